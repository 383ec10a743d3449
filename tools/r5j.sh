#!/bin/bash
# IPC import at the C5 leg: 4 ranks at 2^28 (larger windows) and 8 ranks at 2^27
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "4 16384" "8 11585"; do
  set -- $cfg
  echo "== $1 ranks, side $2"
  GG_IPC_DEBUG=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $((29820+$1)) \
    bench.py --gpus $1 --backend gloo --steps 2 --warmup 2 --nodes 65536 --legs C5 --c5-side $2 --leg-steps 2 --no-cpu-baseline \
    > $O/r$1.json 2> $O/r$1.err &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 20; echo "  $(date +%T) $(grep -c opened $O/r$1.err) opened, $(grep -c 'tables done' $O/r$1.err) done"; done
  wait $pid; echo "  rc=$?"
  grep -h "exchange_bytes_densest" $O/r$1.json | head -c 0
  python - $O/r$1.json <<'PY'
import json, sys
try:
    d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); l=d["legs"]["C5"]
    print({k: l.get(k) for k in ("check","exchange_bytes_densest_round_rank0","ms_per_step","hbm_bytes_max","error")})
except Exception as e: print("no result", e)
PY
done
