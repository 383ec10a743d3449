#!/bin/bash
# C5 at 2^27 on 8 ranks (one GPU): payload per rank, heads (engine exchange over gloo) vs tile segments (IPC)
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
export PYTHONUNBUFFERED=1
for x in engine ipc; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29831 \
    bench.py --gpus 8 --backend gloo --steps 2 --warmup 2 --nodes 65536 --legs C5 --c5-side 11585 --leg-steps 1 --no-cpu-baseline --xchg $x \
    > $O/$x.json 2> $O/$x.err &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 20; echo "  $x $(date +%T) $(grep -c 'bench\[' $O/$x.err)"; done
  wait $pid; echo "  rc=$?"
  python - $O/$x.json <<'PY'
import json, sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); l=d["legs"]["C5"]
print({k: l.get(k) for k in ("check","exchange","exchange_bytes_per_round_rank0","exchange_bytes_densest_round_rank0","ms_per_step","error")})
PY
done
