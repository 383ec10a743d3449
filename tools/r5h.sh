#!/bin/bash
# the C5 2^28 shape on 8 ranks (one GPU, gloo rendezvous, IPC exchange): densest-round
# payload per rank with tile segments (C2 headline at 64K nodes per rank: short)
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
export PYTHONUNBUFFERED=1
NP=${NP:-8}
GG_IPC_DEBUG=1 GG_BENCH_WATCHDOG=${WD:-60} timeout -k 10 ${TL:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port 29811 \
  bench.py --gpus $NP --backend gloo --steps 2 --warmup 2 --nodes 65536 --legs C5 --c5-side ${SIDE:-16384} --leg-steps 2 --no-cpu-baseline \
  > $O/c5_w8.json 2> $O/c5_w8.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; date; wc -l $O/c5_w8.err; done
wait $pid || { tail -30 $O/c5_w8.err; exit 1; }
python - <<'PY'
import json
d=json.loads([l for l in open("gpurun_out/r5h/c5_w8.json") if l.startswith("{")][-1])
l=d["legs"]["C5"]
print({k: l.get(k) for k in ("check","exchange","exchange_bytes_per_round_rank0","exchange_bytes_densest_round_rank0","ms_per_step","hbm_bytes_max","rounds_per_step","error","setup_s")})
print(l.get("checks"))
PY
