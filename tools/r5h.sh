#!/bin/bash
# tile segments: the IPC / dist GPU tests, the bench rehearsal tests, then the
# C5 2^28 shape on 8 ranks (one GPU, gloo rendezvous, IPC exchange)
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread \
  -k "ipc or world8 or halves or bench" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29811 \
  bench.py --gpus 8 --backend gloo --steps 2 --warmup 2 --legs C5 --c5-side 16384 --leg-steps 2 --no-cpu-baseline \
  > $O/c5_w8.json 2> $O/c5_w8.err || { tail -30 $O/c5_w8.err; exit 1; }
python - <<'PY'
import json
d=json.loads([l for l in open("gpurun_out/r5h/c5_w8.json") if l.startswith("{")][-1])
l=d["legs"]["C5"]
print({k: l.get(k) for k in ("check","exchange","exchange_bytes_per_round_rank0","exchange_bytes_densest_round_rank0","ms_per_step","hbm_bytes_max","rounds_per_step","error")})
print(l.get("checks"))
PY
