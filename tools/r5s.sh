#!/bin/bash
# lean digest on vertex parts: parity tests, then the C4 leg on 1 rank (10^8) and rehearsals on 2 / 8 ranks (2^22, gloo)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lsat.py tests/test_gpu_hubs.py \
  "tests/test_gpu_dist.py::test_parts_lean_digest_equals_oracle" "tests/test_gpu_dist.py::test_world8_c4_shape_full_width_equals_oracle" \
  "tests/test_gpu_dist.py::test_lane_halves_equal_oracle" "tests/test_gpu_dist.py::test_ipc_run_episodes_equal_oracle" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  GG_LSAT=$v timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700+v)) \
    bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --nodes 65536 --legs C4 --c4-nodes 4194304 --leg-steps 2 --no-cpu-baseline \
    > $O/c4_r2_lsat$v.json 2> $O/c4_r2_lsat$v.err &
  p=$!; while kill -0 $p 2>/dev/null; do sleep 20; echo "  r2 lsat=$v $(date +%T) $(grep 'bench\[' $O/c4_r2_lsat$v.err | tail -1 | cut -c1-90)"; done
  wait $p || { tail -30 $O/c4_r2_lsat$v.err; exit 1; }
  python3 - $O/c4_r2_lsat$v.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); l = d["legs"]["C4"]
print({k: l.get(k) for k in ("check", "exchange", "ms_per_step", "rounds_per_step", "error")}, l.get("checks", {}).get("failures"))
PY
done
