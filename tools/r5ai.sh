#!/bin/bash
# part labels cached per spec: dist tests with lane halves and parts, then the 2-rank C4 leg rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ai; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lsat.py \
  "tests/test_gpu_dist.py::test_parts_lean_digest_equals_oracle" "tests/test_gpu_dist.py::test_world8_c4_shape_full_width_equals_oracle" \
  "tests/test_gpu_dist.py::test_lane_halves_equal_oracle" "tests/test_gpu_dist.py::test_world8_lane_groups_by_parts_equals_oracle" tests/test_gpu_bench.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29733 \
    bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --nodes 65536 --legs C4 --c4-nodes 4194304 --leg-steps 2 --no-cpu-baseline \
    > $O/c4_r2.json 2> $O/c4_r2.err || { tail -30 $O/c4_r2.err; exit 1; }
python3 - $O/c4_r2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); l = d["legs"]["C4"]
print({k: l.get(k) for k in ("check", "exchange", "ms_per_step", "setup_s", "error")})
PY
