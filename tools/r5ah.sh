#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lsat.py tests/test_gpu_hubs.py \
  "tests/test_gpu_dist.py::test_parts_lean_digest_equals_oracle" tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
