#!/bin/bash
# GPU-box check: smoke, GPU parity tests, short bench. Each step time-limited;
# the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 240 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1 \
&& tail -3 gpurun_out/smoke.log \
&& echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
&& tail -5 gpurun_out/gpu_tests.log \
&& echo "== bench" && timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 \
&& tail -3 gpurun_out/bench.log
rc=$?
echo "rc=$rc"
[ -f gpurun_out/smoke.log ] && tail -20 gpurun_out/smoke.log
[ -f gpurun_out/gpu_tests.log ] && grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_tests.log | tail -40
exit $rc
