#!/bin/bash
# Round 5: the bench rehearsal tests, then the whole GPU suite with durations.
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== $(date +%T) bench tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread \
  > $O/bench_tests.log 2>&1 || { tail -40 $O/bench_tests.log; exit 1; }
tail -3 $O/bench_tests.log
echo "== $(date +%T) suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 \
  > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -32 $O/suite.log
