#!/bin/bash
# C2 per-round stamps, the bench line and a rocprofv3 kernel trace of it (one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=22 timeout -k 10 200 python -u tools/rounds.py C2 > gpurun_out/c2_rounds.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/c2_bench.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2trace -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c2trace.log 2>&1
