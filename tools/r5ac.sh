#!/bin/bash
# C5 (2^30, W = 64) episode trace through the bench leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r5ac; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-headline --legs C5 --leg-steps 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 tools/trace_episode.py $O/tr/run_kernel_trace.csv 1 > $O/ep.txt 2>&1
tail -16 $O/ep.txt
rm -rf $O/tr
