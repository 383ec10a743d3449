#!/bin/bash
# C4 (10^8 R-MAT, W = 4096) on one GPU: one episode's dispatch trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv 1 > $O/episode.txt 2>&1
cat $O/episode.txt
rm -f $O/trace/*.db
