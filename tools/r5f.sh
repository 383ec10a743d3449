#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fresh-sets 0 --legs none > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv > $O/episode.txt 2>&1
cat $O/episode.txt
rm -f $O/trace/*.db
