#!/bin/bash
# rocprofv3 kernel trace + stats of the default C2 bench command (no legs), one episode's dispatches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fresh-sets 0 --legs none > $O/bench.json 2> $O/trace.log || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv 5 > $O/episode.txt 2>&1
tail -22 $O/episode.txt
head -12 $O/trace/run_kernel_stats.csv | cut -c1-150
rm -f $O/trace/*.db
