#!/bin/bash
# two-pair resets: zeroing stream priority A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r5w; mkdir -p $O
for i in 1 2; do
  for v in "GG_TWO_PAIRS=0" "GG_TWO_PAIRS=1 GG_ZPRIO=1" "GG_TWO_PAIRS=1 GG_ZPRIO=0"; do
    env $v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C2 $v', d['ms_per_step'], d['roofline']['event_ms_per_step'])" $O/c2.json
  done
done
GG_ZPRIO=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fresh-sets 0 --legs none > $O/bench_tr.json 2> $O/trace.log || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv 5 > $O/episode.txt 2>&1
head -8 $O/episode.txt; tail -12 $O/episode.txt
rm -f $O/trace/*.db
