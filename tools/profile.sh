#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then one PMC pass per
# TCC counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage: tools/profile.sh <tag> [C2|C4]   -> gpurun_out/prof_<tag>/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
CFG=${2:-C2}
ARGS="--config $CFG --steps ${PROF_STEPS:-5} --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none"
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 \
&& echo "== FETCH_SIZE" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 \
&& echo "== WRITE_SIZE" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -eq 0 ] && python3 tools/traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv "rocprofv3 --pmc passes over: bench.py $ARGS ($TAG)" $OUT/traffic.json $CFG
find $OUT -name "*.csv" | head -20
exit $rc
