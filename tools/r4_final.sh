#!/bin/bash
# Round-4 evidence of the final build: the C2 bench line as the driver runs it,
# rocprofv3 kernel stats + FETCH/WRITE passes of that bench (-> traffic.json);
# with C4=1 also the C4 bench line and its passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r4}
if [ -z "$C4" ]; then
echo "== bench C2" && timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err \
&& tail -c 400 gpurun_out/bench_c2_$TAG.json \
&& echo "== profile C2" && timeout -k 10 700 bash tools/profile.sh $TAG C2
else
echo "== bench C4" && timeout -k 10 500 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err \
&& tail -c 400 gpurun_out/bench_c4_$TAG.json \
&& echo "== profile C4" && PROF_STEPS=2 timeout -k 10 1000 bash tools/profile.sh ${TAG}_c4 C4
fi
