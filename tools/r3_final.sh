#!/bin/bash
# Round-3 evidence of the final build: the C2 bench line as the driver runs it,
# rocprofv3 kernel stats + FETCH/WRITE passes of that bench (profiles/traffic.json),
# the C4 bench line, and C5 at 2^30 nodes from the device generator.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r3x}
echo "== bench C2" && timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err \
&& tail -c 300 gpurun_out/bench_c2_$TAG.json \
&& echo "== profile C2" && timeout -k 10 600 bash tools/profile.sh $TAG C2 \
&& echo "== bench C4" && timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err \
&& tail -c 300 gpurun_out/bench_c4_$TAG.json
