#!/bin/bash
# Checkpoint of a build: the GPU suite, the C2 bench line (driver default), the
# C4 bench line (setup time includes build_rev).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r3}
echo "== GPU tests"
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
echo "== bench C2"
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
tail -c 400 gpurun_out/bench_c2_$TAG.json
echo "== bench C4"
timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
tail -c 300 gpurun_out/bench_c4_$TAG.json
