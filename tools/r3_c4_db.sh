#!/bin/bash
# C4 with double-buffered rounds: the N = 1 bench line and the 8-part
# rehearsal at 2^24 nodes (per-rank kernel times and payloads -> projection).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
echo "== bench C4" && timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/bench_c4_db.json 2> gpurun_out/bench_c4_db.err \
&& tail -c 300 gpurun_out/bench_c4_db.json \
&& echo "== rehearsal 2^24, 8 parts" && timeout -k 10 700 python -u tools/c4_rehearsal.py --nodes 16777216 --parts 8 --lane-groups 1 \
    --out gpurun_out/r3_c4_rehearsal_2p24_p8_db.json > gpurun_out/r3_c4_rehearsal_db.log 2>&1 \
&& tail -3 gpurun_out/r3_c4_rehearsal_db.log
