#!/bin/bash
# C4 evidence: lane-half rehearsal (2048 lanes = one half of C4's 4096) and a
# larger rehearsal (2^24 nodes) on 8 locality-ordered parts; the N = 1 bench
# line; rocprofv3 kernel stats and FETCH/WRITE passes of the C4 bench.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
echo "== rehearsal 2^22, 8 parts, 2048 lanes (one lane half)"
timeout -k 10 600 python -u tools/c4_rehearsal.py --nodes 4194304 --lanes 2048 --parts 8 --lane-groups 1 \
    --out gpurun_out/r3_c4_rehearsal_2p22_p8_half.json > gpurun_out/r3_c4_half.log 2>&1
tail -1 gpurun_out/r3_c4_half.log
echo "== rehearsal 2^24, 8 parts"
timeout -k 10 900 python -u tools/c4_rehearsal.py --nodes 16777216 --parts 8 --lane-groups 1 \
    --out gpurun_out/r3_c4_rehearsal_2p24_p8.json
echo "== bench C4 N=1"
timeout -k 10 600 python -u bench.py --config C4 > gpurun_out/r3_bench_c4.json 2> gpurun_out/r3_bench_c4.err
tail -c 600 gpurun_out/r3_bench_c4.json
echo "== profile C4"
PROF_STEPS=2 timeout -k 10 900 bash tools/profile.sh r3_c4 C4
