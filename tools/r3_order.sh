#!/bin/bash
# Locality-ordered shard rows: the C4 rehearsal at 2^22 nodes on 8 parts with
# the reordered shards, the single engine at native vs degree row order (what
# order is worth at this size), then sync rounds streamed vs tiles.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
echo "== gg_topology_part tests"
timeout -k 10 300 python -u -m pytest "tests/test_gpu_dist.py::test_topology_part_equals_single" -m gpu -v -s \
    --timeout 200 --timeout-method thread > gpurun_out/r3_order_tests2.log 2>&1
tail -2 gpurun_out/r3_order_tests2.log
echo "== rehearsal, reordered shards"
timeout -k 10 600 python -u tools/c4_rehearsal.py --nodes 4194304 --parts 8 --lane-groups 1 \
    --out gpurun_out/r3_c4_rehearsal_2p22_p8_ordered.json
echo "== single engine, native order"
GG_ORDER=native timeout -k 10 300 python -u tools/c4_rehearsal.py --nodes 4194304 --single-only 10
echo "== single engine, degree order"
timeout -k 10 300 python -u tools/c4_rehearsal.py --nodes 4194304 --single-only 10
echo "== sync rounds"
timeout -k 10 600 python -u tools/sync_rounds.py --json gpurun_out/r3_sync_rounds.json
