#!/bin/bash
# Round-3 multi-rank rehearsals on one GPU (gloo): bench's C4 2-D and lane-halves
# modes at 2^20 nodes, the C4 exchange rehearsal at 2^22 nodes (8 parts; 2 lane
# groups x 4 parts), and C5 on 8 device-built ranks at 2^28 nodes.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=29611
run() { echo "== $*" ; "$@"; }
run timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $P bench.py --config C4 --parts 2 --gpus 4 --backend gloo --nodes 1048576 --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r3_bench_c4_2x2_gloo.json
run timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $((P+1)) bench.py --config C4 --parts 2 --halves 2 --gpus 4 --backend gloo --nodes 1048576 \
    --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3_bench_c4_2x2_halves_gloo.json
run timeout -k 10 600 python -u tools/c4_rehearsal.py --nodes 4194304 --parts 8 --lane-groups 1 \
    --out gpurun_out/r3_c4_rehearsal_2p22_p8.json
run timeout -k 10 600 python -u tools/c4_rehearsal.py --nodes 4194304 --parts 4 --lane-groups 2 \
    --out gpurun_out/r3_c4_rehearsal_2p22_l2p4.json
run timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((P+2)) tools/shard_rehearsal.py --side 16384 --json gpurun_out/r3_c5_shard_rehearsal_2p28_w8.json
