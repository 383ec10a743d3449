#!/bin/bash
# Multi-rank rehearsals of bench.py on the one GPU of a gpurun box (gloo, every
# rank on device 0; the N > 1 check compares the sharded run with one engine):
# C2 at 2 and 4 ranks (vertex-range shards), C4 2 x 2 at 2^22 nodes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name nproc args...
  local name=$1 n=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --steps 3 --warmup 1 "$@" \
    > gpurun_out/gloo_$name.json 2> gpurun_out/gloo_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/gloo_$name.err; exit 1; }
  echo "$name: $(tail -1 gpurun_out/gloo_$name.json | cut -c1-400)"
}
run c2_w2 2 && run c2_w4 4 && run c4_2x2 4 --config C4 --parts 2 --nodes 4194304
