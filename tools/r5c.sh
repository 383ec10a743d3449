#!/bin/bash
set -o pipefail
O=gpurun_out/r5c; mkdir -p $O
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
GG_BENCH_DEBUG=1 timeout -k 10 300 $RUN --master-port 29655 bench.py --gpus 2 --backend gloo --steps 3 --warmup 2 \
  --legs none --no-cpu-baseline > $O/dbg.json 2> $O/dbg.err; echo "rc=$?"
grep "^bench" $O/dbg.err | grep -v quiescence | cut -c1-220
