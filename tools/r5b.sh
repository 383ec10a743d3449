#!/bin/bash
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
i=0
for s in DBG_GOLD=1 DBG_FN=1 "DBG_GOLD=1 DBG_FN=1"; do
  i=$((i+1))
  env $s timeout -k 10 200 $RUN --master-port $((29710+i)) tools/dbg_bench.py > $O/dbgc_$i.log 2>&1 || { tail -20 $O/dbgc_$i.log; exit 1; }
  echo "$s"; grep "^rank" $O/dbgc_$i.log | cut -c1-200
done
