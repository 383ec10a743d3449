#!/bin/bash
# bench.py's N > 1 flow on one GPU (ranks share it, gloo rendezvous): C2 weak
# scaling at 2 ranks over the host-staged and the IPC exchange (the line's
# oracle_check compares every timed episode with O2's world-2 counters), and
# C4 at 2^22 nodes on 2 parts over IPC with lane halves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # $1 tag, rest: bench args
  local tag=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29700 + RANDOM % 200)) bench.py --gpus 2 --backend gloo "$@" > gpurun_out/rh_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"
  grep '^{' gpurun_out/rh_$tag.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
c=d['config']
print(' ', d['value'], d['ms_per_step'], c.get('exchange'), '|', c.get('check'), '|', c.get('oracle_check'))" || tail -5 gpurun_out/rh_$tag.log
  return $rc
}
run c2_gloo --steps 5 --warmup 2 --no-cpu-baseline &&
run c2_ipc --steps 5 --warmup 2 --no-cpu-baseline --xchg ipc &&
run c4_ipc_halves --steps 3 --warmup 1 --no-cpu-baseline --config C4 --nodes 4194304 --parts 2 --halves 2 --xchg ipc
