#!/bin/bash
# bench.py's default N > 1 exchange choice (--xchg auto) on one GPU: the
# device-driven exchange after its validation rounds, and the fallback when one
# rank fails (GG_BENCH_IPC_FAIL=1: rank 1 raises after the validation rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29700 + RANDOM % 200)) bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/auto_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"
  grep '^{' gpurun_out/auto_$tag.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print(' ', round(d['ms_per_step'],3), c.get('exchange'), '|', c.get('exchange_note'), '|', bool(c.get('oracle_check')))" || tail -5 gpurun_out/auto_$tag.log
  grep "falling back" gpurun_out/auto_$tag.log | head -2
  return $rc
}
run ipc GG_X=1 && run fallback GG_BENCH_IPC_FAIL=1
