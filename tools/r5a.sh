#!/bin/bash
# Round 5, first GPU pass: the IPC dead-peer test and the IPC suites, the bench
# with its C4/C5 legs at N = 1, and 2-rank one-GPU rehearsals (gloo) of the
# same leg code and of both IPC fallback paths.
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "== $(date +%T) $*"; }
step tests
timeout -k 10 420 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread \
  -k "dead_peer or ipc_exchange_equals or ipc_run_episodes" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
step bench N=1
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
tail -c 600 $O/bench1.json
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step rehearsal 2 ranks gloo
timeout -k 10 400 $RUN --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 2 \
  --c4-nodes 4194304 --c5-side 4096 --no-cpu-baseline > $O/rh2.json 2> $O/rh2.err || { tail -30 $O/rh2.err; exit 1; }
tail -c 600 $O/rh2.json
step rehearsal ipc fail at round 3
GG_BENCH_IPC_FAIL=1:3 GG_IPC_SPIN_LIMIT=65536 timeout -k 10 300 $RUN --master-port 29512 bench.py --gpus 2 \
  --backend gloo --steps 3 --warmup 2 --legs none > $O/rh_ipcfail.json 2> $O/rh_ipcfail.err || { tail -30 $O/rh_ipcfail.err; exit 1; }
tail -c 400 $O/rh_ipcfail.json
step rehearsal episodes fail
GG_BENCH_EPISODES_FAIL=1 timeout -k 10 300 $RUN --master-port 29513 bench.py --gpus 2 \
  --backend gloo --steps 3 --warmup 2 --legs none > $O/rh_epfail.json 2> $O/rh_epfail.err || { tail -30 $O/rh_epfail.err; exit 1; }
tail -c 400 $O/rh_epfail.json
step done
