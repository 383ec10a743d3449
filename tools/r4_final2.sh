#!/bin/bash
# Round-4 evidence on the build with gg_run_episodes and block lists: the C2
# bench line (CPU baseline included), its rocprofv3 kernel stats and counter
# traffic, one episode's dispatch trace, C2/C3 per-round times, and bench's
# N = 2 flow rehearsed on one GPU (gloo rendezvous, IPC exchange).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/f2_bench_c2.json 2> gpurun_out/f2_bench_c2.err && echo bench ok \
&& bash tools/profile.sh r4c C2 > gpurun_out/f2_profile.log 2>&1 && echo profile ok \
&& python3 tools/trace_episode.py gpurun_out/prof_r4c/trace/run_kernel_trace.csv > gpurun_out/f2_episode_trace.txt 2>&1 && echo trace ok \
&& ROUNDS=22 timeout -k 10 120 python tools/rounds.py C2 > gpurun_out/f2_rounds_c2.log 2>&1 && echo c2 rounds ok \
&& ROUNDS=30 timeout -k 10 200 python tools/rounds.py C3 2097152 > gpurun_out/f2_rounds_c3.log 2>&1 && echo c3 rounds ok \
&& GG_BLOCK_LISTS=0 ROUNDS=30 timeout -k 10 200 python tools/rounds.py C3 2097152 > gpurun_out/f2_rounds_c3_nobll.log 2>&1 && echo c3 nobll ok \
&& timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29700 + RANDOM % 200)) bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline --xchg ipc \
      > gpurun_out/f2_rh_c2_ipc.log 2>&1 && echo rehearsal ok
echo rc=$?
rm -f gpurun_out/prof_r4c/*/run_*.db
