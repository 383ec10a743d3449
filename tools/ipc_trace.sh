#!/bin/bash
# Host-side evidence for the device-driven exchange (one GPU, two ranks started
# from this shell): per transport, the enqueue and wall time of whole episodes;
# then rank 0 of an IPC run under rocprofv3 (kernel + HIP API trace, the program
# itself after --; rank 1 runs beside it), so the trace shows which HIP calls a
# multi-round gg_dist_step makes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run_pair() {  # $1 transport, $2 port, $3 tag, rest: extra args
  local t=$1 p=$2 tag=$3; shift 3
  timeout -k 10 240 python -u tools/ipc_rank.py --rank 1 --port $p --transport $t "$@" > gpurun_out/ipc_${tag}_r1.log 2>&1 &
  local pid=$!
  timeout -k 10 240 python -u tools/ipc_rank.py --rank 0 --port $p --transport $t "$@" --out gpurun_out/ipc_${tag}.json > gpurun_out/ipc_${tag}_r0.log 2>&1
  local rc=$?
  wait $pid; local rc1=$?
  echo "$tag rc=$rc/$rc1"; tail -1 gpurun_out/ipc_${tag}_r0.log | cut -c1-400
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ]
}
if [ -z "$TRACE_ONLY" ]; then
run_pair ipc 29612 c2_ipc && run_pair engine 29613 c2_engine &&
run_pair ipc 29614 c4_ipc --config C4 && run_pair engine 29615 c4_engine --config C4 || exit 1
fi
# the trace: rank 1 plain, rank 0 under rocprofv3
timeout -k 10 240 python -u tools/ipc_rank.py --rank 1 --port 29616 --transport ipc --episodes 3 > gpurun_out/ipc_trace_r1.log 2>&1 &
pid=$!
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/ipctrace -o run -- python -u tools/ipc_rank.py --rank 0 --port 29616 --transport ipc --episodes 3 > gpurun_out/ipc_trace_r0.log 2>&1
rc=$?
wait $pid; rc1=$?
echo "trace rc=$rc/$rc1"
[ $rc -eq 0 ] && [ $rc1 -eq 0 ] || exit 1
db=$(find gpurun_out/ipctrace -name "*.db" | head -1)
python3 tools/hip_api_summary.py "$db" > gpurun_out/ipc_hip_api_summary.txt && rm -rf gpurun_out/ipctrace
