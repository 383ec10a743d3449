#!/bin/bash
# Multi-rank rehearsal on ONE GPU: (1) can RCCL put 2 ranks on one device?
# (2) bench.py --gpus 2 with gloo staging (functional), (3) with nccl if (1) works.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 5 90 $TR --master-port 29511 tools/nccl_probe.py > gpurun_out/probe.log 2>&1
prc=$?
echo "probe rc=$prc"; tail -5 gpurun_out/probe.log
case $prc in 124|134|137|139) exit $prc;; esac
timeout -k 10 300 $TR --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/bench2_gloo.log 2>&1
rc=$?
echo "bench gloo rc=$rc"; grep -E '^\{' gpurun_out/bench2_gloo.log | cut -c1-400; tail -3 gpurun_out/bench2_gloo.log
[ $rc -ne 0 ] && exit $rc
if [ $prc -eq 0 ]; then
  timeout -k 10 300 $TR --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench2_nccl.log 2>&1
  rc=$?
  echo "bench nccl rc=$rc"; grep -E '^\{' gpurun_out/bench2_nccl.log | cut -c1-600; tail -3 gpurun_out/bench2_nccl.log
fi
exit $rc
