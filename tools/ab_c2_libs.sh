#!/bin/bash
# Same-box A/B of two engine libraries on C2 (bench ms/step, stamp ms/step,
# stream kernel ms/step), alternated 3 times: cur = libgossip_hip.so, alt = $1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
ALT=${1:?library}
run_c2() {  # name lib
  local name=$1 lib=$2
  GG_HIP_LIB=$P/$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --fresh-sets 0 > gpurun_out/abl_$name.$i.log 2>&1 || { echo FAIL $name; tail -5 gpurun_out/abl_$name.$i.log; exit 1; }
  echo "C2 $name $i $(tail -1 gpurun_out/abl_$name.$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; k=r["kernels"]; print(round(d["ms_per_step"],4), "stamp", round(r["stamp_ms_per_step"],4), "stream_ms/step", round(k["stream"]["total_ms"]/d["steps"],4), "frac", round(r["frac"],3))')"
}
for i in 1 2 3; do
  run_c2 cur libgossip_hip.so
  run_c2 alt $ALT
done
