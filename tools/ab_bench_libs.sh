#!/bin/bash
# bench.py ms/step for two engine builds, alternated three times on one box:
#   tools/ab_bench_libs.sh   (libgossip_hip_base.so vs libgossip_hip.so in the package)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
for i in 1 2 3; do
  for L in libgossip_hip_base.so libgossip_hip.so; do
    GG_HIP_LIB=$P/$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 > gpurun_out/ab_$L.$i.log 2>&1 || { echo FAIL $L; tail -5 gpurun_out/ab_$L.$i.log; exit 1; }
    echo "$L $i $(tail -1 gpurun_out/ab_$L.$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4))')"
  done
done
