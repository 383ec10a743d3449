#!/bin/bash
# Same-box A/B of two engine builds (libgossip_hip_pre.so: before; libgossip_hip.so: after):
# C2 bench ms/step, and C5 at 2^26 nodes per-round kernel times, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
for i in 1 2 3; do
  for L in libgossip_hip_pre.so libgossip_hip.so; do
    GG_HIP_LIB=$P/$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --fresh-sets 0 > gpurun_out/abr3_c2_$L.$i.log 2>&1 || { echo FAIL $L; tail -5 gpurun_out/abr3_c2_$L.$i.log; exit 1; }
    echo "C2 $L $i $(tail -1 gpurun_out/abr3_c2_$L.$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],4), "stream_ms/step", round(r["kernels"]["stream"]["total_ms"]/d["steps"],4))')"
  done
done
for i in 1 2; do
  for L in libgossip_hip_pre.so libgossip_hip.so; do
    GG_HIP_LIB=$P/$L ROUNDS=18 timeout -k 10 200 python3 -u tools/rounds.py C5 8192 > gpurun_out/abr3_c5_$L.$i.log 2>&1 || { echo FAIL $L; tail -5 gpurun_out/abr3_c5_$L.$i.log; exit 1; }
    echo "C5 $L $i: $(grep -E '^r (9|1[0-5]) ' gpurun_out/abr3_c5_$L.$i.log | awk '{print $3}' | tr '\n' ' ') $(tail -1 gpurun_out/abr3_c5_$L.$i.log)"
  done
done
