#!/bin/bash
# Same-box A/B of engine builds, alternated on one box:
#   pre   = libgossip_hip_pre.so (the build before this change set)
#   nodb  = libgossip_hip_ab.so with GG_NO_DB=1 (no double-buffered lean rounds)
#   cur   = libgossip_hip.so
# C2 bench ms/step, then C5 at 2^26 nodes per-round kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
run_c2() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env GG_HIP_LIB=$P/$lib "$@" timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --fresh-sets 0 > gpurun_out/abr3_c2_$name.$i.log 2>&1 || { echo FAIL $name; tail -5 gpurun_out/abr3_c2_$name.$i.log; exit 1; }
  echo "C2 $name $i $(tail -1 gpurun_out/abr3_c2_$name.$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],4), "stamp", round(r["stamp_ms_per_step"],4), "stream_ms/step", round(r["kernels"]["stream"]["total_ms"]/d["steps"],4), "frac", round(r["frac"],3))')"
}
for i in 1 2 3; do
  run_c2 pre libgossip_hip_pre.so
  run_c2 nodb libgossip_hip_ab.so GG_NO_DB=1
  run_c2 cur libgossip_hip.so
done
for i in 1 2; do
  for L in libgossip_hip_pre.so libgossip_hip.so; do
    GG_HIP_LIB=$P/$L ROUNDS=18 timeout -k 10 200 python3 -u tools/rounds.py C5 8192 > gpurun_out/abr3_c5_$L.$i.log 2>&1 || { echo FAIL $L; tail -5 gpurun_out/abr3_c5_$L.$i.log; exit 1; }
    echo "C5 $L $i: $(grep -E '^r (9|1[0-5]) ' gpurun_out/abr3_c5_$L.$i.log | awk '{print $3}' | tr '\n' ' ') $(tail -1 gpurun_out/abr3_c5_$L.$i.log)"
  done
done
GG_HIP_LIB=$P/libgossip_hip.so ROUNDS=22 timeout -k 10 100 python3 -u tools/rounds.py C2 > gpurun_out/abr3_rounds_c2_cur.log 2>&1
