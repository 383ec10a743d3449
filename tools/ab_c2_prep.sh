#!/bin/bash
# Same-box A/B on C2 (bench ms/step and stamp times): round_prep's general
# sparse path (ab) against the 16-nodes-per-thread scan with wave-listed
# out-lists forced at C2's size (wide, GG_PREP_WIDE=1), both from
# libgossip_hip_ab.so, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
run_c2() {  # name env...
  local name=$1; shift
  env GG_HIP_LIB=$P/libgossip_hip_ab.so "$@" timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --fresh-sets 0 > gpurun_out/abc2_$name.$i.log 2>&1 || { echo FAIL $name; tail -5 gpurun_out/abc2_$name.$i.log; exit 1; }
  echo "C2 $name $i $(tail -1 gpurun_out/abc2_$name.$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; k=r["kernels"]; print(round(d["ms_per_step"],4), "stamp", round(r["stamp_ms_per_step"],4), "prep_ms/step", round(k["prep"]["total_ms"]/d["steps"],4), "stream_ms/step", round(k["stream"]["total_ms"]/d["steps"],4))')"
}
for i in 1 2 3; do
  run_c2 ab
  run_c2 wide GG_PREP_WIDE=1
done
GG_HIP_LIB=$P/libgossip_hip_ab.so GG_PREP_WIDE=1 ROUNDS=22 timeout -k 10 100 python3 -u tools/rounds.py C2 > gpurun_out/abc2_rounds_wide.log 2>&1
GG_HIP_LIB=$P/libgossip_hip_ab.so ROUNDS=22 timeout -k 10 100 python3 -u tools/rounds.py C2 > gpurun_out/abc2_rounds_ab.log 2>&1
