#!/bin/bash
# Same-box A/B of two engine builds on C5 at 2^26
# nodes, per-round kernel times, alternated:
#   pre  = libgossip_hip_pre.so (the previous commit)
#   cur  = libgossip_hip.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gossip-glomers-distributed-systems_amd
one() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env GG_HIP_LIB=$P/$lib "$@" ROUNDS=18 timeout -k 10 200 python3 -u tools/rounds.py C5 8192 > gpurun_out/abff_$name.$i.log 2>&1 || { echo FAIL $name; tail -5 gpurun_out/abff_$name.$i.log; exit 1; }
  echo "C5 $name $i: $(grep -E "^r +[0-9]+ " gpurun_out/abff_$name.$i.log | awk "{print \$3}" | cut -c4-8 | tr "\n" " ") $(tail -1 gpurun_out/abff_$name.$i.log)"
}
for i in 1 2; do
  one pre libgossip_hip_pre.so
  one cur libgossip_hip.so
done
# per-kernel times of the current build (rocprofv3 kernel trace)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ROUNDS=18 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5ff -o c5 -- python3 -u tools/rounds.py C5 8192 > gpurun_out/abff_prof.log 2>&1 || { echo FAIL prof; tail -5 gpurun_out/abff_prof.log; exit 1; }
find gpurun_out/prof_c5ff -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/c5ff_kernel_stats.csv
