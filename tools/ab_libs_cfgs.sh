#!/bin/bash
# Episode kernel time per config for several engine builds (per-round logs kept):
#   tools/ab_libs_cfgs.sh "C3 2000000" "C5 4096" -- libA.so libB.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=gossip-glomers-distributed-systems_amd
cfgs=()
while [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
shift
k=0
for C in "${cfgs[@]}"; do
  for L in "$@"; do
    k=$((k+1))
    GG_HIP_LIB=$PKG/$L ROUNDS=${ROUNDS:-40} timeout -k 10 300 python -u tools/rounds.py $C > gpurun_out/abcfg_$k.log 2>&1 || { echo "FAIL $C $L"; tail -5 gpurun_out/abcfg_$k.log; exit 1; }
    echo "$C $L: $(tail -1 gpurun_out/abcfg_$k.log)"
  done
done
