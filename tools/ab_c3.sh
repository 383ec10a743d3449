#!/bin/bash
# C3-shaped A/B (random 8-regular, W = 1024, bisection + sync) of engine builds:
#   tools/ab_c3.sh V lib1 lib2 ...   (library paths relative to the repo; "-" = the default build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$1; shift
for L in "$@"; do
  echo "== $L"
  if [ "$L" = "-" ]; then unset GG_HIP_LIB; else export GG_HIP_LIB=$L; fi
  ROUNDS=32 timeout -k 10 200 python -u tools/rounds.py C3 $V > gpurun_out/ab_c3_$(basename $L).log 2>&1 || { echo FAIL; tail -3 gpurun_out/ab_c3_$(basename $L).log; exit 1; }
  tail -1 gpurun_out/ab_c3_$(basename $L).log
done
