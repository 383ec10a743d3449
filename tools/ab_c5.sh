#!/bin/bash
# C5-shaped A/B (grid + one long link per node, W = 64) of engine builds:
#   tools/ab_c5.sh SIDE lib1 lib2 ...   (library paths relative to the repo; "-" = the default build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=$1; shift
for L in "$@"; do
  echo "== $L"
  if [ "$L" = "-" ]; then unset GG_HIP_LIB; else export GG_HIP_LIB=$L; fi
  ROUNDS=20 timeout -k 10 300 python -u tools/rounds.py C5 $S > gpurun_out/ab_c5_$(basename $L).log 2>&1 || { echo FAIL; tail -3 gpurun_out/ab_c5_$(basename $L).log; exit 1; }
  tail -1 gpurun_out/ab_c5_$(basename $L).log
done
