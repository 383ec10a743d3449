#!/bin/bash
# Per-round diagnostics of C2 for several engine builds: tools/ab_rounds.sh lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=gossip-glomers-distributed-systems_amd
for L in "$@"; do
  echo "== $L"
  GG_HIP_LIB=$PKG/$L timeout -k 10 200 python -u tools/rounds.py ${CFG:-C2} > gpurun_out/rounds_$L.log 2>&1 || { echo FAIL; tail -5 gpurun_out/rounds_$L.log; exit 1; }
  cat gpurun_out/rounds_$L.log
done
