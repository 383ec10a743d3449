#!/bin/bash
# PMC passes over tools/rounds.py (one counter group per pass).
# Usage: tools/pmc.sh TAG "CNT1 CNT2" "CNT3" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/pmc_$TAG
k=0
for grp in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/p$k -o run -- python3 tools/rounds.py C2 > gpurun_out/pmc_$TAG/p$k.log 2>&1 || { echo "pass $k ($grp) failed"; exit 1; }
done
echo done
