#!/bin/bash
# saturation potential on C4-shaped R-MAT (2^20 and 2^22 nodes, W = 4096)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5o; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/sat_potential.py 20 > $O/sat_2p20.txt 2>&1 || { tail -20 $O/sat_2p20.txt; exit 1; }
tail -16 $O/sat_2p20.txt
timeout -k 10 500 python3 tools/sat_potential.py 22 > $O/sat_2p22.txt 2>&1 || { tail -20 $O/sat_2p22.txt; exit 1; }
tail -16 $O/sat_2p22.txt
