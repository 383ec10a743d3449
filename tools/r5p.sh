#!/bin/bash
# C2 per-round device times with the lean digest on and off (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5p; mkdir -p $O
for v in 1 0 1 0; do
  GG_LSAT=$v ROUNDS=22 timeout -k 10 120 python3 tools/rounds.py C2 > $O/c2_rounds_lsat$v.txt 2>&1 || { tail $O/c2_rounds_lsat$v.txt; exit 1; }
  echo "lsat=$v $(tail -1 $O/c2_rounds_lsat$v.txt)"
done
paste <(cut -c1-60 $O/c2_rounds_lsat1.txt) <(cut -c1-60 $O/c2_rounds_lsat0.txt)
