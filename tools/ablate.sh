#!/bin/bash
# Dense-round ablation (timing only): per-round stamps of rounds.py under GG_ABLATE masks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ablate
for m in 0 1 2 4 3 7; do
  GG_ABLATE=$m ROUNDS=22 timeout -k 10 120 python tools/rounds.py C2 > gpurun_out/ablate/m$m.log 2>&1 || exit 1
  echo "mask $m: $(grep -E '^r 1[3-9]' gpurun_out/ablate/m$m.log | awk '{s+=substr($3,4)} END {printf "dense rounds 13-19 avg ms %.4f", s/NR}')  $(tail -1 gpurun_out/ablate/m$m.log)"
done
