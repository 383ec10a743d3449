#!/bin/bash
# Per-round diagnostics of one episode under several environment settings of one
# build: tools/ab_rounds_env.sh "GG_X=0" "GG_X=1"   (CFG=C2 by default, ROUNDS=24)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for E in "$@"; do
  k=$((k+1))
  echo "== $E"
  env $E ROUNDS=${ROUNDS:-24} timeout -k 10 200 python -u tools/rounds.py ${CFG:-C2} > gpurun_out/rounds_env_$k.log 2>&1 || { echo FAIL; tail -5 gpurun_out/rounds_env_$k.log; exit 1; }
  cat gpurun_out/rounds_env_$k.log
done
