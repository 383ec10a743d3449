#!/bin/bash
# C2 A/B of an engine knob: tools/ab_env_c2.sh NAME "VAL1 VAL2 ..." (rounds + bench per value)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $2; do
  echo "== $1=$v"
  env $1=$v ROUNDS=22 timeout -k 10 200 python -u tools/rounds.py C2 > gpurun_out/ab_rounds_$v.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab_rounds_$v.log; exit 1; }
  tail -1 gpurun_out/ab_rounds_$v.log
  env $1=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench_$v.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab_bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench_$v.log').read().strip().splitlines()[-1]); print('ms_per_step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3))"
done
