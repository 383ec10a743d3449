#!/bin/bash
# C2 A/B over settings of several engine knobs at once:
#   tools/ab_env2_c2.sh "A=1 B=2" "A=0" ...   (each argument: one setting, env assignments)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for set in "$@"; do
  i=$((i + 1))
  echo "== $set"
  env $set ROUNDS=22 timeout -k 10 200 python -u tools/rounds.py C2 > gpurun_out/ab2_rounds_$i.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab2_rounds_$i.log; exit 1; }
  tail -1 gpurun_out/ab2_rounds_$i.log
  env $set timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab2_bench_$i.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab2_bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab2_bench_$i.log').read().strip().splitlines()[-1]); print('ms_per_step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'oracle', bool(d['config'].get('oracle_check')))"
done
