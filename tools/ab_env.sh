#!/bin/bash
# A/B the bench across environment settings of one build:
#   tools/ab_env.sh "GG_PREP_BLOCKS=4096" "GG_PREP_BLOCKS=1024"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for rep in 1 2 3; do
for E in "$@"; do
  k=$((k+1))
  echo "== $E rep $rep"
  env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abenv_$k.log 2>&1 || { echo FAIL; tail -5 gpurun_out/abenv_$k.log; exit 1; }
  python - "$E" "gpurun_out/abenv_$k.log" <<'PY'
import json,sys
l=[x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d=json.loads(l); r=d["roofline"]; k=r["kernels"]
print(f'{sys.argv[1]}: value={d["value"]:.4g} ms/step={d["ms_per_step"]:.3f} stamp_ms={r["stamp_ms_per_step"]:.3f} '
      f'prep_ms/step={k["prep"]["total_ms"]/d["steps"]:.3f} stream_ms/step={k["stream"]["total_ms"]/d["steps"]:.3f}')
PY
done
done
