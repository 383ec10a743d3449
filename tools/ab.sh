#!/bin/bash
# A/B the bench across engine builds: tools/ab.sh lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=gossip-glomers-distributed-systems_amd
for rep in 1 2; do
for L in "$@"; do
  echo "== $L rep $rep"
  GG_HIP_LIB=$PKG/$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$L.log 2>&1 || { echo FAIL; tail -5 gpurun_out/ab_$L.log; exit 1; }
  python - "$L" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/ab_{sys.argv[1]}.log") if x.startswith("{")][-1]
d=json.loads(l); r=d["roofline"]
print(f'{sys.argv[1]}: value={d["value"]:.4g} ms/step={d["ms_per_step"]:.3f} launch_ms={r["avg_launch_ms"]:.4f} achieved={r["achieved"]:.0f}GB/s frac={r["frac"]:.3f}')
PY
done
done
