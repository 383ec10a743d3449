#!/bin/bash
# Full bench (or the legs in LEGS) over variant engine builds, alternating: ab_libs/libgossip_hip_<v>.so
mkdir -p gpurun_out/abw
extra=(); [ -n "$LEGS" ] && extra=(--no-headline --legs "$LEGS")
for v in ${VARIANTS:-base w5 base w5}; do
  GG_HIP_LIB=ab_libs/libgossip_hip_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline "${extra[@]}" > gpurun_out/abw/$v.json 2> gpurun_out/abw/$v.err || { echo FAIL $v; tail -5 gpurun_out/abw/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/abw/$v.json') if l.startswith('{')][-1])
print('$v', d.get('ms_per_step'), {k: round(l['ms_per_step'],2) for k,l in d['legs'].items()}, [l['check'] for l in d['legs'].values()])"
done
