mkdir -p gpurun_out/abw
for v in base w5 base w5; do
  GG_HIP_LIB=ab_libs/libgossip_hip_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/abw/$v.json 2> gpurun_out/abw/$v.err || { echo FAIL $v; tail -5 gpurun_out/abw/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/abw/$v.json') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'],4), {k: round(l['ms_per_step'],2) for k,l in d['legs'].items()}, [l['check'] for l in d['legs'].values()], d['config']['oracle_check'][:20])"
done
