#!/bin/bash
# C2: the marking kernel at 5 waves/SIMD (4 VGPRs spilled) vs 4 waves, alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5ae; mkdir -p $O
for i in 1 2 3; do
  for v in cur w5; do
    lib=gossip-glomers-distributed-systems_amd/libgossip_hip.so; [ $v = w5 ] && lib=tools/ablib/libgossip_w5.so
    GG_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c2_$v.json 2> $O/c2_$v.err || { tail -20 $O/c2_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('C2 $v', d['ms_per_step'], 'stream ms/step', r['kernels']['stream']['total_ms']/d['steps'], d['config']['oracle_check'] is not None)" $O/c2_$v.json
  done
done
