#!/bin/bash
# lean digest: parity at every group width, then C2 per-round totals digest off / DPP / shuffles, C4 with DPP
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lsat.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in off dpp shfl; do
    case $v in off) env="GG_LSAT=0";; dpp) env="GG_LSAT=1";; shfl) env="GG_LSAT=1 GG_HIP_LIB=tools/ablib/libgossip_nodpp.so";; esac
    env $env ROUNDS=22 timeout -k 10 120 python3 tools/rounds.py C2 > $O/c2_$v.$i.txt 2>&1 || { tail $O/c2_$v.$i.txt; exit 1; }
    echo "C2 $v $i $(tail -1 $O/c2_$v.$i.txt)"
  done
done
GG_LSAT=1 timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4_dpp.json 2> $O/c4_dpp.err || { tail -20 $O/c4_dpp.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C4 dpp', d['ms_per_step'])" $O/c4_dpp.json
