#!/bin/bash
# lean saturation digest: parity tests, then the C4 episode trace and a C2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lsat.py tests/test_gpu_hubs.py tests/test_gpu_prep_paths.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv 1 > $O/episode.txt 2>&1
tail -14 $O/episode.txt
rm -f $O/trace/*.db
for v in 1 0; do
  GG_LSAT=$v timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4_lsat$v.json 2> $O/c4_lsat$v.err || { tail -20 $O/c4_lsat$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C4 lsat=$v', d['ms_per_step'], d.get('check'))" $O/c4_lsat$v.json
done
for v in 1 0 1 0; do
  GG_LSAT=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --legs none > $O/c2_lsat$v.json 2> $O/c2_lsat$v.err || { tail -20 $O/c2_lsat$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C2 lsat=$v', d['ms_per_step'])" $O/c2_lsat$v.json
done
