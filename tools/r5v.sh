#!/bin/bash
# two-pair resets: tests (parity, prep paths, dense, episodes), C2 A/B alternated, episode trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prep_paths.py tests/test_gpu_parity.py tests/test_gpu_dense.py tests/test_gpu_edge_cases.py -k "not fullsize" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  for v in 1 0; do
    GG_TWO_PAIRS=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --legs none > $O/c2_tp$v.$i.json 2> $O/c2_tp$v.$i.err || { tail -20 $O/c2_tp$v.$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C2 two_pairs=$v', d['ms_per_step'], d['config']['oracle_check'] is not None, d['config']['fresh_injections']['ms_per_step'])" $O/c2_tp$v.$i.json
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fresh-sets 0 --legs none > $O/bench_tr.json 2> $O/trace.log || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_episode.py $O/trace/run_kernel_trace.csv 5 > $O/episode.txt 2>&1
tail -14 $O/episode.txt
rm -f $O/trace/*.db
