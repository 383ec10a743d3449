#!/bin/bash
# vectorized compact_scan: split-compaction tests, full-size tests, C5 trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r5af; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "C5 or c5 or split or compact" tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-headline --legs C5 --leg-steps 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 tools/trace_episode.py $O/tr/run_kernel_trace.csv 1 > $O/ep.txt 2>&1
tail -12 $O/ep.txt
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); l=d['legs']['C5']; print('C5', l['ms_per_step'], l['check'])" $O/c5.json
rm -rf $O/tr
