#!/bin/bash
# learned marking flags: parity tests, C4 episode trace and bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lsat.py tests/test_gpu_hubs.py tests/test_gpu_prep_paths.py tests/test_gpu_parity.py \
  "tests/test_gpu_dist.py::test_parts_lean_digest_equals_oracle" "tests/test_gpu_dist.py::test_world8_c4_shape_full_width_equals_oracle" tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python3 tools/trace_episode.py $O/tr/run_kernel_trace.csv 1 > $O/ep.txt 2>&1
echo "$(grep 'episode:' $O/ep.txt)"
grep -E "expand_stream<" $O/ep.txt | head -10 | awk '{print $2}' | paste -sd' '
rm -rf $O/tr
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4_$i.json 2> $O/c4_$i.err || { tail -20 $O/c4_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C4', d['ms_per_step'])" $O/c4_$i.json
done
