#!/bin/bash
# C4 with double-buffered rounds forced on hub graphs (GG_DB=1) vs the F-row kernels: parity, then bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ad; mkdir -p $O
GG_DB=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hubs.py tests/test_gpu_lsat.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    env GG_DB=$v timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4_db$v.json 2> $O/c4_db$v.err || { tail -20 $O/c4_db$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C4 GG_DB=$v', d['ms_per_step'], d['config']['hbm_bytes_rank0']/2**30)" $O/c4_db$v.json
  done
done
