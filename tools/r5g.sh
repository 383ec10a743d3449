#!/bin/bash
# solo marking rounds: tests, then A/B on one box (C2 bench, no legs)
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_prep_paths.py tests/test_episodes.py tests/test_gpu_parity.py tests/test_gpu_sync_alloc.py -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() { env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --legs none --no-cpu-baseline --fresh-sets 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$*', round(d['ms_per_step'],4), round(r['event_ms_per_step'],4), d['config']['oracle_check'][:12])"; }
for i in 1 2 3; do
run GG_X=1
run GG_SOLO=0
done
