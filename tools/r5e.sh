#!/bin/bash
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_prep_paths.py tests/test_episodes.py tests/test_gpu_sync_alloc.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --legs none > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open("gpurun_out/r5e/bench.json").read().strip().splitlines()[-1])
r=d["roofline"]
print(d["ms_per_step"], d["value"], r["frac"], r["event_ms_per_step"], r["per_call_ms_per_step"], d["config"]["oracle_check"][:40], d["config"]["fresh_injections"]["ms_per_step"])
PY
bash tools/r5f.sh | tail -32
