#!/bin/bash
# the full GPU suite, then the default bench line (N = 1: C2 headline, C4 and C5 legs, CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5r; mkdir -p $O
S=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc in $(( $(date +%s) - S )) s"; tail -3 $O/gpu_suite.log
[ $rc -eq 0 ] || exit 1
[ "${1:-}" = "suite" ] && exit 0
S=$(date +%s)
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err &
p=$!; while kill -0 $p 2>/dev/null; do sleep 30; echo "  bench $(( $(date +%s) - S )) s: $(tail -1 $O/bench.err | cut -c1-100)"; done; wait $p || { tail -20 $O/bench.err; exit 1; }
echo "bench in $(( $(date +%s) - S )) s"
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("C2", round(d["ms_per_step"], 4), "ms/step", f'{d["value"]:.3e}', "frac", round(r["frac"], 3), "line_frac", round(r["line_frac"], 3), r.get("line_source", "")[:60])
for n, l in d.get("legs", {}).items():
    rr = l.get("roofline") or {}
    print(n, round(l.get("ms_per_step", 0), 1), "ms/step", l.get("check"), "line_frac", rr.get("line_frac"), "traffic", rr.get("traffic"))
print("cpu", d.get("cpu_baseline", {}) and d["cpu_baseline"].get("value"))
PY
