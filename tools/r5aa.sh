#!/bin/bash
# C2 with the lean digest forced on vs off (per-round kernel totals, bench), after the pipeline change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5aa; mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    GG_LSAT=$v ROUNDS=22 timeout -k 10 120 python3 tools/rounds.py C2 > $O/c2_rounds_lsat$v.$i.txt 2>&1 || { tail $O/c2_rounds_lsat$v.$i.txt; exit 1; }
    GG_LSAT=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c2_lsat$v.json 2> $O/c2_lsat$v.err || { tail -20 $O/c2_lsat$v.err; exit 1; }
    echo "lsat=$v $i $(tail -1 $O/c2_rounds_lsat$v.$i.txt) bench $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" $O/c2_lsat$v.json)"
  done
done
