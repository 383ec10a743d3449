#!/bin/bash
# One rocprofv3 --pmc pass per counter group over the same command, then a
# per-kernel table of every counter (tools/pmc_table.py).
# Usage: tools/pmc.sh <tag> "<counters of pass 1>" ["<pass 2>" ...] -- <program> [args...]
#   -> gpurun_out/pmc_<tag>/{p1,p2,...}/run_counter_collection.csv, summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
i=0
for g in "${groups[@]}"; do
    i=$((i + 1))
    echo "== pass $i: $g"
    # shellcheck disable=SC2086
    timeout -s KILL 300 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_table.py $(find "$OUT" -name "*counter_collection.csv") | tee "$OUT/summary.txt"
