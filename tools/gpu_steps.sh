#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit.
# Usage: tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
# Output of step <name> goes to gpurun_out/<name>.log. A step that ends with
# status 0 or 1 (a test failure) lets the next one run; anything else (a time
# limit, an abort, a segfault, a GPU fault) ends the script there.
mkdir -p gpurun_out
for spec in "$@"; do
    secs="${spec%%|*}"
    rest="${spec#*|}"
    name="${rest%%|*}"
    cmd="${rest#*|}"
    echo "== $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name exit $rc"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping after $name (exit $rc)"
        exit $rc
    fi
done
exit 0
