#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/trace_rounds
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_rounds -o run -- python3 tools/rounds.py ${1:-C2} > gpurun_out/trace_rounds/log.txt 2>&1
