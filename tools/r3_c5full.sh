#!/bin/bash
# C5 at full size (2^30 nodes, device generator): the episode record, then
# FETCH_SIZE and WRITE_SIZE passes of one episode (per-dispatch HBM bytes of
# expand_stream1 against its algorithmic bytes: tools/pmc_dispatch.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3ff}
FS_TIMEOUT=300 bash tools/fullsize.sh "C5 --device-gen" || exit $?
cp gpurun_out/full/C5_devicegen.json gpurun_out/C5_devicegen_$TAG.json
cp gpurun_out/full/C5_devicegen.log gpurun_out/C5_devicegen_$TAG.log
[ -n "$NO_PMC" ] && exit 0
bash tools/pmc.sh c5full_$TAG "FETCH_SIZE" "WRITE_SIZE" -- python3 -u tools/fullsize.py C5 --device-gen --sample 2000 --max-rounds 19
