#!/bin/bash
# Full-size config runs (tools/fullsize.py), each time-limited; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/full
# heartbeat: host-side graph ingest of 10^8-node inputs prints nothing for minutes
( while sleep 60; do echo "[heartbeat $(date +%T)]"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for spec in "$@"; do
  name=$(echo $spec | tr ' ' '_' | tr -d '-')
  echo "== $spec"
  timeout -k 10 ${FS_TIMEOUT:-500} python -u tools/fullsize.py $spec --json gpurun_out/full/$name.json > gpurun_out/full/$name.log 2>&1
  rc=$?
  tail -4 gpurun_out/full/$name.log | cut -c1-1500
  [ $rc -ne 0 ] && exit $rc
done
exit 0
