#!/bin/bash
# C4: where the lean digest's cost sits — episode traces with the digest off, read-only (no marking), on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5y; mkdir -p $O
for v in off nomark on; do
  case $v in off) env="GG_LSAT=0";; nomark) env="GG_LSAT_NOMARK=1 GG_HIP_LIB=tools/ablib/libgossip_ab.so";; on) env="GG_LSAT=1";; esac
  env $env timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none > $O/c4_$v.json 2> $O/c4_$v.err || { tail -20 $O/c4_$v.err; exit 1; }
  python3 tools/trace_episode.py $O/tr_$v/run_kernel_trace.csv 1 > $O/ep_$v.txt 2>&1
  echo "== $v $(grep 'episode:' $O/ep_$v.txt)"
  grep -E "expand_stream<|hub_chunks<" $O/ep_$v.txt | head -20 | awk '{print $2}' | paste -sd' '
  rm -rf $O/tr_$v
done
