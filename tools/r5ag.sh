#!/bin/bash
# C4 rehearsal at 2^24 nodes on 8 device-built parts (one GPU, ranks one at a time per round), this build (lean digest on parts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ag; mkdir -p $O
timeout -k 10 1000 python3 tools/c4_rehearsal.py --nodes 16777216 --parts 8 --lane-groups 1 --out $O/c4_2p24_p8.json > $O/log.txt 2>&1 &
p=$!; S=$(date +%s); while kill -0 $p 2>/dev/null; do sleep 30; echo "  $(( $(date +%s) - S )) s: $(tail -1 $O/log.txt | cut -c1-100)"; done
wait $p || { tail -30 $O/log.txt; exit 1; }
python3 tools/project_c4.py $O/c4_2p24_p8.json --row-bytes 512 > $O/project.json
python3 -c "import json; d=json.load(open('$O/project.json')); [print(p['link_GBps'], round(p['single_ms'],1), round(p['speedup_exchange_after'],2), round(p['speedup_overlap_bound'],2)) for p in d['projections']]"
