#!/bin/bash
# 8-rank C4 leg rehearsal (2^22 nodes, one GPU, gloo + IPC, lane halves) with the part digest on and off; fullsize.py smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 200 python3 tools/fullsize.py C5 --side 4096 --device-gen --json $O/c5_4096.json > $O/fullsize.log 2>&1 || { tail -20 $O/fullsize.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_4096.json')); print('fullsize C5 4096', d['episode_s'], d['roofline']['line_frac'], d['roofline']['line_source'][:60])"
for v in 1 0; do
  GG_LSAT=$v timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29800+v)) \
    bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --nodes 65536 --legs C4 --c4-nodes 4194304 --leg-steps 2 --no-cpu-baseline \
    > $O/c4_r8_lsat$v.json 2> $O/c4_r8_lsat$v.err &
  p=$!; while kill -0 $p 2>/dev/null; do sleep 20; echo "  r8 lsat=$v $(date +%T) $(grep 'bench\[' $O/c4_r8_lsat$v.err | tail -1 | cut -c1-90)"; done
  wait $p || { tail -30 $O/c4_r8_lsat$v.err; exit 1; }
  python3 - $O/c4_r8_lsat$v.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); l = d["legs"]["C4"]
print({k: l.get(k) for k in ("check", "exchange", "ms_per_step", "setup_s", "exchange_bytes_densest_round_rank0", "error")})
PY
done
