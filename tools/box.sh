#!/bin/bash
# GPU-box tasks (one gpurun call each; every GPU step under its own time limit,
# steps chained so the first failure ends the call):
#   tools/box.sh suite              the GPU suite (-m gpu) with per-test durations
#   tools/box.sh golden CFG [args]  tests/golden/make_fullsize_golden.py on the box's host cores
#                                   (writes gpurun_out/gold/; copy the records to tests/golden/)
#   tools/box.sh bench [args]       bench.py at N = 1 (default: the driver's command)
#   tools/box.sh legs LEGS [args]   bench.py --no-headline --legs LEGS
#   tools/box.sh ipc8               8 ranks on this one GPU (gloo rendezvous, IPC exchange): the C2
#                                   headline, then the C5 leg at 2^28 (tools/r5h.sh)
#   tools/box.sh c4half2 [NODES]    2 ranks on this one GPU: the C4 leg with lane halves (digest mode per rank)
#   tools/box.sh memset             tools/graph_memset_repro: a captured hipMemsetAsync node against our
#                                   zero kernel, one process and two at once
#   tools/box.sh ipcrepro [SCN...]  tools/ipc_reopen_repro: hipIpcOpenMemHandle after close / free / realloc
#   tools/box.sh pmc "CFGS"         tools/pmc_passes.sh (request ceilings, traffic passes)
# Output under gpurun_out/box/ (merged back by gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/box
mkdir -p $O
task=$1
shift
tick() {  # a progress line every 30 s while pid $1 runs (the box's hang rule), then its status
    while kill -0 "$1" 2>/dev/null; do sleep 30; echo "  $2 $(date +%T) $(tail -c 200 "$3" 2>/dev/null | tail -1)"; done
    wait "$1"
}
case $task in
suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=40 \
        "$@" > $O/suite.log 2>&1 &
    tick $! suite $O/suite.log
    rc=$?
    tail -60 $O/suite.log
    exit $rc ;;
golden)
    mkdir -p gpurun_out/gold
    timeout -k 10 1150 python -u tests/golden/make_fullsize_golden.py "$@" --outdir gpurun_out/gold \
        > gpurun_out/gold/$1.log 2>&1 &
    tick $! golden gpurun_out/gold/$1.log
    rc=$?
    tail -30 gpurun_out/gold/$1.log
    exit $rc ;;
bench)
    args=("$@")
    [ ${#args[@]} -eq 0 ] && args=(--gpus 1 --steps 20 --warmup 5)
    timeout -k 10 600 python -u bench.py "${args[@]}" > $O/bench.json 2> $O/bench.err &
    tick $! bench $O/bench.err
    rc=$?
    tail -5 $O/bench.err
    tail -c 3000 $O/bench.json
    exit $rc ;;
legs)
    legs=$1
    shift
    timeout -k 10 600 python -u bench.py --no-headline --legs "$legs" --no-cpu-baseline "$@" > $O/legs.json 2> $O/legs.err &
    tick $! legs $O/legs.err
    rc=$?
    tail -20 $O/legs.err
    tail -c 4000 $O/legs.json
    exit $rc ;;
ipc8)
    bash tools/r5h.sh ;;
c4half2)
    n=${1:-16777216}
    GG_BENCH_WATCHDOG=${WD:-120} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29813 bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 \
        --nodes 65536 --legs C4 --c4-nodes "$n" --leg-steps 2 --no-cpu-baseline $C4HALF2_ARGS \
        > $O/c4half2.json 2> $O/c4half2.err &
    tick $! c4half2 $O/c4half2.err
    rc=$?
    tail -20 $O/c4half2.err
    python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/box/c4half2.json") if l.startswith("{")][-1])
l = d["legs"]["C4"]
print({k: l.get(k) for k in ("check", "lsat", "exchange", "ms_per_step", "hbm_bytes_per_gpu", "error", "exchange_note")})
print(l.get("checks"))
PY
    exit $rc ;;
memset)
    timeout -k 10 120 tools/graph_memset_repro 300 memset > $O/memset_1p.txt 2>&1
    a=$?
    timeout -k 10 120 tools/graph_memset_repro 300 kernel > $O/kernel_1p.txt 2>&1
    b=$?
    [ $a -le 1 ] && [ $b -le 1 ] || { cat $O/*_1p.txt; exit 1; }
    (timeout -k 10 180 tools/graph_memset_repro 300 memset > $O/memset_2p_a.txt 2>&1 &
     timeout -k 10 180 tools/graph_memset_repro 300 memset > $O/memset_2p_b.txt 2>&1 &
     wait)
    (timeout -k 10 180 tools/graph_memset_repro 300 kernel > $O/kernel_2p_a.txt 2>&1 &
     timeout -k 10 180 tools/graph_memset_repro 300 kernel > $O/kernel_2p_b.txt 2>&1 &
     wait)
    tail -n 3 $O/memset_*.txt $O/kernel_*.txt ;;
ipcrepro)
    # each scenario a fresh pair of processes; a step stuck in the runtime is caught by the
    # repro's own watchdog (exit 1) or a failed call (exit 2); a time limit ends the chain
    for sc in ${@:-2 4 3 1}; do
        cached=; [ "${sc%c}" != "$sc" ] && cached=1  # N c: the same with hipMalloc windows
        REPRO_CACHED=$cached timeout -k 10 90 tools/ipc_reopen_repro ${sc%c} > $O/ipc_reopen_$sc.txt 2>&1 \
            || { rc=$?; [ $rc -ge 124 ] && { cat $O/ipc_reopen_$sc.txt; exit $rc; }; }
        echo "== scenario $sc"; cat $O/ipc_reopen_$sc.txt
    done ;;
pmc)
    O=gpurun_out/box/pmc bash tools/pmc_passes.sh "$1" ;;
*)
    echo "unknown task $task"; exit 2 ;;
esac
