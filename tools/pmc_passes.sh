#!/bin/bash
# PMC passes of this build: the request ceilings (gather_bench --calibrate: reads and writes), then C2 / C3 / C5 / C4
# (FETCH_SIZE, WRITE_SIZE, memory-side requests: one counter group per run)
# usage: tools/pmc_passes.sh "CAL C2 C3 C5" | "C4"   (O=<out dir>, default gpurun_out/pmc_passes)
# -> $O/request_ceiling.json, $O/traffic_<cfg>.json: copy them to profiles/ (bench.py reads them there)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=${O:-gpurun_out/pmc_passes}; mkdir -p $O
tick() { while kill -0 $1 2>/dev/null; do sleep 30; echo "  $2 $(date +%T)"; done; wait $1; }
pass() {  # name counters... -- command
  local name=$1; shift
  local cs=(); while [ "$1" != "--" ]; do cs+=("$1"); shift; done; shift
  timeout -s KILL ${PASS_TIMEOUT:-300} rocprofv3 --pmc "${cs[@]}" --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1 &
  tick $! $name || { echo "pass $name failed"; tail -20 $O/$name.log; exit 1; }
  rm -f $O/$name/*.db
}
for cfg in $1; do
  case $cfg in
    CAL)
      timeout -k 10 120 tools/gather_bench --calibrate > $O/gather_cal.txt 2>&1 || { cat $O/gather_cal.txt; exit 1; }
      cat $O/gather_cal.txt
      pass cal_req TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -- tools/gather_bench --calibrate
      python3 tools/request_ceiling.py $O/gather_cal.txt $(ls $O/cal_req/*counter_collection.csv) $O/request_ceiling.json ;;
    C2) cmd=(python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none) ;;
    C3) cmd=(python3 bench.py --no-headline --legs C3 --leg-steps 2 --no-cpu-baseline) ;;
    C4) cmd=(python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --fresh-sets 0 --legs none) ;;
    C5) cmd=(python3 bench.py --no-headline --legs C5 --leg-steps 1 --no-cpu-baseline) ;;
  esac
  [ $cfg = CAL ] && continue
  pass ${cfg}_fetch FETCH_SIZE -- "${cmd[@]}"
  pass ${cfg}_write WRITE_SIZE -- "${cmd[@]}"
  pass ${cfg}_req TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -- "${cmd[@]}"
  out=$O/traffic_$cfg.json
  python3 tools/traffic.py $(ls $O/${cfg}_fetch/*counter_collection.csv) $(ls $O/${cfg}_write/*counter_collection.csv) \
    "rocprofv3 --pmc passes over: ${cmd[*]:1} (tools/pmc_passes.sh)" $out $cfg --req $(ls $O/${cfg}_req/*counter_collection.csv) > $O/traffic_$cfg.txt; head -12 $O/traffic_$cfg.txt
done
