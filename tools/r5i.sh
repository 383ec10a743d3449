#!/bin/bash
# hipIpcOpenMemHandle of a second, larger window after a first one was opened,
# closed and freed (the bench's headline -> leg sequence), two processes, one GPU
O=gpurun_out/r5i; mkdir -p $O
for sizes in "0.01 3.4" "0.01 1.0 3.4 6.8"; do
  n=$(echo $sizes | wc -w)
  echo "== uncached windows: $sizes GiB"
  coproc EXP { timeout -k 5 100 tools/ipc_map_bench exports 1 $sizes; }
  coproc IMP { timeout -k 5 100 tools/ipc_map_bench imports $n 2>&1; }
  for i in $(seq $n); do
    read -r -t 60 h <&"${EXP[0]}" || { echo "no handle"; break; }
    echo "$h" >&"${IMP[1]}"
    read -r -t 60 line <&"${IMP[0]}" && echo "$line" || { echo "import $i: no answer in 60 s"; break; }
    read -r -t 60 nx <&"${IMP[0]}"
    echo next >&"${EXP[1]}"
  done
  kill $EXP_PID $IMP_PID 2>/dev/null; wait
done
