#!/bin/bash
# expand_stream1 (C5) A/B over variant engine builds: per-round episode times (tools/leg_rounds.py)
mkdir -p gpurun_out/ab5
# variant libraries: build with -DGG_STREAM1_WAVES_PER_EU=N / -DGG_STREAM1_ROWS=N into ab_libs/libgossip_hip_<name>.so
for v in base w6r8 w8r8 w4r12 w6r12 base; do
  GG_HIP_LIB=ab_libs/libgossip_hip_$v.so timeout -k 10 200 python -u tools/leg_rounds.py C5 > gpurun_out/ab5/$v.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab5/$v.txt; exit 1; }
  echo "$v: $(grep -E '^r 1[2-5]' gpurun_out/ab5/$v.txt | awk '{print $2}' | tr '\n' ' ') $(tail -1 gpurun_out/ab5/$v.txt)"
done
