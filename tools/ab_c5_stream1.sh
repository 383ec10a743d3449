mkdir -p gpurun_out/ab5
for v in base w6r8 w8r8 w4r12 w6r12 base; do
  GG_HIP_LIB=ab_libs/libgossip_hip_$v.so timeout -k 10 200 python -u tools/leg_rounds.py C5 > gpurun_out/ab5/$v.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab5/$v.txt; exit 1; }
  echo "$v: $(grep -E '^r 1[2-5]' gpurun_out/ab5/$v.txt | awk '{print $2}' | tr '\n' ' ') $(tail -1 gpurun_out/ab5/$v.txt)"
done
