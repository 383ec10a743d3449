#!/bin/bash
# C2 rounds 20-21 (timer rounds): round_prep grid sizes, A/B-knob build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gossip-glomers-distributed-systems_amd
for B in 4096 1024 2048 16384 4096; do
  echo "== GG_SYNC_PREP_BLOCKS=$B"
  GG_HIP_LIB=$P/libgossip_hip_ab.so GG_SYNC_PREP_BLOCKS=$B ROUNDS=22 timeout -k 10 120 python3 -u tools/rounds.py C2 | grep -E "^r (19|20|21)|total"
done
