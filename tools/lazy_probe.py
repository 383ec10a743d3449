#!/usr/bin/env python3
"""Single-step runs of the lazy-sync-buffer scenarios against O2 under env
variants (GG_SYNC_EAGER, GG_SYNC_ALLOC_ROUND, GG_SYNC_DIGEST, ...): prints the
first differing rounds per variant. Usage: tools/lazy_probe.py [scenario index...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = [{}, {"GG_SYNC_EAGER": "1"}, {"GG_SYNC_ALLOC_ROUND": "0"}, {"GG_SYNC_ALLOC_ROUND": "3"},
            {"GG_SYNC_ALLOC_ROUND": "5"}, {"GG_SYNC_DIGEST": "0"}, {"GG_SYNC_DIGEST": "0", "GG_SYNC_EAGER": "1"}]

CHILD = r'''
import sys, os
sys.path[:0] = [os.path.join(sys.argv[1], "tests"), os.path.join(sys.argv[1], "gossip-glomers-distributed-systems_amd"), sys.argv[1]]
from test_gpu_sync_alloc import _scenarios
from helpers import make_engine, diff_stats
from ggamd.engine import HIP_LIB
cpu = os.path.join(sys.argv[1], "oracle", "_build", "libgossip_cpu.so")
sc = _scenarios()[int(sys.argv[2])]
ref = make_engine(cpu, sc).step(sc.rounds)
for mode in ("whole", "single"):
    e = make_engine(HIP_LIB, sc, device=0)
    st = e.step(sc.rounds) if mode == "whole" else [e.step(1)[0] for _ in range(sc.rounds)]
    d = diff_stats(ref, st)
    print(f"  {mode:6s}: {'OK' if not d else d[:3]}", flush=True)
    e.close()
'''

for k in (sys.argv[1:] or ["1", "3"]):
    for v in VARIANTS:
        env = dict(os.environ, GG_SYNC_TILES="0", **v)
        print(f"scenario {k} {v}", flush=True)
        r = subprocess.run([sys.executable, "-c", CHILD, REPO, k], env=env, timeout=120)
        if r.returncode:
            print("  child failed", r.returncode, flush=True)
            sys.exit(1)
