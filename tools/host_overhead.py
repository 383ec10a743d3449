#!/usr/bin/env python3
"""Host-side cost of one C2 bench episode (tools only): wall time of
eng.reset(), inject() and eng.step(R) around the device time of the step's
launch sequence (HIP events), median over episodes."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))
from ggamd import topology as T  # noqa: E402
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402

V, K, R = 1 << 20, 1024, 22
seed = BASE_SEED + 2
eng = Engine(V, K, seed=seed, enable_sync=True, device=0)
eng.topology(T.tree(V, 4))
inj = injection_arrays(uniform_injections(V, K, seed))
rows = []
for ep in range(40):
    t0 = time.perf_counter()
    eng.reset()
    t1 = time.perf_counter()
    inject(eng, inj)
    t2 = time.perf_counter()
    eng.step(R, raw=True)
    t3 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, t3 - t2, eng.step_device_ms() * 1e-3))
rows = rows[5:]
med = [statistics.median(r[i] for r in rows) * 1e6 for i in range(4)]
print(f"reset {med[0]:.1f} us, inject {med[1]:.1f} us, step wall {med[2]:.1f} us, step device (events) {med[3]:.1f} us, "
      f"episode wall {sum(med[:3]):.1f} us")
