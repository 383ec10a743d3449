#!/usr/bin/env python3
"""Per-round diagnostics of one episode: kernel time, active nodes, gathers."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import by_name, inject  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
kw = {}
if len(sys.argv) > 2:
    kw = {"V": int(sys.argv[2])} if name != "C5" else {"side": int(sys.argv[2])}
wl = by_name(name, **kw)
e = Engine(wl.topo.n_nodes, wl.n_lanes, seed=wl.seed, enable_sync=wl.enable_sync, device=0)
wl.apply(e)
rounds = int(os.environ.get("ROUNDS", "40"))
for rep in range(2):
    e.reset()
    inject(e, wl.injections)  # reset keeps topology and partition windows
    st = e.step(rounds)
tot = 0.0
print(f"{name}: V={wl.topo.n_nodes} E={wl.topo.nnz} W={wl.n_lanes}")
for s in st:
    tot += s["kernel_ms"]
    print(f'r{s["round"]:3d} ms={s["kernel_ms"]:.4f} p/e/s={s["prep_ms"]:.4f}/{s["expand_ms"]:.4f}/{s["stream_ms"]:.4f} '
          f'new={s["new_bits"]:>11d} active={s["work_rows"]:>9d} '
          f'gathers={s["work_gathers"]:>9d} fired={s["syncs_fired"]:>7d} sbytes={s["stream_bytes"]/1e6:.1f}MB ebytes={s["expand_bytes"]/1e6:.1f}MB')
print(f"total kernel ms {tot:.3f}")
