#!/usr/bin/env python3
"""How much of a C4-shaped episode's gather work a saturation skip could drop.

R-MAT (C4's parameters) at 2^N nodes, W = 4096 lanes injected in round 0,
stepped one round at a time; after each round every node's set size is read
back. A node is *saturated after r* when its set already holds every lane it
will ever hold (its size equals the size after quiescence: the lanes whose
source lies in its component). Round r+1's in-edge work on saturated nodes
(in-degree weighted, hubs and the rest apart) is what an exact per-node skip
— a digest compared against the lanes reachable from the node's component —
could drop; the plain digest (set size == every injected lane) drops only the
nodes reached by every lane, i.e. none once any source is isolated.

usage: python tools/sat_potential.py [log2 nodes = 22] [hub degree = 512]
"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..",
                                               "gossip-glomers-distributed-systems_amd"))


def main():
    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, uniform_injections
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    hub = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    V, K, seed = 1 << lg, 4096, BASE_SEED + 4
    e = Engine(V, K, seed=seed, enable_sync=False, device=0)
    e.generate(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    topo = e.export_topology()
    deg = np.diff(topo.row_ptr).astype(np.int64)
    del topo
    inject(e, uniform_injections(V, K, seed))
    sizes = []
    t0 = time.time()
    for r in range(40):
        st = e.step(1)[0]
        sizes.append(np.bitwise_count(e.read_bits()).sum(axis=1, dtype=np.int64))
        print(f"round {r}: {st['new_bits']} new bits ({time.time() - t0:.0f} s)", flush=True)
        if st["new_bits"] == 0 and r > 0:
            break
    e.close()
    final = sizes[-1]
    is_hub = deg > hub
    tot_h, tot_o = deg[is_hub].sum(), deg[~is_hub].sum()
    print(f"V = {V}, in-edges {deg.sum()}, hubs (in-degree > {hub}) {is_hub.sum()} holding {tot_h} in-edges; "
          f"nodes reached by every lane: {(final == K).sum()}")
    print("round | in-edge work of nodes saturated after the round before: hubs, others, all")
    for r in range(1, len(sizes)):
        sat = sizes[r - 1] == final
        h = deg[sat & is_hub].sum() / max(1, tot_h)
        o = deg[sat & ~is_hub].sum() / max(1, tot_o)
        a = deg[sat].sum() / max(1, deg.sum())
        print(f"{r:5d} | {h:6.3f} {o:6.3f} {a:6.3f}")


if __name__ == "__main__":
    main()
