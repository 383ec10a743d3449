#!/usr/bin/env python3
"""How much of a vertex-sharded round could run before the exchange lands
(interior-first ordering)? For the device partition's node ranges (generate_sharded:
[V*p/P, V*(p+1)/P) cut at multiples of 64), the share of nodes with no remote
neighbour and the share of the in-edge work they carry, on the C4 generator
(R-MAT) and the C5 generator (grid + long links). CPU only (host builders)."""
import sys
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))
import numpy as np  # noqa: E402

from ggamd import topology as T  # noqa: E402
from ggamd.workload import BASE_SEED  # noqa: E402


def interior(t, P):
    V = t.n_nodes
    plo = [min(V, (V * p // P) // 64 * 64) for p in range(P)] + [V]
    owner = np.searchsorted(np.array(plo[1:]), np.arange(V), side="right")
    rows = np.repeat(np.arange(V), np.diff(t.row_ptr))
    cut = owner[rows] != owner[t.col]
    remote = np.zeros(V, bool)
    np.logical_or.at(remote, rows, cut)
    deg = np.diff(t.row_ptr)
    return float((~remote[deg > 0]).mean()), float(deg[~remote].sum() / deg.sum()), float(cut.mean())


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    for name, t in (("C4 R-MAT", T.rmat(1 << lg, 16, seed=BASE_SEED + 4)),
                    ("C5 grid+links", T.grid_links(1 << (lg // 2), seed=BASE_SEED + 5))):
        for P in (2, 4, 8):
            a, b, c = interior(t, P)
            print(f"{name} 2^{lg} P={P}: interior nodes {a:.3f} (of nodes with edges), "
                  f"interior in-edge work {b:.3f}, cut edges {c:.3f}")


if __name__ == "__main__":
    main()
