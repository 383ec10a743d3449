#!/usr/bin/env python3
"""Per-round device times of one vertex part of C2 (rank 0 of world 2 at
2 x 2^20 nodes, driven through gg_dist_round_begin / _end with an all-zero
receive buffer: the ghosts stay idle) beside the single engine of 2^20 nodes:
what a sharded round adds on the device (prep, stream, exchange kernels).
Usage: tools/dist_rounds.py [rounds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

import torch  # noqa: E402

from ggamd import topology as T  # noqa: E402
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    K, seed = 1024, BASE_SEED + 2
    out = {}
    for name, V, world in (("single", 1 << 20, 1), ("part0", 2 << 20, 2)):
        e = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=0, world=world)
        e.topology(T.tree(V, 4))
        inj = injection_arrays(uniform_injections(V, K, seed))
        for ep in range(3):
            e.reset()
            inject(e, inj)
            if world == 1:
                st = e.step(R)
            else:
                for _ in range(R):
                    e.dist_round_begin()
                    e.dist_round_end(wait=False)
                st = e.dist_flush()
        torch.cuda.synchronize()
        out[name] = st
        e.close()
    print(f"{'r':>3} {'single ms p/s':>16} {'part0 ms p/s':>18}")
    for k in range(R):
        a, b = out["single"][k], out["part0"][k]
        print(f"{k:3d} {a['kernel_ms']:.4f} {a['prep_ms']:.4f}/{a['stream_ms']:.4f}   "
              f"{b['kernel_ms']:.4f} {b['prep_ms']:.4f}/{b['stream_ms']:.4f}")
    for n in out:
        print(n, "total kernel ms", round(sum(s["kernel_ms"] for s in out[n]), 3))


if __name__ == "__main__":
    main()
