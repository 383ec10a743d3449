#!/usr/bin/env python3
"""Host cost of one sharded round on one GPU, without the collective: a world=2
engine (rank 0 of the C2 tree at 2 x 2^20 nodes) driven through
gg_dist_round_begin / gg_dist_round_end with an all-zero receive buffer (the
ghosts stay idle), plus the cost of the torch view / stream plumbing the
ShardedRunner adds. Prints host microseconds per round and the device time of
the same rounds (engine stream synchronised once at the end), i.e. whether a
round is host- or device-bound before RCCL is even involved.

Usage: tools/dist_host_overhead.py [episodes]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

import torch  # noqa: E402

from ggamd import topology as T  # noqa: E402
from ggamd.dist import _view  # noqa: E402
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402


def main():
    eps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    V, K = 2 << 20, 1024
    seed = BASE_SEED + 2
    topo = T.tree(V, 4)
    inj = injection_arrays(uniform_injections(V, K, seed))
    e = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=0, world=2)
    e.topology(topo)
    dev = torch.device("cuda", 0)
    R = 24
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    a2a_send = torch.zeros(4096, dtype=torch.uint8, device=dev)
    a2a_recv = torch.zeros(4096, dtype=torch.uint8, device=dev)
    for mode in ("engine", "engine+views", "engine+views+a2a(world=1)"):
        host_us, dev_ms = [], []
        for ep in range(eps + 1):
            e.reset()
            inject(e, inj)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(R):
                x = e.dist_round_begin()
                if mode != "engine":
                    send = _view(x.send, x.send_total, True, dev)
                    recv = _view(x.recv, x.recv_total, True, dev)
                    ext = torch.cuda.ExternalStream(x.stream, device=dev)
                    with torch.cuda.stream(ext):
                        recv.zero_()
                        if mode.endswith("a2a(world=1)"):
                            dist.all_to_all_single(a2a_recv, a2a_send, [4096], [4096])
                    del send
                e.dist_round_end(wait=False)
            t1 = time.perf_counter()
            st = e.dist_flush()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if ep:
                host_us.append((t1 - t0) / R * 1e6)
                dev_ms.append(sum(s["kernel_ms"] for s in st))
        print(f"{mode}: host {sum(host_us) / len(host_us):.1f} us/round enqueue, "
              f"device {sum(dev_ms) / len(dev_ms):.3f} ms/episode ({R} rounds, "
              f"{sum(dev_ms) / len(dev_ms) / R * 1e3:.1f} us/round), wall {(t2 - t0) * 1e3:.2f} ms/episode",
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
