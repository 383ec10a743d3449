#!/usr/bin/env python3
"""Debug: the bench's sequence on a 2-part C2 job over the IPC exchange (gloo
ranks on one GPU): validation dist_step(R), R single-round steps, a synchronous
episode, then gg_dist_run_episodes; each rank compares every episode's local
counters with its synchronous episode's. Usage: torchrun --nproc-per-node 2 tools/dbg_episodes.py [variant]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gossip-glomers-distributed-systems_amd"))
import torch
import torch.distributed as dist

from ggamd import topology as T
from ggamd.dist import ShardedRunner
from ggamd.engine import COUNT_FIELDS, Engine
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

variant = sys.argv[1] if len(sys.argv) > 1 else "bench"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
V, K, seed = (1 << 20) * world, 1024, BASE_SEED + 2
eng = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=rank, world=world)
eng.topology(T.tree(V, 4))
rn = ShardedRunner(eng, torch.device("cuda", 0), transport="ipc")
arr = injection_arrays(uniform_injections(V, K, seed))
R = int(os.environ.get("DBG_R", "22"))


def ep_sync():
    eng.reset()
    inject(eng, arr)
    return rn.step(R, reduce=False)


def show(tag, a, b):
    d = [(s["round"], f, s[f], t[f]) for s, t in zip(a, b) for f in COUNT_FIELDS if s[f] != t[f]]
    print(f"rank {rank} {tag}: {'OK' if not d else d[:4]}", flush=True)


if variant.startswith("exact"):  # bench.py's headline sequence (exactNN: NN validation rounds)
    nv = int(variant[5:] or R)
    if os.environ.get("DBG_MEMINFO"):
        torch.cuda.mem_get_info(0)
    eng.reset()
    inject(eng, arr)
    v = rn.step(nv, reduce=False)  # validation
    if os.environ.get("DBG_SLEEP"):
        import time
        time.sleep(float(os.environ["DBG_SLEEP"]) * (1 + rank))
    if os.environ.get("DBG_COLL"):
        t = torch.zeros(300, dtype=torch.int64)
        dist.all_reduce(t)
        dist.barrier()
    eng.reset()
    inject(eng, arr)
    for _ in range(R):
        rn.step(1, reduce=False)
    ref = ep_sync()  # warmup - 1 = 1 episode
    show("validation vs warmup", v, ref[:nv])
    print(f"rank {rank} warmup new_bits {[x['new_bits'] for x in ref]}", flush=True)
    for k in range(2):
        dist.barrier()
        torch.cuda.synchronize()
        eng.reset()
        inject(eng, arr)
        eps = rn.run_episodes(R, 3)
        for j, ep in enumerate(eps):
            show(f"exact call {k} ep {j}", ep, ref)
    sys.exit(0)
if variant in ("bench", "noval"):
    if variant == "bench":
        v = ep_sync()
    eng.reset()
    inject(eng, arr)
    for _ in range(R):
        rn.step(1, reduce=False)
ref = ep_sync()
ref2 = ep_sync()
show("sync episode twice", ref2, ref)
eng.reset()
inject(eng, arr)
eps = rn.run_episodes(R, 3)
for k, ep in enumerate(eps):
    show(f"run_episodes ep {k}", ep, ref)
eng.reset()
inject(eng, arr)
eps = rn.run_episodes(R, 3)
for k, ep in enumerate(eps):
    show(f"second run_episodes ep {k}", ep, ref)
eng.close()
dist.destroy_process_group()
