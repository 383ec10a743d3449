#!/usr/bin/env python3
"""Debug: bench.py's headline sequence on a 2-part C2 job (gloo ranks, one GPU),
piece by piece; env DBG_SKIP = comma list of pieces to leave out
(coll: the validation's agree/reduce, qcoll: the per-round allreduce of the
quiescence loop, mem: mem_get_info, free0: the mem_get_info before the engine)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))
import bench  # noqa: E402

skip = set(filter(None, os.environ.get("DBG_SKIP", "").split(",")))
job = bench.Job("gloo", 2)
from ggamd import topology as T  # noqa: E402
from ggamd.dist import ShardedRunner  # noqa: E402
from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402

rank = job.rank
if "free0" not in skip:
    job.free_bytes()
V, K, seed = (1 << 20) * 2, 1024, BASE_SEED + 2
topo = T.tree(V, 4)
eng = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=rank, world=2)
eng.topology(topo)
rn = ShardedRunner(eng, job.device, transport="ipc")
arr = injection_arrays(uniform_injections(V, K, seed))
if os.environ.get("DBG_GOLD"):
    gold = bench.gold_c2(V, K)
if os.environ.get("DBG_FN"):  # the validation inside a function, its arrays dropped on return
    def _val():
        a = injection_arrays(uniform_injections(V, K, seed))
        eng.reset()
        inject(eng, a)
        return rn.step(23, reduce=False)
    val = _val()
else:
    eng.reset()
    inject(eng, arr)
    val = rn.step(23, reduce=False)
if "coll" not in skip:
    job.agree(True)
    bench.reduce_counts(val, job, COUNT_FIELDS)
inj_arr = injection_arrays(uniform_injections(V, K, seed))
eng.reset()
inject(eng, inj_arr)
for r in range(23):
    st = rn.step(1, reduce=False)[0]
    if "qcoll" not in skip:
        job.allreduce([st["new_bits"]])
if "mem" not in skip:
    job.free_bytes()
eng.reset()
inject(eng, inj_arr)
w = rn.step(23, reduce=False)
bad = [(a["round"], f) for a, b in zip(w, val) for f in COUNT_FIELDS if a[f] != b[f]]
print(f"rank {rank} skip {sorted(skip)}: warmup {'OK' if not bad else bad[:3]} new_bits {w[0]['new_bits']}", flush=True)
eng.close()
job.close()
