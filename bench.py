#!/usr/bin/env python3
"""Benchmark: (node,msg) deliveries/s of the gossip-propagation engine.

One *step* = one full propagation episode: reset -> the clients' broadcasts ->
lockstep rounds until the round after the last delivery (quiescence, fixed
during warmup). `value` = all (node,msg) deliveries of the timed episodes on
all ranks / the max-over-ranks wall time.

Headline (--config C2, default; BASELINE.json configs[1]): a 4-ary tree
  (Maelstrom `tree4`) of 2^20 nodes per GPU, K = 1024 fresh messages broadcast
  by clients at seeded uniform nodes in round 0, sync timers on, no partitions.
  On N GPUs the tree has N * 2^20 nodes, vertex-range sharded (locality order)
  with one exchange of ghost payloads per round ("scaling": "weak").
--config C4 (configs[3]) as the headline: R-MAT (.57,.19,.19,.05), edge factor
  16, 10^8 nodes, K = 4096, strong scaling over N = L x P ranks (--parts P).

Legs (--legs, default C3,C4,C5 after a C2 headline; in the same JSON line
under "legs", every N including 1): BASELINE.json's other scale configs, each
built in HBM by the on-device generators and self-checked —
  C3  10^7-node random 8-regular, W = 1024, a seeded bisection in rounds
      [2, 12) healed by the sync timers (the partition-window and sync-heal
      kernels), N vertex parts;
  C4  10^8-node R-MAT, W = 4096, STRONG scaling: N vertex parts (two lane
      halves per GPU, one half's exchange under the other half's kernels);
      ms/step, deliveries/s, HBM per GPU, the dominant kernel's roofline;
  C5  2^30-node grid + one long link per node, W = 64, N vertex parts: HBM per
      GPU, rounds to full delivery, episode time.
  Checks: every timed episode equals the checking episode counter by counter;
  the checking episode's every round (all counters and the delivery hash)
  equals O2's run of the workload on the host-built graph
  (tests/golden/fullsize_*.json); P1 / KAT-3 / ACK (ggamd.checks; C4's
  components from the exported graph); N > 1: every round's global counters
  equal one unsharded engine on rank 0.

N > 1 exchange (--xchg auto): the device-driven IPC exchange when every rank
maps its peers and one whole C2 episode through it equals O2's run of the
same workload (tests/golden/bench_c2.json, every counter and the delivery
hash); else the engine's grouped RCCL send/recv. A failure later in the timed
region rebuilds every rank on the engine exchange and times that.

Usage: python bench.py [--config C2|C4] [--parts P] [--gpus N] [--steps K] [--warmup W]
                       [--legs C4,C5|none] [--leg-steps S] [--no-cpu-baseline]
For N > 1 launch under torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "gossip-glomers-distributed-systems_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

METRIC = "(node,msg) deliveries/sec at 1/2/4/8 GPUs; % of HBM roofline; msgs/op"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
M64 = (1 << 64) - 1

KERNELS = {"prep": "round_prep", "expand": "expand_round", "stream": "expand_stream"}
# the kernels one round launches exactly one of, per kind (the launch count of a kind)
MAIN_KERNELS = {"prep": ["round_prep"], "expand": ["expand_round", "expand_round_lean"],
                "stream": ["expand_stream", "expand_stream_db", "expand_stream_masked", "expand_stream1",
                           "expand_stream_sync", "expand_batched"]}
# the kernels stamping each kind: a kind's "launch" is one round, so its
# counter traffic per launch is the sum over these kernels' dispatches per round
KIND_KERNELS = {
    "prep": ["round_prep", "compact_round", "mark_injections", "hub_mark", "sync_records"],
    "expand": ["expand_round", "expand_round_lean"],
    "stream": ["expand_stream", "expand_stream_db", "expand_stream_db_mark", "expand_stream_masked", "expand_stream1",
               "expand_stream_sync", "hub_chunks", "hub_finish", "hub_sync_chunks", "hub_sync_finish", "hub_sync_push",
               "expand_batched"],
}
TRAFFIC_JSON = {"C2": os.path.join(REPO, "profiles", "traffic.json"),  # committed PMC passes per config
                "C3": os.path.join(REPO, "profiles", "traffic_C3.json"),
                "C4": os.path.join(REPO, "profiles", "traffic_C4.json"),
                "C5": os.path.join(REPO, "profiles", "traffic_C5.json")}
CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
GOLD_C2 = os.path.join(REPO, "tests", "golden", "bench_c2.json")
# the random-row request ceiling (rows of <= 128 B gathered by a per-node index,
# tools/gather_bench.hip): what a kernel whose rows are one line
# each can reach, where the byte roofline cannot be. profiles/request_ceiling.json
# holds it in the L2's memory-side requests (TCC_EA0_RDREQ per second of
# gather_bench under rocprofv3), the unit of line_frac, and the write side
# (TCC_EA0_WRREQ of its random-row stores and coalesced sweep); this constant
# is only the fallback without that file
ROW_CEILING_PER_S = 47e9
REQ_CEILING_JSON = os.path.join(REPO, "profiles", "request_ceiling.json")


def request_ceiling():
    """(read, write) memory-side request ceilings per second and their source: the
    random-row gathers, and the highest of the random-row stores and the coalesced
    store sweep (tools/gather_bench.hip --calibrate, profiles/request_ceiling.json).
    Write requests run far faster than reads (reset_state's sweep: ~86 G/s), so
    counting a kernel's writes against the read ceiling overstated line_frac."""
    try:
        d = json.load(open(REQ_CEILING_JSON))
        return float(d["requests_per_s"]), d.get("write_requests_per_s"), os.path.relpath(REQ_CEILING_JSON, REPO)
    except (OSError, ValueError, KeyError, TypeError):
        return ROW_CEILING_PER_S, None, "tools/gather_bench.hip rows/s (profiles/r2/gather_ceiling.txt)"


def pmc_traffic(kind: str, shape: dict):
    """HBM bytes and memory-side requests per EPISODE of a kernel kind from the
    committed rocprofv3 PMC passes (tools/traffic.py: FETCH_SIZE, WRITE_SIZE and
    TCC_EA0_RDREQ/WRREQ in separate passes over this same bench command,
    FETCH_SIZE doubled for gfx950): the sum over the kind's kernels of value x
    dispatches, over the profiled run's episodes — its reset_state dispatches
    less the one of the topology install (one per episode; a round can launch
    one or both of the marking-round kernels, so rounds are not countable from
    the dispatches). None unless the passes profiled a run of exactly this shape
    (config, nodes, lanes, world, parts, halves): another run's traffic is not
    this run's."""
    path = TRAFFIC_JSON.get(shape["config"])
    try:
        d = json.load(open(path))
    except (OSError, ValueError, TypeError):
        return None, None, None
    if d.get("shape") != shape:
        return None, (f"{os.path.relpath(path, REPO)} profiled {d.get('shape')}, not this run's {shape}: "
                      "no counter traffic for this shape"), None
    base = lambda name: name.split("(")[0].split("<")[0].split("::")[-1]  # noqa: E731
    ents = {}
    resets = sum(ent["dispatches"] for name, ent in d.get("kernels", {}).items() if base(name) == "reset_state")
    for name, ent in d.get("kernels", {}).items():
        b = base(name)
        if b in KIND_KERNELS[kind]:
            e = ents.setdefault(b, [0.0, 0, 0.0, 0.0, "rd_requests_per_dispatch" in ent])
            e[0] += ent["traffic_bytes_per_dispatch"] * ent["dispatches"]
            e[1] += ent["dispatches"]
            e[2] += ent.get("rd_requests_per_dispatch", 0.0) * ent["dispatches"]
            e[3] += ent.get("wr_requests_per_dispatch", 0.0) * ent["dispatches"]
    episodes = resets - 1
    if episodes < 1 or not ents:
        return None, None, None
    per_ep = sum(v[0] for v in ents.values()) / episodes
    reqs = ((sum(v[2] for v in ents.values()) / episodes, sum(v[3] for v in ents.values()) / episodes)
            if all(v[4] for v in ents.values()) else None)
    return per_ep, (f'{os.path.relpath(path, REPO)} ({d.get("source", "")}; kernels {sorted(ents)}; '
                    f'{episodes} episodes)'), reqs


def dense_bytes_per_round(V: int, E: int, nwp: int) -> int:
    """SURVEY.md §8d dense-pull bytes of one round: row_ptr 8(V+1) + col 4E +
    every sender row gathered E*w + read seen, write seen, write F 3*V*w."""
    w = 8 * nwp
    return 8 * (V + 1) + 4 * E + E * w + 3 * V * w


def next_pow2(x: int) -> int:
    p = 1
    while p < x:
        p <<= 1
    return p


def cpu_counts():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return os.cpu_count() or 1, aff or 1


def roofline(rounds_local: list[dict], nwp: int, n_own: int, E_own: int, shape: dict, episodes: int) -> dict:
    """The dominant kernel kind's roofline over a run's rounds (this rank):
    per-kind device times (first block start to last block end of each launch,
    stamped by the kernels) and the algorithmic bytes each launch had to move
    (counted by the kernels). line_frac: the time the kind's
    memory-side requests of an episode (TCC_EA0_RDREQ and WRREQ from the
    committed PMC pass of this shape) need at the measured ceilings — reads at
    the random-row gather rate, writes at the fastest store rate
    (tools/gather_bench.hip --calibrate) — over the kind's measured time per
    episode: random rows of <= 128 B are request-bound, so the byte roofline
    is out of reach for them. null without a request pass of this shape."""
    kinds = {}
    n = max(1, len(rounds_local))
    for kind, name in KERNELS.items():
        ms = sum(s[kind + "_ms"] for s in rounds_local)
        by = sum(s[kind + "_bytes"] for s in rounds_local)
        if kind == "stream":
            name = "expand_stream / expand_stream_db / expand_stream1"
        kinds[kind] = {"kernel": name, "launches": len(rounds_local), "total_ms": ms, "bytes": by,
                       "avg_launch_ms": ms / n, "GBps": by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0}
    dom = max(kinds, key=lambda k: kinds[k]["total_ms"])
    D = kinds[dom]
    traffic_ep, traffic_src, reqs_ep = pmc_traffic(dom, shape)
    R = n / max(1, episodes)  # rounds per episode: one launch of the kind per round
    traffic = traffic_ep / R if traffic_ep else None
    kind_s_ep = D["total_ms"] / max(1, episodes) * 1e-3  # the kind's device time per episode
    rd_ceil, wr_ceil, ceiling_src = request_ceiling()
    line_frac = line_src = line_rd = line_wr = None
    if reqs_ep and kind_s_ep > 0:
        rd, wr = reqs_ep
        # the time the kind's requests need at the ceilings, reads and writes each at its
        # own rate (no write ceiling measured: writes at the read rate, an upper bound);
        # line_frac = line_read_frac + line_write_frac
        line_rd = rd / rd_ceil / kind_s_ep
        line_wr = wr / (wr_ceil or rd_ceil) / kind_s_ep
        need = rd / rd_ceil + wr / (wr_ceil or rd_ceil)
        line_frac = need / kind_s_ep
        line_src = (f"PMC: {rd:.4g} read + {wr:.4g} write memory-side requests per episode of this kind "
                    f"({traffic_src}) need {need * 1e3:.4g} ms at {rd_ceil:.4g} read / "
                    f"{(wr_ceil or rd_ceil):.4g} write requests/s (the random-row gather and the fastest store "
                    f"ceilings, {ceiling_src}); the kind ran {kind_s_ep * 1e3:.4g} ms per episode")
    round_ms = sum(s["kernel_ms"] for s in rounds_local)
    round_bytes = sum(s["prep_bytes"] + s["expand_bytes"] + s["stream_bytes"] for s in rounds_local)
    return {
        "bound": "hbm",
        "kernel": D["kernel"],
        "kind": dom,
        "kind_kernels": "every kernel stamping this kind per round: " + ", ".join(KIND_KERNELS[dom]),
        "achieved": D["GBps"],
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": D["GBps"] / HBM_PEAK_GBS,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "algorithmic_bytes_per_launch": D["bytes"] / n,
        "avg_launch_ms": D["avg_launch_ms"],
        "launches": D["launches"],
        "dense_bytes_per_round": dense_bytes_per_round(n_own, E_own, nwp),
        "line_frac": line_frac,
        "line_read_frac": line_rd,
        "line_write_frac": line_wr,
        "line_source": line_src or "null: no request pass of this shape in profiles/",
        "read_requests_per_launch": reqs_ep[0] / R if reqs_ep else None,
        "write_requests_per_launch": reqs_ep[1] / R if reqs_ep else None,
        "timing": "per launch: device clock (s_memrealtime) from the first block start to the last "
                  "block end of that kernel, stamped by every block (no-op launches included, as in "
                  "rocprofv3's average)",
        "kernels": {k: dict(d) for k, d in kinds.items()},
        "round_GBps": round_bytes / (round_ms * 1e-3) / 1e9 if round_ms > 0 else 0.0,
    }


class Job:
    """This process's rank, device and collectives (one process per GPU)."""

    def __init__(self, backend: str, gpus: int):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != gpus and self.world == 1 and gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
        self.backend = backend
        if backend == "gloo":  # rehearsal: every rank on the one visible GPU
            self.local = 0
        torch.cuda.set_device(self.local)
        self.device = torch.device("cuda", self.local)
        if self.world > 1:
            to = datetime.timedelta(seconds=int(os.environ.get("GG_BENCH_PG_TIMEOUT", "600")))
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=self.device, timeout=to)
            else:
                dist.init_process_group(backend, timeout=to)

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.local])
            else:
                self.dist.barrier()
        self.torch.cuda.synchronize()

    def allreduce(self, vals, op: str = "sum") -> list[int]:
        if self.world == 1:
            return [int(v) for v in vals]
        t = self.torch.tensor([int(v) for v in vals], dtype=self.torch.int64,
                              device=self.device if self.backend == "nccl" else "cpu")
        R = self.dist.ReduceOp
        self.dist.all_reduce(t, op={"sum": R.SUM, "max": R.MAX, "min": R.MIN}[op])
        return t.cpu().tolist()

    def agree(self, ok: bool) -> bool:
        """True iff every rank is ok (every rank calls it at the same point)."""
        return self.allreduce([0 if ok else 1])[0] == 0

    def gather_i64(self, v: int) -> list[int]:
        """Every rank's value, by rank."""
        vals = [0] * self.world
        vals[self.rank] = int(v)
        return self.allreduce(vals)

    def free_bytes(self) -> int:
        return self.torch.cuda.mem_get_info(self.local)[0]

    def close(self):
        if self.world > 1:
            self.barrier()
            self.dist.destroy_process_group()


def reduce_counts(stats, job: Job, fields):
    """Sum one episode's per-round counters over the ranks (seen_hash mod 2^64)."""
    flat = []
    for s in stats:
        for f in fields:
            v = s[f] & M64
            flat.append(v - (1 << 64) if v >= (1 << 63) else v)
    tot = job.allreduce(flat)
    out, k = [], 0
    for s in stats:
        d = dict(s)
        for f in fields:
            d[f] = tot[k] & M64
            k += 1
        out.append(d)
    return out


def count_diffs(a_eps, b_eps, fields, label_a, label_b, limit=8):
    out = []
    for a, b in zip(a_eps, b_eps):
        for f in fields:
            if (a[f] & M64) != (b[f] & M64):
                out.append(f"round {b['round']} {f}: {label_a} {a[f] & M64} != {label_b} {b[f] & M64}")
                if len(out) >= limit:
                    return out
    if len(a_eps) != len(b_eps):
        out.append(f"{label_a} has {len(a_eps)} rounds, {label_b} {len(b_eps)}")
    return out


def gold_c2(nodes: int, lanes: int):
    """O2's per-round global counters of the C2 workload (tests/golden/bench_c2.json)."""
    if not os.path.exists(GOLD_C2):
        return None
    return next((g for g in json.load(open(GOLD_C2))["runs"].values() if g["nodes"] == nodes and g["lanes"] == lanes),
                None)


def gold_full(name: str, V: int, K: int, seed: int):
    """O2's full-size record of a leg's workload (tests/golden/make_fullsize_golden.py),
    or None when there is none of exactly this shape."""
    path = os.path.join(REPO, "tests", "golden", f"fullsize_{name.lower()}.json")
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    return g if (g["nodes"], g["lanes"], g["seed"]) == (V, K, seed) else None


def peer_info(job: Job) -> dict:
    """Where the ranks' GPUs are: distinct devices or not, and peer access from this one."""
    torch = job.torch
    if job.world == 1:
        return {}
    try:
        uuid = str(torch.cuda.get_device_properties(job.local).uuid)
    except Exception:  # noqa: BLE001
        uuid = f"local{job.local}"
    import hashlib
    h = int.from_bytes(hashlib.sha1(uuid.encode()).digest()[:7], "little")
    uuids = job.gather_i64(h)
    locals_ = job.gather_i64(job.local)
    acc = {}
    for q in range(job.world):
        if q != job.rank and locals_[q] != job.local:
            try:
                acc[q] = bool(torch.cuda.can_device_access_peer(job.local, locals_[q]))
            except Exception:  # noqa: BLE001
                acc[q] = None
    return {"distinct_devices": len(set(uuids)) == job.world, "devices": len(set(uuids)),
            "local_device_of_rank": locals_, "can_access_peer_from_rank0": acc if job.rank == 0 else None}


# ---------------------------------------------------------------------------
# headline (C2 weak scaling; or --config C4)

def headline(job: Job, args) -> tuple[dict | None, dict]:
    torch, world, rank, local = job.torch, job.world, job.rank, job.local
    from ggamd import topology as T
    from ggamd.engine import COUNT_FIELDS, Engine, stats_dict
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

    cfg = args.config
    free0 = job.free_bytes()
    t_setup = time.perf_counter()

    def setup(xchg):
        runner = None
        if cfg == "C2":
            V = (args.nodes or (1 << 20)) * world
            K = args.lanes or 1024
            seed = BASE_SEED + 2
            topo = T.tree(V, 4)
            gen = None
            E = int(topo.nnz)
            eng = Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world)
            eng.topology(topo)
            engs = [eng]
            if world > 1:
                from ggamd.dist import ShardedRunner
                runner = ShardedRunner(eng, job.device,
                                       transport=xchg if args.backend == "nccl" or xchg == "ipc" else "engine")
            parallelism = f"vertex-range x{world}" if world > 1 else "single GPU"
            scaling = "weak"
            workload = ("C2: tree4 of 2^20 nodes per GPU, 1024 messages broadcast in round 0 at seeded uniform "
                        "nodes, sync on, no partitions; one step = one episode to quiescence")
        else:
            V = args.nodes or 100_000_000
            K = args.lanes or 4096
            seed = BASE_SEED + 4
            topo = None
            gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
            P = args.parts
            if world % P:
                raise SystemExit(f"--parts {P} does not divide the world size {world}")
            L = world // P
            if args.halves == 2 and P > 1:
                from ggamd.dist import HalvesRunner
                g, q = divmod(rank, P)
                engs = [Engine(V, K, seed=seed, enable_sync=True, device=local, rank=(2 * g + h) * P + q,
                               world=2 * world, lane_groups=2 * L) for h in range(2)]
                E = engs[0].generate(**gen)
                engs[1].generate(**gen)
                eng = engs[0]
                runner = HalvesRunner(engs, job.device, transport=xchg)
            else:
                eng = Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world,
                             lane_groups=L)
                E = eng.generate(**gen)  # this rank's rows of the graph, built in its GPU's HBM (gossip_gen.h)
                engs = [eng]
                if P > 1:
                    from ggamd.dist import ShardedRunner
                    runner = ShardedRunner(eng, job.device,
                                           transport=xchg if args.backend == "nccl" or xchg == "ipc" else "engine")
            if world == 1:
                parallelism = "single GPU"
            elif P == 1:
                parallelism = f"message lanes x{world} (every GPU: whole graph, {K // world} lanes)"
            else:
                parallelism = (f"{L} lane groups x {P} vertex parts (each GPU: 1/{P} of the nodes + ghosts, "
                               f"{K // L} lanes" + (", as two engines of half the lanes each, exchange of one "
                                                    "overlapping the other's kernels)" if len(engs) == 2 else ")"))
            scaling = "strong"
            workload = (f"C4: R-MAT (.57,.19,.19,.05) edge factor 16, symmetrized, {V} nodes, {K} messages "
                        "broadcast in round 0 at seeded uniform nodes, sync on, no partitions; graph built "
                        "in HBM by the on-device generator; one step = one episode to quiescence")
        return dict(runner=runner, V=V, K=K, seed=seed, topo=topo, gen=gen, E=E, eng=eng, engs=engs,
                    parallelism=parallelism, scaling=scaling, workload=workload)

    def close_all(b):
        ipc_release(job, b["engs"] if b is not None else [])
        if b is not None:
            for e in b["engs"]:
                e.close()
        torch.cuda.synchronize()

    # N > 1 exchange: "auto" = the device-driven one (no host wait, captured rounds)
    # if every rank can map its peers and one whole episode through it equals O2
    # (every round's global counters, C2: tests/golden/bench_c2.json), else the
    # engine's RCCL send/recv, rebuilt from scratch on every rank
    xchg = args.xchg
    notes = []
    validation = None
    if xchg == "auto":
        xchg = "ipc" if (world > 1 and (cfg == "C2" or args.parts > 1)) else "engine"
    if args.xchg == "auto" and xchg == "ipc":
        built, validation = validate_ipc(job, args, setup)
        if built is None:
            xchg = "engine"
            notes.append(f"device-driven exchange failed its validation ({validation['result']}): "
                         "every rank rebuilt on --xchg engine")
            b = setup(xchg)
        else:
            b = built
    else:
        b = setup(xchg)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    inj = uniform_injections(b["V"], b["K"], b["seed"])
    inj_arr = injection_arrays(inj)  # converted once, outside the timed loop

    def quiescence(bb) -> int:
        for e in bb["engs"]:
            e.reset()
            inject(e, inj_arr)
        R = 0
        while True:
            rn = bb["runner"]
            st = rn.step(1, reduce=False)[0] if rn else bb["eng"].step(1)[0]
            nb = job.allreduce([st["new_bits"]])[0]
            R += 1
            if nb == 0 and R > 1:
                return R
            if R > 400:
                raise RuntimeError("no quiescence within 400 rounds")

    R = quiescence(b)  # warmup 0: the quiescence round R from per-round global counts
    torch.cuda.synchronize()
    # after the first episode: the engine's second set buffer (double-buffered
    # rounds) is allocated at its first step
    hbm_bytes = free0 - job.free_bytes()

    event_ms = []

    def episode(bb):
        for e in bb["engs"]:
            e.reset()
            inject(e, inj_arr)
        rn = bb["runner"]
        if rn is None:
            st = bb["eng"].step(R, raw=True)
            event_ms.append(bb["eng"].step_device_ms())
            return st
        return rn.step(R, reduce=False)

    for _ in range(max(0, args.warmup - 1)):
        episode(b)
    event_ms.clear()

    # one engine per rank (no vertex parts): the K episodes go back to back through
    # gg_run_episodes — each still a reset, the same client broadcasts and R rounds,
    # its counters read back and checked like the loop's — with one host wait, so
    # no host round trip idles the GPU between episodes; vertex parts over the
    # device-driven exchange: gg_dist_run_episodes, every rank alike. A failure there
    # (every rank agrees) rebuilds every rank on the engine exchange.
    def mode_of(bb):
        rn = bb["runner"]
        if rn is None:
            return "single"
        if getattr(rn, "can_run_episodes", False) and os.environ.get("GG_BENCH_DIST_EPISODES", "1") != "0":
            return "dist_pipe"
        return "sync"

    def timed(bb, mode, warm: bool):
        """(elapsed s, this rank's stats per episode); raises on an exchange failure."""
        eng, rn = bb["eng"], bb["runner"]
        if warm and mode != "sync" and args.warmup > 0:  # (its counter ring is allocated here)
            eng.reset()
            inject(eng, inj_arr)
            if mode == "dist_pipe":
                if os.environ.get("GG_BENCH_EPISODES_FAIL") == str(rank):  # test hook: the rebuild path
                    raise RuntimeError("GG_BENCH_EPISODES_FAIL")
                rn.run_episodes(R, args.steps)
            else:
                eng.run_episodes(R, args.steps, raw=True)
        job.barrier()
        t0 = time.perf_counter()
        if mode == "dist_pipe":
            eng.reset()
            inject(eng, inj_arr)
            local = rn.run_episodes(R, args.steps)
        elif mode == "single":
            eng.reset()
            inject(eng, inj_arr)
            arr = eng.run_episodes(R, args.steps, raw=True)
        else:
            local = [episode(bb) for _ in range(args.steps)]
        job.barrier()
        el = time.perf_counter() - t0
        if mode == "single":
            local = [[arr[k * R + i] for i in range(R)] for k in range(args.steps)]
        return el, local

    mode = mode_of(b)
    fail = None
    try:
        elapsed, local_stats = timed(b, mode, True)
    except Exception as exc:  # noqa: BLE001 — every rank agrees below
        fail = exc
        print(f"bench: rank {rank}: timed {mode} run failed ({exc!r})", file=sys.stderr)
    if not job.agree(fail is None):
        if mode == "single" or xchg == "engine":
            raise SystemExit(f"bench: the timed run failed on some rank ({fail!r})")
        # the device-driven exchange failed after its validation: every rank
        # closes its engines and rebuilds on the engine exchange (the
        # IPC runner cannot be reused — its error word stays set)
        close_all(b)
        xchg = "engine"
        notes.append(f"the timed {mode} run failed on some rank: every rank rebuilt on --xchg engine")
        b = setup(xchg)
        R2 = quiescence(b)
        if R2 != R:
            raise SystemExit(f"bench: the rebuilt job quiesces after {R2} rounds, not {R}")
        mode = mode_of(b)
        elapsed, local_stats = timed(b, mode, False)
    runner, eng, engs, V, K, seed = b["runner"], b["eng"], b["engs"], b["V"], b["K"], b["seed"]
    pipelined = mode in ("single", "dist_pipe")
    per_call_ms = None
    if pipelined:
        ev_pipe = [eng.step_device_ms()] * args.steps
        job.barrier()
        c0 = time.perf_counter()
        for _ in range(args.steps):
            episode(b)
        job.barrier()
        per_call_ms = (time.perf_counter() - c0) / args.steps * 1e3
        event_ms[:] = ev_pipe
        if world > 1:
            per_call_ms = float(job.allreduce([int(per_call_ms * 1e6)], "max")[0]) / 1e6

    # fresh episodes (N = 1): every step broadcasts a different seeded value set, as
    # in a workload whose clients keep sending new values: the injections and each
    # round's offsets into them are uploaded again; the captured launch sequence
    # names neither, so it replays as long as the same rounds inject the same number
    # of lanes (a set with another round pattern would capture once more)
    fresh = None
    if world == 1 and args.fresh_sets > 0:
        sets = [injection_arrays(uniform_injections(V, K, seed + 7919 * (i + 1))) for i in range(args.fresh_sets)]

        def q_rounds(arrs):
            eng.reset()
            inject(eng, arrs)
            n = 0
            while True:
                n += 1
                if eng.step(1)[0]["new_bits"] == 0 and n > 1:
                    return n
                if n > 400:
                    raise RuntimeError("no quiescence within 400 rounds")
        rounds_of = [q_rounds(a) for a in sets]
        n_fresh = max(args.fresh_sets, min(args.steps, 2 * args.fresh_sets))
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        fdl = 0
        for k in range(n_fresh):
            i = k % args.fresh_sets
            eng.reset()
            inject(eng, sets[i])
            st = eng.step(rounds_of[i], raw=True)
            fdl += sum(st[j].new_bits for j in range(rounds_of[i]))
        torch.cuda.synchronize()
        fdt = time.perf_counter() - f0
        fresh = {"sets": args.fresh_sets, "steps": n_fresh, "rounds_per_set": rounds_of,
                 "ms_per_step": fdt / n_fresh * 1e3, "deliveries_per_s": fdl / fdt,
                 "note": "each step uploads its own injection pairs and round offsets, then replays the "
                         "captured launch sequence, which reads both from device memory (the timed `value` "
                         "repeats one set, whose pairs stay resident)"}
    if mode == "single":
        local_stats = [[stats_dict(a[i]) for i in range(R)] for a in local_stats]
    if world > 1:
        elapsed = float(job.allreduce([int(elapsed * 1e9)], "max")[0]) / 1e9
        per_ep = [reduce_counts(s, job, COUNT_FIELDS) for s in local_stats]
    else:
        per_ep = local_stats
    deliveries = sum(s["new_bits"] for ep in per_ep for s in ep)
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in per_ep[-1])

    dinfo = None
    if runner is not None:
        dinfo = eng.dist_info()
        dinfo.update(peer_info(job))
        n_own = dinfo["owned"]
        if b["topo"] is not None:
            owned = eng.dist_owned().astype(np.int64)
            E_own = int((b["topo"].row_ptr[owned + 1] - b["topo"].row_ptr[owned]).sum())
        else:
            E_own = b["E"]  # generate() returned this rank's adjacency entries
    else:
        n_own, E_own = V, b["E"]
    nwp = next_pow2(K // 64 // (world // args.parts * len(engs) if cfg == "C4" else 1))
    rounds_local = [s for ep in local_stats for s in ep]
    shape = {"config": cfg, "nodes": V // world if cfg == "C2" else V, "lanes": K, "world": world,
             "parts": args.parts if cfg == "C4" else world, "halves": len(engs)}
    roof = roofline(rounds_local, nwp, n_own, E_own, shape, args.steps)
    roof["event_ms_per_step"] = (sum(event_ms) / len(event_ms)) if event_ms else None
    roof["per_call_ms_per_step"] = per_call_ms
    roof["stamp_ms_per_step"] = sum(s["kernel_ms"] for s in rounds_local) / args.steps
    roof["timing"] += ("; cross-check: HIP events on the engine stream around episodes 2..K-1 (episode 1 may recapture the batch) of the "
                       "pipelined run (event_ms_per_step)")
    xbytes = None
    if runner is not None:  # payload bytes this rank sent per round (mean over the timed rounds)
        xbytes = sum(s["sent_bytes"] for s in rounds_local) / len(rounds_local)

    # N > 1: the sharded job must reproduce one unsharded engine, round by round
    check = None
    if world > 1 and not args.no_check:
        bad = 0
        close_all(b)  # free every rank's shard before rank 0 builds the whole graph
        if rank == 0:
            ref = Engine(V, K, seed=seed, enable_sync=True, device=local)
            if b["gen"] is None:
                ref.topology(b["topo"])
            else:
                ref.generate(**b["gen"])
            inject(ref, inj_arr)
            want = ref.step(R)
            ref.close()
            diffs = count_diffs(per_ep[-1], want, COUNT_FIELDS, "sharded", "single")
            bad = len(diffs)
            if diffs:
                print("bench: sharded run differs from the single engine:", diffs, file=sys.stderr)
        bad = job.allreduce([bad])[0]
        check = "every round's global counters equal one unsharded engine" if bad == 0 else "FAILED"
        if bad:
            job.close()
            raise SystemExit(1)

    # every timed episode's global counters against the CPU oracle O2's run of the
    # same workload (tests/golden/bench_c2.json, made by make_bench_golden.py for
    # 2^20 x N nodes); a differing episode fails the run
    oracle_check = None
    if cfg == "C2" and K == 1024 and seed == BASE_SEED + 2:
        gold = gold_c2(V, K)
        if gold is not None:
            want = gold["rounds"]
            diffs = [d for k, ep in enumerate(per_ep) for d in
                     count_diffs(ep, want[:len(ep)], COUNT_FIELDS, f"episode {k}", "O2", 2)]
            if len(want) != R:
                diffs.append(f"quiescence round count {R} != O2 {len(want)}")
            if diffs:
                if rank == 0:
                    print("bench: counters differ from O2:", diffs[:8], file=sys.stderr)
                job.close()
                raise SystemExit(1)
            oracle_check = (f"all {len(per_ep)} timed episodes: every round's global counters and delivery hash "
                            f"equal O2's run of this workload (tests/golden/bench_c2.json, {V} nodes)")

    close_all(b)
    info = {"xchg": xchg, "validation": validation}
    if rank != 0:
        return None, info
    value = deliveries / elapsed
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "deliveries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": b["scaling"],
        "vs_baseline": None,
        "dtype": "u64",
        "data": f"synthetic (seeded {'tree4' if cfg == 'C2' else 'R-MAT'} topology, seeded client broadcasts)",
        "config": {
            "workload": b["workload"],
            "nodes": V, "edges": b["E"], "lanes": K, "rounds_per_step": R,
            "deliveries_per_step": deliveries // args.steps,
            "inter_node_msgs_per_step": msgs,
            "msgs_per_op": msgs / K,
            "parallelism": b["parallelism"],
            "exchange": (runner.transport if runner is not None else
                         ("none: lane groups never exchange; one all_reduce of the counters "
                          "after the timed episodes" if world > 1 else None)),
            "exchange_note": "; ".join(notes) or None,
            "exchange_validation": validation,
            "lane_groups": world // args.parts if cfg == "C4" else 1,
            "vertex_parts": args.parts if cfg == "C4" else world,
            "exchange_bytes_per_round_rank0": xbytes,
            "shard": dinfo,
            "hbm_bytes_rank0": hbm_bytes,
            "setup_s_rank0": setup_s,
            "check": check,
            "oracle_check": oracle_check,
            "timed_loop": ({"single": "gg_run_episodes", "dist_pipe": "gg_dist_run_episodes"}.get(mode, "") +
                           ": the K episodes (each a reset, the same client broadcasts and R rounds, its counters "
                           "read back) queued back to back, one host wait; roofline.per_call_ms_per_step times the "
                           "same episodes as K synchronous reset/broadcast/step calls" if pipelined else
                           "one synchronous reset/broadcast/step call sequence per episode"),
            "fresh_injections": fresh,
        },
        "roofline": roof,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline and os.path.exists(CPU_LIB):
        out["cpu_baseline"] = cpu_baseline(cfg, b["topo"], inj, V, K, seed, R)
    return out, info


def ipc_release(job: Job, engs) -> None:
    """Collective (every rank, at the same point): every engine of this rank leaves
    the device-driven exchange (gg_dist_ipc_close; a no-op without it), then a
    barrier — only then may any rank close an engine, whose window goes back to the
    process's pool for a later leg (gossip.h: windows are never freed while the
    process lives; freeing and reallocating them between legs is what stalled the
    8-rank rehearsal)."""
    for e in engs:
        try:
            e.dist_ipc_close()
        except Exception as exc:  # noqa: BLE001 — the barrier below still runs on every rank
            print(f"bench: rank {job.rank}: gg_dist_ipc_close failed ({exc!r})", file=sys.stderr, flush=True)
    job.barrier()


def validate_ipc(job: Job, args, setup):
    """Build the job on the device-driven exchange and run one whole episode
    through it (C2: every round — at least 4, so the consumed-flag waits and the
    reuse of each parity's buffers run — against O2's run of the same workload;
    --config C4: 6 rounds that must finish). Returns (the built job or None,
    a record of the validation). Every rank makes the same collective calls
    whatever fails. Test hook GG_BENCH_IPC_FAIL=rank[:round]: that rank stops
    exchanging after `round` rounds (default 0: at once) — its peers' waits
    run out (GG_EIO) — and reports a failure."""
    from ggamd.engine import COUNT_FIELDS
    from ggamd.workload import inject, injection_arrays, uniform_injections
    hook = os.environ.get("GG_BENCH_IPC_FAIL")
    f_rank, f_round = (None, None)
    if hook:
        p = hook.split(":")
        f_rank, f_round = int(p[0]), int(p[1]) if len(p) > 1 else 0
    ok, built, local, gold, err = True, None, None, None, None
    rounds = 6
    try:
        built = setup("ipc")
        if args.config == "C2":
            gold = gold_c2(built["V"], built["K"])
            if gold is not None:
                rounds = len(gold["rounds"])
        arr = injection_arrays(uniform_injections(built["V"], built["K"], built["seed"]))
        for e in built["engs"]:
            e.reset()
            inject(e, arr)
        n = rounds if job.rank != f_rank else min(rounds, f_round)
        local = built["runner"].step(n, reduce=False) if n else []
        if job.rank == f_rank:
            raise RuntimeError(f"GG_BENCH_IPC_FAIL: stopped after {n} rounds")
    except Exception as exc:  # noqa: BLE001 — every rank falls back together
        ok = False
        err = repr(exc)
        print(f"bench: rank {job.rank}: device-driven exchange failed its validation ({exc!r})", file=sys.stderr)
    rec = {"rounds": rounds, "against": "tests/golden/bench_c2.json (O2), every counter and the delivery hash"
           if gold is not None else "completion only (no golden run of this shape)"}
    if job.agree(ok):
        glob = reduce_counts(local, job, COUNT_FIELDS)
        diffs = count_diffs(glob, gold["rounds"], COUNT_FIELDS, "ipc", "O2") if gold is not None else []
        if not diffs:
            rec["result"] = "passed"
            return built, rec
        rec["result"] = "counters differ from O2: " + "; ".join(diffs[:4])
        if job.rank == 0:
            print(f"bench: device-driven validation episode differs from O2: {diffs}", file=sys.stderr)
    else:
        rec["result"] = f"failed on some rank (rank {job.rank}: {err})" if err else "failed on some rank"
    ipc_release(job, built["engs"] if built is not None else [])
    if built is not None:
        for e in built["engs"]:
            e.close()
    job.torch.cuda.synchronize()
    return None, rec


# ---------------------------------------------------------------------------
# legs: C4 (10^8 R-MAT, W = 4096, strong scaling) and C5 (2^30 grid + links, W = 64)

def run_leg(job: Job, args, name: str, xchg_pref: str) -> dict:
    t0 = time.perf_counter()
    try:
        rec = leg(job, args, name, xchg_pref)
    except LegAbort as exc:
        rec = {"config": name, "error": str(exc)}
    rec["leg_s"] = time.perf_counter() - t0
    return rec


class LegAbort(RuntimeError):
    pass


def leg(job: Job, args, name: str, xchg_pref: str) -> dict:
    """One leg; every phase ends in an agreement (all ranks ok, or LegAbort on
    every rank), so no rank waits in a collective another rank skipped."""
    torch, world, rank, local = job.torch, job.world, job.rank, job.local
    from ggamd.checks import components, episode_failures, expected_from_components
    from ggamd.engine import COUNT_FIELDS, Engine, stats_dict
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

    windows = []  # seeded partition windows (a, b, epoch seed): kept across resets (gossip.h gg_reset)
    if name == "C4":
        V = args.c4_nodes or 100_000_000
        K = 4096
        seed = BASE_SEED + 4
        gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
        workload = (f"C4: R-MAT (.57,.19,.19,.05) edge factor 16, symmetrized, {V} nodes, {K} messages broadcast "
                    "in round 0 at seeded uniform nodes, sync on, no partitions; graph built in HBM by the "
                    "on-device generator; strong scaling (the same graph at every N)")
    elif name == "C3":
        V = args.c3_nodes or 10_000_000
        K = 1024
        seed = BASE_SEED + 3
        gen = dict(kind="random_regular", n=V, k=8, seed=seed)
        windows = [(2, 12, seed ^ 0x5EED)]
        workload = (f"C3: random 8-regular graph, {V} nodes, {K} messages broadcast in round 0 at seeded uniform "
                    "nodes; a seeded bisection of the nodes drops every message across it in rounds [2, 12) "
                    "(Maelstrom --nemesis partition), the sync timers (rounds >= 20) heal it; one step = one "
                    "episode until every node holds every value and a round delivers nothing; graph built in "
                    "HBM by the on-device generator; strong scaling (the same graph at every N)")
    else:
        side = args.c5_side or 32768
        V = side * side
        K = 64
        seed = BASE_SEED + 5
        gen = dict(kind="grid_links", n=side, seed=seed)
        workload = (f"C5: {side}x{side} 4-neighbour grid + one seeded long-range link per node, symmetrized, "
                    f"{V} nodes, {K} messages broadcast in round 0 at seeded uniform nodes, sync on, no "
                    "partitions; graph built in HBM by the on-device generator (each rank its own part)")
    P = args.leg_parts or world
    if world % P:
        raise LegAbort(f"--leg-parts {P} does not divide the world size {world}")
    L = world // P
    halves = 2 if (name == "C4" and P > 1 and K // 64 // L >= 2 and args.leg_halves != 1) else 1
    inj = uniform_injections(V, K, seed)
    inj_arr = injection_arrays(inj)
    log = (lambda *a: print(f"bench[{name}]:", *a, file=sys.stderr, flush=True)) if rank == 0 else (lambda *a: None)

    def phase(fn, what):
        ok, res, err = True, None, None
        try:
            res = fn()
        except Exception as exc:  # noqa: BLE001
            ok, err = False, exc
            print(f"bench[{name}]: rank {rank}: {what} failed ({exc!r})", file=sys.stderr, flush=True)
        if not job.agree(ok):
            raise LegAbort(f"{what} failed on some rank" + (f" (rank {rank}: {err!r})" if err else ""))
        return res

    free0 = job.free_bytes()
    tb = time.perf_counter()
    engs = []

    def build_engines():
        if halves == 2:
            g, q = divmod(rank, P)
            for h in range(2):
                engs.append(Engine(V, K, seed=seed, enable_sync=True, device=local, rank=(2 * g + h) * P + q,
                                   world=2 * world, lane_groups=2 * L))
        else:
            engs.append(Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world,
                               lane_groups=L))
        E = 0
        for e in engs:
            E = e.generate(**gen)  # this rank's rows (gossip_gen.h); halves: the same rows twice
            for a, b, ep in windows:
                e.partition_seeded(a, b, ep)
        return E

    def close_engs():
        ipc_release(job, engs)
        for e in engs:
            e.close()
        engs.clear()
        torch.cuda.synchronize()

    def build_runner(xchg):
        if P == 1 and L == 1:
            return None
        if halves == 2:
            from ggamd.dist import HalvesRunner
            return HalvesRunner(engs, job.device, transport=xchg)
        from ggamd.dist import ShardedRunner
        return ShardedRunner(engs[0], job.device,
                             transport=xchg if (args.backend == "nccl" or xchg == "ipc") else "engine")

    try:
        E_local = phase(build_engines, "engine build")
        xchg = xchg_pref if P > 1 else "none"
        note = None
        try:
            runner = phase(lambda: build_runner(xchg), f"exchange setup ({xchg})")
        except LegAbort as exc:
            if xchg != "ipc":
                raise
            # a window mapping failed or ran out its bound (GG_IPC_OPEN_TIMEOUT_S) on some
            # rank: every rank rebuilds its engines on the engine exchange
            close_engs()
            E_local = phase(build_engines, "engine rebuild")
            xchg = "engine"
            note = f"device-driven exchange setup failed ({exc}): rebuilt on the engine exchange"
            runner = phase(lambda: build_runner(xchg), "exchange setup (engine)")
        setup_s = time.perf_counter() - tb
        log(f"built in {setup_s:.1f} s: {len(engs)} engine(s) per GPU, P={P} L={L}, exchange {xchg}")
        eng = engs[0]

        def reset_all():
            for e in engs:
                e.reset()
                inject(e, inj_arr)

        # checking episode: one round at a time to quiescence (global counters)
        def check_round():
            if runner is None:
                return eng.step(1)[0]
            return runner.step(1, reduce=False)[0]

        reset_all()
        check = []
        delivered = 0
        while True:
            ok, st = True, None
            try:
                st = check_round()
            except Exception as exc:  # noqa: BLE001
                ok = False
                print(f"bench[{name}]: rank {rank}: round {len(check)} failed ({exc!r})", file=sys.stderr)
            vals = [0 if ok else 1] + ([(st[f] & M64) - (1 << 64) if (st[f] & M64) >= (1 << 63) else st[f]
                                        for f in COUNT_FIELDS] if ok else [0] * len(COUNT_FIELDS))
            tot = job.allreduce(vals)
            if tot[0]:
                raise LegAbort(f"checking episode: round {len(check)} failed on some rank")
            g = dict(st)
            for j, f in enumerate(COUNT_FIELDS):
                g[f] = tot[1 + j] & M64
            check.append(g)
            delivered += g["new_bits"]
            if len(check) % 5 == 0:
                log(f"checking episode: round {len(check) - 1}, {g['new_bits']} deliveries")
            # quiescence; a healed partition (C3): only after every node holds every value
            if (g["new_bits"] == 0 and len(check) > 1 and (not windows or delivered == V * K)) or len(check) >= 120:
                break
        R = len(check)
        if check[-1]["new_bits"]:
            raise LegAbort(f"no quiescence within {R} rounds")
        hbm = job.gather_i64(free0 - job.free_bytes())
        log(f"checking episode: {R} rounds, {sum(s['new_bits'] for s in check)} deliveries")

        # timed episodes
        event_ms = None

        def timed():
            nonlocal event_ms
            job.barrier()
            t0 = time.perf_counter()
            if runner is None:
                reset_all()
                arr = eng.run_episodes(R, args.leg_steps, raw=True)
                eps = [[stats_dict(arr[k * R + i]) for i in range(R)] for k in range(args.leg_steps)]
                event_ms = eng.step_device_ms()
            elif getattr(runner, "can_run_episodes", False):
                reset_all()
                eps = runner.run_episodes(R, args.leg_steps)
            else:
                eps = []
                for _ in range(args.leg_steps):
                    reset_all()
                    eps.append(runner.step(R, reduce=False))
            job.barrier()
            return time.perf_counter() - t0, eps

        res = None
        try:
            res = timed()
        except Exception as exc:  # noqa: BLE001
            print(f"bench[{name}]: rank {rank}: timed episodes failed ({exc!r})", file=sys.stderr, flush=True)
        if not job.agree(res is not None):
            if xchg != "ipc":
                raise LegAbort("timed episodes failed on some rank")
            # the device-driven exchange failed: rebuild every rank on the engine exchange
            close_engs()
            phase(build_engines, "engine rebuild")
            xchg = "engine"
            runner = phase(lambda: build_runner(xchg), "exchange setup (engine)")
            eng = engs[0]
            note = "the device-driven exchange failed in the timed episodes: rebuilt on the engine exchange"
            res = phase(timed, "timed episodes (engine exchange)")
        elapsed, eps_local = res
        elapsed = float(job.allreduce([int(elapsed * 1e9)], "max")[0]) / 1e9
        eps = [reduce_counts(ep, job, COUNT_FIELDS) for ep in eps_local] if world > 1 else eps_local
        deliveries = sum(s["new_bits"] for ep in eps for s in ep)
        fails = []
        for k, ep in enumerate(eps):
            d = count_diffs(ep, check, COUNT_FIELDS, f"timed episode {k}", "checking episode", 3)
            fails += d
        rounds_local = [s for ep in eps_local for s in ep]
        # the lean saturation digest on each rank (gossip.h GG_PATH_LSAT / _COMP bits)
        lpath = 0
        for s in rounds_local:
            lpath |= int(s.get("path", 0))
        lsat = [("off", "universe", "component targets")[m]
                for m in job.gather_i64(2 if lpath & 512 else (1 if lpath & 256 else 0))]
        sent = sum(s["sent_bytes"] for s in rounds_local) / max(1, len(rounds_local))
        sent_max = max((s["sent_bytes"] for s in rounds_local), default=0)
        dinfo = eng.dist_info() if world > 1 else None
        n_own = dinfo["owned"] if dinfo else V
        nwp = next_pow2(K // 64 // (L * halves))
        shape = {"config": name, "nodes": V, "lanes": K, "world": world, "parts": P, "halves": halves}
        roof = roofline(rounds_local, nwp, n_own, E_local, shape, args.leg_steps) if rank == 0 else None
        if roof is not None:
            roof["event_ms_per_step"] = event_ms
            roof["stamp_ms_per_step"] = sum(s["kernel_ms"] for s in rounds_local) / args.leg_steps
        # the graph's global adjacency entries: lane group 0's parts hold every row once
        nnz = job.allreduce([E_local if rank < P else 0])[0]
        transport = runner.transport if runner is not None else None
        if dinfo is not None:
            dinfo.update(peer_info(job))

        # properties and, N > 1, one unsharded engine on rank 0 (after every shard is freed)
        export_c4 = []  # N = 1: the C4 graph for its components, exported before the engine goes
        if world == 1 and name == "C4":
            export_c4.append(phase(eng.export_topology, "graph export"))
        close_engs()
        srcs = [n for n, _, _ in inj]
        checks = {}

        def verify():
            if rank != 0:
                return []
            bad = []
            single = None
            if world > 1:
                t = time.perf_counter()
                ref = Engine(V, K, seed=seed, enable_sync=True, device=local)
                try:
                    ref.generate(**gen)
                    for a, b, ep in windows:
                        ref.partition_seeded(a, b, ep)
                    inject(ref, inj_arr)
                    single = ref.step(R)
                    topo = ref.export_topology() if name == "C4" else None
                finally:
                    ref.close()
                torch.cuda.synchronize()
                d = count_diffs(check, single, COUNT_FIELDS, "sharded", "single")
                bad += d
                checks["single_engine"] = ("every round's global counters equal one unsharded engine "
                                           f"({time.perf_counter() - t:.1f} s)" if not d else "FAILED: " + "; ".join(d))
            if name == "C4":
                t = time.perf_counter()
                if world == 1:
                    topo = export_c4.pop()
                lab, size, vol = components(topo.row_ptr, topo.col, device=f"cuda:{local}", log=log)
                del topo
                exp_d, exp_f = expected_from_components(lab, size, vol, srcs)
                checks["components_s"] = time.perf_counter() - t
                ncomp = int((size > 0).sum())
                checks["components"] = ncomp
                if ncomp > 1 and any(m != "component targets" for m in lsat):
                    checks["lsat_note"] = ("a disconnected graph, but some rank ran the lean digest without "
                                           "component targets (slower, still exact): " + ", ".join(lsat))
            elif name == "C3":  # connected; the timers fire, so KAT-3 does not apply
                exp_d, exp_f = V * K, None
            else:  # the grid spans every node: one component
                exp_d, exp_f = V * K, K * (nnz - (V - 1))
            bad += episode_failures(check, exp_d, exp_f)
            checks["properties"] = ("P1 (deliveries = sum of source component sizes), " +
                                    ("" if exp_f is None else "KAT-3 (forwards = sum of vol(comp) - |comp| + 1: no "
                                     "timer fired before quiescence), ") +
                                    "ACK (acks(r+1) = broadcasts delivered in r) hold on the checking episode")
            checks["expected"] = {"deliveries": exp_d, "forwards": exp_f}
            gold = gold_full(name, V, K, seed)
            if gold is not None:  # O2 on the host-built graph, every round (tests/golden/fullsize_*.json)
                d = count_diffs(check, gold["rounds"], COUNT_FIELDS, "checking episode", "O2")
                bad += d
                checks["oracle"] = (f"every round's global counters and delivery hash equal O2's run of this "
                                    f"workload on the host-built graph (tests/golden/fullsize_{name.lower()}.json, "
                                    f"{len(gold['rounds'])} rounds)" if not d else "FAILED: " + "; ".join(d[:4]))
            else:
                checks["oracle"] = "no O2 record of this shape (tests/golden/fullsize_*.json)"
            return bad

        fails += phase(verify, "checks") or []
        ok = not job.allreduce([len(fails)])[0]
        checks["timed_episodes"] = "every timed episode equals the checking episode, counter by counter"
        if fails:
            checks["failures"] = fails[:12]
        last = max((i for i, s in enumerate(check) if s["new_bits"]), default=-1)
        rec = {
            "config": name, "workload": workload, "nodes": V, "edges": nnz, "lanes": K, "n_gpus": world,
            "scaling": "strong", "vertex_parts": P, "lane_groups": L, "lane_halves_per_gpu": halves,
            "exchange": transport, "exchange_note": note,
            "steps": args.leg_steps, "rounds_per_step": R, "rounds_to_full_delivery": last + 1,
            "value": deliveries / elapsed, "unit": "deliveries/s",
            "ms_per_step": elapsed / args.leg_steps * 1e3,
            "deliveries_per_step": deliveries // args.leg_steps,
            "hbm_bytes_per_gpu": hbm, "hbm_bytes_max": max(hbm),
            "lsat": lsat,
            "exchange_bytes_per_round_rank0": sent if world > 1 else None,
            "exchange_bytes_densest_round_rank0": sent_max if world > 1 else None,
            "shard": dinfo, "setup_s": setup_s,
            "check": "passed" if ok else "FAILED", "checks": checks,
            "roofline": roof,
        }
        return rec
    finally:
        close_engs()


# ---------------------------------------------------------------------------

def cpu_baseline(cfg, topo, inj, V, K, seed, R):
    """The oracle restatements on this host's cores (reported beside the GPU
    number, not the target). Legs: O2 (bitset, C++) on the box's CPU share, O2
    on one thread, and O1 (message-level literal restatement of the handlers,
    Python) on C1 per inter-node message — the cost of the reference's own
    per-message Send/handler path in kind. Each leg is a bounded sample."""
    from ggamd import topology as T
    from ggamd.engine import Engine
    from ggamd.workload import inject, uniform_injections
    host_cpus, affinity = cpu_counts()
    # the CPU share this process is given: the runtime's declared thread budget
    # (OMP_NUM_THREADS: the GPU box's per-GPU share of its host cores), else every
    # core this process may run on
    share = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(int(share), affinity)) if share and share.isdigit() else affinity
    basis = "OMP_NUM_THREADS (the declared per-GPU CPU share)" if share and share.isdigit() else \
        "sched_getaffinity (every core this process may use)"

    def o2_episodes(topo_, inj_, V_, K_, seed_, thr, budget_s, rounds=None):
        os.environ["GG_CPU_THREADS"] = str(thr)
        e = Engine(V_, K_, seed=seed_, enable_sync=True, library=CPU_LIB)
        e.topology(topo_)
        if rounds is not None:  # one untimed episode: first-touch page faults, thread start-up
            e.reset()
            inject(e, inj_)
            e.step(rounds)
        dl, eps, t0 = 0, 0, time.perf_counter()
        while True:
            e.reset()
            inject(e, inj_)
            if rounds is None:  # to quiescence
                r = 0
                while True:
                    s = e.step(1)[0]
                    dl += s["new_bits"]
                    r += 1
                    if s["new_bits"] == 0 and r > 1:
                        break
                rounds = r
            else:
                dl += sum(s["new_bits"] for s in e.step(rounds))
            eps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        dt = time.perf_counter() - t0
        e.close()
        return dl / dt, eps, rounds, dt

    scaling = None
    if cfg == "C2":
        v_all, n_all, r_all, _ = o2_episodes(topo, inj, V, K, seed, threads, 8.0, R)
        sample_all = f"{n_all} full C2 episodes ({r_all} rounds each)"
        v_one, n_one, r_one, _ = o2_episodes(topo, inj, V, K, seed, 1, 6.0, R)
        sample_one = f"{n_one} full C2 episode(s) on one thread"
        # thread scaling inside the share (the whole box is not this process's to take)
        scaling = {"1": v_one, str(threads): v_all}
        t = 2
        while t < threads:
            scaling[str(t)] = o2_episodes(topo, inj, V, K, seed, t, 3.0, R)[0]
            t *= 2
        scaling = dict(sorted(scaling.items(), key=lambda kv: int(kv[0])))
    else:  # C4: R-MAT samples of the same generator (the 10^8-node graph needs ~150 GB of host state)
        Va = 1 << 20
        ta = T.rmat(Va, 16, seed=seed)
        v_all, n_all, r_all, _ = o2_episodes(ta, uniform_injections(Va, K, seed), Va, K, seed, threads, 1.0)
        sample_all = f"{n_all} episode(s) to quiescence ({r_all} rounds) of the same R-MAT generator at 2^20 nodes"
        V1 = 1 << 17
        t1 = T.rmat(V1, 16, seed=seed)
        v_one, n_one, r_one, _ = o2_episodes(t1, uniform_injections(V1, K, seed), V1, K, seed, 1, 1.0)
        sample_one = f"{n_one} episode(s) ({r_one} rounds) of the R-MAT generator at 2^17 nodes on one thread"
    o1 = o1_c1_leg()
    return {"value": v_all, "unit": "deliveries/s", "cores": threads, "kind": "port",
            "sample": f"O2 bitset oracle (oracle/o2_bitset.cpp, -O3) on {threads} threads: {sample_all}",
            "host_cpus": host_cpus, "affinity_cpus": affinity, "cores_basis": basis,
            "single_thread": {"value": v_one, "unit": "deliveries/s", "cores": 1, "sample": sample_one},
            "thread_scaling": scaling,
            "whole_box": {"value": None, "cores": affinity,
                          "note": (f"not measured: this process's CPU share is {threads} of the host's {host_cpus} "
                                   "CPUs (OMP_NUM_THREADS on the GPU box; the other GPUs' jobs own the rest), so "
                                   "O2 runs on that share; thread_scaling gives its curve inside the share"
                                   if threads < affinity else "= value (every CPU this process may use)")},
            "o1_per_message": o1}


def o1_c1_leg():
    """O1 (oracle/o1_literal.py: every Send/Reply/RPC a message object through an
    in-memory network, handlers restated statement by statement) on config C1:
    inter-node messages and deliveries per second of one thread."""
    sys.path.insert(0, REPO)
    from oracle.o1_literal import O1Network
    from ggamd.workload import c1
    wl, _ = c1()
    o = O1Network(25, wl.n_lanes, wl.seed, wl.sync_base, wl.sync_jitter, wl.enable_sync)
    o.topology(wl.topo.rows())
    for n, v, r in wl.injections:
        o.broadcast(int(n), int(v), int(r))
    t0 = time.perf_counter()
    st = o.step(wl.max_rounds)
    dt = time.perf_counter() - t0
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in st)
    dl = sum(s["new_bits"] for s in st)
    return {"value": msgs / dt, "unit": "inter-node messages/s", "cores": 1,
            "deliveries_per_s": dl / dt, "messages": msgs, "seconds": dt,
            "sample": f"C1 (25-node tree4, {len(wl.injections)} client broadcasts over 200 rounds, sync on), "
                      f"{wl.max_rounds} rounds through O1's message-level network"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=["C2", "C4"])
    ap.add_argument("--no-headline", action="store_true",
                    help="legs only (profiling a leg's kernels alone); the JSON line then carries only the legs")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, help="C2: nodes per GPU (2^20); C4: nodes (10^8)")
    ap.add_argument("--lanes", type=int, help="C2: 1024; C4: 4096")
    ap.add_argument("--parts", type=int, default=1, help="--config C4: vertex parts P (world = lane groups x P)")
    ap.add_argument("--halves", type=int, default=1, choices=[1, 2],
                    help="--config C4 with --parts > 1: 2 = two engines per GPU over the two halves of its lanes, "
                         "one half's exchange overlapping the other half's kernels (ggamd.dist.HalvesRunner)")
    ap.add_argument("--legs", default=None,
                    help="comma list of C3,C4,C5 (default after a C2 headline: C3,C4,C5; 'none' to skip)")
    ap.add_argument("--leg-steps", type=int, default=3, help="timed episodes per leg")
    ap.add_argument("--leg-parts", type=int, default=0, help="legs: vertex parts P (default N)")
    ap.add_argument("--leg-halves", type=int, default=0, choices=[0, 1], help="legs: 1 = no lane halves for C4")
    ap.add_argument("--c3-nodes", type=int, help="C3 leg nodes (10^7; smaller for rehearsals)")
    ap.add_argument("--c4-nodes", type=int, help="C4 leg nodes (10^8; smaller for rehearsals)")
    ap.add_argument("--c5-side", type=int, help="C5 leg grid side (32768 = 2^30 nodes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fresh-sets", type=int, default=4,
                    help="N = 1: after the timed region, episodes rotating this many distinct seeded injection "
                         "sets (every step re-captures its launch graph and uploads its injections; 0: skip)")
    ap.add_argument("--no-check", action="store_true", help="skip the N > 1 single-engine check")
    ap.add_argument("--xchg", default=os.environ.get("GG_DIST_TRANSPORT", "auto"),
                    choices=["auto", "engine", "ipc", "torch"],
                    help="N > 1 exchange between vertex parts: engine = the engine's grouped RCCL send/recv; "
                         "ipc = device-driven (IPC-mapped peer windows, kernel flags, captured batches of rounds, "
                         "no host wait); torch = torch all_to_all; auto (default) = ipc when every rank maps its "
                         "peers and one whole validation episode through it equals O2, else engine")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 "
                    "(nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    args = ap.parse_args()
    if os.environ.get("GG_BENCH_WATCHDOG"):  # stacks of every thread every N seconds (hang diagnosis)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GG_BENCH_WATCHDOG"]), repeat=True, file=sys.stderr)

    job = Job(args.backend, args.gpus)
    if args.no_headline:
        out, info = {"note": "--no-headline: legs only"}, {"xchg": args.xchg}
    else:
        out, info = headline(job, args)
    legs_arg = args.legs if args.legs is not None else ("C3,C4,C5" if args.config == "C2" else "none")
    names = [x.strip().upper() for x in legs_arg.split(",") if x.strip() and x.strip().lower() != "none"]
    legs = {}
    for name in names:
        if name not in ("C3", "C4", "C5"):
            raise SystemExit(f"--legs: unknown leg {name}")
        pref = info["xchg"] if info["xchg"] in ("ipc", "engine") else "engine"
        if args.backend != "nccl" and pref == "engine":
            pref = "engine"  # (gloo rehearsal: the engine's sequencing over HostTransport)
        legs[name] = run_leg(job, args, name, pref)
    if job.rank == 0:
        if names:
            out["legs"] = legs
        print(json.dumps(out), flush=True)
    job.close()


if __name__ == "__main__":
    main()
