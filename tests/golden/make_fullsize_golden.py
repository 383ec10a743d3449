#!/usr/bin/env python3
"""Generate tests/golden/fullsize_c5.json, fullsize_c4.json and fullsize_c3.json:
BASELINE.json's three largest configs at their FULL size run by the CPU oracle O2
(oracle/o2_bitset.cpp) on graphs built by the host builders
(host/topology.cpp, no GPU involved) — every round's counters and delivery
hash (seen_hash: the fingerprint of every (node, value) first-delivery round,
DESIGN.md §2 item 6) to quiescence. tests/test_gpu_fullsize.py runs the HIP
engine on the device-generated graph and diffs it against these records round
by round: the O2 run takes minutes on the GPU box's host cores (C5: 2^30 nodes,
6.4e9 adjacency entries; C4: 10^8 nodes at 4096 lanes, 1.6 TB of sender rows
per dense round), far beyond the GPU suite's budget, so it runs once here.

  C5  32768 x 32768 grid + one seeded long link per node, W = 64, sync on
  C3  random 8-regular, 10^7 nodes, W = 1024, a seeded bisection in rounds
      [2, 12) healed by the sync timers (bench.py's C3 leg checks every timed
      episode against this record)
  C4  R-MAT (.57,.19,.19,.05) edge factor 16, 10^8 nodes, W = 4096, sync on,
      as L lane-group engines run one after the other (lanes never interact:
      the per-round counters of the groups sum to one engine's, node-level
      counters being counted by group 0 only — the same split the HIP engine's
      gg_config.lane_groups uses), --groups picks which ones a call runs and
      --merge sums the partial records.

The workloads are the bench legs' (bench.py leg(): seeds, uniform injections
in round 0, the engine's default timers). Progress goes to stdout every round
and every 30 s of a long call (the GPU box's hang rule).

Usage (repo root; runs on the GPU box's host CPUs, ~270 GB host memory cap):
  python tests/golden/make_fullsize_golden.py C5
  python tests/golden/make_fullsize_golden.py C4 --lane-groups 4 --groups 0,1
  python tests/golden/make_fullsize_golden.py C4 --lane-groups 4 --groups 2,3
  python tests/golden/make_fullsize_golden.py C4 --merge
"""
import argparse
import glob
import json
import os
import platform
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "gossip-glomers-distributed-systems_amd")]

from ggamd import topology as T  # noqa: E402
from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402

CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
M64 = (1 << 64) - 1
T0 = time.time()


def log(*a):
    print(f"[{time.time() - T0:7.1f} s]", *a, flush=True)


class Heartbeat:
    """A line every 30 s while a long native call runs (no output for 3 min = hung)."""

    def __init__(self, what):
        self.what, self.stop = what, threading.Event()

    def __enter__(self):
        def beat():
            while not self.stop.wait(30):
                log(f"... {self.what}")
        self.t = threading.Thread(target=beat, daemon=True)
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()


def spec(name, size=None):
    if name == "C5":
        side = size or 32768
        V, K, seed = side * side, 64, BASE_SEED + 5
        return dict(V=V, K=K, seed=seed, build=lambda: T.grid_links(side, seed=seed), windows=[],
                    graph=f"grid_links side {side} seed {seed} (ggh_grid_links)", gen=dict(kind="grid_links", n=side,
                                                                                             seed=seed))
    if name == "C3":  # the partition window cuts rounds [2, 12); the timers (round >= 20) heal it
        V, K, seed = size or 10_000_000, 1024, BASE_SEED + 3
        return dict(V=V, K=K, seed=seed, build=lambda: T.random_regular(V, 8, seed), heal=True,
                    windows=[(2, 12, seed ^ 0x5EED)],
                    graph=f"random_regular n {V} k 8 seed {seed} (ggh_random_regular)",
                    gen=dict(kind="random_regular", n=V, k=8, seed=seed))
    V, K, seed = size or 100_000_000, 4096, BASE_SEED + 4
    return dict(V=V, K=K, seed=seed, build=lambda: T.rmat(V, 16, seed=seed), windows=[],
                graph=f"rmat n {V} edge factor 16 (.57,.19,.19) seed {seed} (ggh_rmat)",
                gen=dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19))


def run_group(sp, topo, inj, L, g, cap=120):
    kw = dict(rank=g, world=L, lane_groups=L) if L > 1 else {}
    e = Engine(sp["V"], sp["K"], seed=sp["seed"], enable_sync=True, library=CPU_LIB, **kw)
    try:
        with Heartbeat(f"O2 install (group {g})"):
            e.topology(topo)
        log(f"group {g}/{L}: O2 topology installed")
        for a, b, ep in sp["windows"]:
            e.partition_seeded(a, b, ep)
        inject(e, inj)
        rounds, total = [], 0
        while True:
            with Heartbeat(f"O2 round {len(rounds)} (group {g})"):
                s = e.step(1)[0]
            rounds.append({f: int(s[f]) & M64 for f in ("round",) + tuple(COUNT_FIELDS)})
            total += s["new_bits"]
            log(f"group {g}/{L}: round {s['round']} new_bits {s['new_bits']} fwd {s['fwd_sent']} "
                f"dropped {s['dropped']} syncs {s['syncs_fired']}")
            # the bench legs' rule: the first round after round 0 with no new bits; a healed
            # partition (C3): the first such round after every node holds every value
            done = s["new_bits"] == 0 and len(rounds) > 1
            if sp.get("heal"):
                done = done and total == sp["V"] * sp["K"] // L
            if done or len(rounds) >= cap:
                return rounds
    finally:
        e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["C3", "C4", "C5"])
    ap.add_argument("--lane-groups", type=int, default=1)
    ap.add_argument("--groups", default=None, help="comma list of lane groups this call runs (default all)")
    ap.add_argument("--merge", action="store_true", help="sum the partial records into the golden file")
    ap.add_argument("--outdir", default=HERE, help="where the records go (on the GPU box: under gpurun_out/)")
    ap.add_argument("--size", type=int, help="a smaller C5 side / C4 node count (dry runs; the golden is full size)")
    args = ap.parse_args()
    name = args.config
    os.makedirs(args.outdir, exist_ok=True)
    out = os.path.join(args.outdir, f"fullsize_{name.lower()}.json")
    if args.merge:
        parts = [json.load(open(p)) for p in sorted(glob.glob(os.path.join(args.outdir, f"fullsize_{name.lower()}.part*.json")))]
        L = parts[0]["lane_groups"]
        have = sorted(int(g) for p in parts for g in p["groups"])
        assert have == list(range(L)), f"partial records cover groups {have}, not 0..{L - 1}"
        R = max(len(rs) for p in parts for rs in p["groups"].values())
        for p in parts:  # a group that quiesced earlier adds nothing to the later rounds: no
            for rs in p["groups"].values():  # timer fired, nothing is injected after round 0
                assert all(x["syncs_fired"] == 0 for x in rs) and rs[-1]["new_bits"] == 0
        tot = []
        for r in range(R):
            d = {"round": r}
            for f in COUNT_FIELDS:
                d[f] = 0
                for p in parts:
                    for rs in p["groups"].values():
                        if r < len(rs):
                            d[f] = (d[f] + rs[r][f]) & M64
                        elif f == "seen_hash":  # cumulative: it stays at the group's last value
                            d[f] = (d[f] + rs[-1][f]) & M64
            tot.append(d)
        rec = {k: parts[0][k] for k in ("config", "generator", "oracle", "graph", "nodes", "nnz", "lanes", "seed",
                                         "lane_groups", "workload")}
        rec["rounds"] = tot
        rec["runs"] = [{k: p[k] for k in ("groups_run", "host", "threads", "seconds")} for p in parts]
        json.dump(rec, open(out, "w"), indent=0)
        log(f"merged {len(parts)} partial records: {R} rounds -> {out}")
        return
    sp = spec(name, args.size)
    L = args.lane_groups
    groups = [int(x) for x in args.groups.split(",")] if args.groups else list(range(L))
    with Heartbeat("host graph build"):
        topo = sp["build"]()
    log(f"{name}: host graph built, {sp['V']} nodes, {topo.nnz} adjacency entries")
    inj = injection_arrays(uniform_injections(sp["V"], sp["K"], sp["seed"]))
    res = {}
    for g in groups:
        res[str(g)] = run_group(sp, topo, inj, L, g)
    rec = {
        "config": name, "generator": "tests/golden/make_fullsize_golden.py", "oracle": "O2 (oracle/o2_bitset.cpp)",
        "graph": sp["graph"], "device_generator": sp["gen"], "nodes": sp["V"], "nnz": int(topo.nnz),
        "lanes": sp["K"], "seed": sp["seed"], "lane_groups": L,
        "windows": [list(w) for w in sp["windows"]],
        "workload": "the bench leg's: uniform_injections(V, K, seed) in round 0, sync on (default timers), "
                    "the seeded partition windows listed (C3: [2, 12)); to the first round after round 0 with no "
                    "new bits (C3: the first after every node holds every value)",
        "groups_run": groups, "host": platform.node(), "threads": os.environ.get("OMP_NUM_THREADS"),
        "seconds": time.time() - T0,
    }
    if L == 1:
        rec["rounds"] = res["0"]
        json.dump(rec, open(out, "w"), indent=0)
        log(f"{len(rec['rounds'])} rounds -> {out}")
    else:
        rec["groups"] = res
        p = os.path.join(args.outdir, f"fullsize_{name.lower()}.part{'_'.join(map(str, groups))}.json")
        json.dump(rec, open(p, "w"), indent=0)
        log(f"groups {groups} -> {p}")


if __name__ == "__main__":
    main()
