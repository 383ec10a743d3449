#!/usr/bin/env python3
"""Full-size config runs (BASELINE.json configs C2..C5) on one GPU, checked by
size-independent properties of the reference semantics, plus optional
bit-exact comparison with the CPU oracle O2 (every round's counters and hash).

Properties (no reference fixtures exist at these sizes; SURVEY.md §8c KATs):
  P1 every message reaches exactly its source's weakly connected component:
     total deliveries = sum over messages of |comp(src)|
  P2 no partitions and no sync firing during the run: forwards sent =
     sum over messages of [sum of degrees in comp(src) - (|comp(src)| - 1)]
     (KAT-3: the source excludes nobody, every other node excludes its first
     deliverer), and acks of round r+1 = broadcasts delivered in round r
  P3 without partitions a node first holds message m in round dist(src_m, v):
     after every round r, bit (v, m) == (dist <= r) on a node sample for two
     messages (BFS on the host)
Then a timed episode (one launch sequence, graph-captured) gives deliveries/s,
rounds to full delivery, per-kernel GB/s and the HBM footprint.

Usage: tools/fullsize.py C3|C4|C5|C2 [--nodes V | --side S] [--oracle] [--max-rounds N]
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

import numpy as np  # noqa: E402

from ggamd import topology as T  # noqa: E402
from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import by_name, inject  # noqa: E402


def log(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--nodes", type=int)
    ap.add_argument("--side", type=int)
    ap.add_argument("--lanes", type=int)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--max-rounds", type=int, default=200)
    ap.add_argument("--sample", type=int, default=20000)
    ap.add_argument("--no-sync", action="store_true")
    ap.add_argument("--device-gen", action="store_true",
                    help="build the graph in HBM (gossip_gen.h) instead of on the host; the CSR is "
                         "exported back only for the host-side facts")
    ap.add_argument("--json")
    args = ap.parse_args()
    import torch
    kw = {}
    if args.nodes:
        kw["V"] = args.nodes
    if args.side:
        kw["side"] = args.side
    if args.lanes:
        kw["K"] = args.lanes
    t0 = time.time()
    wl = by_name(args.config, device_gen=args.device_gen, **kw)
    if args.no_sync:
        wl.enable_sync = False
    K = len(wl.injections)
    if wl.topo is not None:
        V = wl.topo.n_nodes
        log(f"{wl.name}: V={V} E={wl.topo.nnz} K={K} W={wl.n_lanes} sync={wl.enable_sync} "
            f"windows={[w[:3] for w in wl.windows]} (host CSR built in {time.time() - t0:.1f}s)")
    else:
        g = wl.gen
        V = g["n"] * g["n"] if g["kind"] == "grid_links" else g["n"]
        log(f"{wl.name}: V={V} K={K} W={wl.n_lanes} sync={wl.enable_sync} "
            f"windows={[w[:3] for w in wl.windows]} (graph built on the device: {g})")
    free0 = torch.cuda.mem_get_info(0)[0]
    t1 = time.time()
    eng = Engine(V, wl.n_lanes, seed=wl.seed, sync_base=wl.sync_base, sync_jitter=wl.sync_jitter,
                 enable_sync=wl.enable_sync, device=0)
    wl.apply(eng)
    torch.cuda.synchronize()
    footprint = free0 - torch.cuda.mem_get_info(0)[0]
    ready_s = time.time() - t1
    log(f"engine ready in {ready_s:.1f}s ({'device-built graph' if wl.topo is None else 'host CSR upload'}), "
        f"HBM footprint {footprint / 2**30:.2f} GiB")
    if wl.topo is None:
        t = time.time()
        wl.topo = eng.export_topology()
        log(f"exported the generated CSR for the host facts in {time.time() - t:.1f}s (E={wl.topo.nnz})")
    topo = wl.topo

    # host-side facts for the properties
    t2 = time.time()
    if wl.name == "C5":
        # the side x side grid is a spanning connected subgraph: one component
        # (skips a serial union-find over 6.4e9 entries at side 2^15)
        lab = np.zeros(V, np.uint32)
    else:
        lab = T.components(topo)
    deg = np.diff(topo.row_ptr)
    comp_size = np.bincount(lab, minlength=V)
    comp_deg = np.bincount(lab, weights=deg.astype(np.float64), minlength=V)
    first = {}
    for n, v, r in wl.injections:  # first injection of each value
        first.setdefault(v, (n, r))
    srcs = np.array([n for n, _ in first.values()], np.int64)
    exp_deliv = int(comp_size[lab[srcs]].sum())
    exp_fwd = int((comp_deg[lab[srcs]] - (comp_size[lab[srcs]] - 1)).sum())
    probe = [int(srcs[0]), int(srcs[len(srcs) // 2])]
    probe_lane = [eng.lane_of(list(first.keys())[0]), eng.lane_of(list(first.keys())[len(srcs) // 2])]
    # a heartbeat while the serial BFS probes run (minutes at 2^30 nodes): a
    # GPU-box run that prints nothing for 3 minutes is taken to be hung
    done = threading.Event()

    def beat():
        while not done.wait(30):
            log(f"  host facts: BFS probes running ({time.time() - t2:.0f}s)")

    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    try:
        dist = [T.bfs(topo, s) for s in probe]
    finally:
        done.set()
        hb.join()
    log(f"host facts in {time.time() - t2:.1f}s: components {len(np.unique(lab))}, expected deliveries "
        f"{exp_deliv}, probe sources {probe}")
    S = min(args.sample, V)
    masked = bool(wl.windows)

    # checking run: round by round
    ref = None
    if args.oracle:
        lib = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
        ref = Engine(V, wl.n_lanes, seed=wl.seed, sync_base=wl.sync_base, sync_jitter=wl.sync_jitter,
                     enable_sync=wl.enable_sync, library=lib)
        wl.apply(ref)
    stats, total, fails = [], 0, []
    for r in range(args.max_rounds):
        s = eng.step(1)[0]
        stats.append(s)
        total += s["new_bits"]
        if ref is not None:
            c = ref.step(1)[0]
            bad = [f for f in COUNT_FIELDS if s[f] != c[f]]
            if bad:
                fails.append(f"round {r}: O2 differs in {bad}")
        if not masked:
            bits = eng.read_bits(0, S)
            for d, lane in zip(dist, probe_lane):
                have = (bits[:, lane >> 6] >> np.uint64(lane & 63)) & np.uint64(1)
                want = (d[:S] >= 0) & (d[:S] <= r)
                if not np.array_equal(have.astype(bool), want):
                    fails.append(f"round {r}: lane {lane} sample bits differ from BFS balls")
        if ref is not None or r % 10 == 0:
            log(f"  round {r}: new {s['new_bits']} kernel {s['kernel_ms']:.2f} ms total {total}")
        if total == exp_deliv and r > 0 and s["new_bits"] == 0:
            break
    R = len(stats)
    last_deliv = max(i for i, s in enumerate(stats) if s["new_bits"]) if total else 0
    # P1
    if total != exp_deliv:
        fails.append(f"P1: deliveries {total} != {exp_deliv}")
    fired = sum(s["syncs_fired"] for s in stats)
    fwd = sum(s["fwd_sent"] for s in stats)
    if not masked and fired == 0:
        if fwd != exp_fwd:
            fails.append(f"P2: forwards {fwd} != {exp_fwd}")
    for a, b in zip(stats, stats[1:]):
        if not masked and b["acks"] != a["fwd_delivered"] + a["push_delivered"]:
            fails.append(f"acks of round {b['round']} != delivered broadcasts of round {a['round']}")
            break
    log(f"checking run: {R} rounds, last delivery in round {last_deliv}, deliveries {total}, "
        f"forwards {fwd} (expected {exp_fwd if fired == 0 else 'n/a: sync fired'}), syncs fired {fired}")

    # timed run: whole episode in one launch sequence
    eng.reset()  # keeps topology and partition windows
    inject(eng, wl.injections)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    st = eng.step(R)
    el = time.perf_counter() - t3
    dl = sum(s["new_bits"] for s in st)
    torch.cuda.synchronize()
    footprint_after = free0 - torch.cuda.mem_get_info(0)[0]
    held = eng.device_bytes()
    kinds = {}
    for k in ("prep", "expand", "stream"):
        ms = sum(s[k + "_ms"] for s in st)
        by = sum(s[k + "_bytes"] for s in st)
        kinds[k] = {"ms": ms, "GB": by / 1e9, "GBps": by / (ms * 1e-3) / 1e9 if ms else 0.0}
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in st)
    out = {"config": wl.name, "nodes": V, "edges": int(topo.nnz), "lanes": wl.n_lanes, "messages": K,
           "rounds": R, "rounds_to_full_delivery": last_deliv + 1, "deliveries": dl,
           "episode_s": el, "deliveries_per_s": dl / el, "device_ms": eng.step_device_ms(),
           "hbm_footprint_GiB": footprint / 2**30,
           "hbm_after_episodes_GiB": footprint_after / 2**30,
           "engine_device_bytes": held["total"], "engine_sync_buffer_bytes": held["sync"],
           "topology_source": "device generator" if args.device_gen else "host CSR", "engine_ready_s": ready_s, "inter_node_msgs": msgs, "msgs_per_op": msgs / K,
           "kernels": kinds, "oracle": bool(ref), "properties_failed": fails}
    # the byte roofline and the request-ceiling fraction (line_frac), as bench.py
    # reports them (PMC requests when profiles/ holds a pass of this shape)
    sys.path.insert(0, REPO)
    import bench as B
    shape = {"config": wl.name, "nodes": V, "lanes": wl.n_lanes, "world": 1, "parts": 1, "halves": 1}
    roof = B.roofline(st, B.next_pow2(max(1, wl.n_lanes // 64)), V, int(topo.nnz), shape, 1)
    out["roofline"] = {k: roof[k] for k in ("kernel", "achieved", "frac", "line_frac", "line_source", "traffic",
                                            "avg_launch_ms")}
    log(json.dumps(out))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)
    if fails:
        log("FAIL:", fails[:10])
        sys.exit(1)
    log("PASS")


if __name__ == "__main__":
    main()
