"""Maelstrom broadcast-workload checker over the engine.

Maelstrom's `broadcast` workload (the reference is tested with `maelstrom test
-w broadcast --node-count 25 --time-limit 20 --rate 100 --latency 100
--topology tree4`, README.md:7-10,26-27; claims README.md:16-18) reports, for
the client operations it issued:
  * stable latency of each broadcast: time until the value is visible in every
    node's read;
  * messages per operation: inter-server messages / client operations;
  * lost values: acknowledged broadcasts missing from the final reads.
Under the lockstep contract a client broadcast of value m to
node s in round r0 is visible at node v from round dr(v, m) on (the engine's
delivery rounds), so with one round per `tick_ms` of simulated latency the
stable latency of m is (max_v dr(v, m) - r0) * tick_ms, and the final reads
are the node sets after the last round. Client reads are operations but not
inter-node messages (they go client -> node), so they only enter the op count.
"""
from __future__ import annotations

import numpy as np


def broadcast_report(eng, injections, n_read_ops: int, stats: list[dict], tick_ms: float = 100.0) -> dict:
    """eng: an Engine created with track_delivery=True that ran `stats` rounds;
    injections: (node, value, round) client broadcasts in call order."""
    first = {}
    for n, v, r in injections:
        first.setdefault(int(v), (int(n), int(r)))
    dr = eng.delivery_rounds()  # [V][W] first-seen round, -1 never
    lat, lost = [], []
    for v, (n, r0) in first.items():
        lane = eng.lane_of(v)
        col = dr[:, lane]
        if (col < 0).any():
            lost.append(v)
            continue
        lat.append((int(col.max()) - r0) * tick_ms)
    V = dr.shape[0]
    final = eng.read_bits()
    lanes = [eng.lane_of(v) for v in first]
    have = np.stack([(final[:, l >> 6] >> np.uint64(l & 63)) & np.uint64(1) for l in lanes], 1)
    missing_reads = int(V * len(lanes) - int(have.sum()))
    fwd = sum(s["fwd_sent"] for s in stats)
    pushes = sum(s["pushes"] for s in stats)
    acks = sum(s["acks"] for s in stats)
    reads = sum(s["reads"] for s in stats)
    read_oks = sum(s["read_oks"] for s in stats)
    msgs = fwd + pushes + acks + reads + read_oks
    ops = len(injections) + n_read_ops
    lat = np.array(lat) if lat else np.zeros(1)
    return {
        "nodes": V,
        "rounds": len(stats),
        "broadcast_ops": len(injections),
        "read_ops": n_read_ops,
        "inter_node_msgs": int(msgs),
        "msgs_per_op": msgs / max(1, ops),
        "msgs_per_broadcast": msgs / max(1, len(injections)),
        "gossip_msgs_per_broadcast": (fwd + acks) / max(1, len(injections)),
        "sync_msgs": int(pushes + reads + read_oks),
        "stable_latency_ms": {"median": float(np.median(lat)), "p95": float(np.percentile(lat, 95)),
                              "p99": float(np.percentile(lat, 99)), "max": float(lat.max())},
        "lost": lost,
        "missing_in_final_reads": missing_reads,
    }
