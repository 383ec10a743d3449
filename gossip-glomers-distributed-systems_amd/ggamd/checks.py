"""Size-independent properties of the reference's propagation (SURVEY.md §8c
KATs), for runs too large for the CPU oracle: the full-size GPU tests and the
bench's C4 / C5 legs use them. These are checkers of results, not a compute
path: nothing here runs a round.

  P1    every message reaches exactly its source's connected component: with no
        partitions, HandleBroadcast floods every new value to every neighbour
        (broadcast.go:50-57, :72-76), so at quiescence total deliveries =
        sum over messages of |comp(src)|
  KAT-3 before any sync timer fires, every reached node forwards each value to
        all its neighbours except the first deliverer (:52), the source to all:
        forwards = sum over messages of [vol(comp(src)) - (|comp(src)| - 1)]
  ACK   every delivered broadcast is acked one round later (:69, :78):
        acks(r + 1) = fwd_delivered(r) + push_delivered(r)
"""
from __future__ import annotations

import time

import numpy as np


def components(row_ptr, col, device="cuda", chunk=1 << 29, log=print):
    """Connected components of a symmetric CSR on the GPU (torch): min-label
    propagation over every adjacency entry (rows and columns resident as int64
    chunks) with pointer jumping, to a fixed point. Returns (label per node,
    component size per label, degree sum per label) as numpy arrays."""
    import torch
    dev = torch.device(device)
    t0 = time.time()
    V = row_ptr.size - 1
    E = int(col.size)
    chunks = []  # (rows, cols) int64 on the device
    for e0 in range(0, E, chunk):
        e1 = min(E, e0 + chunk)
        v0 = int(np.searchsorted(row_ptr, e0, side="right")) - 1
        v1 = int(np.searchsorted(row_ptr, e1 - 1, side="right"))
        rp = torch.from_numpy(np.clip(row_ptr[v0:v1 + 1], e0, e1) - e0).to(dev)
        rows = torch.repeat_interleave(torch.arange(v0, v1, device=dev), rp[1:] - rp[:-1])
        chunks.append((rows, torch.from_numpy(col[e0:e1]).to(dev).long()))
    lab = torch.arange(V, dtype=torch.int64, device=dev)
    it = 0
    while True:
        old = lab.clone()
        for rows, cols in chunks:
            lab.scatter_reduce_(0, rows, lab[cols], reduce="amin")
        for _ in range(8):  # pointer jumping
            lab = lab[lab]
        it += 1
        if log:
            log(f"components: pass {it}, {time.time() - t0:.1f} s")
        if torch.equal(lab, old):
            break
    lab = lab.cpu().numpy()
    del chunks, old
    torch.cuda.empty_cache()
    # per-label sums on the host: the giant component's label would take every
    # device atomic of a bincount on one address
    size = np.bincount(lab, minlength=V)
    vol = np.bincount(lab, weights=(row_ptr[1:] - row_ptr[:-1]).astype(np.float64), minlength=V)
    if log:
        log(f"components: {int((size > 0).sum())} labels, {time.time() - t0:.1f} s")
    return lab, size, vol


def expected_from_components(lab, size, vol, sources) -> tuple[int, int]:
    """(P1 deliveries, KAT-3 forwards) for one message per source node."""
    comp = lab[np.asarray(sources, np.int64)]
    p1 = int(size[comp].sum())
    kat3 = int(round(float(vol[comp].sum()))) - p1 + len(sources)
    return p1, kat3


def episode_failures(stats: list[dict], exp_deliveries: int | None, exp_forwards: int | None) -> list[str]:
    """P1, KAT-3 (only when no sync timer fired: a sync adds reads and pushes)
    and the ack identity over one episode's global per-round counters."""
    bad = []
    dl = sum(s["new_bits"] for s in stats)
    if exp_deliveries is not None and dl != exp_deliveries:
        bad.append(f"P1: deliveries {dl} != {exp_deliveries}")
    fired = sum(s["syncs_fired"] for s in stats)
    fwd = sum(s["fwd_sent"] for s in stats)
    if exp_forwards is not None:
        if fired:
            bad.append(f"KAT-3 not applicable: {fired} sync timers fired before quiescence")
        elif fwd != exp_forwards:
            bad.append(f"KAT-3: forwards {fwd} != {exp_forwards}")
    for a, b in zip(stats, stats[1:]):
        if b["acks"] != a["fwd_delivered"] + a["push_delivered"]:
            bad.append(f"ACK: acks of round {b['round']} != delivered broadcasts of round {a['round']}")
            break
    return bad
