#!/usr/bin/env python3
"""C4 at N GPUs, projected from one-GPU rehearsals (tools/c4_rehearsal.py JSON):
per round, the slowest rank's kernel time (measured, ranks run one at a time)
and the largest per-rank payload (measured bytes) over the xGMI links a rank
uses (P - 1 peers, one link each, at --link GB/s per direction).

  after:   T_r = C_r + X_r / B               (exchange after the kernels)
  overlap: T_r = max(C_r, X_r / B)           (lane halves: one half's exchange
                                              under the other half's kernels)
With --halves JSON (a rehearsal with twice the lane groups: each rank = one
lane half), a GPU's kernels are both halves' (C_A + C_B) and its payload both
halves' (X_A + X_B), overlapped as max(C_A + C_B, (X_A + X_B) / B): the price
of splitting the lanes is in the measured kernel times.

Scale-up to 10^8 nodes (--scale S): kernel times and payloads multiplied by
the single-engine ratio S of the dense rounds (measured: C4 at 10^8 vs the
rehearsal size), stated as a projection, not a measurement.

Host time per round (--host-us U): time the host spends on a round's critical
path, added to every round (the engine's RCCL exchange in exact-size mode
waits for each round's segment sizes before it enqueues the payload, round 3:
~70 us of enqueue per round behind that wait; the device-driven exchange has
none — its whole episode is enqueued ahead in one graph, 17 us per C4 round
measured, profiles/r4/ipc/).

Payload format (--row-bytes R --head-bytes H): the rehearsals measured the
engine exchange's 16-byte head per entry; the device-driven exchange's tile
segments (round 5) ship one 80-byte record per 256 entries instead, so each
payload is scaled by (R + 80/256) / (R + H), R = the F row's bytes.

Payloads measured over the device-driven exchange (--payload-json, from
tools/c4_ipc_payload.py: tile segments, with or without need bits) replace the
rehearsal's per-round payloads as they are.

Usage: python tools/project_c4.py profiles/r3/r3_c4_rehearsal_2p22_p8_ordered.json [--halves H.json] [--scale S] [--host-us U]
       [--row-bytes R --head-bytes 16] [--payload-json P.json --payload-key need|all]
"""
import argparse
import json


def rounds_of(d):
    return d["per_round"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rehearsal")
    ap.add_argument("--halves")
    ap.add_argument("--links", default="64,76.5,153", help="GB/s per link and direction")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--host-us", type=float, default=0.0, help="host time per round on the critical path")
    ap.add_argument("--row-bytes", type=float, default=0.0, help="F row bytes: rescale payloads to tile segments")
    ap.add_argument("--head-bytes", type=float, default=16.0, help="per-entry head bytes the rehearsal measured")
    ap.add_argument("--payload-json", help="tools/c4_ipc_payload.py output: its per-round largest per-rank payload "
                                           "(device-driven exchange, tile segments) replaces the rehearsal's")
    ap.add_argument("--payload-key", default="need", help="need | all (with or without need bits)")
    args = ap.parse_args()
    xs = (args.row_bytes + 80.0 / 256.0) / (args.row_bytes + args.head_bytes) if args.row_bytes else 1.0
    d = json.load(open(args.rehearsal))
    if args.payload_json:  # measured tile-segment payloads: no rescaling
        pj = json.load(open(args.payload_json))
        assert pj["config"]["nodes"] == d["config"]["nodes"] and pj["config"]["parts"] == d["config"]["parts"]
        for r, q in zip(rounds_of(d), pj["per_round"]):
            r["payload_bytes_max"] = q[f"payload_bytes_max_{args.payload_key}"]
        xs = 1.0
    P = d["config"]["parts"]
    h = json.load(open(args.halves)) if args.halves else None
    out = {"rehearsal": args.rehearsal, "halves": args.halves, "parts": P, "lane_groups": d["config"]["lane_groups"],
           "nodes": d["config"]["nodes"], "scale": args.scale, "host_us_per_round": args.host_us,
           "payload_scale": xs, "payload_json": args.payload_json, "payload_key": args.payload_key,
           "projections": []}
    single = sum(r["single_ms"] for r in rounds_of(d)) * args.scale
    for link in [float(x) for x in args.links.split(",")]:
        B = link * 1e9 * min(7, max(1, P - 1))
        t_after = t_ovl = t_half = 0.0
        for i, r in enumerate(rounds_of(d)):
            c = r["rank_ms_max"] * args.scale
            x = r["payload_bytes_max"] * xs * args.scale / B * 1e3
            hst = args.host_us * 1e-3
            t_after += c + x + hst
            t_ovl += max(c, x) + hst
            if h:
                hr = rounds_of(h)[i]
                # a GPU holds two lane-half ranks: both halves' kernels and payloads
                c2 = 2 * hr["rank_ms_mean"] * args.scale if hr["rank_ms_max"] < 1.2 * hr["rank_ms_mean"] else \
                    (hr["rank_ms_max"] + hr["rank_ms_mean"]) * args.scale
                x2 = 2 * hr["payload_bytes_max"] * xs * args.scale / B * 1e3
                t_half += max(c2, x2) + hst
        p = {"link_GBps": link, "single_ms": single, "exchange_after_ms": t_after,
             "speedup_exchange_after": single / t_after, "overlap_bound_ms": t_ovl,
             "speedup_overlap_bound": single / t_ovl}
        if h:
            p.update({"halves_ms": t_half, "speedup_halves": single / t_half})
        out["projections"].append(p)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
