#!/usr/bin/env python3
"""Generate tests/golden/bench_c2.json: the bench's C2 workload (bench.py: tree4
of 2^20 nodes per GPU, 1024 values broadcast in round 0 at seeded uniform
nodes, sync on with the engine's default timers) run by the CPU oracle O2 to
quiescence for world sizes 1, 2, 4 and 8 (V = 2^20 x N): every round's
counters and delivery hash. bench.py checks each timed episode's global
counters against the entry for its node count, so a multi-GPU line is checked
against O2 itself and not only against one engine of the same build.
Usage: python tests/golden/make_bench_golden.py [N ...]   (from the repo root)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "gossip-glomers-distributed-systems_amd")]

from ggamd import topology as T  # noqa: E402
from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402

CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
OUT = os.path.join(HERE, "bench_c2.json")


def run(world: int, K: int = 1024) -> dict:
    V = (1 << 20) * world
    seed = BASE_SEED + 2
    e = Engine(V, K, seed=seed, enable_sync=True, library=CPU_LIB)
    e.topology(T.tree(V, 4))
    inject(e, injection_arrays(uniform_injections(V, K, seed)))
    rounds = []
    while True:  # bench.py's quiescence rule: the first round after round 0 with no new bits
        s = e.step(1)[0]
        rounds.append({f: int(s[f]) for f in ("round",) + tuple(COUNT_FIELDS)})
        if s["new_bits"] == 0 and len(rounds) > 1:
            break
    e.close()
    return {"nodes": V, "lanes": K, "seed": seed, "rounds": rounds}


def main():
    worlds = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    data = json.load(open(OUT)) if os.path.exists(OUT) else {"generator": "tests/golden/make_bench_golden.py",
                                                             "oracle": "O2 (oracle/o2_bitset.cpp)", "runs": {}}
    for w in worlds:
        t = time.time()
        data["runs"][str(w)] = run(w)
        print(f"world {w}: {len(data['runs'][str(w)]['rounds'])} rounds in {time.time() - t:.1f} s", flush=True)
    with open(OUT, "w") as f:
        json.dump(data, f, indent=0)


if __name__ == "__main__":
    main()
