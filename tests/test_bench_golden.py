"""tests/golden/bench_c2.json (the O2 counters bench.py checks its episodes
against) matches O2 run now, for the one-GPU workload (2^20 nodes, ~3 s)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


def test_bench_golden_world1_matches_o2():
    import make_bench_golden as m
    data = json.load(open(m.OUT))
    assert set(data["runs"]) >= {"1", "2", "4", "8"}
    for w, run in data["runs"].items():
        assert run["nodes"] == (1 << 20) * int(w) and run["lanes"] == 1024
        assert run["rounds"][-1]["new_bits"] == 0
        assert sum(r["new_bits"] for r in run["rounds"]) == run["nodes"] * 1024  # P1: a tree is connected
    assert m.run(1) == data["runs"]["1"]
