"""The full-size O2 records (tests/golden/fullsize_*.json, made by
tests/golden/make_fullsize_golden.py on the GPU box's host cores) against the
size-independent properties of broadcast.go's algorithm, and the record
maker's lane-group split against one O2 engine at a small size.

The GPU suite (tests/test_gpu_fullsize.py) and bench.py's legs diff the HIP
engine against these records round by round."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, REPO

MAKER = os.path.join(GOLDEN, "make_fullsize_golden.py")


def _load(name):
    path = os.path.join(GOLDEN, f"fullsize_{name}.json")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    return json.load(open(path))


def _ack(rounds):
    for a, b in zip(rounds, rounds[1:]):
        assert b["acks"] == a["fwd_delivered"] + a["push_delivered"], b["round"]


def test_c5_record_properties():
    g = _load("c5")
    rs, V, K = g["rounds"], g["nodes"], g["lanes"]
    assert V == 1 << 30 and K == 64
    assert rs[-1]["new_bits"] == 0 and all(r["new_bits"] for r in rs[:-1])
    assert all(r["syncs_fired"] == 0 for r in rs)  # quiescence before the first timer (round 20)
    assert sum(r["new_bits"] for r in rs) == V * K  # P1: the grid spans every node
    assert sum(r["fwd_sent"] for r in rs) == K * (g["nnz"] - (V - 1))  # KAT-3
    _ack(rs)


def test_c3_record_properties():
    g = _load("c3")
    rs, V, K = g["rounds"], g["nodes"], g["lanes"]
    assert (V, K, g["windows"]) == (10_000_000, 1024, [[2, 12, g["seed"] ^ 0x5EED]])
    assert sum(r["new_bits"] for r in rs) == V * K  # P1 after the heal
    assert sum(r["dropped"] for r in rs[2:13]) > 0  # the window cut messages
    last = max(r["round"] for r in rs if r["new_bits"])
    assert last >= 20 and rs[-1]["new_bits"] == 0  # the heal needed the timers
    _ack(rs)


def test_c4_record_properties():
    g = _load("c4")
    rs = g["rounds"]
    assert (g["nodes"], g["lanes"], g["lane_groups"]) == (100_000_000, 4096, 4)
    assert rs[-1]["new_bits"] == 0
    assert all(r["syncs_fired"] == 0 for r in rs)
    _ack(rs)


def test_lane_group_records_sum_to_one_engine(tmp_path):
    """make_fullsize_golden.py's C4 split (4 lane-group O2 engines, run as two
    partial records and merged) equals one O2 engine over all 4096 lanes, every
    round, at 2·10^5 nodes."""
    env = dict(os.environ, GG_CPU_THREADS="4")
    run = lambda *a: subprocess.run([sys.executable, MAKER, "C4", "--size", "200000", *a], check=True,  # noqa: E731
                                    cwd=REPO, env=env, capture_output=True, text=True)
    split, whole = tmp_path / "split", tmp_path / "whole"
    run("--lane-groups", "4", "--groups", "0,1", "--outdir", str(split))
    run("--lane-groups", "4", "--groups", "2,3", "--outdir", str(split))
    run("--merge", "--outdir", str(split))
    run("--outdir", str(whole))
    a = json.load(open(split / "fullsize_c4.json"))["rounds"]
    b = json.load(open(whole / "fullsize_c4.json"))["rounds"]
    assert len(a) == len(b) > 3
    assert a == b
