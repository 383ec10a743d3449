"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracles reproduce their committed fixtures exactly.
GPU: the HIP engine reproduces every fixture exactly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from ggamd.engine import COUNT_FIELDS
from helpers import c1_scenario, make_engine, make_o1

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def _check_stats(gold, st):
    assert len(gold["stats"]) == len(st)
    for g, s in zip(gold["stats"], st):
        for f in ["round"] + COUNT_FIELDS:
            assert g[f] == s[f], (g["round"], f, g[f], s[f])


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _scenario_4k(name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import scenario_4k
    return scenario_4k(name)


@pytest.mark.parametrize("name,part", [("c1_tree4", False), ("c1_tree4_bisect", True)])
def test_c1_o1_fixture(name, part):
    gold = _load(name)
    sc = c1_scenario(partition=part)
    o1 = make_o1(sc)
    _check_stats(gold, o1.step(sc.rounds))
    assert [o1.read(v) for v in range(25)] == gold["reads"]


@pytest.mark.parametrize("name,part", [("c1_tree4", False), ("c1_tree4_bisect", True)])
def test_c1_o2_fixture(cpu_lib, name, part):
    gold = _load(name)
    sc = c1_scenario(partition=part)
    e = make_engine(cpu_lib, sc)
    _check_stats(gold, e.step(sc.rounds))
    assert [e.read(v) for v in range(25)] == gold["reads"]
    assert e.delivery_rounds().tolist() == gold["delivery_rounds"]


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_4k_o2_fixture(cpu_lib, name):
    gold = _load(name + "_4k")
    sc = _scenario_4k(name)
    e = make_engine(cpu_lib, sc)
    _check_stats(gold, e.step(sc.rounds))
    assert _sha(e.read_bits()) == gold["sets_sha256"]
    assert _sha(e.delivery_rounds()) == gold["delivery_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_tree4", "c1_tree4_bisect", "c2_4k", "c3_4k", "c4_4k", "c5_4k"])
def test_gpu_fixture(hip_lib, name):
    gold = _load(name)
    if name.startswith("c1"):
        sc = c1_scenario(partition=name.endswith("bisect"))
    else:
        sc = _scenario_4k(name[:2])
    e = make_engine(hip_lib, sc)
    _check_stats(gold, e.step(sc.rounds))
    if name.startswith("c1"):
        assert [e.read(v) for v in range(25)] == gold["reads"]
        assert e.delivery_rounds().tolist() == gold["delivery_rounds"]
    else:
        assert _sha(e.read_bits()) == gold["sets_sha256"]
        assert _sha(e.delivery_rounds()) == gold["delivery_sha256"]
