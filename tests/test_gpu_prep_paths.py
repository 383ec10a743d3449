"""round_prep's grid-capped paths against the CPU oracle, round by round.

round_prep strides over the owned nodes with a capped grid (1024 blocks).
When the cap would need more than four passes, sparse lean rounds take four
nodes per thread from one 32-bit load of each flag array (the "quad" path,
DESIGN.md §7c); at the default cap only graphs above 2^20 nodes take it. The
cap is read once per process, so the case runs in a child process with
GG_PREP_BLOCKS=1 (a one-block grid): every graph above 1024 nodes then takes
the quad path in its sparse rounds, and the sync rounds take the one-node
path with many passes. Counters (including seen_hash), node sets and delivery
rounds must equal O2 in every round.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path[:0] = [%(tests)r, %(pkg)r, %(repo)r]
import numpy as np
from ggamd import topology as T
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine
scs = [
    Scenario(T.tree(5000, 4), 128, 24, uniform_injections(5000, 100, 3), seed=4, enable_sync=False),
    Scenario(T.random_regular(6000, 8, seed=5), 64, 16, uniform_injections(6000, 64, 6), seed=7,
             enable_sync=False),
    Scenario(T.grid_links(70, seed=8), 256, 30, uniform_injections(4900, 200, 9), seed=10,
             enable_sync=False),
    Scenario(T.tree(4100, 4), 1024, 40, uniform_injections(4100, 700, 11), seed=12, sync_base=9,
             sync_jitter=4),
]
bad = []
for k, sc in enumerate(scs):
    g = make_engine(%(hip)r, sc, device=0)
    c = make_engine(%(cpu)r, sc)
    for r in range(sc.rounds):  # round by round: a late candidate mark would show here
        d = diff_stats(g.step(1), c.step(1))
        if d:
            bad.append((k, d[:5]))
            break
        if r %% 4 == 3 and not np.array_equal(g.read_bits(), c.read_bits()):
            bad.append((k, "sets differ at round %%d" %% r))
            break
    if not np.array_equal(g.delivery_rounds(), c.delivery_rounds()):
        bad.append((k, "delivery rounds differ"))
    g.close(); c.close()
print(json.dumps(bad))
"""


def test_prep_quad_path_equals_oracle(hip_lib, cpu_lib):
    code = CHILD % {"tests": os.path.join(REPO, "tests"), "pkg": os.path.join(REPO, "gossip-glomers-distributed-systems_amd"),
                    "repo": REPO, "hip": hip_lib, "cpu": cpu_lib}
    env = dict(os.environ, GG_PREP_BLOCKS="1")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == []


@pytest.mark.parametrize("no_mark", ["0", "1"])
def test_marking_rounds_equal_oracle(hip_lib, cpu_lib, monkeypatch, no_mark):
    """Marking rounds (GG_PATH_NO_PREP): in double-buffered rounds before the
    timers the expand kernel marks the next round's candidates (a changed node
    and its receivers) and clears its flag byte of r-1, and those rounds launch
    no round_prep; GG_NO_MARK=1 keeps round_prep. Sparse and dense rounds,
    injections spread over the rounds, the hand-over to the timer rounds, one
    multi-round step and single steps: every round equals O2."""
    import random

    import numpy as np

    from ggamd import topology as T
    from ggamd.engine import PATH_DB, PATH_NO_PREP
    from ggamd.workload import uniform_injections
    from helpers import Scenario, diff_stats, make_engine
    monkeypatch.setenv("GG_NO_MARK", no_mark)
    monkeypatch.setenv("GG_DB", "1")
    rnd = random.Random(5)
    scs = [Scenario(T.tree(6000, 4), 256, 34, [(n, v, v % 7) for n, v, _ in uniform_injections(6000, 200, 1)],
                    seed=2, sync_base=14, sync_jitter=3),
           Scenario(T.random_regular(5000, 6, seed=3), 128, 30, [(rnd.randrange(5000), v, rnd.randrange(12))
                                                                  for v in range(120)], seed=4, sync_base=9),
           Scenario(T.grid_links(60, seed=5), 512, 26, uniform_injections(3600, 400, 6), seed=7, enable_sync=False)]
    for k, sc in enumerate(scs):
        c = make_engine(cpu_lib, sc)
        want = c.step(sc.rounds)
        for mode in ("whole", "single"):
            g = make_engine(hip_lib, sc, device=0)
            st = g.step(sc.rounds) if mode == "whole" else [g.step(1)[0] for _ in range(sc.rounds)]
            d = diff_stats(want, st)
            assert not d, (k, mode, d[:6])
            assert np.array_equal(g.read_bits(), c.read_bits()), (k, mode)
            assert np.array_equal(g.delivery_rounds(), c.delivery_rounds()), (k, mode)
            n_np = sum(1 for s in st if s["path"] & PATH_NO_PREP)
            assert any(s["path"] & PATH_DB for s in st), k
            assert (n_np > 3) if no_mark == "0" else (n_np == 0), (k, mode, [s["path"] for s in st])
            g.close()
        c.close()


@pytest.mark.parametrize("solo", ["learned", "mark", "db", "alt"])
def test_solo_marking_rounds_equal_oracle(hip_lib, cpu_lib, monkeypatch, solo):
    """Solo marking rounds (GG_PATH_SOLO): once a marking round has run, the
    engine launches only the expand kernel that run needed (the busy flag the
    kernels report) instead of both with one exiting at once. Any schedule is
    exact — a marking kernel in a busy round visits every node, a solo
    expand_stream_db visits every node and the round after it is dense — so the
    forced schedules (GG_SOLO = mark / db / alt, every marking round) must equal
    O2 as the learned one does: three episodes per scenario (the first learns,
    the second recaptures its batch with the schedule, the third replays it and
    runs through gg_run_episodes), every round against O2."""
    import random

    import numpy as np

    from ggamd import topology as T
    from ggamd.engine import PATH_NO_PREP, PATH_SOLO
    from ggamd.workload import inject, uniform_injections
    from helpers import Scenario, diff_stats, make_engine
    monkeypatch.setenv("GG_DB", "1")
    if solo != "learned":
        monkeypatch.setenv("GG_SOLO", solo)
    rnd = random.Random(9)
    scs = [Scenario(T.tree(6000, 4), 256, 34, uniform_injections(6000, 200, 1), seed=2, sync_base=14, sync_jitter=3),
           Scenario(T.tree(3000, 4), 128, 30, [(n, v, v % 5) for n, v, _ in uniform_injections(3000, 100, 4)],
                    seed=3, enable_sync=False),
           Scenario(T.random_regular(5000, 6, seed=3), 128, 24, [(rnd.randrange(5000), v, rnd.randrange(6))
                                                                 for v in range(120)], seed=4, sync_base=9),
           Scenario(T.grid_links(60, seed=5), 512, 26, uniform_injections(3600, 400, 6), seed=7, enable_sync=False)]
    for k, sc in enumerate(scs):
        c = make_engine(cpu_lib, sc)
        want = c.step(sc.rounds)
        g = make_engine(hip_lib, sc, device=0)
        runs = [g.step(sc.rounds)]
        g.reset()
        inject(g, sc.injections)
        runs.append(g.step(sc.rounds))
        g.reset()
        inject(g, sc.injections)
        runs += g.run_episodes(sc.rounds, 2)
        for j, st in enumerate(runs):
            d = diff_stats(want, st)
            assert not d, (k, j, d[:6])
        assert np.array_equal(g.read_bits(), c.read_bits()), k
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds()), k
        n_marking = sum(1 for s in runs[1] if s["path"] & PATH_NO_PREP)
        n_solo = [sum(1 for s in st if s["path"] & PATH_SOLO) for st in runs]
        if solo == "learned":  # (round 0 is always solo: nothing was active before it)
            assert n_solo[0] <= 1 and min(n_solo[1:]) >= 1, (k, n_solo, n_marking)
        else:
            assert min(n_solo) >= 1, (k, n_solo)
        g.close()
        c.close()


@pytest.mark.parametrize("mode", ["learned", "forced"])
def test_busy_rounds_without_list_equal_oracle(hip_lib, cpu_lib, monkeypatch, mode):
    """Lean streaming rounds that are not marking rounds (before the timers on
    non-marking engines, timer rounds, hub graphs) skip compact_round when the
    last run of the round was busy and run dense (RoundArgs::no_list); forced
    (GG_NO_LIST=1) every such round runs dense whatever it finds. Exact either
    way: three episodes per scenario (learning, recapture, replay through
    gg_run_episodes) against O2."""
    import random

    import numpy as np

    from ggamd import topology as T
    from ggamd.workload import inject, uniform_injections
    from helpers import Scenario, diff_stats, make_engine
    if mode == "forced":
        monkeypatch.setenv("GG_NO_LIST", "1")
    monkeypatch.setenv("GG_HUB_DEG", "16")
    rnd = random.Random(19)
    scs = [Scenario(T.tree(6000, 4), 256, 34, uniform_injections(6000, 200, 1), seed=2, sync_base=14, sync_jitter=3),
           Scenario(T.rmat(4096, 16, seed=41), 256, 16, uniform_injections(4096, 256, 42), seed=43, sync_base=9,
                    sync_jitter=2),
           Scenario(T.random_regular(5000, 6, seed=3), 128, 24, [(rnd.randrange(5000), v, rnd.randrange(6))
                                                                 for v in range(120)], seed=4, sync_base=9),
           Scenario(T.grid_links(60, seed=5), 64, 26, uniform_injections(3600, 64, 6), seed=7, enable_sync=False)]
    for k, sc in enumerate(scs):
        c = make_engine(cpu_lib, sc)
        want = c.step(sc.rounds)
        g = make_engine(hip_lib, sc, device=0)
        runs = [g.step(sc.rounds)]
        g.reset()
        inject(g, sc.injections)
        runs.append(g.step(sc.rounds))
        g.reset()
        inject(g, sc.injections)
        runs += g.run_episodes(sc.rounds, 2)
        for j, st in enumerate(runs):
            d = diff_stats(want, st)
            assert not d, (k, j, d[:6])
        assert np.array_equal(g.read_bits(), c.read_bits()), k
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds()), k
        g.close()
        c.close()

