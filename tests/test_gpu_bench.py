"""bench.py's multi-rank code on one GPU: two ranks over gloo (every rank an
engine on cuda:0), the same headline, exchange validation, fallbacks and C4 /
C5 legs the driver's N-GPU runs take, at reduced leg sizes.

* the C2 headline over the device-driven exchange: one whole validation episode
  against O2 (tests/golden/bench_c2.json), then every timed episode against O2
  and one unsharded engine (round 5: replays of a batch captured in the
  validation episode read back garbage counters — the memset node — until the
  engine's own zeroing kernel replaced it);
* the legs: C3 (partition window healed by the timers), strong-scaling C4
  (2 vertex parts x 2 lane halves) and C5, each checked against one unsharded
  engine, P1 / KAT-3 / ACK;
* GG_BENCH_IPC_FAIL: a rank stops exchanging after 3 validation rounds; its
  peer's waits run out (lowered bound) and every rank rebuilds on the engine
  exchange, whose timed episodes still equal O2;
* GG_BENCH_EPISODES_FAIL: gg_dist_run_episodes fails on one rank after the
  validation; every rank rebuilds on the engine exchange.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from helpers import free_port
    return free_port()


def _bench(extra, env=None, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo", "--steps", "2", "--warmup", "2", "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, cwd=REPO, env=dict(os.environ, **(env or {})), capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line), r.stderr


def test_bench_two_ranks_with_legs():
    d, _ = _bench(["--c3-nodes", str(1 << 17), "--c4-nodes", str(1 << 18), "--c5-side", "512", "--leg-steps", "2"])
    c = d["config"]
    assert d["n_gpus"] == 2
    assert c["exchange"].startswith("device-driven"), c["exchange"]
    assert c["exchange_validation"]["result"] == "passed", c["exchange_validation"]
    assert c["check"] == "every round's global counters equal one unsharded engine"
    assert c["oracle_check"] and c["oracle_check"].startswith("all 2 timed episodes")
    assert c["shard"]["devices"] == 1 and c["shard"]["distinct_devices"] is False
    for name in ("C3", "C4", "C5"):
        leg = d["legs"][name]
        assert leg.get("error") is None, leg
        assert leg["check"] == "passed", leg["checks"]
        assert leg["checks"]["single_engine"].startswith("every round's global counters equal")
        assert leg["vertex_parts"] == 2 and leg["steps"] == 2
        assert leg["rounds_to_full_delivery"] >= 1
    assert d["legs"]["C4"]["lane_halves_per_gpu"] == 2
    assert d["legs"]["C5"]["checks"]["expected"]["deliveries"] == 512 * 512 * 64
    # C3: the partition window cut messages and the timers healed it (P1 after the heal)
    c3 = d["legs"]["C3"]
    assert c3["checks"]["expected"]["deliveries"] == (1 << 17) * 1024
    assert c3["rounds_to_full_delivery"] > 20


@pytest.mark.parametrize("hook", ["ipc_fail_round3", "episodes_fail"])
def test_bench_fallback_to_engine_exchange(hook):
    env = ({"GG_BENCH_IPC_FAIL": "1:3", "GG_IPC_SPIN_LIMIT": str(1 << 16)} if hook == "ipc_fail_round3"
           else {"GG_BENCH_EPISODES_FAIL": "1"})
    d, err = _bench(["--legs", "none"], env=env)
    c = d["config"]
    assert c["exchange"].startswith("engine sequencing"), c["exchange"]
    assert "rebuilt on --xchg engine" in (c["exchange_note"] or ""), c["exchange_note"]
    if hook == "ipc_fail_round3":
        assert c["exchange_validation"]["result"].startswith("failed on some rank"), c["exchange_validation"]
    assert c["check"] == "every round's global counters equal one unsharded engine"
    assert c["oracle_check"] and c["oracle_check"].startswith("all 2 timed episodes")
