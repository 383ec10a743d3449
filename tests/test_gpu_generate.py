"""On-device topology generators (include/gossip_gen.h) against the host
builders that define the graphs (host/topology.cpp).

1. CSR identity: gg_topology_generate followed by gg_topology_export gives the
   host builder's row_ptr and col exactly — every kind, edge sizes (1- and
   2-node trees, 2x2 grids, regular graphs small enough for self loops and
   duplicate pairs, R-MAT with rejection at non-power-of-two V and with hubs),
   the multi-part sort plan forced to tiny parts (full-size C5 needs 4 parts),
   and full-size C2 (2^20-node tree4) and a 2^20-node grid.
2. Same episodes: an engine whose topology was generated on the device and one
   given the host CSR through gg_topology run identical seeded episodes
   (sync, partitions) with bit-identical per-round counters and node sets;
   the R-MAT case has in/out hubs, so the hub plan built from the generated
   row pointers is exercised too. The CPU oracle O2 runs beside them on the
   host CSR.
"""
import numpy as np
import pytest

from ggamd import topology as T
from ggamd.engine import Engine
from ggamd.workload import uniform_injections
from helpers import diff_stats

pytestmark = pytest.mark.gpu

HOST = {
    "tree": lambda n, k, seed: T.tree(n, k),
    "random_regular": lambda n, k, seed: T.random_regular(n, k, seed),
    "rmat": lambda n, k, seed: T.rmat(n, k, seed=seed),
    "grid_links": lambda n, k, seed: T.grid_links(n, seed),
}
RMAT_ABC = dict(a=0.57, b=0.19, c=0.19)


def _generate(hip_lib, kind, n, k, seed, lanes=64, **kw):
    V = n * n if kind == "grid_links" else n
    e = Engine(V, lanes, seed=5, library=hip_lib, **kw)
    extra = RMAT_ABC if kind == "rmat" else {}
    nnz = e.generate(kind, n, k=k, seed=seed, **extra)
    return e, nnz


CASES = [
    ("tree", 1, 4, 0), ("tree", 2, 4, 0), ("tree", 25, 4, 0), ("tree", 1000, 3, 0), ("tree", 4097, 4, 0),
    ("tree", 300, 1, 0),
    ("random_regular", 2, 2, 11), ("random_regular", 3, 4, 12), ("random_regular", 17, 8, 13),
    ("random_regular", 5000, 8, 14), ("random_regular", 4099, 6, 15),
    ("rmat", 2, 4, 21), ("rmat", 3, 16, 22), ("rmat", 1000, 16, 23), ("rmat", 4096, 16, 24),
    ("rmat", 1 << 14, 16, 25), ("rmat", 12345, 8, 26),
    ("grid_links", 2, 0, 31), ("grid_links", 3, 0, 32), ("grid_links", 64, 0, 33), ("grid_links", 101, 0, 34),
]


@pytest.mark.parametrize("kind,n,k,seed", CASES, ids=[f"{c[0]}-{c[1]}-{c[2]}" for c in CASES])
def test_generated_csr_equals_host_builder(hip_lib, kind, n, k, seed):
    host = HOST[kind](n, k, seed)
    e, nnz = _generate(hip_lib, kind, n, k, seed)
    got = e.export_topology()
    assert nnz == host.nnz
    assert np.array_equal(got.row_ptr, host.row_ptr)
    assert np.array_equal(got.col, host.col)


MULTI = [("random_regular", 5000, 8, 14), ("rmat", 1 << 14, 16, 25), ("grid_links", 101, 0, 34),
         ("rmat", 3, 16, 22)]


@pytest.mark.parametrize("part_keys", [1, 1000, 20000])
@pytest.mark.parametrize("kind,n,k,seed", MULTI, ids=[f"{c[0]}-{c[1]}" for c in MULTI])
def test_generated_csr_in_many_sort_parts(hip_lib, monkeypatch, kind, n, k, seed, part_keys):
    """The row-range part plan (one radix sort per part, < 2^32 keys each at
    full size) forced down to tiny parts: same CSR as the host builder."""
    monkeypatch.setenv("GG_GEN_PART_KEYS", str(part_keys))
    host = HOST[kind](n, k, seed)
    e, nnz = _generate(hip_lib, kind, n, k, seed)
    got = e.export_topology()
    assert nnz == host.nnz
    assert np.array_equal(got.row_ptr, host.row_ptr)
    assert np.array_equal(got.col, host.col)


@pytest.mark.parametrize("kind,n", [("tree", 1 << 20), ("grid_links", 1024)])
def test_generated_csr_full_size(hip_lib, kind, n):
    host = HOST[kind](n, 4, 0x6A09E667F3BCC909 + 5)
    e, nnz = _generate(hip_lib, kind, n, 4, 0x6A09E667F3BCC909 + 5)
    got = e.export_topology()
    assert nnz == host.nnz
    assert np.array_equal(got.row_ptr, host.row_ptr)
    assert np.array_equal(got.col, host.col)


def test_host_csr_export_roundtrip(hip_lib):
    """gg_topology_export of a host-given symmetric topology returns it unchanged."""
    t = T.grid_links(20, 77)
    e = Engine(t.n_nodes, 64, library=hip_lib)
    e.topology(t)
    got = e.export_topology()
    assert np.array_equal(got.row_ptr, t.row_ptr) and np.array_equal(got.col, t.col)


def test_generate_rejects_bad_specs(hip_lib):
    e = Engine(100, 64, library=hip_lib)
    with pytest.raises(Exception, match="node count"):
        e.generate("tree", 99, k=4)
    with pytest.raises(Exception, match="even"):
        e.generate("random_regular", 100, k=3, seed=1)
    e2 = Engine(100, 64, library=hip_lib)
    e2.generate("tree", 100, k=4)  # a valid spec after nothing installed
    assert e2.export_topology().nnz == 198


EPISODES = [
    ("tree", 4096, 4, 0, 1024, None),
    ("grid_links", 64, 0, 33, 128, (3, 9, 0xBEEF)),
    ("random_regular", 4096, 8, 14, 256, (2, 8, 0xF00D)),
    ("rmat", 1 << 14, 16, 25, 512, None),
]


@pytest.mark.parametrize("kind,n,k,seed,W,window", EPISODES, ids=[e[0] for e in EPISODES])
def test_generated_topology_runs_identical_episodes(hip_lib, cpu_lib, kind, n, k, seed, W, window):
    host = HOST[kind](n, k, seed)
    V = host.n_nodes
    inj = uniform_injections(V, W // 2, 99 + n)
    engines = []
    for lib, gen in ((hip_lib, True), (hip_lib, False), (cpu_lib, False)):
        e = Engine(V, W, seed=7, sync_base=6, sync_jitter=4, enable_sync=True, library=lib)
        if gen:
            extra = RMAT_ABC if kind == "rmat" else {}
            e.generate(kind, n, k=k, seed=seed, **extra)
        else:
            e.topology(host)
        if window:
            e.partition_seeded(*window)
        for node, val, r in inj:
            e.broadcast(int(node), int(val), int(r))
        engines.append(e)
    st = [e.step(30) for e in engines]
    assert sum(s["new_bits"] for s in st[0]) > 0
    d = diff_stats(st[0], st[1])
    assert not d, d[:10]
    d = diff_stats(st[0], st[2])
    assert not d, d[:10]
    assert np.array_equal(engines[0].read_bits(), engines[1].read_bits())
    assert np.array_equal(engines[0].read_bits(), engines[2].read_bits())
