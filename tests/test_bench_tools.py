"""CPU tests of the measurement plumbing: tools/traffic.py (PMC passes ->
profiles/traffic*.json), tools/request_ceiling.py (the random-row request
ceiling) and bench.py's per-episode normalisation of both (pmc_traffic,
roofline.line_frac). Synthetic counter CSVs in rocprofv3's column layout."""
import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _passes(tmp_path, episodes=3):
    """FETCH / WRITE / request passes of a run with `episodes` episodes (+1
    install reset), two stream kernels per round, 4 rounds per episode."""
    fetch, write, req = [], [], []
    d = 0
    for _ in range(episodes + 1):
        fetch.append(dict(Dispatch_Id=d, Kernel_Name="gg::reset_state(gg::ResetArgs)", Counter_Name="FETCH_SIZE",
                          Counter_Value=1.0))
        write.append(dict(Dispatch_Id=d, Kernel_Name="gg::reset_state(gg::ResetArgs)", Counter_Name="WRITE_SIZE",
                          Counter_Value=100.0))
        req += [dict(Dispatch_Id=d, Kernel_Name="gg::reset_state(gg::ResetArgs)", Counter_Name=c, Counter_Value=v)
                for c, v in (("TCC_EA0_RDREQ_sum", 0.0), ("TCC_EA0_WRREQ_sum", 1600.0))]
        d += 1
    for _ in range(episodes * 4):
        for k, fk, wk, rd, wr in (("void gg::expand_stream_db<8, 2, 3>(gg::RoundArgs)", 1000.0, 500.0, 16000.0, 8000.0),
                                  ("void gg::expand_stream_db_mark<8, 2>(gg::RoundArgs)", 10.0, 5.0, 160.0, 80.0)):
            fetch.append(dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name="FETCH_SIZE", Counter_Value=fk))
            write.append(dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name="WRITE_SIZE", Counter_Value=wk))
            req += [dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name="TCC_EA0_RDREQ_sum", Counter_Value=rd),
                    dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name="TCC_EA0_WRREQ_sum", Counter_Value=wr)]
            d += 1
    paths = [tmp_path / n for n in ("fetch.csv", "write.csv", "req.csv")]
    for p, rows in zip(paths, (fetch, write, req)):
        _csv(p, rows)
    return paths


def test_traffic_json_and_bench_normalisation(tmp_path, monkeypatch):
    f, w, r = _passes(tmp_path)
    out = tmp_path / "traffic_C2.json"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "traffic.py"), str(f), str(w), "test", str(out),
                           "C2", "--req", str(r)], stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    k = d["kernels"]["void gg::expand_stream_db<8, 2, 3>(gg::RoundArgs)"]
    assert k["dispatches"] == 12 and k["traffic_bytes_per_dispatch"] == (2 * 1000.0 + 500.0) * 1024
    assert k["rd_requests_per_dispatch"] == 16000.0 and k["wr_requests_per_dispatch"] == 8000.0
    assert d["shape"] == {"config": "C2", "world": 1, "parts": 1, "halves": 1, "nodes": 1 << 20, "lanes": 1024}

    sys.path.insert(0, REPO)
    import bench
    monkeypatch.setitem(bench.TRAFFIC_JSON, "C2", str(out))
    per_ep, src, reqs = bench.pmc_traffic("stream", d["shape"])
    # 3 episodes (4 resets less the install's), 4 rounds each, both kernels every round
    want_bytes = 12 * ((2 * 1000.0 + 500.0) + (2 * 10.0 + 5.0)) * 1024 / 3
    assert per_ep == pytest.approx(want_bytes) and "3 episodes" in src
    assert reqs[0] == pytest.approx(12 * (16000 + 160) / 3) and reqs[1] == pytest.approx(12 * (8000 + 80) / 3)
    # another shape: no traffic, and no line_frac
    other = dict(d["shape"], nodes=1 << 21)
    assert bench.pmc_traffic("stream", other)[0] is None

    # roofline over synthetic rounds: line_frac = (reads at the read ceiling + writes at the
    # write ceiling) per episode / the kind's time per episode
    rounds = [{"round": i % 4, "kernel_ms": 0.5, "prep_ms": 0.0, "expand_ms": 0.0, "stream_ms": 0.4,
               "prep_bytes": 0, "expand_bytes": 0, "stream_bytes": 10 ** 8, "work_gathers": 10, "work_rows": 10}
              for i in range(12)]
    ceil = tmp_path / "ceiling.json"
    ceil.write_text(json.dumps({"requests_per_s": 5e10, "write_requests_per_s": 8e10}))
    monkeypatch.setattr(bench, "REQ_CEILING_JSON", str(ceil))
    roof = bench.roofline(rounds, 16, 1 << 20, 2 * (1 << 20), d["shape"], 3)
    assert roof["line_frac"] == pytest.approx((reqs[0] / 5e10 + reqs[1] / 8e10) / (4 * 0.4e-3))
    assert roof["line_read_frac"] == pytest.approx(reqs[0] / 5e10 / (4 * 0.4e-3))
    assert roof["line_write_frac"] == pytest.approx(reqs[1] / 8e10 / (4 * 0.4e-3))
    assert roof["traffic"] == pytest.approx(per_ep / 4)
    roof2 = bench.roofline(rounds, 16, 1 << 20, 2 * (1 << 20), other, 3)
    assert roof2["line_frac"] is None and "line_model" not in roof2


def test_request_ceiling(tmp_path):
    stdout = tmp_path / "gather.txt"
    stdout.write_text("calibrate rows  64 B G= 4 rows_per_dispatch 1000 rows_per_s 4.0e+10\n"
                      "calibrate rows 512 B G=32 rows_per_dispatch 1000 rows_per_s 1.0e+10\n"
                      "calibrate writes  64 B G= 4 rows_per_dispatch 1000 rows_per_s 5.0e+10\n"
                      "calibrate seqwrite bytes_per_dispatch 2000000 bytes_per_s 5.0e+12\n"
                      "calibrate rows_mall  64 B G= 4 rows_per_dispatch 1000 rows_per_s 6.0e+10\n"
                      "calibrate writes_mall  64 B G= 4 rows_per_dispatch 1000 rows_per_s 5.5e+10\n"
                      "calibrate seqwrite_mall bytes_per_dispatch 1000000 bytes_per_s 6.0e+12\n")
    rows = []
    g = "(uint4 const*, unsigned int const*, unsigned long, uint4*)"
    for d, (name, rd) in enumerate((("void gather<4, 8, 0>" + g, 1050), ("void gather<32, 8, 0>" + g, 4050),
                                    ("void gather<4, 8, 1>" + g, 1020))):
        rows += [dict(Dispatch_Id=d, Kernel_Name=name, Counter_Name="TCC_EA0_RDREQ_sum", Counter_Value=rd),
                 dict(Dispatch_Id=d, Kernel_Name=name, Counter_Name="TCC_EA0_WRREQ_sum", Counter_Value=0)]
    sc = "(uint4*, unsigned int const*, unsigned long)"
    for d, (name, wr) in enumerate((("void scatter<4, 8, 0>" + sc, 1100), ("void seqwrite<0>(uint4*, unsigned long)", 32000),
                                    ("void scatter<4, 8, 1>" + sc, 1000), ("void seqwrite<1>(uint4*, unsigned long)", 16000)),
                                   start=3):
        rows += [dict(Dispatch_Id=d, Kernel_Name=name, Counter_Name="TCC_EA0_RDREQ_sum", Counter_Value=0),
                 dict(Dispatch_Id=d, Kernel_Name=name, Counter_Name="TCC_EA0_WRREQ_sum", Counter_Value=wr)]
    _csv(tmp_path / "req.csv", rows)
    out = tmp_path / "ceiling.json"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "request_ceiling.py"), str(stdout),
                           str(tmp_path / "req.csv"), str(out)], stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    by = {(r["row_bytes"], "HBM" in r["table"]): r for r in d["rows"]}
    assert by[64, True]["requests_per_row"] == pytest.approx(1.05)
    assert by[512, True]["requests_per_row"] == pytest.approx(4.05)
    assert by[64, False]["requests_per_row"] == pytest.approx(1.02)
    # each direction's ceiling: the highest rate over both tables
    assert d["requests_per_s"] == pytest.approx(max(4.0e10 * 1.05, 1.0e10 * 4.05, 6.0e10 * 1.02))
    wby = {"HBM" in r["table"]: r for r in d["write_rows"]}
    assert wby[True]["requests_per_row"] == pytest.approx(1.1) and wby[False]["requests_per_row"] == pytest.approx(1.0)
    sw = {"HBM" in r["table"]: r for r in d["write_sweeps"]}
    assert sw[True]["requests_per_s"] == pytest.approx(32000 / (2e6 / 5e12))
    assert sw[False]["requests_per_s"] == pytest.approx(16000 / (1e6 / 6e12))
    assert d["write_requests_per_s"] == pytest.approx(max(5e10 * 1.1, 5.5e10, 32000 / (2e6 / 5e12), 16000 / (1e6 / 6e12)))
