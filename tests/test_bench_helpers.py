"""CPU checks of bench.py's accounting (no GPU): the algorithmic-bytes model of a level,
the harmonic mean, and the PMC traffic lookup keyed by the kernel source hash."""
import importlib.util
import json
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bottom_up_level_bytes(bench):
    ls = {"direction": 2, "unvisited_in": 1000, "stage2": 100, "claims": 10, "walked": 50, "frontier_out": 600}
    nwords = 64
    # single device: a discovery stores its 4-B parent (the level record gives the distance)
    assert bench.level_bytes(ls, nwords) == 16 * 64 + 4 * 1000 + 16 * 100 + 8 * 10 + 4 * 50 + 4 * 600
    # a packed 8-B state store per discovery (round 3's pull levels)
    assert bench.level_bytes(ls, nwords, found_bytes=8) == 16 * 64 + 4 * 1000 + 16 * 100 + 8 * 10 + 4 * 50 + 8 * 600


def test_pull_level_bytes_with_provenance_codes(bench):
    """Round 5: a single-device pull level stores a 1-B code per discovery plus a 4-B parent for its
    explicit_parents; a partition's pull level stores every parent explicitly and no code (code_bytes 0)."""
    ls = {"direction": 2, "unvisited_in": 1000, "stage2": 100, "claims": 10, "walked": 50, "frontier_out": 600,
          "explicit_parents": 40}
    base = 16 * 64 + 4 * 1000 + 16 * 100 + 8 * 10 + 4 * 50
    assert bench.level_bytes(ls, 64) == base + 1 * 600 + 4 * 40
    dist = dict(ls, explicit_parents=600)
    assert bench.level_bytes(dist, 64, code_bytes=0) == base + 4 * 600
    hy = {"direction": 3, "unvisited_in": 1000, "scanned": 300, "frontier_out": 20, "explicit_parents": 5}
    assert bench.level_bytes(hy, 64) == 16 * 64 + 4 * 1000 + 4 * 300 + 20 + 4 * 5
    acct = bench.LevelAccount(64, 4, code_bytes=0)
    acct.add([dict(dist, kernel_ms=0.1)])
    assert acct.bu_bytes == base + 4 * 600


def test_top_down_level_bytes(bench):
    ls = {"direction": 1, "frontier_in": 10, "mf_in": 300, "frontier_out": 20}
    # uint32 row offsets (the default below 2^32 adjacency entries), then int64 offsets
    assert bench.level_bytes(ls, 1) == 12 * 10 + 4 * 300 + 20 * 20
    assert bench.level_bytes(ls, 1, off_bytes=8) == 20 * 10 + 4 * 300 + 28 * 20


def test_hybrid_level_bytes(bench):
    ls = {"direction": 3, "unvisited_in": 1000, "scanned": 300, "frontier_out": 20}
    # both halves of a hybrid level store the 4-B parent: found_bytes per discovery, like a pull level
    assert bench.level_bytes(ls, 64) == 16 * 64 + 4 * 1000 + 4 * 300 + 4 * 20
    assert bench.level_bytes(ls, 64, found_bytes=8) == 16 * 64 + 4 * 1000 + 4 * 300 + 8 * 20


def test_level_account_whole_bfs(bench):
    acct = bench.LevelAccount(64, 4)
    bu = {"direction": 2, "unvisited_in": 1000, "stage2": 100, "claims": 10, "walked": 50, "frontier_out": 600,
          "kernel_ms": 0.5}
    td = {"direction": 1, "frontier_in": 10, "mf_in": 300, "frontier_out": 20, "kernel_ms": 0.1}
    acct.add([td, bu])
    assert acct.bu_launches == 1 and acct.bu_bytes == bench.level_bytes(bu, 64)
    assert acct.all_bytes == bench.level_bytes(bu, 64) + bench.level_bytes(td, 64)
    w = acct.whole(2.0, 1)  # 2 ms for one BFS
    assert abs(w["achieved"] - round(acct.all_bytes / 2e-3 / 1e9, 1)) < 1e-9
    assert bench.edge_scan_equivalent(1 << 20, 1 << 16, 1.0)["frac_of_peak"] > 0


def test_account_levels_decodes_raw_records(bench):
    """The timed loop keeps one raw LevelStat blob per BFS (Graph.level_stats_raw); account_levels decodes them
    after the region into the same account that the per-BFS dicts would give, keeping roots for --levels-json."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(ROOT, "bfs-with-mapreduce_amd"))
    from bfsx import Graph, LevelStat
    recs = [dict(direction=1, frontier_in=10, mf_in=300, frontier_out=20, kernel_ms=0.1),
            dict(direction=2, unvisited_in=1000, stage2=100, claims=10, walked=1 << 40, frontier_out=600,
                 kernel_ms=0.5)]
    buf = (LevelStat * 2)()
    for i, r in enumerate(recs):
        for k, v in r.items():
            setattr(buf[i], k, v)
    blob = C.string_at(buf, 2 * C.sizeof(LevelStat))
    a, b = bench.LevelAccount(64, 4), bench.LevelAccount(64, 4)
    kept = bench.account_levels(a, Graph, [7, 9], [blob, blob[:C.sizeof(LevelStat)]], True)
    b.add(Graph.level_stats_decode(blob))
    b.add(Graph.level_stats_decode(blob)[:1])
    assert (a.all_bytes, a.bu_bytes, a.bu_ms, a.bu_launches) == (b.all_bytes, b.bu_bytes, b.bu_ms, b.bu_launches)
    assert [k["root"] for k in kept] == [7, 7, 9] and kept[1]["walked"] == 1 << 40
    assert bench.account_levels(bench.LevelAccount(64, 4), Graph, [7], [b""], False) == []


def test_hmean(bench):
    assert bench.hmean([1.0, 1.0]) == 1.0
    assert abs(bench.hmean([1.0, 3.0]) - 1.5) < 1e-12


def test_measured_traffic_requires_matching_source(bench, tmp_path, monkeypatch):
    """A PMC summary counts only while the BFS kernel sources (bench.BFS_SRCS) still hash to the source it was
    measured on; of several k_bu instantiations the one with the most launches is reported."""
    import hashlib
    h = hashlib.sha256()
    for f in bench.BFS_SRCS:
        h.update(open(os.path.join(ROOT, "bfs-with-mapreduce_amd", "csrc", f), "rb").read())
    sha = h.hexdigest()[:16]
    assert sha == bench.bfs_src_sha()
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"bfs_src_sha": sha, "fetch_correction": 2.0,
           "kernels": {"k_bu<a, true>": {"launches": 2, "traffic_B": 9e9, "traffic_raw_B": 5e9, "avg_ms_trace": 1.0},
                       "k_bu<a, false>": {"launches": 90, "traffic_B": 1.2e9, "traffic_raw_B": 7e8,
                                          "avg_ms_trace": 0.25}}}
    (prof / "zz_hbm.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "PKG", os.path.join(ROOT, "bfs-with-mapreduce_amd"))
    out = bench.measured_traffic()
    assert out["traffic"] == 1200.0 and out["traffic_GBs"] == 4800.0
    # and only for the graph size it was measured on (a scale-26 profile says nothing about scale 30)
    rec["nwords"] = 1 << 20
    (prof / "zz_hbm.json").write_text(json.dumps(rec))
    assert bench.measured_traffic(nwords=1 << 20)["traffic"] == 1200.0
    assert bench.measured_traffic(nwords=1 << 24)["traffic"] is None
    rec["bfs_src_sha"] = "0" * 16
    (prof / "zz_hbm.json").write_text(json.dumps(rec))
    assert bench.measured_traffic()["traffic"] is None


def test_pick_roots_skips_tiny_components(bench):
    """Roots in components of under 1/1000 of the tuples are skipped (and listed); the rest keep the
    sampling order; a graph without tiny components keeps exactly the first roots."""
    class G:
        def sample_roots(self, n, seed):
            return list(range(100, 100 + n))

    class A:
        roots, root_seed = 5, 1

    m = 10_000
    small = {101: 3, 104: 9}
    calls = []
    roots, mcomp, errors, skipped = bench.pick_roots(
        A, G(), m, lambda r: small.get(r, 9_000), lambda: calls.append(1) or 0)
    assert roots == [100, 102, 103, 105, 106]
    assert skipped == [{"root": 101, "m_comp": 3}, {"root": 104, "m_comp": 9}]
    assert errors == 0 and len(calls) == 5 and mcomp[100] == 9_000
    roots, _, _, skipped = bench.pick_roots(A, G(), m, lambda r: 10, lambda: 0)
    assert roots == [100, 101, 102, 103, 104] and skipped == []
