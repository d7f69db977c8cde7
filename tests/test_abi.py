"""C-ABI checks that need no GPU: libbfsx.so loads, exports every symbol include/bfsx.h declares,
and its host-side parser (GraphFileUtil.convert semantics) agrees with the oracle, including the
reference's error behaviour on malformed input (GraphFileUtil.java:45-66)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_py as O
from conftest import ROOT, load_bfsx

HEADER = os.path.join(ROOT, "include", "bfsx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bfsx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    bfsx = load_bfsx()
    L = bfsx.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n  # ctypes attribute lookup = dlsym
    assert sorted(bfsx.EXPORTS) == names
    assert L.bfsx_abi_version() == 1


def test_exports_are_plain_c_symbols():
    out = os.popen(f"nm -D --defined-only {os.path.join(ROOT, 'bfs-with-mapreduce_amd', 'libbfsx.so')}").read()
    for n in declared_functions():
        assert re.search(rf"\bT {n}$", out, flags=re.M), n


@pytest.mark.parametrize("name", ["tinyCG.txt", "mediumG.txt", "tinyG.txt"])
def test_parser_matches_oracle(name):
    bfsx = load_bfsx()
    p = os.path.join(ROOT, "tests", "golden", name)
    nv, u, v = bfsx.parse_algs4(p)
    nv2, u2, v2 = O.load_graphfileutil(p)
    assert nv == nv2 and np.array_equal(u, u2) and np.array_equal(v, v2)


MALFORMED = {
    "ok_crlf": "3\r\n2\r\n0 1\r\n1 2\r\n",
    "ok_cr_only": "3\r2\r0 1\r1 2",
    "ok_extra_tokens": "3\n9\n0 1 7\n1 2 x\n",  # tokens beyond the second are ignored
    "ok_plus_sign": "3\n2\n+0 1\n1 +2\n",
    "ok_self_loop_dup": "3\n4\n0 0\n0 1\n1 0\n0 1\n",
    "ok_edge_count_ignored": "3\nbanana\n0 1\n",
    "ok_v0": "0\n1\n0 0\n",  # vertex 0 always exists
    "ok_no_edges": "5\n0\n",
    "ok_only_header": "5",
    "empty_file": "",
    "bad_vcount": "x\n0\n",
    "neg_vcount": "-1\n0\n",
    "vcount_space": " 3\n0\n",
    "double_space": "3\n1\n0  1\n",
    "one_token": "3\n1\n0\n",
    "empty_line": "3\n1\n0 1\n\n",
    "range_hi": "3\n1\n0 3\n",
    "range_neg": "3\n1\n-1 0\n",
    "overflow": "3\n1\n0 2147483648\n",
    "tab_sep": "3\n1\n0\t1\n",
    "ok_trailing_space": "3\n1\n0 1 \n",  # ["0","1",""]: get(0), get(1) parse fine
}


@pytest.mark.parametrize("case", sorted(MALFORMED))
def test_parser_error_behaviour_matches_reference_semantics(tmp_path, case):
    bfsx = load_bfsx()
    p = tmp_path / f"{case}.txt"
    p.write_bytes(MALFORMED[case].encode())
    try:
        got = bfsx.parse_algs4(str(p))
        got_rc = 0
    except bfsx.BfsxError as e:
        got_rc, got = e.code, None
    try:
        exp = O.load_graphfileutil(str(p))
        exp_rc = 0
    except O.OracleError as e:
        exp_rc, exp = e.code, None
    assert got_rc == exp_rc, (got_rc, exp_rc)
    if case.startswith("ok_"):
        assert got_rc == 0
        assert got[0] == exp[0] and np.array_equal(got[1], exp[1]) and np.array_equal(got[2], exp[2])
    else:
        assert got_rc < 0


def test_missing_file_is_io_error():
    bfsx = load_bfsx()
    with pytest.raises(bfsx.BfsxError) as ei:
        bfsx.parse_algs4("/nonexistent/graph.txt")
    assert ei.value.code == bfsx.BFSX_E_IO


def test_init_without_gpu_fails_loudly():
    bfsx = load_bfsx()
    import torch  # noqa: F401  (device counting only; does not initialise HIP)
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(bfsx.BfsxError) as ei:
        bfsx.Context(0)
    assert ei.value.code == bfsx.BFSX_E_NODEV
