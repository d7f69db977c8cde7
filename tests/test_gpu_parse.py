"""K0, the GPU tokenizer of algs4 edge lists (kernels_parse.hip), against the host parser and the oracle.

The host parser is itself pinned to GraphFileUtil.convert's semantics (tests/test_abi.py); the GPU path
must give the same tuples, the same error code and the same first bad line number on every input,
including the malformed cases, CR / CRLF terminators and files without a final newline."""
import os

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN
from test_abi import MALFORMED, malformed_bytes

pytestmark = pytest.mark.gpu


def both(bfsx, ctx, path):
    out = []
    for f in (lambda p: bfsx.parse_algs4(p), lambda p: ctx.parse_algs4_gpu(p)):
        try:
            out.append((0, f(path), ""))
        except bfsx.BfsxError as e:
            out.append((e.code, None, str(e)))
    return out


@pytest.mark.parametrize("name", ["tinyCG.txt", "mediumG.txt", "tinyG.txt"])
def test_gpu_parse_reference_files(bfsx, ctx, name):
    p = os.path.join(GOLDEN, name)
    (rc_h, h, _), (rc_g, g, _) = both(bfsx, ctx, p)
    assert rc_h == rc_g == 0
    assert h[0] == g[0] and np.array_equal(h[1], g[1]) and np.array_equal(h[2], g[2])
    nv, u, v = O.load_graphfileutil(p)
    assert g[0] == nv and np.array_equal(g[1], u) and np.array_equal(g[2], v)


@pytest.mark.parametrize("case", sorted(MALFORMED))
def test_gpu_parse_malformed_like_host(bfsx, ctx, tmp_path, case):
    p = tmp_path / f"{case}.txt"
    p.write_bytes(malformed_bytes(case))
    (rc_h, h, msg_h), (rc_g, g, msg_g) = both(bfsx, ctx, str(p))
    assert rc_h == rc_g
    if rc_h == 0:
        assert h[0] == g[0] and np.array_equal(h[1], g[1]) and np.array_equal(h[2], g[2])
    elif "line " in msg_h:
        assert msg_h.split("line ")[1].split(":")[0] == msg_g.split("line ")[1].split(":")[0]  # same line


@pytest.mark.parametrize("term", ["\n", "\r\n", "\r"])
def test_gpu_parse_large_random_file(bfsx, ctx, tmp_path, term):
    rng = np.random.default_rng(len(term))
    nv, m = 50_000, 300_000
    u = rng.integers(0, nv, m)
    v = rng.integers(0, nv, m)
    extra = rng.random(m) < 0.1  # some lines carry ignored extra tokens / a trailing space
    lines = [f"{a} {b} 7" if x else f"{a} {b}" for a, b, x in zip(u, v, extra)]
    body = f"{nv}{term}{m}{term}" + term.join(lines)  # no final terminator
    p = tmp_path / "big.txt"
    p.write_bytes(body.encode())
    (rc_h, h, _), (rc_g, g, _) = both(bfsx, ctx, str(p))
    assert rc_h == rc_g == 0
    assert np.array_equal(g[1], u.astype(np.uint32)) and np.array_equal(g[2], v.astype(np.uint32))
    assert np.array_equal(h[1], g[1]) and np.array_equal(h[2], g[2])
    # a bad line deep in the file: same code and line number on both paths
    lines[123_456] = f"{nv} 0"  # id == V -> the reference's NullPointerException
    lines[200_000] = "1 x"      # later NumberFormatException must not win
    p.write_bytes((f"{nv}{term}{m}{term}" + term.join(lines)).encode())
    (rc_h, _, msg_h), (rc_g, _, msg_g) = both(bfsx, ctx, str(p))
    assert rc_h == rc_g == bfsx.BFSX_E_RANGE
    assert "line 123459" in msg_h and "line 123459" in msg_g


def test_load_uses_gpu_tokenizer_end_to_end(ctx):
    """bfsx_graph_load_algs4 (GPU tokenizer -> device CSR) gives the reference distances."""
    path = os.path.join(GOLDEN, "mediumG.txt")
    with ctx.load_algs4(path) as g:
        d, _, st = g.bfs(0)
    ref = np.array([int(x.split()[1]) for x in open(os.path.join(GOLDEN, "mediumG.dist"))], np.int32)
    assert np.array_equal(d, ref) and st["levels"] == 14
