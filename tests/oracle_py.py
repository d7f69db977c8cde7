"""ctypes binding of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product path (libbfsx.so and its Python mirror) never does.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None

I64P = C.POINTER(C.c_int64)
U32P = C.POINTER(C.c_uint32)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        L.orc_load_graphfileutil.argtypes = [C.c_char_p, I64P, I64P, C.POINTER(U32P), C.POINTER(U32P)]
        L.orc_load_algs4_graph.argtypes = L.orc_load_graphfileutil.argtypes
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_build_sets.argtypes = [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                     C.POINTER(I64P), C.POINTER(U32P)]
        L.orc_mapreduce_bfs.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                        I64P, C.c_int]
        L.orc_algs4_bfs.argtypes = [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_void_p, C.c_void_p]
        L.orc_algs4_adj.argtypes = [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_void_p, C.c_int64]
        L.orc_algs4_adj.restype = C.c_int64
        L.orc_csr_bfs.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        L.orc_validate.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        L.orc_kronecker.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p]
        L.orc_kronecker_thresholds.argtypes = [U32P, U32P, U32P]
        L.orc_mcomp.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_mcomp.restype = C.c_int64
        L.orc_dist_sha256.argtypes = [C.c_int64, C.c_void_p, C.c_char_p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle error {code}")
        self.code = code


def _load(fn, path):
    nv, m = C.c_int64(), C.c_int64()
    up, vp = U32P(), U32P()
    rc = fn(path.encode(), C.byref(nv), C.byref(m), C.byref(up), C.byref(vp))
    if rc:
        raise OracleError(rc)
    u = np.ctypeslib.as_array(up, shape=(max(m.value, 1),))[: m.value].copy()
    v = np.ctypeslib.as_array(vp, shape=(max(m.value, 1),))[: m.value].copy()
    lib().orc_free(up)
    lib().orc_free(vp)
    return nv.value, u, v


def load_graphfileutil(path):
    """GraphFileUtil.convert parse semantics -> (nv, u, v)."""
    return _load(lib().orc_load_graphfileutil, path)


def load_algs4_graph(path):
    """algs4 Graph(In) parse semantics -> (nv, u, v)."""
    return _load(lib().orc_load_algs4_graph, path)


def build_sets(nv, u, v):
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    op, cp = I64P(), U32P()
    rc = lib().orc_build_sets(nv, len(u), _ptr(u), _ptr(v), C.byref(op), C.byref(cp))
    if rc:
        raise OracleError(rc)
    off = np.ctypeslib.as_array(op, shape=(nv + 1,)).copy()
    nnz = int(off[-1])
    col = np.ctypeslib.as_array(cp, shape=(max(nnz, 1),))[:nnz].copy()
    lib().orc_free(op)
    lib().orc_free(cp)
    return off, col


def mapreduce_bfs(nv, off, col, source=0, nthreads=0, max_iters=1 << 16):
    dist = np.empty(nv, np.int32)
    parent = np.empty(nv, np.int64)
    color = np.empty(nv, np.int8)
    gray = np.zeros(max_iters, np.int64)
    emits = np.zeros(max_iters, np.int64)
    iters = C.c_int64()
    rc = lib().orc_mapreduce_bfs(nv, _ptr(off), _ptr(col), source, _ptr(dist), _ptr(parent),
                                 _ptr(color), _ptr(gray), _ptr(emits), max_iters, C.byref(iters),
                                 nthreads)
    if rc:
        raise OracleError(rc)
    k = min(iters.value, max_iters)
    return dict(dist=dist, parent=parent, color=color, iters=iters.value, gray=gray[:k],
                emits=emits[:k])


def algs4_bfs(nv, u, v, source=0):
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    dist = np.empty(nv, np.int32)
    edge_to = np.empty(nv, np.int64)
    rc = lib().orc_algs4_bfs(nv, len(u), _ptr(u), _ptr(v), source, _ptr(dist), _ptr(edge_to))
    if rc:
        raise OracleError(rc)
    return dist, edge_to


def algs4_adj(nv, u, v, x):
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    out = np.empty(2 * len(u) + 1, np.uint32)
    k = lib().orc_algs4_adj(nv, len(u), _ptr(u), _ptr(v), x, _ptr(out), len(out))
    return out[:k].tolist()


def csr_bfs(nv, off, col, source):
    dist = np.empty(nv, np.int32)
    parent = np.empty(nv, np.int64)
    rc = lib().orc_csr_bfs(nv, _ptr(off), _ptr(col), source, _ptr(dist), _ptr(parent))
    if rc:
        raise OracleError(rc)
    return dist, parent


def validate(nv, off, col, source, dist, parent, rows_sorted=False):
    """Graph500 rules + BreadthFirstPaths.check (orc_validate bisects rows, so they are sorted here
    unless the caller says they already are: device rows are degree-ordered by default)."""
    if not rows_sorted:
        off = np.ascontiguousarray(off, dtype=np.int64)
        rows = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
        col = np.ascontiguousarray(col)[np.lexsort((col, rows))]
    dist = np.ascontiguousarray(dist, dtype=np.int32)
    parent = np.ascontiguousarray(parent, dtype=np.int64)
    return lib().orc_validate(nv, _ptr(off), _ptr(col), source, _ptr(dist), _ptr(parent))


def kronecker(scale, edgefactor, seed):
    m = edgefactor << scale
    u = np.empty(m, np.uint32)
    v = np.empty(m, np.uint32)
    lib().orc_kronecker(scale, edgefactor, seed, _ptr(u), _ptr(v))
    return u, v


def mcomp(u, v, dist):
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    return lib().orc_mcomp(len(u), _ptr(u), _ptr(v), _ptr(np.ascontiguousarray(dist, np.int32)))


def dist_sha256(dist):
    dist = np.ascontiguousarray(dist, dtype=np.int32)
    out = C.create_string_buffer(65)
    lib().orc_dist_sha256(len(dist), _ptr(dist), out)
    return out.value.decode()
