"""Thin ctypes binding of libbfsx.so (include/bfsx.h) used by tests, bench.py and smoke().

This is plumbing, not a fallback: every compute call goes to the HIP library, and loading fails
loudly when libbfsx.so is missing.  The reference-shaped host (BfsSpark / GraphFileUtil / Vertex /
Color / ServiceConfiguration) is the C++ twin in host/ (bfsx_spark); this module mirrors the C-ABI
one-to-one.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# BFSX_LIB: another build of the same library (A/B timing of two builds on one box)
LIB_PATH = os.environ.get("BFSX_LIB") or os.path.join(PKG_DIR, "libbfsx.so")
# the diagnostic build of the same sources (-DBFSX_DIAG): the test hooks and the encoded hub domain of graphs
# built without the relabel; a Context given one of DIAG_OPTIONS (or diag=True) runs on it
DIAG_LIB_PATH = os.environ.get("BFSX_DIAG_LIB") or os.path.join(PKG_DIR, "libbfsx_diag.so")
DIAG_OPTIONS = ("poison_queues", "test_overread", "bu_force_spill", "persist_abort_at", "check_retired", "fail_at",
                "slot_force", "race_probe")

BFSX_OK = 0
BFSX_E_IO = -1
BFSX_E_PARSE = -2
BFSX_E_RANGE = -3
BFSX_E_HIP = -4
BFSX_E_RCCL = -5
BFSX_E_OOM = -6
BFSX_E_ARG = -7
BFSX_E_NODEV = -8

DIR_AUTO, DIR_TOPDOWN, DIR_BOTTOMUP = 0, 1, 2
INF = 2147483647

# Every symbol include/bfsx.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "bfsx_abi_version", "bfsx_last_error", "bfsx_init", "bfsx_finalize", "bfsx_set_option",
    "bfsx_parse_algs4", "bfsx_parse_algs4_gpu", "bfsx_free_host", "bfsx_graph_load_algs4", "bfsx_graph_from_edges",
    "bfsx_graph_kronecker", "bfsx_kronecker_edges", "bfsx_graph_free", "bfsx_graph_nv",
    "bfsx_graph_nnz", "bfsx_graph_m", "bfsx_graph_csr", "bfsx_sample_roots", "bfsx_bfs",
    "bfsx_result", "bfsx_level_times", "bfsx_level_dirs", "bfsx_level_stats",
    "bfsx_device_synchronize", "bfsx_validate", "bfsx_validate_result",
    "bfsx_dist_graph_from_edges", "bfsx_dist_graph_kronecker", "bfsx_graph_partition", "bfsx_graph_degree",
    "bfsx_last_bfs_ms", "bfsx_last_unpack_ms", "bfsx_persist_fallbacks", "bfsx_comm_unique_id", "bfsx_comm_init", "bfsx_comm_local_group",
    "bfsx_dist_bfs", "bfsx_init_group", "bfsx_group_size", "bfsx_dist_graph_load_algs4", "bfsx_last_resolve_ms",
    "bfsx_comm_times",
]
# test-only level primitives (include/bfsx_levels.h): exported for tests/dist_driver.py, not product ABI
TEST_EXPORTS = [
    "bfsx_dist_begin", "bfsx_dist_frontier_info", "bfsx_dist_td_expand", "bfsx_dist_td_claim",
    "bfsx_dist_frontier_slice", "bfsx_dist_bu_step", "bfsx_dist_level_end", "bfsx_dist_finish",
    "bfsx_dist_mcomp",
]
COMM_ID_BYTES = 128


class Stats(C.Structure):
    _fields_ = [
        ("levels", C.c_int32), ("topdown_levels", C.c_int32), ("bottomup_levels", C.c_int32),
        ("persist_retries", C.c_int32), ("reached", C.c_int64), ("m_comp", C.c_int64),
        ("edges_examined", C.c_int64), ("t_bfs_ms", C.c_double), ("t_total_ms", C.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class LevelStat(C.Structure):
    _fields_ = [
        ("direction", C.c_int32), ("level", C.c_int32), ("frontier_in", C.c_int64),
        ("frontier_out", C.c_int64), ("mf_in", C.c_int64), ("unvisited_in", C.c_int64),
        ("scanned", C.c_int64), ("claims", C.c_int64), ("kernel_ms", C.c_double), ("cum_ms", C.c_double),
        ("stage2", C.c_int64), ("walked", C.c_int64), ("explicit_parents", C.c_int64),
    ]


class BfsxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"bfsx error {code}: {msg}")
        self.code = code


_libs = {}
_VP = C.c_void_p
_U32PP = C.POINTER(C.POINTER(C.c_uint32))


def lib(diag=False):
    """The product library (libbfsx.so), or with diag=True its diagnostic build (libbfsx_diag.so).  Both can be
    loaded in one process (ctypes loads them RTLD_LOCAL); every handle belongs to the library that made it."""
    path = DIAG_LIB_PATH if diag else LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built: run `make` (or __graft_entry__.build())")
        _libs[path] = _bind(C.CDLL(path))
    return _libs[path]


def _bind(L):
    if True:
        L.bfsx_last_error.restype = C.c_char_p
        L.bfsx_init.argtypes = [C.c_int, C.POINTER(_VP)]
        L.bfsx_finalize.argtypes = [_VP]
        L.bfsx_finalize.restype = None
        L.bfsx_set_option.argtypes = [_VP, C.c_char_p, C.c_char_p]
        L.bfsx_parse_algs4.argtypes = [C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _U32PP, _U32PP]
        L.bfsx_parse_algs4_gpu.argtypes = [_VP, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _U32PP,
                                           _U32PP]
        L.bfsx_free_host.argtypes = [_VP]
        L.bfsx_free_host.restype = None
        L.bfsx_graph_load_algs4.argtypes = [_VP, C.c_char_p, C.POINTER(_VP)]
        L.bfsx_graph_from_edges.argtypes = [_VP, C.c_int64, _VP, _VP, C.c_int64, C.POINTER(_VP)]
        L.bfsx_graph_kronecker.argtypes = [_VP, C.c_int, C.c_int, C.c_uint64, C.POINTER(_VP)]
        L.bfsx_kronecker_edges.argtypes = [_VP, C.c_int, C.c_int, C.c_uint64, _VP, _VP]
        L.bfsx_graph_free.argtypes = [_VP]
        L.bfsx_graph_free.restype = None
        for f in ("bfsx_graph_nv", "bfsx_graph_nnz", "bfsx_graph_m"):
            getattr(L, f).argtypes = [_VP]
            getattr(L, f).restype = C.c_int64
        L.bfsx_graph_csr.argtypes = [_VP, _VP, _VP]
        L.bfsx_sample_roots.argtypes = [_VP, C.c_int, C.c_uint64, _VP]
        L.bfsx_bfs.argtypes = [_VP, C.c_int64, _VP, _VP, C.POINTER(Stats)]
        L.bfsx_result.argtypes = [_VP, _VP, _VP]
        L.bfsx_level_times.argtypes = [_VP, _VP, C.c_int]
        L.bfsx_level_dirs.argtypes = [_VP, _VP, C.c_int]
        L.bfsx_last_bfs_ms.argtypes = [_VP, C.POINTER(C.c_double)]
        L.bfsx_last_unpack_ms.argtypes = [_VP, C.POINTER(C.c_double)]
        if hasattr(L, "bfsx_last_resolve_ms") or not os.environ.get("BFSX_LIB"):  # an older build (A/B) may lack it
            L.bfsx_last_resolve_ms.argtypes = [_VP, C.POINTER(C.c_double)]
        if hasattr(L, "bfsx_persist_fallbacks") or not os.environ.get("BFSX_LIB"):  # an older build (A/B) may lack it
            L.bfsx_persist_fallbacks.argtypes = [_VP, C.POINTER(C.c_int64)]
        L.bfsx_level_stats.argtypes = [_VP, C.POINTER(LevelStat), C.c_int]
        if hasattr(L, "bfsx_comm_times") or not os.environ.get("BFSX_LIB"):  # an older build (A/B) may lack it
            L.bfsx_comm_times.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        L.bfsx_device_synchronize.argtypes = [_VP]
        I64P = C.POINTER(C.c_int64)
        L.bfsx_validate.argtypes = [_VP, C.c_int64, I64P, I64P, I64P, I64P]
        L.bfsx_validate_result.argtypes = [_VP, C.c_int64, _VP, _VP, I64P, I64P]
        L.bfsx_dist_graph_from_edges.argtypes = [_VP, C.c_int64, _VP, _VP, C.c_int64, C.c_int, C.c_int,
                                                 C.POINTER(_VP)]
        L.bfsx_dist_graph_kronecker.argtypes = [_VP, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, C.POINTER(_VP)]
        L.bfsx_graph_partition.argtypes = [_VP, I64P, I64P, I64P, I64P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.bfsx_graph_degree.argtypes = [_VP, C.c_int64, I64P]
        L.bfsx_dist_begin.argtypes = [_VP, C.c_int64, I64P]
        L.bfsx_dist_frontier_info.argtypes = [_VP, I64P, I64P]
        L.bfsx_dist_td_expand.argtypes = [_VP, _VP, C.c_int64, _VP]
        L.bfsx_dist_td_claim.argtypes = [_VP, _VP, C.c_int64]
        L.bfsx_dist_frontier_slice.argtypes = [_VP, _VP]
        L.bfsx_dist_bu_step.argtypes = [_VP, _VP]
        L.bfsx_dist_level_end.argtypes = [_VP, I64P, I64P]
        L.bfsx_dist_finish.argtypes = [_VP]
        L.bfsx_dist_mcomp.argtypes = [_VP, I64P, I64P]
        L.bfsx_comm_unique_id.argtypes = [_VP]
        L.bfsx_comm_init.argtypes = [_VP, C.c_int, C.c_int, _VP]
        L.bfsx_comm_local_group.argtypes = [_VP, C.c_int]
        L.bfsx_dist_bfs.argtypes = [_VP, C.c_int64, C.POINTER(Stats)]
        L.bfsx_init_group.argtypes = [C.c_int, C.POINTER(_VP)]
        L.bfsx_group_size.argtypes = [_VP]
        L.bfsx_dist_graph_load_algs4.argtypes = [_VP, C.c_char_p, C.c_int, C.c_int, C.POINTER(_VP)]
    return L


def _check(rc, L=None):
    if rc != BFSX_OK:
        raise BfsxError(rc, (L or lib()).bfsx_last_error().decode(errors="replace"))
    return rc


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def comm_unique_id():
    """RCCL unique id (bytes) for bfsx_comm_init; rank 0 creates it, the caller distributes it."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check(lib().bfsx_comm_unique_id(buf))
    return bytes(buf)


def local_group(ctxs):
    """Attach an in-process exchange group to the contexts (rank r = ctxs[r]); each rank must then
    be driven by its own host thread (bfsx_dist_bfs is collective)."""
    L = ctxs[0]._L
    if any(c._L is not L for c in ctxs):
        raise ValueError("the contexts of one group must come from the same library (all diag or none)")
    arr = (_VP * len(ctxs))(*[c._h for c in ctxs])
    _check(L.bfsx_comm_local_group(arr, len(ctxs)), L)


def parse_algs4(path):
    """GraphFileUtil.convert parse (host only, no GPU needed) -> (nv, u, v)."""
    nv, m = C.c_int64(), C.c_int64()
    up, vp = C.POINTER(C.c_uint32)(), C.POINTER(C.c_uint32)()
    _check(lib().bfsx_parse_algs4(os.fsencode(path), C.byref(nv), C.byref(m), C.byref(up), C.byref(vp)))
    try:
        n = m.value
        u = np.ctypeslib.as_array(up, shape=(max(n, 1),))[:n].copy()
        v = np.ctypeslib.as_array(vp, shape=(max(n, 1),))[:n].copy()
    finally:
        lib().bfsx_free_host(up)
        lib().bfsx_free_host(vp)
    return nv.value, u, v


class Context:
    """One device (bfsx_init .. bfsx_finalize), or with group=N a group context of N ranks in this process
    (bfsx_init_group): graphs built on it are partitioned over the ranks, and every call runs all of them."""

    def __init__(self, device=0, group=None, diag=None, **options):
        if diag is None:
            diag = any(k in DIAG_OPTIONS and str(v) != "off" for k, v in options.items())
        self.diag = bool(diag)
        self._L = lib(self.diag)
        h = _VP()
        if group is not None:
            self._check(self._L.bfsx_init_group(int(group), C.byref(h)))
        else:
            self._check(self._L.bfsx_init(device, C.byref(h)))
        self._h = h
        for k, val in options.items():
            self.set_option(k, val)

    def _check(self, rc):
        return _check(rc, self._L)

    @property
    def group_size(self):
        return self._L.bfsx_group_size(self._h)

    def set_option(self, key, value):
        self._check(self._L.bfsx_set_option(self._h, key.encode(), str(value).encode()))

    def parse_algs4_gpu(self, path):
        """The same parse with the edge lines tokenized on this device -> (nv, u, v)."""
        nv, m = C.c_int64(), C.c_int64()
        up, vp = C.POINTER(C.c_uint32)(), C.POINTER(C.c_uint32)()
        self._check(self._L.bfsx_parse_algs4_gpu(self._h, os.fsencode(path), C.byref(nv), C.byref(m), C.byref(up),
                                          C.byref(vp)))
        try:
            n = m.value
            u = np.ctypeslib.as_array(up, shape=(max(n, 1),))[:n].copy()
            v = np.ctypeslib.as_array(vp, shape=(max(n, 1),))[:n].copy()
        finally:
            self._L.bfsx_free_host(up)
            self._L.bfsx_free_host(vp)
        return nv.value, u, v

    def load_algs4(self, path):
        g = _VP()
        self._check(self._L.bfsx_graph_load_algs4(self._h, os.fsencode(path), C.byref(g)))
        return Graph(self, g)

    def from_edges(self, nv, u, v):
        u = np.ascontiguousarray(u, dtype=np.uint32)
        v = np.ascontiguousarray(v, dtype=np.uint32)
        g = _VP()
        self._check(self._L.bfsx_graph_from_edges(self._h, nv, _p(u), _p(v), len(u), C.byref(g)))
        return Graph(self, g)

    def kronecker(self, scale, edgefactor=16, seed=0x5EED2026):
        g = _VP()
        self._check(self._L.bfsx_graph_kronecker(self._h, scale, edgefactor, seed, C.byref(g)))
        return Graph(self, g)

    def dist_from_edges(self, nv, u, v, rank, nranks):
        u = np.ascontiguousarray(u, dtype=np.uint32)
        v = np.ascontiguousarray(v, dtype=np.uint32)
        g = _VP()
        self._check(self._L.bfsx_dist_graph_from_edges(self._h, nv, _p(u), _p(v), len(u), rank, nranks, C.byref(g)))
        return Graph(self, g)

    def dist_load_algs4(self, path, rank, nranks):
        g = _VP()
        self._check(self._L.bfsx_dist_graph_load_algs4(self._h, os.fsencode(path), rank, nranks, C.byref(g)))
        return Graph(self, g)

    def dist_kronecker(self, scale, rank, nranks, edgefactor=16, seed=0x5EED2026):
        g = _VP()
        self._check(self._L.bfsx_dist_graph_kronecker(self._h, scale, edgefactor, seed, rank, nranks, C.byref(g)))
        return Graph(self, g)

    def kronecker_edges(self, scale, edgefactor=16, seed=0x5EED2026):
        m = edgefactor << scale
        u = np.empty(m, np.uint32)
        v = np.empty(m, np.uint32)
        self._check(self._L.bfsx_kronecker_edges(self._h, scale, edgefactor, seed, _p(u), _p(v)))
        return u, v

    def synchronize(self):
        self._check(self._L.bfsx_device_synchronize(self._h))

    def comm_init(self, rank, nranks, uid):
        """Collective over the nranks processes: attach an RCCL communicator to this context."""
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"an RCCL unique id has {COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        self._check(self._L.bfsx_comm_init(self._h, rank, nranks, buf))

    def close(self):
        if self._h:
            self._L.bfsx_finalize(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Graph:
    def __init__(self, ctx, handle):
        self.ctx = ctx
        self._L = ctx._L
        self._h = handle

    def _check(self, rc):
        return _check(rc, self._L)

    @property
    def nv(self):
        return self._L.bfsx_graph_nv(self._h)

    @property
    def nnz(self):
        return self._L.bfsx_graph_nnz(self._h)

    @property
    def m(self):
        return self._L.bfsx_graph_m(self._h)

    def csr(self):
        off = np.empty(self.nv + 1, np.int64)
        col = np.empty(max(self.nnz, 1), np.uint32)
        self._check(self._L.bfsx_graph_csr(self._h, _p(off), _p(col)))
        return off, col[: self.nnz]

    def sample_roots(self, count, seed=0x5EED):
        r = np.empty(count, np.int64)
        self._check(self._L.bfsx_sample_roots(self._h, count, seed, _p(r)))
        return r

    def bfs(self, source, want_dist=True, want_parent=True):
        """Returns (dist int32[nv] or None, parent int64[nv] or None, stats dict)."""
        nv = self.nv
        dist = np.empty(nv, np.int32) if want_dist else None
        parent = np.empty(nv, np.int64) if want_parent else None
        st = Stats()
        self._check(self._L.bfsx_bfs(self._h, source, _p(dist), _p(parent), C.byref(st)))
        return dist, parent, st.as_dict()

    def bfs_device_only(self, source):
        """The timed hot path: results stay on the device, no stats reduction.
        Returns the device time (ms) of source init -> last level complete (hipEvents)."""
        self._check(self._L.bfsx_bfs(self._h, source, None, None, None))
        return self.last_bfs_ms()

    def last_bfs_ms(self):
        """Device time (ms) of the most recent BFS of this graph (bfsx_last_bfs_ms)."""
        ms = C.c_double()
        self._check(self._L.bfsx_last_bfs_ms(self._h, C.byref(ms)))
        return ms.value

    COMM_KINDS = ("allreduce", "count_alltoall", "alltoallv", "allgather")

    def comm_times(self):
        """Device time (ms) and calls of the collectives of the most recent partitioned BFS by kind
        (bfsx_comm_times; option comm_timing=on, else zeros): {"allreduce": (ms, calls), ...}."""
        ms, cnt = (C.c_double * 4)(), (C.c_int64 * 4)()
        self._check(self._L.bfsx_comm_times(self._h, ms, cnt))
        return {k: (ms[i], cnt[i]) for i, k in enumerate(self.COMM_KINDS)}

    def last_unpack_ms(self):
        """Device time (ms) of the unpack kernel of the most recent result copy (bfsx_last_unpack_ms): the
        packed internal-id state -> original-id dist / parent arrays, outside t_bfs; -1 if none ran."""
        ms = C.c_double()
        self._check(self._L.bfsx_last_unpack_ms(self._h, C.byref(ms)))
        return ms.value

    def last_resolve_ms(self):
        """Device time (ms) of the internal-id part of the most recent unpack (bfsx_last_resolve_ms): push log and
        pull records folded into the per-vertex state; -1 if none ran (or an older build, BFSX_LIB)."""
        if not hasattr(self._L, "bfsx_last_resolve_ms"):
            return -1.0
        ms = C.c_double()
        self._check(self._L.bfsx_last_resolve_ms(self._h, C.byref(ms)))
        return ms.value

    def persist_fallbacks(self):
        """BFS runs of this graph re-run without K3p since it was built (bfsx_persist_fallbacks)."""
        if not hasattr(self._L, "bfsx_persist_fallbacks"):  # BFSX_LIB names an older build (A/B timing)
            return -1
        n = C.c_int64()
        self._check(self._L.bfsx_persist_fallbacks(self._h, C.byref(n)))
        return n.value

    def unpack_device_only(self):
        """Materialise the most recent result on the device only (bfsx_result with null outputs); returns the
        unpack kernel's device time (ms)."""
        self._check(self._L.bfsx_result(self._h, None, None))
        return self.last_unpack_ms()

    def result(self, want_parent=True, dist=None, parent=None):
        """Copy the most recent result to host (bfsx_result); dist / parent: caller arrays to fill (reused
        buffers), else new ones."""
        if dist is None:
            dist = np.empty(self.nv, np.int32)
        if parent is None and want_parent:
            parent = np.empty(self.nv, np.int64)
        # explicit checks (not asserts, which python -O drops): bfsx_result writes nv elements into both arrays
        if not (isinstance(dist, np.ndarray) and dist.dtype == np.int32 and dist.size == self.nv
                and dist.flags.c_contiguous and dist.flags.writeable):
            raise ValueError(f"dist must be a writeable C-contiguous int32 array of {self.nv} elements")
        if parent is not None and not (isinstance(parent, np.ndarray) and parent.dtype == np.int64
                                       and parent.size == self.nv and parent.flags.c_contiguous
                                       and parent.flags.writeable):
            raise ValueError(f"parent must be a writeable C-contiguous int64 array of {self.nv} elements")
        self._check(self._L.bfsx_result(self._h, _p(dist), _p(parent)))
        return dist, parent

    def validate(self, source=-1):
        """Graph500-style validation of the most recent BFS on the device (collective on a partitioned
        graph).  Returns {errors, first_bad, reached, entries}; errors == 0 means the distances are
        exactly the graph's BFS distances and the parents form a valid BFS tree."""
        e, f, r, n = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        self._check(self._L.bfsx_validate(self._h, source, C.byref(e), C.byref(f), C.byref(r), C.byref(n)))
        return {"errors": e.value, "first_bad": f.value, "reached": r.value, "entries": n.value}

    def validate_result(self, source, dist, parent):
        """Validate a caller-supplied (dist, parent) for this graph's rows.  Returns (errors, first_bad)."""
        dist = np.ascontiguousarray(dist, np.int32)
        parent = np.ascontiguousarray(parent, np.int64)
        if len(dist) != self.nv or len(parent) != self.nv:
            raise ValueError(f"dist and parent must hold {self.nv} elements")
        e, f = C.c_int64(), C.c_int64()
        self._check(self._L.bfsx_validate_result(self._h, source, _p(dist), _p(parent), C.byref(e), C.byref(f)))
        return e.value, f.value

    def level_times(self, cap=1 << 20):
        buf = np.empty(cap, np.float64)
        n = self._L.bfsx_level_times(self._h, _p(buf), cap)
        return buf[:n].copy()

    def level_dirs(self, cap=1 << 20):
        buf = np.empty(cap, np.int32)
        n = self._L.bfsx_level_dirs(self._h, _p(buf), cap)
        return buf[:n].copy()

    def partition(self):
        a, b, c, d = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        r, p = C.c_int32(), C.c_int32()
        self._check(self._L.bfsx_graph_partition(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d), C.byref(r),
                                          C.byref(p)))
        return dict(nv_global=a.value, v_lo=b.value, nv_local=c.value, chunk=d.value, rank=r.value,
                    nranks=p.value)

    def degree(self, v):
        d = C.c_int64()
        self._check(self._L.bfsx_graph_degree(self._h, v, C.byref(d)))
        return d.value

    # ---- multi-GPU level primitives (device pointers are ints, e.g. torch tensor data_ptr()) ----
    def dist_begin(self, source):
        d = C.c_int64()
        self._check(self._L.bfsx_dist_begin(self._h, source, C.byref(d)))
        return d.value

    def dist_frontier_info(self):
        a, b = C.c_int64(), C.c_int64()
        self._check(self._L.bfsx_dist_frontier_info(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def dist_td_expand(self, send_ptr, send_cap, nranks):
        counts = np.zeros(nranks, np.int64)
        self._check(self._L.bfsx_dist_td_expand(self._h, send_ptr, send_cap, _p(counts)))
        return counts

    def dist_td_claim(self, recv_ptr, n):
        self._check(self._L.bfsx_dist_td_claim(self._h, recv_ptr, n))

    def dist_frontier_slice(self, slice_ptr):
        self._check(self._L.bfsx_dist_frontier_slice(self._h, slice_ptr))

    def dist_bu_step(self, front_ptr):
        self._check(self._L.bfsx_dist_bu_step(self._h, front_ptr))

    def dist_level_end(self):
        a, b = C.c_int64(), C.c_int64()
        self._check(self._L.bfsx_dist_level_end(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def dist_finish(self):
        self._check(self._L.bfsx_dist_finish(self._h))

    def dist_bfs(self, source, want_stats=True):
        """Partitioned BFS, the whole level loop + exchanges in libbfsx (collective: every rank calls
        it with the same source).  Returns the stats dict (m_comp/reached all-reduced) or the device
        time in ms when want_stats is False."""
        if want_stats:
            st = Stats()
            self._check(self._L.bfsx_dist_bfs(self._h, source, C.byref(st)))
            return st.as_dict()
        self._check(self._L.bfsx_dist_bfs(self._h, source, None))
        return self.last_bfs_ms()

    def dist_mcomp(self):
        a, b = C.c_int64(), C.c_int64()
        self._check(self._L.bfsx_dist_mcomp(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def level_stats(self, cap=1 << 16):
        buf = (LevelStat * cap)()
        n = self._L.bfsx_level_stats(self._h, buf, cap)
        return [{k: getattr(buf[i], k) for k, _ in LevelStat._fields_} for i in range(n)]

    def level_stats_raw(self, cap=256):
        """The most recent BFS's level records as one bytes copy, with no per-field conversion (a few us, so a
        timed loop can keep every BFS's records); level_stats_decode turns it into level_stats()'s dicts."""
        buf = getattr(self, "_ls_buf", None)
        if buf is None or len(buf) < cap:
            buf = self._ls_buf = (LevelStat * cap)()
        n = self._L.bfsx_level_stats(self._h, buf, cap)
        return C.string_at(buf, max(n, 0) * C.sizeof(LevelStat))

    @staticmethod
    def level_stats_decode(raw):
        n = len(raw) // C.sizeof(LevelStat)
        buf = (LevelStat * n).from_buffer_copy(raw) if n else ()
        return [{k: getattr(buf[i], k) for k, _ in LevelStat._fields_} for i in range(n)]

    def free(self):
        if self._h:
            self._L.bfsx_graph_free(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.free()
