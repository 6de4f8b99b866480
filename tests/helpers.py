"""Shared test helpers: golden fixtures, digests and the CPU oracle (ctypes).

The oracle (oracle/liboracle.so) is TEST INFRASTRUCTURE: it is only ever used
here as the checker (and by smoke()/bench.py's cpu_baseline).
"""
import ctypes
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")


# --------------------------------------------------------------------------
# tiles as plain dicts of numpy arrays (DCSC: cp int64, jc/ir int32, val f64)
# --------------------------------------------------------------------------
def load_npz(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return dict(m=int(z["m"]), n=int(z["n"]), cp=z["cp"].astype(np.int64), jc=z["jc"].astype(np.int32),
                ir=z["ir"].astype(np.int32), val=z["val"].astype(np.float64))


def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def _mix64(z):
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def tile_cols(t):
    """expanded column index per nonzero"""
    cnt = np.diff(t["cp"])
    return np.repeat(t["jc"].astype(np.int64), cnt)


def digest(t, roff=0, coff=0):
    """Same digest as oracle/ref_driver.cpp tile_digest (tests/golden/make_golden.py)."""
    col = tile_cols(t) + coff
    row = t["ir"].astype(np.int64) + roff
    h = _mix64((col.astype(np.uint64) << np.uint64(32)) | row.astype(np.uint64))
    vb = _mix64(np.ascontiguousarray(t["val"], dtype=np.float64).view(np.uint64))
    with np.errstate(over="ignore"):
        hs = int(np.sum(h, dtype=np.uint64))
        hv = int(np.sum(h * vb, dtype=np.uint64))
    unsorted = 0
    if len(t["jc"]) > 1:
        unsorted += int(np.sum(np.diff(t["jc"].astype(np.int64)) <= 0))
    if len(row) > 1:
        d = np.diff(t["ir"].astype(np.int64))
        same = np.diff(col) == 0
        unsorted += int(np.sum((d <= 0) & same))
    return dict(nnz=int(len(t["ir"])), nzc=int(len(t["jc"])), hs="%016x" % hs, hv="%016x" % hv,
                vsum=float(np.sum(t["val"])), unsorted=unsorted)


def assert_digest_eq(d, g, values=True, vtol=0.0):
    assert d["nnz"] == g["nnz"], (d, g)
    assert d["hs"] == g["hs"], (d, g)
    assert d["unsorted"] == 0
    if values:
        if vtol == 0.0:
            assert d["hv"] == g["hv"], (d, g)
        assert abs(d["vsum"] - g["vsum"]) <= vtol * max(1.0, abs(g["vsum"])), (d, g)


def assert_tiles_equal(c, r, rtol=0.0, bound=None):
    """Indices bit-exact; values exact (rtol=0) or |dc| <= rtol * bound (elementwise)."""
    assert c["m"] == r["m"] and c["n"] == r["n"]
    np.testing.assert_array_equal(np.asarray(c["cp"], np.int64), np.asarray(r["cp"], np.int64))
    np.testing.assert_array_equal(np.asarray(c["jc"]), np.asarray(r["jc"]))
    np.testing.assert_array_equal(np.asarray(c["ir"]), np.asarray(r["ir"]))
    if rtol == 0.0:
        np.testing.assert_array_equal(np.asarray(c["val"]), np.asarray(r["val"]))
    else:
        b = np.abs(r["val"]) if bound is None else bound
        err = np.abs(np.asarray(c["val"]) - np.asarray(r["val"]))
        bad = err > rtol * b + 1e-300
        assert not bad.any(), f"{bad.sum()} values off, max rel {float(np.max(err / (b + 1e-300)))}"


# --------------------------------------------------------------------------
# oracle (ctypes)
# --------------------------------------------------------------------------
class OTile(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("nzc", ctypes.c_int64),
                ("cp", ctypes.POINTER(ctypes.c_int64)), ("jc", ctypes.POINTER(ctypes.c_int32)),
                ("ir", ctypes.POINTER(ctypes.c_int32)), ("val", ctypes.POINTER(ctypes.c_double))]


_lib = None


def oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, capture_output=True)
        _lib = ctypes.CDLL(ORACLE_SO)
        P = ctypes.POINTER(OTile)
        _lib.ocbg_rmat_tile.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, P]
        _lib.ocbg_local_hybrid.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P]
        _lib.ocbg_local_heap.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P]
        _lib.ocbg_summa.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        _lib.ocbg_symbolic.argtypes = [P, P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                       ctypes.c_int]
        _lib.ocbg_rmat_edges.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        _lib.ocbg_free.argtypes = [P]
    return _lib


def _to_otile(t):
    keep = dict(cp=np.ascontiguousarray(t["cp"], np.int64), jc=np.ascontiguousarray(t["jc"], np.int32),
                ir=np.ascontiguousarray(t["ir"], np.int32), val=np.ascontiguousarray(t["val"], np.float64))
    o = OTile(t["m"], t["n"], len(keep["ir"]), len(keep["jc"]),
              keep["cp"].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
              keep["jc"].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
              keep["ir"].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
              keep["val"].ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return o, keep


def _from_otile(o):
    lib = oracle()
    t = dict(m=o.m, n=o.n,
             cp=np.ctypeslib.as_array(o.cp, (o.nzc + 1,)).copy(),
             jc=np.ctypeslib.as_array(o.jc, (max(o.nzc, 1),))[:o.nzc].copy(),
             ir=np.ctypeslib.as_array(o.ir, (max(o.nnz, 1),))[:o.nnz].copy(),
             val=np.ctypeslib.as_array(o.val, (max(o.nnz, 1),))[:o.nnz].copy())
    lib.ocbg_free(ctypes.byref(o))
    return t


SR = {"plus": 0, "plus_times": 0, "minplus": 1, "min_plus": 1}


def oracle_rmat(scale, ef=16, seed=0xDECAFBAD, nthreads=0):
    o = OTile()
    oracle().ocbg_rmat_tile(scale, ef, seed, nthreads, ctypes.byref(o))
    return _from_otile(o)


def oracle_edges(scale, e0, e1, seed=0xDECAFBAD):
    s = np.empty(e1 - e0, np.int64)
    d = np.empty(e1 - e0, np.int64)
    oracle().ocbg_rmat_edges(scale, e0, e1, seed, s.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                             d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return s, d


def oracle_local(A, B, sr="plus", heap=False, nthreads=0):
    a, ka = _to_otile(A)
    b, kb = _to_otile(B)
    c = OTile()
    f = oracle().ocbg_local_heap if heap else oracle().ocbg_local_hybrid
    rc = f(ctypes.byref(a), ctypes.byref(b), SR[sr], nthreads, ctypes.byref(c))
    assert rc == 0
    return _from_otile(c)


def oracle_summa(A, B, pr, algo="doublebuff", sr="plus", nthreads=0):
    a, ka = _to_otile(A)
    b, kb = _to_otile(B)
    c = OTile()
    rc = oracle().ocbg_summa(ctypes.byref(a), ctypes.byref(b), pr, 0 if algo == "doublebuff" else 1, SR[sr],
                             nthreads, ctypes.byref(c))
    assert rc == 0, rc
    return _from_otile(c)


def oracle_symbolic(A, B, nthreads=0):
    a, ka = _to_otile(A)
    b, kb = _to_otile(B)
    nz = len(B["jc"])
    f = np.zeros(max(nz, 1), np.int64)
    n = np.zeros(max(nz, 1), np.int64)
    oracle().ocbg_symbolic(ctypes.byref(a), ctypes.byref(b), f.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                           n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), nthreads)
    return f[:nz], n[:nz]


def abs_tile(t):
    u = dict(t)
    u["val"] = np.abs(t["val"])
    return u


# ---- Galerkin path host restatements (checkers) ----
_M64 = (1 << 64) - 1


def _mix_np(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


POISSON1_CDF = np.array([0.36787944117144233, 0.7357588823428847, 0.9196986029286058, 0.9810118431238463,
                         0.9963401531726563, 0.9994058151824183, 0.999916758850712, 0.9999897508033253,
                         0.999998874797402, 0.9999998885745216, 0.9999999899522336, 0.9999999991683892])


def restriction_host(scale, order=2, seed=0x5EED):
    """global restriction operator of cbg_restriction_tile (csrc/cbg_ops.hip k_restrict_count /
    k_restrict_fill): genrestrict.m:11's sprand(n, n/order, order/n) shape -- Poisson(1)
    nonzeros per fine row (count by inversion of the CDF table), uniform coarse columns,
    values in (0, 1], a column drawn twice in one row summed."""
    n = 1 << scale
    nc = n // order
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _mix_np(np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03)))
        u = (_mix_np(h ^ np.uint64(0x5851F42D4C957F2D)) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        k = np.searchsorted(POISSON1_CDF, u, side="right")
        rows = np.repeat(np.arange(n, dtype=np.int64), k)
        starts = np.repeat(np.cumsum(k) - k, k)
        j = np.arange(len(rows), dtype=np.int64) - starts
        hj = _mix_np(h[rows] + (j + 1).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    cols = (hj % np.uint64(nc)).astype(np.int64)
    vals = ((_mix_np(hj) >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * (1.0 / 9007199254740992.0)
    o = np.lexsort((j, rows, cols))
    r, c, v = rows[o], cols[o], vals[o]
    head = np.ones(len(r), bool)
    head[1:] = (r[1:] != r[:-1]) | (c[1:] != c[:-1])
    run = np.cumsum(head) - 1
    uv = np.zeros(int(head.sum()))
    np.add.at(uv, run, v)  # duplicates summed in draw order
    ur, uc = r[head], c[head]
    jc, start = np.unique(uc, return_index=True)
    return dict(m=n, n=nc, cp=np.append(start, len(ur)).astype(np.int64), jc=jc.astype(np.int32),
                ir=ur.astype(np.int32), val=uv)


def random_values_host(t, seed=0x5EEDF00D, roff=0, coff=0):
    """Tile.set_random_values (csrc/cbg_ops.hip random_value) on a host tile: a copy with
    every (row, col) value = U[-1, 1) from mix(((col << 32) | row) ^ seed * K)."""
    col = tile_cols(t).astype(np.uint64) + np.uint64(coff)
    row = t["ir"].astype(np.uint64) + np.uint64(roff)
    with np.errstate(over="ignore"):
        z = _mix_np(((col << np.uint64(32)) | row) ^ (np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)))
    u = dict(t)
    u["val"] = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 4503599627370496.0) - 1.0
    return u


def transpose_host(d):
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    rows = d["ir"].astype(np.int64)
    o = np.lexsort((cols, rows))
    r, c, v = rows[o], cols[o], d["val"][o]
    jc, start = np.unique(r, return_index=True)
    return dict(m=d["n"], n=d["m"], cp=np.append(start, len(r)).astype(np.int64), jc=jc.astype(np.int32),
                ir=c.astype(np.int32), val=v)


def add_diag_host(d, dv):
    """d + diag(dv) for a host DCSC dict with no diagonal entries (loops removed)."""
    n = len(dv)
    cols = np.concatenate([np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"])), np.arange(n)])
    rows = np.concatenate([d["ir"].astype(np.int64), np.arange(n)])
    vals = np.concatenate([d["val"], dv])
    o = np.lexsort((rows, cols))
    r, c, v = rows[o], cols[o], vals[o]
    jc, start = np.unique(c, return_index=True)
    return dict(m=d["m"], n=d["n"], cp=np.append(start, len(r)).astype(np.int64), jc=jc.astype(np.int32),
                ir=r.astype(np.int32), val=v)
