"""combblas-spmm-test_amd -- MI355X-native CombBLAS 2D-SUMMA SpGEMM hot path.

Python binding of libcbg (C ABI in include/cbg.h) used by tests/ and bench.py.
It mirrors the reference's operator surface for the path:

  reference (include/CombBLAS/...)                 here
  ------------------------------------------------ --------------------------------
  SpDCCols<int32_t,double> (SpDCCols.h)            Tile  (device DCSC tile)
  CommGrid (CommGrid.h, src/CommGrid.cpp:37-75)    CommGrid (RCCL or host transport)
  SpParMat<...> (SpParMat.h)                       SpParMat (tile + grid + global dims)
  PlusTimesSRing / MinPlusSRing (Semirings.h)      PlusTimesSRing / MinPlusSRing
  LocalHybridSpGEMM (mtSpGEMM.h:212-460)           LocalHybridSpGEMM(A, B)
  MergeAll / MultiwayMerge (Friends.h:657,         MergeAll(parts) / MultiwayMerge(parts)
     MultiwayMerge.h:409)
  Mult_AnXBn_DoubleBuff (ParFriends.h:798-997)     Mult_AnXBn_DoubleBuff(A, B, sr)
  Mult_AnXBn_Synch (ParFriends.h:1004-1108)        Mult_AnXBn_Synch(A, B, sr)
  PSpGEMM (SpParMat.h:454-467)                     PSpGEMM(A, B, sr)
  DistEdgeList::GenGraph500Data + SpParMat(DEL)    rmat_tile / SpParMat.rmat
     + RemoveLoops

The reference MPI_Aborts on misuse; here the same codes surface as CbgError.code
(3001 GRIDMISMATCH, 3002 DIMMISMATCH, 3003 NOTSQUARE, 3005 MATRIXALIAS).

There is no CPU fallback: without libcbg.so (built by `make -C
combblas-spmm-test_amd`) or without a GPU every compute call raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CBG_LIB: alternative build of libcbg (tuning experiments: tools/variants.sh)
LIB_PATH = os.environ.get("CBG_LIB") or os.path.join(_HERE, "libcbg.so")

PLUS_TIMES, MIN_PLUS = 0, 1
DOUBLEBUFF, SYNCH = 0, 1
EXEC_PANEL, EXEC_STAGED = 0, 1
RANDOM_VALUES_SEED = 0x5EEDF00D  # Tile.set_random_values default
PHASES_AUTO = -1  # MemEfficientSpGEMM: phase count from the device's free memory (include/cbg.h CBG_PHASES_AUTO)

GRIDMISMATCH, DIMMISMATCH, NOTSQUARE, MATRIXALIAS, INVALIDPARAMS = 3001, 3002, 3003, 3005, 3007
HIPERROR, RCCLERROR, OOM, NOTSUPPORTED = 3100, 3101, 3102, 3103


class CbgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libcbg error {code}: {msg}")
        self.code = code


class CTile(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("nzc", ctypes.c_int64),
                ("cp", ctypes.c_void_p), ("jc", ctypes.c_void_p), ("ir", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("on_device", ctypes.c_int32), ("reserved", ctypes.c_int32)]


BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_size_t)


class CHostComm(ctypes.Structure):
    _fields_ = [("bcast", BCAST_FN), ("allgather", ALLGATHER_FN), ("user", ctypes.c_void_p)]


# every symbol include/cbg.h declares (checked by tests/test_capi.py)
EXPORTS = [
    "cbg_version", "cbg_last_error", "cbg_set_device", "cbg_device_count", "cbg_pool_stats", "cbg_pool_trim",
    "cbg_synchronize", "cbg_hbm_copy_bandwidth", "cbg_tile_upload", "cbg_tile_download", "cbg_tile_free", "cbg_tile_split_cols",
    "cbg_tile_split_rows", "cbg_tile_digest", "cbg_rmat_tile", "cbg_local_spgemm", "cbg_local_symbolic", "cbg_merge",
    "cbg_last_stats", "cbg_get_unique_id", "cbg_grid_create", "cbg_grid_create_host", "cbg_grid_destroy",
    "cbg_grid_info", "cbg_grid_barrier", "cbg_grid_allreduce_max", "cbg_grid_allreduce_sum_i64", "cbg_summa_spgemm",
    "cbg_tile_equal", "cbg_summa_spgemm_phased", "cbg_tile_transpose", "cbg_tile_dim_apply", "cbg_restriction_tile",
    "cbg_tile_random_values",
    "cbg_grid_transpose", "cbg_grid_block_extract", "cbg_grid_agree", "cbg_merge_stats", "cbg_tile_alloc",
    "cbg_tile_concat_cols", "cbg_device_memory", "cbg_last_summa_info", "cbg_summa_spgemm_memeff",
    "cbg_last_summa_comm",
    "cbg_last_phase_plan", "cbg_last_work_stats", "cbg_store_probe",
]
Column, Row = 0, 1  # DimApply dimensions (SpDefs.h Dim)
OP_MULTIPLIES, OP_PLUS, OP_MIN, OP_MAX = 0, 1, 2, 3
_OPS = {"multiplies": OP_MULTIPLIES, "plus": OP_PLUS, "min": OP_MIN, "max": OP_MAX}

# int (*cbg_phase_fn)(void* user, int phase, int64_t col_offset, const cbg_tile* C_phase)
PHASE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p)
EPSILON = 0.01  # SpDefs.h:64, the tolerance of ErrorTolerantEqual

_lib = None


def lib():
    """Load libcbg.so (raises if it has not been built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `make -C {_HERE}` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    T = ctypes.POINTER(CTile)
    i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
    sig = {
        "cbg_version": ([], ctypes.c_char_p),
        "cbg_last_error": ([], ctypes.c_char_p),
        "cbg_set_device": ([i32], i32),
        "cbg_device_count": ([ctypes.POINTER(i32)], i32),
        "cbg_pool_stats": ([ctypes.POINTER(ctypes.c_size_t)] * 2, i32),
        "cbg_pool_trim": ([], i32),
        "cbg_synchronize": ([], i32),
        "cbg_hbm_copy_bandwidth": ([i64, i32, ctypes.POINTER(ctypes.c_double)], i32),
        "cbg_tile_upload": ([T, T], i32),
        "cbg_tile_download": ([T, T], i32),
        "cbg_tile_free": ([T], i32),
        "cbg_tile_split_cols": ([T, i64, T, T], i32),
        "cbg_tile_split_rows": ([T, i64, T, T], i32),
        "cbg_tile_digest": ([T, i64, i64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)], i32),
        "cbg_rmat_tile": ([i32, i32, ctypes.c_uint64, i32, i32, i32, i32, T], i32),
        "cbg_local_spgemm": ([T, T, i32, T, vp], i32),
        "cbg_local_symbolic": ([T, T, ctypes.POINTER(i64), ctypes.POINTER(i64), vp], i32),
        "cbg_merge": ([T, i32, i32, T, vp], i32),
        "cbg_last_stats": ([ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "cbg_last_work_stats": ([ctypes.POINTER(i64), i32], i32),
        "cbg_store_probe": ([i64, i32], i32),
        "cbg_get_unique_id": ([vp], i32),
        "cbg_grid_create": ([i32, i32, i32, i32, vp, ctypes.POINTER(vp)], i32),
        "cbg_grid_create_host": ([i32, i32, i32, i32, ctypes.POINTER(CHostComm), ctypes.POINTER(vp)], i32),
        "cbg_grid_destroy": ([vp], i32),
        "cbg_grid_info": ([vp] + [ctypes.POINTER(i32)] * 6, i32),
        "cbg_grid_barrier": ([vp], i32),
        "cbg_grid_allreduce_max": ([vp, ctypes.POINTER(ctypes.c_double)], i32),
        "cbg_grid_allreduce_sum_i64": ([vp, ctypes.POINTER(i64)], i32),
        "cbg_summa_spgemm": ([vp, T, T, i64, i64, i32, i32, i32, T], i32),
        "cbg_tile_equal": ([T, T, ctypes.c_double, ctypes.POINTER(i32)], i32),
        "cbg_summa_spgemm_phased": ([vp, T, T, i64, i64, i32, i32, i32, i32, PHASE_FN, vp, T], i32),
        "cbg_summa_spgemm_memeff": ([vp, T, T, i64, i64, i32, i32, i32, i32, i64, PHASE_FN, vp, T], i32),
        "cbg_last_phase_plan": ([ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i64), ctypes.POINTER(i64),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double)],
                                i32),
        "cbg_tile_transpose": ([T, T], i32),
        "cbg_tile_dim_apply": ([T, i32, ctypes.POINTER(ctypes.c_double), i32], i32),
        "cbg_restriction_tile": ([i32, i32, ctypes.c_uint64, i32, i32, i32, i32, T], i32),
        "cbg_tile_random_values": ([T, ctypes.c_uint64, i64, i64], i32),
        "cbg_grid_transpose": ([vp, T, T], i32),
        "cbg_grid_block_extract": ([vp, T, i64, i64, i32, i64, i64, T], i32),
        "cbg_grid_agree": ([vp, i32, ctypes.POINTER(i32)], i32),
        "cbg_merge_stats": ([ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double)], i32),
        "cbg_tile_alloc": ([i64, i64, i64, i64, T], i32),
        "cbg_tile_concat_cols": ([T, i32, T], i32),
        "cbg_device_memory": ([ctypes.POINTER(ctypes.c_size_t)] * 2, i32),
        "cbg_last_summa_info": ([ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], i32),
        "cbg_last_summa_comm": ([ctypes.POINTER(i32), ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double)], i32),
    }
    experiment = "CBG_LIB" in os.environ  # an older build under A/B may lack the newest entry points
    for name, (args, res) in sig.items():
        if experiment and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise CbgError(rc, lib().cbg_last_error().decode(errors="replace"))


# --------------------------------------------------------------------------
# tiles
# --------------------------------------------------------------------------
class Tile:
    """A device-resident DCSC tile (SpDCCols<int32_t,double> in HBM)."""

    def __init__(self, ct=None):
        self.c = ct if ct is not None else CTile()

    # shape / counts (SpDCCols::getnrow/getncol/getnnz/getnzc)
    m = property(lambda self: self.c.m)
    n = property(lambda self: self.c.n)
    nnz = property(lambda self: self.c.nnz)
    nzc = property(lambda self: self.c.nzc)

    def isZero(self):
        return self.c.nnz == 0

    @staticmethod
    def from_host(m, n, cp, jc, ir, val):
        cp = np.ascontiguousarray(cp, np.int64)
        jc = np.ascontiguousarray(jc, np.int32)
        ir = np.ascontiguousarray(ir, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        h = CTile(int(m), int(n), len(ir), len(jc), cp.ctypes.data, jc.ctypes.data if len(jc) else None,
                  ir.ctypes.data if len(ir) else None, val.ctypes.data if len(val) else None, 0, 0)
        t = Tile()
        _check(lib().cbg_tile_upload(ctypes.byref(h), ctypes.byref(t.c)))
        return t

    @staticmethod
    def from_dict(d):
        return Tile.from_host(d["m"], d["n"], d["cp"], d["jc"], d["ir"], d["val"])

    def to_host(self):
        c = self.c
        cp = np.empty(c.nzc + 1, np.int64)
        jc = np.empty(max(c.nzc, 1), np.int32)
        ir = np.empty(max(c.nnz, 1), np.int32)
        val = np.empty(max(c.nnz, 1), np.float64)
        h = CTile(0, 0, 0, 0, cp.ctypes.data, jc.ctypes.data, ir.ctypes.data, val.ctypes.data, 0, 0)
        _check(lib().cbg_tile_download(ctypes.byref(c), ctypes.byref(h)))
        return dict(m=int(c.m), n=int(c.n), cp=cp, jc=jc[:c.nzc], ir=ir[:c.nnz], val=val[:c.nnz])

    def digest(self, roff=0, coff=0):
        """nnz, nzc, order-free hashes hs/hv, vsum, and `unsorted`: the number of DCSC
        order violations (rows not strictly ascending in a column, columns not
        ascending, empty columns; 0 for a valid tile, as the reference driver counts)."""
        hs, hv, vs, un = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        _check(lib().cbg_tile_digest(ctypes.byref(self.c), roff, coff, ctypes.byref(hs), ctypes.byref(hv),
                                     ctypes.byref(vs), ctypes.byref(un)))
        return dict(nnz=int(self.c.nnz), nzc=int(self.c.nzc), hs="%016x" % hs.value, hv="%016x" % hv.value,
                    vsum=vs.value, unsorted=int(un.value))

    def equal(self, other, epsilon=EPSILON):
        """SpDCCols::operator== (SpDCCols.h:74-81): exact structure, ErrorTolerantEqual values."""
        eq = ctypes.c_int()
        _check(lib().cbg_tile_equal(ctypes.byref(self.c), ctypes.byref(other.c), epsilon, ctypes.byref(eq)))
        return bool(eq.value)

    def __eq__(self, other):
        return isinstance(other, Tile) and self.equal(other)

    __hash__ = object.__hash__

    def transpose(self):
        """SpDCCols::Transpose (SpDCCols.cpp:853-873) -> new device tile."""
        t = Tile()
        _check(lib().cbg_tile_transpose(ctypes.byref(self.c), ctypes.byref(t.c)))
        return t

    def dim_apply(self, dim, vec, op="multiplies"):
        """SpParMat::DimApply on this tile (in place): vec has n (Column) or m (Row) values."""
        v = np.ascontiguousarray(vec, np.float64)
        if len(v) != (self.n if dim == Column else self.m):
            raise CbgError(INVALIDPARAMS, "DimApply vector length does not match the tile")
        _check(lib().cbg_tile_dim_apply(ctypes.byref(self.c), dim, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        _OPS.get(op, op)))

    def set_random_values(self, seed=RANDOM_VALUES_SEED, row_off=0, col_off=0):
        """Values U[-1, 1) from a hash of (seed, global column, global row) (SURVEY 8(d)'s
        random-valued inputs; the tile's global offsets make it grid-independent); in place."""
        _check(lib().cbg_tile_random_values(ctypes.byref(self.c), seed, int(row_off), int(col_off)))
        return self

    def split_cols(self, cut):
        """SpDCCols::Split (SpDCCols.cpp:905-930)"""
        a, b = Tile(), Tile()
        _check(lib().cbg_tile_split_cols(ctypes.byref(self.c), cut, ctypes.byref(a.c), ctypes.byref(b.c)))
        return a, b

    @staticmethod
    def create(essentials):
        """SpDCCols::Create(essentials) (SpDCCols.cpp:733-745): an uninitialised device tile
        from GetEssentials() = [nnz, m, n, nzc] (a broadcast's receive buffer)."""
        nnz, m, n, nzc = (int(x) for x in essentials)
        t = Tile()
        _check(lib().cbg_tile_alloc(m, n, nnz, nzc, ctypes.byref(t.c)))
        return t

    def GetEssentials(self):
        """SpDCCols::GetEssentials (SpDCCols.cpp:786-795): [nnz, m, n, nzc]"""
        return [int(self.c.nnz), int(self.c.m), int(self.c.n), int(self.c.nzc)]

    def GetArrays(self):
        """SpDCCols::GetArrays (SpDCCols.cpp:825-851): index arrays [cp, jc, ir] and value
        arrays [numx] as (device address, element count, element bytes) -- the buffers a
        broadcast of the tile moves (cp is int64 here, jc/ir int32)."""
        c = self.c
        if c.nnz == 0:
            return dict(indarrs=[(None, 0, 8), (None, 0, 4), (None, 0, 4)], numarrs=[(None, 0, 8)])
        return dict(indarrs=[(c.cp, c.nzc + 1, 8), (c.jc, c.nzc, 4), (c.ir, c.nnz, 4)],
                    numarrs=[(c.val, c.nnz, 8)])

    @staticmethod
    def concat_cols(parts):
        """SpDCCols::ColConcatenate / Merge: parts side by side (columns shifted)."""
        arr = (CTile * len(parts))(*[p.c for p in parts])
        t = Tile()
        _check(lib().cbg_tile_concat_cols(arr, len(parts), ctypes.byref(t.c)))
        return t

    def Merge(self, a, b):
        """SpDCCols::Merge (SpDCCols.cpp:1194-1223): self = [a | b]; a and b are released."""
        t = Tile.concat_cols([a, b])
        a.free()
        b.free()
        self.free()
        self.c = t.c
        t.c = CTile()

    def Transpose(self):
        """SpDCCols::Transpose (SpDCCols.cpp:853-873), in place."""
        t = self.transpose()
        self.free()
        self.c = t.c
        t.c = CTile()

    def ColSplit(self, parts):
        """SpDCCols::ColSplit (SpDCCols.cpp:936-970): `parts` column pieces cut at
        (i+1)*(n/parts), the last taking the rest; this tile is released."""
        w = self.n // parts
        out, rest = [], self
        for i in range(parts - 1):
            left, right = rest.split_cols(w)
            if rest is not self:
                rest.free()
            out.append(left)
            rest = right
        if rest is self:
            rest, _ = self.split_cols(self.n)
            _.free()
        out.append(rest)
        self.free()
        return out

    def split_rows(self, cut):
        a, b = Tile(), Tile()
        _check(lib().cbg_tile_split_rows(ctypes.byref(self.c), cut, ctypes.byref(a.c), ctypes.byref(b.c)))
        return a, b

    def free(self):
        if self.c.on_device and (self.c.cp or self.c.ir):
            _check(lib().cbg_tile_free(ctypes.byref(self.c)))

    def __del__(self):
        try:
            if _lib is not None and self.c.on_device:
                _lib.cbg_tile_free(ctypes.byref(self.c))
        except Exception:
            pass


def restriction_tile(scale, order=2, seed=0x5EED, grid=(1, 1), pos=(0, 0)):
    """Restriction operator tile (n x n/order, one nonzero per fine row, values in (0,1]),
    the role of mfiles/genrestrict.m for the Galerkin driver."""
    t = Tile()
    _check(lib().cbg_restriction_tile(scale, order, seed, grid[0], grid[1], pos[0], pos[1], ctypes.byref(t.c)))
    return t


def rmat_tile(scale, edgefactor=16, seed=0xDECAFBAD, grid=(1, 1), pos=(0, 0)):
    """Graph500 Kronecker R-MAT tile generated on device (GenWriteMatrix.cpp:101-114 semantics)."""
    t = Tile()
    _check(lib().cbg_rmat_tile(scale, edgefactor, seed, grid[0], grid[1], pos[0], pos[1], ctypes.byref(t.c)))
    return t


class PlusTimesSRing:
    """PlusTimesSRing<double,double> (Semirings.h:212-233)"""
    code = PLUS_TIMES


class MinPlusSRing:
    """MinPlusSRing<double,double> (Semirings.h:235-255)"""
    code = MIN_PLUS


def _sr(sr):
    if isinstance(sr, int):
        return sr
    if isinstance(sr, str):
        return {"plus": PLUS_TIMES, "plus_times": PLUS_TIMES, "minplus": MIN_PLUS, "min_plus": MIN_PLUS}[sr]
    return sr.code


def LocalHybridSpGEMM(A, B, sr=PlusTimesSRing, stream=None):
    """C = A*B for device tiles (mtSpGEMM.h:212-460); returns a device Tile (DCSC)."""
    C = Tile()
    _check(lib().cbg_local_spgemm(ctypes.byref(A.c), ctypes.byref(B.c), _sr(sr), ctypes.byref(C.c), stream))
    return C


def LocalSpGEMM(A, B, sr=PlusTimesSRing, stream=None):
    """The reference's heap kernel (mtSpGEMM.h:73-202, HashSpGEMMTest.cpp:75): same C
    structure as LocalHybridSpGEMM (rows ascending per column); the heap's summation
    order only changes fp rounding, so the one device kernel serves both entry points."""
    return LocalHybridSpGEMM(A, B, sr, stream)


def last_stats():
    f, n, nb, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    a, b = ctypes.c_double(), ctypes.c_double()
    lib().cbg_last_stats(ctypes.byref(f), ctypes.byref(n), ctypes.byref(a), ctypes.byref(b), ctypes.byref(nb),
                         ctypes.byref(ns))
    return dict(flops=f.value, nnz=n.value, ms_symbolic=a.value, ms_numeric=b.value, n_big=nb.value,
                n_slabs=ns.value)


# cbg_last_work_stats classes (include/cbg.h CBG_WORK_*), in order
WORK_CLASSES = (["bitmap_small_kept", "bitmap_small_mark", "bitmap_large_kept", "bitmap_large_mark"] +
                ["hash_T%d" % t for t in (512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192)] +
                ["rank_N%d" % n for n in (1024, 2048, 4096)] +
                ["sym_panel_units", "sym_group_units", "sym_deferred_units", "esc_columns", "thin_columns",
                 "single_big_entries", "hash_bin_columns", "wave_bin_columns", "int_accumulate"] +
                ["group_rank_N%d" % n for n in (2048, 4096)])


def last_work_stats():
    """the work of each kernel family in the last call's local multiplies (summed):
    numeric slabs per launch class, symbolic units, small-column passes -- which
    code paths ran (cbg_last_work_stats)"""
    buf = (ctypes.c_int64 * len(WORK_CLASSES))()
    n = lib().cbg_last_work_stats(buf, len(WORK_CLASSES))
    if n != len(WORK_CLASSES):
        raise CbgError(-1, "cbg_last_work_stats reports %d classes, the mirror knows %d" % (n, len(WORK_CLASSES)))
    return dict(zip(WORK_CLASSES, buf))


def summa_info():
    """the last PANEL SUMMA's double buffering: pieces multiplied, broadcast ms of the
    first piece, estimated ms of the rest's broadcast, and the ms an extra piece is taken
    to cost (pipelined when the hidden broadcast is worth it)."""
    a, b, c, d = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    lib().cbg_last_summa_info(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d))
    r, nb, ex = ctypes.c_int(), ctypes.c_int64(), ctypes.c_double()
    if hasattr(lib(), "cbg_last_summa_comm"):  # (absent only from older builds under A/B)
        lib().cbg_last_summa_comm(ctypes.byref(r), ctypes.byref(nb), ctypes.byref(ex))
    return dict(pieces=a.value, bcast_ms_piece0=b.value, est_hidden_ms=c.value, piece_cost_ms=d.value,
                rule=r.value, bytes_recv=nb.value, exposed_comm_ms=ex.value)


def phase_plan():
    """the last MemEfficientSpGEMM's phases: count, whether chosen from memory, this
    rank's product flops and nnz(C) estimate, the C bytes a phase was allowed, and
    phases split in column halves after an out-of-memory."""
    a, b, c, d, e, f = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int()
    g = ctypes.c_double()
    lib().cbg_last_phase_plan(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d), ctypes.byref(e),
                              ctypes.byref(f), ctypes.byref(g))
    return dict(phases=a.value, automatic=bool(b.value), flops=c.value, nnz_est=d.value, c_budget_bytes=e.value,
                oom_splits=f.value, plan_ms=g.value)


def merge_stats():
    """the last call's multiway merges: partial entries in, merged entries out, device ms."""
    a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
    lib().cbg_merge_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return dict(entries_in=a.value, entries_out=b.value, ms=c.value)


def MergeAll(parts, sr=PlusTimesSRing):
    """Merge column-sorted partial tiles, summing duplicates (Friends.h:657-741)."""
    arr = (CTile * len(parts))(*[p.c for p in parts])
    C = Tile()
    _check(lib().cbg_merge(arr, len(parts), _sr(sr), ctypes.byref(C.c), None))
    return C


MultiwayMerge = MergeAll  # MultiwayMerge.h:409-526: same result, threaded in the reference


def synchronize():
    _check(lib().cbg_synchronize())


def hbm_copy_bandwidth(nbytes=4 << 30, reps=10):
    """Measured HBM bandwidth (GB/s) of a 16-B-per-lane device copy: the measured
    roofline peak the bench reports beside the spec peak."""
    g = ctypes.c_double()
    _check(lib().cbg_hbm_copy_bandwidth(nbytes, reps, ctypes.byref(g)))
    return g.value


def store_probe(nbytes, width):
    """writes exactly nbytes of a scratch buffer with width-byte (4 or 8) stores per
    lane, lane-consecutive (the WRITE_SIZE calibration of tools/traffic.py)"""
    _check(lib().cbg_store_probe(nbytes, width))


def device_count():
    c = ctypes.c_int()
    _check(lib().cbg_device_count(ctypes.byref(c)))
    return c.value


def device_memory():
    """(free, total) bytes of the device (hipMemGetInfo)."""
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    _check(lib().cbg_device_memory(ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def pool_stats():
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    lib().cbg_pool_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


# --------------------------------------------------------------------------
# grid / distributed matrix
# --------------------------------------------------------------------------
class CommGrid:
    """CommGrid(world, rows, cols) (src/CommGrid.cpp:37-75); rows=cols=0 -> square.

    transport="rccl": one process per GPU, RCCL row/col communicators over xGMI.
    transport="host": collectives delegated to host callbacks (`host_comm`, an
    object with bcast(comm, np.ndarray(uint8), root) and allgather(comm, bytes)
    -> bytes); used to test the SUMMA logic with several processes per GPU.
    """

    def __init__(self, rank, nranks, rows=0, cols=0, unique_id=None, transport="rccl", host_comm=None):
        self.rank, self.nranks = rank, nranks
        self.h = ctypes.c_void_p()
        self._keep = None
        if transport == "rccl":
            if unique_id is None:
                raise ValueError("unique_id (from CommGrid.unique_id() on rank 0) is required")
            buf = ctypes.create_string_buffer(bytes(unique_id), 128)
            _check(lib().cbg_grid_create(rank, nranks, rows, cols, buf, ctypes.byref(self.h)))
        else:
            hc = host_comm

            def _bcast(user, comm, buf, nbytes, root):
                try:
                    arr = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)), (nbytes,))
                    hc.bcast(comm, arr, root)
                    return 0
                except Exception:  # noqa: BLE001 -- surfaced as CBG_ERR_RCCL
                    import traceback
                    traceback.print_exc()
                    return 1

            def _allgather(user, comm, inp, out, nbytes):
                try:
                    src = ctypes.string_at(inp, nbytes)
                    res = hc.allgather(comm, src)
                    ctypes.memmove(out, res, len(res))
                    return 0
                except Exception:  # noqa: BLE001
                    import traceback
                    traceback.print_exc()
                    return 1

            cb = CHostComm(BCAST_FN(_bcast), ALLGATHER_FN(_allgather), None)
            self._keep = cb
            _check(lib().cbg_grid_create_host(rank, nranks, rows, cols, ctypes.byref(cb), ctypes.byref(self.h)))
        vals = [ctypes.c_int() for _ in range(6)]
        _check(lib().cbg_grid_info(self.h, *[ctypes.byref(v) for v in vals]))
        _, _, self.grid_rows, self.grid_cols, self.prow, self.pcol = [v.value for v in vals]

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(lib().cbg_get_unique_id(buf))
        return buf.raw

    # CommGrid accessors
    def GetGridRows(self):
        return self.grid_rows

    def GetGridCols(self):
        return self.grid_cols

    def GetRankInProcRow(self):
        return self.pcol

    def GetRankInProcCol(self):
        return self.prow

    def barrier(self):
        _check(lib().cbg_grid_barrier(self.h))

    def allreduce_max(self, x):
        v = ctypes.c_double(x)
        _check(lib().cbg_grid_allreduce_max(self.h, ctypes.byref(v)))
        return v.value

    def allreduce_sum(self, x):
        v = ctypes.c_int64(int(x))
        _check(lib().cbg_grid_allreduce_sum_i64(self.h, ctypes.byref(v)))
        return v.value

    def agree(self, local_rc):
        """collective error agreement: the maximum of the ranks' codes (0 = every rank succeeded)."""
        out = ctypes.c_int()
        _check(lib().cbg_grid_agree(self.h, int(local_rc), ctypes.byref(out)))
        return out.value

    def destroy(self):
        if self.h:
            _check(lib().cbg_grid_destroy(self.h))
            self.h = ctypes.c_void_p()


class GlooHostComm:
    """Host transport for CommGrid(transport="host") over torch.distributed (gloo).

    Builds one process group per grid row and per grid column (ranks ascending,
    so the rank inside a row group is the grid column and inside a column group
    the grid row, as CommGrid's MPI_Comm_split keys give, src/CommGrid.cpp:66-67).
    Used to run the SUMMA logic with several processes on one GPU and in CPU tests.
    """

    def __init__(self, grid_rows, grid_cols):
        import torch  # noqa: F401
        import torch.distributed as dist
        self.dist = dist
        self.pr, self.pc = grid_rows, grid_cols
        self.rank = dist.get_rank()
        self.prow, self.pcol = self.rank // grid_cols, self.rank % grid_cols
        self.rows = [dist.new_group([r * grid_cols + c for c in range(grid_cols)]) for r in range(grid_rows)]
        self.cols = [dist.new_group([r * grid_cols + c for r in range(grid_rows)]) for c in range(grid_cols)]

    def _group(self, comm):
        if comm == 1:
            return self.rows[self.prow], lambda root: self.prow * self.pc + root
        if comm == 2:
            return self.cols[self.pcol], lambda root: root * self.pc + self.pcol
        return None, lambda root: root

    def bcast(self, comm, arr, root):
        import torch
        g, glob = self._group(comm)
        t = torch.from_numpy(arr)
        self.dist.broadcast(t, src=glob(root), group=g)

    def allgather(self, comm, data):
        import torch
        g, _ = self._group(comm)
        size = self.dist.get_world_size(g) if g is not None else self.dist.get_world_size()
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(size)]
        self.dist.all_gather(out, t, group=g)
        return b"".join(o.numpy().tobytes() for o in out)


class TcpHostComm:
    """Host transport over plain TCP sockets (rank 0 is the hub), no torch.

    The GPU processes must not import torch: torch's ROCm wheel carries its own
    HIP runtime, and a second runtime in the process corrupts the heap at exit.
    Every collective is world-synchronous (row and column communicators
    partition the world): each rank sends its payload to the hub, which replies
    with what that rank must receive.  Used for the RCCL unique-id rendezvous of
    bench.py and for multi-process tests on one GPU.
    """

    def __init__(self, rank, world, grid_rows=1, grid_cols=None, addr="127.0.0.1", port=29511, timeout=120.0):
        import socket
        import struct
        import time
        self._struct = struct
        self.rank, self.world = rank, world
        self.pr = grid_rows
        self.pc = grid_cols if grid_cols is not None else world // grid_rows
        self.prow, self.pcol = rank // self.pc, rank % self.pc
        self.peers = {}
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(timeout)
            while len(self.peers) < world - 1:
                c, _ = srv.accept()
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                r = struct.unpack("<q", self._recv(c, 8))[0]
                self.peers[r] = c
            srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=timeout)
                    break
                except OSError:
                    if time.time() - t0 > timeout:
                        raise
                    time.sleep(0.05)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.sendall(struct.pack("<q", rank))
            self.hub = c

    @staticmethod
    def _recv(c, n):
        buf = bytearray(n)
        mv = memoryview(buf)
        got = 0
        while got < n:
            k = c.recv_into(mv[got:], n - got)
            if k == 0:
                raise ConnectionError("peer closed")
            got += k
        return bytes(buf)

    def _send_msg(self, c, b):
        c.sendall(self._struct.pack("<q", len(b)) + b)

    def _recv_msg(self, c):
        n = self._struct.unpack("<q", self._recv(c, 8))[0]
        return self._recv(c, n)

    def _members(self, comm, r):
        pr_, pc_ = r // self.pc, r % self.pc
        if comm == 1:
            return [pr_ * self.pc + c for c in range(self.pc)]
        if comm == 2:
            return [q * self.pc + pc_ for q in range(self.pr)]
        return list(range(self.world))

    def _exchange(self, payload, reply_fn):
        if self.world == 1:
            return reply_fn({0: payload}, 0)
        if self.rank != 0:
            self._send_msg(self.hub, payload)
            return self._recv_msg(self.hub)
        got = {0: payload}
        for r, c in self.peers.items():
            got[r] = self._recv_msg(c)
        for r, c in self.peers.items():
            self._send_msg(c, reply_fn(got, r))
        return reply_fn(got, 0)

    def bcast(self, comm, arr, root):
        mine = bytes(arr) if self._members(comm, self.rank)[root] == self.rank else b""
        res = self._exchange(mine, lambda got, r: got[self._members(comm, r)[root]])
        arr[:] = memoryview(res).cast("B")

    def allgather(self, comm, data):
        return self._exchange(bytes(data), lambda got, r: b"".join(got[q] for q in self._members(comm, r)))

    def bcast_object(self, obj, root=0):
        import pickle
        res = self._exchange(pickle.dumps(obj) if self.rank == root else b"", lambda got, r: got[root])
        return pickle.loads(res)

    def close(self):
        for c in getattr(self, "peers", {}).values():
            c.close()
        if hasattr(self, "hub"):
            self.hub.close()


def block_range(total, parts, idx):
    """Block distribution of SpParMat::Owner (SpParMat.cpp:5068-5097): last block takes the remainder."""
    per = total // parts
    lo = idx * per
    hi = total if idx == parts - 1 else lo + per
    return lo, hi


class SpParMat:
    """Distributed sparse matrix: one device tile per rank of a CommGrid."""

    def __init__(self, tile, grid, gm, gn):
        self.tile, self.grid, self.gm, self.gn = tile, grid, gm, gn

    def getnrow(self):
        return self.gm

    def getncol(self):
        return self.gn

    def getnnz(self):
        """global nnz (SpParMat::getnnz Allreduce, SpParMat.cpp:772-778)"""
        return self.grid.allreduce_sum(self.tile.nnz) if self.grid is not None else self.tile.nnz

    def __eq__(self, other):
        """SpParMat::operator== (SpParMat.cpp:2878-2884): local tile equality, AND over the grid."""
        if not isinstance(other, SpParMat):
            return False
        local = 1 if self.tile.equal(other.tile) else 0
        if self.grid is None:
            return bool(local)
        return self.grid.allreduce_sum(1 - local) == 0

    __hash__ = object.__hash__

    def Transpose(self):
        """SpParMat::Transpose (SpParMat.cpp:3528-3590), in place; square grids only."""
        t = Tile()
        _check(lib().cbg_grid_transpose(self.grid.h, ctypes.byref(self.tile.c), ctypes.byref(t.c)))
        self.tile.free()
        self.tile, self.gm, self.gn = t, self.gn, self.gm

    def _block_extract(self, dim, lo, hi):
        t = Tile()
        _check(lib().cbg_grid_block_extract(self.grid.h, ctypes.byref(self.tile.c), self.gm, self.gn, dim, lo, hi,
                                            ctypes.byref(t.c)))
        return SpParMat(t, self.grid, hi - lo if dim == 0 else self.gm, hi - lo if dim == 1 else self.gn)

    def BlockSplit(self, br, bc):
        """SpParMat::BlockSplit (SpParMat.cpp:2974-3058): br x bc blocks, each a
        distributed matrix of its own on this grid in the standard layout; block
        sizes as the reference's (the first n % b blocks one longer).  A row
        split (bc = 1) or a column split (br = 1) -- the splits BlockSpGEMM makes
        (BlockSpGEMM.h:39-45) -- is one collective per block; a 2-D split is
        the row split's blocks split by columns."""
        if (br == 1 and bc == 1) or br > self.gm or bc > self.gn:
            return [[self]]
        roff = _block_offsets(self.gm, br)
        coff = _block_offsets(self.gn, bc)
        rows = [self._block_extract(0, roff[i], roff[i + 1]) if br > 1 else self for i in range(br)]
        out = []
        for R in rows:
            out.append([R._block_extract(1, coff[j], coff[j + 1]) if bc > 1 else R for j in range(bc)])
            if bc > 1 and R is not self:
                R.tile.free()
        return out

    def DimApply(self, dim, vec, op="multiplies"):
        """SpParMat::DimApply (SpParMat.cpp:801) with a dense global vector (host array of
        ncol (Column) or nrow (Row) values); each rank applies its block's slice."""
        total, parts, idx = ((self.gn, self.grid.grid_cols, self.grid.pcol) if dim == Column
                             else (self.gm, self.grid.grid_rows, self.grid.prow))
        lo, hi = block_range(total, parts, idx)
        self.tile.dim_apply(dim, np.asarray(vec, np.float64)[lo:hi], op)

    def __iadd__(self, other):
        """SpParMat::operator+= (SpParMat.cpp:741): union, duplicates added (a MergeAll of the two tiles)."""
        C = MergeAll([self.tile, other.tile], PlusTimesSRing)
        self.tile.free()
        self.tile = C
        return self

    def copy(self):
        """deep copy (the reference's copy constructor)."""
        a, b = self.tile.split_cols(self.tile.n)
        b.free()
        return SpParMat(a, self.grid, self.gm, self.gn)

    @staticmethod
    def restriction(grid, scale, order=2, seed=0x5EED):
        n = 1 << scale
        t = restriction_tile(scale, order, seed, (grid.grid_rows, grid.grid_cols), (grid.prow, grid.pcol))
        return SpParMat(t, grid, n, n // order)

    @staticmethod
    def rmat(grid, scale, edgefactor=16, seed=0xDECAFBAD):
        nv = 1 << scale
        t = rmat_tile(scale, edgefactor, seed, (grid.grid_rows, grid.grid_cols), (grid.prow, grid.pcol))
        return SpParMat(t, grid, nv, nv)

    @staticmethod
    def ReadDistribute(grid, filename, master=0):
        """SpParMat::ReadDistribute (SpParMat.cpp:4211-4540), text or HKDT binary
        triples: every rank parses the file and keeps its block of the block
        distribution (the reference's master reads and scatters; the tiles are
        the same)."""
        return SpParMat.from_global(grid, read_triples(filename))

    @staticmethod
    def ParallelReadMM(grid, filename, onebased=True, binop="max"):
        """SpParMat::ParallelReadMM (SpParMat.cpp:3980-4117): every rank parses the
        file and keeps its block of the block distribution (the reference splits
        the byte range across ranks and redistributes with Alltoallv; the
        resulting tiles are the same)."""
        return SpParMat.from_global(grid, read_mm(filename, onebased, binop))

    @staticmethod
    def from_global(grid, d):
        """Distribute a global host DCSC dict by the block distribution (SpParMat::Owner)."""
        r0, r1 = block_range(d["m"], grid.grid_rows, grid.prow)
        c0, c1 = block_range(d["n"], grid.grid_cols, grid.pcol)
        t = sub_tile(d, r0, r1, c0, c1)
        return SpParMat(Tile.from_dict(t), grid, d["m"], d["n"])


_BINOPS = {"max": np.maximum, "min": np.minimum, "plus": np.add, "first": None}


def _dcsc_from_triples(m, n, rows, cols, vals):
    """tuples -> global host DCSC dict sorted by (col, row) (SpTuples::SortColBased;
    stable, so duplicates keep their file order), duplicates kept like
    SpDCCols::Create(size, m, n, tuples) (SpDCCols.cpp:748)."""
    order = np.lexsort((rows, cols))
    rows, cols, vals = rows[order], cols[order], vals[order]
    jc, start = np.unique(cols, return_index=True)
    return dict(m=int(m), n=int(n), cp=np.append(start, len(rows)).astype(np.int64), jc=jc.astype(np.int32),
                ir=rows.astype(np.int32), val=vals.astype(np.float64))


def read_triples(path):
    """The files of SpParMat::ReadDistribute (SpParMat.cpp:4211-4540) -> global host
    DCSC dict.  Text: '%' comment lines, then "m n nnz", then nnz lines "i j [v]"
    (1-based; a missing value reads as 1, ScalarReadSaveHandler::getNoNum).
    Binary (FileHeader.h ParseHeader): "HKDT", uint64 version, objsize, format, m,
    n, nnz, then nnz records {int64 row, int64 col, double val} (0-based,
    binaryfill, SpParMat.h:250-260)."""
    with open(path, "rb") as f:
        head = f.read(4)
        if head == b"HKDT":
            version, objsize, fmt, m, n, nnz = np.frombuffer(f.read(48), dtype=np.uint64).tolist()
            if fmt != 0:
                raise CbgError(INVALIDPARAMS, f"{path}: Ascii input with binary headers is not supported")
            rec = np.dtype([("r", "<i8"), ("c", "<i8"), ("v", "<f8")])
            t = np.frombuffer(f.read(int(nnz) * rec.itemsize), dtype=rec, count=int(nnz))
            return _dcsc_from_triples(m, n, t["r"].astype(np.int64), t["c"].astype(np.int64),
                                      t["v"].astype(np.float64))
    with open(path) as f:
        line = f.readline()
        while line.startswith("%"):
            line = f.readline()
        m, n, nnz = (int(x) for x in line.split()[:3])
        rows = np.empty(nnz, np.int64)
        cols = np.empty(nnz, np.int64)
        vals = np.ones(nnz, np.float64)
        for k in range(nnz):
            parts = f.readline().split()
            rows[k] = int(parts[0]) - 1
            cols[k] = int(parts[1]) - 1
            if len(parts) > 2:
                vals[k] = float(parts[2])
    return _dcsc_from_triples(m, n, rows, cols, vals)


def read_vector(path):
    """FullyDistVec::ReadDistribute (FullyDistVec.cpp:495 -> FullyDistSpVec.cpp:1397-1437)
    -> dense host vector: header "m n nnz", then "i j v" lines (1-based); the index
    is the row for a column vector (n == 1), else the column; absent entries are 0."""
    with open(path) as f:
        m, n, nnz = (int(x) for x in f.readline().split()[:3])
        glen = m if n == 1 else n
        out = np.zeros(glen, np.float64)
        for _ in range(nnz):
            parts = f.readline().split()
            i = int(parts[0] if n == 1 else parts[1]) - 1
            out[i] = float(parts[2]) if len(parts) > 2 else 1.0
    return out


def read_mm(path, onebased=True, binop="max"):
    """Matrix Market coordinate file -> global host DCSC dict, with the semantics of
    SpParMat::ParallelReadMM (SpParMat.cpp:3980-4117): real / integer / pattern
    (value 1), symmetric or hermitian entries mirrored (SpHelper::push_to_vectors,
    SpHelper.h:75-91), duplicates combined with BinOp after a column-major sort
    (SpTuples::RemoveDuplicates; the reference's MultTest uses maximum<double>)."""
    with open(path) as f:
        banner = f.readline().split()
        if len(banner) < 5 or banner[0].lower() != "%%matrixmarket" or banner[2].lower() != "coordinate":
            raise CbgError(INVALIDPARAMS, f"{path}: not a Matrix Market coordinate file")
        field, sym = banner[3].lower(), banner[4].lower()
        if field not in ("real", "integer", "pattern", "double"):
            raise CbgError(INVALIDPARAMS, f"{path}: unsupported Matrix Market field '{field}'")
        line = f.readline()
        while line.startswith("%") or not line.strip():
            line = f.readline()
        m, n, nz = (int(x) for x in line.split()[:3])
        data = np.loadtxt(f, ndmin=2) if nz else np.zeros((0, 3))
    rows = data[:, 0].astype(np.int64)
    cols = data[:, 1].astype(np.int64)
    vals = np.ones(len(rows)) if field == "pattern" else data[:, 2].astype(np.float64)
    if onebased:
        rows, cols = rows - 1, cols - 1
    if sym in ("symmetric", "hermitian"):
        off = rows != cols
        rows, cols, vals = (np.concatenate([rows, cols[off]]), np.concatenate([cols, rows[off]]),
                            np.concatenate([vals, vals[off]]))
    order = np.lexsort((rows, cols))
    rows, cols, vals = rows[order], cols[order], vals[order]
    if len(rows):
        first = np.ones(len(rows), bool)
        first[1:] = (rows[1:] != rows[:-1]) | (cols[1:] != cols[:-1])
        starts = np.flatnonzero(first)
        op = _BINOPS[binop] if isinstance(binop, str) else binop
        if op is None:
            vals = vals[starts]
        elif isinstance(op, np.ufunc):
            vals = op.reduceat(vals, starts)
        else:
            ends = np.append(starts[1:], len(vals))
            out = []
            for a, b in zip(starts, ends):
                v = vals[a]
                for x in vals[a + 1:b]:
                    v = op(v, x)
                out.append(v)
            vals = np.asarray(out, np.float64)
        rows, cols = rows[starts], cols[starts]
    jc, start = np.unique(cols, return_index=True)
    cp = np.append(start, len(rows)).astype(np.int64)
    return dict(m=m, n=n, cp=cp, jc=jc.astype(np.int32), ir=rows.astype(np.int32), val=vals.astype(np.float64))


def write_mm(path, d):
    """global host DCSC dict -> Matrix Market coordinate real general (1-based)."""
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{d['m']} {d['n']} {len(d['ir'])}\n")
        for r, c, v in zip(d["ir"], cols, d["val"]):
            f.write(f"{int(r) + 1} {int(c) + 1} {float(v)!r}\n")


def sub_tile(d, r0, r1, c0, c1):
    """rows [r0,r1) x cols [c0,c1) of a host DCSC dict, re-based (host helper)."""
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    rows = d["ir"].astype(np.int64)
    keep = (rows >= r0) & (rows < r1) & (cols >= c0) & (cols < c1)
    cols, rows, vals = cols[keep] - c0, rows[keep] - r0, d["val"][keep]
    jc, start = np.unique(cols, return_index=True)
    cp = np.append(start, len(rows)).astype(np.int64)
    return dict(m=r1 - r0, n=c1 - c0, cp=cp, jc=jc.astype(np.int32), ir=rows.astype(np.int32),
                val=vals.astype(np.float64))


def _summa(A, B, sr, algo, exec_mode):
    if A is B:
        raise CbgError(MATRIXALIAS, "Can not multiply, inputs alias (make a temporary copy of one of them first)")
    if A.grid is not B.grid and (A.grid.grid_rows, A.grid.grid_cols) != (B.grid.grid_rows, B.grid.grid_cols):
        raise CbgError(GRIDMISMATCH, "Grids don't confirm for multiplication")
    C = Tile()
    _check(lib().cbg_summa_spgemm(A.grid.h, ctypes.byref(A.tile.c), ctypes.byref(B.tile.c), A.gn, B.gm, _sr(sr),
                                  algo, exec_mode, ctypes.byref(C.c)))
    return SpParMat(C, A.grid, A.gm, B.gn)


def Mult_AnXBn_DoubleBuff(A, B, sr=PlusTimesSRing, exec_mode=EXEC_PANEL):
    """ParFriends.h:798-997 (collective over A.grid)."""
    return _summa(A, B, sr, DOUBLEBUFF, exec_mode)


def Mult_AnXBn_Synch(A, B, sr=PlusTimesSRing, exec_mode=EXEC_PANEL):
    """ParFriends.h:1004-1108 (collective over A.grid)."""
    return _summa(A, B, sr, SYNCH, exec_mode)


def MemEfficientSpGEMM(A, B, phases, sr=PlusTimesSRing, algo=DOUBLEBUFF, exec_mode=EXEC_PANEL, on_phase=None,
                       hardThreshold=0.0, selectNum=0, recoverNum=0, recoverPct=0.0, perProcessMemory=0):
    """ParFriends.h:449-730 with `phases` column pieces of B; the MCL pruning
    arguments must stay at their no-pruning values (pruning is not on this path).

    perProcessMemory > 0 (GB, ParFriends.h:482-535) or phases == PHASES_AUTO (this
    library's extension: the device's free memory) picks the phase count from
    memory (see cbg_summa_spgemm_memeff; phase_plan() reports it); otherwise
    phases < 1 or >= the inner dimension is reset to 1 (ParFriends.h:468-473).

    on_phase=None: C is the column concatenation of the phase products
    (ColConcatenate).  on_phase=fn: fn(phase, col_offset, Tile) is called with
    each phase's device tile (valid during the call only) and None is returned."""
    if hardThreshold > 0 or selectNum > 0 or recoverNum > 0 or recoverPct > 0:
        raise CbgError(INVALIDPARAMS, "MemEfficientSpGEMM pruning (MCL) is not supported on this path")
    errors = []  # (A is B is allowed: the reference copies B, ParFriends.h:547-549)

    def _cb(user, phase, off, ptile):
        try:
            view = Tile(CTile.from_buffer_copy(CTile.from_address(ptile)))
            try:
                on_phase(phase, int(off), view)
            finally:
                view.c = CTile()  # borrowed: libcbg frees the phase tile after the call
            return 0
        except Exception as e:  # noqa: BLE001 -- reported after the collective finishes
            errors.append(e)
            return 1

    fn = PHASE_FN(_cb) if on_phase is not None else PHASE_FN()
    C = Tile() if on_phase is None else None
    rc = lib().cbg_summa_spgemm_memeff(A.grid.h, ctypes.byref(A.tile.c), ctypes.byref(B.tile.c), A.gn, B.gm, _sr(sr),
                                       algo, exec_mode, phases, int(perProcessMemory), fn, None,
                                       ctypes.byref(C.c) if C else None)
    if errors:
        raise errors[0]
    _check(rc)
    return SpParMat(C, A.grid, A.gm, B.gn) if C is not None else None


def _block_offsets(n, nb):
    """block starts of BlockSplit / BlockSpGEMM::getBlockOffsets (BlockSpGEMM.h:114-131):
    n // nb per block, the first n % nb blocks one longer; n at the end."""
    bs, r = divmod(n, nb)
    return [min(b, r) * (bs + 1) + max(b - r, 0) * bs for b in range(nb)] + [n]


class BlockSpGEMM:
    """BlockSpGEMM (BlockSpGEMM.h:14-131): C = A*B computed block by block.  A is
    split into br row blocks, B into bc column blocks (bi = 1, as the reference
    asserts); getNextBlock() multiplies the next (row block, column block) pair
    with Mult_AnXBn_DoubleBuff and returns the C block with its global row and
    column offsets.  Collective over A's grid."""

    def __init__(self, A, B, br, bc, bi=1):
        if bi != 1:
            raise CbgError(NOTSUPPORTED, "BlockSpGEMM with bi != 1 (the reference asserts bi == 1)")
        self.br, self.bc, self.bi, self.cur_block = br, bc, bi, 0
        self.A_blocks = A.BlockSplit(br, bi)
        self.B_blocks = B.BlockSplit(bi, bc)
        self.nr, self.nc = A.getnrow(), B.getncol()

    def hasNext(self):
        return self.cur_block < self.br * self.bc

    def getBlockOffsets(self, is_row):
        return _block_offsets(self.nr, self.br) if is_row else _block_offsets(self.nc, self.bc)

    def getBlockId(self, rbid, cbid, sr=PlusTimesSRing):
        """-> (C block, roffset, coffset)"""
        roff = _block_offsets(self.nr, self.br)[rbid]
        coff = _block_offsets(self.nc, self.bc)[cbid]
        C = Mult_AnXBn_DoubleBuff(self.A_blocks[rbid][0], self.B_blocks[0][cbid], sr)
        return C, roff, coff

    def getNextBlock(self, sr=PlusTimesSRing):
        """-> (C block, roffset, coffset) of block cur_block (row-major over the blocks)"""
        rbid, cbid = divmod(self.cur_block, self.bc)
        self.cur_block += 1
        return self.getBlockId(rbid, cbid, sr)


def PSpGEMM(A, B, sr=PlusTimesSRing):
    """SpParMat.h:454-467: PSpGEMM -> Mult_AnXBn_Synch."""
    return Mult_AnXBn_Synch(A, B, sr)
