"""GPU parity of the HIP local multiply (through the C ABI) against the reference's golden
vectors and the CPU oracle.  Indices bit-exact; fp64 values exact for the integer-valued
R-MAT products and within |dc| <= 1e-12 * (|A||B|)_ij for random-valued inputs
(north_star tolerance); min-plus is exact (order independent)."""
import numpy as np
import pytest

from helpers import (abs_tile, assert_digest_eq, assert_tiles_equal, digest, golden, load_npz, oracle_local)

pytestmark = pytest.mark.gpu
G = golden()
RTOL = 1e-12


@pytest.mark.parametrize("scale", [8, 10, 12, 14, 16, 18])
def test_device_rmat_matches_reference(cbg, scale):
    A = cbg.rmat_tile(scale, 16)
    g = G["rmat"][f"s{scale}_ef16"]["A"]
    d = A.digest()
    assert d["nnz"] == g["nnz"] and d["nzc"] == g["nzc"] and d["hs"] == g["hs"] and d["hv"] == g["hv"]


@pytest.mark.parametrize("scale", [8, 10])
@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_local_full_product_bit_exact(cbg, scale, sr):
    A = cbg.rmat_tile(scale, 16)
    B = cbg.rmat_tile(scale, 16)
    C = cbg.LocalHybridSpGEMM(A, B, sr)
    assert_tiles_equal(C.to_host(), load_npz(f"rmat_s{scale}_ef16_C_local_{sr}.npz"))


@pytest.mark.parametrize("scale", [12, 14, 16, 18])
def test_local_digest_vs_reference(cbg, scale):
    A = cbg.rmat_tile(scale, 16)
    B = cbg.rmat_tile(scale, 16)
    C = cbg.LocalHybridSpGEMM(A, B)
    g = G["rmat"][f"s{scale}_ef16"]["C_local_plus"]
    d = C.digest()  # `unsorted` counted on the device: 0 required
    assert_digest_eq(d, g)
    h = C.to_host()  # order: columns ascending, rows ascending inside each column
    assert np.all(np.diff(h["jc"]) > 0)
    cols = np.repeat(np.arange(len(h["jc"])), np.diff(h["cp"]))
    r = h["ir"].astype(np.int64)
    assert not np.any((np.diff(cols) == 0) & (np.diff(r) <= 0))
    st = cbg.last_stats()
    assert st["nnz"] == g["nnz"] and st["flops"] == G["rmat"][f"s{scale}_ef16"]["symbolic"]["flops"]


@pytest.mark.parametrize("scale", [12, 14])
def test_minplus_digest(cbg, scale):
    A = cbg.rmat_tile(scale, 16)
    B = cbg.rmat_tile(scale, 16)
    C = cbg.LocalHybridSpGEMM(A, B, "minplus")
    assert_digest_eq(C.digest(), G["rmat"][f"s{scale}_ef16"]["C_local_minplus"])


@pytest.mark.parametrize("name", ["sevenvertex", "small_nonsym", "largeseq"])
@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_bundled_inputs(cbg, name, sr):
    Ah = load_npz(f"{name}_A.npz")
    Bh = load_npz(f"{name}_B.npz") if name == "largeseq" else Ah
    A, B = cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh)
    C = cbg.LocalHybridSpGEMM(A, B, sr).to_host()
    ref = load_npz(f"{name}_C_local_{sr}.npz")
    if sr == "plus":
        bound = oracle_local(abs_tile(Ah), abs_tile(Bh))["val"]
        assert_tiles_equal(C, ref, rtol=RTOL, bound=bound)
    else:
        assert_tiles_equal(C, ref)


def _rand_tile(rng, m, n, density, lo=-1.0, hi=1.0, hub_cols=()):
    M = (rng.random((m, n)) < density)
    for c in hub_cols:
        M[:, c] = rng.random(m) < 0.8
    vals = rng.uniform(lo, hi, size=(m, n))
    cols, rows = np.nonzero(M.T)
    jc, start = np.unique(cols, return_index=True)
    return dict(m=m, n=n, cp=np.append(start, len(rows)).astype(np.int64), jc=jc.astype(np.int32),
                ir=rows.astype(np.int32), val=vals[rows, cols].astype(np.float64))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_fp_vs_oracle(cbg, seed):
    rng = np.random.default_rng(seed)
    # hub columns in A and B force the wave, block and big-column (slab) paths
    Ah = _rand_tile(rng, 3000, 2500, 0.004, hub_cols=(3, 77))
    Bh = _rand_tile(rng, 2500, 1800, 0.01, hub_cols=(5,))
    Bh2 = dict(Bh)
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh)).to_host()
    ref = oracle_local(Ah, Bh2)
    bound = oracle_local(abs_tile(Ah), abs_tile(Bh))["val"]
    assert_tiles_equal(C, ref, rtol=RTOL, bound=bound)
    Cm = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), "minplus").to_host()
    assert_tiles_equal(Cm, oracle_local(Ah, Bh, "minplus"))


def _sparse_cols(rng, m, lens, dup_rows=None):
    """DCSC with column j holding lens[j] distinct sorted random rows (0 = empty column dropped)"""
    cols, rows = [], []
    for j, L in enumerate(lens):
        if L == 0:
            continue
        r = np.sort(rng.choice(m if dup_rows is None else dup_rows, L, replace=False))
        cols.append(np.full(L, j))
        rows.append(r)
    cols = np.concatenate(cols)
    rows = np.concatenate(rows)
    jc, start = np.unique(cols, return_index=True)
    return dict(m=m, n=len(lens), cp=np.append(start, len(rows)).astype(np.int64), jc=jc.astype(np.int32),
                ir=rows.astype(np.int32), val=rng.uniform(-1.0, 1.0, len(rows)))


@pytest.mark.parametrize("m", [5000, (1 << 27) + 5])
def test_small_column_esc(cbg, m):
    # columns of <= 512 products run through the expand-sort-compress waves
    # (k_esc_wave: 32 ... 1 columns per wave, 1, 2, 4 or 8 products per lane); rows
    # concentrated on few values force duplicate keys inside a wave, B columns
    # of many entries on empty A columns force several staging rounds, and
    # m >= 2^27 leaves no room for column bits in the sort key (CPW = 1)
    rng = np.random.default_rng(5)
    k = 400
    hot = np.arange(0, m, max(1, m // 40))[:40]      # 40 row values: many duplicates
    lensA = rng.integers(0, 9, k)
    lensA[::7] = 0                                      # empty A columns
    Ah = _sparse_cols(rng, m, lensA, dup_rows=hot)
    Ah["n"] = k
    nB = 3000
    ir, cp = [], [0]
    for j in range(nB):
        target = int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 100, 128, 160, 200, 256, 300, 400, 512]))
        ks, f = [], 0
        for kk in rng.permutation(k):
            L = int(lensA[kk])
            if f + L > target:
                continue
            ks.append(kk)
            f += L
            if f == target or len(ks) > 200:
                break
        ks = sorted(ks) if ks else [int(np.argmax(lensA == 0))]
        ir.extend(ks)
        cp.append(len(ir))
    Bh = dict(m=k, n=nB, cp=np.array(cp, np.int64), jc=np.arange(nB, dtype=np.int32),
              ir=np.array(ir, np.int32), val=rng.uniform(-1.0, 1.0, len(ir)))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh)).to_host()
    bound = oracle_local(abs_tile(Ah), abs_tile(Bh))["val"]
    assert_tiles_equal(C, oracle_local(Ah, Bh), rtol=RTOL, bound=bound)
    Cm = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), "minplus").to_host()
    assert_tiles_equal(Cm, oracle_local(Ah, Bh, "minplus"))


@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_thin_big_columns(cbg, sr):
    # long B columns over A columns of ONE nonzero (GalerkinNew's S * (A*T)):
    # flops per B entry 1 < R / 4, so they take the expand-sort-compress pass of
    # cbg_thin.hip instead of R (column, panel) pairs; A's rows come from a small
    # pool so that products collide; a few ordinary big and small columns too
    rng = np.random.default_rng(21)
    m, k = (1 << 20) + 37, 120000
    pool = rng.choice(m, 30000, replace=False)
    rowsA = rng.choice(pool, k)
    Ah = dict(m=m, n=k, cp=np.arange(k + 1, dtype=np.int64), jc=np.arange(k, dtype=np.int32),
              ir=rowsA.astype(np.int32), val=rng.uniform(0.5, 2.0, k))
    hub = np.sort(rng.choice(m, 20000, replace=False))          # one long A column: a regular big column
    Ah = dict(m=m, n=k + 1, cp=np.append(Ah["cp"], k + len(hub)).astype(np.int64),
              jc=np.arange(k + 1, dtype=np.int32), ir=np.concatenate([Ah["ir"], hub]).astype(np.int32),
              val=np.concatenate([Ah["val"], rng.uniform(0.5, 2.0, len(hub))]))
    lens = list(rng.integers(4100, 30000, 24)) + list(rng.integers(1, 40, 200))
    ir, cp = [], [0]
    for L in lens:
        ir.extend(np.sort(rng.choice(k, int(L), replace=False)))
        cp.append(len(ir))
    ir.extend([0, k])  # the hub column and one short one: a regular big column (one entry alone is a copy)
    cp.append(len(ir))
    nB = len(cp) - 1
    Bh = dict(m=k + 1, n=nB, cp=np.array(cp, np.int64), jc=np.arange(nB, dtype=np.int32),
              ir=np.array(ir, np.int32), val=rng.uniform(-1.0, 1.0, len(ir)))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), sr).to_host()
    ref = oracle_local(Ah, Bh, sr)
    if sr == "plus":
        assert_tiles_equal(C, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
    else:
        assert_tiles_equal(C, ref)
    assert cbg.last_stats()["n_big"] == 1  # the thin columns left the (column, panel) path


@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_single_entry_columns(cbg, sr):
    """B columns with one entry are scaled copies of an A column (k_copy_single /
    k_copy_single_big: no symbolic or hash work): short and hub A columns (above
    the 4096-flop big threshold), zero and negative B values, next to ordinary
    small and big columns; entry by entry against the oracle."""
    rng = np.random.default_rng(5)
    m, k = (1 << 19) + 11, 3000
    lens = np.concatenate([rng.integers(0, 30, k - 6), [5000, 9000, 20000, 70000, 4096, 4097]]).astype(np.int64)
    ir, cp = [], [0]
    for L in lens:
        ir.extend(np.sort(rng.choice(m, int(L), replace=False)))
        cp.append(len(ir))
    Ah = dict(m=m, n=k, cp=np.array(cp, np.int64), jc=np.arange(k, dtype=np.int32), ir=np.array(ir, np.int32),
              val=rng.uniform(-2.0, 2.0, len(ir)))
    bcols = []
    for j in range(400):
        t = j % 4
        if t == 0:    # one entry: a short A column
            bcols.append([int(rng.integers(0, k - 6))])
        elif t == 1:  # one entry: a hub
            bcols.append([int(k - 6 + rng.integers(0, 6))])
        elif t == 2:  # a few short ones
            bcols.append(sorted(rng.choice(k - 6, 5, replace=False).tolist()))
        else:         # hubs and short ones: a big column
            bcols.append(sorted(set(rng.choice(k - 6, 3, replace=False).tolist() + [k - 3, k - 2])))
    cpB = np.cumsum([0] + [len(c) for c in bcols]).astype(np.int64)
    irB = np.concatenate([np.array(c, np.int32) for c in bcols])
    valB = rng.uniform(-1.0, 1.0, len(irB))
    valB[::7] = 0.0  # explicit zero products stay structural entries
    Bh = dict(m=k, n=len(bcols), cp=cpB, jc=np.arange(len(bcols), dtype=np.int32), ir=irB, val=valB)
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), sr).to_host()
    ref = oracle_local(Ah, Bh, sr)
    if sr == "plus":
        assert_tiles_equal(C, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
    else:
        assert_tiles_equal(C, ref)


def test_big_columns_tall_matrix(cbg):
    # m > 2^20 rows exercises multi-pass bitmaps and hash-mode slabs
    rng = np.random.default_rng(7)
    m, k, n = (1 << 21) + 123, 64, 8
    nnz_per = 40000
    cols = np.repeat(np.arange(k), nnz_per)
    rows = np.concatenate([np.sort(rng.choice(m, nnz_per, replace=False)) for _ in range(k)])
    Ah = dict(m=m, n=k, cp=np.arange(k + 1, dtype=np.int64) * nnz_per, jc=np.arange(k, dtype=np.int32),
              ir=rows.astype(np.int32), val=rng.integers(1, 5, len(rows)).astype(np.float64))
    Bh = dict(m=k, n=n, cp=np.arange(n + 1, dtype=np.int64) * k, jc=np.arange(n, dtype=np.int32),
              ir=np.tile(np.arange(k, dtype=np.int32), n), val=rng.integers(1, 3, n * k).astype(np.float64))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh))
    assert cbg.last_stats()["n_big"] == n
    assert_tiles_equal(C.to_host(), oracle_local(Ah, Bh))


@pytest.mark.parametrize("kind", ["f32_exact", "one_inexact", "out_of_f32_range"])
def test_slab_value_narrowing(cbg, kind):
    # slab kernels read A's values as f32 only when every one is exactly an f32
    # (k_vals_f32); otherwise the f64 array: both must give the f64 products
    rng = np.random.default_rng(11)
    m, k, n = (1 << 19) + 5, 48, 6
    nnz_per = 30000
    rows = np.concatenate([np.sort(rng.choice(m, nnz_per, replace=False)) for _ in range(k)])
    val = rng.choice(np.array([0.5, -2.25, 3.0, 1.0, -0.0, 1024.125]), len(rows))
    if kind == "one_inexact":
        val[12345] = 0.1
    elif kind == "out_of_f32_range":
        val[777] = 1e300
        val[778] = 1e-300
    Ah = dict(m=m, n=k, cp=np.arange(k + 1, dtype=np.int64) * nnz_per, jc=np.arange(k, dtype=np.int32),
              ir=rows.astype(np.int32), val=val)
    Bh = dict(m=k, n=n, cp=np.arange(n + 1, dtype=np.int64) * k, jc=np.arange(n, dtype=np.int32),
              ir=np.tile(np.arange(k, dtype=np.int32), n), val=rng.uniform(-1, 1, n * k))
    for sr in ("plus", "minplus"):
        C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), sr)
        assert cbg.last_stats()["n_big"] == n
        ref = oracle_local(Ah, Bh, sr)
        if sr == "plus":
            assert_tiles_equal(C.to_host(), ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
        else:
            assert_tiles_equal(C.to_host(), ref)


@pytest.mark.parametrize("kind", ["rmat", "negative", "scaled_past_bound", "minus_zero", "half_integer"])
def test_int_accumulate_paths(cbg, kind):
    """The slab kernels' exact int32 accumulation (IACC) runs when every value of A and
    B is an integer of magnitude <= 2^24 (not -0.0) and max|A| max_j sum_k |B(k,j)|
    < 2^31 (min-plus: max|A| + max|B| < 2^30), else the f64 path; either way C equals
    the oracle's (integer sums are exact in f64 in any order).  R-MAT scale 14 (bitmap
    and rank slabs), both semirings."""
    Ah = cbg.rmat_tile(14, 16).to_host()
    if kind == "negative":
        Ah["val"] = -Ah["val"]
    elif kind == "scaled_past_bound":
        Ah["val"] = Ah["val"] * float(1 << 16)  # integers whose bound passes 2^31 (sums exact in f64)
    elif kind == "minus_zero":
        Ah["val"] = Ah["val"].copy()
        Ah["val"][123] = -0.0
    elif kind == "half_integer":
        Ah["val"] = Ah["val"] + 0.5  # f32-exact, not integers
    expect = {"rmat": True, "negative": True, "scaled_past_bound": False, "minus_zero": False,
              "half_integer": False}[kind]
    for sr in ("plus", "minplus"):
        A = cbg.Tile.from_dict(Ah)
        B = cbg.Tile.from_dict(Ah)
        C = cbg.LocalHybridSpGEMM(A, B, sr)
        w = cbg.last_work_stats()
        assert w["bitmap_small_kept"] + w["bitmap_large_kept"] > 0, w
        Ch = C.to_host()
        for t in (A, B, C):
            t.free()
        on = w["int_accumulate"] > 0
        if kind == "scaled_past_bound" and sr == "minplus":
            assert on  # |a + b| stays far below 2^30
        else:
            assert on == expect, (kind, sr, w)
        assert_tiles_equal(Ch, oracle_local(Ah, Ah, sr))  # exact: integer (or half-integer) sums


def _panel_group_operands(m=(1 << 20) + 77):
    """Tall A (m = 2^20 + 77: 5 row panels of 2^18, the last one partial) and a B whose
    columns land in every big-column class: panel groups of 4 and 2 (expected products
    per group <= 4096), single-panel hash pairs, bitmap pairs, a group with > 512 B
    entries, and groups whose products crowd into one panel (nnz > one hash slab), which
    must fall back to per-panel slabs."""
    rng = np.random.default_rng(11)
    heavy, light, local = 3000, 1000, 200  # A columns: 100 rows anywhere / 8 rows / 100 rows in panel 0

    def col(nr, hi):
        return np.sort(rng.choice(hi, nr, replace=False))

    acols = [col(100, m) for _ in range(heavy)] + [col(8, m) for _ in range(light)] + \
            [col(100, 1 << 18) for _ in range(local)]
    k = len(acols)
    cnt = np.array([len(c) for c in acols])
    Ah = dict(m=m, n=k, cp=np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64), jc=np.arange(k, dtype=np.int32),
              ir=np.concatenate(acols).astype(np.int32),
              val=rng.integers(1, 5, int(cnt.sum())).astype(np.float64))
    groups = [(100, 5, 40, 0), (100, 44, 48, 0), (100, 78, 84, 0), (50, 140, 160, 0), (30, 280, 320, 0),
              (20, 600, 601, 1), (20, 45, 46, 2)]
    bcols = []
    for num, lo, hi, kind in groups:
        for _ in range(num):
            nb = int(rng.integers(lo, hi))
            if kind == 0:
                bcols.append(np.sort(rng.choice(heavy, nb, replace=False)))
            elif kind == 1:
                bcols.append(np.sort(heavy + rng.choice(light, nb, replace=False)))
            else:
                bcols.append(np.sort(heavy + light + rng.choice(local, nb, replace=False)))
    n = len(bcols)
    perm = rng.permutation(n)
    bcols = [bcols[i] for i in perm]
    bc = np.array([len(c) for c in bcols])
    Bh = dict(m=k, n=n, cp=np.concatenate([[0], np.cumsum(bc)]).astype(np.int64), jc=np.arange(n, dtype=np.int32),
              ir=np.concatenate(bcols).astype(np.int32), val=rng.integers(1, 3, int(bc.sum())).astype(np.float64))
    return Ah, Bh


@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_panel_groups_tall_matrix(cbg, sr):
    """Big columns in panel groups (one hash slab over several row panels), their
    per-panel fallbacks and a partial last panel, bit-exact against the oracle."""
    Ah, Bh = _panel_group_operands()
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), sr)
    assert cbg.last_stats()["n_big"] > 300
    assert_tiles_equal(C.to_host(), oracle_local(Ah, Bh, sr))


@pytest.mark.parametrize("thin", ["0", "1"])
def test_panel_groups_65_panels(cbg, thin, monkeypatch):
    """m = 2^24 + 77 (65 row panels, the scale-24 case): columns of 4400-4800 products
    fall in the 32-panel group class (groups of up to 64 panels, GROUP_LOG_MAX = 6),
    one hash slab spanning 2^23 rows whose emit buckets need 17-bit row offsets;
    bit-exact against the oracle, plus-times and min-plus.  With the thin-column
    pass on, the 20 columns of 600 B entries over 8-row A columns (flops x 4 <
    entries x 65 panels) take it instead."""
    monkeypatch.setenv("CBG_THIN", thin)
    Ah, Bh = _panel_group_operands((1 << 24) + 77)
    for sr in ("plus", "minplus"):
        C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(Ah), cbg.Tile.from_dict(Bh), sr)
        assert cbg.last_stats()["n_big"] == (300 if thin == "1" else 320)
        assert_tiles_equal(C.to_host(), oracle_local(Ah, Bh, sr))


def test_panel_groups_rmat20():
    """R-MAT scale 20 (4 row panels): the panel-group path and the per-pair path
    (CBG_GROUPS=0) give identical C (digest), and nnz(C) equals the reference's
    symbolic total (golden)."""
    import json
    import os
    import subprocess
    import sys
    code = r'''
import sys, json
sys.path.insert(0, "tests")
from conftest import load_cbg
cbg = load_cbg()
A = cbg.rmat_tile(20, 16); B = cbg.rmat_tile(20, 16)
print(json.dumps(cbg.LocalHybridSpGEMM(A, B).digest()))
'''
    res = []
    for env in ({}, {"CBG_GROUPS": "0"}):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **env),
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
    g = G["rmat"]["s20_ef16"]["symbolic"]
    assert res[0]["nnz"] == g["nnzC"]
    assert res[0] == res[1]


def test_edge_cases(cbg):
    # empty operands -> SpTuples(0, m, n) (mtSpGEMM.h:224-227)
    E = dict(m=5, n=4, cp=np.zeros(1, np.int64), jc=np.zeros(0, np.int32), ir=np.zeros(0, np.int32),
             val=np.zeros(0))
    X = dict(m=4, n=3, cp=np.array([0, 2], np.int64), jc=np.array([1], np.int32), ir=np.array([0, 3], np.int32),
             val=np.array([1.0, -1.0]))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(E), cbg.Tile.from_dict(X))
    assert C.nnz == 0 and C.m == 5 and C.n == 3
    # explicit zeros are kept: (+1)(1) + (-1)(1) = 0 stays a structural nonzero
    A = dict(m=2, n=2, cp=np.array([0, 1, 2], np.int64), jc=np.array([0, 1], np.int32), ir=np.array([0, 0], np.int32),
             val=np.array([1.0, -1.0]))
    B = dict(m=2, n=1, cp=np.array([0, 2], np.int64), jc=np.array([0], np.int32), ir=np.array([0, 1], np.int32),
             val=np.array([1.0, 1.0]))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(A), cbg.Tile.from_dict(B)).to_host()
    assert C["ir"].tolist() == [0] and C["val"].tolist() == [0.0] and C["jc"].tolist() == [0]
    # B column whose A columns are all empty produces no output column
    B2 = dict(m=2, n=3, cp=np.array([0, 1, 2], np.int64), jc=np.array([0, 2], np.int32),
              ir=np.array([0, 1], np.int32), val=np.array([2.0, 3.0]))
    A2 = dict(m=2, n=2, cp=np.array([0, 1], np.int64), jc=np.array([1], np.int32), ir=np.array([1], np.int32),
              val=np.array([5.0]))
    C = cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(A2), cbg.Tile.from_dict(B2)).to_host()
    assert C["jc"].tolist() == [2] and C["ir"].tolist() == [1] and C["val"].tolist() == [15.0]
    # dimension mismatch -> DIMMISMATCH (ParFriends.h:162-170)
    with pytest.raises(cbg.CbgError) as e:
        cbg.LocalHybridSpGEMM(cbg.Tile.from_dict(A2), cbg.Tile.from_dict(X))
    assert e.value.code == cbg.DIMMISMATCH


def test_merge_and_split(cbg):
    A = cbg.rmat_tile(10, 16)
    B = cbg.rmat_tile(10, 16)
    A1, A2 = A.split_cols(A.n // 2)
    B1, B2 = B.split_rows(B.m // 2)
    P1 = cbg.LocalHybridSpGEMM(A1, B1)
    P2 = cbg.LocalHybridSpGEMM(A2, B2)
    C = cbg.MergeAll([P1, P2])
    assert_tiles_equal(C.to_host(), load_npz("rmat_s10_ef16_C_local_plus.npz"))
    Cm = cbg.MergeAll([cbg.LocalHybridSpGEMM(A1, B1, "minplus"), cbg.LocalHybridSpGEMM(A2, B2, "minplus")], "minplus")
    assert_tiles_equal(Cm.to_host(), load_npz("rmat_s10_ef16_C_local_minplus.npz"))


@pytest.mark.parametrize("algo", ["doublebuff", "synch"])
@pytest.mark.parametrize("exec_mode", [0, 1])
def test_summa_single_rank(cbg, algo, exec_mode):
    class Self:
        def bcast(self, comm, arr, root):
            pass

        def allgather(self, comm, data):
            return data

    g = cbg.CommGrid(0, 1, transport="host", host_comm=Self())
    A = cbg.SpParMat.rmat(g, 10)
    B = cbg.SpParMat.rmat(g, 10)
    f = cbg.Mult_AnXBn_DoubleBuff if algo == "doublebuff" else cbg.Mult_AnXBn_Synch
    C = f(A, B, exec_mode=exec_mode)
    assert_tiles_equal(C.tile.to_host(), load_npz("rmat_s10_ef16_C_local_plus.npz"))
    with pytest.raises(cbg.CbgError) as e:
        f(A, A)
    assert e.value.code == cbg.MATRIXALIAS
    g.destroy()


@pytest.mark.parametrize("algo", ["doublebuff", "synch"])
@pytest.mark.parametrize("exec_mode", [0, 1])
def test_summa_rccl_single_rank(cbg, algo, exec_mode):
    """The RCCL transport end to end on one GPU (1x1 grid: ncclCommInitRank, ncclCommSplit,
    and every collective of the path executed on one-rank communicators: the grouped
    ncclBroadcast of the A/B tiles (PANEL) and of the stage pieces (STAGED), ncclAllGather
    of the sizes, the agreement allgathers).  MemEfficientSpGEMM with 3 phases on PANEL
    broadcasts B's column pieces one phase ahead and assembles C in the growable arena."""
    g = cbg.CommGrid(0, 1, unique_id=cbg.CommGrid.unique_id(), transport="rccl")
    A = cbg.SpParMat.rmat(g, 10)
    B = cbg.SpParMat.rmat(g, 10)
    f = cbg.Mult_AnXBn_DoubleBuff if algo == "doublebuff" else cbg.Mult_AnXBn_Synch
    C = f(A, B, exec_mode=exec_mode)
    ref = load_npz("rmat_s10_ef16_C_local_plus.npz")
    assert_tiles_equal(C.tile.to_host(), ref)
    Cp = cbg.MemEfficientSpGEMM(A, B, 3, algo=cbg.DOUBLEBUFF if algo == "doublebuff" else cbg.SYNCH,
                                exec_mode=exec_mode)
    assert_tiles_equal(Cp.tile.to_host(), ref)
    assert Cp.tile.digest()["unsorted"] == 0
    assert g.allreduce_max(3.5) == 3.5 and g.allreduce_sum(7) == 7 and g.agree(0) == 0 and g.agree(5) == 5
    T = A.copy()
    T.Transpose()  # 1x1: the diagonal rank transposes locally
    assert T.tile.nnz == A.tile.nnz
    blk = A.BlockSplit(2, 1)  # BlockSplit's broadcasts over the one-rank column communicator
    assert blk[0][0].tile.nnz + blk[1][0].tile.nnz == A.tile.nnz
    g.barrier()
    g.destroy()


@pytest.mark.parametrize("chunk", ["20000", "3000"])
def test_merge_int64_chunks(chunk):
    """MergeAll over column chunks (the path of partials with 2^31 or more entries),
    forced at small sizes by CBG_MERGE_CHUNK: merged tile == the one-product merge,
    chunks laid end to end in the growable arena; merges stay out of last_stats()."""
    import json
    import os
    import subprocess
    import sys
    code = """
import json, sys
sys.path.insert(0, %r)
from conftest import load_cbg
from helpers import load_npz
cbg = load_cbg()
A = cbg.Tile.from_dict(load_npz("rmat_s10_ef16_A.npz"))
AA = cbg.LocalHybridSpGEMM(A, A)
M = cbg.MergeAll([AA, A, A])  # three partials of one shape: A*A + 2A
st, ms = cbg.last_stats(), cbg.merge_stats()
h = M.to_host()
print(json.dumps(dict(nnz=int(M.nnz), d=M.digest(), stats_nnz=st["nnz"], merge_in=ms["entries_in"],
                      cp=h["cp"].tolist()[:50], ir=h["ir"].tolist()[:200], val=h["val"].tolist()[:200])))
""" % os.path.dirname(os.path.abspath(__file__))
    out = {}
    for env in ({}, {"CBG_MERGE_CHUNK": chunk}):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **env))
        assert r.returncode == 0, r.stderr[-3000:]
        out[bool(env)] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out[True] == out[False]
    assert out[True]["d"]["unsorted"] == 0 and out[True]["stats_nnz"] == 0
    assert out[True]["merge_in"] > out[True]["nnz"] > 0


def _add(ds):
    return dict(nnz=sum(d["nnz"] for d in ds), hs="%016x" % (sum(int(d["hs"], 16) for d in ds) % (1 << 64)),
                hv="%016x" % (sum(int(d["hv"], 16) for d in ds) % (1 << 64)),
                unsorted=sum(d["unsorted"] for d in ds))


def _tile_digests(cbg, scale, pr, pc, phases=-1):
    """every rank's C tile of scale-`scale` A*A on a pr x pc grid, computed on this one
    GPU the way the rank computes it (its A block row times its B block column,
    generated on device as the (pr x 1) / (1 x pc) tiles), streamed in B-column
    phases (-1 = PHASES_AUTO: picked from device memory, as the bench does); each phase digested at
    its global offsets (row block start, column block start + phase offset), so the
    sum is the digest of the whole C.  Returns (summed digest, phase plans)."""
    from combblas_spmm_test_amd import block_range
    nv = 1 << scale
    grid = _self_grid_1x1(cbg)
    parts, plans = [], []
    for r in range(pr):
        Ar = cbg.rmat_tile(scale, 16, grid=(pr, 1), pos=(r, 0))
        r0 = block_range(nv, pr, r)[0]
        for c in range(pc):
            Bc = cbg.rmat_tile(scale, 16, grid=(1, pc), pos=(0, c))
            c0 = block_range(nv, pc, c)[0]
            A = cbg.SpParMat(Ar, grid, Ar.m, nv)
            B = cbg.SpParMat(Bc, grid, nv, Bc.n)
            cbg.MemEfficientSpGEMM(A, B, phases, on_phase=lambda ph, off, t: parts.append(t.digest(r0, c0 + off)))
            plans.append(cbg.phase_plan())
            Bc.free()
        Ar.free()
    grid.destroy()
    return _add(parts), plans


def _oracle_large(key):
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        return json.load(f)[key]


@pytest.mark.parametrize("grid", [(2, 2), (4, 2)])
def test_rank_tiles_scale22(cbg, grid):
    """Config 3's per-rank work (2x2) and the bench's 8-GPU grid (4x2) on one GPU: every
    rank's C tile of scale-22 A*A (its A block row times its B block column, phases
    picked from memory), digested at its global offsets; the tiles' digests add up to
    the oracle's digest of the whole C (tests/golden/oracle_large.json s22_ef16:
    structure and values bit-exact), nnz to the reference's symbolic total."""
    d, plans = _tile_digests(cbg, 22, grid[0], grid[1])
    g = _oracle_large("s22_ef16")
    assert (d["nnz"], d["hs"], d["hv"], d["unsorted"]) == (g["nnz"], g["hs"], g["hv"], 0)
    assert d["nnz"] == G["rmat"]["s22_ef16"]["symbolic"]["nnzC"]
    assert all(p["automatic"] and p["phases"] >= 1 for p in plans)


def test_rank_tiles_scale24_2x4(cbg):
    """Config 4's per-rank work on one GPU: the eight C tiles of scale-24 A*A on a 2x4
    grid (about 2.3e10 nonzeros = 275 GB per tile: the phase count is picked from
    device memory, C streamed per phase); their nonzeros add up to the reference's
    symbolic nnz(C) = 183,028,712,946 and every tile is row-sorted."""
    d, plans = _tile_digests(cbg, 24, 2, 4)
    assert d["nnz"] == G["rmat"]["s24_ef16"]["symbolic"]["nnzC"] and d["unsorted"] == 0
    assert all(p["automatic"] and p["phases"] >= 2 for p in plans)  # 275 GB of C per tile does not fit
    g = _oracle_large("s24_ef16") if "s24_ef16" in _oracle_all() else None
    if g is not None:
        assert (d["nnz"], d["hs"], d["hv"]) == (g["nnz"], g["hs"], g["hv"])


def test_rank_tiles_scale24_2x4_values(cbg):
    """Config 4's 2x4 rank tiles with their VALUES pinned on a strided sample of C: column
    pieces p = 16k of 512 (8 in each of the grid's 4 block columns; digests of the CPU
    oracle, tests/golden/oracle_large.json s24_ef16_pieces).  For every sampled piece
    the ranks (r, c) whose block column holds it multiply their A block row (2^23 x 2^24
    rows/columns: R = 32 row panels) by that piece of their B block column -- the work
    their PANEL SUMMA does for those columns after the broadcasts; the two row blocks'
    digests at their global offsets add up to the oracle's digest of the piece
    (structure and values bit-exact, rows sorted)."""
    from combblas_spmm_test_amd import block_range
    g = _oracle_large("s24_ef16_pieces")
    n = 1 << 24
    w = n // g["pieces"]
    sample = sorted(p for p in (int(k) for k in g["digests"]) if p % 16 == 0)
    assert len(sample) >= 32 and {p * w * 4 // n for p in sample} == {0, 1, 2, 3}
    got = {p: [] for p in sample}
    for c in range(4):
        Bc = cbg.rmat_tile(24, 16, grid=(1, 4), pos=(0, c))
        c0 = block_range(n, 4, c)[0]
        mine = [p for p in sample if c0 <= p * w < c0 + Bc.n]
        for r in range(2):
            Ar = cbg.rmat_tile(24, 16, grid=(2, 1), pos=(r, 0))
            r0 = block_range(n, 2, r)[0]
            for p in mine:
                lo = p * w - c0
                left, right = Bc.split_cols(lo + w)
                right.free()
                low, Bp = left.split_cols(lo)
                low.free()
                left.free()
                C = cbg.LocalHybridSpGEMM(Ar, Bp)
                got[p].append(C.digest(r0, p * w))
                C.free()
                Bp.free()
            Ar.free()
        Bc.free()
    for p in sample:
        d, ref = _add(got[p]), g["digests"][str(p)]
        assert (d["nnz"], d["hs"], d["hv"], d["unsorted"]) == (ref["nnz"], ref["hs"], ref["hv"], 0), (p, d, ref)


def _oracle_all():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        return json.load(f)


def test_auto_phases_plan(cbg):
    """MemEfficientSpGEMM's memory-driven phase count (ParFriends.h:482-535): the plan's
    flops are the product's exact flops (from the tiles' count vectors); PHASES_AUTO on
    scale 18 (C = 5 GB) runs one phase; perProcessMemory = 2 GB forces several; the
    streamed phases add up to the reference's digest either way.  phases = 0 without a
    memory budget is the reference's "Resetting to 1" (ParFriends.h:468-473)."""
    grid = _self_grid_1x1(cbg)
    A = cbg.SpParMat.rmat(grid, 18)
    B = cbg.SpParMat.rmat(grid, 18)
    gd = G["rmat"]["s18_ef16"]["C_local_plus"]
    for kw in ({}, {"perProcessMemory": 2}):
        parts = []
        cbg.MemEfficientSpGEMM(A, B, cbg.PHASES_AUTO, on_phase=lambda ph, off, t: parts.append(t.digest(0, off)),
                               **kw)
        plan, st = cbg.phase_plan(), cbg.last_stats()
        d = _add(parts)
        assert (d["nnz"], d["hs"], d["hv"], d["unsorted"]) == (gd["nnz"], gd["hs"], gd["hv"], 0), kw
        assert plan["automatic"] and plan["flops"] == st["flops"] == G["rmat"]["s18_ef16"]["symbolic"]["flops"]
        if kw:
            # 2 GB minus the inputs, 60 % of it for C: 12 B x 4.3e8 entries needs several
            # phases; the flops bound alone asks for more than one, so the compression was
            # sampled and the estimate is close to the true nnz(C)
            assert plan["phases"] >= 4 and plan["c_budget_bytes"] < 1.2e9, plan
            assert 0.8 * gd["nnz"] <= plan["nnz_est"] <= 1.3 * gd["nnz"], plan
        else:
            # the flops bound (12 B x 1.1e9) fits the device: one phase, no sample taken
            assert plan["phases"] == 1 and plan["nnz_est"] == plan["flops"], plan
    for ph in (0, -3):  # the reference's reset to 1, not a memory plan
        parts = []
        cbg.MemEfficientSpGEMM(A, B, ph, on_phase=lambda p, off, t: parts.append((p, t.digest(0, off))))
        plan = cbg.phase_plan()
        assert plan["phases"] == 1 and not plan["automatic"] and {p for p, _ in parts} == {0}, plan
        assert _add([d for _, d in parts])["hs"] == gd["hs"]
    A.tile.free()
    B.tile.free()
    grid.destroy()


def test_phase_split_on_oom(cbg):
    """A phase whose C does not fit (forced with the CBG_FAULT_C_BYTES test hook, read per
    call) is computed as column halves of its B piece, each handed to the consumer at
    its own offset: the digests still add up to the reference's."""
    import os
    grid = _self_grid_1x1(cbg)
    A = cbg.SpParMat.rmat(grid, 14)
    B = cbg.SpParMat.rmat(grid, 14)
    gd = G["rmat"]["s14_ef16"]["C_local_plus"]
    parts = []
    os.environ["CBG_FAULT_C_BYTES"] = str(12 * gd["nnz"] // 5)
    try:
        cbg.MemEfficientSpGEMM(A, B, 2, on_phase=lambda ph, off, t: parts.append((ph, off, t.digest(0, off))))
    finally:
        del os.environ["CBG_FAULT_C_BYTES"]
    plan = cbg.phase_plan()
    d = _add([x[2] for x in parts])
    assert (d["nnz"], d["hs"], d["hv"], d["unsorted"]) == (gd["nnz"], gd["hs"], gd["hv"], 0)
    assert plan["oom_splits"] >= 2 and len(parts) >= 6 and sorted(set(x[0] for x in parts)) == [0, 1]
    A.tile.free()
    B.tile.free()
    grid.destroy()


@pytest.mark.parametrize("env", [{"CBG_BITMAP_BUDGET_GB": "0"}, {"CBG_BIG_FLOPS": "64"},
                                 {"CBG_BIG_FLOPS": "64", "CBG_BITMAP_BUDGET_GB": "0"},
                                 {"CBG_BITMAP_BUDGET_GB": "0.0002"}, {"CBG_CUTS_CAP": "3000"},
                                 {"CBG_CUTS_CAP": "0"}])
def test_big_column_path_variants(env):
    """Same products through the other big-column code paths (subprocess: knobs are
    read once): no kept bitmaps; a budget for a few of them (the general k_num_slab
    with kept and marked slabs mixed); multi-slab pairs' cuts for the first pairs only
    (the others search theirs: both kinds in one launch) or for none."""
    import json
    import os
    import subprocess
    import sys
    code = r'''
import sys, json
sys.path.insert(0, "tests")
from conftest import load_cbg
cbg = load_cbg()
out = {}
for scale in (12, 14):
    A = cbg.rmat_tile(scale, 16); B = cbg.rmat_tile(scale, 16)
    d = cbg.LocalHybridSpGEMM(A, B).digest(); d["n_big"] = cbg.last_stats()["n_big"]
    out[scale] = d
print(json.dumps(out))
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env), cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for scale in (12, 14):
        d = res[str(scale)]
        g = G["rmat"][f"s{scale}_ef16"]["C_local_plus"]
        assert d["nnz"] == g["nnz"] and d["hs"] == g["hs"] and d["hv"] == g["hv"], (env, scale)
        assert d["n_big"] > 0


def _self_grid(cbg):
    class Self:
        def bcast(self, comm, arr, root):
            pass

        def allgather(self, comm, data):
            return data

    return cbg.CommGrid(0, 1, transport="host", host_comm=Self())


def test_tile_equal_semantics(cbg):
    """SpDCCols::operator== / ErrorTolerantEqual (EPSILON 0.01, SpDefs.h:64)."""
    d = load_npz("rmat_s10_ef16_A.npz")
    A = cbg.Tile.from_dict(d)
    assert A == cbg.Tile.from_dict(d)
    v = d["val"].copy()
    v[5] *= 1.005                      # relative error 0.5 % < 1 %
    assert A == cbg.Tile.from_dict(dict(d, val=v))
    v[5] = d["val"][5] * 1.02          # 2 % > 1 %, and |diff| >= 0.01
    assert not A == cbg.Tile.from_dict(dict(d, val=v))
    assert A.equal(cbg.Tile.from_dict(dict(d, val=v)), epsilon=0.05)
    v = d["val"].copy()
    v[7] = np.nan
    assert not A == cbg.Tile.from_dict(dict(d, val=v))
    ir = d["ir"].copy()
    ir[0] += 1 if ir[1] > ir[0] + 1 else 0
    if not np.array_equal(ir, d["ir"]):
        assert not A == cbg.Tile.from_dict(dict(d, ir=ir))
    z0 = cbg.Tile.from_host(3, 4, np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))
    z1 = cbg.Tile.from_host(5, 6, np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))
    assert z0 == z1                    # both empty: equal whatever the shape (SpDCCols.h:76-77)
    assert not A == z0


@pytest.mark.parametrize("phases", [1, 2, 3, 7, 1024])
def test_phased_spgemm_matches_reference(cbg, phases):
    """MemEfficientSpGEMM phases (ColSplit + ColConcatenate) vs the reference's product."""
    g = _self_grid(cbg)
    A = cbg.SpParMat.rmat(g, 10)
    B = cbg.SpParMat.rmat(g, 10)
    C = cbg.MemEfficientSpGEMM(A, B, phases)   # phases >= ncol resets to 1 (ParFriends.h:469-473)
    assert_tiles_equal(C.tile.to_host(), load_npz("rmat_s10_ef16_C_local_plus.npz"))
    Cm = cbg.MemEfficientSpGEMM(A, B, phases, sr="minplus")
    assert_tiles_equal(Cm.tile.to_host(), load_npz("rmat_s10_ef16_C_local_minplus.npz"))
    Calias = cbg.MemEfficientSpGEMM(A, A, phases)  # allowed: the reference copies B
    assert Calias == C
    g.destroy()


def test_staged_phases_regular_matrix(cbg):
    """STAGED MemEfficientSpGEMM on a regular matrix whose two column halves (the
    DoubleBuff stages' A slices) have identical sizes but different entries: every
    stage of every phase frees its slices and the pool hands the same blocks out again,
    so a column-map cache keyed on pointers and sizes would reuse the maps of another A
    slice.  Each phase's product must equal the oracle's."""
    rng = np.random.default_rng(7)
    n = 4096
    cols = np.repeat(np.arange(n), 4)
    rows = (cols + np.tile(np.array([0, 1, 17, 301]), n) + (cols >= n // 2) * 5) % n
    o = np.lexsort((rows, cols))
    r, c = rows[o], cols[o]
    Ah = dict(m=n, n=n, cp=np.arange(0, 4 * n + 1, 4, dtype=np.int64), jc=np.arange(n, dtype=np.int32),
              ir=r.astype(np.int32), val=rng.uniform(-1, 1, 4 * n))
    g = _self_grid(cbg)
    A = cbg.SpParMat(cbg.Tile.from_dict(Ah), g, n, n)
    B = cbg.SpParMat(cbg.Tile.from_dict(Ah), g, n, n)
    ref = oracle_local(Ah, Ah)
    bound = oracle_local(abs_tile(Ah), abs_tile(Ah))["val"]
    for ex in (cbg.EXEC_STAGED, cbg.EXEC_PANEL):
        C = cbg.MemEfficientSpGEMM(A, B, 4, algo=cbg.DOUBLEBUFF, exec_mode=ex)
        assert_tiles_equal(C.tile.to_host(), ref, rtol=RTOL, bound=bound)
        C.tile.free()
    g.destroy()


def test_phased_spgemm_streamed(cbg):
    """on_phase streaming: phase tiles with their column offsets add up to the full digest."""
    g = _self_grid(cbg)
    A = cbg.SpParMat.rmat(g, 12)
    B = cbg.SpParMat.rmat(g, 12)
    seen = []
    cbg.MemEfficientSpGEMM(A, B, 5, on_phase=lambda p, off, t: seen.append((p, off, t.n, t.digest(0, off))))
    assert [s[0] for s in seen] == list(range(5))
    w = 4096 // 5
    assert [s[1] for s in seen] == [p * w for p in range(5)]
    assert [s[2] for s in seen] == [w] * 4 + [4096 - 4 * w]
    hs = sum(int(s[3]["hs"], 16) for s in seen) % (1 << 64)
    hv = sum(int(s[3]["hv"], 16) for s in seen) % (1 << 64)
    gd = golden()["rmat"]["s12_ef16"]["C_local_plus"]
    assert sum(s[3]["nnz"] for s in seen) == gd["nnz"]
    assert "%016x" % hs == gd["hs"] and "%016x" % hv == gd["hv"]
    with pytest.raises(ValueError):
        cbg.MemEfficientSpGEMM(A, B, 2, on_phase=lambda p, off, t: (_ for _ in ()).throw(ValueError("x")))
    with pytest.raises(cbg.CbgError) as e:
        cbg.MemEfficientSpGEMM(A, B, 2, hardThreshold=0.5)
    assert e.value.code == cbg.INVALIDPARAMS
    g.destroy()


def test_multtest_sevenvertex(cbg):
    """ReleaseTests/MultTest.cpp:95-180 SpGEMM part: ParallelReadMM of A, B and
    CControl, then Synch and DoubleBuff must equal CControl (SpParMat::operator==)."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    g = _self_grid(cbg)
    A = cbg.SpParMat.ParallelReadMM(g, os.path.join(gold, "sevenvertex.mtx"), True, "max")
    B = cbg.SpParMat.ParallelReadMM(g, os.path.join(gold, "sevenvertex.mtx"), True, "max")
    CControl = cbg.SpParMat.ParallelReadMM(g, os.path.join(gold, "sevenvertex_C.mtx"), True, "max")
    assert cbg.Mult_AnXBn_Synch(A, B) == CControl
    assert cbg.Mult_AnXBn_DoubleBuff(A, B) == CControl
    assert cbg.MemEfficientSpGEMM(A, B, 2) == CControl
    g.destroy()


def test_hashspgemmtest_largeseq(cbg, tmp_path):
    """ReleaseTests/HashSpGEMMTest.cpp:66-83: read A, B and the control C, then the
    local LocalSpGEMM(Alocal, Blocal) must equal CClocal (SpDCCols::operator==).  A and
    B are the reference's largeseq triples files (ReadDistribute); the control is the
    reference's own product (golden), written as Matrix Market and read back."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    g = _self_grid(cbg)
    A = cbg.SpParMat.ReadDistribute(g, os.path.join(gold, "largeseq_input1_0.triples"))
    B = cbg.SpParMat.ReadDistribute(g, os.path.join(gold, "largeseq_input2_0.triples"))
    cbg.write_mm(str(tmp_path / "C.mtx"), load_npz("largeseq_C_local_plus.npz"))
    CC = cbg.SpParMat.ParallelReadMM(g, str(tmp_path / "C.mtx"), True, "max")
    C = cbg.LocalSpGEMM(A.tile, B.tile)
    assert C == CC.tile
    assert C.nnz == 29677
    g.destroy()


def test_cpp_multtest_driver():
    """tools/multtest (C++ mirror header; built by __graft_entry__.build()) prints the
    reference MultTest's success lines for the bundled sevenvertex inputs."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "tools", "multtest")
    if not os.path.exists(exe):
        pytest.skip("tools/multtest not built (needs MPICH in /opt/conda)")
    g = os.path.join(repo, "tests", "golden")
    r = subprocess.run([exe, os.path.join(g, "sevenvertex.mtx"), os.path.join(g, "sevenvertex.mtx"),
                        os.path.join(g, "sevenvertex_C.mtx")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for line in ("Synchronous Multiplication working correctly", "Double buffered multiplication working correctly",
                 "Phased (MemEfficientSpGEMM) multiplication working correctly"):
        assert line in r.stdout


def test_restriction_tile_restatement(cbg):
    from helpers import restriction_host
    from combblas_spmm_test_amd import sub_tile, block_range
    g = restriction_host(10, 2)
    assert_tiles_equal(cbg.restriction_tile(10, 2).to_host(), g)
    for pos in [(0, 0), (0, 1), (1, 0), (1, 1)]:
        r0, r1 = block_range(g["m"], 2, pos[0])
        c0, c1 = block_range(g["n"], 2, pos[1])
        assert_tiles_equal(cbg.restriction_tile(10, 2, grid=(2, 2), pos=pos).to_host(), sub_tile(g, r0, r1, c0, c1))


def test_tile_transpose_and_dim_apply(cbg):
    from helpers import transpose_host
    d = load_npz("largeseq_A.npz")
    t = cbg.Tile.from_dict(d)
    assert_tiles_equal(t.transpose().to_host(), transpose_host(d))
    assert_tiles_equal(t.transpose().transpose().to_host(), d)
    rng = np.random.default_rng(3)
    vc, vr = rng.uniform(-2, 2, d["n"]), rng.uniform(-2, 2, d["m"])
    t.dim_apply(cbg.Column, vc)
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    assert_tiles_equal(t.to_host(), dict(d, val=d["val"] * vc[cols]))
    t.dim_apply(cbg.Row, vr, "plus")
    assert_tiles_equal(t.to_host(), dict(d, val=d["val"] * vc[cols] + vr[d["ir"]]))
    z = cbg.Tile.from_host(4, 3, np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))
    zt = z.transpose()
    assert (zt.m, zt.n, zt.nnz) == (3, 4, 0)


def test_galerkin_single_rank(cbg):
    """S*(A*T) with S = T^T (GalerkinNew.cpp:96-110) vs the oracle on host-built operands."""
    from helpers import add_diag_host, restriction_host, transpose_host
    g = _self_grid(cbg)
    scale = 10
    n = 1 << scale
    dv = np.random.default_rng(7).uniform(0.5, 1.5, n)
    L = cbg.SpParMat.rmat(g, scale)
    Ah = add_diag_host(L.tile.to_host(), dv)
    A = cbg.SpParMat.from_global(g, Ah)
    T = cbg.SpParMat.restriction(g, scale, 2)
    S = T.copy()
    S.Transpose()
    Th = restriction_host(scale, 2)
    Sh = transpose_host(Th)
    assert_tiles_equal(S.tile.to_host(), Sh)
    SAT = cbg.PSpGEMM(S, cbg.PSpGEMM(A, T))
    ref = oracle_local(Sh, oracle_local(Ah, Th))
    bound = oracle_local(abs_tile(Sh), oracle_local(abs_tile(Ah), abs_tile(Th)))["val"]
    assert_tiles_equal(SAT.tile.to_host(), ref, rtol=1e-12, bound=bound)
    # splitting approach: S*(L*T) + (S*D)*T == S*(A*T)
    SLT = cbg.PSpGEMM(S, cbg.PSpGEMM(L, T))
    SD = S.copy()
    SD.DimApply(cbg.Column, dv)
    SLT += cbg.PSpGEMM(SD, T)
    assert SLT == SAT
    # the min-plus variant (config 5): S*(A*T) on MinPlusSRing, exact against the oracle
    SATm = cbg.PSpGEMM(S, cbg.PSpGEMM(A, T, cbg.MinPlusSRing), cbg.MinPlusSRing)
    refm = oracle_local(Sh, oracle_local(Ah, Th, sr="minplus"), sr="minplus")
    assert_tiles_equal(SATm.tile.to_host(), refm)
    g.destroy()


@pytest.mark.parametrize("layout", ["1x1", "2x4"])
def test_galerkin_scale22_vs_oracle(cbg, layout):
    """Config 5 at its own size: GalerkinNew's S*(A*T) (GalerkinNew.cpp:96-110) for the
    scale-22 R-MAT A (plus a diagonal) and the order-2 restriction T, plus-times within
    1e-12 of the oracle entry by entry (all operands are positive, so |S||A||T| is the
    oracle's product itself) and min-plus bit-exact.  1x1: one rank's PSpGEMMs.  2x4:
    config 5's grid, every rank's two products computed on this GPU the way the PANEL
    SUMMA does after its broadcasts (AT(:, c) = A T(:, c), then S(r, :) AT(:, c)), each
    rank tile checked against its block of the oracle's product."""
    from helpers import restriction_host, transpose_host
    from combblas_spmm_test_amd import block_range, sub_tile
    scale, n = 22, 1 << 22
    dv = np.random.default_rng(7).uniform(0.5, 1.5, n)
    g = _self_grid_1x1(cbg)
    L = cbg.SpParMat.rmat(g, scale)
    D = cbg.Tile.from_host(n, n, np.arange(n + 1, dtype=np.int64), np.arange(n, dtype=np.int32),
                           np.arange(n, dtype=np.int32), dv)
    Ad = cbg.MergeAll([L.tile, D])  # A = L + diag(dv) (L has no loops)
    L.tile.free()
    D.free()
    Ah = Ad.to_host()
    assert len(Ah["ir"]) == G["rmat"]["s22_ef16"]["A"]["nnz"] + n
    Th = restriction_host(scale, 2)
    Sh = transpose_host(Th)
    for sr in ("plus", "minplus"):
        ref = oracle_local(Sh, oracle_local(Ah, Th, sr=sr), sr=sr)
        rtol = 1e-12 if sr == "plus" else 0.0
        if layout == "1x1":
            A = cbg.SpParMat(Ad, g, n, n)
            T = cbg.SpParMat.restriction(g, scale, 2)
            S = T.copy()
            S.Transpose()
            SAT = cbg.PSpGEMM(S, cbg.PSpGEMM(A, T, sr), sr)
            assert_tiles_equal(SAT.tile.to_host(), ref, rtol=rtol, bound=ref["val"])
            for X in (T, S, SAT):
                X.tile.free()
            continue
        pr, pc = 2, 4
        nc = n // 2
        for c in range(pc):
            c0, c1 = block_range(nc, pc, c)
            Tc = cbg.Tile.from_dict(sub_tile(Th, 0, n, c0, c1))
            ATc = cbg.LocalHybridSpGEMM(Ad, Tc, sr)
            for r in range(pr):
                r0, r1 = block_range(nc, pr, r)
                Sr = cbg.Tile.from_dict(sub_tile(Sh, r0, r1, 0, n))
                SATrc = cbg.LocalHybridSpGEMM(Sr, ATc, sr)
                want = sub_tile(ref, r0, r1, c0, c1)
                assert_tiles_equal(SATrc.to_host(), want, rtol=rtol, bound=want["val"])
                for X in (Sr, SATrc):
                    X.free()
            Tc.free()
            ATc.free()
    Ad.free()
    g.destroy()


def test_galerkin_driver():
    """tools/galerkin.py end to end (one rank): splitting check passes, timings reported."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "galerkin.py"), "--scale", "12", "--iters", "1",
                        "--minplus"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["splitting_correct"] and out["full_restriction_s"] > 0 and out["full_restriction_minplus_s"] > 0


def test_cpp_galerkin_driver():
    """tools/galerkin (C++ mirror: Transpose, DimApply, +=, PSpGEMM, operator==) on one rank."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "tools", "galerkin")
    if not os.path.exists(exe):
        pytest.skip("tools/galerkin not built (needs MPICH in /opt/conda)")
    r = subprocess.run([exe, "12", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Splitting approach is correct" in r.stdout


def _write_triples(path, d, binary=False):
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    rows = d["ir"].astype(np.int64)
    if binary:
        rec = np.zeros(len(rows), dtype=[("r", "<i8"), ("c", "<i8"), ("v", "<f8")])
        rec["r"], rec["c"], rec["v"] = rows, cols, d["val"]
        with open(path, "wb") as f:
            f.write(b"HKDT" + np.array([1, 24, 0, d["m"], d["n"], len(rows)], np.uint64).tobytes() + rec.tobytes())
        return
    with open(path, "w") as f:
        f.write(f"%% written by the test\n{d['m']} {d['n']} {len(rows)}\n")
        f.writelines(f"{r + 1} {c + 1} {float(v)!r}\n" for r, c, v in zip(rows, cols, d["val"]))


def test_cpp_galerkin_driver_files(tmp_path):
    """tools/galerkin with the reference's four file arguments (GalerkinNew.cpp:60-101):
    A and the off-diagonal L as text triples, T as HKDT binary, the diagonal as a
    vector file; ReadDistribute on the C++ mirror, then the splitting check."""
    import os
    import subprocess
    from helpers import add_diag_host, load_npz, restriction_host
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "tools", "galerkin")
    if not os.path.exists(exe):
        pytest.skip("tools/galerkin not built (needs MPICH in /opt/conda)")
    n = 1 << 10
    dv = np.random.default_rng(7).uniform(0.5, 1.5, n)
    Lh = load_npz("rmat_s10_ef16_A.npz")
    _write_triples(tmp_path / "A.txt", add_diag_host(Lh, dv))
    _write_triples(tmp_path / "L.txt", Lh)
    _write_triples(tmp_path / "T.bin", restriction_host(10, 2), binary=True)
    with open(tmp_path / "D.txt", "w") as f:
        f.write(f"{n} 1 {n}\n")
        f.writelines(f"{i + 1} 1 {float(v)!r}\n" for i, v in enumerate(dv))
    r = subprocess.run([exe] + [str(tmp_path / x) for x in ("A.txt", "L.txt", "D.txt", "T.bin")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Data read" in r.stdout and "Splitting approach is correct" in r.stdout


def _self_grid_1x1(cbg):
    class Self:
        def bcast(self, comm, arr, root):
            pass

        def allgather(self, comm, data):
            return data

    return cbg.CommGrid(0, 1, transport="host", host_comm=Self())


def test_block_split_and_blockspgemm(cbg):
    """SpParMat::BlockSplit (SpParMat.cpp:2974-3058) and BlockSpGEMM (BlockSpGEMM.h):
    blocks are the reference's sub-matrices (first n % b blocks one longer), and the
    C blocks at their offsets tile the golden A*A exactly (ReleaseTests/BlockedSpGEMM.cpp)."""
    from helpers import load_npz
    g = _self_grid_1x1(cbg)
    Ah = load_npz("rmat_s10_ef16_A.npz")
    Ch = load_npz("rmat_s10_ef16_C_local_plus.npz")
    A = cbg.SpParMat.from_global(g, Ah)
    B = cbg.SpParMat.from_global(g, Ah)
    blocks = A.BlockSplit(3, 2)
    roff, coff = cbg._block_offsets(Ah["m"], 3), cbg._block_offsets(Ah["n"], 2)
    assert roff == [0, 342, 683, 1024] and coff == [0, 512, 1024]
    for i in range(3):
        for j in range(2):
            assert_tiles_equal(blocks[i][j].tile.to_host(), cbg.sub_tile(Ah, roff[i], roff[i + 1], coff[j], coff[j + 1]))
    bs = cbg.BlockSpGEMM(A, B, 3, 2)
    assert bs.getBlockOffsets(True) == roff and bs.getBlockOffsets(False) == coff
    seen = 0
    while bs.hasNext():
        C, r0, c0 = bs.getNextBlock()
        rb, cb = roff.index(r0), coff.index(c0)
        assert (C.getnrow(), C.getncol()) == (roff[rb + 1] - r0, coff[cb + 1] - c0)
        assert_tiles_equal(C.tile.to_host(), cbg.sub_tile(Ch, r0, roff[rb + 1], c0, coff[cb + 1]))
        seen += 1
    assert seen == 6
    C, r0, c0 = bs.getBlockId(2, 1)
    assert (r0, c0) == (683, 512)
    assert A.BlockSplit(1, 1)[0][0] is A
    g.destroy()


def test_cpp_blockedspgemm_driver():
    """tools/blockedspgemm (ReleaseTests/BlockedSpGEMM.cpp on the C++ mirror header): the
    reference's per-block lines, and the blocks' nonzeros add up to nnz(A*B)."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "tools", "blockedspgemm")
    if not os.path.exists(exe):
        pytest.skip("tools/blockedspgemm not built (needs MPICH in /opt/conda)")
    mm = os.path.join(repo, "tests", "golden", "sevenvertex.mtx")
    r = subprocess.run([exe, mm, mm, "2", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()  # (RCCL may print a banner first)
    assert any(ln.startswith("A 7 7 12") for ln in lines) and any(ln.startswith("B 7 7 12") for ln in lines)
    blocks = [ln.split() for ln in lines if ln.startswith("block size")]
    assert [(b[2], b[3], b[6], b[7]) for b in blocks] == [("4", "3", "0", "0"), ("4", "2", "0", "3"),
                                                         ("4", "2", "0", "5"), ("3", "3", "4", "0"),
                                                         ("3", "2", "4", "3"), ("3", "2", "4", "5")]
    assert "BlockSpGEMM blocks cover A*B" in r.stdout


@pytest.mark.parametrize("scale,sr", [(20, "plus"), (21, "plus"), (20, "minplus")])
def test_local_digest_large_vs_oracle(cbg, scale, sr):
    """R-MAT 20/21 (4 and 8 row panels: panel groups, multi-slab pairs) against the
    oracle's digests (tests/golden/oracle_large.json, made by tools/check_scale.py)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        g = json.load(f)[f"s{scale}_ef16" + ("" if sr == "plus" else "_" + sr)]
    A = cbg.rmat_tile(scale, 16)
    B = cbg.rmat_tile(scale, 16)
    C = cbg.LocalHybridSpGEMM(A, B, sr)
    d = C.digest()
    C.free()
    assert d["nnz"] == g["nnz"] and d["nzc"] == g["nzc"] and d["hs"] == g["hs"] and d["hv"] == g["hv"], (d, g)
    assert d["unsorted"] == 0  # rows strictly ascending in every column (Dcsc::operator== compares ir exactly)
    sym = G["rmat"].get(f"s{scale}_ef16", {}).get("symbolic")
    if sym:  # the reference's own symbolic total
        assert d["nnz"] == sym["nnzC"]


def _cols_host(t, keep):
    """the columns j of host tile t with keep(j) (ids kept, same n)"""
    sel = np.flatnonzero(keep(t["jc"].astype(np.int64)))
    cnt = np.diff(t["cp"])[sel]
    starts = t["cp"][sel]
    idx = np.repeat(starts - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(int(cnt.sum()))
    return dict(m=t["m"], n=t["n"], cp=np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64),
                jc=t["jc"][sel].copy(), ir=t["ir"][idx], val=t["val"][idx])


@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_random_values_scale20_vs_oracle(cbg, sr):
    """SURVEY 8(d)'s random-valued variant at multi-panel scale: the R-MAT scale-20
    structure (R = 4 row panels: bitmap and hash (column, panel) pairs, panel groups,
    multi-slab pairs) with values U[-1, 1) from a hash of (row, col), which are not f32
    (the slab kernels' f64-value instantiations run); B = every 16th column of A.
    Entry by entry against the CPU oracle: plus-times within 1e-12 (|A||B|)_ij, min-plus
    exact.  The device values equal the host restatement bit for bit."""
    from helpers import random_values_host
    A = cbg.rmat_tile(20, 16).set_random_values()
    Ah = A.to_host()
    np.testing.assert_array_equal(Ah["val"], random_values_host(Ah)["val"])
    Bh = _cols_host(Ah, lambda j: j % 16 == 0)
    B = cbg.Tile.from_dict(Bh)
    C = cbg.LocalHybridSpGEMM(A, B, sr)
    st = cbg.last_stats()
    assert st["n_big"] > 0 and st["n_slabs"] > 0, st
    w = cbg.last_work_stats()
    # the f64-value instantiations of every family this shape reaches ran:
    # (column, panel) units and panel groups in the symbolic, bitmap slabs with
    # kept bitmaps (both classes), rank and hash slabs, the small-column passes
    for k in ("sym_panel_units", "sym_group_units", "bitmap_small_kept", "bitmap_large_kept", "esc_columns",
              "hash_bin_columns"):
        assert w[k] > 0, (k, w)
    assert sum(w["rank_N%d" % n] for n in (1024, 2048, 4096)) > 0, w
    assert sum(w["hash_T%d" % t] for t in (512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192)) > 0, w
    assert sum(w["group_rank_N%d" % n] for n in (2048, 4096)) > 0, w
    Ch = C.to_host()
    C.free()
    ref = oracle_local(Ah, Bh, sr)
    if sr == "plus":
        assert_tiles_equal(Ch, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
    else:
        assert_tiles_equal(Ch, ref)
    A.free()
    B.free()


def test_random_values_scale24_piece_vs_oracle(cbg):
    """The same at scale 24 (R = 64 row panels, panel groups of up to 64 panels, hash
    slabs spanning up to 2^24 rows): C's B-column piece 0 of 512 (B = A's columns
    [0, n/512)) with random values, entry by entry within 1e-12 (|A||B|)_ij."""
    n = 1 << 24
    A = cbg.rmat_tile(24, 16).set_random_values()
    left, right = A.split_cols(n // 512)
    right.free()
    C = cbg.LocalHybridSpGEMM(A, left)
    Ch = C.to_host()
    C.free()
    Ah, Bh = A.to_host(), left.to_host()
    A.free()
    left.free()
    ref = oracle_local(Ah, Bh)
    bound = oracle_local(abs_tile(Ah), abs_tile(Bh))["val"]
    assert len(Ch["ir"]) == _oracle_large("s24_ef16_pieces")["digests"]["0"]["nnz"]
    assert_tiles_equal(Ch, ref, rtol=RTOL, bound=bound)


S22_VALUE_PIECES = (0, 37, 101, 166, 230, 295, 359, 424, 480, 511)


def test_random_values_scale22_pieces_vs_oracle(cbg):
    """The f64-value path at the headline's own shape: the
    scale-22 R-MAT tile (R = 16 row panels) with values U[-1, 1) from a hash of (row,
    col) -- A's values are then f64, so the slab kernels' f64 instantiations run, not
    the f32 narrowing of R-MAT's integer values -- times B-column pieces of 1/512 of
    the tile (B = A's columns [p n/512, (p+1) n/512)) for 10 pieces spread over the
    columns, the high-id end included.  Every piece has big columns over 16 panels:
    bitmap pairs (single- and multi-slab), rank slabs (single-panel sparse pairs),
    two-level rank slabs (panel groups), hash slabs (the smallest sparse slabs).  Entry by entry against the CPU oracle: plus-times
    within 1e-12 (|A||B|)_ij; min-plus exact on three of the pieces
    (mtSpGEMM.h:362-440 semantics, Dcsc::operator== dcsc.cpp:472-510)."""
    n = 1 << 22
    A = cbg.rmat_tile(22, 16).set_random_values()
    Ah = A.to_host()
    work = None
    for p in S22_VALUE_PIECES:
        c0, c1 = p * (n // 512), (p + 1) * (n // 512)
        left, right = A.split_cols(c1)
        right.free()
        low, B = left.split_cols(c0)
        low.free()
        left.free()
        Bh = B.to_host()  # columns renumbered from 0, as C's
        for sr in (("plus", "minplus") if p in (0, 230, 511) else ("plus",)):
            C = cbg.LocalHybridSpGEMM(A, B, sr)
            st = cbg.last_stats()
            assert st["n_big"] > 0 and st["n_slabs"] > 0, (p, st)
            w = cbg.last_work_stats()
            work = w if work is None else {k: work[k] + w[k] for k in w}
            Ch = C.to_host()
            C.free()
            ref = oracle_local(Ah, Bh, sr)
            if sr == "plus":
                assert_tiles_equal(Ch, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
            else:
                assert_tiles_equal(Ch, ref)
        B.free()
    A.free()
    # every kernel family the docstring names ran with f64 values: symbolic units
    # and panel groups, both bitmap slab classes (kept bitmaps), all three rank
    # classes, both group rank classes, several hash-slab table sizes
    for k in ("sym_panel_units", "sym_group_units", "bitmap_small_kept", "bitmap_large_kept", "rank_N1024",
              "rank_N2048", "rank_N4096", "group_rank_N2048", "group_rank_N4096"):
        assert work[k] > 0, (k, work)
    assert sum(1 for t in (512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192) if work["hash_T%d" % t]) >= 2, work


@pytest.mark.parametrize("grank_min", ["-1", "0"])
def test_group_slabs_hash_or_rank_vs_oracle(cbg, grank_min):
    """Panel-group slabs either way (CBG_GRANK_MIN, read per call): -1 sends every
    group slab to the hash slabs (k_num_slab_hash, the larger tables among them), 0
    every group slab of a span <= 2^22 to the two-level rank (k_num_slab_grank, the
    small ones too).  Scale-20 R-MAT with U[-1,1) values times every 16th column
    (R = 4 panels, groups of 2 and 4), both semirings, entry by entry against the
    oracle (plus-times within 1e-12 (|A||B|)_ij, min-plus exact)."""
    import os
    old = os.environ.get("CBG_GRANK_MIN")
    os.environ["CBG_GRANK_MIN"] = grank_min
    try:
        A = cbg.rmat_tile(20, 16).set_random_values()
        Ah = A.to_host()
        Bh = _cols_host(Ah, lambda j: j % 16 == 0)
        B = cbg.Tile.from_dict(Bh)
        for sr in ("plus", "minplus"):
            C = cbg.LocalHybridSpGEMM(A, B, sr)
            w = cbg.last_work_stats()
            g = w["group_rank_N2048"] + w["group_rank_N4096"]
            big_hash = sum(w["hash_T%d" % t] for t in (2048, 3072, 4096, 6144, 8192))
            if grank_min == "-1":
                assert g == 0 and big_hash > 0, w
            else:
                assert g > 0, w
            Ch = C.to_host()
            C.free()
            ref = oracle_local(Ah, Bh, sr)
            if sr == "plus":
                assert_tiles_equal(Ch, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])
            else:
                assert_tiles_equal(Ch, ref)
        A.free()
        B.free()
    finally:
        if old is None:
            del os.environ["CBG_GRANK_MIN"]
        else:
            os.environ["CBG_GRANK_MIN"] = old


def _subprocess_local(env, code, timeout=600):
    """run `code` (prints one JSON line last) in a fresh process with `env` (the
    library reads its knobs once per process)"""
    import json
    import os
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **env), cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_random_values_scale22_piece_marking_pass(cbg, tmp_path):
    """The general k_num_slab (no kept bitmaps: the numeric marks its rows itself)
    with f64 values at the headline's shape: CBG_BITMAP_BUDGET_GB=0, scale-22 R-MAT
    with U[-1,1) values, B-column piece 230 of 512; entry by entry against the
    oracle within 1e-12 (|A||B|)_ij."""
    n = 1 << 22
    p = 230
    out = str(tmp_path / "c.npz")
    code = r"""
import sys, json, numpy as np
sys.path.insert(0, "tests")
from conftest import load_cbg
cbg = load_cbg()
n = 1 << 22
A = cbg.rmat_tile(22, 16).set_random_values()
left, right = A.split_cols(%d); right.free()
low, B = left.split_cols(%d); low.free(); left.free()
C = cbg.LocalHybridSpGEMM(A, B)
w = cbg.last_work_stats()
Ch = C.to_host()
np.savez(%r, **{k: Ch[k] for k in ("cp", "jc", "ir", "val")})
print(json.dumps(w))
""" % ((p + 1) * (n // 512), p * (n // 512), out)
    w = _subprocess_local({"CBG_BITMAP_BUDGET_GB": "0"}, code)
    assert w["bitmap_small_mark"] > 0 and w["bitmap_large_mark"] > 0, w
    assert w["bitmap_small_kept"] == 0 and w["bitmap_large_kept"] == 0, w
    z = np.load(out)
    Ch = dict(m=n, n=n // 512, cp=z["cp"], jc=z["jc"], ir=z["ir"], val=z["val"])
    A = cbg.rmat_tile(22, 16).set_random_values()
    Ah = A.to_host()
    A.free()
    Bh = _cols_host(Ah, lambda j: (j >= p * (n // 512)) & (j < (p + 1) * (n // 512)))
    Bh["n"] = n // 512
    Bh["jc"] = Bh["jc"] - p * (n // 512)
    ref = oracle_local(Ah, Bh)
    assert_tiles_equal(Ch, ref, rtol=RTOL, bound=oracle_local(abs_tile(Ah), abs_tile(Bh))["val"])


def test_pool_quarantine_scale20(cbg):
    """The pool's debug quarantine (CBG_POOL_QUARANTINE=1: a freed block is poisoned
    at once on another stream and not reused before the multiply's end), so a
    buffer released while a kernel can still read it would corrupt the product: the
    scale-20 A*A digest still equals the oracle's, rows sorted."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        g = json.load(f)["s20_ef16"]
    code = r"""
import sys, json
sys.path.insert(0, "tests")
from conftest import load_cbg
cbg = load_cbg()
A = cbg.rmat_tile(20, 16); B = cbg.rmat_tile(20, 16)
C = cbg.LocalHybridSpGEMM(A, B)
d = C.digest()
print(json.dumps({k: d[k] for k in ("nnz", "nzc", "hs", "hv", "unsorted")}))
"""
    d = _subprocess_local({"CBG_POOL_QUARANTINE": "1"}, code)
    assert (d["nnz"], d["nzc"], d["hs"], d["hv"], d["unsorted"]) == (g["nnz"], g["nzc"], g["hs"], g["hv"], 0), (d, g)


def test_local_scale24_column_pieces_vs_oracle(cbg):
    """Scale 24 (2^24 rows: R = 64 row panels, groups of up to 64 panels) pinned
    against the CPU oracle on a sample of C: column pieces p of 512 (B = A's
    columns [p n/512, (p+1) n/512), the slicing of tools/oracle_digest_pieces.py),
    each one local multiply on the GPU digested at its column offset, equal to the
    oracle's piece digest (tests/golden/oracle_large.json s24_ef16_pieces: the
    first pieces; the whole C, 183 G nonzeros, takes the oracle ~7 h on 6 cores)."""
    g = _oracle_large("s24_ef16_pieces")
    n = 1 << 24
    A = cbg.rmat_tile(24, 16)
    for key, ref in sorted(g["digests"].items(), key=lambda kv: int(kv[0])):
        ph = int(key)
        c0, c1 = ph * (n // g["pieces"]), (ph + 1) * (n // g["pieces"])
        left, right = A.split_cols(c1)
        right.free()
        low, B = left.split_cols(c0)
        low.free()
        left.free()
        C = cbg.LocalHybridSpGEMM(A, B)
        d = C.digest(0, c0)
        C.free()
        B.free()
        assert (d["nnz"], d["nzc"], d["hs"], d["hv"]) == (ref["nnz"], ref["nzc"], ref["hs"], ref["hv"]), (ph, d, ref)
        assert d["unsorted"] == 0
    A.free()


def test_local_scale22_ef8_resident(cbg):
    """SURVEY 8(d)'s scale-22 ef8 case: one local multiply whose C (9.08 G nonzeros,
    109 GB) stays resident on the GPU; its digest equals the oracle's
    (tests/golden/oracle_large.json) and nnz the reference's symbolic total."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        g = json.load(f)["s22_ef8"]
    A = cbg.rmat_tile(22, 8)
    B = cbg.rmat_tile(22, 8)
    assert A.nnz == G["rmat"]["s22_ef8"]["A"]["nnz"]
    C = cbg.LocalHybridSpGEMM(A, B)
    d = C.digest()
    st = cbg.last_stats()
    for t in (C, A, B):
        t.free()
    assert (d["nnz"], d["nzc"], d["hs"], d["hv"], d["unsorted"]) == (g["nnz"], g["nzc"], g["hs"], g["hv"], 0)
    sym = G["rmat"]["s22_ef8"]["symbolic"]
    assert d["nnz"] == sym["nnzC"] and st["flops"] == sym["flops"]


@pytest.mark.parametrize("sr,phases", [("plus", -1), ("plus", 3), ("plus", 4), ("minplus", -1)])
def test_phased_scale22_vs_oracle(cbg, sr, phases):
    """The bench's configuration: R-MAT scale-22 A*A as MemEfficientSpGEMM on one GPU with
    the phase count picked from device memory (PHASES_AUTO, what bench.py times: 2 phases),
    and 3 and 4 phases forced; each phase's C digested on the device as it is
    streamed; the sum equals the oracle's digest of the whole C (24.8 G nonzeros,
    tests/golden/oracle_large.json; min-plus too) and nnz the reference's symbolic total."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_large.json")) as f:
        g = json.load(f)["s22_ef16" + ("" if sr == "plus" else "_minplus")]
    grid = _self_grid_1x1(cbg)
    nv = 1 << 22
    A = cbg.SpParMat(cbg.rmat_tile(22, 16), grid, nv, nv)
    B = cbg.SpParMat(cbg.rmat_tile(22, 16), grid, nv, nv)
    parts = []
    cbg.MemEfficientSpGEMM(A, B, phases, sr=sr, on_phase=lambda ph, off, t: parts.append(t.digest(0, off)))
    plan = cbg.phase_plan()
    assert plan["phases"] == (phases if phases > 0 else plan["phases"]) and plan["automatic"] == (phases < 0)
    if phases < 0:
        assert 2 <= plan["phases"] <= 4 and plan["oom_splits"] == 0, plan
    hs = "%016x" % (sum(int(d["hs"], 16) for d in parts) % (1 << 64))
    hv = "%016x" % (sum(int(d["hv"], 16) for d in parts) % (1 << 64))
    nnz = sum(d["nnz"] for d in parts)
    A.tile.free()
    B.tile.free()
    grid.destroy()
    assert (nnz, hs, hv) == (g["nnz"], g["hs"], g["hv"])
    assert all(d["unsorted"] == 0 for d in parts)
    if sr == "plus":  # and the reference itself (Mult_AnXBn_Synch in 16 B-column phases on the box's host)
        ref = G["rmat"]["s22_ef16"]["C_synch_plus_16phases"]
        assert (nnz, hs, hv) == (ref["nnz"], ref["hs"], ref["hv"])
    assert nnz == G["rmat"]["s22_ef16"]["symbolic"]["nnzC"]


def test_hbm_copy_bandwidth(cbg):
    """The measured roofline peak the bench reports: a plausible HBM3E copy rate."""
    g = cbg.hbm_copy_bandwidth(1 << 30, 5)
    assert 1000.0 < g < 8000.0


def _run_tool(path, args, timeout=300):
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, *path)
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def test_cpp_plugin_surface():
    """The tile type's plugin surface on the C++ mirror (SpMat.h:54-174): Create(essentials),
    GetEssentials, GetArrays (device addresses), Split/Merge, ColSplit/ColConcatenate,
    Transpose, LocalHybridSpGEMM -> SpTuples* -> SpDCCols(tuples, false) == Mult_AnXBn_Synch."""
    rc, out = _run_tool(("tools", "plugin_surface"), ["12"])
    assert rc == 0 and "PLUGIN OK" in out, out[-2000:]


def test_reference_adapter_runs():
    """integration/ParFriends_cbg.h inside a reference-compiled driver (oracle/_ref/adapter_check,
    test infrastructure built against /root/reference): the reference's own
    SpParMat / ParallelReadMM / Mult_AnXBn_Synch and the adapter's DoubleBuff/Synch on
    MI355X give equal products under the reference's SpParMat::operator==."""
    import os
    mm = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sevenvertex.mtx")
    rc, out = _run_tool(("oracle", "_ref", "adapter_check"), [mm])
    assert rc == 0 and "ADAPTER OK" in out, out[-2000:]


def test_reference_multtiming_unmodified_dropin():
    """The drop-in: the reference's ReleaseTests/MultTiming.cpp compiled UNMODIFIED with
    integration/ParFriends_cbg.h as one forced include (oracle/_ref/multtiming_dropin,
    test infrastructure built against /root/reference).  Its
    Mult_AnXBn_DoubleBuff<PlusTimesSRing<double,double>, double, SpDCCols<int,double>>
    and Mult_AnXBn_Synch calls (MultTiming.cpp:58,71,83,92) run on MI355X through the
    adapter's explicit specializations, on the reference's largeseq triples."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    os.environ["CBG_ADAPTER_VERBOSE"] = "1"
    try:
        rc, out = _run_tool(("oracle", "_ref", "multtiming_dropin"),
                            [os.path.join(gold, "largeseq_input1_0.triples"), os.path.join(gold, "largeseq_input2_0.triples")])
    finally:
        del os.environ["CBG_ADAPTER_VERBOSE"]
    assert rc == 0, out[-2000:]
    assert "[cbg adapter] Mult_AnXBn_DoubleBuff on MI355X" in out and "[cbg adapter] Mult_AnXBn_Synch on MI355X" in out
    assert "Double buffered multiplications finished" in out and "Synchronous multiplications finished" in out
    assert "29677" in out  # C's nonzeros, printed by the reference's SpParHelper::Print / PrintInfo


def test_reference_dropin_index_overflow():
    """The drop-in's download (integration/ParFriends_cbg.h cbg_download) fills the
    reference's Dcsc arrays directly and refuses a C whose nonzeros the index type
    cannot hold (the tuples constructor's (IT)t.size() wrapped silently): with the
    limit forced to 1000 (CBG_ADAPTER_IT_MAX) the unmodified MultTiming aborts with
    the message instead of building a wrong matrix (largeseq: 29,677 nonzeros)."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    os.environ["CBG_ADAPTER_IT_MAX"] = "1000"
    try:
        rc, out = _run_tool(("oracle", "_ref", "multtiming_dropin"),
                            [os.path.join(gold, "largeseq_input1_0.triples"), os.path.join(gold, "largeseq_input2_0.triples")])
    finally:
        del os.environ["CBG_ADAPTER_IT_MAX"]
    assert rc != 0, out[-2000:]
    assert "exceeds the index type's range (1000)" in out and "29677 nonzeros" in out, out[-2000:]


def test_tile_plugin_surface_python(cbg):
    """The Python mirror's SpDCCols surface: create(essentials), GetEssentials, GetArrays,
    Merge, ColSplit, concat_cols, Transpose (SpDCCols.cpp:733-970)."""
    ref = load_npz("rmat_s10_ef16_A.npz")
    A = cbg.Tile.from_dict(ref)
    ess = A.GetEssentials()
    assert ess == [len(ref["ir"]), ref["m"], ref["n"], len(ref["jc"])]
    R = cbg.Tile.create(ess)
    assert R.GetEssentials() == ess
    arr = A.GetArrays()
    assert [c for _, c, _ in arr["indarrs"]] == [ess[3] + 1, ess[3], ess[0]] and arr["numarrs"][0][1] == ess[0]
    l, r = A.split_cols(A.n // 2)
    M = cbg.Tile()
    M.Merge(l, r)
    assert_tiles_equal(M.to_host(), ref)
    parts = M.ColSplit(3)
    assert len(parts) == 3 and sum(p.n for p in parts) == ref["n"]
    K = cbg.Tile.concat_cols(parts)
    assert_tiles_equal(K.to_host(), ref)
    K.Transpose()
    K.Transpose()
    assert_tiles_equal(K.to_host(), ref)
