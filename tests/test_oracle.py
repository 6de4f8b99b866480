"""The CPU oracle (oracle/cbg_oracle.c) is pinned against the reference's own outputs
(tests/golden/, produced by oracle/_ref/ref_driver linked with the reference sources)."""
import numpy as np
import pytest

from helpers import (assert_digest_eq, assert_tiles_equal, digest, golden, load_npz, oracle_local, oracle_rmat,
                     oracle_summa, oracle_symbolic, oracle_edges, abs_tile)

G = golden()


@pytest.mark.parametrize("scale", [8, 10, 12, 14, 16])
def test_rmat_generator_matches_reference(scale):
    A = oracle_rmat(scale, 16)
    g = G["rmat"][f"s{scale}_ef16"]["A"]
    assert_digest_eq(digest(A), g)
    assert digest(A)["nzc"] == g["nzc"]


@pytest.mark.parametrize("scale", [8, 10])
def test_rmat_full_tile(scale):
    A = oracle_rmat(scale, 16)
    R = load_npz(f"rmat_s{scale}_ef16_A.npz")
    assert_tiles_equal(A, R)


@pytest.mark.parametrize("scale", [8, 10, 12, 14])
@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_local_hybrid_matches_reference(scale, sr):
    A = oracle_rmat(scale, 16)
    C = oracle_local(A, A, sr)
    assert_digest_eq(digest(C), G["rmat"][f"s{scale}_ef16"][f"C_local_{sr}"])


@pytest.mark.parametrize("scale", [8, 10])
def test_local_full_product(scale):
    A = oracle_rmat(scale, 16)
    for sr in ("plus", "minplus"):
        C = oracle_local(A, A, sr)
        assert_tiles_equal(C, load_npz(f"rmat_s{scale}_ef16_C_local_{sr}.npz"))


@pytest.mark.parametrize("algo", ["doublebuff", "synch"])
@pytest.mark.parametrize("scale", [8, 12])
def test_summa_1x1_and_2x2(algo, scale):
    A = oracle_rmat(scale, 16)
    g = G["rmat"][f"s{scale}_ef16"]
    C1 = oracle_summa(A, A, 1, algo)
    assert_digest_eq(digest(C1), g[f"C_{algo}_plus"])
    if algo == "doublebuff":
        C2 = oracle_summa(A, A, 2, algo)
        d = digest(C2)
        assert d["nnz"] == g["C_doublebuff_plus_p4"]["nnz"] and d["hv"] == g["C_doublebuff_plus_p4"]["hv"]


def test_heap_equals_hybrid():
    A = oracle_rmat(10, 16)
    assert_tiles_equal(oracle_local(A, A, heap=True), oracle_local(A, A))


def test_symbolic_totals():
    A = oracle_rmat(12, 16)
    f, n = oracle_symbolic(A, A)
    s = G["rmat"]["s12_ef16"]["symbolic"]
    assert int(f.sum()) == s["flops"] and int(n.sum()) == s["nnzC"] and int(n.max()) == s["maxcol"]


@pytest.mark.parametrize("name", ["sevenvertex", "small_nonsym", "largeseq"])
@pytest.mark.parametrize("sr", ["plus", "minplus"])
def test_bundled_inputs(name, sr):
    A = load_npz(f"{name}_A.npz")
    B = load_npz(f"{name}_B.npz") if name == "largeseq" else A
    ref = load_npz(f"{name}_C_local_{sr}.npz")
    C = oracle_local(A, B, sr)
    if sr == "plus":
        bound = oracle_local(abs_tile(A), abs_tile(B), "plus")["val"]
        assert_tiles_equal(C, ref, rtol=1e-12, bound=bound)
    else:
        assert_tiles_equal(C, ref)  # min-plus is exact
    for algo in ("doublebuff", "synch"):
        Cs = oracle_summa(A, B, 1, algo, sr)
        assert_tiles_equal(Cs, ref, rtol=1e-12, bound=np.abs(ref["val"]) + 1e-300 if sr == "minplus" else bound)


def test_edge_prefix_is_rank_independent():
    # Global edge ids are independent of the partition (RefGen21::compute_edge_range, RefGen21.h:263-269)
    s0, d0 = oracle_edges(10, 0, 4096)
    s1, d1 = oracle_edges(10, 1000, 2000)
    np.testing.assert_array_equal(s0[1000:2000], s1)
    np.testing.assert_array_equal(d0[1000:2000], d1)
