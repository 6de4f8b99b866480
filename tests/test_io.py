"""Matrix Market reading with SpParMat::ParallelReadMM semantics (CPU, no device work).

The bundled sevenvertex.mtx (a data file of the reference's ReleaseTests) must read
to exactly the tile the reference itself read (golden sevenvertex_A.npz, made by
oracle/_ref readmm); the other cases pin SpHelper::push_to_vectors and
SpTuples::RemoveDuplicates behaviour on small synthetic files."""
import os

import numpy as np

from conftest import load_cbg
from helpers import load_npz

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def dense(d):
    out = np.zeros((d["m"], d["n"]))
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    out[d["ir"], cols] = d["val"]
    return out


def test_sevenvertex_matches_reference_read():
    cbg = load_cbg()
    d = cbg.read_mm(os.path.join(GOLD, "sevenvertex.mtx"))
    r = load_npz("sevenvertex_A.npz")
    for k in ("cp", "jc", "ir", "val"):
        assert np.array_equal(d[k], r[k]), k
    c = cbg.read_mm(os.path.join(GOLD, "sevenvertex_C.mtx"))
    rc = load_npz("sevenvertex_C_local_plus.npz")
    for k in ("cp", "jc", "ir", "val"):
        assert np.array_equal(c[k], rc[k]), k


def test_symmetric_pattern_duplicates(tmp_path):
    cbg = load_cbg()
    p = tmp_path / "s.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n% comment\n4 4 4\n2 1 1.5\n3 3 2.0\n4 2 -1\n2 1 7\n")
    d = cbg.read_mm(str(p))
    D = dense(d)
    assert D[1, 0] == 7 and D[0, 1] == 7           # duplicate (2,1) combined with max, mirrored
    assert D[2, 2] == 2 and D[3, 1] == -1 and D[1, 3] == -1
    assert len(d["ir"]) == 5
    d = cbg.read_mm(str(p), binop="plus")
    assert dense(d)[1, 0] == 8.5
    p.write_text("%%MatrixMarket matrix coordinate pattern general\n3 5 3\n1 5\n3 1\n1 5\n")
    d = cbg.read_mm(str(p))
    D = dense(d)
    assert D.shape == (3, 5) and D[0, 4] == 1 and D[2, 0] == 1 and len(d["ir"]) == 2
    p.write_text("%%MatrixMarket matrix coordinate integer general\n2 2 2\n0 1 5\n1 0 3\n")
    D = dense(cbg.read_mm(str(p), onebased=False))
    assert D[0, 1] == 5 and D[1, 0] == 3
    p.write_text("%%MatrixMarket matrix coordinate real general\n3 3 0\n")
    d = cbg.read_mm(str(p))
    assert d["m"] == 3 and len(d["ir"]) == 0 and len(d["cp"]) == 1


def test_read_distribute_matches_reference():
    """SpParMat::ReadDistribute triples files (data files of the reference's tests:
    ReleaseTests/small_nonsym.mtx, largeseq/input{1,2}_0) read to exactly the
    tiles the reference's own ReadDistribute produced (golden *_A/_B.npz, made by
    oracle/_ref readtriples)."""
    cbg = load_cbg()
    for f, g in (("small_nonsym.triples", "small_nonsym_A.npz"), ("largeseq_input1_0.triples", "largeseq_A.npz"),
                 ("largeseq_input2_0.triples", "largeseq_B.npz")):
        d = cbg.read_triples(os.path.join(GOLD, f))
        r = load_npz(g)
        assert (d["m"], d["n"]) == (r["m"], r["n"]), f
        for k in ("cp", "jc", "ir", "val"):
            assert np.array_equal(d[k], r[k]), (f, k)


def test_read_distribute_binary_and_nonum(tmp_path):
    """HKDT binary triples (FileHeader.h, 0-based int64/int64/double records) and
    text lines without a value (read as 1, ScalarReadSaveHandler::getNoNum)."""
    cbg = load_cbg()
    r = cbg.read_triples(os.path.join(GOLD, "largeseq_input1_0.triples"))
    cols = np.repeat(r["jc"].astype(np.int64), np.diff(r["cp"]))
    rec = np.zeros(len(cols), dtype=[("r", "<i8"), ("c", "<i8"), ("v", "<f8")])
    rec["r"], rec["c"], rec["v"] = r["ir"], cols, r["val"]
    p = tmp_path / "b.bin"
    with open(p, "wb") as f:
        f.write(b"HKDT")
        f.write(np.array([1, 24, 0, r["m"], r["n"], len(cols)], np.uint64).tobytes())
        f.write(rec[np.random.default_rng(0).permutation(len(rec))].tobytes())
    b = cbg.read_triples(str(p))
    for k in ("cp", "jc", "ir", "val"):
        assert np.array_equal(b[k], r[k]), k
    q = tmp_path / "t.txt"
    q.write_text("% c\n3 3 3\n1 1\n3 2 5.5\n2 2\n")
    d = cbg.read_triples(str(q))
    assert dense(d).tolist() == [[1, 0, 0], [0, 1, 0], [0, 5.5, 0]]
    v = tmp_path / "v.txt"
    v.write_text("4 1 2\n2 1 0.5\n4 1 -3\n")
    assert cbg.read_vector(str(v)).tolist() == [0, 0.5, 0, -3]
