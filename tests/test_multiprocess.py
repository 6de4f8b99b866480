"""N>1 path: world-size-2/4 runs launched with torch.distributed.run (127.0.0.1).

CPU (gloo, no device work): the host transport's row/column broadcasts and
allgathers and the SpParMat::Owner block distribution.
GPU: the full SUMMA (panel + staged, DoubleBuff + Synch) with several ranks
sharing one GPU through the same transport, checked against the reference's
global digest (the digest is additive over tiles); and the same over RCCL
communicators of several ranks (one NCCL_HOSTID per rank: RCCL's socket
transport, since RCCL refuses ranks of one host on one GPU)."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    """a port p with p and p+1 (the TCP host-transport hub) free, drawn below the
    Linux ephemeral range so that outgoing connections cannot take it meanwhile"""
    import random
    rng = random.Random(os.getpid() ^ int.from_bytes(os.urandom(4), "little"))
    for _ in range(200):
        p = rng.randrange(20000, 32000, 2)
        try:
            for q in (p, p + 1):
                s = socket.socket()
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                s.bind(("127.0.0.1", q))
                s.close()
            return p
        except OSError:
            continue
    raise RuntimeError("no free port pair")


def launch(nproc, args, timeout=300, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(HERE, "mp_worker.py")] + args
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    # every rank's libcbg error first (the tail alone may show only the agreed code)
    errs = [ln for ln in out.splitlines() if "CbgError" in ln or "[cbg]" in ln]
    return r.returncode, "\n".join(errs[:16]) + "\n" + out


@pytest.mark.parametrize("grid", [(1, 2), (2, 1), (2, 2)])
@pytest.mark.parametrize("case", ["rmat", "largeseq"])
@pytest.mark.parametrize("transport", ["cpu", "cputcp"])
def test_host_transport_cpu(grid, case, transport):
    """gloo (GlooHostComm) and plain-TCP (TcpHostComm) transports: same collectives, same answers."""
    rc, out = launch(grid[0] * grid[1], [transport, str(grid[0]), str(grid[1]), case])
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.parametrize("grid", [(1, 2), (2, 2)])
def test_error_agreement_cpu(grid):
    """cbg_grid_agree over the TCP host transport without a device: one rank's code
    reaches every rank, and a rank that disappears makes the others' next
    collective return CBG_ERR_RCCL instead of hanging (the reference MPI_Aborts)."""
    rc, out = launch(grid[0] * grid[1], ["cputcp", str(grid[0]), str(grid[1]), "agree"], timeout=120)
    assert out.count("MPOK") == grid[0] * grid[1], out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("first", ["0", "1"])
@pytest.mark.parametrize("grid", [(1, 2), (2, 2), (2, 4)])
def test_fault_injection_gpu(grid, first):
    """An OOM-like failure in one rank's local multiply (CBG_FAULT_INJECT) is
    returned by every rank for PANEL and STAGED; the grid then multiplies fine
    (also when the failures are the grid's first calls)."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "fault"], timeout=300,
                     env={"CBG_FAULT_FIRST": first})
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(2, 2), (2, 4)])
def test_summa_scale18_multiprocess_gpu(grid):
    """Scale-18 A*A on 2x2 and 2x4 grids (tiles generated on device): STAGED DoubleBuff
    and Synch (generalized stages on 2x4) and pipelined PANEL == the reference's digest."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "rmat18"], timeout=600)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("min_ms", ["0", "1e9"])
@pytest.mark.parametrize("grid", [(2, 2), (4, 2)])
def test_summa_pipeline_decision_gpu(grid, min_ms):
    """The adaptive double buffering's two outcomes, forced: CBG_PIPELINE_MIN_MS=0 keeps
    the two B-column pieces (piece 1 broadcast while piece 0 multiplies), 1e9 rejoins
    them into one multiply after the rest's broadcast; both equal the reference."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "rmat"], timeout=600,
                     env={"CBG_PIPELINE_MIN_MS": min_ms})
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]
    want = "pieces 2" if min_ms == "0" else "pieces 1"
    assert want in out, out[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(1, 2), (2, 1), (2, 2), (2, 4), (4, 2)])
@pytest.mark.parametrize("case", ["rmat", "largeseq"])
def test_summa_multiprocess_gpu(grid, case):
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), case], timeout=600)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(1, 2), (2, 2)])
def test_multtest_multiprocess_gpu(grid):
    """MultTest's SpGEMM checks (ParallelReadMM + operator== against CControl) on a grid."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "multtest"], timeout=600)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(2, 2)])
def test_galerkin_multiprocess_gpu(grid):
    """GalerkinNew on a 2x2 grid: distributed Transpose + PSpGEMM + DimApply + += (host transport)."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "galerkin"], timeout=600)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(2, 1), (1, 2), (2, 2)])
def test_blockspgemm_multiprocess_gpu(grid):
    """BlockedSpGEMM: BlockSplit's redistribution of row / column blocks over a grid and
    the block products, checked against the golden A*A digest (host transport)."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "blockspgemm"], timeout=600)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid,case", [((1, 2), "rmat"), ((2, 2), "rmat"), ((2, 4), "largeseq"), ((2, 2), "galerkin"),
                                       ((2, 2), "fault"), ((2, 2), "rmat18")])
def test_rccl_multirank_gpu(grid, case):
    """RCCL with several ranks (mp_worker mode "rccl": one NCCL_HOSTID per rank, so the
    ranks sharing this GPU talk through RCCL's socket transport): the PANEL pipeline
    and STAGED SUMMA, phases, Transpose's send/recv and the error agreement on real
    RCCL communicators, against the same golden digests as the host transport."""
    rc, out = launch(grid[0] * grid[1], ["rccl", str(grid[0]), str(grid[1]), case], timeout=300)
    assert rc == 0 and "MPOK" in out and "transport rccl" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [None, "2", "1/4"])
@pytest.mark.parametrize("grid", [(1, 2), (2, 2)])
def test_narrow_uneven_pieces_gpu(grid, pipeline):
    """B tiles 15 and 16 columns wide (31 x 31 on a 1 x 2 grid): every rank cuts the same
    number of pipeline pieces (agreed from the narrowest tile), so PANEL never pairs
    one rank's extra agree() with another's broadcast; products within 1e-12 of the
    oracle for DoubleBuff/Synch, PANEL/STAGED and phases."""
    env = {"CBG_PIPELINE": pipeline} if pipeline else {}
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "narrow"], timeout=300, env=env)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(1, 2), (2, 2)])
def test_layout_mismatch_gpu(grid):
    """A tile off the block layout (one rank's A tile a column short): STAGED's stage
    slices and PANEL's gathered widths both return CBG_ERR_DIMMISMATCH on every rank
    (reference: MPI_Abort(DIMMISMATCH)); the grid multiplies correctly afterwards."""
    rc, out = launch(grid[0] * grid[1], ["gpu", str(grid[0]), str(grid[1]), "mismatch"], timeout=300)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gpu", "rccl"])
def test_redist_fault_gpu(mode):
    """Transpose and BlockSplit under the collective error protocol: a receive-buffer
    allocation that fails on one rank (CBG_FAULT_INJECT_REDIST) is returned by every
    rank of a 2x2 grid, over the host transport and over RCCL; both then work."""
    rc, out = launch(4, [mode, "2", "2", "redist_fault"], timeout=300)
    assert rc == 0 and "MPOK" in out, out[:1500] + out[-3000:]
