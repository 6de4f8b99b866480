#!/usr/bin/env python3
"""bench.py -- nnz(C)/s of R-MAT A*A through the MI355X 2D-SUMMA SpGEMM path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--phases P]
                  [--algo doublebuff|synch] [--exec panel|staged] [--no-cpu-baseline]
                  [--values rmat|random] [--no-f64-leg] [--grid RxC]

One step = one complete Mult_AnXBn_DoubleBuff (reference ParFriends.h:798-997)
of Graph500 R-MAT A (SEED 0xDECAFBAD, ef 16, duplicates summed, loops removed)
by a deep copy of A, inputs resident in HBM in the 2D block layout.  Every N
runs the metric's scale 22 as MemEfficientSpGEMM (ParFriends.h:449) whose
phase count the library picks from device memory inside every step (N=1: C is
297 GB, more than one GPU's HBM: 2 B-column phases of ~149 GB, each phase's C
materialized in HBM and handed to the consumer; a C tile that fits runs as one
phase, the adaptive double-buffered DoubleBuff).  N>1 is launched by
torch.distributed.run, one rank per GPU, RCCL row/column communicators (grids
2x1, 2x2, 4x2 for 2/4/8: DESIGN.md section 6 gives the measured reason; --grid
1x2 / 2x4 runs BASELINE.md's shapes); an RCCL grid that cannot be created ends
the run non-zero (CBG_ALLOW_HOST_TRANSPORT=1 opts into the TCP host transport).
After the headline loop the same structure is timed again with f64 values
(f64_values / roofline.frac_f64_values): R-MAT's integer values let the slab
kernels read A as exact f32, real-valued matrices do not.  --scale 18 gives
configs[1] (C resident on one GPU).

Prints ONE JSON line on rank 0 (see the driver contract in DESIGN.md).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def load_cbg():
    import importlib.util
    name = "combblas_spmm_test_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "combblas-spmm-test_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# row-heavy grids: fewer row panels per rank tile, and the A block row (gathered
# before the first piece, exposed) spans fewer ranks than the B block column
# (broadcast piece by piece behind the multiply); measured per rank tile on one
# GPU: 2x1 7 % and 4x2 2-13 % faster than 1x2 / 2x4.  --grid RxC overrides.
GRIDS = {1: (1, 1), 2: (2, 1), 4: (2, 2), 8: (4, 2), 9: (3, 3), 16: (4, 4)}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scale", type=int, default=None)
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0xDECAFBAD)
    p.add_argument("--algo", choices=["doublebuff", "synch"], default="doublebuff")
    p.add_argument("--exec", dest="exec_mode", choices=["panel", "staged"], default="panel")
    p.add_argument("--phases", type=int, default=None,
                   help="MemEfficientSpGEMM phases (B column pieces): 0 (default) picks them from device "
                        "memory per call and streams C per phase; 1 keeps C resident; P > 1 forces P")
    p.add_argument("--phase-consumer", choices=["none", "digest"], default="none",
                   help="what the phase callback does with each phase's device C tile")
    p.add_argument("--grid", default=None, help="RxC process grid (default: GRIDS[N])")
    p.add_argument("--values", choices=["rmat", "random"], default="rmat",
                   help="rmat: the generator's duplicate counts (small integers); random: U[-1,1) from a hash of "
                        "(row, col) on the same structure (SURVEY 8(d)'s fp variant; A's values are then f64)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-f64-leg", dest="f64_leg", action="store_false",
                   help="skip the second timed loop with f64 (random) values on the same structure")
    p.add_argument("--cpu-threads", type=int, default=0, help="default: the CPUs this job may use")
    p.add_argument("--cpu-scale", type=int, default=20, help="scale of the CPU-baseline sample (reference Synch)")
    return p.parse_args()


def host_cores():
    """CPUs this job may use: the affinity mask capped by the cgroup CPU quota (the
    GPU box gives one GPU's job 16 of the host's cores), plus the host's lscpu shape."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) // int(per)
    except (OSError, ValueError):
        pass
    shape = {}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                shape[k.strip()] = v.strip()
    except (OSError, ValueError):
        pass
    cores = min(n, quota) if quota else n
    return max(cores, 1), dict(affinity=n, cgroup_quota=quota, **shape)


def newest_profile(suffix, accept=lambda d: True, root=None):
    """The newest committed record profiles/rNN_<suffix> (highest round NN) whose
    JSON `accept` takes, as (dict, path relative to the repo), or (None, None)."""
    import re
    root = root or os.path.join(REPO, "profiles")
    pat = re.compile(r"^r(\d+)_" + re.escape(suffix) + "$")
    found = []
    for name in os.listdir(root) if os.path.isdir(root) else []:
        m = pat.match(name)
        if m:
            found.append((int(m.group(1)), name))
    for _, name in sorted(found, reverse=True):
        path = os.path.join(root, name)
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if accept(d):
            return d, os.path.relpath(path, REPO)
    return None, None


def pmc_traffic(scale, ef, phases):
    """HBM bytes of one local multiply (all phases) at this configuration from the
    newest committed PMC passes (profiles/rNN_traffic_s<scale>.json, made by
    tools/profile_round.sh + tools/traffic.py: FETCH_SIZE calibrated on k_digest,
    + WRITE_SIZE), or None."""
    d, path = newest_profile("traffic_s%d.json" % scale, lambda d: d.get("scale") == scale and d.get("ef") == ef
                             and d.get("phases", 1) == phases)
    return (d["traffic_bytes"], path) if d else (None, None)


REF_DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")


def cpu_baseline_reference(scale, ef, threads, algos=("synch",)):
    """The reference itself (oracle/_ref/ref_driver: our driver linked against the
    reference's CombBLAS sources, built by __graft_entry__.build() where the
    reference exists; the binary travels with the tree) timed on host cores:
    GenGraph500Data + RemoveLoops (GenWriteMatrix.cpp:101-114), then
    Mult_AnXBn_<algo> at 1x1 with `threads` OpenMP threads, multiply time only
    (MPI_Wtime around the call); the best of `algos` is reported.
    Synch only by default: at scale 18 it is 2.5x faster than DoubleBuff
    (5.9 s vs 15.6 s, whose serial MergeAll dominates), so it is the better-of.
    None if the binary is absent or fails."""
    import subprocess
    import tempfile
    if not os.path.exists(REF_DRIVER):
        return None
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    with tempfile.TemporaryDirectory() as d:
        a = os.path.join(d, "A.cbgt")
        r = subprocess.run([REF_DRIVER, "gen", str(scale), str(ef), a], capture_output=True, text=True, env=env,
                           timeout=600)
        if r.returncode != 0:
            return None
        best = None
        for algo in algos:
            r = subprocess.run([REF_DRIVER, "mult", algo, "plus", a, a, "-"], capture_output=True, text=True,
                               env=env, timeout=900)
            if r.returncode != 0:
                return None
            nnz = dt = None
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    d_ = json.loads(line)
                    if d_.get("tag", "").startswith("C_"):
                        nnz = d_["nnz"]
                    if d_.get("tag", "").startswith("time_"):
                        dt = d_["seconds"]
            if nnz is None or not dt:
                return None
            if best is None or nnz / dt > best[0]:
                best = (nnz / dt, algo, dt, nnz)
    return best


def cpu_baseline_s22():
    """The newest reference run at the metric's own scale (profiles/rNN_cpu_reference_s22.json,
    tools/cpu_reference_s22.sh on the GPU box: Mult_AnXBn_Synch per B-column phase)."""
    d, path = newest_profile("cpu_reference_s22.json", lambda d: "value" in d)
    if d is not None:
        d["source"] = path
    return d


def cpu_baseline(scale, ef, seed, threads):
    """Oracle (plain-C restatement of the reference MPI+OpenMP path) timed on host cores.

    Times Mult_AnXBn_Synch and Mult_AnXBn_DoubleBuff restated (oracle/cbg_oracle.c)
    at 1x1 on `threads` OpenMP threads and reports the better one."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from helpers import oracle_rmat, oracle_summa  # test infrastructure: the checker/baseline only
    A = oracle_rmat(scale, ef, seed, threads)
    B = dict(A)
    best = None
    for algo in ("synch", "doublebuff"):
        t0 = time.perf_counter()
        C = oracle_summa(A, B, 1, algo, "plus", threads)
        dt = time.perf_counter() - t0
        nnz = len(C["ir"])
        del C
        r = nnz / dt
        if best is None or r > best[0]:
            best = (r, algo, dt, nnz)
    return best


def host_transport_fallback(rank, err, env=None):
    """The RCCL grid could not be created.  An N>1 line measured over the TCP
    host transport says nothing about RCCL over xGMI, so the bench exits
    non-zero (the driver sees a failed run, not a socket number with rc 0)
    unless the fallback is asked for explicitly: CBG_ALLOW_HOST_TRANSPORT=1
    (development runs of the N>1 logic with several ranks on one GPU)."""
    env = os.environ if env is None else env
    if env.get("CBG_ALLOW_HOST_TRANSPORT") != "1":
        raise SystemExit(f"[bench] rank {rank}: RCCL grid unavailable ({err}); not falling back to the TCP "
                         "host transport (set CBG_ALLOW_HOST_TRANSPORT=1 to allow it)")
    print(f"[bench] rank {rank}: RCCL grid unavailable ({err}); using the TCP host transport "
          "(CBG_ALLOW_HOST_TRANSPORT=1)", file=sys.stderr, flush=True)


def roofline_over_ranks(bytes_alg, ms_avg, n, peak_gbs):
    """Roofline of the local multiplies of all ranks as one job: the bytes of
    every rank's local multiply over the SLOWEST rank's device time, per GPU
    (sum of bytes / max ms / N), so a fast rank cannot stand for the grid
    (bytes_alg, ms_avg: per-rank lists).  Also the slowest rank's own rate."""
    slow = max(range(n), key=lambda r: ms_avg[r])
    achieved = sum(bytes_alg) / (ms_avg[slow] * 1e-3) / n / 1e9
    slowest_rank = bytes_alg[slow] / (ms_avg[slow] * 1e-3) / 1e9
    return {"achieved": achieved, "frac": achieved / peak_gbs, "slowest_rank": slow,
            "slowest_rank_achieved": slowest_rank, "slowest_rank_frac": slowest_rank / peak_gbs}


def f64_values_leg(cbg, grid, A, B, a, step, N):
    """The same product with f64 values (U[-1,1) from a hash of (row, col), the
    structure unchanged), timed like the headline: R-MAT's small-integer values
    let the slab kernels read A's values as exact f32 (bit-identical results),
    which real-valued matrices cannot.  Reported beside the headline (rmat
    values only; --values random is this leg as the headline)."""
    if a.values != "rmat":
        return None
    r0_ = cbg.block_range(1 << (a.scale if a.scale is not None else 22), grid.grid_rows, grid.prow)[0]
    c0_ = cbg.block_range(1 << (a.scale if a.scale is not None else 22), grid.grid_cols, grid.pcol)[0]
    A.tile.set_random_values(row_off=r0_, col_off=c0_)
    B.tile.set_random_values(row_off=r0_, col_off=c0_)
    cbg.synchronize()
    for _ in range(a.warmup):
        _, C = step()
        if C is not None:
            C.tile.free()
    step_s, ms = [], []
    for _ in range(a.steps):
        grid.barrier()
        ts = time.perf_counter()
        _, C = step()
        cbg.synchronize()
        step_s.append(grid.allreduce_max(time.perf_counter() - ts))
        if C is not None:
            C.tile.free()
        st = cbg.last_stats()
        ms.append(st["ms_symbolic"] + st["ms_numeric"])
    st = cbg.last_stats()
    col_nnz = [grid.allreduce_sum(B.tile.nnz if grid.pcol == c else 0) for c in range(grid.grid_cols)]
    bytes_alg = 16 * st["flops"] + 12 * st["nnz"] + 32 * col_nnz[grid.pcol] + 8 * B.tile.n
    ms_avg = sum(ms) / len(ms)
    rank = grid.rank
    ms_ranks = [grid.allreduce_max(ms_avg if r == rank else -1.0) for r in range(N)]
    bytes_ranks = [grid.allreduce_sum(bytes_alg if r == rank else 0) for r in range(N)]
    roof = roofline_over_ranks(bytes_ranks, ms_ranks, N, HBM_PEAK_GBS)
    med = sorted(step_s)[len(step_s) // 2]
    return {"values": "U[-1,1) from a hash of (row, col): A's values are f64 (no f32 narrowing)",
            "ms_per_step": med * 1e3, "step_ms": [round(x * 1e3, 3) for x in step_s],
            "achieved": roof["achieved"], "frac": roof["frac"], "ms_avg": ms_ranks[roof["slowest_rank"]]}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    N = max(world, 1)
    scale = a.scale if a.scale is not None else 22
    # phases: PHASES_AUTO (default) = MemEfficientSpGEMM picks them from device memory on
    # every call, inside the timed step (ParFriends.h:482-535; see
    # cbg_summa_spgemm_memeff): scale 22 on one GPU (C = 297 GB) streams C per
    # B-column phase, a C tile that fits runs as one phase (the adaptive
    # double-buffered DoubleBuff).  --phases 1 keeps C resident (Mult_AnXBn_*),
    # --phases P > 1 forces P phases.
    if a.phases is None:
        a.phases = -1  # PHASES_AUTO
    stream_c = a.phases != 1
    rehearsal = N > 1 and os.environ.get("CBG_RANK_HOSTIDS") == "1"
    if rehearsal:
        # several ranks on ONE GPU (a development box): one NCCL_HOSTID per rank
        # makes RCCL accept them (socket transport over loopback), so the N>1
        # code path runs end to end; its times say nothing about xGMI
        os.environ["NCCL_HOSTID"] = "cbg-bench-rank-%d" % rank
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    cbg = load_cbg()  # libcbg first: its HIP/RCCL runtimes are the ones the process uses
    cbg.lib().cbg_set_device(local_rank % max(1, cbg.device_count()))

    if a.grid:
        pr, pc = (int(x) for x in a.grid.lower().split("x"))
    else:
        pr, pc = GRIDS[N]
    if pr * pc != N:
        raise SystemExit(f"grid {pr}x{pc} does not have {N} ranks")
    if N == 1:
        class Self:
            def bcast(self, comm, arr, root):
                pass

            def allgather(self, comm, data):
                return data

        grid = cbg.CommGrid(0, 1, transport="host", host_comm=Self())
        transport = "none"
    else:
        # Host rendezvous for the RCCL unique id over plain TCP (MASTER_PORT+1):
        # the GPU processes never import torch, whose ROCm wheel would load a
        # second HIP runtime into the process.
        hc = cbg.TcpHostComm(rank, N, pr, pc, os.environ.get("MASTER_ADDR", "127.0.0.1"),
                             int(os.environ.get("MASTER_PORT", "29500")) + 1)
        uid = hc.bcast_object(cbg.CommGrid.unique_id() if rank == 0 else None, root=0)
        try:
            grid = cbg.CommGrid(rank, N, pr, pc, unique_id=uid, transport="rccl")
            transport = "rccl (socket rehearsal: all ranks on one GPU)" if rehearsal else "rccl"
            hc.close()
        except cbg.CbgError as e:
            host_transport_fallback(rank, e)  # exits non-zero unless explicitly allowed
            hc.allgather(0, b"0")  # every rank agrees on the fallback
            grid = cbg.CommGrid(rank, N, pr, pc, transport="host", host_comm=hc)
            transport = "host-tcp (opt-in fallback: NOT an RCCL/xGMI number)"

    t_gen = time.perf_counter()
    A = cbg.SpParMat.rmat(grid, scale, a.ef, a.seed)
    B = cbg.SpParMat.rmat(grid, scale, a.ef, a.seed)  # deep copy (aliasing is forbidden)
    if a.values == "random":
        r0_ = cbg.block_range(1 << scale, grid.grid_rows, grid.prow)[0]
        c0_ = cbg.block_range(1 << scale, grid.grid_cols, grid.pcol)[0]
        A.tile.set_random_values(row_off=r0_, col_off=c0_)
        B.tile.set_random_values(row_off=r0_, col_off=c0_)
    cbg.synchronize()
    t_gen = time.perf_counter() - t_gen
    mult = cbg.Mult_AnXBn_DoubleBuff if a.algo == "doublebuff" else cbg.Mult_AnXBn_Synch
    exec_mode = cbg.EXEC_PANEL if a.exec_mode == "panel" else cbg.EXEC_STAGED

    algo = cbg.DOUBLEBUFF if a.algo == "doublebuff" else cbg.SYNCH

    def step():
        """one complete multiply; returns (local nnz(C), resident C or None)"""
        if not stream_c:
            C = mult(A, B, exec_mode=exec_mode)
            return C.tile.nnz, C
        seen = [0]

        def consume(phase, off, t):  # C of one phase, resident until this returns
            seen[0] += t.nnz
            if a.phase_consumer == "digest":
                t.digest(0, off)

        cbg.MemEfficientSpGEMM(A, B, a.phases, algo=algo, exec_mode=exec_mode, on_phase=consume)
        plans.append(cbg.phase_plan())
        return seen[0], None

    C = None
    plans = []
    for _ in range(a.warmup):
        _, C = step()
        if C is not None:
            C.tile.free()
            C = None
    # the measured side of the roofline, before the timed region (and again after)
    peaks = [cbg.hbm_copy_bandwidth(4 << 30, 10) for _ in range(2)] if rank == 0 else []
    # K steps, each bracketed by barrier + synchronize and timed as the max over
    # ranks; the whole loop is bracketed the same way (the driver contract)
    ms_local, step_s, pipe = [], [], []
    grid.barrier()
    cbg.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if C is not None:
            C.tile.free()
        grid.barrier()
        ts = time.perf_counter()
        nnz_local, C = step()
        cbg.synchronize()
        te = time.perf_counter()
        st = cbg.last_stats()
        ms_local.append(st["ms_symbolic"] + st["ms_numeric"])
        step_s.append(te - ts)
        pipe.append(cbg.summa_info())
    cbg.synchronize()
    grid.barrier()
    dt = time.perf_counter() - t0
    dt = grid.allreduce_max(dt)
    step_s = [grid.allreduce_max(x) for x in step_s]
    med = sorted(step_s)[len(step_s) // 2] if len(step_s) % 2 else \
        0.5 * (sorted(step_s)[len(step_s) // 2 - 1] + sorted(step_s)[len(step_s) // 2])
    nnz_c = grid.allreduce_sum(nnz_local)
    st = cbg.last_stats()
    flops = grid.allreduce_sum(st["flops"])
    # algorithmic bytes of this rank's local multiply:
    # 16F + 12 nnz(C) + 32 nnz(B) + 8 n, B = the rank's B block column
    col_nnz = [grid.allreduce_sum(B.tile.nnz if grid.pcol == c else 0) for c in range(pc)]
    bytes_alg = 16 * st["flops"] + 12 * st["nnz"] + 32 * col_nnz[grid.pcol] + 8 * B.tile.n
    ms_avg = sum(ms_local) / len(ms_local)
    # every rank's bytes and device ms (one max-reduction per rank: N <= 16)
    ms_ranks = [grid.allreduce_max(ms_avg if r == rank else -1.0) for r in range(N)]
    bytes_ranks = [grid.allreduce_sum(bytes_alg if r == rank else 0) for r in range(N)]
    roof = roofline_over_ranks(bytes_ranks, ms_ranks, N, HBM_PEAK_GBS)
    achieved = roof["achieved"]
    f64 = None
    if a.f64_leg:
        if C is not None:
            C.tile.free()
            C = None
        n_plans = len(plans)
        f64 = f64_values_leg(cbg, grid, A, B, a, step, N)
        del plans[n_plans:]  # the headline's phase plans only

    phases_run = plans[-1]["phases"] if plans else 1
    if rank == 0:
        traffic, traffic_src = pmc_traffic(scale, a.ef, phases_run) if N == 1 and a.values == "rmat" else (None, None)
        peaks += [cbg.hbm_copy_bandwidth(4 << 30, 10) for _ in range(2)]
        peak_measured = max(peaks)
        out = {
            "metric": "nnz(C)/sec for A·A (R-MAT scale %d) at %d GPUs" % (scale, N),
            "value": nnz_c / med,
            "unit": "nnz(C)/s",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": med * 1e3,
            "higher_is_better": True,
            # every N multiplies the same scale-22 problem (total work fixed)
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic Graph500 R-MAT (SEED 0xDECAFBAD), generated on device" + (
                "; values U[-1,1) from a hash of (row, col)" if a.values == "random" else ""),
            "timing": {"value_from": "median over the steps of (barrier; step; synchronize) max over ranks "
                                     "(BASELINE.md: median of >= 5)",
                       "step_ms": [round(x * 1e3, 3) for x in step_s],
                       "loop_ms_per_step": dt / a.steps * 1e3, "value_loop_mean": nnz_c * a.steps / dt},
            "config": {"workload": "R-MAT scale-%d ef%d A·A, Mult_AnXBn_%s, %s" % (
                scale, a.ef, "DoubleBuff" if a.algo == "doublebuff" else "Synch", a.exec_mode),
                "scale": scale, "edgefactor": a.ef, "grid": "%dx%d" % (grid.grid_rows, grid.grid_cols),
                "values": a.values,
                "nnz_C": nnz_c, "flops": flops, "gen_s": round(t_gen, 3),
                "big_columns": st["n_big"], "slabs": st["n_slabs"], "transport": transport,
                "phases": phases_run,
                "phase_plan": ({"automatic": plans[-1]["automatic"], "phases_per_step": [p_["phases"] for p_ in plans[-a.steps:]],
                                "flops_rank0": plans[-1]["flops"], "nnz_est_rank0": plans[-1]["nnz_est"],
                                "c_budget_gb_rank0": round(plans[-1]["c_budget_bytes"] / 1e9, 1),
                                "oom_splits": plans[-1]["oom_splits"],
                                "plan_ms_per_step": [round(p_["plan_ms"], 2) for p_ in plans[-a.steps:]],
                                "rule": "MemEfficientSpGEMM(phases=PHASES_AUTO): flops of the rank's product from tile count "
                                        "vectors (x the compression of an exact symbolic of a sample when the flops "
                                        "bound asks for > 1 phase), 12 B per entry against 60 % of the free HBM, "
                                        "inside each timed step"}
                               if plans else None),
                "double_buffering": {"pieces": [p_["pieces"] for p_ in pipe],
                                     "decision": [["one piece", "pipelined", "adaptive: pipelined",
                                                   "adaptive: rejoined", "fixed pipeline"][p_["rule"]]
                                                  if p_["pieces"] > 1 or p_["rule"] else "one piece" for p_ in pipe],
                                     "bytes_bcast_rank0": [p_["bytes_recv"] for p_ in pipe],
                                     "exposed_comm_ms": [round(p_["exposed_comm_ms"], 3) for p_ in pipe],
                                     "bcast_ms_piece0": [round(p_["bcast_ms_piece0"], 3) for p_ in pipe],
                                     "est_hidden_ms": [round(p_["est_hidden_ms"], 3) for p_ in pipe],
                                     "piece_cost_ms": [round(p_["piece_cost_ms"], 3) for p_ in pipe],
                                     "rule": "the A block row's gather and B piece 0 (1/8 of the columns) in one "
                                             "broadcast group; on RCCL grids with > 1 remote B tile per grid column "
                                             "piece 1 is broadcast while piece 0 multiplies; with one remote B tile "
                                             "(or the host transport) only when the first group's measured time, "
                                             "scaled to the rest, exceeds what an extra piece costs: max(3 ms, 4 % of "
                                             "the previous step's local multiply).  exposed_comm_ms = rank 0's "
                                             "compute-stream waits for the broadcasts (HIP events)"}
                if N > 1 else None,
                "C": "materialized per phase in HBM, handed to a %s consumer" % a.phase_consumer if stream_c
                     else "resident in HBM"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "peak_measured": peak_measured, "frac_measured": achieved / peak_measured,
                         "peak_measured_method": "16-B/lane device copy of 4 GiB x10 (read+write bytes), "
                                                 "cbg_hbm_copy_bandwidth: the fastest of 8 copy shapes (grid-stride "
                                                 "or one launch streaming the buffer, 1/4/8 loads in flight per "
                                                 "lane, nontemporal or not) swept on the first call; best of 2 "
                                                 "before and 2 after the timed region",
                         "peak_measured_runs": peaks,
                         "traffic_source": traffic_src,
                         "kernel": "local SpGEMM pipeline (symbolic+numeric) of every rank",
                         "achieved_rule": "sum over ranks of bytes_alg / the slowest rank's device ms / N (per GPU)",
                         "ms_avg": ms_ranks[roof["slowest_rank"]], "bytes_alg": sum(bytes_ranks),
                         "ms_avg_ranks": [round(x, 3) for x in ms_ranks], "bytes_alg_ranks": bytes_ranks,
                         "slowest_rank": roof["slowest_rank"], "slowest_rank_frac": roof["slowest_rank_frac"]},
        }
        if f64 is not None:
            out["roofline"]["frac_f64_values"] = f64["frac"]
            out["f64_values"] = f64
        if N == 1 and not a.no_cpu_baseline:
            # the reference at the metric's own scale (a committed run on the GPU box's
            # host, ~6 min) first; cpu_baseline below is the bounded live sample
            s22 = cpu_baseline_s22()
            if s22 is not None and scale == 22:
                s22["scale"] = 22
                s22["gpu_over_cpu"] = out["value"] / s22["value"]
                out["cpu_baseline_s22"] = s22
            cores, host = host_cores()
            threads = a.cpu_threads or cores
            cs = a.cpu_scale
            ref = cpu_baseline_reference(cs, a.ef, threads) if a.seed == 0xDECAFBAD else None
            if ref is not None:
                r, algo_, cdt, cnnz = ref
                out["cpu_baseline"] = {"value": r, "unit": "nnz(C)/s", "cores": threads, "kind": "reference",
                                       "scale": cs, "sample": "R-MAT scale-%d ef%d A*A, the reference's Mult_AnXBn_%s 1x1 "
                                                 "(oracle/_ref/ref_driver), %.1f s on %d threads" % (
                                                     cs, a.ef, algo_.capitalize(), cdt, threads),
                                       "host": host}
                # cross-check at scale 18: the reference vs our restatement on the same cores
                rr = cpu_baseline_reference(18, a.ef, threads)
                pr_ = cpu_baseline(18, a.ef, a.seed, threads)
                if rr and pr_:
                    out["cpu_baseline"]["crosscheck_s18"] = {"reference_synch": rr[0],
                                                             "port_best": pr_[0], "port_algo": pr_[1]}
            else:
                r, algo_, cdt, cnnz = cpu_baseline(cs, a.ef, a.seed, threads)
                out["cpu_baseline"] = {"value": r, "unit": "nnz(C)/s", "cores": threads, "kind": "port",
                                       "scale": cs, "sample": "R-MAT scale-%d ef%d A*A, oracle Mult_AnXBn_%s 1x1, %.1f s" % (
                                           cs, a.ef, algo_.capitalize(), cdt), "host": host}
        print(json.dumps(out), flush=True)
    if C is not None:
        C.tile.free()
    grid.destroy()


if __name__ == "__main__":
    main()
