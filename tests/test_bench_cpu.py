"""bench.py host logic without a GPU: the N>1 transport rule and the per-rank roofline
(Weak 6: an N>1 line must neither report the fastest rank's bandwidth nor
fall back to the TCP host transport silently)."""
import importlib.util
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_rccl_failure_exits_nonzero_without_opt_in():
    b = load_bench()
    with pytest.raises(SystemExit) as e:
        b.host_transport_fallback(3, RuntimeError("ncclCommInitRank failed"), env={})
    assert e.value.code not in (0, None)  # a message: exit status 1
    assert "CBG_ALLOW_HOST_TRANSPORT" in str(e.value.code)
    # opted in: no exit, the caller continues on the host transport
    b.host_transport_fallback(3, RuntimeError("x"), env={"CBG_ALLOW_HOST_TRANSPORT": "1"})


def test_rccl_failure_exit_status_of_a_process():
    """the same rule seen from outside: the interpreter exits with status 1"""
    code = ("import importlib.util,sys;s=importlib.util.spec_from_file_location('b',%r);"
            "m=importlib.util.module_from_spec(s);s.loader.exec_module(m);"
            "m.host_transport_fallback(0, RuntimeError('no RCCL'))") % os.path.join(REPO, "bench.py")
    env = {k: v for k, v in os.environ.items() if k != "CBG_ALLOW_HOST_TRANSPORT"}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert "not falling back" in r.stderr


def test_roofline_over_ranks_uses_the_slowest_rank():
    b = load_bench()
    # rank 1 is slow: the job's per-GPU rate is all bytes over rank 1's time / N
    r = b.roofline_over_ranks([100e9, 100e9], [50.0, 100.0], 2, 8000.0)
    assert r["slowest_rank"] == 1
    assert r["achieved"] == pytest.approx(200e9 / 0.1 / 2 / 1e9)  # 1000 GB/s per GPU
    assert r["frac"] == pytest.approx(1000.0 / 8000.0)
    assert r["slowest_rank_achieved"] == pytest.approx(100e9 / 0.1 / 1e9)
    # never the fastest rank's rate (2000 GB/s here)
    assert r["achieved"] < 100e9 / 0.05 / 1e9
    # one rank: the plain rate
    one = b.roofline_over_ranks([1.22e12], [430.0], 1, 8000.0)
    assert one["achieved"] == pytest.approx(1.22e12 / 0.43 / 1e9)


def test_default_grids_and_flags():
    b = load_bench()
    assert b.GRIDS[1] == (1, 1) and b.GRIDS[2][0] * b.GRIDS[2][1] == 2 and b.GRIDS[8][0] * b.GRIDS[8][1] == 8
    src = open(os.path.join(REPO, "bench.py")).read()
    assert "--no-f64-leg" in src and "frac_f64_values" in src


def test_newest_profile_lookup(tmp_path):
    """the CPU-baseline and traffic records come from the highest round present
    (a hard-coded round list skipped r04)"""
    import json
    b = load_bench()
    for rnd, v in (("r02", 65.6e6), ("r04", 68.9e6), ("r10", 70.0e6), ("r03", 1.0)):
        (tmp_path / ("%s_cpu_reference_s22.json" % rnd)).write_text(json.dumps({"value": v}))
    (tmp_path / "r11_cpu_reference_s22.json").write_text("not json")
    d, path = b.newest_profile("cpu_reference_s22.json", lambda d: "value" in d, root=str(tmp_path))
    assert d["value"] == 70.0e6 and path.endswith("r10_cpu_reference_s22.json")
    # a predicate skips records of other configurations
    d, _ = b.newest_profile("cpu_reference_s22.json", lambda d: d["value"] < 69e6, root=str(tmp_path))
    assert d["value"] == 68.9e6
    # the committed records: the newest round's s22 reference run
    s22 = b.cpu_baseline_s22()
    rounds = sorted(int(n[1:3]) for n in os.listdir(os.path.join(REPO, "profiles"))
                    if n.endswith("_cpu_reference_s22.json"))
    assert s22["source"] == "profiles/r%02d_cpu_reference_s22.json" % rounds[-1]
