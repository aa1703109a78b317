"""bench.py's failure reporting: every leg's parity and
delivery checks and every leg error reach the top level, and the run exits
non-zero on any of them.  CPU only: imports bench.py without running it."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_failed_checks_all_green():
    b = _bench()
    extras = {"c3": {"spot_check": True, "roofline": {"frac": 0.77}},
              "c5_job": {"root_check": True, "encode_ms": 1.0},
              "echo_c1": {"per_read_1c": {"payload_ok": True}, "cpu_reference": {"1c_1t": {"payload_ok": True}}},
              "pcie_inclusive_all_ranks": {"check": True}}
    assert b.failed_checks(extras) == []


def test_failed_checks_finds_misses_and_errors():
    b = _bench()
    extras = {"c3": {"spot_check": False},
              "c4": {"error": "RuntimeError('boom')"},
              "c5_job": {"root_check": True},
              "c5_job_one_process": {"root_check": False},
              "session_batch": {"rx": {"delivered_ok": True}, "tx": {"error": "exit 1"}},
              "echo_c1": {"tcp_loopback": {"gpu_1c_1t": {"payload_ok": False}}},
              "lists": [{"wire_ok": False}]}
    got = b.failed_checks(extras)
    assert "c3.spot_check=False" in got
    assert any(g.startswith("c4:") for g in got)
    assert "c5_job_one_process.root_check=False" in got
    assert any(g.startswith("session_batch.tx:") for g in got)
    assert "echo_c1.tcp_loopback.gpu_1c_1t.payload_ok=False" in got
    assert "lists[0].wire_ok=False" in got
    assert len(got) == 6


def test_bench_gpus_n_starts_n_ranks():
    """`python bench.py --gpus 2` (the driver's N=1 command shape with N=2)
    starts two ranks itself (torch.distributed.run as a child process) and the
    line reports n_gpus 2; --dry-run keeps it to the launch path (gloo, no
    GPU work)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    assert line["root_ingress_expectation_GBps"] == 153.0


def test_bench_world_mismatch_fails():
    """A launch whose WORLD_SIZE is not --gpus exits non-zero instead of
    reporting another N."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=3" in r.stderr
