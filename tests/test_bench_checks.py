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
