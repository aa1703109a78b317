"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer, and the
drop-in compile check (CPU only, no GPU).

* `make -C tests/cpp sanitize` builds the oracle (test infrastructure) and
  the HTTP upgrade parser from their sources with -fsanitize=address,undefined
  and runs a randomized driver over them (tests/cpp/test_host_sanitize.cpp:
  round trips, split streams, garbage streams and frame tables, mutated HTTP
  requests), and the handshake test with the product's host sources
  (ws.cpp, ws_api.cpp, ws_batch.cpp, http.cpp) instrumented;
* `make -C tests/cpp threads` builds the batches' cross-thread test
  (tests/cpp/test_batch_threads.cpp) with the product's host sources under
  ThreadSanitizer and under AddressSanitizer;
* `make -C tests/cpp dropin` compiles code written against the reference's
  WebSocket API signatures (Timespan overloads, PerformClientUpgrade(response,
  UUID), ConnectAsync) against include/server/ws/.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def _make(target):
    jobs = str(min(8, os.cpu_count() or 2))
    r = subprocess.run(["make", "-s", "-j" + jobs, "-C", CPP, target], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def _run(exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "0 failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_sanitized_oracle_and_http():
    _make("sanitize")
    _run(os.path.join(CPP, "_build", "san", "test_host_sanitize"))


def test_sanitized_handshake():
    _make("sanitize")
    _run(os.path.join(CPP, "_build", "san", "test_handshake"))


def test_batch_threads_tsan():
    """Forget / destroy a connection or transport on one thread
    while another flushes, and destroy a session whose frames sit in another
    thread's BatchScope; ADVICE r4: a server's batched receive and send
    switched on and off while IO threads read and send, every frame delivered
    once (tests/cpp/test_batch_threads.cpp, ThreadSanitizer)."""
    _make("threads")
    exe = os.path.join(CPP, "_build", "san", "test_batch_threads_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "0 failures" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_batch_threads_asan():
    _make("threads")
    _run(os.path.join(CPP, "_build", "san", "test_batch_threads_asan"))


def test_concurrent_create_tsan():
    """Eight threads create codec contexts at once (round 4's getenv crash in
    wsg_create): under ThreadSanitizer, without a device every wsg_create
    fails the same clean way (tests/cpp/test_concurrent_create.cpp; the GPU
    run is tests/test_gpu_cpp_api.py::test_concurrent_context_creation)."""
    _make("threads")
    exe = os.path.join(CPP, "_build", "san", "test_concurrent_create_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_reference_api_compiles():
    _make("dropin")
