"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (the reference has
none; GPU sanitizers are unavailable on this pool, so they cover host code only).

`make -C oracle asan` compiles oracle/asan_harness.cpp with the CPU oracle restatement and the
product's host-only sources (gs_params.cpp config reader, gs_plan.cpp Z-slab plan, gs_hostsync.cpp
bounded wait / id hand-off / loopback hub) under
-fsanitize=address,undefined -fno-sanitize-recover=all; any report aborts the harness."""
import os
import subprocess

from conftest import REPO


def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "asan"], check=True, capture_output=True,
                   timeout=600)
    env = dict(os.environ, OMP_NUM_THREADS="4", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(REPO, "oracle", "build", "asan_harness")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan harness ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]


def test_hostsync_under_tsan():
    """The exchange layer's HIP-free host logic (gs_hostsync.cpp: loopback hub barrier/abort across rank
    threads, bounded wait, id file hand-off) under ThreadSanitizer."""
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "tsan"], check=True, capture_output=True,
                   timeout=600)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([os.path.join(REPO, "oracle", "build", "tsan_harness")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan harness ok" in r.stdout
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
