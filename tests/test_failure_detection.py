"""CPU-only tests of the failure-detection logic around the Z-slab exchange (SURVEY.md §5 "failure
detection"; the reference's contract is an `Exception: ...` print, src/main.cpp:107-109).

* The bounded wait that settles every RCCL call and every distributed stream sync
  (gs::boundedWait, gs_comm.cpp): completion, an injected ncclInternalError and a timeout.
* The loopback hub (the single-GPU multi-rank emulation): a rank that fails must release every other
  rank thread from its barriers, and the first failure is what is reported.
The real RCCL communicator's error path (GS_COMM_INJECT_ERROR) is exercised on the GPU in
tests/test_gpu_rccl.py."""
import ctypes as C
import time

import pytest

import gpusolve as gsv


def wait(scenario, k, timeout):
    buf = C.create_string_buffer(512)
    rc = gsv.driver().gs_debug_bounded_wait(scenario, k, timeout, buf, 512)
    return rc, buf.value.decode()


def test_bounded_wait_completes():
    assert wait(0, 1, 1.0) == (0, "")
    assert wait(0, 5000, 5.0) == (0, "")  # past the spin phase into the back-off


def test_bounded_wait_reports_async_error():
    rc, msg = wait(1, 3, 5.0)
    assert rc == 1
    assert msg.startswith("debug wait: ") and "internal error" in msg


def test_bounded_wait_times_out():
    t0 = time.monotonic()
    rc, msg = wait(2, 0, 0.3)
    el = time.monotonic() - t0
    assert rc == 1 and "timed out after" in msg
    assert 0.3 <= el < 5.0


@pytest.mark.parametrize("nranks,failing", [(2, 0), (2, 1), (4, 2), (8, 7), (1, 0)])
def test_loopback_hub_abort_unwinds_every_rank(nranks, failing):
    d = gsv.driver()
    n = d.gs_debug_loopback_abort(nranks, failing)
    assert n == nranks, "a rank thread was left parked in a barrier"
    assert d.gs_last_error().decode() == f"rank {failing} failed"


# ---- the RCCL id's file hand-off of a multi-process GpuSolve-hip run (gs_comm.cpp publishUid / awaitUid)
def _uid(seed):
    return (C.c_ubyte * 128)(*[(seed * 31 + i * 7) % 256 for i in range(128)])


def test_uid_handoff_round_trip(tmp_path):
    d = gsv.driver()
    path = str(tmp_path / "uid").encode()
    sent = _uid(3)
    assert d.gs_uid_publish(path, sent) == 0
    got = (C.c_ubyte * 128)()
    assert d.gs_uid_await(path, 1.0, got) == 0
    assert bytes(got) == bytes(sent)
    assert [p.name for p in tmp_path.iterdir()] == ["uid"]  # the temporary file was renamed into place


def test_uid_handoff_waits_for_a_late_publisher(tmp_path):
    import threading
    d = gsv.driver()
    path = str(tmp_path / "uid").encode()
    sent = _uid(5)
    t = threading.Timer(0.2, lambda: d.gs_uid_publish(path, sent))
    t.start()
    got = (C.c_ubyte * 128)()
    t0 = time.monotonic()
    assert d.gs_uid_await(path, 10.0, got) == 0
    t.join()
    assert bytes(got) == bytes(sent) and time.monotonic() - t0 >= 0.15


def test_uid_handoff_times_out(tmp_path):
    d = gsv.driver()
    got = (C.c_ubyte * 128)()
    t0 = time.monotonic()
    assert d.gs_uid_await(str(tmp_path / "never").encode(), 0.3, got) == 1
    msg = d.gs_last_error().decode()
    assert "timed out after" in msg and "RCCL id" in msg
    assert time.monotonic() - t0 < 5.0


def test_uid_handoff_rejects_a_short_file(tmp_path):
    (tmp_path / "uid").write_bytes(b"x" * 100)
    d = gsv.driver()
    got = (C.c_ubyte * 128)()
    assert d.gs_uid_await(str(tmp_path / "uid").encode(), 1.0, got) == 1
    assert "short RCCL id file" in d.gs_last_error().decode()


def test_uid_default_path_is_per_restart_attempt(monkeypatch):
    """without GS_UID_FILE the id file was /tmp/gpusolve-uid-<ppid>-<port>, the same for every
    torchrun --max-restarts attempt (the agent keeps its pid and port), so a file left behind by an attempt
    whose rank 0 was killed could be read by the next attempt's ranks. The default path now carries
    TORCHELASTIC_RUN_ID and TORCHELASTIC_RESTART_COUNT: attempt 1 never sees attempt 0's stale file."""
    import os
    drv = gsv.driver()

    def path():
        buf = C.create_string_buffer(512)
        n = drv.gs_uid_default_path(buf, 512)
        assert 0 < n < 512
        return buf.value.decode()

    monkeypatch.delenv("GS_UID_FILE", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", f"gs-test-{os.getpid()}")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    p0 = path()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    p1 = path()
    assert p0 != p1 and p0.startswith("/tmp/gpusolve-uid-")
    stale = (C.c_ubyte * 128)(*([7] * 128))
    fresh = (C.c_ubyte * 128)(*range(128))
    got = (C.c_ubyte * 128)()
    try:
        assert drv.gs_uid_publish(p0.encode(), stale) == 0  # attempt 0's rank 0, killed before its cleanup
        t0 = time.perf_counter()
        assert drv.gs_uid_await(p1.encode(), 0.2, got) != 0  # attempt 1 waits for ITS rank 0
        assert time.perf_counter() - t0 >= 0.2
        assert drv.gs_uid_publish(p1.encode(), fresh) == 0
        assert drv.gs_uid_await(p1.encode(), 5.0, got) == 0
        assert bytes(got) == bytes(range(128))
    finally:
        for p in (p0, p1):
            if os.path.exists(p):
                os.unlink(p)
