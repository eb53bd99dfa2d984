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
