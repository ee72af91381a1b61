"""GPU: the launch gate (include/fenv.h fenv_stream_gate) that bench.py's timed window is queued
behind -- it holds the stream's later work until the host stores the flag, releases it, records
how; and with no store it exits by itself at its timeout (every wave reaches an exit)."""
import ctypes
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture()
def blk(flib):
    b = flib.HostBlock(torch.device(DEV), [("flag", np.uint32, (16,)), ("status", np.uint32, (16,))])
    b.flag[:] = 0
    b.status[:] = 0
    return b


def _arm(flib, blk, value, timeout_us):
    st = torch.cuda.current_stream(DEV)
    flib.check(flib.lib().fenv_stream_gate(blk.dev("flag"), value, timeout_us, blk.dev("status"),
                                           None, ctypes.c_void_p(st.cuda_stream)), "fenv_stream_gate")
    return st


def test_gate_holds_then_releases(flib, blk):
    x = torch.zeros(1 << 20, device=DEV)
    torch.cuda.synchronize()
    st = _arm(flib, blk, 7, 5_000_000)
    x.add_(1.0)                                  # queued behind the gate
    ev = torch.cuda.Event()
    ev.record(st)
    time.sleep(0.05)
    assert not ev.query() and blk.status[0] == 0  # still held 50 ms later
    blk.flag[0] = 6                               # a different value does not release it
    time.sleep(0.01)
    assert not ev.query()
    blk.flag[0] = 7
    ev.synchronize()
    assert blk.status[0] == 1 and blk.status[1] >= 2
    assert float(x.sum()) == float(1 << 20)


def test_gate_times_out_without_release(flib, blk):
    t0 = time.perf_counter()
    st = _arm(flib, blk, 3, 30_000)               # 30 ms, never released
    st.synchronize()
    el = time.perf_counter() - t0
    assert blk.status[0] == 2 and blk.status[1] >= 1
    assert 0.025 < el < 5.0
    _arm(flib, blk, 4, 5_000_000)                 # re-armed gate is held again, then released
    blk.flag[0] = 4
    st.synchronize()
    assert blk.status[0] == 1


def test_bound_events_time_the_gated_work(flib, blk):
    """Events bound to the gate wave's exit and to the start of an empty mark kernel
    (fenv_stream_mark) time the work between them like hipEventRecord markers do: a sleep kernel
    of a fixed cycle count measures within 15 % (+ 20 us) of its marker-timed duration."""
    L = flib.lib()
    st = torch.cuda.current_stream(DEV)
    sp = ctypes.c_void_p(st.cuda_stream)
    cycles = 20_000_000
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    torch.cuda._sleep(cycles)
    b.record(st)
    torch.cuda.synchronize()
    ref_ms = a.elapsed_time(b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for e in (e0, e1):
        e.record(st)                              # created (torch makes a HIP event lazily)
    torch.cuda.synchronize()
    flib.check(L.fenv_stream_gate(blk.dev("flag"), 9, 5_000_000, blk.dev("status"),
                                  ctypes.c_void_p(e0.cuda_event), sp), "fenv_stream_gate")
    torch.cuda._sleep(cycles)
    flib.check(L.fenv_stream_mark(ctypes.c_void_p(e1.cuda_event), sp), "fenv_stream_mark")
    time.sleep(0.02)
    blk.flag[0] = 9
    torch.cuda.synchronize()
    assert blk.status[0] == 1
    ms = e0.elapsed_time(e1)
    # the 20 ms the gate was held are not in the span: it starts at the gate's exit
    assert abs(ms - ref_ms) < 0.15 * ref_ms + 0.02, (ms, ref_ms)
