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
                                           ctypes.c_void_p(st.cuda_stream)), "fenv_stream_gate")
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
    held_ms = ((int(blk.status[3]) << 32) | int(blk.status[2])) / 1e6
    assert 55.0 <= held_ms < 5000.0               # the wave's own clock: held > the 60 ms slept
    assert float(x.sum()) == float(1 << 20)


def test_gate_times_out_without_release(flib, blk):
    t0 = time.perf_counter()
    st = _arm(flib, blk, 3, 30_000)               # 30 ms, never released
    st.synchronize()
    el = time.perf_counter() - t0
    assert blk.status[0] == 2 and blk.status[1] >= 1
    assert 0.025 < el < 5.0
    held_ms = ((int(blk.status[3]) << 32) | int(blk.status[2])) / 1e6
    assert 30.0 <= held_ms < 31.0                 # the timeout, by the wave's clock
    _arm(flib, blk, 4, 5_000_000)                 # re-armed gate is held again, then released
    blk.flag[0] = 4
    st.synchronize()
    assert blk.status[0] == 1


def test_gate_holds_work_ordered_after_it_on_other_streams(flib, blk):
    """bench.py's window: the side stream's reductions wait on events recorded on the gated
    stream, so they are held too, and run once the gate is released."""
    main = torch.cuda.current_stream(DEV)
    side = torch.cuda.Stream(DEV)
    y = torch.zeros(4096, device=DEV)
    mark, done = torch.cuda.Event(), torch.cuda.Event()
    torch.cuda.synchronize()
    _arm(flib, blk, 11, 5_000_000)
    y.fill_(2.0)                                  # on the gated stream
    mark.record(main)
    side.wait_event(mark)
    with torch.cuda.stream(side):
        y.mul_(3.0)                               # ordered after the gated fill
    done.record(side)
    time.sleep(0.03)
    assert not done.query() and blk.status[0] == 0
    blk.flag[0] = 11
    done.synchronize()
    assert blk.status[0] == 1
    assert torch.all(y == 6.0).item()
