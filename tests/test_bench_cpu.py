"""CPU checks of bench.py's bookkeeping (no GPU): the launch plan covers exactly the requested
steps (the driver compares the line's `steps`/`warmup` with its command), and the algorithmic
byte model matches DESIGN.md §4 (47.0 B per agent-step at N = 5, D = 8, T = 10)."""
import bench


def test_launch_plan_exact():
    for steps in (1, 5, 9, 10, 11, 20, 25, 5000, 5003):
        for T in (1, 3, 10):
            plan = bench.launch_plan(steps, T)
            assert sum(plan) == steps
            assert all(1 <= L <= T for L in plan)
            assert plan[:-1] == [T] * (len(plan) - 1)
    assert bench.launch_plan(0, 10) == []
    assert bench.launch_plan(20, 10) == [10, 10] and bench.launch_plan(5, 10) == [5]


def test_rollout_bytes_model():
    A, N, D, T = 5 * (1 << 20), 5, 8, 10
    per = bench.rollout_bytes_per_launch(A, N, D, T) / (A * T)
    assert abs(per - 47.0) < 1e-9
    # single step (T = 1): SURVEY §8(d)'s B_step 64.2 B at N=5, D=8 + the 4-B episode counter / N
    assert abs(bench.rollout_bytes_per_launch(A, N, D, 1) / A - (64.2 + 0.8)) < 1e-9
    # timed bytes of a plan = sum over its launches
    plan = bench.launch_plan(25, 10)
    tot = sum(bench.rollout_bytes_per_launch(A, N, D, L) for L in plan)
    assert tot > 25 * A * 45


def test_cpu_share_within_affinity():
    import os
    threads, how = bench.cpu_share()
    assert 1 <= threads <= len(os.sched_getaffinity(0)) and "affinity" in how


def test_window_summary_fields():
    """One window's JSON fields from its max-over-ranks wall and kernel times: value over the
    wall, kernel_value over the event-timed span, fixed overhead = the difference."""
    w = {"elapsed_max": 1.0e-3, "kern_ms_max": 0.9, "host_issue_ms": 0.05}
    s = bench.window_summary(w, total_agents=5_000_000, steps=20)
    assert abs(s["value"] - 1e11) < 1.0
    assert abs(s["kernel_value"] - 1e11 / 0.9) < 1.0
    assert abs(s["ms_per_step"] - 0.05) < 1e-12
    assert abs(s["fixed_overhead_ms"] - 0.1) < 1e-12
    assert s["kernel_ms_timed"] == 0.9 and s["host_issue_ms"] == 0.05


def test_gate_prefix_and_alignment_constants():
    """The gated window queues at most GATE_PREFIX launches before its release, and N > 1 windows
    start ALIGN_MARGIN_NS after the ranks agree."""
    assert bench.GATE_PREFIX >= 2          # the driver's --steps 20 window is gated whole
    assert 0 < bench.ALIGN_MARGIN_NS <= 5_000_000
    assert bench._Gate.TIMEOUT_US <= 60_000_000   # fenv_stream_gate's limit
