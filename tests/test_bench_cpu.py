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
