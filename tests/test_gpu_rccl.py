"""GPU: RCCL executed once on the one-GPU box (RCCL refuses two ranks on one GPU, so the
driver's 8-GPU run would otherwise be its first execution).  bench.py's N > 1 region --
the stats reductions' side-stream all-reduce, max_over_ranks, the per-rank all-gather and the
barriers -- runs in a world-1 process group over backend "nccl" (FENV_DIST_FORCE=1), and its
episode statistics equal, bit for bit, those of the same command with no process group."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the 8-way shard size of config 3; --prewarm-ms 0: a fixed pre-warm (2 regions), so both runs
# step the env through the same launches
ARGS = ["--gpus", "1", "--steps", "20", "--warmup", "5", "--formations", "131072",
        "--prewarm-ms", "0", "--no-policy", "--no-configs", "--no-cpu-baseline"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FENV_DIST_FORCE", "FENV_DIST_BACKEND"):
        env.pop(k, None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_region_over_rccl_world1():
    plain = _bench({})
    rccl = _bench({"FENV_DIST_FORCE": "1", "FENV_DIST_BACKEND": "nccl", "WORLD_SIZE": "1",
                   "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                   "MASTER_PORT": str(_port())})
    assert plain["dist"] == {"backend": "none", "world": 1}
    assert rccl["dist"] == {"backend": "nccl", "world": 1}
    for d in (plain, rccl):
        assert d["issue"] == "gated" and d["gate"]["released"] == 1
        assert d["value"] > 0 and d["host_issued"]["value"] > 0
    # the per-rank timings came through the all-gather (one rank), and agree with the line
    pr = rccl["per_rank"]
    assert set(pr) == {"host", "gated"}
    for w in pr.values():
        assert all(len(v) == 1 for v in w.values())
        # the window started at the agreed instant (1 ms after the agreement), not late
        assert 0.0 <= w["start_late_us"][0] < 1000.0
    assert abs(pr["gated"]["elapsed_ms"][0] - rccl["ms_per_step"] * rccl["steps"]) < 1e-6
    assert "per_rank" not in plain
    # the all-reduced stats equal the unreduced ones bit for bit (same seed, same launches)
    assert rccl["episode_stats"] == plain["episode_stats"]
    assert rccl["episode_stats"]["agent_dones_sampled_rollout"] >= 0


def test_bench_falls_back_to_host_window_when_gate_times_out():
    """A gate that never sees its release (test hook: the store is skipped; the wave times out
    after 20 ms) does not take the line down: it carries the host-issued window, labelled."""
    d = _bench({"FENV_BENCH_GATE_TEST": "no-release"})
    assert d["issue"] == "host" and "did not release" in d["gate_error"]
    assert d["value"] == d["host_issued"]["value"] and "gate" not in d


def test_ppo_collectives_over_rccl_world1():
    """The PPO and stats collectives (policy broadcast, the replicated update's sample all-gather,
    the sharded update's gradient all-reduce, the double-buffered stats all-reduce on a side
    stream, max_over_ranks, the per-rank gather) run once each on RCCL over device tensors in a
    world-1 "nccl" group, and are identities there, bit for bit."""
    env = dict(os.environ)
    env.update({"FENV_DIST_FORCE": "1", "FENV_DIST_BACKEND": "nccl", "WORLD_SIZE": "1",
                "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(_port())})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_child.py")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["world"] == 1 and out["active"]
    assert out["broadcast_equal"] and out["gather_equal"] and out["allreduce_equal"]
    assert out["stats_result"] == [2.0, 2.0]
    assert out["max_over_ranks"] == 3.25 and out["gather_floats"] == [[1.5, 2.5]]


def test_gated_window_absorbs_a_host_stall():
    """What the gate is for: a 400 us host stall injected right before the window's second launch
    is issued (test hook FENV_BENCH_STALL_US) lands inside the host-issued window -- at the 8-way
    shard size its first launch runs only ~55 us -- and outside the gated one, where the whole
    window is queued before t0."""
    d = _bench({"FENV_BENCH_STALL_US": "400"})
    assert d["issue"] == "gated"
    host_ms = d["host_issued"]["ms_per_step"] * d["steps"]
    gated_ms = d["ms_per_step"] * d["steps"]
    # host-issued: the GPU idles between the two launches (inside the event-timed span too)
    assert host_ms > 0.4 and d["host_issued"]["kernel_ms_timed"] > 0.35
    # gated: the ~0.13 ms of the window without a stall (the two launches back to back)
    assert gated_ms < 0.35 and host_ms - gated_ms > 0.25
    assert d["gate"]["prefix_issue_ms"] > 0.4                # the stall happened, before t0
