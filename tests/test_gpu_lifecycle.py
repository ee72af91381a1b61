"""Env lifecycle on the GPU: deterministic release, teardown from
the garbage collector and inside a HIP graph capture, and O(N) formation views.

Round 2 saw one SIGABRT during garbage collection.  Envs then formed a reference
cycle with their formation views, so every dropped env -- its device state, its pinned host
mirrors, its torch buffers -- was torn down by the cyclic collector at arbitrary points.  These
tests churn a few hundred envs over every kernel path with explicit collections in between."""
import gc
import os
import weakref

import numpy as np
import pytest
import torch

from oracle import COracleEnv, synth_actions

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def make_env(venv, F, N, goal=True, seed=0, **kw):
    cfg = {"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": goal}
    return venv.FormationEnv(cfg, device=DEV, seed=seed, **kw)


def test_env_has_no_reference_cycle(venv):
    """A dropped env (views accessed, numpy face used) is freed by reference counting alone."""
    env = make_env(venv, 7, 5)
    env.reset()
    env.step(np.zeros((35, 2), np.float32))
    v = env.formationsim_list[3]
    _ = v.agents, v.goal, v.steps_since_reset
    ref = weakref.ref(env)
    gc.disable()
    try:
        del env
        assert ref() is None, "FormationEnv survived its last reference: a reference cycle"
    finally:
        gc.enable()
    with pytest.raises(ReferenceError):
        _ = v.agents


def test_release_is_deterministic_and_idempotent(venv, flib):
    env = make_env(venv, 16, 5)
    env.reset()
    base = torch.cuda.memory_allocated()
    with make_env(venv, 4096, 5) as big:
        big.reset()
        big.rollout(torch.zeros((3, big.num_envs, 2), device=DEV))
        assert torch.cuda.memory_allocated() > base
    assert big.released
    assert torch.cuda.memory_allocated() <= base  # the env's torch buffers went with it
    big.release()  # idempotent
    with pytest.raises(Exception):
        big.step_tensor(torch.zeros((big.num_envs, 2), device=DEV))
    with pytest.raises(NotImplementedError):  # the reference's close() contract is kept
        env.close()
    assert flib.lib().fenv_destroy(None) == 0
    env.release()


def test_churn_envs_across_paths_with_gc(venv):
    """Create and drop ~300 envs over the wavefront (N <= 64, incl. the staged and role-split
    kernels), workgroup (64 < N <= 1024) and large-formation (N > 1024) paths, both reset modes,
    the numpy face (device-mapped host arrays) and the device faces, some released explicitly, some
    dropped, some left to the collector, with gc.collect() interleaved; every 25th env is checked
    against the C oracle bit for bit."""
    shapes = [(5, 1), (1, 5), (4096, 5), (60, 64), (3, 100), (2, 1024), (2, 1025), (1, 1300),
              (2500, 5), (7, 33)]
    rng = np.random.default_rng(0)
    keep = []
    checked = 0
    for i in range(300):
        F, N = shapes[(i + i // 25) % len(shapes)]
        mode = "philox" if i % 3 == 1 else "mt19937"
        env = make_env(venv, F, N, goal=bool(i % 2), seed=i, reset_mode=mode, max_steps=3)
        A = F * N
        if i % 25 == 0 and mode == "mt19937":
            ref = COracleEnv(F, N, bool(i % 2), i, max_steps=3)
            o = env.reset()
            assert np.array_equal(o.view(np.uint32), ref.reset().view(np.uint32))
            for k in range(6):
                a = synth_actions(i, k, A, 1.2)
                o, r, d, _ = env.step(a)
                ro, rr, rd, _ = ref.step(a)
                assert np.array_equal(o.view(np.uint32), ro.view(np.uint32)), (F, N, k)
                assert np.array_equal(r.view(np.uint32), rr.view(np.uint32)), (F, N, k)
                assert np.array_equal(d, rd), (F, N, k)
            checked += 1
        elif i % 4 == 0:
            env.reset()
            env.step(rng.uniform(-1, 1, (A, 2)).astype(np.float32))
            _ = env.formationsim_list[F - 1].agents
        else:
            env.reset_tensor()
            env.rollout(torch.rand((4, A, 2), device=DEV) * 2 - 1)
            env.metrics()
        if i % 5 == 0:
            env.release()
        elif i % 5 == 1:
            keep.append(env)  # left for the collector below
        del env
        if i % 10 == 9:
            keep.clear()
            gc.collect()
    gc.collect()
    torch.cuda.synchronize()
    assert checked >= 8


def test_env_dropped_inside_graph_capture(venv, flib):
    """A handle dropped while a HIP graph is being captured is parked, not freed inside the
    capture (which would invalidate it); the capture completes and replays, and the parked
    handle is destroyed by the next create."""
    keep = make_env(venv, 64, 5, reset_mode="philox")
    keep.reset_tensor()
    doomed = make_env(venv, 32, 5, reset_mode="philox")
    doomed.reset_tensor()
    acts = torch.rand((2, keep.num_envs, 2), device=DEV) * 2 - 1
    obs = torch.empty((2, keep.num_envs, 8), device=DEV)
    rew = torch.empty((2, keep.num_envs), device=DEV)
    done = torch.empty((2, keep.num_envs), dtype=torch.bool, device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        keep.rollout(acts, obs, rew, done)
        del doomed  # its finalizer runs inside the capture
    assert len(flib._deferred) == 1
    g.replay()
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all()
    make_env(venv, 2, 5).release()  # drains the parked handle
    assert len(flib._deferred) == 0


def test_release_inside_graph_capture(venv, flib):
    """an explicit release() (or a `with` block ending) during a capture must not
    synchronize the capturing stream (that would invalidate the capture): the handle is parked,
    the capture completes and replays, and the next create destroys it."""
    keep = make_env(venv, 64, 5, reset_mode="philox")
    keep.reset_tensor()
    doomed = make_env(venv, 32, 5, reset_mode="philox")
    doomed.reset_tensor()
    acts = torch.rand((2, keep.num_envs, 2), device=DEV) * 2 - 1
    obs = torch.empty((2, keep.num_envs, 8), device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        keep.rollout(acts, obs)
        doomed.release()
    assert doomed.released and len(flib._deferred) == 1
    g.replay()
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all()
    make_env(venv, 2, 5).release()
    assert len(flib._deferred) == 0


def test_view_touches_only_its_formation(venv):
    """formationsim_list[i] on a 1,048,576 x 5 env reads formation i's slice only: the device
    memory it allocates is O(N) (not the O(A) of get_state), and its values equal the full-state
    rows and metrics."""
    F, N = 1 << 20, 5
    env = make_env(venv, F, N, reset_mode="philox", seed=3)
    env.reset_tensor()
    env.rollout(torch.rand((3, F * N, 2), device=DEV) * 2.4 - 1.2)
    torch.cuda.synchronize()
    i = 777_777
    px, py, gx, gy, t = env.get_state()
    full = env.metrics()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    v = env.formationsim_list[i]
    ag, goal, sr = v.agents, v.goal, v.steps_since_reset
    met, comp = v.compute_metrics(), v.reward_components()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert peak < 64 * 1024, f"a view access allocated {peak} B of device memory"
    sl = slice(i * N, (i + 1) * N)
    assert torch.equal(ag, torch.stack([px[sl], py[sl]], 1).cpu())
    assert torch.equal(goal, torch.stack([gx[i], gy[i]]).cpu())
    assert sr == int(t[i])
    row = full[i].tolist()
    assert [met["avg_dist_to_goal"], met["ave_dist_to_neighbor"],
            met["std_dist_to_neighbor"]] == row[:3]
    assert list(comp.values()) == row[4:8]
    # a range in the middle, with rewards, equals the same rows of the full call
    rew = torch.rand(F * N, device=DEV)
    a, b = 1000, 4096
    assert torch.equal(env.metrics_range(a, b, rew[a * N:(a + b) * N]), env.metrics(rew)[a:a + b])
    with pytest.raises(IndexError):
        env.metrics_range(F - 1, 2)


def test_mt_reset_staging_across_streams_and_churn(venv):
    """The MT19937 reset sets are staged into two slots by a DMA on the handle's own stream,
    ordered by events: many reset events inside one rollout call (the slot flips
    at each, and each next launch waits for the set staged at the last), launches
    alternating between two streams (ordered only by stream waits), and staging buffers taken
    back from the process pool by envs of other sizes -- every reward, obs and done bit-exact
    against the C oracle."""
    for F, N in ((40, 5), (3, 100), (700, 5)):  # pooled buffers of other sizes, then reused
        e = make_env(venv, F, N, seed=F, max_steps=2)
        e.rollout(torch.rand((7, F * N, 2), device=DEV) * 2 - 1)
        e.release()
    F, N = 500, 5
    env = make_env(venv, F, N, seed=21, max_steps=2)
    ref = COracleEnv(F, N, True, 21, max_steps=2)
    assert np.array_equal(env.reset().view(np.uint32), ref.reset().view(np.uint32))
    streams = [torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)]
    prev = torch.cuda.current_stream(DEV)
    k = 0
    for call, T in enumerate((30, 5, 1, 9, 4, 13)):
        st = streams[call % 2]
        st.wait_stream(prev)
        acts = np.stack([synth_actions(6, k + j, F * N, 1.1) for j in range(T)])
        with torch.cuda.stream(st):
            a = torch.from_numpy(acts).to(DEV, non_blocking=False)
            obs, rew, done = env.rollout(a)
        prev = st
        st.synchronize()
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        for j in range(T):
            ro, rr, rd, _ = ref.step(acts[j])
            assert np.array_equal(rew[j].view(np.uint32), rr.view(np.uint32)), (call, k + j)
            assert np.array_equal(obs[j].view(np.uint32), ro.view(np.uint32)), (call, k + j)
            assert np.array_equal(done[j], rd), (call, k + j)
        k += T
    assert k > 40  # > 10 reset events at max_steps 2
    env.release()


def _mt_run(venv, F, N, seed, T_calls, hook=None, flib=None, streams=False):
    """MT19937 env vs the C oracle over rollout calls of the given lengths (max_steps 2: a reset
    event every 4 steps); returns the first mismatch or None.  `hook` = (mode, n) arms
    fenv_test_stage_hook right after the ctor."""
    env = make_env(venv, F, N, seed=seed, max_steps=2)
    ref = COracleEnv(F, N, True, seed, max_steps=2)
    if hook is not None:
        flib.lib().fenv_test_stage_hook(*hook)
    try:
        o = env.reset_tensor().cpu().numpy()
        bad = None if np.array_equal(o.view(np.uint32), ref.reset().view(np.uint32)) else "reset"
        ss = [torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)] if streams else None
        prev = torch.cuda.current_stream(DEV)
        k = 0
        for call, T in enumerate(T_calls):
            acts = np.stack([synth_actions(8, k + j, F * N, 1.1) for j in range(T)])
            a = torch.from_numpy(acts).to(DEV)
            if ss is not None:
                st = ss[call % 2]
                st.wait_stream(prev)
                with torch.cuda.stream(st):
                    obs, rew, done = env.rollout(a)
                prev = st
                st.synchronize()
            else:
                obs, rew, done = env.rollout(a)
            obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
            for j in range(T):
                ro, rr, rd, _ = ref.step(acts[j])
                if bad is None and not (np.array_equal(rew[j].view(np.uint32), rr.view(np.uint32))
                                        and np.array_equal(obs[j].view(np.uint32),
                                                           ro.view(np.uint32))
                                        and np.array_equal(done[j], rd)):
                    bad = f"call {call} step {k + j}"
            k += T
        torch.cuda.synchronize()
        return env, bad
    finally:
        if hook is not None:
            flib.lib().fenv_test_stage_hook(0, 0)


def test_mt_staging_ordering_with_delayed_copies(venv, flib):
    """every staging copy of the run is delayed (fenv_test_stage_hook mode 1:
    each staging DMA starts behind a kernel sleeping ~0.35 ms), so a launch that was not
    ordered behind its refill -- same stream, or another stream through the events -- would read
    the slot's previous set.  Results stay bit-exact against the C oracle and the tag check stays
    silent: the consumers wait for the copies."""
    for F, N, streams in ((500, 5, False), (500, 5, True), (24581, 5, False), (3, 1500, False)):
        env, bad = _mt_run(venv, F, N, 21, (8, 5, 1, 9, 13), hook=(1, 1000), flib=flib,
                           streams=streams)
        assert bad is None, (F, N, streams, bad)
        env.check()  # no staging error recorded
        env.release()


def test_mt_staging_check_fires_on_a_stale_set(venv, flib):
    """The tag check is live: with the copies of two refills skipped (hook mode 2) a reset event
    applies the slot's previous set -- exactly the failure of VERDICT r3 weak #1 -- and instead of
    silently wrong rewards the env reports FENV_ESTATE naming the stale set."""
    for F, N in ((500, 5), (24581, 5), (9, 100), (3, 1500)):
        # the ctor's two refills (sets 1, 2) are copied; the hook then skips the copy of set 3
        # (staged by reset()), so the first in-launch reset event reads slot 0's set 1
        env = make_env(venv, F, N, seed=4, max_steps=2)
        flib.lib().fenv_test_stage_hook(2, 1)
        try:
            env.reset_tensor()
            env.rollout(torch.zeros((4, F * N, 2), device=DEV))
            torch.cuda.synchronize()
            with pytest.raises(flib.FenvError, match="previous set"):
                env.check()
            with pytest.raises(flib.FenvError, match="tag check"):
                env.rollout(torch.zeros((1, F * N, 2), device=DEV))
        finally:
            flib.lib().fenv_test_stage_hook(0, 0)
        env.release()


def test_numpy_face_zero_copy_arrays(venv, flib):
    """The numpy faces' arrays live in device-mapped host memory the kernels write in place
    (fenv_host_alloc): every call returns the same arrays (aliasing, like the reference's
    obs_buf.numpy()); the done array holds 0 / 1 bytes; a CUDA action tensor drives the same
    step; arrays a caller kept stay valid after the env is released, and their block goes back
    to the pool only when the last one is gone.  Host blocks are freed once, and only by their
    own device."""
    import ctypes
    L = flib.lib()
    F, N = 300, 5
    A = F * N
    env = make_env(venv, F, N, seed=3, reset_mode="philox", max_steps=4)
    twin = make_env(venv, F, N, seed=3, reset_mode="philox", max_steps=4)
    o0 = env.reset()
    twin.reset_tensor()
    assert np.array_equal(o0.view(np.uint32), twin.obs_dev.cpu().numpy().view(np.uint32))
    for k in range(12):
        a = synth_actions(3, k, A, 1.3)
        if k % 3 == 2:  # the CUDA-tensor form of the same face
            o, r, d, _ = env.step(torch.from_numpy(a).to(DEV))
        else:
            o, r, d, _ = env.step(a)
        to, tr, td = twin.step_tensor(torch.from_numpy(a).to(DEV))
        assert o is o0 and np.shares_memory(o, o0)
        assert np.array_equal(o.view(np.uint32), to.cpu().numpy().view(np.uint32)), k
        assert np.array_equal(r.view(np.uint32), tr.cpu().numpy().view(np.uint32)), k
        assert np.array_equal(d, td.cpu().numpy()), k
        assert set(np.unique(d.view(np.uint8)).tolist()) <= {0, 1}
    assert d.any()  # max_steps 4: resets happened inside the window
    kept = o.copy()
    env.release()
    twin.release()
    del env
    gc.collect()
    assert np.array_equal(o.view(np.uint32), kept.view(np.uint32))  # block still held by `o`
    before = L.fenv_pinned_pool_bytes(0)
    del o, o0, r, d
    gc.collect()
    # back in the pool (a cached buffer of up to 4x the request may have served it), unless the
    # pool was already too full to take it
    blk = 256 + sum((n + 255) // 256 * 256 for n in (A * 8, A * 32, A * 4, A))
    assert L.fenv_pinned_pool_bytes(0) > before or before > (512 << 20) - 4 * blk
    h, dv = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.fenv_host_alloc(0, 4096, ctypes.byref(h), ctypes.byref(dv)) == 0 and h.value and dv.value
    assert L.fenv_host_free(1 if torch.cuda.device_count() > 1 else 99, h) != 0  # other device
    assert L.fenv_host_free(0, h) == 0
    assert L.fenv_host_free(0, h) != 0  # freed once


def test_pinned_pool_bounded_under_growing_sizes(venv, flib):
    """the pinned staging pool is per device and bounded (512 MiB per device): envs of
    growing size churned one after another leave at most that much cached."""
    L = flib.lib()
    for F in (1000, 10_000, 100_000, 400_000, 1_000_000, 2_000_000):
        e = make_env(venv, F, 5, seed=1)
        e.release()
        assert L.fenv_pinned_pool_bytes(0) <= 512 << 20
    small = make_env(venv, 10, 5, seed=2)
    small.reset()
    small.release()
    assert L.fenv_pinned_pool_bytes(0) <= 512 << 20


def test_mt_draw_ahead_across_events_and_release(venv, flib):
    """The next MT19937 set is drawn ahead on a host thread (fenv_api.cpp gen_pending): at
    200,000 x 5 (2.4M draws per set) and a reset event every 4 steps, every staged set equals the
    oracle's, in order, across calls of several lengths and two streams; releasing the env with
    a draw in flight joins it (the host slots it writes are freed after), and the next env --
    which may take the same pinned buffer -- is bit-exact again."""
    env, bad = _mt_run(venv, 200_000, 5, 31, (3, 5, 9, 2, 7))
    assert bad is None, bad
    env.release()
    env, bad = _mt_run(venv, 200_000, 5, 32, (6, 1, 4), streams=True)
    assert bad is None, bad
    env.release()


def test_exit_with_a_draw_in_flight(tmp_path):
    """A process that exits right after creating a large MT19937 env (its next reset set being
    drawn on the host thread) and never releases it: the library joins the thread at unload,
    before the HIP runtime frees the pinned slot it writes, so the process exits cleanly."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import torch, pkgload\n"
            "pkg = pkgload.load()\n"
            "from importlib import import_module\n"
            "ve = import_module(pkg.__name__ + '.vectorized_env')\n"
            "env = ve.FormationEnv({'num_formation': 400000, 'num_agents_per_formation': 5,\n"
            "                       'goal_in_obs': True}, device='cuda:0', seed=3)\n"
            "env.reset_tensor()\n"
            "torch.cuda.synchronize()\n"
            "import os; os._exit(0) if len(sys.argv) > 1 else None\n") % root
    for args in ([], ["hard"]):
        r = subprocess.run([sys.executable, "-c", code] + args, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, (args, r.returncode, r.stderr[-2000:])
