"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: formation sharding, the
sharded MT19937 reset stream, the stats all-reduce used by bench.py / training, and PPO's
once-per-update sample all-gather + shared epoch permutations (uneven shards)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _world1_worker(port, root, q):
    """FENV_DIST_FORCE=1 at WORLD_SIZE 1: a real process group, so every collective of the N > 1
    path runs (the StatsReducer all-reduce, max_over_ranks, gather_floats, the barrier)."""
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", FENV_DIST_FORCE="1")
    import pkgload
    from importlib import import_module
    d = import_module(pkgload.load().__name__ + ".distributed")
    r, w, _ = d.init_from_env(backend="gloo")
    red = d.StatsReducer(2, "cpu")
    bufs = [torch.zeros(2, dtype=torch.float64) for _ in range(2)]
    for k in range(3):
        red.reserve()
        bufs[k % 2].copy_(torch.tensor([float(k), 2.0], dtype=torch.float64))
        red.submit(bufs[k % 2])
    res = red.result().tolist()
    dist.barrier()
    q.put((r, w, d.active(), red.dist, res, d.max_over_ranks(4.5), d.gather_floats([1.0, 2.0]),
           dist.get_backend()))
    dist.destroy_process_group()


def test_forced_world1_process_group_runs_collectives():
    """The N > 1 code path at world size 1 (how the one-GPU box executes RCCL once, tests/
    test_gpu_rccl.py): FENV_DIST_FORCE=1 makes init_from_env start a process group, and the
    stats reducer, max_over_ranks and gather_floats then go through real collectives."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_worker, args=(_free_port(), root, q))
    p.start()
    r, w, active, red_dist, res, mx, per, backend = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert (r, w, active, red_dist, backend) == (0, 1, True, True, "gloo")
    assert res == [2.0, 2.0] and mx == 4.5 and per == [[1.0, 2.0]]


def test_shard_range_partitions(pkg):
    from importlib import import_module
    d = import_module(pkg.__name__ + ".distributed")
    for total in (1, 7, 8, 1 << 20, 1000003):
        for world in (1, 2, 3, 4, 8):
            if world > total:
                continue
            spans = [d.shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (f0, c0), (f1, c1) in zip(spans, spans[1:]):
                assert f0 + c0 == f1 and abs(c0 - c1) <= 1
            assert spans[-1][0] + spans[-1][1] == total
    with pytest.raises(ValueError):
        d.shard_range(10, 2, 2)


def _global_samples(T, A, C):
    """Deterministic stand-in for an unsharded [T, A, C] update buffer (distinct values)."""
    return torch.arange(T * A * C, dtype=torch.float32).reshape(T, A, C) * 0.5 - 7.0


def _worker(rank, world, port, root, q):
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import pkgload
    pkg = pkgload.load()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".distributed")
    lib = import_module(pkg.__name__ + "._lib")
    r, w, _ = d.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    total, N, seed = 11, 5, 99
    first, count = d.shard_range(total, rank, world)
    # each rank's share of reset draw set 1 of the global stream
    px = np.zeros(count * N, np.float32)
    py = np.zeros(count * N, np.float32)
    gx = np.zeros(count, np.float32)
    gy = np.zeros(count, np.float32)
    lib.check(lib.lib().fenv_host_reset_draws(seed, 1, total, first, count, N,
                                              *(lib.ptr(v) for v in (px, py, gx, gy))))
    parts = [None] * world
    dist.all_gather_object(parts, (first, px.tolist(), gx.tolist()))
    # stats all-reduce through the double-buffered reducer
    red = d.StatsReducer(2, "cpu")
    bufs = [torch.zeros(2, dtype=torch.float64) for _ in range(2)]
    for k in range(5):
        red.reserve()
        bufs[k % 2].copy_(torch.tensor([float(rank + k), 1.0], dtype=torch.float64))
        red.submit(bufs[k % 2])
    out = red.result().clone()
    mx = d.max_over_ranks(float(rank) * 3.0)
    per = d.gather_floats([rank, rank * 2.5, -1.0])  # bench's per-rank timings
    # PPO's collectives: rank 0's parameters replicated once; per update ONE all-gather of the
    # [T, A_r, D+5] samples of uneven shards (11 formations x 5 agents: 30 + 25 rows)
    params = torch.full((9669,), float(rank + 1))
    d.broadcast_(params)
    counts = d.shard_counts(total, world, N)
    T, C = 3, 13
    glob = _global_samples(T, total * N, C)
    a0 = sum(counts[:rank])
    local = glob[:, a0:a0 + counts[rank]].clone()
    gathered = d.gather_columns(local, counts)
    # the update's permutations: one randperm per epoch from a generator seeded alike
    ppo = import_module(pkg.__name__ + ".ppo")
    perms = ppo.epoch_permutations(T * total * N, 4, torch.Generator().manual_seed(7), "cpu")
    got = [None] * world
    dist.all_gather_object(got, (gathered.numpy().tobytes(), perms.numpy().tobytes()))
    if rank == 0:
        q.put((parts, out.tolist(), mx, float(params.sum()), counts, got, per))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_draws_and_stats(flib):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts, out, mx, psum, counts, got, per = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the shards' draws concatenate to the unsharded draw set
    total, N, seed = 11, 5, 99
    px = np.zeros(total * N, np.float32)
    py = np.zeros(total * N, np.float32)
    gx = np.zeros(total, np.float32)
    gy = np.zeros(total, np.float32)
    flib.check(flib.lib().fenv_host_reset_draws(seed, 1, total, 0, total, N,
                                                *(flib.ptr(v) for v in (px, py, gx, gy))))
    parts = sorted(parts)
    assert np.array_equal(np.concatenate([np.array(p[1], np.float32) for p in parts]), px)
    assert np.array_equal(np.concatenate([np.array(p[2], np.float32) for p in parts]), gx)
    assert out == [float(0 + 4) + float(1 + 4), 2.0]
    assert mx == 3.0
    assert per == [[0.0, 0.0, -1.0], [1.0, 2.5, -1.0]]  # one list per rank, in rank order
    assert psum == 9669.0                        # rank 0's ones everywhere
    assert counts == [30, 25]                    # uneven shards (6 + 5 formations)
    # both ranks gathered the same buffer, equal to the unsharded (world-1) one, and drew the
    # same permutations as a world-1 run
    want = _global_samples(3, total * N, 13).numpy().tobytes()
    assert got[0][0] == want and got[1][0] == want
    from importlib import import_module
    import pkgload
    ppo = import_module(pkgload.load().__name__ + ".ppo")
    perms = ppo.epoch_permutations(3 * total * N, 4, torch.Generator().manual_seed(7), "cpu")
    assert got[0][1] == got[1][1] == perms.numpy().tobytes()


# ------------------------------------------------------------------ data-parallel PPO update
_DP = dict(D=8, n=(18, 13), epochs=3, batch=8, seed=5)


def _dp_samples(rank):
    """Rank r's local update samples (obs, actions, old_log_prob, advantages, returns)."""
    g = torch.Generator().manual_seed(1000 + rank)
    n, D = _DP["n"][rank], _DP["D"]
    obs = torch.rand((n, D), generator=g) * 2 - 1
    act = torch.randn((n, 2), generator=g) * 0.7
    lp = -torch.rand(n, generator=g) * 3 - 1
    adv = torch.randn(n, generator=g) * 2
    ret = torch.randn(n, generator=g)
    return obs, act, lp, adv, ret


def _dp_init_params():
    from importlib import import_module
    import pkgload
    pol = import_module(pkgload.load().__name__ + ".policy")
    n = sum(int(np.prod(s)) for _, s in pol.param_shapes(_DP["D"]))
    g = torch.Generator().manual_seed(3)
    flat = torch.randn(n, generator=g) * 0.2
    flat[-2:] = torch.tensor([-0.3, 0.1])  # log_std
    return flat


def _dp_cfg():
    from importlib import import_module
    import pkgload
    ppo = import_module(pkgload.load().__name__ + ".ppo")
    return ppo.PPOConfig(n_epochs=_DP["epochs"], batch_size=_DP["batch"], update_mode="sharded")


def _dp_worker(rank, world, port, root, q):
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import pkgload
    pkg = pkgload.load()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".distributed")
    dpu = import_module(pkg.__name__ + ".dp_update")
    d.init_from_env(backend="gloo")
    param = torch.nn.Parameter(_dp_init_params())
    opt = torch.optim.Adam([param], lr=1e-3, eps=1e-5)
    upd = dpu.ShardedUpdate(_dp_cfg(), _DP["D"], list(_DP["n"]), _DP["seed"], "cpu")
    stats = upd.run(param, opt, _dp_samples(rank))
    st = opt.state[param]
    got = [None] * world
    dist.all_gather_object(got, (param.detach().numpy().tobytes(),
                                 st["exp_avg_sq"].numpy().tobytes(), stats))
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_update_equals_concatenated_minibatches():
    """The data-parallel update (dp_update.py: each rank takes batch_size / world rows of every
    global minibatch, one gradient all-reduce per minibatch) on 2 ranks with uneven shards (18 +
    13 samples: the last minibatch has rows on rank 0 only) equals the single-process SB3 update
    whose minibatches are the concatenations of the ranks' rows -- to summation order."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == got[1][0] and got[0][1] == got[1][1]  # replicated state, bit for bit
    # single-process reference: SB3 PPO.train over the concatenated minibatches
    import math
    from importlib import import_module
    import pkgload
    pkg = pkgload.load()
    ppo = import_module(pkg.__name__ + ".ppo")
    dpu = import_module(pkg.__name__ + ".dp_update")
    cfg = _dp_cfg()
    b, M, rows, _ = dpu.minibatch_plan(list(_DP["n"]), cfg.batch_size, 2)
    assert rows[1][-1] == 0 and M == 5
    perms = []
    for r in range(2):
        gen = torch.Generator().manual_seed((_DP["seed"] * 1_000_003 + r) & 0x7FFFFFFFFFFFFFFF)
        perms.append([torch.randperm(_DP["n"][r], generator=gen) for _ in range(cfg.n_epochs)])
    local = [_dp_samples(r) for r in range(2)]
    param = torch.nn.Parameter(_dp_init_params())
    opt = torch.optim.Adam([param], lr=1e-3, eps=1e-5)
    sums = torch.zeros(4, dtype=torch.float64)
    for e in range(cfg.n_epochs):
        for j in range(M):
            parts = [tuple(t[perms[r][e][j * b:j * b + rows[r][j]]] for t in local[r])
                     for r in range(2)]
            obs, act, old_lp, adv, ret = (torch.cat([p[k] for p in parts]) for k in range(5))
            values, log_prob, entropy = ppo.evaluate_actions(_DP["D"], param, obs, act)
            if adv.numel() > 1:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            ratio = torch.exp(log_prob - old_lp)
            l1 = adv * ratio
            l2 = adv * torch.clamp(ratio, 1 - cfg.clip_range, 1 + cfg.clip_range)
            pl = -torch.min(l1, l2).mean()
            vl = torch.nn.functional.mse_loss(ret, values)
            el = -torch.mean(entropy)
            loss = pl + cfg.ent_coef * el + cfg.vf_coef * vl
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_([param], cfg.max_grad_norm)
            opt.step()
            cf = (torch.abs(ratio - 1) > cfg.clip_range).float().mean()
            sums += torch.stack([pl.detach(), vl.detach(), el.detach(), cf]).double()
    want = param.detach()
    have = torch.from_numpy(np.frombuffer(got[0][0], np.float32).copy())
    assert (have - want).abs().max().item() < 2e-6, (have - want).abs().max().item()
    assert not torch.equal(want, _dp_init_params())  # the update moved the parameters
    ref = (sums / (cfg.n_epochs * M)).tolist()
    stats = got[0][2]
    for k, name in enumerate(("policy_gradient_loss", "value_loss", "entropy_loss",
                              "clip_fraction")):
        assert math.isclose(stats[name], ref[k], rel_tol=1e-5, abs_tol=1e-6), (name, stats, ref)


def test_sharded_minibatch_plan(pkg):
    """minibatch_plan: every rank runs the same number of minibatches per epoch; the rows of
    minibatch j over the ranks sum to the global minibatch; batch_size must split evenly."""
    from importlib import import_module
    dpu = import_module(pkg.__name__ + ".dp_update")
    b, M, rows, bg = dpu.minibatch_plan([300, 250], 64, 2)
    assert (b, M) == (32, 10)
    assert all(sum(r) == n for r, n in zip(rows, [300, 250]))
    assert bg == [rows[0][j] + rows[1][j] for j in range(M)] and bg[0] == 64
    assert rows[1][-2:] == [26, 0] or rows[1][-1] == 0
    b, M, rows, bg = dpu.minibatch_plan([50000], 64, 1)
    assert (b, M, bg[-1]) == (64, 782, 16)  # the reference's 1000 x 5 x 10 samples
    with pytest.raises(ValueError):
        dpu.minibatch_plan([10, 10], 63, 2)


def test_sharded_mode_at_world1_draws_sb3_minibatches(pkg):
    """with one rank, update_mode='sharded' shuffles with the generator the replicated
    path draws SB3's per-epoch randperm from, so both modes run the same minibatches, over two
    consecutive updates (the generator advances alike)."""
    from importlib import import_module
    dpu = import_module(pkg.__name__ + ".dp_update")
    ppo = import_module(pkg.__name__ + ".ppo")
    cfg = ppo.PPOConfig(n_epochs=3)
    g_rep = torch.Generator().manual_seed(7)
    g_sh = torch.Generator().manual_seed(7)
    upd = dpu.ShardedUpdate(cfg, 8, [1000], 7, "cpu", gen=g_sh)
    for _ in range(2):
        want = ppo.epoch_permutations(1000, 3, g_rep, "cpu")
        assert torch.equal(upd.permutations(), want)
    # the minibatches: contiguous slices of each epoch's permutation, 64 rows, the last 40
    assert (upd.b, upd.M, upd.bg[-1]) == (64, 16, 40)
