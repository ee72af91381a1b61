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
        q.put((parts, out.tolist(), mx, float(params.sum()), counts, got))
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
    parts, out, mx, psum, counts, got = q.get(timeout=120)
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
