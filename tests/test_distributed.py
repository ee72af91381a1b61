"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: formation sharding, the
sharded MT19937 reset stream and the stats all-reduce used by bench.py / training."""
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
    # PPO's collectives: rank 0's parameters replicated once, gradient bucket averaged
    params = torch.full((9669,), float(rank + 1))
    d.broadcast_(params)
    grad = torch.arange(9669, dtype=torch.float32) * (rank + 1)
    d.allreduce_mean_(grad)
    seeds = [None] * world
    dist.all_gather_object(seeds, d.sample_seed(12345, rank))
    if rank == 0:
        q.put((parts, out.tolist(), mx, float(params.sum()), grad[:4].tolist(), seeds))
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
    parts, out, mx, psum, g4, seeds = q.get(timeout=120)
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
    assert g4 == [0.0, 1.5, 3.0, 4.5]            # mean of k and 2k
    assert seeds[0] == 12345 and seeds[1] != seeds[0]  # rank 0 keeps the single-GPU stream
