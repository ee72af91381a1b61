"""Child process of tests/test_gpu_rccl.py (not a test module): the PPO / stats collectives of the
N > 1 path on device tensors over a world-1 "nccl" process group (FENV_DIST_FORCE=1), so RCCL runs
each of them once.  Prints one JSON line of checks."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    import pkgload
    from importlib import import_module
    d = import_module(pkgload.load().__name__ + ".distributed")
    rank, world, local = d.init_from_env()
    dev = torch.device("cuda", local)
    g = torch.Generator(device=dev).manual_seed(5)
    out = {"backend": dist.get_backend(), "world": world, "active": d.active()}
    # the policy broadcast at PPO construction (9,669 floats at D = 8)
    p = torch.rand(9669, device=dev, generator=g)
    ref = p.clone()
    d.broadcast_(p)
    out["broadcast_equal"] = bool(torch.equal(p, ref))
    # replicated PPO's per-update all-gather of [n_steps, A_r, D + 5] samples (1,000 x 5 agents)
    smp = torch.rand((10, 5000, 13), device=dev, generator=g)
    got = d.gather_columns(smp, d.shard_counts(1000, world, 5))
    out["gather_equal"] = bool(torch.equal(got, smp))
    # sharded PPO's gradient all-reduce (SUM) of the flat gradient
    grad = torch.rand(9669, device=dev, generator=g)
    gref = grad.clone()
    dist.all_reduce(grad)
    out["allreduce_equal"] = bool(torch.equal(grad, gref))
    # the stats reducer on a side stream: reserve -> write -> submit, three rounds, then result
    red = d.StatsReducer(2, dev)
    bufs = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(2)]
    for k in range(3):
        red.reserve()
        bufs[k % 2].fill_(float(k))
        red.submit(bufs[k % 2])
    res = red.result().cpu().tolist()
    out["stats_result"] = res
    out["max_over_ranks"] = d.max_over_ranks(3.25, dev)
    out["gather_floats"] = d.gather_floats([1.5, 2.5], dev)
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
