"""Formation sharding across ranks (one process per GPU) and the only collectives the path
needs: an all-reduce of episode statistics, one broadcast of the initial policy, and (PPO) one
all-gather of every rank's rollout samples per update.  The reference is single-process (SURVEY
§2: no torch.distributed anywhere); this is new, per SURVEY §8(e): formations are independent,
so env stepping needs no communication.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous formation shard [first, first+count) of rank `rank` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(int(total), int(world))
    first = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    return first, count


def init_from_env(backend: str | None = None, force: bool | None = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env vars when WORLD_SIZE > 1, or at any world
    size when ``force`` (default: env ``FENV_DIST_FORCE=1``) -- a world-1 process group runs every
    collective of the N > 1 path for real (the one-GPU box's way to execute RCCL: it refuses two
    ranks on one GPU).

    Returns (rank, world_size, local_rank).  backend defaults to "nccl" (RCCL on ROCm) when a
    GPU is visible, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob: run several ranks on fewer GPUs over gloo (never used by the driver)
    backend = backend or os.environ.get("FENV_DIST_BACKEND") or None
    if torch.cuda.is_available() and torch.cuda.device_count() > 0:
        local = local % torch.cuda.device_count()
    if force is None:
        force = os.environ.get("FENV_DIST_FORCE", "") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


class StatsReducer:
    """Stream-overlapped all-reduce of a small stats vector, two submissions in flight.

    ``submit(v)`` starts an async all-reduce of ``v`` IN PLACE on a side stream, after the
    current stream's work that produced v (or after the event ``after``); the caller alternates
    two buffers.  Before rewriting the buffer of a slot, call ``reserve()``: on the GPU it makes the
    writing stream wait (device-side) for the all-reduce that last used the slot, on the CPU the
    host waits for it.  ``result()`` makes the current stream (or ``stream``) wait for the last
    submission and returns its buffer.  Without an initialised process group there is nothing to
    reduce and ``v`` is returned as is; with one (any world size, world 1 included) every
    submission is a real collective.

    Every cross-stream dependency goes through events created and recorded once in the
    constructor: torch's ``Stream.wait_stream`` creates and records a fresh event per call, and
    a torch event is created lazily at its first record -- host work that would otherwise sit
    inside a caller's timed region (bench.py).  ``stream`` lets the caller hand in the side
    stream it already reduces on, so the collective adds no stream hop.

    Backends: on NCCL (RCCL) ``all_reduce(async_op=True).wait()`` only orders the side stream
    after the collective, so ``submit`` returns at once.  On gloo with CUDA tensors the same
    ``wait()`` blocks the host until the collective is done, so ``submit`` is synchronous there:
    a gloo rehearsal (tools/scale_rehearsal.sh) does not measure the overlapped stats path."""

    def __init__(self, n: int, device, stream=None):
        self.device = torch.device(device)
        self.work = [None, None]
        self.bufs = [None, None]
        self.k = 0
        self.cuda = self.device.type == "cuda"
        self.dist = active()
        self.used = [False, False]
        self.side = None
        if self.cuda:
            self.side = stream if stream is not None else torch.cuda.Stream(self.device)
            self.dep = torch.cuda.Event()
            self.done = [torch.cuda.Event(), torch.cuda.Event()]
            for e in [self.dep] + self.done:
                e.record(self.side)

    def reserve(self, stream=None) -> None:
        """Order a rewrite of the next slot's buffer after the all-reduce that last used the slot
        (call before overwriting the buffer you are about to submit): on the GPU the current
        stream (or ``stream``) waits for that submission's event, on the CPU the host waits."""
        s = self.k % 2
        if self.cuda:
            if self.used[s]:
                (stream or torch.cuda.current_stream(self.device)).wait_event(self.done[s])
            return
        if self.work[s] is not None:
            self.work[s].wait()
            self.work[s] = None

    def submit(self, v: torch.Tensor, after=None, stream=None) -> None:
        """All-reduce ``v`` in place: on ``stream`` if given (v was produced on it, or the caller
        ordered it there), after ``after`` if given, else on the side stream after the current
        stream's work so far."""
        s = self.k % 2
        self.bufs[s] = v
        if self.cuda:
            st = stream if stream is not None else self.side
            if after is not None:
                st.wait_event(after)
            elif stream is None:
                self.dep.record(torch.cuda.current_stream(self.device))
                st.wait_event(self.dep)
            with torch.cuda.stream(st):
                if self.dist:
                    # stream-ordered: wait() only makes the side stream wait for the collective
                    dist.all_reduce(v, async_op=True).wait()
                self.done[s].record(st)
            self.used[s] = True
        else:
            self.reserve()
            if self.dist:
                self.work[s] = dist.all_reduce(v, async_op=True)
        self.k += 1

    def ready(self):
        """The event of the last submission (cuda), None before the first or on the CPU."""
        return self.done[(self.k - 1) % 2] if self.cuda and self.k else None

    def result(self, stream=None) -> torch.Tensor:
        s = (self.k - 1) % 2
        if self.work[s] is not None:
            self.work[s].wait()
            self.work[s] = None
        if self.cuda:
            (stream or torch.cuda.current_stream(self.device)).wait_event(self.done[s])
        return self.bufs[s]


def active() -> bool:
    """True when a process group is initialised: the collectives run (any world size)."""
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(x: float, device=None) -> float:
    """Max of ``x`` over the ranks (one all-reduce; ``x`` itself without a process group)."""
    if not active():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(xs, device=None) -> list[list[float]]:
    """All-gather of a short list of floats from every rank -> one list per rank, in rank order
    (one collective; [xs] without a process group)."""
    xs = [float(x) for x in xs]
    if not active():
        return [xs]
    t = torch.tensor(xs, dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def world_rank() -> tuple[int, int]:
    """(world_size, rank) of the initialised process group, (1, 0) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Replicate ``t`` from rank ``src`` in place (the policy parameters, once at start); a real
    collective whenever a process group is up (world 1 included)."""
    if active():
        dist.broadcast(t, src)
    return t


def shard_counts(total: int, world: int, scale: int = 1) -> list[int]:
    """Rows owned by each rank: shard_range sizes x ``scale`` (agents per formation)."""
    return [shard_range(total, r, world)[1] * int(scale) for r in range(world)]


def gather_columns(local: torch.Tensor, counts: list[int], out: torch.Tensor | None = None):
    """All-gather of a [T, A_r, C] tensor whose middle dimension is sharded contiguously over the
    ranks (sizes ``counts``, which may differ by rank) -> [T, sum(counts), C], concatenated in rank
    order along dim 1: exactly the unsharded tensor.  One collective (shards padded to the largest
    count) whenever a process group is up (world 1 included); without one it is a copy."""
    world, rank = world_rank()
    T, Ar, C = local.shape
    if Ar != counts[rank]:
        raise ValueError(f"rank {rank}: local shard has {Ar} rows, counts say {counts[rank]}")
    total = sum(counts)
    if out is None:
        out = torch.empty((T, total, C), dtype=local.dtype, device=local.device)
    if not active():
        out.copy_(local)
        return out
    amax = max(counts)
    pad = local
    if Ar != amax:
        pad = torch.zeros((T, amax, C), dtype=local.dtype, device=local.device)
        pad[:, :Ar].copy_(local)
    parts = [torch.empty((T, amax, C), dtype=local.dtype, device=local.device)
             for _ in range(world)]
    dist.all_gather(parts, pad.contiguous())
    o = 0
    for r, n in enumerate(counts):
        out[:, o:o + n].copy_(parts[r][:, :n])
        o += n
    return out
