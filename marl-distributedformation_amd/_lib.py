"""ctypes binding of libfenv.so (C ABI declared in include/fenv.h).

The library is the only compute path: there is no CPU fallback.  If ``libfenv.so`` is missing,
or no HIP device is visible, every entry point raises.  torch is imported first so that the
library binds to the HIP runtime torch has already loaded (one runtime per process).
"""
from __future__ import annotations

import ctypes
import os
import re
import weakref

import numpy as np

import torch  # noqa: F401  (must precede loading libfenv.so: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfenv.so")
# developer override for A/B builds of the same sources (never needed in normal use)
LIB_PATH = os.environ.get("FENV_LIB_OVERRIDE") or LIB_PATH
HEADER = os.path.join(os.path.dirname(HERE), "include", "fenv.h")

FENV_RESET_MT19937 = 0
FENV_RESET_PHILOX = 1
RESET_MODES = {"mt19937": FENV_RESET_MT19937, "philox": FENV_RESET_PHILOX}

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64

# name -> (restype, argtypes)
SIGNATURES = {
    "fenv_create": (_I32, [ctypes.POINTER(_P), _I32, _I64, _I32, _I32, ctypes.c_double, _I32,
                           _U32, _I32, _I64, _I64]),
    "fenv_destroy": (_I32, [_P]),
    "fenv_info": (_I32, [_P, _P]),
    "fenv_reset": (_I32, [_P, _P, _P]),
    "fenv_observe": (_I32, [_P, _P, _P]),
    "fenv_step": (_I32, [_P, _P, _P, _P, _P, _P]),
    "fenv_rollout": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P]),
    "fenv_rollout_random": (_I32, [_P, _I32, _U64, _U64, _P, _P, _P, _P, _P, _P]),
    "fenv_partial_count": (_I64, [_P]),
    "fenv_rollout_kernel": (ctypes.c_char_p, [_P, _I32]),
    "fenv_reduce_partials": (_I32, [_P, _I64, _P, _P]),
    "fenv_stream_gate": (_I32, [_P, _U32, _I64, _P, _P]),
    "fenv_metrics": (_I32, [_P, _P, _P, _P, _P]),
    "fenv_get_state": (_I32, [_P, _P, _P, _P, _P, _P, _P]),
    "fenv_get_state_range": (_I32, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P]),
    "fenv_metrics_range": (_I32, [_P, _I64, _I64, _P, _P, _P, _P]),
    "fenv_abi_version": (_I32, []),
    "fenv_set_state": (_I32, [_P, _P, _P, _P, _P, _P, _P]),
    "fenv_host_reset_draws": (_I32, [_U32, _I64, _I64, _I64, _I64, _I32, _P, _P, _P, _P]),
    "fenv_desired_neighbor_dist": (ctypes.c_float, [_I32]),
    "fenv_fp_probe": (_I32, [_I32, _P, _P, _P, _I64, _P]),
    "policy_param_count": (_I32, [_I32]),
    "policy_forward": (_I32, [_P, _I32, _P, _I64, _I64, _P, _P, _P, _P, _P, _U64, _U64, _I32,
                              _P]),
    "rollout_gae": (_I32, [_P, _P, _P, _P, _P, _I32, _I64, ctypes.c_float, ctypes.c_float, _P, _P,
                           _P]),
    "fenv_policy_rollout": (_I32, [_P, _P, _I32, _U64, _U64, _I32, ctypes.c_float,
                                   ctypes.c_float, _P, _P]),
    "ppo_update": (_I32, [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I64, _P, _I32, _I32, _P,
                          _P, _P]),
    "ppo_workspace_bytes": (_I64, []),
    "ppo_update_ws": (_I32, [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I64, _P, _I32, _I32, _P,
                             _P, _P, _P]),
    "ppo_grad": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P, _I32, _I32, ctypes.c_float,
                        ctypes.c_float, _I32, _I32, _P, _P, _P, _P]),
    "ppo_apply": (_I32, [_P, _P, _P, _P, _P, _I32, _P, _P]),
    "fenv_test_ppo_inject": (None, [_I32]),
    "fenv_status": (_I32, [_P]),
    "fenv_test_stage_hook": (None, [_I32, _I32]),
    "fenv_pinned_pool_bytes": (_I64, [_I32]),
    "fenv_host_alloc": (_I32, [_I32, _I64, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "fenv_host_free": (_I32, [_I32, _P]),
    "fenv_debug_staging": (_I32, [_P, _I32, _P, _P]),
    "fenv_last_error": (ctypes.c_char_p, []),
}


class PPOHParams(ctypes.Structure):
    """``ppo_hparams`` (include/fenv.h)."""
    _fields_ = [(k, ctypes.c_float) for k in ("clip_range", "ent_coef", "vf_coef",
                                              "max_grad_norm", "lr", "beta1", "beta2", "eps")] + \
        [("normalize_advantage", ctypes.c_int32)]


class RolloutBufs(ctypes.Structure):
    """``fenv_rollout_bufs`` (include/fenv.h): device pointers of one fused rollout."""
    _fields_ = [(n, _P) for n in ("obs", "last_obs", "mu", "action", "clipped", "value",
                                  "log_prob", "reward", "episode_start", "done", "last_done",
                                  "last_value", "advantage", "ret")]


class FenvError(RuntimeError):
    """A libfenv.so call returned an error code."""


_lib = None


def header_symbols(path: str = HEADER) -> list[str]:
    """Function names declared in include/fenv.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*([a-z_0-9]+)\s*\(", src,
                                 flags=re.M)))


def lib() -> ctypes.CDLL:
    """Load libfenv.so (raises ImportError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: the formation env has no CPU fallback. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C marl-distributedformation_amd/csrc`.")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_deferred: list = []


def destroy_handle(h) -> None:
    """``fenv_destroy`` of a handle, from release() or a finalizer.  While a HIP graph is being
    captured on this thread's current stream the device frees inside it would invalidate the
    capture, so the handle is parked and destroyed at the next create/destroy outside a capture
    (the library also parks any free the runtime refuses, csrc/fenv_api.cpp)."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        _deferred.append(h)
        return
    flush_deferred()
    check(lib().fenv_destroy(h), "fenv_destroy")


def flush_deferred() -> None:
    """Destroy the handles parked by :func:`destroy_handle` (no-op while capturing)."""
    if not _deferred or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        return
    L = lib()
    while _deferred:
        L.fenv_destroy(_deferred.pop())


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().fenv_last_error().decode(errors="replace")
        raise FenvError(f"{what or 'libfenv'} failed (code {rc}): {msg}")


def ptr(t) -> ctypes.c_void_p | None:
    """Raw data pointer of a torch tensor / numpy array (None passes NULL)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return ctypes.c_void_p(t.data_ptr())
    return t.ctypes.data_as(ctypes.c_void_p)


def current_stream(device: torch.device | int | None = None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(device=None) -> torch.device:
    """The HIP device the env runs on; raise loudly when there is none (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the MI355X formation env has no CPU path "
                           "(the CPU restatement under oracle/ is a test checker, not a fallback)")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
    if d.type != "cuda":
        raise ValueError(f"FormationEnv device must be a HIP device, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


# live HostBlocks: host address -> (bytes, device address, device index), for device_address()
_blocks: dict[int, tuple[int, int, int]] = {}


def _host_free(device: int, host: int) -> None:
    _blocks.pop(host, None)
    if _lib is not None:
        _lib.fenv_host_free(device, ctypes.c_void_p(host))


def device_address(a: np.ndarray, device=None, align: int = 16) -> ctypes.c_void_p | None:
    """The device address of a C-contiguous numpy array that lies inside a live HostBlock (e.g.
    an observation array a FormationEnv's numpy face returned), so a kernel can read it in place;
    None for any other array, one not aligned to ``align`` bytes, or (``device`` given) one whose
    block was mapped for another device: a block's device address is only valid on its own."""
    if not isinstance(a, np.ndarray) or not a.flags.c_contiguous:
        return None
    p = a.ctypes.data
    if p % align:
        return None
    want = None if device is None else torch.device(device).index
    for base, (n, dev, di) in _blocks.copy().items():  # a finalizer may drop a block meanwhile
        if base <= p and p + a.nbytes <= base + n:
            if want is not None and want != di:
                return None
            return ctypes.c_void_p(dev + (p - base))
    return None


class HostBlock:
    """Numpy arrays in one block of coherent, device-mapped host memory (``fenv_host_alloc``): the
    kernels read and write them in place, so the numpy faces of reset / step need no DMA copies.
    ``fields`` is [(name, numpy dtype, shape)]; each field is an attribute (the numpy array,
    256-B aligned in the block) and ``dev(name)`` its device address.  The block goes back to the
    library's pool when the last array viewing it is gone, so arrays a caller kept stay valid
    after the env that filled them is released."""

    def __init__(self, device: torch.device, fields):
        offs, total = {}, 0
        for name, dt, shape in fields:
            offs[name] = total
            total += (int(np.prod(shape)) * np.dtype(dt).itemsize + 255) // 256 * 256
        h, d = _P(), _P()
        check(lib().fenv_host_alloc(device.index, max(total, 256), ctypes.byref(h),
                                    ctypes.byref(d)), "fenv_host_alloc")
        raw = (ctypes.c_uint8 * max(total, 256)).from_address(h.value)
        # freed with the last view: the arrays below hold `raw` through their base chain
        weakref.finalize(raw, _host_free, device.index, h.value)
        _blocks[h.value] = (max(total, 256), d.value, device.index)
        base = np.ctypeslib.as_array(raw)
        self._dev = {}
        for name, dt, shape in fields:
            n = int(np.prod(shape)) * np.dtype(dt).itemsize
            setattr(self, name, base[offs[name]:offs[name] + n].view(dt).reshape(shape))
            self._dev[name] = ctypes.c_void_p(d.value + offs[name])

    def dev(self, name: str) -> ctypes.c_void_p:
        return self._dev[name]
