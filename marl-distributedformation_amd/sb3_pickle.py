"""The three pickled entries of an SB3 model zip's ``data`` -- ``policy_class``,
``observation_space``, ``action_space`` -- written without stable-baselines3 or gymnasium.

SB3's ``BaseAlgorithm.save`` stores every non-JSON attribute of the model as
``{":type:": str(type), ":serialized:": base64(cloudpickle.dumps(obj))}`` and ``PPO.load``
(``save_util.json_to_data``) turns it back with ``cloudpickle.loads``.  The reference's playback
(``/root/reference/visualize_policy.py:35``, ``PPO.load(checkpoint_path)`` with no
``custom_objects``) therefore needs these three entries to be real pickles: ``load`` raises
KeyError without the spaces, and the algorithm is rebuilt from ``policy_class``.

What cloudpickle emits for them, and what is emitted here opcode by opcode:
  * a class importable by name (SB3's ``ActorCriticPolicy``, which ``"MlpPolicy"`` resolves to
    for PPO) -> a by-reference GLOBAL, ``stable_baselines3.common.policies ActorCriticPolicy``;
  * a gymnasium ``Box`` instance (no ``__reduce__`` of its own) -> ``copyreg.__newobj__``:
    NEWOBJ of the class with no arguments, then BUILD with the instance ``__dict__``, which
    ``Space.__setstate__`` / ``Box.__setstate__`` take (``gymnasium/spaces/space.py``,
    ``box.py``: dtype, _shape, low, high, bounded_below, bounded_above, low_repr, high_repr,
    _np_random);
  * numpy arrays and dtypes -> their own ``__reduce__`` (``numpy.core.multiarray._reconstruct``
    + BUILD with (version, shape, dtype, fortran, raw bytes); ``numpy.dtype(str, False, True)``
    + BUILD with the dtype state).  ``numpy.core`` is the name numpy 1.x pickles with and numpy
    2.x keeps loadable, so the zip loads under either.

The reference's spaces (``/root/reference/vectorized_env.py:34-35``): action
``Box(-1, 1, (2,), float32)``, observation ``Box(-1, 1, (obs_dim,), float32)``.

Parity against SB3 / gymnasium: unpinned (neither is installed here).  The bytes are checked
by ``tests/test_checkpoint.py`` with ``pickle.loads`` against stand-in classes that restate the
two ``__setstate__`` methods, and the numpy parts against numpy itself.
"""
from __future__ import annotations

import base64
import struct

import numpy as np

_PROTO4 = b"\x80\x04"
_STOP = b"."
_MARK = b"("
_TUPLE = b"t"
_EMPTY_TUPLE = b")"
_EMPTY_DICT = b"}"
_SETITEMS = b"u"
_REDUCE = b"R"
_BUILD = b"b"
_NEWOBJ = b"\x81"
_NONE = b"N"
_TRUE = b"\x88"
_FALSE = b"\x89"


def _global(module: str, name: str) -> bytes:
    return b"c" + module.encode() + b"\n" + name.encode() + b"\n"


def _int(v: int) -> bytes:
    if 0 <= v < 256:
        return b"K" + bytes([v])
    if 0 <= v < 65536:
        return b"M" + struct.pack("<H", v)
    return b"J" + struct.pack("<i", v)


def _str(s: str) -> bytes:
    b = s.encode("utf-8")
    return (b"\x8c" + bytes([len(b)]) if len(b) < 256 else b"X" + struct.pack("<I", len(b))) + b


def _bytes(b: bytes) -> bytes:
    return (b"C" + bytes([len(b)]) if len(b) < 256 else b"B" + struct.pack("<I", len(b))) + b


def _tuple(items: list[bytes]) -> bytes:
    if not items:
        return _EMPTY_TUPLE
    return _MARK + b"".join(items) + _TUPLE


def _dict(items: list[tuple[str, bytes]]) -> bytes:
    return _EMPTY_DICT + _MARK + b"".join(_str(k) + v for k, v in items) + _SETITEMS


def _dtype(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    order = "|" if dt.itemsize == 1 else "<"
    # numpy.dtype.__reduce__: (dtype, (kind+size, False, True), (3, order, None, None, None,
    # -1, -1, flags)); flags 0 for the plain scalar types used here
    return (_global("numpy", "dtype") + _tuple([_str(dt.str[1:]), _FALSE, _TRUE]) + _REDUCE +
            _tuple([_int(3), _str(order), _NONE, _NONE, _NONE, _int_neg1(), _int_neg1(),
                    _int(0)]) + _BUILD)


def _int_neg1() -> bytes:
    return b"J" + struct.pack("<i", -1)


def _ndarray(a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a)
    if a.dtype.byteorder == ">":
        raise ValueError("big-endian arrays are not emitted")
    shape = _tuple([_int(int(s)) for s in a.shape])
    return (_global("numpy.core.multiarray", "_reconstruct") +
            _tuple([_global("numpy", "ndarray"), _tuple([_int(0)]), _bytes(b"b")]) + _REDUCE +
            _tuple([_int(1), shape, _dtype(a.dtype), _FALSE, _bytes(a.tobytes())]) + _BUILD)


def _short_repr(arr: np.ndarray) -> str:
    """gymnasium.spaces.box._short_repr: the scalar when all entries are equal, else the array."""
    if arr.size != 0 and np.min(arr) == np.max(arr):
        return str(np.min(arr))
    return str(arr)


def box_pickle(low: float, high: float, shape: tuple, dtype=np.float32) -> bytes:
    """cloudpickle bytes of ``gymnasium.spaces.Box(low, high, shape, dtype)``."""
    dt = np.dtype(dtype)
    lo = np.full(shape, low, dtype=dt)
    hi = np.full(shape, high, dtype=dt)
    state = [
        ("dtype", _dtype(dt)),
        ("_shape", _tuple([_int(int(s)) for s in shape])),
        ("low", _ndarray(lo)),
        ("high", _ndarray(hi)),
        ("bounded_below", _ndarray(np.asarray(-np.inf < lo))),
        ("bounded_above", _ndarray(np.asarray(np.inf > hi))),
        ("low_repr", _str(_short_repr(lo))),
        ("high_repr", _str(_short_repr(hi))),
        ("_np_random", _NONE),
    ]
    return (_PROTO4 + _global("gymnasium.spaces.box", "Box") + _EMPTY_TUPLE + _NEWOBJ +
            _dict(state) + _BUILD + _STOP)


def class_pickle(module: str, name: str) -> bytes:
    """cloudpickle bytes of a class importable as ``module.name`` (pickled by reference)."""
    return _PROTO4 + _global(module, name) + _STOP


def serialized(type_repr: str, payload: bytes) -> dict:
    """An SB3 ``data`` entry for a pickled object."""
    return {":type:": type_repr, ":serialized:": base64.b64encode(payload).decode()}


def sb3_opaque_entries(obs_dim: int, act_dim: int = 2) -> dict:
    """``policy_class``, ``observation_space`` and ``action_space`` as SB3 writes them for the
    reference's PPO('MlpPolicy', FormationEnv) (vectorized_env.py:34-35, 126)."""
    box_t = "<class 'gymnasium.spaces.box.Box'>"
    return {
        "policy_class": serialized(
            "<class 'abc.ABCMeta'>",
            class_pickle("stable_baselines3.common.policies", "ActorCriticPolicy")),
        "observation_space": serialized(box_t, box_pickle(-1.0, 1.0, (int(obs_dim),))),
        "action_space": serialized(box_t, box_pickle(-1.0, 1.0, (int(act_dim),))),
    }
