"""The north star's floating-point bound for the policy path (BASELINE.json: "within 1e-5
relative (fp32)"), as one assertion shared by the GPU policy tests.

    |got - ref| <= 1e-5 * (|ref| + rms(ref))

* Elementwise 1e-5 relative for every entry at (or above) the output's own scale.
* The absolute floor is derived from the output's magnitude: 1e-5 of the RMS of ``ref`` over the
  batch (per output tensor).  It only matters for entries much smaller than the typical one --
  a head output or log-prob that lands near zero by cancellation in its final dot product or
  sum, where no fp32 evaluation order (torch's included) can promise 1e-5 of the tiny result
  itself.  For the SB3 policy outputs the RMS is O(0.1-1) (mu, value) and O(1) (log_prob), so
  the floor is 1e-6 - 1e-5 absolute, against the 2e-5 + 2e-5|ref| (mu/value) and 1e-4
  (log_prob) bounds of round 1.
"""
import numpy as np
import torch

REL = 1e-5


def bound(ref) -> np.ndarray:
    r = np.asarray(ref, np.float64)
    rms = float(np.sqrt(np.mean(r * r))) if r.size else 0.0
    return REL * (np.abs(r) + rms)


def assert_rel_close(got, ref, name: str = "") -> float:
    """Raise if any entry violates the bound; returns the worst |err| / bound (for reports)."""
    g = (got.detach().cpu().double().numpy() if isinstance(got, torch.Tensor)
         else np.asarray(got, np.float64))
    r = (ref.detach().cpu().double().numpy() if isinstance(ref, torch.Tensor)
         else np.asarray(ref, np.float64))
    assert g.shape == r.shape, (name, g.shape, r.shape)
    b = bound(r)
    err = np.abs(g - r)
    ratio = err / np.maximum(b, 1e-300)
    worst = float(ratio.max()) if ratio.size else 0.0
    if not np.all(err <= b):
        i = np.unravel_index(int(np.argmax(ratio)), ratio.shape)
        raise AssertionError(f"{name}: {int((err > b).sum())} of {err.size} entries exceed "
                             f"1e-5 (|ref| + rms); worst at {i}: got {g[i]!r} ref {r[i]!r} "
                             f"err {err[i]:.3e} bound {b[i]:.3e} ({worst:.2f}x)")
    return worst
