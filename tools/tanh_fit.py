"""Coefficients of the small-argument tanh in csrc/ppo_update.hip (FENV_PPO_TANH_ACC):
tanh(x) = x + x^3 p(x^2) on |x| < 0.55, p of degree 4, fitted by least squares in the relative
error of tanh on Chebyshev nodes; checks the float32 Horner evaluation (fma) against float64
tanh, and the exp form 1 - 2 / (1 + 2^(2 x log2 e)) the kernel uses above 0.55."""
import numpy as np

X, DEG = 0.55, 4
u = (np.cos(np.linspace(0, np.pi, 4000)) + 1) / 2 * X * X
u = u[u > 1e-6]
x = np.sqrt(u)
f = (np.tanh(x) - x) / x ** 3
w = x ** 3 / np.tanh(x)
A = np.vstack([u ** k for k in range(DEG + 1)]).T
c, *_ = np.linalg.lstsq(A * w[:, None], f * w, rcond=None)
c32 = c.astype(np.float32)
print("coefficients (c0..c4):", [float(v) for v in c32])
xs = np.linspace(-X, X, 200001).astype(np.float32)
xs = xs[xs != 0]
u32 = (xs * xs).astype(np.float32)
p = np.float32(c32[-1])
for k in range(DEG - 1, -1, -1):
    p = (p.astype(np.float64) * u32 + c32[k]).astype(np.float32)
t = ((xs * u32).astype(np.float32).astype(np.float64) * p + xs).astype(np.float32)
ref = np.tanh(xs.astype(np.float64))
print("polynomial |x| < 0.55: max ulp", (np.abs(t - ref) / np.spacing(np.abs(ref).astype(np.float32))).max())
xs = np.linspace(-9, 9, 400001).astype(np.float32)
e = np.exp2((xs * np.float32(2.88539008177792681)).astype(np.float32)).astype(np.float32)
r = (1.0 / (np.float32(1) + e).astype(np.float64)).astype(np.float32)
t = (np.float32(1) - np.float32(2) * r).astype(np.float32)
ref = np.tanh(xs.astype(np.float64))
m = np.abs(xs) >= X
print("exp form |x| >= 0.55: max ulp", (np.abs(t - ref) / np.spacing(np.abs(ref).astype(np.float32)))[m].max())
m2 = (np.abs(xs) < X) & (xs != 0)
print("exp form |x| < 0.55: max relative error", (np.abs(t - ref) / np.abs(ref))[m2].max())
