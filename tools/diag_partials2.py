"""Round-3 diagnosis, step 2: test_metrics_and_partials[500-5] fails in the full GPU suite (rewards
of the first step after an in-launch MT19937 reset are wrong for the leading agents) but passes
alone.  The test that runs before it (test_state_roundtrip_and_lockstep_rule) leaves two envs
that are now destroyed at once (no reference cycle since round 3) instead of at a later garbage
collection.  This replays that prelude before the failing sequence, in variants, and reports
where the first mismatch is: the reset positions the launch applied (state after launch 1 vs the
C oracle), or the rewards."""
import gc
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pkgload  # noqa: E402
from oracle import COracleEnv, synth_actions  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

venv = import_module(pkg.__name__ + ".vectorized_env")
lib = import_module(pkg.__name__ + "._lib")
DEV = "cuda:0"


def make(F, N, seed, **kw):
    return venv.FormationEnv({"num_formation": F, "num_agents_per_formation": N,
                              "goal_in_obs": True}, device=DEV, seed=seed, **kw)


def prelude(kind):
    if kind == "none":
        return
    env = make(10, 5, 1)
    env.reset()
    px, py, gx, gy, t = env.get_state()
    env.set_state(px + 1, py, gx, gy, t + 3)
    t_bad = t.clone()
    t_bad[0] += 1
    if kind != "noerr":
        try:
            env.set_state(px, py, gx, gy, t_bad)
        except lib.FenvError:
            pass
    ep = make(10, 5, 1, reset_mode="philox")
    ep.set_state(px, py, gx, gy, t_bad)
    if kind == "keep":
        return env, ep
    del env, ep
    if kind == "gc":
        gc.collect()


def run(kind):
    keep = prelude(kind)
    F, N = 500, 5
    env = make(F, N, 21, max_steps=3)
    ref = COracleEnv(F, N, True, 21, max_steps=3)
    o = env.reset()
    ro = ref.reset()
    obs_reset_ok = np.array_equal(o.view(np.uint32), ro.view(np.uint32))
    acts = np.stack([synth_actions(4, k, F * N, 1.0) for k in range(8)])
    obs, rew, done = env.rollout(torch.from_numpy(acts[:5]).to(DEV))
    st = [v.cpu().numpy() for v in env.get_state()]
    first_bad = None
    for k in range(5):
        ro_k, rr, rd, _ = ref.step(acts[k])
        if first_bad is None and not np.array_equal(rew[k].cpu().numpy().view(np.uint32), rr.view(np.uint32)):
            first_bad = ("reward", k)
    rst = ref.get_state()
    bad_state = [i for i, (a, b) in enumerate(zip(st, rst)) if not np.array_equal(a, b)]
    nbad = int((st[0] != rst[0]).sum()) if 0 in bad_state else 0
    first_idx = int(np.nonzero(st[0] != rst[0])[0][0]) if nbad else -1
    src = ""
    if nbad:  # which MT reset set the launch applied to the wrong agents (2 is right)
        import ctypes
        L = lib.lib()
        bad = np.nonzero(st[0] != rst[0])[0]
        for s_ in (0, 1, 2, 3, 4):
            hp = np.zeros(F * N, np.float32); hq = np.zeros(F * N, np.float32)
            g1 = np.zeros(F, np.float32); g2 = np.zeros(F, np.float32)
            f = lambda a: a.ctypes.data_as(ctypes.c_void_p)
            L.fenv_host_reset_draws(ctypes.c_uint32(21), ctypes.c_int64(s_), ctypes.c_int64(F),
                                    ctypes.c_int64(0), ctypes.c_int64(F), ctypes.c_int32(N),
                                    f(hp), f(hq), f(g1), f(g2))
            src += f" set{s_}:{int((st[0][bad] == hp[bad]).sum())}/{bad.size}"
        src += f" bad agents {bad[:8].tolist()}..{bad[-1]}"
    print(f"{kind:6s}: reset obs ok {obs_reset_ok}; first reward mismatch {first_bad};{src} state after the "
          f"in-launch reset differs in fields {bad_state} (px: {nbad} agents, first {first_idx})",
          flush=True)
    env.release()
    del keep


for rep in range(2):
    for kind in ("none", "full", "noerr", "gc", "keep"):
        run(kind)
