"""Diagnosis of the MT19937 post-reset mismatch, from the failure the round-4
job recorded (gpurun_out/r4a/pytest_new.log: test_mt_reset_staging_across_streams_and_churn,
call 0 step 3 -- the first in-launch reset -- observations wrong for a prefix of the agents).

Replays that test's sequence in variants and, at the first mismatch, records: the handle's
staging state and error words (fenv_debug_staging), which draw set the wrong agents' positions
came from (host replay of the global MT19937 stream), and the device / host contents of both
staging slots against the expected sets.  One JSON line per variant.

    python tools/mt_stage_repro.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pkgload  # noqa: E402
from oracle import COracleEnv, synth_actions  # noqa: E402

pkg = pkgload.load()
from importlib import import_module  # noqa: E402

ve = import_module(pkg.__name__ + ".vectorized_env")
L = import_module(pkg.__name__ + "._lib")
lib = L.lib()
DEV = "cuda:0"


def draws(seed, sset, F, N):
    px = np.zeros(F * N, np.float32)
    py = np.zeros(F * N, np.float32)
    gx = np.zeros(F, np.float32)
    gy = np.zeros(F, np.float32)
    lib.fenv_host_reset_draws(seed, sset, F, 0, F, N, *(a.ctypes.data_as(ctypes.c_void_p)
                                                       for a in (px, py, gx, gy)))
    return px, py, gx, gy


def staging(env, which=-1):
    info = (ctypes.c_int64 * 10)()
    out = None
    if which >= 0:
        out = np.zeros(int(env._stage_floats), np.float32)
    lib.fenv_debug_staging(env._h, which, None if out is None else out.ctypes.data_as(ctypes.c_void_p),
                           info)
    return list(info), out


def run(variant, F=500, N=5, seed=21, pre=True, streams=True, sync_after_reset=False):
    if pre:
        for Fp, Np in ((40, 5), (3, 100), (700, 5)):
            e = ve.FormationEnv({"num_formation": Fp, "num_agents_per_formation": Np,
                                 "goal_in_obs": True}, device=DEV, seed=Fp, max_steps=2)
            e.rollout(torch.rand((7, Fp * Np, 2), device=DEV) * 2 - 1)
            e.release()
    env = ve.FormationEnv({"num_formation": F, "num_agents_per_formation": N, "goal_in_obs": True},
                          device=DEV, seed=seed, max_steps=2)
    A = F * N
    env._stage_floats = 3 * A + 3 * F
    ref = COracleEnv(F, N, True, seed, max_steps=2)
    o = env.reset()
    rep = {"variant": variant}
    if not np.array_equal(o.view(np.uint32), ref.reset().view(np.uint32)):
        rep["reset_mismatch"] = True
    if sync_after_reset:
        torch.cuda.synchronize()
    rep["after_reset"] = staging(env)[0]
    info = rep["after_reset"]
    # where the terminal buffer's end sits relative to the staged sets: the grid's idle lanes
    # (f >= F) index term records a in [A, waves * fpw * N), i.e. bytes [16 A, 16 a_max) of term
    fpw = 64 // N if N <= 64 else 1
    waves = -(-F // fpw)
    groups = -(-waves // 4)
    a_max = groups * 4 * fpw * N + (64 - fpw * N)
    rep["term_end_to_pend_bytes"] = int(info[9] - (info[8] + 16 * A))
    rep["idle_term_bytes_past_end"] = [0, int(16 * (a_max - A))]
    # device slot 0 right after reset()'s refill (generation 3 = draw set 2)
    _, sl0 = staging(env, 0)
    px, py, gx, gy = draws(seed, 2, F, N)
    want = np.concatenate([px, py, gx, gy])
    mis = np.nonzero(sl0[:2 * A + 2 * F].view(np.uint32) != want.view(np.uint32))[0]
    rep["slot0_after_reset"] = {"mismatched": int(mis.size),
                                "first_last": [int(mis[0]), int(mis[-1])] if mis.size else None,
                                "zeros": int((sl0[mis] == 0).sum()) if mis.size else 0}
    ss = [torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)] if streams else None
    prev = torch.cuda.current_stream(DEV)
    k = 0
    for call, T in enumerate((30, 5, 1, 9, 4, 13)):
        acts = np.stack([synth_actions(6, k + j, A, 1.1) for j in range(T)])
        if ss is not None:
            st = ss[call % 2]
            st.wait_stream(prev)
            with torch.cuda.stream(st):
                a = torch.from_numpy(acts).to(DEV, non_blocking=False)
                obs, rew, done = env.rollout(a)
            prev = st
            st.synchronize()
        else:
            obs, rew, done = env.rollout(torch.from_numpy(acts).to(DEV))
            torch.cuda.synchronize()
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        for j in range(T):
            ro, rr, rd, _ = ref.step(acts[j])
            bad = np.nonzero((obs[j].view(np.uint32) != ro.view(np.uint32)).any(1))[0]
            badr = np.nonzero(rew[j].view(np.uint32) != rr.view(np.uint32))[0]
            if bad.size or badr.size or not np.array_equal(done[j], rd):
                rep["first_bad"] = {"call": call, "step": k + j, "obs_agents": int(bad.size),
                                    "rew_agents": int(badr.size)}
                if bad.size:
                    rep["first_bad"]["agents_first_last"] = [int(bad[0]), int(bad[-1])]
                    rep["first_bad"]["cols_wrong"] = np.nonzero(
                        (obs[j][bad].view(np.uint32) != ro[bad].view(np.uint32)).any(0))[0].tolist()
                    rep["first_bad"]["obs_gpu_row0"] = obs[j][bad[0]].tolist()
                    rep["first_bad"]["obs_ref_row0"] = ro[bad[0]].tolist()
                try:
                    env.check()
                    rep["status"] = "ok"
                except L.FenvError as ex:
                    rep["status"] = str(ex)
                info, _ = staging(env)
                rep["staging_info"] = info
                # which draw set the wrong agents' reset positions came from (obs column 0 =
                # px / 400 of the post-reset state when the step reset them)
                if bad.size and rd.any():
                    hits = {}
                    for sset in range(0, 8):
                        px, py, gx, gy = draws(seed, sset, F, N)
                        nx = (px / np.float32(400)).astype(np.float32)
                        hits[sset] = int((obs[j][bad, 0].view(np.uint32) ==
                                          nx[bad].view(np.uint32)).sum())
                    rep["wrong_agents_match_set"] = hits
                    zero = int((obs[j][bad, 0] == 0).sum())
                    rep["wrong_agents_x_zero"] = zero
                # staged slots vs the sets they should hold
                for which in range(4):
                    _, sl = staging(env, which)
                    sset_expected = info[1 + (which & 1)] - 1  # generation g = draw set g - 1
                    px, py, gx, gy = draws(seed, sset_expected, F, N)
                    want = np.concatenate([px, py, gx, gy])
                    got = sl[:2 * A + 2 * F]
                    mis = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
                    rep[f"slot{which}{'dev' if which < 2 else 'host'}"] = {
                        "gen": info[1 + (which & 1)], "mismatched_floats": int(mis.size),
                        "first": int(mis[0]) if mis.size else None,
                        "last": int(mis[-1]) if mis.size else None,
                        "zeros_in_mismatch": int((got[mis] == 0).sum()) if mis.size else 0}
                env.release()
                return rep
        k += T
    rep["ok"] = True
    try:
        env.check()
    except L.FenvError as ex:
        rep["status"] = str(ex)
    env.release()
    return rep


if __name__ == "__main__":
    for name, kw in (("as_test", {}), ("as_test_again", {}), ("no_pre_envs", {"pre": False}),
                     ("one_stream", {"streams": False}), ("sync_after_reset", {"sync_after_reset": True})):
        try:
            print(json.dumps(run(name, **kw)), flush=True)
        except Exception as ex:  # noqa: BLE001
            print(json.dumps({"variant": name, "error": f"{type(ex).__name__}: {ex}"}), flush=True)
