"""Policy playback, the reference's ``python visualize_policy.py name=<run>`` (README.md:21).

Reference: visualize_policy.py:11-51 -- load the newest ``logs/<name>/rl_model_*_steps.zip``
(:29-35), build ``FormationEnv(cfg, visualize=True, log=False)`` with ``num_formation = 1``
(:36-37), and animate ``env.formationsim_list[0].fig`` (:38-48), each frame taking
``model.predict(obs, deterministic=True)`` and ``env.step(actions)`` and printing actions, obs,
rewards and dones (:11-20).  Here the policy is :class:`policy.MlpPolicy` (HIP kernel) loaded
from the zip's ``policy.pth`` and the figure is the host mirror of formation 0 (viz.py).

    python marl-distributedformation_amd/visualize_policy.py name=myrun
    python marl-distributedformation_amd/visualize_policy.py name=myrun steps_to_simulate=200 save=run.gif

Extra keys: ``steps_to_simulate`` (1000, as :39), ``save`` (write the animation to this file
instead of opening a window), ``quiet`` (skip the per-step prints), ``checkpoint`` (an explicit
zip instead of the newest one).
"""
from __future__ import annotations

import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Playback:
    """Env + policy + frame function (visualize_policy.py:11-20) for one formation."""

    def __init__(self, cfg, checkpoint_path: str, device=None, visualize: bool = True,
                 verbose: bool = True):
        from importlib import import_module
        pkg = _pkg()
        venv = import_module(pkg.__name__ + ".vectorized_env")
        pol_mod = import_module(pkg.__name__ + ".policy")
        self.model = pol_mod.MlpPolicy.from_checkpoint(checkpoint_path, device=device)
        cfg.num_formation = 1  # visualize_policy.py:36 (override)
        self.env = venv.FormationEnv(cfg, visualize=visualize, log=False, device=device)
        if self.model.obs_dim != self.env.obs_dim:
            raise ValueError(f"checkpoint obs_dim {self.model.obs_dim} != env obs_dim "
                             f"{self.env.obs_dim} (goal_in_obs mismatch)")
        self.first_env = self.env.formationsim_list[0]
        self.obs = self.env.reset()
        self.verbose = verbose

    def simulate_func(self, i):
        if self.verbose:
            print("-" * 10)
            print(f"Step {i}")
        actions, _states = self.model.predict(self.obs, deterministic=True)
        obs, rewards, dones, info = self.env.step(actions)
        if self.verbose:
            print(f"actions: {actions}")
            print(f"obs: {obs}")
            print(f"rewards: {rewards}")
            print(f"dones: {dones}")
        self.obs = obs
        return rewards, dones


def _pkg():
    if _ROOT not in sys.path:
        sys.path.insert(0, _ROOT)
    import pkgload
    return pkgload.load()


def main(argv: list[str] | None = None) -> Playback:
    argv = list(sys.argv[1:] if argv is None else argv)
    from importlib import import_module
    pkg = _pkg()
    config = import_module(pkg.__name__ + ".config")
    ckpt = import_module(pkg.__name__ + ".checkpoint")
    cfg = config.load_config(overrides=argv)
    path = cfg.get("checkpoint") or ckpt.latest_checkpoint(
        os.path.join(os.getcwd(), "logs", str(cfg.name)))
    print(f"Loading model from {path}")
    pb = Playback(cfg, path, verbose=not cfg.get("quiet", False))
    steps = int(cfg.get("steps_to_simulate", 1000))

    import matplotlib.animation as animation
    import matplotlib.pyplot as plt
    ani = animation.FuncAnimation(pb.first_env.fig, pb.simulate_func, frames=range(steps),
                                  interval=200)
    out = cfg.get("save")
    if out:
        ani.save(str(out), writer="pillow" if str(out).endswith(".gif") else None)
    else:
        plt.show()
    return pb


if __name__ == "__main__":
    main()
