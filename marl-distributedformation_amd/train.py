"""Training entry point, the reference's ``python vectorized_env.py name=<run> key=value ...``.

Reference: ``run(cfg)`` at vectorized_env.py:112-137 (README.md:18): FormationEnv(cfg), an SB3
``CheckpointCallback(save_freq=10, save_path=f'{this_dir}/logs/{cfg.name}/')``,
``PPO('MlpPolicy', env, n_steps=10, learning_rate=1e-3, ent_coef=0.01)``, the no-op
``model.policy.log_std_init = -2`` (quirk Q2, not reproduced because it changes nothing) and
``learn(total_timesteps=5000 * cfg.num_formation, log_interval=4)``.  Here the env, the rollout
and GAE run on the HIP kernels and the PPO update on PyTorch-ROCm (ppo.py); wandb is replaced by
a console log every ``log_interval`` rollouts.

    python marl-distributedformation_amd/train.py name=myrun num_agents_per_formation=5
    torchrun --nproc-per-node 8 marl-distributedformation_amd/train.py name=myrun num_formation=8000

Extra keys (all optional, hydra ``key=value`` syntax): ``num_steps`` (5000, the reference's
constant), ``seed`` (env + policy seed), ``reset_mode`` (mt19937 | philox), ``batch_size`` /
``n_epochs`` (SB3 defaults 64 / 10), ``log_interval`` (4).  With several ranks the formations are
sharded contiguously.  The default update mode is "replicated" (ppo.py ``PPOConfig.update_mode``):
one all-gather of every rank's rollout samples per update (RCCL), then the same update on every
rank, with no gradient all-reduce; ``update_mode="sharded"`` instead all-reduces the flat gradient
once per global minibatch.
"""
from __future__ import annotations

import os
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pkg():
    if _ROOT not in sys.path:
        sys.path.insert(0, _ROOT)
    import pkgload
    return pkgload.load()


def main(argv: list[str] | None = None) -> str:
    """Train; returns the checkpoint directory (``<cwd>/logs/<name>/``)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    pkg = _pkg()
    from importlib import import_module
    config = import_module(pkg.__name__ + ".config")
    venv = import_module(pkg.__name__ + ".vectorized_env")
    ppo_mod = import_module(pkg.__name__ + ".ppo")
    ckpt = import_module(pkg.__name__ + ".checkpoint")
    pdist = import_module(pkg.__name__ + ".distributed")
    import torch

    cfg = config.load_config(overrides=argv)
    rank, world, local = pdist.init_from_env()
    torch.cuda.set_device(local)
    num_steps = int(cfg.get("num_steps", 5000))  # vectorized_env.py:116
    seed = int(cfg.get("seed", 0))
    first, F = pdist.shard_range(int(cfg.num_formation), rank, world)
    shard = dict(cfg.to_dict(), num_formation=F)
    env = venv.FormationEnv(shard, log=False, device=torch.device("cuda", local), seed=seed,
                            reset_mode=cfg.get("reset_mode", "mt19937"), first_formation=first,
                            total_formations=int(cfg.num_formation))
    this_dir = os.getcwd()  # hydra.utils.get_original_cwd()
    save_path = os.path.join(this_dir, "logs", str(cfg.name))
    checkpoint_callback = ckpt.CheckpointCallback(save_freq=10, save_path=save_path)
    pcfg = ppo_mod.PPOConfig(n_steps=10, learning_rate=1e-3, ent_coef=0.01,
                             batch_size=int(cfg.get("batch_size", 64)),
                             n_epochs=int(cfg.get("n_epochs", 10)))
    model = ppo_mod.PPO(env, pcfg, seed=seed)
    log_interval = int(cfg.get("log_interval", 4))
    t0 = time.perf_counter()
    state = {"it": 0}

    def log(m):
        state["it"] += 1
        if rank == 0 and state["it"] % log_interval == 0:
            el = time.perf_counter() - t0
            print(f"iterations {state['it']}  total_timesteps {m.num_timesteps}  "
                  f"fps {m.num_timesteps / el:.0f}  rollout_mean_reward "
                  f"{float(m.buffer.rewards.mean()):.4f}  " +
                  "  ".join(f"{k} {v:.4g}" for k, v in m.stats.items()), flush=True)

    model.learn(total_timesteps=num_steps * int(cfg.num_formation),
                callback=[checkpoint_callback, log])
    if world > 1:
        torch.distributed.destroy_process_group()
    return save_path


if __name__ == "__main__":
    main()
