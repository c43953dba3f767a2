"""Batched training_loop (src/dqn_lib.py:167-244) + the driver of src/double_dqn_conv.py.

Reference -> this build:
  one Board2048 per episode, episodes in sequence   n_boards boards stepped together; an
                                                    "episode" is any board's game
  epsilon = max((D - ep) / D, min_epsilon)          the same formula per board (its own episode
                                                    count), inside the fused step kernel
  train once per episode after 700 episodes         `updates_per_step` updates per rollout step
                                                    once the ring holds `min_fill` transitions
  target sync every 100 episodes                    every `target_sync_every` updates
  experiment.add_episode per episode                the step kernel's episode log, drained every
                                                    `check_every` steps
  snapshot_game every n episodes                    complete games of `track_boards` boards
  experiment.save() every 1000 episodes, at the     the same, plus binary/checkpoint.pt (full
  end and on KeyboardInterrupt / exceptions         state) so the run resumes bit-exactly
"""
from __future__ import annotations

import torch

from .env import ReplayBuffer, VecEnv2048
from .experiment import Experiment
from .learner import DQNLearner, Trainer


def build_trainer(n_boards: int = 65536, net: str = "conv", dtype=torch.float32,
                  batch_size: int = 8192, discount_factor: float = 0.8,
                  replay_buffer_length: int = 1 << 20, learning_rate: float = 1e-2,
                  use_double_dqn: bool = True, target_sync_every: int = 100,
                  no_episodes_to_reach_epsilon: float = 1000.0, min_epsilon: float = 0.01,
                  updates_per_step: int = 1, min_fill: int | None = None, seed: int = 0,
                  device="cuda:0", track_boards: int = 1, episode_log_slots: int = 8,
                  graph: bool = True, board_offset: int = 0, process_group=None,
                  loop_graph: bool | None = None, loss_fn=None) -> Trainer:
    cap = max(n_boards, (replay_buffer_length // n_boards) * n_boards)  # multiple of n
    env = VecEnv2048(n_boards, seed=0x2048 + seed, device=device, board_offset=board_offset)
    replay = ReplayBuffer(cap, device=device)
    learner = DQNLearner(replay, net=net, dtype=dtype, batch_size=batch_size,
                         discount_factor=discount_factor, lr=learning_rate,
                         use_double_dqn=use_double_dqn, target_sync_every=target_sync_every,
                         graph=graph, seed=seed, process_group=process_group, loss_fn=loss_fn)
    return Trainer(env, replay, learner, updates_per_step=updates_per_step, min_fill=min_fill,
                   eps_decay_episodes=no_episodes_to_reach_epsilon, min_epsilon=min_epsilon,
                   episode_log_slots=episode_log_slots, track_boards=track_boards,
                   graph=loop_graph)


def hyperparameters(trainer: Trainer, no_episodes: int, snapshot_game_every_n_episodes: int):
    """The HYPERPARAMS dict of src/configs/double_dqn_conv.py:49-66, for this build's run."""
    L = trainer.learner
    lr = L._adam.lr if L._adam is not None else L.opt.param_groups[0]["lr"]
    return {"batch_size": L.B, "discount_factor": L.gamma, "model": str(L.model),
            "replay_buffer_length": trainer.replay.capacity, "learning_rate": lr,
            "loss_fn": "MSELoss()" if L.loss_fn is None else str(L.loss_fn),
            "optimizer": "Adam (one HIP launch, device t)" if L._adam is not None else str(L.opt),
            "no_episodes": no_episodes, "no_episodes_to_reach_epsilon": trainer.eps_decay,
            "min_epsilon": trainer.min_eps, "use_double_dqn": L.use_double_dqn,
            "snapshot_game_every_n_episodes": snapshot_game_every_n_episodes,
            "n_boards": trainer.env.n, "updates_per_step": trainer.updates_per_step,
            "target_sync_every_updates": L.target_sync_every, "min_fill": trainer.min_fill,
            "dtype": str(L.dtype)}


def training_loop(trainer: Trainer, no_episodes: int, experiment: Experiment | None = None,
                  snapshot_game_every_n_episodes: int = 500, save_every_episodes: int = 1000,
                  check_every: int = 64, max_steps: int | None = None,
                  verbose: bool = False) -> Trainer:
    """Run until `no_episodes` episodes (over all boards) have finished (or max_steps rollout
    steps).  Episodes are logged into `experiment` in completion order; the run saves like the
    reference (every `save_every_episodes` episodes, at the end, on interrupt / error)."""
    done_eps = len(experiment.episodes) if experiment is not None else 0
    next_save = (done_eps // save_every_episodes + 1) * save_every_episodes
    next_snap = (done_eps // snapshot_game_every_n_episodes + 1) * snapshot_game_every_n_episodes

    def save():
        if experiment is not None:
            experiment.model = trainer.learner.model
            experiment.save()
            experiment.save_checkpoint(trainer.state_dict())

    try:
        steps = 0
        while done_eps < no_episodes and (max_steps is None or steps < max_steps):
            trainer.step()
            steps += 1
            if steps % check_every:
                continue
            rec = trainer.collect_episodes(experiment)
            done_eps += int(rec["step"].numel())
            if verbose and rec["step"].numel():
                print(f"step {trainer.steps}: {done_eps} episodes, last max tile "
                      f"{1 << int(rec['max_exp'].max())}, loss {float(trainer.learner.last_loss):.4g}")
            if experiment is not None and done_eps >= next_snap:
                trainer.snapshot_games(experiment)
                next_snap = (done_eps // snapshot_game_every_n_episodes + 1) * snapshot_game_every_n_episodes
            if done_eps >= next_save:
                save()
                next_save = (done_eps // save_every_episodes + 1) * save_every_episodes
        rec = trainer.collect_episodes(experiment)
        if experiment is not None:
            trainer.snapshot_games(experiment)
        save()
    except KeyboardInterrupt as e:
        print(e)
        print(f"\nKeyboard interrupt caught. Saving current experiment in "
              f"{experiment.folder if experiment else '(none)'}")
        save()
    except Exception:
        save()
        raise
    return trainer


def resume(folder_name: str, root: str = ".", **build_kwargs):
    """Reopen an experiment and its trainer at the saved state (binary/checkpoint.pt)."""
    exp = Experiment(folder_name, root=root, resumed=True)
    state = exp.load_checkpoint()
    e = state["env"]
    tr = build_trainer(n_boards=e["n"], seed=e["seed"] - 0x2048, board_offset=e["board_offset"],
                       replay_buffer_length=state["replay"]["capacity"],
                       episode_log_slots=state.get("episode_log", {}).get("slots", 8),
                       **build_kwargs)
    tr.load_state_dict(state)
    exp.model = tr.learner.model
    return exp, tr
