"""g2048: MI355X-native batched 2048 environment + Double-DQN hot path.

Drop-in for the hot path of ribal-aladeeb/reinforcement-learning-2048 (src/board.py,
src/dqn_lib.py): the env step, replay buffer and train_step, batched over tens of thousands of
boards per launch on gfx950.  Native code: csrc/g2048.hip -> libg2048.so (C ABI include/g2048.h).
"""
from ._native import NativeError, load as load_native  # noqa: F401
from .env import ACTIONS, EpisodeLog, ReplayBuffer, VecEnv2048, decode_episodes  # noqa: F401

__all__ = ["VecEnv2048", "ReplayBuffer", "EpisodeLog", "decode_episodes", "ACTIONS", "NativeError",
           "load_native"]
