"""Batched mirror of the reference's src/dqn_lib.py over VecEnv2048 / ReplayBuffer.

Same names, same argument meaning, same numerics (see the parity notes per function); the unit
of work is N boards / B transitions per call instead of one Board2048.  The injected callables
(board_to_tensor_function, extract_samples_function, reward_function) remain the plug points.

Reference findings honoured here: F1 the reference's train_step calls
zero_grad() between backward() and step(), so Adam never moves the weights -- reproduced with
reference_compat=True, the default is the intended zero_grad -> backward -> step; F5 the
epsilon-greedy normalisation bug (fused in the env kernel, "compat" flavour); F6 terminal
self-transitions (s, a, 0, s, 1); F7 float64 learner (dtype follows the model); F10 the target
network is evaluated without autograd.
"""
from __future__ import annotations

from typing import Callable

import torch

from .env import ReplayBuffer, VecEnv2048


# ------------------------------------------------------------------ encoders (src/dqn_lib.py:8-13)
def board_as_4d_tensor(env: VecEnv2048, device=None, dtype=torch.float64) -> torch.Tensor:
    """log_scale().state_as_4d_tensor() for every board: [N, 1, 4, 4] exponents."""
    return env.encode(dtype, conv=True)


def board_as_flattened_tensor(env: VecEnv2048, device=None, dtype=torch.float64) -> torch.Tensor:
    """log_scale().flattened_state_as_tensor() for every board: [N, 16] exponents."""
    return env.encode(dtype, conv=False)


class BoardBatch:
    """A batch of boards that are not an env's (sampled replay rows, the before / after boards
    of a step): the same `board` (u8 [n, 16] exponents), `n`, `device` and `encode()` as
    VecEnv2048, so every board_to_tensor_function -- the reference's two or a caller's own --
    takes either.  The Board2048 accessors a reward_function may use (src/board.py:204-231)
    answer for all n boards at once: `state` (tile values, int64 [n, 4, 4], 0 = empty),
    `merge_score()` (int64 [n], when the batch carries the scores: play_one_step passes the
    scores before / after the move), `simple_score()`, `log_scale()` (a batch whose `state` is
    the exponents) and `number_of_empty_cells()`."""

    def __init__(self, board: torch.Tensor, score: torch.Tensor | None = None, log: bool = False):
        self.board = board
        self.n = board.shape[0]
        self.device = board.device
        self._score = score
        self._log = log

    def encode(self, dtype=torch.float32, conv: bool = True):
        x = self.board.to(dtype)
        return x.view(self.n, 1, 4, 4) if conv else x

    @property
    def state(self) -> torch.Tensor:
        e = self.board.to(torch.int64)
        v = e if self._log else torch.where(e > 0, torch.ones_like(e) << e, torch.zeros_like(e))
        return v.view(self.n, 4, 4)

    def merge_score(self) -> torch.Tensor:
        if self._score is None:
            raise TypeError("merge_score(): this BoardBatch carries no scores (only the before / "
                            "after boards that play_one_step hands a reward_function do)")
        return self._score

    def simple_score(self) -> torch.Tensor:
        # sum of `state` (src/board.py:204-205): tile values, or exponents after log_scale()
        return self.state.flatten(1).sum(1)

    def log_scale(self) -> "BoardBatch":
        return BoardBatch(self.board, self._score, log=True)

    def number_of_empty_cells(self) -> torch.Tensor:
        return (self.board == 0).sum(1)


_FUSED_ENCODERS = (board_as_4d_tensor, board_as_flattened_tensor)


def reward_func_merge_score(board=None, next_board=None, action=None, done=None):
    """src/dqn_lib.py:87-88: next.merge_score() - board.merge_score().  The env kernel computes
    exactly this gain in-register; passing this function selects the fused path."""
    raise RuntimeError("reward_func_merge_score is computed inside the env step kernel")


def _custom_rewards(reward_function, s, s2, action, done, replay_buffer, row0, score0, gain):
    """A caller's reward_function(board, next_board, action, done) (src/dqn_lib.py:97,104) over
    the whole batch -- BoardBatch views of the boards before / after the move (s' = s for
    terminal and invalid moves, as the reference's peek_action) carrying the merge scores before
    (score0) and after (score0 + the kernel's merge gain), so the reference's own
    `next_board.merge_score() - board.merge_score()` works; actions and done flags as tensors --
    written over the kernel's merge-score rewards in the ring rows just appended.  The ring
    stores rewards as int32 (the reference's merge-score rewards are ints)."""
    r = reward_function(BoardBatch(s, score0), BoardBatch(s2, score0 + gain.to(torch.int64)),
                        action, done)
    r = torch.as_tensor(r, device=s.device)
    if r.shape != (s.shape[0],):
        raise ValueError(f"reward_function must return one reward per board ({s.shape[0]})")
    ri = r.to(torch.int32)
    if r.is_floating_point() and not torch.equal(ri.to(r.dtype), r):
        raise TypeError("the replay ring stores int32 rewards; reward_function returned "
                        "non-integer values")
    replay_buffer.r[row0:row0 + s.shape[0]].copy_(ri)
    return ri


# ------------------------------------------------------------------ acting (src/dqn_lib.py:16-30, 91-107)
def _model_dtype(model: torch.nn.Module) -> torch.dtype:
    return next(model.parameters()).dtype


@torch.no_grad()
def q_values(env: VecEnv2048, model: torch.nn.Module, board_to_tensor_function: Callable) -> torch.Tensor:
    dtype = _model_dtype(model)
    return model(board_to_tensor_function(env, env.device, dtype)).reshape(env.n, 4).contiguous()


def epsilon_greedy_policy(env: VecEnv2048, epsilon, model: torch.nn.Module, device=None,
                          board_to_tensor_function: Callable = board_as_4d_tensor,
                          replay_buffer: ReplayBuffer | None = None):
    """src/dqn_lib.py:16-30 for every board, fused with the move it selects (the action is
    applied in the same kernel, so this also advances the env like play_one_step).
    Returns (actions uint8 [N], done uint8 [N], max_q [N])."""
    q = q_values(env, model, board_to_tensor_function)
    action, reward, done = env.step_egreedy(q, epsilon, replay=replay_buffer)
    return action, done, q.amax(1)


def play_one_step(env: VecEnv2048, epsilon, model: torch.nn.Module, replay_buffer: ReplayBuffer,
                  device=None, reward_function: Callable = reward_func_merge_score,
                  board_to_tensor_function: Callable = board_as_4d_tensor):
    """src/dqn_lib.py:91-107 for N boards in one kernel: epsilon-greedy select (compat formula,
    F5), move + spawn, merge-score reward, done flag, replay append.  Terminal boards record
    (s, a, 0, s, 1) and are re-dealt.  With epsilon >= 1 no Q-values are needed and `model`
    may be None (the random branch returns before the forward, :20-21).
    A reward_function other than reward_func_merge_score is called as the reference calls it
    (board, next_board, action, done), batched: board / next_board are BoardBatch objects (the
    Board2048 accessors over all boards, merge scores included), action / done tensors, and it
    returns one reward per board (see _custom_rewards); it needs the replay buffer, where the
    transition's s' lives after the auto-reset.
    Returns (env, actions, rewards, dones, max_q_values)."""
    custom = reward_function is not reward_func_merge_score
    if custom and replay_buffer is None:
        raise ValueError("a custom reward_function needs the replay buffer (it holds s')")
    if model is None or (not isinstance(epsilon, torch.Tensor) and float(epsilon) >= 1.0):
        q = torch.zeros((env.n, 4), dtype=torch.float32, device=env.device)
    else:
        q = q_values(env, model, board_to_tensor_function)
    s = env.board.clone() if custom else None
    score0 = (env.score.to(torch.int64) & 0xFFFFFFFF) if custom else None  # u32 in int32
    row0 = int(env.clock[0]) % (replay_buffer.capacity // env.n) * env.n if custom else 0
    action, reward, done = env.step_egreedy(q, epsilon, replay=replay_buffer)
    if custom:
        reward = _custom_rewards(reward_function, s, replay_buffer.s2[row0:row0 + env.n],
                                 action, done, replay_buffer, row0, score0, reward)
    return env, action, reward, done, q.amax(1)


# ------------------------------------------------------------------ sampling (src/dqn_lib.py:33-84)
def extract_samples_conv(states: torch.Tensor) -> torch.Tensor:
    """Layout of extract_samples_conv (:33-46): [B, 1, 4, 4] (the gather + encode ran in-kernel)."""
    return states.view(states.shape[0], 1, 4, 4)


def extract_samples_dense(states: torch.Tensor) -> torch.Tensor:
    """Layout of extract_samples_dense (:49-64): [B, 16]."""
    return states.view(states.shape[0], 16)


def sample_experiences(batch_size: int, replay_buffer: ReplayBuffer, device=None,
                       board_to_tensor_function: Callable | None = None,
                       extract_sample_function: Callable = extract_samples_conv,
                       dtype=torch.float64, idx: torch.Tensor | None = None):
    """src/dqn_lib.py:67-84: B indices uniform with replacement over the filled rows
    (np.random.randint(len, size=B) -> torch RNG on the device, graph-safe), then the gather +
    encode.  With the reference's encoders (or None) the gather and the log2 encode are one
    fused kernel; any other board_to_tensor_function is applied, as in the reference
    (:71-80), to the sampled boards (BoardBatch views of the gathered rows) before
    extract_sample_function.  Returns (states, actions i64, rewards, next_states, dones)."""
    if idx is None:
        idx = (torch.rand(batch_size, dtype=torch.float64, device=replay_buffer.device)
               * replay_buffer.count.to(torch.float64)).to(torch.int64)
    if board_to_tensor_function is None or board_to_tensor_function in _FUSED_ENCODERS:
        s, a, r, s2, d, _ = replay_buffer.sample_encode(batch_size, dtype, idx=idx)
        return extract_sample_function(s), a, r, extract_sample_function(s2), d
    _, a, r, _, d, _ = replay_buffer.sample_encode(batch_size, dtype, idx=idx, want_s=False,
                                                   want_s2=False)
    dev = replay_buffer.device
    s = board_to_tensor_function(BoardBatch(replay_buffer.s[idx]), dev, dtype)
    s2 = board_to_tensor_function(BoardBatch(replay_buffer.s2[idx]), dev, dtype)

    def layout(x):  # the reference layouts apply to 16 values per board; other encodings pass
        return extract_sample_function(x.reshape(batch_size, 16)) if x[0].numel() == 16 else x

    return layout(s), a, r, layout(s2), d


def one_hot(tensor: torch.Tensor, no_outputs: int, device=None) -> torch.Tensor:
    """src/dqn_lib.py:110-116 (same assertions, float32 result)."""
    assert tensor.max().item() + 1 <= no_outputs, \
        "One hot encoded array size has to be bigger or equal than max scalar value"
    assert len(tensor.shape) == 1, "should be 1D"
    encoded = torch.zeros(tensor.shape[0], no_outputs, device=tensor.device)
    encoded[torch.arange(tensor.shape[0], device=tensor.device), tensor] = 1
    return encoded


# ------------------------------------------------------------------ learning (src/dqn_lib.py:119-164)
def bellman_targets(model, target_model, rewards, next_states, dones, discount_factor,
                    use_double_dqn: bool = True) -> torch.Tensor:
    """y = r + (1 - done) * gamma * Q_target(s', a*) with a* = argmax Q_online(s') (double,
    :125-132) or max_a Q_target(s', a) (vanilla, :133-144).  No autograd (F10).
    Parity: the reference multiplies the int64 (1 - dones) by the Python float gamma, which
    torch evaluates in float32, so gamma enters as float32(0.8) -- reproduced here."""
    with torch.no_grad():
        if use_double_dqn:
            a_star = torch.argmax(model(next_states), dim=1)
            next_q = target_model(next_states).gather(1, a_star[:, None])[:, 0]
        else:
            next_q = torch.max(target_model(next_states), dim=1).values
        disc = (1 - dones).to(torch.float32) * torch.tensor(discount_factor, dtype=torch.float32)
        return rewards.to(next_q.dtype) + disc.to(next_q.dtype) * next_q


def targets_from_q(q_online_next, q_target_next, rewards, dones, discount_factor,
                   use_double_dqn: bool = True) -> torch.Tensor:
    """bellman_targets given precomputed Q_online(s') / Q_target(s') (same float32-gamma parity)."""
    if use_double_dqn:
        a_star = torch.argmax(q_online_next, dim=1)
        next_q = q_target_next.gather(1, a_star[:, None])[:, 0]
    else:
        next_q = torch.max(q_target_next, dim=1).values
    disc = (1 - dones).to(torch.float32) * torch.tensor(discount_factor, dtype=torch.float32)
    return rewards.to(next_q.dtype) + disc.to(next_q.dtype) * next_q


def is_mse_sum(loss_fn) -> bool:
    """None or nn.MSELoss(reduction='sum') -- the loss of the reference configs
    (src/configs/double_dqn_conv.py:38), the one the fused HIP learner kernels implement."""
    return loss_fn is None or (isinstance(loss_fn, torch.nn.MSELoss) and loss_fn.reduction == "sum")


def dqn_loss(model, target_model, states, actions, rewards, next_states, dones, discount_factor,
             use_double_dqn: bool = True, loss_fn: Callable | None = None):
    """loss_fn(Q_online(s)[a], y) against the Bellman target (:146-158); None = MSELoss(sum).
    The reference's one_hot-mask-and-sum picks the same element as gather (exact)."""
    y = bellman_targets(model, target_model, rewards, next_states, dones, discount_factor,
                        use_double_dqn)
    q = model(states).gather(1, actions[:, None].to(torch.int64))[:, 0]
    if loss_fn is None:
        return ((q - y) ** 2).sum(), q, y
    return loss_fn(q, y), q, y


def train_step(batch_size: int, discount_factor: float, model: torch.nn.Module,
               target_model: torch.nn.Module, replay_buffer: ReplayBuffer,
               loss_fn: Callable | None, optimizer: torch.optim.Optimizer, device=None,
               use_double_dqn: bool = True,
               board_to_tensor_function: Callable = board_as_4d_tensor,
               extract_samples_function: Callable = extract_samples_conv,
               reference_compat: bool = False, idx: torch.Tensor | None = None):
    """src/dqn_lib.py:119-164 on one minibatch sampled from the HBM replay ring.
    loss_fn(q, y) as the reference calls it (:158); None = MSELoss(reduction='sum'), the configs'
    loss (src/configs/double_dqn_conv.py:38).  reference_compat=True reproduces the reference's
    backward -> zero_grad -> step order, in which the optimizer never updates (F1)."""
    dtype = _model_dtype(model)
    states, actions, rewards, next_states, dones = sample_experiences(
        batch_size, replay_buffer, device, board_to_tensor_function, extract_samples_function,
        dtype=dtype, idx=idx)
    if reference_compat:
        loss, _, _ = dqn_loss(model, target_model, states, actions, rewards, next_states, dones,
                              discount_factor, use_double_dqn, loss_fn)
        loss.backward()
        optimizer.zero_grad()
        optimizer.step()
        return loss
    optimizer.zero_grad()
    loss, _, _ = dqn_loss(model, target_model, states, actions, rewards, next_states, dones,
                          discount_factor, use_double_dqn, loss_fn)
    loss.backward()
    optimizer.step()
    return loss


def sync_target(model: torch.nn.Module, target_model: torch.nn.Module) -> None:
    """target_model.load_state_dict(copy.deepcopy(model.state_dict())) (src/dqn_lib.py:227-228),
    as an in-place device copy."""
    with torch.no_grad():
        for pt, p in zip(target_model.parameters(), model.parameters()):
            pt.copy_(p)
