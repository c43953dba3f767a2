"""Experiment artefacts in the reference's on-disk layout, plus full-state checkpoints.

Reference: src/experiments.py:40-160 (Experiment), experiments/notebook_utils.py:9-25 (readers).

    <root>/experiments/<name>/
        text/hyperparams.json         json.dump(hyperparameters, indent=4)        (:126-127)
        text/runtime.txt              'HH:MM:SS'                                 (:129-132)
        binary/hyperparameters.p      pickle of the hyperparameter dict          (:134-135)
        binary/runtime.p              pickle of round(elapsed, 2)                (:137-138)
        binary/episodes.p             pickle of the add_episode dict list        (:140-141)
        binary/model.pt               torch.save(nn.Sequential) -- reference module classes,
                                      so the reference notebooks can torch.load it (:143-144)
        binary/board_histories/episode_<n>.p   [(state int64[4,4], 'u'|'d'|'l'|'r', reward)]
        binary/games_played.p         Player histories (:146-160)
      added by this build (weights_only-loadable, no pickled code):
        binary/model_state.pt         state_dict of the online net
        binary/checkpoint.pt          everything needed to resume bit-exactly: online + target
                                      nets, Adam moments + device step, env boards / counters /
                                      reset epoch, replay ring, episode-log ring, trainer cadence

The reference saves neither the optimizer, nor the replay buffer, nor RNG state (SURVEY.md
sec. 5); checkpoint.pt adds them.  Episode dicts carry the reference's seven keys; records that
come from the device episode log also carry 'board' and 'board_episode'.
"""
from __future__ import annotations

import json
import os
import pickle
import time
import uuid

import numpy as np
import torch
from torch import nn

from .nets import Conv2048

EXPERIMENTS_DIRECTORY = "experiments"
ACTION_LETTERS = ("u", "d", "l", "r")  # src/dqn_lib.py:201 board_history action labels
CHECKPOINT_FORMAT = "g2048-checkpoint-1"


def reference_module(model: nn.Module) -> nn.Module:
    """A CPU nn.Sequential with the reference's layer classes and indices holding `model`'s
    weights (state_dict keys are identical), for binary/model.pt."""
    if isinstance(model, Conv2048):
        p = next(model.parameters())
        seq = nn.Sequential(nn.Conv2d(1, 64, kernel_size=2), nn.ReLU(),
                            nn.Conv2d(64, 64, kernel_size=2), nn.ReLU(), nn.Flatten(),
                            nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 4)).to(p.dtype)
        seq.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
        return seq
    if isinstance(model, nn.Sequential):
        # plain nn.Linear / nn.ReLU layers (the build's Linear subclass only changes the fp64
        # backward): the reference notebooks unpickle torch's own classes
        layers = []
        for m in model:
            if isinstance(m, nn.Linear):
                lin = nn.Linear(m.in_features, m.out_features, bias=m.bias is not None)
                layers.append(lin.to(m.weight.dtype))
            else:
                layers.append(type(m)())
        seq = nn.Sequential(*layers)
        seq.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
        return seq
    raise TypeError("model.pt export supports the conv net and nn.Sequential MLPs")


_SAFE_MODULES = [nn.Sequential, nn.Conv2d, nn.Linear, nn.ReLU, nn.Flatten]


def load_reference_module(path: str) -> nn.Module:
    """torch.load of a model.pt holding an nn.Sequential, with weights_only=True and only the
    reference's layer classes allowlisted (nothing else in the file is executed)."""
    with torch.serialization.safe_globals(_SAFE_MODULES):
        return torch.load(path, map_location="cpu", weights_only=True)


def episode_record(max_tile, merge_score, number, reward, q_value, epsilon, number_moves):
    """One Experiment.add_episode dict (src/experiments.py:112-122) with the reference's types."""
    return {"max_tile": np.int64(max_tile), "merge_score": np.int64(merge_score),
            "number": int(number), "reward": np.float64(reward),
            "q_value": None if q_value is None else np.float64(q_value),
            "epsilon": None if epsilon is None else float(epsilon),
            "number_moves": int(number_moves)}


def real_state(exps) -> np.ndarray:
    """Board exponents (u8[16]) -> the reference's Board2048.state (int64 [4, 4] tile values)."""
    e = np.asarray(exps, dtype=np.int64).reshape(4, 4)
    return np.where(e > 0, np.left_shift(1, e), 0).astype(np.int64)


class Experiment:
    """The reference Experiment (src/experiments.py:40-160): same folders, files and pickles.

    Experiment(folder_name, root)                    new experiment under root/experiments/
    Experiment(folder_name, root, resumed=True)      reload hyperparameters, runtime, episodes
    """

    def __init__(self, folder_name: str | None = None, root: str = ".", model=None,
                 resumed: bool = False, python_file_name: str | None = None):
        base = os.path.join(root, EXPERIMENTS_DIRECTORY)
        os.makedirs(base, exist_ok=True)
        self.model = model
        if resumed:
            self.folder = os.path.join(base, folder_name)
            if not os.path.isdir(self.folder):
                raise FileNotFoundError(f"You wish to resume an experiment which does not exist: "
                                        f"{folder_name}")
            with open(self._bin("hyperparameters.p"), "rb") as f:
                self.hyperparameters = pickle.load(f)
            with open(self._bin("runtime.p"), "rb") as f:
                self.runtime = pickle.load(f)
            with open(self._bin("episodes.p"), "rb") as f:
                self.episodes = pickle.load(f)
            if model is None and os.path.exists(self._bin("model.pt")):
                self.model = load_reference_module(self._bin("model.pt"))
            self._t0 = time.time() - float(self.runtime)
        else:
            self.folder = self._new_folder(base, folder_name)
            for sub in ("text", "binary", os.path.join("binary", "board_histories")):
                os.makedirs(os.path.join(self.folder, sub), exist_ok=True)
            self.hyperparameters = {}
            self.episodes = []
            self._t0 = time.time()
            self.runtime = self._t0
            if python_file_name:
                import shutil
                shutil.copyfile(python_file_name, os.path.join(
                    self.folder, os.path.basename(python_file_name) + ".txt"))

    @staticmethod
    def _new_folder(base: str, folder_name: str | None) -> str:
        """create_exp_folder (src/experiments.py:92-105): the given name, else exp_<n+1>_<tag>."""
        if folder_name is not None:
            path = os.path.join(base, folder_name)
            if not os.path.exists(path):
                os.makedirs(path)
                return path
            print(f"File {folder_name} already exists. Different folder name will be used.")
        nums = []
        for f in os.listdir(base):
            if f.startswith("exp_"):
                try:
                    nums.append(int(f[4:f.find("_", 4)]))
                except ValueError:
                    pass
        path = os.path.join(base, f"exp_{max(nums, default=0) + 1}_{uuid.uuid4().int % 10**18}")
        os.makedirs(path)
        return path

    def _bin(self, name: str) -> str:
        return os.path.join(self.folder, "binary", name)

    # ------------------------------------------------------------------ reference API
    def add_hyperparameter(self, mapping: dict) -> None:
        assert type(mapping) == dict, "When adding hyperparameters, pass them as dict"
        self.hyperparameters.update(mapping)

    def add_episode(self, max_tile, merge_score, number, reward, q_value=None, epsilon=None,
                    number_moves=0, **extra) -> dict:
        rec = episode_record(max_tile, merge_score, number, reward, q_value, epsilon,
                             number_moves)
        rec.update(extra)
        self.episodes.append(rec)
        return rec

    def add_episodes_from_log(self, records: dict, eps_decay: float | None = None,
                              min_epsilon: float = 0.0) -> int:
        """Append one add_episode dict per device episode-log record (g2048.EpisodeLog.read()).
        reward = mean per-step reward = score / moves; q_value = mean max-Q = q_sum / moves;
        epsilon = the board's schedule value for that episode (src/dqn_lib.py:184-188)."""
        k = int(records["step"].numel())
        if k == 0:
            return 0
        moves = records["moves"].double().clamp(min=1)
        reward = (records["score"].double() / moves).tolist()
        qv = (records["q_sum"] / moves).tolist()
        ep = records["episode"].double()
        if eps_decay:
            eps = torch.clamp((eps_decay - ep) / eps_decay, min=min_epsilon).tolist()
        else:
            eps = [None] * k
        mx = records["max_exp"].tolist()
        sc = records["score"].tolist()
        mv = records["moves"].tolist()
        bd = records["board"].tolist()
        be = records["episode"].tolist()
        base = len(self.episodes)
        for j in range(k):
            rec = episode_record(1 << mx[j] if mx[j] else 0, sc[j], base + j, reward[j], qv[j],
                                 eps[j], mv[j])
            rec["board"] = int(bd[j])
            rec["board_episode"] = int(be[j])
            self.episodes.append(rec)
        return k

    def snapshot_game(self, board_history, episode) -> None:
        with open(self._bin(os.path.join("board_histories", f"episode_{episode}.p")), "wb") as f:
            pickle.dump(board_history, f)

    def save(self) -> None:
        """The reference's save() (src/experiments.py:124-144) + model_state.pt."""
        with open(os.path.join(self.folder, "text", "hyperparams.json"), "w") as f:
            json.dump(self.hyperparameters, f, indent=4, default=str)
        elapsed = time.time() - self._t0
        with open(os.path.join(self.folder, "text", "runtime.txt"), "w") as f:
            f.write(time.strftime("%H:%M:%S", time.gmtime(elapsed)))
        with open(self._bin("hyperparameters.p"), "wb") as f:
            pickle.dump(self.hyperparameters, f)
        with open(self._bin("runtime.p"), "wb") as f:
            pickle.dump(round(elapsed, 2), f)
        with open(self._bin("episodes.p"), "wb") as f:
            pickle.dump(self.episodes, f)
        if self.model is not None:
            torch.save(reference_module(self.model), self._bin("model.pt"))
            torch.save({k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                       self._bin("model_state.pt"))

    def save_games_played(self, games_history: list) -> None:
        """Append to binary/games_played.p (src/experiments.py:146-160)."""
        path = self._bin("games_played.p")
        total = []
        if os.path.isfile(path):
            with open(path, "rb") as f:
                total = pickle.load(f)
        total += games_history
        with open(path, "wb") as f:
            pickle.dump(total, f)

    # ------------------------------------------------------------------ full state
    def save_checkpoint(self, state: dict) -> str:
        path = self._bin("checkpoint.pt")
        torch.save(dict(state, format=CHECKPOINT_FORMAT), path + ".tmp")
        os.replace(path + ".tmp", path)
        return path

    def load_checkpoint(self, map_location="cpu") -> dict:
        return load_checkpoint(self._bin("checkpoint.pt"), map_location)


def load_checkpoint(path: str, map_location="cpu") -> dict:
    """weights_only load of a checkpoint.pt (tensors, numbers, strings and containers only)."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    if state.get("format") != CHECKPOINT_FORMAT:
        raise ValueError(f"{path}: not a {CHECKPOINT_FORMAT} file")
    return state


def load_pickle(job_name: str, fn: str):
    """experiments/notebook_utils.py:9-12 (our own files only)."""
    with open(os.path.join(job_name, "binary", fn), "rb") as f:
        return pickle.load(f)


def get_max_tile_frequency(max_tiles) -> np.ndarray:
    """experiments/notebook_utils.py:14-16: [[tiles...], [counts...]]."""
    return np.array(np.unique(np.asarray(max_tiles), return_counts=True), dtype=int)
