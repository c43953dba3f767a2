"""Experiment artefacts (g2048.experiment) on CPU: the reference's folder layout and file
formats (src/experiments.py:40-160), the notebook readers (experiments/notebook_utils.py:9-16),
model.pt interchange with the reference's nn.Sequential, and weights_only checkpoints."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

from g2048.experiment import (Experiment, episode_record, get_max_tile_frequency, load_checkpoint,
                              load_pickle, load_reference_module, real_state, reference_module)
from g2048.nets import det_init, make_net

REF_KEYS = {"max_tile", "merge_score", "number", "reward", "q_value", "epsilon", "number_moves"}


def test_layout_and_files(tmp_path):
    model = det_init(make_net("conv", dtype=torch.float64), 0.5)
    exp = Experiment("job", root=str(tmp_path), model=model)
    assert exp.folder == os.path.join(str(tmp_path), "experiments", "job")
    for sub in ("text", "binary", "binary/board_histories"):
        assert os.path.isdir(os.path.join(exp.folder, sub))
    exp.add_hyperparameter({"batch_size": 5000, "discount_factor": 0.8})
    with pytest.raises(AssertionError):
        exp.add_hyperparameter([("x", 1)])
    exp.add_episode(max_tile=256, merge_score=2200, number=0, reward=11.5, q_value=3.25,
                    epsilon=1.0, number_moves=191)
    hist = [(real_state(np.array([1, 0, 0, 0] * 4, np.uint8)), "u", 0)]
    exp.snapshot_game(hist, 0)
    exp.save()
    exp.save_games_played([hist])
    exp.save_games_played([hist, hist])

    hp = json.load(open(os.path.join(exp.folder, "text", "hyperparams.json")))
    assert hp == {"batch_size": 5000, "discount_factor": 0.8}
    rt = open(os.path.join(exp.folder, "text", "runtime.txt")).read()
    assert len(rt.split(":")) == 3
    eps = load_pickle(exp.folder, "episodes.p")
    assert len(eps) == 1 and set(eps[0]) == REF_KEYS
    assert eps[0]["max_tile"] == 256 and isinstance(eps[0]["max_tile"], np.int64)
    assert isinstance(eps[0]["reward"], np.float64)
    assert isinstance(load_pickle(exp.folder, "runtime.p"), float)
    assert load_pickle(exp.folder, "hyperparameters.p")["batch_size"] == 5000
    assert len(load_pickle(exp.folder, "games_played.p")) == 3
    snap = load_pickle(exp.folder, os.path.join("board_histories", "episode_0.p"))
    assert snap[0][1] == "u" and snap[0][0].dtype == np.int64 and snap[0][0][0, 0] == 2

    # model.pt is a plain nn.Sequential of the reference's classes with identical weights
    seq = load_reference_module(os.path.join(exp.folder, "binary", "model.pt"))
    assert isinstance(seq, torch.nn.Sequential) and isinstance(seq[0], torch.nn.Conv2d)
    x = torch.randint(0, 12, (9, 1, 4, 4)).double()
    assert torch.equal(seq(x), model(x))
    sd = torch.load(os.path.join(exp.folder, "binary", "model_state.pt"), weights_only=True)
    assert set(sd) == set(model.state_dict())

    # resume reads everything back
    r = Experiment("job", root=str(tmp_path), resumed=True)
    assert r.hyperparameters == exp.hyperparameters and len(r.episodes) == 1
    assert torch.equal(r.model(x), model(x))
    with pytest.raises(FileNotFoundError):
        Experiment("nope", root=str(tmp_path), resumed=True)


def test_auto_folder_names(tmp_path):
    a = Experiment(root=str(tmp_path))
    b = Experiment(root=str(tmp_path))
    na, nb = os.path.basename(a.folder), os.path.basename(b.folder)
    assert na.startswith("exp_1_") and nb.startswith("exp_2_")
    c = Experiment("fixed", root=str(tmp_path))
    d = Experiment("fixed", root=str(tmp_path))  # exists -> numbered folder instead
    assert os.path.basename(c.folder) == "fixed" and os.path.basename(d.folder).startswith("exp_3_")


def test_dense_model_pt_roundtrip(tmp_path):
    m = det_init(make_net("dense64"), 0.2)
    exp = Experiment("d", root=str(tmp_path), model=m)
    exp.save()
    seq = load_reference_module(os.path.join(exp.folder, "binary", "model.pt"))
    x = torch.rand(5, 16) * 10
    assert torch.equal(seq(x), m(x))
    assert torch.equal(reference_module(m)(x), m(x))


def test_episodes_from_log(tmp_path):
    """Device episode-log records -> reference add_episode dicts."""
    rec = {"step": torch.tensor([40, 45, 49]), "q_sum": torch.tensor([18.5, 0.0, -3.0], dtype=torch.float64),
           "board": torch.tensor([14, 40, 47]), "episode": torch.tensor([0, 0, 3]),
           "score": torch.tensor([168, 272, 316]), "moves": torch.tensor([41, 46, 50]),
           "max_exp": torch.tensor([4, 5, 0])}
    exp = Experiment("log", root=str(tmp_path))
    exp.add_episode(max_tile=2, merge_score=0, number=0, reward=0.0, number_moves=1)
    assert exp.add_episodes_from_log(rec, eps_decay=2.0, min_epsilon=0.01) == 3
    e = exp.episodes[1:]
    assert [d["number"] for d in e] == [1, 2, 3]
    assert [int(d["max_tile"]) for d in e] == [16, 32, 0]
    assert e[0]["reward"] == 168 / 41 and e[0]["q_value"] == 18.5 / 41
    assert e[1]["epsilon"] == 1.0 and e[2]["epsilon"] == 0.01  # max((2 - 3) / 2, 0.01)
    assert e[0]["number_moves"] == 41 and e[2]["board"] == 47 and e[2]["board_episode"] == 3
    assert REF_KEYS <= set(e[0])


def test_notebook_max_tile_frequency():
    f = get_max_tile_frequency([256, 128, 256, 512, 128, 256])
    assert f.tolist() == [[128, 256, 512], [2, 3, 1]]


def test_episode_record_types():
    r = episode_record(1024, 12000, 5, 3.5, None, 0.5, 700)
    assert r["q_value"] is None and r["epsilon"] == 0.5 and isinstance(r["merge_score"], np.int64)


def test_checkpoint_weights_only(tmp_path):
    exp = Experiment("ck", root=str(tmp_path))
    state = {"trainer": {"steps": 3}, "env": {"board": torch.zeros(4, 16, dtype=torch.uint8)},
             "learner": {"model": {"0.weight": torch.ones(2)}, "updates": 7}}
    exp.save_checkpoint(state)
    back = exp.load_checkpoint()
    assert back["trainer"]["steps"] == 3 and back["learner"]["updates"] == 7
    assert torch.equal(back["env"]["board"], state["env"]["board"])
    bad = os.path.join(str(tmp_path), "bad.pt")
    torch.save({"x": 1}, bad)
    with pytest.raises(ValueError):
        load_checkpoint(bad)
    # a pickled object (code) is refused by the weights_only loader
    with open(os.path.join(str(tmp_path), "evil.pt"), "wb") as f:
        pickle.dump({"format": "g2048-checkpoint-1", "obj": Experiment}, f)
    with pytest.raises(Exception):
        load_checkpoint(os.path.join(str(tmp_path), "evil.pt"))
