"""hzamd.manager.ModelManager against the reference ModelManager
(model.py): train_step losses and updated weights from the same initial
weights and batch (tests/golden/train.npz, captured from the reference on
CPU; fp32, atol 1e-6), the reference-written checkpoint loaded with the
safe loader (tests/golden/ref_ckpt_tiny.pth.tar), the forced LR reset on
load (model.py:198-236), and our own save -> load round trip."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from hzamd.manager import ModelManager

MODEL_CFG = {"input_channels": 38, "cnn_filters": 32, "board_size": (5, 7), "action_size": 143,
             "global_feature_size": 42, "value_head_hidden_dim": 64, "num_res_blocks": 1,
             "policy_head_conv_filters": 2, "value_head_conv_filters": 1}           # config.py test_model_config
TRAIN_CFG = {"device": "cpu", "optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 0.0,
             "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 4, "momentum": 0.9,
             "use_scheduler": True, "scheduler_type": "StepLR", "scheduler_step_size": 30,
             "scheduler_gamma": 0.5, "force_lr_reset_on_load": False, "new_forced_lr": 0.000125}


def fixture():
    return np.load(os.path.join(GOLDEN, "train.npz"))


def state(f, prefix):
    return {k[len(prefix):]: torch.from_numpy(f[k]) for k in f.files if k.startswith(prefix)}


def test_train_step_matches_reference():
    f = fixture()
    mm = ModelManager(MODEL_CFG, TRAIN_CFG)
    mm.model.load_state_dict(state(f, "init/"))
    b, g, pi, z = (torch.from_numpy(f[k]) for k in ("board", "glob", "pi", "z"))
    losses = np.array([mm.train_step(b, g, pi, z) for _ in range(3)])
    assert np.abs(losses - f["losses"]).max() <= 1e-6
    for k, v in state(f, "final/").items():
        assert (mm.model.state_dict()[k] - v).abs().max().item() <= 1e-6, k


def test_load_reference_checkpoint():
    f = fixture()
    mm = ModelManager(MODEL_CFG, TRAIN_CFG)
    ok, it = mm.load_checkpoint(folder=GOLDEN, filename="ref_ckpt_tiny.pth.tar")
    assert ok and it == 7
    for k, v in state(f, "final/").items():
        assert torch.equal(mm.model.state_dict()[k], v), k
    assert mm.get_current_lr() == 0.001
    assert len(mm.optimizer.state) == len(list(mm.model.parameters()))


def test_forced_lr_reset_on_load():
    mm = ModelManager(MODEL_CFG, dict(TRAIN_CFG, force_lr_reset_on_load=True))
    ok, it = mm.load_checkpoint(folder=GOLDEN, filename="ref_ckpt_tiny.pth.tar")
    assert ok and it == 7
    assert mm.optimizer.param_groups[0]["lr"] == 0.000125
    # StepLR(last_epoch=7 - 7 % 30 = 0) steps once in its constructor, as in the reference
    assert mm.scheduler.last_epoch == 1 and mm.get_current_lr() == 0.000125


def test_capturable_checkpoint_trains_on_cpu(tmp_path):
    """A checkpoint whose Adam groups say capturable=True (a GPU manager's
    optimizer state) loads into a CPU manager that can still train: the
    flag is set for the loading device and the step counters move to the
    host; our own files are written with capturable=False."""
    torch.manual_seed(4)
    a = ModelManager(MODEL_CFG, TRAIN_CFG)
    b, g = torch.rand(4, 38, 5, 7), torch.rand(4, 42)
    pi = torch.softmax(torch.rand(4, 143), 1)
    a.train_step(b, g, pi, torch.zeros(4, 1))
    a.save_checkpoint(folder=tmp_path, filename="a.pth.tar", iteration=1)
    ck = torch.load(tmp_path / "a.pth.tar", weights_only=True)
    assert all(not gr.get("capturable", False) for gr in ck["optimizer_state_dict"]["param_groups"])
    for gr in ck["optimizer_state_dict"]["param_groups"]:
        gr["capturable"] = True                      # as a GPU-written file of round 2 had it
    torch.save(ck, tmp_path / "gpu.pth.tar")
    c = ModelManager(MODEL_CFG, TRAIN_CFG)
    assert c.load_checkpoint(folder=tmp_path, filename="gpu.pth.tar") == (True, 1)
    assert all(gr["capturable"] is False for gr in c.optimizer.param_groups)
    loss = c.train_step(b, g, pi, torch.zeros(4, 1))
    a.train_step(b, g, pi, torch.zeros(4, 1))
    for k, v in a.model.state_dict().items():
        assert torch.equal(c.model.state_dict()[k], v), k
    assert np.isfinite(loss).all()


def test_checkpoint_round_trip(tmp_path):
    torch.manual_seed(3)
    a = ModelManager(MODEL_CFG, TRAIN_CFG)
    b, g = torch.rand(4, 38, 5, 7), torch.rand(4, 42)
    pi = torch.softmax(torch.rand(4, 143), 1)
    a.train_step(b, g, pi, torch.zeros(4, 1))
    a.step_scheduler()
    a.save_checkpoint(folder=tmp_path, filename="x.pth.tar", iteration=3)
    ck = torch.load(tmp_path / "x.pth.tar", weights_only=True)
    assert set(ck) == {"model_config", "training_config", "model_state_dict", "optimizer_state_dict",
                       "scheduler_state_dict", "iteration"}
    c = ModelManager(MODEL_CFG, TRAIN_CFG)
    assert c.load_checkpoint(folder=tmp_path, filename="x.pth.tar") == (True, 3)
    for k, v in a.model.state_dict().items():
        assert torch.equal(c.model.state_dict()[k], v)
    assert c.scheduler.last_epoch == 1
    assert c.load_checkpoint(folder=tmp_path, filename="missing.pth.tar") == (False, 0)
    p0, v0 = a.predict(b[0], g[0])
    p1, v1 = c.predict(b[0], g[0])
    assert p0.shape == (143,) and np.array_equal(p0, p1) and v0 == v1


def test_head_filters_in_config_are_ignored_like_the_reference():
    """The reference's ModelManager never passes the head conv filter counts
    to AlphaZeroModel (model.py:20-29), so its heads are always 2 / 1 filters
    (model.py:287-288): a config naming other counts builds the same network
    and state dict."""
    mm = ModelManager(dict(MODEL_CFG, policy_head_conv_filters=4, value_head_conv_filters=3), TRAIN_CFG)
    ref = ModelManager(MODEL_CFG, TRAIN_CFG)
    a, b = mm.model.state_dict(), ref.model.state_dict()
    assert list(a) == list(b) and all(a[k].shape == b[k].shape for k in a)
    assert a["policy_conv.weight"].shape[0] == 2 and a["value_conv.weight"].shape[0] == 1
