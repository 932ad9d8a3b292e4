"""ModelManager with the reference's interface and checkpoint format
(model.py:10-259), over hzamd.net.HarmoniesNet (same parameter names as
AlphaZeroModel, so state dicts move between the two unchanged).

  predict(board, glob)          -> (np.f32[143], float)         model.py:80-110
  train_step(board, glob, pi, z) -> (total, policy, value) losses model.py:112-157
  save_checkpoint / load_checkpoint                               model.py:159-252
  get_current_lr / step_scheduler                                 model.py:254-270

Checkpoints are the reference's dict (model_config, training_config,
model_state_dict, optimizer_state_dict, [scheduler_state_dict],
[iteration]) written with torch.save; loading uses weights_only=True, which
accepts every entry the reference writes.  The forced learning-rate reset on
load (training_config force_lr_reset_on_load / new_forced_lr, with the StepLR
re-initialisation at last_epoch = iteration - iteration % step_size) follows
model.py:198-236.
"""
from pathlib import Path

import torch
from torch import nn, optim
from torch.optim.lr_scheduler import ReduceLROnPlateau, StepLR

from .net import HarmoniesNet


def _net_cfg(model_config):
    """The AlphaZeroModel arguments ModelManager passes (model.py:20-29): the
    head conv filter counts are never passed, so the heads are always 2 / 1
    filters whatever the config says (model.py:287-288 defaults)."""
    keys = ("input_channels", "cnn_filters", "board_size", "action_size", "global_feature_size",
            "value_head_hidden_dim", "num_res_blocks")
    return {k: model_config[k] for k in keys if k in model_config}


class ModelManager:
    def __init__(self, model_config, training_config):
        self.model_config = model_config
        self.training_config = training_config
        self.device = torch.device(training_config["device"])
        self.initial_learning_rate = training_config["learning_rate"]
        self.model = HarmoniesNet(_net_cfg(model_config)).to(self.device)
        self.learning_rate = training_config["learning_rate"]
        if training_config["optimizer_type"] == "Adam":
            # capturable on the GPU: the step counter and bias corrections stay
            # on the device, so a training step can be replayed as a HIP graph
            # (hzamd.train.training_phase)
            self.optimizer = optim.Adam(self.model.parameters(), lr=self.initial_learning_rate,
                                        weight_decay=training_config["weight_decay"],
                                        capturable=self.device.type == "cuda")
        else:
            self.optimizer = optim.SGD(self.model.parameters(), lr=self.learning_rate,
                                       momentum=training_config["momentum"],
                                       weight_decay=training_config["weight_decay"])
        self.scheduler = None
        if training_config.get("use_scheduler", False):
            if training_config.get("scheduler_type", "StepLR").lower() == "steplr":
                self.scheduler = StepLR(self.optimizer, step_size=training_config.get("scheduler_step_size", 30),
                                        gamma=training_config.get("scheduler_gamma", 0.5))
        self.value_loss_fn = nn.MSELoss()
        self.value_loss_weight = training_config["value_loss_weight"]
        self.policy_loss_weight = training_config["policy_loss_weight"]
        self._folded = None
        self._folded_sig = None

    # -- inference -------------------------------------------------------------
    def _fast(self):
        """On the GPU: the folded network (hzamd.infer.FoldedNet: the HIP
        stem / tower / head kernels, one state per workgroup at batch 1) of
        the current weights, re-folded whenever any parameter or buffer was
        modified since (PyTorch's per-tensor version counters: optimizer
        steps, load_state_dict, any in-place write).  None on the CPU or for
        shapes the kernels do not cover."""
        if self.device.type != "cuda":
            return None
        tensors = list(self.model.parameters()) + list(self.model.buffers())
        # (invalidate_fold() clears _folded_sig for writes that bump no counter)
        sig = tuple((t.data_ptr(), t._version) for t in tensors)
        if self._folded is None or sig != self._folded_sig:
            from .infer import FoldedNet
            self.model.eval()
            if self._folded is None:
                self._folded = FoldedNet(self.model)
            else:
                self._folded.refresh()
            self._folded_sig = sig
        f = self._folded
        return f if f.stem_packed is not None and f.packed is not None else None

    def predict(self, board_tensor, global_features_tensor):
        """model.py:81-110: eval mode, softmax over all 143 logits."""
        if board_tensor.dim() == 3:
            board_tensor = board_tensor.unsqueeze(0)
        if global_features_tensor.dim() == 1:
            global_features_tensor = global_features_tensor.unsqueeze(0)
        self.model.eval()
        fast = self._fast()
        with torch.no_grad():
            board = board_tensor.to(self.device, torch.float32)
            glob = global_features_tensor.to(self.device, torch.float32)
            if fast is not None:
                from .infer import check_split_timeouts
                probs, value = fast.predict(board.contiguous(), glob.contiguous())
                check_split_timeouts(self.device)  # never hand a timed-out (NaN) prediction back
            else:
                logits, value = self.model(board, glob)
                probs = torch.softmax(logits, dim=1)
        return probs.squeeze(0).detach().cpu().numpy(), value.reshape(-1)[0].item()

    # -- training --------------------------------------------------------------
    def losses(self, board, glob, target_pi, target_z):
        """The reference's loss (model.py:135-147) as tensors (no sync)."""
        logits, value = self.model(board, glob)
        policy_loss = -torch.sum(target_pi * torch.log_softmax(logits, dim=1), dim=1).mean()
        value_loss = self.value_loss_fn(value, target_z)
        total = self.policy_loss_weight * policy_loss + self.value_loss_weight * value_loss
        return total, policy_loss, value_loss

    def train_step_async(self, board, glob, target_pi, target_z):
        """One optimiser step; returns the three losses as device tensors."""
        self.model.train()
        self.optimizer.zero_grad()
        total, pl, vl = self.losses(board.to(self.device), glob.to(self.device), target_pi.to(self.device),
                                    target_z.to(self.device))
        total.backward()
        self.optimizer.step()
        return total.detach(), pl.detach(), vl.detach()

    def train_step(self, board_tensor, global_features_tensor, target_policies, target_values):
        t, p, v = self.train_step_async(board_tensor, global_features_tensor, target_policies, target_values)
        return t.item(), p.item(), v.item()

    def invalidate_fold(self):
        """Weights changed behind PyTorch's version counters (a replayed HIP
        graph's optimizer step does not bump them): re-fold on the next predict."""
        self._folded_sig = None

    # -- checkpoints -----------------------------------------------------------
    def _portable_optimizer_state(self):
        """optimizer.state_dict() in the reference's form: a capturable GPU
        Adam keeps its step counters on the device and saves capturable=True,
        which a CPU Adam (model.py:199) cannot step after loading; the file
        gets capturable=False and host step counters."""
        sd = self.optimizer.state_dict()
        groups = [dict(g, capturable=False) if "capturable" in g else dict(g) for g in sd["param_groups"]]
        state = {k: {kk: (vv.detach().to("cpu", torch.float32) if kk == "step" and torch.is_tensor(vv) else vv)
                     for kk, vv in st.items()} for k, st in sd["state"].items()}
        return {"state": state, "param_groups": groups}

    def _adopt_optimizer_device(self):
        """After optimizer.load_state_dict: the groups' capturable flag comes
        from the file; set it for this device (capturable on the GPU, so that
        training can be graphed; plain on the CPU, as the reference) and move
        the step counters where that mode keeps them."""
        cap = self.device.type == "cuda"
        for g in self.optimizer.param_groups:
            if "capturable" in g:
                g["capturable"] = cap
                for p in g["params"]:
                    st = self.optimizer.state.get(p)
                    if st and torch.is_tensor(st.get("step")):
                        st["step"] = st["step"].to(p.device if cap else "cpu", torch.float32)

    def save_checkpoint(self, folder="checkpoints", filename="checkpoint.pth.tar", iteration=None):
        path = Path(folder)
        path.mkdir(parents=True, exist_ok=True)
        state = {"model_config": self.model_config, "training_config": self.training_config,
                 "model_state_dict": self.model.state_dict(),
                 "optimizer_state_dict": self._portable_optimizer_state()}
        if self.scheduler:
            state["scheduler_state_dict"] = self.scheduler.state_dict()
        if iteration is not None:
            state["iteration"] = iteration
        torch.save(state, path / filename)

    def load_checkpoint(self, folder="checkpoints", filename="checkpoint.pth.tar"):
        """Returns (loaded, iteration) like the reference; (False, 0) when the
        file is missing or unreadable."""
        path = Path(folder) / filename
        if not path.exists():
            return False, 0
        try:
            ck = torch.load(path, map_location=self.device, weights_only=True)
            self.model.load_state_dict(ck["model_state_dict"])
            self.optimizer.load_state_dict(ck["optimizer_state_dict"])
            self._adopt_optimizer_device()
            self.invalidate_fold()
            if self.scheduler and "scheduler_state_dict" in ck:
                self.scheduler.load_state_dict(ck["scheduler_state_dict"])
            it = ck.get("iteration", 0)
            if self.training_config.get("force_lr_reset_on_load", False) and it >= 0:
                forced = self.training_config.get("new_forced_lr")
                if forced is not None and forced > 0:
                    for g in self.optimizer.param_groups:
                        g["lr"] = forced
                    if self.scheduler and self.training_config.get("scheduler_type", "StepLR").lower() == "steplr":
                        step = self.training_config.get("scheduler_step_size", 30)
                        self.scheduler = StepLR(self.optimizer, step_size=step,
                                                gamma=self.training_config.get("scheduler_gamma", 0.5),
                                                last_epoch=it - (it % step))
            return True, it
        except Exception:
            return False, 0

    def get_current_lr(self):
        if self.scheduler:
            return self.scheduler.get_last_lr()[0]
        return self.optimizer.param_groups[0]["lr"]

    def step_scheduler(self, metric=None):
        if self.scheduler:
            if isinstance(self.scheduler, ReduceLROnPlateau):
                if metric is not None:
                    self.scheduler.step(metric)
            else:
                self.scheduler.step()
