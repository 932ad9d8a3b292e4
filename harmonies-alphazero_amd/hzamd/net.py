"""Policy/value network with the reference architecture (model.py:277-394).

This module restates the architecture (training runs it as a plain PyTorch
module) with parameter names matching model.py, so that `model_state_dict`
entries of the reference's checkpoints (model.py:161-182) load unchanged.
Leaf evaluation does not run it as is: hzamd.infer.FoldedNet folds its
eval-mode BatchNorms and runs the stem, the 16 tower convs and the heads as
hand-written HIP MFMA kernels (csrc/hz_net.hip); only the heads' linear
layers stay PyTorch.  (SURVEY §2 row 5 planned a stock-PyTorch leaf
evaluator; the network is 97 % of a 200-sim move, so it was replaced — see
DESIGN.md §0.)

Stem conv3x3 (38 -> F) + BN + ReLU; R residual blocks
(conv-BN-ReLU-conv-BN + skip, ReLU); policy head conv1x1 (F -> 2) + BN + ReLU,
flatten || globals -> Linear(70 + 42, 143); value head conv1x1 (F -> 1) + BN
+ ReLU, flatten || globals -> Linear(35 + 42, H) -> ReLU -> Linear(H, 1) -> tanh.
"""
import torch
from torch import nn

DEFAULT = dict(input_channels=38, cnn_filters=128, board_size=(5, 7), action_size=143,
               global_feature_size=42, value_head_hidden_dim=256, num_res_blocks=8,
               policy_head_conv_filters=2, value_head_conv_filters=1)
TINY = dict(DEFAULT, cnn_filters=32, value_head_hidden_dim=64, num_res_blocks=1)  # config.py:103-113


class _Block(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv1 = nn.Conv2d(ch, ch, 3, padding=1)
        self.bn1 = nn.BatchNorm2d(ch)
        self.conv2 = nn.Conv2d(ch, ch, 3, padding=1)
        self.bn2 = nn.BatchNorm2d(ch)

    def forward(self, x):
        y = torch.relu(self.bn1(self.conv1(x)))
        return torch.relu(self.bn2(self.conv2(y)) + x)


class HarmoniesNet(nn.Module):
    def __init__(self, cfg=None):
        super().__init__()
        c = dict(DEFAULT, **(cfg or {}))
        f, (h, w) = c["cnn_filters"], c["board_size"]
        pf, vf, g = c["policy_head_conv_filters"], c["value_head_conv_filters"], c["global_feature_size"]
        self.conv = nn.Conv2d(c["input_channels"], f, 3, padding=1)
        self.bn = nn.BatchNorm2d(f)
        self.residual_blocks = nn.ModuleList(_Block(f) for _ in range(c["num_res_blocks"]))
        self.policy_conv = nn.Conv2d(f, pf, 1)
        self.policy_bn = nn.BatchNorm2d(pf)
        self.policy_fc = nn.Linear(pf * h * w + g, c["action_size"])
        self.value_conv = nn.Conv2d(f, vf, 1)
        self.value_bn = nn.BatchNorm2d(vf)
        self.value_fc1 = nn.Linear(vf * h * w + g, c["value_head_hidden_dim"])
        self.value_fc2 = nn.Linear(c["value_head_hidden_dim"], 1)

    def forward(self, board, glob):
        x = torch.relu(self.bn(self.conv(board)))
        for blk in self.residual_blocks:
            x = blk(x)
        p = torch.relu(self.policy_bn(self.policy_conv(x))).flatten(1)
        logits = self.policy_fc(torch.cat((p, glob), 1))
        v = torch.relu(self.value_bn(self.value_conv(x))).flatten(1)
        v = torch.tanh(self.value_fc2(torch.relu(self.value_fc1(torch.cat((v, glob), 1)))))
        return logits, v


def flops_per_eval(cfg=None):
    """Forward multiply-adds x 2 for one position (convs + linears)."""
    c = dict(DEFAULT, **(cfg or {}))
    hw = c["board_size"][0] * c["board_size"][1]
    f, cin = c["cnn_filters"], c["input_channels"]
    conv = 2 * hw * 9 * (cin * f + 2 * c["num_res_blocks"] * f * f)
    heads = 2 * hw * f * (c["policy_head_conv_filters"] + c["value_head_conv_filters"])
    g = c["global_feature_size"]
    fc = 2 * ((c["policy_head_conv_filters"] * hw + g) * c["action_size"] +
              (c["value_head_conv_filters"] * hw + g) * c["value_head_hidden_dim"] + c["value_head_hidden_dim"])
    return conv + heads + fc


def load_reference_checkpoint(model, path, device="cpu"):
    """Load `model_state_dict` from a checkpoint written by
    ModelManager.save_checkpoint (model.py:161-182) — tensors only
    (weights_only=True: nothing in the file is executed)."""
    ckpt = torch.load(path, map_location=device, weights_only=True)
    state = ckpt.get("model_state_dict", ckpt) if isinstance(ckpt, dict) else ckpt
    model.load_state_dict(state)
    return ckpt
