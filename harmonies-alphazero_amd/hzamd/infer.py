"""Leaf-eval inference form of the reference network (model.py:325-394).

`ModelManager.predict` (model.py:81-110) runs the network in eval mode, where
every BatchNorm is a fixed per-channel affine map.  On MI355X the stock graph
spends most of its time in those BatchNorms: MIOpen's spatial inference
kernel takes ~1 ms per call on [4096, 128, 5, 7] (~150 GB/s), 19 calls per
forward, against ~0.4 ms for the 3x3 conv itself.  FoldedNet folds each
BatchNorm into the preceding conv's weights and bias once,

    W' = W * g / sqrt(var + eps),   b' = (b - mean) * g / sqrt(var + eps) + beta,

keeps activations NHWC (channels_last: MIOpen's implicit-GEMM NHWC conv runs
at ~106 TFLOP/s fp32 here, NCHW Winograd at ~82) and applies bias / residual
add / ReLU in place.  Arithmetic stays fp32; the results differ from the
unfolded graph only by fp32 rounding (tests/test_infer_gpu.py states the
tolerance).  Rebuild (or call refresh()) after the weights change.
"""
import torch
import torch.nn.functional as F
from torch import nn


def _fold(conv, bn):
    inv = torch.rsqrt(bn.running_var.double() + bn.eps) * bn.weight.double()
    w = (conv.weight.double() * inv.view(-1, 1, 1, 1)).float()
    b0 = conv.bias.double() if conv.bias is not None else torch.zeros_like(inv)
    b = ((b0 - bn.running_mean.double()) * inv + bn.bias.double()).float()
    return w.contiguous(memory_format=torch.channels_last), b.contiguous()


class FoldedNet(nn.Module):
    """Eval-mode HarmoniesNet (or the reference AlphaZeroModel: same module
    names) with BatchNorm folded into the convs; forward(board, glob) ->
    (logits [B,143], value [B,1]) like the source network."""

    def __init__(self, net):
        super().__init__()
        self.src = net
        self.refresh()

    @torch.no_grad()
    def refresh(self):
        n = self.src
        self.stem = _fold(n.conv, n.bn)
        self.blocks = [(_fold(b.conv1, b.bn1), _fold(b.conv2, b.bn2)) for b in n.residual_blocks]
        self.pconv = _fold(n.policy_conv, n.policy_bn)
        self.vconv = _fold(n.value_conv, n.value_bn)
        self.pfc = (n.policy_fc.weight.detach(), n.policy_fc.bias.detach())
        self.vfc1 = (n.value_fc1.weight.detach(), n.value_fc1.bias.detach())
        self.vfc2 = (n.value_fc2.weight.detach(), n.value_fc2.bias.detach())

    @torch.no_grad()
    def forward(self, board, glob):
        x = board.contiguous(memory_format=torch.channels_last)
        w, b = self.stem
        x = F.conv2d(x, w, b, padding=1).relu_()
        for (w1, b1), (w2, b2) in self.blocks:
            y = F.conv2d(x, w1, b1, padding=1).relu_()
            x = F.conv2d(y, w2, b2, padding=1).add_(x).relu_()
        w, b = self.pconv
        p = F.conv2d(x, w, b).relu_().flatten(1)               # NCHW order, as model.py flattens
        logits = F.linear(torch.cat((p, glob), 1), *self.pfc)
        w, b = self.vconv
        v = F.conv2d(x, w, b).relu_().flatten(1)
        v = F.linear(torch.cat((v, glob), 1), *self.vfc1).relu_()
        v = torch.tanh(F.linear(v, *self.vfc2))
        return logits, v
