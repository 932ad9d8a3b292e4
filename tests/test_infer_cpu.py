"""FoldedNet (BatchNorm folded into the convs, NHWC; its HIP epilogue
restated in torch here) computes the eval-mode
reference network up to fp32 rounding: max |diff| <= 1e-4 on logits and
values (non-trivial BatchNorm statistics, default 128x8 architecture)."""
import torch

from hzamd.infer import FoldedNet
from hzamd.net import TINY, HarmoniesNet


def torch_epilogue(x, b, res=None):
    """Plain-torch restatement of hz_bias_act (the HIP epilogue FoldedNet
    uses on the GPU): relu((x + b[c]) + res)."""
    x = x + b.view(1, -1, 1, 1)
    if res is not None:
        x = x + res
    return x.relu()


def _randomise_bn(net, g):
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.2)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)


def _check(cfg, B):
    g = torch.Generator().manual_seed(3)
    torch.manual_seed(0)
    net = HarmoniesNet(cfg).eval()
    _randomise_bn(net, g)
    board = (torch.rand(B, 38, 5, 7, generator=g) > 0.8).float()
    glob = torch.rand(B, 42, generator=g)
    with torch.no_grad():
        l0, v0 = net(board, glob)
        l1, v1 = FoldedNet(net, torch_epilogue)(board, glob)
    assert l1.shape == l0.shape and v1.shape == v0.shape
    assert (l1 - l0).abs().max().item() <= 1e-4
    assert (v1 - v0).abs().max().item() <= 1e-4


def test_folded_matches_eval_default():
    _check(None, 16)


def test_folded_matches_eval_tiny():
    _check(TINY, 64)


def test_refresh_tracks_weight_updates():
    torch.manual_seed(1)
    net = HarmoniesNet(TINY).eval()
    f = FoldedNet(net, torch_epilogue)
    with torch.no_grad():
        net.conv.weight.mul_(1.5)
    f.refresh()
    board = torch.rand(4, 38, 5, 7)
    glob = torch.rand(4, 42)
    with torch.no_grad():
        assert (f(board, glob)[0] - net(board, glob)[0]).abs().max().item() <= 1e-4
