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


def test_split3_bf16_is_exact():
    """The bf16x6 conv's operand split: h + m + l == w exactly for fp32
    values of every magnitude the network sees (and the pieces shrink by
    >= 2^8 each, so the dropped piece products stay below fp32 rounding)."""
    from hzamd.infer import pack_conv3x3_x6, split3_bf16
    g = torch.Generator().manual_seed(0)
    w = torch.cat([torch.randn(100000, generator=g) * s for s in (1e-6, 1e-3, 1.0, 1e3)])
    h, m, lo = split3_bf16(w)
    assert torch.equal(h.double() + m.double() + lo.double(), w.double())
    nz = w != 0
    assert bool((m.float().abs()[nz] <= w.abs()[nz] * 2.0 ** -8).all())
    assert bool((lo.float().abs()[nz] <= w.abs()[nz] * 2.0 ** -16).all())
    wc = torch.randn(128, 128, 3, 3, generator=g)
    p = pack_conv3x3_x6(wc)
    assert p.shape == (9, 4, 3, 128, 32) and p.dtype == torch.bfloat16
    # tap (kh, kw) = (1, 2), ci 70 = chunk 2 lane 6, co 5, plane h
    assert p[5, 2, 0, 5, 6] == wc[5, 70, 1, 2].to(torch.bfloat16)
    rec = p.double().sum(2).permute(2, 1, 3, 0).reshape(128, 128, 3, 3)   # [co][ci][kh][kw]
    assert torch.equal(rec, wc.double())
