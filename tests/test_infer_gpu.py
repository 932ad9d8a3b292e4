"""FoldedNet on the GPU (HIP stem / tower / heads kernels) against the unfolded eval-mode
network run on the CPU in fp32: max |diff| <= 2e-3 on logits and values at
batch 512 with non-trivial BatchNorm statistics (different conv algorithms
and summation orders on the two devices)."""
import pytest
import torch

from hzamd.infer import FoldedNet
from hzamd.mcts import BatchedPredictor
from hzamd.net import HarmoniesNet
from test_infer_cpu import _randomise_bn

pytestmark = pytest.mark.gpu


def test_folded_gpu_matches_cpu_reference():
    g = torch.Generator().manual_seed(5)
    torch.manual_seed(0)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    board = (torch.rand(512, 38, 5, 7, generator=g) > 0.8).float()
    glob = torch.rand(512, 42, generator=g)
    with torch.no_grad():
        l0, v0 = net(board, glob)
    gnet = net.to("cuda")
    fnet = FoldedNet(gnet)
    # the default net must take the native kernels, not the MIOpen fallback
    assert fnet.stem_packed is not None and fnet.packed is not None and fnet.heads is not None
    assert fnet.fc is not None
    l1, v1 = fnet(board.cuda(), glob.cuda())
    assert (l1.cpu() - l0).abs().max().item() <= 2e-3
    assert (v1.cpu() - v0).abs().max().item() <= 2e-3
    p, v = BatchedPredictor(gnet)(board.cuda(), glob.cuda())
    assert (p.cpu() - torch.softmax(l0, 1)).abs().max().item() <= 2e-3
    assert (v.cpu() - v0.reshape(-1)).abs().max().item() <= 2e-3


def test_folded_gpu_matches_fp64_reference_at_leaf_batch():
    """The whole fused forward at the config-3 leaf batch (4096 encoder-like
    boards), random BatchNorm statistics, against the unfolded network run in
    float64 on the CPU: logits and values within 1e-4 (fp32 rounding of ~1,200-
    term sums; the fp32 CPU network itself is checked to the same bound)."""
    g = torch.Generator().manual_seed(11)
    torch.manual_seed(1)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    n = 4096
    board = (torch.rand(n, 38, 5, 7, generator=g) > 0.8).float()
    glob = torch.rand(n, 42, generator=g)
    with torch.no_grad():
        l64, v64 = net.double()(board.double(), glob.double())
        net.float()
        l32, v32 = net(board, glob)
    assert (l32.double() - l64).abs().max().item() <= 1e-4
    fnet = FoldedNet(net.to("cuda"))
    l1, v1 = fnet(board.cuda(), glob.cuda())
    dl = (l1.cpu().double() - l64).abs().max().item()
    dv = (v1.cpu().double() - v64).abs().max().item()
    assert dl <= 1e-4 and dv <= 1e-4, (dl, dv)


def test_folded_live_rows_equal_full_batch():
    """With a device live-row count k, the HIP kernels compute rows [0, k)
    exactly as in the full batch (row results do not depend on the batch)."""
    g = torch.Generator().manual_seed(3)
    torch.manual_seed(2)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    n = 1000
    board = (torch.rand(n, 38, 5, 7, generator=g) > 0.8).float().cuda()
    glob = torch.rand(n, 42, generator=g).cuda()
    fnet = FoldedNet(net.to("cuda"))
    l0, v0 = fnet(board, glob)
    pred = BatchedPredictor(net)
    p0, pv0 = pred(board, glob)
    for k in (0, 1, 7, 8, 9, 333, 1000):
        live = torch.tensor([k], dtype=torch.int32, device="cuda")
        l1, v1 = fnet(board, glob, live=live)
        assert torch.equal(l1[:k], l0[:k]) and torch.equal(v1[:k], v0[:k]), k
        p1, pv1 = pred(board, glob, None, live)
        assert torch.equal(p1[:k], p0[:k]) and torch.equal(pv1[:k], pv0[:k]), k


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("batch", [1, 3, 4096])
def test_bias_act_equals_torch_passes(batch, res):
    """hz_bias_act == the three torch passes it replaces (bias add, add_,
    relu_) exactly: same fp32 operations in the same order."""
    from hzamd.infer import _bias_act
    g = torch.Generator(device="cuda").manual_seed(batch)
    x = torch.randn(batch, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    b = torch.randn(128, device="cuda", generator=g)
    r = torch.randn(batch, 128, 5, 7, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last) if res else None
    want = x + b.view(1, -1, 1, 1)
    if res:
        want.add_(r)
    want.relu_()
    got = _bias_act(x.clone(memory_format=torch.channels_last), b, r)
    assert torch.equal(got, want)


def test_bias_act_rejects_nchw():
    from hzamd._native import NativeError
    from hzamd.infer import _bias_act
    x = torch.randn(2, 128, 5, 7, device="cuda")
    with pytest.raises(NativeError):
        _bias_act(x, torch.zeros(128, device="cuda"))


def _conv_ref(x, w, b, res):
    y = torch.nn.functional.conv2d(x.double(), w.double(), None, padding=1) + b.double().view(1, -1, 1, 1)
    if res is not None:
        y = y + res.double()
    return y.relu()


def _tower_conv(kind):
    from hzamd.infer import _conv3x3_act, _conv3x3_x6_act, pack_conv3x3, pack_conv3x3_x6
    if kind == "f32":
        return _conv3x3_act, pack_conv3x3
    return _conv3x3_x6_act, pack_conv3x3_x6


@pytest.mark.parametrize("kind", ["f32", "x6"])
@pytest.mark.parametrize("batch", [1, 13, 64])
@pytest.mark.parametrize("res", [False, True])
def test_conv3x3_exact_on_integer_data(batch, res, kind):
    """Small-integer inputs and weights: every product and partial sum is
    exact in fp32, so hz_conv3x3_bias_act (f32 MFMA) and
    hz_conv3x3_x6_bias_act (bf16 MFMA, split operands) must equal the fp64
    conv exactly (catches any operand-layout, tap or channel-order mistake;
    asymmetric weights so a transposed tap or swapped co/ci shows)."""
    _conv3x3_act, pack_conv3x3 = _tower_conv(kind)
    g = torch.Generator().manual_seed(batch * 2 + res)
    x = torch.randint(-3, 4, (batch, 128, 5, 7), generator=g).float()
    w = torch.randint(-2, 3, (128, 128, 3, 3), generator=g).float()
    b = torch.randint(-50, 50, (128,), generator=g).float()
    r = torch.randint(-20, 20, (batch, 128, 5, 7), generator=g).float() if res else None
    want = _conv_ref(x, w, b, r).float()
    cl = torch.channels_last
    got = _conv3x3_act(x.cuda().contiguous(memory_format=cl), pack_conv3x3(w).cuda(), b.cuda(),
                       r.cuda().contiguous(memory_format=cl) if res else None)
    assert torch.equal(got.cpu(), want)


@pytest.mark.parametrize("kind", ["f32", "x6"])
@pytest.mark.parametrize("batch", [8, 4096])
def test_conv3x3_matches_miopen_float(batch, kind):
    """Real-valued data at the leaf-eval batch: within fp32 rounding of
    MIOpen's conv + the torch epilogue (|diff| <= 1e-4 on O(1) outputs)."""
    _conv3x3_act, pack_conv3x3 = _tower_conv(kind)
    g = torch.Generator(device="cuda").manual_seed(batch)
    cl = torch.channels_last
    x = torch.randn(batch, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
    w = (torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.05).contiguous(memory_format=cl)
    b = torch.randn(128, device="cuda", generator=g) * 0.1
    r = torch.randn(batch, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=cl)
    want = (torch.nn.functional.conv2d(x, w, b, padding=1) + r).relu()
    got = _conv3x3_act(x, pack_conv3x3(w), b, r)
    assert (got - want).abs().max().item() <= 1e-4


@pytest.mark.parametrize("live", [None, 0, 1, 9, 300])
def test_conv3x3_x6_fp32_accuracy_vs_fp64(live):
    """Real-valued data (values not representable in bf16): the bf16x6 conv's
    error against a float64 conv is at the f32 MFMA conv's level (both are
    fp32 rounding: max |err| <= 2x the f32 kernel's + 1e-7; outputs reach
    ~10, so both are a few 1e-6); with a live-row bound the rows computed
    are unchanged."""
    from hzamd.infer import _conv3x3_act, _conv3x3_x6_act, pack_conv3x3, pack_conv3x3_x6
    n = 300
    g = torch.Generator().manual_seed(21)
    x = torch.randn(n, 128, 5, 7, generator=g).relu()
    w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    b = torch.randn(128, generator=g) * 0.1
    r = torch.randn(n, 128, 5, 7, generator=g)
    want = _conv_ref(x, w, b, r)
    cl = torch.channels_last
    xc, rc = x.cuda().contiguous(memory_format=cl), r.cuda().contiguous(memory_format=cl)
    e32 = (_conv3x3_act(xc, pack_conv3x3(w).cuda(), b.cuda(), rc).cpu().double() - want).abs().max().item()
    full = _conv3x3_x6_act(xc, pack_conv3x3_x6(w).cuda(), b.cuda(), rc)
    e6 = (full.cpu().double() - want).abs().max().item()
    assert e6 <= 2 * e32 + 1e-7, (e6, e32)
    if live is not None:
        lv = torch.tensor([live], dtype=torch.int32, device="cuda")
        part = _conv3x3_x6_act(xc, pack_conv3x3_x6(w).cuda(), b.cuda(), rc, lv)
        assert torch.equal(part[:live], full[:live])


@pytest.mark.parametrize("batch", [1, 7, 15, 29, 300])
def test_kernels_read_nothing_past_their_inputs(batch):
    """Every input is the prefix of a buffer whose tail is NaN: a kernel that
    reads past its last state (or past a state's 38 board channels into the
    next one, which the zero weight rows would otherwise hide) turns
    outputs into NaN.  The stems and tower convs at the small batch sizes the
    arena's routed leaf batches take."""
    from hzamd.infer import (_conv3x3_act, _conv3x3_x6_act, _stem_act, _stem_x6_act, pack_conv3x3,
                             pack_conv3x3_x6, pack_stem, pack_stem_x6)
    g = torch.Generator(device="cuda").manual_seed(batch)
    cl = torch.channels_last
    board = torch.full((batch + 2, 38, 5, 7), float("nan"), device="cuda")
    board[:batch] = (torch.rand(batch, 38, 5, 7, device="cuda", generator=g) > 0.7).float()
    ws = torch.randn(128, 38, 3, 3, device="cuda", generator=g) * 0.1
    b = torch.randn(128, device="cuda", generator=g) * 0.1
    for stem, pack in ((_stem_act, pack_stem), (_stem_x6_act, pack_stem_x6)):
        assert bool(torch.isfinite(stem(board[:batch], pack(ws), b)).all())
    x = torch.full((batch + 2, 128, 5, 7), float("nan"), device="cuda").contiguous(memory_format=cl)
    x[:batch] = torch.randn(batch, 128, 5, 7, device="cuda", generator=g)
    w = torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03
    for conv, pack in ((_conv3x3_act, pack_conv3x3), (_conv3x3_x6_act, pack_conv3x3_x6)):
        y = conv(x[:batch], pack(w), b, x[:batch])
        assert bool(torch.isfinite(y).all())


def test_folded_small_batches_match_large_batch():
    """FoldedNet on the small batches of a routed arena search (1..30 rows)
    gives each row the result it gets in a large batch."""
    g = torch.Generator().manual_seed(8)
    torch.manual_seed(3)
    net = HarmoniesNet().eval().cuda()
    board = (torch.rand(64, 38, 5, 7, generator=g) > 0.8).float().cuda()
    glob = torch.rand(64, 42, generator=g).cuda()
    fnet = FoldedNet(net)
    l0, v0 = fnet(board, glob)
    for k in (1, 2, 7, 15, 30):
        l1, v1 = fnet(board[:k].clone(), glob[:k].clone())
        assert torch.allclose(l1, l0[:k], atol=1e-5) and torch.allclose(v1, v0[:k], atol=1e-5), k


@pytest.mark.parametrize("n", [200, 1000])
def test_stem_x6_fp32_accuracy_vs_fp64(n):
    """Encoder-like boards (0, 1/3, 2/3, 1, bag fractions: not bf16 values):
    the bf16x6 stem's error vs a float64 conv is at the f32 stem's level, in
    the one-state form (200 rows) and the eight-state form with tap classes
    (1000 rows: all six products, the packed second chunk for every block)."""
    from hzamd.infer import _stem_act, _stem_x6_act, pack_stem, pack_stem_x6
    g = torch.Generator().manual_seed(4)
    board = torch.randint(0, 4, (n, 38, 5, 7), generator=g).float() / 3.0
    w = torch.randn(128, 38, 3, 3, generator=g) * 0.1
    b = torch.randn(128, generator=g) * 0.1
    want = _conv_ref(board, w, b, None)
    e32 = (_stem_act(board.cuda(), pack_stem(w).cuda(), b.cuda()).cpu().double() - want).abs().max().item()
    e6 = (_stem_x6_act(board.cuda(), pack_stem_x6(w).cuda(), b.cuda()).cpu().double() - want).abs().max().item()
    assert e6 <= 2 * e32 + 1e-7, (e6, e32)


@pytest.mark.parametrize("batch", [1, 5, 4096])
def test_heads_match_torch(batch):
    """hz_heads == conv1x1 + bias + ReLU, NCHW flatten, concat with glob for
    both heads (model.py:336-351), within fp32 summation-order rounding."""
    from hzamd.infer import _heads
    g = torch.Generator(device="cuda").manual_seed(batch)
    cl = torch.channels_last
    x = torch.randn(batch, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
    glob = torch.rand(batch, 42, device="cuda", generator=g)
    hw = torch.randn(3, 128, device="cuda", generator=g) * 0.1
    hb = torch.randn(3, device="cuda", generator=g) * 0.1
    p = torch.nn.functional.conv2d(x, hw[:2].reshape(2, 128, 1, 1), hb[:2]).relu().flatten(1)
    v = torch.nn.functional.conv2d(x, hw[2:].reshape(1, 128, 1, 1), hb[2:]).relu().flatten(1)
    pcat, vcat = _heads(x, glob, hw.contiguous(), hb.contiguous())
    assert pcat.shape == (batch, 112) and vcat.shape == (batch, 77)
    assert (pcat[:, :70] - p).abs().max().item() <= 1e-5
    assert (vcat[:, :35] - v).abs().max().item() <= 1e-5
    assert torch.equal(pcat[:, 70:], glob) and torch.equal(vcat[:, 35:], glob)


@pytest.mark.parametrize("kind", ["f32", "x6"])
@pytest.mark.parametrize("batch", [1, 13, 64, 1000])
def test_stem_exact_on_integer_data(batch, kind):
    """hz_stem3x3_bias_act / hz_stem3x3_x6_bias_act on small-integer data
    equal the fp64 conv exactly (NCHW board in, NHWC out; channel padding
    38 -> 48 / 64 must contribute 0)."""
    from hzamd.infer import _stem_act, _stem_x6_act, pack_stem, pack_stem_x6
    if kind == "x6":
        _stem_act, pack_stem = _stem_x6_act, pack_stem_x6
    g = torch.Generator().manual_seed(100 + batch)
    board = torch.randint(-3, 4, (batch, 38, 5, 7), generator=g).float()
    w = torch.randint(-2, 3, (128, 38, 3, 3), generator=g).float()
    b = torch.randint(-50, 50, (128,), generator=g).float()
    want = _conv_ref(board, w, b, None).float()
    got = _stem_act(board.cuda(), pack_stem(w).cuda(), b.cuda())
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got.cpu(), want)


@pytest.mark.parametrize("batch", [1, 7, 300, 2048, 2049, 4096])
def test_fused_head_matches_layers(batch):
    """hz_heads_fc (1x1 convs, both linear layers, softmax, tanh in one launch)
    against hz_heads + the PyTorch linear layers + torch.softmax / tanh on
    the same tower output, random BatchNorm statistics: within fp32
    summation-order rounding; with a live-row bound, the live rows match."""
    from hzamd.infer import _heads_fc
    g = torch.Generator().manual_seed(40 + batch)
    torch.manual_seed(batch)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    net = net.cuda()
    fused, split = FoldedNet(net), FoldedNet(net, fused_head=False)
    assert fused.fc is not None and split.fc is None
    cl = torch.channels_last
    x = torch.randn(batch, 128, 5, 7, generator=g).relu().cuda().contiguous(memory_format=cl)
    glob = torch.rand(batch, 42, generator=g).cuda()
    with torch.no_grad():
        pcat = torch.cat((torch.nn.functional.conv2d(x, *split.pconv).relu().flatten(1), glob), 1)
        vcat = torch.cat((torch.nn.functional.conv2d(x, *split.vconv).relu().flatten(1), glob), 1)
        l0 = torch.nn.functional.linear(pcat, *split.pfc)
        v0 = torch.tanh(torch.nn.functional.linear(torch.nn.functional.linear(vcat, *split.vfc1).relu(),
                                                   *split.vfc2)).reshape(-1)
    lo, pr, v = _heads_fc(x, glob, *fused.heads, fused.fc, logits=True, probs=True)
    assert (lo - l0).abs().max().item() <= 2e-5 * max(1.0, l0.abs().max().item())
    assert (pr - torch.softmax(l0, 1)).abs().max().item() <= 1e-6
    assert (v - v0).abs().max().item() <= 2e-6
    assert torch.allclose(pr.sum(1), torch.ones(batch, device="cuda"), atol=1e-5)
    k = max(1, batch // 2 - 3)
    live = torch.tensor([k], dtype=torch.int32, device="cuda")
    lo2, pr2, v2 = _heads_fc(x, glob, *fused.heads, fused.fc, live=live, logits=True, probs=True)
    assert torch.equal(lo2[:k], lo[:k]) and torch.equal(pr2[:k], pr[:k]) and torch.equal(v2[:k], v[:k])
    # the folded forward and predict give the same numbers through either head
    board = (torch.rand(batch, 38, 5, 7, generator=g) > 0.8).float().cuda()
    lf, vf = fused(board, glob)
    ls, vs = split(board, glob)
    assert vf.shape == vs.shape == (batch, 1)
    assert (lf - ls).abs().max().item() <= 2e-5 * max(1.0, ls.abs().max().item())
    assert (vf - vs).abs().max().item() <= 2e-6
    pf, vpf = fused.predict(board, glob)
    assert (pf - torch.softmax(ls, 1)).abs().max().item() <= 1e-6 and vpf.shape == (batch,)


def test_stem_x6_encoder_boards_take_exact_path():
    """Real encoder boards (channels 0-36 in {0, 1}, the phase channel 37 in
    {0, 1/3, 2/3}): every staged value is a bf16 value once channel 37 is
    staged as its three pieces, so the stem issues only the h plane's
    products; the result must still carry all six products of channel 37's
    split: error vs a float64 conv at the f32 stem's level (a lost piece of
    1/3 would show as ~1e-3)."""
    from hzamd.env import BatchedEnv
    from hzamd.infer import _stem_act, _stem_x6_act, pack_stem, pack_stem_x6
    n = 600
    env = BatchedEnv(n, seed_base=21, device="cuda")
    env.reset()
    plies = torch.arange(n, device="cuda") % 50
    for p in range(50):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
    board, _ = env.encode()
    env.close()
    ph = board[:, 37].amax((1, 2))
    assert bool(((ph - 1 / 3).abs() < 1e-6).any()) and bool(((ph - 2 / 3).abs() < 1e-6).any())
    g = torch.Generator().manual_seed(9)
    w = torch.randn(128, 38, 3, 3, generator=g) * 0.1
    b = torch.randn(128, generator=g) * 0.1
    want = _conv_ref(board.cpu(), w, b, None)
    e32 = (_stem_act(board, pack_stem(w).cuda(), b.cuda()).cpu().double() - want).abs().max().item()
    got = _stem_x6_act(board, pack_stem_x6(w).cuda(), b.cuda())
    e6 = (got.cpu().double() - want).abs().max().item()
    assert e6 <= 2 * e32 + 1e-7, (e6, e32)


def test_x6_small_batch_kernel_matches_large_batch_kernel():
    """Batches of at most 768 rows run the one-state-per-workgroup variant of
    the x6 conv and stem: each row's products and sums are issued in the same
    order as in the eight-state variant, so a row's output is bit-identical
    whichever variant computed it."""
    from hzamd.infer import _conv3x3_x6_act, _stem_x6_act, pack_conv3x3_x6, pack_stem_x6
    g = torch.Generator(device="cuda").manual_seed(77)
    cl = torch.channels_last
    big = 1100
    x = torch.randn(big, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
    r = torch.randn(big, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=cl)
    w = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
    b = torch.randn(128, device="cuda", generator=g)
    board = (torch.rand(big, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
    board[:, 37] = (torch.arange(big, device="cuda") % 4).float().view(-1, 1, 1) / 3.0
    ws = pack_stem_x6(torch.randn(128, 38, 3, 3, device="cuda", generator=g) * 0.1)
    full = _conv3x3_x6_act(x, w, b, r)
    sfull = _stem_x6_act(board, ws, b)
    for k in (1, 30, 767):
        sub = _conv3x3_x6_act(x[:k].contiguous(memory_format=cl), w, b, r[:k].contiguous(memory_format=cl))
        assert torch.equal(sub, full[:k]), k
        assert torch.equal(_stem_x6_act(board[:k].contiguous(), ws, b), sfull[:k]), k


def test_x6_eight_state_form_live_rows_and_accuracy():
    """The eight-state tower conv (batches above 768 rows: rows grouped by
    tap class, off-board taps skipped) against float64, and with a live-row
    bound that ends inside a workgroup (517 = 64 x 8 + 5): the live rows are
    the rows of the unbounded run, bit for bit."""
    from hzamd.infer import _conv3x3_x6_act, pack_conv3x3_x6
    n = 1000
    g = torch.Generator().manual_seed(33)
    x = torch.randn(n, 128, 5, 7, generator=g).relu()
    w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    b = torch.randn(128, generator=g) * 0.1
    r = torch.randn(n, 128, 5, 7, generator=g)
    cl = torch.channels_last
    xc, rc = x.cuda().contiguous(memory_format=cl), r.cuda().contiguous(memory_format=cl)
    wp = pack_conv3x3_x6(w).cuda()
    full = _conv3x3_x6_act(xc, wp, b.cuda(), rc)
    want = _conv_ref(x[:64], w, b, r[:64])
    assert (full[:64].cpu().double() - want).abs().max().item() <= 1e-5
    lv = torch.tensor([517], dtype=torch.int32, device="cuda")
    part = _conv3x3_x6_act(xc, wp, b.cuda(), rc, lv)
    assert torch.equal(part[:517], full[:517])


@pytest.mark.parametrize("batch", [769, 803, 4096])
def test_resblock_x6_fused_equals_two_layered_convs(batch):
    """hz_resblock_x6_bias_act as one launch (the 4-wave conv's batch sizes:
    conv1's output relu(acc + b1) staged for conv2 on the CU, through LDS and
    half of it through tmp) gives the bits of the two layered convs,
    with a partly filled last workgroup (803 = 100 x 8 + 3), a live-row bound
    inside a workgroup, and a NaN tail past the input (nothing read past the
    batch); and stays within fp32 rounding of a float64 block."""
    from hzamd._native import lib
    from hzamd.infer import _conv3x3_x6_act, _resblock_x6, pack_conv3x3_x6
    prev = lib().hz_resblock_x6_fused(4096)
    assert lib().hz_resblock_x6_set_fused(1) == 0
    try:
        for table in (0, 1):  # both row placements of the one-launch form (hz_resblock_x6_set_table)
            assert lib().hz_resblock_x6_set_table(table) == 0
            _check_resblock(batch, lib, _conv3x3_x6_act, _resblock_x6, pack_conv3x3_x6)
    finally:
        lib().hz_resblock_x6_set_fused(prev)
        lib().hz_resblock_x6_set_table(1)


def _check_resblock(batch, lib, _conv3x3_x6_act, _resblock_x6, pack_conv3x3_x6):
    assert lib().hz_resblock_x6_fused(batch) == 1
    g = torch.Generator().manual_seed(batch)
    cl = torch.channels_last
    x = torch.randn(batch, 128, 5, 7, generator=g).relu()
    w1 = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    w2 = torch.randn(128, 128, 3, 3, generator=g) * 0.03
    b1 = torch.randn(128, generator=g) * 0.1
    b2 = torch.randn(128, generator=g) * 0.1
    buf = torch.full((batch + 9, 128, 5, 7), float("nan"), device="cuda").contiguous(memory_format=cl)
    buf[:batch] = x.cuda()
    xc = buf[:batch]
    p1, p2 = pack_conv3x3_x6(w1).cuda(), pack_conv3x3_x6(w2).cuda()
    b1c, b2c = b1.cuda(), b2.cuda()
    fused = _resblock_x6(xc, p1, b1c, p2, b2c)
    layered = _conv3x3_x6_act(_conv3x3_x6_act(xc, p1, b1c), p2, b2c, xc)
    assert torch.equal(fused, layered)
    live = torch.tensor([batch - 4], dtype=torch.int32, device="cuda")
    part = _resblock_x6(xc, p1, b1c, p2, b2c, live)
    assert torch.equal(part[:batch - 4], fused[:batch - 4])
    k = 48
    want = _conv_ref(_conv_ref(x[:k], w1, b1, None).float(), w2, b2, x[:k])
    assert (fused[:k].cpu().double() - want).abs().max().item() <= 2e-5


def test_folded_net_fused_blocks_same_bits():
    """The whole folded forward with every residual block as one launch
    (hz_resblock_x6_set_fused(1), the default) gives the layered forward's
    logits and values bit for bit (1,100 encoder-like boards: above the resident
    tower's 1,024, so the layered blocks run; live bound inside a
    workgroup)."""
    from hzamd._native import lib
    g = torch.Generator().manual_seed(12)
    torch.manual_seed(12)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    n = 1100
    board = (torch.rand(n, 38, 5, 7, generator=g) > 0.8).float().cuda()
    board[:, 37] = 2.0 / 3.0
    glob = torch.rand(n, 42, generator=g).cuda()
    fnet = FoldedNet(net.cuda())
    assert n > fnet.resident_max
    live = torch.tensor([n - 5], dtype=torch.int32, device="cuda")
    prev = lib().hz_resblock_x6_fused(4096)
    try:
        assert lib().hz_resblock_x6_set_fused(0) == 0
        l0, v0 = fnet(board, glob, live=live)
        assert lib().hz_resblock_x6_set_fused(1) == 0
        assert lib().hz_resblock_x6_fused(n) == 1
        l1, v1 = fnet(board, glob, live=live)
    finally:
        lib().hz_resblock_x6_set_fused(prev)
    assert torch.equal(l0[:n - 5], l1[:n - 5]) and torch.equal(v0[:n - 5], v1[:n - 5])


@pytest.mark.parametrize("batch", [769, 803, 4096])
def test_tower_one_launch_equals_per_block_launches(batch):
    """hz_tower_x6_blocks (every workgroup carries its 8 states through all
    eight residual blocks in one launch, each block's output written over
    the previous one) gives the bits of eight hz_resblock_x6_bias_act
    launches, with both row tables, a partly filled last workgroup (803), a
    live-row bound inside a workgroup and a NaN tail past the input; the
    input is left unchanged; a batch the per-block path serves is refused
    with -2 (nothing enqueued) and FoldedNet falls back."""
    from hzamd._native import lib
    from hzamd.infer import _resblock_x6, _tower_blocks_x6
    g = torch.Generator().manual_seed(batch)
    torch.manual_seed(batch)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    fnet = FoldedNet(net.cuda())
    cl = torch.channels_last
    x = torch.randn(batch, 128, 5, 7, generator=g).relu()
    buf = torch.full((batch + 9, 128, 5, 7), float("nan"), device="cuda").contiguous(memory_format=cl)
    buf[:batch] = x.cuda()
    xc = buf[:batch]
    x0 = xc.clone()
    live = torch.tensor([batch - 4], dtype=torch.int32, device="cuda")
    try:
        for table in (0, 1):
            assert lib().hz_resblock_x6_set_table(table) == 0
            ref = xc
            for ((_, b1), (_, b2)), (p1, p2) in zip(fnet.blocks, fnet.packed):
                ref = _resblock_x6(ref, p1, b1, p2, b2)
            tw = _tower_blocks_x6(xc, fnet._tw_ptrs, len(fnet.blocks))
            assert tw is not None and torch.equal(tw, ref), table
            part = _tower_blocks_x6(xc, fnet._tw_ptrs, len(fnet.blocks), live)
            assert torch.equal(part[:batch - 4], ref[:batch - 4]), table
            assert torch.equal(xc, x0)
    finally:
        lib().hz_resblock_x6_set_table(1)
    small = torch.zeros(64, 128, 5, 7, device="cuda").contiguous(memory_format=cl)
    assert _tower_blocks_x6(small, fnet._tw_ptrs, len(fnet.blocks)) is None
    # the whole forward with the tower loop on and off: the same bits
    board = (torch.rand(batch, 38, 5, 7, generator=g) > 0.8).float().cuda()
    board[:, 37] = 2.0 / 3.0
    glob = torch.rand(batch, 42, generator=g).cuda()
    prev = fnet.tower_loop
    try:
        fnet.tower_loop = 0
        l0, v0 = fnet(board, glob)
        fnet.tower_loop = 1
        l1, v1 = fnet(board, glob)
    finally:
        fnet.tower_loop = prev
    assert torch.equal(l0, l1) and torch.equal(v0, v1)


_CS4_SCRIPT = """
import sys, torch
sys.path[:0] = [sys.argv[2]]
from hzamd.infer import _conv3x3_x6_act, pack_conv3x3_x6
g = torch.Generator().manual_seed(77)
x = torch.randn(1003, 128, 5, 7, generator=g).relu()
w = torch.randn(128, 128, 3, 3, generator=g) * 0.03
b = torch.randn(128, generator=g) * 0.1
r = torch.randn(1003, 128, 5, 7, generator=g)
cl = torch.channels_last
xc, rc = x.cuda().contiguous(memory_format=cl), r.cuda().contiguous(memory_format=cl)
y = _conv3x3_x6_act(xc, pack_conv3x3_x6(w).cuda(), b.cuda(), rc)
torch.save(y.cpu(), sys.argv[1])
"""


def test_x6_four_state_form_matches_default(tmp_path):
    """The opt-in 4-state tower conv (HZ_X6_CS4=1: two 4-wave workgroups per
    CU, its own tap-class table) gives the default 4-wave form's bits, with a
    partly filled last workgroup (1003 = 250 x 4 + 3); the form is chosen
    once per process, so each runs in a process of its own."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "harmonies-alphazero_amd")
    outs = []
    for flag in ("0", "1"):
        path = str(tmp_path / f"cs4_{flag}.pt")
        env = dict(os.environ, HZ_X6_CS4=flag)
        subprocess.run([sys.executable, "-c", _CS4_SCRIPT, path, pkg], env=env, check=True, timeout=300)
        outs.append(torch.load(path, weights_only=True))
    assert torch.isfinite(outs[0]).all() and torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("batch", [1, 5, 64, 256, 1024])
def test_resident_tower_matches_layered_tower(batch):
    """hz_tower_x6_resident (small batches: the whole tower in one launch,
    activations in LDS) issues each row's products, sums and epilogue in the
    order of the layered one-state x6 convs: logits and values bit-identical,
    with and without a live-row bound."""
    g = torch.Generator().manual_seed(90 + batch)
    torch.manual_seed(batch)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    board = (torch.rand(batch, 38, 5, 7, generator=g) > 0.8).float().cuda()
    board[:, 37] = 1.0 / 3.0
    glob = torch.rand(batch, 42, generator=g).cuda()
    fnet = FoldedNet(net.cuda())
    fnet.resident_max = 1024  # the kernel's own limit (the default dispatch switches earlier)
    assert fnet.resident is not None and batch <= fnet.resident_max
    l0, v0 = fnet(board, glob)
    p0, pv0 = fnet.predict(board, glob)
    split_max = fnet.split_max
    fnet.resident_max = fnet.split_max = 0  # layered
    l1, v1 = fnet(board, glob)
    p1, pv1 = fnet.predict(board, glob)
    assert torch.equal(l0, l1) and torch.equal(v0, v1)
    assert torch.equal(p0, p1) and torch.equal(pv0, pv1)
    fnet.resident_max, fnet.split_max = 1024, split_max
    k = (batch + 1) // 2
    live = torch.tensor([k], dtype=torch.int32, device="cuda")
    l2, v2 = fnet(board, glob, live=live)
    assert torch.equal(l2[:k], l0[:k]) and torch.equal(v2[:k], v0[:k])


def test_resident_tower_reads_nothing_past_its_input():
    """The resident tower on the prefix of a buffer whose tail is NaN."""
    from hzamd.infer import _tower_resident
    batch = 3
    g = torch.Generator().manual_seed(4)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    fnet = FoldedNet(net.cuda())
    x = torch.full((batch + 2, 128, 5, 7), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    x[:batch] = torch.rand(batch, 128, 5, 7, device="cuda")
    y = _tower_resident(x[:batch], *fnet.resident)
    assert bool(torch.isfinite(y).all())


@pytest.mark.parametrize("batch", [1, 3, 10, 11, 32])
def test_split_tower_matches_resident_tower(batch):
    """hz_tower_x6_split (24 one-row-block workgroups per state up to 10
    states, else 8 three-row-block ones; in-launch hand-off of each
    conv's output) == hz_tower_x6_resident bit for bit, no workgroup timed
    out, with a live bound too; repeated launches reuse nothing stale."""
    from hzamd.infer import _tower_resident, _tower_split
    g = torch.Generator().manual_seed(300 + batch)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    fnet = FoldedNet(net.cuda())
    for rep in range(3):
        x = torch.rand(batch, 128, 5, 7, generator=g).cuda().contiguous(memory_format=torch.channels_last)
        want = _tower_resident(x, *fnet.resident)
        sync = []
        got = _tower_split(x, *fnet.resident, sync_out=sync)
        torch.cuda.synchronize()
        assert int(sync[0][32 * 32]) == 0 and not sync[0].any()  # no time-out; counters left zeroed
        assert torch.equal(got, want), rep
    k = (batch + 1) // 2
    live = torch.tensor([k], dtype=torch.int32, device="cuda")
    got = _tower_split(x, *fnet.resident, live)
    assert torch.equal(got[:k], want[:k])


def test_predict_rows_do_not_depend_on_batch_size():
    """A board's priors and value are the same bits whatever batch it is
    evaluated in: every kernel form the batch size selects (split tower <= 32
    rows, resident tower <= 896, one-state and eight-state layered convs,
    k_heads_fc1 <= 2,048 and k_heads_fc above) sums in the same order, so a
    self-play board's search does not depend on how many boards share its
    GPU (config 4 at any boards-per-GPU split)."""
    from hzamd.infer import _heads_fc
    g = torch.Generator().manual_seed(21)
    torch.manual_seed(2)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    n = 4096
    board = (torch.rand(n, 38, 5, 7, generator=g) > 0.8).float()
    board[:, 37] = torch.randint(0, 3, (n, 1, 1), generator=g).float() / 3.0
    glob = torch.rand(n, 42, generator=g)
    fnet = FoldedNet(net.to("cuda"))
    board, glob = board.cuda(), glob.cuda()
    p_full, v_full = fnet.predict(board, glob)
    for s in (1, 7, 10, 11, 32, 33, 300, 768, 769, 896, 897, 1024, 1025, 2048, 2049):
        p, v = fnet.predict(board[:s].contiguous(), glob[:s].contiguous())
        assert torch.equal(p, p_full[:s]) and torch.equal(v, v_full[:s]), s
    # the two head kernels directly: rows of a 2,049-row call (k_heads_fc)
    # equal those of a 300-row call (k_heads_fc1)
    cl = torch.channels_last
    x = torch.randn(2049, 128, 5, 7, generator=g).relu().cuda().contiguous(memory_format=cl)
    gl = torch.rand(2049, 42, generator=g).cuda()
    lo, pr, v = _heads_fc(x, gl, *fnet.heads, fnet.fc, logits=True, probs=True)
    lo1, pr1, v1 = _heads_fc(x[:300].contiguous(memory_format=cl), gl[:300].contiguous(), *fnet.heads, fnet.fc,
                             logits=True, probs=True)
    assert torch.equal(lo1, lo[:300]) and torch.equal(pr1, pr[:300]) and torch.equal(v1, v[:300])


def test_split_tower_refused_when_not_resident_falls_back():
    """hz_tower_x6_split launches only grids the device holds at once
    (CU count x occupancy): with the workgroup limit below a launch's grid it
    enqueues nothing (HZ_E_NOT_RESIDENT) and FoldedNet takes the resident
    tower, bit-identical and finite; never NaN."""
    from hzamd._native import lib
    from hzamd.infer import _tower_split, split_max_batch
    assert split_max_batch(torch.device("cuda", 0)) == 32  # 256 CUs hold every split launch
    g = torch.Generator().manual_seed(77)
    net = HarmoniesNet().eval()
    _randomise_bn(net, g)
    fnet = FoldedNet(net.cuda())
    board = (torch.rand(5, 38, 5, 7, generator=g) > 0.8).float().cuda()
    glob = torch.rand(5, 42, generator=g).cuda()
    p0, v0 = fnet.predict(board, glob)                     # split tower (24 groups per state)
    x = torch.rand(5, 128, 5, 7, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    try:
        assert lib().hz_tower_x6_split_set_limit(5 * 24 - 1) == 0
        assert lib().hz_tower_x6_split_max_batch() == 4
        assert _tower_split(x, *fnet.resident) is None       # refused, nothing enqueued
        p1, v1 = fnet.predict(board, glob)                 # -> resident tower
    finally:
        lib().hz_tower_x6_split_set_limit(0)
    assert torch.equal(p0, p1) and torch.equal(v0, v1) and bool(torch.isfinite(p1).all())


def test_split_tower_timeout_is_loud():
    """A split-tower hand-off that gave up waiting (its state's outputs NaN,
    the timeout word set) raises NativeError at the end of the search or
    predict that used it, instead of letting NaN priors steer PUCT; the word
    is cleared, so the next search runs normally."""
    from hzamd._native import NativeError
    from hzamd.env import BatchedEnv
    from hzamd.infer import SPLIT_TIMEOUT_WORD, _split_sync
    from hzamd.mcts import BatchedMCTS, BatchedPredictor
    torch.manual_seed(0)
    net = HarmoniesNet().cuda().eval()
    ev = BatchedPredictor(net)
    env = BatchedEnv(3, seed_base=5, device="cuda:0")
    env.reset()
    mcts = BatchedMCTS(env, 4)
    v = mcts.search(ev, 2.0)                               # 3 boards: the split tower, no time-out
    assert int(v.sum()) == 3 * (4 - 1)                     # the first simulation expands the root
    sync = _split_sync(torch.device("cuda", 0))
    sync[SPLIT_TIMEOUT_WORD] = 1                            # as a workgroup that gave up would leave it
    with pytest.raises(NativeError, match="timed out"):
        mcts.search(ev, 2.0)
    assert int(sync[SPLIT_TIMEOUT_WORD]) == 0
    v = mcts.search(ev, 2.0)
    assert int(v.sum()) == 3 * (4 - 1)
    mcts.close()
    env.close()
