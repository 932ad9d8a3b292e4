"""Leaf-eval inference form of the reference network (model.py:325-394).

`ModelManager.predict` (model.py:81-110) runs the network in eval mode, where
every BatchNorm is a fixed per-channel affine map.  On MI355X the stock graph
spends most of its time in those BatchNorms: MIOpen's spatial inference
kernel takes ~1 ms per call on [4096, 128, 5, 7] (~150 GB/s), 19 calls per
forward, against ~0.4 ms for the 3x3 conv itself.  FoldedNet folds each
BatchNorm into the preceding conv's weights and bias once,

    W' = W * g / sqrt(var + eps),   b' = (b - mean) * g / sqrt(var + eps) + beta,

keeps activations NHWC (channels_last: MIOpen's implicit-GEMM NHWC conv runs
at ~132 TFLOP/s fp32 here, NCHW Winograd at ~82) and runs each 3x3 conv
without bias, followed by one HIP pass (`hz_bias_act`, csrc/hz_net.hip) that
adds the bias, the residual and applies the ReLU in place (PyTorch would make
three passes over the activation: bias add, add_, relu_).  Arithmetic stays
fp32; the results differ from the unfolded graph only by fp32 rounding
(tests/test_infer_gpu.py states the tolerance).  Rebuild (or call refresh())
after the weights change.
"""
import ctypes
import os

import torch
import torch.nn.functional as F
from torch import nn

from ._native import NativeError, lib


def pack_conv3x3(w):
    """[co][ci][3][3] -> [kh*3+kw][ci/16][co][ci%16], the layout hz_conv3x3_bias_act
    reads (one 16-byte B fragment per lane)."""
    co, ci = w.shape[0], w.shape[1]
    return w.permute(2, 3, 1, 0).reshape(9, ci // 16, 16, co).permute(0, 1, 3, 2).contiguous()


def split3_bf16(w):
    """fp32 -> its three bf16 pieces (h, m, l) with h + m + l == w exactly
    (round-to-nearest at each step), stacked on a new leading dim."""
    w = w.float()
    h = w.to(torch.bfloat16)
    r = w - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack((h, m, lo))


def pack_conv3x3_x6(w):
    """[co][ci][3][3] fp32 -> bf16 planes [kh*3+kw][ci/32][plane][co][ci%32],
    the layout hz_conv3x3_x6_bias_act reads (one 16-byte B fragment per lane)."""
    co, ci = w.shape[0], w.shape[1]
    p = split3_bf16(w)                                   # [3][co][ci][3][3]
    p = p.permute(3, 4, 2, 0, 1).reshape(9, ci // 32, 32, 3, co)  # [tap][q][k][plane][co]
    return p.permute(0, 1, 3, 4, 2).contiguous()         # [tap][q][plane][co][k]


def _live_ptr(live):
    """Device int32 scalar bounding the rows the HIP kernels compute (None = all)."""
    if live is None:
        return None
    if not (live.is_cuda and live.dtype == torch.int32):
        raise NativeError("live row count must be a CUDA int32 tensor")
    return live.data_ptr()


def _conv3x3_act(x, wpack, b, res=None, live=None):
    """relu((conv3x3(x) + b) + res) for a 128-channel NHWC activation, one HIP launch."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_conv3x3_bias_act needs a CUDA fp32 channels_last [B,128,5,7] activation")
    if res is not None and (res.shape != x.shape or res.stride() != x.stride()):
        raise NativeError("hz_conv3x3_bias_act: residual layout differs from the activation")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    rc = lib().hz_conv3x3_bias_act(x.data_ptr(), wpack.data_ptr(), b.data_ptr(),
                                   res.data_ptr() if res is not None else None, out.data_ptr(), x.shape[0],
                                   _live_ptr(live), torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_conv3x3_bias_act failed ({rc})")
    return out


def _tower_resident(x, allw, allb, live=None):
    """The whole x6 tower in one HIP launch (hz_tower_x6_resident): allw
    [nconv] pack_conv3x3_x6 layouts, allb [nconv][128]; bit-identical to the
    per-conv _conv3x3_x6_act chain."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_tower_x6_resident needs a CUDA fp32 channels_last [B,128,5,7] activation")
    if not (allw.is_contiguous() and allb.is_contiguous() and allb.shape == (allw.shape[0], 128)):
        raise NativeError("hz_tower_x6_resident: weights/biases of the wrong layout")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    rc = lib().hz_tower_x6_resident(x.data_ptr(), allw.data_ptr(), allb.data_ptr(), out.data_ptr(), allw.shape[0],
                                    x.shape[0], _live_ptr(live), torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_tower_x6_resident failed ({rc})")
    return out


_SPLIT_SYNC = {}  # (device, stream) -> hand-off counter block (zeroed once; every launch leaves it zeroed)
_SPLIT_CAP = {}   # device -> the largest batch hz_tower_x6_split accepts there (occupancy API)
_SPLIT_PENDING = set()  # devices with split-tower launches since the last check_split_timeouts()
SPLIT_TIMEOUT_WORD = 32 * 32


def _split_sync(device, stream=None):
    """The counter block of the split tower's launches on (device, stream):
    a block is used by the launches of one stream only, in stream order
    (launches on two streams sharing one block would corrupt its counters)."""
    stream = torch.cuda.current_stream(device) if stream is None else stream
    key = (device, stream.cuda_stream)
    t = _SPLIT_SYNC.get(key)
    if t is None:
        t = _SPLIT_SYNC[key] = torch.zeros(33 * 32, dtype=torch.int32, device=device)
    return t


def split_max_batch(device):
    """Largest batch the split tower may run on `device` with all its
    workgroups resident at once (hz_tower_x6_split_max_batch: CU count x
    occupancy); larger batches take the resident tower."""
    cap = _SPLIT_CAP.get(device)
    if cap is None:
        with torch.cuda.device(device):
            cap = _SPLIT_CAP[device] = int(lib().hz_tower_x6_split_max_batch())
    return cap


def check_split_timeouts(device=None):
    """Raise NativeError if a split-tower hand-off on `device` (all devices
    when None) gave up waiting since the last check (its state's outputs
    came out NaN); the timeout word is cleared first, so a caller may retry.
    Reads one word per counter block (a device -> host copy: never call it
    inside a graph capture)."""
    if device is not None:
        device = torch.device(device)
        if device.index is None:
            # "cuda" without an index (a ModelManager's training_config device)
            # may name a model on any GPU: check every device with launches
            device = None
    if not _SPLIT_PENDING or (device is not None and device not in _SPLIT_PENDING):
        return
    if device is None:
        _SPLIT_PENDING.clear()
    else:
        _SPLIT_PENDING.discard(device)
    bad = []
    for (dev, _), t in list(_SPLIT_SYNC.items()):
        if device is not None and torch.device(dev) != device:
            continue
        if int(t[SPLIT_TIMEOUT_WORD].item()) != 0:
            t[SPLIT_TIMEOUT_WORD] = 0
            bad.append(str(dev))
    if bad:
        raise NativeError(f"split tower: a hand-off timed out on {', '.join(bad)} (workgroups not co-resident: is "
                          "another process sharing the GPU?); the affected predictions were NaN and are discarded")


def _tower_split(x, allw, allb, live=None, sync_out=None):
    """_tower_resident with 24 or 8 workgroups per state (hz_tower_x6_split,
    batch <= 32): bit-identical, the weights streamed by 8 CUs per state.
    Returns None (nothing enqueued) when the device cannot hold the launch's
    workgroups at once (the caller takes the resident tower).
    sync_out (list, tests): receives the counter/timeout block."""
    B = x.shape[0]
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_tower_x6_split needs a CUDA fp32 channels_last [B,128,5,7] activation")
    if not (allw.is_contiguous() and allb.is_contiguous() and allb.shape == (allw.shape[0], 128)):
        raise NativeError("hz_tower_x6_split: weights/biases of the wrong layout")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    xch = torch.empty(2 * B * 35 * 128, dtype=torch.float32, device=x.device)
    sync = _split_sync(x.device)
    rc = lib().hz_tower_x6_split(x.data_ptr(), allw.data_ptr(), allb.data_ptr(), out.data_ptr(), xch.data_ptr(),
                                 sync.data_ptr(), allw.shape[0], B, _live_ptr(live),
                                 torch.cuda.current_stream(x.device).cuda_stream)
    if rc == -2:  # HZ_E_NOT_RESIDENT: the grid exceeds what the device holds at once
        return None
    if rc != 0:
        raise NativeError(f"hz_tower_x6_split failed ({rc})")
    _SPLIT_PENDING.add(x.device)
    if sync_out is not None:
        sync_out.append(sync)
    return out


def pack_stem(w):
    """Stem weights [128][38][3][3] with the input channels zero-padded to 48,
    packed like pack_conv3x3 (hz_stem3x3_bias_act's layout)."""
    w48 = torch.zeros(w.shape[0], 48, 3, 3, dtype=w.dtype, device=w.device)
    w48[:, :w.shape[1]] = w
    return pack_conv3x3(w48)


def _conv3x3_x6_act(x, wpack6, b, res=None, live=None):
    """_conv3x3_act on the bf16 MFMA with fp32-exact products (bf16x6 split)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_conv3x3_x6_bias_act needs a CUDA fp32 channels_last [B,128,5,7] activation")
    if res is not None and (res.shape != x.shape or res.stride() != x.stride()):
        raise NativeError("hz_conv3x3_x6_bias_act: residual layout differs from the activation")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    rc = lib().hz_conv3x3_x6_bias_act(x.data_ptr(), wpack6.data_ptr(), b.data_ptr(),
                                      res.data_ptr() if res is not None else None, out.data_ptr(), x.shape[0],
                                      _live_ptr(live), torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_conv3x3_x6_bias_act failed ({rc})")
    return out


def _resblock_x6(x, p1, b1, p2, b2, live=None):
    """One residual block (model.py:376-393, BN folded) on the x6 convs:
    relu(conv2(relu(conv1(x) + b1)) + b2 + x) through hz_resblock_x6_bias_act
    (one launch at the 4-wave conv's batch sizes, else the two layered convs;
    bit-identical either way)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_resblock_x6_bias_act needs a CUDA fp32 channels_last [B,128,5,7] activation")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    tmp = torch.empty_like(x, memory_format=torch.channels_last)
    rc = lib().hz_resblock_x6_bias_act(x.data_ptr(), p1.data_ptr(), b1.data_ptr(), p2.data_ptr(), b2.data_ptr(),
                                       out.data_ptr(), tmp.data_ptr(), x.shape[0], _live_ptr(live),
                                       torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_resblock_x6_bias_act failed ({rc})")
    return out


def _tower_blocks_x6(x, ptrs, nblk, live=None):
    """Every residual block of the tower in one launch (hz_tower_x6_blocks:
    each workgroup carries its 8 states through all blocks); None where the
    batch takes the per-block path.  ptrs: the host pointer arrays built by
    FoldedNet.refresh (kept alive there)."""
    out = torch.empty_like(x, memory_format=torch.channels_last)
    tmp = torch.empty_like(x, memory_format=torch.channels_last)
    w1, b1, w2, b2 = ptrs
    rc = lib().hz_tower_x6_blocks(x.data_ptr(), w1, b1, w2, b2, nblk, out.data_ptr(), tmp.data_ptr(), x.shape[0],
                                  _live_ptr(live), torch.cuda.current_stream(x.device).cuda_stream)
    if rc == -2:
        return None
    if rc != 0:
        raise NativeError(f"hz_tower_x6_blocks failed ({rc})")
    return out


def pack_stem_x6(w):
    """Stem weights [128][38][3][3] in hz_stem3x3_x6_bias_act's layout: bf16
    planes [K-step][q][plane][co][32] over 64 input slots.  Slots 0-37 are
    the channels, then channel 37's weights again in slots 38 and 39, where
    the kernel stages the phase channel's bf16 pieces m and l: slot 38 keeps
    the planes (h, m), slot 39 only h, so each piece meets the weight pieces
    of the six-product split.  Chunk 0 (slots 0-31) is packed as
    pack_conv3x3_x6 (K-step = tap); chunk 1 holds only slots 32-39, so its
    K-steps are tap-packed: step s, k = 8 g + j is slot 32 + j at tap
    4 s + g (zero past tap 8), in the entries of K-steps 0-2."""
    co = w.shape[0]
    w64 = torch.zeros(co, 64, 3, 3, dtype=w.dtype, device=w.device)
    w64[:, :w.shape[1]] = w
    w64[:, 38] = w64[:, 39] = w[:, 37]
    pl = split3_bf16(w64)                                # [3][co][64][3][3]
    pl[2, :, 38] = 0                                     # slot 38: planes h, m
    pl[1:, :, 39] = 0                                    # slot 39: plane h
    pl = pl.reshape(3, co, 64, 9)                        # [plane][co][slot][tap]
    p = torch.zeros(9, 2, 3, co, 32, dtype=pl.dtype, device=w.device)
    p[:, 0] = pl[:, :, :32, :].permute(3, 0, 1, 2)       # [tap][plane][co][slot]
    for st in range(3):
        for g in range(4):
            tap = 4 * st + g
            if tap < 9:
                p[st, 1, :, :, 8 * g:8 * g + 8] = pl[:, :, 32:40, tap]
    return p.contiguous()


def _stem_x6_act(board, wpack6, b, live=None):
    """_stem_act on the bf16 MFMA with fp32-exact products (bf16x6 split)."""
    if not (board.is_cuda and board.dtype == torch.float32 and board.shape[1:] == (38, 5, 7)):
        raise NativeError("hz_stem3x3_x6_bias_act needs a CUDA fp32 [B,38,5,7] board")
    board = board.contiguous()
    out = torch.empty(board.shape[0], 128, 5, 7, dtype=torch.float32, device=board.device,
                      memory_format=torch.channels_last)
    rc = lib().hz_stem3x3_x6_bias_act(board.data_ptr(), wpack6.data_ptr(), b.data_ptr(), out.data_ptr(),
                                      board.shape[0], _live_ptr(live),
                                      torch.cuda.current_stream(board.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_stem3x3_x6_bias_act failed ({rc})")
    return out


def _stem_act(board, wpack, b, live=None):
    """relu(conv3x3(board) + b) from the encoder's NCHW board, NHWC out, one HIP launch."""
    if not (board.is_cuda and board.dtype == torch.float32 and board.shape[1:] == (38, 5, 7)):
        raise NativeError("hz_stem3x3_bias_act needs a CUDA fp32 [B,38,5,7] board")
    board = board.contiguous()
    out = torch.empty(board.shape[0], 128, 5, 7, dtype=torch.float32, device=board.device,
                      memory_format=torch.channels_last)
    rc = lib().hz_stem3x3_bias_act(board.data_ptr(), wpack.data_ptr(), b.data_ptr(), out.data_ptr(),
                                   board.shape[0], _live_ptr(live), torch.cuda.current_stream(board.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_stem3x3_bias_act failed ({rc})")
    return out


def _heads(x, glob, hw, hb, live=None):
    """(relu(policy conv1x1) flattened NCHW || glob, relu(value conv1x1) || glob)
    for the default heads (2 + 1 filters on the 5x7 board), one HIP launch."""
    B = x.shape[0]
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_heads needs a CUDA fp32 channels_last [B,128,5,7] activation")
    glob = glob.to(torch.float32).contiguous()
    pcat = torch.empty(B, 112, dtype=torch.float32, device=x.device)
    vcat = torch.empty(B, 77, dtype=torch.float32, device=x.device)
    rc = lib().hz_heads(x.data_ptr(), hw.data_ptr(), hb.data_ptr(), glob.data_ptr(), pcat.data_ptr(),
                        vcat.data_ptr(), B, _live_ptr(live), torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_heads failed ({rc})")
    return pcat, vcat


def _heads_fc(x, glob, hw, hb, fc, live=None, logits=True, probs=False):
    """The whole head in one HIP launch (hz_heads_fc): -> (logits [B,143] or
    None, softmax probabilities [B,143] or None, value [B])."""
    B = x.shape[0]
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1:] == (128, 5, 7)):
        raise NativeError("hz_heads_fc needs a CUDA fp32 channels_last [B,128,5,7] activation")
    glob = glob.to(torch.float32).contiguous()
    lo = torch.empty(B, 143, dtype=torch.float32, device=x.device) if logits else None
    pr = torch.empty(B, 143, dtype=torch.float32, device=x.device) if probs else None
    v = torch.empty(B, dtype=torch.float32, device=x.device)
    ptr = (lambda t: t.data_ptr() if t is not None else None)
    rc = lib().hz_heads_fc(x.data_ptr(), glob.data_ptr(), hw.data_ptr(), hb.data_ptr(),
                           *(t.data_ptr() for t in fc), ptr(lo), ptr(pr), v.data_ptr(), B, _live_ptr(live),
                           torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_heads_fc failed ({rc})")
    return lo, pr, v


def _nhwc(x):
    """channels_last (a no-op for MIOpen's NHWC output; PyTorch's own conv,
    taken with cudnn disabled, returns NCHW)."""
    return x.contiguous(memory_format=torch.channels_last)


def _bias_act(x, b, res=None):
    """x = relu(x + b[c] (+ res)) in place over an NHWC activation."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)):
        raise NativeError("hz_bias_act needs a CUDA fp32 channels_last activation")
    if res is not None and (res.shape != x.shape or res.stride() != x.stride()):
        raise NativeError("hz_bias_act: residual layout differs from the activation")
    ch = x.shape[1]
    rc = lib().hz_bias_act(x.data_ptr(), b.data_ptr(), res.data_ptr() if res is not None else None,
                           x.numel() // ch, ch, torch.cuda.current_stream(x.device).cuda_stream)
    if rc != 0:
        raise NativeError(f"hz_bias_act failed ({rc})")
    return x


def _fold(conv, bn):
    inv = torch.rsqrt(bn.running_var.double() + bn.eps) * bn.weight.double()
    w = (conv.weight.double() * inv.view(-1, 1, 1, 1)).float()
    b0 = conv.bias.double() if conv.bias is not None else torch.zeros_like(inv)
    b = ((b0 - bn.running_mean.double()) * inv + bn.bias.double()).float()
    return w.contiguous(memory_format=torch.channels_last), b.contiguous()


class FoldedNet(nn.Module):
    """Eval-mode HarmoniesNet (or the reference AlphaZeroModel: same module
    names) with BatchNorm folded into the convs; forward(board, glob) ->
    (logits [B,143], value [B,1]) like the source network.

    `epilogue(x, b, res=None)` is the bias [+ skip] + ReLU pass; the default
    is the HIP kernel (CUDA fp32 activations only; no CPU path).  Tests pass
    a plain-torch restatement to check the folding algebra on the CPU."""

    # stem + tower conv kernels: "x6" = bf16 MFMA with fp32-exact products
    # (bf16x6 split: hz_stem3x3_x6_bias_act, hz_conv3x3_x6_bias_act), "f32" =
    # the f32 MFMA (hz_stem3x3_bias_act, hz_conv3x3_bias_act)
    TOWER_MFMA = ("x6", "f32")
    # batches of at most this many boards run the x6 tower as one resident
    # launch (hz_tower_x6_resident; 0 = always layered).  Measured per
    # predict (tools/resident_bench.py): 262 vs 402 us at 1 board, 986 vs
    # 1047 us at 1024; from 1536 the layered eight-state convs win (1066 vs
    # 1488 us: weights shared by 8 states, off-board taps skipped).  Round 5
    # (tools/rows_dist.py, profiles/r05/rows: the eight-state tower in one
    # launch): 957 vs 979 us at 896, 1080 vs 990 us at 1024
    resident_max = int(os.environ.get("HZ_RESIDENT_MAX", "896"))  # (A/B measurements)
    # ... and at most this many with 8 workgroups per state (hz_tower_x6_split)
    split_max = int(os.environ.get("HZ_SPLIT_MAX", "32"))
    # residual blocks above the one-state forms' batch limit: 1 (the default)
    # = all of them in one launch (hz_tower_x6_blocks), 0 = one launch per
    # block (hz_resblock_x6_bias_act); the same bits either way.  Forward at
    # 4,096 rows, interleaved A/B in one process (tools/tower_ab.py): 2.229 vs
    # 2.261 ms and 2.272 vs 2.286 ms on two boxes; self-play 141.8 vs 141.0
    # games/s (profiles/r05/tower)
    tower_loop = int(os.environ.get("HZ_TOWER_LOOP", "1"))

    def __init__(self, net, epilogue=None, native_conv=True, tower="x6", fused_head=True):
        super().__init__()
        if tower not in self.TOWER_MFMA:
            raise ValueError(f"tower must be one of {self.TOWER_MFMA}")
        self.src = net
        self.tower = tower
        self.fused_head = fused_head
        self.epilogue = epilogue or _bias_act
        self.native_conv = native_conv and epilogue is None
        self.refresh()

    @torch.no_grad()
    def refresh(self):
        n = self.src
        # bumped on every re-fold: a captured HIP graph of this network's
        # kernels (BatchedMCTS's cached simulation) is valid for one generation
        self.generation = getattr(self, "generation", -1) + 1
        self.stem = _fold(n.conv, n.bn)
        self.blocks = [(_fold(b.conv1, b.bn1), _fold(b.conv2, b.bn2)) for b in n.residual_blocks]
        # the tower's 128-channel convs run as one fused HIP kernel each
        # (conv + bias + skip + ReLU); other widths use MIOpen + hz_bias_act
        self.stem_packed = None
        if self.native_conv and self.stem[0].shape == (128, 38, 3, 3):
            self.stem_packed = pack_stem_x6(self.stem[0]) if self.tower == "x6" else pack_stem(self.stem[0])
        self.packed = None
        self.resident = None
        if self.native_conv and self.blocks and self.blocks[0][0][0].shape[:2] == (128, 128):
            pk = pack_conv3x3_x6 if self.tower == "x6" else pack_conv3x3
            if self.tower == "x6":
                # all convs back to back (hz_tower_x6_resident); the per-conv
                # packs are views of it
                allw = torch.stack([pk(w) for blk in self.blocks for (w, _) in blk])
                self.packed = [(allw[2 * i], allw[2 * i + 1]) for i in range(len(self.blocks))]
                if allw.shape[0] <= 64:  # the kernel's bias table holds 64 convs
                    self.resident = (allw, torch.stack([b for blk in self.blocks for (_, b) in blk]).contiguous())
                # hz_tower_x6_blocks' host arrays of device pointers (the
                # biases kept contiguous here so the pointers stay valid)
                self._tw_bias = [(b1.contiguous(), b2.contiguous()) for (_, b1), (_, b2) in self.blocks]
                P = ctypes.c_void_p * len(self.blocks)
                self._tw_ptrs = (P(*[p1.data_ptr() for p1, _ in self.packed]),
                                 P(*[b1.data_ptr() for b1, _ in self._tw_bias]),
                                 P(*[p2.data_ptr() for _, p2 in self.packed]),
                                 P(*[b2.data_ptr() for _, b2 in self._tw_bias]))
            else:
                self.packed = [(pk(w1), pk(w2)) for (w1, _), (w2, _) in self.blocks]
        self.pconv = _fold(n.policy_conv, n.policy_bn)
        self.vconv = _fold(n.value_conv, n.value_bn)
        # snapshots like the folded convs: an optimizer step on the source
        # net changes nothing here until refresh()
        self.pfc = (n.policy_fc.weight.detach().clone(), n.policy_fc.bias.detach().clone())
        self.vfc1 = (n.value_fc1.weight.detach().clone(), n.value_fc1.bias.detach().clone())
        self.vfc2 = (n.value_fc2.weight.detach().clone(), n.value_fc2.bias.detach().clone())
        # both heads' 1x1 convs + ReLU + flatten + concat with glob: one HIP pass
        self.heads = None
        if (self.native_conv and self.pconv[0].shape == (2, 128, 1, 1) and self.vconv[0].shape == (1, 128, 1, 1)
                and n.policy_fc.in_features == 112 and n.value_fc1.in_features == 77):
            self.heads = (torch.cat((self.pconv[0].reshape(2, 128), self.vconv[0].reshape(1, 128))).contiguous(),
                          torch.cat((self.pconv[1], self.vconv[1])).contiguous())
        # ... and, for the default linear shapes, the linear layers, softmax and
        # tanh too (hz_heads_fc: weights transposed so its loads coalesce)
        self.fc = None
        if (self.heads is not None and self.fused_head and n.policy_fc.out_features == 143
                and n.value_fc1.out_features == 256 and n.value_fc2.out_features == 1):
            self.fc = (self.pfc[0].t().contiguous(), self.pfc[1].contiguous(), self.vfc1[0].t().contiguous(),
                       self.vfc1[1].contiguous(), self.vfc2[0].reshape(-1).contiguous(),
                       self.vfc2[1].contiguous())

    @torch.no_grad()
    def forward(self, board, glob, live=None):
        """live (CUDA int32 [1], optional): only rows < live[0] are needed;
        the HIP kernels skip the others (their outputs are unspecified)."""
        return self._run(board, glob, live, probs=False)

    @torch.no_grad()
    def predict(self, board, glob, live=None):
        """ModelManager.predict for a batch (model.py:100-104): (softmax over
        all 143 logits [B,143], value [B])."""
        return self._run(board, glob, live, probs=True)

    def _run(self, board, glob, live, probs):
        ep = self.epilogue
        w, b = self.stem
        if self.stem_packed is None or self.packed is None:
            live = None
        if self.stem_packed is not None:  # reads the NCHW board directly
            x = (_stem_x6_act if self.tower == "x6" else _stem_act)(board, self.stem_packed, b, live)
        else:
            x = ep(_nhwc(F.conv2d(board.contiguous(memory_format=torch.channels_last), w, None, padding=1)), b)
        B = board.shape[0]
        xs = None
        if self.resident is not None and B <= min(self.split_max, split_max_batch(board.device)):
            xs = _tower_split(x, *self.resident, live)
        if xs is not None:
            x = xs
        elif self.resident is not None and B <= max(self.resident_max, min(self.split_max, 32)):
            x = _tower_resident(x, *self.resident, live)
        elif self.packed is not None and self.tower == "x6":
            xt = None
            if self.tower_loop and len(self.blocks) <= 16:
                xt = _tower_blocks_x6(x, self._tw_ptrs, len(self.blocks), live)
            if xt is not None:
                x = xt
            else:
                for ((_, b1), (_, b2)), (p1, p2) in zip(self.blocks, self.packed):
                    x = _resblock_x6(x, p1, b1, p2, b2, live)
        elif self.packed is not None:
            for ((_, b1), (_, b2)), (p1, p2) in zip(self.blocks, self.packed):
                y = _conv3x3_act(x, p1, b1, None, live)
                x = _conv3x3_act(y, p2, b2, x, live)
        else:
            for (w1, b1), (w2, b2) in self.blocks:
                y = ep(_nhwc(F.conv2d(x, w1, None, padding=1)), b1)
                x = ep(_nhwc(F.conv2d(y, w2, None, padding=1)), b2, x)
        if self.fc is not None:
            lo, pr, v = _heads_fc(x, glob, *self.heads, self.fc, live=live, logits=not probs, probs=probs)
            return (pr, v) if probs else (lo, v.unsqueeze(1))
        if self.heads is not None:
            pcat, vcat = _heads(x, glob, *self.heads, live=live)
            logits = F.linear(pcat, *self.pfc)
            v = F.linear(vcat, *self.vfc1).relu_()
            v = torch.tanh(F.linear(v, *self.vfc2))
        else:
            w, b = self.pconv
            p = F.conv2d(x, w, b).relu_().flatten(1)               # NCHW order, as model.py flattens
            logits = F.linear(torch.cat((p, glob), 1), *self.pfc)
            w, b = self.vconv
            v = F.conv2d(x, w, b).relu_().flatten(1)
            v = F.linear(torch.cat((v, glob), 1), *self.vfc1).relu_()
            v = torch.tanh(F.linear(v, *self.vfc2))
        return (torch.softmax(logits, 1), v.reshape(-1)) if probs else (logits, v)
