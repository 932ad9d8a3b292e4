"""Replay-buffer files.

The reference keeps a `collections.deque(maxlen)` of 4-tuples of CPU float
tensors (board f32[38,5,7], glob f32[42], pi f32[143], z f32[1]) and
pickles it whole (buffer.py:7-48): ≈5.9 KB per example, and loading it runs
the unpickler over an arbitrary file.

  * compact format: the packed device records (hzamd.distributed: 6 state
    words + 143 u16 visit counts + z + player = 336 B per example) in a
    NumPy .npz of plain integer arrays (`records`, `maxlen`, `version`),
    read back with allow_pickle=False;
  * export_reference_pickle: the reference's own format, written exactly as
    buffer.save_buffer does (pickle.HIGHEST_PROTOCOL of the deque), so
    buffer.load_buffer / ReplayBufferDataset read it unchanged.
Reference pickles are not imported (that would unpickle foreign files).
"""
import collections
import os
import pickle

import numpy as np
import torch

from . import distributed as hd

VERSION = 1


def save_compact(records, path, maxlen=None):
    rec = records.detach().to("cpu", torch.int64).numpy()
    if rec.ndim != 2 or rec.shape[1] != hd.RECORD_WORDS:
        raise ValueError(f"records must be int64 [M, {hd.RECORD_WORDS}]")
    with open(path, "wb") as f:
        np.savez(f, records=rec, maxlen=np.int64(-1 if maxlen is None else maxlen), version=np.int64(VERSION))


def load_compact(path, device="cpu"):
    """Returns (records int64 [M, 42] on `device`, maxlen or None)."""
    with np.load(path, allow_pickle=False) as f:
        if int(f["version"]) != VERSION:
            raise ValueError(f"unsupported compact buffer version {int(f['version'])}")
        rec = torch.from_numpy(f["records"]).to(device)
        maxlen = int(f["maxlen"])
    return rec, (None if maxlen < 0 else maxlen)


def to_examples(records, chunk=8192):
    """Packed records -> the reference's example tuples, oldest first (HIP
    encoder for board/glob, pi = N / sum N as MCTS.py:378-381, z f32[1])."""
    from .selfplay import encode_states
    out = []
    for s in range(0, records.shape[0], chunk):
        states, visits, z, _ = hd.unpack_records(records[s:s + chunk])
        board, glob = encode_states(states)
        b, g, p, zz = board.cpu(), glob.cpu(), hd.pi_of(visits).cpu(), z.reshape(-1, 1).cpu()
        out += [(b[i].clone(), g[i].clone(), p[i].clone(), zz[i].clone()) for i in range(b.shape[0])]
    return out


def export_reference_pickle(records, path, maxlen):
    """buffer.save_buffer's file for these records (a deque(maxlen) of
    example tuples; the newest `maxlen` are kept, as deque.extend does)."""
    buf = collections.deque(to_examples(records), maxlen=maxlen)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        pickle.dump(buf, f, pickle.HIGHEST_PROTOCOL)
    return len(buf)
