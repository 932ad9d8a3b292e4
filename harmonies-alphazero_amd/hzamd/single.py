"""Single-board bridge for the drop-in facade modules.

The reference mutates Python objects and draws tiles from the process-global
`random` stream (harmonies_engine.py:120-130).  Here every rule evaluation of
a facade call runs on the GPU on a one-board BatchedEnv: the object's state
is packed into the device record, Python's MT19937 state (random.getstate())
is imported as the board's stream, the HIP op runs, and state and stream are
written back (random.setstate) — so a seeded caller sees exactly the draws
the reference would make.
"""
import random

import numpy as np
import torch

from .env import BatchedEnv, unpack_mask
from .state import (SORTED_COORDS, TILE_TYPES, apply_ref_to_object, pack_ref, ref_from_object, unpack_ref,
                    words_to_array)

_BRIDGE = None


def bridge():
    global _BRIDGE
    if _BRIDGE is None:
        _BRIDGE = SingleBoard()
    return _BRIDGE


def action_to_move(a):
    a = int(a)
    if a < 5:
        return a
    t, c = divmod(a - 5, 23)
    return (TILE_TYPES[t], SORTED_COORDS[c])


class SingleBoard:
    def __init__(self, device=None):
        if not torch.cuda.is_available():
            from ._native import NativeError
            raise NativeError("the Harmonies engine runs on the GPU (HIP); no GPU is visible")
        self.device = torch.device(device or "cuda:0")
        self.env = BatchedEnv(1, device=self.device)

    # -- transfer ----------------------------------------------------------------
    def load(self, g, rng=False):
        ref = ref_from_object(g)
        words = torch.from_numpy(np.ascontiguousarray(words_to_array([pack_ref(ref)]).T)).to(self.device)
        if rng:
            _, internal, _ = random.getstate()
            mt = torch.tensor(np.array(internal[:624], dtype=np.uint32).view(np.int32).reshape(1, 624),
                              device=self.device)
            idx = torch.tensor([internal[624]], dtype=torch.int32, device=self.device)
            self.env.import_state(words, mt, idx)
        else:
            self.env.import_state(words)
        return ref

    def store(self, g, rng=False):
        if rng:
            st, mt, idx = self.env.export_state(with_mt=True)
            self._set_python_rng(mt, idx)
        else:
            st = self.env.export_state()
        ref = unpack_ref(st.cpu().numpy()[:, 0])
        apply_ref_to_object(ref, g)
        return ref

    def store_rng(self):
        """Write the board's stream back to Python's `random`, state untouched."""
        _, mt, idx = self.env.export_state(with_mt=True)
        self._set_python_rng(mt, idx)

    @staticmethod
    def _set_python_rng(mt, idx):
        words = mt.cpu().numpy().view(np.uint32)[0].tolist()
        ver, _, gauss = random.getstate()
        random.setstate((ver, tuple(words) + (int(idx.item()),), gauss))

    def legal_current(self):
        """Legal action ids of the board currently loaded."""
        mask = unpack_mask(self.env.legal_mask()[0])[0]
        return torch.nonzero(mask).flatten().tolist()

    # -- operations --------------------------------------------------------------
    def replenish(self, g):
        self.load(g, rng=True)
        self.env.replenish()
        self.store(g, rng=True)

    def end_turn(self, g):
        self.load(g, rng=True)
        self.env.end_turn()
        self.store(g, rng=True)

    def legal_actions(self, g):
        self.load(g)
        return self.legal_current()

    def step(self, g, action):
        """Apply action id in place; returns the HZ_ST_* status (0 = applied)."""
        self.load(g, rng=True)
        status = int(self.env.step(torch.tensor([action], dtype=torch.int16, device=self.device)).item())
        if status == 0:
            self.store(g, rng=True)
        return status

    def score_parts(self, g):
        self.load(g)
        _, parts = self.env.score(parts=True)
        return parts[0].cpu().numpy()  # [2, 5]

    def encode(self, g):
        self.load(g)
        board, glob = self.env.encode()
        return board[0].cpu(), glob[0].cpu()
