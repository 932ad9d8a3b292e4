"""Device-resident training phase and the compact buffer format, on CPU:
training_phase reproduces a DataLoader(shuffle)-style loop of
ModelManager.train_step calls (same permutation, same batches, last
partial batch kept) and the compact .npz round-trips packed records."""
import numpy as np
import torch

from hzamd import distributed as hd
from hzamd.buffer_io import load_compact, save_compact
from hzamd.manager import ModelManager
from hzamd.train import TensorSource, training_phase
from test_manager_cpu import MODEL_CFG, TRAIN_CFG


def test_training_phase_matches_manual_loop():
    g = torch.Generator().manual_seed(7)
    M = 10
    board = (torch.rand(M, 38, 5, 7, generator=g) > 0.8).float()
    glob = torch.rand(M, 42, generator=g)
    pi = torch.softmax(torch.rand(M, 143, generator=g), 1)
    z = torch.randint(-1, 2, (M,), generator=g).float()
    torch.manual_seed(0)
    a = ModelManager(MODEL_CFG, TRAIN_CFG)
    torch.manual_seed(0)
    b = ModelManager(MODEL_CFG, TRAIN_CFG)
    res = training_phase(a, TensorSource(board, glob, pi, z), epochs=2, batch_size=4,
                         generator=torch.Generator().manual_seed(5))
    gen = torch.Generator().manual_seed(5)
    losses = []
    for _ in range(2):
        perm = torch.randperm(M, generator=gen)
        for s in range(0, M, 4):
            i = perm[s:s + 4]
            losses.append(b.train_step(board[i], glob[i], pi[i], z[i].reshape(-1, 1)))
    assert res["batches"] == 6 == len(losses)
    assert abs(res["loss"] - np.mean([l[0] for l in losses])) <= 1e-6
    for k, v in a.model.state_dict().items():
        assert torch.equal(b.model.state_dict()[k], v), k
    assert training_phase(a, TensorSource(board[:3], glob[:3], pi[:3], z[:3]), 1, 4) is None


def test_compact_buffer_round_trip(tmp_path):
    g = torch.Generator().manual_seed(1)
    M = 50
    states = torch.randint(0, 1 << 62, (M, 6), generator=g)
    visits = torch.randint(0, 400, (M, 143), generator=g, dtype=torch.int32)
    z = torch.randint(-1, 2, (M,), generator=g)
    player = torch.randint(0, 2, (M,), generator=g)
    rec = hd.pack_records(states, visits, z, player)
    save_compact(rec, tmp_path / "b.npz", maxlen=50000)
    back, maxlen = load_compact(tmp_path / "b.npz")
    assert maxlen == 50000 and torch.equal(back, rec)
    s2, v2, z2, p2 = hd.unpack_records(back)
    assert torch.equal(s2, states) and torch.equal(v2, visits) and torch.equal(z2, z.float())
