"""Training phase on the GPU from device-resident examples.

Trainer.execute_training_phase (trainer.py:136-193) copies the replay deque
into a Dataset and iterates a shuffled DataLoader of CPU tensors, calling
ModelManager.train_step per batch (one host sync per batch for the loss
logging).  Here the examples stay on the device: either packed records
(hzamd.distributed format: state words + visit counts + z, 336 B each),
featurised per batch by the HIP encoder, or already-featurised tensors.
Batches follow DataLoader(shuffle=True, drop_last=False) semantics (one
permutation per epoch, last partial batch kept); the losses are accumulated
on the device and read once at the end.
"""
import torch

from . import distributed as hd


class RecordSource:
    """Packed records int64 [M, 42] on the GPU; a batch is decoded with the
    HIP encoder (board f32[B,38,5,7], glob f32[B,42]), pi = N / sum N, z."""

    def __init__(self, records):
        self.records = records

    def __len__(self):
        return self.records.shape[0]

    @property
    def device(self):
        return self.records.device

    def batch(self, idx):
        from .selfplay import encode_states
        states, visits, z, _ = hd.unpack_records(self.records.index_select(0, idx))
        board, glob = encode_states(states)
        return board, glob, hd.pi_of(visits), z.reshape(-1, 1)


def featurize(records):
    """All packed records -> TensorSource (board, glob, pi, z) on their device,
    in one pass of the HIP encoder (≈6 KB per example; the reference's
    default 50,000-example buffer is ≈300 MB)."""
    from .selfplay import encode_states
    states, visits, z, _ = hd.unpack_records(records)
    board, glob = encode_states(states)
    return TensorSource(board, glob, hd.pi_of(visits), z)


class TensorSource:
    """Already-featurised examples (board, glob, pi, z[., 1]) on any device."""

    def __init__(self, board, glob, pi, z):
        self.t = (board, glob, pi, z.reshape(-1, 1))

    def __len__(self):
        return self.t[0].shape[0]

    @property
    def device(self):
        return self.t[0].device

    def batch(self, idx):
        return tuple(x.index_select(0, idx) for x in self.t)


def training_phase(manager, source, epochs, batch_size, generator=None):
    """Returns {"loss", "policy_loss", "value_loss", "batches"} averaged over
    batches, or None when there are fewer examples than one batch (the
    reference skips training then)."""
    m = len(source)
    if m < batch_size:
        return None
    dev = source.device
    acc = torch.zeros(3, dtype=torch.float64, device=manager.device)
    batches = 0
    for _ in range(epochs):
        perm = torch.randperm(m, device=dev, generator=generator)
        for s in range(0, m, batch_size):
            b, g, pi, z = source.batch(perm[s:s + batch_size])
            t, p, v = manager.train_step_async(b, g, pi, z)
            acc += torch.stack([t, p, v]).to(torch.float64)
            batches += 1
    a = (acc / batches).tolist()
    return {"loss": a[0], "policy_loss": a[1], "value_loss": a[2], "batches": batches}
