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


class GraphedStep:
    """ModelManager.train_step_async for full batches of one size, replayed
    as a captured HIP graph: a batch of 64 is ~150 small launches (forward,
    backward, Adam), launch-bound at ~4 ms; a replay is one launch after the
    copy into the static inputs.  The first `warmup` batches train eagerly
    on a side stream (PyTorch's capture recipe: the optimizer state and the
    allocator settle); the capture itself executes nothing, and the batch it
    was recorded with is then trained by the first replay, so every batch is
    trained exactly once.  Capture once per phase: the learning rate is
    read when the graph is recorded (the scheduler steps between phases)."""

    def __init__(self, manager, warmup=3):
        self.m = manager
        self.warmup = warmup
        self.graph = None

    def step(self, board, glob, pi, z):
        m = self.m
        if self.warmup > 0:
            self.warmup -= 1
            cur = torch.cuda.current_stream(m.device)
            side = torch.cuda.Stream(m.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                out = m.train_step_async(board, glob, pi, z)
            cur.wait_stream(side)
            return out
        if self.graph is None:
            self.static = [x.to(m.device).clone() for x in (board, glob, pi, z)]
            m.model.train()
            m.optimizer.zero_grad(set_to_none=True)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                total, pl, vl = m.losses(*self.static)
                total.backward()
                m.optimizer.step()
            self.out = (total.detach(), pl.detach(), vl.detach())
        else:
            for dst, x in zip(self.static, (board, glob, pi, z)):
                dst.copy_(x)
        self.graph.replay()
        # the replayed optimizer step bumps no version counter: tell the
        # manager its folded inference copy is stale
        if hasattr(m, "invalidate_fold"):
            m.invalidate_fold()
        return self.out


def graph_capable(manager):
    """Training steps can be graphed: a CUDA model under capturable Adam or
    SGD (no host-side optimizer state)."""
    opt = manager.optimizer
    if manager.device.type != "cuda":
        return False
    if isinstance(opt, torch.optim.Adam):
        return all(g.get("capturable", False) for g in opt.param_groups)
    return isinstance(opt, torch.optim.SGD)


def training_phase(manager, source, epochs, batch_size, generator=None, graph=None):
    """Returns {"loss", "policy_loss", "value_loss", "batches"} averaged over
    batches, or None when there are fewer examples than one batch (the
    reference skips training then).  graph (default: when graph_capable):
    full batches replay one captured training step (GraphedStep); a last
    partial batch runs eagerly."""
    m = len(source)
    if m < batch_size:
        return None
    dev = source.device
    acc = torch.zeros(3, dtype=torch.float64, device=manager.device)
    batches = 0
    graphed = GraphedStep(manager) if (graph_capable(manager) if graph is None else graph) else None
    for _ in range(epochs):
        perm = torch.randperm(m, device=dev, generator=generator)
        for s in range(0, m, batch_size):
            b, g, pi, z = source.batch(perm[s:s + batch_size])
            if graphed is not None and b.shape[0] == batch_size:
                t, p, v = graphed.step(b, g, pi, z)
            else:
                t, p, v = manager.train_step_async(b, g, pi, z)
            acc += torch.stack([t, p, v]).to(torch.float64)
            batches += 1
    a = (acc / batches).tolist()
    return {"loss": a[0], "policy_loss": a[1], "value_loss": a[2], "batches": batches}
