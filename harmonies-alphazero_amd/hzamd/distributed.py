"""Multi-GPU self-play data exchange (BASELINE config 4).

One process per GPU; rank r owns global boards [r*n, (r+1)*n) seeded by
global id, so no board-level state is ever exchanged during self-play.  Once
per iteration the compact training records of every rank are all-gathered
into every rank's replay buffer (the reference pickles whole games back to
the parent process through a Pool, trainer.py:104-127), and rank 0's updated
weights are broadcast (trainer.py:76-94 ships a state_dict per game).

Record = 42 int64 words (336 B): 6 state words | 143 u16 visit counts |
int8 z | int8 player, packed little-endian.  pi = N / sum(N) is rebuilt on
the receiver exactly as MCTS.py:378-381 computes it.
"""
import torch
import torch.distributed as dist

RECORD_WORDS = 42  # 6 + ceil((143*2 + 2) / 8) = 6 + 36


def pack_records(states, visits, z, player):
    """states int64 [M,6], visits int [M,143] (< 65536), z float/int [M] in
    {-1,0,1}, player int [M] -> int64 [M, 42]."""
    m = states.shape[0]
    dev = states.device
    tail = torch.zeros(m, 36 * 8, dtype=torch.uint8, device=dev)
    v16 = visits.to(torch.int32).clamp(0, 65535)
    tail[:, 0:286:2] = (v16 & 255).to(torch.uint8)
    tail[:, 1:286:2] = (v16 >> 8).to(torch.uint8)
    tail[:, 286] = z.to(torch.int8).view(torch.uint8) if z.dtype != torch.uint8 else z
    tail[:, 287] = player.to(torch.uint8)
    return torch.cat([states.to(torch.int64), tail.view(torch.int64).reshape(m, 36)], dim=1)


def unpack_records(rec):
    m = rec.shape[0]
    states = rec[:, :6].contiguous()
    tail = rec[:, 6:].contiguous().view(torch.uint8).reshape(m, 288)
    visits = tail[:, 0:286:2].to(torch.int32) | (tail[:, 1:286:2].to(torch.int32) << 8)
    z = tail[:, 286].view(torch.int8).to(torch.float32)
    player = tail[:, 287].to(torch.int8)
    return states, visits, z, player


def collective_device(group=None):
    """Where a small control tensor must live for a collective: the CPU under
    gloo, the current GPU under RCCL ("nccl")."""
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def pi_of(visits):
    v = visits.to(torch.float64)
    t = v.sum(1, keepdim=True)
    return torch.where(t > 0, v / t.clamp_min(1), torch.zeros_like(v)).to(torch.float32)


def all_gather_records(rec, group=None):
    """Variable-length all-gather: counts first (int64), then one padded
    all_gather_into_tensor of the packed records; rank order preserved.
    Under RCCL the records move GPU to GPU over xGMI; under gloo (CPU
    rehearsals, which cannot all-gather device tensors) they are staged
    through host memory."""
    world = dist.get_world_size(group)
    dev = rec.device
    cdev = collective_device(group)
    src = rec.to(cdev)
    cnt = torch.tensor([src.shape[0]], dtype=torch.int64, device=cdev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    pad = torch.zeros(mx, RECORD_WORDS, dtype=torch.int64, device=cdev)
    pad[:src.shape[0]] = src
    out = torch.empty(world * mx, RECORD_WORDS, dtype=torch.int64, device=cdev)
    if cdev.type == "cuda" and hasattr(dist, "all_gather_into_tensor"):
        dist.all_gather_into_tensor(out, pad, group=group)
    else:
        dist.all_gather(list(out.split(mx)), pad, group=group)
    return torch.cat([out[r * mx: r * mx + counts[r]] for r in range(world)]).to(dev)


def broadcast_weights(model, src=0, group=None):
    """Rank src's parameters and buffers to every rank: one flat tensor per
    dtype, each in its own dtype (float32 weights travel as 4 B, not
    upcast), so a broadcast moves exactly the state_dict's bytes."""
    tensors = [t for t in model.state_dict().values() if torch.is_tensor(t)]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for ts in by_dtype.values():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                k = t.numel()
                t.copy_(flat[off:off + k].reshape(t.shape))
                off += k


class ReplayBuffer:
    """Device ring of packed records with deque(maxlen) semantics: the newest
    `capacity` records are kept (buffer.py / trainer.py:127 extend())."""

    def __init__(self, capacity, device):
        self.capacity = int(capacity)
        self.data = torch.zeros(self.capacity, RECORD_WORDS, dtype=torch.int64, device=device)
        self.size = 0
        self.head = 0  # next write slot

    def extend(self, rec):
        m = rec.shape[0]
        if m >= self.capacity:
            self.data.copy_(rec[m - self.capacity:])
            self.head, self.size = 0, self.capacity
            return
        end = self.head + m
        if end <= self.capacity:
            self.data[self.head:end] = rec
        else:
            k = self.capacity - self.head
            self.data[self.head:] = rec[:k]
            self.data[:m - k] = rec[k:]
        self.head = end % self.capacity
        self.size = min(self.capacity, self.size + m)

    def records(self):
        """Records oldest -> newest."""
        if self.size < self.capacity:
            return self.data[:self.size]
        return torch.cat([self.data[self.head:], self.data[:self.head]])

    def __len__(self):
        return self.size
