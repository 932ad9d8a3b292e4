"""BatchedMCTS: one PUCT search per board of a BatchedEnv, all boards advancing
in lock-step so that every simulation's leaf evaluations form one PyTorch
batch (the reference evaluates one leaf at a time: MCTS.py:291-352).

    select (HIP) -> gather + encode the leaves that need the network (HIP)
    -> evaluator(board, glob) (PyTorch) -> expand + backup (HIP)

Like the reference, which calls predict only for non-terminal leaves
(MCTS.py:297-341), each simulation's batch holds only the active boards
whose selected leaf is not terminal, gathered on the device: in board order
(hz_mcts_gather_leaves), or, for an evaluator that declares
`row_independent = True` (each output row a function of its input row
alone, whatever its position or the batch size: the folded network, the
stub), in arrival order by the fused expand/backup/select/gather launch.

The evaluator is any callable (board f32[k,38,5,7], glob f32[k,42]) ->
(policy f32[k,143] probabilities, value f32[k]) on the same device, e.g.
`BatchedPredictor(model)` wrapping model.py's AlphaZeroModel the way
ModelManager.predict does (softmax over all 143 logits, model.py:81-110).
An evaluator with `device_rows = True` is instead called as
evaluator(board, glob, rows, count) on the full [n]-row buffers, of which
the first count[0] (a device int32) are live and rows[j] is row j's board:
no host round trip per simulation (BatchedPredictor's HIP kernels take
count as their live-row bound).
"""
import os

import torch

from . import _native as nat
from .env import ACTION_SIZE

MAX_CHILDREN = 69


class BatchedMCTS:
    def __init__(self, env, num_simulations, max_nodes=None, max_depth=192, exact_keys=False):
        self.env = env
        self.n = env.n
        self.device = env.device
        self.num_simulations = int(num_simulations)
        self._graph_cache = None  # (key, captured simulation, network) kept by search(graph=True)
        self._capture_stream = None  # this handle's graph-capture stream (own split-tower counter block)
        self.max_nodes = int(max_nodes or 1 + MAX_CHILDREN * self.num_simulations)
        L = nat.lib()
        self._h = L.hz_mcts_create(self.n, self.max_nodes, int(max_depth), int(bool(exact_keys)),
                                   nat.stream_ptr(self.device))
        if not self._h:
            raise nat.NativeError("hz_mcts_create failed (out of device memory?)")
        d = self.device
        self.board = torch.zeros(self.n, 38, 5, 7, dtype=torch.float32, device=d)
        self.glob = torch.zeros(self.n, 42, dtype=torch.float32, device=d)
        self.visits = torch.zeros(self.n, ACTION_SIZE, dtype=torch.int32, device=d)
        self.counts = torch.zeros(self.n, 4, dtype=torch.int32, device=d)
        self.rows = torch.zeros(self.n, dtype=torch.int32, device=d)
        self.count = torch.zeros(1, dtype=torch.int32, device=d)
        # the second leaf-count buffer of the fused gather (search(): the
        # launch that consumes one count builds the next batch's in the other)
        self.count_b = torch.zeros(1, dtype=torch.int32, device=d)
        self.eval_rows = torch.zeros(1, dtype=torch.int64, device=d)  # leaves evaluated, last search
        self.eval_rows_total = torch.zeros(1, dtype=torch.int64, device=d)  # ... all searches (one add each)
        # k_gather adds each simulation's gathered row count to it (no extra kernel)
        nat.check(L.hz_mcts_set_eval_counter(self._h, nat.ptr(self.eval_rows)), "hz_mcts_set_eval_counter")
        # count_edges: after each search, its edges (one apply_move per legal
        # child of every expanded leaf, MCTS.py:171-177; the skipped self-loop
        # children of :189-194 are not edges) are added on the device to
        # edges_total (two small launches per search, no host read)
        self.count_edges = False
        # the next simulation's select inside each expand/backup launch
        # (search(); HZ_FUSE_SELECT=0 runs them as separate launches)
        self.fuse_select = os.environ.get("HZ_FUSE_SELECT", "1") != "0"
        # ... and the next leaf batch's gather + encode too (each board that
        # needs the network takes a row and encodes its leaf in that launch;
        # HZ_FUSE_GATHER=0 keeps hz_mcts_gather_leaves' separate launch)
        self.fuse_gather = os.environ.get("HZ_FUSE_GATHER", "1") != "0"
        self.edges_total = torch.zeros(1, dtype=torch.int64, device=d)
        # count_path: after each search, the edge levels its simulations
        # walked (the sum of the tree's edge visit counts, hz_mcts_path_edges)
        # are added on the device to path_total (one small launch per search)
        self.count_path = False
        self.path_total = torch.zeros(1, dtype=torch.int64, device=d)
        self._nil_pol = torch.zeros(1, ACTION_SIZE, dtype=torch.float32, device=d)
        self._nil_val = torch.zeros(1, dtype=torch.float32, device=d)

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            nat.lib().hz_mcts_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync(self):
        nat.lib().hz_mcts_set_stream(self._h, nat.stream_ptr(self.device))
        self.env._sync_stream()

    # -- the four device stages ----------------------------------------------
    def begin(self, active=None):
        self._sync()
        nat.check(nat.lib().hz_mcts_begin(self._h, self.env.handle, nat.ptr(active)), "hz_mcts_begin")

    def select(self, cpuct, active=None):
        nat.check(nat.lib().hz_mcts_select(self._h, nat.ptr(active), float(cpuct)), "hz_mcts_select")

    def encode_leaves(self):
        nat.check(nat.lib().hz_mcts_encode_leaves(self._h, nat.ptr(self.board), nat.ptr(self.glob)),
                  "hz_mcts_encode_leaves")
        return self.board, self.glob

    def select_gather(self, cpuct, active=None):
        """select then gather_leaves; one launch when the handle has at most
        32 boards (hz_mcts_select_gather)."""
        nat.check(nat.lib().hz_mcts_select_gather(self._h, nat.ptr(active), float(cpuct), nat.ptr(self.board),
                                                  nat.ptr(self.glob), nat.ptr(self.rows), nat.ptr(self.count)),
                  "hz_mcts_select_gather")
        return self.board, self.glob, self.rows, self.count

    def gather_leaves(self):
        """The leaves that need the network, in board order: (board, glob,
        rows, count) with rows [0, count[0]) live (hz_mcts_gather_leaves)."""
        nat.check(nat.lib().hz_mcts_gather_leaves(self._h, nat.ptr(self.board), nat.ptr(self.glob),
                                                  nat.ptr(self.rows), nat.ptr(self.count)),
                  "hz_mcts_gather_leaves")
        return self.board, self.glob, self.rows, self.count

    def expand_backup(self, policy, value, noise=None, eps=0.25, testing=True, gathered=False):
        if policy.numel() == 0:  # no leaf needed the network (never read, but not NULL)
            policy, value = self._nil_pol, self._nil_val
        policy = policy.to(dtype=torch.float32).contiguous()
        value = value.reshape(-1).to(dtype=torch.float32).contiguous()
        if noise is not None:
            noise = noise.to(device=self.device, dtype=torch.float64).contiguous()
        fn = nat.lib().hz_mcts_expand_backup_gathered if gathered else nat.lib().hz_mcts_expand_backup
        nat.check(fn(self._h, self.env.handle, nat.ptr(policy), nat.ptr(value), nat.ptr(noise), float(eps),
                     int(bool(testing))), "hz_mcts_expand_backup")

    def expand_backup_select(self, policy, value, cpuct, active=None, noise=None, eps=0.25, testing=True):
        """expand_backup(gathered=True), then the next simulation's select in
        the same launch (hz_mcts_expand_backup_select)."""
        if policy.numel() == 0:
            policy, value = self._nil_pol, self._nil_val
        policy = policy.to(dtype=torch.float32).contiguous()
        value = value.reshape(-1).to(dtype=torch.float32).contiguous()
        if noise is not None:
            noise = noise.to(device=self.device, dtype=torch.float64).contiguous()
        nat.check(nat.lib().hz_mcts_expand_backup_select(self._h, self.env.handle, nat.ptr(policy), nat.ptr(value),
                                                         nat.ptr(noise), float(eps), int(bool(testing)),
                                                         nat.ptr(active), float(cpuct)),
                  "hz_mcts_expand_backup_select")

    def expand_backup_select_gather(self, policy, value, cpuct, active, noise, eps, testing, count_out, count_prev,
                                    add_prev):
        """expand_backup_select, then the next leaf batch in the same launch
        (hz_mcts_expand_backup_select_gather): rows in arrival order into
        self.board / self.glob / self.rows, its count into count_out (zero on
        entry); count_prev (this batch's) is zeroed, and first added to the
        eval counter when add_prev."""
        if policy.numel() == 0:
            policy, value = self._nil_pol, self._nil_val
        policy = policy.to(dtype=torch.float32).contiguous()
        value = value.reshape(-1).to(dtype=torch.float32).contiguous()
        if noise is not None:
            noise = noise.to(device=self.device, dtype=torch.float64).contiguous()
        nat.check(nat.lib().hz_mcts_expand_backup_select_gather(
            self._h, self.env.handle, nat.ptr(policy), nat.ptr(value), nat.ptr(noise), float(eps), int(bool(testing)),
            nat.ptr(active), float(cpuct), nat.ptr(self.board), nat.ptr(self.glob), nat.ptr(self.rows),
            nat.ptr(count_out), nat.ptr(count_prev), int(bool(add_prev))), "hz_mcts_expand_backup_select_gather")

    def result(self):
        nat.check(nat.lib().hz_mcts_result(self._h, nat.ptr(self.visits)), "hz_mcts_result")
        return self.visits

    def stats(self):
        nat.check(nat.lib().hz_mcts_stats(self._h, nat.ptr(self.counts)), "hz_mcts_stats")
        return self.counts

    # -- one full search per board -------------------------------------------
    def _device_step(self, evaluator, cpuct, active, noise, eps, testing, max_rows=None):
        """One simulation with a device-row evaluator: no host round trip."""
        board, glob, rows, count = self.select_gather(cpuct, active)  # (adds count to eval_rows)
        if max_rows is not None:  # the live rows are a prefix of at most max_rows
            board, glob = board[:max_rows], glob[:max_rows]
        policy, value = evaluator(board, glob, rows, count)
        self.expand_backup(policy, value, noise, eps, testing, gathered=True)

    def _capture_step(self, evaluator, cpuct, active, eps, testing, max_rows=None):
        """One simulation captured as a HIP graph (select, gather + encode,
        the evaluator's kernels, expand + backup): replaying it costs one
        launch instead of ~60.  Noise is passed as NULL: the kernel reads it
        only when it expands the root, which the first (eager) simulation does
        (hz_mcts.hip k_expand_backup: noisy = leaf == 0 && !testing && noise).

        Replay constraint: the graph bakes in the split tower's counter block
        of its capture stream, and capture streams come from PyTorch's stream
        pool, so two handles may share one block.  Replays of captured
        simulations must therefore run one at a time (search() replays on the
        caller's stream, in order); replaying two handles' graphs
        concurrently on different streams would corrupt the hand-off
        counters."""
        g = torch.cuda.CUDAGraph()
        if self._capture_stream is None:
            self._capture_stream = torch.cuda.Stream(self.device)
        # the split tower's counter block for this stream, zeroed now: created
        # inside the capture, its zero-fill would be a graph node replayed
        # with every simulation (hzamd.infer._split_sync)
        from .infer import _split_sync
        _split_sync(self.device, self._capture_stream)
        try:
            with torch.cuda.graph(g, stream=self._capture_stream):
                self._sync()  # the handles launch on the capture stream
                self._device_step(evaluator, cpuct, active, None, eps, testing, max_rows)
        finally:
            self._sync()  # back on the caller's stream, captured or not
        return g

    def search(self, evaluator, cpuct, active=None, noise=None, eps=0.25, testing=True, sims=None,
               gather=True, graph=False, max_rows=None):
        """get_best_action_and_pi's simulation loop (MCTS.py:288-352) for every
        active board; returns root visit counts int32 [n, 143].

        gather (default): each simulation evaluates only the leaves that need
        the network (module docstring); `eval_rows` counts them on the device.
        gather=False evaluates one row per board (terminal leaves and inactive
        boards included, their results unused), as before.

        graph: simulations 2.. replay one captured HIP graph, for small,
        launch-bound batches (the arena's few dozen boards); taken only with
        a device-row evaluator that declares `capturable = True` (no host
        reads, no allocations outside PyTorch's allocator), as
        BatchedPredictor does for the folded network; otherwise ignored.

        max_rows (host int, device-row evaluators): an upper bound on the
        leaves a simulation can gather (e.g. the number of active boards);
        the evaluator then gets the first max_rows rows of the buffers, so
        its kernels are sized (and the small-batch conv form chosen) by it."""
        if active is not None:
            active = active.to(device=self.device, dtype=torch.uint8).contiguous()
        self.begin(active)
        self.eval_rows.zero_()
        device_rows = bool(getattr(evaluator, "device_rows", False))
        total = self.num_simulations if sims is None else int(sims)
        if graph and gather and device_rows and getattr(evaluator, "capturable", False) and total > 1:
            self._device_step(evaluator, cpuct, active, noise, eps, testing, max_rows)
            # an evaluator with a graph_key (the network object and its weight
            # generation) lets the captured simulation be kept for the next
            # search with the same settings (the drop-in's one search per move);
            # only without an `active` mask, whose tensor the graph would bake in
            gk = getattr(evaluator, "graph_key", None)
            key = None if gk is None or active is not None else (
                id(gk[0]), gk[1], float(cpuct), float(eps), bool(testing), max_rows)
            cached = self._graph_cache
            if key is not None and cached is not None and cached[0] == key:
                g = cached[1]
            else:
                self._graph_cache = None
                g = self._capture_step(evaluator, cpuct, active, eps, testing, max_rows)
                if key is not None:
                    self._graph_cache = (key, g, gk[0])  # holds the network: its id stays unique
            for _ in range(total - 1):
                g.replay()
            return self._finish()
        if gather and total > 1 and self.n > 32 and self.fuse_select:
            # the next simulation's select rides in each expand/backup launch
            # (and, fuse_gather, the gather + encode of its leaf batch: the
            # two count buffers alternate, each zeroed by the launch after the
            # one that filled it, so both are zero between searches)
            # rows in arrival order only for an evaluator that opts in: one
            # that maps rows to boards by position, or whose results depend on
            # a row's place in the batch, keeps the board-order gather
            fuse_gather = self.fuse_gather and bool(getattr(evaluator, "row_independent", False))
            if fuse_gather:
                self.count_b.zero_()  # (defensive: a search cut short may have left it set)
            board, glob, rows, count = self.select_gather(cpuct, active)
            bufs, cur = (self.count, self.count_b), 0
            for s in range(total):
                policy, value = self._evaluate(evaluator, device_rows, board, glob, rows, count, max_rows)
                if s + 1 < total:
                    if fuse_gather:
                        self.expand_backup_select_gather(policy, value, cpuct, active, noise, eps, testing,
                                                         bufs[cur ^ 1], bufs[cur], add_prev=s > 0)
                        cur ^= 1
                        count = bufs[cur]
                    else:
                        self.expand_backup_select(policy, value, cpuct, active, noise, eps, testing)
                        board, glob, rows, count = self.gather_leaves()
                else:
                    self.expand_backup(policy, value, noise, eps, testing, gathered=True)
            if fuse_gather:  # the last batch's count: no gather call added it
                self.eval_rows += count
                count.zero_()
            return self._finish()
        for _ in range(total):
            if not gather:
                self.select(cpuct, active)
                board, glob = self.encode_leaves()
                policy, value = evaluator(board, glob)
                self.eval_rows += self.n
                self.expand_backup(policy, value, noise, eps, testing)
                continue
            board, glob, rows, count = self.select_gather(cpuct, active)  # (adds count to eval_rows)
            policy, value = self._evaluate(evaluator, device_rows, board, glob, rows, count, max_rows)
            self.expand_backup(policy, value, noise, eps, testing, gathered=True)
        return self._finish()

    def _evaluate(self, evaluator, device_rows, board, glob, rows, count, max_rows):
        if device_rows:
            if max_rows is not None:
                board, glob = board[:max_rows], glob[:max_rows]
            return evaluator(board, glob, rows, count)
        k = int(count.item())  # one host read per simulation
        if k:
            return evaluator(board[:k], glob[:k])
        return self._nil_pol, self._nil_val

    def _finish(self):
        """Root visits of the search just run, after making sure no leaf
        evaluation of it went through a timed-out split-tower hand-off (whose
        NaN priors would have steered PUCT silently): NativeError if one did."""
        from .infer import check_split_timeouts
        self.eval_rows_total += self.eval_rows
        if self.count_edges:
            self.edges_total += self.stats()[:, 1].sum(dtype=torch.int64)
        if self.count_path:
            nat.check(nat.lib().hz_mcts_path_edges(self._h, nat.ptr(self.path_total)), "hz_mcts_path_edges")
        visits = self.result()
        check_split_timeouts(self.device)
        return visits


def choose_actions(visits, explore, u):
    """Move choice of get_best_action_and_pi (MCTS.py:394-423) from root visit
    counts (edges are in ascending action order, as the search inserts them):
    explore[b] -> sample proportional to N with the uniform u[b] (first action
    whose cumulative count exceeds u * total); else the first action with the
    most visits.  Returns int64 [n] (-1 when a board has no visits)."""
    v = visits.to(torch.int64)
    total = v.sum(1)
    greedy = torch.argmax(v, dim=1)
    cum = v.cumsum(1)
    target = u.to(torch.float64) * total.to(torch.float64)
    sampled = torch.argmax((target.unsqueeze(1) < cum.to(torch.float64)).to(torch.int32), dim=1)
    act = torch.where(explore.to(torch.bool), sampled, greedy)
    return torch.where(total > 0, act, torch.full_like(act, -1))


def pi_from_visits(visits):
    """pi_target = N / sum(N) in float64, stored as float32 by the trainer
    (MCTS.py:378-381, trainer.py:531)."""
    v = visits.to(torch.float64)
    tot = v.sum(1, keepdim=True)
    return torch.where(tot > 0, v / tot.clamp_min(1), torch.zeros_like(v)).to(torch.float32)


class BatchedPredictor:
    """ModelManager.predict (model.py:81-110) for a whole batch: eval mode,
    no grad, softmax over all 143 logits (illegal moves are not masked).
    Called by BatchedMCTS with the device row count (device_rows): the
    folded net's HIP kernels compute only the live rows."""

    device_rows = True

    def __init__(self, model, dtype=None, fold=True):
        self.model = model
        self.dtype = dtype
        # eval-mode BatchNorm folded into the convs (hzamd.infer): same fp32
        # arithmetic up to rounding, ~3x faster on MI355X at batch 4096
        self.fast = None
        if fold and hasattr(model, "residual_blocks"):
            from .infer import FoldedNet
            self.fast = FoldedNet(model)
        # the folded fp32 path is HIP kernels + PyTorch ops only: it can be
        # captured in a HIP graph (BatchedMCTS.search(graph=True))
        self.capturable = self.fast is not None and (dtype is None or dtype == torch.float32)
        # the folded kernels compute every row on its own, in one summation
        # order whatever the batch (test_predict_rows_do_not_depend_on_batch_size);
        # the PyTorch/MIOpen path makes no such promise
        self.row_independent = self.capturable

    def refresh(self):
        """Re-fold after the model's weights changed."""
        if self.fast is not None:
            self.fast.refresh()

    @torch.no_grad()
    def __call__(self, board, glob, rows=None, count=None):
        self.model.eval()
        low = self.dtype is not None and self.dtype != torch.float32
        # the folded net's HIP kernels are fp32-only; autocast runs the source
        # net (on every row: it has no live-row bound)
        if low:
            with torch.autocast(device_type="cuda", dtype=self.dtype):
                logits, value = self.model(board, glob)
        elif self.fast is not None:
            return self.fast.predict(board, glob, live=count)
        else:
            logits, value = self.model(board, glob)
        return torch.softmax(logits.float(), dim=1), value.float().reshape(-1)


def stub_evaluator(board, glob):
    """Deterministic integer-valued evaluator used by the parity tests; the
    same formula as tests/golden/make_golden.py:stub_predict_np, so the GPU
    search and the reference search see identical priors and values."""
    n0 = torch.round(board[:, 0:18].double().sum((1, 2, 3))).long()
    n1 = torch.round(board[:, 18:36].double().sum((1, 2, 3))).long()
    cp = torch.round(board[:, 36].amax((1, 2))).long()
    ph3 = torch.round(board[:, 37].amax((1, 2)) * 3.0).long()
    pc = torch.round(glob[:, 0:36].double() * 3.0).long()
    w = (pc * torch.arange(1, 37, device=board.device, dtype=torch.int64)).sum(1)
    K = (n0 * 73 + n1 * 151 + ph3 * 7 + cp * 3 + w * 13) % (1 << 31)
    a = torch.arange(ACTION_SIZE, device=board.device, dtype=torch.int64)
    h = (a.unsqueeze(0) * 2654435761 + K.unsqueeze(1) * 40503) % (1 << 32)
    pol = ((h >> 22) + 1).to(torch.float32) / 1024.0
    val = ((K % 255) - 127).to(torch.float64) / 128.0
    return pol, val.to(torch.float32)


stub_evaluator.row_independent = True  # a function of each row alone
