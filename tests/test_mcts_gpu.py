"""GPU parity of the batched HIP MCTS (hzamd.mcts) against the reference's
own get_best_action_and_pi (golden fixtures, canonical move order, stub
evaluator) and against the C oracle at full batch size.  Visit counts, the
chosen move, tree sizes and the RNG stream must match exactly."""
import os
from collections import defaultdict

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN
from hzamd.state import pack_ref, unpack_ref, words_to_array

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def make_env(refs, mt_seeds):
    from hzamd.env import BatchedEnv
    env = BatchedEnv(len(refs), device=DEV)
    words = words_to_array([pack_ref(v) for v in refs])
    mts = np.zeros((len(refs), 624), np.uint32)
    idx = np.zeros(len(refs), np.int32)
    for i, s in enumerate(mt_seeds):
        w, k = oracle.mt_seed(int(s)).words()
        mts[i], idx[i] = w, k
    env.import_state(torch.from_numpy(np.ascontiguousarray(words.T)),
                     torch.from_numpy(mts.view(np.int32)), torch.from_numpy(idx))
    return env


def test_mcts_matches_reference_fixtures():
    from hzamd.mcts import BatchedMCTS, choose_actions, stub_evaluator
    f = load("mcts.npz")
    groups = defaultdict(list)
    for k in range(len(f["sims"])):
        groups[(int(f["sims"][k]), float(f["cpuct"][k]), int(f["testing"][k]), float(f["eps"][k]))].append(k)
    checked = 0
    for (sims, cpuct, testing, eps), ks in groups.items():
        env = make_env(f["state"][ks], f["mt_seed"][ks])
        mcts = BatchedMCTS(env, sims)
        noise = torch.from_numpy(np.ascontiguousarray(f["noise"][ks][:, :69]))
        visits = mcts.search(stub_evaluator, cpuct, noise=noise, eps=eps, testing=bool(testing))
        explore = torch.tensor([(not testing) and f["ply"][k] < f["tau0"][k] for k in ks])
        u = torch.tensor([f["u"][k] for k in ks], dtype=torch.float64)
        act = choose_actions(visits.cpu(), explore, u).numpy()
        counts = mcts.stats().cpu().numpy()
        v = visits.cpu().numpy()
        _, mt, mti = env.export_state(with_mt=True)
        mt = mt.cpu().numpy().view(np.uint32)
        mti = mti.cpu().numpy()
        for j, k in enumerate(ks):
            assert (v[j] == f["visits"][k]).all(), (k, v[j][v[j] > 0], f["visits"][k][f["visits"][k] > 0])
            assert act[j] == f["action"][k], k
            assert counts[j, 0] == f["n_nodes"][k] and counts[j, 1] == f["n_edges"][k], k
            assert counts[j, 3] == 0
            m = oracle.mt_from_words(mt[j], mti[j])
            assert oracle.mt_next32(m) == f["next_word"][k], k
            checked += 1
        mcts.close()
        env.close()
    assert checked == len(f["sims"])


def test_mcts_4096_boards_vs_oracle():
    """Full batch: 4096 boards at assorted game positions, 24 simulations,
    testing mode, stub evaluator; every board is searched by the C oracle."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, base, sims, cpuct = 4096, 500, 24, 2.0
    env = BatchedEnv(n, seed_base=base, device=DEV)
    env.reset()
    # advance board b by (b % 61) rule plies to spread positions over the game
    plies = torch.arange(n, device=DEV) % 61
    for p in range(61):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        act = torch.where(plies > p, act, torch.full_like(act, -1))
        env.step(act)
    st0, mt0, idx0 = env.export_state(with_mt=True)
    st0, mt0, idx0 = st0.cpu().numpy(), mt0.cpu().numpy().view(np.uint32), idx0.cpu().numpy()
    active = torch.from_numpy(np.array([not oracle.is_game_over(unpack_ref(st0[:, b])) for b in range(n)]))
    mcts = BatchedMCTS(env, sims)
    visits = mcts.search(stub_evaluator, cpuct, active=active).cpu().numpy()
    counts = mcts.stats().cpu().numpy()
    _, mt1, idx1 = env.export_state(with_mt=True)
    mt1, idx1 = mt1.cpu().numpy().view(np.uint32), idx1.cpu().numpy()
    for b in range(n):
        if not active[b]:
            assert visits[b].sum() == 0
            continue
        m = oracle.mt_from_words(mt0[b], idx0[b])
        a, ov, nn, ne = oracle.mcts_search(unpack_ref(st0[:, b]), m, sims, cpuct, testing=True)
        assert (visits[b] == ov).all(), b
        assert (counts[b, 0], counts[b, 1]) == (nn, ne), b
        m2 = oracle.mt_from_words(mt1[b], idx1[b])
        assert oracle.mt_next32(m2) == oracle.mt_next32(m), b


def test_sibling_dedup_table_matches_serial_walk():
    """k_expand_backup's sibling dedup: the LDS hash table (default) and the
    serial walk it falls back to on a hash collision (forced on every
    expansion by hz_mcts_set_dedup_walk) give the same trees, and both the
    oracle's, on 1024 boards spread over the game (sibling duplicates: two
    equal tiles in hand placed on the same hex)."""
    import hzamd._native as nat
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, sims, cpuct = 1024, 24, 2.0
    env = BatchedEnv(n, seed_base=900, device=DEV)
    env.reset()
    plies = torch.arange(n, device=DEV) % 53
    for p in range(53):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
    st0, mt0, idx0 = env.export_state(with_mt=True)
    active = torch.from_numpy(np.array([not oracle.is_game_over(unpack_ref(st0[:, b].cpu().numpy()))
                                        for b in range(n)]))
    runs = []
    for walk in (0, 1):
        env.import_state(st0, mt0, idx0)
        mcts = BatchedMCTS(env, sims)
        assert nat.lib().hz_mcts_set_dedup_walk(mcts._h, walk) == 0
        v = mcts.search(stub_evaluator, cpuct, active=active).cpu().numpy()
        runs.append((v, mcts.stats().cpu().numpy()))
        mcts.close()
    assert (runs[0][0] == runs[1][0]).all() and (runs[0][1] == runs[1][1]).all()
    st0, mt0, idx0 = st0.cpu().numpy(), mt0.cpu().numpy().view(np.uint32), idx0.cpu().numpy()
    for b in range(0, n, 8):
        if not active[b]:
            continue
        m = oracle.mt_from_words(mt0[b], idx0[b])
        _, ov, nn, ne = oracle.mcts_search(unpack_ref(st0[:, b]), m, sims, cpuct, testing=True)
        assert (runs[0][0][b] == ov).all() and (runs[0][1][b, 0], runs[0][1][b, 1]) == (nn, ne), b


def test_mcts_exact_keys_mode():
    """exact_keys=1 keys transpositions by the true canonical tuple."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, sims = 128, 16
    env = BatchedEnv(n, seed_base=77, device=DEV)
    env.reset()
    st0, mt0, idx0 = env.export_state(with_mt=True)
    st0, mt0, idx0 = st0.cpu().numpy(), mt0.cpu().numpy().view(np.uint32), idx0.cpu().numpy()
    mcts = BatchedMCTS(env, sims, exact_keys=True)
    visits = mcts.search(stub_evaluator, 1.5).cpu().numpy()
    counts = mcts.stats().cpu().numpy()
    for b in range(n):
        m = oracle.mt_from_words(mt0[b], idx0[b])
        _, ov, nn, ne = oracle.mcts_search(unpack_ref(st0[:, b]), m, sims, 1.5, testing=True, exact_keys=True)
        assert (visits[b] == ov).all() and (counts[b, 0], counts[b, 1]) == (nn, ne), b


def test_mcts_gathered_leaf_batch_matches_full_batch():
    """Leaf batches gathered on the device (active boards whose leaf is not
    terminal, MCTS.py:297-341) give every board the same search as the
    one-row-per-board batch: identical visit counts and node/edge counts with
    the stub evaluator, whether the evaluator takes the host-sliced batch or
    the device row count; and fewer rows reach the evaluator.  30 % of the
    boards inactive, positions late in the game so that terminal leaves occur."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, base, sims, cpuct = 700, 900, 16, 1.5
    g = torch.Generator().manual_seed(7)
    active = (torch.rand(n, generator=g) > 0.3).to(DEV)
    plies = 40 + torch.arange(n, device=DEV) % 24

    class DeviceRows:
        device_rows = True
        row_independent = True

        def __init__(self):
            self.calls = []
            self.shapes = []

        def __call__(self, board, glob, rows, count):
            k = int(count.item())
            self.calls.append(k)
            self.shapes.append(board.shape[0])
            assert rows[:k].unique().numel() == k           # one row per board (arrival order when fused)
            pol = torch.full((n, 143), float("nan"), device=DEV)
            val = torch.full((n,), float("nan"), device=DEV)
            p, v = stub_evaluator(board[:k], glob[:k])
            pol[:k], val[:k] = p, v
            return pol, val

    out = []
    for mode in ("full", "host", "device", "device_max"):
        env = BatchedEnv(n, seed_base=base, device=DEV)
        env.reset()
        for p in range(64):
            mask, count = env.legal_mask()
            act = env.rule_actions(mask, count)
            env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
        act_b = active & ~env.done()
        mcts = BatchedMCTS(env, sims)
        calls = []

        def ev(board, glob):
            calls.append(board.shape[0])
            return stub_evaluator(board, glob)
        dr = DeviceRows()
        k_act = int(act_b.sum())
        v = mcts.search(dr if mode.startswith("device") else ev, cpuct, active=act_b, gather=mode != "full",
                        max_rows=k_act if mode == "device_max" else None).clone()
        if mode == "device_max":  # the evaluator saw buffers of the active-board count
            assert dr.shapes == [k_act] * sims
        out.append((v.cpu(), mcts.stats().clone().cpu(), dr.calls if mode.startswith("device") else calls,
                    int(mcts.eval_rows.item())))
        mcts.close()
        env.close()
    (v0, c0, calls0, r0), (v1, c1, calls1, r1), (v2, c2, calls2, r2), (v3, c3, calls3, r3) = out
    assert torch.equal(v0, v1) and torch.equal(v0, v2) and torch.equal(v0, v3)
    assert torch.equal(c0[:, :2], c1[:, :2]) and torch.equal(c0[:, :2], c2[:, :2])
    assert torch.equal(c0[:, :2], c3[:, :2]) and calls3 == calls2 and r3 == r2
    assert calls0 == [n] * sims and r0 == n * sims
    assert sum(calls1) == r1 == r2 == sum(calls2)
    k = int(act_b.sum())
    assert max(calls1) <= k and r1 < k * sims        # terminal leaves were skipped
    assert bool((v1[~act_b.cpu()] == 0).all())


def test_fused_select_equals_separate_launches():
    """search() runs each simulation's select inside the previous one's
    expand/backup launch above 32 boards, and (fuse_gather) the next leaf
    batch's gather + encode there too, rows in arrival order.  Against
    separate launches (select, gather + encode in board order): identical
    visit counts, tree sizes, leaf rows per simulation, next CPython word of
    every board, and every simulation's batch is the same set of boards with
    bit-identical encoded rows (self-play settings, mid-game positions, 20 %
    of the boards inactive)."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    from hzamd.selfplay import NoiseSource
    n, base, sims = 1000, 321, 24
    g = torch.Generator().manual_seed(3)
    active = (torch.rand(n, generator=g) > 0.2).to(DEV)
    out = []
    for fuse, fuse_gather in ((True, True), (True, False), (False, False)):
        env = BatchedEnv(n, seed_base=base, device=DEV)
        env.reset()
        for p in range(20 + (base % 7)):
            mask, count = env.legal_mask()
            env.step(env.rule_actions(mask, count))
        act_b = active & ~env.done()
        _, count = env.legal_mask()
        noise, _ = NoiseSource(base, DEV).draw(5, count, 0.4)
        mcts = BatchedMCTS(env, sims)
        mcts.fuse_select = fuse
        mcts.fuse_gather = fuse_gather
        rows, batches = [], []

        class DeviceRows:
            device_rows = True
            row_independent = True

            def __call__(self, board, glob, r, count):
                rows.append(count.clone())
                k = int(count.item())
                order = torch.argsort(r[:k])
                batches.append((r[:k][order].clone(), board[:k][order].clone(), glob[:k][order].clone()))
                return stub_evaluator(board, glob)
        v = mcts.search(DeviceRows(), 2.0, active=act_b, noise=noise, eps=0.25, testing=False).clone()
        st, mt, idx = env.export_state(with_mt=True)
        out.append((v.cpu(), mcts.stats().clone().cpu(), torch.cat(rows).cpu(), mt.cpu(), idx.cpu(),
                    mcts.eval_rows.clone().cpu(), batches))
        assert int(mcts.count.item()) == 0 or not fuse_gather
        mcts.close()
        env.close()
    for x in out[1:]:
        for a, b in zip(out[0][:6], x[:6]):
            assert torch.equal(a, b)
        assert len(out[0][6]) == len(x[6]) == sims
        for ba, bb in zip(out[0][6], x[6]):
            for ta, tb in zip(ba, bb):
                assert torch.equal(ta, tb)
    assert int(out[0][5]) == int(out[0][2].sum())  # the eval counter holds every batch's rows


def test_fused_gather_only_for_row_independent_evaluators():
    """The fused gather hands rows over in arrival order, so search() takes it
    only for an evaluator that declares row_independent; any other evaluator
    (device rows or host rows) gets every batch in ascending board order, and
    both searches give the same visits."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, sims = 300, 12
    out = []
    for indep in (False, True):
        env = BatchedEnv(n, seed_base=515, device=DEV)
        env.reset()
        for p in range(18):
            mask, count = env.legal_mask()
            env.step(env.rule_actions(mask, count))
        mcts = BatchedMCTS(env, sims)
        assert mcts.fuse_select and mcts.fuse_gather
        ordered = []

        class DeviceRows:
            device_rows = True
            row_independent = indep

            def __call__(self, board, glob, r, count):
                k = int(count.item())
                ordered.append(bool((r[1:k] > r[:k - 1]).all()) if k > 1 else True)
                return stub_evaluator(board, glob)
        v = mcts.search(DeviceRows(), 2.0, testing=True).clone()
        out.append((v.cpu(), ordered))
        mcts.close()
        env.close()
    (v0, ord0), (v1, ord1) = out
    assert torch.equal(v0, v1)
    assert all(ord0) and len(ord0) == sims
    assert not all(ord1)  # arrival order somewhere (the fused gather ran)


def test_mcts_4096_boards_200_sims_selfplay_config_vs_oracle():
    """BASELINE config 3's search at full size: 4096 boards at assorted game
    positions, 200 simulations, self-play settings (testing=False: the root
    Dirichlet mix with eps 0.25, cpuct 2), stub evaluator, gathered leaf
    batches on the device; every board's visit counts, tree sizes and next
    MT word checked against the C oracle's search (run on the host cores)."""
    from concurrent.futures import ThreadPoolExecutor
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator

    class DeviceRows:  # the stub on the device-row protocol (no host read per simulation)
        device_rows = True
        row_independent = True

        def __call__(self, board, glob, rows, count):
            return stub_evaluator(board, glob)

    n, base, sims, cpuct, eps = 4096, 1300, 200, 2.0, 0.25
    env = BatchedEnv(n, seed_base=base, device=DEV)
    env.reset()
    plies = torch.arange(n, device=DEV) % 63
    for p in range(63):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
    st0, mt0, idx0 = env.export_state(with_mt=True)
    st0, mt0, idx0 = st0.cpu().numpy(), mt0.cpu().numpy().view(np.uint32), idx0.cpu().numpy()
    active = ~env.done()
    torch.manual_seed(4)
    noise = torch.distributions.Dirichlet(torch.full((69,), 0.4)).sample((n,)).double()
    mcts = BatchedMCTS(env, sims)
    visits = mcts.search(DeviceRows(), cpuct, active=active, noise=noise, eps=eps, testing=False,
                         max_rows=int(active.sum())).cpu().numpy()
    counts = mcts.stats().cpu().numpy()
    _, mt1, idx1 = env.export_state(with_mt=True)
    mt1, idx1 = mt1.cpu().numpy().view(np.uint32), idx1.cpu().numpy()
    act_np = active.cpu().numpy()
    nz = noise.numpy()

    def one(b):
        m = oracle.mt_from_words(mt0[b], idx0[b])
        _, ov, nn, ne = oracle.mcts_search(unpack_ref(st0[:, b]), m, sims, cpuct, eps=eps, testing=False,
                                           noise=np.concatenate([nz[b], np.zeros(143 - 69)]))
        return ov, nn, ne, oracle.mt_next32(m)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, [b for b in range(n) if act_np[b]]))
    k = 0
    for b in range(n):
        if not act_np[b]:
            assert visits[b].sum() == 0
            continue
        ov, nn, ne, nxt = res[k]
        k += 1
        assert (visits[b] == ov).all(), b
        assert (counts[b, 0], counts[b, 1]) == (nn, ne), b
        assert oracle.mt_next32(oracle.mt_from_words(mt1[b], idx1[b])) == nxt, b
    assert k > 3000
    mcts.close()
    env.close()


@pytest.mark.parametrize("n", [1, 7, 32, 33])
def test_fused_select_gather_matches_separate_launches(n):
    """hz_mcts_select_gather (one launch of select + gather + encode up to 32
    boards) leaves the same leaves, gathered rows, slots, count and encoded
    tensors as hz_mcts_select + hz_mcts_gather_leaves, after a few
    simulations of tree growth with some boards inactive and some terminal."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    env = BatchedEnv(n, seed_base=600, device=DEV)
    env.reset()
    mcts = BatchedMCTS(env, 16)
    active = torch.ones(n, dtype=torch.uint8, device=DEV)
    active[::5] = 0 if n > 1 else 1
    mcts.search(stub_evaluator, 2.0, active=active, sims=6)   # grow the trees (eager, host-row evaluator)
    b1, g1, r1, c1 = (t.clone() for t in mcts.select_gather(2.0, active))
    mcts.board.zero_()
    mcts.glob.zero_()
    mcts.select(2.0, active)
    b2, g2, r2, c2 = mcts.gather_leaves()
    k = int(c1.item())
    assert int(c2.item()) == k and k > 0
    assert torch.equal(r1[:k], r2[:k])
    assert torch.equal(b1[:k], b2[:k]) and torch.equal(g1[:k], g2[:k])
    mcts.close()
    env.close()


def test_gather_encode_equals_layered_gather():
    """hz_mcts_gather_leaves as one k_gather_encode launch (the default) and
    as k_gather + the encoder launches (hz_mcts_set_gather_encode(h, 0)):
    identical rows, count and encoded board/glob tensors, on a partial block
    (1000 boards, 20 % inactive, grown trees with terminal leaves), and
    identical visit counts after a whole search with each form (expand reads
    each board's slot: a wrong slot changes the visits)."""
    import hzamd._native as nat
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n = 1000
    g = torch.Generator().manual_seed(11)
    active = (torch.rand(n, generator=g) > 0.2).to(torch.uint8).to(DEV)
    out = []
    for mode in (1, 0):
        env = BatchedEnv(n, seed_base=77, device=DEV)
        env.reset()
        for p in range(30):
            mask, count = env.legal_mask()
            env.step(env.rule_actions(mask, count))
        mcts = BatchedMCTS(env, 24)
        assert nat.lib().hz_mcts_set_gather_encode(mcts._h, mode) == 0
        v = mcts.search(stub_evaluator, 2.0, active=active, sims=12).clone()
        mcts.board.fill_(float("nan"))
        mcts.glob.fill_(float("nan"))
        mcts.select(2.0, active)
        b, gl, r, c = (t.clone() for t in mcts.gather_leaves())
        k = int(c.item())
        torch.cuda.synchronize()
        out.append((v.cpu(), k, r[:k].cpu(), b[:k].cpu(), gl[:k].cpu()))
        mcts.close()
        env.close()
    (v1, k1, r1, b1, g1), (v0, k0, r0, b0, g0) = out
    assert k1 == k0 and k1 > 0
    assert torch.equal(v1, v0) and torch.equal(r1, r0)
    assert torch.equal(b1, b0) and torch.equal(g1, g0)


def test_path_edges_counts_walked_levels():
    """hz_mcts_path_edges adds the sum of the trees' edge visit counts: every
    simulation after the first (which expands the root) walks at least one
    edge, the second exactly one; so after 2 simulations the sum is the
    number of active boards, and after S it lies in [S - 1, (S - 1) * depth]
    per board with root visits summing to S - 1."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n = 200
    env = BatchedEnv(n, seed_base=818, device=DEV)
    env.reset()
    mcts = BatchedMCTS(env, 24)
    mcts.count_path = True
    mcts.search(stub_evaluator, 2.0, sims=2)
    assert int(mcts.path_total.item()) == n
    mcts.path_total.zero_()
    v = mcts.search(stub_evaluator, 2.0, sims=24)
    tot = int(mcts.path_total.item())
    assert int(v.sum().item()) == 23 * n
    assert 23 * n < tot < 23 * n * 12
    mcts.close()
    env.close()


@pytest.mark.parametrize("sims", [1, 2, 3])
def test_mcts_few_simulations_vs_oracle(sims):
    """The smallest searches (one simulation: the root's expansion alone; two
    and three: the first select steps below it) on a ragged batch of 130
    boards at assorted positions: visits, tree sizes and the next MT word of
    every board vs the C oracle."""
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    n, base, cpuct = 130, 4100 + sims, 1.25
    env = BatchedEnv(n, seed_base=base, device=DEV)
    env.reset()
    plies = torch.arange(n, device=DEV) % 67
    for p in range(67):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
    st0, mt0, idx0 = env.export_state(with_mt=True)
    st0, mt0, idx0 = st0.cpu().numpy(), mt0.cpu().numpy().view(np.uint32), idx0.cpu().numpy()
    active = torch.from_numpy(np.array([not oracle.is_game_over(unpack_ref(st0[:, b])) for b in range(n)]))
    assert int(active.sum()) > 0
    mcts = BatchedMCTS(env, sims)
    visits = mcts.search(stub_evaluator, cpuct, active=active).cpu().numpy()
    counts = mcts.stats().cpu().numpy()
    _, mt1, idx1 = env.export_state(with_mt=True)
    mt1, idx1 = mt1.cpu().numpy().view(np.uint32), idx1.cpu().numpy()
    for b in range(n):
        if not active[b]:
            assert visits[b].sum() == 0
            continue
        m = oracle.mt_from_words(mt0[b], idx0[b])
        _, ov, nn, ne = oracle.mcts_search(unpack_ref(st0[:, b]), m, sims, cpuct, testing=True)
        assert (visits[b] == ov).all(), b
        assert (counts[b, 0], counts[b, 1]) == (nn, ne), b
        assert oracle.mt_next32(oracle.mt_from_words(mt1[b], idx1[b])) == oracle.mt_next32(m), b
    mcts.close()
    env.close()
