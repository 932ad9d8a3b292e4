"""bench.py's N > 1 path (barriers, max-over-ranks time, summed counts, one
JSON line from rank 0) rehearsed with two ranks sharing this box's GPU over
gloo (HZ_BENCH_REHEARSAL=1); the driver's real run uses one GPU per rank and
RCCL.  Also the default single-rank contract fields, the selfplay sub-object
and the config-4 exchange."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu

SMALL_SP = ["--sp-boards", "256", "--sp-sims", "16", "--sp-warmup", "1", "--sp-moves", "2"]


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _torchrun(args, port, timeout=600):
    env = dict(os.environ, HZ_BENCH_REHEARSAL="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2"] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


def _single(args, timeout=600, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


def test_bench_gpus_n_spawns_its_ranks():
    """`bench.py --gpus 2` with no launcher starts two ranks itself (the form
    the driver uses for its N-GPU runs); on this one-GPU box they share it
    over gloo (HZ_BENCH_REHEARSAL=1)."""
    env = dict(os.environ, HZ_BENCH_REHEARSAL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = _single(["--gpus", "2", "--steps", "2", "--warmup", "1", "--launches-per-step", "4", "--no-off-compare",
                 "--no-selfplay"], env=env)
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "shard2"
    assert "8192/8192 boards bit-exact vs C oracle" in d["parity"]
    assert "spawning 2 ranks" in r.stderr


def test_bench_rccl_one_rank():
    """--dist at one rank: the process group is RCCL ("nccl") and the N > 1
    collectives run on device tensors: the parity all-reduces, and the
    complete games' records all-gathered (all_gather_into_tensor) into the
    replay buffer; with one rank the gathered records are the rank's own."""
    r = _single(["--dist", "--steps", "2", "--warmup", "1", "--launches-per-step", "4", "--no-off-compare",
                 "--no-cpu-baseline", "--sp-cpu-seconds", "0"] + SMALL_SP)
    assert "backend nccl" in r.stderr, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 1 and "4096/4096 boards bit-exact" in d["parity"]
    sp = d["selfplay"]
    x = sp["exchange"]
    assert x is not None and x["records"] == x["records_own"] == sp["game"]["moves"]
    assert x["bytes_per_rank_received"] == x["records"] * 336
    assert sp["parity"].startswith("256/256 boards bit-exact vs C twin")
    assert sp["nn_parity"]["rows_checked"] >= 256


def test_config4_rccl_one_rank_equals_plain(tmp_path):
    """Config 4 with the records all-gathered over RCCL at one rank
    (SelfPlay.iteration -> all_gather_records on device tensors) fills the
    replay buffer with exactly the records of the run without a process
    group."""
    _single(CFG4 + ["--dist", "--records-out", str(tmp_path / "rccl")])
    _single(CFG4 + ["--records-out", str(tmp_path / "plain")])
    a = torch.load(tmp_path / "rccl.rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "plain.rank0.pt", weights_only=True)
    assert a["buffer"].shape[0] > 0 and torch.equal(a["buffer"], b["buffer"]) and torch.equal(a["own"], b["own"])


def test_bench_two_ranks_rehearsal():
    r = _torchrun(["--steps", "2", "--warmup", "1", "--launches-per-step", "8", "--no-off-compare"] + SMALL_SP,
                  29517)
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["parallelism"] == "shard2"
    assert d["cpu_baseline"] is None
    sp = d["selfplay"]
    assert sp["n_gpus"] == 2 and sp["sims_per_s"] > 0
    x = sp["exchange"]
    # the complete games' records of both ranks, all-gathered
    assert x["records"] == sp["game"]["moves"] and x["bytes_per_rank_received"] == x["records"] * 336
    assert 2 * 256 * 40 <= x["records"] <= 2 * 256 * 100
    assert sp["games_per_s_basis"].startswith("complete games") and sp["game"]["games"] == 2 * 256
    assert sp["steady"]["games_ended"] >= 2 * 256  # both ranks' continuous legs, summed
    # every rank checked its own boards against the C twin and the oracle
    assert sp["parity"].startswith("512/512 boards bit-exact vs C twin")
    assert "8192/8192 boards bit-exact vs C oracle" in d["parity"]


def test_bench_single_rank_contract():
    r = _single(["--steps", "2", "--warmup", "1", "--launches-per-step", "16", "--cpu-seconds", "1",
                 "--sp-cpu-seconds", "1"] + SMALL_SP)
    d = _last_json(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "selfplay"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["games_per_step"] == 16 * 4096
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "issue_bound"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    assert "4096/4096 boards bit-exact" in d["parity"]
    assert d["env_games_per_s"] > 0 and "games_per_s" not in d
    sp = d["selfplay"]
    for k in ("sims_per_s", "games_per_s", "nn_roofline", "tree_ms_per_move", "cpu_baseline", "exchange",
              "env_steps_per_s", "nn_parity"):
        assert k in sp, k
    assert sp["exchange"] is None
    # env steps: every expansion child plus every real move of the complete games
    g = sp["game"]
    assert g["env_steps"] > 5 * g["moves"] and sp["env_steps_per_s"] == g["env_steps_per_s"]
    assert sp["nn_parity"]["rows_checked"] >= 256 and sp["nn_parity"]["max_abs_dpolicy"] <= 1e-4
    assert sp["nn_parity"]["max_abs_dvalue"] <= 1e-4
    assert sp["sims"] == 256 * 16 * 2 and 0 < sp["nn_rows_evaluated"] <= sp["sims"]
    assert 0 < sp["nn_roofline"]["frac"] < 1 and sp["nn_roofline"]["fp32_mfma_frac"] > 0
    assert sp["parity"].startswith("256/256 boards bit-exact vs C twin")
    # continuous self-play: every board's first game ends inside the 80 moves
    st = sp["steady"]
    assert st["games_ended"] >= 256 and 40 <= st["mean_game_plies"] <= 100 and st["games_per_s"] > 0
    assert sp["steady_games_per_s"] == st["games_per_s"] == d["selfplay_steady_games_per_s"]
    # the caller-facing loop and the counter-derived rates
    assert "replayed by the C oracle" in d["api_caller"]["parity"] and d["api_caller"]["env_steps_per_s"] > 0
    assert d["auto_reset"]["env_steps_per_s"] > 0 and "bit-exact" in d["auto_reset"]["parity"]
    if d["roofline"]["traffic_gbs"] is not None:
        assert 0 < d["roofline"]["traffic_frac"] < 1
    assert sp["tree_roofline"]["path_edge_levels"] >= sp["sims"] // 2
    assert sp["games_per_s_basis"].startswith("complete games") and sp["game"]["games"] == 256
    assert "load_checkpoint" in sp["network"]
    for k in ("value", "unit", "cores", "kind", "sample", "nn_cpu_ms_per_eval"):
        assert k in sp["cpu_baseline"], k


CFG4 = ["--config", "4", "--boards", "48", "--sims", "6", "--iterations", "2", "--warmup", "2"]


def test_config4_exchange_two_ranks_equals_world1(tmp_path):
    """Config 4 rehearsed at world 2 (gloo, both ranks on this GPU): every
    rank's replay buffer holds the same records, in rank order; each rank's
    own records equal a world-1 run over the same global boards bit for bit
    (results do not depend on the GPU count); the example count is the sum of
    the ranks' plies."""
    r = _torchrun(CFG4 + ["--records-out", str(tmp_path / "w2")], 29519)
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["unit"] == "games/s" and d["exchange"]["records"] > 0
    w2 = [torch.load(tmp_path / f"w2.rank{k}.pt", weights_only=True) for k in (0, 1)]
    assert torch.equal(w2[0]["buffer"], w2[1]["buffer"])
    solo = []
    for k in (0, 1):
        _single(CFG4 + ["--seed-base", str(48 * k), "--records-out", str(tmp_path / f"w1_{k}")])
        solo.append(torch.load(tmp_path / f"w1_{k}.rank0.pt", weights_only=True))
        assert torch.equal(w2[k]["own"], solo[k]["own"]), k
    # two iterations: per iteration rank 0's records then rank 1's
    own = [torch.split(w2[k]["own"], w2[k]["own_counts"].tolist()) for k in (0, 1)]
    want = torch.cat([torch.cat((own[0][i], own[1][i])) for i in range(2)])
    assert torch.equal(w2[0]["buffer"], want)
    assert d["exchange"]["records"] == want.shape[0] == d["examples_per_iteration"] * 2


def test_config1_single_game_contract():
    """bench.py --config 1: games played one at a time through the drop-in
    modules (harmonies_engine / MCTS / process_game_state with ModelManager)
    to the end; one JSON line with the contract keys and the reference's
    CPU figure beside it."""
    r = _single(["--config", "1", "--games", "1", "--sims", "2"])
    d = _last_json(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "dtype",
              "config", "plies", "reference_cpu"):
        assert k in d, k
    assert d["unit"] == "games/s" and d["value"] > 0 and d["steps"] == 1
    assert 40 <= d["plies"][0] <= 100


def test_config4_stub_records_replayed_by_oracle(tmp_path):
    """Config 4 at world 2 with the stub evaluator (--stub): each rank's own
    records of both iterations (state, visit counts, z, player) are replayed
    board by board by the C twin's search (oracle.mcts_search with the
    logged root noise and uniforms, MCTS.py:272-441) and engine
    (trainer.py:468-538's ply loop): states, visits, moves and z agree."""
    import numpy as np
    import oracle
    from hzamd import distributed as hd
    from hzamd.state import unpack_ref
    n = 48
    _torchrun(["--config", "4", "--boards", str(n), "--sims", "6", "--iterations", "2", "--warmup", "2", "--stub",
               "--records-out", str(tmp_path / "s")], 29523)
    checked = 0
    for rank in (0, 1):
        d = torch.load(tmp_path / f"s.rank{rank}.pt", weights_only=True)
        assert d["stub"] and d["sims"] == 6
        base = int(d["seed_base"])
        states, visits, z, player = (t.numpy() for t in hd.unpack_records(d["own"]))
        noise, u, act = d["noise"].numpy(), d["u"].numpy(), d["act"].numpy()
        counts = d["own_counts"].tolist()
        off = step = 0
        for it in range(2):
            # env.reset() before the warm-up moves started episode 0; iteration it plays episode it + 1
            ms = [oracle.mt_seed(base + b + ((it + 1) << 32)) for b in range(n)]
            ss = [oracle.reset(m) for m in ms]
            start, ply, ends = off, 0, {}
            while True:
                live = [b for b in range(n) if not oracle.is_game_over(ss[b])]
                if not live:
                    break
                for b in live:
                    r = off
                    assert (unpack_ref(states[r]) == ss[b]).all(), (rank, it, ply, b)
                    assert player[r] == ss[b][72]
                    a, ov, _, _ = oracle.mcts_search(ss[b], ms[b], 6, 2.0, eps=0.25, testing=False, tau0=15,
                                                     ply=ply, u=float(u[step, b]),
                                                     noise=np.concatenate([noise[step, b], np.zeros(143 - 69)]))
                    assert (visits[r] == ov).all(), (rank, it, ply, b)
                    assert a == act[step, b], (rank, it, ply, b)
                    rc, ss[b] = oracle.step(ss[b], a, ms[b])
                    assert rc == 0
                    ends.setdefault(b, []).append(r)
                    off += 1
                    checked += 1
                ply += 1
                step += 1
            assert ply == int(d["plies"][it]) and off - start == counts[it]
            for b, rows in ends.items():
                w = int(ss[b][75])
                outcome = 1.0 if w == 0 else -1.0 if w == 1 else 0.0
                for r in rows:
                    assert z[r] == (outcome if player[r] == 0 else -outcome), (rank, it, b)
    assert checked > 2 * 2 * n * 40
