"""Benchmark: BASELINE config 2 — 4096 concurrent boards per GPU, pure env
step / legal_actions / score HIP kernels, bit-exact vs the CPU engine — with
config 3 (and, at N > 1, config 4's exchange) measured in the same run.

Headline (config 2): one bench step = `--launches-per-step` (256) batched
passes of the env hot path over 4096 boards, each a single hz_play launch:
HarmoniesGameState() on every board (CPython-exact seeding and opening
draws), then play to the end of every game (legal mask -> build-defined
splitmix rule pick -> apply_move, incl. chance draws and final scoring).
The final states of the first and the last timed launch are compared with
the C oracle board by board.
Boards are seeded by their global id (rank * 4096 + b), so N GPUs run N
independent shards (weak scaling, no data-path collective).

`selfplay` sub-object (config 3, profile_self_play.py's loop batched): 4096
boards x 200 MCTS simulations per move with the default 128-filter x
8-block network in fp32, 2 warm-up + 3 timed moves; at N > 1 the timed
moves' (s, pi, player) records are all-gathered over RCCL (config 4's
exchange) and timed separately.

Other configs: --config 3 (self-play moves only, or --full-game), --config 4
(whole self-play iterations + the all-gather into every rank's replay
buffer), --config 5 (the full training loop).

Prints one JSON line (rank 0).  Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W] [--boards 4096]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "harmonies-alphazero_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# SURVEY.md §8(d) algorithmic bytes per unit
BYTES_PER_ENV_STEP = 152   # 64 B state read + 64 B state write + 18 B mask + ~6 B RNG
BYTES_PER_RESET = 2564     # 624x4 B MT init + idx + 64 B state
BYTES_PER_ENCODE = 5488    # f32 [38,5,7] + [42] written per state
TREE_BYTES_POLICY = 576    # f32 [143] policy + value row read per evaluated leaf
TREE_BYTES_CHILD = 88      # per expansion child: 64 B state + 16 B edge + 8 B hash slot
TREE_BYTES_PATH = 16       # per edge level walked by a simulation (~16 B / path edge)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
MAX_PLIES = 96             # rule games end after 56-72 plies
# hz_play launches until every board replays a fully prepared episode, by
# pipeline (1: seed -> draw1 -> draw2 -> play; 2: k_play2's thirteen stages)
PIPELINE_DEPTH = {1: 4, 2: 13}
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
X6_PRODUCTS = 6                # bf16 MFMAs per fp32 product block in the x6 kernels
# bf16 MFMA FLOP the 4096-row forward's kernels issue per state (8-state
# workgroups; v_mfma_f32_16x16x32_bf16 = 16,384 FLOP): the tower's 16 convs x
# 4 chunks x 132 block-taps (the tap classes skip off-board taps: 132 of 162)
# x 8 column blocks x 6 products, and the stem's chunk 0 (132 block-taps x 8
# x 3: an encoder board's values are bf16 values, so only the A plane h
# issues) and its tap-packed chunk 1 (3 K-steps x 18 blocks x 8 x 3), per
# workgroup / 8 (hz_net.hip kX6ClassTaps, k_conv3x3_x6, x6w4_body)
MFMA_FLOP = 16384
X6_ISSUED_FLOP_PER_STATE = (16 * 4 * 132 * 8 * 6 + 132 * 8 * 3 + 3 * 18 * 8 * 3) * MFMA_FLOP / 8
CLOCK_GHZ = 2.4            # MI355X peak engine clock (cycle figures of the issue-bound view)
MT_SEED_STEPS = 1246       # init_by_array's two 623-step passes: the seeding chain per reset
MT_STEP_FLOOR_CYCLES = 17  # tools/alu_chain.py: the bare MT recurrence per step
MEAN_SELFPLAY_PLIES = 62.4  # mean game length


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher, N > 1 starts N ranks itself. Must equal "
                         "WORLD_SIZE when a launcher set it")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (RCCL) even at one rank, so the N > 1 collectives run")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--boards", type=int, default=4096)
    ap.add_argument("--pipeline", type=int, choices=(1, 2), default=2,
                    help="config 2: hz_play's pipeline (1 = chance-ahead k_rollout, 2 = k_play2's thirteen stages; "
                         "identical results)")
    ap.add_argument("--launches-per-step", type=int, default=256,
                    help="config 2: hz_play launches (4096-board batches) per bench step")
    ap.add_argument("--seed-base", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-off-compare", action="store_true",
                    help="skip the chance-ahead-off comparison run (profiling)")
    ap.add_argument("--no-api-path", action="store_true",
                    help="config 2: skip the per-ply API path leg (reset / legal+rule+step per ply / score graphs)")
    ap.add_argument("--no-api-caller", action="store_true",
                    help="config 2: skip the api_caller leg (a Python caller's own moves through legal_actions/step)")
    ap.add_argument("--no-auto-reset", action="store_true",
                    help="config 2: skip the steady-state auto-reset leg (hz_rollout auto_reset launches)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06", "traffic.json"),
                    help="HBM bytes per launch from the counter passes (tools/traffic_r06.sh)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="1: one game at a time through the drop-in modules (profile_self_play.py); "
                         "2: env kernels (default, the headline) + the selfplay sub-object; 3: MCTS self-play "
                         "moves with the network; 4: whole self-play iterations + the RCCL all-gather into "
                         "every rank's replay buffer; 5: whole training iterations "
                         "(self-play -> buffer -> training -> arena)")
    ap.add_argument("--games", type=int, default=4, help="config 1: timed games (seeds 0..games-1)")
    ap.add_argument("--no-selfplay", action="store_true", help="config 2: skip the selfplay sub-object")
    ap.add_argument("--sp-boards", type=int, default=4096, help="selfplay sub-object: boards per GPU")
    ap.add_argument("--sp-sims", type=int, default=200, help="selfplay sub-object: simulations per move")
    ap.add_argument("--sp-warmup", type=int, default=2, help="selfplay sub-object: untimed moves")
    ap.add_argument("--sp-moves", type=int, default=3, help="selfplay sub-object: timed moves")
    ap.add_argument("--sp-cpu-seconds", type=float, default=8.0,
                    help="selfplay sub-object: bound of the one-thread C-twin sample (seconds x 4)")
    ap.add_argument("--sp-steady-moves", type=int, default=80,
                    help="selfplay sub-object: moves of the continuous (steady-state) leg, 0 = off")
    ap.add_argument("--sp-games", type=int, default=1,
                    help="selfplay sub-object: complete games timed on every board (0: estimate games/s from "
                         "the per-move leg)")
    ap.add_argument("--iterations", type=int, default=5,
                    help="config 5: training iterations timed (one evaluation cycle at eval-every 5); "
                         "config 4: self-play iterations timed")
    ap.add_argument("--eval-games", type=int, default=30, help="config 5: arena games per evaluation (config.py:92)")
    ap.add_argument("--eval-every", type=int, default=5, help="config 5: eval_frequency (config.py:94)")
    ap.add_argument("--eval-sims", type=int, default=200, help="config 5: mcts_config_eval sims (config.py:68)")
    ap.add_argument("--sims", type=int, default=None,
                    help="MCTS simulations per move (config 3/4: 200; config 5: 400 = mcts_config_default)")
    ap.add_argument("--records-out", default=None,
                    help="config 4: write this rank's replay buffer and own records (torch.save) for tests")
    ap.add_argument("--checkpoint", default=None,
                    help="self-play network: a model.py-format checkpoint (default: synthesize best_model.pth.tar "
                         "from the torch.manual_seed(0) default net and load it through load_checkpoint)")
    ap.add_argument("--stub", action="store_true",
                    help="config 4 only: the deterministic stub evaluator instead of the network (oracle-replay tests)")
    ap.add_argument("--nn-dtype", default="fp32", choices=["fp32", "bf16"], help="config 3 leaf-eval dtype")
    ap.add_argument("--full-game", action="store_true",
                    help="config 3: time one complete game on every board (games/s measured, not estimated)")
    args = ap.parse_args()
    if args.stub and args.config != 4:
        ap.error("--stub applies to --config 4 only (the other configs time the network)")
    return args


_RED_DEV = None  # device of reduction tensors: the GPU under RCCL, the CPU under gloo


def traffic_entry(args, kernel):
    """The counter passes' figures for one kernel (tools/traffic_r06.py:
    bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE, and the kernel's mean
    rocprof duration in the same command), or None."""
    try:
        with open(args.traffic_json) as f:
            return json.load(f).get("kernels", {}).get(kernel)
    except (OSError, ValueError):
        return None


def traffic_rate(entry, seconds_per_launch=None):
    """Counter bytes per launch as a rate: over `seconds_per_launch` (a live
    measurement of this run) when given, else over the counter run's own
    rocprof mean duration."""
    if not entry:
        return None
    b = entry["bytes_per_launch"]
    t = seconds_per_launch if seconds_per_launch else entry.get("mean_ns", 0) * 1e-9
    if not t:
        return None
    gbs = b / t / 1e9
    return {"bytes_per_launch": b, "traffic_gbs": gbs, "traffic_frac": gbs / HBM_PEAK_GBS,
            "over": "this run's live launch time" if seconds_per_launch else
                    f"the counter run's rocprof mean ({entry.get('mean_ns', 0) / 1e3:.1f} us)",
            "source": "profiles/r06/traffic.json (tools/traffic_r06.sh: FETCH_SIZE x2 + WRITE_SIZE, separate "
                      "--pmc passes of one command)"}


def all_reduce(vals, op):
    """Reduce a list of numbers over ranks (float64: exact for counts)."""
    t = torch.tensor(vals, dtype=torch.float64, device=_RED_DEV)
    dist.all_reduce(t, op=op)
    return t.tolist()


def cpu_baseline(boards, seconds):
    """The C oracle (oracle/hz_oracle.c, the bit-exact CPU port of the
    reference engine) playing the same rule-driven 4096-board batches on the
    host cores, for a bounded wall time."""
    import oracle
    nthreads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    oracle.play_rule_games(64, 10**9, nthreads=nthreads)  # warm the library / threads
    steps = games = 0
    t0 = time.perf_counter()
    k = 0
    while True:
        total, _, _, _ = oracle.play_rule_games(boards, 10**9 + k * boards, nthreads=nthreads)
        steps += total
        games += boards
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    # the same port on one core, a shorter bounded sample (SURVEY §8d ii)
    s1, t1 = 0, time.perf_counter()
    k1 = 0
    while time.perf_counter() - t1 < seconds / 4:
        s1 += oracle.play_rule_games(boards // 4, 2 * 10**9 + k1 * boards, nthreads=1)[0]
        k1 += 1
    dt1 = time.perf_counter() - t1
    return {"value": steps / dt, "unit": "env-steps/s", "cores": nthreads, "kind": "port",
            "games_per_s": games / dt, "value_1core": s1 / dt1,
            "sample": f"{k} batches x {boards} rule-driven games ({steps} env steps) in {dt:.1f}s, "
                      f"C oracle with OpenMP, {nthreads} threads; 1 core: {k1} batches x {boards // 4} games "
                      f"in {dt1:.1f}s"}


def bench_single_game(args, dev):
    """BASELINE config 1: profile_self_play.py:17-77's loop, one game at a
    time through the drop-in modules (harmonies_engine.HarmoniesGameState,
    process_game_state.create_state_tensors, MCTS.get_best_action_and_pi)
    with hzamd.manager.ModelManager as the model manager (predict: the folded
    HIP network at batch 1), 32 simulations per move, mcts_config_default
    otherwise, default network random-initialised with torch.manual_seed(0);
    game g seeded random.seed(g), np.random.seed(g) as in BASELINE.md.  One
    host round trip per simulation, as the reference's evaluator contract
    has it.  Reports games/s over `games` games after one warm-up game."""
    import random

    import numpy as np
    from harmonies_engine import HarmoniesGameState
    from MCTS import get_best_action_and_pi
    from process_game_state import create_state_tensors

    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    from hzamd.selfplay import MCTS_DEFAULT
    sims = args.sims or 32
    cfg = dict(MCTS_DEFAULT, num_simulations=sims)
    torch.manual_seed(0)
    mm = ModelManager(dict(DEFAULT), {"device": str(dev), "optimizer_type": "Adam", "learning_rate": 0.001,
                                      "weight_decay": 0.0001, "value_loss_weight": 1.0,
                                      "policy_loss_weight": 1.0})

    def one(g):
        random.seed(g)
        np.random.seed(g)
        game, turn = HarmoniesGameState(), 0
        while not game.is_game_over():
            create_state_tensors(game)  # the reference loop builds the inputs every ply
            action, _ = get_best_action_and_pi(game.clone(), mm, cfg, turn)
            if action is None:
                raise RuntimeError(f"config 1: no move for seed {g} at ply {turn}")
            game = game.apply_move(action)
            turn += 1
        return turn

    one(1000)  # warm-up: kernels, allocator, the folded network
    torch.cuda.synchronize(dev)
    times, plies = [], []
    for g in range(args.games):
        t0 = time.perf_counter()
        plies.append(one(g))
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    total = sum(times)
    line = {"metric": "config 1: one self-play game at a time through the drop-in modules (games/s)",
            "value": len(times) / total, "unit": "games/s", "n_gpus": 1, "steps": len(times), "warmup": 1,
            "ms_per_step": total / len(times) * 1e3, "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic: random-init network, seeded games",
            "config": {"workload": f"config1: 1 game at a time, {sims} sims/move, mcts_config_default, "
                                   "default 128fx8 net", "games": len(times), "sims": sims},
            "s_per_game": [round(t, 3) for t in times], "plies": plies,
            "plies_per_s": sum(plies) / total, "sims_per_s": sum(plies) * sims / total,
            "reference_cpu": {"s_per_game": 13.80, "games_per_s": 0.0725, "plies_per_s": 4.35,
                              "source": "BASELINE.md: the reference on 8 CPU cores, seeds 0-3, measured in the "
                                        "survey container (not published)"}}
    print(json.dumps(line), flush=True)


def bench_loop(args, dev, rank, world):
    """BASELINE config 5: the reference's main.py loop (trainer.Trainer) on
    the batched engine, one step = one training iteration: `boards` games per
    rank of self-play with the best model (mcts_config_default: 400 sims per
    move, self-play noise), RCCL all-gather of the records into every rank's
    replay buffer, rank-0 training (reference training config: Adam, batch
    64, 2 epochs over the buffer, buffer 50,000), weight broadcast,
    checkpoint, buffer file, and every `eval_every` (5) iterations an arena
    of `eval_games` (30) games between candidate and best
    (mcts_config_eval, 200 sims), sharded over the ranks.  Reports
    games/hour over `iterations` (default 5 = one evaluation cycle)."""
    import tempfile
    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    from hzamd.trainer import Trainer
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    sims = args.sims or 400
    model_cfg = dict(DEFAULT, board_size=(5, 7))
    train_cfg = {"device": str(dev), "optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 0.0001,
                 "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64, "momentum": 0.9,
                 "use_scheduler": True, "scheduler_type": "StepLR", "scheduler_step_size": 30,
                 "scheduler_gamma": 0.5, "force_lr_reset_on_load": False, "new_forced_lr": 0.000125}
    mcts_cfg = {"num_simulations": sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
                "fpu_value": 0.25, "turns_until_tau0": 15, "action_size": 143, "testing": False}
    tmp = tempfile.mkdtemp(prefix=f"hz_loop_r{rank}_")
    sp_cfg = {"num_iterations": args.iterations + 1, "num_games_per_iter": args.boards, "epochs_per_iter": 2,
              "replay_buffer_size": 50000, "checkpoint_folder": os.path.join(tmp, "ck"),
              "replay_buffer_folder": os.path.join(tmp, "buf"), "replay_buffer_filename": "replay_buffer.pkl",
              "eval_frequency": args.eval_every, "eval_episodes": args.eval_games, "eval_win_rate_threshold": 0.51,
              "best_model_filename": "best_model.pth.tar"}
    mm = ModelManager(model_cfg, train_cfg)
    tr = Trainer(mm, mcts_cfg, sp_cfg, train_cfg, eval_mcts_config={"num_simulations": args.eval_sims},
                 seed_base=args.seed_base,
                 log=lambda *a: print(f"[config5 r{rank}]", *a, file=sys.stderr, flush=True))
    # warm-up iteration (kernels, allocator), then the timed ones
    tr.iteration = 0
    tr.execute_self_play_phase(tr.best_model_manager)
    tr.execute_training_phase()
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    t0 = time.perf_counter()
    phases = {"self_play": 0.0, "training": 0.0, "evaluation": 0.0}
    games, evals = 0, 0
    for it in range(1, args.iterations + 1):
        tr.iteration = it
        a = time.perf_counter()
        sp = tr.execute_self_play_phase(tr.best_model_manager)
        b = time.perf_counter()
        tr.execute_training_phase()
        tr.model_manager.step_scheduler()
        if rank == 0:
            tr.model_manager.save_checkpoint(folder=sp_cfg["checkpoint_folder"], filename="latest_candidate.pth.tar",
                                             iteration=it)
        tr.save_buffer()
        torch.cuda.synchronize(dev)
        c = time.perf_counter()
        if it % args.eval_every == 0:
            tr.evaluate_model()
            evals += 1
        torch.cuda.synchronize(dev)
        d = time.perf_counter()
        phases["self_play"] += b - a
        phases["training"] += c - b
        phases["evaluation"] += d - c
        games += sp["games"]
        print(f"[config5] iteration {it}: self-play {b - a:.1f}s training {c - b:.1f}s eval {d - c:.1f}s",
              file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dd():
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    if rank == 0:
        ref = (sims == 400 and args.eval_sims == 200 and args.eval_games == 30 and args.eval_every == 5)
        print(json.dumps({
            "metric": "full loop self-play games/hour (self-play -> buffer -> training -> arena)",
            "value": games / elapsed * 3600.0, "unit": "games/hour", "n_gpus": world, "steps": args.iterations,
            "warmup": 1, "ms_per_step": elapsed * 1000.0 / args.iterations, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic: random-init network, seeded games",
            "config": {"workload": f"config5: {args.boards} games/rank/iteration, {sims} sims/move, arena "
                                   f"{args.eval_games} games x {args.eval_sims} sims every {args.eval_every} "
                                   f"iterations, default 128fx8 net"
                                   + ("" if ref else " (deviates from config.py:53-99)"),
                       "boards_per_gpu": args.boards, "sims": sims, "eval_sims": args.eval_sims,
                       "eval_games": args.eval_games, "eval_frequency": args.eval_every,
                       "reference_config": ref, "parallelism": f"shard{world}"},
            "phase_seconds": phases, "games": games, "evaluations": evals,
        }))
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)  # the run's checkpoints and buffer files


class TimedEvaluator:
    """Wraps the leaf evaluator: HIP events around every call (the current
    stream, where the network's kernels run); `rows` = the rows it computed
    since reset(), read from the search's own device counter (k_gather adds
    each simulation's live-row count; one add per search), so the timed
    region holds no counting kernel of the benchmark's."""

    device_rows = True

    def __init__(self, pred, dev):
        self.pred = pred
        # the fused (arrival-order) leaf gather exactly when the wrapped
        # evaluator allows it (hzamd.mcts.BatchedMCTS.search)
        self.row_independent = bool(getattr(pred, "row_independent", False))
        self.events = []
        self.mcts = None  # attach(): the BatchedMCTS whose searches call this evaluator
        self._base = torch.zeros(1, dtype=torch.int64, device=dev)
        self._ebase = torch.zeros(1, dtype=torch.int64, device=dev)
        self._pbase = torch.zeros(1, dtype=torch.int64, device=dev)
        self.calls = 0
        self.snap_at = None  # call index whose leaf batch + outputs are kept (device copies) for nn_guard
        self.snap = None
        # HZ_BENCH_CALL_DUMP=path: each call's live-row count is kept too (a
        # device copy after the event pair) and call_stats() writes the
        # per-call (rows, ms) lists there (tools/tail_trace.py)
        self.dump = os.environ.get("HZ_BENCH_CALL_DUMP")
        self.rowlog = []

    def attach(self, mcts):
        self.mcts = mcts
        mcts.count_edges = True  # expansion env steps counted on the device (edges_total)
        mcts.count_path = True  # edge levels walked by the simulations (path_total)

    def __call__(self, board, glob, rows=None, count=None):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = self.pred(board, glob, rows, count)
        b.record()
        self.events.append((a, b))
        if self.dump:
            self.rowlog.append(count.clone() if torch.is_tensor(count) else
                               torch.full((1,), board.shape[0] if count is None else int(count),
                                          dtype=torch.int32, device=board.device))
        if self.calls == self.snap_at:  # after the event pair: not part of the forward's time
            self.snap = (board.clone(), glob.clone(), None if count is None else count.clone(),
                         out[0].clone(), out[1].clone())
        self.calls += 1
        return out

    @property
    def rows(self):
        return self.mcts.eval_rows_total - self._base

    @property
    def edges(self):
        """Expansion env steps (apply_move per legal child) since reset()."""
        return self.mcts.edges_total - self._ebase

    @property
    def path_edges(self):
        """Edge levels walked by the simulations (select + backup) since reset()."""
        return self.mcts.path_total - self._pbase

    def reset(self):
        torch.cuda.synchronize()
        self.events.clear()
        self.rowlog.clear()
        self._base = self.mcts.eval_rows_total.clone()
        self._ebase = self.mcts.edges_total.clone()
        self._pbase = self.mcts.path_total.clone()

    def ms(self):
        return sum(a.elapsed_time(b) for a, b in self.events)

    def call_stats(self):
        """Per-call forward durations (HIP events, no profiler): the tail of
        the distribution shows whether slow launches exist outside rocprof."""
        import numpy as np
        t = np.array([a.elapsed_time(b) for a, b in self.events])
        if not t.size:
            return None
        q = np.percentile(t, [50, 90, 99, 99.9])
        if self.dump and self.rowlog:
            rows = torch.cat([r.view(-1)[:1].to(torch.int64) for r in self.rowlog]).cpu().numpy()
            with open(self.dump, "w") as f:
                json.dump({"rows": rows.tolist(), "ms": t.tolist()}, f)
        return {"calls": int(t.size), "mean_ms": float(t.mean()), "std_ms": float(t.std()), "p50_ms": float(q[0]),
                "p90_ms": float(q[1]), "p99_ms": float(q[2]), "p999_ms": float(q[3]), "max_ms": float(t.max()),
                "calls_over_2x_p50": int((t > 2 * q[0]).sum())}


REF_TRAIN_CFG = {"optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 0.0001,
                 "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64, "momentum": 0.9,
                 "use_scheduler": True, "scheduler_type": "StepLR", "scheduler_step_size": 30,
                 "scheduler_gamma": 0.5, "force_lr_reset_on_load": False, "new_forced_lr": 0.000125}


def load_selfplay_model(args, dev):
    """BASELINE config 3's network: best_model.pth.tar through
    ModelManager.load_checkpoint (model.py:184-256).  The reference's file is
    absent offline, so unless --checkpoint names one, a
    checkpoint is synthesized first: the default network initialised with
    torch.manual_seed(0), written by save_checkpoint in the model.py:161-182
    dict.  Returns (model in eval mode, description)."""
    import tempfile
    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    cfg = dict(REF_TRAIN_CFG, device=str(dev))
    mm = ModelManager(dict(DEFAULT, board_size=(5, 7)), cfg)

    def load(path):
        ok, _ = mm.load_checkpoint(folder=os.path.dirname(os.path.abspath(path)), filename=os.path.basename(path))
        if not ok:
            raise SystemExit(f"could not load {path} with ModelManager.load_checkpoint")

    if args.checkpoint is None:
        with tempfile.TemporaryDirectory(prefix="hz_ckpt_") as folder:  # removed after the load
            torch.manual_seed(0)
            ModelManager(dict(DEFAULT, board_size=(5, 7)), cfg).save_checkpoint(folder=folder,
                                                                                filename="best_model.pth.tar")
            load(os.path.join(folder, "best_model.pth.tar"))
        what = "synthesized best_model.pth.tar (torch.manual_seed(0) default net, model.py:161-182 format)"
    else:
        load(args.checkpoint)
        what = f"checkpoint {args.checkpoint}"
    return mm.model.eval(), what + " loaded by ModelManager.load_checkpoint"


def _selfplay_setup(args, dev, rank, sims, n):
    from hzamd.mcts import BatchedPredictor
    from hzamd.selfplay import SelfPlay
    torch.backends.cudnn.benchmark = True
    cfg = {"num_simulations": sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
           "turns_until_tau0": 15, "testing": False}
    if getattr(args, "stub", False):
        # the deterministic integer evaluator of the parity fixtures (tests
        # replay such runs with the C twin's search, board by board)
        from hzamd.mcts import stub_evaluator
        return SelfPlay(n, stub_evaluator, cfg, seed_base=args.seed_base + rank * n, device=dev), None
    net, what = load_selfplay_model(args, dev)
    dtype = torch.bfloat16 if args.nn_dtype == "bf16" else None
    ev = TimedEvaluator(BatchedPredictor(net, dtype=dtype), dev)
    ev.network = what
    sp = SelfPlay(n, ev, cfg, seed_base=args.seed_base + rank * n, device=dev)
    ev.attach(sp.mcts)
    return sp, ev


def bench_selfplay(args, dev, rank, world):
    """BASELINE config 3: 4096 boards x `sims` MCTS simulations per move with
    the default 128-filter x 8-block network (random init, torch.manual_seed(0),
    BatchedPredictor = ModelManager.predict batched).  One step = one move of
    every board (full search + choice + env step)."""
    from hzamd.net import flops_per_eval
    n, sims = args.boards, args.sims or 200
    sp, ev = _selfplay_setup(args, dev, rank, sims, n)
    if args.full_game:
        return bench_selfplay_games(args, sp, ev, dev, rank, world, sims)
    sp.env.reset()
    for w in range(args.warmup):
        sp.move(w)
    ev.reset()
    if dd():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    moves = []
    for k in range(args.steps):
        moves.append(sp.move(args.warmup + k)[2].sum())
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sp.check_steps()  # the last timed move's env step (move() reports one move late)
    nn_ms = ev.ms()
    rows = int(ev.rows.item())
    env_steps = int(ev.edges.item()) + int(sum(int(m) for m in moves))  # expansion children + real moves
    sims_done = n * sims * args.steps
    if dd():
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    sims_all = sims_done * world
    per_move = elapsed / args.steps
    fl = flops_per_eval()
    if rank == 0:
        print(json.dumps({
            "metric": "self-play MCTS simulations/sec @4096 boards x 200 sims",
            "value": sims_all / elapsed, "unit": "sims/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": per_move * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.nn_dtype,
            "data": "synthetic: seeded games; network = synthesized best_model.pth.tar (seed-0 random init)",
            "config": {"workload": f"config3: {n} boards x {sims} sims/move, default 128fx8 net",
                       "boards_per_gpu": n, "sims": sims, "parallelism": f"shard{world}"},
            "games_per_s_est": world * n / (per_move * MEAN_SELFPLAY_PLIES),
            "env_steps_per_s": env_steps * world / elapsed,
            "nn_rows_evaluated": rows, "nn_ms_per_move": nn_ms / args.steps,
            "tree_ms_per_move": per_move * 1e3 - nn_ms / args.steps,
            "nn_tflops": fl * rows / (nn_ms * 1e-3) / 1e12 if nn_ms else None,
            "note": f"games/s estimated from ms per move x mean game length {MEAN_SELFPLAY_PLIES} plies",
        }))


def bench_selfplay_games(args, sp, ev, dev, rank, world, sims):
    """Config 3, measured end to end: after `warmup` moves of a throw-away
    game, every board plays one whole self-play game (search + choice + env
    step per ply, records kept on the device as SelfPlay.play does); games/s
    = boards of all ranks / the slowest rank's time."""
    from hzamd.net import flops_per_eval
    n = sp.n
    sp.env.reset()
    for w in range(args.warmup):
        sp.move(w)
    ev.reset()
    orig_move = sp.move

    def move(ply, done=None, **kw):  # progress on stderr (a long run must not look hung)
        out = orig_move(ply, done, **kw)
        if ply % 8 == 0:
            print(f"[config3 full game] ply {ply}", file=sys.stderr, flush=True)
        return out

    sp.move = move
    if dd():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rec = sp.play(reset=True)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    sp.move = orig_move
    moves = int(rec["valid"].sum().item())
    nn_ms = ev.ms()
    rows = int(ev.rows.item())
    env_steps = int(ev.edges.item()) + moves
    if dd():
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    if rank == 0:
        print(json.dumps({
            "metric": "self-play games/sec @4096 boards x 200 MCTS sims (complete games, measured)",
            "value": world * n / elapsed, "unit": "games/s", "n_gpus": world, "steps": 1, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.nn_dtype,
            "data": "synthetic: seeded games; network = synthesized best_model.pth.tar (seed-0 random init)",
            "config": {"workload": f"config3: {n} boards x {sims} sims/move, one whole game per board",
                       "boards_per_gpu": n, "sims": sims, "parallelism": f"shard{world}"},
            "plies": rec["plies"], "moves": moves, "sims_per_s": world * moves * sims / elapsed,
            "env_steps_per_s": world * env_steps / elapsed,
            "nn_rows_evaluated": rows, "nn_rows_skipped": moves * sims - rows, "nn_s": nn_ms * 1e-3,
            "nn_tflops": flops_per_eval() * rows / (nn_ms * 1e-3) / 1e12 if nn_ms else None,
            "nn_call_ms": ev.call_stats(),
        }))


def selfplay_probe(args, dev, rank, world):
    """The `selfplay` sub-object of the default line (config 3,
    profile_self_play.py:17-77's loop batched; at N > 1 also config 4's
    exchange).  Three legs on every rank:
      1. per move: `sp_moves` timed moves at the full leaf batch (sims/s and
         the network's roofline at batch 4096);
      2. complete games: `sp_games` whole self-play games on every board, timed
         end to end (games_per_s is measured, not extrapolated); at N > 1 the
         games' (s, pi, z) records are all-gathered over RCCL into every
         rank's replay buffer and the exchange is timed (config 4);
      3. parity guard: the first timed move's roots, chance streams and root
         noise searched again on the GPU with the deterministic stub
         evaluator, and by the C twin (or_mcts_search, MCTS.py:272-441
         restated) on the host: root visit counts, tree sizes and the next
         word of every board's CPython stream must agree, board by board,
         on every rank (the count of mismatches is all-reduced).
    Returns the sub-object on rank 0."""
    from hzamd import distributed as hd
    from hzamd.net import flops_per_eval
    n, sims = args.sp_boards, args.sp_sims
    sp, ev = _selfplay_setup(args, dev, rank, sims, n)
    fl = flops_per_eval()
    sp.env.reset()
    for w in range(args.sp_warmup):
        sp.move(w)
    torch.cuda.synchronize(dev)
    # the first timed move's roots + streams (device copies): the guard's input
    roots = tuple(t.clone() for t in sp.env.export_state(with_mt=True))
    active0 = ~sp.env.done()
    sp.keep_noise = True
    sp.noise_log.clear()
    step0 = sp.step_counter

    # -- leg 1: per move at the full leaf batch.  The same moves run twice
    # from the same positions (states, streams and noise keys restored:
    # every result is the same): first as the workload alone, which gives
    # the move time, then with a HIP event pair around every leaf
    # evaluation, which gives the network's time; the pairs' markers add
    # ~10 us per simulation to a move (tools/event_cost.py,
    # profiles/r04/event_cost.json), which the first pass leaves out
    def timed_moves(evaluator):
        sp.evaluator = evaluator
        recs = []
        if dd():
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(args.sp_moves):
            recs.append(sp.move(args.sp_warmup + k))
        torch.cuda.synchronize(dev)
        if dd():
            dist.barrier()
        dt = time.perf_counter() - t0
        sp.check_steps()
        return recs, dt

    recs, elapsed = timed_moves(ev.pred)
    noise0 = sp.noise_log[0][0].clone()
    sp.keep_noise = False
    sp.noise_log.clear()
    sp.env.import_state(*roots)
    sp.step_counter = step0
    ev.reset()
    ev.calls, ev.snap_at, ev.snap = 0, sims // 2, None  # the NN guard's leaf batch: mid first timed move
    recs_i, elapsed_i = timed_moves(ev)
    sp.evaluator = ev
    nn_ms = ev.ms()
    rows = int(ev.rows.item())
    board_moves = int(sum(int(a.sum().item()) for _, _, a in recs))
    assert board_moves == int(sum(int(a.sum().item()) for _, _, a in recs_i))
    env_steps = int(ev.edges.item()) + board_moves  # expansion children + real moves
    sims_done = board_moves * sims
    if dd():
        elapsed, elapsed_i = all_reduce([elapsed, elapsed_i], dist.ReduceOp.MAX)
        sims_all, rows_all, env_all = (int(x) for x in all_reduce([sims_done, rows, env_steps], dist.ReduceOp.SUM))
    else:
        sims_all, rows_all, env_all = sims_done, rows, env_steps
    per_move = elapsed / args.sp_moves
    nn_tf = fl * rows / (nn_ms * 1e-3) / 1e12 if nn_ms else None
    # the tree kernels' roofline (per simulation, the leaf's
    # encoded row written and its policy/value row read, and per expansion
    # child its state, edge and hash slot), over the move time the network
    # does not take (select, expand, backup, gather + encode, noise, choice)
    edges = int(ev.edges.item())
    path = int(ev.path_edges.item())
    # both from the instrumented pass: the network's event-timed share and
    # that pass's own move time (the uninstrumented pass's time minus the
    # instrumented pass's network time mixed two passes' clocks: 9.7-18.1 ms
    # per move across boxes for the same code, against 12.6-12.9 this way;
    # the event records, ~2 per simulation, count as tree time here)
    tree_s = elapsed_i - nn_ms * 1e-3
    tree_bytes = rows * (BYTES_PER_ENCODE + TREE_BYTES_POLICY) + edges * TREE_BYTES_CHILD + path * TREE_BYTES_PATH
    tree_gbs = tree_bytes / tree_s / 1e9 if tree_s > 0 else None
    tree_roofline = {"bound": "latency (a wave per board walks, expands and backs up one path per simulation)",
                     "achieved": tree_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": tree_gbs / HBM_PEAK_GBS if tree_gbs else None,
                     "alg_bytes_per_move": tree_bytes / args.sp_moves,
                     "basis": f"{BYTES_PER_ENCODE} B encoded + {TREE_BYTES_POLICY} B policy/value read per "
                              f"evaluated leaf ({rows} rows), {TREE_BYTES_CHILD} B per expansion child (state, key "
                              f"digest, edge, hash slot; {edges} children), {TREE_BYTES_PATH} B per edge level "
                              f"walked (select's read + backup's N/W update; {path} levels = the sum of the trees' "
                              "edge visit counts, hz_mcts_path_edges), over the instrumented pass's move time "
                              "minus its event-timed network time",
                     "path_edge_levels": path, "mean_path_depth": path / max(1, board_moves * sims),
                     "traffic": traffic_rate(traffic_entry(args, "k_expand_backup<4, true, true, 16, false>"))}
    # the network's numerics in the measured run: rows of a timed leaf batch
    # against the checkpoint's network in float64 on the CPU
    nn_parity = nn_guard(ev, dev)
    # -- leg 2: complete games (+ config 4's exchange at N > 1)
    game = selfplay_games_leg(args, sp, ev, dev, rank, world, sims, fl) if args.sp_games > 0 else None
    steady = selfplay_steady_leg(args, sp, ev, dev, rank, world, sims, fl) if args.sp_steady_moves > 0 else None
    # -- leg 3: the parity guard (every rank), with the CPU twin's timing
    guard = selfplay_guard(roots, active0, noise0, sims, dev, rank, world,
                           cpu_sample=rank == 0 and world == 1 and args.sp_cpu_seconds > 0,
                           one_core_s=min(2.0, args.sp_cpu_seconds / 4))
    out = None
    if rank == 0:
        emu_peak = BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS
        out = {"workload": f"config3: {n} boards/GPU x {sims} sims/move, default 128fx8 net, fp32; "
                           f"per move: {args.sp_warmup} warm-up + {args.sp_moves} timed moves from the game start; "
                           f"complete games: {args.sp_games} whole game(s) on every board",
               "sims_per_s": sims_all / elapsed, "nn_evals_per_s": rows_all / elapsed,
               "env_steps_per_s_per_move_leg": env_all / elapsed,
               "ms_per_move": per_move * 1e3, "nn_ms_per_move": nn_ms / args.sp_moves,
               "tree_ms_per_move": (elapsed_i - nn_ms * 1e-3) / args.sp_moves * 1e3,
               "tree_ms_per_move_two_pass": per_move * 1e3 - nn_ms / args.sp_moves,
               "ms_per_move_instrumented": elapsed_i / args.sp_moves * 1e3,
               "per_move_basis": "ms_per_move: the timed moves alone; nn_ms_per_move: the same moves replayed from "
                                 "the same positions with a HIP event pair around every leaf evaluation "
                                 "(ms_per_move_instrumented is that pass's move time); tree_ms_per_move = "
                                 "ms_per_move_instrumented - nn_ms_per_move (one pass: the event records count "
                                 "as tree time)",
               "nn_rows_evaluated": rows, "sims": sims_done,
               "nn_roofline": {"bound": "mfma", "achieved": nn_tf, "peak": emu_peak, "unit": "TFLOP/s",
                               "frac": nn_tf / emu_peak if nn_tf else None,
                               "fp32_mfma_peak": FP32_MFMA_PEAK_TFLOPS,
                               "fp32_mfma_frac": nn_tf / FP32_MFMA_PEAK_TFLOPS if nn_tf else None,
                               "mfma_issued": {
                                   "bf16_flop_per_eval": X6_ISSUED_FLOP_PER_STATE,
                                   "achieved": (X6_ISSUED_FLOP_PER_STATE * rows / (nn_ms * 1e-3) / 1e12
                                                if nn_ms else None),
                                   "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                   "frac": (X6_ISSUED_FLOP_PER_STATE * rows / (nn_ms * 1e-3) / 1e12
                                            / BF16_MFMA_PEAK_TFLOPS if nn_ms else None),
                                   "basis": "bf16 MFMA FLOP the stem and tower kernels issue per state (the tap "
                                            "classes skip off-board taps, the stem's bf16-exact inputs issue one "
                                            "A plane) over the same event time, against the bf16 dense peak: the "
                                            "matrix pipes' delivered rate, where frac above credits the dense fp32 "
                                            "conv"},
                               "flop_per_eval": fl,
                               "basis": "fp32 FLOP of the whole leaf-eval forward at the 4096-row batch (HIP events "
                                        "around each call, incl. the heads) over the emulated-fp32 roof: the stem "
                                        "and tower convs compute fp32-exact products as six bf16 MFMAs per fp32 "
                                        "product block, so their ceiling is the bf16 dense peak / 6 = "
                                        f"{emu_peak:.1f} TFLOP/s; fp32_mfma_frac is the same figure against the "
                                        f"f32 MFMA's dense peak ({FP32_MFMA_PEAK_TFLOPS} TFLOP/s), which this path "
                                        "does not use",
                               "traffic": traffic_rate(traffic_entry(args, "k_x6w4_tower<true>"))},
               "tree_roofline": tree_roofline,
               "dtype": "fp32", "n_gpus": world, "network": ev.network, "parity": guard["parity"],
               "nn_parity": nn_parity}
        if game is not None:
            out.update({"games_per_s": game["games_per_s"], "games_per_s_basis": game["basis"],
                        "env_steps_per_s": game["env_steps_per_s"],
                        "env_steps_basis": "complete-games leg: expansion children (one apply_move per legal "
                                           "child, MCTS.py:171-177, counted on the device) + real moves, all "
                                           "ranks, over the slowest rank's time",
                        "game": game})
            out["exchange"] = game.get("exchange")
        else:
            out.update({"env_steps_per_s": env_all / elapsed,
                        "env_steps_basis": "per-move leg: expansion children + real moves",
                        "games_per_s": world * n / (per_move * MEAN_SELFPLAY_PLIES),
                        "games_per_s_basis": f"estimate: ms per move x mean game length {MEAN_SELFPLAY_PLIES} "
                                             "plies (--sp-games 0)", "exchange": None})
        out["steady"] = steady
        out["steady_games_per_s"] = steady["games_per_s"] if steady is not None else None
        if guard.get("cpu_baseline") is not None:
            out["cpu_baseline"] = guard["cpu_baseline"]
    sp.mcts.close()
    sp.env.close()
    return out


def selfplay_games_leg(args, sp, ev, dev, rank, world, sims, fl):
    """Leg 2 of the selfplay sub-object: `sp_games` complete games on every
    board (SelfPlay.play: search + choice + env step per ply, records kept on
    the device), timed end to end with barriers; at N > 1 the compacted
    records (z from each recorded player's side) are all-gathered into every
    rank's replay buffer over RCCL, timed separately (config 4's exchange,
    trainer.py:104-127)."""
    from hzamd import distributed as hd
    n = sp.n
    orig_move = sp.move

    def move(ply, done=None, **kw):  # progress on stderr: a long run must not look hung
        out = orig_move(ply, done, **kw)
        if ply % 16 == 0:
            print(f"[selfplay game] rank {rank} ply {ply}", file=sys.stderr, flush=True)
        return out

    sp.move = move
    ev.reset()
    plies, moves, t_play, packed = [], 0, 0.0, []
    try:
        for _ in range(args.sp_games):
            if dd():
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            rec = sp.play(reset=True)
            torch.cuda.synchronize(dev)
            t_play += time.perf_counter() - t0
            plies.append(rec["plies"])
            moves += int(rec["valid"].sum().item())
            if dd():
                comp = sp.compact(rec)
                packed.append(hd.pack_records(comp["states"], comp["visits"], comp["z"], comp["player"]))
            del rec
    finally:
        sp.move = orig_move
    nn_ms, rows = ev.ms(), int(ev.rows.item())
    nn_calls = ev.call_stats()
    env_steps = int(ev.edges.item()) + moves  # expansion children + real moves
    exchange = None
    if dd():
        t_play = all_reduce([t_play], dist.ReduceOp.MAX)[0]
        moves_all, rows_all, env_all = (int(x) for x in all_reduce([moves, rows, env_steps], dist.ReduceOp.SUM))
        own = torch.cat(packed)
        buf = hd.ReplayBuffer(max(1, own.shape[0]) * world, dev)
        torch.cuda.synchronize(dev)
        dist.barrier()
        x0 = time.perf_counter()
        gathered = hd.all_gather_records(own)
        buf.extend(gathered)
        torch.cuda.synchronize(dev)
        xdt = all_reduce([time.perf_counter() - x0], dist.ReduceOp.MAX)[0]
        nbytes = gathered.numel() * 8
        exchange = {"collective": "all_gather (counts) + all_gather_into_tensor (records), into every rank's "
                                  "device replay buffer",
                    "records": int(gathered.shape[0]), "records_own": int(own.shape[0]),
                    "bytes_per_rank_received": nbytes, "ms": xdt * 1e3, "GBps": nbytes / xdt / 1e9,
                    "note": "the complete games' (s, pi, z) records, 336 B each (config 4's exchange)"}
    else:
        moves_all, rows_all, env_all = moves, rows, env_steps
    if rank != 0:
        return None
    games = world * n * args.sp_games
    return {"games_per_s": games / t_play,
            "basis": f"complete games: {args.sp_games} whole game(s) on each of the {world} x {n} boards, timed "
                     "end to end (slowest rank)",
            "seconds": t_play, "games": games, "plies_per_game_batch": plies, "moves": moves_all,
            "sims_per_s": moves_all * sims / t_play, "env_steps": env_all, "env_steps_per_s": env_all / t_play,
            "nn_rows_evaluated": rows_all,
            "nn_rows_skipped": moves_all * sims - rows_all, "nn_s_rank0": nn_ms * 1e-3,
            "nn_tflops_rank0": fl * rows / (nn_ms * 1e-3) / 1e12 if nn_ms else None,
            "nn_call_ms_rank0": nn_calls, "exchange": exchange}


def selfplay_steady_leg(args, sp, ev, dev, rank, world, sims, fl):
    """Leg 2b of the selfplay sub-object: continuous self-play
    (SelfPlay.play_steady: the reference's self_play_worker run game after
    game on every board, trainer.py:434-541; a board whose game ended starts
    its next game, seeded by global id and game index, before the next move),
    `sp_steady_moves` moves from a fresh reset, timed end to end.  Every
    move searches all boards, so no leaf batch shrinks as games end.
    games_per_s = board-moves per second / the mean length of the games that
    ended in the run (the long-run rate of a renewal process: both factors
    measured here); games_ended_per_s, the raw count over the same time, is
    beside it (games still running when the window closes are not counted
    there)."""
    n, M = sp.n, args.sp_steady_moves
    ev.reset()

    def progress(m):  # a long run must not look hung
        if m % 16 == 0:
            print(f"[selfplay steady] rank {rank} move {m}", file=sys.stderr, flush=True)
    if dd():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rec = sp.play_steady(M, progress=progress)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ended = rec["ended"]
    games = int(ended.sum().item())
    plies = int(rec["plies"][ended].to(torch.int64).sum().item())
    nn_ms, rows = ev.ms(), int(ev.rows.item())
    edges = int(ev.edges.item())
    moves = n * M
    del rec
    if dd():
        dt = all_reduce([dt], dist.ReduceOp.MAX)[0]
        games, plies, moves, rows, edges = (int(x) for x in all_reduce([games, plies, moves, rows, edges],
                                                                          dist.ReduceOp.SUM))
    if rank != 0:
        return None
    mean_len = plies / max(1, games)
    return {"games_per_s": moves / dt / mean_len,
            "basis": f"continuous self-play, {M} moves of every board from a fresh reset (finished boards start "
                     "their next game before the next move): board-moves/s over the mean length of the games that "
                     "ended in the run",
            "seconds": dt, "moves_per_board": M, "board_moves_per_s": moves / dt, "games_ended": games,
            "mean_game_plies": mean_len, "games_ended_per_s": games / dt, "sims_per_s": moves * sims / dt,
            "env_steps_per_s": (edges + moves) / dt, "nn_rows_evaluated": rows,
            "nn_rows_skipped": moves * sims - rows, "nn_s_rank0": nn_ms * 1e-3,
            "nn_tflops_rank0": fl * rows / world / (nn_ms * 1e-3) / 1e12 if nn_ms else None}


def selfplay_guard(roots, active, noise, sims, dev, rank, world, cpu_sample=False, one_core_s=2.0):
    """Leg 3: the first timed move's roots (states, CPython streams, root
    noise) searched on the GPU (BatchedMCTS with the stub evaluator, the
    timed move's settings: cpuct 2, eps 0.25, testing False) and on the host
    by the C twin's or_mcts_search, all boards spread over threads (ctypes
    releases the GIL).  Root visit counts, node and edge counts and the next
    CPython word of every board must be equal; mismatches are summed over
    ranks.  The CPU run's rate doubles as the selfplay cpu_baseline (rank 0,
    N = 1), with a one-thread sample and the reference network's batch-1 CPU
    forward beside it."""
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    import oracle  # test infrastructure: the checker and the CPU baseline only
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    from hzamd.state import unpack_ref
    st_d, mt_d, idx_d = roots
    n = st_d.shape[1]
    env = BatchedEnv(n, device=dev)
    env.import_state(st_d, mt_d, idx_d)
    mcts = BatchedMCTS(env, sims)
    visits = mcts.search(stub_evaluator, 2.0, active=active, noise=noise, eps=0.25, testing=False)
    counts = mcts.stats()
    _, mt1, idx1 = env.export_state(with_mt=True)
    torch.cuda.synchronize(dev)
    visits, counts = visits.cpu().numpy(), counts.cpu().numpy()
    mt1, idx1 = mt1.cpu().numpy().view(np.uint32), idx1.cpu().numpy()
    st, mt, idx = st_d.cpu().numpy(), mt_d.cpu().numpy().view(np.uint32), idx_d.cpu().numpy()
    nz = np.zeros((n, 143), np.float64)
    nz[:, :noise.shape[1]] = noise.cpu().numpy()
    act = active.cpu().numpy()
    mcts.close()
    env.close()
    nthreads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))

    def search(b):
        m = oracle.mt_from_words(mt[b], idx[b])
        _, ov, nn, ne = oracle.mcts_search(unpack_ref(st[:, b]), m, sims, 2.0, eps=0.25, testing=False, tau0=15,
                                           ply=0, noise=nz[b])
        return ov, nn, ne, m

    def check(b):
        ov, nn, ne, m = search(b)
        ok = ((visits[b] == ov).all() and counts[b, 0] == nn and counts[b, 1] == ne
              and oracle.mt_next32(m) == oracle.mt_next32(oracle.mt_from_words(mt1[b], idx1[b])))
        return int(not ok)

    boards = [b for b in range(n) if act[b]]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(nthreads) as pool:
        bad = sum(pool.map(check, boards, chunksize=8))
    cpu_dt = time.perf_counter() - t0
    checked = len(boards)
    if dd():
        bad, checked = (int(x) for x in all_reduce([bad, checked], dist.ReduceOp.SUM))
    assert bad == 0, f"selfplay parity: {bad} of {checked} boards' searches differ from the C twin"
    out = {"parity": f"{checked}/{checked} boards bit-exact vs C twin (first timed move's roots, streams and root "
                     f"noise, {sims} sims, stub evaluator: root visits, tree sizes, next MT word"
                     + (f"; {world} ranks, each its own boards)" if world > 1 else ")")}
    if not cpu_sample:
        return out
    # one thread, bounded, for the per-core figure
    t1, k1, s1 = time.perf_counter(), 0, 0
    while time.perf_counter() - t1 < one_core_s and k1 < len(boards):
        search(boards[k1])
        s1 += sims
        k1 += 1
    dt1 = time.perf_counter() - t1
    from hzamd.net import HarmoniesNet
    net = HarmoniesNet().eval()
    prev = torch.get_num_threads()
    torch.set_num_threads(nthreads)
    with torch.no_grad():
        b, g = torch.zeros(1, 38, 5, 7), torch.zeros(1, 42)
        for _ in range(5):
            net(b, g)
        t2 = time.perf_counter()
        for _ in range(40):
            net(b, g)
        nn_s = (time.perf_counter() - t2) / 40
    torch.set_num_threads(prev)
    tree_1 = s1 / dt1
    done = len(boards) * sims
    out["cpu_baseline"] = {
        "value": done / cpu_dt, "unit": "sims/s", "cores": nthreads, "kind": "port",
        "value_1core": tree_1, "nn_cpu_ms_per_eval": nn_s * 1e3,
        "est_sims_per_s_one_process": 1.0 / (1.0 / tree_1 + nn_s),
        "sample": f"the first timed move's {len(boards)} roots searched ({done} sims, {sims} per board) in "
                  f"{cpu_dt:.1f}s by the C twin's or_mcts_search on {nthreads} threads with the stub evaluator "
                  f"(tree work only; the same run is the parity guard); 1 thread: {k1} searches in {dt1:.1f}s; "
                  f"the reference net's batch-1 CPU forward ({nthreads} intra-op threads) timed separately; "
                  "est_sims_per_s_one_process = one reference-shaped process (one tree, one predict per leaf)"}
    return out


NN_GUARD_TOL = 1e-4  # tests/test_infer_gpu.py:38's bound against the float64 network


def nn_guard(ev, dev, rows_each=256):
    """The leaf evaluator's numerics inside the measured run (model.py:81-110):
    the first and the last `rows_each` live rows of one timed leaf batch
    (TimedEvaluator.snap: the batch the kernels saw and the probabilities and
    values they returned) evaluated again by the checkpoint's own network in
    float64 on the host CPU (softmax over all 143 logits, tanh value, as
    ModelManager.predict); max |diff| of probabilities and values must be
    within NN_GUARD_TOL on every rank (all-reduced)."""
    import copy
    if ev.snap is None:
        raise RuntimeError("nn_guard: no leaf batch was kept")
    board, glob, count, pol, val = ev.snap
    ev.snap = None
    k = int(count.item()) if count is not None else board.shape[0]
    idx = sorted(set(range(min(rows_each, k))) | set(range(max(0, k - rows_each), k)))
    it = torch.tensor(idx, dtype=torch.long, device=board.device)
    b64, g64 = board.index_select(0, it).cpu().double(), glob.index_select(0, it).cpu().double()
    p_gpu, v_gpu = pol.index_select(0, it).cpu().double(), val.reshape(-1).index_select(0, it).cpu().double()
    net64 = copy.deepcopy(ev.pred.model).cpu().double().eval()
    prev = torch.get_num_threads()
    torch.set_num_threads(max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))))
    t0 = time.perf_counter()
    with torch.no_grad():
        logits, v64 = net64(b64, g64)
    cpu_s = time.perf_counter() - t0
    torch.set_num_threads(prev)
    dp = (p_gpu - torch.softmax(logits, 1)).abs().max().item() if idx else 0.0
    dv = (v_gpu - v64.reshape(-1)).abs().max().item() if idx else 0.0
    checked = len(idx)
    if dd():
        dp, dv = all_reduce([dp, dv], dist.ReduceOp.MAX)
        checked = int(all_reduce([checked], dist.ReduceOp.SUM)[0])
    assert dp <= NN_GUARD_TOL and dv <= NN_GUARD_TOL, f"nn guard: max |dp| {dp:.3g}, |dv| {dv:.3g} > {NN_GUARD_TOL}"
    return {"rows_checked": checked, "live_rows_in_batch": k, "max_abs_dpolicy": dp, "max_abs_dvalue": dv,
            "tol": NN_GUARD_TOL, "cpu_s": cpu_s,
            "basis": f"the first and last {rows_each} live rows of one timed leaf batch (mid first timed move) "
                     "against the loaded network in float64 on the CPU: softmax probabilities and tanh values"}


def bench_exchange(args, dev, rank, world):
    """BASELINE config 4: every rank plays `iterations` self-play iterations
    (SelfPlay.iteration: one whole game on each of its 4096 boards, seeded by
    global board id) and all-gathers the packed (s, pi, z) records over RCCL
    into every rank's device replay buffer (trainer.py:104-127's Pool
    fan-out + replay_buffer.extend).  Self-play and the exchange are timed
    separately; value = games of all ranks / total time."""
    from hzamd import distributed as hd
    n, sims = args.boards, args.sims or 200
    sp, ev = _selfplay_setup(args, dev, rank, sims, n)
    buf = hd.ReplayBuffer(max(50000, 2 * n * 80 * world), dev)
    # warm-up: a few moves (kernels, allocator) and one exchange
    sp.env.reset()
    for w in range(min(2, args.warmup)):
        sp.move(w)
    if dd():
        hd.all_gather_records(torch.zeros(1, hd.RECORD_WORDS, dtype=torch.int64, device=dev))
    torch.cuda.synchronize(dev)
    own, plies = [], []
    t_play = t_x = 0.0
    games = examples = 0
    # --records-out: keep each move's root noise, uniforms and choices, so a
    # test can replay the records with the C twin (tests/test_bench_gpu.py)
    sp.keep_noise = bool(args.records_out)
    sp.noise_log.clear()
    if dd():
        dist.barrier()
    t0 = time.perf_counter()
    for it in range(args.iterations):
        tm = {}
        gathered, rec = sp.iteration(buf, timings=tm)
        plies.append(rec["plies"])
        del rec
        t_play += tm["play_s"]
        t_x += tm["exchange_s"]
        games += n * world
        examples += int(gathered.shape[0])
        own.append(tm["own_records"])
        print(f"[config4] iteration {it}: self-play {tm['play_s']:.1f}s exchange {tm['exchange_s'] * 1e3:.1f} ms "
              f"({int(gathered.shape[0])} records)", file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dd():
        elapsed, t_play, t_x = all_reduce([elapsed, t_play, t_x], dist.ReduceOp.MAX)
    if args.records_out:
        log = sp.noise_log
        torch.save({"buffer": buf.records().cpu(), "own": torch.cat(own).cpu(),
                    "own_counts": torch.tensor([o.shape[0] for o in own]), "rank": rank, "world": world,
                    "seed_base": args.seed_base + rank * n, "plies": torch.tensor(plies),
                    "noise": torch.stack([x[0] for x in log]).cpu(), "u": torch.stack([x[1] for x in log]).cpu(),
                    "act": torch.stack([x[2] for x in log]).cpu(), "sims": sims, "stub": bool(args.stub)},
                   f"{args.records_out}.rank{rank}.pt")
    nbytes = examples * hd.RECORD_WORDS * 8
    if rank == 0:
        print(json.dumps({
            "metric": "self-play games/sec @4096 boards/GPU x 200 MCTS sims + RCCL all-gather of (s, pi, z)",
            "value": games / elapsed, "unit": "games/s", "n_gpus": world, "steps": args.iterations,
            "warmup": 1, "ms_per_step": elapsed * 1e3 / args.iterations, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.nn_dtype,
            "data": ("synthetic: stub evaluator (parity runs), seeded games" if args.stub else
                     "synthetic: seeded games; network = synthesized best_model.pth.tar (seed-0 random init) "
                     "loaded through ModelManager.load_checkpoint"),
            "config": {"workload": f"config4: {n} boards/GPU x {sims} sims/move, whole games, records "
                                   f"all-gathered into every rank's replay buffer",
                       "boards_per_gpu": n, "sims": sims, "parallelism": f"shard{world}"},
            "self_play_s": t_play, "exchange": {"ms": t_x * 1e3, "records": examples,
                                                "bytes_per_rank_received": nbytes,
                                                "GBps": nbytes / t_x / 1e9 if t_x > 0 and dd() else None,
                                                "collective": "all_gather (counts) + all_gather_into_tensor"
                                                if dd() else "none (one rank)"},
            "examples_per_iteration": examples / args.iterations,
        }))


def dd():
    """True when torch.distributed carries this run's collectives (N > 1, or
    --dist at N = 1)."""
    return dist.is_available() and dist.is_initialized()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per
    GPU) as `torch.distributed.run` children on 127.0.0.1 and exit with their
    status.  The parent touches no GPU (torch.cuda.device_count() does not
    initialise one on this image); it only checks that N GPUs are visible."""
    import subprocess
    rehearsal = os.environ.get("HZ_BENCH_REHEARSAL") == "1"
    if not rehearsal and torch.cuda.device_count() < n:
        raise SystemExit(f"bench.py --gpus {n}: only {torch.cuda.device_count()} GPU(s) visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] spawning {n} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    r = subprocess.run(cmd)
    if r.returncode != 0:
        print(f"[bench] a rank failed (exit {r.returncode})", file=sys.stderr, flush=True)
    sys.exit(r.returncode)


def main():
    args = parse()
    if args.stub and args.config != 4:
        raise SystemExit("--stub is config 4's evaluator (oracle-replay runs); pass --config 4")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        spawn_ranks(args.gpus)  # exits
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HZ_BENCH_REHEARSAL=1 (tests only): ranks share the visible GPUs
    # (local % device_count) and reduce over gloo, to exercise the N > 1 path
    # on a one-GPU box; the real multi-GPU run uses one GPU per rank and RCCL
    rehearsal = os.environ.get("HZ_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = local % max(1, torch.cuda.device_count())
    elif world > 1 and local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but {torch.cuda.device_count()} GPU(s) visible")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    global _RED_DEV
    _RED_DEV = "cpu" if rehearsal else dev
    if world > 1 or args.dist:
        # --dist at N = 1: a one-rank process group, so the RCCL collectives
        # of the N > 1 path (records all-gather, parity all-reduce) run
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        print(f"[bench] rank {rank}/{world}: process group backend {dist.get_backend()}", file=sys.stderr,
              flush=True)
    if args.config == 1:
        if world > 1:
            raise SystemExit("config 1 is one game at a time on one GPU")
        bench_single_game(args, dev)
        return
    if args.config == 5:
        bench_loop(args, dev, rank, world)
        if dd():
            dist.destroy_process_group()
        return
    if args.config in (3, 4):
        (bench_selfplay if args.config == 3 else bench_exchange)(args, dev, rank, world)
        if dd():
            dist.destroy_process_group()
        return

    from hzamd.env import BatchedEnv
    from hzamd.state import unpack_ref

    n, L = args.boards, args.launches_per_step
    env = BatchedEnv(n, seed_base=args.seed_base + rank * n, device=dev)
    env.set_pipeline(args.pipeline)
    kname = "k_play2" if args.pipeline == 2 else "k_rollout"
    games = torch.zeros(n, dtype=torch.int32, device=dev)
    steps = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    launches = [0]  # hz_play launches so far: launch k plays every board's episode k

    def one_launch(_unused=None, g=games, s=steps):
        # hz_play: HarmoniesGameState() on every board fused with rule-driven
        # play to the end of the game, one launch
        env.rollout(MAX_PLIES, games_done=g, steps_done=s, reset=True)
        launches[0] += 1

    # first batch (episode 0: board b seeded seed_base + rank*n + b) doubles as
    # a parity guard: its env-step count must equal the C oracle's
    one_launch()
    torch.cuda.synchronize(dev)
    first_steps = int(steps.sum().item())
    # the chance-ahead pipeline (seed -> draw1 -> draw2 -> play) is primed
    # after three launches; warm-up is at least that many
    prime = max(0, PIPELINE_DEPTH[args.pipeline] - args.warmup * L)
    for _ in range(max(0, args.warmup * L - 1) + prime):
        one_launch()
    torch.cuda.synchronize(dev)

    # per-launch counters of the timed launches (each launch plays a new episode)
    T = args.steps * L
    games_t = torch.zeros(T, n, dtype=torch.int32, device=dev)
    steps_t = torch.zeros(T, n, dtype=torch.int32, device=dev)
    first_ep = launches[0]
    first_state = torch.empty(6, n, dtype=torch.int64, device=dev)
    # the timed launches call hz_play through the C-ABI with their arguments
    # made beforehand (env.rollout's per-call Python work, and a tracer's
    # per-call interception on top of it, would otherwise leave the GPU
    # waiting between 13-us launches); the same entry point and arguments
    import ctypes
    from hzamd import _native as nat
    env._sync_stream()
    play, h = nat.lib().hz_play, env._h
    gp = [ctypes.c_void_p(games_t[i].data_ptr()) for i in range(T)]
    spp = [ctypes.c_void_p(steps_t[i].data_ptr()) for i in range(T)]

    def fast_launch(i):
        rc = play(h, MAX_PLIES, 0, None, None, None, gp[i], spp[i])
        if rc:
            raise nat.NativeError(f"hz_play failed with code {rc}")
        launches[0] += 1

    if dd():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(T):
        fast_launch(i)
        if i == 0:  # the first timed batch's final states, for the oracle check (a 196 KB copy)
            first_state.copy_(env.export_state())
            env._sync_stream()
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    last_ep = launches[0] - 1
    last_state = env.export_state()
    # the dominant kernel's average launch duration: HIP events on the env's
    # stream around a block of K back-to-back launches (no markers between
    # them), outside the timed region; rocprofv3's per-dispatch average for
    # k_rollout (profiles/<round>/stats) is the figure it must agree with
    K = min(T, 512)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    env._sync_stream()
    gp = [ctypes.c_void_p(games.data_ptr())] * K
    spp = [ctypes.c_void_p(steps.data_ptr())] * K
    ev0.record(stream)
    for i in range(K):
        fast_launch(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = ev0.elapsed_time(ev1) / K
    env.epoch += 1  # (games were started outside env.rollout)
    env.check_errors()  # no pipeline wave gave up waiting in any launch so far (else NativeError)

    timed_steps, timed_games = int(steps_t.sum(dtype=torch.int64)), int(games_t.sum(dtype=torch.int64))
    longest = int(steps_t.max())
    if dd():
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
        c = all_reduce([timed_steps, timed_games], dist.ReduceOp.SUM)
        env_steps_all, games_all = int(c[0]), int(c[1])
    else:
        env_steps_all, games_all = timed_steps, timed_games

    value = env_steps_all / elapsed
    games_per_s = games_all / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps

    # roofline of the dominant kernel (hz_play = k_rollout with reset, or
    # k_play2), per launch
    alg_bytes = (timed_steps * BYTES_PER_ENV_STEP + timed_games * BYTES_PER_RESET) / T
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get(f"{kname}_bytes_per_launch")
        except Exception:
            traffic = None
    tr = traffic_rate(traffic_entry(args, kname), kern_ms * 1e-3)
    cycles = kern_ms * 1e-3 * CLOCK_GHZ * 1e9
    issue = {"kernel_cycles": cycles, "longest_game_plies": longest,
             "cycles_per_ply_longest_game": cycles / max(1, longest),
             "cycles_per_mt_seed_step": cycles / MT_SEED_STEPS, "mt_step_floor_cycles": MT_STEP_FLOOR_CYCLES,
             "note": (f"a launch is the longest serial per-lane chain of its roles (one board's whole game, or a "
                      f"stream's {MT_SEED_STEPS}-step seeding) at {CLOCK_GHZ} GHz; the bare MT recurrence costs "
                      f"{MT_STEP_FLOOR_CYCLES} cycles/step (tools/alu_chain.py), DESIGN.md §3"
                      if kname == "k_rollout" else
                      f"k_play2 runs thirteen stages side by side, one per episode in flight: the game cut into four "
                      f"play stages, the {MT_SEED_STEPS}-step seeding chain into five stages of 207-312 steps, the "
                      f"draws into four; a launch lasts as long as its longest stage (tools/p2_roles.py), so "
                      f"cycles_per_mt_seed_step and cycles_per_ply_longest_game are the launch divided by the whole "
                      f"chain, a per-launch proxy; the bare recurrence costs {MT_STEP_FLOOR_CYCLES} cycles/step and "
                      f"a step with its b32 LDS read and HBM store ~56 (tools/alu_chain.py), DESIGN.md §3")}

    # the same workload with chance-ahead off (every launch seeds and draws
    # in-kernel), for comparison; not the headline number
    off_steps, off_elapsed = 0, float("nan")
    if not args.no_off_compare:
        off_steps, off_elapsed = off_compare(env, one_launch, games, args, dev, world)

    api = None if args.no_api_path else api_path_leg(args, dev, rank, world)
    caller = None if args.no_api_caller else api_caller_leg(args, dev, rank, world)
    auto = None if args.no_auto_reset else auto_reset_leg(args, dev, rank, world)
    enc = encoder_roofline(dev, n, args.seed_base) if rank == 0 else None

    # parity guard on every rank, over its own boards (global ids
    # seed_base + rank * n + b): the first batch's env-step count and the
    # final states of the first and the last timed batches against the C
    # oracle; the mismatch counts are summed over ranks
    import oracle  # test infrastructure: parity guard + cpu_baseline only
    my_base = args.seed_base + rank * n
    ref_total = oracle.play_rule_games(n, my_base, nthreads=8)[0]
    bad_steps = int(ref_total != first_steps)
    bad_boards = 0
    for ep, stt in ((first_ep, first_state), (last_ep, last_state)):
        got = stt.cpu().numpy()
        _, finals, _, _ = oracle.play_rule_games(n, my_base, nthreads=8, episode=ep)
        bad = [b for b in range(n) if not (unpack_ref(got[:, b]) == finals[b]).all()]
        if bad:
            print(f"[parity] rank {rank} episode {ep}: boards {bad[:8]} differ from the C oracle", file=sys.stderr)
        bad_boards += len(bad)
    if dd():
        bad_steps, bad_boards = (int(x) for x in all_reduce([bad_steps, bad_boards], dist.ReduceOp.SUM))
    assert bad_steps == 0 and bad_boards == 0, (bad_steps, bad_boards)
    parity = (f"first batch: {first_steps} env steps == C oracle ({ref_total}); final states of the first and "
              f"last timed batches (episodes {first_ep}, {last_ep}): {world * n}/{world * n} boards bit-exact vs "
              "C oracle" + (f" ({world} ranks, each its own boards)" if world > 1 else ""))
    sp = None
    if not args.no_selfplay:
        env.close()
        sp = selfplay_probe(args, dev, rank, world)

    if rank == 0:
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(n, args.cpu_seconds)
        out = {
            "metric": "self-play env-steps/sec + games/sec @4096 boards, 1/2/4/8 GPUs; bit-exact vs CPU",
            "value": value,
            "unit": "env-steps/s",
            "headline_basis": "value = config 2: rule-driven env play (reset, legal mask, step, chance draws, "
                              "final scoring) on 4096 boards/GPU, NO MCTS and no network; the self-play "
                              "(config 3: 200-sim MCTS + network per move) figures are selfplay_env_steps_per_s "
                              "and selfplay_games_per_s",
            "selfplay_env_steps_per_s": (sp or {}).get("env_steps_per_s"),
            "selfplay_games_per_s": (sp or {}).get("games_per_s"),
            "selfplay_steady_games_per_s": (sp or {}).get("steady_games_per_s"),
            "env_games_per_s": games_per_s,
            "env_games_basis": "rule-driven env games (config 2, no MCTS) per second; the self-play games/s "
                               "is selfplay.games_per_s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: CPython-seeded games, seeds = global board id, build-defined splitmix rule policy",
            "config": {"workload": f"config2: 4096 concurrent boards/GPU, reset + rule-driven play to game end "
                                   f"(legal mask, step, chance draws, final scoring); one step = {L} hz_play "
                                   f"launches of 4096 boards",
                       "boards_per_gpu": n, "launches_per_step": L, "env_steps_per_step": timed_steps / args.steps,
                       "games_per_step": timed_games / args.steps, "parallelism": f"shard{world}"},
            "roofline": {"bound": "latency (per-lane chains)", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_gbs": tr["traffic_gbs"] if tr else None,
                         "traffic_frac": tr["traffic_frac"] if tr else None,
                         "traffic_basis": "counter bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/r06/"
                                          "traffic.json) over this run's kernel_ms" if tr else None,
                         "kernel": kname, "kernel_ms": kern_ms, "kernel_ms_launches": K,
                         "alg_bytes_per_launch": alg_bytes, "issue_bound": issue,
                         "bound_note": "priced against HBM (peak 8 TB/s), but the launch is bound by its serial "
                                       "per-lane chains (a board's whole game, a stream's seeding): counter "
                                       "traffic is below the algorithmic bytes, see issue_bound and DESIGN.md §3"},
            "chance_ahead": {"on": True, "pipeline": args.pipeline,
                             "note": ("each hz_play also prepares every board's next three episodes as a pipeline "
                                      "on the other CUs (stream seeding, pile draws and rule hashes, none of which "
                                      "depends on moves); steady state: one preparation per game in the timed region"
                                      if args.pipeline == 1 else
                                      "k_play2: each hz_play runs thirteen stages on thirteen consecutive episodes "
                                      "of every board (seeding pass 1 in two stages, pass 2 in three, pile draws 0-5, "
                                      "6-11, 12-17, 18-23 + rule hashes, plies 0-23, 24-39, 40-55, the rest + scoring); "
                                      "steady "
                                      "state: one episode's worth of every stage per call, i.e. one game per board per "
                                      "call"),
                             "pipeline_prime": prime,
                             "value_off": (off_steps / off_elapsed) if off_steps else None,
                             "ms_per_step_off": (off_elapsed * 1000.0 / args.steps) if off_steps else None},
            "encoder_roofline": enc,
            "cpu_baseline": cpu,
            "parity": parity,
            "selfplay": sp,
        }
        out["api_path"] = api
        out["api_caller"] = caller
        out["auto_reset"] = auto
        print(json.dumps(out))
    if args.no_selfplay:
        env.close()
    if dd():
        dist.destroy_process_group()


def encoder_roofline(dev, n, seed_base):
    """hz_encode_states (create_state_tensors) over one batch of recorded game
    states (every ply of n rule-driven games): output bytes / time vs HBM peak."""
    from hzamd.env import BatchedEnv
    from hzamd.selfplay import encode_states
    env = BatchedEnv(n, seed_base=seed_base + (1 << 40), device=dev)
    env.reset()
    _, _, (ts, _, ta) = env.rollout(MAX_PLIES, record=True)
    states = ts.permute(0, 2, 1).reshape(-1, 6)[(ta >= 0).reshape(-1)].contiguous()
    m = states.shape[0]
    for _ in range(3):
        encode_states(states)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        encode_states(states)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    gbs = m * BYTES_PER_ENCODE / (ms * 1e-3) / 1e9
    env.close()
    return {"kernel": "k_encode_board + k_encode_glob", "states": m, "ms": ms, "achieved": gbs,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "bytes_per_state": BYTES_PER_ENCODE}


def off_compare(env, one_launch, games, args, dev, world):
    """Time the same workload with chance-ahead off (every launch seeds and
    draws in-kernel; pipeline 1); returns (env steps of all ranks, max elapsed)."""
    env.set_seed_ahead(False)
    env.set_pipeline(1)
    for _ in range(2):
        one_launch()
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    T = args.steps * args.launches_per_step
    steps_o = torch.zeros(T, env.n, dtype=torch.int32, device=dev)
    t1 = time.perf_counter()
    for i in range(T):
        one_launch(None, games, steps_o[i])
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    elapsed = time.perf_counter() - t1
    total = int(steps_o.sum(dtype=torch.int64))
    if dd():
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
        total = int(all_reduce([total], dist.ReduceOp.SUM)[0])
    env.set_seed_ahead(True)
    env.set_pipeline(args.pipeline)
    for _ in range(PIPELINE_DEPTH[args.pipeline]):  # (refill before anything else times this env)
        one_launch()
    return total, elapsed


def _oracle_check(env, n, base, ep, plies=None):
    """Boards whose final state (and ply count) differ from the C oracle's
    episode-ep game (test infrastructure: parity guard only)."""
    import oracle
    from hzamd.state import unpack_ref
    got = env.export_state().cpu().numpy()
    total, finals, ref_plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=ep)
    bad = [b for b in range(n) if not (unpack_ref(got[:, b]) == finals[b]).all()]
    return bad, total


def api_path_leg(args, dev, rank, world, plies=MAX_PLIES, reps=10):
    """The batched per-ply surface (harmonies_engine.py:145-298, :357-367) as
    a caller of the reference API drives it: reset, then per ply
    legal_actions -> the rule pick -> step, then score; one batch = every
    board's whole game.  Each ply is one launch (hz_rule_ply: the three
    calls' outputs, bit-identical), the batch one replayed HIP graph
    (reset + `plies` ply launches + score); the three-launch form is timed
    beside it.  Each replay's reset starts every board's next episode.  Env
    steps per batch are the episodes' step counts (the C oracle's, for the
    same seeds); the first and the last timed episodes' final states are
    checked against it board by board."""
    import oracle
    from hzamd.env import BatchedEnv
    n = args.boards
    base = args.seed_base + rank * n
    env = BatchedEnv(n, seed_base=base, device=dev)
    mask = torch.zeros(n, 3, dtype=torch.int64, device=dev)
    count = torch.zeros(n, dtype=torch.int32, device=dev)
    act = torch.zeros(n, dtype=torch.int16, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)

    def fused():
        env.reset()
        for _ in range(plies):
            env.rule_ply(mask, count, act, status)
        env.score()

    def layered():
        env.reset()
        for _ in range(plies):
            env.legal_mask(mask, count)
            env.rule_actions(mask, count, act)
            env.step(act, status)
        env.score()

    def graph_of(body):
        body()  # (eager once: episode k)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                body()
        torch.cuda.current_stream(dev).wait_stream(s)
        return g

    episodes = [0]  # resets so far: the next batch plays episode episodes[0]

    def timed(g):
        g.replay()
        episodes[0] += 1
        torch.cuda.synchronize(dev)
        if dd():
            dist.barrier()
        e0 = episodes[0]
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        episodes[0] += reps
        return dt, e0

    g_l = graph_of(layered)
    episodes[0] += 1
    dt_l, _ = timed(g_l)
    g_f = graph_of(fused)
    episodes[0] += 1
    bad_first = None
    g_f.replay()  # (episode e_first, checked below)
    e_first = episodes[0]
    episodes[0] += 1
    torch.cuda.synchronize(dev)
    bad_first, _ = _oracle_check(env, n, base, e_first)
    dt_f, e0 = timed(g_f)
    e_last = episodes[0] - 1
    bad_last, _ = _oracle_check(env, n, base, e_last)
    steps = sum(int(oracle.play_rule_games(n, base, nthreads=8, episode=e)[0]) for e in range(e0, e0 + reps))
    resets = n * reps
    env.close()
    bad = len(bad_first) + len(bad_last)
    if dd():
        dt_f, dt_l = all_reduce([dt_f, dt_l], dist.ReduceOp.MAX)
        steps, resets, bad = (int(x) for x in all_reduce([steps, resets, bad], dist.ReduceOp.SUM))
    assert bad == 0, f"api path: {bad} boards differ from the C oracle"
    alg = steps * BYTES_PER_ENV_STEP + resets * BYTES_PER_RESET
    gbs = alg / dt_f / 1e9
    return {"env_steps_per_s": steps / dt_f, "games_per_s": resets / dt_f,
            "ms_per_batch": dt_f / reps * 1e3, "launches_per_batch": plies + 2,
            "ms_per_batch_three_launches": dt_l / reps * 1e3, "launches_per_batch_three_launches": 3 * plies + 2,
            "env_steps_per_s_three_launches": steps / dt_l,
            "boards": n, "plies_per_batch": plies, "batches_timed": reps,
            "roofline": {"bound": "latency (one launch per ply: a board's ply is one lane's chain)",
                         "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "alg_bytes_per_batch": alg / reps / world,
                         "basis": f"{BYTES_PER_ENV_STEP} B per env step + {BYTES_PER_RESET} B per reset over the "
                                  "replayed graphs' wall time"},
            "parity": f"final states of timed episodes {e0} and {e_last} (and {e_first} before timing): "
                      f"{world * n}/{world * n} boards bit-exact vs C oracle each; env steps = the oracle's "
                      "step counts of the timed episodes",
            "note": "one HIP graph per batch: hz_reset, then per ply hz_rule_ply (get_legal_moves -> rule pick -> "
                    "apply_move in one launch), then hz_score"}


def api_caller_leg(args, dev, rank, world, plies=MAX_PLIES, reps=5):
    """The caller-facing batched loop (harmonies_engine.py:145-298 through
    process_game_state.py:156-179's action index), as a Python caller drives
    it: reset every board with its episode's seed, then per ply
    BatchedEnv.legal_actions() (bool [n, 143], one hz_legal_actions launch)
    -> the caller's own move, chosen OUTSIDE the env kernels with PyTorch ops
    on a device tensor (uniform over the legal moves: a seeded device
    generator's scores, masked, arg-max) -> BatchedEnv.step().  Eager launches
    from a plain Python loop, no host read per ply; `plies` plies per batch
    (finished boards get an empty mask and a no-op).  Every timed batch's
    actions are kept and replayed by the C oracle from the same seeds: final
    states bit-exact, no move rejected, every game over; env steps are the
    moves applied."""
    import numpy as np
    import oracle
    from hzamd.env import BatchedEnv
    from hzamd.state import unpack_ref
    n = args.boards
    base = args.seed_base + rank * n
    env = BatchedEnv(n, seed_base=base, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(20_251 + rank)
    bidx = torch.arange(n, device=dev, dtype=torch.int64)
    acts = torch.full((reps + 1, plies, n), -1, dtype=torch.int16, device=dev)
    finals = torch.zeros(reps + 1, 6, n, dtype=torch.int64, device=dev)
    none = torch.full((n,), -1, dtype=torch.int64, device=dev)

    def batch(r):
        env.reset(seeds=base + bidx + (r << 32))  # episode r of every board
        for p in range(plies):
            legal = env.legal_actions()                        # bool [n, 143] on the device
            score = torch.rand(n, 143, device=dev, generator=gen)
            score.masked_fill_(~legal, -1.0)
            a = torch.where(legal.any(1), score.argmax(1), none)  # the caller's pick
            acts[r, p] = a.to(torch.int16)
            env.step(acts[r, p])
        finals[r] = env.export_state()

    batch(0)  # warm-up (allocator, first launches)
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    t0 = time.perf_counter()
    for r in range(1, reps + 1):
        batch(r)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    a_np = acts.cpu().numpy()
    f_np = finals.cpu().numpy()
    steps, bad, over = 0, 0, 0
    for r in range(1, reps + 1):
        seeds = (base + np.arange(n, dtype=np.uint64) + (np.uint64(r) << np.uint64(32))).astype(np.uint64)
        total, ref, rej = oracle.replay_actions(seeds, a_np[r], nthreads=8)
        got = f_np[r]
        bad += int((rej != 0).sum()) + sum(1 for b in range(n) if not (unpack_ref(got[:, b]) == ref[b]).all())
        over += sum(1 for b in range(n) if oracle.is_game_over(ref[b]))
        steps += int(total)
        assert total == int((a_np[r] >= 0).sum())
    env.close()
    resets = n * reps
    if dd():
        dt = all_reduce([dt], dist.ReduceOp.MAX)[0]
        steps, resets, bad, over = (int(x) for x in all_reduce([steps, resets, bad, over], dist.ReduceOp.SUM))
    assert bad == 0, f"api caller: {bad} boards differ from the C oracle's replay of the same actions"
    assert over == resets, f"api caller: {resets - over} games not over after {plies} plies"
    alg = steps * BYTES_PER_ENV_STEP + resets * BYTES_PER_RESET
    gbs = alg / dt / 1e9
    return {"env_steps_per_s": steps / dt, "games_per_s": resets / dt, "ms_per_batch": dt / reps * 1e3,
            "boards": n, "plies_per_batch": plies, "batches_timed": reps,
            "launches_per_ply": "hz_legal_actions + rand + masked_fill + any + argmax + where + copy + hz_step "
                                "(~8 eager launches)",
            "roofline": {"bound": "launch (a Python loop of ~8 eager launches per ply)",
                         "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "alg_bytes_per_batch": alg / reps / world,
                         "basis": f"{BYTES_PER_ENV_STEP} B per env step + {BYTES_PER_RESET} B per reset over the "
                                  "loop's wall time"},
            "parity": f"every timed batch ({reps} x {world * n} games): the caller's recorded actions replayed by the "
                      "C oracle (or_replay_actions) from the same seeds: final states bit-exact, 0 moves rejected, "
                      "every game over",
            "note": "legal_actions() -> the caller's own choice (PyTorch ops on a device tensor, seeded device "
                    "generator) -> step(), one eager Python loop per batch; the fused rule path is api_path"}


def auto_reset_leg(args, dev, rank, world, plies=MAX_PLIES, warmup=4, launches=40):
    """Config 2 in steady-state auto-reset mode: hz_rollout(plies,
    auto_reset=1) launch after launch, every board starting its next episode
    as soon as a game ends (mid-launch), so every launch plays exactly
    `plies` env steps per board.  Steps and games are counted on the device;
    after the last launch every board's state and game count are checked
    against the C oracle's restatement (or_play_rule_auto) of the whole run."""
    import oracle
    from hzamd.env import BatchedEnv
    from hzamd.state import unpack_ref
    n = args.boards
    base = args.seed_base + rank * n
    env = BatchedEnv(n, seed_base=base, device=dev)
    env.reset()
    # per-launch counters (hz_rollout writes each launch's games / steps)
    games = torch.zeros(warmup + launches, n, dtype=torch.int32, device=dev)
    steps = torch.zeros(warmup + launches, n, dtype=torch.int32, device=dev)
    for i in range(warmup):
        env.rollout(plies, auto_reset=True, games_done=games[i], steps_done=steps[i])
    torch.cuda.synchronize(dev)
    if dd():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + launches):
        env.rollout(plies, auto_reset=True, games_done=games[i], steps_done=steps[i])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    env.check_errors()
    st = env.export_state().cpu().numpy()
    g_all = games.sum(0).cpu().numpy()
    total_games = int(g_all.sum())
    all_steps = int(steps.sum(dtype=torch.int64))
    timed_steps = int(steps[warmup:].sum(dtype=torch.int64))
    timed_games = int(games[warmup:].sum(dtype=torch.int64))
    ref_steps, finals, ref_games, _ = oracle.play_rule_auto(n, base, (warmup + launches) * plies, ep0=0, nthreads=8)
    bad = sum(1 for b in range(n) if not ((unpack_ref(st[:, b]) == finals[b]).all() and g_all[b] == ref_games[b]))
    bad += int(all_steps != ref_steps)
    env.close()
    if dd():
        dt = all_reduce([dt], dist.ReduceOp.MAX)[0]
        timed_steps, timed_games, bad = (int(x) for x in all_reduce([timed_steps, timed_games, bad],
                                                                     dist.ReduceOp.SUM))
    assert bad == 0, f"auto-reset leg: {bad} boards differ from the C oracle"
    alg = timed_steps * BYTES_PER_ENV_STEP + timed_games * BYTES_PER_RESET
    gbs = alg / dt / 1e9
    tr = traffic_rate(traffic_entry(args, "k_rollout<true, false>"), dt / launches)
    return {"env_steps_per_s": timed_steps / dt, "games_per_s": timed_games / dt,
            "ms_per_launch": dt / launches * 1e3, "launches_timed": launches, "plies_per_launch": plies,
            "traffic": tr,
            "boards": n, "kernel": "k_rollout<true, false>",
            "roofline": {"bound": "latency (per-lane chains: plies and in-kernel seeding of the next episode)",
                         "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "alg_bytes_per_launch": alg / launches / world,
                         "basis": f"{BYTES_PER_ENV_STEP} B per env step + {BYTES_PER_RESET} B per game started"},
            "parity": f"after {warmup + launches} launches ({(warmup + launches) * plies} env steps per board, "
                      f"{total_games} games ended on rank 0): {world * n}/{world * n} boards' states and game counts "
                      "bit-exact vs the C oracle's auto-reset restatement",
            "note": "hz_rollout(max_plies, auto_reset=1) continued launch after launch: a board whose game ends "
                    "seeds and starts its next episode in the same launch"}


if __name__ == "__main__":
    main()
