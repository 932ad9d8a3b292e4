"""Benchmark: BASELINE config 2 — 4096 concurrent boards per GPU, pure env
step / legal_actions / score HIP kernels, bit-exact vs the CPU engine.

One bench step = one batched pass of the env hot path over 4096 boards, a
single hz_play launch: HarmoniesGameState() on every board (CPython-exact
seeding and opening draws), then play to the end of every game (legal mask ->
build-defined splitmix rule pick -> apply_move, incl. chance draws and final
scoring).
Boards are seeded by their global id (rank * 4096 + b), so N GPUs run N
independent shards (weak scaling, no data-path collective).

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
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
MAX_PLIES = 96             # rule games end after 56-72 plies
PIPELINE_DEPTH = 4         # hz_play launches until every board replays a fully prepared episode


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--boards", type=int, default=4096)
    ap.add_argument("--seed-base", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-off-compare", action="store_true",
                    help="skip the chance-ahead-off comparison run (profiling)")
    ap.add_argument("--api-mode", action="store_true",
                    help="also time the unfused per-ply API path (legal_mask/rule/step launches)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_traffic.json"))
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5],
                    help="2: env kernels (default, the headline); 3: MCTS self-play moves with the network; "
                         "5: whole training iterations (self-play -> buffer -> training -> arena)")
    ap.add_argument("--iterations", type=int, default=2, help="config 5: training iterations timed")
    ap.add_argument("--eval-games", type=int, default=32, help="config 5: arena games per evaluation")
    ap.add_argument("--sims", type=int, default=200, help="config 3: MCTS simulations per move")
    ap.add_argument("--nn-dtype", default="fp32", choices=["fp32", "bf16"], help="config 3 leaf-eval dtype")
    ap.add_argument("--full-game", action="store_true",
                    help="config 3: time one complete game on every board (games/s measured, not estimated)")
    return ap.parse_args()


_RED_DEV = None  # device of reduction tensors: the GPU under RCCL, the CPU under gloo


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


def bench_loop(args, dev, rank, world):
    """BASELINE config 5: the reference's main.py loop (trainer.Trainer) on
    the batched engine, one step = one training iteration: `boards` games per
    rank of self-play with the best model (MCTS `sims` per move, self-play
    noise), RCCL all-gather of the records into every rank's replay buffer,
    rank-0 training (reference training config: Adam, batch 64, 2 epochs over
    the buffer, buffer 50,000), weight broadcast, checkpoint, buffer file, and
    every iteration an arena of `eval_games` games between candidate and best
    (mcts_config_eval with `sims` simulations).  Reports games/hour."""
    import tempfile
    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    from hzamd.trainer import Trainer
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    model_cfg = dict(DEFAULT, board_size=(5, 7))
    train_cfg = {"device": str(dev), "optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 0.0001,
                 "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64, "momentum": 0.9,
                 "use_scheduler": True, "scheduler_type": "StepLR", "scheduler_step_size": 30,
                 "scheduler_gamma": 0.5, "force_lr_reset_on_load": False, "new_forced_lr": 0.000125}
    mcts_cfg = {"num_simulations": args.sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
                "fpu_value": 0.25, "turns_until_tau0": 15, "action_size": 143, "testing": False}
    tmp = tempfile.mkdtemp(prefix=f"hz_loop_r{rank}_")
    sp_cfg = {"num_iterations": args.iterations + 1, "num_games_per_iter": args.boards, "epochs_per_iter": 2,
              "replay_buffer_size": 50000, "checkpoint_folder": os.path.join(tmp, "ck"),
              "replay_buffer_folder": os.path.join(tmp, "buf"), "replay_buffer_filename": "replay_buffer.pkl",
              "eval_frequency": 1, "eval_episodes": args.eval_games, "eval_win_rate_threshold": 0.51,
              "best_model_filename": "best_model.pth.tar"}
    mm = ModelManager(model_cfg, train_cfg)
    tr = Trainer(mm, mcts_cfg, sp_cfg, train_cfg, eval_mcts_config={"num_simulations": args.sims},
                 seed_base=args.seed_base, log=lambda *_: None)
    # warm-up iteration (kernels, MIOpen algorithm search), then the timed ones
    tr.iteration = 0
    tr.execute_self_play_phase(tr.best_model_manager)
    tr.execute_training_phase()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    phases = {"self_play": 0.0, "training": 0.0, "evaluation": 0.0}
    games = 0
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
        tr.evaluate_model()
        torch.cuda.synchronize(dev)
        d = time.perf_counter()
        phases["self_play"] += b - a
        phases["training"] += c - b
        phases["evaluation"] += d - c
        games += sp["games"]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    if rank == 0:
        print(json.dumps({
            "metric": "full loop self-play games/hour (self-play -> buffer -> training -> arena)",
            "value": games / elapsed * 3600.0, "unit": "games/hour", "n_gpus": world, "steps": args.iterations,
            "warmup": 1, "ms_per_step": elapsed * 1000.0 / args.iterations, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic: random-init network, seeded games",
            "config": {"workload": f"config5: {args.boards} games/rank/iteration, {args.sims} sims/move, "
                                   f"arena {args.eval_games} games every iteration, default 128fx8 net",
                       "boards_per_gpu": args.boards, "sims": args.sims, "parallelism": f"shard{world}"},
            "phase_seconds": phases, "games": games,
        }))


def bench_selfplay(args, dev, rank, world):
    """BASELINE config 3: 4096 boards x `sims` MCTS simulations per move with
    the default 128-filter x 8-block network (random init, torch.manual_seed(0),
    BatchedPredictor = ModelManager.predict batched).  One step = one move of
    every board (full search + choice + env step)."""
    from hzamd.mcts import BatchedPredictor
    from hzamd.net import HarmoniesNet, flops_per_eval
    from hzamd.selfplay import SelfPlay
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    net = HarmoniesNet().to(dev).eval()
    dtype = torch.bfloat16 if args.nn_dtype == "bf16" else None
    pred = BatchedPredictor(net, dtype=dtype)
    nn_ev = []

    def evaluator(board, glob):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = pred(board, glob)
        b.record()
        nn_ev.append((a, b))
        return out

    n = args.boards
    cfg = {"num_simulations": args.sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
           "turns_until_tau0": 15, "testing": False}
    sp = SelfPlay(n, evaluator, cfg, seed_base=args.seed_base + rank * n, device=dev)
    if args.full_game:
        return bench_selfplay_games(args, sp, nn_ev, dev, rank, world)
    sp.env.reset()
    for w in range(args.warmup):
        sp.move(w)
    torch.cuda.synchronize(dev)
    nn_ev.clear()
    edges = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        _, v, active = sp.move(args.warmup + k)
        edges += int(sp.mcts.stats()[:, 1].sum().item())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nn_ms = sum(a.elapsed_time(b) for a, b in nn_ev)
    sims_done = n * args.sims * args.steps
    if world > 1:
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    sims_all = sims_done * world
    per_move = elapsed / args.steps
    avg_plies = 62.4  # mean game length
    fl = flops_per_eval()
    if rank == 0:
        print(json.dumps({
            "metric": "self-play MCTS simulations/sec (= NN leaf evals/s) @4096 boards x 200 sims",
            "value": sims_all / elapsed, "unit": "sims/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": per_move * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.nn_dtype, "data": "synthetic: random-init network, seeded games",
            "config": {"workload": f"config3: {n} boards x {args.sims} sims/move, default 128fx8 net",
                       "boards_per_gpu": n, "sims": args.sims, "parallelism": f"shard{world}"},
            "games_per_s_est": world * n / (per_move * avg_plies),
            "env_steps_per_s": (edges + n * args.steps) * world / elapsed,
            "nn_ms_per_move": nn_ms / args.steps, "tree_ms_per_move": per_move * 1e3 - nn_ms / args.steps,
            "nn_tflops": fl * n * args.sims * args.steps / (nn_ms * 1e-3) / 1e12,
            "note": "games/s estimated from ms per move x mean game length 62.4 plies",
        }))


def bench_selfplay_games(args, sp, nn_ev, dev, rank, world):
    """Config 3, measured end to end: after `warmup` moves of a throw-away
    game, every board plays one whole self-play game (search + choice + env
    step per ply, records kept on the device as SelfPlay.play does); games/s
    = boards of all ranks / the slowest rank's time."""
    from hzamd.net import flops_per_eval
    n = sp.n
    sp.env.reset()
    for w in range(args.warmup):
        sp.move(w)
    torch.cuda.synchronize(dev)
    nn_ev.clear()
    plies = [0]
    orig_move = sp.move

    def move(ply, done=None):  # progress on stderr (a long run must not look hung)
        out = orig_move(ply, done)
        plies[0] = ply + 1
        if ply % 8 == 0:
            print(f"[config3 full game] ply {ply}", file=sys.stderr, flush=True)
        return out

    sp.move = move
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rec = sp.play(reset=True)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    sp.move = orig_move
    evals = int(rec["valid"].sum().item()) * args.sims
    nn_ms = sum(a.elapsed_time(b) for a, b in nn_ev)
    if world > 1:
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
    if rank == 0:
        print(json.dumps({
            "metric": "self-play games/sec @4096 boards x 200 MCTS sims (complete games, measured)",
            "value": world * n / elapsed, "unit": "games/s", "n_gpus": world, "steps": 1, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.nn_dtype, "data": "synthetic: random-init network, seeded games",
            "config": {"workload": f"config3: {n} boards x {args.sims} sims/move, one whole game per board",
                       "boards_per_gpu": n, "sims": args.sims, "parallelism": f"shard{world}"},
            "plies": rec["plies"], "moves": int(rec["valid"].sum().item()),
            "sims_per_s": world * evals / elapsed, "nn_s": nn_ms * 1e-3,
            "nn_tflops": flops_per_eval() * n * args.sims * len(nn_ev) / args.sims / (nn_ms * 1e-3) / 1e12
            if nn_ms else None,
        }))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HZ_BENCH_REHEARSAL=1 (tests only): ranks share the visible GPUs
    # (local % device_count) and reduce over gloo, to exercise the N > 1 path
    # on a one-GPU box; the real multi-GPU run uses one GPU per rank and RCCL
    rehearsal = os.environ.get("HZ_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    global _RED_DEV
    _RED_DEV = "cpu" if rehearsal else dev
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if args.config == 5:
        bench_loop(args, dev, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config == 3:
        bench_selfplay(args, dev, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return

    from hzamd.env import BatchedEnv

    n = args.boards
    env = BatchedEnv(n, seed_base=args.seed_base + rank * n, device=dev)
    games = torch.zeros(n, dtype=torch.int32, device=dev)
    steps = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def one_step(ev=None, g=games, s=steps):
        # hz_play: HarmoniesGameState() on every board fused with rule-driven
        # play to the end of the game, one launch
        if ev:
            ev[0].record(stream)
        env.rollout(MAX_PLIES, games_done=g, steps_done=s, reset=True)
        if ev:
            ev[1].record(stream)

    # first batch (episode 0: board b seeded seed_base + rank*n + b) doubles as
    # the parity guard: its env-step count must equal the C oracle's
    one_step()
    torch.cuda.synchronize(dev)
    first_steps = int(steps.sum().item())
    # the chance-ahead pipeline (seed -> draw1 -> draw2 -> play) is primed
    # after three launches; fewer warm-up steps than that get extra untimed
    # priming launches, reported as pipeline_prime
    prime = max(0, PIPELINE_DEPTH - args.warmup)
    for _ in range(max(0, args.warmup - 1) + prime):
        one_step()
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    # per-step counters of the timed launches (each step plays a new episode)
    games_t = torch.zeros(args.steps, n, dtype=torch.int32, device=dev)
    steps_t = torch.zeros(args.steps, n, dtype=torch.int32, device=dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(None, games_t[i], steps_t[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the dominant kernel's average launch duration, from HIP events around
    # each launch on its stream, in a separate loop of the same launches (the
    # event markers would otherwise sit between the timed launches)
    for i in range(args.steps):
        one_step(evs[i], games, steps)
    torch.cuda.synchronize(dev)
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    timed_steps, timed_games = int(steps_t.sum(dtype=torch.int64)), int(games_t.sum(dtype=torch.int64))
    if world > 1:
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
        c = all_reduce([timed_steps, timed_games], dist.ReduceOp.SUM)
        env_steps_all, games_all = int(c[0]), int(c[1])
    else:
        env_steps_all, games_all = timed_steps, timed_games

    value = env_steps_all / elapsed
    games_per_s = games_all / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps

    # roofline of the dominant kernel (hz_play = k_rollout with reset), per launch
    alg_bytes = (timed_steps * BYTES_PER_ENV_STEP + timed_games * BYTES_PER_RESET) / args.steps
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get("k_rollout_bytes_per_launch")
        except Exception:
            traffic = None

    # the same workload with chance-ahead off (every launch seeds and draws
    # in-kernel), for comparison; not the headline number
    off_steps, off_elapsed = 0, float("nan")
    if not args.no_off_compare:
        off_steps, off_elapsed = off_compare(env, one_step, games, args, dev, world)

    api = None
    if args.api_mode and rank == 0:
        api = api_mode(env, dev, stream)
    enc = encoder_roofline(dev, n, args.seed_base) if rank == 0 else None

    if rank == 0:
        import oracle  # test infrastructure: parity guard + cpu_baseline only
        ref_total = oracle.play_rule_games(n, args.seed_base, nthreads=8)[0]
        assert ref_total == first_steps, (ref_total, first_steps)
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(n, args.cpu_seconds)
        out = {
            "metric": "self-play env-steps/sec + games/sec @4096 boards, 1/2/4/8 GPUs; bit-exact vs CPU",
            "value": value,
            "unit": "env-steps/s",
            "games_per_s": games_per_s,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: CPython-seeded games, seeds = global board id, build-defined splitmix rule policy",
            "config": {"workload": "config2: 4096 concurrent boards/GPU, reset + rule-driven play to game end "
                                   "(legal mask, step, chance draws, final scoring), one hz_play launch",
                       "boards_per_gpu": n, "env_steps_per_step": timed_steps / args.steps,
                       "games_per_step": timed_games / args.steps, "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_rollout", "kernel_ms": kern_ms,
                         "alg_bytes_per_launch": alg_bytes},
            "chance_ahead": {"on": True, "note": "each hz_play also prepares every board's next three episodes "
                                                 "as a pipeline on the other CUs (stream seeding, pile draws and "
                                                 "rule hashes, none of which depends on moves); steady state: one "
                                                 "preparation per game in the timed region",
                             "pipeline_prime": prime,
                             "value_off": (off_steps / off_elapsed) if off_steps else None,
                             "ms_per_step_off": (off_elapsed * 1000.0 / args.steps) if off_steps else None},
            "encoder_roofline": enc,
            "cpu_baseline": cpu,
            "parity": f"first batch: {first_steps} env steps == C oracle ({ref_total})",
        }
        if api:
            out["api_path"] = api
        print(json.dumps(out))
    env.close()
    if world > 1:
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


def off_compare(env, one_step, games, args, dev, world):
    """Time the same workload with chance-ahead off (every launch seeds and
    draws in-kernel); returns (env steps of all ranks, max elapsed)."""
    env.set_seed_ahead(False)
    for _ in range(2):
        one_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    steps_o = torch.zeros(args.steps, env.n, dtype=torch.int32, device=dev)
    t1 = time.perf_counter()
    for i in range(args.steps):
        one_step(None, games, steps_o[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t1
    total = int(steps_o.sum(dtype=torch.int64))
    if world > 1:
        elapsed = all_reduce([elapsed], dist.ReduceOp.MAX)[0]
        total = int(all_reduce([total], dist.ReduceOp.SUM)[0])
    env.set_seed_ahead(True)
    return total, elapsed


def api_mode(env, dev, stream, plies=MAX_PLIES, reps=5):
    """Unfused path: per ply hz_legal_mask + hz_rule_actions + hz_step
    (3 launches), then hz_score — captured once into a HIP graph."""
    n = env.n
    mask = torch.zeros(n, 3, dtype=torch.int64, device=dev)
    count = torch.zeros(n, dtype=torch.int32, device=dev)
    act = torch.zeros(n, dtype=torch.int16, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)

    def body():
        env.reset()
        for _ in range(plies):
            env.legal_mask(mask, count)
            env.rule_actions(mask, count, act)
            env.step(act, status)
        env.score()

    body()
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"ms_per_batch": dt * 1e3, "launches_per_batch": 3 * plies + 2,
            "note": "graph-captured per-ply launches over a 4096-board batch", "boards": n}


if __name__ == "__main__":
    main()
