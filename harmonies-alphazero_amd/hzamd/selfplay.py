"""Batched self-play: `self_play_worker` (trainer.py:434-541) for n boards at
once on one GPU.

Per ply, for every board still playing: record the state and the player to
move, run get_best_action_and_pi's search (BatchedMCTS, one PyTorch leaf
batch per simulation), choose the move (tau = 1 sampling for the first
`turns_until_tau0` plies unless testing, else the first most-visited move),
apply it (HIP step, chance draws from the board's CPython stream).  When a
board's game ends its examples get z = outcome from the recorded player's
perspective (trainer.py:517-538).

Records stay on the device in compact form: state words int64 [T, 6, n],
player int8 [T, n], visit counts int32 [T, n, 143], valid bool [T, n].
`examples()` turns them into the reference's example tuples
(board f32[38,5,7], glob f32[42], pi f32[143], z f32[1]).
"""
import torch

from . import _native as nat
from .env import BatchedEnv
from .mcts import MAX_CHILDREN, BatchedMCTS, choose_actions, pi_from_visits

MCTS_DEFAULT = {  # config.py:53-65 (the self-play config)
    "num_simulations": 400, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
    "fpu_value": 0.25, "turns_until_tau0": 15, "action_size": 143, "testing": False,
}


class NoiseSource:
    """Root Dirichlet noise (MCTS.py:314-316) and the tau=1 uniforms, drawn on
    the device by hz_root_noise from a counter-based generator keyed by
    (seed, global board id = board_base + b, move counter): a board's draws
    are the same whatever batch it sits in and whatever the GPU count."""

    def __init__(self, board_base, device, seed=0):
        self.board_base = int(board_base)
        self.seed = int(seed)
        self.device = torch.device(device)

    def draw(self, step, counts, alpha):
        n = counts.numel()
        counts = counts.to(device=self.device, dtype=torch.int32).contiguous()
        noise = torch.empty(n, MAX_CHILDREN, dtype=torch.float64, device=self.device)
        u = torch.empty(n, dtype=torch.float64, device=self.device)
        nat.check(nat.lib().hz_root_noise(nat.ptr(counts), n, self.seed & (2**64 - 1),
                                          self.board_base & (2**64 - 1), int(step) & (2**64 - 1), float(alpha),
                                          nat.ptr(noise), nat.ptr(u), nat.stream_ptr(self.device)),
                  "hz_root_noise")
        return noise, u


class SelfPlay:
    def __init__(self, n_boards, evaluator, mcts_config=None, seed_base=0, device="cuda", max_plies=200,
                 env=None, exact_keys=False):
        self.cfg = dict(MCTS_DEFAULT, **(mcts_config or {}))
        self.device = torch.device(device)
        self.env = env or BatchedEnv(n_boards, seed_base=seed_base, device=self.device)
        self.n = self.env.n
        self.evaluator = evaluator
        self.mcts = BatchedMCTS(self.env, self.cfg["num_simulations"], exact_keys=exact_keys)
        self.max_plies = int(max_plies)
        self.noise = NoiseSource(seed_base, self.device)
        self.keep_noise = False
        self.noise_log = []
        self.step_counter = 0
        # move() holds the host back only after its search is queued: the
        # previous move's step status and active-board count come back
        # through a pinned buffer and an event recorded after that step
        self._n_active = self.n  # an upper bound on the active boards (sizes the network's launches) ...
        self._n_active_epoch = -1  # ... while the env's epoch (no game started since) is this
        self._flags = torch.zeros(2, dtype=torch.int64, pin_memory=self.device.type == "cuda")
        self._flags_ev = None
        self._bad_dev = None

    def move(self, ply, done=None, _bound=None):
        """One ply for every board that is still playing: search, choose,
        step.  Returns (state words before the move, visits, active mask).

        A step failure of this move is reported by the next move() or by
        check_steps(): a caller that stops after a move must end with
        check_steps().  `done` (optional) is the caller's finished-board mask;
        the network's launches are then sized for every board, since the
        active-board bound kept from the last step holds only for the env's
        own done() (play() passes its bound for the mask it computed)."""
        env, n, d, cfg = self.env, self.n, self.device, self.cfg
        testing = bool(cfg.get("testing", False))
        if done is None:
            done = env.done()
            bound = self._active_bound()  # done() only shrinks the active set between resets
        else:
            bound = n if _bound is None else int(_bound)
        active = ~done
        st = env.export_state()
        _, count = env.legal_mask()
        noise, u = self.noise.draw(self.step_counter, count, cfg["dirichlet_alpha"])
        self.step_counter += 1
        # the leaf batch holds at most one row per active board: size the
        # network's launches by that (late in the games most boards are done);
        # an upper bound from an earlier move, so no host read waits here
        v = self.mcts.search(self.evaluator, cfg["cpuct"], active=active, noise=noise,
                             eps=cfg["dirichlet_epsilon"], testing=testing, max_rows=max(1, bound))
        self.check_steps()  # the previous move's step, done long before this search runs
        if torch.is_tensor(ply):
            explore = (ply < cfg["turns_until_tau0"]) & (not testing)
        else:
            explore = torch.full((n,), (not testing) and ply < cfg["turns_until_tau0"], dtype=torch.bool, device=d)
        act = choose_actions(v, explore, u)
        if self.keep_noise:
            self.noise_log.append((noise.clone(), u.clone(), act.clone()))
        act = torch.where(active, act, torch.full_like(act, -1)).to(torch.int16)
        status = env.step(act)
        bad = active & (status != 0)
        # read back by the next move (or check_steps()) after its search is queued
        flags = torch.stack([bad.sum(dtype=torch.int64), (~env.done()).sum(dtype=torch.int64)])
        self._flags.copy_(flags, non_blocking=True)
        self._flags_ev = torch.cuda.Event() if d.type == "cuda" else None
        if self._flags_ev is not None:
            self._flags_ev.record()
        self._bad_dev = bad
        self._flags_epoch = env.epoch
        return st, v, active

    def _active_bound(self):
        return self._n_active if self.env.epoch == self._n_active_epoch else self.n

    def check_steps(self):
        """Raise RuntimeError if the last move's env step failed on a board
        (waits for that step only); updates the active-board bound."""
        if self._bad_dev is None:
            return
        if self._flags_ev is not None:
            self._flags_ev.synchronize()
        nbad, nact = (int(x) for x in self._flags.tolist())
        bad, self._bad_dev = self._bad_dev, None
        self._n_active, self._n_active_epoch = nact, self._flags_epoch
        if nbad:
            raise RuntimeError(f"self-play step failed on boards {torch.nonzero(bad).flatten().tolist()[:8]}")

    def play(self, reset=True):
        """Play one game on every board; returns the device records."""
        env, n, d = self.env, self.n, self.device
        if reset:
            env.reset()
        T = self.max_plies
        states = torch.zeros(T, 6, n, dtype=torch.int64, device=d)
        players = torch.zeros(T, n, dtype=torch.int8, device=d)
        visits = torch.zeros(T, n, 143, dtype=torch.int32, device=d)
        valid = torch.zeros(T, n, dtype=torch.bool, device=d)
        done = env.done()
        ply = 0
        while ply < T:
            n_active = int((~done).sum())  # (one host read per ply: the loop stops exactly)
            if n_active == 0:
                break
            self._n_active, self._n_active_epoch = n_active, env.epoch
            st, v, active = self.move(ply, done, _bound=n_active)
            states[ply] = st
            players[ply] = ((st[5] >> 41) & 1).to(torch.int8)
            valid[ply] = active
            visits[ply] = v
            done = env.done()
            ply += 1
        self.check_steps()
        final = env.export_state()
        return {"states": states[:ply], "players": players[:ply], "visits": visits[:ply],
                "valid": valid[:ply], "final": final, "plies": ply}

    def play_steady(self, moves, reset=True, progress=None):
        """Continuous self-play: the reference's self_play_worker
        (trainer.py:434-541) run game after game on every board, `moves`
        moves in all.  A board whose game ended at a move starts its next
        game before the following move (HarmoniesGameState() after
        random.seed(seed_base + b + (k << 32)) for its k-th game, k = 0, 1,
        ... per board: the seeds hz_rollout(auto_reset=1) uses), so every
        board searches at every move and no leaf batch shrinks while games
        end.  Each move's records keep the board's game index; z comes from
        that game's outcome once it has ended (games still running at the
        end give no examples; compact_steady()).  progress(move) is called
        after each move (host side only)."""
        env, n, d = self.env, self.n, self.device
        bidx = torch.arange(n, device=d, dtype=torch.int64)
        base = int(self.env.seed_base)
        game = torch.zeros(n, dtype=torch.int64, device=d)
        ply = torch.zeros(n, dtype=torch.int64, device=d)
        if reset:
            env.reset(seeds=base + bidx)
        M = int(moves)
        states = torch.zeros(M, 6, n, dtype=torch.int64, device=d)
        visits = torch.zeros(M, n, 143, dtype=torch.int32, device=d)
        games = torch.zeros(M, n, dtype=torch.int32, device=d)
        ended = torch.zeros(M, n, dtype=torch.bool, device=d)
        outcome = torch.zeros(M, n, dtype=torch.float32, device=d)
        plies = torch.zeros(M, n, dtype=torch.int16, device=d)
        none = torch.zeros(n, dtype=torch.bool, device=d)
        for m in range(M):
            self._n_active, self._n_active_epoch = n, env.epoch
            st, v, _ = self.move(ply, none, _bound=n)
            states[m] = st
            visits[m] = v
            games[m] = game.to(torch.int32)
            fin = env.export_state()
            over = env.done()
            ended[m] = over
            outcome[m] = torch.where(over, self.outcomes(fin), torch.zeros_like(outcome[m]))
            plies[m] = (ply + 1).to(torch.int16)
            # the boards whose game just ended start their next one (a
            # selected-board reset: nothing moves where over is false)
            game = game + over.to(torch.int64)
            ply = torch.where(over, torch.zeros_like(ply), ply + 1)
            env.reset(sel=over, seeds=base + bidx + (game << 32))
            if progress is not None:
                progress(m)
        self.check_steps()
        players = ((states[:, 5] >> 41) & 1).to(torch.int8)
        return {"states": states, "visits": visits, "players": players, "game": games, "ended": ended,
                "outcome": outcome, "plies": plies, "moves": M}

    def compact_steady(self, rec):
        """play_steady's records of the games that ended inside the run, in
        (move, board) order: as compact() (states, visits, pi, z from the
        recorded player's side, player, board), plus each record's game
        index, and per ended game its length (`lengths`: plies)."""
        M, n, d = rec["moves"], self.n, self.device
        game = rec["game"].to(torch.int64)                         # [M, n]
        K = int(game.max().item()) + 1 if M else 1
        key = game * n + torch.arange(n, device=d).unsqueeze(0)    # (game, board)
        res = torch.zeros(K * n, dtype=torch.float32, device=d)
        has = torch.zeros(K * n, dtype=torch.bool, device=d)
        em = rec["ended"]
        res[key[em]] = rec["outcome"][em]
        has[key[em]] = True
        mask = has[key]                                            # records of ended games
        player = rec["players"].to(torch.float32)
        out = res[key]
        z = torch.where(player == 0, out, -out)
        states = rec["states"].permute(0, 2, 1)[mask]
        visits = rec["visits"][mask]
        board_id = torch.arange(n, device=d).expand(M, n)[mask].to(torch.int32)
        return {"states": states.contiguous(), "visits": visits, "pi": pi_from_visits(visits),
                "z": z[mask].contiguous(), "player": rec["players"][mask], "board": board_id,
                "game": game[mask].to(torch.int32), "lengths": rec["plies"][em].to(torch.int64)}

    @staticmethod
    def outcomes(final):
        """get_game_outcome per board (+1 P0 won, -1 P1 won, 0 draw)."""
        win = (final[5] >> 46) & 3
        return torch.where(win == 1, 1, torch.where(win == 2, -1, 0)).to(torch.float32)

    def compact(self, rec):
        """Flatten the valid records: states int64 [M, 6], visits int32
        [M, 143], pi f32 [M, 143], z f32 [M] (trainer.py:517-538), player
        int8 [M], board id int32 [M]."""
        out = self.outcomes(rec["final"])                       # [n]
        T = rec["plies"]
        mask = rec["valid"]                                      # [T, n]
        player = rec["players"].to(torch.float32)
        z = torch.where(player == 0, out.unsqueeze(0), -out.unsqueeze(0))  # 0 stays 0 for draws
        states = rec["states"].permute(0, 2, 1)[mask]            # [M, 6]
        visits = rec["visits"][mask]
        pi = pi_from_visits(visits)                              # [M, 143]
        board_id = torch.arange(self.n, device=self.device).expand(T, self.n)[mask].to(torch.int32)
        return {"states": states.contiguous(), "visits": visits, "pi": pi, "z": z[mask].contiguous(),
                "player": rec["players"][mask], "board": board_id}

    def iteration(self, buffer=None, group=None, timings=None):
        """One self-play phase: every board plays a game; with torch.distributed
        initialised the packed records of all ranks are all-gathered (RCCL)
        into `buffer` (a distributed.ReplayBuffer) on every rank, in rank
        order.  timings (a dict, optional) gets "play_s" and "exchange_s"
        (device-synchronised; the exchange starts after a barrier)."""
        from . import distributed as hd
        import time
        import torch.distributed as dist
        t0 = time.perf_counter()
        rec = self.play()
        comp = self.compact(rec)
        packed = hd.pack_records(comp["states"], comp["visits"], comp["z"], comp["player"])
        distributed = dist.is_available() and dist.is_initialized()
        if timings is not None:
            torch.cuda.synchronize(self.device)
            timings["play_s"] = time.perf_counter() - t0
            timings["own_records"] = packed
            if distributed:
                dist.barrier(group)
        t1 = time.perf_counter()
        out = hd.all_gather_records(packed, group) if distributed else packed
        if buffer is not None:
            buffer.extend(out)
        if timings is not None:
            torch.cuda.synchronize(self.device)
            timings["exchange_s"] = time.perf_counter() - t1
        return out, rec

    def examples(self, compact):
        """The reference's replay-buffer tuples (trainer.py:529-538), on CPU."""
        board, glob = encode_states(compact["states"])
        b, g, p, z = board.cpu(), glob.cpu(), compact["pi"].cpu(), compact["z"].cpu()
        return [(b[i], g[i], p[i], z[i:i + 1]) for i in range(b.shape[0])]


def encode_states(states):
    """create_state_tensors for an int64 [M, 6] array of state words."""
    m = states.shape[0]
    dev = states.device
    board = torch.empty(m, 38, 5, 7, dtype=torch.float32, device=dev)
    glob = torch.empty(m, 42, dtype=torch.float32, device=dev)
    if m:
        st = states.contiguous()
        nat.check(nat.lib().hz_encode_states(nat.ptr(st), 1, 6, None, m, nat.ptr(board), nat.ptr(glob),
                                             nat.stream_ptr(dev)), "hz_encode_states")
    return board, glob
