"""Batched evaluation games between two agents.

The reference plays its evaluation games one at a time:
  * Trainer.evaluate_model / play_one_eval_game (trainer.py:293-431): the
    candidate network against the best one, both searching with
    mcts_config_eval (200 sims, no noise, testing=True -> most-visited move),
    the candidate playing P0 in even games; win rate = wins / decisive games
    (0.5 when there are none), promotion when it exceeds the threshold;
  * evaluation.run_tournament / play_game (evaluation.py:7-133): an MCTS agent
    against choose_move_greedy, alternating who plays P0.
Here every game is a board of one BatchedEnv; each ply, the boards whose
player to move belongs to agent A move by A and the others by B.  Two MCTS
agents with the same search settings share one batched search per ply whose
leaf batch is routed row by row to the searching player's network.
"""
import torch

from .env import BatchedEnv
from .mcts import BatchedMCTS, choose_actions

MCTS_EVAL = {  # config.py mcts_config_eval
    "num_simulations": 200, "cpuct": 2, "dirichlet_alpha": 0.1, "dirichlet_epsilon": 0,
    "fpu_value": 0.25, "turns_until_tau0": 0, "action_size": 143, "testing": True,
}


class GreedyAgent:
    """evaluation.choose_move_greedy for a batch of boards (hz_greedy_actions)."""

    def act(self, env, mask, ply):
        return env.greedy_actions(sel=mask).to(torch.int64)


class MctsAgent:
    """get_best_action_and_pi with an evaluator (e.g. BatchedPredictor(model))
    and an evaluation config (deterministic: testing=True, no noise)."""

    def __init__(self, evaluator, mcts_config=None, exact_keys=False, graph=True):
        self.evaluator = evaluator
        # device-row evaluators replay each search's simulation as a HIP graph
        # (BatchedMCTS.search(graph=True)): the arena's batches are launch-bound
        self.graph = graph
        self.cfg = dict(MCTS_EVAL, **(mcts_config or {}))
        if not self.cfg.get("testing", False) or self.cfg.get("dirichlet_epsilon", 0) != 0:
            raise ValueError("arena MctsAgent plays the deterministic evaluation search (testing=True, eps=0)")
        self.exact_keys = exact_keys
        self.mcts = None

    def _search(self, env, mask, evaluator):
        if self.mcts is None or self.mcts.env is not env:
            self.mcts = BatchedMCTS(env, self.cfg["num_simulations"], exact_keys=self.exact_keys)
        v = self.mcts.search(evaluator, self.cfg["cpuct"], active=mask, noise=None, eps=0.0, testing=True,
                             graph=self.graph and env.device.type == "cuda")
        zeros = torch.zeros(env.n, dtype=torch.bool, device=env.device)
        return choose_actions(v, zeros, torch.zeros(env.n, dtype=torch.float64, device=env.device))

    def act(self, env, mask, ply):
        return self._search(env, mask, self.evaluator)


class _Routed:
    """One leaf batch, each row evaluated by its board's searching agent.
    BatchedMCTS gathers the leaves that need the network (device_rows):
    row j belongs to board rows[j], so the agent is picked by rows[j], never
    by the row's position.  When both evaluators take device row counts
    (BatchedPredictor), both run on the whole gathered batch and each row
    keeps its agent's result: no host round trip per simulation (the arena's
    batches are a few dozen rows, so two whole forwards cost what two halves
    do); otherwise the rows are split on the host."""

    device_rows = True

    def __init__(self, eval_a, eval_b, a_rows):
        self.eval_a, self.eval_b, self.a_rows = eval_a, eval_b, a_rows
        self.both_device = bool(getattr(eval_a, "device_rows", False) and getattr(eval_b, "device_rows", False))
        self.capturable = self.both_device and all(getattr(e, "capturable", False) for e in (eval_a, eval_b))
        # agents are picked by rows[j], never by position
        self.row_independent = all(getattr(e, "row_independent", False) for e in (eval_a, eval_b))

    def __call__(self, board, glob, rows=None, count=None):
        if rows is not None and self.both_device:
            pa, va = self.eval_a(board, glob, rows, count)
            pb, vb = self.eval_b(board, glob, rows, count)
            a = self.a_rows.index_select(0, rows.to(torch.int64).clamp(0, self.a_rows.numel() - 1))
            return (torch.where(a.unsqueeze(1), pa.to(torch.float32), pb.to(torch.float32)),
                    torch.where(a, va.reshape(-1).to(torch.float32), vb.reshape(-1).to(torch.float32)))
        if rows is not None:
            k = int(count.item())
            board, glob = board[:k], glob[:k]
            a = self.a_rows.index_select(0, rows[:k].to(torch.int64))
        else:
            a = self.a_rows
        n = board.shape[0]
        policy = torch.zeros(n, 143, dtype=torch.float32, device=board.device)
        value = torch.zeros(n, dtype=torch.float32, device=board.device)
        for idx, ev in ((torch.nonzero(a).flatten(), self.eval_a), (torch.nonzero(~a).flatten(), self.eval_b)):
            if idx.numel():
                p, v = ev(board.index_select(0, idx), glob.index_select(0, idx))
                policy.index_copy_(0, idx, p.to(torch.float32))
                value.index_copy_(0, idx, v.reshape(-1).to(torch.float32))
        return policy, value


def summarize(outcome_a):
    """Counts from agent A's perspective (+1 win, -1 loss, 0 draw/error) and
    the reference's win rate: wins / decisive games, 0.5 if there are none
    (trainer.py:333-338)."""
    o = outcome_a.to(torch.int64).cpu()
    wins, losses = int((o == 1).sum()), int((o == -1).sum())
    draws = int(o.numel() - wins - losses)
    decisive = wins + losses
    return {"wins": wins, "losses": losses, "draws": draws,
            "win_rate": 0.5 if decisive == 0 else wins / decisive}


def play_games(agent_a, agent_b, n_games, seed_base=0, device="cuda", max_plies=200, env=None, first_game=0):
    """Play games first_game .. first_game + n_games - 1 (game g seeded
    seed_base + g); A plays P0 in even games.  Returns (outcome from A's
    perspective int64 [n], final state words [6, n], plies played)."""
    env = env or BatchedEnv(n_games, seed_base=seed_base + first_game, device=device)
    env.reset()
    n, d = env.n, env.device
    a_is_p0 = ((torch.arange(n, device=d) + first_game) % 2) == 0
    shared = (isinstance(agent_a, MctsAgent) and isinstance(agent_b, MctsAgent)
              and agent_a.cfg == agent_b.cfg and agent_a.exact_keys == agent_b.exact_keys)
    ply = 0
    while ply < max_plies:
        done = env.done()
        if bool(done.all()):
            break
        st = env.export_state()
        to_move = (st[5] >> 41) & 1
        a_turn = ((to_move == 0) == a_is_p0) & ~done
        b_turn = ~a_turn & ~done
        if shared:
            act = agent_a._search(env, ~done, _Routed(agent_a.evaluator, agent_b.evaluator, a_turn))
        else:
            act = torch.full((n,), -1, dtype=torch.int64, device=d)
            for agent, mask in ((agent_a, a_turn), (agent_b, b_turn)):
                if bool(mask.any()):
                    act = torch.where(mask, agent.act(env, mask, ply), act)
        act = torch.where(done, torch.full_like(act, -1), act)
        status = env.step(act.to(torch.int16))
        bad = ~done & (status != 0)
        if bool(bad.any()):
            raise RuntimeError(f"arena step failed on boards {torch.nonzero(bad).flatten().tolist()[:8]}")
        ply += 1
    final = env.export_state()
    win = (final[5] >> 46) & 3                          # 1 P0, 2 P1, 3 draw, 0 unfinished
    outcome_p0 = torch.where(win == 1, 1, torch.where(win == 2, -1, 0)).to(torch.int64)
    outcome_a = torch.where(a_is_p0, outcome_p0, -outcome_p0)
    return outcome_a, final, ply


def shard(n_games, rank, world):
    """Games [first, first + count) of rank `rank` when n_games are split
    over `world` ranks as evenly as possible (the first n % world ranks get
    one more)."""
    q, r = divmod(int(n_games), int(world))
    count = q + (1 if rank < r else 0)
    return rank * q + min(rank, r), count


def evaluate_model(candidate_evaluator, best_evaluator, n_games=30, threshold=0.51, mcts_config=None,
                   seed_base=0, device="cuda", group=None):
    """Trainer.evaluate_model (trainer.py:293-375) batched: returns the
    summary from the candidate's perspective plus `passed` (win_rate >
    threshold, i.e. the candidate becomes the best model).

    With torch.distributed initialised the n_games are sharded over the
    ranks (game g is the same game at any world size: seed seed_base + g,
    candidate P0 in even g) and the win/loss/draw counts are all-reduced, so
    every rank returns the same summary and promotion decision."""
    import torch.distributed as dist
    from . import distributed as hd
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    first, count = shard(n_games, rank, world)
    counts = torch.zeros(3, dtype=torch.int64)
    if count:
        cand = MctsAgent(candidate_evaluator, mcts_config)
        best = MctsAgent(best_evaluator, mcts_config)
        outcome, _, _ = play_games(cand, best, count, seed_base=seed_base, device=device, first_game=first)
        o = outcome.cpu()
        counts = torch.tensor([int((o == 1).sum()), int((o == -1).sum()), int((o == 0).sum())])
    if world > 1:
        t = counts.to(hd.collective_device(group))
        dist.all_reduce(t, group=group)
        counts = t.cpu()
    wins, losses, draws = (int(c) for c in counts)
    decisive = wins + losses
    s = {"wins": wins, "losses": losses, "draws": draws, "win_rate": 0.5 if decisive == 0 else wins / decisive}
    s["passed"] = s["win_rate"] > threshold
    return s
