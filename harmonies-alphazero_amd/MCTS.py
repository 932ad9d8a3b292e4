"""Drop-in `MCTS` (reference MCTS.py) backed by the batched HIP search.

get_best_action_and_pi(game_state, model_manager, mcts_config,
game_move_number) keeps the reference signature and contract
(MCTS.py:272-441): it runs mcts_config["num_simulations"] PUCT simulations
from game_state with model_manager.predict(board, glob) as the leaf
evaluator and returns (move, pi) with pi a float64 array over 143 actions.
The tree, selection, expansion (including chance draws from Python's global
`random` stream), backup and visit counting run as HIP kernels on a one-board
search; root Dirichlet noise and tau = 1 sampling draw from numpy's global
stream like the reference (np.random.dirichlet / np.random.choice).

Moves are expanded in ascending action-index order; the reference uses
set iteration order (PYTHONHASHSEED-dependent), see DESIGN.md.  For
thousands of concurrent games use hzamd.mcts.BatchedMCTS / hzamd.selfplay.
"""
import os
import random

import numpy as np
import torch

from hzamd.mcts import BatchedMCTS
from hzamd.single import action_to_move, bridge
from process_game_state import get_action_index


class Node:
    """Tree node record (MCTS.py:8-20); the search itself lives on the GPU."""

    def __init__(self, state):
        self.state = state
        self.current_player = state.current_player
        self.id = hash(state)
        self.edges = {}

    def is_leaf(self):
        return len(self.edges) == 0


class Edge:
    """Tree edge record (MCTS.py:23-39)."""

    def __init__(self, in_node, out_node, prior, action):
        self.in_node = in_node
        self.out_node = out_node
        self.current_player = in_node.current_player
        self.action = action
        self.stats = {"N": 0, "W": 0, "Q": 0, "P": prior}


class MCTS:
    """Name kept for imports (profile_self_play.py:12); searches run through
    get_best_action_and_pi or hzamd.mcts.BatchedMCTS."""

    def __init__(self, root_node, mcts_config):
        self.root = root_node
        self.mcts_config = mcts_config
        self.tree = {root_node.id: root_node}

    def __len__(self):
        return len(self.tree)

    def add_node(self, node):
        self.tree[node.id] = node

    def get_root_edges(self):
        return self.root.edges


_SEARCH = {}
# simulations 2.. of a search replay one captured HIP graph, kept across moves
# while the network's weights do not change (hzamd.mcts.BatchedMCTS.search);
# taken only with hzamd's ModelManager (the device-row evaluator);
# HZ_DROPIN_GRAPH=0 runs every simulation eagerly (A/B measurements)
GRAPH = os.environ.get("HZ_DROPIN_GRAPH", "1") != "0"


def _search_for(sims):
    br = bridge()
    s = _SEARCH.get(sims)
    if s is None:
        _SEARCH.clear()
        s = _SEARCH[sims] = BatchedMCTS(br.env, sims)
    return s


class _PredictAdapter:
    """Batch-of-one evaluator calling model_manager.predict (model.py:81-110)."""

    def __init__(self, model_manager, device):
        self.mm = model_manager
        self.device = device

    def __call__(self, board, glob):
        pol, val = self.mm.predict(board[0].cpu(), glob[0].cpu())
        p = torch.as_tensor(np.asarray(pol, dtype=np.float32), device=self.device).reshape(1, -1)
        v = torch.tensor([float(val)], dtype=torch.float32, device=self.device)
        return p, v


class _FoldedRows:
    """hzamd.manager.ModelManager.predict's own computation (the folded HIP
    network, softmax) on the device-row protocol: the leaf stays on the GPU,
    no host round trip per simulation.  Used only for that ModelManager; any
    other model manager goes through its predict()."""

    device_rows = True
    capturable = True  # HIP kernels + PyTorch ops only: one simulation is replayed as a HIP graph
    row_independent = True  # each row computed on its own (arrival-order leaf batches are fine)

    def __init__(self, folded):
        self.f = folded

    @property
    def graph_key(self):  # the captured simulation stays valid for this network generation
        return self.f, self.f.generation

    def __call__(self, board, glob, rows=None, count=None):
        return self.f.predict(board, glob, live=count)


def _evaluator(model_manager, device):
    fast = getattr(model_manager, "_fast", None)
    f = fast() if callable(fast) else None
    return _FoldedRows(f) if f is not None else _PredictAdapter(model_manager, device)


def get_best_action_and_pi(game_state, model_manager, mcts_config, game_move_number):
    br = bridge()
    sims = int(mcts_config["num_simulations"])
    testing = bool(mcts_config.get("testing", False))
    action_size = int(mcts_config["action_size"])
    search = _search_for(sims)
    br.load(game_state, rng=True)
    legal = br.legal_current()
    terminal = game_state.is_game_over()
    noise = None
    if not testing and not terminal and legal and sims > 0:
        vec = np.random.dirichlet([mcts_config["dirichlet_alpha"]] * len(legal))  # MCTS.py:314-316
        noise = torch.zeros(1, 69, dtype=torch.float64)
        noise[0, :len(vec)] = torch.from_numpy(np.asarray(vec, dtype=np.float64))
    visits = search.search(_evaluator(model_manager, br.device), float(mcts_config["cpuct"]),
                           noise=noise, eps=float(mcts_config["dirichlet_epsilon"]), testing=testing,
                           graph=GRAPH)
    v = visits[0].cpu().numpy().astype(np.int64)
    br.store_rng()

    # root edges exist once the root was expanded, in ascending action order
    root_actions = legal if (sims > 0 and not terminal) else []
    total = int(sum(v[a] for a in root_actions))
    pi = np.zeros(action_size, dtype=int)  # MCTS.py:356-358
    for a in root_actions:
        pi[a] = v[a]
    if total > 0:
        pi = pi / total
    best = None
    if (not testing) and game_move_number < mcts_config["turns_until_tau0"]:
        if total > 0:
            probs = np.array([v[a] for a in root_actions], dtype=float) / total
            best = action_to_move(root_actions[np.random.choice(len(root_actions), p=probs)])
    else:
        max_visits = -1
        for a in root_actions:
            if v[a] > max_visits:
                max_visits, best = v[a], action_to_move(a)
    if best is None:  # MCTS.py:425-439
        moves = [action_to_move(a) for a in legal]
        if not moves:
            return None, pi
        best = random.choice(moves)
    return best, pi


__all__ = ["Node", "Edge", "MCTS", "get_best_action_and_pi", "get_action_index"]
