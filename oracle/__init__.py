"""CPU oracle for the Harmonies hot path — TEST INFRASTRUCTURE ONLY.

A C restatement (oracle/hz_oracle.c) of the reference engine
(harmonies_engine.py), encoder (process_game_state.py) and MCTS (MCTS.py),
pinned by fixtures captured from the reference itself (tests/golden/).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product (harmonies-alphazero_amd/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

REFSTATE = 78


class MT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("idx", ctypes.c_int32)]

    def words(self):
        return np.ctypeslib.as_array(self.mt).copy(), int(self.idx)


class MctsCfg(ctypes.Structure):
    _fields_ = [("sims", ctypes.c_int32), ("cpuct", ctypes.c_float), ("eps", ctypes.c_double),
                ("testing", ctypes.c_int32), ("tau0", ctypes.c_int32), ("ply", ctypes.c_int32),
                ("u", ctypes.c_double), ("exact_keys", ctypes.c_int32), ("negate_value", ctypes.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.POINTER
        L.or_mt_seed.argtypes = [P(MT), ctypes.c_uint64]
        L.or_mt_next32.argtypes = [P(MT)]
        L.or_mt_next32.restype = ctypes.c_uint32
        L.or_randbelow.argtypes = [P(MT), ctypes.c_uint32]
        L.or_randbelow.restype = ctypes.c_uint32
        L.or_sample.argtypes = [P(MT), ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.or_reset.argtypes = [P(MT), ctypes.c_void_p]
        L.or_legal.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_legal.restype = ctypes.c_int
        L.or_step.argtypes = [ctypes.c_void_p, ctypes.c_int, P(MT)]
        L.or_step.restype = ctypes.c_int
        L.or_score_board.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_is_game_over.argtypes = [ctypes.c_void_p]
        L.or_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.or_canonical.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.or_rule.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_rule.restype = ctypes.c_uint64
        L.or_play_rule_games.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.or_play_rule_games.restype = ctypes.c_int64
        L.or_play_rule_games_ep.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.or_play_rule_games_ep.restype = ctypes.c_int64
        L.or_play_rule_auto.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.or_play_rule_auto.restype = ctypes.c_int64
        L.or_replay_actions.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.or_replay_actions.restype = ctypes.c_int64
        L.or_mcts_search.argtypes = [ctypes.c_void_p, P(MT), P(MctsCfg), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.or_mcts_search.restype = ctypes.c_int
        L.or_stub_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def mt_seed(seed):
    m = MT()
    lib().or_mt_seed(ctypes.byref(m), ctypes.c_uint64(seed))
    return m


def mt_from_words(words, idx):
    m = MT()
    for i in range(624):
        m.mt[i] = int(words[i])
    m.idx = int(idx)
    return m


def mt_next32(m):
    return lib().or_mt_next32(ctypes.byref(m))


def sample(m, n, k):
    out = np.zeros(3, np.int32)
    lib().or_sample(ctypes.byref(m), n, k, _p(out))
    return out[:k]


def reset(m):
    st = np.zeros(REFSTATE, np.int16)
    lib().or_reset(ctypes.byref(m), _p(st))
    return st


def legal(st):
    st = np.ascontiguousarray(st, np.int16)
    mask = np.zeros(143, np.uint8)
    lib().or_legal(_p(st), _p(mask))
    return mask


def step(st, action, m):
    """Returns (status, new_state).  State unchanged on a non-zero status."""
    st = np.array(st, np.int16, copy=True)
    r = lib().or_step(_p(st), int(action), ctypes.byref(m))
    return r, st


def greedy_move(st, m):
    """choose_move_greedy's action index (consumes m like the reference)."""
    st = np.ascontiguousarray(st, np.int16)
    return lib().or_greedy_move(_p(st), ctypes.byref(m))


def score_board(cells23):
    cells = np.ascontiguousarray(cells23, np.uint8)
    out = np.zeros(5, np.int32)
    lib().or_score_board(_p(cells), _p(out))
    return out


def is_game_over(st):
    st = np.ascontiguousarray(st, np.int16)
    return bool(lib().or_is_game_over(_p(st)))


def encode(st):
    st = np.ascontiguousarray(st, np.int16)
    b = np.zeros((38, 5, 7), np.float32)
    g = np.zeros(42, np.float32)
    lib().or_encode(_p(st), _p(b), _p(g))
    return b, g


def canonical(st, pyhash=False):
    st = np.ascontiguousarray(st, np.int16)
    k = np.zeros(128, np.uint8)
    lib().or_canonical(_p(st), _p(k), int(bool(pyhash)))
    return k.tobytes()


def rule(seed, ply):
    return lib().or_rule(ctypes.c_uint64(seed), ctypes.c_uint64(ply))


def play_rule_games(n, seed_base, nthreads=0, episode=0):
    """Every board b plays its episode-`episode` game (seed = seed_base + b +
    (episode << 32)) with the build-defined rule policy to the end."""
    finals = np.zeros((n, REFSTATE), np.int16)
    plies = np.zeros(n, np.int32)
    nxt = np.zeros(n, np.uint32)
    total = lib().or_play_rule_games_ep(n, ctypes.c_uint64(seed_base), int(episode), _p(finals), _p(plies),
                                        _p(nxt), nthreads)
    return total, finals, plies, nxt


def play_rule_auto(n, seed_base, plies, ep0=0, nthreads=0):
    """hz_rollout(auto_reset) restated: every board plays `plies` rule-driven
    env steps from episode ep0's reset, starting its next episode whenever a
    game ends.  Returns (steps, finals [n, 78], games ended [n], episode [n])."""
    finals = np.zeros((n, REFSTATE), np.int16)
    games = np.zeros(n, np.int32)
    ep = np.zeros(n, np.int32)
    total = lib().or_play_rule_auto(n, ctypes.c_uint64(seed_base), int(ep0), int(plies), _p(finals), _p(games),
                                    _p(ep), nthreads)
    return total, finals, games, ep


def replay_actions(seeds, actions, nthreads=0):
    """Every board b reset after random.seed(seeds[b]) and then given
    actions[p, b] for each ply p (negative = no-op; a rejected move leaves
    the state unchanged).  Returns (moves applied, finals [n, 78], rejected
    moves per board [n])."""
    seeds = np.ascontiguousarray(seeds, np.uint64)
    actions = np.ascontiguousarray(actions, np.int16)
    plies, n = actions.shape
    assert seeds.shape == (n,)
    finals = np.zeros((n, REFSTATE), np.int16)
    rejected = np.zeros(n, np.int32)
    total = lib().or_replay_actions(n, _p(seeds), plies, _p(actions), _p(finals), _p(rejected), nthreads)
    return total, finals, rejected


def mcts_search(st, m, sims, cpuct, eps=0.25, testing=True, tau0=15, ply=0, u=0.0, noise=None,
                exact_keys=False, negate_value=False):
    st = np.ascontiguousarray(st, np.int16)
    cfg = MctsCfg(sims, cpuct, eps, int(bool(testing)), tau0, ply, u, int(bool(exact_keys)),
                  int(bool(negate_value)))
    nz = np.zeros(143, np.float64) if noise is None else np.ascontiguousarray(noise, np.float64)
    visits = np.zeros(143, np.int32)
    nn = ctypes.c_int32(0)
    ne = ctypes.c_int32(0)
    a = lib().or_mcts_search(_p(st), ctypes.byref(m), ctypes.byref(cfg), _p(nz), _p(visits),
                             ctypes.byref(nn), ctypes.byref(ne))
    return a, visits, nn.value, ne.value


def stub_eval(st):
    st = np.ascontiguousarray(st, np.int16)
    pol = np.zeros(143, np.float32)
    val = ctypes.c_double(0)
    lib().or_stub_eval(_p(st), _p(pol), ctypes.byref(val))
    return pol, val.value
