"""Compact board record <-> Python views.

The device record of one board is six u64 words (layout in
csrc/hz_device.hpp).  This module converts it to and from

  * the reference's own Python objects (HarmoniesGameState attributes,
    harmonies_engine.py:66-79) for the drop-in facade, and
  * REFSTATE, a flat int16[78] view (tile ids in TILE_TYPES order, stack codes
    per cell) used by the tests and the golden fixtures.

Pure format conversion: no game rule is evaluated here.
"""
import numpy as np

TILE_TYPES = ["water", "plant", "wood", "stone", "building", "field"]
PHASES = ["choose_pile", "place_tile_1", "place_tile_2", "place_tile_3", "game_over"]
BAG_KEYS = ["water", "plant", "wood", "stone", "field", "building"]  # INITIAL_BAG insertion order
STACKS = [
    (),
    ("water",), ("plant",), ("wood",), ("stone",), ("building",), ("field",),
    ("wood", "plant"), ("stone", "stone"), ("stone", "stone", "stone"),
    ("wood", "building"), ("stone", "building"), ("building", "building"),
]
STACK_CODE = {s: i for i, s in enumerate(STACKS)}
SORTED_COORDS = sorted([
    (-1, -2), (0, -2), (1, -2), (2, -2), (3, -2), (-1, -1), (0, -1), (1, -1), (2, -1),
    (-2, 0), (-1, 0), (0, 0), (1, 0), (2, 0), (-2, 1), (-1, 1), (0, 1), (1, 1),
    (-3, 2), (-2, 2), (-1, 2), (0, 2), (1, 2)])
CELL_OF = {c: i for i, c in enumerate(SORTED_COORDS)}
WORDS = 6
REFSTATE = 78

_M64 = (1 << 64) - 1


class NotRepresentable(ValueError):
    """A Python state the native record cannot hold (e.g. arbitrary tile names)."""


def _winner_code(w):
    return {None: 0, 0: 1, 1: 2, -1: 3}[w]


def _winner_of(code):
    return [None, 0, 1, -1][code]


def pack_ref(v):
    """REFSTATE int16[78] -> six u64 words (as Python ints)."""
    v = [int(x) for x in v]
    pl = [0, 0, 0, 0]
    for p in (0, 1):
        for c in range(23):
            code = v[p * 23 + c]
            for k in range(4):
                if (code >> k) & 1:
                    pl[k] |= 1 << (32 * p + c)
    piles = 0
    for i in range(5):
        for j in range(3):
            t = v[46 + 3 * i + j]
            piles |= (t if t >= 0 else 7) << (9 * i + 3 * j)
    piles |= v[61] << 45
    misc = 0
    for j in range(3):
        t = v[62 + j]
        misc |= (t if t >= 0 else 7) << (3 * j)
    misc |= v[65] << 9
    for t in range(6):
        misc |= v[66 + t] << (11 + 5 * t)
    misc |= v[72] << 41
    misc |= v[73] << 42
    misc |= v[74] << 45
    misc |= _winner_code(None if v[75] == -2 else v[75]) << 46
    misc |= v[76] << 48
    misc |= v[77] << 56
    return pl + [piles, misc]


def unpack_ref(words):
    """six u64 words (ints or a uint64/int64 array) -> REFSTATE int16[78]."""
    w = [int(x) & _M64 for x in words]
    v = np.zeros(REFSTATE, np.int16)
    for p in (0, 1):
        for c in range(23):
            code = 0
            for k in range(4):
                code |= ((w[k] >> (32 * p + c)) & 1) << k
            v[p * 23 + c] = code
    piles = w[4]
    for i in range(5):
        for j in range(3):
            t = (piles >> (9 * i + 3 * j)) & 7
            v[46 + 3 * i + j] = -1 if t == 7 else t
    v[61] = (piles >> 45) & 7
    misc = w[5]
    for j in range(3):
        t = (misc >> (3 * j)) & 7
        v[62 + j] = -1 if t == 7 else t
    v[65] = (misc >> 9) & 3
    for t in range(6):
        v[66 + t] = (misc >> (11 + 5 * t)) & 31
    v[72] = (misc >> 41) & 1
    v[73] = (misc >> 42) & 7
    v[74] = (misc >> 45) & 1
    wn = _winner_of((misc >> 46) & 3)
    v[75] = -2 if wn is None else wn
    v[76] = (misc >> 48) & 255
    v[77] = (misc >> 56) & 255
    return v


def words_to_array(rows):
    """list of 6-int lists -> int64 array [n, 6] (two's complement view)."""
    a = np.array([[x & _M64 for x in r] for r in rows], dtype=np.uint64)
    return a.view(np.int64)


def ref_from_object(g):
    """HarmoniesGameState-like object -> REFSTATE (raises NotRepresentable)."""
    v = np.zeros(REFSTATE, np.int16)
    try:
        for p in (0, 1):
            for coord, stack in g.player_boards[p].items():
                v[p * 23 + CELL_OF[tuple(coord)]] = STACK_CODE[tuple(stack)]
        piles = list(g.available_piles)
        if len(piles) > 5:
            raise NotRepresentable("more than 5 piles")
        v[46:61] = -1
        for i, pile in enumerate(piles):
            if not 1 <= len(pile) <= 3:
                raise NotRepresentable("pile size outside 1..3")
            for j, t in enumerate(pile):
                v[46 + 3 * i + j] = TILE_TYPES.index(t)
        v[61] = len(piles)
        hand = list(g.tiles_in_hand)
        if len(hand) > 3:
            raise NotRepresentable("more than 3 tiles in hand")
        v[62:65] = -1
        for j, t in enumerate(hand):
            v[62 + j] = TILE_TYPES.index(t)
        v[65] = len(hand)
        if list(g.tile_bag.keys()) != BAG_KEYS:
            raise NotRepresentable("tile_bag keys/order differ from INITIAL_BAG")
        for t, name in enumerate(TILE_TYPES):
            cnt = int(g.tile_bag[name])
            if not 0 <= cnt <= 31:
                raise NotRepresentable("bag count outside 0..31")
            v[66 + t] = cnt
        v[72] = int(g.current_player)
        v[73] = PHASES.index(g.turn_phase)
        v[74] = int(bool(g.game_over))
        v[75] = -2 if g.winner is None else int(g.winner)
        for p in (0, 1):
            s = int(g.final_scores[p])
            if not 0 <= s <= 255:
                raise NotRepresentable("score outside 0..255")
            v[76 + p] = s
    except (KeyError, ValueError, TypeError, AttributeError, IndexError) as e:
        if isinstance(e, NotRepresentable):
            raise
        raise NotRepresentable(f"state not representable by the native engine: {e!r}") from e
    return v


def apply_ref_to_object(v, g):
    """Write REFSTATE into a HarmoniesGameState-like object's attributes
    (fresh containers, so previously shared lists/dicts are not mutated)."""
    v = [int(x) for x in v]
    g.player_boards = [{}, {}]
    for p in (0, 1):
        for c in range(23):
            code = v[p * 23 + c]
            if code:
                g.player_boards[p][SORTED_COORDS[c]] = list(STACKS[code])
    g.tile_bag = {name: v[66 + TILE_TYPES.index(name)] for name in BAG_KEYS}
    g.available_piles = []
    for i in range(v[61]):
        g.available_piles.append([TILE_TYPES[t] for t in v[46 + 3 * i: 49 + 3 * i] if t >= 0])
    g.tiles_in_hand = [TILE_TYPES[t] for t in v[62:62 + v[65]]]
    g.current_player = v[72]
    g.turn_phase = PHASES[v[73]]
    g.game_over = bool(v[74])
    g.winner = None if v[75] == -2 else v[75]
    g.final_scores = [v[76], v[77]]
    return g
