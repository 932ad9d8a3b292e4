"""Drop-in `harmonies_engine` (reference harmonies_engine.py) backed by the
MI355X engine.

HarmoniesGameState keeps the reference's public attributes and methods
(player_boards, tile_bag, available_piles, current_player, tiles_in_hand,
turn_phase, game_over, winner, final_scores; get_legal_moves, apply_move,
_end_turn_actions, scoring, clone, hashing) so trainer.py, evaluation.py and
the UIs run unchanged.  Every rule evaluation — legal moves, placement and
turn transitions, chance draws, habitat scoring — runs as a HIP kernel on a
one-board engine (hzamd.single); chance draws consume Python's global
`random` stream exactly as the reference does.  For throughput use the
batched engine (hzamd.BatchedEnv / hzamd.selfplay) instead of this facade.

Differences from the reference, by design:
  * get_legal_moves returns moves in ascending action-index order (the
    reference returns list(set(...)), whose order depends on PYTHONHASHSEED);
  * states must hold real tiles and reachable stacks; anything else raises
    hzamd.state.NotRepresentable (a ValueError) when a rule is evaluated —
    hashing, equality and cloning accept arbitrary contents as before.
"""
import copy

from constants import *  # noqa: F401,F403  (the reference re-exports them, text_game.py:5)
from constants import (AXIAL_DIRECTIONS, INITIAL_BAG, PILE_SIZE, TILE_TYPES, VALID_HEXES,
                       coordinate_to_index_map)
from hzamd.single import action_to_move, bridge

PLAYER_BOARD_HEX_COUNT = len(VALID_HEXES)
WATER_SCORES = {1: 0, 2: 2, 3: 5, 4: 8, 5: 11, 6: 15}
_PHASES = ("choose_pile", "place_tile_1", "place_tile_2", "place_tile_3")


def get_water_score(length):
    """River length -> points (harmonies_engine.py:18-27)."""
    if length <= 0:
        return 0
    return WATER_SCORES.get(length, WATER_SCORES[6] + (length - 6) * 4)


def get_neighbors(coord):
    """Valid axial neighbours of a hex (harmonies_engine.py:31-43)."""
    if coord not in VALID_HEXES:
        return []
    q, r = coord
    return [(q + dq, r + dr) for dq, dr in AXIAL_DIRECTIONS if (q + dq, r + dr) in VALID_HEXES]


class HarmoniesGameState:
    def __init__(self, initial_state=None):
        if initial_state:
            self.__dict__.update(initial_state)
            return
        self.player_boards = [{}, {}]
        self.tile_bag = INITIAL_BAG.copy()
        self.available_piles = []
        self.current_player = 0
        self.tiles_in_hand = []
        self.turn_phase = "choose_pile"
        self.game_over = False
        self.winner = None
        self.final_scores = [0, 0]
        self._replenish_piles()

    # -- identity (pure Python, accepts arbitrary contents) -------------------
    def get_canonical_tuple(self):
        boards = tuple(tuple((c, tuple(s)) for c, s in sorted(b.items())) for b in self.player_boards[:2])
        return (
            self.current_player,
            self.turn_phase,
            tuple(sorted(self.tiles_in_hand)),
            tuple(tuple(sorted(p)) for p in self.available_piles),
            tuple(sorted(self.tile_bag.items())),
            boards[0],
            boards[1],
        )

    def __hash__(self):
        return hash(self.get_canonical_tuple())

    def __eq__(self, other):
        if not isinstance(other, HarmoniesGameState):
            return NotImplemented
        return self.get_canonical_tuple() == other.get_canonical_tuple()

    def clone(self):
        return copy.deepcopy(self)

    def get_current_player(self):
        return self.current_player

    # -- rules (HIP) ------------------------------------------------------------
    def _replenish_piles(self):
        bridge().replenish(self)

    def _end_turn_actions(self):
        bridge().end_turn(self)

    def get_legal_moves(self):
        return [action_to_move(a) for a in bridge().legal_actions(self)]

    def apply_move(self, move):
        new_state = self.clone()
        phase = new_state.turn_phase
        if phase == "choose_pile":
            if not isinstance(move, int) or not 0 <= move < len(new_state.available_piles):
                raise ValueError(f"Invalid pile index: {move}")
            action = move
        elif isinstance(phase, str) and phase.startswith("place_tile"):
            if not (isinstance(move, tuple) and len(move) == 2 and isinstance(move[0], str)
                    and move[0] in TILE_TYPES and isinstance(move[1], tuple)):
                raise ValueError(f"Invalid move format for placement phase: {move}. Expected (tile_type, (q, r))")
            tile, coord = move
            if coord not in VALID_HEXES:
                raise ValueError(f"Invalid coordinate: {coord}")
            action = 5 + TILE_TYPES.index(tile) * 23 + coordinate_to_index_map[coord]
        else:
            raise ValueError(f"Invalid turn phase: {phase}")
        hand_before = list(new_state.tiles_in_hand)
        status = bridge().step(new_state, action)
        if status == 0:
            return new_state
        if status == 1:
            raise ValueError(f"Invalid pile index: {move}")
        if status == 3:
            raise ValueError(f"Illegal move attempted: Tile '{move[0]}' not found in hand {hand_before}")
        if status == 4:
            hand_after = list(hand_before)
            hand_after.remove(move[0])
            stack = new_state.player_boards[new_state.current_player].get(move[1])
            raise ValueError(f"Illegal move attempted in apply_move: Cannot place {move[0]} on {move[1]} with stack "
                             f"{stack} (Hand was: {hand_after} after removal attempt)")
        raise ValueError(f"Invalid turn phase: {phase}")

    def is_game_over(self):
        return self.game_over and self.winner is not None

    def get_game_outcome(self):
        if not self.is_game_over():
            return None
        return {0: 1, 1: -1}.get(self.winner, 0)

    def _calculate_final_scores(self):
        parts = bridge().score_parts(self)
        self.final_scores[0] = int(parts[0].sum())
        self.final_scores[1] = int(parts[1].sum())

    def _determine_winner(self):
        s0, s1 = self.final_scores
        self.winner = 0 if s0 > s1 else 1 if s1 > s0 else -1

    def calculate_score_for_player(self, player_id):
        return int(bridge().score_parts(self)[player_id].sum())

    def _score_board_part(self, board, k):
        probe = HarmoniesGameState({"player_boards": [board, {}], "tile_bag": INITIAL_BAG.copy(),
                                    "available_piles": [], "current_player": 0, "tiles_in_hand": [],
                                    "turn_phase": "choose_pile", "game_over": False, "winner": None,
                                    "final_scores": [0, 0]})
        return int(bridge().score_parts(probe)[0][k])

    def _score_grass(self, board, player):
        return self._score_board_part(board, 0)

    def _score_mountains(self, board, player):
        return self._score_board_part(board, 1)

    def _score_fields(self, board, player):
        return self._score_board_part(board, 2)

    def _score_buildings(self, board, player):
        return self._score_board_part(board, 3)

    def _score_water(self, board, player):
        return self._score_board_part(board, 4)

    def _get_top_tile(self, board, coord):
        return board.get(coord, [None])[-1]

    def __str__(self):
        lines = [
            "--- Harmonies State (Grid: 5-4-5-4-5 rows) ---",
            f"Player Turn: {self.current_player}, Phase: {self.turn_phase}",
            f"Game Over: {self.is_game_over()}, Winner: {self.winner}, Scores: {self.final_scores}",
            f"Bag: {dict(sorted(self.tile_bag.items()))}",
            f"Available Piles: {self.available_piles}",
            f"Player {self.current_player} Hand: {self.tiles_in_hand}",
        ]
        for p in (0, 1):
            lines.append(f"Player {p} Board ({len(self.player_boards[p])}/{PLAYER_BOARD_HEX_COUNT} hexes):")
            lines.append(f"  { {str(c): s for c, s in sorted(self.player_boards[p].items())} }")
        lines.append("---------------------------------------------")
        return "\n".join(lines) + "\n"


__all__ = ["HarmoniesGameState", "get_neighbors", "get_water_score", "PILE_SIZE", "PLAYER_BOARD_HEX_COUNT"]
