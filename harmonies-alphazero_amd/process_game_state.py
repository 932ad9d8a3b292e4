"""Drop-in `process_game_state` (reference process_game_state.py) backed by the
MI355X encoder kernel.

create_state_tensors(state) -> (f32 [38, 5, 7], f32 [42]) CPU tensors with
the reference's channel layout (:19-137); the values come from the HIP
encoder (hz_encode) run on a one-board engine.  get_action_index is the
reference's index map (:156-179): pile i -> i, (tile, coord) -> 5 + 23*tile
+ cell.  Batched encoding of many states: hzamd.env.BatchedEnv.encode /
hzamd.selfplay.encode_states.
"""
from constants import NUM_HEXES, NUM_PILES, TILE_TYPES, VALID_HEXES, coordinate_to_index_map
from hzamd.single import bridge

q_min = min(q for q, _ in VALID_HEXES)
q_max = max(q for q, _ in VALID_HEXES)
r_min = min(r for _, r in VALID_HEXES)
r_max = max(r for _, r in VALID_HEXES)


def create_state_tensors(game_state):
    return bridge().encode(game_state)


def create_board_tensor(game_state):
    return create_state_tensors(game_state)[0]


def create_global_features(game_state):
    return create_state_tensors(game_state)[1]


def get_action_index(action, hand_tiles=None):
    """Game move -> flat policy index in [0, 143)."""
    if isinstance(action, int):
        if 0 <= action < NUM_PILES:
            return action
        raise ValueError(f"Invalid pile index action: {action}")
    if isinstance(action, tuple) and len(action) == 2:
        tile_type, coord = action
        if tile_type not in TILE_TYPES:
            raise ValueError(f"Invalid tile type in action: {tile_type}")
        if coord not in coordinate_to_index_map:
            raise ValueError(f"Invalid coordinate in action: {coord}")
        return NUM_PILES + TILE_TYPES.index(tile_type) * NUM_HEXES + coordinate_to_index_map[coord]
    raise ValueError(f"Invalid action format: {action}")
