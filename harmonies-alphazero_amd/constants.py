"""Board constants of the Harmonies engine, same names and values as the
reference's constants.py (:1-52), for drop-in imports."""

TILE_TYPES = ["water", "plant", "wood", "stone", "building", "field"]
WATER, PLANT, WOOD, STONE, BUILDING, FIELD = TILE_TYPES

# 23 hexes in a 5-4-5-4-5 pattern: rows r = -2..2, each row a run of q values
_ROWS = {-2: range(-1, 4), -1: range(-1, 3), 0: range(-2, 3), 1: range(-2, 2), 2: range(-3, 2)}
VALID_HEXES = {(q, r) for r, qs in _ROWS.items() for q in qs}

AXIAL_DIRECTIONS = [(1, 0), (-1, 0), (0, 1), (0, -1), (1, -1), (-1, 1)]
BOARD_SIZE = (5, 7)

# insertion order matters: the draw order of the bag follows it
INITIAL_BAG = dict(zip([WATER, PLANT, WOOD, STONE, FIELD, BUILDING], [23, 19, 21, 23, 19, 15]))
NUM_PILES = 5
PILE_SIZE = 3
NUM_HEXES = len(VALID_HEXES)
EMPTY_HEX_END_THRESHOLD = 2

sorted_coords = sorted(VALID_HEXES)
coordinate_to_index_map = {c: i for i, c in enumerate(sorted_coords)}
INPUT_CHANNELS = 2 * 3 * len(TILE_TYPES) + 2
GLOBAL_FEATURE_SIZE = NUM_PILES * len(TILE_TYPES) + 2 * len(TILE_TYPES)
ACTION_SIZE = NUM_PILES + len(TILE_TYPES) * NUM_HEXES
