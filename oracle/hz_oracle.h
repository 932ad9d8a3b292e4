/* hz_oracle.h — CPU restatement of the reference Harmonies engine, encoder
 * and MCTS.  TEST INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, never by the product path.
 *
 * States cross this interface in the REFSTATE layout (int16[78]) written by
 * tests/golden/make_golden.py:
 *   [0:23]  player-0 stack code per cell (cell = index into sorted(VALID_HEXES))
 *   [23:46] player-1 stack codes
 *   [46:61] piles 5x3 tile ids (TILE_TYPES order), -1 = absent
 *   [61]    number of piles
 *   [62:65] hand tile ids, -1 = absent      [65] hand size
 *   [66:72] bag counts in TILE_TYPES order
 *   [72] current_player  [73] phase (0 choose_pile,1..3 place_tile_k,4 game_over)
 *   [74] game_over flag  [75] winner (-2 None, -1 draw, 0, 1)  [76:78] final_scores
 * Stack codes: 0 empty, 1+t singleton of tile t, 7 wood/plant, 8 stone/stone,
 * 9 stone/stone/stone, 10 wood/building, 11 stone/building, 12 building/building.
 */
#ifndef HZ_ORACLE_H
#define HZ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_REFSTATE 78

typedef struct { uint32_t mt[624]; int32_t idx; } or_mt;

/* CPython random.seed(int) / getrandbits / _randbelow / sample(range(n), k). */
void     or_mt_seed(or_mt *m, uint64_t seed);
uint32_t or_mt_next32(or_mt *m);
uint32_t or_randbelow(or_mt *m, uint32_t n);
void     or_sample(or_mt *m, uint32_t n, int k, int32_t *out);

/* Engine (reference harmonies_engine.py). */
void or_reset(or_mt *m, int16_t *st);
int  or_legal(const int16_t *st, uint8_t *mask143);          /* returns #legal */
int  or_step(int16_t *st, int action, or_mt *m);             /* 0 ok, else status */
void or_score_board(const uint8_t *cells23, int32_t *out5);   /* grass,mount,field,bldg,water */
int  or_is_game_over(const int16_t *st);
void or_encode(const int16_t *st, float *board1330, float *glob42);
void or_canonical(const int16_t *st, uint8_t *key128, int pyhash);

/* evaluation.py choose_move_greedy; consumes m like the reference. */
int or_greedy_move(const int16_t *st, or_mt *m);

/* Build-defined action rule used by the env benchmark / fixtures. */
uint64_t or_rule(uint64_t seed, uint64_t ply);

/* Play n games (board b seeded seed_base+b) with the rule; returns total env
 * steps.  finals: n*78, plies: n, next_word: n (CPython next getrandbits(32)). */
int64_t or_play_rule_games(int n, uint64_t seed_base, int16_t *finals, int32_t *plies,
                           uint32_t *next_word, int nthreads);
int64_t or_play_rule_games_ep(int n, uint64_t seed_base, int episode, int16_t *finals, int32_t *plies,
                              uint32_t *next_word, int nthreads);
/* Steady-state auto-reset play: `plies` env steps per board from episode
 * ep0's reset, each ended game followed by the board's next episode. */
int64_t or_play_rule_auto(int n, uint64_t seed_base, int ep0, int64_t plies, int16_t *finals, int32_t *games,
                          int32_t *episode_out, int nthreads);
/* a caller's own moves replayed from random.seed(seeds[b]) resets (the api_caller leg's check) */
int64_t or_replay_actions(int n, const uint64_t *seeds, int plies, const int16_t *actions, int16_t *finals,
                          int32_t *rejected, int nthreads);

/* MCTS (reference MCTS.py get_best_action_and_pi) with the deterministic stub
 * evaluator of tests/golden/make_golden.py, canonical (ascending action index)
 * move order.  noise: per-legal-rank Dirichlet values used when !testing.
 * Outputs: visits[143], returns chosen action (or -1). */
typedef struct {
  int32_t sims;
  float   cpuct;
  double  eps;
  int32_t testing;
  int32_t tau0;
  int32_t ply;
  double  u;            /* uniform for tau=1 sampling */
  int32_t exact_keys;   /* 0: key nodes like hash(state) (reference); 1: exact canonical */
  int32_t negate_value; /* 1: the stub's value negated (a second, different evaluator) */
} or_mcts_cfg;

int or_mcts_search(const int16_t *root, or_mt *m, const or_mcts_cfg *cfg, const double *noise,
                   int32_t *visits143, int32_t *n_nodes, int32_t *n_edges);

/* Stub evaluator (integer formula over the encoder's inputs). */
void or_stub_eval(const int16_t *st, float *policy143, double *value);

#ifdef __cplusplus
}
#endif
#endif
