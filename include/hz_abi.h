/* hz_abi.h — C-ABI of libhz.so, the MI355X-native Harmonies self-play engine.
 *
 * The reference (IllyaArtemchuk/Harmonies-Alphazero) is pure Python with no
 * FFI; its hot path is reached through duck-typed Python surfaces.  Each entry
 * point below is the batched device form of one of those surfaces (cited as
 * /root/reference file:line).  The Python package
 * harmonies-alphazero_amd/hzamd binds them with ctypes; INTEGRATION.md shows
 * the binding a maintainer would add.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer (e.g. torch tensor.data_ptr())
 *    unless stated otherwise; it must stay valid until the work enqueued on
 *    the handle's stream has run.  Calls are asynchronous, stream-ordered on
 *    the handle's stream, and never allocate or synchronize.
 *  - Return value: 0 = enqueued; <0 = invalid argument (nothing enqueued);
 *    >0 = hipError_t of the failed launch.
 *  - Per-board rule violations are not errors of the call: they come back as
 *    per-board status codes (HZ_ST_*), where the reference raises ValueError.
 *  - Board b's state is the structure-of-arrays record documented in
 *    harmonies-alphazero_amd/csrc/hz_device.hpp (six u64 words, word w at
 *    state[w * n + b]); its chance stream is a CPython MT19937 (624 words at
 *    mt[b * 624 + i] plus a cursor).
 */
#ifndef HZ_ABI_H
#define HZ_ABI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-board status codes (reference ValueError sites in parentheses) */
enum {
  HZ_ST_OK = 0,
  HZ_ST_BAD_PILE = 1,        /* harmonies_engine.py:216-220 "Invalid pile index"      */
  HZ_ST_BAD_FORMAT = 2,      /* :227-236 "Invalid move format for placement phase"     */
  HZ_ST_NOT_IN_HAND = 3,     /* :244-248 "Illegal move attempted: Tile ... not in hand" */
  HZ_ST_ILLEGAL_STACK = 4,   /* :281-283 "Cannot place ... on ... with stack"           */
  HZ_ST_BAD_PHASE = 5,       /* :296-297 "Invalid turn phase"                           */
  HZ_ST_BAD_ACTION = 6,      /* action id outside [0,143) (process_game_state.py:156-179) */
  HZ_ST_NOOP = 7             /* negative action: board left untouched                    */
};

typedef struct hz_env hz_env;

/* ---- lifecycle ---------------------------------------------------------- */
/* n_boards boards; board b's k-th game is seeded like
 * random.seed(seed_base + b + (k << 32)) followed by HarmoniesGameState()
 * (harmonies_engine.py:66-79).  stream: hipStream_t, NULL = null stream.
 * The handle owns all device buffers (48 B state + 2.5 KB MT per board). */
hz_env *hz_env_create(int32_t n_boards, uint64_t seed_base, void *stream);
void hz_env_destroy(hz_env *env);
int32_t hz_env_size(const hz_env *env);
int hz_env_set_stream(hz_env *env, void *stream);
/* device pointers of the handle's own buffers (for zero-copy views) */
uint64_t *hz_env_state_ptr(hz_env *env);     /* [6][n]            */
uint32_t *hz_env_mt_ptr(hz_env *env);        /* [n][624]          */
int32_t *hz_env_mt_pos_ptr(hz_env *env);     /* [n]               */
int32_t *hz_env_ply_ptr(hz_env *env);        /* [n] plies played in the current game */
uint64_t *hz_env_seed_ptr(hz_env *env);      /* [n] seed of the current game */

/* ---- env surface (step / reset / legal_actions / score) ----------------- */
/* reset: HarmoniesGameState() for every board with sel[b] != 0 (sel NULL =
 * all boards).  seeds (optional, [n]) overrides the per-board seed. */
int hz_reset(hz_env *env, const uint8_t *sel, const uint64_t *seeds);

/* legal_actions: get_legal_moves (harmonies_engine.py:145-208) mapped through
 * get_action_index (process_game_state.py:156-179) to a 143-bit mask per
 * board, mask[b*3 + w] bit i = action 64*w + i.  count[b] = #legal (may be
 * NULL).  A finished board has an empty mask. */
int hz_legal_mask(hz_env *env, uint64_t *mask, int32_t *count);
/* the same legal moves as one byte per action: legal[b*143 + a] = 1 when
 * action a is legal on board b (a bool [n][143] tensor; legal 16-B aligned),
 * count as above.  One launch for BatchedEnv.legal_actions(). */
int hz_legal_actions(hz_env *env, uint8_t *legal, int32_t *count);

/* step: apply_move (harmonies_engine.py:210-298) in place, including
 * _end_turn_actions (:301-329) and chance draws.  action[b] < 0 = no-op.
 * status[b] (may be NULL) gets an HZ_ST_* code; on a non-zero status the
 * board is unchanged (the reference raises before committing its clone). */
int hz_step(hz_env *env, const int16_t *action, int32_t *status);

/* _replenish_piles (harmonies_engine.py:132-137) / _end_turn_actions
 * (:301-329) on the selected boards (sel NULL = all), drawing from each
 * board's stream.  The Python facade uses them for HarmoniesGameState() and
 * for callers that invoke _end_turn_actions directly (text_game.py:212). */
int hz_replenish(hz_env *env, const uint8_t *sel);
int hz_end_turn(hz_env *env, const uint8_t *sel);

/* score: calculate_score_for_player(p) (:357-367) for both players of every
 * board, out[b*2 + p].  parts (may be NULL): out_parts[(b*2+p)*5 + k] for
 * grass, mountains, fields, buildings, water (:369-523). */
int hz_score(hz_env *env, int32_t *out, int32_t *out_parts);

/* encode: create_state_tensors (process_game_state.py:15-137) for boards
 * idx[0..m) (idx NULL = boards 0..m-1): board[m][38][5][7], glob[m][42], f32. */
int hz_encode(hz_env *env, const int32_t *idx, int32_t m, float *board, float *glob);

/* Stateless encoder over any state array (replay records, tree nodes): item j
 * is idx[j] (idx NULL = j); its word w is states[item * item_stride +
 * w * word_stride].  idx[j] < 0 yields zeros.  Enqueued on `stream`. */
int hz_encode_states(const uint64_t *states, int64_t word_stride, int64_t item_stride, const int32_t *idx,
                     int32_t m, float *board, float *glob, void *stream);

/* Build-defined deterministic policy used by the env benchmark and the golden
 * traces: pick legal action k = ((splitmix64(seed, ply) >> 32) * L) >> 32 in
 * ascending action order.  Writes action[b] (-1 if no legal move). */
int hz_rule_actions(hz_env *env, const uint64_t *mask, const int32_t *count, int16_t *action);

/* One ply of the per-ply surface for every board in ONE launch:
 * get_legal_moves (harmonies_engine.py:145-208, as hz_legal_mask) -> the
 * rule pick above (as hz_rule_actions) -> apply_move (:210-298, as hz_step).
 * Each output pointer may be NULL; those given get exactly what the three
 * separate calls would write (mask, count, action, status).  The batched
 * API path's graph replays one of these per ply instead of three launches. */
int hz_rule_ply(hz_env *env, uint64_t *mask, int32_t *count, int16_t *action, int32_t *status);

/* evaluation.py:137-196 choose_move_greedy for every selected board (sel may
 * be NULL = all): the legal move whose resulting board scores highest for the
 * player to move, first strictly best in ascending action order.  Like the
 * reference, whose simulated apply_move calls refill the piles from the
 * global `random` at the end of a turn, it consumes each board's chance
 * stream once per candidate when the phase is place_tile_3; apply the
 * returned move with hz_step.  action[b] = -1 when unselected, finished or
 * without a legal move. */
int hz_greedy_actions(hz_env *env, const uint8_t *sel, int16_t *action);

/* Fused env loop: every board plays up to max_plies rule-driven plies
 * (legal mask -> rule pick -> step), stopping at game end (auto_reset = 0) or
 * starting its next game (auto_reset != 0).  Optional per-ply records
 * (NULL = off): traj_state[(ply*6 + w)*n + b], traj_mask[(ply*n + b)*3 + w],
 * traj_action[ply*n + b] (-1 after the game ended).  games_done[b] counts
 * games finished during the call, steps_done[b] env steps taken. */
int hz_rollout(hz_env *env, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state,
               uint64_t *traj_mask, int16_t *traj_action, int32_t *games_done,
               int32_t *steps_done);
/* hz_reset (all boards) fused with hz_rollout in one launch: the chance
 * streams are seeded and consumed in LDS and written to HBM once.  With
 * chance-ahead on (the default), the other blocks of the same launch run,
 * concurrently with the play, a three-stage pipeline over every board's
 * next episodes (a game's chance draws and the benchmark rule's hashes do
 * not depend on its moves): the stream seeded three calls ahead, its piles
 * drawn two and one calls ahead, with the rule hashes; a call replays the
 * prepared piles instead of seeding and drawing (identical results; a board
 * whose episode counter was moved by anything else seeds in place, a game
 * needing more piles continues on the prepared stream). */
int hz_play(hz_env *env, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state,
            uint64_t *traj_mask, int16_t *traj_action, int32_t *games_done,
            int32_t *steps_done);
/* chance-ahead for hz_play: draws = piles prepared per board (0 = off,
 * capped at 24 = the default). */
int hz_env_set_seed_ahead(hz_env *env, int32_t draws);
/* hz_play's pipeline: 2 (the default; HZ_PIPELINE=1 in the environment at
 * hz_env_create makes 1 the default) = every board's game spread over
 * thirteen consecutive calls, one stage per call (seeding pass 1 in two
 * stages, pass 2 in three, four draw stages, four play stages), all thirteen
 * running in each launch on different episodes; 1 = the chance-ahead
 * pipeline above.  Same results either way; pipeline 2 applies to calls with
 * auto_reset = 0, no trajectory outputs and max_plies >= 96 (others take
 * pipeline 1).  Returns -1 for a value other than 1 or 2. */
int hz_env_set_pipeline(hz_env *env, int32_t pipeline);
/* hz_rollout with auto_reset: on != 0 (the default, unless HZ_AR_AHEAD=0
 * at hz_env_create) lets each such call's extra blocks prepare every board's
 * episodes two and three ahead of its counter (seeded stream, pile script of
 * the first 24 draws, cursors), so that a board whose game ends starts the
 * next one from its script instead of seeding in place
 * (harmonies_engine.py:66-79 + :120-137 restated ahead of time; a game's
 * chance sequence does not depend on its moves).  Same results either way. */
int hz_env_set_auto_ahead(hz_env *env, int32_t on);
/* Both hz_play pipelines hand rows from one wave to another inside a block
 * through an LDS progress counter; a waiting wave spins at most spin_limit
 * s_sleep rounds.  A wait that gives up ORs a bit into the env's error word
 * (1: the chance-ahead seed stage's row wait, 2: k_play2's twist wave) and
 * the call's streams are then untrusted: the caller must raise.  word is a
 * device int32 the caller reads (and clears) after a sync; NULL = the
 * handle's own word.  No reference counterpart (the reference has no
 * concurrency). */
int hz_env_set_error_word(hz_env *env, int32_t *word);
/* Test knob: the spin bound of those waits (0 = the default, 2^22 rounds);
 * a bound of 1 makes waits give up almost at once. */
int hz_env_set_spin_limit(hz_env *env, int32_t limit);

/* ---- state transfer (Python facade and tests) --------------------------- */
/* export: state[6][n] and, optionally, the MT streams in CPython getstate()
 * form (mt[n][624], mt_index[n] in [0, 624]).  Finishes any partially
 * twisted generation in place (the stream's future outputs are unchanged). */
int hz_export_state(hz_env *env, uint64_t *state, uint32_t *mt, int32_t *mt_index);
/* import: the inverse; mt/mt_index may be NULL to keep the current streams. */
int hz_import_state(hz_env *env, const uint64_t *state, const uint32_t *mt, const int32_t *mt_index);

/* ---- batched MCTS (MCTS.py) ---------------------------------------------- */
/* One single-tree PUCT search per board of an hz_env, all boards advancing
 * one simulation per call sequence select -> encode_leaves -> (caller's
 * policy/value inference, e.g. PyTorch) -> expand_backup.  Semantics follow
 * get_best_action_and_pi (MCTS.py:272-441) with moves in ascending action
 * order (the reference's order is set iteration order).
 * Transpositions are keyed like the reference's hash(state) (exact_keys = 0)
 * or by the exact canonical tuple (exact_keys = 1).  max_nodes bounds nodes
 * and edges per board per search (1 + sims * 69 never overflows); it must be
 * below 2^24 (edge ids are packed into 24 bits of the walk's hints), else
 * create returns NULL. */
typedef struct hz_mcts hz_mcts;
hz_mcts *hz_mcts_create(int32_t n_boards, int32_t max_nodes, int32_t max_depth, int32_t exact_keys, void *stream);
void hz_mcts_destroy(hz_mcts *mcts);
int hz_mcts_set_stream(hz_mcts *mcts, void *stream);
/* new tree per board with root = the env board's current state (MCTS.py:288);
 * active[b] == 0 (or NULL = all active) leaves board b out of this search */
int hz_mcts_begin(hz_mcts *mcts, hz_env *env, const uint8_t *active);
/* move_to_leaf (MCTS.py:63-149) for every active board */
int hz_mcts_select(hz_mcts *mcts, const uint8_t *active, float cpuct);
/* create_state_tensors of every board's selected leaf into board[n][38][5][7],
 * glob[n][42]; rows of terminal leaves / inactive boards are zero */
int hz_mcts_encode_leaves(hz_mcts *mcts, float *board, float *glob);
/* The leaves that need the network, gathered: the active boards whose
 * selected leaf is not terminal (MCTS.py:297-341 calls predict only for
 * those), in ascending board order.  count[0] (device) = k; rows[j] (may be
 * NULL, [n]) = board of row j; board[j] / glob[j] for j < k get the leaf's
 * create_state_tensors, rows >= k are not written.  No host round trip: the
 * leaf-eval kernels below take `count` as their live-row bound.  Pair with
 * hz_mcts_expand_backup_gathered. */
int hz_mcts_gather_leaves(hz_mcts *mcts, float *board, float *glob, int32_t *rows, int32_t *count);
/* hz_mcts_select followed by hz_mcts_gather_leaves (board and glob both
 * required), as one launch when the handle has at most 32 boards (config 1's
 * one-board searches, the arena): same results, two launch latencies less
 * per simulation. */
int hz_mcts_select_gather(hz_mcts *mcts, const uint8_t *active, float cpuct, float *board, float *glob,
                          int32_t *rows, int32_t *count);
/* counter (device int64, may be NULL to detach): every later
 * hz_mcts_gather_leaves adds its row count k to counter[0] on the device
 * (the number of leaf evaluations of a search without a separate kernel). */
int hz_mcts_set_eval_counter(hz_mcts *mcts, int64_t *counter);
/* Test switch (no reference counterpart): on != 0 makes every expansion's
 * sibling dedup take its serial walk instead of the LDS hash table (the path
 * the table leaves to the walk only on a hash collision), so tests can check
 * both give the same trees.  Off by default. */
int hz_mcts_set_dedup_walk(hz_mcts *mcts, int32_t on);
/* Test / A-B switch (no reference counterpart): how hz_mcts_gather_leaves
 * runs on this handle: 1 = one k_gather_encode launch, 0 = k_gather + the
 * encoder launches (same rows, slots, count and tensors), -1 = the process
 * default (HZ_GATHER_ENCODE, fused unless it is 0). */
int hz_mcts_set_gather_encode(hz_mcts *mcts, int32_t mode);
/* expand_leaf (MCTS.py:151-218) with policy[n][143] (probabilities, as
 * ModelManager.predict returns them, model.py:81-110), root Dirichlet mix
 * (MCTS.py:308-327) when !testing using noise[n][69] (i-th legal move), then
 * back_fill (MCTS.py:220-266) with value[n] (terminal leaves use the game
 * outcome, MCTS.py:333-341).  Children's chance draws consume the env
 * board's MT stream in child order, like the reference's apply_move calls. */
int hz_mcts_expand_backup(hz_mcts *mcts, hz_env *env, const float *policy, const float *value,
                          const double *noise, double eps, int32_t testing);
/* the same with policy[k][143] / value[k] in the row order of the last
 * hz_mcts_gather_leaves (board b reads row j where rows[j] = b) */
int hz_mcts_expand_backup_gathered(hz_mcts *mcts, hz_env *env, const float *policy, const float *value,
                                   const double *noise, double eps, int32_t testing);
/* hz_mcts_expand_backup_gathered followed by the next simulation's
 * hz_mcts_select(active, cpuct), in one launch (each board's wave walks its
 * tree right after its backup; same leaves and paths as the two calls).
 * A search then runs select once, and per simulation gather_leaves, the
 * network and this (the last simulation: hz_mcts_expand_backup_gathered).
 * Replaces the select of MCTS.py:297-305's next iteration. */
int hz_mcts_expand_backup_select(hz_mcts *mcts, hz_env *env, const float *policy, const float *value,
                                 const double *noise, double eps, int32_t testing, const uint8_t *active,
                                 float cpuct);
/* hz_mcts_expand_backup_select, then, in the same launch, the next leaf
 * batch (hz_mcts_gather_leaves' outputs): each board whose new leaf needs
 * the network takes the next row of *count_out (atomically: rows in
 * arrival order, not board order; rows[j] = board of row j, as before) and
 * encodes its leaf into board[j], glob[j].  *count_out must be 0 at launch;
 * *count_prev (the count of the batch this launch consumes) is set to 0,
 * after being added to the eval counter when add_prev != 0 (a count that no
 * gather call added).  Every result (visits, trees, streams) equals the
 * separate launches'; the evaluator must treat rows independently. */
int hz_mcts_expand_backup_select_gather(hz_mcts *mcts, hz_env *env, const float *policy, const float *value,
                                        const double *noise, double eps, int32_t testing, const uint8_t *active,
                                        float cpuct, float *board, float *glob, int32_t *rows, int32_t *count_out,
                                        int32_t *count_prev, int32_t add_prev);
/* Self-play root noise (MCTS.py:314-316, np.random.dirichlet([alpha] * L)
 * over the L = count[b] legal moves, in legal-move order) into noise[n][69]
 * (zeros past L) and the tau = 1 move-choice uniform (MCTS.py:411,
 * np.random.choice) into u[n] (may be NULL), from a counter-based generator
 * keyed by (seed, global board id = board_base + b, move): a board's draws do
 * not depend on the batch or the GPU count.  Enqueued on `stream`. */
int hz_root_noise(const int32_t *count, int32_t n, uint64_t seed, uint64_t board_base, uint64_t move, double alpha,
                  double *noise, double *u, void *stream);
/* root visit counts by action id: visits[n][143] (MCTS.py:355-376) */
int hz_mcts_result(hz_mcts *mcts, int32_t *visits);
/* per-board [nodes, edges, search generation, overflow flag] -> counts[n][4] */
int hz_mcts_stats(hz_mcts *mcts, int32_t *counts);
/* out[0] (device int64) += the sum of every edge's visit count over every
 * board's current tree, i.e. the edge levels its simulations walked (each
 * back_fill, MCTS.py:220-266, visits every edge of its path once): the
 * path-walk term of the tree kernels' algorithmic bytes (bench.py). */
int hz_mcts_path_edges(hz_mcts *mcts, int64_t *out);
/* host pointers to the device arrays leaf[n] / leaf_gidx[n] (debugging) */
int hz_mcts_leaf_ptrs(hz_mcts *mcts, int32_t **leaf, int32_t **leaf_gidx);

/* ---- leaf-eval kernels (hzamd/infer.py) ---------------------------------- */
/* `live` (device pointer, may be NULL) bounds the rows computed: rows
 * >= min(batch, *live) are neither read nor written (gathered leaf batches
 * whose size is known only on the device). */
/* x[rows][ch] = relu((x + bias[c]) + res) in place (res may be NULL): the
 * eval-mode BatchNorm (folded into the conv) -> [+ skip] -> ReLU tail of
 * model.py:376-393 (ResidualBlock.forward) and model.py:325-330 (stem) over an
 * NHWC activation.  ch % 4 == 0, pointers 16-byte aligned. */
int hz_bias_act(float *x, const float *bias, const float *res, int64_t rows, int32_t ch, void *stream);

/* out = relu((conv3x3(x, w) + bias[co]) + res) for the residual tower's
 * 128 -> 128 channel convs (model.py:362-371, kernel 3, padding 1) on the
 * 5x7 board: x, res, out NHWC [batch][5][7][128] (res may be NULL; out must
 * not alias x or res), wpack = w[co][ci][kh][kw] repacked as
 * [kh*3+kw][ci/16][co][ci%16] (hzamd/infer.py:pack_conv3x3).  f32 MFMA, exact
 * fp32 products and sums (summation order differs from MIOpen's). */
int hz_conv3x3_bias_act(const float *x, const float *wpack, const float *bias, const float *res, float *out,
                        int32_t batch, const int32_t *live, void *stream);

/* hz_conv3x3_bias_act on the bf16 MFMA (v_mfma_f32_16x16x32_bf16) with
 * fp32-exact products: x and w are split exactly into three bf16 pieces each
 * and the six piece products of order <= 2 are accumulated in fp32 (the
 * dropped ones are below one fp32 rounding).  wpack6 = bf16 planes
 * [kh*3+kw][ci/32][plane h,m,l][co][ci%32] (hzamd/infer.py:pack_conv3x3_x6). */
int hz_conv3x3_x6_bias_act(const float *x, const void *wpack6, const float *bias, const float *res, float *out,
                           int32_t batch, const int32_t *live, void *stream);

/* One residual block of the tower (model.py:376-393, ResidualBlock.forward
 * with BN folded): out = relu(conv2(relu(conv1(x) + b1)) + b2 + x), w1/w2
 * packed as for hz_conv3x3_x6_bias_act; x, out NHWC [batch][5][7][128] (out
 * must not alias x); tmp = scratch of batch*35*128 floats.  Bit-identical to
 * hz_conv3x3_x6_bias_act(x, w1, b1, NULL, tmp) followed by
 * hz_conv3x3_x6_bias_act(tmp, w2, b2, x, out); in its one-launch form
 * (hz_resblock_x6_fused(batch) == 1) the intermediate activation stays on
 * the CU (tmp holds half of it, briefly: a [2][288][32]-float slice per
 * 8-state group, which the one-launch form is taken only to fit in the
 * batch*35*128 floats above, i.e. never below 5 rows). */
int hz_resblock_x6_bias_act(const float *x, const void *w1, const float *b1, const void *w2, const float *b2,
                            float *out, float *tmp, int32_t batch, const int32_t *live, void *stream);
int32_t hz_resblock_x6_fused(int32_t batch);
/* on = 1 (the default, unless HZ_X6_BLOCK=0): hz_resblock_x6_bias_act takes
 * the one-launch form where it applies; 0: the two layered convs (A/B
 * measurements); results are bit-identical. */
int hz_resblock_x6_set_fused(int32_t on);
/* The one-launch form's row placement: 1 (the default, unless
 * HZ_BLK_TABLE=0) the LDS-bank-conflict-free row table the layered conv
 * uses, 0 round 3's (A/B measurements; results are bit-identical). */
int hz_resblock_x6_set_table(int32_t cf);
/* The residual tower (model.py:332-334: nblk <= 16 ResidualBlock.forward,
 * :376-393) in ONE launch where
 * hz_resblock_x6_fused(batch) holds: each workgroup carries its 8 states
 * through every block, block k's output written over block k-1's in out
 * (block 0 reads x, which is only read).  w1/b1/w2/b2 are HOST arrays of
 * nblk device pointers (each block's packed conv weights and folded
 * biases, as hz_resblock_x6_bias_act takes them); tmp as there.  The same
 * bits as nblk hz_resblock_x6_bias_act calls.  Returns -2 (nothing
 * enqueued) for a batch the per-block path serves. */
int hz_tower_x6_blocks(const float *x, const void *const *w1, const float *const *b1, const void *const *w2,
                       const float *const *b2, int32_t nblk, float *out, float *tmp, int32_t batch,
                       const int32_t *live, void *stream);
/* A/B knob (no reference counterpart): hz_tower_x6_blocks' first-round
 * workgroups on every other CU of each XCD start `units` x 8,128 cycles late
 * (default 4, HZ_TOWER_STAGGER overrides; 0: none), so the blocks' epilogue
 * bursts of all CUs stop coinciding.  Results are the same bits either way. */
int hz_tower_x6_set_stagger(int32_t units);

/* out = relu(conv3x3(board, w) + bias[co]) for the stem (model.py:328-330,
 * 38 -> 128 channels, padding 1): board NCHW [batch][38][5][7] as the
 * encoder writes it, out NHWC [batch][5][7][128], wpack = w with the input
 * channels zero-padded to 48, packed as for hz_conv3x3_bias_act. */
int hz_stem3x3_bias_act(const float *board, const float *wpack, const float *bias, float *out, int32_t batch,
                        const int32_t *live, void *stream);
/* the stem on the bf16 MFMA with fp32-exact products (as hz_conv3x3_x6_bias_act);
 * wpack6 = w with the input channels zero-padded to 64, packed as there
 * (hzamd/infer.py:pack_stem_x6). */
int hz_stem3x3_x6_bias_act(const float *board, const void *wpack6, const float *bias, float *out, int32_t batch,
                           const int32_t *live, void *stream);
/* The whole residual tower (model.py:332-333 over ResidualBlock.forward,
 * model.py:376-393, BN folded) in one launch for small batches: nconv
 * (even) convs, conv 2i without and 2i+1 with the skip of block i's input;
 * x0 = the stem's output, out = the tower's, both NHWC [batch][5][7][128]
 * (distinct buffers).  wpack6 = the nconv convs' pack_conv3x3_x6 layouts
 * back to back, bias [nconv][128].  One workgroup per state, activations
 * resident in LDS; bit-identical to nconv hz_conv3x3_x6_bias_act calls. */
int hz_tower_x6_resident(const float *x0, const void *wpack6, const float *bias, float *out, int32_t nconv,
                         int32_t batch, const int32_t *live, void *stream);
/* hz_tower_x6_resident for batch <= 32 with 24 (batch <= 10) or 8
 * workgroups per state (16 output channels each) exchanging each conv's
 * output through HBM in-launch: xch = scratch of 2 * batch * 35 * 128
 * floats, sync = 33 * 32 words, zero-initialised ONCE by the caller and left
 * zeroed by every launch (calls sharing one sync block must be ordered on
 * one stream); sync[32 * 32] != 0 means a workgroup gave up waiting (1 s)
 * since the block was zeroed, and that state's output is NaN.  Bit-identical
 * to hz_tower_x6_resident. */
int hz_tower_x6_split(const float *x0, const void *wpack6, const float *bias, float *out, float *xch, uint32_t *sync,
                      int32_t nconv, int32_t batch, const int32_t *live, void *stream);

/* Every workgroup of an hz_tower_x6_split launch must be resident at once
 * (its hand-offs wait on all of them).  hz_tower_x6_split returns
 * HZ_E_NOT_RESIDENT (-2), enqueuing nothing, when the launch's grid
 * (24 workgroups per state up to 10 states, else 8) exceeds what the current
 * device holds at once (CU count x the kernel's occupancy per CU, from the
 * occupancy API) or the limit set here; callers then take
 * hz_tower_x6_resident.  max_batch: the largest batch up to which it accepts
 * every batch on the current device (0: none).  set_limit: cap the workgroups (0 = no cap
 * beyond the device's), e.g. when other work shares the GPU. */
int32_t hz_tower_x6_split_max_batch(void);
int hz_tower_x6_split_set_limit(int32_t groups);

/* The heads of model.py:336-351 up to their linear layers, BN folded:
 * pcat[b] = relu(hw[0..1] . x[b][cell] + hb[0..1]) in NCHW flatten order (70)
 * || glob[b] (42); vcat[b] = relu(hw[2] . x[b][cell] + hb[2]) (35) || glob[b].
 * x NHWC [batch][5][7][128] (16-byte aligned), hw [3][128], hb [3]. */
int hz_heads(const float *x, const float *hw, const float *hb, const float *glob, float *pcat, float *vcat,
             int32_t batch, const int32_t *live, void *stream);
/* The whole head for the default shapes (2 + 1 head filters, 143 actions,
 * 256 hidden units, 42 globals): the 1x1 convs as hz_heads, then
 * logits = pcat . wpT + bp (model.py:341-344; wpT = policy_fc.weight^T
 * [112][143]), value = tanh(w2 . relu(vcat . w1T + b1) + b2) (model.py:352-355;
 * w1T [77][256], w2 [256], b2 [1]) and ModelManager.predict's softmax
 * (model.py:100-104).  logits [batch][143] and probs [batch][143] are
 * optional (NULL: not written); value [batch]. */
int hz_heads_fc(const float *x, const float *glob, const float *hw, const float *hb, const float *wpT,
                const float *bp, const float *w1T, const float *b1, const float *w2, const float *b2, float *logits,
                float *probs, float *value, int32_t batch, const int32_t *live, void *stream);

/* ---- build info ---------------------------------------------------------- */
const char *hz_version(void);

#ifdef __cplusplus
}
#endif
#endif
