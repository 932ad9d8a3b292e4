/* hz_oracle.c — CPU restatement of the reference engine / encoder / MCTS.
 *
 * TEST INFRASTRUCTURE (the parity checker and the cpu_baseline of bench.py).
 * Nothing in the product path links or calls this file.
 *
 * It deliberately follows the *reference's* structure (stack lists per cell,
 * BFS over get_neighbors, canonical-tuple transposition table, Python/NumPy
 * scalar promotion) rather than the GPU design (bitboards), so that the two
 * are independent statements of the same rules.  Citations are
 * /root/reference file:line.
 *
 * Pinned by the .npz fixtures under tests/golden/ captured from the reference itself
 * (tests/golden/make_golden.py); see tests/test_oracle_golden.py.
 */
#include "hz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- geometry
 * constants.py:1-52, harmonies_engine.py:31-43 (get_neighbors). */
enum { WATER = 0, PLANT, WOOD, STONE, BUILDING, FIELD };
static const int CELL_Q[23] = {-3, -2, -2, -2, -1, -1, -1, -1, -1, 0, 0, 0, 0, 0,
                               1,  1,  1,  1,  1,  2,  2,  2,  3};
static const int CELL_R[23] = {2, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, 1, 2,
                               -2, -1, 0, 1, 2, -2, -1, 0, -2};
static const int AXIAL[6][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, -1}, {-1, 1}};
static const int INITIAL_TT[6] = {23, 19, 21, 23, 15, 19};   /* INITIAL_BAG, TILE_TYPES order */
/* flat_bag iterates tile_bag in INITIAL_BAG insertion order (constants.py:41):
 * water, plant, wood, stone, field, building. */
static const int BAG_ORDER[6] = {WATER, PLANT, WOOD, STONE, FIELD, BUILDING};

/* stack codes <-> tile lists (bottom -> top) */
static const int CODE_H[13] = {0, 1, 1, 1, 1, 1, 1, 2, 2, 3, 2, 2, 2};
static const int CODE_T[13][3] = {
    {-1, -1, -1}, {WATER, -1, -1}, {PLANT, -1, -1}, {WOOD, -1, -1}, {STONE, -1, -1},
    {BUILDING, -1, -1}, {FIELD, -1, -1}, {WOOD, PLANT, -1}, {STONE, STONE, -1},
    {STONE, STONE, STONE}, {WOOD, BUILDING, -1}, {STONE, BUILDING, -1}, {BUILDING, BUILDING, -1}};

static int g_nbr[23][6], g_nnbr[23];
static int g_geom_ready = 0;

static int cell_of(int q, int r) {
  for (int c = 0; c < 23; c++)
    if (CELL_Q[c] == q && CELL_R[c] == r) return c;
  return -1;
}

static void geom_init(void) {
  if (g_geom_ready) return;
  for (int c = 0; c < 23; c++) {
    g_nnbr[c] = 0;
    for (int d = 0; d < 6; d++) {
      int n = cell_of(CELL_Q[c] + AXIAL[d][0], CELL_R[c] + AXIAL[d][1]);
      if (n >= 0) g_nbr[c][g_nnbr[c]++] = n;
    }
  }
  g_geom_ready = 1;
}

/* ------------------------------------------------------------------ MT19937
 * CPython Modules/_randommodule.c (init_genrand, init_by_array, genrand_uint32,
 * random_seed for int arguments) and Lib/random.py:239-249 (_randbelow),
 * :480-503 (sample). */
void or_mt_seed(or_mt *m, uint64_t seed) {
  uint32_t key[2];
  int klen;
  key[0] = (uint32_t)seed;
  key[1] = (uint32_t)(seed >> 32);
  klen = key[1] ? 2 : 1;
  uint32_t *mt = m->mt;
  mt[0] = 19650218U;
  for (int i = 1; i < 624; i++) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int i = 1, j = 0;
  for (int k = 624; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
    i++; j++;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = 623; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
    i++;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
  }
  mt[0] = 0x80000000U;
  m->idx = 624;
}

uint32_t or_mt_next32(or_mt *m) {
  uint32_t *mt = m->mt, y;
  static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
  if (m->idx >= 624) {
    int kk;
    for (kk = 0; kk < 624 - 397; kk++) {
      y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
      mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1U];
    }
    for (; kk < 623; kk++) {
      y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
      mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1U];
    }
    y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
    mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1U];
    m->idx = 0;
  }
  y = mt[m->idx++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return y;
}

static int bit_length(uint32_t n) { int k = 0; while (n) { k++; n >>= 1; } return k; }

uint32_t or_randbelow(or_mt *m, uint32_t n) {
  if (!n) return 0;
  int k = bit_length(n);
  uint32_t r = or_mt_next32(m) >> (32 - k);
  while (r >= n) r = or_mt_next32(m) >> (32 - k);
  return r;
}

void or_sample(or_mt *m, uint32_t n, int k, int32_t *out) {
  /* k <= 5, so setsize = 21 (random.py:484-486) */
  if (n <= 21) {
    int32_t pool[21];
    for (uint32_t i = 0; i < n; i++) pool[i] = (int32_t)i;
    for (int i = 0; i < k; i++) {
      uint32_t j = or_randbelow(m, n - (uint32_t)i);
      out[i] = pool[j];
      pool[j] = pool[n - (uint32_t)i - 1];
    }
  } else {
    for (int i = 0; i < k; i++) {
      uint32_t j;
      int dup;
      do {
        j = or_randbelow(m, n);
        dup = 0;
        for (int q = 0; q < i; q++) if ((uint32_t)out[q] == j) dup = 1;
      } while (dup);
      out[i] = (int32_t)j;
    }
  }
}

/* ------------------------------------------------------------------- state */
typedef struct {
  int h;
  int t[3];
} stack_t_;

typedef struct {
  stack_t_ board[2][23];
  int piles[5][3], pile_len[5], npiles;
  int hand[3], nhand;
  int bag[6];
  int player, phase, game_over, winner, scores[2];
} ostate;

static int code_of_stack(const stack_t_ *s) {
  for (int c = 0; c < 13; c++) {
    if (CODE_H[c] != s->h) continue;
    int ok = 1;
    for (int i = 0; i < s->h; i++) if (CODE_T[c][i] != s->t[i]) ok = 0;
    if (ok) return c;
  }
  return -1;
}

static void from_ref(const int16_t *v, ostate *s) {
  memset(s, 0, sizeof(*s));
  for (int p = 0; p < 2; p++)
    for (int c = 0; c < 23; c++) {
      int code = v[p * 23 + c];
      s->board[p][c].h = CODE_H[code];
      for (int i = 0; i < 3; i++) s->board[p][c].t[i] = CODE_T[code][i];
    }
  s->npiles = v[61];
  for (int i = 0; i < 5; i++) {
    s->pile_len[i] = 0;
    for (int j = 0; j < 3; j++) {
      s->piles[i][j] = v[46 + 3 * i + j];
      if (v[46 + 3 * i + j] >= 0) s->pile_len[i]++;
    }
  }
  s->nhand = v[65];
  for (int j = 0; j < 3; j++) s->hand[j] = v[62 + j];
  for (int t = 0; t < 6; t++) s->bag[t] = v[66 + t];
  s->player = v[72]; s->phase = v[73]; s->game_over = v[74]; s->winner = v[75];
  s->scores[0] = v[76]; s->scores[1] = v[77];
}

static void to_ref(const ostate *s, int16_t *v) {
  for (int p = 0; p < 2; p++)
    for (int c = 0; c < 23; c++) v[p * 23 + c] = (int16_t)code_of_stack(&s->board[p][c]);
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 3; j++)
      v[46 + 3 * i + j] = (int16_t)((i < s->npiles && j < s->pile_len[i]) ? s->piles[i][j] : -1);
  v[61] = (int16_t)s->npiles;
  for (int j = 0; j < 3; j++) v[62 + j] = (int16_t)(j < s->nhand ? s->hand[j] : -1);
  v[65] = (int16_t)s->nhand;
  for (int t = 0; t < 6; t++) v[66 + t] = (int16_t)s->bag[t];
  v[72] = (int16_t)s->player; v[73] = (int16_t)s->phase; v[74] = (int16_t)s->game_over;
  v[75] = (int16_t)s->winner; v[76] = (int16_t)s->scores[0]; v[77] = (int16_t)s->scores[1];
}

/* harmonies_engine.py:120-130 _draw_tiles; returns number drawn into out */
static int draw_tiles(ostate *s, or_mt *m, int num, int *out) {
  int n = 0;
  for (int t = 0; t < 6; t++) n += s->bag[t];
  if (n == 0) return 0;
  int k = num < n ? num : n;
  int32_t idx[3];
  or_sample(m, (uint32_t)n, k, idx);
  for (int i = 0; i < k; i++) {
    int rem = idx[i], t = 0;
    for (int o = 0; o < 6; o++) {
      int tt = BAG_ORDER[o];
      if (rem < s->bag[tt]) { t = tt; break; }
      rem -= s->bag[tt];
    }
    out[i] = t;
  }
  for (int i = 0; i < k; i++) s->bag[out[i]]--;
  return k;
}

/* :132-137 _replenish_piles */
static void replenish(ostate *s, or_mt *m) {
  while (s->npiles < 5) {
    int tiles[3];
    int k = draw_tiles(s, m, 3, tiles);
    if (!k) break;
    for (int j = 0; j < 3; j++) s->piles[s->npiles][j] = j < k ? tiles[j] : -1;
    s->pile_len[s->npiles] = k;
    s->npiles++;
  }
}

/* :66-79 __init__ */
void or_reset(or_mt *m, int16_t *st) {
  ostate s;
  memset(&s, 0, sizeof(s));
  for (int t = 0; t < 6; t++) s.bag[t] = INITIAL_TT[t];
  s.winner = -2;
  for (int i = 0; i < 5; i++) for (int j = 0; j < 3; j++) s.piles[i][j] = -1;
  for (int j = 0; j < 3; j++) s.hand[j] = -1;
  replenish(&s, m);
  to_ref(&s, st);
}

/* ------------------------------------------------------------- legal moves
 * :145-208 get_legal_moves (+ process_game_state.py:156-179 get_action_index) */
static int can_place(const stack_t_ *st, int tile) {
  if (st->h == 0) return 1;
  int top = st->t[st->h - 1], h = st->h;
  if (tile == PLANT && top == WOOD && h <= 2) return 1;
  if (tile == STONE && top == STONE && h < 3) return 1;
  if (tile == BUILDING && (top == WOOD || top == STONE || top == BUILDING) && h < 2) return 1;
  return 0;
}

static int legal_of(const ostate *s, uint8_t *mask) {
  memset(mask, 0, 143);
  int n = 0;
  if (s->phase == 0) {
    for (int i = 0; i < s->npiles; i++) { mask[i] = 1; n++; }
    return n;
  }
  if (s->phase >= 1 && s->phase <= 3) {
    if (!s->nhand) return 0;
    for (int j = 0; j < s->nhand; j++) {
      int t = s->hand[j];
      for (int c = 0; c < 23; c++) {
        if (can_place(&s->board[s->player][c], t)) {
          int a = 5 + t * 23 + c;
          if (!mask[a]) { mask[a] = 1; n++; }
        }
      }
    }
    return n;
  }
  return 0;
}

int or_legal(const int16_t *st, uint8_t *mask143) {
  ostate s;
  geom_init();
  from_ref(st, &s);
  return legal_of(&s, mask143);
}

/* ----------------------------------------------------------------- scoring
 * :357-523 calculate_score_for_player and the five _score_* functions. */
static int top_of(const stack_t_ *b, int c) { return b[c].h ? b[c].t[b[c].h - 1] : -1; }

static int water_points(int len) {               /* :18-27 get_water_score */
  static const int W[7] = {0, 0, 2, 5, 8, 11, 15};
  if (len <= 0) return 0;
  if (len <= 6) return W[len];
  return 15 + (len - 6) * 4;
}

static int components(const stack_t_ *b, int type, int comp[23][23], int *csize) {
  int visited[23] = {0}, nc = 0;
  for (int s0 = 0; s0 < 23; s0++) {
    if (top_of(b, s0) != type || visited[s0]) continue;
    int q[23], qh = 0, qt = 0, sz = 0;
    q[qt++] = s0; visited[s0] = 1;
    while (qh < qt) {
      int cur = q[qh++];
      comp[nc][sz++] = cur;
      for (int k = 0; k < g_nnbr[cur]; k++) {
        int n = g_nbr[cur][k];
        if (!visited[n] && top_of(b, n) == type) { visited[n] = 1; q[qt++] = n; }
      }
    }
    csize[nc++] = sz;
  }
  return nc;
}

static void score_parts(const stack_t_ *b, int32_t *out) {
  geom_init();
  int grass = 0, mount = 0, fields = 0, bld = 0, water = 0;
  for (int c = 0; c < 23; c++) {
    if (!b[c].h) continue;
    int top = b[c].t[b[c].h - 1], h = b[c].h;
    if (top == PLANT) {                                   /* :369-390 */
      if (h == 1) grass += 1;
      else if (h == 2 && b[c].t[0] == WOOD) grass += 3;
      else if (h == 3 && b[c].t[0] == WOOD && b[c].t[1] == WOOD) grass += 7;
    }
    if (top == STONE) {                                   /* :392-422 */
      int adj = 0;
      for (int k = 0; k < g_nnbr[c]; k++) if (top_of(b, g_nbr[c][k]) == STONE) adj = 1;
      if (adj) mount += (h == 1) ? 1 : (h == 2) ? 3 : (h == 3) ? 7 : 0;
    }
    if (top == BUILDING && h == 2) {                      /* :454-478 */
      int seen[6] = {0}, nt = 0;
      for (int k = 0; k < g_nnbr[c]; k++) {
        int t = top_of(b, g_nbr[c][k]);
        if (t >= 0 && !seen[t]) { seen[t] = 1; nt++; }
      }
      if (nt >= 3) bld += 5;
    }
  }
  int comp[23][23], csz[23];
  int nc = components(b, FIELD, comp, csz);               /* :424-452 */
  for (int i = 0; i < nc; i++) if (csz[i] >= 2) fields += 5;
  nc = components(b, WATER, comp, csz);                   /* :480-523 */
  for (int i = 0; i < nc; i++) {
    if (csz[i] < 2) continue;
    int in[23] = {0};
    for (int j = 0; j < csz[i]; j++) in[comp[i][j]] = 1;
    int diameter = 0;
    for (int j = 0; j < csz[i]; j++) {
      int dist[23], q[23], qh = 0, qt = 0, maxd = 0;
      for (int x = 0; x < 23; x++) dist[x] = -1;
      q[qt++] = comp[i][j]; dist[comp[i][j]] = 0;
      while (qh < qt) {
        int cur = q[qh++];
        if (dist[cur] > maxd) maxd = dist[cur];
        for (int k = 0; k < g_nnbr[cur]; k++) {
          int n = g_nbr[cur][k];
          if (in[n] && dist[n] < 0) { dist[n] = dist[cur] + 1; q[qt++] = n; }
        }
      }
      if (maxd > diameter) diameter = maxd;
    }
    water += water_points(diameter + 1);
  }
  out[0] = grass; out[1] = mount; out[2] = fields; out[3] = bld; out[4] = water;
}

void or_score_board(const uint8_t *cells23, int32_t *out5) {
  stack_t_ b[23];
  for (int c = 0; c < 23; c++) {
    b[c].h = CODE_H[cells23[c]];
    for (int i = 0; i < 3; i++) b[c].t[i] = CODE_T[cells23[c]][i];
  }
  score_parts(b, out5);
}

static int score_player(const ostate *s, int p) {
  int32_t parts[5];
  score_parts(s->board[p], parts);
  return parts[0] + parts[1] + parts[2] + parts[3] + parts[4];
}

/* ------------------------------------------------------------- transitions */
static void finish_game(ostate *s) {                      /* :344-354 */
  s->phase = 4;
  s->scores[0] = score_player(s, 0);
  s->scores[1] = score_player(s, 1);
  s->winner = s->scores[0] > s->scores[1] ? 0 : s->scores[1] > s->scores[0] ? 1 : -1;
}

static void end_turn(ostate *s, or_mt *m) {               /* :301-329 */
  int filled = 0;
  for (int c = 0; c < 23; c++) if (s->board[s->player][c].h) filled++;
  int player_trigger = (23 - filled) <= 2;
  int total = 0;
  for (int t = 0; t < 6; t++) total += s->bag[t];
  int bag_empty_before = total == 0;
  replenish(s, m);
  int bag_trigger = bag_empty_before && s->npiles == 0;
  int end = player_trigger || bag_trigger;
  if (end && !s->game_over) {
    s->game_over = 1;
    if (s->player == 0) { s->player = 1; s->phase = 0; }
    else finish_game(s);
  } else if (s->game_over) {
    finish_game(s);
  } else {
    s->player = 1 - s->player;
    s->phase = 0;
  }
}

/* :210-298 apply_move.  Status: 1 invalid pile index, 2 invalid move format,
 * 3 tile not in hand, 4 illegal stacking, 5 invalid phase, 6 bad action id. */
static int step_state(ostate *s, int a, or_mt *m) {
  if (a < 0 || a >= 143) return 6;
  if (s->phase == 0) {
    if (a >= 5 || a >= s->npiles) return 1;
    s->nhand = s->pile_len[a];
    for (int j = 0; j < 3; j++) s->hand[j] = s->piles[a][j];
    for (int i = a; i < s->npiles - 1; i++) {
      for (int j = 0; j < 3; j++) s->piles[i][j] = s->piles[i + 1][j];
      s->pile_len[i] = s->pile_len[i + 1];
    }
    s->npiles--;
    for (int j = 0; j < 3; j++) s->piles[s->npiles][j] = -1;
    s->pile_len[s->npiles] = 0;
    s->phase = 1;
    return 0;
  }
  if (s->phase >= 1 && s->phase <= 3) {
    if (a < 5) return 2;
    int t = (a - 5) / 23, c = (a - 5) % 23;
    int pos = -1;
    for (int j = 0; j < s->nhand; j++) if (s->hand[j] == t) { pos = j; break; }
    if (pos < 0) return 3;
    stack_t_ *st = &s->board[s->player][c];
    if (!can_place(st, t)) return 4;
    for (int j = pos; j < s->nhand - 1; j++) s->hand[j] = s->hand[j + 1];
    s->nhand--;
    s->hand[s->nhand] = -1;
    st->t[st->h++] = t;
    if (s->phase < 3) s->phase++;
    else end_turn(s, m);
    return 0;
  }
  return 5;
}

int or_step(int16_t *st, int action, or_mt *m) {
  ostate s;
  geom_init();
  from_ref(st, &s);
  int r = step_state(&s, action, m);
  if (r == 0) to_ref(&s, st);
  return r;
}

int or_is_game_over(const int16_t *st) { return st[74] && st[75] != -2; }

/* ------------------------------------------------------------------ encoder
 * process_game_state.py:15-137 */
void or_encode(const int16_t *v, float *board, float *glob) {
  ostate s;
  from_ref(v, &s);
  memset(board, 0, sizeof(float) * 1330);
  for (int p = 0; p < 2; p++)
    for (int c = 0; c < 23; c++) {
      int y = CELL_R[c] + 2, x = CELL_Q[c] + 3;
      const stack_t_ *st = &s.board[p][c];
      for (int pos = 0; pos < st->h && pos < 3; pos++)
        board[(p * 18 + st->t[pos] * 3 + pos) * 35 + y * 7 + x] = 1.0f;
    }
  float phase_val = (s.phase >= 0 && s.phase <= 3) ? (float)((double)s.phase / 3.0) : 0.0f;
  for (int c = 0; c < 23; c++) {
    int y = CELL_R[c] + 2, x = CELL_Q[c] + 3;
    board[36 * 35 + y * 7 + x] = (float)s.player;
    board[37 * 35 + y * 7 + x] = phase_val;
  }
  memset(glob, 0, sizeof(float) * 42);
  for (int i = 0; i < 5 && i < s.npiles; i++)
    for (int t = 0; t < 6; t++) {
      int cnt = 0;
      for (int j = 0; j < s.pile_len[i]; j++) if (s.piles[i][j] == t) cnt++;
      glob[i * 6 + t] = (float)((double)cnt / 3.0);
    }
  if (s.nhand)
    for (int t = 0; t < 6; t++) {
      int cnt = 0;
      for (int j = 0; j < s.nhand; j++) if (s.hand[j] == t) cnt++;
      glob[30 + t] = (float)((double)cnt / 3.0);
    }
  for (int t = 0; t < 6; t++) glob[36 + t] = (float)((double)s.bag[t] / (double)INITIAL_TT[t]);
}

/* :81-110 get_canonical_tuple as a fixed-width byte key:
 * player, phase, sorted hand, piles (each sorted, in order), bag, boards.
 *
 * pyhash=1 reproduces how MCTS.py actually keys its transposition table:
 * by hash(state) (MCTS.py:14,177,185), and CPython's hash(-1) == hash(-2), so
 * an axial coordinate component -1 hashes like -2.  Board items are hashed in
 * sorted-coordinate order (harmonies_engine.py:84-87), so two boards collide
 * iff their occupied cells, listed in cell-index order, agree pairwise on
 * (coordinate with -1 -> -2, stack).  pyhash=0 is the exact canonical tuple. */
#define KEYLEN 128
static int hash_class(int c) {
  int q = CELL_Q[c] == -1 ? -2 : CELL_Q[c], r = CELL_R[c] == -1 ? -2 : CELL_R[c];
  for (int d = 0; d < 23; d++) {
    int qd = CELL_Q[d] == -1 ? -2 : CELL_Q[d], rd = CELL_R[d] == -1 ? -2 : CELL_R[d];
    if (qd == q && rd == r) return d;
  }
  return c;
}

static void canonical_of(const ostate *s, uint8_t *k, int pyhash) {
  memset(k, 0xFF, KEYLEN);
  k[0] = (uint8_t)s->player;
  k[1] = (uint8_t)s->phase;
  int h[3], n = s->nhand;
  for (int j = 0; j < n; j++) h[j] = s->hand[j];
  for (int a = 0; a < n; a++) for (int b = a + 1; b < n; b++) if (h[b] < h[a]) { int t = h[a]; h[a] = h[b]; h[b] = t; }
  k[2] = (uint8_t)n;
  for (int j = 0; j < n; j++) k[3 + j] = (uint8_t)h[j];
  k[6] = (uint8_t)s->npiles;
  for (int i = 0; i < s->npiles; i++) {
    int p[3], m = s->pile_len[i];
    for (int j = 0; j < m; j++) p[j] = s->piles[i][j];
    for (int a = 0; a < m; a++) for (int b = a + 1; b < m; b++) if (p[b] < p[a]) { int t = p[a]; p[a] = p[b]; p[b] = t; }
    for (int j = 0; j < m; j++) k[7 + 3 * i + j] = (uint8_t)p[j];
  }
  for (int t = 0; t < 6; t++) k[22 + t] = (uint8_t)s->bag[t];
  for (int p = 0; p < 2; p++) {
    uint8_t *o = k + 28 + p * 46;
    int w = 0;
    for (int c = 0; c < 23; c++) {
      int code = code_of_stack(&s->board[p][c]);
      if (pyhash) {
        if (!code) continue;
        o[w++] = (uint8_t)hash_class(c);
        o[w++] = (uint8_t)code;
      } else {
        o[c] = (uint8_t)code;
      }
    }
  }
}

void or_canonical(const int16_t *st, uint8_t *key128, int pyhash) {
  ostate s;
  geom_init();
  from_ref(st, &s);
  canonical_of(&s, key128, pyhash);
}

/* ------------------------------------------------------------ action rule */
uint64_t or_rule(uint64_t seed, uint64_t ply) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ULL + ply;
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static int kth_legal(const uint8_t *mask, int k) {
  for (int a = 0; a < 143; a++) if (mask[a] && k-- == 0) return a;
  return -1;
}

int64_t or_play_rule_games(int n, uint64_t seed_base, int16_t *finals, int32_t *plies,
                           uint32_t *next_word, int nthreads) {
  return or_play_rule_games_ep(n, seed_base, 0, finals, plies, next_word, nthreads);
}

/* the same for every board's episode e: seed = seed_base + b + (e << 32)
 * (the env's hz_reset / hz_play seeding of a board's (e+1)-th game) */
int64_t or_play_rule_games_ep(int n, uint64_t seed_base, int episode, int16_t *finals, int32_t *plies,
                              uint32_t *next_word, int nthreads) {
  geom_init();
  int64_t total = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
#endif
  for (int b = 0; b < n; b++) {
    or_mt m;
    uint64_t seed = seed_base + (uint64_t)b + ((uint64_t)(uint32_t)episode << 32);
    or_mt_seed(&m, seed);
    int16_t st[78];
    or_reset(&m, st);
    ostate s;
    from_ref(st, &s);
    int ply = 0;
    uint8_t mask[143];
    while (!(s.game_over && s.winner != -2)) {
      int L = legal_of(&s, mask);
      if (!L) break;
      uint64_t z = or_rule(seed, (uint64_t)ply);
      int k = (int)(((z >> 32) * (uint64_t)L) >> 32);
      step_state(&s, kth_legal(mask, k), &m);
      ply++;
    }
    if (finals) to_ref(&s, finals + (size_t)b * 78);
    if (plies) plies[b] = ply;
    if (next_word) next_word[b] = or_mt_next32(&m);
    total += ply;
  }
  return total;
}

/* Steady-state auto-reset play (hz_rollout with auto_reset, the env loop of
 * a self-play worker that starts a new HarmoniesGameState() whenever a game
 * ends, trainer.py:434-541 with the rule in place of the search): board b
 * plays `plies` rule-driven env steps from its episode ep0's reset, starting
 * episode e + 1 (seed_base + b + ((e + 1) << 32)) whenever episode e ends
 * with steps left.  finals: the state after the last step; games: the games
 * that ended within the steps; episode_out: the episode being played (or
 * just ended) at the end.  Returns the steps taken (n * plies). */
int64_t or_play_rule_auto(int n, uint64_t seed_base, int ep0, int64_t plies, int16_t *finals, int32_t *games,
                          int32_t *episode_out, int nthreads) {
  geom_init();
  int64_t total = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
#endif
  for (int b = 0; b < n; b++) {
    int64_t left = plies;
    int e = ep0, done = 0;
    ostate s;
    memset(&s, 0, sizeof(s));
    for (;;) {
      or_mt m;
      uint64_t seed = seed_base + (uint64_t)b + ((uint64_t)(uint32_t)e << 32);
      or_mt_seed(&m, seed);
      int16_t st[78];
      or_reset(&m, st);
      from_ref(st, &s);
      int ply = 0;
      uint8_t mask[143];
      while (left > 0 && !(s.game_over && s.winner != -2)) {
        int L = legal_of(&s, mask);
        if (!L) {
          /* stuck (no legal move, game not over): the kernel's auto-reset
           * path stops such a board for the rest of the call, so does this */
          left = 0;
          break;
        }
        uint64_t z = or_rule(seed, (uint64_t)ply);
        int k = (int)(((z >> 32) * (uint64_t)L) >> 32);
        step_state(&s, kth_legal(mask, k), &m);
        ply++;
        left--;
        total++;
      }
      if (s.game_over && s.winner != -2) done++;
      if (left <= 0) break;
      e++;
    }
    if (finals) to_ref(&s, finals + (size_t)b * 78);
    if (games) games[b] = done;
    if (episode_out) episode_out[b] = e;
  }
  return total;
}

/* A caller's own moves replayed: board b starts HarmoniesGameState() after
 * random.seed(seeds[b]) (harmonies_engine.py:66-79) and applies
 * actions[p * n + b] for p < plies with apply_move (:210-298; a negative
 * action is the batched step's no-op), the state kept unchanged on a
 * rejected move like the reference's clone-then-commit.  finals: the last
 * state; rejected[b]: the moves that were rejected.  Returns the moves
 * applied. */
int64_t or_replay_actions(int n, const uint64_t *seeds, int plies, const int16_t *actions, int16_t *finals,
                          int32_t *rejected, int nthreads) {
  geom_init();
  int64_t total = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
#endif
  for (int b = 0; b < n; b++) {
    or_mt m;
    or_mt_seed(&m, seeds[b]);
    int16_t st[78];
    or_reset(&m, st);
    ostate s;
    from_ref(st, &s);
    int bad = 0;
    for (int p = 0; p < plies; p++) {
      int a = actions[(size_t)p * n + b];
      if (a < 0) continue;
      ostate t = s;
      if (step_state(&t, a, &m) == 0) {
        s = t;
        total++;
      } else {
        bad++;
      }
    }
    if (finals) to_ref(&s, finals + (size_t)b * 78);
    if (rejected) rejected[b] = bad;
  }
  return total;
}

/* -------------------------------------------------------------------- MCTS
 * MCTS.py:8-441.  Node = state + ordered edge list; Edge = (player of the
 * in-node, action, child, N int, W/Q float64, P float32).  Transpositions are
 * found through the canonical key (MCTS.py:177-204 via hash(state)). */
typedef struct { int node, action, child, N; double W, Q; float P; int player; } oedge;
typedef struct { ostate s; uint8_t key[KEYLEN]; int e0, ne; } onode;
typedef struct {
  onode *nodes; int nn, cap_n;
  oedge *edges; int ne, cap_e;
  int *hslot; int hcap;
  int pyhash;
} otree;

static uint64_t key_hash(const uint8_t *k) {
  uint64_t h = 1469598103934665603ULL;
  for (int i = 0; i < KEYLEN; i++) { h ^= k[i]; h *= 1099511628211ULL; }
  return h;
}

static int tree_find(otree *t, const uint8_t *key) {
  uint64_t h = key_hash(key);
  for (int i = (int)(h & (uint64_t)(t->hcap - 1));; i = (i + 1) & (t->hcap - 1)) {
    int v = t->hslot[i];
    if (v < 0) return -1;
    if (!memcmp(t->nodes[v].key, key, KEYLEN)) return v;
  }
}

static void tree_insert_slot(otree *t, int v) {
  uint64_t h = key_hash(t->nodes[v].key);
  int i = (int)(h & (uint64_t)(t->hcap - 1));
  while (t->hslot[i] >= 0) i = (i + 1) & (t->hcap - 1);
  t->hslot[i] = v;
}

static int tree_add(otree *t, const ostate *s) {
  if (t->nn == t->cap_n) { t->cap_n *= 2; t->nodes = realloc(t->nodes, sizeof(onode) * t->cap_n); }
  if (2 * (t->nn + 1) > t->hcap) {
    t->hcap *= 2;
    free(t->hslot);
    t->hslot = malloc(sizeof(int) * t->hcap);
    for (int i = 0; i < t->hcap; i++) t->hslot[i] = -1;
    for (int v = 0; v < t->nn; v++) tree_insert_slot(t, v);
  }
  onode *nd = &t->nodes[t->nn];
  nd->s = *s;
  canonical_of(s, nd->key, t->pyhash);
  nd->e0 = -1; nd->ne = 0;
  tree_insert_slot(t, t->nn);
  return t->nn++;
}

static int st_game_over(const ostate *s) { return s->game_over && s->winner != -2; }

void or_stub_eval(const int16_t *st, float *policy, double *value) {
  ostate s;
  from_ref(st, &s);
  int64_t n0 = 0, n1 = 0;
  for (int c = 0; c < 23; c++) {
    n0 += s.board[0][c].h < 3 ? s.board[0][c].h : 3;
    n1 += s.board[1][c].h < 3 ? s.board[1][c].h : 3;
  }
  int64_t cp = s.player, ph3 = (s.phase >= 0 && s.phase <= 3) ? s.phase : 0, w = 0;
  for (int i = 0; i < 5 && i < s.npiles; i++)
    for (int t = 0; t < 6; t++) {
      int cnt = 0;
      for (int j = 0; j < s.pile_len[i]; j++) if (s.piles[i][j] == t) cnt++;
      w += (int64_t)cnt * (i * 6 + t + 1);
    }
  for (int t = 0; t < 6; t++) {
    int cnt = 0;
    for (int j = 0; j < s.nhand; j++) if (s.hand[j] == t) cnt++;
    w += (int64_t)cnt * (30 + t + 1);
  }
  int64_t K = (n0 * 73 + n1 * 151 + ph3 * 7 + cp * 3 + w * 13) % (1LL << 31);
  for (int a = 0; a < 143; a++) {
    uint64_t h = ((uint64_t)a * 2654435761ULL + (uint64_t)K * 40503ULL) % (1ULL << 32);
    policy[a] = (float)((h >> 22) + 1) / 1024.0f;
  }
  *value = (double)((K % 255) - 127) / 128.0;
}

static void stub_eval_state(const ostate *s, float *policy, double *value) {
  int16_t v[78];
  to_ref(s, v);
  or_stub_eval(v, policy, value);
}

int or_mcts_search(const int16_t *root_ref, or_mt *m, const or_mcts_cfg *cfg, const double *noise,
                   int32_t *visits, int32_t *n_nodes, int32_t *n_edges) {
  geom_init();
  otree t;
  t.cap_n = 1024; t.nodes = malloc(sizeof(onode) * t.cap_n); t.nn = 0;
  t.cap_e = 4096; t.edges = malloc(sizeof(oedge) * t.cap_e); t.ne = 0;
  t.hcap = 2048; t.hslot = malloc(sizeof(int) * t.hcap);
  t.pyhash = !cfg->exact_keys;
  for (int i = 0; i < t.hcap; i++) t.hslot[i] = -1;
  ostate root;
  from_ref(root_ref, &root);
  tree_add(&t, &root);
  int path[512];
  uint8_t mask[143];
  float pol[143];
  for (int sim = 0; sim < cfg->sims; sim++) {
    int node = 0, depth = 0;
    /* move_to_leaf (MCTS.py:63-149) */
    while (t.nodes[node].ne > 0) {
      if (!legal_of(&t.nodes[node].s, mask)) break;
      int ns = 0;
      for (int e = 0; e < t.nodes[node].ne; e++) ns += t.edges[t.nodes[node].e0 + e].N;
      double sqrt_ns = sqrt(ns > 1 ? (double)ns : 1.0);
      double best = -INFINITY;
      int sel = -1;
      for (int e = 0; e < t.nodes[node].ne; e++) {
        oedge *ed = &t.edges[t.nodes[node].e0 + e];
        if (!mask[ed->action]) continue;
        float cp = cfg->cpuct * ed->P;                       /* float32 * float32 */
        double u = (double)cp * sqrt_ns / (double)(1 + ed->N);
        double qu = ed->Q + u;
        if (qu > best) { best = qu; sel = t.nodes[node].e0 + e; }
      }
      if (sel < 0) break;
      path[depth++] = sel;
      node = t.edges[sel].child;
    }
    double value;
    const ostate *ls = &t.nodes[node].s;
    int leaf_player = ls->player;
    if (!st_game_over(ls)) {
      stub_eval_state(ls, pol, &value);
      if (cfg->negate_value) value = -value;
      if (node == 0 && !cfg->testing) {                    /* MCTS.py:308-327 */
        int L = legal_of(ls, mask);
        float one_m_eps = (float)(1.0 - cfg->eps);
        int i = 0;
        for (int a = 0; a < 143 && L; a++) {
          if (!mask[a]) continue;
          float a32 = one_m_eps * pol[a];
          double b64 = cfg->eps * noise[i++];
          pol[a] = (float)((double)a32 + b64);
        }
      }
      /* expand_leaf (MCTS.py:151-218) */
      int L = legal_of(&t.nodes[node].s, mask);
      if (L) {
        int e0 = t.ne, cnt = 0;
        for (int a = 0; a < 143; a++) {
          if (!mask[a]) continue;
          ostate child = t.nodes[node].s;
          step_state(&child, a, m);
          uint8_t key[KEYLEN];
          canonical_of(&child, key, t.pyhash);
          int c = tree_find(&t, key);
          if (c == node) continue;
          if (c < 0) c = tree_add(&t, &child);
          if (t.ne == t.cap_e) { t.cap_e *= 2; t.edges = realloc(t.edges, sizeof(oedge) * t.cap_e); }
          oedge *ed = &t.edges[t.ne++];
          ed->node = node; ed->action = a; ed->child = c; ed->N = 0; ed->W = 0; ed->Q = 0;
          ed->P = pol[a]; ed->player = t.nodes[node].s.player;
          cnt++;
        }
        t.nodes[node].e0 = e0;
        t.nodes[node].ne = cnt;
      }
    } else {
      int outcome = ls->winner == 0 ? 1 : ls->winner == 1 ? -1 : 0;
      value = leaf_player == 0 ? (double)outcome : -(double)outcome;
      if (outcome == 0) value = 0.0;
    }
    /* back_fill (MCTS.py:220-266) */
    for (int d = depth - 1; d >= 0; d--) {
      oedge *ed = &t.edges[path[d]];
      double dir = ed->player == leaf_player ? 1.0 : -1.0;
      ed->N += 1;
      ed->W += value * dir;
      ed->Q = ed->W / (double)ed->N;
    }
  }
  /* MCTS.py:354-441 */
  memset(visits, 0, sizeof(int32_t) * 143);
  int total = 0;
  for (int e = 0; e < t.nodes[0].ne; e++) {
    oedge *ed = &t.edges[t.nodes[0].e0 + e];
    visits[ed->action] = ed->N;
    total += ed->N;
  }
  int best = -1;
  int explore = !cfg->testing && cfg->ply < cfg->tau0;
  if (explore) {
    if (total > 0) {
      double target = cfg->u * (double)total;
      int cum = 0;
      for (int e = 0; e < t.nodes[0].ne; e++) {
        oedge *ed = &t.edges[t.nodes[0].e0 + e];
        cum += ed->N;
        if (target < (double)cum) { best = ed->action; break; }
      }
    }
  } else {
    int maxv = -1;
    for (int e = 0; e < t.nodes[0].ne; e++) {
      oedge *ed = &t.edges[t.nodes[0].e0 + e];
      if (ed->N > maxv) { maxv = ed->N; best = ed->action; }
    }
  }
  if (best < 0) {                                          /* random.choice fallback */
    int L = legal_of(&t.nodes[0].s, mask);
    if (L) best = kth_legal(mask, (int)or_randbelow(m, (uint32_t)L));
  }
  if (n_nodes) *n_nodes = t.nn;
  if (n_edges) *n_edges = t.ne;
  free(t.nodes); free(t.edges); free(t.hslot);
  return best;
}

/* ---------------------------------------------------------- greedy agent
 * evaluation.py:137-196 choose_move_greedy: apply every legal move (in the
 * canonical ascending action order) to a copy of the state — each apply
 * consumes the chance stream exactly like the reference's apply_move, whose
 * turn end refills the piles from the global `random` — score the copy for
 * the player to move, keep the first strictly best.  Returns the action, or
 * -1 when there is no legal move. */
int or_greedy_move(const int16_t *st, or_mt *m) {
  uint8_t mask[143];
  int L = or_legal(st, mask);
  if (!L) return -1;
  int p = st[72];
  int best = -1, best_score = -1;
  for (int a = 0; a < 143; a++) {
    if (!mask[a]) continue;
    int16_t t[OR_REFSTATE];
    memcpy(t, st, sizeof(t));
    if (or_step(t, a, m)) continue; /* the reference skips moves that raise */
    uint8_t cells[23];
    for (int c = 0; c < 23; c++) cells[c] = (uint8_t)t[p * 23 + c];
    int32_t parts[5];
    or_score_board(cells, parts);
    int sc = parts[0] + parts[1] + parts[2] + parts[3] + parts[4];
    if (sc > best_score) {
      best_score = sc;
      best = a;
    }
  }
  return best;
}
