// hz_device.hpp — the Harmonies rules as CDNA4 device code.
//
// One lane owns one board ("lane-per-board"): every rule below is a handful
// of 32/64-bit bitboard operations, so a wave advances 64 independent games
// per instruction and the SoA state loads/stores are fully coalesced.
//
// Board state (48 B, six u64 words, stored SoA in HBM: word w of board b at
// st[w * N + b]):
//   pl[0..3]  bit-planes of the 4-bit stack code of every cell;
//             player 0 in bits 0..22, player 1 in bits 32..54
//             (cell = index into sorted(VALID_HEXES), constants.py:47-49)
//   piles     5 piles x 3 tiles x 3 bits (7 = no tile), bits 45..47 = #piles
//   misc      hand 3x3 bits | #hand 2 | bag 6x5 bits (TILE_TYPES order) |
//             player 1 | phase 3 | game_over 1 | winner 2 | score0 8 | score1 8
// Stack codes (every stack the placement rules can build,
// harmonies_engine.py:183-194): 0 empty, 1+t a single tile t,
// 7 wood+plant, 8 stone+stone, 9 stone x3, 10 wood+building,
// 11 stone+building, 12 building+building.
//
// Chance: each board owns a CPython MT19937 stream (624 words SoA + a cursor)
// seeded exactly like random.seed(int), consumed exactly like
// random.sample(range(n), k) (Lib/random.py:239-249, :480-503).  The twist is
// done lazily one word at a time (cursor in [624,1248) = "words below
// cursor-624 are already twisted"), which is bit-identical to CPython's
// batch twist for the consumed outputs; hz_mt_normalize turns it back into
// CPython's (mt, index) form.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hz {

constexpr int kCells = 23;
constexpr uint32_t kAll23 = (1u << 23) - 1;
constexpr int kActions = 143;
enum { WATER = 0, PLANT = 1, WOOD = 2, STONE = 3, BUILDING = 4, FIELD = 5 };
enum { PH_CHOOSE = 0, PH_P1 = 1, PH_P2 = 2, PH_P3 = 3, PH_OVER = 4 };
enum {
  ST_OK = 0, ST_BAD_PILE = 1, ST_BAD_FORMAT = 2, ST_NOT_IN_HAND = 3, ST_ILLEGAL_STACK = 4,
  ST_BAD_PHASE = 5, ST_BAD_ACTION = 6, ST_NOOP = 7
};

// INITIAL_BAG (constants.py:41) in TILE_TYPES order.
__host__ __device__ constexpr int initial_count(int t) {
  return t == WATER ? 23 : t == PLANT ? 19 : t == WOOD ? 21 : t == STONE ? 23 : t == BUILDING ? 15 : 19;
}

struct State {
  uint64_t pl[4];
  uint64_t piles;
  uint64_t misc;
};

// ------------------------------------------------------------------ fields
__device__ __forceinline__ int hand_tile(uint64_t m, int j) { return (int)((m >> (3 * j)) & 7); }
__device__ __forceinline__ int hand_n(uint64_t m) { return (int)((m >> 9) & 3); }
__device__ __forceinline__ int bag_n(uint64_t m, int t) { return (int)((m >> (11 + 5 * t)) & 31); }
__device__ __forceinline__ int player_of(uint64_t m) { return (int)((m >> 41) & 1); }
__device__ __forceinline__ int phase_of(uint64_t m) { return (int)((m >> 42) & 7); }
__device__ __forceinline__ int over_flag(uint64_t m) { return (int)((m >> 45) & 1); }
__device__ __forceinline__ int winner_code(uint64_t m) { return (int)((m >> 46) & 3); }  // 0 None,1 P0,2 P1,3 draw
__device__ __forceinline__ int score_of(uint64_t m, int p) { return (int)((m >> (48 + 8 * p)) & 255); }
__device__ __forceinline__ int npiles_of(uint64_t piles) { return (int)((piles >> 45) & 7); }
__device__ __forceinline__ int pile_tile(uint64_t piles, int i, int j) { return (int)((piles >> (9 * i + 3 * j)) & 7); }

__device__ __forceinline__ uint64_t set_bits(uint64_t w, int lo, int width, uint64_t v) {
  uint64_t mask = ((1ull << width) - 1) << lo;
  return (w & ~mask) | ((v << lo) & mask);
}

__device__ __forceinline__ int bag_total(uint64_t m) {
  int s = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) s += bag_n(m, t);
  return s;
}

// is_game_over(): game_over and winner is not None (harmonies_engine.py:332-333)
__device__ __forceinline__ bool game_done(uint64_t m) { return over_flag(m) && winner_code(m) != 0; }

// ------------------------------------------------------------- bitboards
__device__ __forceinline__ void planes_of(const State& s, int p, uint32_t b[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = (uint32_t)(s.pl[k] >> (32 * p)) & kAll23;
}

template <int C>
__device__ __forceinline__ uint32_t is_code(const uint32_t b[4]) {
  uint32_t m = kAll23;
  m &= (C & 1) ? b[0] : ~b[0];
  m &= (C & 2) ? b[1] : ~b[1];
  m &= (C & 4) ? b[2] : ~b[2];
  m &= (C & 8) ? b[3] : ~b[3];
  return m;
}

__device__ __forceinline__ int code_at(const State& s, int p, int c) {
  int sh = 32 * p + c;
  return (int)(((s.pl[0] >> sh) & 1) | (((s.pl[1] >> sh) & 1) << 1) | (((s.pl[2] >> sh) & 1) << 2) |
               (((s.pl[3] >> sh) & 1) << 3));
}

__device__ __forceinline__ void set_code(State& s, int p, int c, int code) {
  int sh = 32 * p + c;
#pragma unroll
  for (int k = 0; k < 4; k++) s.pl[k] = (s.pl[k] & ~(1ull << sh)) | ((uint64_t)((code >> k) & 1) << sh);
}

// New stack code after placing tile t on a stack, or -1 if illegal
// (harmonies_engine.py:254-283; same rules as get_legal_moves :183-194).
__device__ __forceinline__ int place_code(int code, int t) {
  if (code == 0) return 1 + t;
  if (t == PLANT && code == 3) return 7;
  if (t == STONE && code == 4) return 8;
  if (t == STONE && code == 8) return 9;
  if (t == BUILDING && code == 3) return 10;
  if (t == BUILDING && code == 4) return 11;
  if (t == BUILDING && code == 5) return 12;
  return -1;
}

// Tile at stack position pos (0 = bottom) for a code; 7 = none.
__host__ __device__ constexpr uint64_t pack_tab(const int* v) {
  uint64_t r = 0;
  for (int i = 0; i < 13; i++) r |= (uint64_t)v[i] << (3 * i);
  return r;
}
constexpr int kTab0[13] = {7, 0, 1, 2, 3, 4, 5, 2, 3, 3, 2, 3, 4};
constexpr int kTab1[13] = {7, 7, 7, 7, 7, 7, 7, 1, 3, 3, 4, 4, 4};
constexpr int kTab2[13] = {7, 7, 7, 7, 7, 7, 7, 7, 7, 3, 7, 7, 7};
constexpr uint64_t kStackPos0 = pack_tab(kTab0);
constexpr uint64_t kStackPos1 = pack_tab(kTab1);
constexpr uint64_t kStackPos2 = pack_tab(kTab2);

__device__ __forceinline__ int tile_at(int code, int pos) {
  uint64_t t = pos == 0 ? kStackPos0 : pos == 1 ? kStackPos1 : kStackPos2;
  return (int)((t >> (3 * code)) & 7);
}

// ----------------------------------------------------------- hex geometry
// 5x7 grid layout for neighbour shifts: bit = (r+2)*7 + (q+3)
// (process_game_state.py:9-12,36-37).  Axial direction (dq,dr) is a shift by
// 7*dr + dq; every wrap-around lands on an invalid cell, masked by kValid35.
__host__ __device__ constexpr int grid_bit(int c) {
  // sorted(VALID_HEXES) -> (q, r)
  constexpr int Q[23] = {-3, -2, -2, -2, -1, -1, -1, -1, -1, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 3};
  constexpr int R[23] = {2, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, -2};
  return (R[c] + 2) * 7 + (Q[c] + 3);
}
__host__ __device__ constexpr uint64_t valid35() {
  uint64_t v = 0;
  for (int c = 0; c < 23; c++) v |= 1ull << grid_bit(c);
  return v;
}
constexpr uint64_t kValid35 = valid35();

// Scoring layout: column-major with a guard row, bit = (q+3)*6 + (r+2).
// Axial direction (dq,dr) is a shift by 6*dq + dr (+-1, +-5, +-6); every
// wrap-around lands on a guard row (r = 3) or outside the 7 columns, masked
// by kValid42.  A column's cells are consecutive cell indices with
// consecutive r, so the conversion from the 23-bit cell set is 7 runs.
__host__ __device__ constexpr int col_bit(int c) {
  constexpr int Q[23] = {-3, -2, -2, -2, -1, -1, -1, -1, -1, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 3};
  constexpr int R[23] = {2, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, 1, 2, -2, -1, 0, -2};
  return (Q[c] + 3) * 6 + (R[c] + 2);
}
__host__ __device__ constexpr uint64_t valid42() {
  uint64_t v = 0;
  for (int c = 0; c < 23; c++) v |= 1ull << col_bit(c);
  return v;
}
constexpr uint64_t kValid42 = valid42();
static_assert(col_bit(0) == 4 && col_bit(1) == 8 && col_bit(4) == 12 && col_bit(9) == 18 && col_bit(14) == 24 &&
                  col_bit(19) == 30 && col_bit(22) == 36,
              "column runs");

__device__ __forceinline__ uint64_t to42(uint32_t m) {
  uint32_t lo = ((m & 1u) << 4) | (((m >> 1) & 7u) << 8) | (((m >> 4) & 31u) << 12) | (((m >> 9) & 31u) << 18) |
                (((m >> 14) & 31u) << 24) | (((m >> 19) & 3u) << 30);
  uint32_t hi = ((m >> 21) & 1u) | (((m >> 22) & 1u) << 4);  // bits 32 and 36
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t nbr42(uint64_t s) {
  return ((s << 1) | (s >> 1) | (s << 5) | (s >> 5) | (s << 6) | (s >> 6)) & kValid42;
}

// ------------------------------------------------------------------ scoring
// calculate_score_for_player (harmonies_engine.py:357-523) on bitboards.
__device__ __forceinline__ int water_points(int len) {  // :18-27
  if (len <= 0) return 0;
  if (len <= 6) return (int)((0x000F0B0805020000ull >> (8 * len)) & 0xFF);
  return 15 + (len - 6) * 4;
}

// The connected-component part of scoring for one 23-bit cell set S:
// low byte  = number of components of size >= 2 (fields, :424-452: +5 each),
// high byte = sum over those components of get_water_score(d + 1) with d the
// component's graph diameter (water, :480-523).  Flood fill + BFS from every
// cell; evaluated for all 2^23 sets once per process into kCompTable.
__device__ __forceinline__ uint32_t comp_stats(uint32_t set23) {
  uint64_t all = to42(set23);
  uint64_t two = all & nbr42(all);  // cells of components of size >= 2
  int ncomp = 0, wpts = 0;
  while (two) {
    uint64_t comp = two & (~two + 1);
    for (;;) {
      uint64_t nx = (comp | nbr42(comp)) & two;
      if (nx == comp) break;
      comp = nx;
    }
    two &= ~comp;
    ncomp++;
    int diam = 0;
    uint64_t todo = comp;
    while (todo) {
      uint64_t reach = todo & (~todo + 1);
      todo &= ~reach;
      int d = 0;
      for (;;) {
        uint64_t nx = (reach | nbr42(reach)) & comp;
        if (nx == reach) break;
        reach = nx;
        d++;
      }
      diam = d > diam ? d : diam;
    }
    wpts += water_points(diam + 1);
  }
  return (uint32_t)ncomp | ((uint32_t)wpts << 8);
}

constexpr uint32_t kCompTableSize = 1u << 23;  // u16 entries (16 MiB)

namespace {
// this translation unit's copy of the table pointer (install_comp_table)
__device__ const uint16_t *g_comp_table;

__global__ void __launch_bounds__(256) k_comp_table(uint16_t *__restrict__ t) {
  uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s < kCompTableSize) t[s] = (uint16_t)comp_stats(s);
}

// Build the component table once per device (for this translation unit) and
// point g_comp_table at it.  Host side; returns 0 on success.
inline int install_comp_table() {
  static const uint16_t *tables[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!tables[dev]) {
    uint16_t *t = nullptr;
    if (hipMalloc(&t, kCompTableSize * sizeof(uint16_t)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_comp_table, dim3(kCompTableSize / 256), dim3(256), 0, 0, t);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(t);
      return 1;
    }
    tables[dev] = t;
  }
  const uint16_t *p = tables[dev];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_comp_table), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
}  // namespace

struct ScoreParts { int grass, mount, field, bldg, water; };

__device__ __forceinline__ ScoreParts score_parts(const uint32_t b23[4]) {
  // fields and water: one table load each (issued first)
  uint32_t f23 = is_code<6>(b23), w23 = is_code<1>(b23);
  uint32_t tf = g_comp_table[f23], tw = g_comp_table[w23];
  uint64_t b[4];
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = to42(b23[k]);
  auto is = [&](int c) -> uint64_t {
    uint64_t m = kValid42;
    m &= (c & 1) ? b[0] : ~b[0];
    m &= (c & 2) ? b[1] : ~b[1];
    m &= (c & 4) ? b[2] : ~b[2];
    m &= (c & 8) ? b[3] : ~b[3];
    return m;
  };
  ScoreParts r;
  // grass :369-390 (h1 plant 1; wood+plant 3; the h3 case is unreachable)
  r.grass = __popc(is_code<2>(b23)) + 3 * __popc(is_code<7>(b23));
  // mountains :392-422: stone tops with a stone-top neighbour, by height
  uint64_t st1 = is(4), st2 = is(8), st3 = is(9);
  uint64_t stone = st1 | st2 | st3;
  uint64_t adj = stone & nbr42(stone);
  r.mount = __popcll(adj & st1) + 3 * __popcll(adj & st2) + 7 * __popcll(adj & st3);
  // buildings :454-478 — a building on top at height 2 with >= 3 distinct
  // neighbouring top types: per cell, count the types among its neighbours
  // with a bit-sliced adder over the six "next to a t-top" sets
  uint64_t bh2 = is(10) | is(11) | is(12);
  r.bldg = 0;
  if (bh2) {
    uint64_t x0 = nbr42(is(1));                                 // water
    uint64_t x1 = nbr42(is(2) | is(7));                         // plant
    uint64_t x2 = nbr42(is(3));                                 // wood
    uint64_t x3 = nbr42(stone);                                 // stone
    uint64_t x4 = nbr42(is(5) | is(10) | is(11) | is(12));      // building
    uint64_t x5 = nbr42(is(6));                                 // field
    uint64_t s1 = x0 ^ x1 ^ x2, c1 = (x0 & x1) | (x2 & (x0 ^ x1));
    uint64_t s2 = x3 ^ x4 ^ x5, c2 = (x3 & x4) | (x5 & (x3 ^ x4));
    uint64_t ge3 = (c1 & c2) | ((c1 | c2) & (s1 | s2));
    r.bldg = 5 * __popcll(ge3 & bh2);
  }
  r.field = 5 * (int)(tf & 0xFF);
  r.water = (int)(tw >> 8);
  return r;
}

__device__ __forceinline__ int score_player(const State& s, int p) {
  uint32_t b[4];
  planes_of(s, p, b);
  ScoreParts r = score_parts(b);
  return r.grass + r.mount + r.field + r.bldg + r.water;
}

// ------------------------------------------------------------------ MT19937
// A board's stream: 624 words at w[0..623] (board-major in HBM, or an LDS
// copy) and a cursor packed as pos | tw << 16:
//   pos = outputs consumed in the current generation (CPython's index),
//   tw  = words of the current generation already twisted in place.
// CPython twists all 624 words when index reaches N; we twist 8 at a time,
// on demand, in one memory round trip per block.  The outputs are identical;
// hz_mt_normalize finishes the twist (tw = 624) to recover CPython's state.
constexpr int kMT = 624;
constexpr int kMTSeeded = 624 | (624 << 16);  // CPython state right after seed()

__device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t twist_word(uint32_t cur, uint32_t next, uint32_t far) {
  uint32_t y = (cur & 0x80000000U) | (next & 0x7fffffffU);
  return far ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
}

// twist words [start, start + k), k = min(8, 624 - start), start == tw, of a
// stream whose word i is at w[i * S]: sources below tw are new, from tw on
// old, so all loads issue together.  Returns k.
template <class Ptr>
__device__ __forceinline__ int twist_block(Ptr w, int S, int start) {
  int k = kMT - start < 8 ? kMT - start : 8;
  uint32_t cur[9], far[8];
#pragma unroll
  for (int j = 0; j < 9; j++) {
    int i = start + j;
    cur[j] = (j <= k) ? w[(i < kMT ? i : 0) * S] : 0u;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    int i = start + j;
    int fi = i < 227 ? i + 397 : (i < 623 ? i - 227 : 396);
    far[j] = (j < k) ? w[fi * S] : 0u;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (j < k) w[(start + j) * S] = twist_word(cur[j], cur[j + 1], far[j]);
  }
  return k;
}

// twist_block for a board-major stream in global memory with 16-B accesses:
// a wave's dword loads of 64 streams touch 64 lines each, so the vector
// form moves the same lines with a quarter of the instructions.  start is a
// multiple of 8 (the cursor's tw); the far words of block start are 8
// consecutive words at 1 mod 4 (i + 397 or i - 227), except for start = 224
// (they wrap from word 623 to 0: dword loads there).
__device__ __forceinline__ int twist_block_vec(uint32_t* w, int start) {
  const uint4 c0 = *(const uint4*)(w + start), c1 = *(const uint4*)(w + start + 4);
  const uint32_t c8 = w[start + 8 < kMT ? start + 8 : 0];
  uint32_t far[8];
  if (start == 224) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int i = start + j;
      far[j] = w[i < 227 ? i + 397 : i - 227];
    }
  } else {
    const int f0 = start < 227 ? start + 397 : start - 227;  // = 1 mod 4
    const uint4 a = *(const uint4*)(w + f0 - 1), b = *(const uint4*)(w + f0 + 3), c = *(const uint4*)(w + f0 + 7);
    far[0] = a.y; far[1] = a.z; far[2] = a.w; far[3] = b.x;
    far[4] = b.y; far[5] = b.z; far[6] = b.w; far[7] = c.x;
  }
  const uint32_t cur[9] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c8};
  uint32_t o[8];
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = twist_word(cur[j], cur[j + 1], far[j]);
  *(uint4*)(w + start) = make_uint4(o[0], o[1], o[2], o[3]);
  *(uint4*)(w + start + 4) = make_uint4(o[4], o[5], o[6], o[7]);
  return 8;
}

// A board's stream in global memory (board-major, contiguous): used by the
// one-draw-per-call kernels (hz_step, hz_end_turn, ...) and the MCTS chance
// replay.  Cursor = pos | tw << 16: pos = CPython's index, tw = words of the
// current generation already twisted in place (8 at a time, on demand);
// hz_mt_normalize finishes the twist to recover CPython's (mt, index).
template <int S>
struct MTS {
  uint32_t* w;  // word i at w[i * S]
  int pos, tw;

  __device__ __forceinline__ MTS(uint32_t* words, int cursor) : w(words), pos(cursor & 0xFFFF), tw(cursor >> 16) {}
  __device__ __forceinline__ int cursor() const { return pos | (tw << 16); }
  __device__ __forceinline__ void prefetch() {}

  // genrand_uint32
  __device__ __forceinline__ uint32_t next() {
    if (pos >= kMT) { pos = 0; tw = 0; }
    if (pos >= tw) tw += twist_block(w, S, tw);
    return temper(w[(pos++) * S]);
  }

  // finish the current generation's twist (CPython form afterwards)
  __device__ __forceinline__ void normalize() {
    if (pos >= kMT) return;
    while (tw < kMT) tw += twist_block(w, S, tw);
  }
};
using MT = MTS<1>;

// MT with a read-ahead window, for the one-draw-per-call kernels of the
// per-ply surface (hz_step, hz_rule_ply): at the start of a draw, prefetch()
// twists in place up to W words past the cursor (twist_block: one round trip
// per 8 words) and loads those W words at once; the draw's picks then pop
// them from a register queue (shifted, never indexed: a per-lane dynamic
// index would put the window in scratch) instead of waiting one memory round
// trip per word.  Past the window next() is MT's.  The words read and the
// cursor left are MT's: a turn-ending ply no longer waits ~5 dependent loads.
template <int W>
struct WinGMT {
  uint32_t* w;
  int pos, tw, left;
  bool fresh;  // the window was fetched and nothing popped since (an early prefetch: the draw's is a no-op)
  uint32_t q[W];

  __device__ __forceinline__ WinGMT(uint32_t* words, int cursor)
      : w(words), pos(cursor & 0xFFFF), tw(cursor >> 16), left(0), fresh(false) {}
  __device__ __forceinline__ int cursor() const { return pos | (tw << 16); }

  __device__ __forceinline__ void prefetch() {
    static_assert(W % 4 == 0, "window of whole 16-B loads");
    if (fresh) return;
    fresh = true;
    if (pos >= kMT) { pos = 0; tw = 0; }
    while (tw < kMT && tw < pos + W) tw += twist_block_vec(w, tw);
    left = tw - pos < W ? tw - pos : W;
    // words [pos, pos + W) from W / 4 + 1 aligned 16-B loads (a load past
    // the stream's end rereads its last four words: positions >= 624 are
    // never used), shifted by pos & 3 with selects (no dynamic index)
    const int a = pos & ~3, sh = pos & 3;
    uint32_t f[W + 4];
#pragma unroll
    for (int k = 0; k < W / 4 + 1; k++) {
      const int o = a + 4 * k <= kMT - 4 ? a + 4 * k : kMT - 4;
      const uint4 v = *(const uint4*)(w + o);
      f[4 * k] = v.x; f[4 * k + 1] = v.y; f[4 * k + 2] = v.z; f[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < W; j++) q[j] = sh == 0 ? f[j] : sh == 1 ? f[j + 1] : sh == 2 ? f[j + 2] : f[j + 3];
  }

  __device__ __forceinline__ uint32_t next() {
    fresh = false;
    if (left > 0) {
      const uint32_t v = q[0];
#pragma unroll
      for (int j = 0; j + 1 < W; j++) q[j] = q[j + 1];
      left--;
      pos++;
      return temper(v);
    }
    if (pos >= kMT) { pos = 0; tw = 0; }
    if (pos >= tw) tw += twist_block(w, 1, tw);
    return temper(w[pos++]);
  }
};
using WinMT12 = WinGMT<12>;

// Dynamic LDS of the lane-per-board kernels: the wave's 64 streams as
// [624][65] words (word i of lane l at i*65 + l).  Addressing through this
// __shared__ symbol keeps every access a 32-bit LDS address.
constexpr int kLdsStride = 65;
extern __shared__ uint32_t hz_lds[];

// A board's stream resident in LDS (k_reset / k_rollout).  Draws scan the
// next <= 24 twisted words in place, branch-free; prefetch() twists ahead
// at a point the whole wave reaches together (the start of a draw).
struct LdsMT {
  int lane, pos, tw;
  __device__ __forceinline__ LdsMT(int l, int cursor) : lane(l), pos(cursor & 0xFFFF), tw(cursor >> 16) {}
  __device__ __forceinline__ int cursor() const { return pos | (tw << 16); }
  __device__ __forceinline__ uint32_t* w() const { return hz_lds + lane; }

  __device__ __forceinline__ void prefetch() {
    if (pos >= kMT) { pos = 0; tw = 0; }
    while (tw < kMT && tw < pos + 24) tw += twist_block(w(), kLdsStride, tw);
  }

  __device__ __forceinline__ uint32_t word(int i) const {  // tempered output i (i < tw)
    return temper(hz_lds[(i < kMT ? i : kMT - 1) * kLdsStride + lane]);
  }

  __device__ __forceinline__ uint32_t next() {
    if (pos >= kMT) { pos = 0; tw = 0; }
    if (pos >= tw) tw += twist_block(w(), kLdsStride, tw);
    return word(pos++);
  }

  __device__ __forceinline__ void normalize() {
    if (pos >= kMT) return;
    while (tw < kMT) tw += twist_block(w(), kLdsStride, tw);
  }

  // start the next generation now and twist its first `target` words
  // (k_seed_ahead: a typical game then never twists)
  __device__ __forceinline__ void twist_ahead(int target) {
    if (pos >= kMT) { pos = 0; tw = 0; }
    while (tw < target) tw += twist_block(w(), kLdsStride, tw);
  }
};

// cursor of a seeded-ahead stream: fresh generation, kAheadTwist words twisted
constexpr int kAheadTwist = 224;
constexpr int kMTAhead = 0 | (kAheadTwist << 16);

// init_genrand(19650218) (_randommodule.c), the starting array of
// init_by_array: the same for every seed, so it is a constant table read
// through the scalar cache instead of a per-step multiply chain.
struct InitGen { uint32_t v[kMT]; };
constexpr InitGen make_init_gen() {
  InitGen g{};
  uint32_t x = 19650218u;
  g.v[0] = x;
  for (int i = 1; i < kMT; i++) {
    x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
    g.v[i] = x;
  }
  return g;
}
__constant__ InitGen kInitGen = make_init_gen();

// random.seed(int) for 0 <= seed < 2^64 (_randommodule.c random_seed +
// init_by_array with key = the seed's 32-bit words) into w[i * stride].
// Both passes are serial recurrences; the code keeps each step to its five
// dependent ALU ops (key selection unrolled by two, pass-1 words read eight
// ahead in pass 2).  The stream's cursor afterwards is kMTSeeded.  After
// each group of pass 2, `prog(r)` reports rows [2, r) final (the seed stage
// publishes them to waves that store them meanwhile).
struct NoProgress {
  __device__ __forceinline__ void operator()(int) const {}
};
template <class Ptr, class Prog = NoProgress>
__device__ __forceinline__ void mt_seed(Ptr w, int stride, uint64_t seed, Prog prog = Prog()) {
  uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  // key[j] + j for j = (i - 1) % keylen: odd i -> kA, even i -> kB
  uint32_t kA = key0, kB = key1 ? key1 + 1u : key0;
  uint32_t prev = 19650218u;  // mt[i-1]
  // first pass: i = 1..623 (mt[0] = mt[623] afterwards, then one more step
  // at i = 1); table words fetched a group of eight ahead
  uint32_t iv[8];
#pragma unroll
  for (int u = 0; u < 8; u++) iv[u] = kInitGen.v[1 + u];
  for (int g = 1; g < kMT - 7; g += 8) {  // g = 1, 9, ..., 609 (groups end at 616)
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = kInitGen.v[g + 8 + u < kMT ? g + 8 + u : kMT - 1];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      w[(g + u) * stride] = v;
      prev = v;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = nx[u];
  }
#pragma unroll
  for (int u = 0; u < 7; u++) {  // i = 617..623
    uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
    w[(617 + u) * stride] = v;
    prev = v;
  }
  // iteration 624 at i = 1 with j = 623 % keylen (-> kB)
  uint32_t m1 = w[1 * stride];
  prev = (m1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB;
  w[1 * stride] = prev;
  uint32_t first1 = prev;
  // second pass: i = 2..623, pass-1 words fetched eight ahead
  uint32_t cur[8];
#pragma unroll
  for (int u = 0; u < 8; u++) cur[u] = w[(2 + u) * stride];
  for (int g = 2; g < kMT - 6; g += 8) {  // g = 2, 10, ..., 610 (groups end at 617)
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = w[(g + 8 + u < kMT ? g + 8 + u : kMT - 1) * stride];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (cur[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(g + u);
      w[(g + u) * stride] = v;
      prev = v;
    }
    prog(g + 8);
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = nx[u];
  }
#pragma unroll
  for (int u = 0; u < 6; u++) {  // i = 618..623
    uint32_t v = (cur[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(618 + u);
    w[(618 + u) * stride] = v;
    prev = v;
  }
  // mt[0] = mt[623]; last step at i = 1; then mt[0] = 0x80000000
  w[1 * stride] = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
  w[0] = 0x80000000U;
}

// mt_seed with init_genrand's table read from an LDS copy (`tab`, 624
// words, the same for every board: broadcast reads) instead of through the
// scalar cache, whose waits also drain the pending LDS stores; rows at
// w[i * S] (S a compile-time stride).
template <int S, class Prog = NoProgress>
__device__ __forceinline__ void mt_seed_tab(uint32_t *w, const uint32_t *tab, uint64_t seed, Prog prog = Prog()) {
  uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  uint32_t kA = key0, kB = key1 ? key1 + 1u : key0;
  uint32_t prev = 19650218u;
  uint32_t iv[8];
#pragma unroll
  for (int u = 0; u < 8; u++) iv[u] = tab[1 + u];
#pragma unroll 2
  for (int g = 1; g < kMT - 7; g += 8) {  // i = 1..616
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = tab[g + 8 + u < kMT ? g + 8 + u : kMT - 1];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      w[(g + u) * S] = v;
      prev = v;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = nx[u];
  }
#pragma unroll
  for (int u = 0; u < 7; u++) {  // i = 617..623
    uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
    w[(617 + u) * S] = v;
    prev = v;
  }
  uint32_t m1 = w[1 * S];
  prev = (m1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB;
  w[1 * S] = prev;
  uint32_t first1 = prev;
  uint32_t cur[8];
#pragma unroll
  for (int u = 0; u < 8; u++) cur[u] = w[(2 + u) * S];
#pragma unroll 2
  for (int g = 2; g < kMT - 6; g += 8) {  // i = 2..617
    uint32_t kneg = __builtin_amdgcn_readfirstlane(0u - (uint32_t)g);
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = w[(g + 8 + u < kMT ? g + 8 + u : kMT - 1) * S];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      // (cur ^ p) - (g + u) as one v_xad_u32 with the offset in an SGPR
      uint32_t p = (prev ^ (prev >> 30)) * 1566083941U, v;
      asm("v_xad_u32 %0, %1, %2, %3" : "=v"(v) : "v"(p), "v"(cur[u]), "s"(kneg - (uint32_t)u));
      w[(g + u) * S] = v;
      prev = v;
    }
    prog(g + 8);
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = nx[u];
  }
#pragma unroll
  for (int u = 0; u < 6; u++) {  // i = 618..623
    uint32_t v = (cur[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(618 + u);
    w[(618 + u) * S] = v;
    prev = v;
  }
  w[1 * S] = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
  w[0] = 0x80000000U;
}

// init_by_array (random.seed) split at its pass boundary, the stream word-
// major in global memory (word i of the board at w[i * ns]), so that the
// chain's wave issues no LDS operation (hz_play's second pipeline, hz_env.hip
// "pipeline 2"): pass 1 leaves mt[1] (the 624th iteration's value) and
// mt[2..623] as pass 2 reads them; pass 2 finishes the array (cursor
// kMTSeeded).  The two together write exactly mt_seed's words.
__device__ __forceinline__ void mt_seed_pass1_g(uint32_t* __restrict__ w, size_t ns, uint64_t seed) {
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  const uint32_t kA = key0, kB = key1 ? key1 + 1u : key0;
  uint32_t prev = 19650218u, m1 = 0;
  for (int g = 1; g < kMT - 7; g += 8) {  // i = 1..616
    uint32_t iv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = kInitGen.v[g + u];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      if (u || g > 1) w[(size_t)(g + u) * ns] = v;
      else m1 = v;
      prev = v;
    }
  }
#pragma unroll
  for (int u = 0; u < 7; u++) {  // i = 617..623
    const uint32_t v = (kInitGen.v[617 + u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
    w[(size_t)(617 + u) * ns] = v;
    prev = v;
  }
  // mt[0] = mt[623]; the 624th iteration at i = 1 (key j = 623 % keylen -> kB)
  w[ns] = (m1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB;
}
template <int PF = 16>
__device__ __forceinline__ void mt_seed_pass2_g(uint32_t* __restrict__ w, size_t ns) {
  const uint32_t first1 = w[ns];
  uint32_t prev = first1;
  uint32_t ring[PF];  // pass-1 words PF iterations ahead
#pragma unroll
  for (int u = 0; u < PF; u++) ring[u] = w[(size_t)(2 + u) * ns];
  constexpr int kFull = 2 + ((kMT - 2) / PF) * PF;
  for (int g = 2; g < kFull; g += PF) {
#pragma unroll
    for (int u = 0; u < PF; u++) {
      const uint32_t cur = ring[u];
      const int nx = g + PF + u;
      ring[u] = nx < kMT ? w[(size_t)nx * ns] : 0u;
      const uint32_t v = (cur ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(g + u);
      w[(size_t)(g + u) * ns] = v;
      prev = v;
    }
  }
#pragma unroll
  for (int u = 0; u < (kMT - 2) % PF; u++) {
    const uint32_t v = (ring[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(kFull + u);
    w[(size_t)(kFull + u) * ns] = v;
    prev = v;
  }
  w[ns] = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
  w[0] = 0x80000000U;
}
// rows [0, rows) of a seeded stream (rows <= 227: every source still old)
// twisted in place, the next generation's start: the stream afterwards has
// cursor 0 | rows << 16 (kMTAhead for rows = kAheadTwist)
__device__ __forceinline__ void mt_pretwist_g(uint32_t* __restrict__ w, size_t ns, int rows) {
  constexpr int B = 8;
  for (int i0 = 0; i0 < rows; i0 += B) {
    uint32_t cur[B + 1], far[B];
#pragma unroll
    for (int j = 0; j <= B; j++) cur[j] = w[(size_t)(i0 + j) * ns];
#pragma unroll
    for (int j = 0; j < B; j++) far[j] = w[(size_t)(i0 + j + 397) * ns];
#pragma unroll
    for (int j = 0; j < B; j++)
      if (i0 + j < rows) w[(size_t)(i0 + j) * ns] = twist_word(cur[j], cur[j + 1], far[j]);
  }
}

// A board's stream in global memory with a runtime word stride (a pipeline-2
// stream slot, word-major: stride = the slot's row length).  As MTS.
struct MTR {
  uint32_t* w;
  int stride, pos, tw;
  __device__ __forceinline__ MTR(uint32_t* words, int s, int cursor)
      : w(words), stride(s), pos(cursor & 0xFFFF), tw(cursor >> 16) {}
  __device__ __forceinline__ int cursor() const { return pos | (tw << 16); }
  __device__ __forceinline__ void prefetch() {}
  __device__ __forceinline__ uint32_t next() {
    if (pos >= kMT) { pos = 0; tw = 0; }
    if (pos >= tw) tw += twist_block(w, stride, tw);
    return temper(w[(size_t)(pos++) * stride]);
  }
};

template <class M>
__device__ __forceinline__ uint32_t randbelow(M& m, uint32_t n) {
  if (!n) return 0;
  int k = 32 - __clz(n);
  uint32_t r = m.next() >> (32 - k);
  while (r >= n) r = m.next() >> (32 - k);
  return r;
}

// random.sample(range(n), k), k <= 3 (so setsize = 21, random.py:484-486),
// one word at a time (slow path); resumes after `got` picks.
template <class M>
__device__ __forceinline__ void sample3_serial(M& m, uint32_t n, int k, uint32_t j[3], int got) {
  if (n <= 21) {
    for (int i = got; i < k; i++) j[i] = randbelow(m, n - (uint32_t)i);
  } else {
    for (int i = got; i < k; i++) {
      uint32_t v;
      bool dup;
      do {
        v = randbelow(m, n);
        dup = (i > 0 && j[0] == v) || (i > 1 && j[1] == v);
      } while (dup);
      j[i] = v;
    }
  }
}

// The raw picks of random.sample(range(n), k) (k <= 3): the set method
// (n > 21) keeps every value < n not already taken; the pool method (n <= 21)
// takes the i-th value < n - i.  A word whose value is out of range is
// rejected (_randbelow, random.py:239-249).
template <class M>
__device__ __forceinline__ void sample3_raw(M& m, uint32_t n, int k, uint32_t j[3]) {
  sample3_serial(m, n, k, j, 0);
}

// LDS stream: branch-free scan of the next <= 24 twisted words (the wave
// leaves early once every lane has its picks; a lane needs more than 24
// words with probability ~1e-5 and then finishes serially).  The words are
// read a step ahead at immediate offsets from the lane's cursor row (Clamp:
// near the end of a generation, rows clamped to 623; the rows past tw are
// never live).  The reads are volatile so that the compiler issues them
// where they are written, ahead of the branch that may leave the scan,
// instead of sinking them to their first use.
typedef __attribute__((address_space(3))) const volatile uint32_t LdsVolatileWord;
template <bool Clamp>
__device__ __forceinline__ uint32_t scan_word(const LdsMT& m, int t) {
  LdsVolatileWord* lds = (LdsVolatileWord*)hz_lds;
  if (Clamp) {
    int i = m.pos + t < kMT ? m.pos + t : kMT - 1;
    return lds[i * kLdsStride + m.lane];
  }
  return lds[(m.pos + t) * kLdsStride + m.lane];
}

// the top 14 bits of temper(y): its last step (y ^= y >> 18) leaves them
// unchanged; every draw keeps at most 7 (the bag never exceeds 120 tiles).
// With the masks held in SGPRs each "y ^= (y << s) & mask" is a shift and
// one v_bitop3 (a VOP3 op on gfx950 takes no literal).
__device__ __forceinline__ uint32_t sgpr_const(uint32_t v) {
  uint32_t r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(v));
  return r;
}
struct TemperMasks {
  uint32_t b, c;
  __device__ __forceinline__ TemperMasks() : b(sgpr_const(0x9d2c5680u)), c(sgpr_const(0xefc60000u)) {}
};
// (x & m) ^ y in one instruction
__device__ __forceinline__ uint32_t and_xor(uint32_t x, uint32_t m, uint32_t y) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6a" : "=v"(r) : "v"(x), "s"(m), "v"(y));
  return r;
}
__device__ __forceinline__ uint32_t temper_top14(uint32_t y, const TemperMasks& k) {
  y ^= y >> 11;
  y = and_xor(y << 7, k.b, y);
  y = and_xor(y << 15, k.c, y);
  return y;
}
__device__ __forceinline__ uint32_t temper_top14(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y;
}

// Three picks (k = 3, the only size a full bag draws) by a scan of the next
// <= 24 words in steps of four, the next step's words read while this one's
// are tested.  Kept values shift through j0 <- j1 <- j2 (j0 the newest), so
// a word costs one mask for all three selects.  Set method (Pool = false,
// n > 21): a value is kept when < n and unlike the two kept before it.  Pool
// method (n <= 21): pick i keeps a value < n - i, read with bit_length(n - i)
// bits.  Returns the picks in draw order in p0, p1, p2 and the count made;
// fewer than three when the window ran out (rare; serial continuation).
template <bool Clamp, bool Pool>
__device__ __forceinline__ int scan3(LdsMT& m, uint32_t n, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  int avail = m.tw - m.pos;
  uint32_t lim = n;
  int sh = __clz(n);
  uint32_t j0 = 0xffffffffu, j1 = 0xffffffffu, j2 = 0xffffffffu;
  int got = 0, used = 0;
  TemperMasks tk;
  uint32_t w[4], nx[4];
#pragma unroll
  for (int u = 0; u < 4; u++) nx[u] = scan_word<Clamp>(m, u);
#pragma unroll
  for (int seg = 0; seg < 6; seg++) {
#pragma unroll
    for (int u = 0; u < 4; u++) w[u] = nx[u];
    if (seg < 5) {
#pragma unroll
      for (int u = 0; u < 4; u++) nx[u] = scan_word<Clamp>(m, 4 * seg + 4 + u);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      int t = 4 * seg + u;
      bool live = got < 3;
      if (Clamp) live = live && t < avail;
      uint32_t v = temper_top14(w[u], tk) >> sh;
      bool ok = live && v < lim;
      if (!Pool) ok = ok && v != j0 && v != j1;
      j2 = ok ? j1 : j2;
      j1 = ok ? j0 : j1;
      j0 = ok ? v : j0;
      got += ok ? 1 : 0;
      used += live ? 1 : 0;
      if (Pool) {
        lim -= ok ? 1u : 0u;
        sh = __clz(lim);
      }
    }
    if (__all(got >= 3)) break;
  }
  m.pos += used;
  // newest first -> draw order
  p0 = got == 3 ? j2 : got == 2 ? j1 : j0;
  p1 = got == 3 ? j1 : j0;
  p2 = j0;
  return got;
}

__device__ __forceinline__ void sample3_raw(LdsMT& m, uint32_t n, int k, uint32_t j[3]) {
  if (k != 3) {  // fewer than three tiles left: only after the bag's count stopped being a multiple of 3
    sample3_serial(m, n, k, j, 0);
    return;
  }
  uint32_t j0, j1, j2;
  int got;
  bool far = __any(m.pos > kMT - 24);
  if (__all(n > 21)) {
    if (far) got = scan3<true, false>(m, n, j0, j1, j2);
    else got = scan3<false, false>(m, n, j0, j1, j2);
  } else if (__all(n <= 21)) {
    if (far) got = scan3<true, true>(m, n, j0, j1, j2);
    else got = scan3<false, true>(m, n, j0, j1, j2);
  } else {  // a wave whose bags differ in method (boards out of lockstep)
    if (n > 21) got = scan3<true, false>(m, n, j0, j1, j2);
    else got = scan3<true, true>(m, n, j0, j1, j2);
  }
  j[0] = j0; j[1] = j1; j[2] = j2;
  if (got < k) sample3_serial(m, n, k, j, got);  // window exhausted (rare)
}

// A window of a pre-twisted stream in LDS: rows [0, lim) only (hz_env.hip's
// pipeline-2 draw stages, three windows side by side).  Reads never twist:
// past the window next() returns 0, and the caller discards any draw whose
// cursor ends past lim (its picks depend only on the words it consumed, all
// below the cursor).  The scan reads rows up to pos + 23, in bounds while
// pos <= lim.
struct WinMT : LdsMT {
  int lim;
  __device__ __forceinline__ WinMT(int l, int cursor, int rows) : LdsMT(l, cursor), lim(rows) {}
  __device__ __forceinline__ void prefetch() {}
  __device__ __forceinline__ uint32_t next() {
    const int i = pos++;
    return i < lim ? temper(hz_lds[i * kLdsStride + lane]) : 0u;
  }
};
__device__ __forceinline__ void sample3_raw(WinMT& m, uint32_t n, int k, uint32_t j[3]) {
  if (k != 3) {
    sample3_serial(m, n, k, j, 0);
    return;
  }
  uint32_t j0, j1, j2;
  int got;
  LdsMT& lm = m;
  if (__all(n > 21)) got = scan3<false, false>(lm, n, j0, j1, j2);
  else if (__all(n <= 21)) got = scan3<false, true>(lm, n, j0, j1, j2);
  else if (n > 21) got = scan3<false, false>(lm, n, j0, j1, j2);
  else got = scan3<false, true>(lm, n, j0, j1, j2);
  j[0] = j0; j[1] = j1; j[2] = j2;
  if (got < k) sample3_serial(m, n, k, j, got);
}

// _draw_tiles(3) (harmonies_engine.py:120-130): flat_bag follows the bag's
// insertion order water, plant, wood, stone, field, building (constants.py:41).
// Produces the pile as 3x3 bits (7 = none); returns the number of tiles drawn.
// The bag itself is decremented by the caller (apply_pile).
template <class M>
__device__ __forceinline__ int draw_pile(uint64_t misc, M& m, uint32_t& pile9) {
  int cnt[6];
#pragma unroll
  for (int t = 0; t < 6; t++) cnt[t] = bag_n(misc, t);
  uint32_t n = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) n += (uint32_t)cnt[t];
  pile9 = 0x1FF;
  if (!n) return 0;
  int k = n < 3 ? (int)n : 3;
  uint32_t j[3] = {0, 0, 0};
  sample3_raw(m, n, k, j);
  uint32_t idx[3];
  if (n <= 21) {
    // pool method bookkeeping: result[i] = pool[j_i]; pool[j_i] = pool[n-i-1];
    // pool[x] == x except at <= 3 recorded positions (random.py:488-493)
    uint32_t mp0 = 0xffffffffu, mp1 = 0xffffffffu, mv0 = 0, mv1 = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      uint32_t ji = j[i], last = n - (uint32_t)i - 1;
      uint32_t vj = ji, vl = last;
      if (i > 0 && mp0 == ji) vj = mv0;
      if (i > 1 && mp1 == ji) vj = mv1;
      if (i > 0 && mp0 == last) vl = mv0;
      if (i > 1 && mp1 == last) vl = mv1;
      idx[i] = vj;
      if (i == 0) { mp0 = ji; mv0 = vl; }
      if (i == 1) { mp1 = ji; mv1 = vl; }
    }
  } else {
    idx[0] = j[0]; idx[1] = j[1]; idx[2] = j[2];
  }
  // the tile at flat index x: how many of the order's prefix counts are <= x
  // picks the tile from the packed order (no per-tile select chain)
  constexpr uint32_t kOrder = WATER | (PLANT << 3) | (WOOD << 6) | (STONE << 9) | (FIELD << 12) | (BUILDING << 15);
  uint32_t e0 = (uint32_t)cnt[WATER], e1 = e0 + (uint32_t)cnt[PLANT], e2 = e1 + (uint32_t)cnt[WOOD];
  uint32_t e3 = e2 + (uint32_t)cnt[STONE], e4 = e3 + (uint32_t)cnt[FIELD];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    uint32_t x = idx[i];
    uint32_t o = (uint32_t)(x >= e0) + (uint32_t)(x >= e1) + (uint32_t)(x >= e2) + (uint32_t)(x >= e3) +
                 (uint32_t)(x >= e4);
    uint32_t tile = i < k ? __builtin_amdgcn_ubfe(kOrder, 3 * o, 3) : 7u;
    pile9 = (pile9 & ~(7u << (3 * i))) | (tile << (3 * i));
  }
  return k;
}

// apply_pile without branches: each drawn tile's count field minus one (a
// tile drawn is in the bag, so no field borrows); 7 = none
__device__ __forceinline__ void apply_pile_fast(uint64_t& misc, uint32_t pile9) {
  uint64_t dec = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    uint32_t t = (pile9 >> (3 * i)) & 7u;
    dec += t < 6u ? 1ull << (11 + 5 * t) : 0ull;
  }
  misc -= dec;
}

// Every drawn tile decrements the bag (:126-129).
__device__ __forceinline__ void apply_pile(uint64_t& misc, uint32_t pile9) {
#pragma unroll
  for (int i = 0; i < 3; i++) {
    int t = (int)((pile9 >> (3 * i)) & 7);
    if (t != 7) misc = set_bits(misc, 11 + 5 * t, 5, (uint64_t)(bag_n(misc, t) - 1));
  }
}

// Sources of piles for _replenish_piles: the live stream ...
// (holds the stream by value: a reference member would force the stream
// state out of registers into scratch)
template <class M>
struct StreamDraw {
  M m;
  __device__ __forceinline__ uint32_t operator()(uint64_t misc) {
    m.prefetch();  // the one point where the wave's refills line up
    uint32_t p9;
    return draw_pile(misc, m, p9) ? p9 : 0x1FFu;
  }
};
// ... or a recorded script of up to 5 piles (9 bits each, 0x1FF = stop),
// used when an MCTS expansion replays the draws its children made in the
// reference's child order.
struct ScriptDraw {
  uint64_t script;
  __device__ __forceinline__ uint32_t operator()(uint64_t) {
    uint32_t p9 = (uint32_t)(script & 0x1FF);
    script = (script >> 9) | (0x1FFull << 36);
    return p9;
  }
};

// _replenish_piles (:132-137); returns the piles drawn as a script.
template <class Draw>
__device__ __forceinline__ uint64_t replenish(State& s, Draw& draw) {
  int np = npiles_of(s.piles);
  uint64_t script = (1ull << 45) - 1;
  int d = 0;
  while (np < 5) {
    uint32_t pile9 = draw(s.misc);
    if (pile9 == 0x1FFu) break;
    apply_pile(s.misc, pile9);
    s.piles = set_bits(s.piles, 9 * np, 9, pile9);
    script = set_bits(script, 9 * d, 9, pile9);
    np++;
    d++;
    s.piles = set_bits(s.piles, 45, 3, (uint64_t)np);
  }
  return script;
}

// HarmoniesGameState.__init__ (:66-79)
template <class Draw>
__device__ __forceinline__ void reset_state(State& s, Draw& d) {
  s.pl[0] = s.pl[1] = s.pl[2] = s.pl[3] = 0;
  s.piles = (1ull << 45) - 1;  // every tile slot = 7 (none), 0 piles
  uint64_t misc = 0x1FF;        // empty hand
#pragma unroll
  for (int t = 0; t < 6; t++) misc = set_bits(misc, 11 + 5 * t, 5, (uint64_t)initial_count(t));
  s.misc = misc;  // player 0, choose_pile, not over, winner None, scores 0
  replenish(s, d);
}

// ------------------------------------------------------------- legal mask
// get_legal_moves (:145-208) + get_action_index (process_game_state.py:156-179):
// action = pile index during choose_pile, else 5 + tile*23 + cell.
__device__ __forceinline__ void or_range(uint64_t mask[3], int lo, uint32_t m23) {
  int w = lo >> 6, off = lo & 63;
  uint64_t v = (uint64_t)m23;
  mask[w] |= v << off;
  if (off + 23 > 64) mask[w + 1] |= v >> (64 - off);
}

__device__ __forceinline__ int legal_mask(const State& s, uint64_t mask[3]) {
  mask[0] = mask[1] = mask[2] = 0;
  int ph = phase_of(s.misc);
  if (ph == PH_CHOOSE) {
    int np = npiles_of(s.piles);
    mask[0] = (1ull << np) - 1;
    return np;
  }
  if (ph < PH_P1 || ph > PH_P3) return 0;
  int nh = hand_n(s.misc);
  if (!nh) return 0;
  uint32_t b[4];
  planes_of(s, player_of(s.misc), b);
  uint32_t empty = kAll23 & ~(b[0] | b[1] | b[2] | b[3]);
  uint32_t wood1 = is_code<3>(b), stone1 = is_code<4>(b), stone2 = is_code<8>(b), bld1 = is_code<5>(b);
  uint32_t has = 0;
  for (int j = 0; j < nh; j++) has |= 1u << hand_tile(s.misc, j);
  int count = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) {
    uint32_t m = empty;
    if (t == PLANT) m |= wood1;
    if (t == STONE) m |= stone1 | stone2;
    if (t == BUILDING) m |= wood1 | stone1 | bld1;
    m = (has >> t) & 1u ? m : 0u;  // branch-free: same instructions on every lane
    or_range(mask, 5 + 23 * t, m);
    count += __popc(m);
  }
  return count;
}

// position of the k-th (0-based) set bit of a 32-bit word, branch-free
__device__ __forceinline__ int select32(uint32_t w, int k) {
  int pos = 0;
#pragma unroll
  for (int s = 16; s > 0; s >>= 1) {
    uint32_t lo = w & ((1u << s) - 1);
    int c = __popc(lo);
    bool up = k >= c;
    k = up ? k - c : k;
    w = up ? w >> s : lo;
    pos += up ? s : 0;
  }
  return pos;
}

// k-th (0-based) legal action in ascending action order: the 32-bit word
// holding it is found by prefix popcounts, then one branch-free select
// (every lane runs the same instructions whatever word its action is in).
__device__ __forceinline__ int kth_action(const uint64_t mask[3], int k) {
  uint32_t w[5] = {(uint32_t)mask[0], (uint32_t)(mask[0] >> 32), (uint32_t)mask[1], (uint32_t)(mask[1] >> 32),
                   (uint32_t)mask[2]};
  uint32_t word = w[4];
  int base = 128, pre = 0;
  bool found = false;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int c = __popc(w[i]);
    bool here = !found && k - pre < c;
    word = here ? w[i] : word;
    base = here ? 32 * i : base;
    found = found || here;
    pre += found ? 0 : c;
  }
  return base + select32(word, k - pre);
}

// The benchmark rule's action without materialising the 143-bit mask (the
// fused rollout when no trajectory is recorded): with h the rule hash's top
// 32 bits, the action is the k-th legal one, k = (h * L) >> 32, in ascending
// action order; for placements that is tile-major over the hand's distinct
// tiles, so the tile is found by prefix counts and the cell by one select.
// Returns -1 when there is no legal move.
__device__ __forceinline__ int rule_action(const State& s, uint32_t h) {
  int ph = phase_of(s.misc);
  if (ph == PH_CHOOSE) {
    int np = npiles_of(s.piles);
    return np ? (int)(((uint64_t)h * (uint32_t)np) >> 32) : -1;
  }
  uint32_t b[4];
  planes_of(s, player_of(s.misc), b);
  uint32_t empty = kAll23 & ~(b[0] | b[1] | b[2] | b[3]);
  uint32_t wood1 = is_code<3>(b), stone1 = is_code<4>(b), stone2 = is_code<8>(b), bld1 = is_code<5>(b);
  int nh = (ph >= PH_P1 && ph <= PH_P3) ? hand_n(s.misc) : 0;
  uint32_t has = 0;
#pragma unroll
  for (int j = 0; j < 3; j++) has |= j < nh ? 1u << hand_tile(s.misc, j) : 0u;
  uint32_t m[6];
  int c[6], L = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) {
    uint32_t mt = empty;
    if (t == PLANT) mt |= wood1;
    if (t == STONE) mt |= stone1 | stone2;
    if (t == BUILDING) mt |= wood1 | stone1 | bld1;
    m[t] = (has >> t) & 1u ? mt : 0u;
    c[t] = __popc(m[t]);
    L += c[t];
  }
  if (L == 0) return -1;
  int k = (int)(((uint64_t)h * (uint32_t)L) >> 32);
  uint32_t word = m[5];
  int tt = 5, pre = 0;
  bool found = false;
#pragma unroll
  for (int t = 0; t < 5; t++) {
    bool here = !found && k - pre < c[t];
    word = here ? m[t] : word;
    tt = here ? t : tt;
    found = found || here;
    pre += found ? 0 : c[t];
  }
  return 5 + 23 * tt + select32(word, k - pre);
}

// ------------------------------------------------------------------- step
__device__ __forceinline__ void finish_game(State& s) {  // :344-354
  int s0 = score_player(s, 0), s1 = score_player(s, 1);
  uint64_t m = s.misc;
  m = set_bits(m, 42, 3, PH_OVER);
  m = set_bits(m, 48, 8, (uint64_t)s0);
  m = set_bits(m, 56, 8, (uint64_t)s1);
  m = set_bits(m, 46, 2, s0 > s1 ? 1 : s1 > s0 ? 2 : 3);
  s.misc = m;
}

// A finished game whose scoring is deferred (Defer = true, k_rollout): phase
// game_over with winner None, a combination no reference state has.  The
// caller scores it with finish_game at a point where the whole wave can do
// it together.
__device__ __forceinline__ void mark_over(State& s) { s.misc = set_bits(s.misc, 42, 3, PH_OVER); }
__device__ __forceinline__ bool score_pending(uint64_t m) {
  return phase_of(m) == PH_OVER && winner_code(m) == 0;
}

template <bool Defer = false, class Draw>
__device__ __forceinline__ void end_turn(State& s, Draw& draw) {  // :301-329
  int p = player_of(s.misc);
  uint32_t b[4];
  planes_of(s, p, b);
  int filled = __popc(b[0] | b[1] | b[2] | b[3]);
  bool player_trigger = (kCells - filled) <= 2;
  bool bag_empty_before = bag_total(s.misc) == 0;
  replenish(s, draw);
  bool bag_trigger = bag_empty_before && npiles_of(s.piles) == 0;
  bool end = player_trigger || bag_trigger;
  bool finish = false;
  if (end && !over_flag(s.misc)) {
    s.misc = set_bits(s.misc, 45, 1, 1);
    if (p == 0) {
      s.misc = set_bits(s.misc, 41, 1, 1);
      s.misc = set_bits(s.misc, 42, 3, PH_CHOOSE);
    } else {
      finish = true;
    }
  } else if (over_flag(s.misc)) {
    finish = true;
  } else {
    s.misc = set_bits(s.misc, 41, 1, (uint64_t)(1 - p));
    s.misc = set_bits(s.misc, 42, 3, PH_CHOOSE);
  }
  if (finish) {
    if constexpr (Defer) mark_over(s);
    else finish_game(s);
  }
}

// apply_move (:210-298) in place; returns a status (state untouched unless OK).
template <bool Defer = false, class Draw>
__device__ __forceinline__ int step_state(State& s, int a, Draw& draw) {
  if (a < 0 || a >= kActions) return ST_BAD_ACTION;
  int ph = phase_of(s.misc);
  if (ph == PH_CHOOSE) {
    int np = npiles_of(s.piles);
    if (a >= 5 || a >= np) return ST_BAD_PILE;
    uint32_t pile9 = (uint32_t)(s.piles >> (9 * a)) & 0x1FF;
    int len = ((pile9 & 7) != 7) + (((pile9 >> 3) & 7) != 7) + (((pile9 >> 6) & 7) != 7);
    uint64_t lower = s.piles & ((1ull << (9 * a)) - 1);
    uint64_t upper = (s.piles & ((1ull << 45) - 1)) >> (9 * (a + 1));
    uint64_t np_piles = lower | (upper << (9 * a));
    np_piles |= 0x1FFull << 36;  // vacated top slot
    s.piles = set_bits(np_piles, 45, 3, (uint64_t)(np - 1));
    uint64_t m = set_bits(s.misc, 0, 9, pile9);
    m = set_bits(m, 9, 2, (uint64_t)len);
    s.misc = set_bits(m, 42, 3, PH_P1);
    return ST_OK;
  }
  if (ph >= PH_P1 && ph <= PH_P3) {
    if (a < 5) return ST_BAD_FORMAT;
    int t = (a - 5) / 23, c = (a - 5) % 23;
    int nh = hand_n(s.misc), j = -1;
    for (int q = nh - 1; q >= 0; q--)
      if (hand_tile(s.misc, q) == t) j = q;
    if (j < 0) return ST_NOT_IN_HAND;
    int p = player_of(s.misc);
    int nc = place_code(code_at(s, p, c), t);
    if (nc < 0) return ST_ILLEGAL_STACK;
    // hand.remove(tile): drop entry j, shift the rest down
    uint32_t h9 = (uint32_t)(s.misc & 0x1FF);
    uint32_t low = h9 & ((1u << (3 * j)) - 1);
    uint32_t high = h9 >> (3 * (j + 1));
    uint32_t nh9 = (low | (high << (3 * j)) | (7u << 6)) & 0x1FF;
    uint64_t m = set_bits(s.misc, 0, 9, nh9);
    s.misc = set_bits(m, 9, 2, (uint64_t)(nh - 1));
    set_code(s, p, c, nc);
    if (ph < PH_P3) s.misc = set_bits(s.misc, 42, 3, (uint64_t)(ph + 1));
    else end_turn<Defer>(s, draw);
    return ST_OK;
  }
  return ST_BAD_PHASE;
}

// apply_move for an action taken from the legal mask (the fused rollout):
// the same transitions as step_state without its validation, written
// branch-free so that every lane of a wave runs the same instructions.
template <bool Defer, class Draw>
__device__ __forceinline__ void step_trusted(State& s, int a, Draw& draw) {
  int ph = phase_of(s.misc);
  if (ph == PH_CHOOSE) {
    int np = npiles_of(s.piles);
    uint32_t pile9 = (uint32_t)(s.piles >> (9 * a)) & 0x1FF;
    int len = ((pile9 & 7) != 7) + (((pile9 >> 3) & 7) != 7) + (((pile9 >> 6) & 7) != 7);
    uint64_t lower = s.piles & ((1ull << (9 * a)) - 1);
    uint64_t upper = (s.piles & ((1ull << 45) - 1)) >> (9 * (a + 1));
    uint64_t np_piles = lower | (upper << (9 * a)) | (0x1FFull << 36);
    s.piles = set_bits(np_piles, 45, 3, (uint64_t)(np - 1));
    uint64_t m = set_bits(s.misc, 0, 9, pile9);
    m = set_bits(m, 9, 2, (uint64_t)len);
    s.misc = set_bits(m, 42, 3, PH_P1);
    return;
  }
  int t = (a - 5) / 23, c = (a - 5) - 23 * t;
  int nh = hand_n(s.misc);
  uint32_t h9 = (uint32_t)(s.misc & 0x1FF);
  // hand.remove(tile): the first entry equal to t
  int j = (int)(h9 & 7) == t ? 0 : (int)((h9 >> 3) & 7) == t ? 1 : 2;
  int p = player_of(s.misc);
  int code = code_at(s, p, c);
  // place_code for a legal placement: empty -> 1 + t; plant on wood 7;
  // stone on stone 8 / on stone-stone 9; building on wood/stone/building 10/11/12
  int nc = t == PLANT ? 7 : t == STONE ? (code == 4 ? 8 : 9) : code + 7;
  nc = code == 0 ? 1 + t : nc;
  uint32_t low = h9 & ((1u << (3 * j)) - 1);
  uint32_t high = h9 >> (3 * (j + 1));
  uint32_t nh9 = (low | (high << (3 * j)) | (7u << 6)) & 0x1FF;
  uint64_t m = set_bits(s.misc, 0, 9, nh9);
  s.misc = set_bits(m, 9, 2, (uint64_t)(nh - 1));
  set_code(s, p, c, nc);
  if (ph < PH_P3) s.misc = set_bits(s.misc, 42, 3, (uint64_t)(ph + 1));
  else end_turn<Defer>(s, draw);
}

// ------------------------------------------------------- transposition key
// MCTS.py keys its DAG by hash(state) (MCTS.py:14,177,185) of
// get_canonical_tuple() (harmonies_engine.py:81-110).  Because CPython hashes
// the int -1 like -2, two canonical tuples collide exactly when they agree
// after mapping every axial coordinate component -1 to -2, with board items
// still listed in sorted real-coordinate order.  The key below encodes that
// equivalence exactly (pyhash = true); pyhash = false gives the true
// canonical tuple.
//   w0: player | phase<<1 | #hand<<4 | sorted hand<<6 | #piles<<15 | bag<<18
//   w1: the piles in order, each sorted (5 x 9 bits)
//   w2..w4 / w5..w7: player 0 / 1 board: one byte (class << 4 | stack code)
//   per occupied cell in cell order (pyhash), or 23 stack-code nibbles.
struct CKey {
  uint64_t w[8];
};

// cell -> coordinate class under (-1 -> -2): {1,6} {2,7} {3,8} {4,5} {9,10}
// {14,15} {19,20} collide; classes numbered 0..15 in order of first cell.
constexpr int kHashClass[23] = {0, 1, 2, 3, 4, 4, 1, 2, 3, 5, 5, 6, 7, 8, 9, 9, 10, 11, 12, 13, 13, 14, 15};
__host__ __device__ constexpr uint64_t pack_class(int lo) {
  uint64_t r = 0;
  for (int c = lo; c < 23 && c < lo + 16; c++) r |= (uint64_t)kHashClass[c] << (4 * (c - lo));
  return r;
}
constexpr uint64_t kClassLo = pack_class(0), kClassHi = pack_class(16);

__device__ __forceinline__ void sort3(uint32_t& a, uint32_t& b, uint32_t& c) {
  uint32_t t;
  if (b < a) { t = a; a = b; b = t; }
  if (c < b) { t = b; b = c; c = t; }
  if (b < a) { t = a; a = b; b = t; }
}

__device__ __forceinline__ uint32_t sorted9(uint32_t v9) {
  uint32_t a = v9 & 7, b = (v9 >> 3) & 7, c = (v9 >> 6) & 7;
  sort3(a, b, c);
  return a | (b << 3) | (c << 6);
}

// w0, w1: player, phase, hand, piles, bag
__device__ __forceinline__ void canon_key_head(const State& s, CKey& k) {
  uint64_t m = s.misc;
  k.w[0] = (uint64_t)player_of(m) | ((uint64_t)phase_of(m) << 1) | ((uint64_t)hand_n(m) << 4) |
           ((uint64_t)sorted9((uint32_t)(m & 0x1FF)) << 6) | ((uint64_t)npiles_of(s.piles) << 15) |
           (((m >> 11) & ((1ull << 30) - 1)) << 18);
  uint64_t pw = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) pw |= (uint64_t)sorted9((uint32_t)(s.piles >> (9 * i)) & 0x1FF) << (9 * i);
  k.w[1] = pw;
}

__device__ __forceinline__ CKey canon_key(const State& s, bool pyhash) {
  CKey k;
  canon_key_head(s, k);
#pragma unroll
  for (int p = 0; p < 2; p++) {
    uint64_t a0 = 0, a1 = 0, a2 = 0;
    if (pyhash) {
      int cnt = 0;
#pragma unroll
      for (int c = 0; c < 23; c++) {
        int code = code_at(s, p, c);
        uint64_t cls = c < 16 ? (kClassLo >> (4 * c)) & 15 : (kClassHi >> (4 * (c - 16))) & 15;
        uint64_t byte = (cls << 4) | (uint64_t)code;
        int sh = (cnt & 7) * 8;
        if (code) {
          if (cnt < 8) a0 |= byte << sh;
          else if (cnt < 16) a1 |= byte << sh;
          else a2 |= byte << sh;
          cnt++;
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < 23; c++) {
        uint64_t code = (uint64_t)code_at(s, p, c);
        if (c < 16) a0 |= code << (4 * c);
        else a1 |= code << (4 * (c - 16));
      }
    }
    k.w[2 + 3 * p] = a0;
    k.w[3 + 3 * p] = a1;
    k.w[4 + 3 * p] = a2;
  }
  return k;
}

// The key of the child that action a leads to from `parent` (whose key is
// pk), equal to canon_key(child, pyhash) for every child step_state makes
// from parent: a child's boards differ from its parent's at most at the
// placed cell of the mover's board (a pile choice and the end of turn leave
// the boards as they are, and the key holds no scores), so the board words
// are the parent's with that one entry rewritten: in the pyhash form the
// occupied cells are listed in cell order one byte each, so a tile on an
// occupied cell replaces the byte at the cell's rank among them and a tile
// on an empty cell inserts one there (the bytes from that rank on move up a
// byte of the 192-bit list); in the exact form the cell's nibble.  w0/w1 are
// rebuilt from the child's state.  ~70 instructions against ~1,300 for the
// 46-cell walk of canon_key (the expansion computes one key per child).
__device__ __forceinline__ CKey canon_key_child(const CKey& pk, const State& parent, const State& child, int a,
                                                bool pyhash) {
  CKey k = pk;
  canon_key_head(child, k);
  if (a < 5) return k;
  const int p = player_of(parent.misc), c = (a - 5) % 23;
  const uint64_t nc = (uint64_t)code_at(child, p, c);
  uint64_t w0 = p ? pk.w[5] : pk.w[2], w1 = p ? pk.w[6] : pk.w[3], w2 = p ? pk.w[7] : pk.w[4];
  if (pyhash) {
    const uint64_t any = parent.pl[0] | parent.pl[1] | parent.pl[2] | parent.pl[3];
    const uint32_t occ = (uint32_t)(any >> (32 * p)) & 0x7FFFFFu;
    const bool occupied = (occ >> c) & 1u;
    const int bp = 8 * __popc(occ & ((1u << c) - 1u)), be = bp + 8;  // the entry's bits [bp, be) of the list
    const uint64_t cls = c < 16 ? (kClassLo >> (4 * c)) & 15 : (kClassHi >> (4 * (c - 16))) & 15;
    const uint64_t byte = cls << 4 | nc;
    // the bits of word j below bit position b of the list
    auto below = [](int b, int j) -> uint64_t {
      const int d = b - 64 * j;
      return d <= 0 ? 0ull : d >= 64 ? ~0ull : (1ull << d) - 1;
    };
    auto entry = [&](int j) -> uint64_t {
      const int d = bp - 64 * j;
      return d >= 0 && d < 64 ? byte << d : 0ull;
    };
    // the bytes above the entry: the list itself (replace) or the list moved up a byte (insert)
    const uint64_t s0 = occupied ? w0 : w0 << 8;
    const uint64_t s1 = occupied ? w1 : (w1 << 8) | (w0 >> 56);
    const uint64_t s2 = occupied ? w2 : (w2 << 8) | (w1 >> 56);
    w0 = (w0 & below(bp, 0)) | (s0 & ~below(be, 0)) | entry(0);
    w1 = (w1 & below(bp, 1)) | (s1 & ~below(be, 1)) | entry(1);
    w2 = (w2 & below(bp, 2)) | (s2 & ~below(be, 2)) | entry(2);
  } else if (c < 16) {
    w0 = (w0 & ~(15ull << (4 * c))) | nc << (4 * c);
  } else {
    w1 = (w1 & ~(15ull << (4 * (c - 16)))) | nc << (4 * (c - 16));
  }
  if (p) {
    k.w[5] = w0;
    k.w[6] = w1;
    k.w[7] = w2;
  } else {
    k.w[2] = w0;
    k.w[3] = w1;
    k.w[4] = w2;
  }
  return k;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t key_hash(const CKey& k) {
  uint64_t h = 0x243F6A8885A308D3ULL;
#pragma unroll
  for (int i = 0; i < 8; i++) h = mix64(h ^ (k.w[i] + 0x9E3779B97F4A7C15ULL * (uint64_t)(i + 1)));
  return h;
}

__device__ __forceinline__ bool key_eq(const CKey& a, const CKey& b) {
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; i++) eq = eq && (a.w[i] == b.w[i]);
  return eq;
}

// ------------------------------------------------------------ action rule
__device__ __forceinline__ uint64_t rule_key(uint64_t seed) {  // the per-game part of rule_hash
  return seed * 0x9E3779B97F4A7C15ULL + 0x9E3779B97F4A7C15ULL;
}
__device__ __forceinline__ uint64_t rule_hash_k(uint64_t key, uint64_t ply) {
  uint64_t z = key + ply;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rule_hash(uint64_t seed, uint64_t ply) {
  return rule_hash_k(rule_key(seed), ply);
}

__device__ __forceinline__ uint32_t rule_h32(uint64_t key, int ply) {
  return (uint32_t)(rule_hash_k(key, (uint64_t)ply) >> 32);
}
__device__ __forceinline__ int rule_pick_k(uint64_t key, int ply, int n_legal) {
  uint32_t hi = (uint32_t)(rule_hash_k(key, (uint64_t)ply) >> 32);
  return (int)(((uint64_t)hi * (uint32_t)n_legal) >> 32);
}
__device__ __forceinline__ int rule_pick(uint64_t seed, int ply, int n_legal) {
  return rule_pick_k(rule_key(seed), ply, n_legal);
}

// ------------------------------------------------ turn-structured rollout
// Every turn is exactly four plies: choose a pile (always three tiles: the
// bag starts at 120 and every draw takes three), then place the three
// (harmonies_engine.py:210-298); the turn ends after place_tile_3.  Boards
// started together therefore move in lockstep: within a turn the phase, and
// across a pair of turns the player, are compile-time constants, so a
// placement works on the mover's 32-bit plane halves directly and the hand
// lives in a register until the turn ends.  turn_pair_safe() admits a board
// only when both turns of the pair are sure to complete their four plies.
template <int P>
__device__ __forceinline__ uint32_t half(uint64_t w) {
  return P ? (uint32_t)(w >> 32) : (uint32_t)w;
}
template <int P>
__device__ __forceinline__ uint64_t with_half(uint64_t w, uint32_t v) {
  return P ? (w & 0xFFFFFFFFull) | ((uint64_t)v << 32) : (w & 0xFFFFFFFF00000000ull) | (uint64_t)v;
}

// player 0 to choose a pile, game running, >= 1 pile and every pile full,
// bag a multiple of three (so every later pile is full) and either five
// piles or an empty bag (so a turn end draws at most one pile), and three
// empty cells on each board (so each placement has a legal cell).  All of it
// holds for every reachable state at a pair boundary.
__device__ __forceinline__ bool turn_pair_safe(const State& s) {
  uint64_t m = s.misc;
  bool ok = (m & ((1ull << 41) | (7ull << 42) | (1ull << 45))) == 0;  // player 0, choose_pile, not over
  int np = npiles_of(s.piles);
  uint64_t p = s.piles;
  uint64_t absent = p & (p >> 1) & (p >> 2) & 0x1249249249249ull & ((1ull << (9 * np)) - 1);  // a slot == 7
  int bag = bag_total(m);
  ok = ok && np >= 1 && absent == 0 && bag % 3 == 0 && (np == 5 || bag == 0);
  uint64_t occ = s.pl[0] | s.pl[1] | s.pl[2] | s.pl[3];
  ok = ok && __popc((uint32_t)occ) <= kCells - 3 && __popc((uint32_t)(occ >> 32)) <= kCells - 3;
  return ok;
}

// Legal cells by tile class (harmonies_engine.py:183-194): water, wood and
// field go on an empty cell (class 0); plant also on wood (1); stone also on
// one or two stones (2); building also on wood, stone or building (3).
// kTileClass5: the class of tile t times 8 in bits 5t..5t+4.
constexpr uint32_t kTileClass5 = (0u << 0) | (8u << 5) | (0u << 10) | (16u << 15) | (24u << 20) | (0u << 25);
__device__ __forceinline__ uint32_t class_off(uint32_t t) { return __builtin_amdgcn_ubfe(kTileClass5, 5 * t, 5); }
// place_code step of a tile onto a non-empty legal cell (code + add): plant
// on wood 3 -> 7 (+4), building on 3/4/5 -> +7, stone on 8 -> 9 (+1) and on
// 4 -> 8 (+4, patched below); 4 bits per tile
constexpr uint32_t kAddTab = 1u | (4u << 4) | (1u << 8) | (1u << 12) | (7u << 16) | (1u << 20);

// The turn path below is branch-free by construction: every choice among
// more than two values is a bit-field extract from a packed word, never a
// chain of selects (which the compiler turns into divergent branches).
//
// One placement ply of player P with NH tiles in hand (hand9: NH 3-bit tiles
// in hand order): the rule's action is the k-th legal move, k = (h * L) >> 32,
// in ascending action order = tile-major over the hand's distinct tiles
// (get_action_index, process_game_state.py:156-179), then the placement and
// hand.remove(tile) of apply_move (:244-276).
template <int P, int NH>
__device__ __forceinline__ void place_fast(State& s, uint32_t& hand9, uint32_t h) {
  uint32_t b0 = half<P>(s.pl[0]), b1 = half<P>(s.pl[1]), b2 = half<P>(s.pl[2]), b3 = half<P>(s.pl[3]);
  uint32_t o01 = b0 | b1, o23 = b2 | b3;
  uint32_t mE = ~(o01 | o23) & kAll23;
  uint32_t wood1 = b0 & b1 & ~o23;             // code 3
  uint32_t stone1 = b2 & ~(o01 | b3);          // code 4
  uint32_t stone2 = b3 & ~(o01 | b2);          // code 8
  uint32_t bld1 = b0 & b2 & ~(b1 | b3);        // code 5
  uint32_t mP = mE | wood1, mS = mE | stone1 | stone2, mB = mP | stone1 | bld1;
  // legal-cell counts of the four classes, one byte each
  uint32_t cw = (uint32_t)__popc(mE) | ((uint32_t)__popc(mP) << 8) | ((uint32_t)__popc(mS) << 16) |
                ((uint32_t)__popc(mB) << 24);
  uint32_t t0 = hand9 & 7u, t1 = (hand9 >> 3) & 7u, t2 = (hand9 >> 6) & 7u;
  uint32_t tile, idx;
  if constexpr (NH == 1) {
    uint32_t c0 = __builtin_amdgcn_ubfe(cw, class_off(t0), 8);
    idx = (uint32_t)(((uint64_t)h * c0) >> 32);
    tile = t0;
  } else if constexpr (NH == 2) {
    uint32_t lo = min(t0, t1), hi = max(t0, t1);
    uint32_t c0 = __builtin_amdgcn_ubfe(cw, class_off(lo), 8);
    uint32_t c1 = __builtin_amdgcn_ubfe(cw, class_off(hi), 8) & (0u - (uint32_t)(hi != lo));
    uint32_t k = (uint32_t)(((uint64_t)h * (c0 + c1)) >> 32);
    bool up = k >= c0;
    tile = up ? hi : lo;
    idx = k - (up ? c0 : 0u);
  } else {
    // the distinct tiles ascending (min/max network), their counts, the
    // k-th move's tile (w = how many prefixes k passes) by one extract
    uint32_t a = min(t0, t1), bb = max(t0, t1);
    uint32_t u2 = max(bb, t2), m12 = min(bb, t2);
    uint32_t u0 = min(a, m12), u1 = max(a, m12);
    uint32_t c0 = __builtin_amdgcn_ubfe(cw, class_off(u0), 8);
    uint32_t c1 = __builtin_amdgcn_ubfe(cw, class_off(u1), 8) & (0u - (uint32_t)(u1 != u0));
    uint32_t c2 = __builtin_amdgcn_ubfe(cw, class_off(u2), 8) & (0u - (uint32_t)(u2 != u1));
    uint32_t c01 = c0 + c1;
    uint32_t k = (uint32_t)(((uint64_t)h * (c01 + c2)) >> 32);
    uint32_t w = (uint32_t)(k >= c0) + (uint32_t)(k >= c01);
    tile = __builtin_amdgcn_ubfe(u0 | (u1 << 3) | (u2 << 6), 3 * w, 3);
    idx = k - __builtin_amdgcn_ubfe((c0 << 8) | (c01 << 16), 8 * w, 8);
  }
  // the tile's legal cells: class bits q1 (plant, building), q2 (stone, building)
  uint32_t cls = class_off(tile) >> 3;
  uint32_t q1 = 0u - (cls & 1u), q2 = 0u - (cls >> 1);
  uint32_t m = mE | (wood1 & q1) | (stone1 & q2) | (stone2 & q2 & ~q1) | (bld1 & q2 & q1);
  int c = select32(m, (int)idx);
  // place_code for a legal placement (see step_trusted): empty -> 1 + t;
  // otherwise code + add (kAddTab), stone on one stone 4 -> 8
  uint32_t code = __builtin_amdgcn_ubfe(b0, c, 1) | (__builtin_amdgcn_ubfe(b1, c, 1) << 1) |
                  (__builtin_amdgcn_ubfe(b2, c, 1) << 2) | (__builtin_amdgcn_ubfe(b3, c, 1) << 3);
  // (as arithmetic on 0/1 values: a select here was sunk into a branch)
  uint32_t add = __builtin_amdgcn_ubfe(kAddTab, 4 * tile, 4);
  uint32_t empty = (uint32_t)(code == 0u);
  add += 3u * ((uint32_t)(code == 4u) & (uint32_t)(add == 1u));
  uint32_t nc = code + add + empty * (1u + tile - add);  // empty: 0 + (1 + tile)
  uint32_t d = code ^ nc;
  uint32_t bit = 1u << c;
  b0 ^= bit & (0u - (d & 1u));
  b1 ^= bit & (0u - ((d >> 1) & 1u));
  b2 ^= bit & (0u - ((d >> 2) & 1u));
  b3 ^= bit & (0u - ((d >> 3) & 1u));
  s.pl[0] = with_half<P>(s.pl[0], b0);
  s.pl[1] = with_half<P>(s.pl[1], b1);
  s.pl[2] = with_half<P>(s.pl[2], b2);
  s.pl[3] = with_half<P>(s.pl[3], b3);
  // hand.remove(tile): the first entry equal to it goes, the rest keep
  // their order (field p = 0, 1 or 2 removed by one bit-field insert)
  if constexpr (NH == 2) {
    hand9 = t0 == tile ? t1 : t0;
  } else if constexpr (NH == 3) {
    uint32_t p = (1u - (uint32_t)(t0 == tile)) * (2u - (uint32_t)(t1 == tile));
    uint32_t low = (1u << (3 * p)) - 1u;
    hand9 = (hand9 & low) | ((hand9 >> 3) & ~low);
  }
}

// _end_turn_actions (:301-329) for player P after a full turn (hand empty).
// Under turn_pair_safe the refill is at most one pile: four piles are left
// unless the bag ran dry at an earlier refill.  Pop: the caller guarantees
// the refill happens and comes from the draw's script (draw.pop()).
template <int P, class Draw, bool Pop = false>
__device__ __forceinline__ void end_turn_fast(State& s, Draw& draw) {
  uint32_t occ = half<P>(s.pl[0] | s.pl[1] | s.pl[2] | s.pl[3]);
  bool player_trigger = __popc(occ) >= kCells - 2;
  uint64_t m = s.misc;
  bool bag_empty_before = (m & (((1ull << 30) - 1) << 11)) == 0;
  int np = npiles_of(s.piles);
  bool want = Pop || (np < 5 && !bag_empty_before);
  uint32_t pile9;  // a full pile (the bag holds a multiple of three); 0x1FF if !want
  if constexpr (Pop) pile9 = draw.pop();
  else pile9 = draw.take(m, want);
  apply_pile_fast(m, pile9);
  uint64_t refilled = (s.piles & ~((0x1FFull << (9 * np)) | (7ull << 45))) | ((uint64_t)pile9 << (9 * np)) |
                      ((uint64_t)(np + 1) << 45);
  s.piles = want ? refilled : s.piles;
  np += want ? 1 : 0;
  bool bag_trigger = bag_empty_before && np == 0;
  bool end = player_trigger || bag_trigger;
  bool over = over_flag(m);
  // next: the other player chooses; P0's trigger sets game_over and gives
  // P1 its last turn; P1's trigger (or a turn after game_over) ends the game
  bool fin = P ? (end || over) : over;
  bool flag = end && !over;
  m = (m & ~((1ull << 41) | (7ull << 42))) | ((uint64_t)(1 - P) << 41);  // player switch, choose_pile
  m |= flag ? (1ull << 45) : 0ull;
  m = fin ? (m & ~(1ull << 41)) | ((uint64_t)P << 41) | ((uint64_t)PH_OVER << 42) : m;  // mark_over, player kept
  s.misc = m;
}

// One whole turn of player P (the rule policy at plies g_ply .. g_ply + 3).
// (CheapRule: a multiplicative stand-in for the rule hash, for the
// microbenchmarks in tools/ only.)
template <int P, bool CheapRule = false>
__device__ __forceinline__ uint32_t turn_rule(uint64_t rkey, int ply) {
  return CheapRule ? ((uint32_t)rkey + (uint32_t)ply) * 0x9E3779B9u : rule_h32(rkey, ply);
}
// ... given the four rule hashes of its plies (h[j] for ply g_ply + j)
template <int P, class Draw, bool Pop = false>
__device__ __forceinline__ void play_turn_h(State& s, Draw& draw, uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3) {
  uint32_t hand9;
  {  // choose_pile: the pile leaves the row, later piles shift down (:221)
    int np = npiles_of(s.piles);
    int a = (int)(((uint64_t)h0 * (uint32_t)np) >> 32);
    hand9 = (uint32_t)(s.piles >> (9 * a)) & 0x1FF;
    uint64_t lower = s.piles & ((1ull << (9 * a)) - 1);
    uint64_t upper = (s.piles & ((1ull << 45) - 1)) >> (9 * (a + 1));
    s.piles = lower | (upper << (9 * a)) | (0x1FFull << 36) | ((uint64_t)(np - 1) << 45);
  }
  place_fast<P, 3>(s, hand9, h1);
  place_fast<P, 2>(s, hand9, h2);
  place_fast<P, 1>(s, hand9, h3);
  s.misc = (s.misc & ~0x7FFull) | 0x1FFull;  // empty hand
  end_turn_fast<P, Draw, Pop>(s, draw);
}
template <int P, class Draw, bool CheapRule = false>
__device__ __forceinline__ void play_turn(State& s, Draw& draw, uint64_t rkey, int g_ply) {
  play_turn_h<P>(s, draw, turn_rule<P, CheapRule>(rkey, g_ply), turn_rule<P, CheapRule>(rkey, g_ply + 1),
                 turn_rule<P, CheapRule>(rkey, g_ply + 2), turn_rule<P, CheapRule>(rkey, g_ply + 3));
}

// ------------------------------------------------------------ SoA access
__device__ __forceinline__ State load_state(const uint64_t* __restrict__ st, int n, int b) {
  State s;
#pragma unroll
  for (int k = 0; k < 4; k++) s.pl[k] = st[(size_t)k * n + b];
  s.piles = st[(size_t)4 * n + b];
  s.misc = st[(size_t)5 * n + b];
  return s;
}

__device__ __forceinline__ void store_state(uint64_t* __restrict__ st, int n, int b, const State& s) {
#pragma unroll
  for (int k = 0; k < 4; k++) st[(size_t)k * n + b] = s.pl[k];
  st[(size_t)4 * n + b] = s.piles;
  st[(size_t)5 * n + b] = s.misc;
}

}  // namespace hz
