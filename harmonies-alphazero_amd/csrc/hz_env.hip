// hz_env.hip — batched Harmonies env kernels and their C-ABI (include/hz_abi.h).
//
// Every env kernel is lane-per-board: thread b owns board b, loads its 48 B
// SoA record (coalesced: 64 lanes x 8 B per word), runs the rules from
// hz_device.hpp in registers and stores the record back.  The encoder is
// element-parallel instead (it writes 5,488 B per board and is HBM-bound).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/hz_abi.h"
#include "hz_device.hpp"
#include "hz_encode.hpp"

using namespace hz;

// pipeline-2 hand-offs (k_play2), per board, rows of nrow
struct P2Draw {   // a draw stage's output: the pile script so far
  int32_t *tag;   // [nrow] episode * 8 + draw stages done
  int32_t *k;     // [nrow] draws done
  uint64_t *q;    // [4][nrow] the script: draw i at bits 9 i ..
  uint64_t *bag;  // [nrow] bag fields (misc layout) after those draws
  int32_t *c;     // [nrow] stream cursor after those draws
};
struct P2Mid {    // a play stage's end state, for the next play stage
  int32_t *tag;   // [nrow] episode
  uint64_t *st;   // [6][nrow] state
  uint64_t *q;    // [4][nrow] the rest of the script
  int32_t *i;     // [3][nrow] script entries used, plies played, stream cursor if fell (else -1)
};

struct hz_env {
  int32_t n;
  uint64_t seed_base;
  hipStream_t stream;
  uint64_t *state;   // [6][n]
  uint32_t *mt;      // [n][624] board-major MT19937 words
  int32_t *pos;      // [n] MT cursor (pos | tw << 16, see hz_device.hpp)
  int32_t *ply;      // [n]
  int32_t *episode;  // [n]
  uint64_t *seed;    // [n]
  // chance-ahead (hz_play): extra blocks of the same launch prepare each
  // board's next episodes (seed, draw1, draw2 stages; see the stages and
  // launch_rollout) while the playing blocks play the current one
  int seed_ahead;            // scripted draws prepared per board (0: off; default kAheadDraws)
  uint32_t *ahead_mt[2];     // [n][624] seeded streams
  int32_t *ahead_tag[2];     // [n] episode each slot holds (-1: none)
  uint64_t *ahead_pile[2];   // [kAheadWords][n] prepared pile scripts
  int32_t *ahead_cur[2];     // [kAheadDraws + 1][n] stream cursor after each scripted draw
  uint32_t *ahead_rule[2];   // [kRulePlies][nrow] rule hashes (top 32 bits) per ply
  int32_t *ep_final[2];      // [n] episode counter after the k_rollout that read the slot
  size_t nrow;               // n rounded up to 64: row stride of the ring slots
  uint32_t *ring_mt[3];      // [624][nrow] word-major streams, three calls / two calls ahead
  int32_t *ring_tag[3];      // [nrow] episode * 4 + stage done
  uint64_t *ring_pile[3];    // [3][nrow] draw1's partial scripts
  int32_t *ring_cur[3];      // [kD1Draws + 1][nrow] cursors
  int32_t *ring_k1[3];       // [nrow] draws draw1 completed
  int calls;                 // hz_play calls (ring and play-slot rotation)
  int primed, slot_valid[2];
  // where board b's current stream lives: -1 = mt (its own), k = ahead_mt[k]
  // (an hz_play board that replayed a prepared episode keeps playing on the
  // prepared copy; it is copied into mt only when something else needs it:
  // materialize(), before any other entry point that reads streams)
  int32_t *mt_src;           // [n]
  int lazy;                  // some board may have mt_src >= 0
  // pipeline 2 (hz_env_set_pipeline(e, 2); see k_play2): every board's game
  // spread over thirteen consecutive hz_play calls, one stage per call
  int pipeline;              // 1: chance-ahead (k_rollout's roles), 2: k_play2
  int calls2, primed2;
  int p2_cut[4];             // the play stages' ply boundaries (HZ_P2_CUTS)
  uint32_t *p2_s[14];        // [624][nrow] stream slots (kP2Stream)
  int32_t *p2_s_tag[14];     // [nrow] episode * 8 + 1 P1a / 2 pass 1 / 3 P2a / 4 P2b / 5 seeded, rows 0-223 twisted
  int32_t *p2_s_cur[14];     // [kAheadDraws + 1][nrow] the slot's cursor before draw 0 and after each draw
  uint32_t *p2_ph[2];        // [3][nrow] P2x -> P2y, by call parity
  P2Draw p2_x[4][2];         // D1 -> D2 -> .. -> D5, by call parity
  P2Draw p2_pl[6];           // D5 -> play0 .. play4: a ring of six
  P2Mid p2_m[4][2];          // play0 -> play1 -> .. -> play4, by call parity
  uint32_t *p2_h[6];         // [kRulePlies][nrow] rule hashes, a ring of six
  int32_t *p2_h_tag[6];      // [nrow] their episode
  int32_t *p2_ep[2];         // [nrow] episode counter each board ended the call with
  // a pipeline wave that gives up waiting for its publisher (a bounded spin
  // on an LDS progress counter) ORs a bit into *wait_err (kWaitErr*), so the
  // host raises instead of trusting the call's streams (hz_env_set_error_word)
  int32_t *wait_err_own;     // [1] the handle's own word
  int32_t *wait_err;         // the word the kernels OR into (caller's or own)
  int spin_limit;            // s_sleep rounds before a wait gives up (hz_env_set_spin_limit)
};

#ifdef HZ_DIAG
// diagnostic build only (tools/diag.py): per-lane phase clocks; g_role_only
// >= 0 runs only that k_rollout role (0 draw2, 1 draw1, 2 seed, 3 play)
__device__ uint64_t *g_stamps;
__device__ int g_role_only = -1;
#define HZ_STAMP(slot)                                                    \
  do {                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                    \
    if (g_stamps) g_stamps[(size_t)b * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                    \
  } while (0)
#ifndef HZ_DIAG_ROLES_ONLY
#define HZ_ACC(slot, t0)                                                  \
  do {                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                    \
    uint64_t _t = __builtin_amdgcn_s_memtime();                           \
    acc##slot += _t - (t0);                                               \
    t0 = _t;                                                              \
    __builtin_amdgcn_sched_barrier(0);                                    \
  } while (0)
#else  // role durations only (tools/libhz_roles.so): no stamps inside the ply loop
#define HZ_ACC(slot, t0) \
  do {                   \
  } while (0)
#endif
// phase boundary inside a preparation role: cycles since the role began
#define HZ_PHASE(slot, t0, b)                                                                 \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (g_stamps) g_stamps[(size_t)(b) * 16 + (slot)] = __builtin_amdgcn_s_memtime() - (t0); \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#else
#define HZ_STAMP(slot) \
  do {                 \
  } while (0)
#define HZ_PHASE(slot, t0, b) \
  do {                        \
  } while (0)
#define HZ_ACC(slot, t0) \
  do {                   \
  } while (0)
#endif

namespace {

constexpr int kBlock = 64;  // one wave per workgroup: 4096 boards -> 64 waves

inline int grid_for(int n) { return (n + kBlock - 1) / kBlock; }

// The 64-board LDS kernels (k_reset, k_rollout) run 256
// threads per block: wave 0 plays (lane = board), waves 1-3 only help move
// the block's streams between HBM and LDS (one 162 KB block per CU, so the
// extra waves cost no occupancy) and wait at the barriers meanwhile.
constexpr int kStageThreads = 256;
constexpr size_t kResetLds = (size_t)kMT * kLdsStride * sizeof(uint32_t);  // 162,240 B

// Copy the streams of boards set in `mask` between HBM (one contiguous span
// of nb x 624 words, board-major) and LDS ([624][65]); 16 B per thread-load,
// eight loads in flight per thread.
__device__ __forceinline__ void stage_mt(uint32_t *__restrict__ g, int nb, int tid, uint64_t mask, bool to_lds) {
  uint32_t *lds = hz_lds;
  constexpr int U = 8;
  int total4 = nb * (kMT / 4);
  for (int q0 = 0; q0 < total4; q0 += kStageThreads * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      int o = q * 4, bl = o / kMT, i = o - bl * kMT;
      if (q < total4 && ((mask >> bl) & 1)) {
        if (to_lds) {
          v[u] = reinterpret_cast<const uint4 *>(g)[q];
        } else {
          v[u].x = lds[i * kLdsStride + bl];
          v[u].y = lds[(i + 1) * kLdsStride + bl];
          v[u].z = lds[(i + 2) * kLdsStride + bl];
          v[u].w = lds[(i + 3) * kLdsStride + bl];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      int o = q * 4, bl = o / kMT, i = o - bl * kMT;
      if (q < total4 && ((mask >> bl) & 1)) {
        if (to_lds) {
          lds[i * kLdsStride + bl] = v[u].x;
          lds[(i + 1) * kLdsStride + bl] = v[u].y;
          lds[(i + 2) * kLdsStride + bl] = v[u].z;
          lds[(i + 3) * kLdsStride + bl] = v[u].w;
        } else {
          reinterpret_cast<uint4 *>(g)[q] = v[u];
        }
      }
    }
  }
}

// ------------------------------------------------------------------ reset
// Lane-per-board with the 64 boards' MT arrays staged in LDS as [624][65]
// words (stride 65: the per-lane seeding writes and the board-major write-out
// reads are both bank-conflict free).  Seeding (two serial 623-step passes)
// and the 15 opening draws run at LDS latency; one coalesced pass then writes
// the block's contiguous 64 x 2,496 B of HBM.
__global__ void __launch_bounds__(kStageThreads) k_reset(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                  int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                  int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                  int n, uint64_t seed_base, const uint8_t *__restrict__ sel,
                                                  const uint64_t *__restrict__ seeds) {
  int tid = threadIdx.x;
  int lane = tid & 63;
  bool w0 = tid < 64;
  int b0 = blockIdx.x * kBlock;
  int b = b0 + lane;
  bool act = b < n && (!sel || sel[b]);
  uint64_t actmask = __ballot(act);  // the same in every wave
  if (w0 && act) {
    uint64_t sd;
    if (seeds) {
      sd = seeds[b];
    } else {
      int e = episode[b];
      sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
      episode[b] = e + 1;
    }
    HZ_STAMP(0);
    mt_seed(hz_lds + lane, kLdsStride, sd);
    HZ_STAMP(1);
    StreamDraw<LdsMT> d{LdsMT(lane, kMTSeeded)};
    State s;
    reset_state(s, d);
    HZ_STAMP(2);
    store_state(st, n, b, s);
    pos[b] = d.m.cursor();
    ply[b] = 0;
    seed[b] = sd;
  }
  __syncthreads();
  int nb = n - b0 < kBlock ? n - b0 : kBlock;
  if (w0 && act) HZ_STAMP(3);
  stage_mt(mt + (size_t)b0 * kMT, nb, tid, actmask, false);
  if (w0 && act) HZ_STAMP(4);
}

// ------------------------------------------------------------- legal mask
__global__ void __launch_bounds__(kBlock) k_legal(const uint64_t *__restrict__ st, int n,
                                                  uint64_t *__restrict__ mask, int32_t *__restrict__ count) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  State s = load_state(st, n, b);
  uint64_t m[3];
  int c = legal_mask(s, m);
  if (game_done(s.misc)) { m[0] = m[1] = m[2] = 0; c = 0; }
  mask[(size_t)b * 3 + 0] = m[0];
  mask[(size_t)b * 3 + 1] = m[1];
  mask[(size_t)b * 3 + 2] = m[2];
  if (count) count[b] = c;
}

// ------------------------------------------------------------------- step
__global__ void __launch_bounds__(kBlock) k_step(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                 int32_t *__restrict__ pos, int32_t *__restrict__ ply, int n,
                                                 const int16_t *__restrict__ action, int32_t *__restrict__ status) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  int a = action[b];
  if (a < 0) {
    if (status) status[b] = ST_NOOP;
    return;
  }
  State s = load_state(st, n, b);
  StreamDraw<MT> d{MT(mt + (size_t)b * kMT, pos[b])};
  int r = step_state(s, a, d);
  if (r == ST_OK) {
    store_state(st, n, b, s);
    pos[b] = d.m.cursor();
    ply[b] += 1;
  }
  if (status) status[b] = r;
}

// -------------------------------------------- replenish / end-turn (facade)
__global__ void __launch_bounds__(kBlock) k_turn_op(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                    int32_t *__restrict__ pos, int n, const uint8_t *__restrict__ sel,
                                                    int op) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n || (sel && !sel[b])) return;
  State s = load_state(st, n, b);
  StreamDraw<MT> d{MT(mt + (size_t)b * kMT, pos[b])};
  if (op == 0) replenish(s, d);
  else end_turn(s, d);
  store_state(st, n, b, s);
  pos[b] = d.m.cursor();
}

// ------------------------------------------------------------------ score
__global__ void __launch_bounds__(kBlock) k_score(const uint64_t *__restrict__ st, int n, int32_t *__restrict__ out,
                                                  int32_t *__restrict__ parts) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  State s = load_state(st, n, b);
  for (int p = 0; p < 2; p++) {
    uint32_t pb[4];
    planes_of(s, p, pb);
    ScoreParts r = score_parts(pb);
    if (out) out[(size_t)b * 2 + p] = r.grass + r.mount + r.field + r.bldg + r.water;
    if (parts) {
      int32_t *o = parts + ((size_t)b * 2 + p) * 5;
      o[0] = r.grass; o[1] = r.mount; o[2] = r.field; o[3] = r.bldg; o[4] = r.water;
    }
  }
}

// ------------------------------------------------------------ rule policy
__global__ void __launch_bounds__(kBlock) k_rule(const uint64_t *__restrict__ seed, const int32_t *__restrict__ ply,
                                                 int n, const uint64_t *__restrict__ mask,
                                                 const int32_t *__restrict__ count, int16_t *__restrict__ action) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  uint64_t m[3] = {mask[(size_t)b * 3], mask[(size_t)b * 3 + 1], mask[(size_t)b * 3 + 2]};
  int L = count ? count[b] : __popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]);
  action[b] = L > 0 ? (int16_t)kth_action(m, rule_pick(seed[b], ply[b], L)) : (int16_t)-1;
}

// ------------------------------------------------ one ply of the surface
// The per-ply API path in one launch: get_legal_moves -> the benchmark's
// rule pick -> apply_move (harmonies_engine.py:145-298) for every board,
// with the three calls' outputs written as hz_legal_mask, hz_rule_actions
// and hz_step write them (bit-identical: the same device functions in the
// same order).  One 48 B state load and store per board instead of two loads
// and a store across three launches.
__global__ void __launch_bounds__(kBlock) k_ply(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                const uint64_t *__restrict__ seed, int n,
                                                uint64_t *__restrict__ mask, int32_t *__restrict__ count,
                                                int16_t *__restrict__ action, int32_t *__restrict__ status) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  State s = load_state(st, n, b);
  uint64_t m[3];
  int c = legal_mask(s, m);
  if (game_done(s.misc)) { m[0] = m[1] = m[2] = 0; c = 0; }
  if (mask) {
    mask[(size_t)b * 3 + 0] = m[0];
    mask[(size_t)b * 3 + 1] = m[1];
    mask[(size_t)b * 3 + 2] = m[2];
  }
  if (count) count[b] = c;
  const int p = ply[b];
  const int a = c > 0 ? kth_action(m, rule_pick(seed[b], p, c)) : -1;
  if (action) action[b] = (int16_t)a;
  if (a < 0) {
    if (status) status[b] = ST_NOOP;
    return;
  }
  StreamDraw<MT> d{MT(mt + (size_t)b * kMT, pos[b])};
  int r = step_state(s, a, d);
  if (r == ST_OK) {
    store_state(st, n, b, s);
    pos[b] = d.m.cursor();
    ply[b] = p + 1;
  }
  if (status) status[b] = r;
}

// ---------------------------------------------------------------- rollout
// Lane-per-board with the block's 64 MT streams resident in LDS for the
// whole call ([624][65] words, as in k_reset): every draw reads and twists at
// LDS latency instead of paying a scattered HBM round trip per draw.  The
// streams are staged in (or seeded in place when reset_first) and written
// back once.
// ------------------------------------------------------------ chance-ahead
// The piles a game draws do not depend on its moves: only a turn end draws
// (one pile: a turn takes exactly one of the five), the bag changes only by
// draws, and the stream only by draws.  So a board's whole chance sequence
// for an episode is fixed by its seed.  The preparing blocks of one hz_play
// launch (on CUs the playing blocks leave idle) seed the stream of each
// board's next episode and run its first kAheadDraws pile draws on the
// initial bag: they store the piles (9 bits each, packed), the stream
// cursor after each draw, and the stream.  The next launch plays such a
// board from the pile script; a game that needs more draws continues on the
// stored stream (slot, global memory) from the cursor after the last
// scripted draw.
constexpr int kAheadDraws = 24;             // 5 opening + 19 turn ends (rule games: at most 23)
constexpr int kAheadWords = (9 * kAheadDraws + 63) / 64;  // 4 u64: the piles, 9 bits each

// The draws that do not come from the script (boards not prepared ahead, and
// a script's rare overrun) live out of line: one copy of the sampling code
// instead of one per refill site keeps the ply loop's code small.  State
// goes in and out by value so the caller's copy stays in registers.
struct SlowDrawOut {
  uint32_t p9;
  int mpos, mtw, gpos, gtw;
};

__device__ __noinline__ SlowDrawOut play_draw_slow(uint64_t misc, int lane, int mpos, int mtw, int scripted,
                                                    uint32_t *gw, int gcursor) {
  SlowDrawOut o;
  uint32_t p9;
  if (scripted) {
    MT gm(gw, gcursor);
    o.p9 = draw_pile(misc, gm, p9) ? p9 : 0x1FFu;
    o.mpos = mpos;
    o.mtw = mtw;
    o.gpos = gm.pos;
    o.gtw = gm.tw;
  } else {
    LdsMT m(lane, mpos | (mtw << 16));
    m.prefetch();
    o.p9 = draw_pile(misc, m, p9) ? p9 : 0x1FFu;
    o.mpos = m.pos;
    o.mtw = m.tw;
    o.gpos = gcursor & 0xFFFF;
    o.gtw = gcursor >> 16;
  }
  return o;
}

struct PlayDraw {
  LdsMT m;                 // stream in LDS (boards not prepared ahead, auto-reset games)
  bool scripted;           // replaying the prepared pile script
  bool fell;               // script exhausted: drawing from the slot stream
  int d;                   // script entries consumed
  int nd;                  // script length (<= kAheadDraws)
  uint64_t q0, q1, q2, q3; // the rest of the script, next entry in the low 9 bits
  MT gm;                   // slot stream (valid once fell)
  const int32_t *cur_tail; // cursor after the last scripted draw (global)

  __device__ __forceinline__ uint32_t operator()(uint64_t misc) { return take(misc, true); }

  // one draw per lane, any source
  __device__ __forceinline__ uint32_t draw_one(uint64_t misc) {
    if (scripted && d < nd) {
      // pop the next 9-bit entry: a shift queue (a select over the four
      // words would become a dynamic index into a scratch copy)
      uint32_t p9 = (uint32_t)q0 & 0x1FFu;
      q0 = (q0 >> 9) | (q1 << 55);
      q1 = (q1 >> 9) | (q2 << 55);
      q2 = (q2 >> 9) | (q3 << 55);
      q3 >>= 9;
      d++;
      return p9;
    }
    if (scripted && !fell) {
      gm = MT(gm.w, *cur_tail);
      fell = true;
    }
    SlowDrawOut o = play_draw_slow(misc, m.lane, m.pos, m.tw, scripted, gm.w, gm.cursor());
    m.pos = o.mpos;
    m.tw = o.mtw;
    gm.pos = o.gpos;
    gm.tw = o.gtw;
    return o.p9;
  }

  // the next script entry, unconditionally (the caller checked d < nd)
  __device__ __forceinline__ uint32_t pop() {
    uint32_t p9 = (uint32_t)q0 & 0x1FFu;
    q0 = (q0 >> 9) | (q1 << 55);
    q1 = (q1 >> 9) | (q2 << 55);
    q2 = (q2 >> 9) | (q3 << 55);
    q3 >>= 9;
    d++;
    return p9;
  }
  // both refills of a turn pair come from the script: two entries left (a
  // script holds <= 24 draws, so the bag still has >= 48 tiles and every
  // turn end refills exactly one pile)
  __device__ __forceinline__ bool pair_pops() const { return scripted && d + 2 <= nd; }

  // reset_state when the lane replays a script of >= 5 entries
  __device__ __forceinline__ void scripted_reset(State &s) {
    s.pl[0] = s.pl[1] = s.pl[2] = s.pl[3] = 0;
    uint64_t open = q0 & ((1ull << 45) - 1);
    s.piles = open | (5ull << 45);
    uint64_t misc = 0x1FF;  // empty hand, player 0, choose_pile
#pragma unroll
    for (int t = 0; t < 6; t++) misc = set_bits(misc, 11 + 5 * t, 5, (uint64_t)initial_count(t));
#pragma unroll
    for (int i = 0; i < 5; i++) apply_pile_fast(misc, (uint32_t)(open >> (9 * i)) & 0x1FFu);
    s.misc = misc;
    q0 = (q0 >> 45) | (q1 << 19);
    q1 = (q1 >> 45) | (q2 << 19);
    q2 = (q2 >> 45) | (q3 << 19);
    q3 >>= 45;
    d = 5;
  }

  // a draw by the lanes with `want` (0x1FF for the others): while every such
  // lane replays its script (wave-uniform test) a plain masked pop, else the
  // general per-lane path
  __device__ __forceinline__ uint32_t take(uint64_t misc, bool want) {
    bool fast = scripted && d < nd;
    if (__all(!want || fast)) {
      uint32_t p9 = want ? (uint32_t)q0 & 0x1FFu : 0x1FFu;
      uint64_t n0 = (q0 >> 9) | (q1 << 55), n1 = (q1 >> 9) | (q2 << 55), n2 = (q2 >> 9) | (q3 << 55);
      q0 = want ? n0 : q0;
      q1 = want ? n1 : q1;
      q2 = want ? n2 : q2;
      q3 = want ? q3 >> 9 : q3;
      d += want ? 1 : 0;
      return p9;
    }
    uint32_t p9 = 0x1FFu;
    if (want) p9 = draw_one(misc);
    return p9;
  }
};

// Chance-ahead preparation: a three-stage pipeline in the blocks of each
// hz_play launch beyond the playing ones (4 x 64 blocks of 162 KB LDS: one
// per CU, every CU of the chip).  Stage k works on each board's episode k
// calls ahead (the episode counter the previous launch left, plus k):
//   seed  (k = 3) blocks [3 nblk, 4 nblk): the stream seeded in LDS and
//     stored as seeded to a word-major ring slot (waves 1-3 store rows while
//     wave 0 still seeds);
//   draw1 (k = 2) blocks [2 nblk, 3 nblk): rows [0, kAheadTwist) staged
//     into LDS twisted on the way in (every source still old: no serial
//     chain), the first kD1Draws pile draws run
//     (a lane stops at a draw that would twist further; the next stage
//     redoes it), the partial script, cursors and draw count written beside
//     the slot;
//   draw2 (k = 1) blocks [nblk, 2 nblk): the whole slot staged and twisted
//     likewise, the remaining draws run, and stream (board-major), script,
//     cursors and tag written to the play slot the next call's playing
//     blocks replay.
// Each ring slot carries one tag per board, episode * 4 + stage done, so a
// stage only continues work its predecessor finished for the same
// episode; otherwise it redoes the earlier stages itself in LDS.  A slot's
// contents depend only on (board, episode), so a matching tag is always
// right, whatever happened between the calls.
constexpr int kD1Draws = 16;
// the rule hashes of an episode's first kRulePlies plies (rule games end by
// ply 72), computed by draw2's otherwise idle waves 1-3 and read by the
// playing wave a turn pair ahead; plies past them are hashed in place
constexpr int kRulePlies = 80;
constexpr int kRing = 3;
static_assert(kD1Draws <= kAheadDraws && 9 * kD1Draws <= 192, "draw1's script sits in words 0-2");

// one ring slot: the stream word-major (row r of board b at mt[r * nrow + b],
// nrow = n rounded up to 64, so a wave's row is 256 contiguous bytes), and
// per board the tag, draw1's script, cursors and draw count
// wait-error bits (hz_env_set_error_word): a bounded wait gave up
constexpr int32_t kWaitErrSeedRows = 1;  // k_rollout's seed stage: wave 0's pass-2 row progress
constexpr int32_t kWaitErrP2Twist = 2;   // k_play2's twist wave: P2c's progress
constexpr int kSpinLimitDefault = 1 << 22;
__device__ __forceinline__ void wait_failed(int32_t *err, int32_t bit) {
  if (err) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Ring {
  uint32_t *mt;
  int32_t *tag;   // [nrow] episode * 4 + stage (1 seeded, 2 draw1 done); -1 none
  uint64_t *pile; // [kAheadWords][nrow]
  int32_t *cur;   // [kD1Draws + 1][nrow] cursor before draw 0 and after each draw
  int32_t *k1;    // [nrow] draws draw1 completed
  int32_t *err;   // the env's wait-error word (seed stage)
  int spin;       // spin bound of the seed stage's row wait
};

// rows [r0, r1) of the block's 64 boards, word-major HBM -> LDS [row][65];
// 16 B per thread-load, eight in flight (conflict-free LDS writes: a wave
// covers four rows, whose banks are shifted by one)
__device__ __forceinline__ void stage_rows(const uint32_t *__restrict__ slot, size_t nrow, int b0, int r0, int r1,
                                           int tid) {
  constexpr int U = 8;
  int total = (r1 - r0) * 16;
  for (int q0 = 0; q0 < total; q0 += kStageThreads * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      q = q < total ? q : total - 1;
      v[u] = *reinterpret_cast<const uint4 *>(slot + (size_t)(r0 + (q >> 4)) * nrow + b0 + (q & 15) * 4);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      if (q < total) {
        uint32_t *d = hz_lds + (r0 + (q >> 4)) * kLdsStride + (q & 15) * 4;
        d[0] = v[u].x;
        d[1] = v[u].y;
        d[2] = v[u].z;
        d[3] = v[u].w;
      }
    }
  }
}

// all rows of the boards in `mask`, LDS -> word-major HBM (coalesced rows)
__device__ __forceinline__ void unstage_rows(uint32_t *__restrict__ slot, size_t nrow, int b0, int tid,
                                             uint64_t mask) {
  int lane = tid & 63;
  if (!((mask >> lane) & 1)) return;
  for (int r = tid >> 6; r < kMT; r += kStageThreads / 64)
    slot[(size_t)r * nrow + b0 + lane] = hz_lds[r * kLdsStride + lane];
}

// run script entries [from, to) of a board's chance sequence on its LDS
// stream, recording packed piles and the cursor after each draw at
// cur[(i + 1) * cs] (a rolled loop: one copy of the sampling code, so the
// instruction cache holds it; the script word is picked by selects, not by
// a dynamic index).  StopOnTwist: end before a draw that twisted (the rows
// past the staged ones are not in LDS).  Returns the entries completed.
template <bool StopOnTwist = false>
__device__ __forceinline__ int run_script(StreamDraw<LdsMT> &d, uint64_t &bag, uint64_t q[kAheadWords],
                                          int32_t *__restrict__ cur, size_t cs, int from, int to) {
  static_assert(kAheadWords == 4, "script words");
  uint64_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  int i = from;
#pragma unroll 1
  for (; i < to; i++) {
    uint32_t p9 = d(bag);
    if (StopOnTwist && d.m.tw != kAheadTwist) break;
    apply_pile_fast(bag, p9);  // 0x1FF: no tiles
    // entry i at bit 9 i of the 256-bit script (PlayDraw pops 9 bits at a time)
    int bit = 9 * i, wd = bit >> 6, off = bit & 63;
    uint64_t lo = (uint64_t)p9 << off;
    uint64_t hi = off > 55 ? (uint64_t)p9 >> (64 - off) : 0ull;
    q0 |= wd == 0 ? lo : 0ull;
    q1 |= wd == 1 ? lo : wd == 0 ? hi : 0ull;
    q2 |= wd == 2 ? lo : wd == 1 ? hi : 0ull;
    q3 |= wd == 3 ? lo : wd == 2 ? hi : 0ull;
    cur[(size_t)(i + 1) * cs] = d.m.cursor();
  }
  q[0] = q0; q[1] = q1; q[2] = q2; q[3] = q3;
  return i;
}

__device__ __forceinline__ uint64_t initial_bag() {
  uint64_t bag = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) bag = set_bits(bag, 11 + 5 * t, 5, (uint64_t)initial_count(t));
  return bag;
}

__device__ __forceinline__ uint64_t episode_seed(uint64_t seed_base, int b, int e) {
  return seed_base + (uint64_t)b + ((uint64_t)e << 32);
}

// Rows [0, kAheadTwist) of the block's 64 boards from a slot holding the
// streams as seeded, word-major HBM -> LDS [row][65], written as the next
// generation's: row i from rows i, i + 1 and i + 397 of the slot (all still
// old), read straight from HBM (16 B per load, 12 in flight per thread), so
// the twist needs no LDS round trip and no barrier.
__device__ __forceinline__ void stage_rows_twisted(const uint32_t *__restrict__ slot, size_t nrow, int b0, int tid) {
  constexpr int U = 4;
  constexpr int total = kAheadTwist * 16;
  for (int q0 = 0; q0 < total; q0 += kStageThreads * U) {
    uint4 c[U], c1[U], f[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      q = q < total ? q : total - 1;
      const uint32_t *p = slot + b0 + (q & 15) * 4;
      int r = q >> 4;
      c[u] = *reinterpret_cast<const uint4 *>(p + (size_t)r * nrow);
      c1[u] = *reinterpret_cast<const uint4 *>(p + (size_t)(r + 1) * nrow);
      f[u] = *reinterpret_cast<const uint4 *>(p + (size_t)(r + 397) * nrow);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      int q = q0 + u * kStageThreads + tid;
      if (q < total) {
        uint32_t *d = hz_lds + (q >> 4) * kLdsStride + (q & 15) * 4;
        d[0] = twist_word(c[u].x, c1[u].x, f[u].x);
        d[1] = twist_word(c[u].y, c1[u].y, f[u].y);
        d[2] = twist_word(c[u].z, c1[u].z, f[u].z);
        d[3] = twist_word(c[u].w, c1[u].w, f[u].w);
      }
    }
  }
}

// a board's stream seeded and pre-twisted in its LDS column (cursor kMTAhead)
__device__ __forceinline__ void seed_in_lds(int lane, uint64_t sd) {
  mt_seed(hz_lds + lane, kLdsStride, sd);
  LdsMT m(lane, kMTSeeded);
  m.twist_ahead(kAheadTwist);
}

// pass-2 progress of the seed stage's wave 0, published to waves 1-3 in
// LDS every 32 rows and at the end of the group loop.  A wave's LDS
// operations execute in order, so a plain store of the counter after the
// rows' stores is seen after them (the empty asm only keeps the compiler
// from reordering; a release fence would wait for every pending LDS read
// of the prefetch); readers load it with acquire.  mt_seed_tab reports
// rows = 10, 18, ..., 618; published: 34, 66, ..., 610, 618.
constexpr int kLastPub = 618;
constexpr int kSeedChunk = (kStageThreads - 64) / 16;  // rows per pass of waves 1-3
constexpr int kOverlapEnd = 2 + (kLastPub - 2) / kSeedChunk * kSeedChunk;
struct SeedProgress {
  int *flag;
  __device__ __forceinline__ void operator()(int rows) const {
    if ((rows & 31) == 2 || rows == kLastPub) {
      asm volatile("" ::: "memory");
      __hip_atomic_store(flag, rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
};

// The seed stage's LDS: init_genrand's table at offset 0 (its reads are
// immediate offsets) and the 64 streams after it as [624][64] (row-major,
// so four boards of a row are one aligned 16-B read): kMT + kMT * 64 words
// = the block's 162,240 B.
constexpr int kSeedStride = 64;
static_assert((kMT * kSeedStride + kMT) * 4 <= (int)kResetLds, "seed stage LDS");

__device__ __forceinline__ void seed_stage(int blk, Ring rs, size_t nrow, const int32_t *__restrict__ ep_final,
                                           int n, uint64_t seed_base) {
  __shared__ int s_rows;  // pass-2 rows [2, s_rows) of every board are final
  int tid = threadIdx.x;
  int lane = tid & 63;
  int b = blk * kBlock + lane;
  bool act = b < n;
#ifdef HZ_DIAG
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  int e = act ? ep_final[b] + 3 : 0;
  uint32_t *tab = hz_lds, *rows = hz_lds + kMT;
  for (int i = tid; i < kMT; i += kStageThreads) tab[i] = kInitGen.v[i];
  if (tid == 0) s_rows = 0;
  __syncthreads();
  // Stores: four boards of a row per thread (one 16-B LDS read, one 16-B
  // store; a wave covers four rows), the stream as seeded (the draw stages
  // twist rows [0, kAheadTwist) as they stage them, stage_rows_twisted).  Waves 1-3
  // store rows [2, kOverlapEnd) chunk by chunk as wave 0 publishes its pass-2
  // progress; after the barrier all four waves store the rest (the last
  // rows and rows 0, 1, final last).  Columns past n hold whatever LDS held;
  // the next stages never read them.
  int c4 = (tid & 15) * 4;
  uint32_t *out = rs.mt + (size_t)blk * kBlock + c4;
  auto row4 = [&](int r) { return *reinterpret_cast<const uint4 *>(rows + r * kSeedStride + c4); };
  if (tid < 64) {
    if (act) {
      mt_seed_tab<kSeedStride>(rows + lane, tab, episode_seed(seed_base, b, e), SeedProgress{&s_rows});
      HZ_PHASE(0, t0, b);
    }
  } else {
    int done = 0;
#pragma unroll 1
    for (int r0 = 2; r0 < kOverlapEnd; r0 += kSeedChunk) {
      // wave 0 publishes every row up to kLastPub; the bound only guards
      // against a hang should that ever change, and giving up is reported
      for (int spin = 0; done < r0 + kSeedChunk && spin < rs.spin; spin++) {
        __builtin_amdgcn_s_sleep(1);
        done = __hip_atomic_load(&s_rows, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (done < r0 + kSeedChunk) {
        done = r0 + kSeedChunk;  // (one report per chunk at most; the rows stored are then untrusted)
        wait_failed(rs.err, kWaitErrSeedRows);
      }
      int r = r0 + ((tid - 64) >> 4);
      *reinterpret_cast<uint4 *>(out + (size_t)r * nrow) = row4(r);
    }
#ifdef HZ_DIAG_ROLES_ONLY
    if (tid < 128 && act) HZ_PHASE(11, t0, b);
#endif
  }
  __syncthreads();
#ifdef HZ_DIAG_ROLES_ONLY
  if (tid < 64 && act) HZ_PHASE(12, t0, b);
#endif
  {  // rows [kOverlapEnd, 624) and 0, 1: 12 rows, one per 16-thread group
    int i = tid >> 4, r = i < kMT - kOverlapEnd ? kOverlapEnd + i : i - (kMT - kOverlapEnd);
    if (r < 2 || r >= kOverlapEnd) *reinterpret_cast<uint4 *>(out + (size_t)r * nrow) = row4(r);
  }
  if (tid < 64 && act) {
    rs.tag[b] = e * 4 + 1;
    HZ_PHASE(1, t0, b);
  }
}

__device__ __forceinline__ void draw1_stage(int blk, Ring r1, size_t nrow, const int32_t *__restrict__ ep_final,
                                            int n, uint64_t seed_base, int draws) {
  int tid = threadIdx.x;
  int lane = tid & 63;
  int b0 = blk * kBlock;
  int b = b0 + lane;
  bool act = b < n;
#ifdef HZ_DIAG
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  int e = act ? ep_final[b] + 2 : 0;
  bool seeded = act && r1.tag[b] == e * 4 + 1;
  uint64_t smask = __ballot(seeded), fmask = __ballot(act && !seeded);  // the same in every wave
  // rows [0, kAheadTwist), twisted on the way in
  if (smask) stage_rows_twisted(r1.mt, nrow, b0, tid);
  // boards the seed stage missed: seeded here, their stream (as seeded,
  // like the seed stage's) to the slot, then twisted in place
  if (tid < 64 && act && !seeded) mt_seed(hz_lds + lane, kLdsStride, episode_seed(seed_base, b, e));
  __syncthreads();
  if (fmask) {
    unstage_rows(r1.mt, nrow, b0, tid, fmask);
    __syncthreads();
  }
  if (tid < 64 && act) {
    HZ_PHASE(2, t0, b);
    if (!seeded) {
      LdsMT m(lane, kMTSeeded);
      m.twist_ahead(kAheadTwist);
    }
    StreamDraw<LdsMT> d{LdsMT(lane, kMTAhead)};
    uint64_t bag = initial_bag(), q[kAheadWords] = {};
    int32_t *cur = r1.cur + b;
    cur[0] = kMTAhead;
    int k = draws < kD1Draws ? draws : kD1Draws;
    // only the twisted rows are live: a lane stops before a draw that would
    // twist further (draw2, holding the whole stream, redoes it), so the
    // slot's stream stays as seeded and every cursor's tw is kAheadTwist
    int k1 = run_script<true>(d, bag, q, cur, nrow, 0, k);
#pragma unroll
    for (int w = 0; w < 3; w++) r1.pile[(size_t)w * nrow + b] = q[w];
    r1.k1[b] = k1;
    r1.tag[b] = e * 4 + 2;
    HZ_PHASE(3, t0, b);
  }
}

__device__ __forceinline__ void draw2_stage(int blk, Ring r2, size_t nrow, uint32_t *__restrict__ out_mt,
                                            int32_t *__restrict__ tag, uint64_t *__restrict__ pile,
                                            int32_t *__restrict__ cur, uint32_t *__restrict__ rule,
                                            const int32_t *__restrict__ ep_final, int n, uint64_t seed_base,
                                            int draws) {
  int tid = threadIdx.x;
  int lane = tid & 63;
  int b0 = blk * kBlock;
  int b = b0 + lane;
  bool act = b < n;
  uint64_t actmask = __ballot(act);
  int nb = n - b0 < kBlock ? n - b0 : kBlock;
#ifdef HZ_DIAG
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  int e = act ? ep_final[b] + 1 : 0;
  bool ok = act && r2.tag[b] == e * 4 + 2;
  uint64_t okmask = __ballot(ok);
  if (okmask) {  // the slot holds the stream as seeded; draw1's cursors say 224 rows twisted
    stage_rows_twisted(r2.mt, nrow, b0, tid);
    stage_rows(r2.mt, nrow, b0, kAheadTwist, kMT, tid);
  }
  __syncthreads();
  if (tid < 64 && act) HZ_PHASE(4, t0, b);
  if (tid >= 64 && act) {  // waves 1-3, while wave 0 draws: the episode's rule hashes
    uint64_t rk = rule_key(episode_seed(seed_base, b, e));
#pragma unroll 1
    for (int j = (tid >> 6) - 1; j < kRulePlies; j += 3) rule[(size_t)j * nrow + b] = rule_h32(rk, j);
  }
  if (tid < 64 && act) {
    uint64_t bag = initial_bag(), q[kAheadWords] = {};
    int start = 0, c0 = kMTAhead;
    if (ok) {  // continue after draw1's draws
      int k1 = r2.k1[b];
      c0 = r2.cur[(size_t)k1 * nrow + b];
#pragma unroll
      for (int w = 0; w < 3; w++) q[w] = r2.pile[(size_t)w * nrow + b];
      // draw1's cursors over (all loads issued before the stores) and the
      // bag replayed from its script; entries past k1 unused
      int32_t cv[kD1Draws];
#pragma unroll
      for (int i = 0; i < kD1Draws; i++) cv[i] = r2.cur[(size_t)i * nrow + b];
#pragma unroll
      for (int i = 0; i < kD1Draws; i++)
        if (i < k1) cur[(size_t)i * n + b] = cv[i];
#pragma unroll
      for (int i = 0; i < kD1Draws; i++) {
        uint32_t p9 = (uint32_t)(q[(9 * i) >> 6] >> ((9 * i) & 63));
        if ((9 * i & 63) > 55) p9 |= (uint32_t)(q[((9 * i) >> 6) + 1] << (64 - ((9 * i) & 63)));
        apply_pile_fast(bag, i < k1 ? p9 & 0x1FFu : 0x1FFu);
      }
      start = k1;
    } else {
      seed_in_lds(lane, episode_seed(seed_base, b, e));
    }
    cur[(size_t)start * n + b] = c0;
    StreamDraw<LdsMT> d{LdsMT(lane, c0)};
    run_script(d, bag, q, cur + b, n, start, draws);
    HZ_PHASE(14, t0, b);
#pragma unroll
    for (int w = 0; w < kAheadWords; w++) pile[(size_t)w * n + b] = q[w];
    tag[b] = e;
  }
  __syncthreads();
  stage_mt(out_mt + (size_t)b0 * kMT, nb, tid, actmask, false);
}

// AutoReset / Record are template parameters so that the common variant
// (play to the end, no trajectory) has a plain loop: no reset path, no
// record stores, fewer live scalar values across the ply loop.
template <bool AutoReset, bool Record>
__global__ void __launch_bounds__(kStageThreads) k_rollout(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                    int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                    int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                    int n, uint64_t seed_base, int max_plies, int auto_reset,
                                                    int reset_first, uint64_t *__restrict__ traj_state,
                                                    uint64_t *__restrict__ traj_mask,
                                                    int16_t *__restrict__ traj_action, int32_t *__restrict__ games_done,
                                                    int32_t *__restrict__ steps_done,
                                                    uint32_t *__restrict__ ahead_mt,
                                                    const int32_t *__restrict__ ahead_tag,
                                                    const uint64_t *__restrict__ ahead_pile,
                                                    const int32_t *__restrict__ ahead_cur, int ahead_draws,
                                                    int32_t *__restrict__ ep_final, int nblk,
                                                    uint32_t *__restrict__ prep_mt, int32_t *__restrict__ prep_tag,
                                                    uint64_t *__restrict__ prep_pile, int32_t *__restrict__ prep_cur,
                                                    const int32_t *__restrict__ prep_ep, Ring rs, Ring r1,
                                                    Ring r2, long nrow, const uint32_t *__restrict__ ahead_rule,
                                                    uint32_t *__restrict__ prep_rule, int32_t *__restrict__ mt_src,
                                                    int src_slot) {
#ifdef HZ_DIAG
  uint64_t role_t0 = __builtin_amdgcn_s_memtime();
#endif
  if ((int)blockIdx.x >= nblk) {  // chance-ahead roles (uniform per block)
    int blk = (int)blockIdx.x - nblk;
    int role = blk / nblk;
    blk -= role * nblk;
#ifdef HZ_PREP_DELAY
    if (role < 2) __builtin_amdgcn_s_sleep(HZ_PREP_DELAY);
#endif
#ifdef HZ_DIAG
    if (g_role_only >= 0 && g_role_only != role) return;
#endif
    if (role == 0)
      draw2_stage(blk, r2, (size_t)nrow, prep_mt, prep_tag, prep_pile, prep_cur, prep_rule, prep_ep, n, seed_base,
                  ahead_draws);
    else if (role == 1)
      draw1_stage(blk, r1, (size_t)nrow, prep_ep, n, seed_base, ahead_draws);
    else
      seed_stage(blk, rs, (size_t)nrow, prep_ep, n, seed_base);
#ifdef HZ_DIAG
    {  // role durations: slot 6 (draw2 blocks), 15 (draw1), 7 (seed), per board of the block
      int bb = blk * kBlock + (threadIdx.x & 63);
      if (g_stamps && threadIdx.x < 64 && bb < n)
        g_stamps[(size_t)bb * 16 + (role == 0 ? 6 : role == 1 ? 15 : 7)] = __builtin_amdgcn_s_memtime() - role_t0;
    }
#endif
    return;
  }
#ifdef HZ_DIAG
  if (g_role_only >= 0 && g_role_only != 3) return;
#endif
  __shared__ uint64_t s_lds_mask;
  int tid = threadIdx.x;
  int lane = tid & 63;
  bool w0 = __builtin_amdgcn_readfirstlane(tid) < 64;  // wave-uniform: wave 0 plays
  int b0 = blockIdx.x * kBlock;
  int b = b0 + lane;
  bool act = b < n;
  uint64_t actmask = __ballot(act);  // the same in every wave
  int nb = n - b0 < kBlock ? n - b0 : kBlock;
  uint32_t *g = mt + (size_t)b0 * kMT;
  // reset_first: a board whose episode was prepared ahead plays its pile
  // script; the others seed their stream in LDS below
  // the script words are read with the tag (one memory round trip); they
  // are used only when the tag matches
  uint64_t pq0 = 0, pq1 = 0, pq2 = 0, pq3 = 0;
  if (reset_first && act && ahead_pile && w0) {
    pq0 = ahead_pile[b];
    pq1 = ahead_pile[(size_t)n + b];
    pq2 = ahead_pile[(size_t)2 * n + b];
    pq3 = ahead_pile[(size_t)3 * n + b];
  }
  int ep0 = act ? episode[b] : 0;
  bool seeded = reset_first && act && ahead_tag && ahead_tag[b] == ep0;
  // the episode's rule hashes into rows [0, kRulePlies) of each seeded
  // lane's LDS column (a seeded lane replays its script and never keeps its
  // stream in LDS), all four waves, issued with the tag loads
  // (16-B loads: four boards of a row per thread; an unseeded lane's column
  // is overwritten by its seeding after the barrier)
  if (reset_first && ahead_rule) {
    constexpr int K = kRulePlies * 16 / kStageThreads;
    static_assert(kRulePlies * 16 % kStageThreads == 0, "hash rows per pass");
    uint4 hv[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      int q = k * kStageThreads + tid;
      hv[k] = *reinterpret_cast<const uint4 *>(ahead_rule + (size_t)(q >> 4) * nrow + b0 + (q & 15) * 4);
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      int q = k * kStageThreads + tid;
      uint32_t *d = hz_lds + (q >> 4) * kLdsStride + (q & 15) * 4;
      d[0] = hv[k].x;
      d[1] = hv[k].y;
      d[2] = hv[k].z;
      d[3] = hv[k].w;
    }
  }
  if (!reset_first) stage_mt(g, nb, tid, actmask, true);
  __syncthreads();
#ifdef HZ_DIAG_ROLES_ONLY
  if (w0 && act) HZ_PHASE(13, role_t0, b);
#endif
  // a board replaying a prepared episode plays on to the end on the
  // prepared stream in ahead_mt (mt_src); it reaches the board's own mt
  // only if something else needs it (materialize)
  if (w0 && act) {
    PlayDraw draw{LdsMT(lane, reset_first ? kMTSeeded : pos[b]), seeded, false, 0, ahead_draws, 0, 0, 0, 0,
                  MT(ahead_mt ? ahead_mt + (size_t)b * kMT : nullptr, 0),
                  ahead_cur ? ahead_cur + (size_t)ahead_draws * n + b : nullptr};
    if (seeded) {
      draw.q0 = pq0;
      draw.q1 = pq1;
      draw.q2 = pq2;
      draw.q3 = pq3;
    }
    State s;
    int g_ply, games = 0, steps = 0;
    uint64_t sd, rkey;
    if (reset_first) {
      int e = ep0;
      sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
      rkey = rule_key(sd);
      episode[b] = e + 1;
      if (!seeded) mt_seed(hz_lds + lane, kLdsStride, sd);
      if (__all(seeded) && ahead_draws >= 5) {
        // HarmoniesGameState() from the script: its first five entries are
        // the opening piles (a full bag always fills them), 45 bits laid out
        // as the piles word
        draw.scripted_reset(s);
      } else {
        reset_state(s, draw);
      }
      g_ply = 0;
#ifdef HZ_DIAG_ROLES_ONLY
      HZ_PHASE(8, role_t0, b);
#endif
    } else {
      s = load_state(st, n, b);
      g_ply = ply[b];
      sd = seed[b];
      rkey = rule_key(sd);
    }
#ifdef HZ_DIAG
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint64_t acc8 = 0, acc9 = 0, acc10 = 0, acc11 = 0, acc12 = 0, acc13 = 0;
#endif
    bool lds_used = !seeded;  // the LDS copy of the stream is live
    bool pre = seeded && ahead_rule != nullptr;  // the episode's rule hashes are in LDS
    for (int i = 0; i < max_plies; i++) {
      if (phase_of(s.misc) == PH_OVER) {  // finished (scored, or scoring deferred)
        if constexpr (!AutoReset) {
          if (Record && traj_action) {
            for (int j = i; j < max_plies; j++) traj_action[(size_t)j * n + b] = -1;
          }
          break;
        }
        if (score_pending(s.misc)) finish_game(s);  // the finished game is scored all the same
        int e = episode[b];
        sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
        rkey = rule_key(sd);
        episode[b] = e + 1;
        mt_seed(hz_lds + lane, kLdsStride, sd);
        draw.m = LdsMT(lane, kMTSeeded);
        draw.scripted = false;
        lds_used = true;
        pre = false;
        reset_state(s, draw);
        g_ply = 0;
      }
      if constexpr (!Record) {
        // a pair of whole turns at once while every board of the wave still
        // playing is at a pair boundary (always, for boards reset together)
        if (__all(i + 8 <= max_plies && turn_pair_safe(s))) {
          uint32_t h[8];
          if (__all(pre && g_ply + 8 <= kRulePlies)) {
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = hz_lds[(g_ply + j) * kLdsStride + lane];
          } else {
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = rule_h32(rkey, g_ply + j);
          }
          int done = 4;
          if (__all(draw.pair_pops())) {  // the refills are plain pops
            play_turn_h<0, PlayDraw, true>(s, draw, h[0], h[1], h[2], h[3]);
            if (phase_of(s.misc) != PH_OVER) {
              play_turn_h<1, PlayDraw, true>(s, draw, h[4], h[5], h[6], h[7]);
              done = 8;
            }
          } else {
            play_turn_h<0>(s, draw, h[0], h[1], h[2], h[3]);
            if (phase_of(s.misc) != PH_OVER) {
              play_turn_h<1>(s, draw, h[4], h[5], h[6], h[7]);
              done = 8;
            }
          }
          g_ply += done;
          steps += done;
          i += done - 1;
          if (phase_of(s.misc) == PH_OVER) games++;
          continue;
        }
      }
      int a;
      HZ_ACC(8, t0);
      if constexpr (Record) {
        uint64_t mk[3];
        int L = legal_mask(s, mk);
        HZ_ACC(9, t0);
        if (traj_state) {
          uint64_t *o = traj_state + (size_t)i * 6 * n + b;
          o[0] = s.pl[0]; o[(size_t)n] = s.pl[1]; o[(size_t)2 * n] = s.pl[2]; o[(size_t)3 * n] = s.pl[3];
          o[(size_t)4 * n] = s.piles; o[(size_t)5 * n] = s.misc;
        }
        if (traj_mask) {
          uint64_t *o = traj_mask + ((size_t)i * n + b) * 3;
          o[0] = mk[0]; o[1] = mk[1]; o[2] = mk[2];
        }
        a = L ? kth_action(mk, rule_pick_k(rkey, g_ply, L)) : -1;
        if (traj_action) traj_action[(size_t)i * n + b] = (int16_t)a;
      } else {
        a = rule_action(s, rule_h32(rkey, g_ply));  // legal mask + rule pick, fused
        HZ_ACC(9, t0);
      }
      if (a < 0) break;  // stuck board (unreachable from HarmoniesGameState())
      HZ_ACC(10, t0);
      bool te = phase_of(s.misc) == PH_P3;
      step_trusted<true>(s, a, draw);
      if (te) HZ_ACC(12, t0);
      else HZ_ACC(11, t0);
      g_ply++;
      steps++;
      if (phase_of(s.misc) == PH_OVER) games++;
    }
#ifdef HZ_DIAG_ROLES_ONLY
    HZ_PHASE(9, role_t0, b);
#endif
    // final scoring of the games that ended in this call, the whole wave at once
    if (score_pending(s.misc)) finish_game(s);
#ifdef HZ_DIAG_ROLES_ONLY
    HZ_PHASE(10, role_t0, b);
#endif
    HZ_ACC(13, t0);
    store_state(st, n, b, s);
    if (lds_used) pos[b] = draw.m.cursor();
    else if (draw.fell) pos[b] = draw.gm.cursor();
    else pos[b] = ahead_cur[(size_t)draw.d * n + b];
    mt_src[b] = lds_used ? -1 : src_slot;
    ply[b] = g_ply;
    seed[b] = sd;
#if defined(HZ_DIAG) && !defined(HZ_DIAG_ROLES_ONLY)
    if (g_stamps) {
      uint64_t *o = g_stamps + (size_t)b * 16;
      o[8] = acc8; o[9] = acc9; o[10] = acc10; o[11] = acc11; o[12] = acc12; o[13] = acc13;
    }
#endif
    if (games_done) games_done[b] = games;
    if (steps_done) steps_done[b] = steps;
    if (ep_final) ep_final[b] = episode[b];
    uint64_t lm = __ballot(lds_used);
    if (lane == 0) s_lds_mask = lm;
  }
  if (w0 && !act && lane == 0 && actmask == 0) s_lds_mask = 0;
  __syncthreads();
  uint64_t lds_mask = s_lds_mask & actmask;
  if (lds_mask) stage_mt(g, nb, tid, lds_mask, false);
#ifdef HZ_DIAG
  if (g_stamps && threadIdx.x < 64 && act) g_stamps[(size_t)b * 16 + 5] = __builtin_amdgcn_s_memtime() - role_t0;
#endif
}

// ============================================================= pipeline 2
// hz_play's second pipeline (hz_env_set_pipeline(e, 2)).  Each of
// k_rollout's roles runs one serial per-board chain of ~60 k cycles (a whole
// game, a whole seeding, 16 pile draws), and a launch lasts as long as its
// longest chain.  Here every board's episode is cut into thirteen stages,
// one per consecutive hz_play call, and one launch runs all thirteen at
// once, each on a different episode of the board (ep = the episode counter
// the previous call left, p2_ep; stage s works on episode ep + 12 - s):
//   s = 0  P1     seeding pass 1, steps 1-624          seed blocks, wave 3
//   s = 1  P2x    pass 2, steps 2-312                  seed blocks, wave 0
//   s = 2  P2y    pass 2, steps 313-624; rows 0-223    seed blocks, wave 1
//                 of the next generation twisted       (twist: wave 2)
//   s = 3  D1     pile draws 0-4                       draw-X blocks, wave 0
//   s = 4  D2     draws 5-9                            draw-X blocks, wave 1
//   s = 5  D3     draws 10-14                          draw-X blocks, wave 2
//   s = 6  D4     draws 15-19                          draw-Y blocks, wave 0
//   s = 7  D5     draws 20-23                          draw-Y blocks, wave 1
//          (the episode's rule hashes meanwhile:       draw-X blocks, wave 3)
//   s = 8  play0  plies [0, cut0)                      draw-Y blocks, wave 2
//   s = 9  play1  plies [cut0, cut1)                   play blocks, wave 3
//   s = 10 play2  plies [cut1, cut2)                   play blocks, wave 2
//   s = 11 play3  plies [cut2, cut3)                   play blocks, wave 1
//   s = 12 play4  the rest, final scoring, the board's play blocks, wave 0
//                 state, cursor and counters
// The stream slots are quad-interleaved (row r of board b at
// slot[(r >> 2) * 4 * nrow + 4 * b + (r & 3)]): a lane's four consecutive
// words are one 16-B access and a wave's 64 boards' quads are 1 KB
// contiguous, so the seeding chains store one 16-B word per four steps
// (a chain step with a b32 LDS read and a b32 store cost ~56 cycles, with
// 16-B operations per four steps ~29: tools/alu_chain.py), which lets pass
// 1 run as one stage and pass 2 as two, and frees the waves for a fifth draw
// stage and a fifth play stage.
// An episode's stream lives in one slot of a ring of kP2Stream from P1 to
// play4 (and afterwards as the board's current stream until materialize or
// the next call); stage s of call c uses slot (c - s) mod kP2Stream.  A stage
// uses an input only when its tag names the stage's episode, so a wrong
// prediction costs time, never results: the stages skip the board and play4
// plays its whole game from scratch (seeding and drawing in LDS, like
// k_rollout's unprepared boards).  The results are k_rollout's: the board ends
// the call with episode ep's final state, cursor and counters, and
// games_done / steps_done count that game (its first plies ran in the four
// calls before, in play0 .. play3).  In steady state a call does every stage
// once per board: one game's worth of work per board per call.
constexpr int kP2Win = 96;        // rows a draw stage stages, from its wave's lowest cursor
constexpr int kP2WinRows = kP2Win + 24;  // LDS rows per window (a scan reads up to 23 rows past its cursor)
constexpr int kP2Draw = 5;        // draw stages
constexpr int kP2Play = 5;        // play stages
constexpr int kP2FirstDraw = 3;   // stage of D1
constexpr int kP2FirstPlay = kP2FirstDraw + kP2Draw;  // stage of play0
constexpr int kP2Stages = kP2FirstPlay + kP2Play;     // 13
constexpr int kP2Last = kP2Stages - 1;  // stage s works on episode ep + kP2Last - s
constexpr int kP2Ring = kP2Play + 1;    // D5's scripts and the rule hashes: read by the play stages 1..kP2Play calls later
constexpr int kP2Stream = kP2Stages + 1;  // stream slots (the last play stage's slot stays the board's stream)
constexpr int kP2MinPlies = 96;   // hz_play max_plies from which pipeline 2 applies (rule games end by ply 80)
constexpr int kP2xEnd = 313;      // P2x: pass-2 steps [2, 313), P2y [313, 624) and the last one, at i = 1
constexpr int kP2Quads = kMT / 4; // 156 quads per stream
constexpr int kP2LdsY = 79;       // P2y's LDS quads start here (P2x's: 0-78, pass-1 rows 0-315)
__device__ __forceinline__ constexpr int p2_draw_cut(int d) { return d >= kP2Draw ? kAheadDraws : 5 * d; }
#ifdef HZ_DIAG
constexpr int kP2Stamps = 48;  // stamp slots per board in k_play2 (tools/p2_roles.py)
#define P2_PHASE(slot, t0)                                                                                       \
  do {                                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                                           \
    if (g_stamps && b < a.n) g_stamps[(size_t)b * kP2Stamps + (slot)] = __builtin_amdgcn_s_memtime() - (t0); \
    __builtin_amdgcn_sched_barrier(0);                                                                           \
  } while (0)
#else
#define P2_PHASE(slot, t0) \
  do {                     \
  } while (0)
#endif
static_assert(p2_draw_cut(kP2Draw - 1) < kAheadDraws && p2_draw_cut(kP2Draw) == kAheadDraws, "draw stages cover the script");
static_assert(3 * kP2WinRows * kLdsStride * 4 <= (int)kResetLds, "three windows per draw block");
static_assert((kP2LdsY + kP2Quads - 78) * 64 * 16 <= (int)kResetLds, "P2x's and P2y's LDS quads fit");
static_assert(kMT % 4 == 0, "whole quads");

struct P2Args {
  uint64_t *st;
  uint32_t *mt;
  int32_t *pos, *ply, *episode;
  uint64_t *seed;
  int n, max_plies, draws;
  int cut[kP2Play - 1];
  uint64_t seed_base;
  long nrow;
  int32_t *games_done, *steps_done, *mt_src;
  const int32_t *ep_in;
  int32_t *ep_out;
  uint32_t *s_mt[kP2Stages];  // the stream slot of each stage this call (quad-interleaved)
  int32_t *s_tag[kP2Stages];  // [nrow] episode * 8 + 2 pass 1 / 3 P2x / 5 seeded, rows 0-223 twisted
  int32_t *s_cur[kP2Stages];  // [kAheadDraws + 1][nrow] cursor before draw 0 and after each draw
  int s_idx_last;             // the last play stage's slot index (materialize: mt_src = 2 + index)
  uint32_t *ph_w;             // [3][nrow] P2x -> P2y: pass 2's last value, pass 1's row-1 word, row 2's final word
  const uint32_t *ph_r;
  P2Draw x_w[kP2Draw - 1], x_r[kP2Draw - 1];  // D1 -> D2 -> .. -> D5 (tag: episode * 8 + stages done)
  P2Draw pl_w, pl_r[kP2Play];     // D5's script: written this call; read by play stage st (st + 1 calls later)
  P2Mid m_w[kP2Play - 1], m_r[kP2Play - 1];  // play stage st -> st + 1 (written / read this call)
  uint32_t *h_w;                  // [kRulePlies][nrow] rule hashes
  const uint32_t *h_r[kP2Play];
  int32_t *ht_w;                  // [nrow] their episode
  const int32_t *ht_r[kP2Play];
  int32_t *err;                   // the env's wait-error word
  int spin;                       // spin bound of the twist wave's waits
};

// PlayDraw for the prepared stages: the pile script in registers, then (a
// script shorter than the game needs) the episode's stream slot in HBM
struct PlayDraw2 {
  uint64_t q0, q1, q2, q3;
  int d, nd;
  bool fell;
  MTQ gm;                  // valid once fell
  const int32_t *cur_nd;   // the slot's cursor after the last scripted draw (read when the script runs out)
  __device__ __forceinline__ uint32_t pop() {
    uint32_t p9 = (uint32_t)q0 & 0x1FFu;
    q0 = (q0 >> 9) | (q1 << 55);
    q1 = (q1 >> 9) | (q2 << 55);
    q2 = (q2 >> 9) | (q3 << 55);
    q3 >>= 9;
    d++;
    return p9;
  }
  __device__ __forceinline__ bool pair_pops() const { return d + 2 <= nd; }
  __device__ __forceinline__ uint32_t draw_one(uint64_t misc) {
    if (d < nd) return pop();
    if (!fell) {
      gm = MTQ(gm.w, gm.s4, *cur_nd);
      fell = true;
    }
    uint32_t p9;
    return draw_pile(misc, gm, p9) ? p9 : 0x1FFu;
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t misc) { return take(misc, true); }
  __device__ __forceinline__ uint32_t take(uint64_t misc, bool want) {
    if (__all(!want || d < nd)) {
      uint32_t p9 = want ? (uint32_t)q0 & 0x1FFu : 0x1FFu;
      uint64_t n0 = (q0 >> 9) | (q1 << 55), n1 = (q1 >> 9) | (q2 << 55), n2 = (q2 >> 9) | (q3 << 55);
      q0 = want ? n0 : q0;
      q1 = want ? n1 : q1;
      q2 = want ? n2 : q2;
      q3 = want ? q3 >> 9 : q3;
      d += want ? 1 : 0;
      return p9;
    }
    return want ? draw_one(misc) : 0x1FFu;
  }
  __device__ __forceinline__ void scripted_reset(State &s) {  // >= 5 entries: the opening piles
    s.pl[0] = s.pl[1] = s.pl[2] = s.pl[3] = 0;
    uint64_t open = q0 & ((1ull << 45) - 1);
    s.piles = open | (5ull << 45);
    uint64_t misc = 0x1FF;
#pragma unroll
    for (int t = 0; t < 6; t++) misc = set_bits(misc, 11 + 5 * t, 5, (uint64_t)initial_count(t));
#pragma unroll
    for (int i = 0; i < 5; i++) apply_pile_fast(misc, (uint32_t)(open >> (9 * i)) & 0x1FFu);
    s.misc = misc;
    q0 = (q0 >> 45) | (q1 << 19);
    q1 = (q1 >> 45) | (q2 << 19);
    q2 = (q2 >> 45) | (q3 << 19);
    q3 >>= 45;
    d = 5;
  }
};

// the rule policy's plies [g, g_end) of one board (k_rollout's ply loop, no
// reset, no recording): turn pairs while the wave allows, single plies
// otherwise; hashes from a pipeline slot when `hs` (row stride nr) holds the
// episode's, else computed.  Returns the plies played.
template <class Draw>
__device__ __forceinline__ int p2_plies(State &s, Draw &draw, int g, int g_end, uint64_t rkey, const uint32_t *hs,
                                        size_t nr) {
  const int g0 = g;
  auto hash = [&](int ply) -> uint32_t { return hs && ply < kRulePlies ? hs[(size_t)ply * nr] : rule_h32(rkey, ply); };
  // the next turn pair's hashes, read one pair ahead (a slot's are in HBM).
  // Wave-uniform choices: a per-lane select would evaluate both sides, i.e.
  // compute all eight hashes and issue their loads every pair.
  const bool all_hs = __all(hs != nullptr);
  uint32_t hn[8];
  int hn_g = -1;  // (wave-uniform)
  while (g < g_end) {
    if (phase_of(s.misc) == PH_OVER) break;
    if (__all(g + 8 <= g_end && turn_pair_safe(s))) {
      uint32_t h[8];
      if (__all(hn_g == g)) {
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = hn[j];
      } else if (all_hs && __all(g + 8 <= kRulePlies)) {
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = hs[(size_t)(g + j) * nr];
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = hash(g + j);
      }
      if (all_hs && __all(g + 16 <= g_end && g + 16 <= kRulePlies)) {
#pragma unroll
        for (int j = 0; j < 8; j++) hn[j] = hs[(size_t)(g + 8 + j) * nr];
        hn_g = __builtin_amdgcn_readfirstlane(g + 8);
      }
      int done = 4;
      if (__all(draw.pair_pops())) {
        play_turn_h<0, Draw, true>(s, draw, h[0], h[1], h[2], h[3]);
        if (phase_of(s.misc) != PH_OVER) {
          play_turn_h<1, Draw, true>(s, draw, h[4], h[5], h[6], h[7]);
          done = 8;
        }
      } else {
        play_turn_h<0>(s, draw, h[0], h[1], h[2], h[3]);
        if (phase_of(s.misc) != PH_OVER) {
          play_turn_h<1>(s, draw, h[4], h[5], h[6], h[7]);
          done = 8;
        }
      }
      g += done;
      continue;
    }
    const int a = rule_action(s, hash(g));
    if (a < 0) break;  // stuck board (unreachable from HarmoniesGameState())
    step_trusted<true>(s, a, draw);
    g++;
  }
  return g - g0;
}

__device__ __forceinline__ int p2_wait(int *flag, int need, int limit, int32_t *err) {
  int v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
  // every publisher reaches kMT + 1 (or kMT rows); the bound only guards
  // against a hang should that ever change, and giving up is reported (the
  // caller goes on with rows that may not be final: the host raises)
  for (int spin = 0; v < need && spin < limit; spin++) {
    __builtin_amdgcn_s_sleep(1);
    v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (v < need) {
    wait_failed(err, kWaitErrP2Twist);
    v = kMT + 1;  // no further waits this launch
  }
  return v;
}
__device__ __forceinline__ void p2_publish(int *flag, int v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// ---- quad-interleaved stream slots
typedef uint32_t p2u4 __attribute__((ext_vector_type(4)));
typedef uint32_t p2u3 __attribute__((ext_vector_type(3)));
typedef uint32_t p2u2 __attribute__((ext_vector_type(2)));
// the slot's quads of boards [b0, b0 + 64) as a buffer: lane l's quad of
// rows [4 q, 4 q + 4) at voffset 16 l, soffset q * 16 nrow (a scalar: no
// 64-bit address arithmetic in the chains)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t p2_rsrc(uint32_t *slot, int b0, size_t nr) {
  const uint64_t base = (uint64_t)(slot + 4 * (size_t)b0);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)((size_t)kP2Quads * 16 * nr - (size_t)b0 * 16));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}
__device__ __forceinline__ void p2_st4(__amdgpu_buffer_rsrc_t rs, int lane, int soff, uint32_t x, uint32_t y,
                                       uint32_t z, uint32_t w) {
  const p2u4 v = {x, y, z, w};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, lane * 16, __builtin_amdgcn_readfirstlane(soff), 0);
}
__device__ __forceinline__ uint4 p2_ld4(__amdgpu_buffer_rsrc_t rs, int lane, int soff) {
  const p2u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, __builtin_amdgcn_readfirstlane(soff), 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// a lane's LDS quad k (the seed blocks stage pass-1 words in the slot's own
// quad layout: 1 KB per quad row of the wave's 64 boards, 16-B accesses)
__device__ __forceinline__ uint4 &p2_lq(int k, int lane) { return reinterpret_cast<uint4 *>(hz_lds)[k * 64 + lane]; }

__device__ __forceinline__ void p2_keys(uint64_t seed, uint32_t &kA, uint32_t &kB) {
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  kA = key0;
  kB = key1 ? key1 + 1u : key0;
}

// P1 (seed blocks, wave 3): init_by_array's pass 1 (random.seed(int) ->
// init_by_array(key), key = the seed's 32-bit words) in one chain: steps
// 1-623 (odd steps key word kA, even ones kB), then the 624th at i = 1 (its
// mt[0] = mt[623] is the chain's last value); one 16-B store per four
// steps.  Row 0 is never read by pass 2.  No LDS.
__device__ __forceinline__ void p2_p1(const P2Args &a, int b0, int lane) {
  const int b = b0 + lane;
  const size_t nr = (size_t)a.nrow;
  const int e = a.ep_in[b] + kP2Last;
  uint32_t kA, kB;
  p2_keys(episode_seed(a.seed_base, b, e), kA, kB);
  const __amdgpu_buffer_rsrc_t rs = p2_rsrc(a.s_mt[0], b0, nr);
  const int qb = (int)(nr * 16);
  uint32_t prev = 19650218u;
  auto step = [&](uint32_t iv, uint32_t k) {
    const uint32_t v = (iv ^ ((prev ^ (prev >> 30)) * 1664525U)) + k;
    prev = v;
    return v;
  };
  const uint32_t w1 = step(kInitGen.v[1], kA), w2 = step(kInitGen.v[2], kB), w3 = step(kInitGen.v[3], kA);
  // init_genrand's table words a group ahead (scalar loads: their wait would
  // otherwise sit in the chain once per group)
  uint32_t iv[8];
#pragma unroll
  for (int u = 0; u < 8; u++) iv[u] = kInitGen.v[4 + u];
#pragma unroll 1
  for (int g = 4; g < 620; g += 8) {  // rows 4-619: two quads per group
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = kInitGen.v[g + 8 + u < kMT ? g + 8 + u : kMT - 1];
    const uint32_t v0 = step(iv[0], kB), v1 = step(iv[1], kA), v2 = step(iv[2], kB), v3 = step(iv[3], kA);
    p2_st4(rs, lane, (g >> 2) * qb, v0, v1, v2, v3);
    const uint32_t v4 = step(iv[4], kB), v5 = step(iv[5], kA), v6 = step(iv[6], kB), v7 = step(iv[7], kA);
    p2_st4(rs, lane, ((g >> 2) + 1) * qb, v4, v5, v6, v7);
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = nx[u];
  }
  {  // rows 620-623 (iv: table words 620-623)
    const uint32_t v0 = step(iv[0], kB), v1 = step(iv[1], kA), v2 = step(iv[2], kB), v3 = step(iv[3], kA);
    p2_st4(rs, lane, (kP2Quads - 1) * qb, v0, v1, v2, v3);
  }
  // the 624th step at i = 1 (key j = 623 % keylen -> kB), prev = mt[623] = mt[0]
  const uint32_t r1 = (w1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB;
  p2_st4(rs, lane, 0, 0u, r1, w2, w3);
  a.s_tag[0][b] = e * 8 + 2;
}

// Pass 2 in two stages, P2x (steps 2-312) and P2y (313-623 and the last
// step, at i = 1), in one seed block on disjoint LDS quads (the pass-1 words
// of two different episodes).  Every step reads the next pass-1 word, too
// close ahead for an HBM round trip, so each chain first stages its half of
// the pass-1 words into LDS (16-B loads and LDS writes, all of a piece in
// flight at once, the slot's own quad layout), then runs on 16-B LDS reads
// two quads ahead and stores one 16-B word per four steps.  The stage's rows
// come in three pieces, each next piece's loads issued before the chain runs
// over the piece before it: two thirds of the staging reads leave the
// launch's opening burst.  Rows 2-223 of the slot are read only by the
// twist, which needs from each row r only its twist part (rows r and r + 1's
// words): P2x stores that instead of the final word (one step late), so the
// twist is one xor per word with the far row.  P2x hands (prev, pass 1's
// row-1 word, row 2's final word) to P2y, which keeps its final words in LDS
// for the twist and writes rows 0 and 1 of the next generation.
// twist_word(cur, next, far) = far ^ twist_part(cur, next)
__device__ __forceinline__ uint32_t twist_part(uint32_t cur, uint32_t next) {
  const uint32_t y = (cur & 0x80000000U) | (next & 0x7fffffffU);
  return (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
}
__device__ __forceinline__ uint32_t p2_step(uint32_t p1, uint32_t &prev, int i) {
  const uint32_t v = (p1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)i;
  prev = v;
  return v;
}
// HBM quads [Q0, Q1) of the lane's board -> LDS quads from Q0 + D
template <int Q0, int Q1>
struct P2QPiece {
  uint4 v[Q1 - Q0];
};
template <int Q0, int Q1>
__device__ __forceinline__ void p2_qload(P2QPiece<Q0, Q1> &pc, __amdgpu_buffer_rsrc_t rs, int lane, int qb) {
#pragma unroll
  for (int u = 0; u < Q1 - Q0; u++) pc.v[u] = p2_ld4(rs, lane, (Q0 + u) * qb);
}
template <int D, int Q0, int Q1>
__device__ __forceinline__ void p2_qput(const P2QPiece<Q0, Q1> &pc, int lane) {
#pragma unroll
  for (int u = 0; u < Q1 - Q0; u++) p2_lq(Q0 + u + D, lane) = pc.v[u];
  // (a wave's LDS operations execute in order: its later reads see these)
}
// groups k in [K0, K1) of four steps 4k .. 4k + 3 on LDS quads k + D, reads
// two quads ahead.  Part: step 4k completes row 4k - 1's part (quad k - 1
// stored), steps 4k + 1 .. 4k + 3 give rows 4k .. 4k + 2 (acc.x-z).  Final:
// quad k's final words stored; Keep also writes them over the pass-1 quad
// in LDS and publishes progress every two groups.
enum { kP2Part = 0, kP2Final = 1, kP2Keep = 2 };
template <int K0, int K1, int D, int Mode>
__device__ __forceinline__ void p2_groups(int lane, __amdgpu_buffer_rsrc_t rs, int qb, uint32_t &prev, uint4 &acc,
                                          int *prog) {
  static_assert(Mode != kP2Keep || (K1 - K0) % 2 == 0, "Keep: pairs of groups");
  uint4 p0 = p2_lq(K0 + D, lane), p1 = p2_lq((K0 + 1 < K1 ? K0 + 1 : K1 - 1) + D, lane);
#pragma unroll 2
  for (int k = K0; k < K1; k++) {
    const uint4 p2 = p2_lq((k + 2 < K1 ? k + 2 : K1 - 1) + D, lane);
    const int i = 4 * k;
    if constexpr (Mode == kP2Part) {
      const uint32_t c = prev;
      const uint32_t v0 = p2_step(p0.x, prev, i);
      acc.w = twist_part(c, v0);
      p2_st4(rs, lane, (k - 1) * qb, acc.x, acc.y, acc.z, acc.w);
      const uint32_t v1 = p2_step(p0.y, prev, i + 1);
      acc.x = twist_part(v0, v1);
      const uint32_t v2 = p2_step(p0.z, prev, i + 2);
      acc.y = twist_part(v1, v2);
      const uint32_t v3 = p2_step(p0.w, prev, i + 3);
      acc.z = twist_part(v2, v3);
    } else {
      const uint32_t v0 = p2_step(p0.x, prev, i), v1 = p2_step(p0.y, prev, i + 1);
      const uint32_t v2 = p2_step(p0.z, prev, i + 2), v3 = p2_step(p0.w, prev, i + 3);
      p2_st4(rs, lane, k * qb, v0, v1, v2, v3);
      if constexpr (Mode == kP2Keep) {
        p2_lq(k + D, lane) = make_uint4(v0, v1, v2, v3);
        if ((k - K0) & 1) p2_publish(prog, 4 * k + 4);  // rows below final in LDS
      }
    }
    p0 = p1;
    p1 = p2;
  }
}

// P2x (seed blocks, wave 0): the episode whose pass 1 completed in the
// previous call; pass-1 quads 0-78 (rows 0-315) on LDS quads 0-78.
__device__ __forceinline__ void p2_x(const P2Args &a, int b0, int lane, int e, bool ok) {
  if (!__any(ok)) return;
  const int b = b0 + lane;
  const size_t nr = (size_t)a.nrow;
  const __amdgpu_buffer_rsrc_t rs = p2_rsrc(a.s_mt[1], b0, nr);
  const int qb = (int)(nr * 16);
#ifdef HZ_DIAG
  const uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
  {
    P2QPiece<0, 27> pc;
    p2_qload(pc, rs, lane, qb);
    p2_qput<0>(pc, lane);
  }
  P2QPiece<27, 53> pc1;
  p2_qload(pc1, rs, lane, qb);
  P2_PHASE(32, tq);
  // steps 2, 3 (rows 0 and 1 of the slot are P2y's: quad 0 gets rows 2, 3)
  const uint4 q0 = p2_lq(0, lane);
  const uint32_t first1 = q0.y;
  uint32_t prev = first1;
  const uint32_t row2 = p2_step(q0.z, prev, 2);
  const uint32_t v3 = p2_step(q0.w, prev, 3);
  uint4 acc = make_uint4(0u, 0u, twist_part(row2, v3), 0u);
  {  // group 1: row 3's part completes quad 0 (rows 2, 3 only)
    const uint4 p = p2_lq(1, lane);
    const uint32_t v4 = p2_step(p.x, prev, 4);
    const p2u2 h = {acc.z, twist_part(v3, v4)};
    __builtin_amdgcn_raw_buffer_store_b64(h, rs, lane * 16 + 8, 0, 0);
    const uint32_t v5 = p2_step(p.y, prev, 5);
    acc.x = twist_part(v4, v5);
    const uint32_t v6 = p2_step(p.z, prev, 6);
    acc.y = twist_part(v5, v6);
    const uint32_t v7 = p2_step(p.w, prev, 7);
    acc.z = twist_part(v6, v7);
  }
  p2_groups<2, 27, 0, kP2Part>(lane, rs, qb, prev, acc, nullptr);  // parts of rows .. 107
  p2_qput<0>(pc1, lane);
  P2QPiece<53, 79> pc2;
  p2_qload(pc2, rs, lane, qb);
  p2_groups<27, 53, 0, kP2Part>(lane, rs, qb, prev, acc, nullptr);  // .. 211
  p2_qput<0>(pc2, lane);
  p2_groups<53, 56, 0, kP2Part>(lane, rs, qb, prev, acc, nullptr);  // .. 223 (acc: rows 220-222)
  {  // group 56: row 223's part completes quad 55; row 224 on is final
    const uint4 p = p2_lq(56, lane);
    const uint32_t c = prev;
    const uint32_t v0 = p2_step(p.x, prev, 224);
    p2_st4(rs, lane, 55 * qb, acc.x, acc.y, acc.z, twist_part(c, v0));
    const uint32_t v1 = p2_step(p.y, prev, 225), v2 = p2_step(p.z, prev, 226), v3b = p2_step(p.w, prev, 227);
    p2_st4(rs, lane, 56 * qb, v0, v1, v2, v3b);
  }
  p2_groups<57, 78, 0, kP2Final>(lane, rs, qb, prev, acc, nullptr);  // rows 228-311
  {  // step 312: row 312 (rows 313-315 of quad 78 are P2y's)
    const uint32_t v = p2_step(p2_lq(78, lane).x, prev, 312);
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 16, __builtin_amdgcn_readfirstlane(78 * qb), 0);
  }
  if (ok) {
    a.ph_w[b] = prev;
    a.ph_w[nr + b] = first1;
    a.ph_w[2 * nr + b] = row2;
    a.s_tag[1][b] = e * 8 + 3;
  }
}

// P2y (seed blocks, wave 1): pass-1 quads 78-155 on LDS quads 79-156; final
// words kept in LDS (the twist reads rows 397-620), progress in *prog
constexpr int kP2YD = kP2LdsY - 78;
__device__ __forceinline__ void p2_y(const P2Args &a, int b0, int lane, int e, bool ok, int *prog) {
  if (!__any(ok)) {
    p2_publish(prog, kMT + 1);  // (the twist wave's waits end: nothing to twist)
    return;
  }
  const int b = b0 + lane;
  const bool act = b < a.n;
  const size_t nr = (size_t)a.nrow;
  const __amdgpu_buffer_rsrc_t rs = p2_rsrc(a.s_mt[2], b0, nr);
  const int qb = (int)(nr * 16);
#ifdef HZ_DIAG
  const uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
  {
    P2QPiece<78, 104> pc;
    p2_qload(pc, rs, lane, qb);
    p2_qput<kP2YD>(pc, lane);
  }
  P2QPiece<104, 130> pc1;
  p2_qload(pc1, rs, lane, qb);
  P2_PHASE(33, tq);
  uint32_t prev = act ? a.ph_r[b] : 0u;
  const uint32_t first1 = act ? a.ph_r[nr + b] : 0u, row2 = act ? a.ph_r[2 * nr + b] : 0u;
  uint4 acc = make_uint4(0u, 0u, 0u, 0u);
  {  // steps 313-315 (row 312 of quad 78 is P2x's)
    const uint4 p = p2_lq(78 + kP2YD, lane);
    const p2u3 v = {p2_step(p.y, prev, 313), p2_step(p.z, prev, 314), p2_step(p.w, prev, 315)};
    __builtin_amdgcn_raw_buffer_store_b96(v, rs, lane * 16 + 4, __builtin_amdgcn_readfirstlane(78 * qb), 0);
  }
  p2_groups<79, 103, kP2YD, kP2Keep>(lane, rs, qb, prev, acc, prog);  // rows 316-411 (an even count of groups)
  p2_qput<kP2YD>(pc1, lane);
  P2QPiece<130, 156> pc2;
  p2_qload(pc2, rs, lane, qb);
  p2_groups<103, 129, kP2YD, kP2Keep>(lane, rs, qb, prev, acc, prog);  // .. 515
  p2_qput<kP2YD>(pc2, lane);
  p2_groups<129, 155, kP2YD, kP2Keep>(lane, rs, qb, prev, acc, prog);  // .. 619
  {  // rows 620-623
    const uint4 p = p2_lq(155 + kP2YD, lane);
    const uint32_t v0 = p2_step(p.x, prev, 620), v1 = p2_step(p.y, prev, 621);
    const uint32_t v2 = p2_step(p.z, prev, 622), v3 = p2_step(p.w, prev, 623);
    p2_st4(rs, lane, 155 * qb, v0, v1, v2, v3);
    p2_lq(155 + kP2YD, lane) = make_uint4(v0, v1, v2, v3);
  }
  p2_publish(prog, kMT);
  // the last step, at i = 1 (mt[0] = mt[623] = prev); then mt[0] =
  // 0x80000000 and rows 0, 1 of the next generation: row 1's next row is
  // row 2, the far rows are 397, 398 (this chain's)
  const uint32_t row1 = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
  const uint4 f = p2_lq(99 + kP2YD, lane);  // rows 396-399
  const p2u2 h = {f.y ^ twist_part(0x80000000u, row1), f.z ^ twist_part(row1, row2)};
  __builtin_amdgcn_raw_buffer_store_b64(h, rs, lane * 16, 0, 0);
  if (ok) a.s_tag[2][b] = e * 8 + 5;
}

// The twist (seed blocks, wave 2): rows [0, kAheadTwist) of the next
// generation into P2y's slot (the stream at cursor kMTAhead): row r's new
// word is the far row r + 397 (P2y's, from LDS) xor row r's twist part,
// which P2x left in the slot (rows 2-223).  Lane = board, quad q = rows 4 q
// .. 4 q + 3, whose far rows are the slot's quads q + 99 (rows 4 q + 397 ..
// 399) and q + 100 (row 4 q + 400), in LDS once P2y has published past them; rows
// 0 and 1 (from row 1, P2y's last step, and row 2's final word) are P2y's.
// All its loads precede its stores.
constexpr int kTwQuads = kAheadTwist / 4;  // 56
__device__ __forceinline__ uint4 xor4(const uint4 &a, const uint4 &b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ void p2_twist(const P2Args &a, int b0, int lane, bool any, int *s_prog) {
  if (!any) return;
  const size_t nr = (size_t)a.nrow;
  const __amdgpu_buffer_rsrc_t rs = p2_rsrc(a.s_mt[2], b0, nr);
  const int qb = (int)(nr * 16);
#ifdef HZ_DIAG
  const int b = b0 + lane;
  const uint64_t tz = __builtin_amdgcn_s_memtime();
#endif
  // (the wave has slack: its loads wait until P2y is 64 rows in, out of the
  // launch's opening burst, where every other stage's inputs arrive)
  int have = p2_wait(s_prog, kP2xEnd + 64, a.spin, a.err);
  P2_PHASE(35, tz);
  uint4 pt[kTwQuads];
#pragma unroll
  for (int q = 0; q < kTwQuads; q++) pt[q] = p2_ld4(rs, lane, q * qb);
  uint4 A = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int q = 0; q < kTwQuads; q += 2) {
    const int need = 4 * (q + 1) + 401;  // the pair's far rows final (below need)
    if (have < need) have = p2_wait(s_prog, need, a.spin, a.err);
    if (q == 0) A = p2_lq(99 + kP2YD, lane);
    const uint4 B = p2_lq(q + 100 + kP2YD, lane), C = p2_lq(q + 101 + kP2YD, lane);
    const uint4 o0 = xor4(make_uint4(A.y, A.z, A.w, B.x), pt[q]);
    const uint4 o1 = xor4(make_uint4(B.y, B.z, B.w, C.x), pt[q + 1]);
    if (q == 0) {
      const p2u2 h = {o0.z, o0.w};
      __builtin_amdgcn_raw_buffer_store_b64(h, rs, lane * 16 + 8, 0, 0);
    } else {
      p2_st4(rs, lane, q * qb, o0.x, o0.y, o0.z, o0.w);
    }
    p2_st4(rs, lane, (q + 1) * qb, o1.x, o1.y, o1.z, o1.w);
    if (q == 0) P2_PHASE(36, tz);
    A = C;
  }
  P2_PHASE(37, tz);
  // (rows 224..623 keep pass 2's words: the current generation's tail)
}

// seed blocks: wave 0 P2x, wave 1 P2y, wave 2 the twist of P2y's episode,
// wave 3 P1
__device__ __forceinline__ void p2_seed(const P2Args &a, int blk) {
  __shared__ int s_prog;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock, b = b0 + lane;
  const bool act = b < a.n;
  if (tid == 0) s_prog = 0;
  // each pass-2 stage's episode and decision (and P2y's for the twist
  // wave), read before the barrier, so before any wave rewrites a tag
  const int k = w == 0 ? 1 : 2;
  const int e = act ? a.ep_in[b] + kP2Last - k : 0;
  const bool ok = act && a.s_tag[k][b] == e * 8 + (k == 1 ? 2 : 3);
  __syncthreads();
  if (w == 0) p2_x(a, b0, lane, e, ok);
  else if (w == 1) p2_y(a, b0, lane, e, ok, &s_prog);
  else if (w == 2) p2_twist(a, b0, lane, __any(ok), &s_prog);
  else if (act) p2_p1(a, b0, lane);
}

// a draw stage d (stage kP2FirstDraw + d): draws [d0, d1) of its episode on
// its stream slot, from an LDS window (at `base`) of kP2Win rows starting at
// the wave's lowest start cursor (the wave's 64 boards' quads, staged
// here); `in` (d > 0) holds the draws so far, `out` gets them plus these;
// the cursors go to the slot's cursor table
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ void p2_draw_stage(const P2Args &a, int b0, int lane, int d, int base) {
  const int b = b0 + lane;
#ifdef HZ_DIAG
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  const bool act = b < a.n;
  const size_t nr = (size_t)a.nrow;
  const int s = kP2FirstDraw + d;
  const int d0 = p2_draw_cut(d), d1 = d == kP2Draw - 1 ? a.draws : min(a.draws, p2_draw_cut(d + 1));
  const int e = act ? a.ep_in[b] + kP2Last - s : 0;
  uint32_t *slot = a.s_mt[s];
  int32_t *cur = a.s_cur[s] + b;
  const P2Draw &in = a.x_r[d > 0 ? d - 1 : 0];
  const P2Draw &out = d == kP2Draw - 1 ? a.pl_w : a.x_w[d];
  bool ok = act && a.s_tag[s][b] == e * 8 + 5;
  int k0 = 0, c0 = kMTAhead;
  uint64_t bag = initial_bag(), q[kAheadWords] = {0, 0, 0, 0};
  if (d > 0 && act) {  // (one round trip: used only if the tag matches)
    const int itag = in.tag[b];
    k0 = in.k[b];
    c0 = in.c[b];
    bag = in.bag[b];
#pragma unroll
    for (int i = 0; i < kAheadWords; i++) q[i] = in.q[(size_t)i * nr + b];
    ok = ok && itag == e * 8 + d;
  }
  const bool draws = ok && k0 >= d0 && d0 < d1;
  const int r0 = wave_min_i(draws ? (c0 & 0xFFFF) : kAheadTwist) & ~3;
  if (r0 < kAheadTwist) {  // the window: rows [r0, r0 + kP2Win), each lane its board's quads, all in flight
    constexpr int U = kP2Win / 4;
    const __amdgpu_buffer_rsrc_t rs = p2_rsrc(slot, b0, nr);
    const int qb = (int)(nr * 16), q0 = r0 >> 2;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = p2_ld4(rs, lane, (q0 + u) * qb);
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t *dd = hz_lds + base + 4 * u * kLdsStride + lane;
      dd[0] = v[u].x;
      dd[kLdsStride] = v[u].y;
      dd[2 * kLdsStride] = v[u].z;
      dd[3 * kLdsStride] = v[u].w;
    }
  }
  P2_PHASE(27 + d, t0);  // window staged
  if (!act) return;
  if (!ok) {
    out.tag[b] = -1;
    return;
  }
  if (d == 0) cur[0] = kMTAhead;
  int k = k0, cc = c0;
  if (draws) {  // every earlier draw is done: continue in the window
    const int lim = min(r0 + kP2Win, kAheadTwist);
    StreamDraw<WinMT> dr{WinMT(base - r0 * kLdsStride + lane, c0, lim)};
#pragma unroll 1
    for (int i = d0; i < d1; i++) {
      if (dr.m.pos >= lim) break;
      const uint32_t p9 = dr(bag);
      // a draw that consumed words past the window is discarded: the next
      // stage (or a play stage, from the stream slot) redoes it from the
      // last cursor kept
      if (dr.m.pos > lim) break;
      apply_pile_fast(bag, p9);
      const int bit = 9 * i, wd = bit >> 6, off = bit & 63;
      const uint64_t lo9 = (uint64_t)p9 << off, hi9 = off > 55 ? (uint64_t)p9 >> (64 - off) : 0ull;
      q[0] |= wd == 0 ? lo9 : 0ull;
      q[1] |= wd == 1 ? lo9 : wd == 0 ? hi9 : 0ull;
      q[2] |= wd == 2 ? lo9 : wd == 1 ? hi9 : 0ull;
      q[3] |= wd == 3 ? lo9 : wd == 2 ? hi9 : 0ull;
      cc = dr.m.cursor();
      cur[(size_t)(i + 1) * nr] = cc;
      k = i + 1;
    }
  }
  out.k[b] = k;
  out.c[b] = cc;
  out.bag[b] = bag;
#pragma unroll
  for (int i = 0; i < kAheadWords; i++) out.q[(size_t)i * nr + b] = q[i];
  out.tag[b] = e * 8 + d + 1;
}

// the rule hashes of D5's episode (read by the play stages in the next
// kP2Play calls)
__device__ __forceinline__ void p2_hashes(const P2Args &a, int b) {
  const size_t nr = (size_t)a.nrow;
  const int e = a.ep_in[b] + kP2Last - (kP2FirstPlay - 1);
  const uint64_t rk = rule_key(episode_seed(a.seed_base, b, e));
#pragma unroll 1
  for (int j = 0; j < kRulePlies; j++) a.h_w[(size_t)j * nr + b] = rule_h32(rk, j);
  a.ht_w[b] = e;
}

// a play stage's state after its plies, for the next play stage
__device__ __forceinline__ void p2_mid_put(const P2Mid &m, size_t nr, int b, const State &s, const PlayDraw2 &d, int g,
                                           int e) {
#pragma unroll
  for (int k = 0; k < 4; k++) m.st[(size_t)k * nr + b] = s.pl[k];
  m.st[4 * nr + b] = s.piles;
  m.st[5 * nr + b] = s.misc;
  m.q[b] = d.q0;
  m.q[nr + b] = d.q1;
  m.q[2 * nr + b] = d.q2;
  m.q[3 * nr + b] = d.q3;
  m.i[b] = d.d;
  m.i[nr + b] = g;
  m.i[2 * nr + b] = d.fell ? d.gm.cursor() : -1;
  m.tag[b] = e;
}
// the previous play stage's state; the draw source continues its script
// (nd entries, cursors in `cur`) or the slot stream it fell onto (sw: the
// board's quads in the slot, quad stride s4)
__device__ __forceinline__ PlayDraw2 p2_mid_get(const P2Mid &m, size_t nr, int b, State &s, int &g, int nd,
                                               uint32_t *sw, int s4, const int32_t *cur) {
#pragma unroll
  for (int k = 0; k < 4; k++) s.pl[k] = m.st[(size_t)k * nr + b];
  s.piles = m.st[4 * nr + b];
  s.misc = m.st[5 * nr + b];
  const int d = m.i[b], fc = m.i[2 * nr + b];
  g = m.i[nr + b];
  return PlayDraw2{m.q[b], m.q[nr + b], m.q[2 * nr + b], m.q[3 * nr + b], d, nd, fc >= 0,
                   MTQ(sw, s4, fc >= 0 ? fc : 0), cur + (size_t)nd * nr};
}

// play stage st (stage kP2FirstPlay + st) of the lane's board: its plies of
// episode ep + kP2Play - 1 - st (the last stage: the rest of episode ep, or
// all of it); returns whether the board's stream ended in LDS (the last
// stage's unprepared fallback)
__device__ __forceinline__ bool p2_play_stage(const P2Args &a, int b0, int lane, int st) {
  const int b = b0 + lane;
  if (b >= a.n) return false;
  const size_t nr = (size_t)a.nrow;
#ifdef HZ_DIAG
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  const bool last = st == kP2Play - 1;
  const int s = kP2FirstPlay + st;
  const int e = last ? a.episode[b] : a.ep_in[b] + kP2Last - s;
  const P2Draw &pl = a.pl_r[st];
  const uint32_t *hsrc = a.h_r[st];
  const int32_t *htag = a.ht_r[st];
  uint32_t *sw = a.s_mt[s] + 4 * (size_t)b;
  const int s4 = (int)(4 * nr);
  const int32_t *cur = a.s_cur[s] + b;
  const int g_end = last ? a.max_plies : min(a.cut[st], a.max_plies);
  const uint64_t sd = episode_seed(a.seed_base, b, e), rk = rule_key(sd);
  // every input's loads issued together (used only if the tags match)
  const int ptag = pl.tag[b], nd = pl.k[b];
  const int mtag = st > 0 ? a.m_r[st - 1].tag[b] : e;
  const uint32_t *hs = htag[b] == e ? hsrc + b : nullptr;
  State s0;
  int g = 0;
  PlayDraw2 draw = st == 0 ? PlayDraw2{pl.q[b], pl.q[nr + b], pl.q[2 * nr + b], pl.q[3 * nr + b], 0, nd, false,
                                       MTQ(sw, s4, 0), cur + (size_t)nd * nr}
                           : p2_mid_get(a.m_r[st - 1], nr, b, s0, g, nd, sw, s4, cur);
  const bool prep = ptag == e * 8 + kP2Draw && mtag == e;
  if (prep) {
    if (st == 0) {
      if (__all(nd >= 5)) draw.scripted_reset(s0);
      else reset_state(s0, draw);
    }
    P2_PHASE(16 + 2 * st, t0);
    g += p2_plies(s0, draw, g, g_end, rk, hs, nr);
    P2_PHASE(17 + 2 * st, t0);
  }
  if (!last) {
    const P2Mid &mo = a.m_w[st];
    if (prep) p2_mid_put(mo, nr, b, s0, draw, g, e);
    else mo.tag[b] = -1;
    return false;
  }
  int cursor, src;
  bool lds_used = false;
  if (prep) {
    cursor = draw.fell ? draw.gm.cursor() : cur[(size_t)draw.d * nr];
    src = 2 + a.s_idx_last;
  } else {  // unprepared: the whole game, the stream seeded and drawn in LDS
    mt_seed(hz_lds + lane, kLdsStride, sd);
    PlayDraw fb{LdsMT(lane, kMTSeeded), false, false, 0, 0, 0, 0, 0, 0, MT(nullptr, 0), nullptr};
    reset_state(s0, fb);
    g = p2_plies(s0, fb, 0, a.max_plies, rk, nullptr, nr);
    cursor = fb.m.cursor();
    src = -1;
    lds_used = true;
  }
  a.episode[b] = e + 1;
  if (score_pending(s0.misc)) finish_game(s0);
  P2_PHASE(26, t0);
  store_state(a.st, a.n, b, s0);
  a.pos[b] = cursor;
  a.mt_src[b] = src;
  a.ply[b] = g;
  a.seed[b] = sd;
  a.ep_out[b] = e + 1;
  // the game this call completes, as hz_play's other pipeline counts it
  if (a.games_done) a.games_done[b] = phase_of(s0.misc) == PH_OVER ? 1 : 0;
  if (a.steps_done) a.steps_done[b] = g;
  return lds_used;
}

// draw-X blocks: D1, D2, D3 (waves 0-2), the rule hashes (wave 3); draw-Y
// blocks: D4, D5 (waves 0, 1), play0 (wave 2).  Each draw wave stages its
// own window and reads only it.
__device__ __forceinline__ void p2_draw(const P2Args &a, int blk, int y) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock;
  if (!y) {
    if (w < 3) p2_draw_stage(a, b0, lane, w, w * kP2WinRows * kLdsStride);
    else if (b0 + lane < a.n) p2_hashes(a, b0 + lane);
  } else {
    if (w < 2) p2_draw_stage(a, b0, lane, 3 + w, w * kP2WinRows * kLdsStride);
    else if (w == 2) p2_play_stage(a, b0, lane, 0);
  }
}

// play blocks: wave 3 - w runs play stage kP2Play - 1 - w (wave 0 the last:
// the rest of episode ep, or all of it).  The stages run one code path (st
// wave-uniform), so the block's four waves share one copy of the ply loop
// in the instruction cache (one inlined copy per stage, ~50 KB each,
// thrashed the cache the two CUs of a pair share).
__device__ __forceinline__ void p2_play(const P2Args &a, int blk) {
  __shared__ uint64_t s_lds_mask;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock, b = b0 + lane;
  const bool act = b < a.n;
  const uint64_t actmask = __ballot(act);
  const int nb = a.n - b0 < kBlock ? a.n - b0 : kBlock;
#ifdef HZ_DIAG
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  const int st = __builtin_amdgcn_readfirstlane(kP2Play - 1 - w);
  const bool lds_used = p2_play_stage(a, b0, lane, st);
#ifdef HZ_DIAG
  if (g_stamps && act) g_stamps[(size_t)b * kP2Stamps + w] = __builtin_amdgcn_s_memtime() - t0;  // play4 .. play1
#endif
  if (w == 0) {
    const uint64_t lm = __ballot(lds_used);
    if (lane == 0) s_lds_mask = lm;
  }
  __syncthreads();
  const uint64_t lds_mask = s_lds_mask & actmask;
  if (lds_mask) stage_mt(a.mt + (size_t)b0 * kMT, nb, tid, lds_mask, false);
}

// one 162 KB-LDS block per CU, so one wave per SIMD: every wave may use the
// whole register file (the twist wave keeps 56 quads in registers)
__global__ void __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) k_play2(P2Args a, int nblk) {
  const int blk = (int)blockIdx.x;
  const int role = blk / nblk;  // 0 play, 1 draw X, 2 draw Y, 3 seed blocks
  const int rb = blk - role * nblk;
#ifdef HZ_DIAG
  if (g_role_only >= 0 && g_role_only != role) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  if (role == 0) p2_play(a, rb);
  else if (role == 3) p2_seed(a, rb);
  else p2_draw(a, rb, role - 1);
#ifdef HZ_DIAG
  {  // wave durations per board, slot 4 role + wave: 0-3 play (play4 .. play1:
     // stamped in p2_play, before its barrier), 4-7 draw X (D1, D2, D3,
     // hashes), 8-10 draw Y (D4, D5, play0), 12-15 seed (P2x, P2y, twist, P1)
    const int w = threadIdx.x >> 6, bb = rb * kBlock + (threadIdx.x & 63);
    const bool idle = role == 2 && w == 3;
    if (g_stamps && role > 0 && !idle && bb < a.n) g_stamps[(size_t)bb * kP2Stamps + 4 * role + w] = __builtin_amdgcn_s_memtime() - t0;
  }
#endif
}

// boards whose stream lives in a pipeline-2 slot (mt_src = 2 + slot): the
// slot's quads of the board into the board's own stream, one wave per board
struct P2Slots {
  uint32_t *s[kP2Stream];
};
__global__ void __launch_bounds__(64) k_mt_materialize2(uint32_t *__restrict__ mt, P2Slots slots,
                                                       int32_t *__restrict__ mt_src, long nrow) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int src = mt_src[b];
  if (src < 2 || src >= 2 + kP2Stream) return;
  const QuadPtr from{slots.s[src - 2] + 4 * (size_t)b, (int)(4 * nrow)};
  uint32_t *to = mt + (size_t)b * kMT;
  uint32_t v[(kMT + 63) / 64];
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++) v[k] = lane + 64 * k < kMT ? from[lane + 64 * k] : 0u;
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++)
    if (lane + 64 * k < kMT) to[lane + 64 * k] = v[k];
  if (lane == 0) mt_src[b] = -1;
}

// ---------------------------------------------------------- greedy agent
// evaluation.py:137-196 choose_move_greedy, one wave per board: lane l scores
// legal moves l, l+64 (canonical ascending order) by applying the placement
// to a register copy and scoring the mover's board; a shuffle reduction keeps
// the first strictly best.  The reference applies every candidate with
// apply_move, whose place_tile_3 turn end refills the piles from the global
// `random`: lane 0 replays those L refills (identical bag and piles for every
// candidate) on the board's stream before the real move is stepped.
struct NoDraw {
  __device__ __forceinline__ uint32_t operator()(uint64_t) { return 0x1FFu; }
};

__global__ void __launch_bounds__(64) k_greedy(const uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                               int32_t *__restrict__ pos, int n, const uint8_t *__restrict__ sel,
                                               int16_t *__restrict__ action) {
  int b = blockIdx.x, lane = threadIdx.x;
  if (b >= n) return;
  bool on = !sel || sel[b];
  State s = load_state(st, n, b);
  uint64_t mk[3];
  int L = legal_mask(s, mk);
  if (!on || game_done(s.misc) || L == 0) {
    if (lane == 0) action[b] = -1;
    return;
  }
  int ph = phase_of(s.misc), p = player_of(s.misc);
  int best_sc = -1, best_k = 0x7fffffff;
  for (int k = lane; k < L; k += 64) {
    int sc;
    if (ph == PH_CHOOSE) {
      sc = score_player(s, p);  // choosing a pile leaves the board as it is
    } else {
      State t = s;
      NoDraw nd;
      step_state<true>(t, kth_action(mk, k), nd);
      sc = score_player(t, p);
    }
    if (sc > best_sc) { best_sc = sc; best_k = k; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    int osc = __shfl_xor(best_sc, off), ok = __shfl_xor(best_k, off);
    if (osc > best_sc || (osc == best_sc && ok < best_k)) { best_sc = osc; best_k = ok; }
  }
  if (lane == 0) {
    if (ph == PH_P3) {
      StreamDraw<MT> d{MT(mt + (size_t)b * kMT, pos[b])};
      for (int k = 0; k < L; k++) {
        State t = s;
        replenish(t, d);
      }
      pos[b] = d.m.cursor();
    }
    action[b] = (int16_t)kth_action(mk, best_k);
  }
}

// ---------------------------------------------------------- state transfer
__global__ void __launch_bounds__(kBlock) k_mt_normalize(uint32_t *__restrict__ mt, int32_t *__restrict__ pos,
                                                         int n, int32_t *__restrict__ index) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  MT m(mt + (size_t)b * kMT, pos[b]);
  m.normalize();
  pos[b] = m.cursor();
  if (index) index[b] = m.pos;
}

__global__ void __launch_bounds__(kBlock) k_mt_import(int32_t *__restrict__ pos, int n,
                                                      const int32_t *__restrict__ index) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  pos[b] = index[b] | (kMT << 16);  // CPython states are fully twisted
}

inline int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

// ======================================================================= ABI
// boards whose stream lives in a play slot (mt_src >= 0): copy it into the
// board's own stream, one wave per board
__global__ void __launch_bounds__(64) k_mt_materialize(uint32_t *__restrict__ mt, const uint32_t *__restrict__ a0,
                                                      const uint32_t *__restrict__ a1, int32_t *__restrict__ mt_src,
                                                      int n) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int src = mt_src[b];
  if (src < 0 || src > 1) return;  // (pipeline-2 slots: k_mt_materialize2)
  const uint32_t *from = (src ? a1 : a0) + (size_t)b * kMT;
  uint32_t *to = mt + (size_t)b * kMT;
  uint32_t v[(kMT + 63) / 64];
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++) v[k] = lane + 64 * k < kMT ? from[lane + 64 * k] : 0u;
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++)
    if (lane + 64 * k < kMT) to[lane + 64 * k] = v[k];
  if (lane == 0) mt_src[b] = -1;
}

static int materialize(hz_env *e) {
  if (!e->lazy) return 0;
  hipLaunchKernelGGL(k_mt_materialize, dim3(e->n), dim3(64), 0, e->stream, e->mt, e->ahead_mt[0], e->ahead_mt[1],
                     e->mt_src, e->n);
  if (e->p2_s[0]) {
    P2Slots sl;
    for (int k = 0; k < kP2Stream; k++) sl.s[k] = e->p2_s[k];
    hipLaunchKernelGGL(k_mt_materialize2, dim3(e->n), dim3(64), 0, e->stream, e->mt, sl, e->mt_src,
                       (long)e->nrow);
  }
  e->lazy = 0;
  return launch_err();
}

// ---------------------------------------------------------- pipeline 2 host
static_assert(sizeof(((hz_env *)0)->p2_s) / sizeof(uint32_t *) == kP2Stream, "slot ring");
static_assert(sizeof(((hz_env *)0)->p2_pl) / sizeof(P2Draw) == kP2Ring && sizeof(((hz_env *)0)->p2_h) / sizeof(uint32_t *) == kP2Ring,
              "script and hash rings");
static_assert(sizeof(((hz_env *)0)->p2_x) / sizeof(P2Draw) == 2 * (kP2Draw - 1) &&
                  sizeof(((hz_env *)0)->p2_m) / sizeof(P2Mid) == 2 * (kP2Play - 1) &&
                  sizeof(((hz_env *)0)->p2_cut) / sizeof(int) == kP2Play - 1,
              "hand-off rings");
static void free_p2(hz_env *e) {
  auto f = [](auto *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
  };
  for (int k = 0; k < kP2Stream; k++) {
    f(e->p2_s[k]);
    f(e->p2_s_tag[k]);
    f(e->p2_s_cur[k]);
  }
  auto fd = [&](P2Draw &d) {
    f(d.tag);
    f(d.k);
    f(d.q);
    f(d.bag);
    f(d.c);
  };
  for (int k = 0; k < kP2Draw - 1; k++) fd(e->p2_x[k][0]), fd(e->p2_x[k][1]);
  for (int k = 0; k < kP2Ring; k++) fd(e->p2_pl[k]);
  for (int k = 0; k < kP2Play - 1; k++)
    for (int j = 0; j < 2; j++) {
      P2Mid &m = e->p2_m[k][j];
      f(m.tag);
      f(m.st);
      f(m.q);
      f(m.i);
    }
  for (int k = 0; k < kP2Ring; k++) {
    f(e->p2_h[k]);
    f(e->p2_h_tag[k]);
  }
  for (int k = 0; k < 2; k++) {
    f(e->p2_ph[k]);
    f(e->p2_ep[k]);
  }
}

// every hand-off tag to "none" (a tag names the episode its slot holds, and a
// slot's contents depend only on (board, episode), so this is never needed
// for correctness; it keeps a fresh pipeline from trusting fresh memory)
static int p2_clear_tags(hz_env *e) {
  const size_t bytes = e->nrow * sizeof(int32_t);
  auto c = [&](int32_t *t) { return hipMemsetAsync(t, 0xff, bytes, e->stream) != hipSuccess; };
  for (int k = 0; k < kP2Stream; k++)
    if (c(e->p2_s_tag[k])) return 1;
  for (int k = 0; k < kP2Draw - 1; k++)
    if (c(e->p2_x[k][0].tag) || c(e->p2_x[k][1].tag)) return 1;
  for (int k = 0; k < kP2Ring; k++)
    if (c(e->p2_pl[k].tag) || c(e->p2_h_tag[k])) return 1;
  for (int k = 0; k < kP2Play - 1; k++)
    if (c(e->p2_m[k][0].tag) || c(e->p2_m[k][1].tag)) return 1;
  return 0;
}

// allocated on first use: 14 stream slots of 2.5 KB per board plus ~1.9 KB
// of hand-offs per board
static int alloc_p2(hz_env *e) {
  if (e->p2_s[0]) return 0;
  const size_t nr = e->nrow;
  auto m = [](auto **p, size_t bytes) { return hipMalloc((void **)p, bytes) == hipSuccess; };
  bool ok = true;
  for (int k = 0; ok && k < kP2Stream; k++)
    ok = m(&e->p2_s[k], nr * kMT * 4) && m(&e->p2_s_tag[k], nr * 4) &&
         m(&e->p2_s_cur[k], (kAheadDraws + 1) * nr * 4);
  auto md = [&](P2Draw &d) {
    return m(&d.tag, nr * 4) && m(&d.k, nr * 4) && m(&d.q, kAheadWords * nr * 8) && m(&d.bag, nr * 8) &&
           m(&d.c, nr * 4);
  };
  for (int k = 0; ok && k < kP2Draw - 1; k++) ok = md(e->p2_x[k][0]) && md(e->p2_x[k][1]);
  for (int k = 0; ok && k < kP2Ring; k++)
    ok = md(e->p2_pl[k]) && m(&e->p2_h[k], kRulePlies * nr * 4) && m(&e->p2_h_tag[k], nr * 4);
  for (int k = 0; ok && k < kP2Play - 1; k++)
    for (int j = 0; ok && j < 2; j++) {
      P2Mid &mm = e->p2_m[k][j];
      ok = m(&mm.tag, nr * 4) && m(&mm.st, 6 * nr * 8) && m(&mm.q, 4 * nr * 8) && m(&mm.i, 3 * nr * 4);
    }
  for (int k = 0; ok && k < 2; k++)
    ok = m(&e->p2_ph[k], 3 * nr * 4) &&
         m(&e->p2_ep[k], nr * 4);
  if (!ok || p2_clear_tags(e)) {
    free_p2(e);
    return 1;
  }
  e->primed2 = 0;
  return 0;
}

// one hz_play call of pipeline 2 (k_play2).  Call c uses stream slot
// (c - s) % kP2Stream for stage s; the D1 -> D2 -> D3 -> D4 hand-offs, P1a ->
// P1b and play stage st -> st + 1 by call parity; D4's script and the rule
// hashes in rings of kP2Ring (read by play stage st st + 1 calls later).  Every slot written by call c is read by call c + 1 or later,
// so launch order on the stream is the only synchronisation.
static int launch_play2(hz_env *e, int32_t max_plies, int32_t *games_done, int32_t *steps_done) {
  if (alloc_p2(e)) return 1;
  const int c = e->calls2, r = c & 1, w = r ^ 1;
  if (!e->primed2) {
    if (hipMemcpyAsync(e->p2_ep[w], e->episode, (size_t)e->n * sizeof(int32_t), hipMemcpyDeviceToDevice,
                       e->stream))
      return 1;
    e->primed2 = 1;
  }
  P2Args a{};
  a.st = e->state;
  a.mt = e->mt;
  a.pos = e->pos;
  a.ply = e->ply;
  a.episode = e->episode;
  a.seed = e->seed;
  a.n = e->n;
  a.max_plies = max_plies;
  a.draws = e->seed_ahead;
  a.err = e->wait_err;
  a.spin = e->spin_limit;
  for (int k = 0; k < kP2Play - 1; k++) a.cut[k] = e->p2_cut[k];
  a.seed_base = e->seed_base;
  a.nrow = (long)e->nrow;
  a.games_done = games_done;
  a.steps_done = steps_done;
  a.mt_src = e->mt_src;
  a.ep_in = e->p2_ep[w];
  a.ep_out = e->p2_ep[r];
  auto sl = [c](int s) { return ((c - s) % kP2Stream + kP2Stream) % kP2Stream; };
  for (int s = 0; s < kP2Stages; s++) {
    a.s_mt[s] = e->p2_s[sl(s)];
    a.s_tag[s] = e->p2_s_tag[sl(s)];
    a.s_cur[s] = e->p2_s_cur[sl(s)];
  }
  a.s_idx_last = sl(kP2Last);
  a.ph_w = e->p2_ph[r];
  a.ph_r = e->p2_ph[w];
  for (int k = 0; k < kP2Draw - 1; k++) {
    a.x_w[k] = e->p2_x[k][r];
    a.x_r[k] = e->p2_x[k][w];
  }
  a.pl_w = e->p2_pl[c % kP2Ring];
  a.h_w = e->p2_h[c % kP2Ring];
  a.ht_w = e->p2_h_tag[c % kP2Ring];
  for (int st = 0; st < kP2Play; st++) {  // written by call c - 1 - st
    const int k = (c + kP2Ring - 1 - st) % kP2Ring;
    a.pl_r[st] = e->p2_pl[k];
    a.h_r[st] = e->p2_h[k];
    a.ht_r[st] = e->p2_h_tag[k];
  }
  for (int st = 0; st < kP2Play - 1; st++) {
    a.m_w[st] = e->p2_m[st][r];
    a.m_r[st] = e->p2_m[st][w];
  }
  const int nblk = grid_for(e->n);
  hipLaunchKernelGGL(k_play2, dim3(4 * nblk), dim3(kStageThreads), kResetLds, e->stream, a, nblk);
  if (int err = launch_err()) return err;
  e->lazy = 1;
  e->calls2 = (c + 1) % (kP2Stream * kP2Ring * 2);  // (a multiple of every ring length)
  e->primed = 0;  // the other pipeline's episode prediction is stale now
  return 0;
}

extern "C" {

hz_env *hz_env_create(int32_t n_boards, uint64_t seed_base, void *stream) {
  if (n_boards <= 0) return nullptr;
  if (install_comp_table()) return nullptr;  // scoring's component table (hz_device.hpp)
  hz_env *e = (hz_env *)calloc(1, sizeof(hz_env));
  if (!e) return nullptr;
  e->n = n_boards;
  e->seed_base = seed_base;
  e->stream = (hipStream_t)stream;
  size_t n = (size_t)n_boards;
  // k_reset / k_rollout stage 64 boards' MT words in 158 KiB of LDS
  if (hipFuncSetAttribute((const void *)k_reset, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResetLds) !=
          hipSuccess ||
      hipFuncSetAttribute((const void *)k_rollout<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)kResetLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)k_rollout<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)kResetLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)k_rollout<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)kResetLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)k_rollout<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)kResetLds) != hipSuccess ||
      hipFuncSetAttribute((const void *)k_play2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResetLds) !=
          hipSuccess) {
    free(e);
    return nullptr;
  }
  bool ok = hipMalloc(&e->state, n * 6 * sizeof(uint64_t)) == hipSuccess &&
            hipMalloc(&e->mt, n * 624 * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&e->pos, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->ply, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->episode, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->seed, n * sizeof(uint64_t)) == hipSuccess &&
            hipMalloc(&e->mt_src, n * sizeof(int32_t)) == hipSuccess;
  if (ok) {
    ok = hipMemset(e->state, 0, n * 6 * sizeof(uint64_t)) == hipSuccess &&
         hipMemset(e->pos, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->ply, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->episode, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->seed, 0, n * sizeof(uint64_t)) == hipSuccess &&
         hipMemset(e->mt_src, 0xff, n * sizeof(int32_t)) == hipSuccess;
  }
  for (int k = 0; ok && k < 2; k++) {
    ok = hipMalloc(&e->ahead_mt[k], n * kMT * sizeof(uint32_t)) == hipSuccess &&
         hipMalloc(&e->ahead_tag[k], n * sizeof(int32_t)) == hipSuccess &&
         hipMalloc(&e->ahead_pile[k], n * kAheadWords * sizeof(uint64_t)) == hipSuccess &&
         hipMalloc(&e->ahead_cur[k], n * (kAheadDraws + 1) * sizeof(int32_t)) == hipSuccess &&
         hipMalloc(&e->ahead_rule[k], (n + kBlock - 1) / kBlock * kBlock * kRulePlies * sizeof(uint32_t)) ==
             hipSuccess &&
         hipMalloc(&e->ep_final[k], n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->ahead_tag[k], 0xff, n * sizeof(int32_t)) == hipSuccess;
  }
  e->nrow = (n + kBlock - 1) / kBlock * kBlock;
  for (int k = 0; ok && k < kRing; k++) {
    size_t nr = e->nrow;
    ok = hipMalloc(&e->ring_mt[k], nr * kMT * sizeof(uint32_t)) == hipSuccess &&
         hipMalloc(&e->ring_tag[k], nr * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->ring_tag[k], 0xff, nr * sizeof(int32_t)) == hipSuccess &&
         hipMalloc(&e->ring_pile[k], nr * 3 * sizeof(uint64_t)) == hipSuccess &&
         hipMalloc(&e->ring_cur[k], nr * (kD1Draws + 1) * sizeof(int32_t)) == hipSuccess &&
         hipMalloc(&e->ring_k1[k], nr * sizeof(int32_t)) == hipSuccess;
  }
  ok = ok && hipDeviceSynchronize() == hipSuccess;
  e->seed_ahead = kAheadDraws;
  {  // hz_play's pipeline: 2 by default, HZ_PIPELINE=1 for the first (hz_env_set_pipeline)
    const char *pv = getenv("HZ_PIPELINE");
    e->pipeline = pv && atoi(pv) == 1 ? 1 : 2;
    // HZ_P2_CUTS="a,b,c,d": pipeline 2's play stage boundaries (plies,
    // increasing multiples of 4: whole turns; a stage that starts at player
    // 1's turn plays single plies up to the next turn pair)
    e->p2_cut[0] = 20;
    e->p2_cut[1] = 32;
    e->p2_cut[2] = 44;
    e->p2_cut[3] = 56;
    const char *cv = getenv("HZ_P2_CUTS");
    int c[4];
    if (cv && sscanf(cv, "%d,%d,%d,%d", &c[0], &c[1], &c[2], &c[3]) == 4 && c[0] > 0 && c[1] > c[0] && c[2] > c[1] &&
        c[3] > c[2] && c[0] % 4 == 0 && c[1] % 4 == 0 && c[2] % 4 == 0 && c[3] % 4 == 0)
      for (int k = 0; k < 4; k++) e->p2_cut[k] = c[k];
  }
  ok = ok && hipMalloc(&e->wait_err_own, sizeof(int32_t)) == hipSuccess &&
       hipMemset(e->wait_err_own, 0, sizeof(int32_t)) == hipSuccess;
  e->wait_err = e->wait_err_own;
  e->spin_limit = kSpinLimitDefault;
  if (!ok) {
    hz_env_destroy(e);
    return nullptr;
  }
  return e;
}

void hz_env_destroy(hz_env *e) {
  if (!e) return;
  free_p2(e);
  if (e->wait_err_own) (void)hipFree(e->wait_err_own);
  for (int k = 0; k < 2; k++) {
    if (e->ahead_mt[k]) (void)hipFree(e->ahead_mt[k]);
    if (e->ahead_tag[k]) (void)hipFree(e->ahead_tag[k]);
    if (e->ahead_pile[k]) (void)hipFree(e->ahead_pile[k]);
    if (e->ahead_cur[k]) (void)hipFree(e->ahead_cur[k]);
    if (e->ahead_rule[k]) (void)hipFree(e->ahead_rule[k]);
    if (e->ep_final[k]) (void)hipFree(e->ep_final[k]);
  }
  for (int k = 0; k < kRing; k++) {
    if (e->ring_mt[k]) (void)hipFree(e->ring_mt[k]);
    if (e->ring_tag[k]) (void)hipFree(e->ring_tag[k]);
    if (e->ring_pile[k]) (void)hipFree(e->ring_pile[k]);
    if (e->ring_cur[k]) (void)hipFree(e->ring_cur[k]);
    if (e->ring_k1[k]) (void)hipFree(e->ring_k1[k]);
  }
  if (e->state) (void)hipFree(e->state);
  if (e->mt) (void)hipFree(e->mt);
  if (e->pos) (void)hipFree(e->pos);
  if (e->ply) (void)hipFree(e->ply);
  if (e->episode) (void)hipFree(e->episode);
  if (e->seed) (void)hipFree(e->seed);
  if (e->mt_src) (void)hipFree(e->mt_src);
  free(e);
}

int32_t hz_env_size(const hz_env *e) { return e ? e->n : -1; }

int hz_env_set_error_word(hz_env *e, int32_t *word) {
  if (!e) return -1;
  e->wait_err = word ? word : e->wait_err_own;
  return 0;
}

int hz_env_set_spin_limit(hz_env *e, int32_t limit) {
  if (!e || limit < 0) return -1;
  e->spin_limit = limit ? limit : kSpinLimitDefault;
  return 0;
}

int hz_env_set_pipeline(hz_env *e, int32_t pipeline) {
  if (!e || (pipeline != 1 && pipeline != 2)) return -1;
  e->pipeline = pipeline;
  e->primed = 0;
  e->primed2 = 0;
  return 0;
}

int hz_env_set_stream(hz_env *e, void *stream) {
  if (!e) return -1;
  e->stream = (hipStream_t)stream;
  return 0;
}

uint64_t *hz_env_state_ptr(hz_env *e) { return e ? e->state : nullptr; }
uint32_t *hz_env_mt_ptr(hz_env *e) {  // the streams are made current first (materialize)
  if (!e || materialize(e)) return nullptr;
  return e->mt;
}
int32_t *hz_env_mt_pos_ptr(hz_env *e) { return e ? e->pos : nullptr; }
int32_t *hz_env_ply_ptr(hz_env *e) { return e ? e->ply : nullptr; }
uint64_t *hz_env_seed_ptr(hz_env *e) { return e ? e->seed : nullptr; }

int hz_env_set_seed_ahead(hz_env *e, int32_t draws) {
  if (!e || draws < 0) return -1;
  e->seed_ahead = draws > kAheadDraws ? kAheadDraws : draws;
  e->primed = 0;
  e->primed2 = 0;
  if (e->p2_s[0] && p2_clear_tags(e)) return 1;
  // draw1's work depends on the draw count: start the ring afresh
  for (int k = 0; k < kRing; k++)
    if (hipMemsetAsync(e->ring_tag[k], 0xff, e->nrow * sizeof(int32_t), e->stream)) return 1;
  return 0;
}

int hz_reset(hz_env *e, const uint8_t *sel, const uint64_t *seeds) {
  if (!e) return -1;
  if (int err = materialize(e)) return err;  // unselected boards keep their streams
  e->primed = 0;  // episode counters move outside hz_play's plan
  e->primed2 = 0;
  hipLaunchKernelGGL(k_reset, dim3(grid_for(e->n)), dim3(kStageThreads), kResetLds, e->stream, e->state, e->mt, e->pos,
                     e->ply, e->episode, e->seed, e->n, e->seed_base, sel, seeds);
  return launch_err();
}

int hz_legal_mask(hz_env *e, uint64_t *mask, int32_t *count) {
  if (!e || !mask) return -1;
  hipLaunchKernelGGL(k_legal, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->n, mask, count);
  return launch_err();
}

int hz_step(hz_env *e, const int16_t *action, int32_t *status) {
  if (!e || !action) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_step, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->n, action, status);
  return launch_err();
}

int hz_rule_ply(hz_env *e, uint64_t *mask, int32_t *count, int16_t *action, int32_t *status) {
  if (!e) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_ply, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->seed, e->n, mask, count, action, status);
  return launch_err();
}

int hz_score(hz_env *e, int32_t *out, int32_t *out_parts) {
  if (!e || (!out && !out_parts)) return -1;
  hipLaunchKernelGGL(k_score, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->n, out, out_parts);
  return launch_err();
}

int hz_encode(hz_env *e, const int32_t *idx, int32_t m, float *board, float *glob) {
  if (!e || m < 0 || (!board && !glob)) return -1;
  if (!idx && m > e->n) return -2;
  if (m == 0) return 0;
  launch_encode(e->state, (long)e->n, 1, idx, m, board, glob, e->stream);
  return launch_err();
}

int hz_rule_actions(hz_env *e, const uint64_t *mask, const int32_t *count, int16_t *action) {
  if (!e || !mask || !action) return -1;
  hipLaunchKernelGGL(k_rule, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->seed, e->ply, e->n, mask, count,
                     action);
  return launch_err();
}

int hz_greedy_actions(hz_env *e, const uint8_t *sel, int16_t *action) {
  if (!e || !action) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_greedy, dim3(e->n), dim3(64), 0, e->stream, e->state, e->mt, e->pos, e->n, sel, action);
  return launch_err();
}

// hz_play's chance-ahead pipeline: one launch per call c.  Blocks [0, nblk)
// play from play slot r = c & 1; draw2 blocks [nblk, 2 nblk) fill play slot
// w = r ^ 1 for call c + 1 from ring slot (c + 1) % 3; draw1 blocks
// continue ring slot (c + 2) % 3 for call c + 2; seed blocks refill ring
// slot c % 3 for call c + 3.  Launch order on the stream is the only
// synchronisation: a slot written by call c is read by call c + 1; the
// preparing blocks read ep_final[w], written by call c - 1's playing blocks
// (the episode counter each board ended with).  The prediction (call c + k
// resets to that counter plus k) only decides which boards skip seeding and
// drawing: a board replays a slot only when the slot's tag equals its
// episode counter, so results never depend on it.  Anything else that moves
// episode counters (hz_reset, hz_rollout) makes the next call re-prime
// ep_final from the counters.
static int launch_rollout(hz_env *e, int32_t max_plies, int32_t auto_reset, int reset_first, uint64_t *traj_state,
                          uint64_t *traj_mask, int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  if (!e || max_plies < 0) return -1;
  e->primed2 = 0;  // (pipeline 2's episode prediction is stale after this launch)
  // hz_rollout continues the current games on their streams; hz_play starts
  // every board's next game (its old stream is dead)
  if (!reset_first)
    if (int err = materialize(e)) return err;
  uint32_t *ahead_mt = nullptr;
  const int32_t *ahead_tag = nullptr;
  const uint64_t *ahead_pile = nullptr;
  const int32_t *ahead_cur = nullptr;
  const uint32_t *ahead_rule = nullptr;
  int32_t *ep_final = nullptr;
  int nblk = grid_for(e->n), grid = nblk;
  bool pipe = reset_first && e->seed_ahead > 0;
  int r = e->calls & 1, w = r ^ 1;
  int c3 = e->calls % kRing;
  auto ring = [e](int k) {
    return Ring{e->ring_mt[k], e->ring_tag[k], e->ring_pile[k], e->ring_cur[k], e->ring_k1[k], e->wait_err,
                e->spin_limit};
  };
  if (pipe) {
    size_t n = (size_t)e->n;
    if (!e->primed) {
      if (hipMemcpyAsync(e->ep_final[w], e->episode, n * sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream))
        return 1;
      e->slot_valid[r] = 0;
      e->primed = 1;
    }
    if (e->slot_valid[r]) {
      ahead_mt = e->ahead_mt[r];
      ahead_tag = e->ahead_tag[r];
      ahead_pile = e->ahead_pile[r];
      ahead_cur = e->ahead_cur[r];
      ahead_rule = e->ahead_rule[r];
    }
    ep_final = e->ep_final[r];
    grid = 4 * nblk;
  } else {
    e->primed = 0;
  }
  bool rec = traj_state || traj_mask || traj_action;
  auto kern = auto_reset ? (rec ? k_rollout<true, true> : k_rollout<true, false>)
                         : (rec ? k_rollout<false, true> : k_rollout<false, false>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kStageThreads), kResetLds, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->episode, e->seed, e->n, e->seed_base, max_plies, auto_reset, reset_first, traj_state,
                     traj_mask, traj_action, games_done, steps_done, ahead_mt, ahead_tag, ahead_pile, ahead_cur,
                     e->seed_ahead, ep_final, nblk, e->ahead_mt[w], e->ahead_tag[w], e->ahead_pile[w],
                     e->ahead_cur[w], e->ep_final[w], ring(c3), ring((c3 + 2) % kRing), ring((c3 + 1) % kRing),
                     (long)e->nrow, ahead_rule, e->ahead_rule[w], e->mt_src, ahead_mt ? r : -1);
  int err = launch_err();
  if (err) return err;
  if (ahead_mt) e->lazy = 1;
  if (pipe) {
    e->slot_valid[w] = 1;
    e->calls++;
  }
  return 0;
}

int hz_rollout(hz_env *e, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state, uint64_t *traj_mask,
               int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  return launch_rollout(e, max_plies, auto_reset, 0, traj_state, traj_mask, traj_action, games_done, steps_done);
}

int hz_play(hz_env *e, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state, uint64_t *traj_mask,
            int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  if (e && e->pipeline == 2 && !auto_reset && !traj_state && !traj_mask && !traj_action &&
      max_plies >= kP2MinPlies)
    return launch_play2(e, max_plies, games_done, steps_done);
  return launch_rollout(e, max_plies, auto_reset, 1, traj_state, traj_mask, traj_action, games_done, steps_done);
}

int hz_export_state(hz_env *e, uint64_t *state, uint32_t *mt, int32_t *mt_index) {
  if (!e) return -1;
  size_t n = (size_t)e->n;
  if (state && hipMemcpyAsync(state, e->state, n * 6 * sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream))
    return 1;
  if (mt || mt_index) {
    if (int err = materialize(e)) return err;
    hipLaunchKernelGGL(k_mt_normalize, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->mt, e->pos, e->n,
                       mt_index);
    int r = launch_err();
    if (r) return r;
    if (mt && hipMemcpyAsync(mt, e->mt, n * kMT * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
  }
  return 0;
}

int hz_import_state(hz_env *e, const uint64_t *state, const uint32_t *mt, const int32_t *mt_index) {
  if (!e) return -1;
  if ((mt == nullptr) != (mt_index == nullptr)) return -2;
  size_t n = (size_t)e->n;
  if (state && hipMemcpyAsync(e->state, state, n * 6 * sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream))
    return 1;
  if (mt) {
    if (int err = materialize(e)) return err;  // (then every board's stream is its own)
    if (hipMemcpyAsync(e->mt, mt, n * kMT * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
    hipLaunchKernelGGL(k_mt_import, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->pos, e->n, mt_index);
    return launch_err();
  }
  return 0;
}

int hz_replenish(hz_env *e, const uint8_t *sel) {
  if (!e) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_turn_op, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->n, sel,
                     0);
  return launch_err();
}

int hz_end_turn(hz_env *e, const uint8_t *sel) {
  if (!e) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_turn_op, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->n, sel,
                     1);
  return launch_err();
}

int hz_encode_states(const uint64_t *states, int64_t word_stride, int64_t item_stride, const int32_t *idx, int32_t m,
                     float *board, float *glob, void *stream) {
  if (!states || m < 0 || (!board && !glob)) return -1;
  if (m == 0) return 0;
  launch_encode(states, (long)word_stride, (long)item_stride, idx, m, board, glob, (hipStream_t)stream);
  return launch_err();
}

const char *hz_version(void) { return "hz 0.1 gfx950"; }

#ifdef HZ_DIAG
int hz_diag_set_stamps(uint64_t *p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
int hz_diag_set_role_only(int r) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_role_only), &r, sizeof(r)) == hipSuccess ? 0 : 1;
}
#endif

}  // extern "C"
