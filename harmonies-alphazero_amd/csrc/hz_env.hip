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
  // auto-reset episodes prepared ahead (hz_rollout with auto_reset; see
  // ar_prep_stage): slot s of board b holds one episode's pile script,
  // cursors and stream, tagged with the episode; mt_src = kArSrc + s while a
  // board plays on slot s's stream
  int ar_ahead;              // on unless HZ_AR_AHEAD=0 / hz_env_set_auto_ahead(e, 0)
  uint32_t *ar_mt;           // [kArSlots][n][624]
  int32_t *ar_tag;           // [kArSlots][n] episode held (-1: none)
  uint64_t *ar_pile;         // [kArSlots][kAheadWords][n]
  int32_t *ar_cur;           // [kArSlots][kAheadDraws + 1][n]
  int32_t *ar_ep[2];         // [n] episode counter at the start of an auto-reset call, by call parity
  int ar_calls, ar_primed;
  // per-ply draw windows (k_step / k_ply; see PlyWin): 12 stream words per
  // board saved by the ply before a turn end, tagged with the cursor and
  // the stream epoch, which every other entry point that can move or
  // rewrite streams bumps
  uint32_t *pw_words;        // [kPlyWin][nrow]
  int32_t *pw_tag;           // [nrow] cursor the words start at (-1: none)
  int32_t *pw_ep;            // [nrow] stream epoch of the words
  int32_t mt_epoch;
  // pipeline 2 (hz_env_set_pipeline(e, 2); see k_play2): every board's game
  // spread over thirteen consecutive hz_play calls, one stage per call
  int pipeline;              // 1: chance-ahead (k_rollout's roles), 2: k_play2
  int calls2, primed2;
  int p2_cut[3];             // the play stages' ply boundaries (HZ_P2_CUTS)
  uint32_t *p2_s[14];        // [624][nrow] stream slots (kP2Stream)
  int32_t *p2_s_tag[14];     // [nrow] episode * 8 + 1 P1a / 2 pass 1 / 3 P2a / 4 P2b / 5 seeded, rows 0-223 twisted
  int32_t *p2_s_cur[14];     // [kAheadDraws + 1][nrow] the slot's cursor before draw 0 and after each draw
  uint32_t *p2_p1h[2];       // [nrow] P1a -> P1b
  uint32_t *p2_p2h[2];       // [2][nrow] P2a -> P2b
  uint32_t *p2_p3h[2];       // [2][nrow] P2b -> P2c
  P2Draw p2_x[3][2];         // D1 -> D2 -> D3 -> D4, by call parity
  P2Draw p2_pl[5];           // D4 -> playA, playB, playC, playD: a ring of five
  P2Mid p2_m[3][2];          // playA -> playB -> playC -> playD, by call parity
  uint32_t *p2_h[5];         // [kRulePlies][nrow] rule hashes, a ring of five
  int32_t *p2_h_tag[5];      // [nrow] their episode
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

// ---------------------------------------------------- per-ply draw windows
// A turn end draws one pile (harmonies_engine.py:301-329 -> :132-137):
// ~4 stream words, a twist of the generation in place every other time.
// The per-ply kernels (k_step, k_ply) spread that memory work over the turn
// instead of putting it on the turn-ending ply: the ply that makes a turn's
// first placement twists the stream ahead until 12 words past the cursor
// are twisted; the ply that makes the second saves those 12 words in the
// board's slot (word-major, so the turn-ending ply loads them coalesced,
// with its state, in the same round trip), tagged with the cursor and the
// env's stream epoch.  The turn-ending ply draws from the slot when both
// tags match (WinGMT's window, marked fresh: no load), from memory
// otherwise.  The words are the stream's own and every other entry point
// that can move or rewrite a stream bumps the epoch, so results never
// depend on the slot.
constexpr int kPlyWin = 12;
static_assert(kPlyWin == 12, "WinMT12's window");
struct PlyWin {
  uint32_t *w;   // [kPlyWin][nrow]
  int32_t *tag;  // [nrow]
  int32_t *ep;   // [nrow]
  long nrow;
  int32_t epoch;
};
struct PlyWinIn {  // a board's slot, loaded with its state
  uint32_t q[kPlyWin];
  int32_t tag, ep;
};
__device__ __forceinline__ PlyWinIn win_load(const PlyWin &pw, int b) {
  PlyWinIn in;
#pragma unroll
  for (int j = 0; j < kPlyWin; j++) in.q[j] = pw.w[(size_t)j * pw.nrow + b];
  in.tag = pw.tag[b];
  in.ep = pw.ep[b];
  return in;
}
// the turn-ending ply: draw from the saved words when they are this cursor's
__device__ __forceinline__ void win_take(const PlyWin &pw, const PlyWinIn &in, WinMT12 &m, int cursor) {
  if (in.tag == cursor && in.ep == pw.epoch) {
#pragma unroll
    for (int j = 0; j < kPlyWin; j++) m.q[j] = in.q[j];
    m.left = kPlyWin;
    m.fresh = true;
  }
}
// after a successful non-drawing step: twist ahead (a first placement made),
// or save the next 12 words (a second placement made: the next ply ends the
// turn).  m's cursor may move tw only (written back by the caller).
__device__ __forceinline__ void win_prepare(const PlyWin &pw, WinMT12 &m, int b, int phase_after) {
  if (phase_after != PH_P2 && phase_after != PH_P3) return;
  if (m.pos >= kMT) return;  // (a generation's end: the draw's own prefetch handles it)
  while (m.tw < kMT && m.tw < m.pos + kPlyWin) m.tw += twist_block_vec(m.w, m.tw);
  if (phase_after != PH_P3) return;
  if (m.tw - m.pos < kPlyWin) {  // the generation ends inside the window
    pw.tag[b] = -1;
    return;
  }
  const int a = m.pos & ~3, sh = m.pos & 3;
  uint32_t f[kPlyWin + 4];
#pragma unroll
  for (int k = 0; k < kPlyWin / 4 + 1; k++) {
    const int o = a + 4 * k <= kMT - 4 ? a + 4 * k : kMT - 4;
    const uint4 v = *(const uint4 *)(m.w + o);
    f[4 * k] = v.x; f[4 * k + 1] = v.y; f[4 * k + 2] = v.z; f[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int j = 0; j < kPlyWin; j++)
    pw.w[(size_t)j * pw.nrow + b] = sh == 0 ? f[j] : sh == 1 ? f[j + 1] : sh == 2 ? f[j + 2] : f[j + 3];
  pw.tag[b] = m.cursor();
  pw.ep[b] = pw.epoch;
}

// the same masks unpacked to one byte per action (bool [n][143], what
// BatchedEnv.legal_actions() hands a caller): each lane unpacks its board's
// three words into LDS, then the block writes its 64 boards' 9,152
// contiguous bytes with 16-B stores (a byte store per action and lane
// would touch 64 lines per instruction)
__global__ void __launch_bounds__(kBlock) k_legal_bytes(const uint64_t *__restrict__ st, int n,
                                                        uint8_t *__restrict__ out, int32_t *__restrict__ count) {
  __shared__ uint4 s_out[kBlock * kActions / 16];
  const int lane = threadIdx.x, b0 = blockIdx.x * kBlock, b = b0 + lane;
  const int nb = n - b0 < kBlock ? n - b0 : kBlock;
  uint64_t m[3] = {0, 0, 0};
  int c = 0;
  if (b < n) {
    const State s = load_state(st, n, b);
    c = legal_mask(s, m);
    if (game_done(s.misc)) { m[0] = m[1] = m[2] = 0; c = 0; }
    if (count) count[b] = c;
  }
  uint8_t *o = reinterpret_cast<uint8_t *>(s_out) + lane * kActions;
#pragma unroll 8
  for (int a = 0; a < kActions; a++) o[a] = (uint8_t)((m[a >> 6] >> (a & 63)) & 1);
  __syncthreads();
  const int total = nb * kActions;  // bytes of this block's boards
  uint8_t *dst = out + (size_t)b0 * kActions;
  // (out + b0 * 143 is 16-B aligned only when b0 is: 64 * 143 = 9,152 = 572 x 16 keeps it so from an aligned base)
  for (int q = lane; q < total / 16; q += kBlock) reinterpret_cast<uint4 *>(dst)[q] = s_out[q];
  for (int i = total / 16 * 16 + lane; i < total; i += kBlock) dst[i] = reinterpret_cast<const uint8_t *>(s_out)[i];
}

// ------------------------------------------------------------------- step
__global__ void __launch_bounds__(kBlock) k_step(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                 int32_t *__restrict__ pos, int32_t *__restrict__ ply, int n,
                                                 const int16_t *__restrict__ action, int32_t *__restrict__ status,
                                                 PlyWin pw) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  // every load of the step issued with the action's (one memory round trip;
  // a no-op board's loads go unused)
  const int a = action[b];
  State s = load_state(st, n, b);
  const int c0 = pos[b];
  const PlyWinIn win = win_load(pw, b);
  // (the compiler would sink these loads past the no-op branch: a second
  // round trip; naming them here keeps all of them in the first)
  asm volatile("" ::"v"(s.pl[0]), "v"(s.pl[1]), "v"(s.pl[2]), "v"(s.pl[3]), "v"(s.piles), "v"(s.misc), "v"(c0),
               "v"(win.tag), "v"(win.ep), "v"(win.q[0]), "v"(win.q[1]), "v"(win.q[2]), "v"(win.q[3]), "v"(win.q[4]),
               "v"(win.q[5]), "v"(win.q[6]), "v"(win.q[7]), "v"(win.q[8]), "v"(win.q[9]), "v"(win.q[10]),
               "v"(win.q[11]));
  if (a < 0) {
    if (status) status[b] = ST_NOOP;
    return;
  }
  StreamDraw<WinMT12> d{WinMT12(mt + (size_t)b * kMT, c0)};
  if (phase_of(s.misc) == PH_P3) win_take(pw, win, d.m, c0);
  int r = step_state(s, a, d);
  if (r == ST_OK) {
    store_state(st, n, b, s);
    win_prepare(pw, d.m, b, phase_of(s.misc));
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
                                                int16_t *__restrict__ action, int32_t *__restrict__ status,
                                                PlyWin pw) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  State s = load_state(st, n, b);
  const int c0 = pos[b];
  const PlyWinIn win = win_load(pw, b);
  // the rule's inputs loaded with the state: read after the mask stores, they
  // were a second dependent memory round trip on every ply
  const int p = ply[b];
  const uint64_t sd = seed[b];
  StreamDraw<WinMT12> d{WinMT12(mt + (size_t)b * kMT, c0)};
  // a third placement ends the turn, whose refill draws: from the words the
  // previous ply saved (PlyWin), or else the stream's read-ahead window (and
  // the twist it may need) fetched now, under the legal-mask and rule work
  const bool early = phase_of(s.misc) == PH_P3 && !game_done(s.misc);
  if (early) {
    win_take(pw, win, d.m, c0);
    d.m.prefetch();  // (a no-op after win_take)
  }
  uint64_t m[3];
  int c = legal_mask(s, m);
  if (game_done(s.misc)) { m[0] = m[1] = m[2] = 0; c = 0; }
  if (mask) {
    mask[(size_t)b * 3 + 0] = m[0];
    mask[(size_t)b * 3 + 1] = m[1];
    mask[(size_t)b * 3 + 2] = m[2];
  }
  if (count) count[b] = c;
  const int a = c > 0 ? kth_action(m, rule_pick(sd, p, c)) : -1;
  if (action) action[b] = (int16_t)a;
  if (a < 0) {
    // (the early prefetch may have twisted words in place: its cursor, the
    // same stream position, goes back with them)
    if (early) pos[b] = d.m.cursor();
    if (status) status[b] = ST_NOOP;
    return;
  }
  int r = step_state(s, a, d);
  if (r == ST_OK) {
    store_state(st, n, b, s);
    win_prepare(pw, d.m, b, phase_of(s.misc));
    ply[b] = p + 1;
  }
  if (r == ST_OK || early) pos[b] = d.m.cursor();
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

// ------------------------------------------------- auto-reset chance-ahead
// hz_rollout(auto_reset = 1) plays every board on and on, starting its next
// episode (seed_base + b + (e << 32)) whenever a game ends: about 1.5 game
// ends per board per 96-ply call.  Seeding a stream is a 1,246-step serial
// chain (~60 k cycles); in-kernel, the wave of a board whose game ended had
// to wait for it.  As with hz_play's chance-ahead, a game's chance sequence
// does not depend on its moves, so extra blocks of each auto-reset launch
// prepare every board's episodes e0 + 2 and e0 + 3 (e0 = the board's episode
// counter when the call starts: it starts e0 and at most e0 + 1 in the call
// when it takes prepared ones) into a ring of four slots by episode: the
// stream seeded and pre-twisted, its first kAheadDraws pile draws from the
// initial bag run into a script with the cursor after each draw, the stream
// after them.  A board whose game ends then starts episode e from slot e & 3
// when the slot's tag says e (prepared by an earlier call: this call's blocks
// write slots e0 + 2, e0 + 3, never the ones it reads) and e - e0 < 2: a
// scripted reset, no chain, no wait for the rest of the wave; otherwise it
// seeds in place as before.  A slot is tagged only when none of its draws
// twisted past the pre-twisted rows, so the stream as stored and every cursor
// agree (materialize copies it to the board's own stream after the call).
// The preparation only decides where a board's chance draws come from, never
// what they are: results are the same with it off (hz_env_set_auto_ahead).
constexpr int kArSlots = 4;
constexpr int kArSrc = 16;  // mt_src codes kArSrc + slot (0, 1: pipeline 1; 2..15: pipeline 2)
struct ArArgs {
  uint32_t *mt;          // [kArSlots][n][624]
  int32_t *tag;          // [kArSlots][n]
  uint64_t *pile;        // [kArSlots][kAheadWords][n]
  int32_t *cur;          // [kArSlots][kAheadDraws + 1][n]
  const int32_t *ep_in;  // [n] the counters the previous call ended with (the preparing blocks' e0)
  int on;
};

__device__ __forceinline__ void ar_prep_stage(int blk, int k, const ArArgs &ar, int n, uint64_t seed_base) {
  __shared__ uint64_t s_ar_mask[kArSlots];
  const int tid = threadIdx.x, lane = tid & 63, b0 = blk * kBlock, b = b0 + lane;
  const bool act = b < n;
  const int nb = n - b0 < kBlock ? n - b0 : kBlock;
  const int e = act ? ar.ep_in[b] + 2 + k : 0;
  const int sl = e & (kArSlots - 1);
  const bool need = act && ar.tag[(size_t)sl * n + b] != e;  // (prepared by an earlier call: kept)
  if (tid < 64) {
#pragma unroll
    for (int q = 0; q < kArSlots; q++) {
      const uint64_t m = __ballot(need && sl == q);
      if (lane == 0) s_ar_mask[q] = m;
    }
    if (need) {
      seed_in_lds(lane, episode_seed(seed_base, b, e));
      uint64_t bag = initial_bag(), q[kAheadWords] = {};
      int32_t *cur = ar.cur + (size_t)sl * (kAheadDraws + 1) * n + b;
      cur[0] = kMTAhead;
      StreamDraw<LdsMT> d{LdsMT(lane, kMTAhead)};
      run_script(d, bag, q, cur, n, 0, kAheadDraws);
      // the stored stream matches every cursor only if no draw twisted past
      // the pre-twisted rows (a bag of >= 48 tiles: in practice never)
      const bool clean = d.m.tw == kAheadTwist;
#pragma unroll
      for (int w = 0; w < kAheadWords; w++) ar.pile[((size_t)sl * kAheadWords + w) * n + b] = q[w];
      ar.tag[(size_t)sl * n + b] = clean ? e : -1;
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int q = 0; q < kArSlots; q++) {
    const uint64_t m = s_ar_mask[q];
    if (m) stage_mt(ar.mt + ((size_t)q * n + b0) * kMT, nb, tid, m, false);
  }
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
                                                    int src_slot, ArArgs ar) {
#ifdef HZ_DIAG
  uint64_t role_t0 = __builtin_amdgcn_s_memtime();
#endif
  if ((int)blockIdx.x >= nblk) {  // chance-ahead roles (uniform per block)
    int blk = (int)blockIdx.x - nblk;
    int role = blk / nblk;
    blk -= role * nblk;
    if constexpr (AutoReset && !Record) {
      if (ar.on) {  // hz_rollout's auto-reset preparation: episodes e0 + 2 (role 0), e0 + 3 (role 1)
        ar_prep_stage(blk, role, ar, n, seed_base);
        return;
      }
    }
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
    // where the lane's scripted stream lives: the play slot of a prepared
    // hz_play episode, or an auto-reset slot (set below when one is taken)
    const int32_t *cur_b = ahead_cur ? ahead_cur + b : nullptr;
    int src_b = src_slot;
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
    if constexpr (AutoReset) {
      // A board whose game ends starts its next episode: seeding its stream
      // is a 1,246-step chain (~60 k cycles) that the whole wave waits for.
      // Each lane counts its own plies (used), and a lane whose game ended
      // waits until no lane of the wave can play on; then every waiting lane
      // seeds together, in one pass, and play resumes.  Every board plays the
      // same plies in the same order as with a reset at its own ply (lanes
      // share nothing), so results are the same; the wave seeds once or
      // twice per launch instead of once per distinct game end.
      int used = 0;
      bool stuck = false;
#ifdef HZ_DIAG_ROLES_ONLY
      int n_pass = 0, n_iter = 0;
#endif
      while (true) {
        if constexpr (!Record) {
          // a prepared episode (ar_prep_stage): a scripted reset at once, the
          // lane's own, with no seeding pass for the wave to wait for
          if (ar.on && phase_of(s.misc) == PH_OVER && !stuck && used < max_plies) {
            const int e = episode[b];
            const int sl = e & (kArSlots - 1);
            if (e - ep0 < 2 && ar.tag[(size_t)sl * n + b] == e) {
              if (score_pending(s.misc)) finish_game(s);  // the finished game is scored all the same
              const uint64_t *pq = ar.pile + (size_t)sl * kAheadWords * n + b;
              draw.q0 = pq[0];
              draw.q1 = pq[(size_t)n];
              draw.q2 = pq[(size_t)2 * n];
              draw.q3 = pq[(size_t)3 * n];
              draw.scripted = true;
              draw.fell = false;
              draw.d = 0;
              draw.nd = kAheadDraws;
              draw.gm = MT(ar.mt + ((size_t)sl * n + b) * kMT, 0);
              cur_b = ar.cur + (size_t)sl * (kAheadDraws + 1) * n + b;
              draw.cur_tail = cur_b + (size_t)kAheadDraws * n;
              src_b = kArSrc + sl;
              sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
              rkey = rule_key(sd);
              episode[b] = e + 1;
              lds_used = false;
              pre = false;
              draw.scripted_reset(s);
              g_ply = 0;
            }
          }
        }
        const bool over = phase_of(s.misc) == PH_OVER;
        const bool can = !over && !stuck && used < max_plies;
#ifdef HZ_DIAG_ROLES_ONLY
        n_iter++;
#endif
        if (!__any(can)) {
          const bool want = over && !stuck && used < max_plies;
          if (!__any(want)) break;
#ifdef HZ_DIAG_ROLES_ONLY
          n_pass++;
#endif
          if (want) {  // the next episode of every waiting board, seeded together
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
          continue;
        }
        if (!can) continue;
        if constexpr (!Record) {
          // a pair of whole turns at once while every playing board of the
          // wave is at a pair boundary with 8 plies of budget
          if (__all(used + 8 <= max_plies && turn_pair_safe(s))) {
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
            used += done;
            if (phase_of(s.misc) == PH_OVER) games++;
            continue;
          }
        }
        int a;
        if constexpr (Record) {
          uint64_t mk[3];
          int L = legal_mask(s, mk);
          if (traj_state) {
            uint64_t *o = traj_state + (size_t)used * 6 * n + b;
            o[0] = s.pl[0]; o[(size_t)n] = s.pl[1]; o[(size_t)2 * n] = s.pl[2]; o[(size_t)3 * n] = s.pl[3];
            o[(size_t)4 * n] = s.piles; o[(size_t)5 * n] = s.misc;
          }
          if (traj_mask) {
            uint64_t *o = traj_mask + ((size_t)used * n + b) * 3;
            o[0] = mk[0]; o[1] = mk[1]; o[2] = mk[2];
          }
          a = L ? kth_action(mk, rule_pick_k(rkey, g_ply, L)) : -1;
          if (traj_action) traj_action[(size_t)used * n + b] = (int16_t)a;
        } else {
          a = rule_action(s, rule_h32(rkey, g_ply));  // legal mask + rule pick, fused
        }
        if (a < 0) {  // stuck board (unreachable from HarmoniesGameState())
          stuck = true;
          continue;
        }
        step_trusted<true>(s, a, draw);
        g_ply++;
        steps++;
        used++;
        if (phase_of(s.misc) == PH_OVER) games++;
      }
#ifdef HZ_DIAG_ROLES_ONLY
      if (g_stamps && lane == 0) {  // the wave's reseeding passes and loop iterations (tools/ar_passes.py)
        g_stamps[(size_t)b * 16 + 11] = n_pass;
        g_stamps[(size_t)b * 16 + 12] = n_iter;
      }
#endif
    } else {
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
    else pos[b] = cur_b[(size_t)draw.d * n];
    mt_src[b] = lds_used ? -1 : src_b;
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
// longest chain.  Here every board's episode is cut into thirteen stages of
// 20-30 k cycles, one per consecutive hz_play call, and one launch runs all
// thirteen at once, each on a different episode of the board (ep = the
// episode counter the previous call left, p2_ep; stage s works on episode
// ep + 12 - s):
//   s = 0  P1a   seeding pass 1, steps 1-312          draw-Y blocks, wave 2
//   s = 1  P1b   pass 1, steps 313-624                draw-X blocks, wave 2
//   s = 2  P2a   pass 2, steps 2-208                  seed blocks, wave 0
//   s = 3  P2b   pass 2, steps 209-416                seed blocks, wave 1
//   s = 4  P2c   pass 2, steps 417-624; rows 0-223    seed blocks, wave 2
//                of the next generation twisted       (twist: wave 3)
//   s = 5  D1    pile draws 0-5                       draw-X blocks, wave 0
//   s = 6  D2    draws 6-11                           draw-X blocks, wave 1
//   s = 7  D3    draws 12-17                          draw-Y blocks, wave 0
//   s = 8  D4    draws 18-23                          draw-Y blocks, wave 1
//          (the episode's rule hashes meanwhile:      draw-X blocks, wave 3)
//   s = 9  playA plies [0, cut0)                      play blocks, wave 3
//   s = 10 playB plies [cut0, cut1)                   play blocks, wave 2
//   s = 11 playC plies [cut1, cut2)                   play blocks, wave 1
//   s = 12 playD the rest, final scoring, the board's play blocks, wave 0
//                state, cursor and counters
// An episode's stream lives in one slot of a ring of kP2Stream from P1a to
// playD (and afterwards as the board's current stream until materialize or
// the next call); stage s of call c uses slot (c - s) mod kP2Stream.  A stage
// uses an input only when its tag names the stage's episode, so a wrong
// prediction costs time, never results: the stages skip the board and playD
// plays its whole game from scratch (seeding and drawing in LDS, like
// k_rollout's unprepared boards).  The results are k_rollout's: the board ends
// the call with episode ep's final state, cursor and counters, and
// games_done / steps_done count that game (its first plies ran in the three
// calls before, in playA, playB and playC).  In steady state a call does
// every stage once per board: one game's worth of work per board per call.
#ifndef HZ_P2_ST_WT
// 1: the hand-off stores (hashes, cursors, scripts, mid-game states) write-
// through too (global_store ... sc1): 17.0 G against 18.3 G with them plain
// (profiles/r05/p2_writethrough), so plain by default
#define HZ_P2_ST_WT 0
#endif
#ifndef HZ_P2_AUX
// cache policy of the seeding stages' and the twist's stream-slot stores
// (~24 MB per 4096-board launch): 16 = sc1, write-through, the line dropped
// from the XCD's L2 (the next call's stages read them, from the MALL), so
// the kernel's end finds no dirty slot lines to write back: 14.1 vs 15.8 us
// per launch against plain stores (0), 15.5 with nt (2)
// (profiles/r05/p2_writethrough; A/B builds -DHZ_P2_AUX=0 / 2)
#define HZ_P2_AUX 16
#endif
constexpr int kP2Win = 96;        // rows a draw stage stages, from its wave's lowest cursor
constexpr int kP2WinRows = kP2Win + 24;  // LDS rows per window (a scan reads up to 23 rows past its cursor)
constexpr int kP2Play = 4;        // play stages
constexpr int kP2Stages = 9 + kP2Play;
constexpr int kP2Last = kP2Stages - 1;  // stage s works on episode ep + kP2Last - s
constexpr int kP2Ring = kP2Play + 1;    // D4's scripts and the rule hashes: read by the play stages 1..kP2Play calls later
constexpr int kP2Stream = 14;     // stream slots (>= kP2Stages + 1: the last play stage's slot stays the board's stream)
constexpr int kP2DrawsPer = 6;    // pile draws per draw stage (4 x 6 = kAheadDraws)
#ifndef HZ_P2_DCUT
// the draw stages' first draws: D1 0-6, D2 7-12, D3 13-17, D4 18-23.  With
// six each, D3 was the longest stage (13.8 us against 10.5 for D1) once the
// slot stores were written through: 19.37 vs 18.24 G env-steps/s, 13.2 vs
// 14.1 us per launch (profiles/r05/p2_dcut; A/B builds -DHZ_P2_DCUT=...)
#define HZ_P2_DCUT 0, 7, 13, 18
#endif
constexpr int kP2DCut[4] = {HZ_P2_DCUT};
constexpr int kP2MinPlies = 96;   // hz_play max_plies from which pipeline 2 applies (rule games end by ply 80)
constexpr int kP1Split = 313;
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
#endif     // pass 1: P1a runs steps [1, 313), P1b [313, 624) and the 624th
static_assert(4 * kP2DrawsPer == kAheadDraws, "four draw stages cover the script");
static_assert(2 * kP2WinRows * kLdsStride * 4 <= (int)kResetLds, "two windows per draw block");
static_assert((kP1Split - 1) % 8 == 0 && (617 - kP1Split) % 8 == 0, "pass-1 halves in groups of eight");

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
  uint32_t *s_mt[kP2Stages];  // the stream slot of each stage this call
  int32_t *s_tag[kP2Stages];  // [nrow] episode * 8 + 1 P1a / 2 pass 1 / 3 P2a / 4 P2b / 5 seeded, rows 0-223 twisted
  int32_t *s_cur[kP2Stages];  // [kAheadDraws + 1][nrow] cursor before draw 0 and after each draw
  int s_idx_last;             // the last play stage's slot index (materialize: mt_src = 2 + index)
  uint32_t *p1h_w;            // [nrow] P1a -> P1b: pass 1's last value
  const uint32_t *p1h_r;
  uint32_t *p2h_w;            // [3][nrow] P2a -> P2b: pass 2's last value, pass 1's row-1 word, row 2's final word
  const uint32_t *p2h_r;
  uint32_t *p3h_w;            // [2][nrow] P2b -> P2c: the same
  const uint32_t *p3h_r;
  P2Draw x_w[3], x_r[3];      // D1 -> D2 -> D3 -> D4 (tag: episode * 8 + stages done)
  P2Draw pl_w, pl_r[kP2Play];     // D4's script: written this call; read by play stage st (st + 1 calls later)
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
  MTR gm;                  // valid once fell
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
      gm = MTR(gm.w, gm.stride, *cur_nd);
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
// init_by_array's pass 1, steps [i0, i1) (i0 odd, groups of eight: odd
// steps take key word kA, even ones kB), rows at w[i * ns]; step 1's value
// goes to row 1 (the 624th step reads it back)
// (wb = the slot's column of the wave's first board, wave-uniform, so a
// row's address is a scalar base plus the lane: no 64-bit address
// arithmetic per step in the chain)
// the slot's columns of boards [b0, b0 + 64) as a buffer (rows of nr words)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t p2_slot_rsrc(uint32_t *slot, int b0, size_t nr) {
  const uint64_t base = (uint64_t)(slot + b0);
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base), hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)((size_t)kMT * nr * 4 - (size_t)b0 * 4));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}
#ifndef HZ_P2_LDNT
#define HZ_P2_LDNT 0  // 1: the stages' 16-B slot reads (staging, windows, the twist's rows) non-temporal (A/B builds)
#endif
__device__ __forceinline__ uint4 p2_ld4(const uint32_t *p) {
  if constexpr (HZ_P2_LDNT) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load((const v4u *)p);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const uint4 *>(p);
}
// a store read by another stage in a later call only: write-through (sc1)
// like the slot stores (HZ_P2_AUX), so the kernel's end has no dirty lines
// of it to write back
template <class T>
__device__ __forceinline__ void p2_st(T *p, T v) {
  if constexpr (HZ_P2_AUX == 16 && HZ_P2_ST_WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
// (the stream slots' stores: written by one stage, read by another in the
// next call, never by this one: HZ_P2_AUX write-through (sc1) leaves no
// dirty lines in the XCD's L2 for the end of the kernel to write back)
__device__ __forceinline__ void mt_pass1_span(uint32_t *__restrict__ slot, int b0, int lane, size_t ns, uint32_t kA,
                                              uint32_t kB, int i0, int i1, uint32_t &prev) {
  const __amdgpu_buffer_rsrc_t rs = p2_slot_rsrc(slot, b0, ns);
  const int row_bytes = __builtin_amdgcn_readfirstlane((int)(ns * 4));
  // init_genrand's table words a group ahead (scalar loads: their wait
  // would otherwise sit in the chain once per group)
  uint32_t iv[8];
#pragma unroll
  for (int u = 0; u < 8; u++) iv[u] = kInitGen.v[i0 + u];
#pragma unroll 1
  for (int g = i0; g < i1; g += 8) {
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = kInitGen.v[g + 8 + u < kMT ? g + 8 + u : kMT - 1];
    const int soff = __builtin_amdgcn_readfirstlane(g * row_bytes);
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, soff + u * row_bytes, HZ_P2_AUX);
      prev = v;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = nx[u];
  }
}
__device__ __forceinline__ void p2_keys(uint64_t seed, uint32_t &kA, uint32_t &kB) {
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  kA = key0;
  kB = key1 ? key1 + 1u : key0;
}

// P1a (seed blocks, wave 0) and P1b (draw-X blocks, wave 2): no LDS
__device__ __forceinline__ void p2_p1a(const P2Args &a, int b0, int lane) {
  const int b = b0 + lane;
  const size_t nr = (size_t)a.nrow;
  const int e = a.ep_in[b] + kP2Last;
  uint32_t kA, kB;
  p2_keys(episode_seed(a.seed_base, b, e), kA, kB);
  uint32_t prev = 19650218u;
  mt_pass1_span(a.s_mt[0], b0, lane, nr, kA, kB, 1, kP1Split, prev);
  a.p1h_w[b] = prev;
  a.s_tag[0][b] = e * 8 + 1;
}
__device__ __forceinline__ void p2_p1b(const P2Args &a, int b0, int lane) {
  const int b = b0 + lane;
  const size_t nr = (size_t)a.nrow;
  const int e = a.ep_in[b] + kP2Last - 1;
  if (a.s_tag[1][b] != e * 8 + 1) return;
  uint32_t kA, kB;
  p2_keys(episode_seed(a.seed_base, b, e), kA, kB);
  uint32_t prev = a.p1h_r[b];
  const uint32_t *w = a.s_mt[1] + b;
  const uint32_t row1 = w[nr];  // (P1a's step-1 word, read before any store of this wave)
  mt_pass1_span(a.s_mt[1], b0, lane, nr, kA, kB, kP1Split, 617, prev);
  const __amdgpu_buffer_rsrc_t rs = p2_slot_rsrc(a.s_mt[1], b0, nr);
  const int row_bytes = __builtin_amdgcn_readfirstlane((int)(nr * 4));
#pragma unroll
  for (int u = 0; u < 7; u++) {  // steps 617..623
    const uint32_t v = (kInitGen.v[617 + u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, (617 + u) * row_bytes, HZ_P2_AUX);
    prev = v;
  }
  // mt[0] = mt[623]; the 624th step at i = 1 (key j = 623 % keylen -> kB)
  __builtin_amdgcn_raw_buffer_store_b32((row1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB, rs, lane * 4, row_bytes,
                                        HZ_P2_AUX);
  a.s_tag[1][b] = e * 8 + 2;
}

// Pass 2 in three stages, P2a (steps 2-208), P2b (209-416) and P2c
// (417-623 and the last step at i = 1), in one seed block on disjoint rows
// of its [624][65] LDS array (the rows of three different episodes).  Every
// step reads the next pass-1 word, too close ahead for an HBM round trip (a
// chain reading the slot through a register ring stalled on the memory
// counter: ~220 k cycles per half), so each chain first stages its third of
// the pass-1 words into its own rows (all loads in flight at once), then
// runs on LDS reads, storing each final word to the slot with a buffer store
// (the row offset a scalar: no address arithmetic in the chain).  A chain
// step costs ~70 cycles with one wave per SIMD (the four dependent VALU
// operations of the recurrence plus the step's memory instructions; staging
// transposed, four words per LDS access, changed nothing), so the chain is
// cut into thirds rather than made cheaper per step.
constexpr int kP2aEnd = 209, kP2bEnd = 417;
constexpr int kTwKeep = 397;  // P2c's final rows from here on stay in LDS (the twist reads rows 397-620)
// Rows [R0, R1) of the wave's 64 boards staged from the slot into LDS, in
// two halves: p2_load issues the 16-B loads (four boards of a row per lane,
// four rows per instruction) into registers, p2_put writes them to LDS.  A
// pass-2 stage stages its first piece, issues the next piece's loads and
// runs its chain over the first piece while they land: two thirds of the
// staging reads leave the launch's opening burst, where every stage's first
// inputs arrive.
template <int R0, int R1>
struct P2Piece {
  uint4 v[(R1 - R0 + 3) / 4];
};
template <int R0, int R1>
__device__ __forceinline__ void p2_load(P2Piece<R0, R1> &pc, const uint32_t *__restrict__ slot, size_t nr, int b0,
                                        int lane) {
  constexpr int U = (R1 - R0 + 3) / 4;
  const int c4 = (lane & 15) * 4;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int r = R0 + 4 * u + (lane >> 4);
    if (r < R1) pc.v[u] = p2_ld4(slot + (size_t)r * nr + b0 + c4);
  }
}
template <int R0, int R1>
__device__ __forceinline__ void p2_put(const P2Piece<R0, R1> &pc, int lane) {
  constexpr int U = (R1 - R0 + 3) / 4;
  const int c4 = (lane & 15) * 4;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int r = R0 + 4 * u + (lane >> 4);
    if (r < R1) {
      uint32_t *d = hz_lds + r * kLdsStride + c4;
      d[0] = pc.v[u].x;
      d[1] = pc.v[u].y;
      d[2] = pc.v[u].z;
      d[3] = pc.v[u].w;
    }
  }
  // (a wave's LDS operations execute in order: its later reads see these)
}
// twist_word(cur, next, far) = far ^ twist_part(cur, next): the part of row
// r's next-generation word that rows r and r + 1 decide
__device__ __forceinline__ uint32_t twist_part(uint32_t cur, uint32_t next) {
  const uint32_t y = (cur & 0x80000000U) | (next & 0x7fffffffU);
  return (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
}
// What a pass-2 step stores: its final word to its row (kP2Final), the same
// and over the pass-1 word in LDS (kP2Keep, P2c), or the previous row's
// twist part (kP2Part: rows 2-223, which only the twist reads)
enum { kP2Final = 0, kP2Keep = 1, kP2Part = 2 };
// steps [G0, G1) of pass 2 (G1 - G0 a multiple of 8) on the lane's LDS
// column, pass-1 words read 8 steps ahead (rows below G1), stores to the
// slot (buffer stores: voffset the lane, soffset the row) as Mode says (in
// LDS in place: the read-ahead is always past the rows written), with
// kP2Keep publishing progress every 8 steps
template <int G0, int G1, int Mode>
__device__ __forceinline__ void p2_span(int lane, __amdgpu_buffer_rsrc_t rs, int row_bytes, uint32_t &prev,
                                        int *prog) {
  constexpr bool KeepLds = Mode == kP2Keep;
  static_assert((G1 - G0) % 8 == 0, "groups of eight");
  uint32_t *l = hz_lds + lane;
  constexpr int S = kLdsStride;
  uint32_t cur[8];
#pragma unroll
  for (int u = 0; u < 8; u++) cur[u] = l[(G0 + u) * S];
#pragma unroll 2
  for (int g = G0; g < G1; g += 8) {
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = l[(g + 8 + u < G1 ? g + 8 + u : G1 - 1) * S];
    const uint32_t kneg = __builtin_amdgcn_readfirstlane(0u - (uint32_t)g);
    const int soff = __builtin_amdgcn_readfirstlane((Mode == kP2Part ? g - 1 : g) * row_bytes);
#pragma unroll
    for (int u = 0; u < 8; u++) {
      // (cur ^ p) - (g + u) as one v_xad_u32 with the offset in an SGPR
      const uint32_t p = (prev ^ (prev >> 30)) * 1566083941U;
      uint32_t v;
      asm("v_xad_u32 %0, %1, %2, %3" : "=v"(v) : "v"(p), "v"(cur[u]), "s"(kneg - (uint32_t)u));
      __builtin_amdgcn_raw_buffer_store_b32(Mode == kP2Part ? twist_part(prev, v) : v, rs, lane * 4,
                                            soff + u * row_bytes, HZ_P2_AUX);
      if (KeepLds) l[(g + u) * S] = v;
      prev = v;
    }
    if (KeepLds) p2_publish(prog, g + 8);  // rows [G0, g + 8) final in LDS
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = nx[u];
  }
}
// the last steps [G, G1) one by one
template <int G, int G1, int Mode>
__device__ __forceinline__ void p2_tail(int lane, __amdgpu_buffer_rsrc_t rs, int row_bytes, uint32_t &prev) {
#pragma unroll
  for (int i = G; i < G1; i++) {
    const uint32_t v = (hz_lds[i * kLdsStride + lane] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)i;
    if (Mode == kP2Part) __builtin_amdgcn_raw_buffer_store_b32(twist_part(prev, v), rs, lane * 4, (i - 1) * row_bytes, HZ_P2_AUX);
    else __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, i * row_bytes, HZ_P2_AUX);
    if (Mode == kP2Keep) hz_lds[i * kLdsStride + lane] = v;
    prev = v;
  }
}

// P2a (seed blocks, wave 0): the seed blocks' P2a episode, whose pass 1
// completed in the previous call; P2b (wave 1) the next older; P2c (wave 2,
// with wave 3's twist) the one before.  Each hands (prev, pass 1's row-1
// word, row 2's final word) to the next.  Rows 2-223 of the slot are read
// only by the twist, which needs from each row r only its twist part
// (rows r and r + 1's words): P2a and P2b store that instead of the final
// word (one step late, when row r + 1 is known), so the twist is one xor
// per word with the far row.  (e, ok: the board's episode and whether the
// stage's input is this episode's, read by every wave of the block before
// its barrier, so before P2c rewrites its tag.)
template <int K>  // 0 P2a, 1 P2b, 2 P2c
__device__ __forceinline__ void p2_third(const P2Args &a, int b0, int lane, int e, bool ok, int *s_prog) {
  const int b = b0 + lane;
  const bool act = b < a.n;
  const size_t nr = (size_t)a.nrow;
  if (!__any(ok)) {
    if (K == 2) p2_publish(s_prog, kMT + 1);  // (the twist wave's waits end: nothing to twist)
    return;
  }
  uint32_t *slot = a.s_mt[2 + K];
#ifdef HZ_DIAG
  const uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
  // the stage's rows in three pieces, P0 staged now; each later piece's
  // loads issued before the chain runs over the piece before it
  constexpr int P0 = K == 0 ? 1 : K == 1 ? kP2aEnd : kP2bEnd;
  constexpr int P1 = K == 0 ? 67 : K == 1 ? 289 : 481;
  constexpr int P2 = K == 0 ? 139 : K == 1 ? 353 : 553;
  constexpr int P3 = K == 0 ? kP2aEnd : K == 1 ? kP2bEnd : kMT;
  {
    P2Piece<P0, P1> pc;
    p2_load(pc, slot, nr, b0, lane);
    p2_put(pc, lane);
  }
  P2Piece<P1, P2> pc1;
  p2_load(pc1, slot, nr, b0, lane);
#ifdef HZ_DIAG
  if (g_stamps && act) g_stamps[(size_t)b * kP2Stamps + 32 + K] = __builtin_amdgcn_s_memtime() - tq;  // staged
#endif
  uint32_t prev, first1, row2;
  if (K == 0) {
    first1 = hz_lds[1 * kLdsStride + lane];
    prev = first1;
  } else {
    const uint32_t *h = K == 1 ? a.p2h_r : a.p3h_r;
    prev = act ? h[b] : 0u;
    first1 = act ? h[nr + b] : 0u;
    row2 = act ? h[2 * nr + b] : 0u;
  }
  const __amdgpu_buffer_rsrc_t rs = p2_slot_rsrc(slot, b0, nr);
  const int row_bytes = (int)(nr * 4);
  P2Piece<P2, P3> pc2;
  if constexpr (K == 0) {  // step 2: row 2's final word, handed on (row 1's part needs row 1, P2c's last step)
    row2 = (hz_lds[2 * kLdsStride + lane] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 2U;
    prev = row2;
    p2_span<3, P1, kP2Part>(lane, rs, row_bytes, prev, s_prog);  // parts of rows 2 ..
    p2_put(pc1, lane);
    p2_load(pc2, slot, nr, b0, lane);
    p2_span<P1, P2, kP2Part>(lane, rs, row_bytes, prev, s_prog);
    p2_put(pc2, lane);
    constexpr int G = P2 + 8 * ((kP2aEnd - P2) / 8);
    p2_span<P2, G, kP2Part>(lane, rs, row_bytes, prev, s_prog);
    p2_tail<G, kP2aEnd, kP2Part>(lane, rs, row_bytes, prev);    // .. 207
  } else if constexpr (K == 1) {
    static_assert(kAheadTwist + 1 - kP2aEnd == 16, "P2b's part steps: two groups");
    p2_span<kP2aEnd, kAheadTwist + 1, kP2Part>(lane, rs, row_bytes, prev, s_prog);  // parts of rows 208-223
    __builtin_amdgcn_raw_buffer_store_b32(prev, rs, lane * 4, kAheadTwist * row_bytes, HZ_P2_AUX);  // row 224's final word
    p2_span<kAheadTwist + 1, P1, kP2Final>(lane, rs, row_bytes, prev, s_prog);
    p2_put(pc1, lane);
    p2_load(pc2, slot, nr, b0, lane);
    p2_span<P1, P2, kP2Final>(lane, rs, row_bytes, prev, s_prog);
    p2_put(pc2, lane);
    p2_span<P2, kP2bEnd, kP2Final>(lane, rs, row_bytes, prev, s_prog);
  } else {
    // rows 0 and 1 of the next generation are P2c's own last words: their
    // far rows (397, 398: P2b's) loaded now, used after the chain
    const uint32_t f0 = act ? slot[(size_t)397 * nr + b] : 0u, f1 = act ? slot[(size_t)398 * nr + b] : 0u;
    p2_span<kP2bEnd, P1, kP2Keep>(lane, rs, row_bytes, prev, s_prog);
    p2_put(pc1, lane);
    p2_load(pc2, slot, nr, b0, lane);
    p2_span<P1, P2, kP2Keep>(lane, rs, row_bytes, prev, s_prog);
    p2_put(pc2, lane);
    constexpr int G = P2 + 8 * ((kMT - P2) / 8);
    p2_span<P2, G, kP2Keep>(lane, rs, row_bytes, prev, s_prog);
    p2_tail<G, kMT, kP2Keep>(lane, rs, row_bytes, prev);
    p2_publish(s_prog, kMT);
    const uint32_t row1 = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;  // the last step, at i = 1
    // mt[0] = 0x80000000 after init_by_array; row 1's next row is row 2
    __builtin_amdgcn_raw_buffer_store_b32(f0 ^ twist_part(0x80000000u, row1), rs, lane * 4, 0, HZ_P2_AUX);
    __builtin_amdgcn_raw_buffer_store_b32(f1 ^ twist_part(row1, row2), rs, lane * 4, row_bytes, HZ_P2_AUX);
  }
  if (K < 2) {
    if (ok) {
      uint32_t *h = K == 0 ? a.p2h_w : a.p3h_w;
      h[b] = prev;
      h[nr + b] = first1;
      h[2 * nr + b] = row2;
      a.s_tag[2 + K][b] = e * 8 + 3 + K;
    }
  } else if (ok) {
    a.s_tag[4][b] = e * 8 + 5;
  }
}

// The twist (seed blocks, wave 3): rows [0, kAheadTwist) of the next
// generation into P2c's slot (the stream at cursor kMTAhead): row r's new
// word is the far row r + 397 (P2b's below row 417, from HBM; P2c's from
// LDS) xor row r's twist part, which P2a and P2b left in the slot (rows
// 2-223).  Lane: four boards, rows grp + 4 i, grp = lane / 16, so iteration
// i needs P2c's rows up to 4 i + 400 and follows P2c's progress (s_prog),
// two iterations per publish of P2c's; rows 0 and 1 (from row 1, P2c's last
// step, and row 2's final word) are P2c's own.  All its loads precede its
// stores.  (Before the parts, the wave shuffled each row's
// successor in from the next lane group and ran at ~350 cycles per
// iteration, ending ~8 k cycles after P2c: profiles/r04/p2/.)
constexpr int kTwIters = kAheadTwist / 4;
constexpr int kTwHbm = (kP2bEnd - 397 + 3) / 4;  // iterations whose rows r + 397 are P2b's (HBM)
__device__ __forceinline__ uint4 xor4(const uint4 &a, const uint4 &b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ void p2_twist(const P2Args &a, int b0, int lane, bool any, int *s_prog) {
  if (!any) return;
  const size_t nr = (size_t)a.nrow;
  uint32_t *slot = a.s_mt[4];
  const int grp = lane >> 4, c4 = (lane & 15) * 4;
  uint32_t *col = slot + b0 + c4;
  auto row = [&](int r) { return p2_ld4(col + (size_t)r * nr); };
  const __amdgpu_buffer_rsrc_t rs = p2_slot_rsrc(slot, b0, nr);
  const int row_bytes = __builtin_amdgcn_readfirstlane((int)(nr * 4));
  auto store = [&](int r, const uint4 &v) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    // (r = grp + 4 i differs across the lane groups: per-lane voffset, no soffset)
    __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, rs, c4 * 4 + r * row_bytes, 0, HZ_P2_AUX);
  };
#ifdef HZ_DIAG
  const int b = b0 + lane;
  const uint64_t tz = __builtin_amdgcn_s_memtime();
#endif
  // (the wave has ~16 k cycles of slack: its 4 MB of loads wait until P2c is
  // 64 rows in, out of the launch's opening burst, where every other
  // stage's inputs arrive)
  int have = p2_wait(s_prog, kP2bEnd + 64, a.spin, a.err);
  P2_PHASE(35, tz);
  uint4 pt[kTwIters], fh[kTwHbm];
#pragma unroll
  for (int i = 0; i < kTwIters; i++) {
    const int r = grp + 4 * i;
    pt[i] = r >= 2 ? row(r) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < kTwHbm; i++) {
    const int r = grp + 4 * i + 397;
    fh[i] = r < kP2bEnd ? row(r) : make_uint4(0, 0, 0, 0);
  }
  auto far = [&](int i) -> uint4 {
    const int r = grp + 4 * i;
    if (i < kTwHbm && r + 397 < kP2bEnd) return fh[i < kTwHbm ? i : 0];
    const uint32_t *d = hz_lds + (r + 397) * kLdsStride + c4;
    return make_uint4(d[0], d[1], d[2], d[3]);
  };
#pragma unroll
  for (int i = 0; i < kTwIters; i += 2) {
    const int need = 4 * (i + 1) + 3 + 397 + 1;  // the pair's far rows final
    if (need > kP2bEnd && have < need) have = p2_wait(s_prog, need, a.spin, a.err);
    const uint4 f0 = far(i), f1 = far(i + 1);
    if (i > 0 || grp >= 2) store(grp + 4 * i, xor4(f0, pt[i]));
    store(grp + 4 * (i + 1), xor4(f1, pt[i + 1]));
    if (i == 0) P2_PHASE(36, tz);
  }
  P2_PHASE(37, tz);
  // (rows 224..623 keep pass 2's words: the current generation's tail)
}

// seed blocks: waves 0-2 P2a, P2b, P2c; wave 3 the twist of P2c's episode
__device__ __forceinline__ void p2_seed(const P2Args &a, int blk) {
  __shared__ int s_prog;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock, b = b0 + lane;
  const bool act = b < a.n;
  if (tid == 0) s_prog = 0;
  // each stage's episode and decision (and P2c's for the twist wave), read
  // before the barrier, so before any wave rewrites a tag
  const int k = w < 3 ? w : 2;
  const int e = act ? a.ep_in[b] + kP2Last - 2 - k : 0;
  const bool ok = act && a.s_tag[2 + k][b] == e * 8 + 2 + k;
  __syncthreads();
  if (w == 0) p2_third<0>(a, b0, lane, e, ok, &s_prog);
  else if (w == 1) p2_third<1>(a, b0, lane, e, ok, &s_prog);
  else if (w == 2) p2_third<2>(a, b0, lane, e, ok, &s_prog);
  else p2_twist(a, b0, lane, __any(ok), &s_prog);
}

// a draw stage: draws [d0, d1) of episode e on its stream slot, from an LDS
// window (at `base`) of kP2Win rows starting at the wave's lowest start
// cursor (the wave's 64 boards, staged here); `in` (stage > 0) holds the
// draws so far, `out` gets them plus these; the cursors go to the slot's
// cursor table
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ void p2_draw_stage(const P2Args &a, int b0, int lane, int stage, int base) {
  const int b = b0 + lane;
#ifdef HZ_DIAG
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  const bool act = b < a.n;
  const size_t nr = (size_t)a.nrow;
  const int d0 = kP2DCut[stage], d1 = stage == 3 ? a.draws : min(a.draws, kP2DCut[stage + 1]);
  const int e = act ? a.ep_in[b] + kP2Last - 5 - stage : 0;
  const uint32_t *slot = a.s_mt[5 + stage];
  int32_t *cur = a.s_cur[5 + stage] + b;
  const P2Draw &in = a.x_r[stage > 0 ? stage - 1 : 0];
  const P2Draw &out = stage == 3 ? a.pl_w : a.x_w[stage];
  bool ok = act && a.s_tag[5 + stage][b] == e * 8 + 5;
  int k0 = 0, c0 = kMTAhead;
  uint64_t bag = initial_bag(), q[kAheadWords] = {0, 0, 0, 0};
  if (stage > 0 && act) {  // (one round trip: used only if the tag matches)
    const int itag = in.tag[b];
    k0 = in.k[b];
    c0 = in.c[b];
    bag = in.bag[b];
#pragma unroll
    for (int i = 0; i < kAheadWords; i++) q[i] = in.q[(size_t)i * nr + b];
    ok = ok && itag == e * 8 + stage;
  }
  const bool draws = ok && k0 >= d0 && d0 < d1;
  const int r0 = wave_min_i(draws ? (c0 & 0xFFFF) : kAheadTwist) & ~3;
  if (r0 < kAheadTwist) {  // the window: rows [r0, r0 + kP2Win), 16-B loads (four boards of a row per lane), all in flight
    constexpr int U = kP2Win / 4;
    const int c4 = (lane & 15) * 4;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int r = r0 + 4 * u + (lane >> 4);
      v[u] = p2_ld4(slot + (size_t)r * nr + b0 + c4);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t *dd = hz_lds + base + (4 * u + (lane >> 4)) * kLdsStride + c4;
      dd[0] = v[u].x;
      dd[1] = v[u].y;
      dd[2] = v[u].z;
      dd[3] = v[u].w;
    }
  }
  P2_PHASE(28 + stage, t0);  // window staged
  if (!act) return;
  if (!ok) {
    out.tag[b] = -1;
    return;
  }
  if (stage == 0) cur[0] = kMTAhead;
  int k = k0, cc = c0;
  if (draws) {  // every earlier draw is done: continue in the window
    const int lim = min(r0 + kP2Win, kAheadTwist);
    StreamDraw<WinMT> d{WinMT(base - r0 * kLdsStride + lane, c0, lim)};
#pragma unroll 1
    for (int i = d0; i < d1; i++) {
      if (d.m.pos >= lim) break;
      const uint32_t p9 = d(bag);
      // a draw that consumed words past the window is discarded: the next
      // stage (or a play stage, from the stream slot) redoes it from the
      // last cursor kept
      if (d.m.pos > lim) break;
      apply_pile_fast(bag, p9);
      const int bit = 9 * i, wd = bit >> 6, off = bit & 63;
      const uint64_t lo9 = (uint64_t)p9 << off, hi9 = off > 55 ? (uint64_t)p9 >> (64 - off) : 0ull;
      q[0] |= wd == 0 ? lo9 : 0ull;
      q[1] |= wd == 1 ? lo9 : wd == 0 ? hi9 : 0ull;
      q[2] |= wd == 2 ? lo9 : wd == 1 ? hi9 : 0ull;
      q[3] |= wd == 3 ? lo9 : wd == 2 ? hi9 : 0ull;
      cc = d.m.cursor();
      p2_st(&cur[(size_t)(i + 1) * nr], cc);
      k = i + 1;
    }
  }
  p2_st(&out.k[b], k);
  p2_st(&out.c[b], cc);
  p2_st(&out.bag[b], bag);
#pragma unroll
  for (int i = 0; i < kAheadWords; i++) p2_st(&out.q[(size_t)i * nr + b], q[i]);
  p2_st(&out.tag[b], e * 8 + stage + 1);
}

// the rule hashes of D4's episode (read by the play stages in the next
// kP2Play calls)
__device__ __forceinline__ void p2_hashes(const P2Args &a, int b) {
  const size_t nr = (size_t)a.nrow;
  const int e = a.ep_in[b] + kP2Last - 8;
  const uint64_t rk = rule_key(episode_seed(a.seed_base, b, e));
#pragma unroll 1
  for (int j = 0; j < kRulePlies; j++) p2_st(&a.h_w[(size_t)j * nr + b], rule_h32(rk, j));
  a.ht_w[b] = e;
}

// draw-X blocks: D1 (wave 0), D2 (wave 1), P1b (wave 2), the rule hashes
// (wave 3); draw-Y blocks: D3, D4 (waves 0, 1), P1a (wave 2).  Each draw
// wave stages its own window and reads only it.
__device__ __forceinline__ void p2_draw(const P2Args &a, int blk, int y) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock;
  if (w < 2) {
    p2_draw_stage(a, b0, lane, 2 * y + w, w * kP2WinRows * kLdsStride);
  } else if (w == 2 && b0 + lane < a.n) {
    if (y) p2_p1a(a, b0, lane);
    else p2_p1b(a, b0, lane);
  } else if (w == 3 && !y && b0 + lane < a.n) {
    p2_hashes(a, b0 + lane);
  }
}

// a play stage's state after its plies, for the next play stage
__device__ __forceinline__ void p2_mid_put(const P2Mid &m, size_t nr, int b, const State &s, const PlayDraw2 &d, int g,
                                           int e) {
#pragma unroll
  for (int k = 0; k < 4; k++) p2_st(&m.st[(size_t)k * nr + b], s.pl[k]);
  p2_st(&m.st[4 * nr + b], s.piles);
  p2_st(&m.st[5 * nr + b], s.misc);
  p2_st(&m.q[b], d.q0);
  p2_st(&m.q[nr + b], d.q1);
  p2_st(&m.q[2 * nr + b], d.q2);
  p2_st(&m.q[3 * nr + b], d.q3);
  p2_st(&m.i[b], d.d);
  p2_st(&m.i[nr + b], g);
  p2_st(&m.i[2 * nr + b], d.fell ? d.gm.cursor() : -1);
  p2_st(&m.tag[b], e);
}
// the previous play stage's state; the draw source continues its script
// (nd entries, cursors in `cur`) or the slot stream it fell onto
__device__ __forceinline__ PlayDraw2 p2_mid_get(const P2Mid &m, size_t nr, int b, State &s, int &g, int nd,
                                               uint32_t *slot, const int32_t *cur) {
#pragma unroll
  for (int k = 0; k < 4; k++) s.pl[k] = m.st[(size_t)k * nr + b];
  s.piles = m.st[4 * nr + b];
  s.misc = m.st[5 * nr + b];
  const int d = m.i[b], fc = m.i[2 * nr + b];
  g = m.i[nr + b];
  return PlayDraw2{m.q[b], m.q[nr + b], m.q[2 * nr + b], m.q[3 * nr + b], d, nd, fc >= 0,
                   MTR(slot, (int)nr, fc >= 0 ? fc : 0), cur + (size_t)nd * nr};
}

// play blocks: wave 3 - st runs play stage st on episode ep + kP2Play - 1 -
// st (the last stage, wave 0: the rest of episode ep, or all of it).  The
// stages run one code path (st wave-uniform), so the block's four waves
// share one copy of the ply loop in the instruction cache (one inlined copy
// per stage, ~50 KB each, thrashed the cache the two CUs of a pair share).
__device__ __forceinline__ void p2_play(const P2Args &a, int blk) {
  __shared__ uint64_t s_lds_mask;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = blk * kBlock, b = b0 + lane;
  const bool act = b < a.n;
  const uint64_t actmask = __ballot(act);
  const int nb = a.n - b0 < kBlock ? a.n - b0 : kBlock;
  const size_t nr = (size_t)a.nrow;
#ifdef HZ_DIAG
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  const int st = __builtin_amdgcn_readfirstlane(kP2Play - 1 - w);  // 0 playA .. kP2Play - 1 the last
  const bool last = st == kP2Play - 1;
  bool lds_used = false;
  if (act) {
    const int e = last ? a.episode[b] : a.ep_in[b] + kP2Play - 1 - st;
    const P2Draw &pl = a.pl_r[st];
    const uint32_t *hsrc = a.h_r[st];
    const int32_t *htag = a.ht_r[st];
    uint32_t *slot = a.s_mt[9 + st] + b;
    const int32_t *cur = a.s_cur[9 + st] + b;
    const int g_end = last ? a.max_plies : min(a.cut[st], a.max_plies);
    const uint64_t sd = episode_seed(a.seed_base, b, e), rk = rule_key(sd);
    // every input's loads issued together (used only if the tags match)
    const int ptag = pl.tag[b], nd = pl.k[b];
    const int mtag = st > 0 ? a.m_r[st - 1].tag[b] : e;
    const uint32_t *hs = htag[b] == e ? hsrc + b : nullptr;
    State s;
    int g = 0;
    PlayDraw2 draw = st == 0 ? PlayDraw2{pl.q[b], pl.q[nr + b], pl.q[2 * nr + b], pl.q[3 * nr + b], 0, nd, false,
                                         MTR(slot, (int)nr, 0), cur + (size_t)nd * nr}
                             : p2_mid_get(a.m_r[st - 1], nr, b, s, g, nd, slot, cur);
    const bool prep = ptag == e * 8 + 4 && mtag == e;
    if (prep) {
      if (st == 0) {
        if (__all(nd >= 5)) draw.scripted_reset(s);
        else reset_state(s, draw);
      }
      P2_PHASE(16 + 3 * st, t0);
      g += p2_plies(s, draw, g, g_end, rk, hs, nr);
      P2_PHASE(17 + 3 * st, t0);
    }
    if (!last) {
      const P2Mid &mo = a.m_w[st];
      if (prep) p2_mid_put(mo, nr, b, s, draw, g, e);
      else mo.tag[b] = -1;
    } else {
      int cursor, src;
      if (prep) {
        cursor = draw.fell ? draw.gm.cursor() : cur[(size_t)draw.d * nr];
        src = 2 + a.s_idx_last;
      } else {  // unprepared: the whole game, the stream seeded and drawn in LDS
        mt_seed(hz_lds + lane, kLdsStride, sd);
        PlayDraw fb{LdsMT(lane, kMTSeeded), false, false, 0, 0, 0, 0, 0, 0, MT(nullptr, 0), nullptr};
        reset_state(s, fb);
        g = p2_plies(s, fb, 0, a.max_plies, rk, nullptr, nr);
        cursor = fb.m.cursor();
        src = -1;
        lds_used = true;
      }
      a.episode[b] = e + 1;
      if (score_pending(s.misc)) finish_game(s);
      P2_PHASE(27, t0);
      store_state(a.st, a.n, b, s);
      a.pos[b] = cursor;
      a.mt_src[b] = src;
      a.ply[b] = g;
      a.seed[b] = sd;
      a.ep_out[b] = e + 1;
      // the game this call completes, as hz_play's other pipeline counts it
      if (a.games_done) a.games_done[b] = phase_of(s.misc) == PH_OVER ? 1 : 0;
      if (a.steps_done) a.steps_done[b] = g;
    }
#ifdef HZ_DIAG
    if (g_stamps) g_stamps[(size_t)b * kP2Stamps + w] = __builtin_amdgcn_s_memtime() - t0;  // last .. playA
#endif
  }
  if (w == 0) {
    const uint64_t lm = __ballot(lds_used);
    if (lane == 0) s_lds_mask = lm;
  }
  __syncthreads();
  const uint64_t lds_mask = s_lds_mask & actmask;
  if (lds_mask) stage_mt(a.mt + (size_t)b0 * kMT, nb, tid, lds_mask, false);
}

// one 162 KB-LDS block per CU, so one wave per SIMD: every wave may use the
// whole register file (the P2b twist wave keeps 57 rows in registers)
__global__ void __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) k_play2(P2Args a, int nblk) {
  const int blk = (int)blockIdx.x;
  const int role = blk / nblk;  // 0 play, 1 draw X, 2 draw Y, 3 seed blocks
  const int rb = blk - role * nblk;
#ifdef HZ_DIAG
  if (g_role_only >= 0 && g_role_only != role) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (role == 0) p2_play(a, rb);
  else if (role == 3) p2_seed(a, rb);
  else p2_draw(a, rb, role - 1);
#ifdef HZ_DIAG
  {  // wave durations per board, slot 4 role + wave: 0-3 play (D, C, B, A:
     // stamped in p2_play, before its barrier), 4-7 draw X (D1, D2, P1b,
     // hashes), 8-10 draw Y (D3, D4, P1a), 12-15 seed (P2a, P2b, P2c, twist)
    const int w = threadIdx.x >> 6, bb = rb * kBlock + (threadIdx.x & 63);
    const bool idle = role == 2 && w == 3;
    if (g_stamps && role > 0 && !idle && bb < a.n) g_stamps[(size_t)bb * kP2Stamps + 4 * role + w] = __builtin_amdgcn_s_memtime() - t0;
    // the wave's realtime (100 MHz) start and end and its clock cycles, per
    // (role, wave): slot 40 of the block's boards 16 role + 4 w + k
    // (tools/p2_span.py: the launch's span against its waves')
    if (g_stamps && bb < a.n && (threadIdx.x & 63) < 4) {
      const int k = threadIdx.x & 63;
      const uint64_t v = k == 0 ? r0 : k == 1 ? __builtin_amdgcn_s_memrealtime() : k == 2 ? t0 : __builtin_amdgcn_s_memtime();
      g_stamps[(size_t)(rb * kBlock + 16 * role + 4 * w + k) * kP2Stamps + 40] = v;
      // where the wave ran: HW_ID (cu, sh, se in bits 8-14) and XCC_ID
      if (k == 0)
        g_stamps[(size_t)(rb * kBlock + 16 * role + 4 * w) * kP2Stamps + 41] =
            (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
    }
  }
#endif
}

// boards whose stream lives in a pipeline-2 slot (mt_src = 2 + slot): the
// slot's column (word-major) into the board's own stream, one wave per board
struct P2Slots {
  uint32_t *s[kP2Stream];
};
__global__ void __launch_bounds__(64) k_mt_materialize2(uint32_t *__restrict__ mt, P2Slots slots,
                                                       int32_t *__restrict__ mt_src, long nrow) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int src = mt_src[b];
  if (src < 2 || src >= 2 + kP2Stream) return;
  const uint32_t *from = slots.s[src - 2] + b;
  uint32_t *to = mt + (size_t)b * kMT;
  uint32_t v[(kMT + 63) / 64];
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++) v[k] = lane + 64 * k < kMT ? from[(size_t)(lane + 64 * k) * nrow] : 0u;
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

// boards whose stream lives in an auto-reset slot (mt_src = kArSrc + slot)
__global__ void __launch_bounds__(64) k_mt_materialize_ar(uint32_t *__restrict__ mt, const uint32_t *__restrict__ ar_mt,
                                                         int32_t *__restrict__ mt_src, int n) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int src = mt_src[b];
  if (src < kArSrc || src >= kArSrc + kArSlots) return;
  const uint32_t *from = ar_mt + ((size_t)(src - kArSrc) * n + b) * kMT;
  uint32_t *to = mt + (size_t)b * kMT;
  uint32_t v[(kMT + 63) / 64];
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++) v[k] = lane + 64 * k < kMT ? from[lane + 64 * k] : 0u;
#pragma unroll
  for (int k = 0; k < (kMT + 63) / 64; k++)
    if (lane + 64 * k < kMT) to[lane + 64 * k] = v[k];
  if (lane == 0) mt_src[b] = -1;
}

static PlyWin ply_win(hz_env *e) { return PlyWin{e->pw_words, e->pw_tag, e->pw_ep, (long)e->nrow, e->mt_epoch}; }

static int materialize(hz_env *e) {
  if (!e->lazy) return 0;
  e->mt_epoch++;  // streams rewritten (PlyWin's saved words are stale)
  if (e->ar_mt)
    hipLaunchKernelGGL(k_mt_materialize_ar, dim3(e->n), dim3(64), 0, e->stream, e->mt, e->ar_mt, e->mt_src, e->n);
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
  for (int k = 0; k < 3; k++) fd(e->p2_x[k][0]), fd(e->p2_x[k][1]);
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
    f(e->p2_p1h[k]);
    f(e->p2_p2h[k]);
    f(e->p2_p3h[k]);
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
  for (int k = 0; k < 3; k++)
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
  for (int k = 0; ok && k < 3; k++) ok = md(e->p2_x[k][0]) && md(e->p2_x[k][1]);
  for (int k = 0; ok && k < kP2Ring; k++)
    ok = md(e->p2_pl[k]) && m(&e->p2_h[k], kRulePlies * nr * 4) && m(&e->p2_h_tag[k], nr * 4);
  for (int k = 0; ok && k < kP2Play - 1; k++)
    for (int j = 0; ok && j < 2; j++) {
      P2Mid &mm = e->p2_m[k][j];
      ok = m(&mm.tag, nr * 4) && m(&mm.st, 6 * nr * 8) && m(&mm.q, 4 * nr * 8) && m(&mm.i, 3 * nr * 4);
    }
  for (int k = 0; ok && k < 2; k++)
    ok = m(&e->p2_p1h[k], nr * 4) && m(&e->p2_p2h[k], 3 * nr * 4) && m(&e->p2_p3h[k], 3 * nr * 4) &&
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
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
  a.p1h_w = e->p2_p1h[r];
  a.p1h_r = e->p2_p1h[w];
  a.p2h_w = e->p2_p2h[r];
  a.p2h_r = e->p2_p2h[w];
  a.p3h_w = e->p2_p3h[r];
  a.p3h_r = e->p2_p3h[w];
  for (int k = 0; k < 3; k++) {
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
  e->ar_primed = 0;
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
  {
    const char *av = getenv("HZ_AR_AHEAD");
    e->ar_ahead = av && atoi(av) == 0 ? 0 : 1;
  }
  {  // hz_play's pipeline: 2 by default, HZ_PIPELINE=1 for the first (hz_env_set_pipeline)
    const char *pv = getenv("HZ_PIPELINE");
    e->pipeline = pv && atoi(pv) == 1 ? 1 : 2;
    // HZ_P2_CUTS="a,b,c": pipeline 2's play stage boundaries (plies,
    // increasing multiples of 4: whole turns; a stage that starts at player
    // 1's turn plays single plies up to the next turn pair)
    e->p2_cut[0] = 24;
    e->p2_cut[1] = 40;
    e->p2_cut[2] = 56;
    const char *cv = getenv("HZ_P2_CUTS");
    int c[3];
    if (cv && sscanf(cv, "%d,%d,%d", &c[0], &c[1], &c[2]) == 3 && c[0] > 0 && c[1] > c[0] && c[2] > c[1] &&
        c[0] % 4 == 0 && c[1] % 4 == 0 && c[2] % 4 == 0)
      for (int k = 0; k < 3; k++) e->p2_cut[k] = c[k];
  }
  ok = ok && hipMalloc(&e->pw_words, e->nrow * kPlyWin * sizeof(uint32_t)) == hipSuccess &&
       hipMalloc(&e->pw_tag, e->nrow * sizeof(int32_t)) == hipSuccess &&
       hipMalloc(&e->pw_ep, e->nrow * sizeof(int32_t)) == hipSuccess &&
       hipMemset(e->pw_tag, 0xff, e->nrow * sizeof(int32_t)) == hipSuccess &&
       hipMemset(e->pw_ep, 0, e->nrow * sizeof(int32_t)) == hipSuccess;
  e->mt_epoch = 1;
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
  if (e->pw_words) (void)hipFree(e->pw_words);
  if (e->pw_tag) (void)hipFree(e->pw_tag);
  if (e->pw_ep) (void)hipFree(e->pw_ep);
  if (e->ar_mt) (void)hipFree(e->ar_mt);
  if (e->ar_tag) (void)hipFree(e->ar_tag);
  if (e->ar_pile) (void)hipFree(e->ar_pile);
  if (e->ar_cur) (void)hipFree(e->ar_cur);
  for (int k = 0; k < 2; k++)
    if (e->ar_ep[k]) (void)hipFree(e->ar_ep[k]);
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

int hz_env_set_auto_ahead(hz_env *e, int32_t on) {
  if (!e) return -1;
  e->ar_ahead = on ? 1 : 0;
  e->ar_primed = 0;
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
  e->mt_epoch++;  // the caller may move or rewrite streams (PlyWin)
  return e->mt;
}
int32_t *hz_env_mt_pos_ptr(hz_env *e) {
  if (!e) return nullptr;
  e->mt_epoch++;
  return e->pos;
}
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
  if (!e) return -1;
  if (int err = materialize(e)) return err;  // unselected boards keep their streams
  e->primed = 0;  // episode counters move outside hz_play's plan
  e->primed2 = 0;
  e->ar_primed = 0;
  hipLaunchKernelGGL(k_reset, dim3(grid_for(e->n)), dim3(kStageThreads), kResetLds, e->stream, e->state, e->mt, e->pos,
                     e->ply, e->episode, e->seed, e->n, e->seed_base, sel, seeds);
  return launch_err();
}

int hz_legal_actions(hz_env *e, uint8_t *legal, int32_t *count) {
  if (!e || !legal || ((uintptr_t)legal & 15)) return -1;
  hipLaunchKernelGGL(k_legal_bytes, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->n, legal, count);
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
                     e->n, action, status, ply_win(e));
  return launch_err();
}

int hz_rule_ply(hz_env *e, uint64_t *mask, int32_t *count, int16_t *action, int32_t *status) {
  if (!e) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_ply, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->seed, e->n, mask, count, action, status, ply_win(e));
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
  if (!e || !action) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_greedy, dim3(e->n), dim3(64), 0, e->stream, e->state, e->mt, e->pos, e->n, sel, action);
  return launch_err();
}

// auto-reset preparation slots, allocated at the first auto-reset hz_rollout
// (40 MB of streams at 4096 boards)
static int alloc_ar(hz_env *e) {
  if (e->ar_mt) return 0;
  const size_t n = (size_t)e->n;
  bool ok = hipMalloc(&e->ar_mt, kArSlots * n * kMT * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&e->ar_tag, kArSlots * n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->ar_pile, kArSlots * kAheadWords * n * sizeof(uint64_t)) == hipSuccess &&
            hipMalloc(&e->ar_cur, kArSlots * (kAheadDraws + 1) * n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->ar_ep[0], n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->ar_ep[1], n * sizeof(int32_t)) == hipSuccess &&
            hipMemsetAsync(e->ar_tag, 0xff, kArSlots * n * sizeof(int32_t), e->stream) == hipSuccess;
  if (!ok) {
    auto f = [](auto *&p) {
      if (p) (void)hipFree((void *)p);
      p = nullptr;
    };
    f(e->ar_mt);
    f(e->ar_tag);
    f(e->ar_pile);
    f(e->ar_cur);
    f(e->ar_ep[0]);
    f(e->ar_ep[1]);
    return 1;
  }
  e->ar_primed = 0;
  return 0;
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
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
  // hz_rollout with auto-reset: episodes prepared ahead (ar_prep_stage) by
  // 2 x nblk extra blocks; the playing blocks leave the counters they end
  // with for the next call's preparing blocks (ep_final)
  ArArgs ar{};
  const bool ar_on = auto_reset && !reset_first && !rec && e->ar_ahead;
  if (ar_on) {
    if (alloc_ar(e)) return 1;
    const int ar_r = e->ar_calls & 1;
    if (!e->ar_primed) {
      if (hipMemcpyAsync(e->ar_ep[ar_r], e->episode, (size_t)e->n * sizeof(int32_t), hipMemcpyDeviceToDevice,
                         e->stream))
        return 1;
      e->ar_primed = 1;
    }
    ar = ArArgs{e->ar_mt, e->ar_tag, e->ar_pile, e->ar_cur, e->ar_ep[ar_r], 1};
    ep_final = e->ar_ep[ar_r ^ 1];
    grid = 3 * nblk;
  } else {
    e->ar_primed = 0;  // episode counters move outside the auto-reset plan
  }
  auto kern = auto_reset ? (rec ? k_rollout<true, true> : k_rollout<true, false>)
                         : (rec ? k_rollout<false, true> : k_rollout<false, false>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kStageThreads), kResetLds, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->episode, e->seed, e->n, e->seed_base, max_plies, auto_reset, reset_first, traj_state,
                     traj_mask, traj_action, games_done, steps_done, ahead_mt, ahead_tag, ahead_pile, ahead_cur,
                     e->seed_ahead, ep_final, nblk, e->ahead_mt[w], e->ahead_tag[w], e->ahead_pile[w],
                     e->ahead_cur[w], e->ep_final[w], ring(c3), ring((c3 + 2) % kRing), ring((c3 + 1) % kRing),
                     (long)e->nrow, ahead_rule, e->ahead_rule[w], e->mt_src, ahead_mt ? r : -1, ar);
  int err = launch_err();
  if (err) return err;
  if (ahead_mt) e->lazy = 1;
  if (ar_on) {
    e->lazy = 1;
    e->ar_calls++;
  }
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
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
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
  if (!e) return -1;
  if (int err = materialize(e)) return err;
  hipLaunchKernelGGL(k_turn_op, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->n, sel,
                     0);
  return launch_err();
}

int hz_end_turn(hz_env *e, const uint8_t *sel) {
  if (e) e->mt_epoch++;  // (may move or rewrite streams: PlyWin)
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
