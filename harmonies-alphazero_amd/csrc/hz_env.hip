// hz_env.hip — batched Harmonies env kernels and their C-ABI (include/hz_abi.h).
//
// Every env kernel is lane-per-board: thread b owns board b, loads its 48 B
// SoA record (coalesced: 64 lanes x 8 B per word), runs the rules from
// hz_device.hpp in registers and stores the record back.  The encoder is
// element-parallel instead (it writes 5,488 B per board and is HBM-bound).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "../../include/hz_abi.h"
#include "hz_device.hpp"
#include "hz_encode.hpp"

using namespace hz;

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
};

#ifdef HZ_DIAG
// diagnostic build only (tools/diag.py): per-lane phase clocks
__device__ uint64_t *g_stamps;
#define HZ_STAMP(slot)                                                    \
  do {                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                    \
    if (g_stamps) g_stamps[(size_t)b * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                    \
  } while (0)
#define HZ_ACC(slot, t0)                                                  \
  do {                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                    \
    uint64_t _t = __builtin_amdgcn_s_memtime();                           \
    acc##slot += _t - (t0);                                               \
    t0 = _t;                                                              \
    __builtin_amdgcn_sched_barrier(0);                                    \
  } while (0)
#else
#define HZ_STAMP(slot) \
  do {                 \
  } while (0)
#define HZ_ACC(slot, t0) \
  do {                   \
  } while (0)
#endif

namespace {

constexpr int kBlock = 64;  // one wave per workgroup: 4096 boards -> 64 waves

inline int grid_for(int n) { return (n + kBlock - 1) / kBlock; }

// ------------------------------------------------------------------ reset
// Lane-per-board with the 64 boards' MT arrays staged in LDS as [624][65]
// words (stride 65: the per-lane seeding writes and the board-major write-out
// reads are both bank-conflict free).  Seeding (two serial 623-step passes)
// and the 15 opening draws run at LDS latency; one coalesced pass then writes
// the block's contiguous 64 x 2,496 B of HBM.
constexpr size_t kResetLds = (size_t)kMT * kLdsStride * sizeof(uint32_t);  // 162,240 B

__global__ void __launch_bounds__(kBlock) k_reset(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                  int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                  int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                  int n, uint64_t seed_base, const uint8_t *__restrict__ sel,
                                                  const uint64_t *__restrict__ seeds) {
  uint32_t *lds = hz_lds;
  int lane = threadIdx.x;
  int b0 = blockIdx.x * kBlock;
  int b = b0 + lane;
  bool act = b < n && (!sel || sel[b]);
  if (act) {
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
  uint64_t actmask = __ballot(act);
  __syncthreads();
  int nb = n - b0 < kBlock ? n - b0 : kBlock;
  uint32_t *g = mt + (size_t)b0 * kMT;
  HZ_STAMP(3);
  // board by board: lanes copy words lane, lane + 64, ... (LDS banks distinct,
  // 256 B coalesced stores, ten LDS reads in flight per board)
  for (int bl = 0; bl < nb; bl++) {
    if (!((actmask >> bl) & 1)) continue;
    uint32_t v[10];
#pragma unroll
    for (int k = 0; k < 10; k++) {
      int i = lane + kBlock * k;
      v[k] = i < kMT ? lds[i * kLdsStride + bl] : 0u;
    }
    uint32_t *gb = g + (size_t)bl * kMT;
#pragma unroll
    for (int k = 0; k < 10; k++) {
      int i = lane + kBlock * k;
      if (i < kMT) gb[i] = v[k];
    }
  }
  HZ_STAMP(4);
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

// ---------------------------------------------------------------- rollout
// Lane-per-board with the block's 64 MT streams resident in LDS for the
// whole call ([624][65] words, as in k_reset): every draw reads and twists at
// LDS latency instead of paying a scattered HBM round trip per draw.  The
// streams are staged in (or seeded in place when reset_first) and written
// back once.
__device__ __forceinline__ void stage_mt(uint32_t *__restrict__ lds, uint32_t *__restrict__ g, int nb, int lane,
                                         uint64_t actmask, bool to_lds) {
  // the block's streams are one contiguous span of nb * 624 words in HBM
  int total4 = nb * (kMT / 4);
  for (int q0 = 0; q0 < total4; q0 += kBlock * 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      int q = q0 + u * kBlock + lane;
      int o = q * 4, bl = o / kMT, i = o - bl * kMT;
      if (q < total4 && ((actmask >> bl) & 1)) {
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
    for (int u = 0; u < 4; u++) {
      int q = q0 + u * kBlock + lane;
      int o = q * 4, bl = o / kMT, i = o - bl * kMT;
      if (q < total4 && ((actmask >> bl) & 1)) {
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

__global__ void __launch_bounds__(kBlock) k_rollout(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                    int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                    int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                    int n, uint64_t seed_base, int max_plies, int auto_reset,
                                                    int reset_first, uint64_t *__restrict__ traj_state,
                                                    uint64_t *__restrict__ traj_mask,
                                                    int16_t *__restrict__ traj_action, int32_t *__restrict__ games_done,
                                                    int32_t *__restrict__ steps_done) {
  uint32_t *lds = hz_lds;
  int lane = threadIdx.x;
  int b0 = blockIdx.x * kBlock;
  int b = b0 + lane;
  bool act = b < n;
  uint64_t actmask = __ballot(act);
  int nb = n - b0 < kBlock ? n - b0 : kBlock;
  uint32_t *g = mt + (size_t)b0 * kMT;
  if (!reset_first) stage_mt(lds, g, nb, lane, actmask, true);
  __syncthreads();
  if (act) {
    StreamDraw<LdsMT> draw{LdsMT(lane, reset_first ? kMTSeeded : pos[b])};
    State s;
    int g_ply, games = 0, steps = 0;
    uint64_t sd;
    if (reset_first) {
      int e = episode[b];
      sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
      episode[b] = e + 1;
      mt_seed(hz_lds + lane, kLdsStride, sd);
      reset_state(s, draw);
      g_ply = 0;
    } else {
      s = load_state(st, n, b);
      g_ply = ply[b];
      sd = seed[b];
    }
#ifdef HZ_DIAG
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint64_t acc8 = 0, acc9 = 0, acc10 = 0, acc11 = 0, acc12 = 0;
#endif
    for (int i = 0; i < max_plies; i++) {
      if (game_done(s.misc)) {
        if (!auto_reset) {
          if (traj_action) {
            for (int j = i; j < max_plies; j++) traj_action[(size_t)j * n + b] = -1;
          }
          break;
        }
        int e = episode[b];
        sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
        episode[b] = e + 1;
        mt_seed(hz_lds + lane, kLdsStride, sd);
        draw.m = LdsMT(lane, kMTSeeded);
        reset_state(s, draw);
        g_ply = 0;
      }
      uint64_t mk[3];
      HZ_ACC(8, t0);
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
      if (L == 0) {  // stuck board (unreachable from HarmoniesGameState())
        if (traj_action) traj_action[(size_t)i * n + b] = -1;
        break;
      }
      int a = kth_action(mk, rule_pick(sd, g_ply, L));
      if (traj_action) traj_action[(size_t)i * n + b] = (int16_t)a;
      HZ_ACC(10, t0);
      bool te = phase_of(s.misc) == PH_P3;
      step_state(s, a, draw);
      if (te) HZ_ACC(12, t0);
      else HZ_ACC(11, t0);
      g_ply++;
      steps++;
      if (game_done(s.misc)) games++;
    }
    store_state(st, n, b, s);
    pos[b] = draw.m.cursor();
    ply[b] = g_ply;
    seed[b] = sd;
#ifdef HZ_DIAG
    if (g_stamps) {
      uint64_t *o = g_stamps + (size_t)b * 16;
      o[8] = acc8; o[9] = acc9; o[10] = acc10; o[11] = acc11; o[12] = acc12;
    }
#endif
    if (games_done) games_done[b] = games;
    if (steps_done) steps_done[b] = steps;
  }
  __syncthreads();
  stage_mt(lds, g, nb, lane, actmask, false);
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
extern "C" {

hz_env *hz_env_create(int32_t n_boards, uint64_t seed_base, void *stream) {
  if (n_boards <= 0) return nullptr;
  hz_env *e = (hz_env *)calloc(1, sizeof(hz_env));
  if (!e) return nullptr;
  e->n = n_boards;
  e->seed_base = seed_base;
  e->stream = (hipStream_t)stream;
  size_t n = (size_t)n_boards;
  // k_reset / k_rollout stage 64 boards' MT words in 158 KiB of LDS
  if (hipFuncSetAttribute((const void *)k_reset, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResetLds) !=
          hipSuccess ||
      hipFuncSetAttribute((const void *)k_rollout, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResetLds) !=
          hipSuccess) {
    free(e);
    return nullptr;
  }
  bool ok = hipMalloc(&e->state, n * 6 * sizeof(uint64_t)) == hipSuccess &&
            hipMalloc(&e->mt, n * 624 * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&e->pos, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->ply, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->episode, n * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&e->seed, n * sizeof(uint64_t)) == hipSuccess;
  if (ok) {
    ok = hipMemset(e->state, 0, n * 6 * sizeof(uint64_t)) == hipSuccess &&
         hipMemset(e->pos, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->ply, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->episode, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(e->seed, 0, n * sizeof(uint64_t)) == hipSuccess;
  }
  if (!ok) {
    hz_env_destroy(e);
    return nullptr;
  }
  return e;
}

void hz_env_destroy(hz_env *e) {
  if (!e) return;
  if (e->state) (void)hipFree(e->state);
  if (e->mt) (void)hipFree(e->mt);
  if (e->pos) (void)hipFree(e->pos);
  if (e->ply) (void)hipFree(e->ply);
  if (e->episode) (void)hipFree(e->episode);
  if (e->seed) (void)hipFree(e->seed);
  free(e);
}

int32_t hz_env_size(const hz_env *e) { return e ? e->n : -1; }

int hz_env_set_stream(hz_env *e, void *stream) {
  if (!e) return -1;
  e->stream = (hipStream_t)stream;
  return 0;
}

uint64_t *hz_env_state_ptr(hz_env *e) { return e ? e->state : nullptr; }
uint32_t *hz_env_mt_ptr(hz_env *e) { return e ? e->mt : nullptr; }
int32_t *hz_env_mt_pos_ptr(hz_env *e) { return e ? e->pos : nullptr; }
int32_t *hz_env_ply_ptr(hz_env *e) { return e ? e->ply : nullptr; }
uint64_t *hz_env_seed_ptr(hz_env *e) { return e ? e->seed : nullptr; }

int hz_reset(hz_env *e, const uint8_t *sel, const uint64_t *seeds) {
  if (!e) return -1;
  hipLaunchKernelGGL(k_reset, dim3(grid_for(e->n)), dim3(kBlock), kResetLds, e->stream, e->state, e->mt, e->pos,
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
  hipLaunchKernelGGL(k_step, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->n, action, status);
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

static int launch_rollout(hz_env *e, int32_t max_plies, int32_t auto_reset, int reset_first, uint64_t *traj_state,
                          uint64_t *traj_mask, int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  if (!e || max_plies < 0) return -1;
  hipLaunchKernelGGL(k_rollout, dim3(grid_for(e->n)), dim3(kBlock), kResetLds, e->stream, e->state, e->mt, e->pos,
                     e->ply, e->episode, e->seed, e->n, e->seed_base, max_plies, auto_reset, reset_first, traj_state,
                     traj_mask, traj_action, games_done, steps_done);
  return launch_err();
}

int hz_rollout(hz_env *e, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state, uint64_t *traj_mask,
               int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  return launch_rollout(e, max_plies, auto_reset, 0, traj_state, traj_mask, traj_action, games_done, steps_done);
}

int hz_play(hz_env *e, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state, uint64_t *traj_mask,
            int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  return launch_rollout(e, max_plies, auto_reset, 1, traj_state, traj_mask, traj_action, games_done, steps_done);
}

int hz_export_state(hz_env *e, uint64_t *state, uint32_t *mt, int32_t *mt_index) {
  if (!e) return -1;
  size_t n = (size_t)e->n;
  if (state && hipMemcpyAsync(state, e->state, n * 6 * sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream))
    return 1;
  if (mt || mt_index) {
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
    if (hipMemcpyAsync(e->mt, mt, n * kMT * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
    hipLaunchKernelGGL(k_mt_import, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->pos, e->n, mt_index);
    return launch_err();
  }
  return 0;
}

int hz_replenish(hz_env *e, const uint8_t *sel) {
  if (!e) return -1;
  hipLaunchKernelGGL(k_turn_op, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->n, sel,
                     0);
  return launch_err();
}

int hz_end_turn(hz_env *e, const uint8_t *sel) {
  if (!e) return -1;
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
#endif

}  // extern "C"
