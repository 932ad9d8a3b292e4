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

using namespace hz;

struct hz_env {
  int32_t n;
  uint64_t seed_base;
  hipStream_t stream;
  uint64_t *state;   // [6][n]
  uint32_t *mt;      // [624][n]
  int32_t *pos;      // [n]
  int32_t *ply;      // [n]
  int32_t *episode;  // [n]
  uint64_t *seed;    // [n]
};

namespace {

constexpr int kBlock = 64;  // one wave per workgroup: 4096 boards -> 64 waves

inline int grid_for(int n) { return (n + kBlock - 1) / kBlock; }

// ------------------------------------------------------------------ reset
__global__ void __launch_bounds__(kBlock) k_reset(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                  int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                  int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                  int n, uint64_t seed_base, const uint8_t *__restrict__ sel,
                                                  const uint64_t *__restrict__ seeds) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  if (sel && !sel[b]) return;
  uint64_t sd;
  if (seeds) {
    sd = seeds[b];
  } else {
    int e = episode[b];
    sd = seed_base + (uint64_t)b + ((uint64_t)e << 32);
    episode[b] = e + 1;
  }
  MTRef m{mt, pos, n, b};
  mt_seed(m, sd);
  int p = 624;
  State s;
  reset_state(s, m, p);
  store_state(st, n, b, s);
  pos[b] = p;
  ply[b] = 0;
  seed[b] = sd;
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
  MTRef m{mt, pos, n, b};
  int p = pos[b];
  int r = step_state(s, a, m, p);
  if (r == ST_OK) {
    store_state(st, n, b, s);
    pos[b] = p;
    ply[b] += 1;
  }
  if (status) status[b] = r;
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
__global__ void __launch_bounds__(kBlock) k_rollout(uint64_t *__restrict__ st, uint32_t *__restrict__ mt,
                                                    int32_t *__restrict__ pos, int32_t *__restrict__ ply,
                                                    int32_t *__restrict__ episode, uint64_t *__restrict__ seed,
                                                    int n, uint64_t seed_base, int max_plies, int auto_reset,
                                                    uint64_t *__restrict__ traj_state, uint64_t *__restrict__ traj_mask,
                                                    int16_t *__restrict__ traj_action, int32_t *__restrict__ games_done,
                                                    int32_t *__restrict__ steps_done) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  MTRef m{mt, pos, n, b};
  State s = load_state(st, n, b);
  int p = pos[b], g_ply = ply[b], games = 0, steps = 0;
  uint64_t sd = seed[b];
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
      mt_seed(m, sd);
      p = 624;
      reset_state(s, m, p);
      g_ply = 0;
    }
    uint64_t mk[3];
    int L = legal_mask(s, mk);
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
    step_state(s, a, m, p);
    g_ply++;
    steps++;
    if (game_done(s.misc)) games++;
  }
  store_state(st, n, b, s);
  pos[b] = p;
  ply[b] = g_ply;
  seed[b] = sd;
  if (games_done) games_done[b] = games;
  if (steps_done) steps_done[b] = steps;
}

// ----------------------------------------------------------------- encode
// Column-major (x-major) valid-cell mask: sorted(VALID_HEXES) order is
// (q, r) lexicographic = column-major over the 5x7 grid, so a cell's index is
// the number of valid cells before it in this order.
__host__ __device__ constexpr uint64_t valid_cm() {
  uint64_t v = 0;
  for (int c = 0; c < 23; c++) {
    int g = grid_bit(c);
    int y = g / 7, x = g % 7;
    v |= 1ull << (x * 5 + y);
  }
  return v;
}
constexpr uint64_t kValidCM = valid_cm();

__global__ void __launch_bounds__(256) k_encode_board(const uint64_t *__restrict__ st, int n,
                                                      const int32_t *__restrict__ idx, int m,
                                                      float *__restrict__ board) {
  // one thread per float2 of the [m][38][5][7] output (1330 floats / board)
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)m * 665;
  if (i >= total) return;
  int j = (int)(i / 665);
  int e0 = (int)(i - (size_t)j * 665) * 2;
  int b = idx ? idx[j] : j;
  float v[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    int e = e0 + q;
    int ch = e / 35, yx = e - ch * 35;
    int y = yx / 7, x = yx - y * 7;
    int cm = x * 5 + y;
    float val = 0.f;
    if ((kValidCM >> cm) & 1) {
      int cell = __popcll(kValidCM & ((1ull << cm) - 1));
      if (ch < 36) {
        int p = ch >= 18 ? 1 : 0;
        int r = ch - 18 * p;
        int t = r / 3, sp = r - 3 * t;
        int sh = 32 * p + cell;
        int code = (int)(((st[b] >> sh) & 1) | (((st[(size_t)n + b] >> sh) & 1) << 1) |
                         (((st[(size_t)2 * n + b] >> sh) & 1) << 2) | (((st[(size_t)3 * n + b] >> sh) & 1) << 3));
        val = tile_at(code, sp) == t ? 1.f : 0.f;
      } else {
        uint64_t misc = st[(size_t)5 * n + b];
        if (ch == 36) {
          val = (float)player_of(misc);
        } else {
          int ph = phase_of(misc);
          val = ph <= PH_P3 ? (float)((double)ph / 3.0) : 0.f;
        }
      }
    }
    v[q] = val;
  }
  reinterpret_cast<float2 *>(board)[i] = make_float2(v[0], v[1]);
}

__global__ void __launch_bounds__(256) k_encode_glob(const uint64_t *__restrict__ st, int n,
                                                     const int32_t *__restrict__ idx, int m,
                                                     float *__restrict__ glob) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m * 42) return;
  int j = i / 42, f = i - j * 42;
  int b = idx ? idx[j] : j;
  uint64_t misc = st[(size_t)5 * n + b];
  float val = 0.f;
  if (f < 30) {
    uint64_t piles = st[(size_t)4 * n + b];
    int pi = f / 6, t = f - pi * 6;
    if (pi < npiles_of(piles)) {
      int cnt = (pile_tile(piles, pi, 0) == t) + (pile_tile(piles, pi, 1) == t) + (pile_tile(piles, pi, 2) == t);
      val = (float)((double)cnt / 3.0);
    }
  } else if (f < 36) {
    int t = f - 30, nh = hand_n(misc), cnt = 0;
    for (int q = 0; q < nh; q++) cnt += hand_tile(misc, q) == t;
    val = (float)((double)cnt / 3.0);
  } else {
    int t = f - 36;
    val = (float)((double)bag_n(misc, t) / (double)initial_count(t));
  }
  glob[i] = val;
}

// ---------------------------------------------------------- state transfer
__global__ void __launch_bounds__(kBlock) k_mt_normalize(uint32_t *__restrict__ mt, int32_t *__restrict__ pos,
                                                         int n) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  int p = pos[b];
  if (p >= 1248) p = 624;
  pos[b] = p;
  // p < 624: already CPython form.  p == 624: CPython's "index = N" (the next
  // call twists), identical representation.
  if (p <= 624) return;
  MTRef m{mt, pos, n, b};
  int start = p - 624;
  for (int i = start; i < 624; i++) {
    uint32_t nw;
    if (i < 227) nw = twist_word(m.w(i), m.w(i + 1), m.w(i + 397));
    else if (i < 623) nw = twist_word(m.w(i), m.w(i + 1), m.w(i - 227));
    else nw = twist_word(m.w(623), m.w(0), m.w(396));
    m.w(i) = nw;
  }
  // all 624 words are now the current generation, as after CPython's twist
  pos[b] = start;
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
  hipLaunchKernelGGL(k_reset, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos,
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
  if (board) {
    size_t total = (size_t)m * 665;
    hipLaunchKernelGGL(k_encode_board, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, e->stream, e->state,
                       e->n, idx, m, board);
  }
  if (glob) {
    hipLaunchKernelGGL(k_encode_glob, dim3((unsigned)((m * 42 + 255) / 256)), dim3(256), 0, e->stream, e->state,
                       e->n, idx, m, glob);
  }
  return launch_err();
}

int hz_rule_actions(hz_env *e, const uint64_t *mask, const int32_t *count, int16_t *action) {
  if (!e || !mask || !action) return -1;
  hipLaunchKernelGGL(k_rule, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->seed, e->ply, e->n, mask, count,
                     action);
  return launch_err();
}

int hz_rollout(hz_env *e, int32_t max_plies, int32_t auto_reset, uint64_t *traj_state, uint64_t *traj_mask,
               int16_t *traj_action, int32_t *games_done, int32_t *steps_done) {
  if (!e || max_plies < 0) return -1;
  hipLaunchKernelGGL(k_rollout, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->state, e->mt, e->pos, e->ply,
                     e->episode, e->seed, e->n, e->seed_base, max_plies, auto_reset, traj_state, traj_mask,
                     traj_action, games_done, steps_done);
  return launch_err();
}

int hz_export_state(hz_env *e, uint64_t *state, uint32_t *mt, int32_t *mt_index) {
  if (!e) return -1;
  size_t n = (size_t)e->n;
  if (state && hipMemcpyAsync(state, e->state, n * 6 * sizeof(uint64_t), hipMemcpyDeviceToDevice, e->stream))
    return launch_err() ? launch_err() : 1;
  if (mt || mt_index) {
    hipLaunchKernelGGL(k_mt_normalize, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->mt, e->pos, e->n);
    int r = launch_err();
    if (r) return r;
    if (mt && hipMemcpyAsync(mt, e->mt, n * 624 * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
    if (mt_index && hipMemcpyAsync(mt_index, e->pos, n * sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream))
      return 1;
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
    if (hipMemcpyAsync(e->mt, mt, n * 624 * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
    if (hipMemcpyAsync(e->pos, mt_index, n * sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream)) return 1;
  }
  return 0;
}

const char *hz_version(void) { return "hz 0.1 gfx950"; }

}  // extern "C"
