// hz_encode.hpp — create_state_tensors (process_game_state.py:15-137) as two
// kernels.  The encoder is the one HBM-bound stage of the hot path: 5,488 B
// of f32 per board against 48 B read, so it is written for store bandwidth
// (per-board work done once per channel, float4 stores contiguous per pair).
// States are read through (word_stride, item_stride) so the same kernels
// encode env boards (SoA: word w of board b at b + w*n) and MCTS leaf nodes
// (AoS: node j at 6*j + w).  idx[j] < 0 encodes an all-zero record.
#pragma once
#include "hz_device.hpp"

namespace hz {


namespace {  // each translation unit gets its own copy of the kernels

// Board planes, one wave per pair of states (a pair's 10,640 B output starts
// 16 B aligned).  Lanes first build the pair's 76 channel masks in grid
// order (channel = player*18 + tile*3 + stack position: the cells whose stack
// holds that tile at that height; channels 36/37: the valid cells, with the
// value current_player / phase index / 3), keep them in LDS, then write the
// pair's 665 float4 contiguously (each element one bit test): the store
// stream is the only HBM traffic.
constexpr int kEncWaves = 4;  // waves (pairs) per 256-thread block

// 23-bit cell set -> the 35-bit tensor-position set (bit y*7 + x, y = r+2,
// x = q+3).  A column's cells are consecutive cell indices with consecutive
// y, i.e. positions 7 apart: one multiply spreads a column's run (v * 0x1041041
// puts bit i at 7 i, masked by 0x10204081).
__device__ __forceinline__ uint64_t to_grid35(uint32_t m) {
  auto col = [&](int c0, int k, int base) -> uint64_t {
    uint32_t v = (m >> c0) & ((1u << k) - 1);
    uint32_t sp = k == 1 ? v : (v * 0x1041041u) & 0x10204081u;
    return (uint64_t)sp << base;
  };
  static_assert(grid_bit(0) == 28 && grid_bit(1) == 15 && grid_bit(4) == 2 && grid_bit(9) == 3 &&
                    grid_bit(14) == 4 && grid_bit(19) == 5 && grid_bit(22) == 6,
                "column bases");
  return col(0, 1, 28) | col(1, 3, 15) | col(4, 5, 2) | col(9, 5, 3) | col(14, 5, 4) | col(19, 3, 5) |
         col(22, 1, 6);
}

// For channel tile*3 + pos (18 of them): the 13-bit set of stack codes whose
// tile at height pos is that tile (code 0, the empty stack, never).
__host__ __device__ constexpr uint32_t code_set(int rem) {
  constexpr int kTabs[3][13] = {{7, 0, 1, 2, 3, 4, 5, 2, 3, 3, 2, 3, 4},
                                {7, 7, 7, 7, 7, 7, 7, 1, 3, 3, 4, 4, 4},
                                {7, 7, 7, 7, 7, 7, 7, 7, 7, 3, 7, 7, 7}};
  uint32_t s = 0;
  for (int c = 1; c < 13; c++) s |= (uint32_t)(kTabs[rem % 3][c] == rem / 3) << c;
  return s;
}
__host__ __device__ constexpr uint64_t code_sets(int from, int cnt) {
  uint64_t r = 0;
  for (int i = 0; i < cnt; i++) r |= (uint64_t)code_set(from + i) << (13 * i);
  return r;
}
constexpr uint64_t kCodeSetLo = code_sets(0, 4), kCodeSetMid = code_sets(4, 4), kCodeSetHi = code_sets(8, 4),
                   kCodeSetTop = code_sets(12, 4), kCodeSetEnd = code_sets(16, 2);

// feature f of item j's global vector (process_game_state.py:98-137)
__device__ __forceinline__ float glob_value(const uint64_t *__restrict__ st, long word_stride, long item_stride,
                                            const int32_t *__restrict__ idx, long j, int f) {
  long b = idx ? (long)idx[j] : j;
  float val = 0.f;
  if (b >= 0) {
    const uint64_t *sb = st + b * item_stride;
    uint64_t misc = sb[5 * word_stride];
    if (f < 30) {
      uint64_t piles = sb[4 * word_stride];
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
  }
  return val;
}

// One wave encodes the pair of items (j0, j0 + 1): its channel masks in the
// wave's own LDS rows (smask / sval: 76 entries each), then the pair's 665
// float4.  Glob: the wave also writes its pair's global features (small
// batches: one launch instead of two; at 4096 items two launches measured
// faster).  Only the wave's own LDS rows are touched, so a wave barrier
// separates the two phases.
template <bool Glob>
__device__ __forceinline__ void encode_pair(const uint64_t *__restrict__ st, long word_stride, long item_stride,
                                            const int32_t *__restrict__ idx, int m, float *__restrict__ board,
                                            float *__restrict__ glob, int lane, long j0, uint64_t *smask,
                                            float *sval) {
  bool live = j0 < m;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    int c = lane + 64 * r;
    if (live && c < 76) {
      long jb = j0 + (c >= 38 ? 1 : 0);
      int ch = c >= 38 ? c - 38 : c;
      uint64_t mask = 0;
      float val = 0.f;
      long bi = jb < m ? (idx ? (long)idx[jb] : jb) : -1;
      if (bi >= 0) {
        const uint64_t *sb = st + bi * item_stride;
        if (ch < 36) {
          int p = ch >= 18 ? 1 : 0;
          int rem = ch - 18 * p;  // tile * 3 + stack position
          int sh = 32 * p;
          uint32_t b0 = (uint32_t)(sb[0] >> sh), b1 = (uint32_t)(sb[word_stride] >> sh);
          uint32_t b2 = (uint32_t)(sb[2 * word_stride] >> sh), b3 = (uint32_t)(sb[3 * word_stride] >> sh);
          // the stack codes whose tile at this height is this tile, then the
          // cells holding one of them (bit-sliced over the 4 code planes)
          uint32_t set = (uint32_t)(kCodeSetLo >> (13 * (rem < 4 ? rem : 0))) & 0x1FFFu;
          set = rem >= 4 && rem < 8 ? (uint32_t)(kCodeSetMid >> (13 * (rem - 4))) & 0x1FFFu : set;
          set = rem >= 8 && rem < 12 ? (uint32_t)(kCodeSetHi >> (13 * (rem - 8))) & 0x1FFFu : set;
          set = rem >= 12 && rem < 16 ? (uint32_t)(kCodeSetTop >> (13 * (rem - 12))) & 0x1FFFu : set;
          set = rem >= 16 ? (uint32_t)(kCodeSetEnd >> (13 * (rem - 16))) & 0x1FFFu : set;
          uint32_t n0 = ~b0, n1 = ~b1, n2 = ~b2, n3 = ~b3, m23 = 0;
#pragma unroll
          for (int code = 1; code < 13; code++) {
            uint32_t hit = ((code & 1) ? b0 : n0) & ((code & 2) ? b1 : n1) & ((code & 4) ? b2 : n2) &
                           ((code & 8) ? b3 : n3);
            m23 |= ((set >> code) & 1u) ? hit : 0u;
          }
          mask = to_grid35(m23);
          val = 1.f;
        } else {
          uint64_t misc = sb[5 * word_stride];
          mask = kValid35;
          if (ch == 36) {
            val = (float)player_of(misc);
          } else {
            int ph = phase_of(misc);
            val = ph <= PH_P3 ? (float)((double)ph / 3.0) : 0.f;
          }
        }
      }
      smask[c] = mask;
      sval[c] = val;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!live) return;
  int nfl = j0 + 1 < m ? 2660 : 1330;
  float *out = board + j0 * 1330;
  // element e = 4 q + u of the pair: channel c = 38 (e >= 1330) + el / 35,
  // position yx = el % 35; tracked incrementally (q advances by 64: e by 256
  // = 7 channels + 11 positions)
  int e0 = 4 * lane, c0 = e0 / 35, y0 = e0 - 35 * c0;
  for (int q = lane; q < nfl / 4; q += 64) {
    // the four elements lie in channel c0 and possibly c0 + 1 (boards
    // switch at element 1330 = 38 x 35: channel 38 onward is the second)
    uint64_t ma = smask[c0], mb = smask[c0 + 1 < 76 ? c0 + 1 : c0];
    float va = sval[c0], vb = sval[c0 + 1 < 76 ? c0 + 1 : c0];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      int yx = y0 + u;
      bool nxt = yx >= 35;
      int pos = nxt ? yx - 35 : yx;
      v[u] = (((nxt ? mb : ma) >> pos) & 1) ? (nxt ? vb : va) : 0.f;
    }
    reinterpret_cast<float4 *>(out)[q] = make_float4(v[0], v[1], v[2], v[3]);
    c0 += 7;
    y0 += 11;
    if (y0 >= 35) { y0 -= 35; c0++; }
  }
  if (nfl == 1330 && lane < 2) {  // odd tail: floats 1328, 1329
    int el = 1328 + lane, ch = el / 35, yx = el - 35 * ch;
    out[el] = ((smask[ch] >> yx) & 1) ? sval[ch] : 0.f;
  }
  if constexpr (Glob) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int i = lane + 64 * r;
      const long j = j0 + (i >= 42 ? 1 : 0);
      if (i < 84 && j < m) glob[j * 42 + i - 42 * (i >= 42 ? 1 : 0)] = glob_value(st, word_stride, item_stride, idx, j, i % 42);
    }
  }
}

// One wave encodes one state (the six words at ns[0..5], AoS as a tree node
// stores them) into its board row (1,330 floats, 8-B aligned: any row of
// the batch) and its global row (42 floats): lanes 0-37 build the 38 channel
// masks into the wave's LDS rows (smask / sval: 38 entries each), then the
// row's 665 float2 are written contiguously.  The same masks, values and
// element order as encode_pair (so the same bits).  The MCTS kernel that
// selects a leaf encodes it with this in place of a separate gather launch.
// In two parts: encode_one_values builds the row in the lane's registers
// (its 11 float2 of the board row, its global), encode_one_store writes it;
// the MCTS kernel builds before it knows the row's batch slot.
constexpr int kEncQ = (665 + 63) / 64;  // float2 of the board row per lane
__device__ __forceinline__ void encode_one_values(const uint64_t *__restrict__ ns, int lane, uint64_t *smask,
                                                  float *sval, float2 (&vals)[kEncQ], float &gv_out) {
  if (lane < 38) {
    const int ch = lane;
    uint64_t mask;
    float val;
    if (ch < 36) {
      const int p = ch >= 18 ? 1 : 0;
      const int rem = ch - 18 * p;
      const int sh = 32 * p;
      const uint32_t b0 = (uint32_t)(ns[0] >> sh), b1 = (uint32_t)(ns[1] >> sh);
      const uint32_t b2 = (uint32_t)(ns[2] >> sh), b3 = (uint32_t)(ns[3] >> sh);
      uint32_t set = (uint32_t)(kCodeSetLo >> (13 * (rem < 4 ? rem : 0))) & 0x1FFFu;
      set = rem >= 4 && rem < 8 ? (uint32_t)(kCodeSetMid >> (13 * (rem - 4))) & 0x1FFFu : set;
      set = rem >= 8 && rem < 12 ? (uint32_t)(kCodeSetHi >> (13 * (rem - 8))) & 0x1FFFu : set;
      set = rem >= 12 && rem < 16 ? (uint32_t)(kCodeSetTop >> (13 * (rem - 12))) & 0x1FFFu : set;
      set = rem >= 16 ? (uint32_t)(kCodeSetEnd >> (13 * (rem - 16))) & 0x1FFFu : set;
      const uint32_t n0 = ~b0, n1 = ~b1, n2 = ~b2, n3 = ~b3;
      uint32_t m23 = 0;
#pragma unroll
      for (int code = 1; code < 13; code++) {
        const uint32_t hit = ((code & 1) ? b0 : n0) & ((code & 2) ? b1 : n1) & ((code & 4) ? b2 : n2) &
                             ((code & 8) ? b3 : n3);
        m23 |= ((set >> code) & 1u) ? hit : 0u;
      }
      mask = to_grid35(m23);
      val = 1.f;
    } else {
      const uint64_t misc = ns[5];
      mask = kValid35;
      if (ch == 36) {
        val = (float)player_of(misc);
      } else {
        const int ph = phase_of(misc);
        val = ph <= PH_P3 ? (float)((double)ph / 3.0) : 0.f;
      }
    }
    smask[ch] = mask;
    sval[ch] = val;
  }
  float gv = 0.f;
  if (lane < 42) gv = glob_value(ns, 1, 6, nullptr, 0, lane);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // float2 q = elements 2 q, 2 q + 1: channel c0, position y0 (q advances by
  // 64: elements by 128 = 3 channels + 23 positions)
  int c0 = (2 * lane) / 35, y0 = 2 * lane - 35 * c0;
#pragma unroll
  for (int k = 0; k < kEncQ; k++) {
    float v0 = 0.f, v1 = 0.f;
    if (lane + 64 * k < 665) {
      const uint64_t ma = smask[c0], mb = smask[c0 + 1 < 38 ? c0 + 1 : c0];
      const float va = sval[c0], vb = sval[c0 + 1 < 38 ? c0 + 1 : c0];
      v0 = ((ma >> y0) & 1) ? va : 0.f;
      const bool nxt = y0 + 1 >= 35;
      const int p1 = nxt ? 0 : y0 + 1;
      v1 = (((nxt ? mb : ma) >> p1) & 1) ? (nxt ? vb : va) : 0.f;
    }
    vals[k] = make_float2(v0, v1);
    c0 += 3;
    y0 += 23;
    if (y0 >= 35) { y0 -= 35; c0++; }
  }
  gv_out = gv;
}
__device__ __forceinline__ void encode_one_store(float *__restrict__ board_row, float *__restrict__ glob_row, int lane,
                                                 const float2 (&vals)[kEncQ], float gv) {
#pragma unroll
  for (int k = 0; k < kEncQ; k++)
    if (lane + 64 * k < 665) reinterpret_cast<float2 *>(board_row)[lane + 64 * k] = vals[k];
  if (lane < 42) glob_row[lane] = gv;
}
__device__ __forceinline__ void encode_one(const uint64_t *__restrict__ ns, float *__restrict__ board_row,
                                           float *__restrict__ glob_row, int lane, uint64_t *smask, float *sval) {
  float2 vals[kEncQ];
  float gv;
  encode_one_values(ns, lane, smask, sval, vals, gv);
  encode_one_store(board_row, glob_row, lane, vals, gv);
}

template <bool Glob>
__global__ void __launch_bounds__(256) k_encode_board(const uint64_t *__restrict__ st, long word_stride,
                                                      long item_stride, const int32_t *__restrict__ idx, int m,
                                                      const int32_t *__restrict__ mcount, float *__restrict__ board,
                                                      float *__restrict__ glob) {
  __shared__ uint64_t smask[kEncWaves][76];
  __shared__ float sval[kEncWaves][76];
  int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (mcount) m = *mcount < m ? *mcount : m;  // device-side item count (compacted leaf batches)
  encode_pair<Glob>(st, word_stride, item_stride, idx, m, board, glob, lane,
                    2 * ((long)blockIdx.x * kEncWaves + w), smask[w], sval[w]);
}

__global__ void __launch_bounds__(256) k_encode_glob(const uint64_t *__restrict__ st, long word_stride,
                                                     long item_stride, const int32_t *__restrict__ idx, int m,
                                                     const int32_t *__restrict__ mcount, float *__restrict__ glob) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (mcount) m = *mcount < m ? *mcount : m;
  if (i >= m * 42) return;
  int j = i / 42, f = i - j * 42;
  glob[i] = glob_value(st, word_stride, item_stride, idx, j, f);
}

// mcount (device pointer, may be NULL): only items [0, min(m, *mcount)) are
// written; the grid is sized for m.
constexpr int kEncFuseMax = 512;  // items up to this: board and glob in one launch

inline void launch_encode(const uint64_t *st, long word_stride, long item_stride, const int32_t *idx, int m,
                          float *board, float *glob, hipStream_t stream, const int32_t *mcount = nullptr) {
  if (board) {
    long pairs = ((long)m + 1) / 2;
    const dim3 grid((unsigned)((pairs + kEncWaves - 1) / kEncWaves));
    if (glob && m <= kEncFuseMax) {  // one launch for both tensors
      hipLaunchKernelGGL(k_encode_board<true>, grid, dim3(256), 0, stream, st, word_stride, item_stride, idx, m,
                         mcount, board, glob);
      return;
    }
    hipLaunchKernelGGL(k_encode_board<false>, grid, dim3(256), 0, stream, st, word_stride, item_stride, idx, m,
                       mcount, board, nullptr);
  }
  if (glob) {
    hipLaunchKernelGGL(k_encode_glob, dim3((unsigned)((m * 42 + 255) / 256)), dim3(256), 0, stream, st,
                       word_stride, item_stride, idx, m, mcount, glob);
  }
}

}  // namespace
}  // namespace hz
