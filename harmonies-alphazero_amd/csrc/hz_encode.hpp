// hz_encode.hpp — create_state_tensors (process_game_state.py:15-137) as two
// element-parallel kernels.  The encoder is the one HBM-bound stage of the
// hot path: 5,488 B of f32 per board against 48 B read, so it is written
// for store bandwidth (one float2 per thread, contiguous across the grid).
// States are read through (word_stride, item_stride) so the same kernels
// encode env boards (SoA: word w of board b at b + w*n) and MCTS leaf nodes
// (AoS: node j at 6*j + w).  idx[j] < 0 encodes an all-zero record.
#pragma once
#include "hz_device.hpp"

namespace hz {

// sorted(VALID_HEXES) is (q, r) lexicographic = column-major over the 5x7
// grid, so a valid cell's index is the number of valid cells before it in
// column-major order.
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

namespace {  // each translation unit gets its own copy of the kernels

__global__ void __launch_bounds__(256) k_encode_board(const uint64_t *__restrict__ st, long word_stride,
                                                      long item_stride, const int32_t *__restrict__ idx, int m,
                                                      float *__restrict__ board) {
  // one thread per float2 of the [m][38][5][7] output (1330 floats / board)
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)m * 665;
  if (i >= total) return;
  int j = (int)(i / 665);
  int e0 = (int)(i - (size_t)j * 665) * 2;
  long b = idx ? (long)idx[j] : (long)j;
  float v[2] = {0.f, 0.f};
  if (b >= 0) {
    const uint64_t *sb = st + b * item_stride;
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
          int code = (int)(((sb[0] >> sh) & 1) | (((sb[word_stride] >> sh) & 1) << 1) |
                           (((sb[2 * word_stride] >> sh) & 1) << 2) | (((sb[3 * word_stride] >> sh) & 1) << 3));
          val = tile_at(code, sp) == t ? 1.f : 0.f;
        } else {
          uint64_t misc = sb[5 * word_stride];
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
  }
  reinterpret_cast<float2 *>(board)[i] = make_float2(v[0], v[1]);
}

__global__ void __launch_bounds__(256) k_encode_glob(const uint64_t *__restrict__ st, long word_stride,
                                                     long item_stride, const int32_t *__restrict__ idx, int m,
                                                     float *__restrict__ glob) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m * 42) return;
  int j = i / 42, f = i - j * 42;
  long b = idx ? (long)idx[j] : (long)j;
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
  glob[i] = val;
}

inline void launch_encode(const uint64_t *st, long word_stride, long item_stride, const int32_t *idx, int m,
                          float *board, float *glob, hipStream_t stream) {
  if (board) {
    size_t total = (size_t)m * 665;
    hipLaunchKernelGGL(k_encode_board, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, st,
                       word_stride, item_stride, idx, m, board);
  }
  if (glob) {
    hipLaunchKernelGGL(k_encode_glob, dim3((unsigned)((m * 42 + 255) / 256)), dim3(256), 0, stream, st,
                       word_stride, item_stride, idx, m, glob);
  }
}

}  // namespace
}  // namespace hz
