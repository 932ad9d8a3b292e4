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

__global__ void __launch_bounds__(256) k_encode_board(const uint64_t *__restrict__ st, long word_stride,
                                                      long item_stride, const int32_t *__restrict__ idx, int m,
                                                      float *__restrict__ board) {
  __shared__ uint64_t smask[kEncWaves][76];
  __shared__ float sval[kEncWaves][76];
  int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  long j0 = 2 * ((long)blockIdx.x * kEncWaves + w);
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
          int rem = ch - 18 * p, t = rem / 3, sp = rem - 3 * t;
          int sh = 32 * p;
          uint32_t b0 = (uint32_t)(sb[0] >> sh), b1 = (uint32_t)(sb[word_stride] >> sh);
          uint32_t b2 = (uint32_t)(sb[2 * word_stride] >> sh), b3 = (uint32_t)(sb[3 * word_stride] >> sh);
          uint64_t tab = sp == 0 ? kStackPos0 : sp == 1 ? kStackPos1 : kStackPos2;
#pragma unroll
          for (int cell = 0; cell < 23; cell++) {
            int code = (int)(((b0 >> cell) & 1) | (((b1 >> cell) & 1) << 1) | (((b2 >> cell) & 1) << 2) |
                             (((b3 >> cell) & 1) << 3));
            mask |= (uint64_t)((int)((tab >> (3 * code)) & 7) == t) << grid_bit(cell);
          }
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
      smask[w][c] = mask;
      sval[w][c] = val;
    }
  }
  __syncthreads();
  if (!live) return;
  int nfl = j0 + 1 < m ? 2660 : 1330;
  float *out = board + j0 * 1330;
  for (int q = lane; q < nfl / 4; q += 64) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      int e = 4 * q + u;
      int bsel = e >= 1330 ? 1 : 0;
      int el = e - 1330 * bsel;
      int ch = el / 35, yx = el - 35 * ch;
      int c = 38 * bsel + ch;
      v[u] = ((smask[w][c] >> yx) & 1) ? sval[w][c] : 0.f;
    }
    reinterpret_cast<float4 *>(out)[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
  if (nfl == 1330 && lane < 2) {  // odd tail: floats 1328, 1329
    int el = 1328 + lane, ch = el / 35, yx = el - 35 * ch;
    out[el] = ((smask[w][ch] >> yx) & 1) ? sval[w][ch] : 0.f;
  }
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
    long pairs = ((long)m + 1) / 2;
    hipLaunchKernelGGL(k_encode_board, dim3((unsigned)((pairs + kEncWaves - 1) / kEncWaves)), dim3(256), 0, stream,
                       st, word_stride, item_stride, idx, m, board);
  }
  if (glob) {
    hipLaunchKernelGGL(k_encode_glob, dim3((unsigned)((m * 42 + 255) / 256)), dim3(256), 0, stream, st,
                       word_stride, item_stride, idx, m, glob);
  }
}

}  // namespace
}  // namespace hz
