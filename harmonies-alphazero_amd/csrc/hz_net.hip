// Leaf-eval epilogues of the folded network (hzamd/infer.py).
//
// The reference network (model.py:325-394) in eval mode is conv -> BN ->
// ReLU (-> + skip -> ReLU).  With BN folded into the conv, what is left
// after each 3x3 conv is a per-channel bias, the residual add and the ReLU.
// PyTorch-ROCm runs those as three passes over the [B, 5, 7, 128] NHWC
// activation (bias add after MIOpen's conv, add_, relu_: ~76 us of HBM
// traffic per residual conv at B = 4096, against ~320 us for the conv
// itself).  hz_bias_act does them in one pass, in the same order and the
// same fp32 operations, so it gives the values the three passes give:
//     x = relu((x + bias[c]) + res)
// HBM-bound: 8 B (12 B with res) per element.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "../../include/hz_abi.h"

namespace {

template <bool Res>
__global__ void __launch_bounds__(256) k_bias_act(float4 *__restrict__ x, const float4 *__restrict__ bias,
                                                  const float4 *__restrict__ res, int64_t n4, int32_t ch4) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 v = x[i];
  float4 b = bias[(int32_t)(i % ch4)];
  v.x = v.x + b.x;
  v.y = v.y + b.y;
  v.z = v.z + b.z;
  v.w = v.w + b.w;
  if constexpr (Res) {
    float4 r = res[i];
    v.x = v.x + r.x;
    v.y = v.y + r.y;
    v.z = v.z + r.z;
    v.w = v.w + r.w;
  }
  v.x = v.x > 0.f ? v.x : 0.f;
  v.y = v.y > 0.f ? v.y : 0.f;
  v.z = v.z > 0.f ? v.z : 0.f;
  v.w = v.w > 0.f ? v.w : 0.f;
  x[i] = v;
}

}  // namespace

extern "C" int hz_bias_act(float *x, const float *bias, const float *res, int64_t rows, int32_t ch, void *stream) {
  if (!x || !bias || rows < 0 || ch <= 0 || (ch & 3)) return -1;
  if (((uintptr_t)x | (uintptr_t)bias | (uintptr_t)res) & 15) return -1;
  int64_t n4 = rows * (ch / 4);
  if (n4 == 0) return 0;
  dim3 grid((unsigned)((n4 + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (res)
    hipLaunchKernelGGL(k_bias_act<true>, grid, block, 0, s, (float4 *)x, (const float4 *)bias,
                       (const float4 *)res, n4, ch / 4);
  else
    hipLaunchKernelGGL(k_bias_act<false>, grid, block, 0, s, (float4 *)x, (const float4 *)bias, nullptr, n4,
                       ch / 4);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- 3x3 conv (128 -> 128 channels, 5x7 board, pad 1) with the epilogue ----
//
// The residual tower's convs (model.py:376-393) as an implicit GEMM on the
// f32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 fma chains):
//     out[(s, cell), co] = sum_{tap, ci} x[s, cell + tap, ci] * w[co, ci, tap]
// One 512-thread workgroup = 8 states = 280 rows as 18 blocks of 16 (the
// last 8 rows repeat row 279 and are not stored).  Wave w = (row half
// rh = w >> 2, output channels 32 (w & 3) .. +32): 9 row blocks x 2 column
// blocks x 4 registers = 72 accumulators, so two waves share each SIMD and
// cover each other's LDS and memory waits.  The input is staged through LDS
// 32 channels at a time on a zero-halo [8][7 x 9][36] grid, double-buffered,
// the next chunk's global loads in flight while the current one is consumed.
// A step is 16 channels of one tap: lane (r = l & 15, kg = l >> 4) reads
// channels 16 gs + 4 kg .. +3 of its row with one 16-B LDS read, and MFMA j
// takes channel 16 gs + 4 kg + j (B alike: weights prepacked
// [tap][ci/16][co][ci%16], one 16-B fragment per lane, loaded a step ahead).
// Epilogue: out = relu((acc + bias[co]) + res), as hz_bias_act.
// (The 4-wave 32x32x2 form with 144 accumulators per wave measured the same
// 336 us; PMC: MFMA pipes busy 81 % at 2.42 GHz, profiles/r01.)
namespace {

constexpr int kCS = 8;             // states per workgroup
constexpr int kRows = kCS * 35;    // 280 output rows
constexpr int kRB = 9;             // row blocks of 16 per wave (two row halves)
constexpr int kLdsRow = 36;        // floats per padded cell (32 channels + 4)
constexpr int kBuf = kCS * 63 * kLdsRow;  // floats per staging buffer

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kStage8 = (kRows * 8 + 511) / 512;  // float4 per thread per chunk (5)

#ifdef HZ_NET_DIAG
// diagnostic build only (tools/conv_phases.py): per-workgroup phase stamps of
// waves 0 and 4, written to this buffer alone
__device__ uint64_t g_conv_stamps[1024][2][16];
#define HZ_STAMP(k)                                                                   \
  if ((t & 255) == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][t >> 8][k] = __builtin_amdgcn_s_memtime();
#else
#define HZ_STAMP(k)
#endif

__global__ void __launch_bounds__(512, 1)
    k_conv3x3_w8(const float *__restrict__ x, const float4 *__restrict__ wp, const float *__restrict__ bias,
                 const float *__restrict__ res, float *__restrict__ out, int32_t batch,
                 const int32_t *__restrict__ live) {
  extern __shared__ float4 lds4[];
  float *lds = (float *)lds4;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kg = lane >> 4, rh = w >> 2;
  const int s0 = blockIdx.x * kCS;
  if (live) batch = *live < batch ? *live : batch;  // rows past the live count are not computed
  if (s0 >= batch) return;
  const int ns = batch - s0 < kCS ? batch - s0 : kCS;
  HZ_STAMP(0)
#ifdef HZ_NET_DIAG
  if ((t & 255) == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][t >> 8][8] = __builtin_amdgcn_s_memrealtime();
#endif

  for (int i = t; i < 2 * kCS * 63; i += 512) {
    int pc = i % 63, ph = pc / 9, pw = pc - 9 * ph;
    if (ph == 0 || ph == 6 || pw == 0 || pw == 8) {
      float4 *p = (float4 *)(lds + (size_t)i * kLdsRow);
#pragma unroll
      for (int k = 0; k < kLdsRow / 4; k++) p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  f32x4 stg[kStage8];
  int gsrc[kStage8], ldst[kStage8];
#pragma unroll
  for (int it = 0; it < kStage8; it++) {
    int f = it * 512 + t;
    f = f < kRows * 8 ? f : kRows * 8 - 1;
    int sc = f >> 3, part = f & 7, s = sc / 35, cell = sc - 35 * s, ch = cell / 7, cw = cell - 7 * ch;
    gsrc[it] = (s < ns ? s0 * 35 + sc : (s0 + ns - 1) * 35 + cell) * 128 + 4 * part;
    ldst[it] = (s * 63 + (ch + 1) * 9 + cw + 1) * kLdsRow + 4 * part;
  }
#define HZ_STAGE_LOAD8(q)                                                                 \
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                        \
  _Pragma("unroll") for (int it = 0; it < kStage8; it++)                                  \
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(stg[it]) : "v"(x + gsrc[it] + 32 * (q)));
#define HZ_STAGE_STORE8(buf)                                                              \
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                        \
  _Pragma("unroll") for (int it = 0; it < kStage8; it++) *(f32x4 *)(lds + (buf) * kBuf + ldst[it]) = stg[it];

  int abase[kRB];
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) {
    int r = (rh * kRB + rb) * 16 + (lane & 15);
    r = r < kRows ? r : kRows - 1;
    int s = r / 35, cell = r - 35 * s, ch = cell / 7, cw = cell - 7 * ch;
    abase[rb] = (s * 63 + ch * 9 + cw) * kLdsRow + 4 * kg;
  }

  f32x4 acc[kRB][2];
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) acc[rb][0] = acc[rb][1] = (f32x4){};

  const int co0 = 32 * (w & 3) + (lane & 15);
  // B fragment of step L = (q * 9 + tap) * 2 + gs, column block cb:
  // wp[((tap * 8 + 2 q + gs) * 128 + co0 + 16 cb) * 4 + kg]
  const float4 *wl = wp + co0 * 4 + kg;
  auto bload = [&](int L, int cb) -> float4 {
    int q2 = L / 18, r = L - 18 * q2, t2 = r >> 1, g2 = r & 1;
    return wl[(t2 * 8 + 2 * q2 + g2) * 512 + 64 * cb];
  };

  HZ_STAMP(1)
  HZ_STAGE_LOAD8(0)
  HZ_STAGE_STORE8(0)
  __syncthreads();
  HZ_STAMP(2)

  float4 b[2][2];
  b[0][0] = bload(0, 0);
  b[0][1] = bload(0, 1);
  float4 acur[kRB];

#pragma unroll
  for (int q = 0; q < 4; q++) {
    const float *lb = lds + (q & 1) * kBuf;
#pragma unroll
    for (int rb = 0; rb < kRB; rb++) acur[rb] = *(const float4 *)(lb + abase[rb]);
    if (q < 3) { HZ_STAGE_LOAD8(q + 1) }
    for (int tap = 0; tap < 9; tap++) {
      const int toff = ((tap / 3) * 9 + tap % 3) * kLdsRow;
      const int tn = tap < 8 ? tap + 1 : 8;
      const int toffn = ((tn / 3) * 9 + tn % 3) * kLdsRow;
      const int L0 = (q * 9 + tap) * 2;
#pragma unroll
      for (int gs = 0; gs < 2; gs++) {
        const int Ln = L0 + gs + 1 < 72 ? L0 + gs + 1 : 71;
        b[(gs + 1) & 1][0] = bload(Ln, 0);
        b[(gs + 1) & 1][1] = bload(Ln, 1);
        float4 a[kRB];
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) a[rb] = acur[rb];
        const int noff = gs == 0 ? toff + 16 : toffn;
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) acur[rb] = *(const float4 *)(lb + abase[rb] + noff);
        const float4 b0 = b[gs][0], b1 = b[gs][1];
#define HZ_MF(c)                                                                              \
  _Pragma("unroll") for (int rb = 0; rb < kRB; rb++) {                                        \
    acc[rb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb].c, b0.c, acc[rb][0], 0, 0, 0);    \
    acc[rb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb].c, b1.c, acc[rb][1], 0, 0, 0);    \
  }
        HZ_MF(x)
        HZ_MF(y)
        HZ_MF(z)
        HZ_MF(w)
#undef HZ_MF
      }
    }
    if (q < 3) {
      HZ_STAGE_STORE8((q + 1) & 1)
      __syncthreads();
    }
    HZ_STAMP(3 + q)
  }

  // epilogue: C/D row = 4 kg + reg, column = lane & 15
  const float bc0 = bias[co0], bc1 = bias[co0 + 16];
  float *ob = out + (size_t)s0 * 35 * 128 + co0;
  const float *rsb = res ? res + (size_t)s0 * 35 * 128 + co0 : nullptr;
  const int nrow = ns * 35;
  // all 72 residual values requested at once (the A/B/staging registers are
  // dead here): one memory round trip instead of one per row block
  float rv[kRB][2][4];
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) {
    const int rbase = (rh * kRB + rb) * 16 + 4 * kg;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const bool ok = rbase + j < nrow;
      rv[rb][0][j] = rsb && ok ? rsb[(rbase + j) * 128] : 0.f;
      rv[rb][1][j] = rsb && ok ? rsb[(rbase + j) * 128 + 16] : 0.f;
    }
  }
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) {
    const int rbase = (rh * kRB + rb) * 16 + 4 * kg;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (rbase + j < nrow) {
        float v0 = acc[rb][0][j] + bc0, v1 = acc[rb][1][j] + bc1;
        if (rsb) {
          v0 = v0 + rv[rb][0][j];
          v1 = v1 + rv[rb][1][j];
        }
        ob[(rbase + j) * 128] = v0 > 0.f ? v0 : 0.f;
        ob[(rbase + j) * 128 + 16] = v1 > 0.f ? v1 : 0.f;
      }
    }
  }
  HZ_STAMP(7)
#ifdef HZ_NET_DIAG
  if ((t & 255) == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][t >> 8][9] = __builtin_amdgcn_s_memrealtime();
#endif
}
#undef HZ_STAGE_LOAD8
#undef HZ_STAMP
#undef HZ_STAGE_STORE8

}  // namespace

extern "C" int hz_conv3x3_bias_act(const float *x, const float *wpack, const float *bias, const float *res,
                                   float *out, int32_t batch, const int32_t *live, void *stream) {
  if (!x || !wpack || !bias || !out || batch < 0) return -1;
  if (((uintptr_t)x | (uintptr_t)wpack | (uintptr_t)out | (uintptr_t)res) & 15) return -1;
  if (batch == 0) return 0;
  // the 145 KB dynamic-LDS opt-in, once per device
  static std::atomic<uint64_t> init_mask{0};
  const size_t lds = 2 * (size_t)kBuf * sizeof(float);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_conv3x3_w8, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL(k_conv3x3_w8, dim3((batch + kCS - 1) / kCS), dim3(512), lds, (hipStream_t)stream, x,
                     (const float4 *)wpack, bias, res, out, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- the same conv on the bf16 MFMA, fp32-exact products (bf16x6) ---------
//
// v_mfma_f32_16x16x32_bf16 runs 16x the MACs per cycle of the f32 form
// (MI355X_MICROARCH.md: 16 vs 32 cycles for 8192 vs 1024 MACs).  Every fp32
// operand is split exactly into three bf16 pieces, a = a_h + a_m + a_l
// (round-to-nearest at each step: |a_m| <= 2^-8 |a|, |a_l| <= 2^-16 |a|, and
// the three pieces sum to a with no error), and
//     a * b = sum over the pairs (i, j) with i + j <= 2 of a_i * b_j
// up to the dropped pairs (m,l), (l,m), (l,l): |error| <= ~2^-23 |a b|, the
// size of one fp32 rounding.  Each bf16 x bf16 product is exact in the MFMA's
// fp32 accumulation, so the conv keeps fp32 accuracy (tests compare both
// kernels against a float64 conv) with 6 bf16 MFMAs per product block:
// 16/6 = 2.7x the f32 MFMA rate.
//
// Tiling as k_conv3x3_w8 (8 states = 280 rows per 512-thread workgroup;
// wave = row half x 32 output channels: 9 x 2 accumulator tiles of 16x16).
// The input is staged 32 channels at a time (one K-step of 32 per tap),
// split into its three bf16 planes on the way into LDS (the split costs
// VALU once per staged element, not per use); a cell is 3 x 64 B + 32 B of
// padding (224 B: ds_read_b128 conflict-free for the A fragment's lane
// groups), the grid has no halo: a neighbour outside the 5x7 board reads one
// shared zero cell.  Weights are prepacked as bf16 planes
// [tap][ci/32][plane][co][32].  Epilogue as k_conv3x3_w8 (fp32 in HBM).
#ifdef HZ_NET_DIAG
#define HZ_STAMP(k)                                                                   \
  if ((t & 255) == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][t >> 8][k] = __builtin_amdgcn_s_memtime();
#define HZ_STAMP_RT(k)                                                                \
  if ((t & 255) == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][t >> 8][k] = __builtin_amdgcn_s_memrealtime();
#else
#define HZ_STAMP(k)
#define HZ_STAMP_RT(k)
#endif
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
constexpr int kX6Cell = 224;                         // bytes per staged cell
constexpr int kBoardC = 38;                           // encoder board channels (stem input)
constexpr int kX6Zero = 512;                          // bytes of zeros after the cells
constexpr int kX6Buf = kCS * 35 * kX6Cell + kX6Zero;  // one chunk of 8 states + the zero region
static_assert(kCS * 35 * kX6Cell % 256 == 0 && kX6Buf % 256 == 0, "zero region and buffers 256-B aligned");
// padding rows of the class tables read at kX6PadBase + 32 k (+ tap offsets
// of at most 8 cells either way, + 3 planes): a 256-B-aligned point in the
// middle of a chunk buffer, in bounds for every form
constexpr int kX6PadBase = (4 * 35 * kX6Cell) & ~255;
static_assert(kX6PadBase >= 8 * kX6Cell && kX6PadBase + 256 + 64 * 3 + 8 * kX6Cell <= 8 * 35 * kX6Cell,
              "padding reads stay inside an 8-state chunk buffer");
constexpr int kX6SmallMax = 768;                      // batches up to this run one state per workgroup
constexpr int kX6TinyMax = 256;                       // ... and up to this, 8 waves of 16 channels each

__device__ __forceinline__ uint32_t bf16_bits(float v) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)v);
}
__device__ __forceinline__ float bf16_value(uint32_t b) { return __uint_as_float(b << 16); }

// two floats rounded to bf16 (nearest-even) in one v_cvt_pk_bf16_f32: a in
// the low half, b in the high half
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_v;
typedef __attribute__((ext_vector_type(2))) float f32x2_v;
__device__ __forceinline__ uint32_t bf16_pair(float a, float b) {
  const f32x2_v f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_v));
}
__device__ __forceinline__ float bf16_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// the three bf16 planes of four consecutive channels: 8 B per plane; each
// plane's pairs come out of one paired conversion already packed (22 VALU
// per float4 instead of ~38 for per-element conversions and packing; the
// same roundings, so the same bits)
__device__ __forceinline__ void split4(const f32x4 v, uint2 &h, uint2 &m, uint2 &l) {
  const uint32_t h01 = bf16_pair(v[0], v[1]), h23 = bf16_pair(v[2], v[3]);
  const float r0 = v[0] - bf16_lo(h01), r1 = v[1] - bf16_hi(h01);
  const float r2 = v[2] - bf16_lo(h23), r3 = v[3] - bf16_hi(h23);
  const uint32_t m01 = bf16_pair(r0, r1), m23 = bf16_pair(r2, r3);
  const float s0 = r0 - bf16_lo(m01), s1 = r1 - bf16_hi(m01);
  const float s2 = r2 - bf16_lo(m23), s3 = r3 - bf16_hi(m23);
  h = make_uint2(h01, h23);
  m = make_uint2(m01, m23);
  l = make_uint2(bf16_pair(s0, s1), bf16_pair(s2, s3));
}

// Tap classes (8-state tower conv).  On the 5x7 board with zero padding a
// cell on the top row has no dh = -1 neighbours, one on the left column no
// dw = -1 neighbours, and so on: of the 315 (cell, tap) pairs of a state only
// 247 read the board.  The 280 rows of a workgroup are regrouped into 18
// blocks of 16 rows whose cells share (a superset of) their valid taps, and
// a block issues MFMAs only for its taps: 132 block-taps instead of 162
// (-18.5 % MFMA work).  Blocks 0-8 are row half 0, 9-17 row half 1, each
// 66 block-taps: 4 interior blocks (9 taps) and 5 edge blocks (6 taps; the
// corner cells ride in edge blocks whose taps cover theirs).
// kX6ClassRow: the block's rows as state * 35 + cell (-1 - k: padding row,
// not stored, that reads LDS bank slot 2k: see kX6PadBase); kX6ClassTaps:
// each block's taps (bit t = tap t = (dh + 1) * 3 + dw + 1).
// Bank-conflict-free A reads (round 4): a cell's 224-B stride puts row r's
// 16-B K slice kg in bank slot (14 r + kg) mod 16, and a ds_read_b128 serves
// 16 lanes per LDS cycle, lanes {0-3, 12-15} of K slice 2j with lanes {4-11}
// of K slice 2j + 1 (and the reverse): all 16 slots differ exactly when the
// block's positions {0-3, 12-15} hold one row of every residue r mod 8 and
// positions {4-11} another.  Every class has every residue equally often
// (state s adds 35 s = 3 s mod 8), so each block takes two rows per residue;
// the corner rows (one per residue) ride in one block of their class with
// one row per residue of the class (as before), and the 8 padding rows (one
// per residue) in one interior block.  tools/class_table.py generates this
// table and checks it (1,584 LDS cycles per chunk and row half pair for the
// A reads against 3,456 for the round-3 table).
alignas(16) __constant__ int16_t kX6ClassRow[18][16] = {
    {8, 9, 10, 11, 16, 17, 18, 19, 44, 53, 46, 23, 12, 45, 22, 15},  // MM
    {24, 25, 26, 43, 80, 57, 50, 51, 60, 85, 78, 79, 52, 61, 54, 47},  // MM
    {88, 81, 58, 59, 96, 89, 82, 115, 116, 117, 94, 95, 92, 93, 86, 87},  // MM
    {120, 113, 114, 123, 128, 121, 122, 131, 148, 157, 158, 151, 124, 149, 150, 127},  // MM
    {40, 1, 2, 3, 72, 73, 74, 75, 36, 37, 110, 71, 4, 5, 38, 39},  // TM
    {144, 145, 106, 107, 176, 177, 178, 179, 180, 141, 214, 215, 108, 109, 142, 143},  // TM
    {32, 33, 66, 67, 64, 65, 138, 99, 100, 101, 102, 103, 68, 29, 30, 31},  // BM
    {56, 49, 42, 91, 112, 161, 154, 147, 196, 77, 126, 119, 84, 21, 14, 7},  // ML
    {48, 97, 90, 27, 160, 153, 202, 83, 132, 125, 118, 167, 20, 13, 62, 55},  // MR
    {152, 129, 130, 155, 184, 185, 162, 163, 164, 197, 190, 183, 156, 165, 166, 159},  // MM
    {192, 193, 186, 187, 200, 201, 194, 219, 228, 229, 222, 199, 220, 221, 198, 191},  // MM
    {232, 225, 218, 227, 256, 233, 226, 235, 260, 261, 262, 263, 236, 253, 254, 255},  // MM
    {264, 257, 234, 267, -1, -2, -3, -4, -5, -6, -7, -8, 268, 269, 270, 271},  // MM
    {0, 105, 210, 35, 248, 249, 250, 211, 212, 245, 246, 247, 140, 213, 70, 175},  // TM+TL
    {136, 137, 170, 171, 208, 169, 242, 243, 204, 205, 206, 207, 172, 173, 134, 135},  // BM
    {104, 209, 34, 139, 240, 241, 274, 275, 276, 277, 278, 279, 244, 69, 174, 239},  // BM+BR
    {168, 217, 98, 203, 224, 273, 266, 259, 252, 189, 238, 231, 28, 133, 182, 63},  // ML+BL
    {216, 41, 146, 195, 272, 265, 258, 251, 188, 237, 230, 223, 76, 181, 6, 111},  // MR+TR
};
// kX6ClassRowBlk: the same classes with round 3's row placement, for the
// fused residual block: there kX6ClassRow's bank-conflict-free placement
// measured 1.1 % slower per 4,096-row forward (2.303 vs 2.289 ms, same box,
// alternating processes, bit-identical; profiles/r04/blk3/fwd_ab.log): the
// block's LDS energy saved came back as a lower clock elsewhere
alignas(16) __constant__ int16_t kX6ClassRowBlk[18][16] = {
    {8, 9, 10, 11, 12, 15, 16, 17, 18, 19, 22, 23, 24, 25, 26, 43},  // MM
    {44, 45, 46, 47, 50, 51, 52, 53, 54, 57, 58, 59, 60, 61, 78, 79},  // MM
    {80, 81, 82, 85, 86, 87, 88, 89, 92, 93, 94, 95, 96, 113, 114, 115},  // MM
    {116, 117, 120, 121, 122, 123, 124, 127, 128, 129, 130, 131, 148, 149, 150, 151},  // MM
    {1, 2, 3, 4, 5, 36, 37, 38, 39, 40, 71, 72, 73, 74, 75, 106},  // TM
    {107, 108, 109, 110, 141, 142, 143, 144, 145, 176, 177, 178, 179, 180, 211, 212},  // TM
    {29, 30, 31, 32, 33, 64, 65, 66, 67, 68, 99, 100, 101, 102, 103, 134},  // BM
    {7, 14, 21, 42, 49, 56, 77, 84, 91, 112, 119, 126, 147, 154, 161, 182},  // ML
    {13, 20, 27, 48, 55, 62, 83, 90, 97, 118, 125, 132, 153, 160, 167, 188},  // MR
    {152, 155, 156, 157, 158, 159, 162, 163, 164, 165, 166, 183, 184, 185, 186, 187},  // MM
    {190, 191, 192, 193, 194, 197, 198, 199, 200, 201, 218, 219, 220, 221, 222, 225},  // MM
    {226, 227, 228, 229, 232, 233, 234, 235, 236, 253, 254, 255, 256, 257, 260, 261},  // MM
    {262, 263, 264, 267, 268, 269, 270, 271, -1, -1, -1, -1, -1, -1, -1, -1},  // MM
    {213, 214, 215, 246, 247, 248, 249, 250, 0, 35, 70, 105, 140, 175, 210, 245},  // TM
    {135, 136, 137, 138, 169, 170, 171, 172, 173, 204, 205, 206, 207, 208, 239, 240},  // BM
    {241, 242, 243, 274, 275, 276, 277, 278, 34, 69, 104, 139, 174, 209, 244, 279},  // BM
    {189, 196, 217, 224, 231, 252, 259, 266, 28, 63, 98, 133, 168, 203, 238, 273},  // ML
    {195, 202, 223, 230, 237, 258, 265, 272, 6, 41, 76, 111, 146, 181, 216, 251},  // MR
};
// kX6ClassSel: the block taps some of whose rows (the corner cells) read
// off the board: only those need the zero-region redirect
constexpr uint32_t kX6ClassSel[3][9] = {
    {0x000, 0x000, 0x000, 0x000, 0x000, 0x000, 0x000, 0x000, 0x000},
    {0x000, 0x000, 0x000, 0x000, 0x048, 0x000, 0x024, 0x180, 0x003},
    {0x000, 0x000, 0x000, 0x1c0, 0x000, 0x168, 0x000, 0x180, 0x0c0},  // 4-state groups (kX6C4Row)
};
constexpr uint32_t kX6ClassTaps[3][9] = {
    {0x1ff, 0x1ff, 0x1ff, 0x1ff, 0x1f8, 0x1f8, 0x03f, 0x1b6, 0x0db},
    {0x1ff, 0x1ff, 0x1ff, 0x1ff, 0x1f8, 0x03f, 0x03f, 0x1b6, 0x0db},
    {0x1ff, 0x1ff, 0x1ff, 0x1ff, 0x1f8, 0x1f8, 0x03f, 0x1b6, 0x0db},  // 4-state groups (kX6C4Row)
};
// The same grouping for 4 states (140 rows, 9 blocks; class index 2 of the
// tables above): 4 nine-tap blocks (the 60 interior cells and 4 BM cells),
// TM (+ the TL, TR corners: two blocks, 4 padding rows), BM, ML (+ BL), MR
// (+ BR): 66 block-taps, half of the 8-state groups' 132 (tools: the
// generator in DESIGN.md §3, k_conv3x3_x6 CS = 4 row)
alignas(16) __constant__ int16_t kX6C4Row[9][16] = {
    {8, 9, 10, 11, 12, 15, 16, 17, 18, 19, 22, 23, 24, 25, 26, 43},
    {44, 45, 46, 47, 50, 51, 52, 53, 54, 57, 58, 59, 60, 61, 78, 79},
    {80, 81, 82, 85, 86, 87, 88, 89, 92, 93, 94, 95, 96, 113, 114, 115},
    {116, 117, 120, 121, 122, 123, 124, 127, 128, 129, 130, 131, 135, 136, 137, 138},
    {1, 2, 3, 4, 5, 36, 37, 38, 39, 40, 71, 72, 73, 74, 75, 106},
    {107, 108, 109, 110, 0, 35, 70, 105, 6, 41, 76, 111, -1, -1, -1, -1},
    {29, 30, 31, 32, 33, 64, 65, 66, 67, 68, 99, 100, 101, 102, 103, 134},
    {7, 14, 21, 42, 49, 56, 77, 84, 91, 112, 119, 126, 28, 63, 98, 133},
    {13, 20, 27, 48, 55, 62, 83, 90, 97, 118, 125, 132, 34, 69, 104, 139},
};

// NQ chunks of 32 input channels.  Stem: x is the encoder's NCHW board
// [B][38][5][7] (channels >= 38 stage as zeros; NQ = 2), else an NHWC
// [B][5][7][128] activation (NQ = 4).
// CS states per workgroup: 8 (8 waves: row half x 32 output channels, 9 row
// blocks each), or 1 for small batches (4 waves: 32 output channels, the
// state's 35 rows as 3 row blocks): a workgroup's time is its waves' MFMA
// chain (8 states: ~175 k cycles, ~73 us, however few states are live), and
// the arena's batches of a few dozen boards fill only a few CUs; one state
// per group cuts each wave's chain to a third at 48/35 rows of waste.
template <int NQ, bool Stem, int CS, int NCB>
__global__ void __launch_bounds__((CS == 8 ? 2 : 1) * (8 / NCB) * 64, CS == 4 ? 2 : 1)
    k_conv3x3_x6(const float *__restrict__ x, const bf16x8 *__restrict__ wp, const float *__restrict__ bias,
                 const float *__restrict__ res, float *__restrict__ out, int32_t batch,
                 const int32_t *__restrict__ live) {
  static_assert(CS == 8 || CS == 4 || CS == 1, "8, 4 or 1 states per workgroup");
  static_assert(NCB == 2 || NCB == 1, "column blocks of 16 output channels per wave");
  constexpr int kRowsT = CS * 35;                  // output rows of the group
  constexpr int kRBT = CS == 1 ? 3 : 9;            // row blocks of 16 per wave
  constexpr int kCG = 8 / NCB;                     // column groups (waves per row group)
  constexpr int kThreads = (CS == 8 ? 2 : 1) * kCG * 64;
  constexpr int kStg = (kRowsT * 8 + kThreads - 1) / kThreads;  // float4 staged per thread per chunk
  constexpr int kZero = (CS * 35 * kX6Cell + 255) / 256 * 256;   // zero region: 256-B aligned (banks)
  constexpr int kBufT = kZero + kX6Zero;                          // one chunk's buffer + zero region
  static_assert((CS == 8 ? 2 : 1) * kRBT * 16 >= kRowsT, "row blocks cover the rows");
  extern __shared__ float4 lds4[];
  char *lds = (char *)lds4;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kg = lane >> 4, rh = w / kCG, cg = w % kCG;
  const int s0 = blockIdx.x * CS;
  if (live) batch = *live < batch ? *live : batch;  // rows past the live count are not computed
  if (s0 >= batch) return;
  const int ns = batch - s0 < CS ? batch - s0 : CS;
  HZ_STAMP(0)
  HZ_STAMP_RT(8)

  if (t < 2 * kX6Zero / 16) {  // both buffers' zero regions
    const int b = t / (kX6Zero / 16), k = t - b * (kX6Zero / 16);
    *(float4 *)(lds + b * kBufT + kZero + 16 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // staging: float4 f of a chunk = (row sc, channels 4 (f & 7) ..), sc = f >> 3
  // with bits 0 and 1 swapped: the 16 lanes of an LDS store cycle cover rows
  // r and r + 2, whose plane slices fall in disjoint bank halves (as
  // k_conv3x3_x6w4's srow; rows stay within their group of four, so every
  // row index stays below kRowsT)
  f32x4 stg[kStg];
  int gsrc[kStg], ldst[kStg];
#pragma unroll
  for (int it = 0; it < kStg; it++) {
    int f = it * kThreads + t;
    f = f < kRowsT * 8 ? f : kRowsT * 8 - 1;
    const int r0 = f >> 3;
    const int sc = (r0 & ~3) | ((r0 & 1) << 1) | ((r0 >> 1) & 1), part = f & 7, s = sc / 35, cell = sc - 35 * s;
    if constexpr (Stem)  // board element (state, channel 4 part, cell); channel offset added per chunk
      gsrc[it] = (s < ns ? s0 + s : s0 + ns - 1) * (kBoardC * 35) + 4 * part * 35 + cell;
    else
      gsrc[it] = (s < ns ? s0 * 35 + sc : (s0 + ns - 1) * 35 + cell) * 128 + 4 * part;
    ldst[it] = sc * kX6Cell + 8 * part;
  }
  // stem: the four channels 32 q + 4 part + j of a slot (part from the
  // clamped slot index, as in gsrc: an unclamped part would read up to 26
  // channels past a state, beyond the end of the last one).  Channel 37
  // (phase / 3: 1/3 and 2/3 are not bf16 values) stages as its three bf16
  // pieces in slots 37, 38, 39, whose weights are packed as the planes
  // (h, m, l), (h, m, 0), (h, 0, 0) of w37: the same six products as
  // splitting it in place, but every staged value of an encoder board is then
  // a bf16 value, which lets the chunk skip the A pieces' products (below).
  // Slots past 39 stage as zeros.
  // The second chunk stages slots 32-39 in every K slice pair (part p as
  // part p & 1): its tap-packed K-steps read slice 0 in lane groups kg = 0, 2
  // and the copy in slice 1 in kg = 1, 3 (aoff_tp), so the 16 lanes of an
  // LDS cycle (positions {0-3, 12-15} of one group, {4-11} of the next: the
  // class table's pairing) fall in even and odd bank slots; all reading
  // slice 0 put them on the even slots only: 2-way conflicts on a third of
  // the stem's A reads (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.236)
  auto stem_load = [&](int it, int q) -> f32x4 {
    f32x4 v;
    int f = it * kThreads + t;
    f = f < kRowsT * 8 ? f : kRowsT * 8 - 1;
    const int part = f & 7, pe = q == 1 ? (part & 1) : part;
    const int c0 = 32 * q + 4 * pe, src = gsrc[it] + 4 * (pe - part) * 35;
    if (c0 == 36) {
      v[0] = x[src + (32 * q) * 35];
      const float p = x[src + (32 * q + 1) * 35];
      const float h = bf16_value(bf16_bits(p)), r = p - h, m = bf16_value(bf16_bits(r));
      v[1] = h;
      v[2] = m;
      v[3] = bf16_value(bf16_bits(r - m));
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = c0 + j < kBoardC - 1 ? x[src + (32 * q + j) * 35] : 0.f;
    }
    return v;
  };
  static_assert(kBoardC == 38, "stem_load places the phase channel 37 in slots 37-39");
#define HZ_X6_LOAD(q)                                                                     \
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                        \
  if constexpr (Stem) {                                                                   \
    _Pragma("unroll") for (int it = 0; it < kStg; it++) stg[it] = stem_load(it, q);       \
  } else {                                                                                \
    _Pragma("unroll") for (int it = 0; it < kStg; it++)                                   \
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(stg[it]) : "v"(x + gsrc[it] + 32 * (q))); \
  }
  // the wait names the staged registers, so the split's arithmetic (which,
  // unlike an LDS store, could move above a plain asm statement) waits too
  static_assert(kStg == 5 || kStg == 2 || kStg == 1, "HZ_X6_STORE ties five, two or one staging registers");
#define HZ_X6_STORE(buf)                                                                  \
  if constexpr (kStg == 5)                                                                \
    asm volatile("s_waitcnt vmcnt(0)"                                                     \
                 : "+v"(stg[0]), "+v"(stg[1]), "+v"(stg[2]), "+v"(stg[3]), "+v"(stg[4])    \
                 :                                                                        \
                 : "memory");                                                             \
  else if constexpr (kStg == 2)                                                           \
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(stg[0]), "+v"(stg[1]) : : "memory");         \
  else                                                                                    \
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(stg[0]) : : "memory");                       \
  _Pragma("unroll") for (int it = 0; it < kStg; it++) {                                   \
    uint2 h_, m_, l_;                                                                     \
    split4(stg[it], h_, m_, l_);                                                          \
    char *d_ = lds + (buf) * kBufT + ldst[it];                                            \
    *(uint2 *)d_ = h_;                                                                    \
    *(uint2 *)(d_ + 64) = m_;                                                             \
    *(uint2 *)(d_ + 128) = l_;                                                            \
    pieces |= m_.x | m_.y | l_.x | l_.y;                                                  \
  }
  // the chunk's A pieces m, l are all zero (every staged value is a bf16
  // value: an encoder board's stem input): only the h plane's three products
  // are issued.  Workgroup-uniform; the tower always takes all six.
#define HZ_X6_SYNC(dst)                                                                   \
  if constexpr (Stem) {                                                                   \
    dst = __builtin_amdgcn_readfirstlane(__syncthreads_or(pieces != 0));                  \
    pieces = 0;                                                                           \
  } else {                                                                                \
    __syncthreads();                                                                      \
  }

  // A fragment of row block rb, tap: the lane's row r = (rh*9 + rb)*16 + (lane & 15)
  // (clamped), its cell (h, w) of state s; neighbour (h + dh - 1, w + dw - 1)
  // or, off the board, the zero region at the same offset mod 256 (so the
  // lane keeps the LDS banks its row would use).
  // valid[rb] bit tap = the neighbour is on the board.
  // the 8-state tower groups its rows by tap class (above)
  constexpr bool kClassed = CS != 1 && NCB == 2;  // the 8-state forms (tower conv, stem), the 4-state one
  // the class table's row of block idx (CS = 4: its own 9-block table, class index 2)
  auto class_row = [&](int idx, int i) -> int { return CS == 4 ? kX6C4Row[idx][i] : kX6ClassRow[idx][i]; };
  int cbase[kRBT];
  uint32_t valid[kRBT];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++) {
    int r = (rh * kRBT + rb) * 16 + (lane & 15);
    int pad = -1;  // CS = 8: a padding row (-1 - k) reads anything in bounds at bank slot 2k (kX6ClassRow)
    if constexpr (kClassed) {
      r = class_row(rh * kRBT + rb, lane & 15);
      if constexpr (CS == 8) {
        pad = r >= 0 ? -1 : -1 - r;
        r = r >= 0 ? r : 0;
      } else {
        r = r >= 0 ? r : class_row(rh * kRBT + rb, 0);  // CS = 4: padding rows read a real row (not stored)
      }
    }
    r = r < kRowsT ? r : kRowsT - 1;
    const int s = r / 35, cell = r - 35 * s, ch = cell / 7, cw = cell - 7 * ch;
    cbase[rb] = (pad < 0 ? r * kX6Cell : kX6PadBase + 32 * pad) + 16 * kg;
    uint32_t v = 0;
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
      const int hh = ch + tap / 3 - 1, ww = cw + tap % 3 - 1;
      v |= (uint32_t)(hh >= 0 && hh < 5 && ww >= 0 && ww < 7) << tap;
    }
    valid[rb] = pad < 0 ? v : 0x1ffu;
  }
  // classed: the epilogue's rows (transposed tiles: lane -> row lane >> 2),
  // read from the table now so that their latency is long hidden
  int erow[kClassed ? kRBT : 1];
  if constexpr (kClassed) {
#pragma unroll
    for (int rb = 0; rb < kRBT; rb++) erow[rb] = class_row(rh * kRBT + rb, lane >> 2);
  }
  auto aoff = [&](int rb, int tap) -> int {
    const int d = ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell;
    const int a = cbase[rb] + d;
    return (valid[rb] >> tap) & 1 ? a : kZero + (a & 255);
  };
  // the stem's second chunk holds only slots 32-39 (channels 32-36, the
  // phase channel's three pieces): its K-steps take 8 channels x 4 taps
  // instead of 32 channels x 1 tap, lane group kg reading tap 4 s + kg
  // (zero past tap 8): 3 K-steps instead of 9 (weights packed to match,
  // hzamd/infer.py pack_stem_x6)
  auto aoff_tp = [&](int rb, int st) -> int {
    const int tap = 4 * st + kg, base = cbase[rb] - 16 * kg + 16 * (kg & 1);  // slice 0 or its copy in 1
    if (tap >= 9) return kZero + (base & 255);
    const int a = base + ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell;
    return (valid[rb] >> tap) & 1 ? a : kZero + (a & 255);
  };

  f32x4 acc[kRBT][NCB];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++)
#pragma unroll
    for (int cb = 0; cb < NCB; cb++) acc[rb][cb] = (f32x4){};

  const int co0 = 16 * NCB * cg + (lane & 15);
  // B fragment of K-step L = q * 9 + tap, plane p, column block cb:
  // wp[(((tap * NQ + q) * 3 + p) * 128 + co0 + 16 cb) * 4 + kg]   (bf16x8 units)
  const bf16x8 *wl = wp + co0 * 4 + kg;
  auto bload = [&](int L, int p, int cb) -> bf16x8 {
    const int q2 = L / 9, t2 = L - 9 * q2;
    return wl[((t2 * NQ + q2) * 3 + p) * 512 + 64 * cb];
  };

  uint32_t pieces = 0;
  int npa = 3, npa_next = 3;  // A planes issued for this chunk, the next one
  HZ_STAMP(1)
  HZ_X6_LOAD(0)
  HZ_X6_STORE(0)
  HZ_X6_SYNC(npa)
  if constexpr (Stem) npa = npa ? 3 : 1;
  HZ_STAMP(2)

  bf16x8 b[3][NCB], bn[3][NCB];  // this K-step's B fragments, the next step's (loaded a step ahead)
#pragma unroll
  for (int p = 0; p < 3; p++)
#pragma unroll
    for (int cb = 0; cb < NCB; cb++) b[p][cb] = bload(0, p, cb);

  // classed main loop: the chunk loop rolled, the taps unrolled, one copy
  // per row half (its blocks' tap sets are compile-time constants).  The
  // stem (two chunks, unrolled): its second chunk is tap-packed (a K-step
  // holds 4 taps), where every block issues all 3 K-steps as in the
  // unclassed loop
  auto classed = [&](auto half) {
    constexpr int H = decltype(half)::value;
    auto taps = [&](int q, const char *lb) __attribute__((always_inline)) {
#pragma unroll
      for (int tap = 0; tap < 9; tap++) {
        const int L = q * 9 + tap, Ln = L + 1 < 9 * NQ ? L + 1 : 9 * NQ - 1;
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
          for (int cb = 0; cb < NCB; cb++) bn[p][cb] = bload(Ln, p, cb);
#pragma unroll
        for (int pa = 0; pa < 3; pa++) {
          if (Stem && pa >= npa) break;  // the chunk's A pieces m, l are zero (stem on encoder boards)
          bf16x8 a[kRBT];
#pragma unroll
          for (int rb = 0; rb < kRBT; rb++) {
            if (!((kX6ClassTaps[H][rb] >> tap) & 1)) continue;
            // a tap every row of the block reads on the board: base + a
            // non-negative immediate (lbm is lb less the largest negative
            // neighbour offset), no per-tap address register
            constexpr int kNeg = 8 * kX6Cell;
            const int d = ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell + kNeg + 64 * pa;
            a[rb] = (kX6ClassSel[H][rb] >> tap) & 1 ? *(const bf16x8 *)(lb + aoff(rb, tap) + 64 * pa)
                                                    : *(const bf16x8 *)(lb - kNeg + cbase[rb] + d);
          }
#pragma unroll
          for (int pb = 0; pb < 3 - pa; pb++)
#pragma unroll
            for (int rb = 0; rb < kRBT; rb++)
              if ((kX6ClassTaps[H][rb] >> tap) & 1)
#pragma unroll
                for (int cb = 0; cb < NCB; cb++)
                  acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[pb][cb], acc[rb][cb], 0, 0, 0);
        }
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
          for (int cb = 0; cb < NCB; cb++) b[p][cb] = bn[p][cb];
        __builtin_amdgcn_sched_barrier(0);  // taps stay in order (registers: no hoisting across)
      }
    };
    if constexpr (Stem) {
      static_assert(NQ == 2, "the stem has two chunks");
      HZ_X6_LOAD(1)
      taps(0, lds);
      HZ_X6_STORE(1)
      HZ_X6_SYNC(npa_next)
      npa = npa_next ? 3 : 1;
      HZ_STAMP(3)
      const char *lb = lds + kBufT;
#pragma unroll
      for (int st = 0; st < 3; st++) {
        const int L = 9 + st, Ln = L + 1;
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
          for (int cb = 0; cb < NCB; cb++) bn[p][cb] = bload(Ln, p, cb);
#pragma unroll
        for (int pa = 0; pa < 3; pa++) {
          if (pa >= npa) break;
          bf16x8 a[kRBT];
#pragma unroll
          for (int rb = 0; rb < kRBT; rb++) a[rb] = *(const bf16x8 *)(lb + aoff_tp(rb, st) + 64 * pa);
#pragma unroll
          for (int pb = 0; pb < 3 - pa; pb++)
#pragma unroll
            for (int rb = 0; rb < kRBT; rb++)
#pragma unroll
              for (int cb = 0; cb < NCB; cb++)
                acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[pb][cb], acc[rb][cb], 0, 0, 0);
        }
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
          for (int cb = 0; cb < NCB; cb++) b[p][cb] = bn[p][cb];
      }
      HZ_STAMP(4)
    } else {
      for (int q = 0; q < NQ; q++) {
        const char *lb = lds + (q & 1) * kBufT;
        if (q < NQ - 1) { HZ_X6_LOAD(q + 1) }
        taps(q, lb);
        if (q < NQ - 1) {
          HZ_X6_STORE((q + 1) & 1)
          HZ_X6_SYNC(npa_next)
        }
        HZ_STAMP(3 + q)
      }
    }
  };
  if constexpr (kClassed && CS == 4) {
    classed(std::integral_constant<int, 2>{});
  } else if constexpr (kClassed) {
    if (rh == 0)
      classed(std::integral_constant<int, 0>{});
    else
      classed(std::integral_constant<int, 1>{});
  } else

  {
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const char *lb = lds + (q & 1) * kBufT;
      if (q < NQ - 1) { HZ_X6_LOAD(q + 1) }
      const bool packed = Stem && q == 1;  // tap-packed K-steps (above)
      for (int tap = 0; tap < (packed ? 3 : 9); tap++) {
        const int L = q * 9 + tap, Ln = L + 1 < 9 * NQ ? L + 1 : 9 * NQ - 1;
  #pragma unroll
        for (int p = 0; p < 3; p++)
  #pragma unroll
          for (int cb = 0; cb < NCB; cb++) bn[p][cb] = bload(Ln, p, cb);
        // plane a of A against the planes b with a + b <= 2
  #pragma unroll
        for (int pa = 0; pa < 3; pa++) {
          if (pa >= npa) break;
          bf16x8 a[kRBT];
  #pragma unroll
          for (int rb = 0; rb < kRBT; rb++)
            a[rb] = *(const bf16x8 *)(lb + (packed ? aoff_tp(rb, tap) : aoff(rb, tap)) + 64 * pa);
  #pragma unroll
          for (int pb = 0; pb < 3 - pa; pb++) {
  #pragma unroll
            for (int rb = 0; rb < kRBT; rb++)
  #pragma unroll
              for (int cb = 0; cb < NCB; cb++)
                acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[pb][cb], acc[rb][cb], 0, 0, 0);
          }
        }
  #pragma unroll
        for (int p = 0; p < 3; p++)
  #pragma unroll
          for (int cb = 0; cb < NCB; cb++) b[p][cb] = bn[p][cb];
      }
      if (q < NQ - 1) {
        HZ_X6_STORE((q + 1) & 1)
        HZ_X6_SYNC(npa_next)
        if constexpr (Stem) npa = npa_next ? 3 : 1;
      }
      HZ_STAMP(3 + q)
    }
  }

  // Epilogue, out = relu((acc + bias) + res), through a per-wave LDS
  // transpose of each 16x16 tile: a lane then holds 4 consecutive output
  // channels of one row, so the residual loads and the stores are float4
  // (a quarter of the memory instructions of per-element ones, which took
  // ~17-21 k cycles per workgroup with the MFMA pipes idle).  The tile lives
  // in buffer 0, which no wave reads after the last chunk's barrier (the last
  // chunk is in buffer 1: NQ is even).
  static_assert(NQ % 2 == 0, "the last chunk is staged in buffer 1");
  // tile row stride (floats): 16-B aligned rows, conflict-free column writes
  // (16 where 20 would not fit: one state, 8 waves)
  constexpr int kTS = kThreads / 64 * 16 * 20 * 4 <= kZero ? 20 : 16;
  static_assert(kThreads / 64 * 16 * kTS * 4 <= kBufT, "per-wave tiles fit in buffer 0");
  // kT tiles per round (one wave barrier pair per round): 6 where they fit
  constexpr int kT = kThreads / 64 * 6 * 16 * kTS * 4 <= kZero && (kRBT * NCB) % 6 == 0 ? 6 : 1;
  float *tile = (float *)lds + w * 16 * kTS * kT;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  const int cow = 16 * NCB * cg + tcol;  // this lane's first output channel (column block 0)
  const int nrow = ns * 35;
  const size_t gbase = (size_t)s0 * 35 * 128;
  // the lane's output row (within the group) of block rb; -1: not stored
  auto orow = [&](int rb) -> int {
    int row = (rh * kRBT + rb) * 16 + trow;
    if constexpr (kClassed) row = erow[rb];
    return row >= 0 && row < nrow ? row : -1;
  };
  float4 rv[kRBT][NCB];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++) {
    const int row = orow(rb);
#pragma unroll
    for (int cb = 0; cb < NCB; cb++)
      rv[rb][cb] = res && row >= 0 ? *(const float4 *)(res + gbase + (size_t)row * 128 + cow + 16 * cb)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 bv[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; cb++) bv[cb] = *(const float4 *)(bias + cow + 16 * cb);
#pragma unroll
  for (int r0 = 0; r0 < kRBT * NCB; r0 += kT) {
#pragma unroll
    for (int k = 0; k < kT; k++) {
      const int rb = (r0 + k) / NCB, cb = (r0 + k) % NCB;
#pragma unroll
      for (int j = 0; j < 4; j++) tile[k * 16 * kTS + (4 * kg + j) * kTS + (lane & 15)] = acc[rb][cb][j];
    }
    __builtin_amdgcn_wave_barrier();
    float4 a4[kT];
#pragma unroll
    for (int k = 0; k < kT; k++) a4[k] = *(const float4 *)(tile + k * 16 * kTS + trow * kTS + tcol);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < kT; k++) {
      const int rb = (r0 + k) / NCB, cb = (r0 + k) % NCB;
      const int row = orow(rb);
      if (row >= 0) {
        float4 v;
        v.x = a4[k].x + bv[cb].x;
        v.y = a4[k].y + bv[cb].y;
        v.z = a4[k].z + bv[cb].z;
        v.w = a4[k].w + bv[cb].w;
        if (res) {
          v.x = v.x + rv[rb][cb].x;
          v.y = v.y + rv[rb][cb].y;
          v.z = v.z + rv[rb][cb].z;
          v.w = v.w + rv[rb][cb].w;
        }
        v.x = v.x > 0.f ? v.x : 0.f;
        v.y = v.y > 0.f ? v.y : 0.f;
        v.z = v.z > 0.f ? v.z : 0.f;
        v.w = v.w > 0.f ? v.w : 0.f;
        *(float4 *)(out + gbase + (size_t)row * 128 + cow + 16 * cb) = v;
      }
    }
  }
  HZ_STAMP(7)
  HZ_STAMP_RT(9)
}
#undef HZ_X6_LOAD
#undef HZ_X6_STORE
#undef HZ_X6_SYNC

}  // namespace

// ---- the tower conv with one wave per SIMD (the default at > 768 rows) ----
//
// k_conv3x3_x6<4, false, 8, 2>'s arithmetic (the same bf16x6 products in the
// same K order per output, the same epilogue: bit-identical outputs) with 4
// waves of up to 512 registers instead of 8 of 256: wave w = (row half
// rh = w >> 1, output channels 64 (w & 1) .. +64), 9 row blocks x 4 column
// blocks = 36 accumulator tiles (144 registers).
//  - every A fragment read from LDS feeds twice the MFMAs: half the LDS read
//    bytes per MFMA (LDS bytes cost power, and the chip holds its clock down
//    under this kernel);
//  - the next chunk's staging no longer runs as a block before the chunk's
//    barrier: its global loads are issued after tap 0's wait and each staged
//    float4 is split and stored between the MFMAs of taps 2-7, so only the
//    barrier itself separates the chunks;
//  - every vector-memory load of the main loop is an asm statement, issued in
//    program order, so one counted wait per tap (vmcnt 12: the next K-step's
//    B fragments stay in flight) covers this K-step's B fragments and the
//    staged chunk.
#ifndef HZ_KO
#define HZ_KO 0  // knock-out bits of diagnostic builds (tools/Makefile variants): results are wrong
#endif
namespace {
constexpr int kW4Stg = (kRows * 8 + 255) / 256;  // float4 staged per thread per chunk (9)

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// row blocks of row half h whose tap set holds tap
constexpr int x6_class_blocks(int h, int tap) {
  int k = 0;
  for (int rb = 0; rb < 9; rb++) k += (kX6ClassTaps[h][rb] >> tap) & 1;
  return k;
}

// Block = true: the whole residual block (model.py:287-299, BN folded),
// out = relu(conv2(relu(conv1(x) + b1)) + b2 + x), in one launch.  The chunk
// loop runs over NG = 8 chunks (conv1's four, then conv2's); at the switch
// each wave turns its conv1 accumulators into relu(acc + b1) (the values the
// layered conv1 stores) and conv2's chunks are staged from them exactly as
// the layered conv2 stages them from HBM (same split, same planes), so the
// result is bit-identical to the two layered convs.  Wave (rh, chf) holds
// output channels 64 chf .. +64 of its row half; at the switch
//  - chunk 0 (chf = 0, column blocks 0-1) goes into buffer 0 (last read in
//    conv1's chunk 2) as bf16 planes, chunk 2 (chf = 1, blocks 0-1) into
//    region E as fp32 rows;
//  - chunks 1 and 3 (blocks 2-3) go to tmp, the group's slice of a global
//    scratch ([2][288][32] fp32 per group: L2-resident until read);
// then conv2's chunks 0, 1, 2 stage chunk 1 (tmp), 2 (E) and 3 (tmp) into
// the other buffer as the HBM staging does.
// LDS: two chunk buffers + E (280 rows x 32 fp32) = 162,304 B.
// Cf (Block only): the fused block with the bank-conflict-free row table
// kX6ClassRow instead of round 3's kX6ClassRowBlk (hz_resblock_x6_set_table;
// the same bits: the table only places the rows)
template <bool Block, bool Cf = false>
__device__ __forceinline__ const int16_t (*x6_tab())[16] {
  if constexpr (Block && !Cf) return kX6ClassRowBlk;
  return kX6ClassRow;
}
// Tower (Block only): the body runs once per residual block of a tower in
// one launch (k_x6w4_tower): the activation it reads was written by this
// workgroup's previous block, so its loads (staging, the skip, tmp) are
// non-temporal (they bypass the CU's L1, which may hold the previous
// block's lines) and the thread index is made opaque per block (nothing
// derived from it is hoisted across blocks into registers)
template <bool NT>
__device__ __forceinline__ f32x4 x6_ld4(const float *p) {
  if constexpr (NT) return __builtin_nontemporal_load((const f32x4 *)p);
  return *(const f32x4 *)p;
}
template <bool NT>
__device__ __forceinline__ float4 x6_ld4f(const float *p) {
  if constexpr (NT) {
    const f32x4 v = __builtin_nontemporal_load((const f32x4 *)p);
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  return *(const float4 *)p;
}
// Tower: from the second block on, x and out are the same buffer (the skip
// input is the block input, overwritten by the block's output), so they are
// not declared __restrict__ there
template <bool Tower>
using X6In = std::conditional_t<Tower, const float *, const float *__restrict__>;
template <bool Tower>
using X6Out = std::conditional_t<Tower, float *, float *__restrict__>;
template <bool Block, bool Cf, bool Tower>
__device__ __forceinline__ void x6w4_body(X6In<Tower> x, const bf16x8 *__restrict__ wp,
                                          const float *__restrict__ bias, X6In<Tower> res,
                                          X6Out<Tower> out, int32_t batch, const int32_t *__restrict__ live,
                                          const bf16x8 *__restrict__ wp2, const float *__restrict__ bias2,
                                          float *__restrict__ tmp) {
  constexpr int NQ = 4, kRBT = 9, NCB = 4, NG = Block ? 8 : 4;
  constexpr int kZero = kCS * 35 * kX6Cell;  // 62,720 B: 256-B aligned
  constexpr int kBufT = kZero + kX6Zero;
  constexpr int kE = 2 * kBufT;              // Block: region E, fp32 [280][32]
  static_assert(kZero % 256 == 0, "zero region 256-B aligned");
  // E has a 281st row and a dummy cell after it: the padding rows of the
  // switch write there (no branch per value)
  constexpr int kDummyCell = kE + (kRows + 1) * 128;
  static_assert(kDummyCell + kX6Cell <= 160 * 1024, "buffers, E and the dummy cell fit the LDS");
  extern __shared__ float4 lds4[];
  char *lds = (char *)lds4;
  int t0 = threadIdx.x;
  if constexpr (Tower) asm volatile("" : "+v"(t0));
  __builtin_assume(t0 >= 0 && t0 < 256);
  const int t = t0, lane = t & 63, w = t >> 6, kg = lane >> 4, rh = w >> 1, chf = w & 1;
  const int s0 = blockIdx.x * kCS;
  if (live) batch = *live < batch ? *live : batch;
  if (s0 >= batch) return;
  const int ns = batch - s0 < kCS ? batch - s0 : kCS;
  HZ_STAMP(0)
  HZ_STAMP_RT(8)

  if (t < 2 * kX6Zero / 16) {
    const int b = t / (kX6Zero / 16), k = t - b * (kX6Zero / 16);
    *(float4 *)(lds + b * kBufT + kZero + 16 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // staging: float4 f of a chunk = (row sc = srow(f), channels 4 (f & 7) ..);
  // srow swaps bits 0 and 1 of f >> 3, so that the 16 lanes of each LDS
  // store cycle (ds_write_b64: 16 contiguous lanes, 32 banks) cover rows r
  // and r + 2, whose 64-B plane slices fall in disjoint bank halves (rows r,
  // r + 1 at the 224-B cell stride share a quarter: 2-way conflicts; tools/
  // class_table.py); the addresses are recomputed per use (registers are the
  // constraint here)
  f32x4 stg[kW4Stg];
  auto stage_f = [&](int it) {
    const int f = it * 256 + t;
    return f < kRows * 8 ? f : kRows * 8 - 1;
  };
  auto srow = [](int f) {
    const int r = f >> 3;
    return (r & ~3) | ((r & 1) << 1) | ((r >> 1) & 1);
  };
  const int last_row = s0 * 35 + ns * 35 - 1;  // rows past the batch reread its last one
  // Block: the thread index made opaque per chunk, so the staging addresses
  // of the three sources are recomputed at each use, not kept in registers
  auto opaque_t = [&]() __attribute__((always_inline)) {
    int tt = t;
    if constexpr (Block) asm volatile("" : "+v"(tt));
    return tt;
  };
  auto stage_issue = [&](int q) __attribute__((always_inline)) {
    const int tt = opaque_t();
#pragma unroll
    for (int it = 0; it < kW4Stg; it++) {
      int f = it * 256 + tt;
      f = f < kRows * 8 ? f : kRows * 8 - 1;
      const int sc = s0 * 35 + srow(f);
      stg[it] = x6_ld4<Tower>(x + (size_t)(sc < last_row ? sc : last_row) * 128 + 4 * (f & 7) + 32 * q);
    }
  };
  // Block: conv2's chunk 2 from region E, chunks 1 and 3 from tmp (fp32 rows of 32 channels)
  constexpr int kTmpRows = 288;  // a group's tmp slice: [2][288][32] (row 280: padding rows' writes)
  float *const tmpg = Block ? tmp + (size_t)blockIdx.x * 2 * kTmpRows * 32 : nullptr;
  auto stage_issue_e = [&]() __attribute__((always_inline)) {
    const int tt = opaque_t();
#pragma unroll
    for (int it = 0; it < kW4Stg; it++) {
      int f = it * 256 + tt;
      f = f < kRows * 8 ? f : kRows * 8 - 1;
      stg[it] = *(const f32x4 *)(lds + kE + 128 * srow(f) + 16 * (f & 7));
    }
  };
  auto stage_issue_tmp = [&](int half) __attribute__((always_inline)) {
    const int tt = opaque_t();
#pragma unroll
    for (int it = 0; it < kW4Stg; it++) {
      int f = it * 256 + tt;
      f = f < kRows * 8 ? f : kRows * 8 - 1;
      stg[it] = x6_ld4<Tower>(tmpg + half * kTmpRows * 32 + 32 * srow(f) + 4 * (f & 7));
    }
  };
  auto stage_put = [&](int it, int buf) {
    uint2 h, m, l;
    split4(stg[it], h, m, l);
    const int f = stage_f(it);
    char *d = lds + buf * kBufT + srow(f) * kX6Cell + 8 * (f & 7);
    *(uint2 *)d = h;
    *(uint2 *)(d + 64) = m;
    *(uint2 *)(d + 128) = l;
  };
  // B fragment of K-step L = q * 9 + tap, plane p, column block cb:
  // wp[(((tap * NQ + q) * 3 + p) * 128 + co0 + 16 cb) * 4 + kg]   (bf16x8 units);
  // S = the K-step over all NG chunks (Block: conv2's from S = 36, in wp2)
  const int co0 = 64 * chf + (lane & 15);
  const bf16x8 *wl = wp + co0 * 4 + kg;
  const bf16x8 *wl2 = (Block ? wp2 : wp) + co0 * 4 + kg;
  auto bissue = [&](bf16x8(&dst)[3][NCB], int S) {
    S = S < 9 * NG ? S : 9 * NG - 1;
    const bf16x8 *w = wl;
    if constexpr (Block) {
      w = S < 9 * NQ ? wl : wl2;
      S = S < 9 * NQ ? S : S - 9 * NQ;
    }
    const int q2 = S / 9, t2 = S - 9 * q2;
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
      for (int cb = 0; cb < NCB; cb++) dst[p][cb] = w[((t2 * NQ + q2) * 3 + p) * 512 + 64 * cb];
  };
  // the class table's rows first (vmcnt counts loads in issue order: the
  // setup's wait for them then covers them alone), then chunk 0's loads and
  // the first K-step's B fragments, under whose latency the setup runs
  int rtab[kRBT];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++) rtab[rb] = x6_tab<Block, Cf>()[rh * kRBT + rb][lane & 15];
  stage_issue(0);
  bf16x8 b[3][NCB], bn[3][NCB];
  bissue(b, 0);

  int cbase[kRBT];
  uint32_t valid[kRBT];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++) {
    const int r = rtab[rb] >= 0 ? rtab[rb] : 0;
    const int s = r / 35, cell = r - 35 * s, ch = cell / 7, cw = cell - 7 * ch;
    uint32_t v = 0;
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
      const int hh = ch + tap / 3 - 1, ww = cw + tap % 3 - 1;
      v |= (uint32_t)(hh >= 0 && hh < 5 && ww >= 0 && ww < 7) << tap;
    }
    // a padding row (-1 - k, not stored) reads anything in bounds at bank
    // slot 2k (its residue in the class table)
    cbase[rb] = (rtab[rb] >= 0 ? r * kX6Cell : kX6PadBase + 32 * (-1 - rtab[rb])) + 16 * kg;
    valid[rb] = rtab[rb] >= 0 ? v : 0x1ffu;
  }
  auto aoff = [&](int rb, int tap) -> int {
    const int d = ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell;
    const int a = cbase[rb] + d;
    return (valid[rb] >> tap) & 1 ? a : kZero + (a & 255);
  };

  f32x4 acc[kRBT][NCB];
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++)
#pragma unroll
    for (int cb = 0; cb < NCB; cb++) acc[rb][cb] = (f32x4){};
  HZ_STAMP(1)
#pragma unroll
  for (int it = 0; it < kW4Stg; it++) stage_put(it, 0);
  __syncthreads();
  HZ_STAMP(2)

  // One wave per SIMD: every instruction that is not an MFMA costs issue
  // cycles unless it sits in an MFMA's shadow (an MFMA holds the wave's issue
  // for 8 of its 16 cycles), so the loop is built as regions of MFMAs with
  // their "fillers" spread one per MFMA (sched_group_barrier; taps and planes
  // are compile-time, so every count is): the LDS reads of the next A plane
  // (plane pa + 1 of the tap, or plane 0 of the next tap: each read has a
  // plane's MFMAs to land in), the next K-step's B fragments (plane-0
  // region: a whole tap to land in) and the next chunk's staging (issued in
  // tap 0, split and stored in the plane-1 regions of taps 2-7).  Loads are
  // compiler-tracked, so its counted waits follow them.
  // Block, between the convs: conv1's outputs relu(acc + b1) (as the layered
  // conv1's epilogue computes them) to where conv2's chunks are staged from
  // (above); then the accumulators restart for conv2
  auto switch_convs = [&]() __attribute__((always_inline)) {
    float b1v[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; cb++) b1v[cb] = bias[64 * chf + 16 * cb + (lane & 15)];
    uint2 rows[kRBT];  // the lane's 4 rows of each row block, all loads in flight at once
#pragma unroll
    for (int rb = 0; rb < kRBT; rb++) rows[rb] = *(const uint2 *)&x6_tab<Block, Cf>()[rh * kRBT + rb][4 * kg];
    // chf is wave-uniform: one branch; a padding row (-1) writes to the
    // dummy cell / row 280, so no value takes a branch of its own
    auto put_all = [&](auto chfc) __attribute__((always_inline)) {
      constexpr int C = decltype(chfc)::value;
      static_for<0, kRBT>([&](auto rbc) {
        constexpr int rb = decltype(rbc)::value;
        static_for<0, 4>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const int r = (int)(int16_t)((j < 2 ? rows[rb].x : rows[rb].y) >> (16 * (j & 1)));
          const bool pad = r < 0;
          static_for<0, NCB>([&](auto cbc) {
            constexpr int cb = decltype(cbc)::value;
            float v = acc[rb][cb][j] + b1v[cb];
            v = v > 0.f ? v : 0.f;
            const int k = 16 * (cb & 1) + (lane & 15);
            if constexpr (cb >= 2) {
              tmpg[C * kTmpRows * 32 + (pad ? kRows : r) * 32 + k] = v;
            } else if constexpr (C == 0) {
              const uint32_t h = bf16_bits(v);
              const float r1 = v - bf16_value(h);
              const uint32_t m = bf16_bits(r1);
              const uint32_t l = bf16_bits(r1 - bf16_value(m));
              char *d = lds + (pad ? kDummyCell : r * kX6Cell) + 2 * k;
              *(unsigned short *)d = (unsigned short)h;
              *(unsigned short *)(d + 64) = (unsigned short)m;
              *(unsigned short *)(d + 128) = (unsigned short)l;
            } else {
              *(float *)(lds + kE + (pad ? kRows : r) * 128 + 4 * k) = v;
            }
          });
        });
        static_for<0, NCB>([&](auto cbc) { acc[rb][decltype(cbc)::value] = (f32x4){}; });
      });
    };
    if (chf == 0)
      put_all(std::integral_constant<int, 0>{});
    else
      put_all(std::integral_constant<int, 1>{});
    __syncthreads();
  };
  auto classed = [&](auto half) {
    constexpr int H = decltype(half)::value;
    auto aread = [&](bf16x8(&dst)[kRBT], const char *lb, auto tapc, int pa) {
      constexpr int tap = decltype(tapc)::value;
      static_for<0, kRBT>([&](auto rbc) {
        constexpr int rb = decltype(rbc)::value;
        if constexpr ((kX6ClassTaps[H][rb] >> tap) & 1) {
          constexpr int kNeg = 8 * kX6Cell;
          const int d = ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell + kNeg + 64 * pa;
          if constexpr ((kX6ClassSel[H][rb] >> tap) & 1)
            dst[rb] = *(const bf16x8 *)(lb + aoff(rb, tap) + 64 * pa);
          else
            dst[rb] = *(const bf16x8 *)(lb - kNeg + cbase[rb] + d);
        }
      });
    };
    for (int g = 0; g < NG; g++) {
      const int q = g & (NQ - 1);  // the chunk of the current conv
      if constexpr (Block)
        if (g == NQ) {
          switch_convs();
          HZ_STAMP(10)
        }
      const char *lb = lds + (q & 1) * kBufT;
      // workgroup-uniform: the next chunk staged by every thread (from HBM,
      // or Block: conv2's chunks 2 and 3 from E and tmp)
      const bool stage = g < NQ - 1 || (Block && g >= NQ && g < NG - 1);
      const bool sync = g < NQ - 1 || (Block && g >= NQ && g < NG - 1);
      const int nb = (q + 1) & 1;
      bf16x8 a[2][kRBT];  // [plane parity]: the plane in use, the one being read
      aread(a[0], lb, std::integral_constant<int, 0>{}, 0);
      static_for<0, 9>([&](auto tapc) {
        constexpr int tap = decltype(tapc)::value;
        const int L = g * 9 + tap;
        static_for<0, 3>([&](auto pac) {
          constexpr int pa = decltype(pac)::value;
          constexpr int cur = (3 * tap + pa) & 1, nxt = cur ^ 1;
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (HZ_KO & 32) {
          } else if constexpr (pa < 2)
            aread(a[nxt], lb, tapc, pa + 1);
          else if constexpr (tap < 8)
            aread(a[nxt], lb, std::integral_constant<int, tap + 1>{}, 0);
          if constexpr (pa == 0) {
            if constexpr (!(HZ_KO & 16)) bissue(bn, L + 1);  // Block: conv2's first after conv1's last
            if (tap == 0 && stage && !(HZ_KO & 1)) {
              if (Block && g == NQ + 1)
                stage_issue_e();
              else if (Block && g >= NQ)
                stage_issue_tmp(g == NQ + 2);
              else
                stage_issue(q + 1);
            }
          }
          if constexpr (HZ_KO & 2) {
            if (tap == 7 && pa == 1 && stage)
#pragma unroll
              for (int it = 0; it < kW4Stg; it++) asm volatile("" ::"v"(stg[it]));
          } else if constexpr (pa == 1 && !(HZ_KO & 1)) {
            if (stage) {
              if constexpr (tap >= 2 && tap <= 4) {
                stage_put(2 * (tap - 2), nb);
                stage_put(2 * (tap - 2) + 1, nb);
              } else if constexpr (tap >= 5 && tap <= 7) {
                stage_put(tap + 1, nb);
              }
            }
          }
#pragma unroll
          for (int pb = 0; pb < 3 - pa; pb++)
            static_for<0, kRBT>([&](auto rbc) {
              constexpr int rb = decltype(rbc)::value;
              if constexpr ((kX6ClassTaps[H][rb] >> tap) & 1) {
#pragma unroll
                for (int cb = 0; cb < NCB; cb++)
                  acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(HZ_KO & 32) ? 0 : cur][rb], b[pb][cb],
                                                                        acc[rb][cb], 0, 0, 0);
              }
            });
          // one filler (VALU, LDS read or write, global load) after each MFMA
          constexpr int nm = (3 - pa) * x6_class_blocks(H, tap) * NCB;
          static_for<0, nm>([&](auto) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x322, 1, 0);
          });
        });
        if constexpr (!(HZ_KO & 16)) {
#pragma unroll
          for (int p = 0; p < 3; p++)
#pragma unroll
            for (int cb = 0; cb < NCB; cb++) b[p][cb] = bn[p][cb];
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      if (sync) __syncthreads();
      if (g < NQ) {
        HZ_STAMP(3 + g)
      } else {
        HZ_STAMP(7 + g)  // Block: conv2's chunks in slots 11-14
      }
    }
  };
  if (rh == 0)
    classed(std::integral_constant<int, 0>{});
  else
    classed(std::integral_constant<int, 1>{});

  // Epilogue as k_conv3x3_x6: relu((acc + bias) + res) through a per-wave LDS
  // transpose of each 16x16 tile (buffer 0: last read in chunk 2, before the
  // barrier that closed it), float4 residual loads and stores.
  constexpr int kTS = 20, kT = 6;
  static_assert(4 * kT * 16 * kTS * 4 <= kZero, "per-wave tiles fit in buffer 0");
  float *tile = (float *)lds + w * 16 * kTS * kT;
  const int trow = lane >> 2, tcol = 4 * (lane & 3);
  const int cow = 64 * chf + tcol;
  const int nrow = ns * 35;
  const size_t gbase = (size_t)s0 * 35 * 128;
  int erow[kRBT];  // the lane's output row of each block (transposed tiles: lane -> row lane >> 2)
#pragma unroll
  for (int rb = 0; rb < kRBT; rb++) erow[rb] = x6_tab<Block, Cf>()[rh * kRBT + rb][lane >> 2];
  auto orow = [&](int rb) -> int {
    const int row = erow[rb];
    return row >= 0 && row < nrow ? row : -1;
  };
  // every residual load in flight at once (36 float4 per lane); Block: the
  // skip input is the block input x, the bias conv2's
  const float *eres = Block ? x : res, *ebias = Block ? bias2 : bias;
  float4 rv[kRBT * NCB];
#pragma unroll
  for (int k = 0; k < kRBT * NCB; k++) {
    const int rb = k / NCB, cb = k % NCB;
    const int row = orow(rb);
    rv[k] = eres && row >= 0 && !(HZ_KO & 64) ? x6_ld4f<Tower>(eres + gbase + (size_t)row * 128 + cow + 16 * cb)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // (Tower: x and out are the same buffer from the second block on; every
  // skip load is issued before any store, and the compiler keeps it so)
  if constexpr (Tower) asm volatile("" ::: "memory");
  float4 bv[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; cb++) bv[cb] = *(const float4 *)(ebias + cow + 16 * cb);
#pragma unroll
  for (int r0 = 0; r0 < kRBT * NCB; r0 += kT) {
#pragma unroll
    for (int k = 0; k < kT; k++) {
      const int rb = (r0 + k) / NCB, cb = (r0 + k) % NCB;
#pragma unroll
      for (int j = 0; j < 4; j++) tile[k * 16 * kTS + (4 * kg + j) * kTS + (lane & 15)] = acc[rb][cb][j];
    }
    __builtin_amdgcn_wave_barrier();
    float4 a4[kT];
#pragma unroll
    for (int k = 0; k < kT; k++) a4[k] = *(const float4 *)(tile + k * 16 * kTS + trow * kTS + tcol);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < kT; k++) {
      const int rb = (r0 + k) / NCB, cb = (r0 + k) % NCB;
      const int row = orow(rb);
      if (row >= 0) {
        float4 v;
        v.x = a4[k].x + bv[cb].x;
        v.y = a4[k].y + bv[cb].y;
        v.z = a4[k].z + bv[cb].z;
        v.w = a4[k].w + bv[cb].w;
        if (eres) {
          v.x = v.x + rv[r0 + k].x;
          v.y = v.y + rv[r0 + k].y;
          v.z = v.z + rv[r0 + k].z;
          v.w = v.w + rv[r0 + k].w;
        }
        v.x = v.x > 0.f ? v.x : 0.f;
        v.y = v.y > 0.f ? v.y : 0.f;
        v.z = v.z > 0.f ? v.z : 0.f;
        v.w = v.w > 0.f ? v.w : 0.f;
        if constexpr (HZ_KO & 4) {
          int never = 0;
          asm volatile("" : "+v"(never));
          if (never) *(float4 *)(out + gbase + (size_t)row * 128 + cow + 16 * cb) = v;
        } else
          *(float4 *)(out + gbase + (size_t)row * 128 + cow + 16 * cb) = v;
      }
    }
  }
  HZ_STAMP(7)
  HZ_STAMP_RT(9)
}
template <bool Block, bool Cf = false>
__global__ void __launch_bounds__(256, 1)
    k_conv3x3_x6w4(const float *__restrict__ x, const bf16x8 *__restrict__ wp, const float *__restrict__ bias,
                   const float *__restrict__ res, float *__restrict__ out, int32_t batch,
                   const int32_t *__restrict__ live, const bf16x8 *__restrict__ wp2,
                   const float *__restrict__ bias2, float *__restrict__ tmp) {
  x6w4_body<Block, Cf, false>(x, wp, bias, res, out, batch, live, wp2, bias2, tmp);
}
// A tower of residual blocks in one launch (hz_tower_x6_blocks): each
// workgroup carries its 8 states through every block (a block's rows depend
// only on the same rows of the block before), writing each block's output
// over the previous one in `out` (block 0 reads x); between blocks only the
// workgroup's own barrier, after its stores have completed.  No launch
// boundary per block: the workgroups drift apart, so their epilogue bursts
// stop coinciding.  Same arithmetic per block as k_conv3x3_x6w4<true>.
constexpr int kTowerMax = 16;
struct X6Tower {
  const bf16x8 *w1[kTowerMax], *w2[kTowerMax];
  const float *b1[kTowerMax], *b2[kTowerMax];
  int32_t nblk;
  int32_t stagger;  // A/B knob (hz_tower_x6_set_stagger): first-round start delay, units of 8,128 cycles
  int32_t round;    // workgroups of the first round (the CU count)
};
template <bool Cf>
__global__ void __launch_bounds__(256, 1)
    k_x6w4_tower(const float *__restrict__ x, float *out, int32_t batch, const int32_t *__restrict__ live,
                 float *__restrict__ tmp, X6Tower tw) {
  // every first-round workgroup starts together, so their epilogues (a
  // residual load and store burst of every CU at once) coincide; a start
  // delay on every other CU of each XCD shifts half of them by part of a
  // block (the second round inherits the shift)
  if (tw.stagger > 0 && (int)blockIdx.x < tw.round && ((blockIdx.x >> 3) & 1))
    for (int i = 0; i < tw.stagger; i++) __builtin_amdgcn_s_sleep(127);
#pragma unroll 1
  for (int k = 0; k < tw.nblk; k++) {
    x6w4_body<true, Cf, true>(k == 0 ? x : out, tw.w1[k], tw.b1[k], nullptr, out, batch, live, tw.w2[k], tw.b2[k],
                              tmp);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's stores done before the barrier
    __syncthreads();
  }
}
}  // namespace
#undef HZ_STAMP
#undef HZ_STAMP_RT

template <int NQ, bool Stem, int CS, int NCB>
static int launch_x6_cs(const float *x, const void *wpack6, const float *bias, const float *res, float *out,
                        int32_t batch, const int32_t *live, void *stream) {
  static std::atomic<uint64_t> init_mask{0};
  const size_t lds = 2 * (size_t)((CS * 35 * kX6Cell + 255) / 256 * 256 + kX6Zero);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_conv3x3_x6<NQ, Stem, CS, NCB>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL((k_conv3x3_x6<NQ, Stem, CS, NCB>), dim3((batch + CS - 1) / CS),
                     dim3((CS == 8 ? 2 : 1) * (8 / NCB) * 64), lds, (hipStream_t)stream, x, (const bf16x8 *)wpack6,
                     bias, res, out, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// batches of at most this many rows (the buffer's, known on the host) run
// one state per workgroup; HZ_X6_SMALL_MAX overrides it (tools/conv_bench.py)
static int32_t x6_small_max() {
  static const int32_t v = [] {
    const char *e = getenv("HZ_X6_SMALL_MAX");
    return e ? (int32_t)atoi(e) : (int32_t)kX6SmallMax;
  }();
  return v;
}

// ... and up to this many, one state per workgroup with 8 waves of 16
// output channels (half of each wave's MFMA chain; HZ_X6_TINY_MAX overrides)
static int32_t x6_tiny_max() {
  static const int32_t v = [] {
    const char *e = getenv("HZ_X6_TINY_MAX");
    return e ? (int32_t)atoi(e) : (int32_t)kX6TinyMax;
  }();
  return v;
}

// the tower's 8-state conv: the 4-wave form (k_conv3x3_x6w4, bit-identical;
// complete self-play games 131.6 vs 127.4-127.7 games/s on one box,
// profiles/r03/ab_w4_fullgame.json) unless HZ_X6_W4=0 (A/B measurements)
static bool x6_w4() {
  static const bool v = [] {
    const char *e = getenv("HZ_X6_W4");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

template <bool Block, bool Cf = false>
static int launch_x6w4(const float *x, const void *wpack6, const float *bias, const float *res, float *out,
                       int32_t batch, const int32_t *live, void *stream, const void *wpack6_2 = nullptr,
                       const float *bias2 = nullptr, float *tmp = nullptr) {
  static std::atomic<uint64_t> init_mask{0};
  const size_t lds = 2 * (size_t)(kCS * 35 * kX6Cell + kX6Zero) + (Block ? (size_t)(kRows + 1) * 128 + kX6Cell : 0);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_conv3x3_x6w4<Block, Cf>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL((k_conv3x3_x6w4<Block, Cf>), dim3((batch + kCS - 1) / kCS), dim3(256), lds, (hipStream_t)stream, x,
                     (const bf16x8 *)wpack6, bias, res, out, batch, live, (const bf16x8 *)wpack6_2, bias2, tmp);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <bool Cf>
static int launch_x6w4_tower(const float *x, float *out, float *tmp, const X6Tower &tw, int32_t batch,
                             const int32_t *live, void *stream) {
  static std::atomic<uint64_t> init_mask{0};
  const size_t lds = 2 * (size_t)(kCS * 35 * kX6Cell + kX6Zero) + (size_t)(kRows + 1) * 128 + kX6Cell;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_x6w4_tower<Cf>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL((k_x6w4_tower<Cf>), dim3((batch + kCS - 1) / kCS), dim3(256), lds, (hipStream_t)stream, x, out,
                     batch, live, tmp, tw);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// residual blocks run as one launch (k_conv3x3_x6w4<true>) where the tower
// conv takes the 4-wave form, unless HZ_X6_BLOCK=0: one block alone measures
// at parity with the two layered launches (282.2 vs 284.1 us, tools/block_ab.py,
// whose layered convs re-read a cached input), but in the forward chain the
// intermediate activation's write and re-read are gone: 2.29 vs 2.41 ms per
// 4096-row forward, 138.4-138.8 vs 132.9-133.6 complete self-play games/s
// on one box (profiles/r03/block)
static std::atomic<int32_t> g_x6_block{-1};  // -1: from HZ_X6_BLOCK on first use
static bool x6_block() {
  int32_t v = g_x6_block.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = getenv("HZ_X6_BLOCK");
    int32_t want = e && atoi(e) == 0 ? 0 : 1, expect = -1;
    g_x6_block.compare_exchange_strong(expect, want);
    v = g_x6_block.load(std::memory_order_relaxed);
  }
  return v == 1;
}

// the fused block's row table: 1 (the default since round 5) the
// bank-conflict-free kX6ClassRow, 0 round 3's kX6ClassRowBlk
// (HZ_BLK_TABLE=0, hz_resblock_x6_set_table).  Whole forwards at 4,096 rows,
// interleaved in one process (tools/blk_table_ab.py, 12 rounds x 20
// forwards each): 2.2378 vs 2.2368 ms and 2.3143 vs 2.3073 ms on two boxes
// (profiles/r05/blk_table), bit-identical
static std::atomic<int32_t> g_x6_blk_cf{-1};
static bool x6_blk_cf() {
  int32_t v = g_x6_blk_cf.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = getenv("HZ_BLK_TABLE");
    int32_t want = e && atoi(e) == 0 ? 0 : 1, expect = -1;
    g_x6_blk_cf.compare_exchange_strong(expect, want);
    v = g_x6_blk_cf.load(std::memory_order_relaxed);
  }
  return v == 1;
}

// HZ_X6_CS4=1: the tower conv above the one-state forms' limit as the
// 4-state form (k_conv3x3_x6<4, false, 4, 2>: two 4-wave workgroups per CU,
// each one's epilogue and staging free to overlap the other's MFMAs;
// A/B measurements)
// the stem above the one-state forms in 4-state workgroups (64 KB of LDS:
// two per CU, one's loads and stores under the other's MFMAs) instead of 8:
// 47.8 vs 49.6 us at 4,096 encoder rows, bit-identical (tools/stem_ab.py,
// alternating processes, profiles/r06/stem_cs4); HZ_STEM_CS4=0: 8 states
static bool stem_cs4() {
  static const bool v = [] {
    const char *e = getenv("HZ_STEM_CS4");
    return !(e && atoi(e) == 0);
  }();
  return v;
}
static bool x6_cs4() {
  static const bool v = [] {
    const char *e = getenv("HZ_X6_CS4");
    return e && atoi(e) == 1;
  }();
  return v;
}

template <int NQ, bool Stem>
static int launch_x6(const float *x, const void *wpack6, const float *bias, const float *res, float *out,
                     int32_t batch, const int32_t *live, void *stream) {
  if (batch <= x6_tiny_max()) return launch_x6_cs<NQ, Stem, 1, 1>(x, wpack6, bias, res, out, batch, live, stream);
  if constexpr (Stem)
    if (batch > x6_small_max() && stem_cs4()) return launch_x6_cs<NQ, Stem, 4, 2>(x, wpack6, bias, res, out, batch, live, stream);
  if constexpr (NQ == 4 && !Stem)
    if (batch > x6_small_max() && x6_cs4()) return launch_x6_cs<NQ, Stem, 4, 2>(x, wpack6, bias, res, out, batch, live, stream);
  if constexpr (NQ == 4 && !Stem)
    if (batch > x6_small_max() && x6_w4()) return launch_x6w4<false>(x, wpack6, bias, res, out, batch, live, stream);
  return batch <= x6_small_max() ? launch_x6_cs<NQ, Stem, 1, 2>(x, wpack6, bias, res, out, batch, live, stream)
                                 : launch_x6_cs<NQ, Stem, 8, 2>(x, wpack6, bias, res, out, batch, live, stream);
}

extern "C" int hz_conv3x3_x6_bias_act(const float *x, const void *wpack6, const float *bias, const float *res,
                                      float *out, int32_t batch, const int32_t *live, void *stream) {
  if (!x || !wpack6 || !bias || !out || batch < 0) return -1;
  if (((uintptr_t)x | (uintptr_t)wpack6 | (uintptr_t)out | (uintptr_t)res) & 15) return -1;
  if (batch == 0) return 0;
  return launch_x6<4, false>(x, wpack6, bias, res, out, batch, live, stream);
}

// One residual block of the tower (model.py:287-299): out = relu(conv2(
// relu(conv1(x) + b1)) + b2 + x).  Where the tower conv takes the 4-wave form
// (batch above the one-state forms' limit) it is one launch whose
// intermediate activation stays on the CU; otherwise the two layered convs
// through tmp (the same bits either way).
extern "C" int hz_resblock_x6_bias_act(const float *x, const void *w1, const float *b1, const void *w2,
                                       const float *b2, float *out, float *tmp, int32_t batch, const int32_t *live,
                                       void *stream) {
  if (!x || !w1 || !b1 || !w2 || !b2 || !out || !tmp || batch < 0) return -1;
  if (((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)w2 | (uintptr_t)out | (uintptr_t)tmp) & 15) return -1;
  if (batch == 0) return 0;
  if (hz_resblock_x6_fused(batch))
    return x6_blk_cf() ? launch_x6w4<true, true>(x, w1, b1, nullptr, out, batch, live, stream, w2, b2, tmp)
                       : launch_x6w4<true>(x, w1, b1, nullptr, out, batch, live, stream, w2, b2, tmp);
  const int rc = launch_x6<4, false>(x, w1, b1, nullptr, tmp, batch, live, stream);
  return rc ? rc : launch_x6<4, false>(tmp, w2, b2, x, out, batch, live, stream);
}

// nblk residual blocks in one launch (k_x6w4_tower: each workgroup carries
// its 8 states through all of them), where hz_resblock_x6_fused(batch)
// holds; w1/b1/w2/b2 are HOST arrays of nblk device pointers (each block's
// packed conv weights and folded biases).  out gets the last block's
// output (and holds the intermediate ones); x is only read.  The same bits
// as nblk hz_resblock_x6_bias_act calls.  -2: this batch takes the
// per-block path (hz_resblock_x6_fused(batch) == 0).
extern "C" int32_t hz_resblock_x6_fused(int32_t batch);
// the default stagger (4 units, ~33 k cycles): 0.3-0.6 % per 4096-row forward
// against none, bit-identical (tools/tower_stagger_ab.py, profiles/r06/s6d,
// s6e); HZ_TOWER_STAGGER overrides it
static std::atomic<int32_t> g_tower_stagger{[] {
  const char *e = getenv("HZ_TOWER_STAGGER");
  return e ? (int32_t)atoi(e) : (int32_t)4;
}()};
static int32_t tower_round() {  // the device's CU count: workgroups of the tower's first round
  static std::atomic<int32_t> cus{0};
  int32_t v = cus.load(std::memory_order_relaxed);
  if (!v) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      v = n;
    else
      v = 256;
    cus.store(v, std::memory_order_relaxed);
  }
  return v;
}
// A/B knob (no reference counterpart): the tower launch's stagger (above)
extern "C" int hz_tower_x6_set_stagger(int32_t units) {
  if (units < 0 || units > 1000) return -1;
  g_tower_stagger.store(units, std::memory_order_relaxed);
  return 0;
}
extern "C" int hz_tower_x6_blocks(const float *x, const void *const *w1, const float *const *b1,
                                  const void *const *w2, const float *const *b2, int32_t nblk, float *out,
                                  float *tmp, int32_t batch, const int32_t *live, void *stream) {
  if (!x || !w1 || !b1 || !w2 || !b2 || !out || !tmp || batch < 0 || nblk < 1 || nblk > kTowerMax) return -1;
  if (((uintptr_t)x | (uintptr_t)out | (uintptr_t)tmp) & 15) return -1;
  if (batch == 0) return 0;
  if (!hz_resblock_x6_fused(batch)) return -2;
  X6Tower tw{};
  for (int k = 0; k < nblk; k++) {
    if (!w1[k] || !b1[k] || !w2[k] || !b2[k] || (((uintptr_t)w1[k] | (uintptr_t)w2[k]) & 15)) return -1;
    tw.w1[k] = (const bf16x8 *)w1[k];
    tw.w2[k] = (const bf16x8 *)w2[k];
    tw.b1[k] = b1[k];
    tw.b2[k] = b2[k];
  }
  tw.nblk = nblk;
  tw.stagger = g_tower_stagger.load(std::memory_order_relaxed);
  tw.round = tower_round();
  return x6_blk_cf() ? launch_x6w4_tower<true>(x, out, tmp, tw, batch, live, stream)
                     : launch_x6w4_tower<false>(x, out, tmp, tw, batch, live, stream);
}

// 1: residual blocks at the 4-wave conv's batch sizes run as one launch, 0:
// as the two layered convs (the same bits either way; A/B and tests)
extern "C" int hz_resblock_x6_set_fused(int32_t on) {
  if (on != 0 && on != 1) return -1;
  g_x6_block.store(on, std::memory_order_relaxed);
  return 0;
}

// the fused block's row table (A/B and tests; the same bits either way)
extern "C" int hz_resblock_x6_set_table(int32_t cf) {
  if (cf != 0 && cf != 1) return -1;
  g_x6_blk_cf.store(cf, std::memory_order_relaxed);
  return 0;
}

// 1 when hz_resblock_x6_bias_act runs batch rows as one launch.  The fused
// kernel's scratch is a [2][288][32]-float slice per 8-state group in tmp,
// which the ABI sizes batch x 35 x 128 floats: the fused form is taken only
// when the slices fit (any batch > 4; the default routing needs > 768)
extern "C" int32_t hz_resblock_x6_fused(int32_t batch) {
  const bool fits = (int64_t)((batch + kCS - 1) / kCS) * 2 * 288 * 32 <= (int64_t)batch * 35 * 128;
  return fits && batch > x6_tiny_max() && batch > x6_small_max() && x6_w4() && x6_block() ? 1 : 0;
}

extern "C" int hz_stem3x3_x6_bias_act(const float *board, const void *wpack6, const float *bias, float *out,
                                      int32_t batch, const int32_t *live, void *stream) {
  if (!board || !wpack6 || !bias || !out || batch < 0) return -1;
  if (((uintptr_t)wpack6 | (uintptr_t)out) & 15) return -1;
  if (batch == 0) return 0;
  return launch_x6<2, true>(board, wpack6, bias, nullptr, out, batch, live, stream);
}

// Resident tower for small batches (config 1's one-board predict, the
// arena's batches of a few dozen boards): one workgroup carries one state
// through every conv of the tower (model.py:376-393, BN folded), its
// activation never leaving LDS, the convs following each other after one
// barrier.  A one-state conv's time is its workgroup streaming the conv's
// 885 KB of weights into one CU (~20 us per conv layered: the B fragments
// were loaded one K-step ahead, latency-bound); here the weight stream runs
// kTRAhead K-steps ahead, across conv boundaries too.
// Same arithmetic as k_conv3x3_x6<4, false, 1, 1> (8 waves of 16 output
// channels, the state's 35 rows as 3 row blocks, the same K order and
// epilogue), so the result is bit-identical to the layered tower.
// LDS: two activation buffers (the conv's input, its output = the next
// conv's input), each the state's four 32-channel chunks as bf16 planes in
// k_conv3x3_x6's cell layout, every chunk followed by its own zero region
// (chunk stride a multiple of 256 B: an off-board tap's offset within the
// chunk does not depend on the chunk); the block input in fp32 for the skip
// (35 x 128 floats).  85,504 B.
namespace {
constexpr int kTRZero = 31 * 256;                          // zero region of a chunk (after 35 cells)
constexpr int kTRChunk = kTRZero + 256 + 256;              // chunk stride
constexpr int kTRBuf = 4 * kTRChunk;                       // one activation buffer
constexpr int kTRLds = 2 * kTRBuf + 35 * 128 * 4;          // + the fp32 skip (+ the biases)
constexpr int kTRMaxConv = 64;
constexpr int kTRConvW = 9 * 4 * 3 * 128 * 4;              // one conv's packed weights (bf16x8 units)
constexpr int kTRAhead = 4;                                // K-steps of B fragments in flight
static_assert(35 * kX6Cell <= kTRZero && kTRZero + 255 + 128 + 16 <= kTRChunk, "cells and zero region fit");
static_assert(36 % kTRAhead == 0, "the B ring's slots repeat every conv");

__global__ void __launch_bounds__(512, 1)
    k_tower_x6_resident(const float *__restrict__ x0, const bf16x8 *__restrict__ wp,
                        const float *__restrict__ bias, float *__restrict__ out, int32_t nconv, int32_t batch,
                        const int32_t *__restrict__ live) {
  extern __shared__ float4 lds4[];
  char *lds = (char *)lds4;
  float *skip = (float *)(lds + 2 * kTRBuf);
  float *biasl = skip + 35 * 128;  // every conv's bias (no plain global load in the conv loop: see bissue)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kg = lane >> 4;
  const int s = blockIdx.x;
  if (live) batch = *live < batch ? *live : batch;
  if (s >= batch) return;
  for (int i = t; i < nconv * 128; i += 512) biasl[i] = bias[i];

  if (t < 2 * 4 * 32) {  // every chunk's zero region (512 B = 32 float4)
    const int c = t >> 5, k = t & 31;
    *(float4 *)(lds + c * kTRChunk + kTRZero + 16 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // the stem's output x0 (NHWC [35][128]) into buffer 0 and the skip:
  // float4 f = cell f >> 5, channels 4 (f & 31) ..
  const float *xs = x0 + (size_t)s * 35 * 128;
  for (int f = t; f < 35 * 32; f += 512) {
    const f32x4 v = *(const f32x4 *)(xs + 4 * f);
    const int cell = f >> 5, part = f & 31;
    uint2 h, m, l;
    split4(v, h, m, l);
    char *d = lds + (part >> 3) * kTRChunk + cell * kX6Cell + 8 * (part & 7);
    *(uint2 *)d = h;
    *(uint2 *)(d + 64) = m;
    *(uint2 *)(d + 128) = l;
    *(f32x4 *)(skip + 4 * f) = v;
  }

  // A fragment of row block rb, tap, chunk q: chunk base + aoff[rb][tap]
  // (+ 64 pa), the lane's row 16 rb + (lane & 15) (clamped) as in
  // k_conv3x3_x6; off the board the chunk's zero region at the same offset
  // mod 256 (the chunk stride is a multiple of 256: the LDS banks the row
  // would use)
  int aoff[3][9];
#pragma unroll
  for (int rb = 0; rb < 3; rb++) {
    int r = 16 * rb + (lane & 15);
    r = r < 35 ? r : 34;
    const int ch = r / 7, cw = r - 7 * ch;
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
      const int hh = ch + tap / 3 - 1, ww = cw + tap % 3 - 1;
      const int a = r * kX6Cell + 16 * kg + ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell;
      aoff[rb][tap] = hh >= 0 && hh < 5 && ww >= 0 && ww < 7 ? a : kTRZero + (a & 255);
    }
  }
  const int co = 16 * w + (lane & 15);
  const bf16x8 *wl = wp + co * 4 + kg;
  // B fragments of conv l (clamped: the stream runs past the last conv),
  // K-step L = q * 9 + tap, planes 0-2 (pack_conv3x3_x6 layout), requested
  // by asm loads: the compiler would sink plain loads to their use and wait
  // for all of them (one step in flight); program order and the explicit
  // waits below keep kTRAhead - 1 steps in flight
  auto bissue = [&](bf16x8(&dst)[3], int l, int L) {
    l = l < nconv ? l : nconv - 1;
    const int q2 = L / 9, t2 = L - 9 * q2;
    const bf16x8 *src = wl + (size_t)l * kTRConvW + (t2 * 4 + q2) * 3 * 512;
#pragma unroll
    for (int p = 0; p < 3; p++) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[p]) : "v"(src + p * 512));
  };
  // the B ring: K-step L of any conv in slot L % kTRAhead
  bf16x8 bq[kTRAhead][3];
#pragma unroll
  for (int L = 0; L < kTRAhead - 1; L++) bissue(bq[L], 0, L);
  __syncthreads();

  for (int l = 0; l < nconv; l++) {
    const char *lb = lds + (l & 1) * kTRBuf;
    char *ob = lds + ((l + 1) & 1) * kTRBuf;
    const float bv = biasl[l * 128 + co];
    f32x4 acc[3] = {};
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int tap = 0; tap < 9; tap++) {
        const int L = q * 9 + tap, Lf = L + kTRAhead - 1;  // Lf: the step whose B this step requests
        if (Lf < 36)
          bissue(bq[Lf % kTRAhead], l, Lf);
        else
          bissue(bq[Lf % kTRAhead], l + 1, Lf - 36);
        // this step's fragments have landed: only the 3 (kTRAhead - 1)
        // requested after them may be outstanding (vmcnt counts in order)
        bf16x8 *b = bq[L % kTRAhead];
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]) : "n"(3 * (kTRAhead - 1)));
#pragma unroll
        for (int pa = 0; pa < 3; pa++) {
          bf16x8 a[3];
#pragma unroll
          for (int rb = 0; rb < 3; rb++)
            a[rb] = *(const bf16x8 *)(lb + q * kTRChunk + aoff[rb][tap] + 64 * pa);
#pragma unroll
          for (int pb = 0; pb < 3 - pa; pb++)
#pragma unroll
            for (int rb = 0; rb < 3; rb++)
              acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[pb], acc[rb], 0, 0, 0);
        }
      }
    }
    // epilogue: relu((acc + bias) [+ skip]); conv 2 of a block adds the
    // block input and its output becomes the next block input
    const bool second = l & 1, last = l == nconv - 1;
    char *od = ob + (co >> 5) * kTRChunk + 2 * (co & 31);
#pragma unroll
    for (int rb = 0; rb < 3; rb++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int r = 16 * rb + 4 * kg + j;
        if (r >= 35) continue;
        float v = acc[rb][j] + bv;
        if (second) v = v + skip[r * 128 + co];
        v = v > 0.f ? v : 0.f;
        if (last) {
          out[((size_t)s * 35 + r) * 128 + co] = v;
          continue;
        }
        if (second) skip[r * 128 + co] = v;
        const uint32_t hb = bf16_bits(v);
        const float r1 = v - bf16_value(hb);
        const uint32_t mb = bf16_bits(r1);
        const uint32_t lo = bf16_bits(r1 - bf16_value(mb));
        char *d = od + r * kX6Cell;
        *(uint16_t *)d = (uint16_t)hb;
        *(uint16_t *)(d + 64) = (uint16_t)mb;
        *(uint16_t *)(d + 128) = (uint16_t)lo;
      }
    __syncthreads();  // the output buffer is the next conv's input
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's requests past the last conv
}
}  // namespace

extern "C" int hz_tower_x6_resident(const float *x0, const void *wpack6, const float *bias, float *out,
                                    int32_t nconv, int32_t batch, const int32_t *live, void *stream) {
  if (!x0 || !wpack6 || !bias || !out || batch < 0 || nconv < 2 || nconv > kTRMaxConv || (nconv & 1)) return -1;
  if (((uintptr_t)x0 | (uintptr_t)wpack6 | (uintptr_t)out) & 15) return -1;
  if (batch == 0) return 0;
  static std::atomic<uint64_t> init_mask{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_tower_x6_resident, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kTRLds + kTRMaxConv * 128 * 4) != hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL(k_tower_x6_resident, dim3(batch), dim3(512), kTRLds + nconv * 128 * 4, (hipStream_t)stream, x0,
                     (const bf16x8 *)wpack6, bias, out, nconv, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Split tower for the smallest batches (config 1's one-board predict): the
// resident tower's workgroup is bound by one CU taking in the whole tower's
// weights (14 MB at ~62 GB/s).  Here kTSG workgroups share a state, each
// owning 16 output channels (3 waves: the state's 3 row blocks), so each
// reads an eighth of the weights; workgroup g of every state runs on the
// same XCD (blocks are dealt round-robin), whose L2 then holds only that
// eighth.  After each conv the groups exchange the activation through HBM
// (xch, double-buffered by conv parity) with the write-through hand-off of
// the HIP guide's Guideline 16, table row 1: every payload store sc1 (16 B), each
// storing wave drains (vmcnt 0), a barrier, ONE lane's agent-scope atomic
// add to the state's counter; ONE lane polls it relaxed (bounded spin),
// a barrier, and every load of the payload is an sc1 load.  The counter
// block (sync: one 128-B line per state holding its hand-off counter and
// its done counter; the timeout word at line kTSMaxBatch) is zeroed once by
// the caller, and the last group of a state to finish zeroes the state's
// counters again (no memset ahead of each launch).  All groups of a launch must be
// resident together: the host caps the batch (kTSMaxBatch x kTSG groups,
// at most one per CU).
// Per (row block, 16 channels) tile the products, sums and epilogue are
// issued in the layered convs' order: bit-identical to them.
namespace {
constexpr int kTSG = 8;                       // workgroups per state
constexpr int kTSMaxBatch = 32;               // kTSMaxBatch * kTSG <= 256 CUs
constexpr int kTSFlag = kTRBuf + kTRMaxConv * 16 * 4 + 3 * 16 * 20 * 4;  // input, biases, tiles, then
constexpr int kTSLds = kTSFlag + 16;                                       // the timeout flag
constexpr int kTSAAhead = 2;                 // K-steps of A fragments read ahead from LDS
constexpr int kTSRb1Max = 10;                // batches up to this: one row block per workgroup
constexpr int kTSAhead = 4;                  // K-steps of B fragments in flight (4-18 measured alike)
constexpr uint64_t kTSSpinTicks = 100000000;  // 1 s at the 100 MHz s_memrealtime clock: give up
typedef __attribute__((address_space(1))) unsigned gu32;
#ifdef HZ_NET_DIAG  // per conv phase stamps of state 0's groups (tools/split_phases.py)
__device__ uint64_t g_split_stamps[8][64][6];
#define HZ_SSTAMP(k) \
  if (t == 0 && s == 0 && l < 64) g_split_stamps[g][l][k] = __builtin_amdgcn_s_memtime();
#else
#define HZ_SSTAMP(k)
#endif

template <int Ahead, int RBG>
__global__ void __launch_bounds__(192, 1)
    k_tower_x6_split(const float *__restrict__ x0, const bf16x8 *__restrict__ wp, const float *__restrict__ bias,
                     float *__restrict__ out, float *xch, unsigned *sync, int32_t nconv, int32_t batch,
                     const int32_t *__restrict__ live) {
  static_assert(36 % Ahead == 0 && 3 * (Ahead - 1) <= 63, "the B ring's slots repeat every conv; vmcnt range");
  // RBG = row blocks per workgroup: 3 (wave w computes row block w; kTSG groups
  // per state) or 1 (the group owns one row block, computed by wave 0; 3 *
  // kTSG groups per state, so a CU streams its B fragments once instead of
  // three times; the other waves only share the staging)
  static_assert(RBG == 3 || RBG == 1, "3 or 1 row blocks per workgroup");
  constexpr int G = kTSG * 3 / RBG;  // workgroups per state
  extern __shared__ float4 lds4[];
  char *lds = (char *)lds4;
  float *biasl = (float *)(lds + kTRBuf);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kg = lane >> 4;
  // group g of every state on XCD g (blocks are dealt round-robin)
  const int s = blockIdx.x / G, g = blockIdx.x % kTSG;
  const int rb = RBG == 3 ? w : (blockIdx.x / kTSG) % 3;
  const bool compute = RBG == 3 || w == 0;  // wave-uniform
  float *tile = (float *)(lds + kTRBuf + kTRMaxConv * 16 * 4) + (RBG == 3 ? w : 0) * 16 * 20;  // transpose tile
  int nb = batch;
  if (live) nb = *live < batch ? *live : batch;
  if (s >= nb) return;  // every group of a state leaves together

  for (int i = t; i < nconv * 16; i += 192) biasl[i] = bias[(i >> 4) * 128 + 16 * g + (i & 15)];
  if (t < 4 * 32) {  // every chunk's zero region
    const int c = t >> 5, k = t & 31;
    *(float4 *)(lds + c * kTRChunk + kTRZero + 16 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto put = [&](int f, const f32x4 v) {  // float4 f of a [35][128] activation into the LDS planes
    const int cell = f >> 5, part = f & 31;
    uint2 h, m, l;
    split4(v, h, m, l);
    char *d = lds + (part >> 3) * kTRChunk + cell * kX6Cell + 8 * (part & 7);
    *(uint2 *)d = h;
    *(uint2 *)(d + 64) = m;
    *(uint2 *)(d + 128) = l;
  };
  const float *xs = x0 + (size_t)s * 35 * 128;
  for (int f = t; f < 35 * 32; f += 192) put(f, *(const f32x4 *)(xs + 4 * f));
  int *flagl = (int *)(lds + kTSFlag);  // set by thread 0 when a hand-off wait gave up
  if (t == 0) *flagl = 0;
  bool failed = false;
  const int co = 16 * g + (lane & 15);
  float sk[4];  // the block input (skip) of this lane's outputs
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int r = 16 * rb + 4 * kg + j;
    sk[j] = r < 35 ? xs[r * 128 + co] : 0.f;
  }

  int aoff[9];
  {
    int r = 16 * rb + (lane & 15);
    r = r < 35 ? r : 34;
    const int ch = r / 7, cw = r - 7 * ch;
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
      const int hh = ch + tap / 3 - 1, ww = cw + tap % 3 - 1;
      const int a = r * kX6Cell + 16 * kg + ((tap / 3 - 1) * 7 + (tap % 3 - 1)) * kX6Cell;
      aoff[tap] = hh >= 0 && hh < 5 && ww >= 0 && ww < 7 ? a : kTRZero + (a & 255);
    }
  }
  const bf16x8 *wl = wp + co * 4 + kg;
  auto bissue = [&](bf16x8(&dst)[3], int l, int L) {  // as k_tower_x6_resident
    l = l < nconv ? l : nconv - 1;
    const int q2 = L / 9, t2 = L - 9 * q2;
    const bf16x8 *src = wl + (size_t)l * kTRConvW + (t2 * 4 + q2) * 3 * 512;
#pragma unroll
    for (int p = 0; p < 3; p++) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[p]) : "v"(src + p * 512));
  };
  bf16x8 bq[Ahead][3];
  if (compute) {
#pragma unroll
    for (int L = 0; L < Ahead - 1; L++) bissue(bq[L], 0, L);
  }
  __syncthreads();

  gu32 *cnt = (gu32 *)(sync + 32 * s);
  for (int l = 0; l < nconv; l++) {
    HZ_SSTAMP(0)
    const bool second = l & 1, last = l == nconv - 1;
    float *xo = xch + ((size_t)(l & 1) * batch + s) * 35 * 128;
    if (compute) {
    const float bv = biasl[l * 16 + (lane & 15)];
    f32x4 acc = {};
    // A fragments kTSAAhead K-steps ahead (a ring of kTSAAhead + 1 slots):
    // with the reads issued just before their MFMAs, every K-step paid the
    // LDS latency (~275 cycles per K-step against 96 of MFMA issue)
    bf16x8 af[kTSAAhead + 1][3];
    auto aread = [&](bf16x8(&dst)[3], int L) {
      const int q2 = L / 9, t2 = L - 9 * q2;
#pragma unroll
      for (int pa = 0; pa < 3; pa++) dst[pa] = *(const bf16x8 *)(lds + q2 * kTRChunk + aoff[t2] + 64 * pa);
    };
#pragma unroll
    for (int L = 0; L < kTSAAhead; L++) aread(af[L], L);
#pragma unroll
    for (int L = 0; L < 36; L++) {
      const int Lf = L + Ahead - 1;
      if (Lf < 36)
        bissue(bq[Lf % Ahead], l, Lf);
      else
        bissue(bq[Lf % Ahead], l + 1, Lf - 36);
      if (L + kTSAAhead < 36) aread(af[(L + kTSAAhead) % (kTSAAhead + 1)], L + kTSAAhead);
      bf16x8 *b = bq[L % Ahead];
      asm volatile("s_waitcnt vmcnt(%3)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]) : "n"(3 * (Ahead - 1)));
      const bf16x8 *a = af[L % (kTSAAhead + 1)];
#pragma unroll
      for (int pa = 0; pa < 3; pa++)
#pragma unroll
        for (int pb = 0; pb < 3 - pa; pb++) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[pa], b[pb], acc, 0, 0, 0);
    }
    HZ_SSTAMP(1)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int r = 16 * rb + 4 * kg + j;
      if (r >= 35) continue;
      float v = acc[j] + bv;
      if (second) v = v + sk[j];
      v = v > 0.f ? v : 0.f;
      if (second) sk[j] = v;
      if (last)  // a state whose hand-off timed out comes out as NaN (loud, never silently wrong)
        out[((size_t)s * 35 + r) * 128 + co] = failed ? __builtin_nanf("") : v;
      else
        tile[(4 * kg + j) * 20 + (lane & 15)] = v;
    }
    // payload: the wave's 16 x 16 tile transposed through LDS, then one
    // 16-B write-through (sc1) store per lane (narrow sc1 stores are one
    // fabric write each)
    if (!last) {
      __builtin_amdgcn_wave_barrier();
      const int r = 16 * rb + (lane >> 2);
      const f32x4 v4 = *(const f32x4 *)(tile + (lane >> 2) * 20 + 4 * (lane & 3));
      if (r < 35)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1"
                     :
                     : "v"(xo + r * 128 + 16 * g + 4 * (lane & 3)), "v"(v4)
                     : "memory");
    }
    }  // compute
    if (last) {
      // the state's last group to get here (every group is past its last
      // wait) zeroes the state's counters for the next launch
      if (t == 0 && __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its payload stores
    HZ_SSTAMP(2)
    __syncthreads();                                    // ... and every wave is done reading the LDS planes
    if (t == 0) {
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = G * (l + 1);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTSSpinTicks) {  // give up: flag it, finish
          __hip_atomic_store((gu32 *)(sync + 32 * kTSMaxBatch), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *flagl = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    HZ_SSTAMP(3)
    __syncthreads();
    failed = failed || *flagl != 0;
    // the whole activation (every group's channels), every load sc1
    const float *xi = xo;
    f32x4 v[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      int f = t + 192 * k;
      f = f < 35 * 32 ? f : 35 * 32 - 1;
      asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[k]) : "v"(xi + 4 * f));
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]));
#pragma unroll
    for (int k = 0; k < 6; k++)
      if (t + 192 * k < 35 * 32) put(t + 192 * k, v[k]);
    HZ_SSTAMP(4)
    __syncthreads();
    HZ_SSTAMP(5)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's requests past the last conv
}
}  // namespace

// Workgroups of k_tower_x6_split the current device holds at once (its CU
// count x the kernel's occupancy per CU, from the occupancy API), cached per
// device; 0 if the query fails.  A launch whose grid exceeds it could leave
// groups waiting for groups that cannot start, so hz_tower_x6_split refuses
// it (HZ_E_NOT_RESIDENT) and the caller takes the resident tower.
static std::atomic<int32_t> g_split_group_limit{0};  // hz_tower_x6_split_set_limit (0: none)

static int32_t split_resident_groups_device();
static int32_t split_resident_groups() {
  const int32_t v = split_resident_groups_device(), lim = g_split_group_limit.load(std::memory_order_relaxed);
  return lim > 0 && lim < v ? lim : v;
}

static int32_t split_resident_groups_device() {
  static std::atomic<int32_t> cache[64];
  static std::atomic<uint64_t> known{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (known.load(std::memory_order_acquire) >> dev & 1) return cache[dev].load(std::memory_order_relaxed);
  hipDeviceProp_t prop;
  int per_cu = 0, per_cu3 = 0;
  int32_t v = 0;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess &&
      hipFuncSetAttribute((const void *)k_tower_x6_split<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kTSLds) == hipSuccess &&
      hipFuncSetAttribute((const void *)k_tower_x6_split<4, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kTSLds) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_tower_x6_split<4, 1>, 192, kTSLds) ==
          hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu3, (const void *)k_tower_x6_split<4, 3>, 192, kTSLds) ==
          hipSuccess) {
    const int pc = per_cu < per_cu3 ? per_cu : per_cu3;
    v = pc > 0 ? (int32_t)(pc * prop.multiProcessorCount) : 0;
  }
  cache[dev].store(v, std::memory_order_relaxed);
  known.fetch_or(1ull << dev, std::memory_order_release);
  return v;
}

// the split tower's workgroups per state at a batch (the one-row-block form
// up to rb1max states, 24 per state; else 8)
static int32_t split_groups_per_state(int32_t batch, int32_t rb1max) { return batch <= rb1max ? 3 * kTSG : kTSG; }

static int32_t split_rb1max() {
  // one row block per workgroup (3 x kTSG groups per state) up to this batch
  // (HZ_TS_RB1_MAX; at most 256 / (3 x kTSG))
  static const int rb1max = [] {
    const char *e = getenv("HZ_TS_RB1_MAX");
    const int v = e ? atoi(e) : kTSRb1Max;
    return v < 0 ? 0 : v > 256 / (3 * kTSG) ? 256 / (3 * kTSG) : v;
  }();
  return rb1max;
}

extern "C" int hz_tower_x6_split_set_limit(int32_t groups) {
  if (groups < 0) return -1;
  g_split_group_limit.store(groups, std::memory_order_relaxed);
  return 0;
}

extern "C" int32_t hz_tower_x6_split_max_batch(void) {
  const int32_t cap = split_resident_groups(), rb1max = split_rb1max();
  int32_t best = 0;  // every batch up to it fits (callers route by batch <= max_batch)
  for (int32_t b = 1; b <= kTSMaxBatch; b++) {
    const int32_t g = b * split_groups_per_state(b, rb1max);
    if (g > cap || g > 256) break;
    best = b;
  }
  return best;
}

extern "C" int hz_tower_x6_split(const float *x0, const void *wpack6, const float *bias, float *out, float *xch,
                                 uint32_t *sync, int32_t nconv, int32_t batch, const int32_t *live, void *stream) {
  if (!x0 || !wpack6 || !bias || !out || !xch || !sync || batch < 0 || batch > kTSMaxBatch || nconv < 2 ||
      nconv > kTRMaxConv || (nconv & 1))
    return -1;
  if (((uintptr_t)x0 | (uintptr_t)wpack6 | (uintptr_t)out | (uintptr_t)xch | (uintptr_t)sync) & 15) return -1;
  if (batch == 0) return 0;
  // every workgroup of the launch must be resident at once (the hand-off
  // waits on all of them): refuse a grid the device cannot hold
  if (batch * split_groups_per_state(batch, split_rb1max()) > split_resident_groups()) return -2;
  // K-steps of B fragments in flight (HZ_TS_AHEAD=12 for measurements; 4,
  // 6, 9, 12 and 18 measured alike with three row blocks per workgroup)
  static const int ahead = [] {
    const char *e = getenv("HZ_TS_AHEAD");
    return e && atoi(e) == 12 ? 12 : kTSAhead;
  }();
  const bool rb1 = batch <= split_rb1max();
  static std::atomic<uint64_t> init_mask{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    for (const void *f : {(const void *)k_tower_x6_split<4, 1>, (const void *)k_tower_x6_split<12, 1>,
                          (const void *)k_tower_x6_split<4, 3>, (const void *)k_tower_x6_split<12, 3>})
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kTSLds) != hipSuccess) return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  const bf16x8 *wp = (const bf16x8 *)wpack6;
  unsigned *sy = (unsigned *)sync;
  const dim3 grid(batch * kTSG * (rb1 ? 3 : 1)), block(192);
  const hipStream_t st = (hipStream_t)stream;
  if (rb1) {
    if (ahead == 4)
      hipLaunchKernelGGL((k_tower_x6_split<4, 1>), grid, block, kTSLds, st, x0, wp, bias, out, xch, sy, nconv, batch, live);
    else
      hipLaunchKernelGGL((k_tower_x6_split<12, 1>), grid, block, kTSLds, st, x0, wp, bias, out, xch, sy, nconv, batch, live);
  } else {
    if (ahead == 4)
      hipLaunchKernelGGL((k_tower_x6_split<4, 3>), grid, block, kTSLds, st, x0, wp, bias, out, xch, sy, nconv, batch, live);
    else
      hipLaunchKernelGGL((k_tower_x6_split<12, 3>), grid, block, kTSLds, st, x0, wp, bias, out, xch, sy, nconv, batch, live);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

#ifdef HZ_NET_DIAG
extern "C" int hz_net_diag_split_stamps(uint64_t *host) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_split_stamps), sizeof(g_split_stamps)) == hipSuccess ? 0 : 1;
}
extern "C" int hz_net_diag_stamps(uint64_t *host) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_conv_stamps), sizeof(g_conv_stamps)) == hipSuccess ? 0 : 1;
}
#endif

// ---- policy / value heads up to the linear layers ---------------------------
//
// model.py:336-351 after the tower: policy = relu(BN(conv1x1(x))) (2
// channels), value = relu(BN(conv1x1(x))) (1 channel), each flattened in
// NCHW order and concatenated with the 42 global features.  With BN folded
// (hzamd/infer.py), one pass over the [B][35][128] activation writes both
// concatenated inputs of the linear layers: pcat[B][70 + 42], vcat[B][35 + 42].
// Wave per state; lane c < 35 owns cell c (its 128 channels are 512
// contiguous bytes); the weights hw[3][128] (policy 0, 1, value) sit in LDS.
namespace {

__global__ void __launch_bounds__(256) k_heads(const float *__restrict__ x, const float *__restrict__ hw,
                                               const float *__restrict__ hb, const float *__restrict__ glob,
                                               float *__restrict__ pcat, float *__restrict__ vcat, int32_t batch,
                                               const int32_t *__restrict__ live) {
  __shared__ float4 w4[3][32];
  const int t = threadIdx.x, lane = t & 63;
  if (live) batch = *live < batch ? *live : batch;
  if (blockIdx.x * 4 >= batch) return;
  if (t < 96) w4[t >> 5][t & 31] = ((const float4 *)hw)[t];
  __syncthreads();
  const int b = blockIdx.x * 4 + (t >> 6);
  if (b >= batch) return;
  if (lane < 35) {
    const float4 *xr = (const float4 *)(x + ((size_t)b * 35 + lane) * 128);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; k++) {
      const float4 v = xr[k], a = w4[0][k], c = w4[1][k], d = w4[2][k];
      s0 += v.x * a.x + v.y * a.y + v.z * a.z + v.w * a.w;
      s1 += v.x * c.x + v.y * c.y + v.z * c.z + v.w * c.w;
      s2 += v.x * d.x + v.y * d.y + v.z * d.z + v.w * d.w;
    }
    s0 += hb[0];
    s1 += hb[1];
    s2 += hb[2];
    pcat[(size_t)b * 112 + lane] = s0 > 0.f ? s0 : 0.f;
    pcat[(size_t)b * 112 + 35 + lane] = s1 > 0.f ? s1 : 0.f;
    vcat[(size_t)b * 77 + lane] = s2 > 0.f ? s2 : 0.f;
  }
  if (lane < 42) {
    const float g = glob[(size_t)b * 42 + lane];
    pcat[(size_t)b * 112 + 70 + lane] = g;
    vcat[(size_t)b * 77 + 35 + lane] = g;
  }
}

}  // namespace

extern "C" int hz_heads(const float *x, const float *hw, const float *hb, const float *glob, float *pcat,
                        float *vcat, int32_t batch, const int32_t *live, void *stream) {
  if (!x || !hw || !hb || !glob || !pcat || !vcat || batch < 0) return -1;
  if (((uintptr_t)x | (uintptr_t)hw) & 15) return -1;
  if (batch == 0) return 0;
  hipLaunchKernelGGL(k_heads, dim3((batch + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, hw, hb, glob, pcat,
                     vcat, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- the whole head: 1x1 convs, linear layers, softmax, tanh ----------------
//
// model.py:336-357 after the tower, plus ModelManager.predict's softmax
// (model.py:100-104), for the default head shapes (2 + 1 head filters, 143
// actions, 256 hidden units, 42 globals): one launch instead of hz_heads,
// three GEMMs and five elementwise passes (38 us against 86-98 us at batch
// 4096, tools/conv_bench.py).  kHS = 8 states per 256-thread workgroup:
//   1. wave w computes the 1x1 convs of states w and w + 4 (lane = cell, as
//      k_heads) into LDS, state-minor: pin[112][8] (policy 70 || glob 42),
//      vin[77][8] (value 35 || glob 42);
//   2. thread a < 143 computes logit a of the 8 states (wpT[j][a]: the
//      threads' weight loads are coalesced; the inputs are LDS broadcasts);
//   3. thread h computes hidden unit h of the 8 states, relu, times w2[h];
//      the 256 products are summed per state (wave reduction + 4 partials);
//   4. wave w applies the softmax to states w and w + 4.
// Phase stamps (tools/head_phases.py): ~30 k cycles for the 1x1 convs (the
// 73 MB read of the tower output), ~23 k for the policy layer, ~18 k for the
// value layer: every workgroup reads all 143 KB of the linear weights from
// L2 (73 MB in total, as much as the activations; 16 states per workgroup
// would halve that but spills).
// fp32 throughout; the sums run in a different order than hipBLASLt's, so
// results agree with the PyTorch layers to fp32 rounding.
namespace {

constexpr int kHS = 8, kAct = 143, kHid = 256, kGlob = 42, kPIn = 70 + kGlob, kVIn = 35 + kGlob;

#ifdef HZ_NET_DIAG  // phase stamps of wave 0 (tools/head_phases.py)
#define HZ_HSTAMP(k)                                                                  \
  if (t == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][0][k] = __builtin_amdgcn_s_memtime();
#define HZ_HSTAMP_RT(k)                                                               \
  if (t == 0 && blockIdx.x < 1024) g_conv_stamps[blockIdx.x][0][k] = __builtin_amdgcn_s_memrealtime();
#else
#define HZ_HSTAMP(k)
#define HZ_HSTAMP_RT(k)
#endif

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// out[s] = sum_j w[j * ld + col] * in[j][s] over the kHS states, as NB blocks
// of JB rows (the last one cut at J).  A workgroup visits the blocks starting
// from block blockIdx % NB: the workgroups, which all run at once, then read
// different weight rows at a time rather than all queueing on the same L2
// lines (all starting at row 0 made the policy layer 57 k cycles).  The
// block partials are added in block order, so the result does not depend on
// the workgroup.  The blocks are k_heads_fc1's input chunks (policy 7 x 16,
// value 4 x 20 with the last cut at 17) and every sum runs in its order, so
// the two head kernels give bit-identical rows: a board's priors do not
// depend on the size of the batch it was evaluated in.  The next block's
// weight loads are in flight while the current block is summed (one exposed
// L2 round trip instead of NB).
template <int J, int NB, int JB = J / NB>
__device__ __forceinline__ void fcn_pipe(const float *__restrict__ w, int ld, int col,
                                         const float4 (*in)[kHS / 4], float (&out)[kHS]) {
  static_assert(NB * JB >= J && (NB - 1) * JB < J, "NB blocks of JB rows cover J");
  constexpr bool ragged = NB * JB != J;
  float part[NB][kHS];
  const int r0 = blockIdx.x % NB;
  auto block_of = [&](int bi) {
    const int blk = r0 + bi;
    return blk >= NB ? blk - NB : blk;
  };
  auto load = [&](float(&dst)[JB], int blk) {
    const float *wb = w + blk * JB * ld + col;
#pragma unroll
    for (int j = 0; j < JB; j++) dst[j] = ragged && blk * JB + j >= J ? 0.f : wb[(ragged && blk * JB + j >= J ? 0 : j) * ld];
  };
  float wc[JB], wn[JB];
  load(wc, block_of(0));
  for (int bi = 0; bi < NB; bi++) {
    const int blk = block_of(bi);
    if (bi + 1 < NB) load(wn, block_of(bi + 1));
    const float4(*ib)[kHS / 4] = in + blk * JB;
    const int jn = ragged && J - blk * JB < JB ? J - blk * JB : JB;  // block-uniform
    float p[kHS] = {};
#pragma unroll
    for (int j = 0; j < JB; j++) {
      if (!ragged || j < jn) {  // (rows past J are not read: they are not in the input)
        const float wv = wc[j];
#pragma unroll
        for (int q = 0; q < kHS / 4; q++) {
          const float4 v = ib[j][q];
          p[4 * q] += wv * v.x, p[4 * q + 1] += wv * v.y, p[4 * q + 2] += wv * v.z, p[4 * q + 3] += wv * v.w;
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
      for (int s = 0; s < kHS; s++) part[b][s] = b == blk ? p[s] : part[b][s];
#pragma unroll
    for (int j = 0; j < JB; j++) wc[j] = wn[j];
  }
#pragma unroll
  for (int s = 0; s < kHS; s++) {
    float o = part[0][s];
#pragma unroll
    for (int b = 1; b < NB; b++) o += part[b][s];
    out[s] = o;
  }
}

__global__ void __launch_bounds__(256) k_heads_fc(const float *__restrict__ x, const float *__restrict__ glob,
                                                  const float *__restrict__ hw, const float *__restrict__ hb,
                                                  const float *__restrict__ wpT, const float *__restrict__ bp,
                                                  const float *__restrict__ w1T, const float *__restrict__ b1,
                                                  const float *__restrict__ w2, const float *__restrict__ b2,
                                                  float *__restrict__ logits, float *__restrict__ probs,
                                                  float *__restrict__ value, int32_t batch,
                                                  const int32_t *__restrict__ live) {
  // the 1x1 convs' weights, [filter][group][4 float4 + 1 pad]: a lane reads
  // its group kk's float4 k4, and the eight groups of a wave sit 20 words
  // apart (8 distinct 4-bank quads); unpadded, groups kk and kk + 2 were 32
  // words apart, the same banks: 4-way conflicts on 108 ds_read_b128 per
  // thread, most of the kernel's SQ_LDS_BANK_CONFLICT (ratio 0.379 in round 6)
  __shared__ float4 w4[3][8][5];
  __shared__ float4 pin[kPIn][kHS / 4];
  __shared__ float4 vin[kVIn][kHS / 4];
  __shared__ float lg[kHS][kAct + 1];
  __shared__ float vpart[4][kHS];
  // the 1x1 convs' partial sums per 16-channel group, [filter][group][state
  // cell] with a row stride of 292 = 4 mod 32 words: the writers (item i =
  // 8 (state cell) + group, consecutive lanes) and the readers (one state
  // cell per lane, groups in order) both touch 32 distinct banks per 32 lanes
  // (round 5's [item][filter] layout read at a 24-word lane stride; the
  // measured conflict ratio stayed at 0.379 without it: the w4 reads above)
  constexpr int kHpRow = 292;
  static_assert(kHpRow >= kHS * 35 && kHpRow % 32 == 4, "hpart row stride");
  __shared__ float hpart[3][8][kHpRow];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (live) batch = *live < batch ? *live : batch;
  const int s0 = blockIdx.x * kHS;
  if (s0 >= batch) return;
  const int ns = batch - s0 < kHS ? batch - s0 : kHS;
  HZ_HSTAMP(0)
  HZ_HSTAMP_RT(8)
  if (t < 96) w4[t >> 5][(t >> 2) & 7][t & 3] = ((const float4 *)hw)[t];
  for (int i = t; i < kHS * kGlob; i += 256) {
    const int sl = i / kGlob, g = i - kGlob * sl;
    const float v = glob[(size_t)(s0 + (sl < ns ? sl : ns - 1)) * kGlob + g];
    ((float *)pin[70 + g])[sl] = v;
    ((float *)vin[35 + g])[sl] = v;
  }
  __syncthreads();
  HZ_HSTAMP(1)

  // 1. heads' 1x1 convs (rows past the batch reread its last state).  Work
  // item = (state, cell, 16-channel group): every lane busy and every load of
  // the thread issued before any is used (one memory round trip instead of
  // four); the group's three partial sums go to LDS and each (state, cell)
  // adds its eight in group order: k_heads_fc1's split and order, the same
  // bits
  {
    constexpr int kItems = kHS * 35 * 8, kIt = (kItems + 255) / 256;
    f32x4 u[kIt][4];
#pragma unroll
    for (int it = 0; it < kIt; it++) {
      int i = it * 256 + t;
      i = i < kItems ? i : kItems - 1;
      const int sl = i / 280, rem = i - 280 * sl, cell = rem >> 3, kk = rem & 7;
      const f32x4 *xr = (const f32x4 *)(x + ((size_t)(s0 + (sl < ns ? sl : ns - 1)) * 35 + cell) * 128) + 4 * kk;
#pragma unroll
      for (int k4 = 0; k4 < 4; k4++) u[it][k4] = xr[k4];
    }
#pragma unroll
    for (int it = 0; it < kIt; it++) {
      const int i = it * 256 + t;
      if (i < kItems) {
        const int kk = i & 7;
        float e0 = 0.f, e1 = 0.f, e2 = 0.f;
#pragma unroll
        for (int k4 = 0; k4 < 4; k4++) {
          const f32x4 v = u[it][k4];
          const float4 p = w4[0][kk][k4], q = w4[1][kk][k4], r = w4[2][kk][k4];
          e0 += v[0] * p.x + v[1] * p.y + v[2] * p.z + v[3] * p.w;
          e1 += v[0] * q.x + v[1] * q.y + v[2] * q.z + v[3] * q.w;
          e2 += v[0] * r.x + v[1] * r.y + v[2] * r.z + v[3] * r.w;
        }
        hpart[0][kk][i >> 3] = e0;
        hpart[1][kk][i >> 3] = e1;
        hpart[2][kk][i >> 3] = e2;
      }
    }
    __syncthreads();
    const float h0 = hb[0], h1 = hb[1], h2 = hb[2];
    for (int i = t; i < kHS * 35; i += 256) {
      const int sl = i / 35, cell = i - 35 * sl;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; kk++) {
        a0 += hpart[0][kk][i];
        a1 += hpart[1][kk][i];
        a2 += hpart[2][kk][i];
      }
      a0 += h0, a1 += h1, a2 += h2;
      ((float *)pin[cell])[sl] = a0 > 0.f ? a0 : 0.f;
      ((float *)pin[35 + cell])[sl] = a1 > 0.f ? a1 : 0.f;
      ((float *)vin[cell])[sl] = a2 > 0.f ? a2 : 0.f;
    }
  }
  __syncthreads();
  HZ_HSTAMP(2)

  // 2. policy logits
  if (t < kAct) {
    float acc[kHS];
    fcn_pipe<kPIn, 7>(wpT, kAct, t, pin, acc);
    const float bb = bp[t];
#pragma unroll
    for (int s = 0; s < kHS; s++) lg[s][t] = acc[s] + bb;
  }
  HZ_HSTAMP(3)

  // 3. value: hidden unit t, relu, times w2[t], summed over the units
  {
    float acc[kHS];
    fcn_pipe<kVIn, 4, 20>(w1T, kHid, t, vin, acc);
    const float bb = b1[t], wo = w2[t];
#pragma unroll
    for (int s = 0; s < kHS; s++) {
      float hv = acc[s] + bb;
      hv = hv > 0.f ? hv : 0.f;
      const float c = wave_sum(hv * wo);
      if (lane == 0) vpart[w][s] = c;
    }
  }
  __syncthreads();
  HZ_HSTAMP(4)
  if (t < ns) value[s0 + t] = tanhf(((vpart[0][t] + vpart[1][t]) + (vpart[2][t] + vpart[3][t])) + b2[0]);

  // 4. softmax over all 143 logits (model.py:104: no legality mask)
#pragma unroll
  for (int k = 0; k < kHS / 4; k++) {
    const int sl = w + 4 * k;
    if (sl >= ns) break;
    const bool has2 = lane + 128 < kAct;
    const float l0 = lg[sl][lane], l1 = lg[sl][lane + 64], l2 = has2 ? lg[sl][lane + 128] : -INFINITY;
    const size_t o = (size_t)(s0 + sl) * kAct;
    if (logits) {
      logits[o + lane] = l0;
      logits[o + lane + 64] = l1;
      if (has2) logits[o + lane + 128] = l2;
    }
    if (probs) {
      const float m = wave_max(fmaxf(fmaxf(l0, l1), l2));
      const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = has2 ? expf(l2 - m) : 0.f;
      const float inv = 1.f / wave_sum((e0 + e1) + e2);
      probs[o + lane] = e0 * inv;
      probs[o + lane + 64] = e1 * inv;
      if (has2) probs[o + lane + 128] = e2 * inv;
    }
  }
  HZ_HSTAMP(5)
  HZ_HSTAMP_RT(9)
}
#undef HZ_HSTAMP
#undef HZ_HSTAMP_RT

// The same head for the smallest batches (config 1's one-board predict, the
// arena's few dozen rows): one state per 1024-thread workgroup, every layer
// split over the inputs so that each thread has at most 20 weight loads,
// all in flight at once (k_heads_fc's 8-state workgroup walks its weight
// rows in 7 + 4 dependent blocks: ~24 us at any batch up to 8).  Partial
// sums are added in k_heads_fc's order, so rows are bit-identical between
// the two kernels.
constexpr int kH1Max = 2048;  // batches up to this take k_heads_fc1 (HZ_HEADS1_MAX overrides; equal at 2048, 0.8 % slower at 4096)
__global__ void __launch_bounds__(1024) k_heads_fc1(const float *__restrict__ x, const float *__restrict__ glob,
                                                    const float *__restrict__ hw, const float *__restrict__ hb,
                                                    const float *__restrict__ wpT, const float *__restrict__ bp,
                                                    const float *__restrict__ w1T, const float *__restrict__ b1,
                                                    const float *__restrict__ w2, const float *__restrict__ b2,
                                                    float *__restrict__ logits, float *__restrict__ probs,
                                                    float *__restrict__ value, int32_t batch,
                                                    const int32_t *__restrict__ live) {
  __shared__ float c1p[105][9];  // 1x1 convs: (head channel, cell) x 8 channel chunks (+1 pad)
  __shared__ float pin[kPIn], vin[kVIn];
  __shared__ float p2[7][kAct];  // policy: 7 chunks of 16 inputs
  __shared__ float p3[4][kHid];  // value: 4 chunks of 20 (the last 17) inputs
  __shared__ float lg[kAct + 1];
  __shared__ float vpart[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (live) batch = *live < batch ? *live : batch;
  const int s = blockIdx.x;
  if (s >= batch) return;
  // 1. the heads' 1x1 convs: output o = head channel * 35 + cell, 16 input channels per thread
  if (t < 105 * 8) {
    const int o = t >> 3, part = t & 7, hc = o / 35, cell = o - 35 * hc;
    const float4 *xv = (const float4 *)(x + ((size_t)s * 35 + cell) * 128 + 16 * part);
    const float4 *wv = (const float4 *)(hw + hc * 128 + 16 * part);
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const float4 u = xv[k], q = wv[k];
      a += u.x * q.x + u.y * q.y + u.z * q.z + u.w * q.w;
    }
    c1p[o][part] = a;
  } else if (t < 105 * 8 + kGlob) {
    const float v = glob[(size_t)s * kGlob + t - 105 * 8];
    pin[70 + t - 105 * 8] = v;
    vin[35 + t - 105 * 8] = v;
  }
  __syncthreads();
  if (t < 105) {
    const int hc = t / 35, cell = t - 35 * hc;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) a += c1p[t][k];
    a += hb[hc];
    a = a > 0.f ? a : 0.f;
    if (hc < 2)
      pin[t] = a;
    else
      vin[cell] = a;
  }
  __syncthreads();
  // 2. policy partials (t < 1001: chunk t / 143 of 16 inputs, column t % 143)
  //    and value partials (all threads: chunk t / 256, hidden unit t % 256)
  float pp = 0.f, vp = 0.f;
  const int pc = t / kAct, pcol = t - kAct * pc;
  if (pc < 7) {
    float wr[16];
#pragma unroll
    for (int j = 0; j < 16; j++) wr[j] = wpT[(size_t)(16 * pc + j) * kAct + pcol];
#pragma unroll
    for (int j = 0; j < 16; j++) pp += wr[j] * pin[16 * pc + j];
  }
  {
    const int vc = t >> 8, u = t & 255, j0 = 20 * vc, nj = vc < 3 ? 20 : kVIn - 60;
    float wr[20];
#pragma unroll
    for (int j = 0; j < 20; j++) wr[j] = j < nj ? w1T[(size_t)(j0 + j) * kHid + u] : 0.f;
#pragma unroll
    for (int j = 0; j < 20; j++)
      if (j < nj) vp += wr[j] * vin[j0 + j];
    p3[vc][u] = vp;
  }
  if (pc < 7) p2[pc][pcol] = pp;
  __syncthreads();
  if (t < kAct) {
    float a = p2[0][t];
#pragma unroll
    for (int c = 1; c < 7; c++) a += p2[c][t];
    lg[t] = a + bp[t];
  } else if (t >= 256 && t < 512) {
    const int u = t - 256;
    float h = (((p3[0][u] + p3[1][u]) + p3[2][u]) + p3[3][u]) + b1[u];  // k_heads_fc's order
    h = h > 0.f ? h : 0.f;
    const float c = wave_sum(h * w2[u]);
    if (lane == 0) vpart[w - 4] = c;
  }
  __syncthreads();
  // 3. value (tanh) and the softmax over all 143 logits (model.py:104)
  if (w == 1 && lane == 0) value[s] = tanhf(((vpart[0] + vpart[1]) + (vpart[2] + vpart[3])) + b2[0]);
  if (w == 0) {
    const bool has2 = lane + 128 < kAct;
    const float l0 = lg[lane], l1 = lg[lane + 64], l2 = has2 ? lg[lane + 128] : -INFINITY;
    const size_t o = (size_t)s * kAct;
    if (logits) {
      logits[o + lane] = l0;
      logits[o + lane + 64] = l1;
      if (has2) logits[o + lane + 128] = l2;
    }
    if (probs) {
      const float m = wave_max(fmaxf(fmaxf(l0, l1), l2));
      const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = has2 ? expf(l2 - m) : 0.f;
      const float inv = 1.f / wave_sum((e0 + e1) + e2);
      probs[o + lane] = e0 * inv;
      probs[o + lane + 64] = e1 * inv;
      if (has2) probs[o + lane + 128] = e2 * inv;
    }
  }
}

}  // namespace

extern "C" int hz_heads_fc(const float *x, const float *glob, const float *hw, const float *hb, const float *wpT,
                           const float *bp, const float *w1T, const float *b1, const float *w2, const float *b2,
                           float *logits, float *probs, float *value, int32_t batch, const int32_t *live,
                           void *stream) {
  if (!x || !glob || !hw || !hb || !wpT || !bp || !w1T || !b1 || !w2 || !b2 || !value || batch < 0) return -1;
  if (((uintptr_t)x | (uintptr_t)hw) & 15) return -1;
  if (batch == 0) return 0;
  static const int32_t h1max = [] {
    const char *e = getenv("HZ_HEADS1_MAX");
    return e ? (int32_t)atoi(e) : (int32_t)kH1Max;
  }();
  if (batch <= h1max)
    hipLaunchKernelGGL(k_heads_fc1, dim3(batch), dim3(1024), 0, (hipStream_t)stream, x, glob, hw, hb, wpT, bp, w1T,
                       b1, w2, b2, logits, probs, value, batch, live);
  else
    hipLaunchKernelGGL(k_heads_fc, dim3((batch + kHS - 1) / kHS), dim3(256), 0, (hipStream_t)stream, x, glob, hw,
                       hb, wpT, bp, w1T, b1, w2, b2, logits, probs, value, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- the stem: 3x3 conv 38 -> 128 channels + bias + ReLU (model.py:328-330) -
//
// Same tiling as k_conv3x3_w8 (8 states per workgroup, wave = row half x 32
// output channels, 9 x 2 tiles of v_mfma_f32_16x16x4_f32), but the input is
// the encoder's NCHW board [B][38][5][7] read directly (no layout copy),
// staged once per workgroup into a zero-halo LDS grid with the channels
// padded to 48 (three 16-channel steps per tap; the weights are packed with
// zero rows for channels 38-47).
namespace {

constexpr int kStemC = 38, kStemCP = 48;
constexpr int kStemRow = kStemCP + 4;  // floats per padded cell
constexpr int kStemLds = kCS * 63 * kStemRow;
constexpr int kStemN = kCS * kStemC * 35;        // board floats per workgroup
constexpr int kStemIt = (kStemN + 511) / 512;    // per thread (21)

__global__ void __launch_bounds__(512, 1)
    k_stem3x3(const float *__restrict__ board, const float4 *__restrict__ wp, const float *__restrict__ bias,
              float *__restrict__ out, int32_t batch, const int32_t *__restrict__ live) {
  extern __shared__ float4 lds4[];
  float *lds = (float *)lds4;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kg = lane >> 4, rh = w >> 2;
  const int s0 = blockIdx.x * kCS;
  if (live) batch = *live < batch ? *live : batch;
  if (s0 >= batch) return;
  const int ns = batch - s0 < kCS ? batch - s0 : kCS;

  // all of this thread's board loads are issued first (coalesced along the
  // NCHW board), the grid is zeroed (halo and channels 38-47) while they are
  // in flight, then the interior is written
  float v[kStemIt];
#pragma unroll
  for (int k = 0; k < kStemIt; k++) {
    const int i = t + 512 * k;
    if (i < kStemN) {
      const int s = i / (kStemC * 35);
      const int sg = s < ns ? s0 + s : s0 + ns - 1;
      v[k] = board[(size_t)sg * (kStemC * 35) + (i - s * (kStemC * 35))];
    }
  }
  for (int i = t; i < kStemLds / 4; i += 512) lds4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kStemIt; k++) {
    const int i = t + 512 * k;
    if (i < kStemN) {
      int s = i / (kStemC * 35), r = i - s * (kStemC * 35), c = r / 35, cell = r - 35 * c;
      int ch = cell / 7, cw = cell - 7 * ch;
      lds[(s * 63 + (ch + 1) * 9 + cw + 1) * kStemRow + c] = v[k];
    }
  }
  __syncthreads();

  int abase[kRB];
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) {
    int r = (rh * kRB + rb) * 16 + (lane & 15);
    r = r < kRows ? r : kRows - 1;
    int s = r / 35, cell = r - 35 * s, ch = cell / 7, cw = cell - 7 * ch;
    abase[rb] = (s * 63 + ch * 9 + cw) * kStemRow + 4 * kg;
  }
  f32x4 acc[kRB][2];
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) acc[rb][0] = acc[rb][1] = (f32x4){};

  const int co0 = 32 * (w & 3) + (lane & 15);
  // B fragment of step L = tap * 3 + gs: wp[((tap * 3 + gs) * 128 + co0 + 16 cb) * 4 + kg]
  const float4 *wl = wp + co0 * 4 + kg;
  // one slot per channel step (static registers), loaded a step ahead
  float4 b[3][2];
  b[0][0] = wl[0];
  b[0][1] = wl[64];
  for (int tap = 0; tap < 9; tap++) {
    const int toff = ((tap / 3) * 9 + tap % 3) * kStemRow;
#pragma unroll
    for (int gs = 0; gs < 3; gs++) {
      const int L = tap * 3 + gs, Ln = L + 1 < 27 ? L + 1 : 26;
      b[(gs + 1) % 3][0] = wl[Ln * 512];
      b[(gs + 1) % 3][1] = wl[Ln * 512 + 64];
      float4 a[kRB];
#pragma unroll
      for (int rb = 0; rb < kRB; rb++) a[rb] = *(const float4 *)(lds + abase[rb] + toff + 16 * gs);
      const float4 b0 = b[gs][0], b1 = b[gs][1];
#define HZ_MF(c)                                                                              \
  _Pragma("unroll") for (int rb = 0; rb < kRB; rb++) {                                        \
    acc[rb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb].c, b0.c, acc[rb][0], 0, 0, 0);    \
    acc[rb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb].c, b1.c, acc[rb][1], 0, 0, 0);    \
  }
      HZ_MF(x)
      HZ_MF(y)
      HZ_MF(z)
      HZ_MF(w)
#undef HZ_MF
    }
  }

  const float bc0 = bias[co0], bc1 = bias[co0 + 16];
  float *ob = out + (size_t)s0 * 35 * 128 + co0;
  const int nrow = ns * 35;
#pragma unroll
  for (int rb = 0; rb < kRB; rb++) {
    const int rbase = (rh * kRB + rb) * 16 + 4 * kg;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (rbase + j < nrow) {
        float v0 = acc[rb][0][j] + bc0, v1 = acc[rb][1][j] + bc1;
        ob[(rbase + j) * 128] = v0 > 0.f ? v0 : 0.f;
        ob[(rbase + j) * 128 + 16] = v1 > 0.f ? v1 : 0.f;
      }
    }
  }
}

}  // namespace

extern "C" int hz_stem3x3_bias_act(const float *board, const float *wpack, const float *bias, float *out,
                                   int32_t batch, const int32_t *live, void *stream) {
  if (!board || !wpack || !bias || !out || batch < 0) return -1;
  if (((uintptr_t)wpack | (uintptr_t)out) & 15) return -1;
  if (batch == 0) return 0;
  static std::atomic<uint64_t> init_mask{0};
  const size_t lds = (size_t)kStemLds * sizeof(float);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1;
  if (!(init_mask.load(std::memory_order_acquire) >> dev & 1)) {
    if (hipFuncSetAttribute((const void *)k_stem3x3, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return 1;
    init_mask.fetch_or(1ull << dev, std::memory_order_release);
  }
  hipLaunchKernelGGL(k_stem3x3, dim3((batch + kCS - 1) / kCS), dim3(512), lds, (hipStream_t)stream, board,
                     (const float4 *)wpack, bias, out, batch, live);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
