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
#include <cstdint>

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
