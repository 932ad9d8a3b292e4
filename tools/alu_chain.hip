// Dependent-chain cycle costs of the integer ops the MT seeding recurrence
// can be built from (tools/alu_chain.py): one wave per SIMD, 1024 steps.
#include <hip/hip_runtime.h>
#include <cstdint>

// v_mul_u32_u24 as an opaque op (the compiler would fold the pieces back
// into one v_mul_lo_u32)
__device__ __forceinline__ uint32_t mul24(uint32_t c, uint32_t a) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(c), "v"(a));
  return r;
}

template <int K>
__device__ __forceinline__ uint32_t step(uint32_t x, uint32_t k) {
  if constexpr (K == 0) {  // v_mul_lo_u32 chain
    return x * 1664525u;
  } else if constexpr (K == 1) {  // v_mul_u32_u24 chain
    return mul24(1664525u, x);
  } else if constexpr (K == 2) {  // xor-shift chain (2 plain ops)
    return x ^ (x >> 3);
  } else if constexpr (K == 3) {  // the seeding step as written
    return ((x ^ (x >> 30)) * 1664525u ^ k) + 7u;
  } else if constexpr (K == 4) {  // the seeding step, multiply by 24-bit halves
    uint32_t t = x ^ (x >> 30);
    uint32_t p = mul24(1664525u, t) + (mul24(1664525u, t >> 24) << 24);
    return (p ^ k) + 7u;
  } else if constexpr (K == 5) {  // pass-2 step as written
    return ((x ^ (x >> 30)) * 1566083941u ^ k) - 7u;
  } else {  // pass-2 step, multiply by 24-bit pieces (C = lo24 + hi8 << 24)
    uint32_t t = x ^ (x >> 30);
    constexpr uint32_t lo = 1566083941u & 0xFFFFFFu, hi = 1566083941u >> 24;
    uint32_t p = mul24(lo, t) + ((mul24(lo, t >> 24) + mul24(hi, t)) << 24);
    return (p ^ k) - 7u;
  }
}

template <int K>
__global__ void __launch_bounds__(64) k_chain(uint32_t *out, uint64_t *cyc, uint32_t k) {
  uint32_t x = threadIdx.x * 2654435761u + 1;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < 1024; i++) x = step<K>(x, k);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int alu_chain(int kind, void *out, void *cyc, int blocks) {
  dim3 g(blocks), b(64);
  uint32_t k = 0x12345u;
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_chain<0>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 1: hipLaunchKernelGGL(k_chain<1>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 2: hipLaunchKernelGGL(k_chain<2>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 3: hipLaunchKernelGGL(k_chain<3>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 4: hipLaunchKernelGGL(k_chain<4>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 5: hipLaunchKernelGGL(k_chain<5>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    case 6: hipLaunchKernelGGL(k_chain<6>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, k); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- seeding variants (cycles per wave for one 64-board seeding)
#include "../harmonies-alphazero_amd/csrc/hz_device.hpp"
using namespace hz;

// pass 1 as mt_seed runs it, with or without the LDS stores
template <bool Store>
__device__ __forceinline__ uint32_t pass1(uint32_t *w, int stride, uint32_t kA, uint32_t kB) {
  uint32_t prev = 19650218u, acc = 0;
  uint32_t iv[8];
#pragma unroll
  for (int u = 0; u < 8; u++) iv[u] = kInitGen.v[1 + u];
  for (int g = 1; g < kMT - 7; g += 8) {
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = kInitGen.v[g + 8 + u < kMT ? g + 8 + u : kMT - 1];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      if (Store) w[(g + u) * stride] = v;
      else acc ^= v;
      prev = v;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = nx[u];
  }
  return prev ^ acc;
}

// pass 1 with the table words read from LDS (a block copy) instead of SMEM
__device__ __forceinline__ uint32_t pass1_ldstab(uint32_t *w, int stride, const uint32_t *tab, uint32_t kA,
                                                 uint32_t kB) {
  uint32_t prev = 19650218u;
  for (int g = 1; g < kMT - 7; g += 8) {
    uint32_t iv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) iv[u] = tab[g + u];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (iv[u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
      w[(g + u) * stride] = v;
      prev = v;
    }
  }
  return prev;
}

// pass 2 alone over an already seeded column: Mode 0 as mt_seed_tab, 1 no
// stores (values folded into a register), 2 no loads (a register stands in)
template <int Mode>
__device__ __forceinline__ uint32_t pass2(uint32_t *w, uint32_t prev) {
  constexpr int S = 64;
  uint32_t acc = 0;
  uint32_t cur[8];
#pragma unroll
  for (int u = 0; u < 8; u++) cur[u] = Mode == 2 ? prev + u : w[(2 + u) * S];
#pragma unroll 2
  for (int g = 2; g < kMT - 6; g += 8) {
    uint32_t nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) nx[u] = Mode == 2 ? cur[u] ^ 0x9e3779b9u : w[(g + 8 + u < kMT ? g + 8 + u : kMT - 1) * S];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      uint32_t v = (cur[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)(g + u);
      if (Mode == 1) acc ^= v;
      else w[(g + u) * S] = v;
      prev = v;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = nx[u];
  }
  return prev ^ acc;
}

// random.seed(int) (init_by_array) with every word in global memory,
// word-major w[i * ns]: the chain wave issues no LDS operation (its stores
// are fire-and-forget vector stores; pass 2 reads its pass-1 words PF steps
// ahead), init_genrand's table through the scalar cache (no LDS waits mix
// with it).  Same words as mt_seed.
template <int PF>
__device__ __forceinline__ void mt_seed_global(uint32_t *w, size_t ns, uint64_t seed) {
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
      w[(size_t)(g + u) * ns] = v;
      if (u == 0 && g == 1) m1 = v;
      prev = v;
    }
  }
#pragma unroll
  for (int u = 0; u < 7; u++) {  // i = 617..623
    const uint32_t v = (kInitGen.v[617 + u] ^ ((prev ^ (prev >> 30)) * 1664525U)) + ((u & 1) ? kB : kA);
    w[(size_t)(617 + u) * ns] = v;
    prev = v;
  }
  // mt[0] = mt[623]; the 624th step at i = 1 (key j = 623 % keylen -> kB)
  prev = (m1 ^ ((prev ^ (prev >> 30)) * 1664525U)) + kB;
  const uint32_t first1 = prev;
  // pass 2: i = 2..623 over the pass-1 words, read PF steps ahead
  uint32_t ring[PF];
#pragma unroll
  for (int u = 0; u < PF; u++) ring[u] = w[(size_t)(2 + u) * ns];
  for (int g = 2; g < 2 + ((kMT - 2) / PF) * PF; g += PF) {
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
    const int i = 2 + ((kMT - 2) / PF) * PF + u;
    const uint32_t v = (ring[u] ^ ((prev ^ (prev >> 30)) * 1566083941U)) - (uint32_t)i;
    w[(size_t)i * ns] = v;
    prev = v;
  }
  w[ns] = (first1 ^ ((prev ^ (prev >> 30)) * 1566083941U)) - 1U;
  w[0] = 0x80000000U;
}

template <int PF>
__global__ void __launch_bounds__(64) k_seedglob(uint32_t *out, uint64_t *cyc, uint32_t *ws, size_t ns) {
  const int lane = threadIdx.x, b = blockIdx.x * 64 + lane;
  const uint64_t sd = 1234 + (uint64_t)b;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  mt_seed_global<PF>(ws + b, ns, sd);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[b] = ws[7 * ns + b];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// the same seeds through mt_seed (LDS), for the comparison of the words
__global__ void __launch_bounds__(64) k_seedref(uint32_t *ws, size_t ns) {
  const int lane = threadIdx.x, b = blockIdx.x * 64 + lane;
  mt_seed(hz_lds + lane, 64, 1234 + (uint64_t)b);
  __syncthreads();
  for (int i = 0; i < kMT; i++) ws[(size_t)i * ns + b] = hz_lds[i * 64 + lane];
}

extern "C" int seed_glob(int pf, void *out, void *cyc, void *ws, long ns, int blocks) {
  dim3 g(blocks), b(64);
  if (pf == 8) hipLaunchKernelGGL(k_seedglob<8>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, (uint32_t *)ws, (size_t)ns);
  else if (pf == 16) hipLaunchKernelGGL(k_seedglob<16>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, (uint32_t *)ws, (size_t)ns);
  else if (pf == 24) hipLaunchKernelGGL(k_seedglob<24>, g, b, 0, 0, (uint32_t *)out, (uint64_t *)cyc, (uint32_t *)ws, (size_t)ns);
  else if (pf == 0) {
    size_t lds = (size_t)kMT * 64 * 4;
    hipFuncSetAttribute((const void *)k_seedref, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_seedref, g, b, lds, 0, (uint32_t *)ws, (size_t)ns);
  } else return -1;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int V>
__global__ void __launch_bounds__(64) k_seedvar(uint32_t *out, uint64_t *cyc) {
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t tab[kMT];
  int lane = threadIdx.x;
  for (int i = lane; i < kMT; i += 64) tab[i] = kInitGen.v[i];
  __syncthreads();
  uint64_t sd = 1234 + blockIdx.x * 64 + lane;
  uint32_t kA = (uint32_t)sd, kB = (uint32_t)(sd >> 32) ? (uint32_t)(sd >> 32) + 1 : kA;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
  if constexpr (V == 0) mt_seed(hz_lds + lane, 64, sd);
  if constexpr (V == 1) r = pass1<true>(hz_lds + lane, 64, kA, kB);
  if constexpr (V == 2) r = pass1<false>(hz_lds + lane, 64, kA, kB);
  if constexpr (V == 3) r = pass1_ldstab(hz_lds + lane, 64, tab, kA, kB);
  if constexpr (V == 4) mt_seed_tab<64>(hz_lds + lane, tab, sd);
  if constexpr (V >= 8 && V <= 10) {
    mt_seed_tab<64>(hz_lds + lane, tab, sd);
    t0 = __builtin_amdgcn_s_memtime();
    r = pass2<V - 8>(hz_lds + lane, kA);
  }
  if constexpr (V == 5) mt_seed_tab<65>(hz_lds + lane, tab, sd);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = r ^ hz_lds[7 * 64 + lane];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int seed_var(int v, void *out, void *cyc, int blocks) {
  dim3 g(blocks), b(64);
  size_t lds = (size_t)kMT * 64 * 4;
  static bool init = false;
  if (!init) {
    hipFuncSetAttribute((const void *)k_seedvar<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<9>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void *)k_seedvar<10>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    init = true;
  }
  switch (v) {
    case 0: hipLaunchKernelGGL(k_seedvar<0>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 1: hipLaunchKernelGGL(k_seedvar<1>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 2: hipLaunchKernelGGL(k_seedvar<2>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 3: hipLaunchKernelGGL(k_seedvar<3>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 4: hipLaunchKernelGGL(k_seedvar<4>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 6: hipLaunchKernelGGL(k_seedvar<0>, dim3(256), b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 7: hipLaunchKernelGGL(k_seedvar<4>, dim3(256), b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 8: hipLaunchKernelGGL(k_seedvar<8>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 9: hipLaunchKernelGGL(k_seedvar<9>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    case 10: hipLaunchKernelGGL(k_seedvar<10>, g, b, lds, 0, (uint32_t *)out, (uint64_t *)cyc); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- pass-2 chain forms, one wave per CU (tools/alu_chain.py "p2chain"):
// cycles per step of pass 2's recurrence over 616 steps with the step's
// memory operations of each candidate layout (V):
//  0 LDS column (stride 65) read 8 ahead + a b32 buffer store per step (P2a)
//  1 LDS column read 8 ahead, no store
//  2 no LDS (operand from registers) + a b32 buffer store per step
//  3 no LDS, no store: the recurrence alone
//  4 LDS board-major (lane's words contiguous, stride S words): b128 reads, no store
//  5 as 4 + a b128 buffer store per 4 steps (board-major global)
//  6 as 4 + a b32 buffer store per step (word-major global)
//  7 no LDS + a b128 buffer store per 4 steps (board-major global)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <int V, int S>
__global__ void __launch_bounds__(64) k_p2chain(uint32_t *gout, uint32_t *out, uint64_t *cyc) {
  const int lane = threadIdx.x, b = blockIdx.x * 64 + lane;
  constexpr bool BM = V >= 4 && V <= 6;  // board-major LDS
  for (int i = 0; i < kMT; i++) {
    if (BM) hz_lds[lane * S + i] = i * 2654435761u + b;
    else hz_lds[i * 65 + lane] = i * 2654435761u + b;
  }
  __syncthreads();
  const uint64_t base = (uint64_t)(gout + (size_t)blockIdx.x * 64 * kMT);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base), hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, 64 * kMT * 4, 0x00020000);
  uint32_t prev = b * 7u + 1u, acc = 0;
  const uint32_t *l = hz_lds + (BM ? lane * S : lane);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  if constexpr (V <= 3 || V == 7) {
    uint32_t cur[8], nx[8];
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = V <= 1 ? l[(2 + u) * 65] : prev + u;
#pragma unroll 2
    for (int g = 2; g < 618; g += 8) {
#pragma unroll
      for (int u = 0; u < 8; u++) nx[u] = V <= 1 ? l[(g + 8 + u) * 65] : cur[u] ^ 0x9e3779b9u;
      const uint32_t kneg = __builtin_amdgcn_readfirstlane(0u - (uint32_t)g);
      const int soff = __builtin_amdgcn_readfirstlane(g * 64 * 4);
      uint32_t q[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t p = (prev ^ (prev >> 30)) * 1566083941U;
        uint32_t v;
        asm("v_xad_u32 %0, %1, %2, %3" : "=v"(v) : "v"(p), "v"(cur[u]), "s"(kneg - (uint32_t)u));
        if (V == 0 || V == 2) __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, soff + u * 256, 0);
        else if (V == 7) q[u] = v;
        else acc ^= v;
        prev = v;
      }
      if (V == 7) {
        __builtin_amdgcn_raw_buffer_store_b128(v4u{q[0], q[1], q[2], q[3]}, rs, lane * kMT * 4, g * 4, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v4u{q[4], q[5], q[6], q[7]}, rs, lane * kMT * 4, g * 4 + 16, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; u++) cur[u] = nx[u];
    }
  } else {
    uint4 c0 = *reinterpret_cast<const uint4 *>(l + 4), c1 = *reinterpret_cast<const uint4 *>(l + 8);
#pragma unroll 2
    for (int g = 4; g < 620; g += 8) {
      const uint4 n0 = *reinterpret_cast<const uint4 *>(l + g + 8), n1 = *reinterpret_cast<const uint4 *>(l + g + 12);
      const uint32_t kneg = __builtin_amdgcn_readfirstlane(0u - (uint32_t)g);
      const int soff = __builtin_amdgcn_readfirstlane(g * 64 * 4);
      const uint32_t cur[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      uint32_t q[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t p = (prev ^ (prev >> 30)) * 1566083941U;
        uint32_t v;
        asm("v_xad_u32 %0, %1, %2, %3" : "=v"(v) : "v"(p), "v"(cur[u]), "s"(kneg - (uint32_t)u));
        if (V == 6) __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, soff + u * 256, 0);
        else if (V == 5) q[u] = v;
        else acc ^= v;
        prev = v;
      }
      if (V == 5) {
        __builtin_amdgcn_raw_buffer_store_b128(v4u{q[0], q[1], q[2], q[3]}, rs, lane * kMT * 4, g * 4, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v4u{q[4], q[5], q[6], q[7]}, rs, lane * kMT * 4, g * 4 + 16, 0);
      }
      c0 = n0;
      c1 = n1;
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[b] = prev ^ acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int p2chain(int v, int s, void *gout, void *out, void *cyc, int blocks) {
  dim3 g(blocks), bl(64);
  const int lds = 160 * 1024;
#define P2C(V, S)                                                                                               \
  do {                                                                                                          \
    hipFuncSetAttribute((const void *)k_p2chain<V, S>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);       \
    hipLaunchKernelGGL((k_p2chain<V, S>), g, bl, lds, 0, (uint32_t *)gout, (uint32_t *)out, (uint64_t *)cyc); \
  } while (0)
  switch (v * 1000 + s) {
    case 0 * 1000 + 0: P2C(0, 628); break;
    case 1 * 1000 + 0: P2C(1, 628); break;
    case 2 * 1000 + 0: P2C(2, 628); break;
    case 3 * 1000 + 0: P2C(3, 628); break;
    case 4 * 1000 + 628: P2C(4, 628); break;
    case 4 * 1000 + 632: P2C(4, 632); break;
    case 5 * 1000 + 628: P2C(5, 628); break;
    case 5 * 1000 + 632: P2C(5, 632); break;
    case 6 * 1000 + 628: P2C(6, 628); break;
    case 7 * 1000 + 0: P2C(7, 628); break;
    default: return -1;
  }
#undef P2C
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
