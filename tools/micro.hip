// Microbenchmarks of the device rules in isolation (tools/micro.py).
#include <hip/hip_runtime.h>
#include "../harmonies-alphazero_amd/csrc/hz_device.hpp"
using namespace hz;

__global__ void __launch_bounds__(64) k_draws(uint32_t *mt, int32_t *cur, int n, int reps, uint32_t *sink) {
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  StreamDraw<MT> d{MT(mt + (size_t)b * kMT, cur[b])};
  uint64_t misc = 0;
  for (int t = 0; t < 6; t++) misc = set_bits(misc, 11 + 5 * t, 5, (uint64_t)initial_count(t));
  uint32_t acc = 0;
  for (int r = 0; r < reps; r++) {
    uint32_t p9 = d(misc);
    apply_pile(misc, p9);
    acc += p9;
    if (bag_total(misc) < 6) misc = set_bits(misc, 11, 30, 0x3fffffffULL & 0x2108421ULL * 17);
  }
  sink[b] = acc;
  cur[b] = d.m.cursor();
}

__global__ void __launch_bounds__(64) k_next(uint32_t *mt, int32_t *cur, int n, int reps, uint32_t *sink) {
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  MT m(mt + (size_t)b * kMT, cur[b]);
  uint32_t acc = 0;
  for (int r = 0; r < reps; r++) acc ^= m.next();
  sink[b] = acc;
  cur[b] = m.cursor();
}

__global__ void __launch_bounds__(64) k_score(const uint64_t *pl, int n, int reps, uint32_t *sink) {
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  State s;
  for (int k = 0; k < 4; k++) s.pl[k] = pl[(size_t)k * n + b];
  s.piles = 0; s.misc = 0;
  uint32_t acc = 0;
  for (int r = 0; r < reps; r++) {
    acc += score_player(s, r & 1);
    s.pl[0] ^= (uint64_t)(acc & 1);
  }
  sink[b] = acc;
}

__global__ void __launch_bounds__(64) k_seed(uint32_t *mt, int n, uint32_t *sink) {
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  mt_seed(mt + (size_t)b * kMT, 1, 1234 + b);
  sink[b] = mt[(size_t)b * kMT + 5];
}

__global__ void __launch_bounds__(64) k_seed_lds(uint32_t *mt, int n, uint32_t *sink) {
  uint32_t *lds = hz_lds;
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  mt_seed(lds + threadIdx.x, 65, 1234 + b);
  sink[b] = lds[5 * 65 + threadIdx.x];
}

__global__ void __launch_bounds__(64) k_pick(const uint64_t *seedv, int n, int reps, uint32_t *sink) {
  int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  uint64_t mk[3] = {0x5555555555555555ull ^ b, 0x3333333333333333ull, 0x0f0f0f0f0f0full};
  uint32_t acc = 0;
  for (int r = 0; r < reps; r++) {
    int L = __popcll(mk[0]) + __popcll(mk[1]) + __popcll(mk[2]);
    acc += kth_action(mk, rule_pick(seedv[b], r, L));
    mk[0] ^= acc;
  }
  sink[b] = acc;
}

extern "C" {
int micro_run(int which, void *a, void *b, int n, int reps, void *sink, void *stream) {
  if (install_comp_table()) return -1;
  dim3 g((n + 63) / 64), blk(64);
  hipStream_t s = (hipStream_t)stream;
  switch (which) {
    case 0: hipLaunchKernelGGL(k_draws, g, blk, 0, s, (uint32_t *)a, (int32_t *)b, n, reps, (uint32_t *)sink); break;
    case 1: hipLaunchKernelGGL(k_next, g, blk, 0, s, (uint32_t *)a, (int32_t *)b, n, reps, (uint32_t *)sink); break;
    case 2: hipLaunchKernelGGL(k_score, g, blk, 0, s, (const uint64_t *)a, n, reps, (uint32_t *)sink); break;
    case 3: hipLaunchKernelGGL(k_seed, g, blk, 0, s, (uint32_t *)a, n, (uint32_t *)sink); break;
    case 4:
      hipFuncSetAttribute((const void *)k_seed_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 624 * 65 * 4);
      hipLaunchKernelGGL(k_seed_lds, g, blk, 624 * 65 * 4, s, (uint32_t *)a, n, (uint32_t *)sink);
      break;
    case 5: hipLaunchKernelGGL(k_pick, g, blk, 0, s, (const uint64_t *)a, n, reps, (uint32_t *)sink); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}

// draws with the stream in LDS (as in k_rollout).  mode 0: fresh seeding
// (twists on demand), bag 120 -> 40; modes 1-4: stream pre-twisted like a
// seeded-ahead one and the bag kept in a game's range (105 -> 57):
// 1 full draw (prefetch + draw_pile + apply_pile), 2 sample3_raw only,
// 3 draw_pile only (no prefetch), 4 prefetch only.
__global__ void __launch_bounds__(64) k_draws_lds(uint32_t *mt, int n, int reps, uint32_t *sink, uint64_t *cyc,
                                                  int mode) {
  uint32_t *lds = hz_lds;
  int lane = threadIdx.x, b = blockIdx.x * 64 + lane;
  mt_seed(lds + lane, 65, 99 + b);
  StreamDraw<LdsMT> d{LdsMT(lane, kMTSeeded)};
  if (mode > 0) d.m.twist_ahead(kAheadTwist);
  int lo = mode ? 57 : 40;
  uint64_t misc0 = 0;
  for (int t = 0; t < 6; t++) misc0 = set_bits(misc0, 11 + 5 * t, 5, (uint64_t)initial_count(t));
  if (mode) {  // 15 tiles out, as after the opening piles
    misc0 = set_bits(misc0, 11, 5, 20);
    misc0 = set_bits(misc0, 16, 5, 16);
    misc0 = set_bits(misc0, 21, 5, 18);
    misc0 = set_bits(misc0, 26, 5, 20);
    misc0 = set_bits(misc0, 31, 5, 13);
    misc0 = set_bits(misc0, 36, 5, 18);
  }
  uint64_t misc = misc0;
  uint32_t acc = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    uint32_t p9 = 0;
    if (mode <= 1) {
      p9 = d(misc);
    } else if (mode == 2) {
      uint32_t j[3];
      sample3_raw(d.m, (uint32_t)bag_total(misc), 3, j);
      p9 = j[0] ^ (j[1] << 3) ^ (j[2] << 6);
    } else if (mode == 3) {
      draw_pile(misc, d.m, p9);
    } else {
      d.m.prefetch();
      d.m.pos += 5;
      p9 = d.m.tw;
    }
    if (mode <= 3) apply_pile(misc, p9 & 0x1FF);
    acc += p9;
    if (bag_total(misc) < lo) misc = misc0;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[b] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int micro_draws_lds(void *mt, int n, int reps, void *sink, void *cyc, void *stream, int mode) {
  hipFuncSetAttribute((const void *)k_draws_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 624 * 65 * 4);
  hipLaunchKernelGGL(k_draws_lds, dim3((n + 63) / 64), dim3(64), 624 * 65 * 4, (hipStream_t)stream, (uint32_t *)mt, n,
                     reps, (uint32_t *)sink, (uint64_t *)cyc, mode);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Turn-structured play in isolation (k_rollout's fast path): pairs of turns
// from a reset state, the piles coming from a fixed cyclic script, restarted
// when the game ends.  mode 0: as in k_rollout; 1: rule hash replaced by a
// multiply (hash cost); 2: no end-of-turn refill draw (draw cost).
struct CycleDraw {
  uint32_t k;
  __device__ __forceinline__ uint32_t operator()(uint64_t misc) {
    if (bag_total(misc) < 3) return 0x1FFu;
    // three tiles the bag still holds, cycling through the types
    uint32_t p9 = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      uint32_t t = (k + i) % 6;
#pragma unroll
      for (int s = 0; s < 6; s++) {
        uint32_t tt = (k + i + s) % 6;
        t = bag_n(misc, (int)t) > i ? t : tt;
      }
      p9 |= t << (3 * i);
    }
    k++;
    return p9;
  }
  __device__ __forceinline__ uint32_t take(uint64_t misc, bool want) { return want ? (*this)(misc) : 0x1FFu; }
};

template <int Mode>
__global__ void __launch_bounds__(64) k_turns(int n, int pairs, uint32_t *sink, uint64_t *cyc) {
  int lane = threadIdx.x, b = blockIdx.x * 64 + lane;
  CycleDraw d{(uint32_t)b};
  State s0;
  reset_state(s0, d);
  State s = s0;
  uint64_t rkey = rule_key((uint64_t)b);
  int g = 0;
  uint32_t acc = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < pairs; r++) {
    if (phase_of(s.misc) == PH_OVER) {
      acc += (uint32_t)s.pl[0];
      s = s0;
      g = 0;
    }
    play_turn<0, CycleDraw, Mode == 1>(s, d, rkey, g);
    if (phase_of(s.misc) != PH_OVER) play_turn<1, CycleDraw, Mode == 1>(s, d, rkey, g + 4);
    g += 8;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[b] = acc + (uint32_t)s.pl[1];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int micro_turns(int mode, int n, int pairs, void *sink, void *cyc, void *stream) {
  dim3 g((n + 63) / 64), blk(64);
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0) hipLaunchKernelGGL(k_turns<0>, g, blk, 0, st, n, pairs, (uint32_t *)sink, (uint64_t *)cyc);
  if (mode == 1) hipLaunchKernelGGL(k_turns<1>, g, blk, 0, st, n, pairs, (uint32_t *)sink, (uint64_t *)cyc);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
