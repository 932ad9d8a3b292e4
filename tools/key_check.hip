// canon_key_child against canon_key (tools/key_check.py): for every legal
// action of every given state, the child's key built from its parent's equals
// the key built from the child's state, in both key forms.  One thread per
// (state, action); turn-ending children draw piles from a per-pair script.
#include <hip/hip_runtime.h>
#include "../harmonies-alphazero_amd/csrc/hz_device.hpp"
using namespace hz;

__global__ void __launch_bounds__(256) k_key_check(const uint64_t *st, int n, unsigned long long *out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * kActions) return;
  const int b = (int)(i / kActions), a = (int)(i % kActions);
  State s;
  for (int k = 0; k < 4; k++) s.pl[k] = st[(size_t)k * n + b];
  s.piles = st[(size_t)4 * n + b];
  s.misc = st[(size_t)5 * n + b];
  if (game_done(s.misc)) return;
  uint64_t mk[3];
  legal_mask(s, mk);
  if (!((mk[a >> 6] >> (a & 63)) & 1)) return;
  unsigned long long bad = 0;
  for (int py = 0; py < 2; py++) {
    State ch = s;
    // a pile script of valid tiles (three tiles per pile, 0..5)
    uint64_t z = mix64(((uint64_t)b << 8) ^ (uint64_t)a), script = 0;
    for (int q = 0; q < 5; q++) {
      uint64_t p9 = (z % 6) | ((z / 6) % 6) << 3 | ((z / 36) % 6) << 6;
      script |= p9 << (9 * q);
      z = mix64(z);
    }
    ScriptDraw sd{script};
    if (step_state(ch, a, sd) != ST_OK) {
      bad |= 4;
      continue;
    }
    const CKey want = canon_key(ch, py), pk = canon_key(s, py);
    const CKey got = canon_key_child(pk, s, ch, a, py);
    if (!key_eq(want, got)) bad |= 1ull << py;
  }
  atomicAdd(&out[0], 1ull);
  if (bad) atomicAdd(&out[1], 1ull);
  if (bad & 4) atomicAdd(&out[2], 1ull);
}

extern "C" int hz_key_check(const uint64_t *st, int n, unsigned long long *out) {
  const long long pairs = (long long)n * kActions;
  hipLaunchKernelGGL(k_key_check, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, 0, st, n, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
