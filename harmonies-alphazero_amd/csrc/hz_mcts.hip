// hz_mcts.hip — batched PUCT MCTS over the boards of an hz_env.
//
// Reference: MCTS.py (Node :8-20, Edge :23-39, move_to_leaf :63-149,
// expand_leaf :151-218, back_fill :220-266, get_best_action_and_pi :272-441).
// Every board runs its own single-tree search; all boards advance one
// simulation per "sim step" in lock-step, so the leaf evaluations of all
// boards form one PyTorch batch.  Boards are independent, so lock-stepping
// preserves each board's sequential semantics exactly (no virtual loss).
//
// One wave (64 lanes) owns one board in every tree kernel: lanes are edges
// in selection and backup, children in expansion.  Per board, in HBM:
//   node pool  [max_nodes] : 48 B state, 64 B canonical key, first edge, #edges
//   edge pool  [max_edges] : action, child node, N (int), W (f64), P (f32), player,
//                            hint (the child's first edge / edge count / terminal flag)
//   hash table [hcap] u64  : search generation << 32 | node id (linear probing;
//                            entries of older searches read as empty, so the
//                            table is never cleared)
// Arithmetic follows the reference's NumPy/Python types exactly (see select
// and expand) so that visit counts are bit-identical to the CPU engine.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/hz_abi.h"
#include "hz_device.hpp"
#include "hz_encode.hpp"

using namespace hz;

struct hz_env;  // defined in hz_env.hip; accessed through the ABI getters

struct hz_mcts {
  int32_t n, max_nodes, max_edges, hcap, max_depth;
  int32_t exact_keys;
  int32_t dedup_walk;    // hz_mcts_set_dedup_walk (tests): every sibling dedup takes the serial walk
  int32_t gather_mode;   // hz_mcts_set_gather_encode: -1 process default (HZ_GATHER_ENCODE), 0 layered, 1 fused
  hipStream_t stream;
  uint64_t *node_state;  // [n][max_nodes][6]
  uint64_t *node_key;    // [n][max_nodes][8] canonical key (a probe compares it whole: no key rebuilt)
  int32_t *node_e0;      // [n][max_nodes]
  int32_t *node_ne;      // [n][max_nodes]
  int16_t *edge_action;  // [n][max_edges]
  int32_t *edge_child;   // [n][max_edges]
  int32_t *edge_n;       // [n][max_edges]
  double *edge_w;        // [n][max_edges]
  float *edge_p;         // [n][max_edges]
  uint8_t *edge_player;  // [n][max_edges]
  // [n][max_edges] the child node's e0 << 8 | terminal << 7 | ne as far as
  // known: ne = 0 means "not expanded when last seen" (select then reads the
  // node itself and repairs the hint), so the walk takes one memory round
  // trip per level (edges + hints) instead of two (node, then its edges)
  int32_t *edge_hint;
  uint64_t *ht;          // [n][hcap]
  int32_t *counts;       // [n][4]: nodes, edges, generation, overflow
  int32_t *path;         // [n][max_depth]
  int32_t *depth;        // [n]
  int32_t *leaf;         // [n]  leaf node of the current simulation, -1 = inactive
  int32_t *leaf_gidx;    // [n]  b*max_nodes + leaf for the encoder, -1 = no eval
  int32_t *slot;         // [n]  row of board b in the gathered leaf batch, -1 = not evaluated
  int32_t *gidx_c;       // [n]  leaf_gidx of the gathered rows, in board order
  int64_t *eval_ctr;     // optional (hz_mcts_set_eval_counter): k_gather adds each simulation's row count
};

namespace {

constexpr int kWave = 64;
constexpr int kMaxChildren = 69;  // measured max legal moves
constexpr int kChildSlots = 128;  // two per lane (loop bound: lanes c and c + 64)
constexpr int kChildLds = 72;     // LDS rows per child array: every access has c < nl <= kMaxChildren
constexpr int kDedupSlots = 128;  // sibling-dedup table (load factor <= 69/128)

inline int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

__device__ __forceinline__ uint64_t ht_entry(int gen, int node) {
  return ((uint64_t)(uint32_t)gen << 32) | (uint32_t)node;
}

__device__ __forceinline__ State load_node(const uint64_t *ns) {
  State s;
#pragma unroll
  for (int k = 0; k < 4; k++) s.pl[k] = ns[k];
  s.piles = ns[4];
  s.misc = ns[5];
  return s;
}

__device__ __forceinline__ void store_node(uint64_t *ns, const State &s) {
#pragma unroll
  for (int k = 0; k < 4; k++) ns[k] = s.pl[k];
  ns[4] = s.piles;
  ns[5] = s.misc;
}

// ------------------------------------------------------------------- begin
// Fresh tree per move (MCTS.py:288-289): node 0 = the board's game state.
__global__ void __launch_bounds__(kWave) k_begin(hz_mcts m, const uint64_t *__restrict__ game, int n_env,
                                                 const uint8_t *__restrict__ active) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.n) return;
  int32_t *cnt = m.counts + (size_t)b * 4;
  bool act = !active || active[b];
  if (!act) {
    m.leaf[b] = -1;
    m.leaf_gidx[b] = -1;
    cnt[0] = 0;
    cnt[1] = 0;
    return;
  }
  State s = load_state(game, n_env, b);
  size_t nb = (size_t)b * m.max_nodes;
  store_node(m.node_state + nb * 6, s);
  CKey key = canon_key(s, !m.exact_keys);
  uint64_t h = key_hash(key);
#pragma unroll
  for (int w = 0; w < 8; w++) m.node_key[nb * 8 + w] = key.w[w];
  m.node_e0[nb] = 0;
  m.node_ne[nb] = 0;
  int gen = cnt[2] + 1;
  cnt[0] = 1;
  cnt[1] = 0;
  cnt[2] = gen;
  cnt[3] = 0;
  uint64_t *ht = m.ht + (size_t)b * m.hcap;
  ht[h & (uint64_t)(m.hcap - 1)] = ht_entry(gen, 0);
}

// ------------------------------------------------------------------ select
// move_to_leaf (MCTS.py:63-149).  Per node: U = cpuct*P*sqrt(max(1,sum N))/(1+N)
// with NumPy promotion: cpuct*P in float32, the rest float64; Q = W/N
// (0 while N == 0); the first edge (insertion = ascending action order)
// with the largest Q+U by strict '>' wins.
// The walk reads each level's edges with their hints (the child's first
// edge and edge count): one dependent memory round trip per level.  A hint
// with ne = 0 (the child was unexpanded when the edge was written, or is a
// transposition target expanded through another parent since) is checked
// against the node and repaired; a terminal child (never expanded) needs no
// check.
constexpr int kHintNe = 127, kHintTerm = 128;
// Wave reductions of the walk: within each row of 16 lanes by DPP moves (a
// VALU operand modifier: quad_perm xor 1, xor 2, then row_ror 4, 8), across
// the four rows by two ds_bpermute rounds (xor 16, 32): 2 LDS-crossbar
// round trips per reduction instead of 6.  Every lane ends with the result.
template <int Ctrl>
__device__ __forceinline__ int dpp_mov(int v) {
  return __builtin_amdgcn_update_dpp(0, v, Ctrl, 0xf, 0xf, false);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppRor4 = 0x124, kDppRor8 = 0x128;
__device__ __forceinline__ int wave_sum_i(int v) {
  v += dpp_mov<kDppXor1>(v);
  v += dpp_mov<kDppXor2>(v);
  v += dpp_mov<kDppRor4>(v);
  v += dpp_mov<kDppRor8>(v);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
// (value, index): the largest value, the smallest index among equal values
// (MCTS.py:102-121's first strict '>' in insertion order); associative and
// commutative, so the reduction order does not change the result
__device__ __forceinline__ void argmax_take(double ob, int oi, double &best, int &bi) {
  if (ob > best || (ob == best && oi < bi)) {
    best = ob;
    bi = oi;
  }
}
template <int Ctrl>
__device__ __forceinline__ void argmax_dpp(double &best, int &bi) {
  const long long b = __double_as_longlong(best);
  const int lo = dpp_mov<Ctrl>((int)b), hi = dpp_mov<Ctrl>((int)(b >> 32)), oi = dpp_mov<Ctrl>(bi);
  argmax_take(__longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo)), oi, best,
              bi);
}
__device__ __forceinline__ void wave_argmax(double &best, int &bi) {
  argmax_dpp<kDppXor1>(best, bi);
  argmax_dpp<kDppXor2>(best, bi);
  argmax_dpp<kDppRor4>(best, bi);
  argmax_dpp<kDppRor8>(best, bi);
#pragma unroll
  for (int o = 16; o < kWave; o <<= 1) argmax_take(__shfl_xor(best, o), __shfl_xor(bi, o), best, bi);
}
// edge_hint = first edge << 8 | terminal << 7 | edge count: the first edge
// must fit in 24 bits, so hz_mcts_create refuses max_nodes >= kMaxNodesHint
constexpr int32_t kMaxNodesHint = 1 << 24;
__device__ __forceinline__ int32_t edge_hint_of(int e0, int ne, bool term) {
  return (int32_t)((uint32_t)e0 << 8 | (term ? (uint32_t)kHintTerm : 0u) | (uint32_t)ne);
}
// Fresh: the edges' N and W are read past the CU's L1 (relaxed agent-scope
// loads), for a walk in the launch whose backup just added to them at L2
// Returns the leaf's encoder index (b * max_nodes + leaf, wave-uniform), -1
// when the board is inactive or its leaf is terminal (no network row)
template <bool Fresh = false>
__device__ __forceinline__ int select_board(const hz_mcts &m, int b, int lane, const uint8_t *__restrict__ active,
                                            float cpuct) {
  int32_t *cnt = m.counts + (size_t)b * 4;
  size_t nb = (size_t)b * m.max_nodes, eb = (size_t)b * m.max_edges;
  // the board's flags and its root's edges in one memory round trip (the
  // root's words are in bounds whether or not the board has a tree)
  const bool act = !active || active[b];
  const int n_nodes = cnt[0];
  int ne = m.node_ne[nb], e0 = m.node_e0[nb];  // the root
  if (!act || n_nodes == 0) {
    if (lane == 0) {
      m.leaf[b] = -1;
      m.leaf_gidx[b] = -1;
    }
    return -1;
  }
  int node = 0, d = 0;
  int32_t *path = m.path + (size_t)b * m.max_depth;
  bool term = false;                           // an active board's root is not terminal
  bool known = true;                           // ne came from the node itself
  for (;;) {
    if (ne <= 0) {
      if (known || term) break;
      // the hint says unexpanded: the node decides (and the hint is repaired)
      ne = m.node_ne[nb + node];
      e0 = m.node_e0[nb + node];
      if (ne <= 0) break;
      if (lane == 0) m.edge_hint[eb + path[d - 1]] = edge_hint_of(e0, ne, false);
    }
    int n0 = 0, n1 = 0, c0 = 0, c1 = 0, h0 = 0, h1 = 0;
    double w0 = 0, w1 = 0;
    float p0 = 0, p1 = 0;
    // each edge's child and hint are read with its statistics (one memory
    // round trip per level)
    auto ld_n = [&](size_t e) {
      return Fresh ? __hip_atomic_load(&m.edge_n[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : m.edge_n[e];
    };
    auto ld_w = [&](size_t e) {
      return Fresh ? __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(&m.edge_w[e]),
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                   : m.edge_w[e];
    };
    if (lane < ne) {
      n0 = ld_n(eb + e0 + lane);
      w0 = ld_w(eb + e0 + lane);
      p0 = m.edge_p[eb + e0 + lane];
      c0 = m.edge_child[eb + e0 + lane];
      h0 = m.edge_hint[eb + e0 + lane];
    }
    if (lane + kWave < ne) {
      n1 = ld_n(eb + e0 + lane + kWave);
      w1 = ld_w(eb + e0 + lane + kWave);
      p1 = m.edge_p[eb + e0 + lane + kWave];
      c1 = m.edge_child[eb + e0 + lane + kWave];
      h1 = m.edge_hint[eb + e0 + lane + kWave];
    }
    const int ns = wave_sum_i(n0 + n1);
    double sqrt_ns = __dsqrt_rn(ns > 1 ? (double)ns : 1.0);
    double best = -INFINITY;
    int bi = 0x7fffffff;
    if (lane < ne) {
      double u = __ddiv_rn(__dmul_rn((double)__fmul_rn(cpuct, p0), sqrt_ns), (double)(1 + n0));
      double q = n0 ? __ddiv_rn(w0, (double)n0) : 0.0;
      best = __dadd_rn(q, u);
      bi = lane;
    }
    if (lane + kWave < ne) {
      double u = __ddiv_rn(__dmul_rn((double)__fmul_rn(cpuct, p1), sqrt_ns), (double)(1 + n1));
      double q = n1 ? __ddiv_rn(w1, (double)n1) : 0.0;
      double v = __dadd_rn(q, u);
      if (v > best) { best = v; bi = lane + kWave; }
    }
    wave_argmax(best, bi);
    int sel = e0 + bi;
    if (d >= m.max_depth) {
      if (lane == 0) cnt[3] = 1;
      break;
    }
    if (lane == 0) path[d] = sel;
    d++;
    const int src = bi & (kWave - 1);
    node = __shfl(bi < kWave ? c0 : c1, src);  // edge_child[sel], from the winner's lane
    const int hint = __shfl(bi < kWave ? h0 : h1, src);
    ne = hint & kHintNe;
    e0 = (int)((uint32_t)hint >> 8);
    term = (hint & kHintTerm) != 0;
    known = false;
  }
  if (d == 0) term = game_done(m.node_state[(nb + node) * 6 + 5]);
  const int gidx = term ? -1 : (int)(nb + node);
  if (lane == 0) {
    m.leaf[b] = node;
    m.depth[b] = d;
    m.leaf_gidx[b] = gidx;
  }
  return gidx;
}

__global__ void __launch_bounds__(kWave) k_select(hz_mcts m, const uint8_t *__restrict__ active, float cpuct) {
  select_board(m, blockIdx.x, threadIdx.x, active, cpuct);
}

// ------------------------------------------------------------ gather leaves
// The boards whose selected leaf needs the network (active, not terminal:
// MCTS.py:297-341 never calls predict on a terminal leaf), in board order:
// rows[j] = board of gathered row j, slot[b] = j (or -1), count[0] = rows.
// One workgroup; thread t owns boards [t*per, (t+1)*per) (contiguous, so the
// exclusive scan of the per-thread counts keeps board order).
constexpr int kGatherThreads = 1024;
__global__ void __launch_bounds__(kGatherThreads) k_gather(hz_mcts m, int32_t *__restrict__ rows,
                                                           int32_t *__restrict__ count) {
  __shared__ int32_t part[kGatherThreads];
  const int t = threadIdx.x;
  const int per = (m.n + kGatherThreads - 1) / kGatherThreads;
  const int b0 = t * per < m.n ? t * per : m.n, b1 = b0 + per < m.n ? b0 + per : m.n;
  int c = 0;
  for (int b = b0; b < b1; b++) c += m.leaf_gidx[b] >= 0;
  part[t] = c;
  __syncthreads();
  for (int o = 1; o < kGatherThreads; o <<= 1) {
    int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int j = part[t] - c;
  for (int b = b0; b < b1; b++) {
    int g = m.leaf_gidx[b];
    if (g >= 0) {
      m.slot[b] = j;
      m.gidx_c[j] = g;
      if (rows) rows[j] = b;
      j++;
    } else {
      m.slot[b] = -1;
    }
  }
  if (t == kGatherThreads - 1) {
    count[0] = part[t];
    if (m.eval_ctr) m.eval_ctr[0] += part[t];  // one workgroup, stream-ordered: no atomic needed
  }
}

// ------------------------------------------------- gather + encode, one launch
// k_gather's result and both encoders in one launch for any batch: every
// workgroup owns leaf rows [8 g, 8 g + 8) (a pair per wave) and finds their
// boards itself: it scans all n leaf flags (thread t: boards [t per, (t + 1)
// per), per = ceil(n / 256); 16 KB of L2 reads per workgroup at 4096 boards),
// so no workgroup waits for another and there is no separate gather launch
// (k_gather: 7 us of one 1024-thread workgroup, then two encoder launches).
// Rows, slots, gidx_c and the count are exactly k_gather's (board order);
// workgroup 0 writes the count, the eval counter and the slots of the boards
// that need no network.
// 8 waves (16 rows) per workgroup: 14.3 us per sim step at 4096 boards against 16.0 with 4 and 16.4 with 16
// (profiles/r04/tree/r4p_ge*): fewer workgroups scan the flags, the encoders keep 2048 waves
constexpr int kGEWaves = 8, kGERows = 2 * kGEWaves, kGEThreads = kGEWaves * kWave, kGELoads = 16;
constexpr int kBoardFloats = 38 * 35, kGlobFloats = 42;  // one encoded state (hz_encode.hpp)
__global__ void __launch_bounds__(kGEThreads) k_gather_encode(hz_mcts m, int32_t *__restrict__ rows,
                                                               int32_t *__restrict__ count,
                                                               float *__restrict__ board, float *__restrict__ glob) {
  __shared__ uint64_t smask[kGEWaves][76];
  __shared__ float sval[kGEWaves][76];
  __shared__ int32_t wsum[kGEWaves];
  __shared__ int32_t s_gidx[kGERows];  // this workgroup's rows' leaves (gidx_c's entries), for its encoder waves
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int per = (m.n + kGEThreads - 1) / kGEThreads;
  const int b0 = t * per < m.n ? t * per : m.n, b1 = b0 + per < m.n ? b0 + per : m.n;
  const int r0 = (int)blockIdx.x * kGERows;
  // up to 4096 boards (per <= kGELoads) the thread's leaf flags stay in
  // registers from the count to the row assignment: one round trip, not two
  const bool one = per <= kGELoads;
  int gk[kGELoads];
  int c = 0;
  if (one) {
#pragma unroll
    for (int k = 0; k < kGELoads; k++) gk[k] = b0 + k < b1 ? m.leaf_gidx[b0 + k] : -1;
#pragma unroll
    for (int k = 0; k < kGELoads; k++) c += gk[k] >= 0;
  } else {
    for (int base = b0; base < b1; base += kGELoads) {  // all of a pass's loads in flight
      int g[kGELoads];
#pragma unroll
      for (int k = 0; k < kGELoads; k++) g[k] = base + k < b1 ? m.leaf_gidx[base + k] : -1;
#pragma unroll
      for (int k = 0; k < kGELoads; k++) c += g[k] >= 0;
    }
  }
  // exclusive prefix of the per-thread counts: wave scan, then the waves' totals
  int incl = c;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  int before = 0, total = 0;
#pragma unroll
  for (int k = 0; k < kGEWaves; k++) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  int r = before + incl - c;  // rank of the thread's first needed board
  const bool first = blockIdx.x == 0;
  auto assign = [&](int b, int g) {
    if (g >= 0) {
      if (r >= r0 && r < r0 + kGERows) {
        m.slot[b] = r;
        m.gidx_c[r] = g;
        s_gidx[r - r0] = g;
        if (rows) rows[r] = b;
      }
      r++;
    } else if (first) {
      m.slot[b] = -1;
    }
  };
  if (first || (r < r0 + kGERows && r + c > r0)) {
    if (one) {
#pragma unroll
      for (int k = 0; k < kGELoads; k++)
        if (b0 + k < b1) assign(b0 + k, gk[k]);
    } else {
      for (int b = b0; b < b1; b++) assign(b, m.leaf_gidx[b]);
    }
  }
  if (first && t == 0) {
    count[0] = total;
    if (m.eval_ctr) m.eval_ctr[0] += total;  // one thread of one workgroup, stream-ordered
  }
  if (r0 >= total) return;
  __syncthreads();  // s_gidx complete
  // the workgroup's rows from 0: its leaves from LDS, its outputs from row r0
  encode_pair<true>(m.node_state, 1, 6, s_gidx, total - r0, board + (size_t)r0 * kBoardFloats,
                    glob + (size_t)r0 * kGlobFloats, lane, 2 * w, smask[w], sval[w]);
}

// --------------------------------- select + gather + encode for small batches
// At most kFusedMax boards (config 1's one-board searches, the arena's few
// dozen games): one workgroup runs move_to_leaf for every board (wave per
// board), gathers the leaves that need the network (one wave's ballot
// prefix: board order kept) and encodes them (wave per pair of rows), so a
// simulation's tree side before the network is one launch instead of three
// (each a few us of launch latency at this size).  Same results as
// k_select + k_gather + the encoder.
constexpr int kFusedMax = 32;
constexpr int kFusedWaves = 16;
static_assert(kFusedMax <= 2 * kFusedWaves && kFusedMax <= kWave, "one pair per wave, one gather wave");
__global__ void __launch_bounds__(kFusedWaves * kWave) k_select_gather_encode(hz_mcts m,
                                                                           const uint8_t *__restrict__ active,
                                                                           float cpuct, int32_t *__restrict__ rows,
                                                                           int32_t *__restrict__ count,
                                                                           float *__restrict__ board,
                                                                           float *__restrict__ glob) {
  __shared__ uint64_t smask[kFusedWaves][76];
  __shared__ float sval[kFusedWaves][76];
  __shared__ int32_t s_count;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int b = w; b < m.n; b += kFusedWaves) select_board(m, b, lane, active, cpuct);
  __syncthreads();  // every board's leaf_gidx (written by its wave) is visible to the workgroup
  if (w == 0) {
    const int g = lane < m.n ? m.leaf_gidx[lane] : -1;
    const uint64_t need = __ballot(g >= 0);
    const int j = __popcll(need & ((1ull << lane) - 1));
    if (lane < m.n) {
      m.slot[lane] = g >= 0 ? j : -1;
      if (g >= 0) {
        m.gidx_c[j] = g;
        if (rows) rows[j] = lane;
      }
    }
    if (lane == 0) {
      const int c = __popcll(need);
      count[0] = c;
      s_count = c;
      if (m.eval_ctr) m.eval_ctr[0] += c;
    }
  }
  __syncthreads();
  encode_pair<true>(m.node_state, 1, 6, m.gidx_c, s_count, board, glob, lane, 2 * w, smask[w], sval[w]);
}

// ------------------------------------------------ turn-end chance, in parallel
// At a turn end (phase place_tile_3) every child of the leaf refills the one
// missing pile from the same bag: _draw_tiles(3) = random.sample(range(n), 3)
// over the same flat bag (harmonies_engine.py:120-137), child after child on
// the board's stream (MCTS.py:171-176).  Only the stream position couples the
// children.  With n > 21 (random.py's set method: every pick is
// _randbelow(n), a repeat of the child's own earlier pick is drawn again),
// the wave produces 64 tempered words at a time (twisting the generation in
// place 64 words at a time: a block's sources are either old words beyond
// it or new words before it), each lane tests its word against n and the
// accepted values are appended, in stream order, to an LDS list.  The list
// is then cut into the children's picks speculatively: lane k takes child
// c + k's three picks as list entries s + 3k .. s + 3k + 2, which is right
// for every child before the first whose triple holds a repeat (or runs past
// the list); that child is resolved serially (skipping its repeats), and the
// cut resumes after it.  A window therefore costs one parallel step per
// repeat (~5 % of triples) instead of a serial step per pick.  Returns the
// stream cursor (pos | tw << 16, as MTS) after the last child's third pick;
// script[c] = the pile the c-th child draws, as replenish() records it.
constexpr int kAccRing = 512;  // accepted-value ring (entries in flight: < 64 + 3)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int turn_end_draws_parallel(uint32_t *w, int cursor, uint64_t misc, int nl, int lane,
                                                       uint64_t *script, uint32_t *acc) {
  int cnt[6];
  uint32_t n = 0;
#pragma unroll
  for (int t = 0; t < 6; t++) {
    cnt[t] = bag_n(misc, t);
    n += (uint32_t)cnt[t];
  }
  // flat bag index -> tile (insertion order water, plant, wood, stone,
  // field, building: constants.py:41); three picks -> the pile's script
  constexpr uint32_t kOrder = WATER | (PLANT << 3) | (WOOD << 6) | (STONE << 9) | (FIELD << 12) | (BUILDING << 15);
  const uint32_t e0 = (uint32_t)cnt[WATER], e1 = e0 + (uint32_t)cnt[PLANT], e2 = e1 + (uint32_t)cnt[WOOD];
  const uint32_t e3 = e2 + (uint32_t)cnt[STONE], e4 = e3 + (uint32_t)cnt[FIELD];
  auto tile = [&](uint32_t x) {
    const uint32_t o = (uint32_t)(x >= e0) + (uint32_t)(x >= e1) + (uint32_t)(x >= e2) + (uint32_t)(x >= e3) +
                       (uint32_t)(x >= e4);
    return (uint64_t)__builtin_amdgcn_ubfe(kOrder, 3 * o, 3);
  };
  auto pile = [&](uint32_t a, uint32_t b, uint32_t c) {
    return (((1ull << 45) - 1) & ~0x1FFull) | tile(a) | tile(b) << 3 | tile(c) << 6;
  };
  const int kb = 32 - __clz(n);
  int pos = cursor & 0xFFFF, tw = cursor >> 16;
  int c = 0;      // next child to resolve (wave-uniform)
  int s = 0;      // its first list entry
  int k_end = 0;  // list length
  for (;;) {
    if (pos >= kMT) {  // next generation
      pos = 0;
      tw = 0;
    }
    const int need = pos + kWave < kMT ? pos + kWave : kMT;
    while (tw < need) {  // twist [tw, tw + 64) of the current generation
      const int i = tw + lane;
      uint32_t nw = 0;
      if (i < kMT) {
        const uint32_t cur = w[i], nxt = w[i + 1 < kMT ? i + 1 : 0];
        const uint32_t far = w[i < 227 ? i + 397 : (i < 623 ? i - 227 : 396)];
        nw = twist_word(cur, nxt, far);
      }
      __builtin_amdgcn_wave_barrier();  // every lane has read before any writes
      if (i < kMT) w[i] = nw;
      __builtin_amdgcn_wave_barrier();
      tw = tw + kWave < kMT ? tw + kWave : kMT;
    }
    {  // append this window's accepted values (value | window offset << 16)
      const int i = pos + lane;
      const uint32_t r = i < kMT ? temper(w[i]) >> (32 - kb) : n;
      const uint64_t ok = __ballot(r < n);
      if (r < n) acc[(k_end + __popcll(ok & ((1ull << lane) - 1))) & (kAccRing - 1)] = r | (uint32_t)lane << 16;
      k_end += __popcll(ok);
      wave_lds_sync();
    }
    int last = -1;  // window offset of the word that completed the last child
    for (;;) {
      // speculative cut: lane k -> child c + k, entries s + 3k .. s + 3k + 2
      const int ck = c + lane, sk = s + 3 * lane;
      bool good = false;
      uint32_t a0 = 0, a1 = 0, a2 = 0;
      if (ck < nl && sk + 2 < k_end) {
        a0 = acc[sk & (kAccRing - 1)] & 0xFFFFu;
        a1 = acc[(sk + 1) & (kAccRing - 1)] & 0xFFFFu;
        a2 = acc[(sk + 2) & (kAccRing - 1)] & 0xFFFFu;
        good = a1 != a0 && a2 != a0 && a2 != a1;
      }
      const uint64_t bad = ~__ballot(good);
      const int f = bad ? __builtin_ctzll(bad) : kWave;  // children c .. c + f - 1 are cut right
      if (lane < f) script[ck] = pile(a0, a1, a2);
      c += f;
      s += 3 * f;
      if (f > 0 && c >= nl) {
        last = (int)(acc[(s - 1) & (kAccRing - 1)] >> 16);
        break;
      }
      if (f == kWave) continue;
      // child c: a repeat among its first three entries, or the list ends:
      // serially, as random.sample draws (wave-uniform values)
      uint32_t j0 = 0, j1 = 0, v = 0;
      int got = 0, e = s;
      while (got < 3 && e < k_end) {
        v = __builtin_amdgcn_readfirstlane(acc[e & (kAccRing - 1)]) & 0xFFFFu;
        e++;
        if ((got >= 1 && v == j0) || (got >= 2 && v == j1)) continue;  // repeat: drawn again
        if (got == 0) j0 = v;
        else if (got == 1) j1 = v;
        got++;
      }
      if (got < 3) break;  // the list ends inside child c: next window
      if (lane == 0) script[c] = pile(j0, j1, v);
      c++;
      s = e;
      if (c >= nl) {
        last = (int)(acc[(s - 1) & (kAccRing - 1)] >> 16);
        break;
      }
    }
    if (last >= 0) {
      pos += last + 1;
      break;
    }
    pos = need;
  }
  wave_lds_sync();  // lane 0's script entries before the children read them
  return pos | (tw << 16);
}

// ---------------------------------------------------------- expand + backup
#ifdef HZ_DIAG
// diagnostic build only (tools/expand_phases.py): per board, s_memtime at the
// phase boundaries of k_expand_backup + flags; written to this buffer alone,
// by the fused launches only (Sel: the search's simulations 1..S-1), so the
// buffer holds the last fused launch's stamps; slots 12-14: after the next
// simulation's select, after its leaf's encode, after the row-slot barriers
__device__ uint64_t g_exp_stamps[16384][16];
// one asm statement fenced by scheduling barriers, so the stamp stays where it
// is written (cdna_hip_programming.md §7, in-kernel stamps)
__device__ __forceinline__ uint64_t xstamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define HZ_XSTAMP(k) \
  {                                                          \
    const uint64_t t_ = xstamp();                            \
    if (dg && lane == 0 && b < 16384) g_exp_stamps[b][k] = t_; \
  }
#define HZ_XFLAG(k, v) \
  if (dg && lane == 0 && b < 16384) g_exp_stamps[b][k] = (uint64_t)(v);
#else
#define HZ_XSTAMP(k)
#define HZ_XFLAG(k, v)
#endif
#ifdef HZ_KEYCHECK
// diagnostic build only (tools/Makefile libhz_kc.so): children whose key
// differs from canon_key of their state, leaves whose stored key differs from
// canon_key of their stored state, children checked
__device__ unsigned long long g_kc[3];
#endif
static_assert(kChildLds >= kMaxChildren, "child arrays hold every legal move");
// 9.8 KB (was 12.3 KB, 19.5 KB before that): 16 waves fit a CU.  The turn-end
// stream copy and the children's states share their bytes (the stream is
// written back before the first child state is stored); the sibling-dedup
// table shares the chance scripts' (read by the children only).  The children's keys stay in LDS:
// rebuilding a key from the child's state at each hash match instead (most
// children of a placement meet an existing node: tile orders transpose)
// made the kernel 3x slower (209 vs 64 us per sim step, profiles/r03).
struct ExpandLds {
  union {
    uint32_t mt[kMT];
    uint64_t state[kChildLds][6];
  };
  union {
    uint64_t script[kChildLds];
    // sibling dedup: open addressing, slot word = (hash tag << 8) | lowest child index
    uint32_t dslot[kDedupSlots];
  };
  union {
    uint64_t key[kChildLds][8];
    uint32_t acc[kAccRing];  // turn-end draws' accepted values (before any key is built)
  };
  uint64_t hash[kChildLds];
  int32_t child[kChildLds];
  int32_t flag[kChildLds];  // 0 new, 1 existing node, 2 self-loop (skipped), 3 sibling duplicate
  float prior[kChildLds];   // the children's priors (policy row, by action)
};
static_assert(kDedupSlots * sizeof(uint32_t) <= kChildLds * sizeof(uint64_t), "the dedup table fits the scripts");
static_assert(kDedupSlots > kMaxChildren && kChildLds <= 256, "a free slot for every child, 8-bit child index");
static_assert(sizeof(uint64_t) * kChildLds * 6 >= sizeof(uint32_t) * kMT, "the states cover the stream copy");


// expand_leaf (MCTS.py:151-218) + back_fill (:220-266) + the root Dirichlet
// mix (:308-327).  noise[b*69 + i] is the i-th legal move's Dirichlet sample.
// (board b, one wave; the kernel below adds the next simulation's select)
__device__ __forceinline__ void expand_backup_board(ExpandLds &L, const hz_mcts &m, uint32_t *__restrict__ mtw,
                                                    int32_t *__restrict__ mtcur, const float *__restrict__ policy,
                                                    const float *__restrict__ value,
                                                    const double *__restrict__ noise, double eps,
                                                    float one_minus_eps, int testing,
                                                    const int32_t *__restrict__ row_of, int prio, int b, int lane,
                                                    bool dg) {
  (void)dg;  // (HZ_DIAG: stamp this launch)
  HZ_XSTAMP(0)
  HZ_XFLAG(10, 0)
  int leaf = m.leaf[b];
  const int d = m.depth[b];
  if (leaf < 0) return;
  int32_t *cnt = m.counts + (size_t)b * 4;
  size_t nb = (size_t)b * m.max_nodes, eb = (size_t)b * m.max_edges;
  const int32_t *path = m.path + (size_t)b * m.max_depth;
  // the edge into the leaf: its hint gets the leaf's edges once expanded
  // (loaded now, used at the end)
  const int in_edge = d > 0 ? path[d - 1] : -1;
  State ls = load_node(m.node_state + (nb + leaf) * 6);
  // the leaf's stored key (same round trip): its children's keys are built
  // from it (canon_key_child); wave-uniform, moved to scalar registers where
  // the children start (the wait for these loads is not taken before then)
  uint64_t lkv[8];
  {
    const uint64_t *lkp = m.node_key + (nb + leaf) * 8;
#pragma unroll
    for (int w = 0; w < 8; w++) lkv[w] = lkp[w];
  }
  const int leaf_ne = m.node_ne[nb + leaf];  // (same round trip) 0: not expanded yet
  int leaf_player = player_of(ls.misc);
  // policy/value row of this board: its own (per-board batch) or its row in
  // the gathered batch (hz_mcts_gather_leaves)
  const size_t row = (size_t)__builtin_amdgcn_readfirstlane(row_of ? row_of[b] : b);
  double v;
  if (game_done(ls.misc)) {
    // MCTS.py:333-341: outcome from the leaf player's perspective
    int wc = winner_code(ls.misc);
    double outcome = wc == 1 ? 1.0 : wc == 2 ? -1.0 : 0.0;
    v = (wc == 3) ? 0.0 : (leaf_player == 0 ? outcome : -outcome);
  } else {
    v = (double)value[row];
    uint64_t mk[3];
    int nl = legal_mask(ls, mk);
    bool noisy = leaf == 0 && !testing && noise;
    HZ_XSTAMP(1)
    if (nl > 0 && nl <= kMaxChildren && leaf_ne == 0) {
      bool turn_end = phase_of(ls.misc) == PH_P3;
      // the children's actions and priors (lane's c = lane, lane + 64): the
      // policy row is read now, its latency under the chance replay and the
      // rule work of the first child
      int cact[2];
      float cpri[2];
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const int c = lane + r * kWave;
        cact[r] = c < nl ? kth_action(mk, c) : 0;
        cpri[r] = c < nl ? policy[row * kActions + cact[r]] : 0.f;
      }
      // the launch lasts as long as its slowest waves, the turn-end
      // expansions (chance replay + ~21 children: ~58 k cycles median against
      // ~41 k for the others, profiles/r03/expand_phases_spec_draws.json);
      // they take issue priority over the three other waves of their SIMD
      if (turn_end && prio) __builtin_amdgcn_s_setprio(2);
      HZ_XFLAG(10, 1 | (turn_end ? 2 : 0) | (nl << 8))
      if (turn_end) {
        // the children's _end_turn_actions draw from the board's stream in
        // child order (MCTS.py:171-176): replay that sequence once, serially,
        // on an LDS copy of the stream
        uint32_t *g = mtw + (size_t)b * kMT;
        {  // all ten of the lane's words in flight at once (one memory round trip)
          uint32_t v[(kMT + kWave - 1) / kWave];
#pragma unroll
          for (int k = 0; k < (kMT + kWave - 1) / kWave; k++) {
            const int i = lane + kWave * k;
            v[k] = i < kMT ? g[i] : 0u;
          }
#pragma unroll
          for (int k = 0; k < (kMT + kWave - 1) / kWave; k++) {
            const int i = lane + kWave * k;
            if (i < kMT) L.mt[i] = v[k];
          }
        }
        wave_lds_sync();
        HZ_XSTAMP(8)
        int bag = 0;
#pragma unroll
        for (int t = 0; t < 6; t++) bag += bag_n(ls.misc, t);
        if (npiles_of(ls.piles) == 4 && bag > 21) {
          // one pile per child, random.sample's set method: the wave-parallel form
          const int cur = turn_end_draws_parallel(L.mt, mtcur[b], ls.misc, nl, lane, L.script, L.acc);
          if (lane == 0) mtcur[b] = cur;
        } else if (lane == 0) {  // fewer piles or the pool method: one lane, serially
          StreamDraw<MT> draw{MT(L.mt, mtcur[b])};
          for (int c = 0; c < nl; c++) {
            State tmp = ls;
            L.script[c] = replenish(tmp, draw);
          }
          mtcur[b] = draw.m.cursor();
        }
        wave_lds_sync();
        HZ_XSTAMP(9)
        for (int i = lane; i < kMT; i += kWave) g[i] = L.mt[i];  // stores: no round trip to wait for
        wave_lds_sync();  // the stream copy is read before the children's states overwrite it
      }
      HZ_XSTAMP(2)
      CKey lk;
#pragma unroll
      for (int w = 0; w < 8; w++)
        lk.w[w] = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(lkv[w] >> 32)) << 32 |
                  (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)lkv[w]);
      // children: lane handles child c = lane and lane + 64 (one at a time:
      // the rule work of two children at once held 38 more registers than fit)
#pragma unroll 1
      for (int r = 0; r < 2; r++) {
        const int c = lane + r * kWave;
        if (c < nl) {
          const int a = r == 0 ? cact[0] : cact[1];
          L.prior[c] = r == 0 ? cpri[0] : cpri[1];
          State ch = ls;
          ScriptDraw sd{turn_end ? L.script[c] : ~0ull};
          step_state(ch, a, sd);
          CKey k = canon_key_child(lk, ls, ch, a, !m.exact_keys);
#ifdef HZ_KEYCHECK
          {
            const CKey want = canon_key(ch, !m.exact_keys), lw = canon_key(ls, !m.exact_keys);
            if (!key_eq(want, k)) atomicAdd(&g_kc[0], 1ull);
            if (!key_eq(lw, lk)) atomicAdd(&g_kc[1], 1ull);
            atomicAdd(&g_kc[2], 1ull);
          }
#endif
#pragma unroll
          for (int w = 0; w < 8; w++) L.key[c][w] = k.w[w];
#pragma unroll
          for (int w = 0; w < 4; w++) L.state[c][w] = ch.pl[w];
          L.state[c][4] = ch.piles;
          L.state[c][5] = ch.misc;
          L.hash[c] = key_hash(k);
          L.child[c] = -1;
          L.flag[c] = 0;
        }
      }
      wave_lds_sync();
      HZ_XSTAMP(3)
      // the board's counters (written by this wave alone, at the end); loaded
      // after the children's rule work, whose registers they would have held
      const int gen = __builtin_amdgcn_readfirstlane(cnt[2]), base_n = __builtin_amdgcn_readfirstlane(cnt[0]),
                base_e = __builtin_amdgcn_readfirstlane(cnt[1]);
      // transpositions (MCTS.py:177-204): a child whose key is already in the
      // tree reuses that node (flag 1), or is skipped if it is the leaf itself
      // (flag 2) ...
      for (int s = lane; s < kDedupSlots; s += kWave) L.dslot[s] = 0u;  // empty (no entry is 0, see below)
      uint64_t *ht = m.ht + (size_t)b * m.hcap;
      uint64_t hmask = (uint64_t)(m.hcap - 1);
      // the free slot each probe ended on and the word it held: a new child's
      // insertion (below) swaps its entry in there with one atomic, instead
      // of reloading the slot first (a sibling may have taken it meanwhile:
      // the swap then fails and the insertion probes on)
      uint32_t fslot[2] = {0u, 0u};
      uint64_t fold[2] = {0ull, 0ull};
      // the lane's two children (c = lane, lane + 64) probe in lockstep, so
      // a wide expansion's second child adds no chain of round trips of its
      // own: each step loads both table words, then both candidates' keys
      uint64_t pslot[2];
      bool open[2];
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const int c = lane + r * kWave;
        open[r] = c < nl;
        pslot[r] = open[r] ? L.hash[c] & hmask : 0;
      }
      while (open[0] || open[1]) {
        uint64_t e[2] = {0ull, 0ull};
#pragma unroll
        for (int r = 0; r < 2; r++)
          if (open[r]) e[r] = ht[pslot[r]];
        bool cand[2];
#pragma unroll
        for (int r = 0; r < 2; r++) {
          cand[r] = open[r] && (int)(e[r] >> 32) == gen;
          if (open[r] && !cand[r]) {  // a free slot: the child is not in the tree
            fslot[r] = (uint32_t)pslot[r];
            fold[r] = e[r];
            open[r] = false;
          }
        }
        // the candidate nodes' stored canonical keys against the children's
        // (one memory round trip after the table's; no key is rebuilt from a
        // state), with their edges and terminal marks
        uint64_t nk[2][8];
        int nne[2] = {0, 0}, ne0[2] = {0, 0};
#pragma unroll
        for (int r = 0; r < 2; r++) {
          if (cand[r]) {
            const int nid = (int)(uint32_t)e[r];
            const uint64_t *kp = m.node_key + (nb + nid) * 8;
#pragma unroll
            for (int w = 0; w < 8; w++) nk[r][w] = kp[w];
            nne[r] = m.node_ne[nb + nid];
            ne0[r] = m.node_e0[nb + nid];
          }
        }
#pragma unroll
        for (int r = 0; r < 2; r++) {
          if (!cand[r]) continue;
          const int c = lane + r * kWave, nid = (int)(uint32_t)e[r];
          bool eq = true;
#pragma unroll
          for (int w = 0; w < 8; w++) eq = eq && nk[r][w] == L.key[c][w];
          if (eq) {
            L.flag[c] = nid == leaf ? 2 : 1;
            L.child[c] = nid;
            // the edge's hint: the node's own edges and terminal mark (its
            // stored state decides, as the reference's Node does: equal keys
            // do not imply equal game_over); kept in the child's hash word,
            // which only new children read from here on
            L.hash[c] = (uint64_t)(uint32_t)edge_hint_of(nne[r] > 0 ? ne0[r] : 0, nne[r] > 0 ? nne[r] : 0,
                                                         nne[r] < 0);
            open[r] = false;
          } else {
            pslot[r] = (pslot[r] + 1) & hmask;
          }
        }
      }
      wave_lds_sync();
      HZ_XSTAMP(4)
      // ... and among the remaining children the first of equal keys creates
      // the node, later siblings reuse it (flag 3: child[c] = that sibling;
      // a target is never itself a duplicate: it has no earlier equal sibling).
      // Every new child enters its hash into an LDS open-addressing table:
      // home slot = hash bits 32-38, tag = bits 40-62 with bit 23 set (so no
      // entry is 0, the empty word); the slot word keeps tag << 8 | the lowest
      // child index of that tag (atomicMin over words of one tag).  Equal
      // keys have equal hashes, so when the slot's lowest index f < c holds
      // c's key, f is the first of c's equal siblings.  When f's key differs
      // (hashes equal in those 30 bits only) the lane is unresolved and the
      // serial walk below decides it; it runs only if some lane needs it.
      // (The walk alone cost up to ~30k cycles at 60+ children, profiles/r02.)
      {
        const int c0 = lane, c1 = lane + kWave;
        const bool new0 = c0 < nl && L.flag[c0] == 0, new1 = c1 < nl && L.flag[c1] == 0;
        const uint64_t h0 = new0 ? L.hash[c0] : 0, h1 = new1 ? L.hash[c1] : 0;
        auto enter = [&](uint64_t h, int c) {
          const uint32_t mine = ((uint32_t)(h >> 40) | 0x800000u) << 8 | (uint32_t)c;
          for (int s = (int)(h >> 32) & (kDedupSlots - 1);; s = (s + 1) & (kDedupSlots - 1)) {
            const uint32_t prev = atomicCAS(&L.dslot[s], 0u, mine);
            if (prev == 0u) return s;
            if ((prev >> 8) == (mine >> 8)) {
              atomicMin(&L.dslot[s], mine);
              return s;
            }
          }
        };
        const int s0 = new0 ? enter(h0, c0) : 0;
        const int s1 = new1 ? enter(h1, c1) : 0;
        wave_lds_sync();
        auto same_key = [&](int f, int c) {
          bool eq = L.hash[f] == L.hash[c];
#pragma unroll
          for (int w = 0; w < 8; w++) eq = eq && L.key[f][w] == L.key[c][w];
          return eq;
        };
        int dup0 = -1, dup1 = -1;
        bool open0 = false, open1 = false;  // unresolved lanes
        if (new0) {
          const int f = (int)(L.dslot[s0] & 0xFFu);
          if (f < c0) {
            if (same_key(f, c0) && !m.dedup_walk) dup0 = f;
            else open0 = true;
          }
        }
        if (new1) {
          const int f = (int)(L.dslot[s1] & 0xFFu);
          if (f < c1) {
            if (same_key(f, c1) && !m.dedup_walk) dup1 = f;
            else open1 = true;
          }
        }
        // the serial walk for unresolved lanes: over the new children c2 in
        // ascending order, c2's hash broadcast from its lane (readlane); the
        // first c2 < c of equal key is the target
        const bool any_open = __ballot(open0 || open1) != 0ull;
        const uint64_t cand[2] = {any_open ? __ballot(new0) : 0ull, any_open ? __ballot(new1) : 0ull};
#pragma unroll
        for (int r = 0; r < 2; r++) {
          uint64_t rest = cand[r];
          while (rest) {
            const int src = __builtin_ctzll(rest);  // wave-uniform
            rest &= rest - 1;
            const int c2 = src + r * kWave;
            const uint64_t hv = r == 0 ? h0 : h1;
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)hv, src);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(hv >> 32), src);
            const uint64_t hc2 = (uint64_t)hi << 32 | lo;
            if (open0 && dup0 < 0 && c2 < c0 && h0 == hc2 && same_key(c2, c0)) dup0 = c2;
            if (open1 && dup1 < 0 && c2 < c1 && h1 == hc2 && same_key(c2, c1)) dup1 = c2;
          }
        }
        wave_lds_sync();  // every lane has read the flags before any is rewritten
        if (dup0 >= 0) {
          L.flag[c0] = 3;
          L.child[c0] = dup0;
        }
        if (dup1 >= 0) {
          L.flag[c1] = 3;
          L.child[c1] = dup1;
        }
      }
      wave_lds_sync();
      // new nodes get consecutive ids in child order; edges keep child order
      int n_new = 0, n_edges = 0;
      for (int r = 0; r < 2; r++) {
        int c = lane + r * kWave;
        bool isnew = c < nl && L.flag[c] == 0;
        bool hasedge = c < nl && L.flag[c] != 2;
        uint64_t bn = __ballot(isnew), be = __ballot(hasedge);
        uint64_t below = (1ull << lane) - 1;
        if (isnew) L.child[c] = base_n + n_new + __popcll(bn & below);
        if (hasedge) L.flag[c] |= (n_edges + __popcll(be & below)) << 4;  // edge rank
        n_new += __popcll(bn);
        n_edges += __popcll(be);
      }
      wave_lds_sync();
      HZ_XSTAMP(5)
      if (base_n + n_new > m.max_nodes || base_e + n_edges > m.max_edges) {
        if (lane == 0) cnt[3] = 1;  // capacity exhausted: leave the leaf unexpanded
      } else {
#pragma unroll
        for (int r = 0; r < 2; r++) {
          const int c = lane + r * kWave;
          if (c >= nl) continue;
          int f = L.flag[c] & 15;
          int node_id = f == 3 ? L.child[L.child[c]] : L.child[c];
          if (f == 0) {
            uint64_t *ns = m.node_state + (nb + node_id) * 6;
#pragma unroll
            for (int w = 0; w < 6; w++) ns[w] = L.state[c][w];
#pragma unroll
            for (int w = 0; w < 8; w++) m.node_key[(nb + node_id) * 8 + w] = L.key[c][w];
            m.node_e0[nb + node_id] = 0;
            m.node_ne[nb + node_id] = game_done(L.state[c][5]) ? -1 : 0;  // -1: terminal (never expanded)
            // the probe's free slot first (the word it held is the expected
            // value); a failed swap names the slot's new word: taken by a
            // sibling (this generation) -> the next slot, loaded
            uint64_t slot = fslot[r];
            unsigned long long old = fold[r];
            for (;;) {
              const unsigned long long prev =
                  atomicCAS((unsigned long long *)&ht[slot], old, (unsigned long long)ht_entry(gen, node_id));
              if (prev == old) break;
              old = prev;
              while ((int)(old >> 32) == gen) {
                slot = (slot + 1) & hmask;
                old = ht[slot];
              }
            }
          }
          if (f != 2) {
            const int a = cact[r];
            float p = L.prior[c];
            if (noisy) p = __double2float_rn(__dadd_rn((double)__fmul_rn(one_minus_eps, p),
                                                       __dmul_rn(eps, noise[(size_t)b * kMaxChildren + c])));
            int e = base_e + (L.flag[c] >> 4);
            m.edge_action[eb + e] = (int16_t)a;
            m.edge_child[eb + e] = node_id;
            m.edge_n[eb + e] = 0;
            m.edge_w[eb + e] = 0.0;
            m.edge_p[eb + e] = p;
            m.edge_player[eb + e] = (uint8_t)leaf_player;
            // the child node's edges and terminal mark: an existing node's
            // from the probe; a new node has no edges, and is terminal as the
            // state it was created from (a sibling duplicate's: its target's)
            m.edge_hint[eb + e] =
                f == 1 ? (int32_t)(uint32_t)L.hash[c]
                       : edge_hint_of(0, 0, game_done(L.state[f == 3 ? L.child[c] : c][5]));
          }
        }
        if (lane == 0) {
          m.node_e0[nb + leaf] = base_e;
          m.node_ne[nb + leaf] = n_edges;
          if (in_edge >= 0) m.edge_hint[eb + in_edge] = edge_hint_of(base_e, n_edges, false);
          cnt[0] = base_n + n_new;
          cnt[1] = base_e + n_edges;
        }
      }
    } else if (nl > kMaxChildren && lane == 0) {
      cnt[3] = 2;
    }
  }
  HZ_XSTAMP(6)
  // back_fill: every path edge gets N += 1, W += v * (+1 if the edge's mover
  // is the leaf's player else -1)
  // (the path's edges are distinct: the adds are read-modify-writes done by
  // the memory side, one round trip less; the f64 add rounds as __dadd_rn)
  for (int i = lane; i < d; i += kWave) {
    const size_t e = eb + path[i];
    double dir = m.edge_player[e] == leaf_player ? 1.0 : -1.0;
    atomicAdd(&m.edge_n[e], 1);
    unsafeAtomicAdd(&m.edge_w[e], v * dir);
  }
#ifdef HZ_DIAG
  __builtin_amdgcn_s_waitcnt(0);
#endif
  HZ_XSTAMP(7)
  HZ_XFLAG(11, d)
}

// Sel: the wave then walks its board's tree for the next simulation
// (select_board, as k_select would in the next launch): the walk starts
// while the path it just backed up is hot in L2, and a simulation has one
// launch fewer.  Same tree, same leaf, same path: the board's wave does in
// one kernel what two consecutive kernels did.
// Gather (with Sel): the wave then also takes its leaf's row of the next
// leaf batch, if the leaf needs the network: the row is the next value of
// count_out (one atomic add per such board: rows in arrival order, not board
// order; every network row is computed independently of its batch, so the
// results are the same bits), and the wave encodes its leaf into that row of
// board/glob itself (encode_one).  This replaces the separate gather +
// encode launch (k_gather_encode: every workgroup scanning every board's
// leaf flag) by work spread over the waves that found the leaves.
// count_out must be zero at launch; count_prev (the count of the batch this
// launch consumed) is zeroed here for the launch after next, and added to
// the eval counter first when add_prev (a count no gather kernel added).
// BPW boards per workgroup (one wave each, each with its own LDS record; the
// expansion synchronises its own wave only): with Gather, the workgroup's
// boards take their rows with one atomic add (16 boards: 256 adds per
// simulation at 4096 boards instead of 4096 to one address, which cost ~20
// us of same-address serialisation at L2).
// WaveSlot (BPW > 1): each wave takes its row with its own atomic add as
// soon as its walk is done, instead of the workgroup's one add after a
// barrier that waits for the workgroup's slowest wave (A/B: HZ_SLOT_WAVE)
template <int Waves, bool Sel, bool Gather = false, int BPW = 1, bool WaveSlot = false>  // Waves: minimum waves per SIMD the register allocation must allow (3: none forced)
__global__ void __launch_bounds__(kWave * BPW) __attribute__((amdgpu_waves_per_eu(Waves, 8))) k_expand_backup(hz_mcts m, uint32_t *__restrict__ mtw,
                                                         int32_t *__restrict__ mtcur,
                                                         const float *__restrict__ policy,
                                                         const float *__restrict__ value,
                                                         const double *__restrict__ noise, double eps,
                                                         float one_minus_eps, int testing,
                                                         const int32_t *__restrict__ row_of, int prio,
                                                         const uint8_t *__restrict__ active, float cpuct,
                                                         float *__restrict__ board, float *__restrict__ glob,
                                                         int32_t *__restrict__ rows, int32_t *__restrict__ count_out,
                                                         int32_t *__restrict__ count_prev, int add_prev) {
  __shared__ ExpandLds Ls[BPW];
  __shared__ int32_t s_need[BPW > 1 ? BPW : 1];
  __shared__ int32_t s_base;
  // (wave-uniform: the record's base is a scalar)
  const int w = BPW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int lane = (int)threadIdx.x & (kWave - 1);
  ExpandLds &L = Ls[w];
  const int b = (int)blockIdx.x * BPW + w;
  const bool live = BPW == 1 || b < m.n;
  if (live)
    expand_backup_board(L, m, mtw, mtcur, policy, value, noise, eps, one_minus_eps, testing, row_of, prio, b, lane,
                        Sel);
  if (Sel) {
    __builtin_amdgcn_s_setprio(0);
    // the walk reads N and W past L1: the backup's adds were done at L2 (the
    // wave's own stores and adds to an address stay in order; an agent-scope
    // fence here, i.e. an L2 writeback and invalidate per wave, made the
    // launch 223 us instead of 38).  The workgroup-scope release fence makes
    // the backup's atomic adds complete (s_waitcnt vmcnt(0) on gfx950, no
    // cache maintenance) before the walk's loads issue, so the walk does not
    // rest on same-address requests reaching L2 in issue order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    const int g = live ? select_board<true>(m, b, lane, active, cpuct) : -1;
    // Gather: the leaf's six state words loaded and its row built in the
    // lane's registers (encode_one_values) before the row-slot barriers,
    // under the wait for the workgroup's slowest wave; after them only the
    // row's stores remain
    float2 evals[kEncQ];
    float egv = 0.f;
    if constexpr (Gather) {
      if (g >= 0) {
        uint64_t lsw[6];
#pragma unroll
        for (int k = 0; k < 6; k++) lsw[k] = m.node_state[(size_t)g * 6 + k];
        encode_one_values(lsw, lane, &L.key[0][0], reinterpret_cast<float *>(&L.key[40][0]), evals, egv);
      }
    }
#ifdef HZ_DIAG
    const bool dg = live;
#endif
    HZ_XSTAMP(12)
    if constexpr (Gather) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (add_prev && m.eval_ctr) m.eval_ctr[0] += *count_prev;  // final: its batch was evaluated
        *count_prev = 0;
      }
      int slot = -1;
      if constexpr (BPW > 1 && !WaveSlot) {
        if (lane == 0) s_need[w] = g >= 0;
        __syncthreads();
        if (threadIdx.x == 0) {
          int tot = 0;
#pragma unroll
          for (int k = 0; k < BPW; k++) tot += s_need[k];
          s_base = tot ? atomicAdd(count_out, tot) : 0;
        }
        __syncthreads();
        if (g >= 0) {
          slot = s_base;
          for (int k = 0; k < w; k++) slot += s_need[k];
        }
      } else if (g >= 0) {
        if (lane == 0) slot = atomicAdd(count_out, 1);
        slot = __builtin_amdgcn_readfirstlane(slot);
      }
      if (slot >= m.n) slot = -1;  // (count_out was not zero: never with the host's protocol)
      HZ_XSTAMP(14)
      if (live && lane == 0) {
        m.slot[b] = slot;
        if (slot >= 0) {
          m.gidx_c[slot] = g;
          if (rows) rows[slot] = b;
        }
      }
      if (slot >= 0) {
        encode_one_store(board + (size_t)slot * kBoardFloats, glob + (size_t)slot * kGlobFloats, lane, evals, egv);
      }
#ifdef HZ_DIAG
      __builtin_amdgcn_s_waitcnt(0);
#endif
      HZ_XSTAMP(13)
    }
  }
}

// ------------------------------------------------------------- root noise
// The self-play root noise of get_best_action_and_pi (MCTS.py:314-316:
// np.random.dirichlet([alpha] * L) over the L legal moves) and the tau = 1
// uniform of its move choice (MCTS.py:411, np.random.choice), drawn from a
// counter-based generator keyed by (seed, global board id, move) instead of
// the process-global np.random: every board's draws are the same whatever
// the batch it sits in or the number of GPUs.  One wave per
// board; lane c draws child c's Gamma(alpha) (and c + 64's): Marsaglia-Tsang
// for alpha + 1 with a standard normal from Box-Muller, times U^(1/alpha)
// for alpha < 1.  The live children's sum is a fixed butterfly over the
// wave, so the result does not depend on anything but the key.
struct NoiseStream {
  uint64_t key, ctr;
  __device__ double uniform() {  // (0, 1], 53 bits
    uint64_t z = mix64(key + 0x9E3779B97F4A7C15ULL * ++ctr);
    return ((double)(z >> 11) + 1.0) * 0x1.0p-53;
  }
};

__device__ double gamma_draw(NoiseStream &s, double alpha) {
  const double a = alpha < 1.0 ? alpha + 1.0 : alpha;
  const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  double g;
  for (;;) {
    double x, v;
    do {
      double u1 = s.uniform(), u2 = s.uniform();
      x = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
      v = 1.0 + c * x;
    } while (v <= 0.0);
    v = v * v * v;
    double u = s.uniform();
    if (u < 1.0 - 0.0331 * x * x * x * x || log(u) < 0.5 * x * x + d * (1.0 - v + log(v))) {
      g = d * v;
      break;
    }
  }
  if (alpha < 1.0) g *= pow(s.uniform(), 1.0 / alpha);
  return g;
}

__global__ void __launch_bounds__(kWave) k_root_noise(const int32_t *__restrict__ count, int n, uint64_t seed,
                                                      uint64_t board_base, uint64_t move, double alpha,
                                                      double *__restrict__ noise, double *__restrict__ u) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const uint64_t key = mix64(mix64(mix64(seed ^ 0x6A09E667F3BCC908ULL) ^ (board_base + (uint64_t)b)) ^ move);
  const int nl = count ? min(max(count[b], 0), kMaxChildren) : 0;
  double g[2];
  double sum = 0.0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int c = lane + kWave * k;
    NoiseStream s{mix64(key ^ (0xD1B54A32D192ED03ULL * (uint64_t)(c + 1))), 0};
    g[k] = c < nl ? gamma_draw(s, alpha) : 0.0;
    sum += g[k];
  }
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) sum += __shfl_xor(sum, off);
  const double inv = sum > 0.0 ? 1.0 / sum : 0.0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int c = lane + kWave * k;
    if (c < kMaxChildren) noise[(size_t)b * kMaxChildren + c] = g[k] * inv;
  }
  if (lane == 0 && u) {
    NoiseStream s{mix64(key ^ 0x5851F42D4C957F2DULL), 0};
    u[b] = s.uniform() - 0x1.0p-53;  // [0, 1)
  }
}

// root visit counts by action (MCTS.py:355-376)
__global__ void __launch_bounds__(kWave) k_result(hz_mcts m, int32_t *__restrict__ visits) {
  int b = blockIdx.x;
  int lane = threadIdx.x;
  int32_t *out = visits + (size_t)b * kActions;
  for (int a = lane; a < kActions; a += kWave) out[a] = 0;
  __syncthreads();
  if (m.counts[(size_t)b * 4] == 0) return;
  size_t nb = (size_t)b * m.max_nodes, eb = (size_t)b * m.max_edges;
  int ne = m.node_ne[nb], e0 = m.node_e0[nb];
  for (int i = lane; i < ne; i += kWave) out[m.edge_action[eb + e0 + i]] = m.edge_n[eb + e0 + i];
}

template <class T>
bool alloc(T **p, size_t count) {
  return hipMalloc((void **)p, count * sizeof(T)) == hipSuccess;
}

}  // namespace

namespace {
// Sum of every edge's visit count over the board's tree: each simulation
// adds one visit to every edge of its path in back_fill (MCTS.py:220-266),
// so this is the number of edge levels the searches walked (the path-walk
// term of the tree's algorithmic bytes).  Wave per board, one vector atomic.
__global__ void __launch_bounds__(kWave) k_path_edges(hz_mcts m, unsigned long long *__restrict__ out) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int ne = m.counts[(size_t)b * 4 + 1];
  const int32_t *en = m.edge_n + (size_t)b * m.max_edges;
  unsigned long long acc = 0;
  for (int e = lane; e < ne; e += kWave) acc += (unsigned)en[e];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, kWave);
  if (lane == 0 && acc) atomicAdd(out, acc);
}
}  // namespace

extern "C" {

hz_mcts *hz_mcts_create(int32_t n_boards, int32_t max_nodes, int32_t max_depth, int32_t exact_keys, void *stream) {
  if (n_boards <= 0 || max_nodes < 2 || max_depth < 1) return nullptr;
  if (max_nodes >= kMaxNodesHint) return nullptr;  // edge ids (max_edges = max_nodes) must fit edge_hint_of
  if (install_comp_table()) return nullptr;  // terminal expansions score boards
  hz_mcts *m = (hz_mcts *)calloc(1, sizeof(hz_mcts));
  if (!m) return nullptr;
  m->n = n_boards;
  m->max_nodes = max_nodes;
  m->max_edges = max_nodes;
  int h = 1;
  while (h < 2 * max_nodes) h <<= 1;
  m->hcap = h;
  m->max_depth = max_depth;
  m->exact_keys = exact_keys;
  m->gather_mode = -1;
  m->stream = (hipStream_t)stream;
  size_t n = (size_t)n_boards, N = n * max_nodes, E = n * m->max_edges;
  bool ok = alloc(&m->node_state, N * 6) && alloc(&m->node_key, N * 8) && alloc(&m->node_e0, N) &&
            alloc(&m->node_ne, N) && alloc(&m->edge_action, E) && alloc(&m->edge_child, E) &&
            alloc(&m->edge_n, E) && alloc(&m->edge_w, E) && alloc(&m->edge_p, E) && alloc(&m->edge_player, E) &&
            alloc(&m->edge_hint, E) &&
            alloc(&m->ht, n * m->hcap) && alloc(&m->counts, n * 4) && alloc(&m->path, n * max_depth) &&
            alloc(&m->depth, n) && alloc(&m->leaf, n) && alloc(&m->leaf_gidx, n) && alloc(&m->slot, n) &&
            alloc(&m->gidx_c, n);
  if (ok) {
    ok = hipMemset(m->ht, 0, n * m->hcap * sizeof(uint64_t)) == hipSuccess &&
         hipMemset(m->counts, 0, n * 4 * sizeof(int32_t)) == hipSuccess &&
         hipMemset(m->depth, 0, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(m->leaf, 0xff, n * sizeof(int32_t)) == hipSuccess &&
         hipMemset(m->leaf_gidx, 0xff, n * sizeof(int32_t)) == hipSuccess;
  }
  if (!ok) {
    hz_mcts_destroy(m);
    return nullptr;
  }
  return m;
}

void hz_mcts_destroy(hz_mcts *m) {
  if (!m) return;
  void *ptrs[] = {m->node_state, m->node_key, m->node_e0,   m->node_ne, m->edge_action, m->edge_child,
                  m->edge_n,     m->edge_w,    m->edge_p,    m->edge_player, m->edge_hint, m->ht, m->counts,
                  m->path,       m->depth,     m->leaf,      m->leaf_gidx, m->slot, m->gidx_c};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  free(m);
}

int hz_mcts_set_eval_counter(hz_mcts *m, int64_t *counter) {
  if (!m) return -1;
  m->eval_ctr = counter;
  return 0;
}

int hz_mcts_set_dedup_walk(hz_mcts *m, int32_t on) {
  if (!m) return -1;
  m->dedup_walk = on ? 1 : 0;
  return 0;
}

int hz_mcts_set_gather_encode(hz_mcts *m, int32_t mode) {
  if (!m || mode < -1 || mode > 1) return -1;
  m->gather_mode = mode;
  return 0;
}

int hz_mcts_set_stream(hz_mcts *m, void *stream) {
  if (!m) return -1;
  m->stream = (hipStream_t)stream;
  return 0;
}

int hz_mcts_begin(hz_mcts *m, hz_env *env, const uint8_t *active) {
  if (!m || !env || hz_env_size(env) != m->n) return -1;
  hipLaunchKernelGGL(k_begin, dim3((m->n + kWave - 1) / kWave), dim3(kWave), 0, m->stream, *m,
                     hz_env_state_ptr(env), m->n, active);
  return launch_err();
}

int hz_mcts_select(hz_mcts *m, const uint8_t *active, float cpuct) {
  if (!m) return -1;
  hipLaunchKernelGGL(k_select, dim3(m->n), dim3(kWave), 0, m->stream, *m, active, cpuct);
  return launch_err();
}

int hz_mcts_encode_leaves(hz_mcts *m, float *board, float *glob) {
  if (!m || (!board && !glob)) return -1;
  launch_encode(m->node_state, 1, 6, m->leaf_gidx, m->n, board, glob, m->stream);
  return launch_err();
}

int hz_mcts_select_gather(hz_mcts *m, const uint8_t *active, float cpuct, float *board, float *glob, int32_t *rows,
                          int32_t *count) {
  if (!m || !count || !board || !glob) return -1;
  if (m->n > kFusedMax) {
    const int rc = hz_mcts_select(m, active, cpuct);
    return rc ? rc : hz_mcts_gather_leaves(m, board, glob, rows, count);
  }
  hipLaunchKernelGGL(k_select_gather_encode, dim3(1), dim3(kFusedWaves * kWave), 0, m->stream, *m, active, cpuct,
                     rows, count, board, glob);
  return launch_err();
}

int hz_mcts_gather_leaves(hz_mcts *m, float *board, float *glob, int32_t *rows, int32_t *count) {
  if (!m || !count || (!board && !glob)) return -1;
  // default: k_gather_encode (one launch); HZ_GATHER_ENCODE=0: k_gather + the
  // encoder launches (same results)
  static const bool fused_default = [] {
    const char *e = getenv("HZ_GATHER_ENCODE");
    return !(e && atoi(e) == 0);
  }();
  const bool fused = m->gather_mode < 0 ? fused_default : m->gather_mode == 1;
  if (fused && board && glob) {
    hipLaunchKernelGGL(k_gather_encode, dim3((m->n + kGERows - 1) / kGERows), dim3(kGEThreads), 0, m->stream, *m,
                       rows, count, board, glob);
    return launch_err();
  }
  hipLaunchKernelGGL(k_gather, dim3(1), dim3(kGatherThreads), 0, m->stream, *m, rows, count);
  launch_encode(m->node_state, 1, 6, m->gidx_c, m->n, board, glob, m->stream, count);
  return launch_err();
}

// boards per workgroup of the gathering expand launch (one atomic add per
// workgroup): 16 by default, HZ_GATHER_BPW=8 (A/B: two workgroups per CU)
constexpr int kGatherBPW = 16;
static_assert(kGatherBPW * sizeof(ExpandLds) <= 160 * 1024, "the workgroup's records fit the LDS");
static int gather_bpw() {
  static const int v = [] {
    const char *e = getenv("HZ_GATHER_BPW");
    return e && atoi(e) == 8 ? 8 : kGatherBPW;
  }();
  return v;
}

static int expand_backup(hz_mcts *m, hz_env *env, const float *policy, const float *value, const double *noise,
                         double eps, int32_t testing, const int32_t *slot, bool sel = false,
                         const uint8_t *active = nullptr, float cpuct = 0.f, float *board = nullptr,
                         float *glob = nullptr, int32_t *rows = nullptr, int32_t *count_out = nullptr,
                         int32_t *count_prev = nullptr, int add_prev = 0) {
  if (!m || !env || !policy || !value || hz_env_size(env) != m->n) return -1;
  float ome = (float)(1.0 - eps);
  // default: registers capped for four waves per SIMD (38 VGPRs spilled;
  // with the 9.8 KB LDS, 4096 boards fit the chip in one round): 44.7 vs
  // 47.3 us per sim step for three waves (HZ_EXPAND_WAVES=3), profiles/r03
  static const int waves = [] {
    const char *e = getenv("HZ_EXPAND_WAVES");
    return e && atoi(e) == 3 ? 3 : 4;
  }();
  // HZ_EXPAND_PRIO=0: the turn-end waves keep the default issue priority (A/B)
  static const int prio = [] {
    const char *e = getenv("HZ_EXPAND_PRIO");
    return e && atoi(e) == 0 ? 0 : 1;
  }();
  static const bool wave_slot = [] {
    const char *e = getenv("HZ_SLOT_WAVE");
    return e && atoi(e) == 1;
  }();
#define HZ_EXPAND_LAUNCH(W, S, G, BP, ...)                                                                      \
  hipLaunchKernelGGL((k_expand_backup<W, S, G, BP, ##__VA_ARGS__>), dim3((m->n + (BP) - 1) / (BP)), dim3(kWave * (BP)), \
                     0, m->stream, *m, hz_env_mt_ptr(env),                                                        \
                     hz_env_mt_pos_ptr(env), policy, value, noise, eps, ome, testing, slot, prio, active, cpuct,     \
                     board, glob, rows, count_out, count_prev, add_prev)
  const bool gat = sel && count_out;
  if (waves == 4) {
    if (gat && gather_bpw() == 8) HZ_EXPAND_LAUNCH(4, true, true, 8);
    else if (gat && wave_slot) HZ_EXPAND_LAUNCH(4, true, true, kGatherBPW, true);
    else if (gat) HZ_EXPAND_LAUNCH(4, true, true, kGatherBPW);
    else if (sel) HZ_EXPAND_LAUNCH(4, true, false, 1);
    else HZ_EXPAND_LAUNCH(4, false, false, 1);
  } else {
    if (gat && gather_bpw() == 8) HZ_EXPAND_LAUNCH(3, true, true, 8);
    else if (gat) HZ_EXPAND_LAUNCH(3, true, true, kGatherBPW);
    else if (sel) HZ_EXPAND_LAUNCH(3, true, false, 1);
    else HZ_EXPAND_LAUNCH(3, false, false, 1);
  }
#undef HZ_EXPAND_LAUNCH
  return launch_err();
}

int hz_mcts_expand_backup(hz_mcts *m, hz_env *env, const float *policy, const float *value, const double *noise,
                          double eps, int32_t testing) {
  return expand_backup(m, env, policy, value, noise, eps, testing, nullptr);
}

int hz_mcts_expand_backup_gathered(hz_mcts *m, hz_env *env, const float *policy, const float *value,
                                   const double *noise, double eps, int32_t testing) {
  return m ? expand_backup(m, env, policy, value, noise, eps, testing, m->slot) : -1;
}

int hz_mcts_expand_backup_select(hz_mcts *m, hz_env *env, const float *policy, const float *value,
                                 const double *noise, double eps, int32_t testing, const uint8_t *active,
                                 float cpuct) {
  return m ? expand_backup(m, env, policy, value, noise, eps, testing, m->slot, true, active, cpuct) : -1;
}

int hz_mcts_expand_backup_select_gather(hz_mcts *m, hz_env *env, const float *policy, const float *value,
                                        const double *noise, double eps, int32_t testing, const uint8_t *active,
                                        float cpuct, float *board, float *glob, int32_t *rows, int32_t *count_out,
                                        int32_t *count_prev, int32_t add_prev) {
  if (!m || !board || !glob || !count_out || !count_prev || count_out == count_prev) return -1;
  return expand_backup(m, env, policy, value, noise, eps, testing, m->slot, true, active, cpuct, board, glob, rows,
                       count_out, count_prev, add_prev);
}

int hz_root_noise(const int32_t *count, int32_t n, uint64_t seed, uint64_t board_base, uint64_t move, double alpha,
                  double *noise, double *u, void *stream) {
  if (n < 0 || !count || !noise || !(alpha > 0.0)) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_root_noise, dim3(n), dim3(kWave), 0, (hipStream_t)stream, count, n, seed, board_base, move,
                     alpha, noise, u);
  return launch_err();
}

int hz_mcts_result(hz_mcts *m, int32_t *visits) {
  if (!m || !visits) return -1;
  hipLaunchKernelGGL(k_result, dim3(m->n), dim3(kWave), 0, m->stream, *m, visits);
  return launch_err();
}

int hz_mcts_stats(hz_mcts *m, int32_t *counts) {
  if (!m || !counts) return -1;
  return hipMemcpyAsync(counts, m->counts, (size_t)m->n * 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, m->stream)
             ? 1
             : 0;
}

#ifdef HZ_DIAG
int hz_mcts_diag_stamps(uint64_t *host) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_exp_stamps), sizeof(g_exp_stamps)) == hipSuccess ? 0 : 1;
}
#endif

int hz_mcts_path_edges(hz_mcts *m, int64_t *out) {
  if (!m || !out) return -1;
  hipLaunchKernelGGL(k_path_edges, dim3(m->n), dim3(kWave), 0, m->stream, *m, (unsigned long long *)out);
  return launch_err();
}

int hz_mcts_leaf_ptrs(hz_mcts *m, int32_t **leaf, int32_t **leaf_gidx) {
  if (!m) return -1;
  if (leaf) *leaf = m->leaf;
  if (leaf_gidx) *leaf_gidx = m->leaf_gidx;
  return 0;
}

}  // extern "C"

#ifdef HZ_KEYCHECK
extern "C" int hz_keycheck_counts(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kc), sizeof(g_kc)) == hipSuccess ? 0 : 1;
}
#endif
