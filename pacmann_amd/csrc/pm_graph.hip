// pm_graph.hip — graph construction and ground truth on the GPU (SURVEY.md
// §8f rank 1: the reference builds its degree-m graph with NGT candidates,
// robustPrune (alpha = 1.2), reverse-edge sampling and a random fill,
// graphann/build_graph.go:169-236,314-523; NGT is not in the image, so the
// candidates here are the exact k nearest neighbours).
//
//   k_to_bf16     rows -> bf16 rows padded to DP (a multiple of 64) + f32 norms
//   k_knn_bf16    per query row, the 64 smallest (bf16 distance, id) keys over
//                 all base rows: MFMA 32x32x16 bf16 tiles, per-row thresholds,
//                 LDS insertion buffers merged into a sorted top-64 per row
//   k_knn_rerank  the 64 prefilter candidates re-ranked by the reference's own
//                 L2Dist (l2_distance_amd64.s order) and id: top K, self dropped
//   k_prune       robustPrune (build_graph.go:169-236) per vertex: candidate
//                 distances in L2Dist order, stable sort, the alpha test of each
//                 candidate against every accepted neighbour in parallel
//
// Integer-valued inputs up to 255 (SIFT bvecs semantics, loader.go:46-51) are
// exact in bf16 and every bf16 product/partial sum is an exact f32 integer, so
// the prefilter distances are exact and the top-64 holds the exact top-K: the
// result equals a brute-force L2Dist ranking bit for bit.  For general float
// data the prefilter ranks by bf16-rounded distances and keeps 64 candidates
// for the exact re-rank of the top K (K <= 48 in the graph build).
#include <hip/hip_runtime.h>

#include "pm_internal.h"

namespace pm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kKnnRows = 64;      // query rows per workgroup
constexpr int kKnnCols = 128;     // base rows per tile
constexpr int kKnnTop = 64;       // prefilter keys kept per query row
constexpr int kKnnThreads = 512;  // 8 waves: 2 row blocks x 4 column blocks of 32x32
constexpr uint64_t kNoKey = ~0ull;

// rows [n][dim] f32 -> out [n][dp] bf16 (zero padded), norms [n] = sum of the
// squared bf16 values in element order (exact for integer-valued rows)
__global__ void __launch_bounds__(kBlock) k_to_bf16(const float* __restrict__ rows, uint64_t n, uint32_t dim,
                                                    uint32_t dp, __bf16* __restrict__ out,
                                                    float* __restrict__ norms) {
  const uint64_t r = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (r >= n) return;
  float s = 0.0f;
  for (uint32_t c0 = 0; c0 < dp; c0 += 64) {
    const uint32_t c = c0 + lane;
    const float v = c < dim ? rows[r * dim + c] : 0.0f;
    const __bf16 b = (__bf16)v;
    out[r * dp + c] = b;
    const float f = (float)b;
    float sq = __fmul_rn(f, f);
    // fixed-order wave sum (xor tree), then chunk order
    for (int o = 1; o < 64; o <<= 1) sq = __fadd_rn(sq, __shfl_xor(sq, o));
    s = __fadd_rn(s, sq);
  }
  if (lane == 0) norms[r] = s;
}

template <int DP>
struct KnnLds {
  uint64_t top[kKnnRows][kKnnTop];          // sorted ascending per row
  uint64_t buf[kKnnRows][kKnnCols];         // this tile's keys below the row threshold
  uint32_t cnt[kKnnRows];
  uint32_t any[2];
  __bf16 b[kKnnCols][DP + 8];               // padded rows: conflict-free 16-B fragment reads
};

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  const uint32_t lo = __shfl_up((uint32_t)v, d), hi = __shfl_up((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

// Merge the row's insertion buffer into its sorted top-64 (lane i holds entry i).
__device__ __forceinline__ void knn_merge_row(uint64_t* top, const uint64_t* buf, uint32_t n, uint32_t lane) {
  uint64_t t = top[lane];
  for (uint32_t e = 0; e < n; ++e) {
    const uint64_t x = buf[e];
    const uint64_t last = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(t >> 32), 63) << 32) |
                          __builtin_amdgcn_readlane((uint32_t)t, 63);
    if (x >= last) continue;   // uniform: x and last are wave-uniform
    const uint32_t pos = __popcll(__ballot(t < x));
    const uint64_t up = shfl_up64(t, 1);
    t = lane < pos ? t : (lane == pos ? x : up);
  }
  top[lane] = t;
}

template <int DP>
__global__ void __launch_bounds__(kKnnThreads) k_knn_bf16(const __bf16* __restrict__ X, const float* __restrict__ xn,
                                                          uint64_t N, const __bf16* __restrict__ Q,
                                                          const float* __restrict__ qn, uint64_t M,
                                                          uint32_t* __restrict__ out) {
  constexpr int KS = DP / 16;                       // MFMA k-steps
  constexpr int CH = kKnnCols * DP / 8;             // 16-B chunks per tile
  constexpr int PER = CH / kKnnThreads;             // per thread
  static_assert(CH % kKnnThreads == 0, "tile chunks");
  __shared__ KnnLds<DP> L;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t rb = 32 * (w & 1), cb = 32 * (w >> 1);
  const uint32_t r32 = lane & 31, h = lane >> 5;
  const uint64_t row0 = (uint64_t)blockIdx.x * kKnnRows;

  for (uint32_t i = tid; i < kKnnRows * kKnnTop; i += kKnnThreads) (&L.top[0][0])[i] = kNoKey;
  if (tid < kKnnRows) L.cnt[tid] = 0;
  if (tid < 2) L.any[tid] = 0;

  // A fragments of this wave's 32 query rows (whole K), kept in registers
  bf16x8 a[KS];
  {
    const uint64_t qr = row0 + rb + r32;
    for (int s = 0; s < KS; ++s) {
      if (qr < M) a[s] = *(const bf16x8*)(Q + qr * DP + 16 * s + 8 * h);
      else for (int j = 0; j < 8; ++j) a[s][j] = (__bf16)0.0f;
    }
  }
  // query norms and thresholds of the lane's 16 output rows
  float qnr[16];
  uint32_t thi[16];
  for (int i = 0; i < 16; ++i) {
    const uint64_t qr = row0 + rb + (i & 3) + 8 * (i >> 2) + 4 * h;
    qnr[i] = qr < M ? qn[qr] : 0.0f;
    thi[i] = 0xffffffffu;
  }
  const uint64_t T = (N + kKnnCols - 1) / kKnnCols;
  uint4 pre[PER];
  auto load_tile = [&](uint64_t t) {
    const uint64_t c0 = t * kKnnCols;
    for (int p = 0; p < PER; ++p) {
      const uint32_t q = tid + p * kKnnThreads;
      const uint32_t j = q / (DP / 8), off = (q % (DP / 8)) * 8;
      if (c0 + j < N) pre[p] = *(const uint4*)(X + (c0 + j) * DP + off);
      else pre[p] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&]() {
    for (int p = 0; p < PER; ++p) {
      const uint32_t q = tid + p * kKnnThreads;
      const uint32_t j = q / (DP / 8), off = (q % (DP / 8)) * 8;
      *(uint4*)&L.b[j][off] = pre[p];
    }
  };
  load_tile(0);
  store_tile();
  __syncthreads();
  for (uint64_t t = 0; t < T; ++t) {
    if (t + 1 < T) load_tile(t + 1);   // in flight during the MFMAs
    f32x16 acc = {};
    for (int s = 0; s < KS; ++s) {
      const bf16x8 bb = *(const bf16x8*)&L.b[cb + r32][16 * s + 8 * h];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], bb, acc, 0, 0, 0);
    }
    const uint64_t col = t * kKnnCols + cb + r32;
    if (col < N) {
      const float cn = xn[col];
      for (int i = 0; i < 16; ++i) {
        const uint32_t lr = rb + (i & 3) + 8 * (i >> 2) + 4 * h;
        float d = __fsub_rn(__fadd_rn(qnr[i], cn), __fmul_rn(2.0f, acc[i]));
        d = d < 0.0f ? 0.0f : d;
        const uint32_t db = __float_as_uint(d);
        if (db <= thi[i]) {
          const uint64_t key = ((uint64_t)db << 32) | (uint32_t)col;
          if (db < thi[i] || key < L.top[lr][kKnnTop - 1]) {
            const uint32_t slot = atomicAdd(&L.cnt[lr], 1u);
            L.buf[lr][slot] = key;
            L.any[t & 1] = 1;
          }
        }
      }
    }
    if (tid == 0) L.any[(t + 1) & 1] = 0;
    __syncthreads();
    const bool merged = L.any[t & 1] != 0;   // uniform
    if (merged) {
      for (uint32_t r = w * 8; r < w * 8 + 8; ++r) {
        const uint32_t n = L.cnt[r];
        if (n) knn_merge_row(L.top[r], L.buf[r], n, lane);
      }
    }
    if (t + 1 < T) store_tile();
    __syncthreads();
    if (merged) {
      if (lane < 8) L.cnt[w * 8 + lane] = 0;   // every row of this wave's merge set
      for (int i = 0; i < 16; ++i) {
        const uint32_t lr = rb + (i & 3) + 8 * (i >> 2) + 4 * h;
        thi[i] = (uint32_t)(L.top[lr][kKnnTop - 1] >> 32);
      }
    }
    // cnt resets must land before the next tile's inserts
    if (merged) __syncthreads();
  }
  for (uint32_t r = w * 8; r < w * 8 + 8; ++r) {
    const uint64_t qr = row0 + r;
    if (qr < M) out[qr * kKnnTop + lane] = (uint32_t)L.top[r][lane];
  }
}

// 8-lane L2Dist of a (global f32) and b (global f32) in the reference order;
// every lane of the group returns the distance.
__device__ __forceinline__ float l2_group8(const float* __restrict__ a, const float* __restrict__ b, uint32_t dim,
                                           uint32_t k) {
  const uint32_t dimS = dim & ~7u;
  float acc = 0.0f;
  for (uint32_t t = k; t < dimS; t += 8) {
    const float d = __fsub_rn(a[t], b[t]);
    acc = __fadd_rn(acc, __fmul_rn(d, d));
  }
  acc = __fadd_rn(acc, __shfl_xor(acc, 1));
  acc = __fadd_rn(acc, __shfl_xor(acc, 2));
  acc = __fadd_rn(acc, __shfl_xor(acc, 4));
  float d = dimS ? acc : 0.0f;
  for (uint32_t i = dimS; i < dim; ++i) {   // build_graph.go:122-125 scalar tail
    const float t = __fsub_rn(a[i], b[i]);
    d = __fadd_rn(d, __fmul_rn(t, t));
  }
  return d;
}

// Bitonic sort of 64 u64 keys held one per lane (ascending by lane).
__device__ __forceinline__ uint64_t wave_sort64(uint64_t x, uint32_t lane) {
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)x, j), hi = __shfl_xor((uint32_t)(x >> 32), j);
      const uint64_t y = ((uint64_t)hi << 32) | lo;
      const bool up = (lane & k) == 0, lower = (lane & j) == 0;
      const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
      x = (up == lower) ? mn : mx;
    }
  }
  return x;
}

// One wave per query row: exact L2Dist of the 64 candidates, keys (dist, id),
// sorted; the first K (self dropped when self_base) go to out[row][K], their
// count to len[row].
__global__ void __launch_bounds__(kBlock) k_knn_rerank(const float* __restrict__ X, uint64_t N, uint32_t dim,
                                                       const float* __restrict__ Q, uint64_t M,
                                                       const uint32_t* __restrict__ cand, uint32_t K,
                                                       int self_base, uint32_t* __restrict__ out,
                                                       float* __restrict__ dist_out, uint32_t* __restrict__ len) {
  __shared__ uint64_t keys[kBlock / 64][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t row = (uint64_t)blockIdx.x * (kBlock / 64) + w;
  if (row >= M) return;
  const float* q = Q + row * dim;
  const uint32_t g = lane >> 3, k = lane & 7;
  for (uint32_t r = 0; r < 8; ++r) {
    const uint32_t c = r * 8 + g;
    const uint32_t id = cand[row * kKnnTop + c];
    const bool ok = id < N;
    const float d = l2_group8(X + (ok ? (uint64_t)id : 0) * dim, q, dim, k);
    if (k == 0) keys[w][c] = ok ? (((uint64_t)__float_as_uint(d) << 32) | id) : kNoKey;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // this wave's LDS keys visible to its lanes
  __builtin_amdgcn_wave_barrier();
  uint64_t x = wave_sort64(keys[w][lane], lane);
  // the first K keys; self dropped (the reference removes u from NGT's K results)
  const uint32_t id = (uint32_t)x;
  const bool in = lane < K && x != kNoKey;
  const bool self = self_base && id == (uint32_t)row;
  const uint64_t keep = __ballot(in && !self);
  const uint32_t pos = __popcll(keep & ((1ull << lane) - 1));
  if (in && !self) {
    out[row * K + pos] = id;
    if (dist_out) dist_out[row * K + pos] = __uint_as_float((uint32_t)(x >> 32));
  }
  if (lane == 0) len[row] = __popcll(keep);
}

constexpr int kPruneMaxL = 4096;   // candidates per vertex held in LDS
constexpr int kPruneMaxM = 64;
constexpr int kPruneMaxD = 256;

struct PruneLds {
  uint64_t key[kPruneMaxL];        // (L2Dist to u, position): stable order
  float dist[kPruneMaxL];          // by position
  uint32_t disc[kPruneMaxL];       // discarded ids in order
  float acc[kPruneMaxM + 1][kPruneMaxD + 8];   // accepted vectors; slot na = the candidate under test
  uint32_t acc_id[kPruneMaxM];
};

// robustPrune(vectors, u, candidates, m, alpha) (build_graph.go:169-236) for
// vertex verts[b] (or b): candidates ids[offs[u] .. offs[u] + lens[u]) (offs
// null: u * stride).  Lists of at most m are kept as they are (:170-172).
// Writes out[u][0..len) and out_len[u]; err = 1 if a list exceeds kPruneMaxL.
// Presorted mode (lists above kPruneMaxL, hub vertices): sorted_pos[off + s]
// is the position of the s-th candidate in (L2Dist, position) order and
// dist_g[off + pos] its distance (k_cand_dist, sorted on the host); only the
// first kPruneMaxL discards are kept (the top-up needs at most m).
__global__ void __launch_bounds__(kBlock) k_prune(const float* __restrict__ X, uint32_t dim,
                                                  const uint32_t* __restrict__ verts, uint64_t nverts,
                                                  const uint64_t* __restrict__ offs, uint64_t stride,
                                                  const uint32_t* __restrict__ lens,
                                                  const uint32_t* __restrict__ ids, uint32_t m, float alpha,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ out_len,
                                                  uint32_t* __restrict__ err,
                                                  const uint32_t* __restrict__ sorted_pos,
                                                  const float* __restrict__ dist_g) {
  __shared__ PruneLds L;
  const uint64_t b = blockIdx.x;
  if (b >= nverts) return;
  const uint64_t u = verts ? verts[b] : b;
  const uint32_t tid = threadIdx.x, g = tid >> 3, k = tid & 7;
  const uint64_t off = offs ? offs[u] : u * stride;
  const uint32_t n = lens[u];
  const uint32_t* c = ids + off;
  if (n <= m) {
    for (uint32_t i = tid; i < n; i += kBlock) out[u * m + i] = c[i];
    if (tid == 0) out_len[u] = n;
    return;
  }
  const bool pre = sorted_pos != nullptr;
  if (n > kPruneMaxL && !pre) {
    if (tid == 0) { atomicOr(err, 1u); out_len[u] = 0; }
    return;
  }
  const float* xu = X + u * dim;
  if (!pre) {
    // dist2u (:176-182) in L2Dist order; 32 candidates per round
    for (uint32_t r = 0; r < n; r += kBlock / 8) {
      const uint32_t i = r + g;
      const uint32_t id = i < n ? c[i] : 0;
      const float d = l2_group8(xu, X + (uint64_t)id * dim, dim, k);
      if (i < n && k == 0) {
        L.dist[i] = d;
        L.key[i] = ((uint64_t)__float_as_uint(d) << 32) | i;
      }
    }
    uint32_t np2 = 64;
    while (np2 < n) np2 <<= 1;
    for (uint32_t i = n + tid; i < np2; i += kBlock) L.key[i] = kNoKey;
    __syncthreads();
    // sort.Slice by distance (:184-186); ties by position (stable)
    for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
      for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
        for (uint32_t i = tid; i < np2; i += kBlock) {
          const uint32_t p = i ^ j;
          if (p > i) {
            const uint64_t x = L.key[i], y = L.key[p];
            const bool up = (i & kk) == 0;
            if ((x > y) == up) { L.key[i] = y; L.key[p] = x; }
          }
        }
        __syncthreads();
      }
    }
  }   // !pre
  // the greedy pass (:188-212): candidate v is accepted unless an accepted a_j
  // has L2Dist(a_j, v) * alpha < dist(u, v); all a_j are tested at once
  uint32_t na = 0, nd = 0;
  for (uint32_t s = 0; s < n; ++s) {
    const uint32_t pos = pre ? sorted_pos[off + s] : (uint32_t)L.key[s];
    const uint32_t v = c[pos];
    const float duv = pre ? dist_g[off + pos] : L.dist[pos];
    const float* xv = X + (uint64_t)v * dim;
    for (uint32_t i = tid; i < dim; i += kBlock) L.acc[na][i] = xv[i];
    __syncthreads();
    bool rej = false;
    if (g < na) {
      const float d = l2_group8(L.acc[g], L.acc[na], dim, k);
      rej = __fmul_rn(d, alpha) < duv;
    }
    const bool any = __syncthreads_or(rej);
    if (!any) {
      if (tid == 0) L.acc_id[na] = v;
      ++na;
      if (na == m) break;
    } else {
      if (tid == 0 && nd < kPruneMaxL) L.disc[nd] = v;
      ++nd;
    }
  }
  __syncthreads();
  // too few accepted: the discarded ones in order (:216-223)
  for (uint32_t i = tid; i < na; i += kBlock) out[u * m + i] = L.acc_id[i];
  const uint32_t fill = na < m ? (m - na < nd ? m - na : nd) : 0;
  for (uint32_t i = tid; i < fill; i += kBlock) out[u * m + na + i] = L.disc[i];
  if (tid == 0) out_len[u] = na + fill;
}

// L2Dist(x_u, x_v) of every candidate v of vertex verts[b]'s list, in the
// reference's order (dist2u, build_graph.go:176-182), into dist_g[offs[u] + i]:
// the keys the host sorts for the presorted k_prune of hub vertices.
__global__ void __launch_bounds__(kBlock) k_cand_dist(const float* __restrict__ X, uint32_t dim,
                                                      const uint32_t* __restrict__ verts,
                                                      const uint64_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ lens,
                                                      const uint32_t* __restrict__ ids, float* __restrict__ dist_g) {
  const uint64_t u = verts[blockIdx.x];
  const uint32_t g = threadIdx.x >> 3, k = threadIdx.x & 7, n = lens[u];
  const uint64_t off = offs[u];
  const float* xu = X + u * dim;
  for (uint32_t i = g; i < n; i += kBlock / 8) {
    const float d = l2_group8(xu, X + (uint64_t)ids[off + i] * dim, dim, k);
    if (k == 0) dist_g[off + i] = d;
  }
}

}  // namespace pm

namespace pmk {
static inline unsigned gcdiv(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }

uint32_t knn_pad_dim(uint32_t dim) { return dim <= 128 ? 128 : (dim <= 192 ? 192 : 0); }
uint32_t knn_top() { return kKnnTop; }
uint32_t prune_max_list() { return kPruneMaxL; }
uint32_t prune_max_dim() { return kPruneMaxD; }
uint32_t prune_max_m() { return kPruneMaxM; }

void to_bf16(hipStream_t st, const float* rows, uint64_t n, uint32_t dim, uint32_t dp, void* out, float* norms) {
  if (!n) return;
  hipLaunchKernelGGL(k_to_bf16, dim3(gcdiv(n, kBlock / 64)), dim3(kBlock), 0, st, rows, n, dim, dp, (__bf16*)out,
                     norms);
}
void knn_prefilter(hipStream_t st, const void* X, const float* xn, uint64_t N, const void* Q, const float* qn,
                   uint64_t M, uint32_t dp, uint32_t* out) {
  if (!M) return;
  const dim3 grid(gcdiv(M, kKnnRows));
  if (dp == 128)
    hipLaunchKernelGGL(k_knn_bf16<128>, grid, dim3(kKnnThreads), 0, st, (const __bf16*)X, xn, N, (const __bf16*)Q,
                       qn, M, out);
  else
    hipLaunchKernelGGL(k_knn_bf16<192>, grid, dim3(kKnnThreads), 0, st, (const __bf16*)X, xn, N, (const __bf16*)Q,
                       qn, M, out);
}
void knn_rerank(hipStream_t st, const float* X, uint64_t N, uint32_t dim, const float* Q, uint64_t M,
                const uint32_t* cand, uint32_t K, bool self_base, uint32_t* out, float* dist, uint32_t* len) {
  if (!M) return;
  hipLaunchKernelGGL(k_knn_rerank, dim3(gcdiv(M, kBlock / 64)), dim3(kBlock), 0, st, X, N, dim, Q, M, cand, K,
                     (int)self_base, out, dist, len);
}
void prune(hipStream_t st, const float* X, uint32_t dim, const uint32_t* verts, uint64_t nverts,
           const uint64_t* offs, uint64_t stride, const uint32_t* lens, const uint32_t* ids, uint32_t m,
           float alpha, uint32_t* out, uint32_t* out_len, uint32_t* err, const uint32_t* sorted_pos,
           const float* dist_g) {
  if (!nverts) return;
  hipLaunchKernelGGL(k_prune, dim3((unsigned)nverts), dim3(kBlock), 0, st, X, dim, verts, nverts, offs, stride, lens,
                     ids, m, alpha, out, out_len, err, sorted_pos, dist_g);
}
void cand_dist(hipStream_t st, const float* X, uint32_t dim, const uint32_t* verts, uint64_t nverts,
               const uint64_t* offs, const uint32_t* lens, const uint32_t* ids, float* dist_g) {
  if (!nverts) return;
  hipLaunchKernelGGL(k_cand_dist, dim3((unsigned)nverts), dim3(kBlock), 0, st, X, dim, verts, offs, lens, ids, dist_g);
}
}  // namespace pmk
