// pm_shard.hip — kernels of private graph search over a sharded graph DB
// (VERDICT r02 row ‡): the synthetic graph DB of the
// BIGANN-scale configs, and the per-id records a shard contributes to a
// shared step's combine.
//
// A shard (rank) holds the partitions p % nshards == shard of the batch PIR
// (batch-pir.go:62-85) and answers only their sub-queries.  Every rank runs
// the same sessions' searches in lock-step, so after each shared step the
// ranks exchange, per id of every session's GetVertexInfo batch
// (private-search.go:441-506), what the search reads of its entry: the
// neighbour list, the L2 distance of its vector to the session's query
// (computed by k_answer next to the decode) and the success flag.  Exactly
// one rank answers an id, the others contribute zero words, so one integer
// all-reduce SUM of the records is the unsharded answer bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pm_internal.h"

namespace pm {

__global__ void __launch_bounds__(kBlock) k_graph_synth(uint32_t* __restrict__ dst, uint64_t r0, uint64_t nel,
                                                        uint32_t epr, uint64_t n, uint32_t dim, uint32_t m,
                                                        uint64_t kv, uint64_t kg) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < nel; f += stride) {
    const uint64_t v = r0 + f / epr;
    const uint32_t e = (uint32_t)(f % epr);
    __builtin_nontemporal_store(graph_synth_elem(kv, kg, n, dim, m, v, e), dst + f);
  }
}

__global__ void __launch_bounds__(kBlock) k_graph_synth_vecs(const uint64_t* __restrict__ ids, uint64_t nel,
                                                             uint32_t dim, uint64_t kv, float* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < nel; f += stride)
    out[f] = graph_synth_vec(kv, ids[f / dim], dim, (uint32_t)(f % dim));
}

// One thread per record word.  map >= 0: the step-wide sub-query that
// answered this id (last wins, as SimpleBatchPianoPIR.Query's response map,
// batch-pir.go:216-236); an in-step duplicate (ST_DUP) carries no row of its
// own and is followed to the sub-query it repeats (post_results does the same
// on the host for the unsharded path).
__global__ void __launch_bounds__(kBlock) k_pack_records(const int32_t* __restrict__ map, uint32_t nrec,
                                                         const PmOutHdr* __restrict__ hdr,
                                                         const uint64_t* __restrict__ rows, uint32_t E, uint32_t w0,
                                                         uint32_t W, uint64_t* __restrict__ rec, uint32_t nsub,
                                                         uint32_t* __restrict__ st2, uint64_t errw) {
  const uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (f == 0) rec[(uint64_t)nrec * W] = errw;   // the records' error word (pm_engine.cpp group_exchange)
  if (f < (uint64_t)nrec * W) {
    const uint32_t r = (uint32_t)(f / W), w = (uint32_t)(f % W);
    int32_t s = map[r];
    uint64_t v = 0;
    if (s >= 0) {
      for (int hop = 0; hdr[s].status == ST_DUP && hop < 2; ++hop) s = (int32_t)hdr[s].ref;
      const uint32_t st = hdr[s].status;
      if (st == ST_OK || st == ST_CACHED) {
        if (w + 1 < W) v = rows[(uint64_t)s * E + w0 + w];
        else v = (1ull << 32) | __float_as_uint(hdr[s].dist);
      }
    }
    rec[f] = v;
  }
  if (f < nsub) {
    st2[2 * f] = hdr[f].status;
    st2[2 * f + 1] = hdr[f].ref;
  }
}

// Eight lanes per record (the reference's 8-lane L2 order, as k_l2_rows);
// only records another shard of a modelled layout answers (map == -2).
__global__ void __launch_bounds__(kBlock) k_synth_records(const int32_t* __restrict__ map,
                                                          const uint64_t* __restrict__ ids, uint32_t nrec,
                                                          uint32_t npos, const float* __restrict__ qbuf,
                                                          uint32_t dim, uint32_t m, uint64_t n, uint64_t kv,
                                                          uint64_t kg, uint32_t w0, uint32_t W,
                                                          uint64_t* __restrict__ rec) {
  const uint64_t g = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 3;
  const uint32_t k = threadIdx.x & 7;
  const bool live = g < nrec && map[g] == -2;   // uniform per 8-lane group
  if (!__any(live)) return;
  const uint64_t v = live ? ids[g] : 0;
  const float* q = qbuf + (uint64_t)(live ? g / npos : 0) * dim;
  const uint32_t dimS = dim & ~7u;
  float acc = 0.0f;
  if (live)
    for (uint32_t t = k; t < dimS; t += 8) {
      const float d = __fsub_rn(graph_synth_vec(kv, v, dim, t), q[t]);
      acc = __fadd_rn(acc, __fmul_rn(d, d));
    }
  acc = __fadd_rn(acc, __shfl_xor(acc, 1));
  acc = __fadd_rn(acc, __shfl_xor(acc, 2));
  acc = __fadd_rn(acc, __shfl_xor(acc, 4));
  if (!live) return;
  uint64_t* o = rec + g * W;
  for (uint32_t w = k; w + 1 < W; w += 8) {
    const uint32_t e0 = 2 * (w0 + w);
    o[w] = (uint64_t)graph_synth_elem(kv, kg, n, dim, m, v, e0) |
           ((uint64_t)graph_synth_elem(kv, kg, n, dim, m, v, e0 + 1) << 32);
  }
  if (k == 0) {
    float d = dimS ? acc : 0.0f;
    for (uint32_t i = dimS; i < dim; ++i) {   // L2Dist's scalar tail (build_graph.go:123-126)
      const float x = __fsub_rn(graph_synth_vec(kv, v, dim, i), q[i]);
      d = __fadd_rn(d, __fmul_rn(x, x));
    }
    o[W - 1] = (1ull << 32) | __float_as_uint(d);
  }
}

}  // namespace pm

namespace pmk {
using namespace pm;
static inline unsigned cdiv_(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }

void graph_synth(hipStream_t st, uint64_t* dst, uint64_t r0, uint64_t rows, uint64_t n, uint32_t dim, uint32_t m,
                 uint64_t seed) {
  const uint32_t epr = dim + m;   // u32 elements per row (E = epr / 2 words)
  const uint64_t nel = rows * epr;
  unsigned grid = cdiv_(nel, kBlock);
  if (grid > 256 * 32) grid = 256 * 32;
  if (grid == 0) return;
  hipLaunchKernelGGL(k_graph_synth, dim3(grid), dim3(kBlock), 0, st, (uint32_t*)dst, r0, nel, epr, n, dim, m,
                     sm64(seed + DOM_SYNTH_VEC), sm64(seed + DOM_SYNTH_NB));
}
void graph_synth_vecs(hipStream_t st, const uint64_t* ids, uint64_t nids, uint32_t dim, uint64_t seed, float* out) {
  const uint64_t nel = nids * dim;
  unsigned grid = cdiv_(nel, kBlock);
  if (grid > 256 * 16) grid = 256 * 16;
  if (grid == 0) return;
  hipLaunchKernelGGL(k_graph_synth_vecs, dim3(grid), dim3(kBlock), 0, st, ids, nel, dim, sm64(seed + DOM_SYNTH_VEC),
                     out);
}
void pack_records(hipStream_t st, const int32_t* map, uint32_t nrec, const PmOutHdr* hdr, const uint64_t* rows,
                  uint32_t E, uint32_t w0, uint32_t W, uint64_t* rec, uint32_t nsub, uint32_t* st2, uint64_t errw) {
  const uint64_t nthr = std::max<uint64_t>({(uint64_t)nrec * W, (uint64_t)nsub, 1});
  hipLaunchKernelGGL(k_pack_records, dim3(cdiv_(nthr, kBlock)), dim3(kBlock), 0, st, map, nrec, hdr, rows, E, w0, W,
                     rec, nsub, st2, errw);
}
void synth_records(hipStream_t st, const int32_t* map, const uint64_t* ids, uint32_t nrec, uint32_t npos,
                   const float* qbuf, uint32_t dim, uint32_t m, uint64_t n, uint64_t seed, uint32_t w0, uint32_t W,
                   uint64_t* rec) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_synth_records, dim3(cdiv_((uint64_t)nrec * 8, kBlock)), dim3(kBlock), 0, st, map, ids, nrec,
                     npos, qbuf, dim, m, n, sm64(seed + DOM_SYNTH_VEC), sm64(seed + DOM_SYNTH_NB), w0, W, rec);
}
}  // namespace pmk
