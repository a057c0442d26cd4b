// pm_drl.hip — the device-resident team round of the batched serving loop
// (pm_search_loop_batched's device loop).
//
// The host round of a lock-step team (pm_engine.cpp run_batched_pool: per
// session the results' post-processing, GetVertexInfo's decode and success
// count, SearchKNN's update and next batch, SimpleBatchPianoPIR.Query's
// bucketing) as ONE launch of one kDrlThreads (256-thread) workgroup per session, so a team's
// 20 rounds chain on its stream as [match + resolve, answer, round] with no
// host round trip.  Same operations in the same order as the host restatement
// (and the oracle), with Go's tie rules:
//   * results (pm_engine.cpp post_results / bq_emit_fast, batch-pir.go:216-236):
//     an ST_OK sub-query's row enters the localCache (pir.go:468-470); each id
//     takes the LAST sub-query made for it; an in-step duplicate (ST_DUP) reads
//     the row and distance of the sub-query it repeats; ids dropped by the
//     overflow get the zero entry;
//   * GetVertexInfo (private-search.go:441-506): the neighbour list of each
//     entry, the success count against the true graph;
//   * SearchKNN's update (graphann/search.go:185-207): positions in order; an
//     id already known, or with an all-zero neighbour list, is skipped; the
//     rest become known and are pushed on the min-heap -- container/heap's
//     exact Push (up) and Pop (swap, down), so equal distances pop in Go's
//     order;
//   * the next batch (search.go:153-171): `parallel` pops, each one's m
//     neighbours, or m ids of the SplitMix stream when the heap is empty;
//   * the bucketing (batch-pir.go:175-200, pm_engine.cpp bq_prepare/add_sub):
//     ids per partition in order, the first queryNumToMake kept, the rest
//     dropped, the partition padded with dummy queries; a localCache hit is a
//     HOSTCACHE sub-query.
// The query's start (search.go:129-148: the first `parallel` start vertices
// by (distance, position)) and end (search.go:211-233: top k by (distance,
// id)) are the kernel's BEGIN and END modes.  The caller guarantees that no
// partition reaches its query budget during the rounds it chains (the gate in
// pm_engine.cpp drl_schedule), i.e. that the host would take the one-step path.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>

#include "pm_internal.h"

namespace pm {

struct HeapE { float d; uint32_t slot; };

// Open-addressing tables of u64 entries {key + 1 | value << 32} (0 = empty).
// A session's tables are only touched by its own workgroup (one CU) within a
// launch, and across launches through the stream's kernel boundaries, so
// workgroup-scope atomics suffice (no L2 write-back or invalidate: MI355X's
// L2s are per XCD, and an agent-scope fence would write one back).
__device__ __forceinline__ bool tab_find(const uint64_t* t, uint32_t mask, uint32_t key, uint32_t* val) {
  for (uint32_t i = drl_hash(key) & mask;; i = (i + 1) & mask) {
    const uint64_t e = __hip_atomic_load(const_cast<uint64_t*>(t) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (e == 0) return false;
    if ((uint32_t)e == key + 1u) { *val = (uint32_t)(e >> 32); return true; }
  }
}
__device__ __forceinline__ void tab_put(uint64_t* t, uint32_t mask, uint32_t key, uint32_t val) {
  const uint64_t ne = ((uint64_t)val << 32) | (uint64_t)(key + 1u);
  for (uint32_t i = drl_hash(key) & mask;; i = (i + 1) & mask) {
    uint64_t e = 0;
    if (__hip_atomic_compare_exchange_strong(t + i, &e, ne, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP))
      return;
    if ((uint32_t)e == key + 1u) {   // insert or overwrite (FlatMap::put)
      __hip_atomic_store(t + i, ne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
  }
}

// container/heap.Push: append, then up().  up() swaps the new element with its
// parent while it is strictly Less (dist <); the ancestors on its path are
// non-increasing upward (heap order), so the elements it passes are exactly the
// c nearest ancestors with dist > x.  Lane l >= 1 holds the ancestor l levels
// up (0-based index ((n + 1) >> l) - 1): one LDS read per lane, one ballot, and
// the c passed ancestors move one level down while x lands at ancestor c.
__device__ __forceinline__ void heap_push(HeapE* hp, uint32_t& nh, HeapE x, uint32_t lane) {
  const uint32_t j1 = nh + 1;   // 1-based position of the new element
  const bool valid = lane >= 1 && lane < 32 && (j1 >> lane) >= 1u;
  HeapE a{0.0f, 0u};
  if (valid) a = hp[(j1 >> lane) - 1];
  const uint64_t b = __ballot(valid && x.d < a.d);
  const uint32_t c = (uint32_t)__builtin_ctzll(~(b >> 1));   // consecutive passed ancestors from lane 1
  if (lane >= 1 && lane <= c) hp[(j1 >> (lane - 1)) - 1] = a;
  if (lane == c) hp[(j1 >> c) - 1] = x;
  nh = j1;   // (one wave: its LDS operations complete in order, so the next push reads these stores)
}
// A run of container/heap.Push calls with the insertion path cached in
// registers (lane l >= 1: the value of ancestor level l of the next insertion
// position j, 1-based, node (j >> l) - 1), so a push costs one ballot and its
// stores, not an LDS round trip: after a push the next position j + 1 shares
// every ancestor above the lowest zero bit of j, whose new values are known
// (shifted down one level through c, x at level c); only the levels below
// it are read from LDS (after this push's stores; none of them is on j's path,
// except the root when j = 2^t - 1, also taken from the registers).  The same
// result as heap_push push by push (restated and checked against Go's
// container/heap with ties in tools/sim_heap_path.py).
__device__ __forceinline__ HeapE dpp_from_up(HeapE v) {   // lane l <- lane l + 1 (wave_shl:1)
  HeapE r;
  r.d = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v.d), 0x130, 0xf, 0xf, true));
  r.slot = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.slot, 0x130, 0xf, 0xf, true);
  return r;
}
__device__ __forceinline__ HeapE dpp_from_down(HeapE v) {   // lane l <- lane l - 1 (wave_shr:1)
  HeapE r;
  r.d = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v.d), 0x138, 0xf, 0xf, true));
  r.slot = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.slot, 0x138, 0xf, 0xf, true);
  return r;
}
__device__ __forceinline__ HeapE path_load(const HeapE* hp, uint32_t j, uint32_t lane) {
  const uint32_t a = lane >= 1 && lane < 32 ? j >> lane : 0u;
  return a ? hp[a - 1] : HeapE{0.0f, 0u};
}
__device__ __forceinline__ void path_push(HeapE* hp, uint32_t& j, HeapE& pv, HeapE x, uint32_t lane) {
  const uint32_t jn = j + 1;
  const uint32_t aj = lane >= 1 && lane < 32 ? j >> lane : 0u;
  const uint64_t b = __ballot(aj >= 1 && x.d < pv.d);
  const uint32_t c = (uint32_t)__builtin_ctzll(~(b >> 1));
  if (lane >= 1 && lane <= c) hp[(j >> (lane - 1)) - 1] = pv;
  if (lane == c) hp[(j >> c) - 1] = x;
  const HeapE up = dpp_from_up(pv), dn = dpp_from_down(pv);
  const uint32_t an = lane >= 1 && lane < 32 ? jn >> lane : 0u;
  HeapE nv{0.0f, 0u};
  if (an >= 1) {
    if (an == aj) nv = lane < c ? up : (lane == c ? x : pv);
    else if (an == (j >> (lane - 1))) nv = lane - 1 < c ? pv : (lane - 1 == c ? x : dn);
    else nv = hp[an - 1];
  }
  pv = nv;
  j = jn;
}

// container/heap.Pop: swap(0, n-1), down(0, n-1), remove the last.  down()
// moves the larger-index child only when strictly Less than the smaller-index
// one, and stops when the chosen child is not Less than the element.
__device__ __forceinline__ HeapE heap_pop(HeapE* hp, uint32_t& nh, uint32_t lane) {
  const uint32_t n1 = nh - 1;
  const HeapE top = hp[0];
  const HeapE x = hp[n1];
  uint32_t i = 0;
  for (;;) {
    const uint32_t j1 = 2 * i + 1;
    if (j1 >= n1) break;
    uint32_t j = j1;
    HeapE e = hp[j1];
    if (j1 + 1 < n1) {
      const HeapE e2 = hp[j1 + 1];
      if (e2.d < e.d) { j = j1 + 1; e = e2; }
    }
    if (!(e.d < x.d)) break;
    if (lane == 0) hp[i] = e;
    i = j;
  }
  if (lane == 0) hp[i] = x;
  nh = n1;
  return top;
}

// wave-wide lexicographic minimum of (d, id)
__device__ __forceinline__ void wave_min2(float& d, uint32_t& id) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float od = __shfl_xor(d, o);
    const uint32_t oi = __shfl_xor(id, o);
    if (od < d || (od == d && oi < id)) { d = od; id = oi; }
  }
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
__device__ __forceinline__ double wave_sumd(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Occurrences of x among a[0 .. len) (LDS, 16-B aligned): 4 ids per read,
// no early exit, so the reads of the loop pipeline.
__device__ __forceinline__ uint32_t lds_count(const uint32_t* a, uint32_t len, uint32_t x) {
  const uint4* a4 = (const uint4*)a;
  uint32_t c = 0;
  const uint32_t n4 = len / 4;
#pragma unroll 4
  for (uint32_t j = 0; j < n4; ++j) {
    const uint4 v = a4[j];
    c += (v.x == x) + (v.y == x) + (v.z == x) + (v.w == x);
  }
  for (uint32_t j = n4 * 4; j < len; ++j) c += a[j] == x;
  return c;
}

// One workgroup of kDrlThreads per session.  The per-position and per-sub-
// query work is spread over all its lanes in a few phases whose global loads
// are all in flight together (a handful of round trips per round); wave 0
// alone runs the order-dependent part (the heap's pushes and pops).
constexpr uint32_t kDrlThreads = 256;
__device__ __forceinline__ void block_sync() { __syncthreads(); }
// the workgroup's global stores visible to its other waves (one CU: no cache maintenance)
__device__ __forceinline__ void wg_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

#ifndef PM_CHAIN_PRIO
#define PM_CHAIN_PRIO 0
#endif
__global__ void __launch_bounds__(kDrlThreads) k_team_round(const DrlArgs A) {
  if (PM_CHAIN_PRIO) __builtin_amdgcn_s_setprio(PM_CHAIN_PRIO);
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint64_t t_prev = A.stamps ? __builtin_amdgcn_s_memtime() : 0;
  auto stamp = [&](int k) {   // diagnostics: phase k's shader clocks (thread 0, MID rounds)
    if (!A.stamps || A.mode != DRL_MID) return;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)(t - t_prev));
    t_prev = t;
  };
  const uint32_t s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t n = A.n, m = A.m, kcap = A.kcap, P = A.P, qn = A.qn, nsq = P * qn;
  // (every array starts 16-B aligned: lds_count and the vector decode read 16 B at a time)
  const uint32_t n4 = (n + 3) & ~3u, q4 = (nsq + 3) & ~3u;
  HeapE* hp = (HeapE*)lds;                                   // [kcap] the heap
  uint32_t* nbuf = (uint32_t*)(lds + (size_t)kcap * 8);     // [n][m] the round's neighbour lists
  uint32_t* bat = nbuf + (((size_t)n * m + 3) & ~(size_t)3); // [n] the round's ids
  float* dbuf = (float*)(bat + n4);                          // [n] their distances
  uint32_t* pbuf = bat + 2 * n4;                             // [n] partitions; then slots of new vertices
  uint32_t* flg = bat + 3 * n4;                              // [n] bit 0 mismatch, 1 non-zero, 2 known
  int32_t* srcj = (int32_t*)(bat + 4 * n4);                  // [n] the answering sub-query (session-local) or -1
  uint32_t* sst = bat + 5 * n4;                              // [nsq] status of the session's sub-queries
  uint32_t* sref = sst + q4;                                 // [nsq] DUP: the repeated sub-query (session-local)
  float* sdist = (float*)(sref + q4);                        // [nsq]
  uint32_t* sgid = sref + 2 * q4;                            // [nsq] global id (~0: dummy)
  __shared__ uint32_t s_wcnt[kDrlThreads / 64];
  __shared__ uint64_t s_wmask[kDrlThreads / 64];
  __shared__ uint32_t s_nknown, s_nheap;

  DrlSess* SS = A.sess + s;
  uint64_t rng = SS->rng;
  uint32_t nknown = SS->nknown, nheap = SS->nheap;
  HeapE* gheap = (HeapE*)(A.heap + (uint64_t)s * kcap);
  uint64_t* ktab = A.ktab + (uint64_t)s * 2 * kcap;
  const uint32_t kmask = 2 * kcap - 1;
  uint32_t* knb = A.knb + (uint64_t)s * kcap * m;
  float* kdist = A.kdist + (uint64_t)s * kcap;
  uint32_t* kid = A.kid + (uint64_t)s * kcap;
  uint32_t* gbat = A.batch + (uint64_t)s * n;
  uint64_t* ctab = A.ctab[s];
  const uint32_t cap = A.cmask + 1;
  const uint32_t base = s * nsq;   // this session's first sub-query of the shared step
  const uint32_t PS = (uint32_t)A.PS;

  if (A.mode == DRL_BEGIN) {
    // knn_reset: an empty known set and heap
    for (uint32_t i = tid; i < 2 * kcap; i += kDrlThreads) ktab[i] = 0;
    wg_fence();
    block_sync();
    if (wave == 0) {
      // knn_begin_finish (search.go:130-146): the first `parallel` start
      // vertices in (distance, position) order become known (with their true
      // neighbour lists: GetStartVertex is non-private) and go on the heap
      nknown = 0;
      nheap = 0;
      const float* sd = A.start_dist + (uint64_t)s * A.ns;
      const uint32_t* sid = A.start_ids + (uint64_t)s * A.ns;
      const uint32_t take = min(A.parallel, A.ns);
      float pd = 0.0f;
      uint32_t ppos = 0;
      for (uint32_t t = 0; t < take; ++t) {
        float bd = __builtin_inff();
        uint32_t bp = 0xffffffffu;
        for (uint32_t j = lane; j < A.ns; j += 64) {
          const float d = sd[j];
          const bool after = t == 0 || d > pd || (d == pd && j > ppos);
          if (after && (d < bd || (d == bd && j < bp))) { bd = d; bp = j; }
        }
        wave_min2(bd, bp);
        pd = bd; ppos = bp;
        const uint32_t id = sid[bp], slot = nknown++;
        if (lane < m) knb[(uint64_t)slot * m + lane] = A.graph[(uint64_t)id * m + lane];
        if (lane == 0) {
          kdist[slot] = bd;
          kid[slot] = id;
          tab_put(ktab, kmask, id, slot);
        }
        heap_push(hp, nheap, HeapE{bd, slot}, lane);
      }
      if (lane == 0) { s_nknown = nknown; s_nheap = nheap; }
    }
    wg_fence();
    block_sync();
    nknown = s_nknown;
    nheap = s_nheap;
  } else {
    // ---- phase 1: the heap, the ids, the session's sub-query results; the
    // localCache entries of its ST_OK answers (post_results, pir.go:468-470)
    for (uint32_t i = tid; i < nheap; i += kDrlThreads) hp[i] = gheap[i];
    for (uint32_t i = tid; i < n; i += kDrlThreads) bat[i] = gbat[i];
    for (uint32_t j = tid; j < nsq; j += kDrlThreads) {
      const PmOutHdr h = A.hdr[base + j];
      const uint64_t g = A.gid[base + j];
      sst[j] = h.status;
      sref[j] = h.ref - base;
      sdist[j] = h.dist;
      sgid[j] = g == ~0ull ? 0xffffffffu : (uint32_t)g;
      if (h.status == ST_OK) {
        const uint32_t p = j / qn;
        tab_put(ctab + (uint64_t)p * cap, A.cmask, (uint32_t)A.subs[base + j].idx, h.ref);
      }
    }
    block_sync();
    stamp(1);
    // ---- phase 2: each position's response (bq_emit_fast: the last sub-query
    // made for its id; an in-step duplicate follows the one it repeats), its
    // distance, whether the id is known, whether an earlier position has it
    for (uint32_t i = tid; i < n; i += kDrlThreads) {
      const uint32_t id = bat[i];
      const uint32_t p = id / PS;
      int32_t src = -1;
      for (uint32_t j = 0; j < qn; ++j)
        if (sgid[p * qn + j] == id) src = (int32_t)(p * qn + j);   // last wins
      for (int hop = 0; src >= 0 && sst[src] == ST_DUP && hop < 2; ++hop) src = (int32_t)sref[src];
      srcj[i] = src;
      dbuf[i] = src >= 0 ? sdist[src] : 0.0f;
      const bool dup = lds_count(bat, i, id) != 0;   // an earlier position has it: known by then
      uint32_t v;
      const bool known = dup || tab_find(ktab, kmask, id, &v);
      flg[i] = known ? 4u : 0u;   // bit 2: not new
    }
    block_sync();
    stamp(2);
    // ---- phase 3: GetVertexInfo's decode (Entry2VectorAndNeighbors) and the
    // success check against the true neighbour list.  Vector form: m / 4
    // lanes per position, 16-B loads all in flight, the position's flags ORed
    // across its lanes by shuffles (m / 4 a power of two <= 64, 16-B aligned rows)
    const uint32_t* rows32 = (const uint32_t*)A.rows;
    const uint32_t cpp = m / 4;   // 16-B chunks per neighbour list
    if (A.vec16) {
      constexpr int kU = 4;   // items per thread in flight
      for (uint32_t e0 = 0; e0 < n * cpp; e0 += kDrlThreads * kU) {
        uint4 rv[kU], tv[kU];
        uint32_t ii[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t e = e0 + u * kDrlThreads + tid;
          rv[u] = make_uint4(0, 0, 0, 0); tv[u] = make_uint4(1, 1, 1, 1); ii[u] = 0xffffffffu;
          if (e < n * cpp) {
            const uint32_t i = e / cpp, c = e - i * cpp;
            ii[u] = i;
            const int32_t src = srcj[i];
            if (src >= 0) rv[u] = *(const uint4*)(rows32 + (uint64_t)(base + src) * 2 * A.E + A.dim + 4 * c);
            tv[u] = *(const uint4*)(A.graph + (uint64_t)bat[i] * m + 4 * c);
          }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t e = e0 + u * kDrlThreads + tid;
          uint32_t f = 0;
          if (ii[u] != 0xffffffffu) {
            ((uint4*)nbuf)[e] = rv[u];
            f = ((rv[u].x != tv[u].x) | (rv[u].y != tv[u].y) | (rv[u].z != tv[u].z) | (rv[u].w != tv[u].w)) ? 1u : 0u;
            f |= (rv[u].x | rv[u].y | rv[u].z | rv[u].w) ? 2u : 0u;
          }
          for (uint32_t o = 1; o < cpp; o <<= 1) f |= __shfl_xor(f, o);   // the position's cpp lanes are adjacent
          if (ii[u] != 0xffffffffu && (e % cpp) == 0) flg[ii[u]] |= f;
        }
      }
    } else {
      for (uint32_t e = tid; e < n * m; e += kDrlThreads) {
        const uint32_t i = e / m, k = e - i * m;
        const int32_t src = srcj[i];
        const uint32_t v = src >= 0 ? rows32[(uint64_t)(base + src) * 2 * A.E + A.dim + k] : 0u;
        const uint32_t t = A.graph[(uint64_t)bat[i] * m + k];
        nbuf[e] = v;
        if (v != t) atomicOr(&flg[i], 1u);
        if (v != 0) atomicOr(&flg[i], 2u);
      }
    }
    block_sync();
    stamp(3);
    // ---- phase 4: the new vertices in position order (SearchKNN's update,
    // search.go:185-207): known slots, rows, the known table
    uint64_t succ = 0;
    bool nw = false;
    uint32_t i4 = tid;
    if (tid < n) {
      const uint32_t f = flg[tid];
      succ = (f & 1u) == 0;
      nw = (f & 2u) && !(f & 4u);
    }
    const uint64_t bal = __ballot(nw);
    if (lane == 0 && wave < kDrlThreads / 64) { s_wcnt[wave] = (uint32_t)__builtin_popcountll(bal); s_wmask[wave] = bal; }
    succ = wave_sum(succ);
    if (lane == 0 && succ) atomicAdd((unsigned long long*)&SS->succ, (unsigned long long)succ);
    block_sync();
    stamp(8);
    uint32_t before = nknown;
    for (uint32_t w = 0; w < wave; ++w) before += s_wcnt[w];
    uint32_t total_new = 0;
    for (uint32_t w = 0; w < kDrlThreads / 64; ++w) total_new += s_wcnt[w];
    float* ndist = (float*)srcj;   // [total_new] the new vertices' distances by rank (srcj is done with)
    if (nw) {
      const uint32_t slot = before + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      pbuf[i4] = slot;
      ndist[slot - nknown] = dbuf[i4];
      kdist[slot] = dbuf[i4];
      kid[slot] = bat[i4];
      tab_put(ktab, kmask, bat[i4], slot);
    }
    block_sync();
    stamp(9);
    for (uint32_t e = tid; e < n * m; e += kDrlThreads) {   // the new vertices' neighbour lists
      const uint32_t i = e / m;
      if ((s_wmask[i >> 6] >> (i & 63)) & 1ull) knb[(uint64_t)pbuf[i] * m + (e - i * m)] = nbuf[e];
    }
    // ---- the heap pushes, in position order (wave 0): new vertex r has slot
    // nknown + r; its distance is read from a register of lane r % 64
    stamp(10);
    if (wave == 0 && total_new) {
      uint32_t j = nheap + 1;
      HeapE pv = path_load(hp, j, lane);
      for (uint32_t r0 = 0; r0 < total_new; r0 += 64) {
        const float dl = r0 + lane < total_new ? ndist[r0 + lane] : 0.0f;
        const uint32_t cnt = min(64u, total_new - r0);
        for (uint32_t r = 0; r < cnt; ++r) {
          const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dl), (int)r));
          path_push(hp, j, pv, HeapE{d, nknown + r0 + r}, lane);
        }
      }
      nheap = j - 1;
    }
    nknown += total_new;
    stamp(11);
    wg_fence();   // the new known rows are read back by this launch's pops
    block_sync();
    stamp(4);
  }

  if (A.mode != DRL_END) {
    // ---- the next batch (search.go:153-171): wave 0 pops, then every lane
    // gathers the popped vertices' neighbours (or the SplitMix ids)
    // (wave 0: each pop's neighbour row is loaded while the next pops run)
    if (wave == 0) {
      uint64_t r0 = rng;   // the id stream consumed by the empty-heap positions in order
      uint32_t v[pmk::kDrlMaxParallel];
#pragma unroll
      for (uint32_t r = 0; r < pmk::kDrlMaxParallel; ++r) {
        if (r >= A.parallel) break;
        if (nheap) {
          const uint32_t slot = heap_pop(hp, nheap, lane).slot;
          v[r] = lane < m ? knb[(uint64_t)slot * m + lane] : 0u;   // in flight during the next pops
        } else {
          v[r] = (uint32_t)(sm64(r0 + (uint64_t)lane * 0x9e3779b97f4a7c15ULL) % A.N);
          r0 += (uint64_t)m * 0x9e3779b97f4a7c15ULL;
        }
      }
#pragma unroll
      for (uint32_t r = 0; r < pmk::kDrlMaxParallel; ++r)
        if (r < A.parallel && lane < m) bat[r * m + lane] = v[r];
      if (lane == 0) s_nheap = nheap;
      rng = r0;
    }
    block_sync();
    nheap = s_nheap;
    stamp(5);
    // ---- SimpleBatchPianoPIR.Query's bucketing into the next shared step
    uint32_t* pcnt = flg;   // [P] ids per partition (flg is done with; P <= n)
    for (uint32_t p = tid; p < P; p += kDrlThreads) pcnt[p] = 0;
    block_sync();
    for (uint32_t i = tid; i < n; i += kDrlThreads) {
      const uint32_t p = bat[i] / PS;
      pbuf[i] = p;
      atomicAdd(&pcnt[p], 1u);
    }
    block_sync();
    double bytes = 0.0;
    uint32_t nreal = 0;
    for (uint32_t i = tid; i < n; i += kDrlThreads) {
      const uint32_t id = bat[i], p = pbuf[i];
      const uint32_t rank = lds_count(pbuf, i, p);
      if (rank < qn) {   // the first queryNumToMake ids of a partition; the rest are dropped
        const uint32_t j = base + p * qn + rank;
        const uint32_t local = id - p * PS;
        uint32_t slot;
        PmSub sub{s * P + p, SUB_REAL, local};
        if (tab_find(ctab + (uint64_t)p * cap, A.cmask, local, &slot)) {
          sub.kind = SUB_HOSTCACHE;
          sub.idx = slot;
        } else {
          bytes += A.part_bytes[p];
          nreal++;
        }
        A.subs[j] = sub;
        A.gid[j] = id;
      }
    }
    for (uint32_t p = tid; p < P; p += kDrlThreads) {   // dummy padding (batch-pir.go:182-190)
      const uint32_t cnt = pcnt[p];
      uint64_t dc = A.dummy[(uint64_t)s * P + p];
      for (uint32_t j = cnt; j < qn; ++j) {
        A.subs[base + p * qn + j] = PmSub{s * P + p, SUB_DUMMY, dc++};
        A.gid[base + p * qn + j] = ~0ull;
        bytes += A.part_bytes[p];
      }
      A.dummy[(uint64_t)s * P + p] = dc;
    }
    if (A.step_bytes) {   // (timing runs) the step's exact answer bytes and real sub-queries
      bytes = wave_sumd(bytes);
      const uint64_t nr = wave_sum(nreal);
      if (lane == 0) {
        atomicAdd(&A.step_bytes[(uint64_t)A.seq * A.S + s], bytes);
        atomicAdd(&A.step_real[(uint64_t)A.seq * A.S + s], (uint32_t)nr);
      }
    }
    stamp(6);
    for (uint32_t i = tid; i < n; i += kDrlThreads) gbat[i] = bat[i];
    for (uint32_t i = tid; i < nheap; i += kDrlThreads) gheap[i] = hp[i];
    stamp(7);
    if (A.stamps && A.mode == DRL_MID && threadIdx.x == 0) atomicAdd((unsigned long long*)&A.stamps[15], 1ull);
  } else {
    // ---- the top k by (distance, id) (search.go:211-233), -1 padded
    float* ld = (float*)lds;                          // the heap's LDS, no longer needed
    uint32_t* li = (uint32_t*)(lds + (size_t)kcap * 4);
    for (uint32_t j = tid; j < nknown; j += kDrlThreads) { ld[j] = kdist[j]; li[j] = kid[j]; }
    block_sync();
    if (wave == 0) {
      int64_t* out = A.answers + ((uint64_t)s * A.q + A.qi) * A.k;
      float pd = 0.0f;
      uint32_t pi = 0;
      for (uint32_t t = 0; t < A.k; ++t) {
        float bd = __builtin_inff();
        uint32_t bi = 0xffffffffu;
        bool any = false;
        for (uint32_t j = lane; j < nknown; j += 64) {
          const float d = ld[j];
          const uint32_t id = li[j];
          const bool after = t == 0 || d > pd || (d == pd && id > pi);
          if (after && (!any || d < bd || (d == bd && id < bi))) { bd = d; bi = id; any = true; }
        }
        const bool found = __ballot(any) != 0;
        wave_min2(bd, bi);   // lanes without a candidate hold (inf, ~0): never below a real one
        if (lane == 0) out[t] = found ? (int64_t)bi : -1;
        if (!found) {
          for (uint32_t u = t + 1 + lane; u < A.k; u += 64) out[u] = -1;
          break;
        }
        pd = bd; pi = bi;
      }
    }
  }
  if (tid == 0) {
    SS->rng = rng;
    SS->nknown = nknown;
    SS->nheap = A.mode == DRL_END ? 0u : nheap;
  }
}

static uint32_t team_round_lds_impl(uint32_t kcap, uint32_t n, uint32_t m) {
  const uint32_t n4 = (n + 3) & ~3u;   // heap, rows, per-position arrays, per-sub-query arrays (P * qn <= n)
  return kcap * 8 + ((n * m + 3) & ~3u) * 4 + 5 * n4 * 4 + 4 * n4 * 4;
}

static void team_round_impl(hipStream_t st, const DrlArgs& A, hipEvent_t a, hipEvent_t b) {
  const uint32_t lds = team_round_lds_impl(A.kcap, A.n, A.m);
  if (a) hipExtLaunchKernelGGL(k_team_round, dim3(A.S), dim3(kDrlThreads), lds, st, a, b, 0, A);
  else hipLaunchKernelGGL(k_team_round, dim3(A.S), dim3(kDrlThreads), lds, st, A);
}

}  // namespace pm

namespace pmk {
void team_round(hipStream_t st, const DrlArgs& A, PmEvents ev) { pm::team_round_impl(st, A, ev.a, ev.b); }
uint32_t team_round_lds(uint32_t kcap, uint32_t n, uint32_t m) { return pm::team_round_lds_impl(kcap, n, m); }
}  // namespace pmk
