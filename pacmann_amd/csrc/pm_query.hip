// pm_query.hip — one batched online step of PianoPIR over every partition
// (SimpleBatchPianoPIR.Query, batch-pir.go:189-216 -> Client.Query,
// pir.go:354-471), as four launches:
//
//   k_match   (wide)        HOT LOOP C for every (real sub-query, primary hint)
//                           pair against the state at the start of the step:
//                           one bit per hint.  Also stages the step descriptor
//                           from pinned host memory into device memory.
//
// No AES runs here: every PRF(tag, chunk) & (CS-1) the online phase needs is a
// lookup in the partition's resident PRF table (PmPart::tab, built by
// k_prep_offsets), because every tag is a hint index in [0, H).
//   k_resolve (1 WG/part.)  the sequential part of Client.Query: cache /
//                           budget checks, first matching hint (stale bits +
//                           re-evaluation of hints refreshed earlier in the
//                           step), refresh of tag / program point / counters.
//                           State is prefetched into LDS; the chain runs on one
//                           wave with no dependent global loads in the common case.
//   k_answer  (1 WG/sub)    set expansion (HOT LOOP D) + programmed point +
//                           replacement substitution, the server's XOR gather
//                           (HOT LOOP E, PrivateQuery pir.go:65-88), decode and
//                           parity refresh (pir.go:450-468), the L2 distance of
//                           the decoded vector to the search query, and the
//                           write of the result straight into host-mapped memory.
//                           The last workgroup to finish (arrival counter,
//                           agent-scope release/acquire) then decodes, in
//                           order, the rare sub-queries whose hint was already
//                           refreshed earlier in the same step.
#include <hip/hip_ext.h>

#include "pm_aes.h"
#include "pm_internal.h"
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>

namespace pm {

constexpr int kAnsBlock = 512;
#ifndef PM_ANSWER_NTLOAD
#define PM_ANSWER_NTLOAD 0   // k_answer_p's row gather with nontemporal loads (streamed past the caches)
#endif
#ifndef PM_STEP_KG
#define PM_STEP_KG 12   // k_step's answer role: rows per thread in flight together (configs[2]: 11 per thread)
#endif
#ifndef PM_ANSWER_KG
#define PM_ANSWER_KG 6   // k_answer gather: rows per thread in flight together (no VGPR spill at 8 waves;
                         // alone 76.0-76.7 us vs 77.3 at 8 and 81-82 at 10, which spills 9 VGPRs)
#endif
constexpr uint32_t kNone = 0xffffffffu;

#ifdef PM_STAMPS
#define STAMP(i)                                                                 \
  do {                                                                           \
    if (threadIdx.x == 0 && S.stamps) {                                          \
      uint64_t t_;                                                               \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      S.stamps[blockIdx.x * 64 + (i)] = t_;                                      \
    }                                                                            \
  } while (0)
// stamps of one workgroup of the other step kernels at fixed slots
#define STAMP_AT(cond, slot)                                                     \
  do {                                                                           \
    if ((cond) && threadIdx.x == 0 && S.stamps) {                                \
      uint64_t t_;                                                               \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      S.stamps[slot] = t_;                                                       \
    }                                                                            \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#define STAMP_AT(cond, slot) do { (void)(cond); } while (0)
#endif
// PM_STEP_STAMPS diagnostic builds: per k_step workgroup, s_memrealtime
// (100 MHz, one clock for every XCD) at slots 0 start, 1 after its wait,
// 2 end, 3 (match: after the counter add)
#ifdef PM_STEP_STAMPS
#define TS(i)                                                                     \
  do {                                                                            \
    if (threadIdx.x == 0 && S.stamps)                                             \
      S.stamps[(uint64_t)blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// slot 3: where the workgroup ran, XCC_ID << 32 | HW_ID
#define TS_HWID()                                                                  \
  do {                                                                             \
    if (threadIdx.x == 0 && S.stamps)                                              \
      S.stamps[(uint64_t)blockIdx.x * 4 + 3] =                                     \
          ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |           \
          (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);                      \
  } while (0)
// answer workgroups: slot 3 = time the resolver's flag was seen << 1 | guess kept
#define TS_SEEN(kept)                                                                          \
  do {                                                                                         \
    if (threadIdx.x == 0 && S.stamps)                                                          \
      S.stamps[(uint64_t)blockIdx.x * 4 + 3] = (__builtin_amdgcn_s_memrealtime() << 1) | (kept); \
  } while (0)
// answer phases (k_step): stamps[gridDim.x * 4 + blockIdx.x * 4 + i], at
// points that follow a barrier anyway (no added waits)
#define AS(i)                                                                                \
  do {                                                                                       \
    if (GRAN && threadIdx.x == 0 && S.stamps)                                                \
      S.stamps[(uint64_t)gridDim.x * 4 + blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AS(i) do {} while (0)
#define TS(i) do {} while (0)
#define TS_HWID() do {} while (0)
#define TS_SEEN(kept) do {} while (0)
#endif
// slots: k_resolve partition 0: 0..40; k_match block (0,0): 41..47; k_answer block 0: 48..63

// PM_ANSWER_STAMPS diagnostic builds: k_answer (three-kernel path) records
// s_memrealtime (100 MHz, one clock for all XCDs) at its phase boundaries,
// stamps[blockIdx * 8 + i]: 0 start, 1 resolution read, 2 query set in LDS,
// 3 gather reduced, 4 decoded, 5 results issued, 6 XCC_ID << 16 | CU/SE ids.
#ifdef PM_ANSWER_STAMPS
#define AST(i)                                                                                   \
  do {                                                                                           \
    if (!GRAN && threadIdx.x == 0 && S.stamps)                                                   \
      S.stamps[(uint64_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#else
#define AST(i) do {} while (0)
#endif


// PM_MR_STAMPS diagnostic builds: k_match_resolve_s records s_memrealtime at
// its phase boundaries (thread 0), stamps[blockIdx * 8 + i]: 0 start,
// 1 partition record loaded, 2 match issued + ballots done (wave 0),
// 3 every wave's match in LDS, 4 candidates' tags / program points loaded,
// 5 chain done and flushed, 6 expansion guesses loaded, 7 query sets issued.
#ifdef PM_MR_STAMPS
#define MRST(i)                                                                                  \
  do {                                                                                           \
    if (threadIdx.x == 0 && S.stamps)                                                            \
      S.stamps[(uint64_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#else
#define MRST(i) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// LDS staging limits of the fast resolve path (SIFT1M / MS-MARCO shapes);
// larger configurations take the global-memory path of the same kernel.
constexpr uint32_t kLdsPH = 8192, kLdsBitWords = 2048, kSpecSubs = 64;   // staging: 8 items per thread

// Descriptor accessors: kernel arguments when they carry it, else the device copies.
// (Two explicit branches: a select of the two addresses would merge them into
// one generic pointer and a flat load.)
__device__ __forceinline__ PmSub step_sub(const PmStep& S, uint32_t s) {
  if (S.args_valid) return S.subs_a[s];
  PmSub v = S.subs[s];
  __builtin_amdgcn_sched_barrier(0);
  return v;
}
__device__ __forceinline__ uint32_t step_sb(const PmStep& S, uint32_t p) {
  return S.args_valid ? S.sb_a[p] : S.sb[p];
}

// The descriptor as k_match sees it: kernel arguments, else the pinned host
// copy (the device copy is being written by this very kernel).
__device__ __forceinline__ PmSub desc_sub(const PmStep& S, uint32_t i) {
  if (S.args_valid) return S.subs_a[i];
  PmSub v = S.subs_h[i];
  __builtin_amdgcn_sched_barrier(0);
  return v;
}
__device__ __forceinline__ uint32_t desc_sb(const PmStep& S, uint32_t p) {
  if (S.args_valid) return S.sb_a[p];
  uint32_t v = S.sb_h[p];
  __builtin_amdgcn_sched_barrier(0);
  return v;
}

// Stores / loads of data handed between the roles of one fused launch
// (k_step): write-through sc1 stores drained before a flag or counter, and
// sc1 loads after the poll (MI355X_MICROARCH.md § inter-workgroup visibility,
// first row of the sc1 table).  Plain accesses in the separate kernels.
template <bool SC1> __device__ __forceinline__ void st32(PM_G uint32_t* p, uint32_t v) {
  if (SC1) __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool SC1> __device__ __forceinline__ void st64(PM_G uint64_t* p, uint64_t v) {
  if (SC1) __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool SC1> __device__ __forceinline__ uint32_t ld32(const PM_G uint32_t* p) {
  if (SC1) return __hip_atomic_load((uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}
template <bool SC1> __device__ __forceinline__ uint64_t ld64(const PM_G uint64_t* p) {
  if (SC1) return __hip_atomic_load((uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

// k_step hand-offs: data-tagged 8-byte granules {value, step token}, each
// written by ONE sc1 store, read with sc1 loads until the token is this
// step's (MI355X_MICROARCH.md, handoff-1to1: no drain, no flag, no counter).
// A spin longer than kSpinTicks (20 ms of s_memrealtime) flags an error in
// pinned host memory, which the host turns into a failed step.
constexpr uint64_t kSpinTicks = 2000000;
__device__ __forceinline__ void put_g(PM_G uint64_t* p, uint32_t v, uint32_t tok) {
  st64<true>(p, ((uint64_t)tok << 32) | v);
}
__device__ __forceinline__ uint32_t get_g(const PM_G uint64_t* p, const PmStep& S) {
  uint64_t v = ld64<true>(p);
  if ((uint32_t)(v >> 32) != S.token) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    do {
      __builtin_amdgcn_s_sleep(1);
      v = ld64<true>(p);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        __hip_atomic_store((uint32_t*)S.err_h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    } while ((uint32_t)(v >> 32) != S.token);
  }
  return (uint32_t)v;
}
// granule layouts (k_step): rec[s][8] = {c1, t1, p1, c2, t2, p2, hist0, sing};
// spec[s][64]; bits[s][words][2] (low, high halves); res[s][8] (PmRes fields)
enum : uint32_t { G_REC = 8, G_RES = 8 };
template <bool GRAN> __device__ __forceinline__ void put_res(const PmStep& S, uint32_t s, const PmRes& r) {
  if (GRAN) {
    const uint32_t* f = reinterpret_cast<const uint32_t*>(&r);
#pragma unroll
    for (int i = 0; i < 8; ++i) put_g(S.resg + (uint64_t)s * G_RES + i, f[i], S.token);
  } else {
    S.res[s] = r;
  }
}
// a resolution record read by the step's finisher (granules: sc1, token-checked)
template <bool GRAN> __device__ __forceinline__ PmRes res_after_acquire(const PmStep& S, uint32_t s) {
  if (!GRAN) return S.res[s];
  PmRes r;
  uint32_t* f = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = get_g(S.resg + (uint64_t)s * G_RES + i, S);
  return r;
}

constexpr uint32_t kMatchHints = 1024;   // hints per match workgroup (any block size)

// In-chunk index the k-th of a partition's pn sub-queries (those from pb0 on)
// gets if every earlier one succeeds: its chunk's QueryHistogram h0k plus the
// earlier valid first occurrences in the same chunk.  One whole wave, pn <= 64;
// lane t returns sub-query pb0 + t in `st` and whether it is valid in `validt`.
__device__ __forceinline__ uint32_t predict_ing(const PmStep& S, const PmPart& P, uint32_t pb0, uint32_t pn,
                                                uint32_t k, uint32_t chunk, uint32_t h0k, PmSub& st,
                                                bool& validt, const PmSub* ls = nullptr) {
  const uint32_t lane = threadIdx.x & 63;
  st = PmSub{0, SUB_NONE, ~0ull};
  if (lane < pn) st = ls ? ls[lane] : desc_sub(S, pb0 + lane);
  validt = lane < pn && st.kind == SUB_REAL && st.idx < P.N;
  const uint32_t cht = (uint32_t)(st.idx >> P.log2CS);
  bool first = validt;
  for (uint32_t t = 0; t + 1 < pn; ++t) {
    const uint64_t it = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(st.idx >> 32), t) << 32) |
                        __builtin_amdgcn_readlane((uint32_t)st.idx, t);
    const bool rt = __builtin_amdgcn_readlane(st.kind == SUB_REAL ? 1u : 0u, t) != 0;
    if (t < lane && rt && it == st.idx) first = false;
  }
  const uint64_t mk = __ballot(lane < k && validt && first && cht == chunk);
  return h0k + (uint32_t)__builtin_popcountll(mk);
}

// One match workgroup (HOT LOOP C): hints [blk*kMatchHints, +kMatchHints) of
// sub-query s against the state at the start of the step; `sub` is uniform.
template <int NT, int kMatchHPT, bool GRAN>
__device__ __forceinline__ void match_role(const PmStep& S, uint32_t s, uint32_t blk, PmSub sub,
                                           uint32_t (&s_cand)[NT / 64][6]) {
  const bool stamp_wg = blk == 0 && s == 0;
  STAMP_AT(stamp_wg, 41);
  if (sub.kind != SUB_REAL) return;
  const PmPart P = S.parts[sub.part];
  const uint32_t base = blk * NT * kMatchHPT;
  if (base >= P.PH) return;
  STAMP_AT(stamp_wg, 42);
  const uint32_t mask = P.CS - 1, chunk = (uint32_t)(sub.idx >> P.log2CS),
                 offset = (uint32_t)(sub.idx & mask);
  const PM_G uint16_t* crow = P.cur + cur_row(P.PH, P.curk, chunk);   // the hint search row of this chunk
  const bool live = sub.idx < P.N;
  // Block 0 of a sub-query also prepares k_resolve's prediction: its chunk's
  // QueryHistogram now, the rest below (loads overlap the match loads).
  const bool meta_wg = blk == 0;
  const uint32_t h0k = (meta_wg && live) ? P.hist[chunk] : 0;
  uint32_t sing_rec = 0;   // GRAN: thread 0's copy for the record
  // kMatchHPT hints per thread: their search-row values (contiguous u16).  A
  // hint matches iff its value is the offset: a refreshed hint's programmed
  // chunk is its backup tag's own chunk, kSkip in its row, so the program
  // point check (pir.go:407) needs no load.
  uint16_t rv[kMatchHPT];
#pragma unroll
  for (int u = 0; u < kMatchHPT; ++u) {
    const uint32_t h = base + u * NT + threadIdx.x;
    rv[u] = (live && h < P.PH) ? crow[cur_row_off(P.curk, h)] : kSkip;
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (meta_wg && wave == 0) {
    // In-chunk index this sub-query gets if every earlier one of its partition
    // succeeds (QueryHistogram + earlier valid first occurrences in the same
    // chunk), and the PRF values at the later sub-queries' chunks of the tag
    // that refresh would hand out: spec[s][j] (k_resolve's re-evaluation).
    const uint32_t pb0 = desc_sb(S, sub.part), pn = desc_sb(S, sub.part + 1) - pb0, k = s - pb0;
    if (pn <= kSpecSubs) {
      PmSub st;
      bool validt;
      const uint32_t sing = predict_ing(S, P, pb0, pn, k, chunk, h0k, st, validt);
      const uint32_t cht = (uint32_t)(st.idx >> P.log2CS);
      const uint32_t pred = (live && sing < P.Qpc && chunk < P.SS) ? P.PH + chunk * P.Qpc + sing : kNone;
      uint32_t v = kSkip;
      if (lane < pn && lane > k && validt && cht < P.SS && pred != kNone) v = P.tabT[tabT_index(P.H, pred, cht)];
      if (GRAN) {
        if (lane < pn) put_g(S.specg + (uint64_t)s * kSpecSubs + lane, v, S.token);
        sing_rec = sing;
      } else {
        if (lane < pn) S.spec[(uint64_t)s * kSpecSubs + lane] = v;
        if (lane == 0) { S.meta[2 * (uint64_t)s] = h0k; S.meta[2 * (uint64_t)s + 1] = sing; }
      }
    }
  }
  // match bits, and the wave's first two matches with their tag / program
  // point (k_resolve's usual candidates)
  uint32_t h0 = kNone, t0 = 0, p0 = 0, h1 = kNone, t1 = 0, p1 = 0;   // wave-uniform
#pragma unroll
  for (int u = 0; u < kMatchHPT; ++u) {
    if (base + u * NT >= P.PH) break;
    const uint32_t h = base + u * NT + threadIdx.x;
    const bool m = rv[u] == offset;
    uint64_t b = __ballot(m);
    if (lane == 0 && (h - lane) < P.PH) {
      if (GRAN) {
        PM_G uint64_t* g = S.bitsg + ((uint64_t)s * S.words + (h >> 6)) * 2;
        put_g(g, (uint32_t)b, S.token);
        put_g(g + 1, (uint32_t)(b >> 32), S.token);
      } else {
        S.bits[(uint64_t)s * S.words + (h >> 6)] = b;
      }
    }
    if (b && h1 == kNone) {   // in hint order within this wave
      const uint32_t hl = h - lane + (uint32_t)__builtin_ctzll(b);
      if (h0 == kNone) {
        h0 = hl;
        b &= b - 1;
        if (b) h1 = h - lane + (uint32_t)__builtin_ctzll(b);
      } else {
        h1 = hl;
      }
    }
  }
  if (h0 != kNone) { t0 = P.tag[h0]; p0 = P.pp[h0]; }
  if (h1 != kNone) { t1 = P.tag[h1]; p1 = P.pp[h1]; }
  if (lane == 0) {
    s_cand[wave][0] = h0; s_cand[wave][1] = t0; s_cand[wave][2] = p0;
    s_cand[wave][3] = h1; s_cand[wave][4] = t1; s_cand[wave][5] = p1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // merge the waves' pairs by hint index
    uint32_t o[6] = {kNone, 0, 0, kNone, 0, 0};
    for (uint32_t w = 0; w < NT / 64; ++w)
      for (int k = 0; k < 2; ++k) {
        const uint32_t h = s_cand[w][3 * k];
        if (h < o[0]) {
          o[3] = o[0]; o[4] = o[1]; o[5] = o[2];
          o[0] = h; o[1] = s_cand[w][3 * k + 1]; o[2] = s_cand[w][3 * k + 2];
        } else if (h < o[3]) {
          o[3] = h; o[4] = s_cand[w][3 * k + 1]; o[5] = s_cand[w][3 * k + 2];
        }
      }
    if (GRAN) {   // one record per sub-query (blk 0 covers every hint), prediction included
      PM_G uint64_t* g = S.recg + (uint64_t)s * G_REC;
      for (int i = 0; i < 6; ++i) put_g(g + i, o[i], S.token);
      put_g(g + 6, h0k, S.token);
      put_g(g + 7, sing_rec, S.token);
    } else {
      PM_G uint32_t* dst = S.cand + ((uint64_t)s * S.cblk + blk) * 6;
      for (int i = 0; i < 6; ++i) dst[i] = o[i];
    }
  }
  STAMP_AT(stamp_wg, 43);
}

__global__ void __launch_bounds__(kBlock) k_match(PmStep S) {
  __shared__ uint32_t s_cand[kBlock / 64][6];
  const uint32_t s = blockIdx.y;
  PmSub sub;
  if (S.args_valid) {
    sub = S.subs_a[s];
    __builtin_amdgcn_sched_barrier(0);
  } else {   // zero-copy read of the host descriptor; staged for the later kernels
    __shared__ PmSub s_sub;
    if (threadIdx.x == 0) {
      s_sub = S.subs_h[s];
      if (blockIdx.x == 0 && S.subs != S.subs_h) S.subs[s] = s_sub;
    }
    if (blockIdx.x == 0 && s == 0 && S.sb != S.sb_h)
      for (uint32_t i = threadIdx.x; i <= S.np; i += kBlock) S.sb[i] = S.sb_h[i];
    __syncthreads();
    sub = s_sub;
  }
  // the descriptor is workgroup-uniform; say so, so the partition header is
  // fetched once with scalar loads
  sub.part = __builtin_amdgcn_readfirstlane(sub.part);
  sub.kind = __builtin_amdgcn_readfirstlane(sub.kind);
  sub.idx = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(sub.idx >> 32)) << 32) |
            __builtin_amdgcn_readfirstlane((uint32_t)sub.idx);
  match_role<kBlock, kMatchHints / kBlock, false>(S, s, blockIdx.x, sub, s_cand);
}

// k_match with the sub-queries of a partition grouped, for steps over many
// partitions with several sub-queries each (batched serving: S x 16
// partitions, 6 sub-queries each).  A workgroup owns (partition, block of
// kMatchHints hints): it loads the hints' state (tag, program point: 8 B per
// hint) once for all of the partition's sub-queries, gathers each one's
// PRF-table values (2 B per hint, G sub-queries' loads in flight together)
// and writes exactly the bits, records and predictions of match_role.
#ifndef PM_MATCHPART_WAVES
#define PM_MATCHPART_WAVES 6
#endif
#ifndef PM_MATCHPART_G
#define PM_MATCHPART_G 6
#endif
// k_resolve's predictions for sub-queries k = k0, k0 + kstep, ... of a
// partition (one wave each): the chunk's QueryHistogram, the predicted
// in-chunk index and the PRF values the refreshed hints would need.
__device__ __forceinline__ void match_part_predict(const PmStep& S, const PmPart& P, uint32_t pb0, uint32_t pn,
                                                   uint32_t k0, uint32_t kstep, const PmSub* ls = nullptr) {
  if (pn > kSpecSubs) return;
  const uint32_t lane = threadIdx.x & 63, lg = P.log2CS;
  for (uint32_t k = k0; k < pn; k += kstep) {
    PmSub sub = ls ? ls[k] : desc_sub(S, pb0 + k);
    sub.kind = __builtin_amdgcn_readfirstlane(sub.kind);
    if (sub.kind != SUB_REAL) continue;
    const bool live = sub.idx < P.N;
    const uint32_t chunk = (uint32_t)(sub.idx >> lg);
    const uint32_t h0k = live ? P.hist[chunk] : 0;
    PmSub st;
    bool validt;
    const uint32_t sing = predict_ing(S, P, pb0, pn, k, chunk, h0k, st, validt, ls);
    const uint32_t cht = (uint32_t)(st.idx >> lg);
    const uint32_t pred = (live && sing < P.Qpc && chunk < P.SS) ? P.PH + chunk * P.Qpc + sing : kNone;
    uint32_t v = kSkip;
    if (lane < pn && lane > k && validt && cht < P.SS && pred != kNone) v = P.tabT[tabT_index(P.H, pred, cht)];
    const uint64_t s = pb0 + k;
    if (lane < pn) S.spec[s * kSpecSubs + lane] = v;
    if (lane == 0) { S.meta[2 * s] = h0k; S.meta[2 * s + 1] = sing; }
  }
}

// Hints [blk * NT * HPT, +NT * HPT) of partition p against each of its pn
// sub-queries: the match bits and each sub-query's first two matches with
// their tag and program point (the block's record in S.cand).  `tid` is the
// thread's index in its team of NT threads; a workgroup may run several
// teams side by side on different blocks (k_match_resolve), so every barrier
// here is reached by the whole workgroup: a team whose block lies past PH
// (`act` false) runs the same loop and barriers without loads or stores.
template <int HPT, int NT, int G>
__device__ __forceinline__ void match_part_block(const PmStep& S, const PmPart& P, uint32_t pb0, uint32_t pn,
                                                 uint32_t blk, uint32_t tid, uint32_t (&s_cand)[G][NT / 64][6]) {
  const uint32_t lane = tid & 63, wave = tid >> 6;
  const uint32_t base = blk * NT * HPT;
  const bool act = base < P.PH;   // team-uniform
  const uint32_t mask = P.CS - 1, lg = P.log2CS;
  for (uint32_t j0 = 0; j0 < pn; j0 += G) {
    uint32_t kind[G], off[G];
    uint16_t rv[G][HPT];
    // each sub-query's search-row values of this block's hints (contiguous
    // u16: 2 B per hint; a hint matches iff its value is the offset, see
    // match_role); the loads of all G sub-queries in flight together
#pragma unroll
    for (int g = 0; g < G; ++g) {
      PmSub sub{0, SUB_NONE, 0};
      if (j0 + g < pn) sub = desc_sub(S, pb0 + j0 + g);
      kind[g] = __builtin_amdgcn_readfirstlane(sub.kind);
      const uint64_t idx = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(sub.idx >> 32)) << 32) |
                           __builtin_amdgcn_readfirstlane((uint32_t)sub.idx);
      const bool lv = act && kind[g] == SUB_REAL && idx < P.N;
      const uint32_t chk = (uint32_t)(idx >> lg);
      off[g] = (uint32_t)(idx & mask);
      const PM_G uint16_t* crow = P.cur + cur_row(P.PH, P.curk, chk);
#pragma unroll
      for (int u = 0; u < HPT; ++u) {
        const uint32_t h = base + u * NT + tid;
        rv[g][u] = (lv && h < P.PH) ? crow[cur_row_off(P.curk, h)] : kSkip;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!act || j0 + g >= pn || kind[g] != SUB_REAL) continue;   // team-uniform
      const uint64_t s = pb0 + j0 + g;
      uint32_t h0 = kNone, t0 = 0, p0 = 0, h1 = kNone, t1 = 0, p1 = 0;   // wave-uniform
#pragma unroll
      for (int u = 0; u < HPT; ++u) {
        if (base + u * NT >= P.PH) break;
        const uint32_t h = base + u * NT + tid;
        uint64_t b = __ballot(rv[g][u] == off[g]);   // kSkip never equals an offset
        if (lane == 0 && (h - lane) < P.PH) S.bits[s * S.words + (h >> 6)] = b;
        if (b && h1 == kNone) {   // in hint order within this wave
          const uint32_t hl = h - lane + (uint32_t)__builtin_ctzll(b);
          if (h0 == kNone) {
            h0 = hl;
            b &= b - 1;
            if (b) h1 = h - lane + (uint32_t)__builtin_ctzll(b);
          } else {
            h1 = hl;
          }
        }
      }
      if (h0 != kNone) { t0 = P.tag[h0]; p0 = P.pp[h0]; }
      if (h1 != kNone) { t1 = P.tag[h1]; p1 = P.pp[h1]; }
      if (lane == 0) {
        s_cand[g][wave][0] = h0; s_cand[g][wave][1] = t0; s_cand[g][wave][2] = p0;
        s_cand[g][wave][3] = h1; s_cand[g][wave][4] = t1; s_cand[g][wave][5] = p1;
      }
    }
    __syncthreads();
    if (act && tid < (uint32_t)G && j0 + tid < pn) {   // merge each sub-query's wave pairs
      const uint32_t g = tid;
      const PmSub sub = desc_sub(S, pb0 + j0 + g);
      if (sub.kind == SUB_REAL) {
        uint32_t o[6] = {kNone, 0, 0, kNone, 0, 0};
        for (uint32_t w = 0; w < NT / 64; ++w)
          for (int k = 0; k < 2; ++k) {
            const uint32_t h = s_cand[g][w][3 * k];
            if (h < o[0]) {
              o[3] = o[0]; o[4] = o[1]; o[5] = o[2];
              o[0] = h; o[1] = s_cand[g][w][3 * k + 1]; o[2] = s_cand[g][w][3 * k + 2];
            } else if (h < o[3]) {
              o[3] = h; o[4] = s_cand[g][w][3 * k + 1]; o[5] = s_cand[g][w][3 * k + 2];
            }
          }
        PM_G uint32_t* dst = S.cand + ((uint64_t)(pb0 + j0 + g) * S.cblk + blk) * 6;
        for (int i = 0; i < 6; ++i) dst[i] = o[i];
      }
    }
    if (j0 + G < pn) __syncthreads();
  }
}

template <int HPT>
__global__ void __launch_bounds__(kBlock, PM_MATCHPART_WAVES) k_match_part(PmStep S) {
  constexpr int NT = kBlock, G = PM_MATCHPART_G;
  __shared__ uint32_t s_cand[G][NT / 64][6];
  const uint32_t p = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x, wave = tid >> 6;
  const uint32_t pb0 = desc_sb(S, p), pn = desc_sb(S, p + 1) - pb0;
  if (!S.args_valid && blk == 0 && S.subs != S.subs_h) {   // stage the descriptor for the later kernels
    for (uint32_t i = tid; i < pn; i += NT) S.subs[pb0 + i] = S.subs_h[pb0 + i];
    if (p == 0)
      for (uint32_t i = tid; i <= S.np; i += NT) S.sb[i] = S.sb_h[i];
  }
  if (pn == 0) return;
  const PmPart P = S.parts[p];
  if (blk * NT * HPT >= P.PH) return;
  // predictions spread over the partition's hint blocks (sub-query k: block
  // k % nb, wave k / nb)
  const uint32_t nb = (P.PH + NT * HPT - 1) / (NT * HPT);
  match_part_predict(S, P, pb0, pn, blk + nb * wave, nb * (NT / 64));
  match_part_block<HPT, NT, G>(S, P, pb0, pn, blk, tid, s_cand);
}

// k_match_part for steps whose partitions all have PH % 8 == 0 (16-B aligned
// search rows): one WAVE per (partition, kMatchHints block).  Lane l holds
// hints 8l.. and 512 + 8l.. of its block (two 16-B loads per sub-query, G
// sub-queries in flight), so the block's match bits are 128 contiguous bytes
// (lane l writes bytes l and 64 + l) and its first two matches come from two
// ballots of the lanes' 8-bit masks: no LDS, no barrier, NW blocks per
// workgroup.  Same bits, records and predictions as k_match_part.
#ifndef PM_MATCHPART8_NW
#define PM_MATCHPART8_NW 4
#endif
#ifndef PM_MATCHPART8_G
#define PM_MATCHPART8_G 4   // sub-queries' search rows in flight together (BIGANN-100M: 4 35-38 us, 6 38-40 us)
#endif
#ifndef PM_MATCHPART8_WAVES
#define PM_MATCHPART8_WAVES 1   // min waves per SIMD (launch bounds)
#endif
constexpr uint32_t kPart8Subs = 256;   // a partition's descriptors held in LDS (more: read in place)
__device__ __forceinline__ uint32_t match8(uint4 v, uint32_t off) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    m |= (((w[i] & 0xffffu) == off) ? 1u : 0u) << (2 * i) | (((w[i] >> 16) == off) ? 1u : 0u) << (2 * i + 1);
  return m;
}
#ifndef PM_MATCH8_NT
#define PM_MATCH8_NT 0   // k_match_part8's search-row loads nontemporal
#endif
template <int NW>
__global__ void __launch_bounds__(64 * NW, PM_MATCHPART8_WAVES) k_match_part8(PmStep S) {
  constexpr int G = PM_MATCHPART8_G;
  constexpr uint32_t kHalf = kMatchHints / 2;   // 512: the second load's hints
  static_assert(kMatchHints == 1024, "one wave x 16 hints per lane");
  const uint32_t p = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the partition's descriptors, read once per workgroup into LDS instead of
  // once per wave and sub-query (BIGANN-100M: 35-38 vs 40-42 us per team
  // step); launched only when every partition has <= kPart8Subs sub-queries
  __shared__ uint32_t s_sb[2];
  __shared__ PmSub s_sub[kPart8Subs];
  if (tid < 2) s_sb[tid] = desc_sb(S, p + tid);
  __syncthreads();
  const uint32_t pb0 = s_sb[0], pn = min(s_sb[1] - pb0, kPart8Subs);
  for (uint32_t i = tid; i < pn; i += 64 * NW) s_sub[i] = desc_sub(S, pb0 + i);
  __syncthreads();
  if (!S.args_valid && blockIdx.x == 0 && S.subs != S.subs_h) {   // stage the descriptor for the later kernels
    for (uint32_t i = tid; i < pn; i += 64 * NW) S.subs[pb0 + i] = s_sub[i];
    if (p == 0)
      for (uint32_t i = tid; i <= S.np; i += 64 * NW) S.sb[i] = S.sb_h[i];
  }
  if (pn == 0) return;
  const PmPart P = S.parts[p];
  const uint32_t nb = (P.PH + kMatchHints - 1) / kMatchHints, nwg = (nb + NW - 1) / NW;
  if (blockIdx.x >= nwg) return;
  match_part_predict(S, P, pb0, pn, blockIdx.x + nwg * wave, nwg * NW, s_sub);
  const uint32_t blk = blockIdx.x * NW + wave;
  if (blk >= nb) return;   // whole wave; nothing below synchronises
  const uint32_t base = blk * kMatchHints, mask = P.CS - 1, lg = P.log2CS;
  const uint32_t hA = base + 8 * lane, hB = hA + kHalf;   // first hint of each load
  for (uint32_t j0 = 0; j0 < pn; j0 += G) {
    uint32_t kind[G], off[G];
    uint4 rv[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      PmSub sub{0, SUB_NONE, 0};
      if (j0 + g < pn) sub = s_sub[j0 + g];
      kind[g] = __builtin_amdgcn_readfirstlane(sub.kind);
      const uint64_t idx = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(sub.idx >> 32)) << 32) |
                           __builtin_amdgcn_readfirstlane((uint32_t)sub.idx);
      const bool lv = kind[g] == SUB_REAL && idx < P.N;
      off[g] = (uint32_t)(idx & mask);
      // (16-B blocks of the row are 16 curk B apart: cur_index)
      const PM_G uint4* crow = reinterpret_cast<const PM_G uint4*>(P.cur + cur_row(P.PH, P.curk, (uint32_t)(idx >> lg)));
      // unconditional 16-B loads (a dead lane reads the partition's first
      // vector), then kSkip x 8 by value: a select of the loaded VALUE keeps
      // them global_load_dwordx4
      const bool okA = lv && hA < P.PH, okB = lv && hB < P.PH;
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const PM_G u32x4* pa = reinterpret_cast<const PM_G u32x4*>(okA ? crow + (hA >> 3) * P.curk : reinterpret_cast<const PM_G uint4*>(P.cur));
      const PM_G u32x4* pb = reinterpret_cast<const PM_G u32x4*>(okB ? crow + (hB >> 3) * P.curk : reinterpret_cast<const PM_G uint4*>(P.cur));
      const u32x4 xa = PM_MATCH8_NT ? __builtin_nontemporal_load(pa) : *pa;
      const u32x4 xb = PM_MATCH8_NT ? __builtin_nontemporal_load(pb) : *pb;
      const uint4 a = make_uint4(xa.x, xa.y, xa.z, xa.w), b = make_uint4(xb.x, xb.y, xb.z, xb.w);
      rv[g][0] = okA ? a : make_uint4(~0u, ~0u, ~0u, ~0u);
      rv[g][1] = okB ? b : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (j0 + g >= pn || kind[g] != SUB_REAL) continue;   // wave-uniform
      const uint64_t s = pb0 + j0 + g;
      const uint32_t mA = match8(rv[g][0], off[g]), mB = match8(rv[g][1], off[g]);
      PM_G uint8_t* bb = reinterpret_cast<PM_G uint8_t*>(S.bits + s * S.words);
      // every byte of a 64-hint word that starts below PH (zero past PH)
      if ((hA & ~63u) < P.PH) bb[hA >> 3] = (uint8_t)mA;
      if ((hB & ~63u) < P.PH) bb[hB >> 3] = (uint8_t)mB;
      uint32_t h0 = kNone, h1 = kNone;   // the block's first two matches, wave-uniform
      auto scan = [&](uint32_t mu, uint32_t hbase) {   // lanes in hint order
        uint64_t bal = __ballot(mu != 0);
        while (bal && h1 == kNone) {
          const uint32_t fl = (uint32_t)__builtin_ctzll(bal);
          uint32_t mm = __builtin_amdgcn_readlane(mu, fl);
          const uint32_t hb = hbase + 8 * fl;
          while (mm && h1 == kNone) {
            const uint32_t hh = hb + (uint32_t)__builtin_ctz(mm);
            mm &= mm - 1;
            if (h0 == kNone) h0 = hh;
            else h1 = hh;
          }
          bal &= bal - 1;
        }
      };
      scan(mA, base);
      if (h1 == kNone) scan(mB, base + kHalf);
      uint32_t t0 = 0, p0 = 0, t1 = 0, p1 = 0;
      if (h0 != kNone) { t0 = P.tag[h0]; p0 = P.pp[h0]; }
      if (h1 != kNone) { t1 = P.tag[h1]; p1 = P.pp[h1]; }
      if (lane < 6) {
        const uint32_t v = lane == 0 ? h0 : lane == 1 ? t0 : lane == 2 ? p0 : lane == 3 ? h1 : lane == 4 ? t1 : p1;
        S.cand[(s * S.cblk + blk) * 6 + lane] = v;
      }
    }
  }
}

// First set bit at position >= start in a sub-query's match bitmask (one wave).
__device__ __forceinline__ uint32_t find_next(const uint64_t* __restrict__ bw, uint32_t nw, uint32_t start) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w0 = start >> 6; w0 < nw; w0 += 64) {
    const uint32_t w = w0 + lane;
    uint64_t v = w < nw ? bw[w] : 0;
    if (w == (start >> 6)) v &= ~0ull << (start & 63);
    const uint64_t m = __ballot(v != 0);
    if (m) {
      const uint32_t fl = (uint32_t)__builtin_ctzll(m);
      const uint64_t vf = __shfl(v, fl);
      return (w0 + fl) * 64 + (uint32_t)__builtin_ctzll(vf);
    }
  }
  return kNone;
}

// The same over sub-query `sub`'s match bits in global memory (granules in k_step).
template <bool GRAN>
__device__ __forceinline__ uint32_t find_next_g(const PmStep& S, uint64_t sub, uint32_t nw, uint32_t start) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w0 = start >> 6; w0 < nw; w0 += 64) {
    const uint32_t w = w0 + lane;
    uint64_t v = 0;
    if (w < nw) {
      if (GRAN) {
        const PM_G uint64_t* g = S.bitsg + (sub * S.words + w) * 2;
        v = get_g(g, S) | ((uint64_t)get_g(g + 1, S) << 32);
      } else {
        v = S.bits[sub * S.words + w];
      }
    }
    if (w == (start >> 6)) v &= ~0ull << (start & 63);
    const uint64_t m = __ballot(v != 0);
    if (m) {
      const uint32_t fl = (uint32_t)__builtin_ctzll(m);
      const uint64_t vf = __shfl(v, fl);
      return (w0 + fl) * 64 + (uint32_t)__builtin_ctzll(vf);
    }
  }
  return kNone;
}

// The same from the hint search rows (k_match_resolve_s, which keeps no match
// bits): the first primary hint h >= start whose search-row value in `chunk`
// is `off`, against the state at the start of the step (nothing writes cur
// before the step's k_answer).  One wave, 8 hints per lane (PH % 8 == 0).
__device__ __forceinline__ uint32_t find_cur(const PmPart& P, uint32_t chunk, uint32_t off, uint32_t start) {
  const uint32_t lane = threadIdx.x & 63;
  const PM_G uint16_t* row = P.cur + cur_row(P.PH, P.curk, chunk);
  for (uint32_t h0 = start & ~7u; h0 < P.PH; h0 += 512) {
    const uint32_t h = h0 + lane * 8;
    uint32_t f = kNone;
    if (h < P.PH) {
      const uint4 v = *reinterpret_cast<const PM_G uint4*>(row + cur_row_off(P.curk, h));
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 7; e >= 0; --e) {
        const uint32_t val = (w[e >> 1] >> (16 * (e & 1))) & 0xffffu;
        if (val == off && h + e >= start) f = h + e;
      }
    }
    const uint64_t m = __ballot(f != kNone);
    if (m) return __builtin_amdgcn_readlane(f, (uint32_t)__builtin_ctzll(m));
  }
  return kNone;
}

// Minimum over the wave of a per-lane candidate.
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor(x, o));
  return x;
}


constexpr int kMaxSubPerPart = 256;

// Resolver LDS.  MODE 0: state read from global memory (large partitions);
// 1: the fast prologue (match records) or, where that does not fit, the
// staged one; 2: the fast prologue only (k_step: n <= kSpecSubs sub-queries,
// nw <= 128 match words, one match record per sub-query).
template <int MODE>
struct ResolveLds {
  static constexpr int NS = MODE >= 2 ? kSpecSubs : kMaxSubPerPart;
  static constexpr bool STG = MODE == 1;
  static constexpr uint32_t NB = kLdsBitWords;
  uint64_t s_idx[NS];
  uint32_t s_kind[NS], s_chunk[NS], s_st[NS], s_hist0[NS], s_c1[NS], s_c2[NS], s_t1[NS],
      s_p1[NS], s_t2[NS], s_p2[NS], s_sing[NS];
  uint32_t m_h[NS], m_tag[NS], m_pp[NS], m_sub[NS], m_pt[NS];
  uint32_t s_fqn, fin, s_chain[NS];
  PmRes s_res[NS];
  // staging: match bits, tags / program points; speculative re-evaluation values
  uint64_t bits_l[STG ? NB : 1];
  uint32_t tag_l[STG ? kLdsPH : 1], pp_l[STG ? kLdsPH : 1];
  uint16_t spec_v[kSpecSubs * kSpecSubs];
};

// Step completion counter, 64 bits at done[0..1]: the high half counts the
// live partitions' resolvers, the low half holds (answer workgroups arrived)
// - (workgroups the resolvers declared involved in refresh chains) + 2^31.
// A resolver adds 2^32 - (its involved workgroups), an involved answer
// workgroup adds 1 once its refresh is released; the bias keeps the low half
// from borrowing, so the value is np_live << 32 | 2^31 exactly after the last
// add of the step, in any order of the adds.  That add's workgroup decodes
// the chain list (done[2] entries from done[3]) and re-arms the counters.
// (k_match_resolve_s steps set np_live 0: their resolvers all finish before
// the answer kernel starts, so only chains are counted, the value returns to
// 2^31 after the last involved arrival, and no resolver waits for an atomic.)
constexpr uint64_t kChainBias = 1ull << 31;
__device__ __forceinline__ uint64_t chain_add(const PmStep& S, uint64_t d) {
  const uint64_t prev = __hip_atomic_fetch_add(reinterpret_cast<PM_G uint64_t*>(S.done), d, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
  return (prev + d == (((uint64_t)S.np_live << 32) | kChainBias)) ? 1u : 0u;
}
__device__ __forceinline__ void chain_rearm(const PmStep& S) {
  *reinterpret_cast<PM_G uint64_t*>(S.done) = kChainBias;
  S.done[2] = 0;
}
// Called by wave 0 of a resolver, after its chain list entries.
template <class LdsT>
__device__ __forceinline__ void resolver_count(const PmStep& S, LdsT& L, uint32_t nchain, uint32_t cadd) {
  if ((threadIdx.x & 63) != 0) return;
  if (nchain) {   // chain list and results must be visible to the finisher
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  }
  L.fin = (uint32_t)chain_add(S, (1ull << 32) - cadd);
}

// One partition's share of Client.Query for every sub-query of the step, in
// order (wave 0 runs the chain; the other waves only help the prologue and
// return early).  L.fin: this workgroup made the step's last chain-count add.
template <int MODE, int NT, bool GRAN>
__device__ __forceinline__ void resolve_role(const PmStep& S, uint32_t p, ResolveLds<MODE>& L) {
  constexpr bool LDS = MODE != 0;
  auto& s_idx = L.s_idx; auto& s_kind = L.s_kind; auto& s_chunk = L.s_chunk; auto& s_st = L.s_st;
  auto& s_hist0 = L.s_hist0; auto& s_c1 = L.s_c1; auto& s_c2 = L.s_c2; auto& s_t1 = L.s_t1;
  auto& s_p1 = L.s_p1; auto& s_t2 = L.s_t2; auto& s_p2 = L.s_p2; auto& s_sing = L.s_sing;
  auto& m_h = L.m_h; auto& m_tag = L.m_tag; auto& m_pp = L.m_pp; auto& m_sub = L.m_sub; auto& m_pt = L.m_pt;
  auto& s_fqn = L.s_fqn; auto& s_chain = L.s_chain; auto& s_res = L.s_res;
  auto& bits_l = L.bits_l; auto& tag_l = L.tag_l; auto& pp_l = L.pp_l; auto& spec_v = L.spec_v;
  const PmPart P = S.parts[p];   // a copy: the chain loop's memory clobbers must not reload it
  const uint32_t b0 = step_sb(S, p), n = step_sb(S, p + 1) - b0;
  if (n == 0) return;
  const uint32_t lg = P.log2CS, mask = P.CS - 1, nw = (P.PH + 63) / 64, H = P.H;
  const uint32_t tid = threadIdx.x;
  STAMP(0);
  const uint32_t wave = tid >> 6, lane = tid & 63;
  // fast prologue (n <= 64 sub-queries, the usual shape): no staging of tags,
  // program points or match bits; two independent chains of two round trips
  // (MODE 0, partitions too large to stage: the same from global memory,
  // the match records read ten blocks at a time)
  // (MODE 3: k_match_resolve_s filled the fast prologue's LDS itself)
  const bool fast = MODE >= 2 || (MODE == 1 && n <= kSpecSubs && nw <= 128) || (MODE == 0 && n <= kSpecSubs);
  // match bits, tags and program points: LDS-staged by the staged prologue,
  // read from global memory on the (rare) paths of the fast one that need them
  const bool staged = MODE == 1 && !fast;
  auto find_bits = [&](uint32_t j, uint32_t start) -> uint32_t {
    if constexpr (MODE == 3) return find_cur(P, s_chunk[j], (uint32_t)(s_idx[j] & mask), start);
    if (staged) return find_next(bits_l + (uint64_t)j * nw, nw, start);
    return find_next_g<GRAN>(S, b0 + j, nw, start);
  };
  auto tag_of = [&](uint32_t h) -> uint32_t { return staged ? tag_l[h] : P.tag[h]; };
  auto pp_of = [&](uint32_t h) -> uint32_t { return staged ? pp_l[h] : P.pp[h]; };
  if (MODE == 3) {
  } else if (fast) {
    constexpr uint32_t NFW = NT / 64 - 1;   // candidate waves; the last wave predicts
    if (wave < NFW) {
      // first two stale candidates of each real sub-query, with their tag and
      // program point: the per-block records k_match wrote (blocks in hint order)
      const uint32_t nblk = MODE == 2 ? 1u : (P.PH + kMatchHints - 1) / kMatchHints;
      for (uint32_t j = wave; j < n; j += NFW) {
        const PmSub sub = step_sub(S, b0 + j);
        uint32_t c1 = kNone, c2 = kNone, t1 = 0, p1 = 0, t2 = 0, p2 = 0;
        if (sub.kind == SUB_REAL && sub.idx < P.N) {
          // the records of up to 16 x 10 blocks, all loads in flight together
          // (lanes 6b..6b+5 of window w: block 10w + b's {h, tag, pp} x 2)
          constexpr uint32_t kWin = 16;
          const uint32_t nwin = (nblk + 9) / 10;
          uint32_t vv[kWin];
#pragma unroll
          for (uint32_t w = 0; w < kWin; ++w) {
            vv[w] = kNone;
            const uint32_t nb = w < nwin ? min(10u, nblk - 10 * w) : 0;
            if (GRAN) {
              if (w == 0 && lane < 6) vv[w] = get_g(S.recg + (uint64_t)(b0 + j) * G_REC + lane, S);
            } else if (lane < nb * 6) {
              vv[w] = S.cand[((uint64_t)(b0 + j) * S.cblk + 10 * w) * 6 + lane];
            }
          }
          // the first two records in hint order: the non-empty hint slots
          // (lanes 3k), window by window
          auto take = [&](uint32_t v) {
            uint64_t m = __ballot(lane < 60 && lane % 3 == 0 && v != kNone);
            while (m && c2 == kNone) {
              const uint32_t l = (uint32_t)__builtin_ctzll(m);
              m &= m - 1;
              const uint32_t h = __builtin_amdgcn_readlane(v, l), t = __builtin_amdgcn_readlane(v, l + 1),
                             pp = __builtin_amdgcn_readlane(v, l + 2);
              if (c1 == kNone) { c1 = h; t1 = t; p1 = pp; } else { c2 = h; t2 = t; p2 = pp; }
            }
          };
#pragma unroll
          for (uint32_t w = 0; w < kWin; ++w)
            if (w < nwin && c2 == kNone) take(vv[w]);   // uniform
          // beyond 160 blocks (PH > 163,840; none of the configurations): the rest
          for (uint32_t w = kWin; w < nwin && c2 == kNone; ++w) {
            const uint32_t nb = min(10u, nblk - 10 * w);
            take(lane < nb * 6 ? S.cand[((uint64_t)(b0 + j) * S.cblk + 10 * w) * 6 + lane] : kNone);
          }
        }
        if (lane == 0) { s_c1[j] = c1; s_c2[j] = c2; s_t1[j] = t1; s_p1[j] = p1; s_t2[j] = t2; s_p2[j] = p2; }
      }
    } else {
      // The last wave: the request of every sub-query, its chunk's
      // QueryHistogram and predicted in-chunk index, and the predicted
      // re-evaluation values (k_match's records; all loads independent)
      const uint32_t k = lane;
      const uint32_t fq = lane == 0 ? *P.fqn : 0;
      PmSub sub{0, SUB_NONE, 0};
      if (k < n) sub = step_sub(S, b0 + k);
      const bool valid = k < n && sub.kind == SUB_REAL && sub.idx < P.N;
      uint32_t h0 = 0, sg = kNone;
      if (valid) {
        if (GRAN) {
          h0 = get_g(S.recg + (uint64_t)(b0 + k) * G_REC + 6, S);
          sg = get_g(S.recg + (uint64_t)(b0 + k) * G_REC + 7, S);
        } else {
          h0 = S.meta[2 * (uint64_t)(b0 + k)];
          sg = S.meta[2 * (uint64_t)(b0 + k) + 1];
        }
      }
      for (uint32_t e0 = 0; e0 < n * n; e0 += 64) {   // spec_v[kk][j], kk < j
        const uint32_t e = e0 + lane, kk = (e / n) & 63, j = e % n;
        // written by real sub-queries' match workgroups only (never read for others)
        const bool rk = __shfl(sub.kind, kk) == SUB_REAL;
        if (e < n * n && kk < j && rk)
          spec_v[kk * kSpecSubs + j] = (uint16_t)(GRAN ? get_g(S.specg + (uint64_t)(b0 + kk) * kSpecSubs + j, S)
                                                       : S.spec[(uint64_t)(b0 + kk) * kSpecSubs + j]);
      }
      if (k < n) {
        s_kind[k] = sub.kind; s_idx[k] = sub.idx; s_chunk[k] = (uint32_t)(sub.idx >> lg); s_st[k] = kNone;
        s_hist0[k] = h0; s_sing[k] = sg;
      }
      if (lane == 0) s_fqn = fq;
    }
  } else if constexpr (MODE < 2) {
    // --- phase 0: prefetch sub-queries, counters, match bits, tags ------------
    // Every global load of the staging is issued before the first LDS store:
    // the kernel is latency-bound, so one round trip instead of one per item.
    {
      constexpr int U = 8;
      PmSub sv[2];
      uint32_t hv[2];
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // (uint4 is a union: no SROA)
      uint64_t bv[U];
      u32x4 tv[U], pv[U];
      const uint32_t nb = LDS ? n * nw : 0, ph4 = LDS ? P.PH / 4 : 0;
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t j = tid + u * NT;
        if (j < n) sv[u] = step_sub(S, b0 + j);
      }
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + u * NT;
        if (i < nb) bv[u] = S.bits[(uint64_t)(b0 + i / nw) * S.words + (i % nw)];
        if (i < ph4) {
          tv[u] = reinterpret_cast<const PM_G u32x4*>(P.tag)[i];
          pv[u] = reinterpret_cast<const PM_G u32x4*>(P.pp)[i];
        }
      }
      const uint32_t fq = tid == 0 ? *P.fqn : 0;
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t j = tid + u * NT;
        hv[u] = (j < n && sv[u].kind == SUB_REAL && sv[u].idx < P.N) ? P.hist[(uint32_t)(sv[u].idx >> lg)] : 0;
      }
      for (uint32_t j = tid + 2 * NT; j < n; j += NT) {   // n > 512: rare
        const PmSub sub = step_sub(S, b0 + j);
        s_kind[j] = sub.kind; s_idx[j] = sub.idx; s_chunk[j] = (uint32_t)(sub.idx >> lg); s_st[j] = kNone;
        s_hist0[j] = (sub.kind == SUB_REAL && sub.idx < P.N) ? P.hist[(uint32_t)(sub.idx >> lg)] : 0;
      }
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t j = tid + u * NT;
        if (j < n) {
          s_kind[j] = sv[u].kind; s_idx[j] = sv[u].idx; s_chunk[j] = (uint32_t)(sv[u].idx >> lg);
          s_hist0[j] = hv[u]; s_st[j] = kNone;
        }
      }
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + u * NT;
        if (i < nb) bits_l[i] = bv[u];
        if (i < ph4) {
          reinterpret_cast<u32x4*>(tag_l)[i] = tv[u];
          reinterpret_cast<u32x4*>(pp_l)[i] = pv[u];
        }
      }
      if (tid == 0) s_fqn = fq;
    }
    __syncthreads();
    STAMP(1);
    // --- phase 1: first two stale candidates per real sub-query + their state;
    //     speculative in-group index of every sub-query (all earlier succeed)
    for (uint32_t j = wave; j < n; j += NT / 64) {
      if (s_kind[j] != SUB_REAL) continue;
      const uint32_t c1 = find_bits(j, 0);
      const uint32_t c2 = c1 == kNone ? kNone : find_bits(j, c1 + 1);
      if (lane == 0) {
        s_c1[j] = c1; s_c2[j] = c2;
        s_t1[j] = c1 == kNone ? 0 : tag_of(c1); s_p1[j] = c1 == kNone ? 0 : pp_of(c1);
        s_t2[j] = c2 == kNone ? 0 : tag_of(c2); s_p2[j] = c2 == kNone ? 0 : pp_of(c2);
      }
    }
    if (LDS && n <= kSpecSubs && wave == NT / 64 - 1) {
      // The last wave (the one with the least candidate work above) predicts, in
      // registers, the in-chunk index each sub-query would get if every earlier
      // one succeeds, and issues the table loads of the values the re-evaluation
      // in phase 2 would then need:
      //   spec_v[k][j] = PRF(tag the refresh of sub k would hand out, chunk of j)
      const uint32_t k = lane;
      const bool real = k < n && s_kind[k] == SUB_REAL;
      const uint64_t idx = k < n ? s_idx[k] : ~0ull;
      const uint32_t ch = k < n ? s_chunk[k] : kNone;
      bool first = real;                 // not a repeat of an earlier real sub-query
      for (uint32_t t = 0; t + 1 < n; ++t) {
        const uint64_t it = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(idx >> 32), t) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)idx, t);
        const bool rt = __builtin_amdgcn_readlane(real ? 1u : 0u, t) != 0;
        if (k > t && rt && it == idx) first = false;
      }
      uint32_t ing = k < n ? s_hist0[k] : 0;
      for (uint32_t q = 0; q + 1 < n; ++q) {
        const bool fq = __builtin_amdgcn_readlane(first ? 1u : 0u, q) != 0;
        const uint32_t cq = __builtin_amdgcn_readlane(ch, q);
        if (k > q && fq && cq == ch) ++ing;
      }
      if (k < n) s_sing[k] = ing;
      for (uint32_t e0 = 0; e0 < n * n; e0 += 64) {   // uniform: every lane joins the shuffles
        const uint32_t e = e0 + lane, kk = (e / n) & 63, j = e % n;
        const uint32_t sk = __shfl(ing, kk), ck = __shfl(ch, kk), cj = __shfl(ch, j);
        const bool rk = __shfl(real ? 1u : 0u, kk) != 0, rj = __shfl(real ? 1u : 0u, j) != 0;
        if (e < n * n && kk < j && rk && rj && ck < P.SS && cj < P.SS && sk < P.Qpc)
          spec_v[kk * kSpecSubs + j] = P.tabT[tabT_index(H, P.PH + ck * P.Qpc + sk, cj)];
      }
    }
  }
  __syncthreads();
  STAMP(2);
  STAMP(3);
  if (wave != 0) return;
  if (n <= 64) {
    // --- phase 2 (n <= 64): the chain in wave-0 registers -------------------
    // Lane k holds sub-query k (request, stale candidates, result) and entry k
    // of the list of hints refreshed so far in this step; each iteration reads
    // the current sub-query with v_readlane and decides with ballots, so the
    // only memory access per iteration is the re-evaluation value of each
    // refreshed hint (LDS when predicted, else the PRF table).
    const uint32_t k = lane;
    const bool in = k < n;
    const uint32_t kd = in ? s_kind[k] : SUB_NONE;
    const uint64_t ix = in ? s_idx[k] : 0;
    const uint32_t ch = in ? s_chunk[k] : kNone, h0 = in ? s_hist0[k] : 0;
    const bool real = in && kd == SUB_REAL;
    const uint32_t c1 = real ? s_c1[k] : kNone, c2 = real ? s_c2[k] : kNone;
    const uint32_t t1 = real ? s_t1[k] : 0, p1 = real ? s_p1[k] : 0;
    const uint32_t t2 = real ? s_t2[k] : 0, p2 = real ? s_p2[k] : 0;
    const bool spec = n <= kSpecSubs && (LDS || fast);
    const uint32_t sg = (spec && real) ? s_sing[k] : kNone;
    // tag sub k's refresh would hand out if every earlier sub-query succeeds
    const uint32_t pred = (sg < P.Qpc && ch < P.SS) ? P.PH + ch * P.Qpc + sg : kNone;
    // per sub-query result
    uint32_t st = kNone, rhit = 0, ring = 0, rtag = 0, rpp = 0, rslot = 0, rfl = 0;
    // per refreshed-hint entry: hint, current tag / program point, last holder, its predicted tag
    uint32_t mh = kNone, mt = 0, mp = 0, ms = 0, mpt = kNone;
    uint32_t cl = 0;   // chain list entry
    uint32_t fqn = s_fqn, nmod = 0, nchain = 0, cadd = 0;
    auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane(v, l); };
    // --- parallel prefix ---------------------------------------------------
    // A sub-query's outcome depends on the earlier ones only through (a) a
    // local-cache hit (an earlier success with the same index), (b) the budget
    // and per-chunk counters, (c) whether its first stale candidate was
    // refreshed earlier, and (d) whether a hint refreshed earlier now matches
    // it below that candidate.  Assuming every earlier valid first occurrence
    // succeeds on its first candidate, (a)-(d) are decided for all lanes at
    // once ((d) with the predicted table values).  The first valid first
    // occurrence that would not succeed that plainly ends the prefix; the chain
    // below resumes there, from the state the prefix leaves.
    uint32_t jf = n;
    {
      const uint32_t off = (uint32_t)(ix & mask);
      bool firstocc = real;
      uint32_t src = k;   // first real sub-query with this index
      for (uint32_t t = 0; t + 1 < n; ++t) {
        const uint64_t it = ((uint64_t)rl((uint32_t)(ix >> 32), t) << 32) | rl((uint32_t)ix, t);
        if (firstocc && t < k && rl(kd, t) == SUB_REAL && it == ix) { firstocc = false; src = t; }
      }
      const bool cand = real && ix < P.N && firstocc;
      const uint64_t okm = __ballot(cand), below = (1ull << k) - 1;   // k < 64
      uint32_t hist = h0;
      for (uint32_t t = 0; t + 1 < n; ++t)
        if (t < k && ((okm >> t) & 1) && rl(ch, t) == ch) ++hist;
      const uint32_t fk = fqn + (uint32_t)__builtin_popcountll(okm & below);
      const uint32_t ntag = P.PH + ch * P.Qpc + hist;   // the refresh this sub-query makes
      bool simple = cand && hist < P.Qpc && fk < P.MaxQ && c1 != kNone;
      for (uint32_t t = 0; t + 1 < n; ++t) {
        if (!((okm >> t) & 1)) continue;
        const uint32_t c1t = rl(c1, t), cht = rl(ch, t), ntt = rl(ntag, t), prt = rl(pred, t);
        if (t < k) {
          if (c1t == c1) simple = false;                      // (c)
          if (cht != ch && c1t < c1 &&                          // (d): unpredicted, or a match
              (ntt != prt || (uint32_t)spec_v[t * kSpecSubs + k] == off))
            simple = false;
        }
      }
      const uint64_t hard = __ballot(cand && !simple);
      jf = hard ? (uint32_t)__builtin_ctzll(hard) : n;
      if (in && k < jf) {
        if (kd == SUB_DUMMY) st = ST_DUMMY;
        else if (kd == SUB_HOSTCACHE) { st = ST_CACHED; rslot = (uint32_t)ix; }
        else if (kd != SUB_REAL) st = ST_SKIP;
        else if (ix >= P.N) st = ST_ERANGE;
        else if (!firstocc) { st = ST_DUP; rslot = b0 + src; }
        else { st = ST_OK; rhit = c1; ring = hist; rtag = t1; rpp = p1; rslot = fk; }
      }
      // the prefix's refreshed hints become the first entries, in order
      const uint64_t okp = okm & (jf >= 64 ? ~0ull : ((1ull << jf) - 1));
      if ((okp >> k) & 1) {
        const uint32_t e = (uint32_t)__builtin_popcountll(okp & below);
        m_h[e] = c1; m_tag[e] = ntag; m_pp[e] = (uint32_t)ix; m_sub[e] = k; m_pt[e] = pred;
      }
      nmod = (uint32_t)__builtin_popcountll(okp);
      fqn += nmod;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (k < nmod) { mh = m_h[k]; mt = m_tag[k]; mp = m_pp[k]; ms = m_sub[k]; mpt = m_pt[k]; }
    }
    STAMP(38);
    for (uint32_t j = jf; j < n; ++j) {
      const uint32_t kind = rl(kd, j), chunk = rl(ch, j);
      const uint64_t idx = ((uint64_t)rl((uint32_t)(ix >> 32), j) << 32) | rl((uint32_t)ix, j);
      uint32_t status = kNone, hit = 0, hist = 0, tag = 0, pp = 0, slot = 0, fl = 0;
      if (kind == SUB_DUMMY) status = ST_DUMMY;
      else if (kind == SUB_HOSTCACHE) { status = ST_CACHED; slot = (uint32_t)idx; }
      else if (kind != SUB_REAL) status = ST_SKIP;
      else if (idx >= P.N) status = ST_ERANGE;
      else {
        const uint32_t off = (uint32_t)(idx & mask);
        // local cache hit inside this step (pir.go:381-383)
        const uint64_t dup = __ballot(k < j && real && ix == idx && st == ST_OK);
        if (dup) { status = ST_DUP; slot = b0 + (uint32_t)__builtin_ctzll(dup); }
        else if (fqn >= P.MaxQ) status = ST_EBUDGET;                        // pir.go:386-391
        else {
          hist = rl(h0, j) + (uint32_t)__builtin_popcountll(__ballot(k < j && st == ST_OK && ch == chunk));
          if (hist >= P.Qpc) status = ST_ECHUNK;                            // pir.go:396-400
        }
        if (status == kNone) {
          // first stale match not refreshed earlier in this step
          uint32_t c = rl(c1, j), which = 1;
          while (c != kNone && __ballot(k < nmod && mh == c)) {
            if (which == 1) { c = rl(c2, j); which = 2; }
            else { c = find_bits(j, c + 1); which = 3; }
          }
          // hints refreshed earlier in this step, with their current tag / program point
          uint32_t cand = kNone;
          if (k < nmod) {
            const uint32_t o = mt == mpt ? (uint32_t)spec_v[ms * kSpecSubs + j]
                                         : (uint32_t)P.tabT[tabT_index(H, mt, chunk)];
            if (o == off && (mp == kDefaultProgramPoint || (mp >> lg) != chunk)) cand = mh;
          }
          uint32_t bm = kNone, bk = 0;
          for (uint64_t cm = __ballot(cand != kNone); cm; cm &= cm - 1) {   // usually 0 or 1 bits
            const uint32_t b = (uint32_t)__builtin_ctzll(cm), v = rl(cand, b);
            if (v < bm) { bm = v; bk = b; }
          }
          hit = min(c, bm);
          if (hit == kNone) {
            status = ST_ENOHIT;                                              // pir.go:416-419
          } else {
            const bool chained = hit == bm;
            if (chained) { tag = rl(mt, bk); pp = rl(mp, bk); }
            else if (which == 1) { tag = rl(t1, j); pp = rl(p1, j); }
            else if (which == 2) { tag = rl(t2, j); pp = rl(p2, j); }
            else { tag = tag_of(hit); pp = pp_of(hit); }
            status = ST_OK; slot = fqn; fl = chained ? 1u : 0u;
            // refresh (pir.go:460-470): backup hint (chunk, hist) has tag PH + chunk*Qpc + hist
            const uint32_t ntag = P.PH + chunk * P.Qpc + hist, npred = rl(pred, j);
            if (chained) {
              // the previous holder must publish its parity refresh; this chained
              // sub-query counts itself, the chain head is counted once
              const uint32_t prev = rl(ms, bk), pf = rl(rfl, prev);
              cadd += 1u + ((!(pf & 1u) && !(pf & 4u)) ? 1u : 0u);
              if (k == prev) rfl = pf | 2u | 4u;
              if (k == nchain) cl = b0 + j;
              if (k == bk) { mt = ntag; mp = (uint32_t)idx; ms = j; mpt = npred; }
              ++nchain;
            } else {
              if (k == nmod) { mh = hit; mt = ntag; mp = (uint32_t)idx; ms = j; mpt = npred; }
              ++nmod;
            }
            ++fqn;
          }
        }
      }
      if (k == j) { st = status; rhit = hit; ring = hist; rtag = tag; rpp = pp; rslot = slot; rfl = fl; }
      if (j < 32) STAMP(4 + j);
    }
    STAMP(39);
    // --- flush (one writer per result / hint / chunk) -----------------------
    if (in) {
      const bool ok = st == ST_OK;
      const PmRes rr{st, ok ? rhit : 0u, ok ? ch : 0u, ok ? ring : 0u, ok ? rtag : 0u,
                     ok ? rpp : 0u, (ok || st == ST_DUP || st == ST_CACHED) ? rslot : 0u, ok ? rfl : 0u};
      put_res<GRAN>(S, b0 + k, rr);
      if constexpr (MODE == 3) s_res[k] = rr;   // k_match_resolve_s expands the query sets from LDS
    }
    if (k < nmod) { P.tag[mh] = mt; P.pp[mh] = mp; }
    bool last = in && st == ST_OK;   // QueryHistogram: the last success per chunk writes
    for (uint32_t t = 0; t < n; ++t)
      if (t > k && rl(st, t) == ST_OK && rl(ch, t) == ch) last = false;
    if (last) P.hist[ch] = ring + 1;
    if (nchain) {   // this partition's chained sub-queries, contiguous and in order
      uint32_t pos = 0;
      if (k == 0) pos = atomicAdd(&S.done[2], nchain);
      pos = __builtin_amdgcn_readfirstlane(pos);
      if (k < nchain) S.done[3 + pos + k] = cl;
    }
    if (k == 0) *P.fqn = fqn;
    if constexpr (MODE == 3) {
      // k_match_resolve_s (S.np_live == 0): the answer kernel starts after every
      // resolver is done, so resolvers do not count in; a partition with refresh
      // chains subtracts its involved answer workgroups (no returned value, no
      // wait), and the counter is back at its bias after their arrivals
      if (k == 0 && cadd)
        __hip_atomic_fetch_add(reinterpret_cast<PM_G uint64_t*>(S.done), (uint64_t)0 - cadd, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    } else {
      resolver_count(S, L, nchain, cadd);
    }
    STAMP(40);
    return;
  }
  if constexpr (MODE < 2) {
  // --- phase 2 (n > 64): the sequential chain of Client.Query calls, on wave 0
  // The chain state lives in plain LDS arrays: lane 0 writes, every lane of the
  // same wave reads in a later iteration (LDS instructions of one wave complete
  // in order); an empty asm memory clobber at the end of each iteration keeps
  // the compiler from reusing values across it.  (volatile pointers here would
  // compile to flat accesses that also wait for the outstanding global stores.)
  // Nothing is written to global memory inside the loop (on CDNA vmcnt counts
  // stores too, so any load wait there would also wait for them): results,
  // refreshed tags / program points, counters and the chain list are kept in
  // LDS and flushed by the whole wave afterwards.
  const bool spec = LDS && n <= kSpecSubs;
  uint32_t fqn = s_fqn, nmod = 0, nchain = 0, cadd = 0;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t s = b0 + j, kind = s_kind[j];
    PmRes r{kNone, 0, 0, 0, 0, 0, 0, 0};
    if (kind == SUB_DUMMY) { r.status = ST_DUMMY; }
    else if (kind == SUB_HOSTCACHE) { r.status = ST_CACHED; r.slot = (uint32_t)s_idx[j]; }
    else if (kind != SUB_REAL) { r.status = ST_SKIP; }
    else {
      const uint64_t idx = s_idx[j];
      const uint32_t chunk = s_chunk[j], off = (uint32_t)(idx & mask);
      if (idx >= P.N) r.status = ST_ERANGE;
      if (r.status == kNone) {   // local cache hit inside this step (pir.go:381-383)
        for (uint32_t k0 = 0; k0 < j; k0 += 64) {
          const uint32_t k = k0 + lane;
          const bool d = k < j && s_kind[k] == SUB_REAL && s_idx[k] == idx && s_st[k] == ST_OK;
          const uint64_t m = __ballot(d);
          if (m) { r.status = ST_DUP; r.slot = b0 + k0 + (uint32_t)__builtin_ctzll(m); break; }
        }
      }
      if (r.status == kNone && fqn >= P.MaxQ) r.status = ST_EBUDGET;     // pir.go:386-391
      uint32_t hist = s_hist0[j];
      if (r.status == kNone) {
        for (uint32_t k0 = 0; k0 < j; k0 += 64) {
          const uint32_t k = k0 + lane;
          hist += (uint32_t)__builtin_popcountll(
              __ballot(k < j && s_st[k] == ST_OK && s_chunk[k] == chunk));
        }
        if (hist >= P.Qpc) r.status = ST_ECHUNK;                          // pir.go:396-400
      }
      if (r.status == kNone) {
        // first unrefreshed stale match
        uint32_t c = s_c1[j], which = 1;
        for (;;) {
          if (c == kNone) break;
          bool mod = false;
          for (uint32_t k0 = 0; k0 < nmod; k0 += 64)
            mod |= __ballot(k0 + lane < nmod && m_h[k0 + lane] == c) != 0;
          if (!mod) break;
          if (which == 1) { c = s_c2[j]; which = 2; }
          else { c = find_bits(j, c + 1); which = 3; }
        }
        // hints refreshed earlier in this step, with their current tag / program point
        uint32_t bm = kNone, bk = kNone;
        for (uint32_t k0 = 0; k0 < nmod; k0 += 64) {
          const uint32_t k = k0 + lane;
          uint32_t cand = kNone;
          if (k < nmod) {
            const uint32_t pp = m_pp[k], tg = m_tag[k], ks = m_sub[k];
            // the speculative value holds when sub ks received its predicted tag
            const uint32_t o = (spec && s_sing[ks] < P.Qpc && tg == P.PH + s_chunk[ks] * P.Qpc + s_sing[ks])
                                   ? (uint32_t)spec_v[ks * kSpecSubs + j]
                                   : (uint32_t)P.tabT[tabT_index(H, tg, chunk)];
            if (o == off && (pp == kDefaultProgramPoint || (pp >> lg) != chunk)) cand = m_h[k];
          }
          const uint32_t mn = wave_min(cand);
          if (mn < bm) {
            bm = mn;
            const uint64_t who = __ballot(cand == mn && mn != kNone);
            bk = k0 + (uint32_t)__builtin_ctzll(who);
          }
        }
        const uint32_t hit = min(c, bm);
        if (hit == kNone) {
          r.status = ST_ENOHIT;                                              // pir.go:416-419
        } else {
          const bool chained = hit == bm;
          uint32_t tag, pp;
          if (chained) { tag = m_tag[bk]; pp = m_pp[bk]; }
          else if (which == 1) { tag = s_t1[j]; pp = s_p1[j]; }
          else if (which == 2) { tag = s_t2[j]; pp = s_p2[j]; }
          else { tag = tag_of(hit); pp = pp_of(hit); }
          r = PmRes{ST_OK, hit, chunk, hist, tag, pp, fqn, chained ? 1u : 0u};
          // refresh (pir.go:460-470): backup hint (chunk, hist) has tag PH + chunk*Qpc + hist
          const uint32_t ntag = P.PH + chunk * P.Qpc + hist;
          if (chained) {
            // the previous holder of this hint must publish its parity refresh;
            // this chained sub-query counts itself, the chain head is counted once
            const uint32_t prev = m_sub[bk];
            const uint32_t pf = s_res[prev].flags;
            cadd += 1u + ((!(pf & 1u) && !(pf & 4u)) ? 1u : 0u);
            if (lane == 0) {
              s_res[prev].flags = pf | 2u | 4u;
              s_chain[nchain] = s;
              m_tag[bk] = ntag; m_pp[bk] = (uint32_t)idx; m_sub[bk] = j;
            }
            ++nchain;
          } else {
            if (lane == 0) { m_h[nmod] = hit; m_tag[nmod] = ntag; m_pp[nmod] = (uint32_t)idx; m_sub[nmod] = j; }
            ++nmod;
          }
          ++fqn;
        }
      }
    }
    if (lane == 0) { s_st[j] = r.status; s_res[j] = r; }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (j < 32) STAMP(4 + j);
  }
  // --- flush (pir.go:460-470 refresh; one writer per hint / chunk) ----------
  for (uint32_t k = lane; k < n; k += 64) put_res<GRAN>(S, b0 + k, s_res[k]);
  for (uint32_t k = lane; k < nmod; k += 64) {
    P.tag[m_h[k]] = m_tag[k];
    P.pp[m_h[k]] = m_pp[k];
  }
  for (uint32_t k = lane; k < n; k += 64) {   // QueryHistogram: the last success per chunk writes
    if (s_st[k] != ST_OK) continue;
    const uint32_t c = s_chunk[k];
    bool last = true;
    for (uint32_t t = k + 1; t < n; ++t) last &= !(s_st[t] == ST_OK && s_chunk[t] == c);
    if (last) P.hist[c] = s_res[k].ing + 1;
  }
  if (nchain) {   // this partition's chained sub-queries, contiguous and in order
    uint32_t pos = 0;
    if (lane == 0) pos = atomicAdd(&S.done[2], nchain);
    pos = __builtin_amdgcn_readfirstlane(pos);
    for (uint32_t k = lane; k < nchain; k += 64) S.done[3 + pos + k] = s_chain[k];
  }
  if (lane == 0) *P.fqn = fqn;
  resolver_count(S, L, nchain, cadd);
  STAMP(40);
  }
}

// (large partitions, MODE 0: 512 threads, so each sub-query of a partition
// has a candidate wave of its own)
constexpr int kResolveBlockG = 512;
template <bool LDS>
__global__ void __launch_bounds__(LDS ? kBlock : kResolveBlockG) k_resolve(PmStep S) {
  __shared__ ResolveLds<LDS ? 1 : 0> L;
  const uint32_t p = blockIdx.x;
  if (step_sb(S, p + 1) == step_sb(S, p)) return;
  resolve_role<LDS ? 1 : 0, LDS ? kBlock : kResolveBlockG, false>(S, p, L);
  __syncthreads();
  // last add here: no answer workgroup is involved in a chain, nothing to decode
  if (L.fin && threadIdx.x == 0) chain_rearm(S);
}

// k_match_part + k_resolve in one launch, one 512-thread workgroup per
// partition (batched serving: the resolver's MODE-0 fast prologue, <= 64
// sub-queries per partition).  The match writes exactly what k_match_part
// writes (bits, per-block records, predictions) to global memory, two 1,024-
// hint blocks at a time (two teams of 256 threads), and after a workgroup
// barrier the same workgroup resolves the partition from them, out of L2.
// Saves the match kernel's launch and its ~4 workgroups per partition.  The
// descriptor must already be in device memory (S.subs == S.subs_h): nothing
// here stages it, as every resolver reads the whole step's sb.
template <int HPT>
__global__ void __launch_bounds__(kResolveBlockG) k_match_resolve(PmStep S) {
  constexpr int NT = kBlock, G = PM_MATCHPART_G, TEAMS = kResolveBlockG / kBlock;
  __shared__ ResolveLds<0> L;
  __shared__ uint32_t s_cand[TEAMS][G][NT / 64][6];
  const uint32_t p = blockIdx.x, tid = threadIdx.x;
  const uint32_t pb0 = step_sb(S, p), pn = step_sb(S, p + 1) - pb0;
  if (pn == 0) return;
  {
    const PmPart P = S.parts[p];
    const uint32_t team = tid / NT, ttid = tid % NT;
    match_part_predict(S, P, pb0, pn, tid >> 6, kResolveBlockG / 64);
    const uint32_t nb = (P.PH + NT * HPT - 1) / (NT * HPT);
    for (uint32_t b = 0; b < nb; b += TEAMS)
      match_part_block<HPT, NT, G>(S, P, pb0, pn, b + team, ttid, s_cand[team]);
  }
  __syncthreads();   // the match's global stores, visible to this workgroup's resolver
  resolve_role<0, kResolveBlockG, false>(S, p, L);
  __syncthreads();
  if (L.fin && threadIdx.x == 0) chain_rearm(S);
}

// k_match_resolve for the search-sized shapes (<= 64 sub-queries per
// partition, PH % 8 == 0 and PH <= 8 * 512 * NU: SIFT1M's 3,584 and MS-MARCO's
// 7,168 hints): one 512-thread workgroup per partition, and the match in ONE
// round trip.  Every thread loads the 8 * NU contiguous search-row values
// (PmPart::cur, 16-B loads) of its hints for every sub-query of a group of G,
// all in flight together; each wave's first two matches (hint order = lane
// order) come out of a ballot, and the resolver's fast prologue is filled in
// LDS directly: no match bits, records or predictions pass through global
// memory (the rare third candidate is re-read from cur, find_cur).  The last
// wave reads the requests, QueryHistogram and FinishedQueryNum and makes the
// predictions of resolve_role's staged prologue (in-chunk index, re-evaluation
// values) meanwhile.  Results are identical to k_match_resolve's.
// Measured alone at the bench's 64-session groups (k_match_resolve_s<2,256>):
// 19.1-19.3 us with the defaults; 19.7 with all 6 sub-queries' search rows in
// one round trip (PM_MR_G 0: 8 per round trip for NU <= 2, 6 for NU 4, 82
// VGPRs and SGPR spills), with or without the candidates' tags loaded by the
// matching wave (PM_MR_TAGPF 1) instead of by wave 0 after the barrier.
#ifndef PM_MR_TAGPF
#define PM_MR_TAGPF 0
#endif
#ifndef PM_MR_G
#define PM_MR_G 8       // search rows of 8 / NU sub-queries per round trip (0: see above)
#endif
#ifndef PM_MR_EARLY
#define PM_MR_EARLY 1   // k_match_resolve_s: row block 0 first, the rest only where fewer than two matches
                        // (+0.6 %, ABBA, profiles/r05/ab/match_early_exit.log)
#endif
#ifndef PM_MR_NTLOAD
#define PM_MR_NTLOAD 1   // k_match_resolve_s' search-row loads nontemporal: streamed, not kept in the Infinity Cache
                     // the answer's DB rows reuse (with PM_REFRESH_NT +2.0 %, ABBA, profiles/r05/ab/nontemporal_*)
#endif
#ifndef PM_REFRESH_NT
#define PM_REFRESH_NT 1   // k_answer_p's refresh stores nontemporal (the same reason)
#endif
#ifndef PM_DEC_NT
#define PM_DEC_NT 0   // k_answer_p's decode operands (replacement row, parities, the new tag's offsets) nontemporal
#endif
#ifndef PM_EPI_NT
#define PM_EPI_NT 1   // k_answer_p's parity and localCache stores nontemporal (+0.5 %, within noise; written
                      // once per refresh, read back rounds later if at all)
#endif
#ifndef PM_CHAIN_PRIO
#define PM_CHAIN_PRIO 0   // s_setprio of the device loop's chain kernels (match + resolve, the team round)
#endif
template <int NU, int NT>
__global__ void __launch_bounds__(NT) k_match_resolve_s(PmStep S) {
  if (PM_CHAIN_PRIO) __builtin_amdgcn_s_setprio(PM_CHAIN_PRIO);
  // G sub-queries' search rows in flight together (the usual 6 per partition:
  // one round trip); 2 * G * NU <= 64 candidates per wave, one per lane
  constexpr int NW = NT / 64, G = PM_MR_G ? PM_MR_G / NU : NU <= 2 ? 8 : NU == 4 ? 6 : 8 / NU;
  static_assert(2 * G * NU <= 64, "one lane per candidate");
  __shared__ ResolveLds<3> L;
  // each (sub-query, row block, wave): first two matches, their tags and program points
  __shared__ uint32_t s_m[kSpecSubs][NU][NW][2], s_mt[kSpecSubs][NU][NW][PM_MR_TAGPF ? 2 : 1],
      s_mp[kSpecSubs][NU][NW][PM_MR_TAGPF ? 2 : 1];
  const uint32_t p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  MRST(0);
  // the partition record is loaded with the descriptor range (its field in the
  // exit test keeps the load ahead of the branch: one round trip, not two)
  const uint32_t b0 = S.sb[p], n = S.sb[p + 1] - b0;   // device descriptor (never in the arguments here)
  const PmPart P = S.parts[p];
  if (n == 0 || P.CS == 0) return;
  const uint32_t lg = P.log2CS, mask = P.CS - 1;
#ifdef PM_MR_STAMPS
  if (tid == 0 && S.stamps) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); MRST(1); }
#endif
  if (wave == NW - 1) {
    // requests, counters and predictions (resolve_role's staged prologue, from global memory)
    const uint32_t k = lane;
    PmSub sub{0, SUB_NONE, 0};
    if (k < n) sub = step_sub(S, b0 + k);
    const bool real = k < n && sub.kind == SUB_REAL;
    const uint64_t idx = k < n ? sub.idx : ~0ull;
    const uint32_t ch = k < n ? (uint32_t)(sub.idx >> lg) : kNone;
    const uint32_t h0 = (real && sub.idx < P.N) ? P.hist[ch] : 0;
    const uint32_t fq = lane == 0 ? *P.fqn : 0;
    bool first = real;   // not a repeat of an earlier real sub-query
    for (uint32_t t = 0; t + 1 < n; ++t) {
      const uint64_t it = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(idx >> 32), t) << 32) |
                          __builtin_amdgcn_readlane((uint32_t)idx, t);
      const bool rt = __builtin_amdgcn_readlane(real ? 1u : 0u, t) != 0;
      if (k > t && rt && it == idx) first = false;
    }
    uint32_t ing = h0;
    for (uint32_t q = 0; q + 1 < n; ++q) {
      const bool fq2 = __builtin_amdgcn_readlane(first ? 1u : 0u, q) != 0;
      const uint32_t cq = __builtin_amdgcn_readlane(ch, q);
      if (k > q && fq2 && cq == ch) ++ing;
    }
    for (uint32_t e0 = 0; e0 < n * n; e0 += 64) {   // uniform: every lane joins the shuffles
      const uint32_t e = e0 + lane, kk = (e / n) & 63, j = e % n;
      const uint32_t sk = __shfl(ing, kk), ck = __shfl(ch, kk), cj = __shfl(ch, j);
      const bool rk = __shfl(real ? 1u : 0u, kk) != 0, rj = __shfl(real ? 1u : 0u, j) != 0;
      if (e < n * n && kk < j && rk && rj && ck < P.SS && cj < P.SS && sk < P.Qpc)
        L.spec_v[kk * kSpecSubs + j] = P.tabT[tabT_index(P.H, P.PH + ck * P.Qpc + sk, cj)];
    }
    if (k < n) {
      L.s_kind[k] = sub.kind; L.s_idx[k] = sub.idx; L.s_chunk[k] = ch; L.s_st[k] = kNone;
      L.s_hist0[k] = h0; L.s_sing[k] = ing;
    }
    if (lane == 0) L.s_fqn = fq;
  }
  // every request of the partition at once, lane k of each wave holding
  // sub-query k (n <= 64): one round trip, then the search-row loads of G
  // sub-queries at a time.  (Loaded per sub-query inside the batch, each
  // descriptor load's wait also drained the previous sub-query's row loads:
  // the batch's loads were serialised.)
  PmSub mine{0, SUB_NONE, 0};
  if (lane < n) mine = step_sub(S, b0 + lane);
  // the match: sub-queries j0 .. j0 + G - 1 at a time, over the row blocks u
  // in umask of the sub-queries in jmask (bit j)
  auto match_pass = [&](uint32_t umask, uint64_t jmask) {
  for (uint32_t j0 = 0; j0 < n; j0 += G) {
    uint32_t cand = kNone;   // lane q: candidate i = q % 2 of (g, u) = (q / (2 NU), (q / 2) % NU)
    uint32_t off[G];
    uint4 v[G][NU];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t jj = min(j0 + g, n - 1);   // uniform
      const uint32_t kind = j0 + g < n ? (uint32_t)__builtin_amdgcn_readlane(mine.kind, jj) : (uint32_t)SUB_NONE;
      const uint64_t idx = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(mine.idx >> 32), jj) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((uint32_t)mine.idx, jj);
      const bool lv = kind == SUB_REAL && idx < P.N && j0 + g < 64 && ((jmask >> (j0 + g)) & 1);
      off[g] = lv ? (uint32_t)(idx & mask) : kNone;
      const PM_G uint16_t* crow = P.cur + cur_row(P.PH, P.curk, lv ? (uint32_t)(idx >> lg) : 0u);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const uint32_t h = (u * NT + tid) * 8;
        v[g][u] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);   // kSkip x 8
        if (lv && ((umask >> u) & 1) && h < P.PH) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const PM_G u32x4* src = reinterpret_cast<const PM_G u32x4*>(crow + cur_row_off(P.curk, h));
          const u32x4 x = PM_MR_NTLOAD ? __builtin_nontemporal_load(src) : *src;
          v[g][u] = make_uint4(x.x, x.y, x.z, x.w);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (j0 + g >= n) break;   // uniform
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const uint32_t w[4] = {v[g][u].x, v[g][u].y, v[g][u].z, v[g][u].w};
        uint32_t bm = 0;   // this lane's 8 hints that match, bit e = hint (u * NT + tid) * 8 + e
#pragma unroll
        for (int e = 0; e < 8; ++e)
          bm |= (((w[e >> 1] >> (16 * (e & 1))) & 0xffffu) == off[g] ? 1u : 0u) << e;
        uint64_t b = __ballot(bm != 0);
        uint32_t a0 = kNone, a1 = kNone;
        if (b) {
          const uint32_t l0 = (uint32_t)__builtin_ctzll(b);
          const uint32_t hb = (u * NT + wave * 64) * 8;
          uint32_t m0 = __builtin_amdgcn_readlane(bm, l0);
          a0 = hb + l0 * 8 + (uint32_t)__builtin_ctz(m0);
          m0 &= m0 - 1;
          if (m0) {
            a1 = hb + l0 * 8 + (uint32_t)__builtin_ctz(m0);
          } else {
            b &= b - 1;
            if (b) {
              const uint32_t l1 = (uint32_t)__builtin_ctzll(b);
              a1 = hb + l1 * 8 + (uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(bm, l1));
            }
          }
        }
        if (lane == 2 * (g * NU + u)) cand = a0;
        if (lane == 2 * (g * NU + u) + 1) cand = a1;
      }
    }
    // the candidates' tags and program points, one lane each, all in flight
    // together (the resolver's chain and the set expansion read them from LDS)
    uint32_t ct = 0, cp = 0;
    if (PM_MR_TAGPF && cand != kNone) { ct = P.tag[cand]; cp = P.pp[cand]; }
    const uint32_t qg = lane / (2 * NU), qu = (lane / 2) % NU, qi = lane % 2;
    if (lane < 2 * G * NU && j0 + qg < n && ((umask >> qu) & 1) && ((jmask >> (j0 + qg)) & 1)) {
      s_m[j0 + qg][qu][wave][qi] = cand;
      if (PM_MR_TAGPF) { s_mt[j0 + qg][qu][wave][qi % 2] = ct; s_mp[j0 + qg][qu][wave][qi % 2] = cp; }
    }
  }
  };
#if PM_MR_EARLY
  // Row block 0 first (hints 0 .. 8 NT - 1); the other blocks only for the
  // sub-queries with fewer than two matches there (the candidates are the
  // first two in hint order): ~9 % of them at SIFT1M's PH, and ~40 % fewer
  // search-row bytes per step for one more round trip where any needs them
  match_pass(1u, ~0ull);
  if (NU > 1) {
    for (uint32_t x = tid; x < n * (NU - 1) * NW * 2; x += NT) {   // the other blocks' slots: none yet
      const uint32_t j = x / ((NU - 1) * NW * 2), r = x % ((NU - 1) * NW * 2);
      s_m[j][1 + r / (NW * 2)][(r / 2) % NW][r % 2] = kNone;
    }
    __syncthreads();
    uint64_t need = 0;
    for (uint32_t j = 0; j < n && j < 64; ++j) {
      uint32_t c = 0;
      for (int w = 0; w < NW; ++w) c += (s_m[j][0][w][0] != kNone) + (s_m[j][0][w][1] != kNone);
      if (L.s_kind[j] == SUB_REAL && c < 2) need |= 1ull << j;
    }
    if (need) match_pass(((1u << NU) - 1) & ~1u, need);   // block-uniform (from LDS)
  }
#else
  match_pass((1u << NU) - 1, ~0ull);
#endif
  MRST(2);
  __syncthreads();
  MRST(3);
  if (wave == 0 && lane < n) {
    // each sub-query's first two matches in hint order, with their tag and program point
    const uint32_t j = lane;
    uint32_t c1 = kNone, c2 = kNone, t1 = 0, p1 = 0, t2 = 0, p2 = 0;
    if (L.s_kind[j] == SUB_REAL) {
      for (int u = 0; u < NU && c2 == kNone; ++u)
        for (int w = 0; w < NW && c2 == kNone; ++w)
          for (int i = 0; i < 2; ++i) {
            const uint32_t h = s_m[j][u][w][i];
            if (h == kNone || c2 != kNone) continue;
            const uint32_t ti = PM_MR_TAGPF ? i : 0;
            if (c1 == kNone) { c1 = h; t1 = s_mt[j][u][w][ti]; p1 = s_mp[j][u][w][ti]; }
            else { c2 = h; t2 = s_mt[j][u][w][ti]; p2 = s_mp[j][u][w][ti]; }
          }
      if (!PM_MR_TAGPF && c1 != kNone) { t1 = P.tag[c1]; p1 = P.pp[c1]; }
      if (!PM_MR_TAGPF && c2 != kNone) { t2 = P.tag[c2]; p2 = P.pp[c2]; }
    }
    L.s_c1[j] = c1; L.s_c2[j] = c2; L.s_t1[j] = t1; L.s_p1[j] = p1; L.s_t2[j] = t2; L.s_p2[j] = p2;
  }
  __syncthreads();
  MRST(4);
  resolve_role<3, NT, false>(S, p, L);
  MRST(5);
  // The query set of every successful sub-query (pir.go:424-444: the hit
  // hint's offsets, its program point, the chunk's replacement), expanded
  // here so that k_answer_s reads it with its resolution record in one round
  // trip instead of gathering the tag's PRF row after the record arrives.
  // One 16-B tabT tile (8 chunks) per thread; S.qw words per sub-query.
  // Thread tid takes tile x = (tid - 64) mod NT first: waves 1.. get here
  // while wave 0 still runs the chain, and load that tile (and the chunk's
  // replacement row) for the usual outcome -- hit = the first candidate (tag
  // s_t1), in-chunk index = the prediction (s_sing) -- so that after the chain
  // the expansion only checks the guess.
  const uint32_t nt8 = S.qset ? S.qw / 8 : 0;
  const uint32_t x0 = (tid + NT - 64) % NT;
  uint4 gv = make_uint4(0, 0, 0, 0);
  uint32_t gr = 0, gtag = kNone, ging = kNone;
  if (tid >= 64 && x0 < n * nt8) {
    const uint32_t j = x0 / nt8, c0 = 8 * (x0 % nt8);
    if (L.s_kind[j] == SUB_REAL && L.s_c1[j] != kNone) {
      gtag = L.s_t1[j];
      if (c0 < P.SS) gv = *reinterpret_cast<const PM_G uint4*>(P.tabT + tabT_index(P.H, gtag, c0));
      const uint32_t ch = L.s_chunk[j], sg = L.s_sing[j];
      if (ch - c0 < 8u && sg < P.Qpc) { ging = sg; gr = P.ridx[ch * P.Qpc + sg]; }
    }
  }
  __syncthreads();
  MRST(6);
  if (S.qset) {
    for (uint32_t x = x0; x < n * nt8; x += NT) {
      const uint32_t j = x / nt8, t = x % nt8;
      const PmRes r = L.s_res[j];
      if (r.status != ST_OK) continue;
      const uint32_t c0 = 8 * t;
      const bool rc = r.chunk - c0 < 8u;
      const bool first = x == x0 && tid >= 64;   // this thread's guessed tile
      const uint32_t ro = rc ? (first && r.ing == ging ? gr : P.ridx[r.chunk * P.Qpc + r.ing]) & mask : 0u;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (first && r.tag == gtag) v = gv;
      else if (c0 < P.SS) v = *reinterpret_cast<const PM_G uint4*>(P.tabT + tabT_index(P.H, r.tag, c0));
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
      auto put = [&](uint32_t e, uint32_t o) {
        w[e >> 1] = (w[e >> 1] & ~(0xffffu << (16 * (e & 1)))) | ((o & 0xffffu) << (16 * (e & 1)));
      };
      if (r.pp != kDefaultProgramPoint && (r.pp >> lg) - c0 < 8u) put((r.pp >> lg) - c0, r.pp & mask);
      if (rc) put(r.chunk - c0, ro);
      *reinterpret_cast<PM_G uint4*>(S.qset + (uint64_t)(b0 + j) * S.qw + c0) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  MRST(7);
}

// L2Dist of the first `dim` floats of an LDS row against q (device), one
// 8-lane group; bit-exact (see k_l2_rows).  Call with lanes 0..7 of a wave.
__device__ __forceinline__ float l2_lds(const float* row, const float* __restrict__ q, uint32_t dim) {
  const uint32_t k = threadIdx.x & 7;
  const uint32_t dimS = dim & ~7u;
  float acc = 0.0f;
#pragma unroll 8   // the loads of 8 terms issued ahead of the (ordered) sum
  for (uint32_t t = k; t < dimS; t += 8) {
    const float d = __fsub_rn(row[t], q[t]);
    acc = __fadd_rn(acc, __fmul_rn(d, d));
  }
  acc = __fadd_rn(acc, __shfl_xor(acc, 1));
  acc = __fadd_rn(acc, __shfl_xor(acc, 2));
  acc = __fadd_rn(acc, __shfl_xor(acc, 4));
  float d = dimS ? acc : 0.0f;
  for (uint32_t i = dimS; i < dim; ++i) {
    const float t = __fsub_rn(row[i], q[i]);
    d = __fadd_rn(d, __fmul_rn(t, t));
  }
  return d;
}

constexpr uint32_t kMaxSSLds = 4096, kMaxELds = 2048;

template <uint32_t ME>
union RowBufT {   // one decoded entry (up to ME words); the L2 reads its leading floats
  uint64_t w[ME];
  float f[2 * ME];
};
using RowBuf = RowBufT<kMaxELds>;

// PmOutHdr::csum: the position-keyed hash of the row words [pf_w0, pf_w1)
// as written (the LDS copy, or zeros), pm_internal.h row_hash_mult.  Wave 0
// only; every lane returns the result.
template <class RB>
__device__ __forceinline__ uint64_t row_csum(const PmStep& S, const RB& row, bool has_row) {
  uint64_t x = 0;
  for (uint32_t w = S.pf_w0 + (threadIdx.x & 63); w < S.pf_w1; w += 64)
    x += (has_row ? row.w[w] : 0) * row_hash_mult(w);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Result publication into pinned (fine-grained) host memory.  The default
// (PM_PUBLISH 0): lane 0 stores the header as soon as the row is final in
// LDS, and no wave waits for its row stores to be acknowledged.  The token is
// a progress mark only: the host takes the step's results after the step's
// completion event (system-scope release after the last kernel, pm_engine.cpp
// wait_step), and checks the row hash there as an assertion (pm_internal.h
// PmOutHdr).  (4: row stores acknowledged before a workgroup barrier and the
// header, as in round 1 — rows still arrive after the token, measured.)  Two
// in-kernel ordered forms, both measured with 0 torn rows in 49M but 2.8x /
// 4.4x the kernel time, are kept as build options:
//   1: lane 0 stores the other header fields, then a SYSTEM-scope release
//      (buffer_wbl2 sc0 sc1: the XCD L2's dirty lines, every wave's included,
//      are written back) and an explicit s_waitcnt vmcnt(0) — inline asm, so
//      the compiler cannot drop the wait after the write-back
//      (MI355X_MICROARCH.md "Compiler hazard") — then the token as ONE 8-byte
//      system-scope store {dist, token};
//   3: every row and header word stored write-through at system scope
//      (sc0 sc1), each wave's stores acknowledged before the barrier, the
//      token stored after lane 0's header stores are acknowledged.
#ifndef PM_PUBLISH
#define PM_PUBLISH 0
#endif
__device__ __forceinline__ void row_store(PM_G uint64_t* p, uint64_t v) {
  if (PM_PUBLISH >= 2) __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else *p = v;
}
__device__ __forceinline__ void publish_hdr(const PmStep& S, uint32_t s, uint32_t status, uint32_t ref,
                                            float d, uint64_t csum) {
  PM_G PmOutHdr* h = S.hdr_h + s;
  if (PM_PUBLISH == 0) {   // lane 0 (it holds d and csum) as soon as the row is final in LDS
    if (threadIdx.x == 0) *h = PmOutHdr{status, ref, d, S.token, csum + S.token * kCsumMix, 0};
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint64_t tok = ((uint64_t)S.token << 32) | __float_as_uint(d);   // {dist, token}: bytes 8..15
  if (PM_PUBLISH == 4) {   // round 1's drained form: row stores acknowledged, then the plain header
    *h = PmOutHdr{status, ref, d, S.token, csum + S.token * kCsumMix, 0};
    return;
  }
  PM_G uint64_t* w = reinterpret_cast<PM_G uint64_t*>(h);
  if (PM_PUBLISH == 3) {   // every byte written through at system scope: no L2 write-back needed
    __hip_atomic_store((uint64_t*)w, ((uint64_t)ref << 32) | status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store((uint64_t*)(w + 2), csum + S.token * kCsumMix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store((uint64_t*)(w + 1), tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  w[0] = ((uint64_t)ref << 32) | status;
  w[2] = csum + S.token * kCsumMix;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store((uint64_t*)(w + 1), tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// What a k_answer workgroup does for its sub-query.
enum : uint32_t { A_ZERO = 0, A_FINAL = 1, A_CHAINED = 2, A_CACHED = 3, A_DUMMY = 4 };

// The hint search row of a refreshed hint (PmPart::cur): hint r.hit now carries
// backup hint (r.chunk, r.ing)'s tag, whose PRF values tabT holds (pir.go:
// 460-462).  Written by the hint's final holder in this step (flags bit 1
// clear); read by the next step's hint search, after this launch ends.
__device__ __forceinline__ void refresh_cur(const PmPart& P, const PmRes& r, uint32_t tid, uint32_t nt) {
  const uint32_t ntag = P.PH + r.chunk * P.Qpc + r.ing;
  for (uint32_t c = tid; c < P.SS; c += nt) P.cur[cur_index(P.PH, P.curk, c, r.hit)] = P.tabT[tabT_index(P.H, ntag, c)];
}

// Decode one chained sub-query (its hint was refreshed earlier in this step)
// once every earlier refresh is visible; the whole workgroup participates.
template <bool GRAN, class RB>
__device__ void decode_chained(const PmStep& S, uint32_t s, RB& row) {
  const PmSub sub = step_sub(S, s);
  const PmRes r = res_after_acquire<GRAN>(S, s);
  const PmPart& P = S.parts[sub.part];
  const uint32_t E = S.E, EX = E & ~3u, tid = threadIdx.x;
  const uint64_t slot = (uint64_t)r.chunk * P.Qpc + r.ing;
  const uint64_t* rv = P.rval + slot * E;
  const uint64_t* bp = P.parity + ((uint64_t)P.PH + slot) * E;
  uint64_t* pp = P.parity + (uint64_t)r.hit * E;
  const uint64_t* a = S.ans + (uint64_t)s * E;
  for (uint32_t w = tid; w < E; w += blockDim.x) {
    uint64_t v = 0;
    if (w < EX) {
      v = a[w] ^ rv[w] ^ pp[w];
      pp[w] = bp[w] ^ v;
    } else {
      pp[w] = bp[w];
    }
    row.w[w] = v;
  }
  if (!(r.flags & 2u)) refresh_cur(P, r, tid, blockDim.x);
  __syncthreads();
  PM_G uint64_t* orow = S.rows_h + (uint64_t)s * E;
  uint64_t* ar = P.arena + (uint64_t)r.slot * E;
  for (uint32_t w = tid; w < E; w += blockDim.x) ar[w] = row.w[w];
  for (uint32_t w = (S.rows_partial ? S.pf_w0 : 0) + tid; w < (S.rows_partial ? S.pf_w1 : E); w += blockDim.x)
    row_store(orow + w, row.w[w]);
  float d = 0.0f;
  const float* qq = P.qv ? P.qv : S.q;
  if (qq && tid < 8) d = l2_lds(row.f, qq, S.dim);
  uint64_t cs = 0;
  if (tid < 64) cs = row_csum(S, row, true);
  publish_hdr(S, s, r.status, r.slot, d, cs);
  __syncthreads();
}

// The finisher of a step (see resolver_count), after its acquire: decodes the
// chained sub-queries in list order and re-arms the counters.  Whole workgroup.
template <bool GRAN, class RB>
__device__ void finish_step(const PmStep& S, RB& row) {
  const uint32_t nchain = S.done[2];
  for (uint32_t k = 0; k < nchain; ++k) decode_chained<GRAN>(S, S.done[3 + k], row);
  if (threadIdx.x == 0) chain_rearm(S);
}

// MSS / ME: the largest SetSize / entry words the instance serves (the
// generic instance: every shape of step_max_ss / step_max_e).
template <int NT, uint32_t MSS = kMaxSSLds, uint32_t ME = kMaxELds>
struct AnswerLds {
  uint32_t f[17];   // k_step: granule fields, per-wave first candidates, predicted index
  __attribute__((aligned(16))) uint16_t qo[MSS];   // the query set: in-chunk offsets < ChunkSize <= 32768
  uint64_t red[NT * 2];
  __attribute__((aligned(16))) RowBufT<ME> row;
  uint32_t s_last;
};

// What the answer of sub-query s needs from its resolution: query set,
// gathered row, decode operands.
__device__ __forceinline__ uint32_t answer_mode(const PmRes& r) {
  return r.status == ST_OK ? ((r.flags & 1u) ? A_CHAINED : A_FINAL)
       : r.status == ST_CACHED ? A_CACHED
       : r.status == ST_DUMMY ? A_DUMMY : A_ZERO;
}

// The query set of (r, mode) for chunks [lo, hi) into qo (pir.go:363-371
// dummy; :424-444 real): PRF row of the tag, program point and replacement
// substituted.
template <int NT>
__device__ __forceinline__ void set_range(const PmPart& P, const PmSub& sub, const PmRes& r, uint32_t mode,
                                          uint16_t* qo, uint32_t lo, uint32_t hi) {
  const uint32_t tid = threadIdx.x, mask = P.CS - 1, lg = P.log2CS;
  if (mode == A_FINAL || mode == A_CHAINED) {
    const uint32_t pchunk = r.pp != kDefaultProgramPoint ? (r.pp >> lg) : kNone;
    for (uint32_t i = lo + tid; i < hi; i += NT) {
      uint32_t o = P.tabT[tabT_index(P.H, r.tag, i)];
      if (i == pchunk) o = r.pp & mask;
      if (i == r.chunk) o = P.ridx[r.chunk * P.Qpc + r.ing] & mask;
      qo[i] = (uint16_t)o;
    }
  } else if (mode == A_DUMMY) {
    for (uint32_t i = lo + tid; i < hi; i += NT)
      qo[i] = (uint16_t)(hash4(P.seed, DOM_DUMMY, P.idx, sub.idx, i) & mask);
  }
}

// The server XOR gather (HOT LOOP E) of the set's chunks [lo, hi) into
// row.w[0..EX): every row load of a batch is issued before the first is
// consumed, so the gather is one HBM round trip per kG rows a thread reads.
template <int W, int NT, int kG, class RB>
__device__ __forceinline__ void gather_range(const PmStep& S, const PmPart& P, const uint16_t* qo, uint64_t* red,
                                             RB& row, uint32_t lo, uint32_t hi) {
  const uint32_t tid = threadIdx.x, E = S.E, EX = E & ~3u, NSEG = EX / W;
  const PM_G uint64_t* base = S.db + P.row0 * E;
  for (uint32_t seg0 = 0; seg0 < NSEG; seg0 += NT) {
    const uint32_t nseg = min(NSEG - seg0, (uint32_t)NT);
    const uint32_t nsl = NT / nseg;
    const uint32_t sl = tid / nseg, seg = seg0 + tid % nseg;
    uint64_t a0 = 0, a1 = 0;
    if (sl < nsl) {
      typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
      for (uint32_t i0 = lo + sl; i0 < hi; i0 += kG * nsl) {
        uint32_t rr[kG];   // partition rows (< 2^32): 32-bit, so the batch fits 64 VGPRs
        // the batch's set offsets: unconditional LDS reads (clamped index),
        // all in flight before one wait (a read inside each bounds branch
        // waited for its own result before the next was issued)
#pragma unroll
        for (int u = 0; u < kG; ++u) rr[u] = qo[min(i0 + u * nsl, hi - 1)];
#pragma unroll
        for (int u = 0; u < kG; ++u) {
          const uint32_t i = i0 + u * nsl;
          rr[u] = i < hi ? i * P.CS + rr[u] : ~0u;
        }
        u64x2 x[kG];
#pragma unroll
        for (int u = 0; u < kG; ++u) {
          x[u] = u64x2{0, 0};
          if (rr[u] < P.N) {
            const PM_G uint64_t* q = base + (uint64_t)rr[u] * E + (uint64_t)seg * W;
            if (W == 2) x[u] = *reinterpret_cast<const PM_G u64x2*>(q);
            else x[u].x = *q;
          }
        }
#pragma unroll
        for (int u = 0; u < kG; ++u) { a0 ^= x[u].x; a1 ^= x[u].y; }
      }
    }
    red[tid * 2] = a0;
    red[tid * 2 + 1] = a1;
    __syncthreads();
    if (tid < nseg) {
      uint64_t x0 = 0, x1 = 0;
      for (uint32_t k = 0; k < nsl; ++k) {
        x0 ^= red[(k * nseg + tid) * 2];
        x1 ^= red[(k * nseg + tid) * 2 + 1];
      }
      row.w[seg * W] = x0;
      if (W == 2) row.w[seg * W + 1] = x1;
    }
    __syncthreads();
  }
}

// k_step's guess of sub-query s's resolution (see answer_role): a dummy's set
// needs none; a real one's first stale candidate over every hint (the match
// role's predicate and state; one tag load per wave), with the in-chunk
// index predicted from the chunk's QueryHistogram.  Whole workgroup (LDS:
// L.f, L.red).  Returns the guessed answer mode (kNone: no guess).
template <int NT, class LDS>
__device__ __forceinline__ uint32_t step_guess(const PmStep& S, uint32_t s, const PmSub& sub, const PmPart& P, LDS& L,
                                               PmRes& g) {
  constexpr bool GRAN = true;   // (stamps)
  (void)GRAN;
  g = PmRes{kNone, 0, 0, 0, 0, 0, 0, 0};
  if (S.no_guess) return kNone;
  if (sub.kind == SUB_DUMMY) {
    g.status = ST_DUMMY;
    return A_DUMMY;
  }
  if (!(sub.kind == SUB_REAL && sub.idx < P.N)) return kNone;
  const uint32_t tid = threadIdx.x, mask = P.CS - 1, lg = P.log2CS;
  constexpr int HPT = kLdsPH / NT;   // k_step: PH <= kLdsPH
  const uint32_t ch = (uint32_t)(sub.idx >> lg), off = (uint32_t)(sub.idx & mask);
  const uint32_t wave = tid >> 6, lane = tid & 63;
  uint32_t rv[HPT];
  const PM_G uint16_t* crow = P.cur + cur_row(P.PH, P.curk, ch);   // match: value == offset (see match_role)
#pragma unroll
  for (int u = 0; u < HPT; ++u) rv[u] = u * NT + tid < P.PH ? crow[cur_row_off(P.curk, u * NT + tid)] : kNone;
  const uint32_t h0k = wave == 0 ? P.hist[ch] : 0;
  // per wave the lowest matching hint (lower u first: hints u*NT + tid)
  uint32_t wh = kNone, wt = 0, wp = 0;
#pragma unroll
  for (int u = 0; u < HPT; ++u) {
    const uint64_t bm = __ballot(rv[u] == off);
    if (bm && wh == kNone) wh = u * NT + wave * 64 + (uint32_t)__builtin_ctzll(bm);
  }
  if (wh != kNone) { wt = P.tag[wh]; wp = P.pp[wh]; }
  if (lane == 0) { L.f[wave] = wh; L.red[2 * wave] = wt; L.red[2 * wave + 1] = wp; }
  if (wave == 0) {
    const uint32_t pb0 = step_sb(S, sub.part), pn = step_sb(S, sub.part + 1) - pb0;
    PmSub st;
    bool validt;
    const uint32_t sg0 = predict_ing(S, P, pb0, pn, s - pb0, ch, h0k, st, validt);
    if (lane == 0) L.f[16] = sg0;
  }
  __syncthreads();
  uint32_t c1 = kNone, t1 = 0, p1 = 0;
  const uint32_t sg = L.f[16];
  AS(0);
  for (uint32_t w = 0; w < NT / 64; ++w)
    if (L.f[w] < c1) { c1 = L.f[w]; t1 = (uint32_t)L.red[2 * w]; p1 = (uint32_t)L.red[2 * w + 1]; }
  __syncthreads();
  if (c1 != kNone && sg < P.Qpc && ch < P.SS) {
    g = PmRes{ST_OK, c1, ch, sg, t1, p1, 0, 0};
    return A_FINAL;
  }
  return kNone;
}

// One sub-query's answer (HOT LOOPs D + E, decode, outputs).  GRAN: inside
// k_step.  There the answer starts before its partition's resolver is done:
// a dummy sub-query's set does not depend on the resolution at all, and a
// real one's usually is the one its first stale candidate gives (hint c1 with
// its tag / program point, the in-chunk index predicted from the chunk's
// QueryHistogram — its match workgroup's record).  The set is expanded, the
// rows gathered and the decode operands loaded for that guess while the
// resolver runs; its result then either equals the guess in every field the
// answer reads (kept) or the work is redone for the actual result.
template <int W, bool GRAN, int NT, class LDS>
__device__ __forceinline__ void answer_role(const PmStep& S, uint32_t s, LDS& L) {
  uint16_t* const qo = L.qo;
  uint64_t* const red = L.red;
  auto& row = L.row;
  const uint32_t tid = threadIdx.x;
  const uint32_t E = S.E, EX = E & ~3u;
  const PmSub sub = step_sub(S, s);
  const PmPart& P = S.parts[sub.part];
  PM_G uint64_t* const orow = S.rows_h + (uint64_t)s * E;
  const bool stamp_wg = s == 0;
  STAMP_AT(stamp_wg, 48);
  AST(0);
#ifdef PM_ANSWER_STAMPS
  if (!GRAN && threadIdx.x == 0 && S.stamps)
    S.stamps[(uint64_t)blockIdx.x * 8 + 6] = ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                             (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
  // the search query the decoded row is scored against (L2): loaded now, in
  // flight with everything else, and put into LDS once the gather is done
  const float* const qq = P.qv ? P.qv : S.q;
  const bool q_lds = qq && S.dim <= 2 * NT;   // red[] holds 2 * NT floats... as NT u64 pairs
  float qreg0 = 0.0f, qreg1 = 0.0f;
  if (q_lds) {
    if (tid < S.dim) qreg0 = qq[tid];
    if (tid + NT < S.dim) qreg1 = qq[tid + NT];
  }
  // the pre-expanded query set (S.qset, three-kernel path after k_match_resolve_s),
  // loaded now, in flight with the resolution record
  const bool qpre = !GRAN && S.qset != nullptr;
  uint4 qpv = make_uint4(0, 0, 0, 0);
  if (qpre && tid < S.qw / 8) qpv = *reinterpret_cast<const PM_G uint4*>(S.qset + (uint64_t)s * S.qw + 8 * tid);
  uint64_t e_rv = 0, e_bp = 0, e_pp = 0;
  uint32_t e_cur = kSkip;   // the refreshed hint's new search-row value at chunk tid (refresh_cur)
  // set expansion + gather into row.w[0..EX) and the decode operands for (r, mode)
  auto gather = [&](const PmRes& r, uint32_t mode, uint32_t lo, uint32_t hi) {
    // a pre-expanded set goes to LDS before any later load is issued (its wait
    // then covers only the loads issued with the record)
    if (qpre && (mode == A_FINAL || mode == A_CHAINED) && tid < S.qw / 8)
      *reinterpret_cast<uint4*>(qo + 8 * tid) = qpv;
    // decode operands: independent of the gather, issued first (pir.go:450-468)
    const uint64_t dslot = (uint64_t)r.chunk * P.Qpc + r.ing;
    if (mode == A_FINAL && !(r.flags & 2u) && tid < P.SS)   // the new tag's PRF row (backup hint (chunk, ing))
      e_cur = P.tabT[tabT_index(P.H, P.PH + r.chunk * P.Qpc + r.ing, tid)];
    if (mode == A_FINAL && tid < E) {
      e_rv = P.rval[dslot * E + tid];
      e_bp = P.parity[((uint64_t)P.PH + dslot) * E + tid];
      e_pp = P.parity[(uint64_t)r.hit * E + tid];
    }
    if (!GRAN && S.nsplit > 1) {   // k_gather did the set: fold its partial XORs
      if (mode == A_FINAL || mode == A_CHAINED || mode == A_DUMMY) {
        const PM_G uint64_t* px = S.part_x + (uint64_t)s * S.nsplit * EX;
        const uint32_t G = NT >= 2 * EX ? NT / EX : 1;   // partial groups folded side by side
        if (G == 1) {
          for (uint32_t w = tid; w < EX; w += NT) {
            uint64_t x = 0;
            for (uint32_t j = 0; j < S.nsplit; ++j) x ^= px[(uint64_t)j * EX + w];
            row.w[w] = x;
          }
        } else {
          if (tid < EX * G) {
            const uint32_t w = tid % EX, g0 = tid / EX;
            uint64_t x = 0;
            for (uint32_t j = g0; j < S.nsplit; j += G) x ^= px[(uint64_t)j * EX + w];
            red[tid] = x;
          }
          __syncthreads();
          if (tid < EX) {
            uint64_t x = 0;
            for (uint32_t g0 = 0; g0 < G; ++g0) x ^= red[g0 * EX + tid];
            row.w[tid] = x;
          }
        }
      }
      __syncthreads();
      return;
    }
    // ---- query set (pir.go:363-371 dummy; :424-444 real) -------------------
    if (qpre && (mode == A_FINAL || mode == A_CHAINED)) {
      // expanded by k_match_resolve_s: in LDS already (above)
    } else {
      set_range<NT>(P, sub, r, mode, qo, lo, hi);
    }
    STAMP_AT(stamp_wg && mode == A_FINAL, 49);
    __syncthreads();
    AS(1);
    STAMP_AT(stamp_wg, 50);
    AST(2);
    // ---- server XOR gather (HOT LOOP E) into row.w[0..EX) ------------------
    // (k_step, GRAN: one client's rows, a thread's whole share in one batch)
    if (mode == A_FINAL || mode == A_CHAINED || mode == A_DUMMY)
      gather_range<W, NT, GRAN ? PM_STEP_KG : PM_ANSWER_KG>(S, P, qo, red, row, lo, hi);
  };
  PmRes r;
  uint32_t mode;
  if (GRAN) {
    // ---- the guess (see above), from this sub-query's match record ---------
    PmRes g;
    const uint32_t gmode = step_guess<NT>(S, s, sub, P, L, g);
    // with gather helpers (S.nhelp) this workgroup gathers the set's first
    // range only; the helpers' partials of the others are merged below
    const bool helped = S.nhelp && (gmode == A_FINAL || gmode == A_DUMMY);
    if (gmode != kNone) gather(g, gmode, 0, helped ? P.SS / (S.nhelp + 1) : P.SS);
    // the helpers' partials, merged while the resolver still runs (a later
    // redo overwrites row.w anyway).  Each helper's guess must be this one
    // (the state it read may have been refreshed by then).  Every granule
    // load of a thread is in flight before the first is checked.
    bool help_ok = true;
    if (helped) {
      // one round trip: a thread's partial words of every helper and (lanes
      // < nhelp) that helper's guess fields are all in flight before the
      // first is checked; a granule not yet written is then polled
      const PM_G uint64_t* const hbase = S.helpg + (uint64_t)s * kStepHelpMax * kHelpGran;
      const uint32_t w = tid;   // EX <= kHelpWords <= NT: one word per thread
      uint64_t v[2 * kStepHelpMax], fv[6];
#pragma unroll
      for (uint32_t k = 0; k < kStepHelpMax; ++k) {
        const bool ld = k < S.nhelp && w < EX;
        v[2 * k] = ld ? ld64<true>(hbase + k * kHelpGran + 2 * w) : 0;
        v[2 * k + 1] = ld ? ld64<true>(hbase + k * kHelpGran + 2 * w + 1) : 0;
      }
      const PM_G uint64_t* const hf = hbase + (uint64_t)min(tid, kStepHelpMax - 1) * kHelpGran + 2 * kHelpWords;
#pragma unroll
      for (int i = 0; i < 6; ++i) fv[i] = tid < S.nhelp ? ld64<true>(hf + i) : 0;
      if (tid < S.nhelp) {
        uint32_t f[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) f[i] = (uint32_t)(fv[i] >> 32) == S.token ? (uint32_t)fv[i] : get_g(hf + i, S);
        L.f[8 + tid] = f[0] == gmode && (gmode == A_DUMMY || (f[1] == g.hit && f[2] == g.chunk && f[3] == g.ing &&
                                                              f[4] == g.tag && f[5] == g.pp)) ? 1u : 0u;
      }
      __syncthreads();
      for (uint32_t k = 0; k < S.nhelp; ++k) help_ok = help_ok && L.f[8 + k] != 0;
      if (help_ok && w < EX) {
        uint64_t x = row.w[w];
#pragma unroll
        for (uint32_t k = 0; k < kStepHelpMax; ++k) {
          if (k >= S.nhelp) break;
          const PM_G uint64_t* hp = hbase + k * kHelpGran + 2 * w;
          const uint32_t lo = (uint32_t)(v[2 * k] >> 32) == S.token ? (uint32_t)v[2 * k] : get_g(hp, S);
          const uint32_t hi = (uint32_t)(v[2 * k + 1] >> 32) == S.token ? (uint32_t)v[2 * k + 1] : get_g(hp + 1, S);
          x ^= (uint64_t)lo | ((uint64_t)hi << 32);
        }
        row.w[w] = x;
      }
      __syncthreads();
    }
    TS(1);
    // ---- the resolver's record of this sub-query ----------------------------
    if (tid < G_RES) L.f[tid] = get_g(S.resg + (uint64_t)s * G_RES + tid, S);
    __syncthreads();
    r = PmRes{L.f[0], L.f[1], L.f[2], L.f[3], L.f[4], L.f[5], L.f[6], L.f[7]};
    mode = answer_mode(r);
    const bool kept = mode == gmode &&
                      (mode == A_DUMMY || (r.hit == g.hit && r.chunk == g.chunk && r.ing == g.ing &&
                                           r.tag == g.tag && r.pp == g.pp));
    TS_SEEN(kept ? 1u : 0u);
    const bool redo = !kept || !help_ok;
    if (redo) {
      e_rv = e_bp = e_pp = 0;
      gather(r, mode, 0, P.SS);
    }
  } else {
    r = S.res[s];
    mode = answer_mode(r);
    AST(1);
    gather(r, mode, 0, P.SS);
  }
  const uint64_t dslot = (uint64_t)r.chunk * P.Qpc + r.ing;
  const uint64_t* rv = P.rval + dslot * E;
  const uint64_t* bp = P.parity + ((uint64_t)P.PH + dslot) * E;
  uint64_t* pp = P.parity + (uint64_t)r.hit * E;
  STAMP_AT(stamp_wg, 51);
  AST(3);
  // ---- decode + refresh, or the cached row -----------------------------
  if (mode == A_FINAL) {
    if (!(r.flags & 2u)) {   // refresh_cur with the row prefetched with the decode operands
      if (tid < P.SS) P.cur[cur_index(P.PH, P.curk, tid, r.hit)] = (uint16_t)e_cur;
      if (P.SS > NT) refresh_cur(P, r, tid + NT, NT);   // SetSize > workgroup (BIGANN): the rest
    }
    for (uint32_t w = tid; w < E; w += NT) {
      const uint64_t rvw = w < NT ? e_rv : rv[w], bpw = w < NT ? e_bp : bp[w],
                     ppw = w < NT ? e_pp : pp[w];
      uint64_t v = 0;
      if (w < EX) v = row.w[w] ^ rvw ^ ppw;
      const uint64_t nw = w < EX ? bpw ^ v : bpw;
      if (PM_EPI_NT) __builtin_nontemporal_store(nw, pp + w);
      else pp[w] = nw;
      row.w[w] = v;
    }
  } else if (mode == A_CHAINED) {
    for (uint32_t w = tid; w < E; w += NT) S.ans[(uint64_t)s * E + w] = w < EX ? row.w[w] : 0;
  } else if (mode == A_CACHED) {
    const uint64_t* a = P.arena + (uint64_t)r.slot * E;
    for (uint32_t w = tid; w < E; w += NT) row.w[w] = a[w];
  }
  float* const qf = reinterpret_cast<float*>(red);   // free since the gather's last barrier
  if (q_lds) {
    if (tid < S.dim) qf[tid] = qreg0;
    if (tid + NT < S.dim) qf[tid + NT] = qreg1;
  }
  __syncthreads();
  STAMP_AT(stamp_wg, 52);
  AST(4);
  // ---- results: row + header into pinned host memory, arena copy -----------
  if (mode != A_CHAINED) {
    const bool has_row = (mode == A_FINAL || mode == A_CACHED);
    // to the host: the whole row, or only the words its caller reads (graph search:
    // the neighbour list; the distance travels in the header)
    for (uint32_t w = (S.rows_partial ? S.pf_w0 : 0) + tid; w < (S.rows_partial ? S.pf_w1 : E); w += NT)
      row_store(orow + w, has_row ? row.w[w] : 0);
    if (mode == A_FINAL) {
      uint64_t* ar = P.arena + (uint64_t)r.slot * E;
      for (uint32_t w = tid; w < E; w += NT) {
        if (PM_EPI_NT) __builtin_nontemporal_store(row.w[w], ar + w);
        else ar[w] = row.w[w];
      }
    }
    float d = 0.0f;
    if (has_row && qq && tid < 8) d = l2_lds(row.f, q_lds ? qf : qq, S.dim);
    uint64_t cs = 0;
    if (tid < 64) cs = row_csum(S, row, has_row);
    publish_hdr(S, s, r.status, r.slot, d, cs);
  }
  STAMP_AT(stamp_wg, 53);
  AST(5);
  // ---- arrival: workgroups of refresh chains count in; the last one decodes
  // the chained sub-queries in order.  Producer side: drain this wave's stores,
  // barrier, one lane releases at agent scope and counts (MI355X_MICROARCH.md
  // § visibility).  Workgroups outside every chain skip all of this.
  if (!(r.status == ST_OK && (r.flags & 3u))) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    L.s_last = (uint32_t)chain_add(S, 1);
    if (L.s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!L.s_last) return;
  finish_step<GRAN>(S, row);
}

template <int W>
#ifndef PM_ANSWER_WGS
#define PM_ANSWER_WGS 8   // min waves per SIMD (HIP launch bounds): <= 64 VGPRs, four 512-thread workgroups per CU
#endif
__global__ void __launch_bounds__(kAnsBlock, PM_ANSWER_WGS) k_answer(PmStep S) {
  __shared__ AnswerLds<kAnsBlock> L;
  answer_role<W, false, kAnsBlock>(S, blockIdx.x, L);
}

// The same answer for the search-sized shapes (SetSize <= 1024, entries <= 256
// words: SIFT1M's 124 x 80, MS-MARCO's 196 x 112) with NT-thread workgroups
// and a 7-8 KB LDS footprint.  The generic instance's 33 KB of LDS (sets up
// to 4096 chunks, entries up to 2048 words) holds a CU to four workgroups,
// i.e. four sub-queries in flight; here registers alone bound it (64 VGPRs:
// 32 waves per CU), so a CU holds 32 / (NT / 64) sub-queries whose latency-
// bound phases (resolution, set expansion, decode, publication) overlap the
// others' row gathers.
constexpr uint32_t kSmallSS = 1024, kSmallE = 256;
template <int W, int NT>
__global__ void __launch_bounds__(NT, PM_ANSWER_WGS) k_answer_s(PmStep S) {
  __shared__ AnswerLds<NT, kSmallSS, kSmallE> L;
  answer_role<W, false, NT>(S, blockIdx.x, L);
}

// ---- k_answer_p: two sub-queries per workgroup, software-pipelined --------
// k_answer_s at the batched serving shape (6,144 sub-queries over 4,096
// resident slots) starts every resident workgroup in its latency phases at
// once (record + query set, then decode and publication), so HBM idles at the
// kernel's start, between the two rounds of workgroups and at its end: 75 us
// alone for 332 MB, where the bare gather of 480 MB takes 66 us
// (tools/gather_bench.hip, fresh rows every launch).  Here a workgroup owns
// sub-queries A = blockIdx.x and B = blockIdx.x + gridDim.x (grid = nsub / 2:
// every workgroup resident from the start), loads both records and query sets
// in one round trip, gathers A, issues B's first row batch, and decodes and
// publishes A while those rows are in flight: B's prologue hides behind A's
// gather and A's epilogue behind B's first batch.  Same results as
// answer_role (pre-expanded query sets, S.qset; no split gather).
constexpr int kAnsPNT = 128;
template <int NT>
struct AnswerPLds {
  __attribute__((aligned(16))) uint16_t qo[2][kSmallSS];
  uint64_t red[NT * 2];
  __attribute__((aligned(16))) RowBufT<kSmallE> row;
  uint32_t s_last;
};
struct AnsQ {   // one sub-query's operands in k_answer_p
  uint32_t s, part, mode;
  PmRes r;
  uint64_t idx;   // the sub-query's index (DUMMY: the dummy counter)
  uint64_t e_rv, e_bp, e_pp;
  uint32_t e_cur;
  float q0, q1;
};
template <int W, int NT>
__device__ __forceinline__ void ansp_decode_ops(const PmStep& S, AnsQ& a) {
  const PmPart& P = S.parts[a.part];
  const uint32_t tid = threadIdx.x, E = S.E;
  a.e_rv = a.e_bp = a.e_pp = 0;
  a.e_cur = kSkip;
  if (a.mode != A_FINAL) return;
  const PmRes& r = a.r;
  const uint64_t dslot = (uint64_t)r.chunk * P.Qpc + r.ing;
  if (PM_DEC_NT) {
    if (!(r.flags & 2u) && tid < P.SS)
      a.e_cur = __builtin_nontemporal_load(P.tabT + tabT_index(P.H, P.PH + r.chunk * P.Qpc + r.ing, tid));
    if (tid < E) {
      a.e_rv = __builtin_nontemporal_load(P.rval + dslot * E + tid);
      a.e_bp = __builtin_nontemporal_load(P.parity + ((uint64_t)P.PH + dslot) * E + tid);
      a.e_pp = __builtin_nontemporal_load(P.parity + (uint64_t)r.hit * E + tid);
    }
    return;
  }
  if (!(r.flags & 2u) && tid < P.SS) a.e_cur = P.tabT[tabT_index(P.H, P.PH + r.chunk * P.Qpc + r.ing, tid)];
  if (tid < E) {
    a.e_rv = P.rval[dslot * E + tid];
    a.e_bp = P.parity[((uint64_t)P.PH + dslot) * E + tid];
    a.e_pp = P.parity[(uint64_t)r.hit * E + tid];
  }
}
// the query set of a gathering sub-query into qo (pre-expanded, or the dummy's)
__device__ __forceinline__ void ansp_set(const PmStep& S, const AnsQ& a, uint4 qpv, uint16_t* qo) {
  const uint32_t tid = threadIdx.x;
  if (a.mode == A_FINAL || a.mode == A_CHAINED) {
    if (tid < S.qw / 8) *reinterpret_cast<uint4*>(qo + 8 * tid) = qpv;
  } else if (a.mode == A_DUMMY) {
    const PmPart& P = S.parts[a.part];
    const uint32_t mask = P.CS - 1;
    for (uint32_t i = tid; i < P.SS; i += blockDim.x) qo[i] = (uint16_t)(hash4(P.seed, DOM_DUMMY, P.idx, a.idx, i) & mask);
  }
}
template <int W, int NT, int KG>
struct AnsGather {   // one thread's share of a sub-query's XOR gather (HOT LOOP E)
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  uint32_t seg, sl, nsl;
  uint64_t a0 = 0, a1 = 0;
  u64x2 x[KG];
  __device__ __forceinline__ void init(uint32_t E) {
    const uint32_t NSEG = (E & ~3u) / W;   // <= NT at the shapes this kernel serves (E <= kSmallE, W 2)
    nsl = NT / NSEG;
    sl = threadIdx.x / NSEG;
    seg = threadIdx.x % NSEG;
  }
  // batch b: rows i = sl + (b * KG + u) * nsl
  __device__ __forceinline__ void load(const PmStep& S, const PmPart& P, const uint16_t* qo, uint32_t b) {
    const uint32_t i0 = sl + b * KG * nsl;
    uint32_t rr[KG];
#pragma unroll
    for (int u = 0; u < KG; ++u) rr[u] = qo[min(i0 + u * nsl, P.SS - 1)];
#pragma unroll
    for (int u = 0; u < KG; ++u) {
      const uint32_t i = i0 + u * nsl;
      rr[u] = (sl < nsl && i < P.SS) ? i * P.CS + rr[u] : ~0u;
    }
    const PM_G uint64_t* base = S.db + P.row0 * S.E;
#pragma unroll
    for (int u = 0; u < KG; ++u) {
      x[u] = u64x2{0, 0};
      if (rr[u] < P.N) {
        const PM_G uint64_t* q = base + (uint64_t)rr[u] * S.E + (uint64_t)seg * W;
#if PM_ANSWER_NTLOAD
        if (W == 2) x[u] = __builtin_nontemporal_load(reinterpret_cast<const PM_G u64x2*>(q));
        else x[u].x = __builtin_nontemporal_load(q);
#else
        if (W == 2) x[u] = *reinterpret_cast<const PM_G u64x2*>(q);
        else x[u].x = *q;
#endif
      }
    }
  }
  __device__ __forceinline__ void fold() {
#pragma unroll
    for (int u = 0; u < KG; ++u) { a0 ^= x[u].x; a1 ^= x[u].y; }
  }
  __device__ __forceinline__ uint32_t batches(const PmPart& P) const { return (P.SS + KG * nsl - 1) / (KG * nsl); }
  // the slices' partial XORs -> row.w[0 .. E & ~3)
  template <class LDS>
  __device__ __forceinline__ void reduce(LDS& L, uint32_t E) {
    const uint32_t tid = threadIdx.x, NSEG = (E & ~3u) / W;
    L.red[tid * 2] = a0;
    L.red[tid * 2 + 1] = a1;
    __syncthreads();
    if (tid < NSEG) {
      uint64_t x0 = 0, x1 = 0;
      for (uint32_t k = 0; k < nsl; ++k) {
        x0 ^= L.red[(k * NSEG + tid) * 2];
        x1 ^= L.red[(k * NSEG + tid) * 2 + 1];
      }
      L.row.w[tid * W] = x0;
      if (W == 2) L.row.w[tid * W + 1] = x1;
    }
    __syncthreads();
  }
};
// decode + refresh, publication and the refresh-chain arrival of sub-query a
// whose gathered row is in L.row (answer_role's epilogue)
template <int W, int NT, class LDS>
__device__ __forceinline__ void ansp_epilogue(const PmStep& S, const AnsQ& a, LDS& L) {
  const PmPart& P = S.parts[a.part];
  const PmRes& r = a.r;
  const uint32_t tid = threadIdx.x, E = S.E, EX = E & ~3u, s = a.s, mode = a.mode;
  auto& row = L.row;
  const uint64_t dslot = (uint64_t)r.chunk * P.Qpc + r.ing;
  uint64_t* pp = P.parity + (uint64_t)r.hit * E;
  if (mode == A_FINAL) {   // pir.go:450-468
    if (!(r.flags & 2u)) {
      if (tid < P.SS) {
        PM_G uint16_t* dst = P.cur + cur_index(P.PH, P.curk, tid, r.hit);
        if (PM_REFRESH_NT) __builtin_nontemporal_store((uint16_t)a.e_cur, dst);
        else *dst = (uint16_t)a.e_cur;
      }
      if (P.SS > NT) refresh_cur(P, r, tid + NT, NT);
    }
    const uint64_t* rv = P.rval + dslot * E;
    const uint64_t* bp = P.parity + ((uint64_t)P.PH + dslot) * E;
    for (uint32_t w = tid; w < E; w += NT) {
      const uint64_t rvw = w < NT ? a.e_rv : rv[w], bpw = w < NT ? a.e_bp : bp[w], ppw = w < NT ? a.e_pp : pp[w];
      uint64_t v = 0;
      if (w < EX) v = row.w[w] ^ rvw ^ ppw;
      const uint64_t nw = w < EX ? bpw ^ v : bpw;
      if (PM_EPI_NT) __builtin_nontemporal_store(nw, pp + w);
      else pp[w] = nw;
      row.w[w] = v;
    }
  } else if (mode == A_CHAINED) {
    for (uint32_t w = tid; w < E; w += NT) S.ans[(uint64_t)s * E + w] = w < EX ? row.w[w] : 0;
  } else if (mode == A_CACHED) {
    const uint64_t* ar = P.arena + (uint64_t)r.slot * E;
    for (uint32_t w = tid; w < E; w += NT) row.w[w] = ar[w];
  }
  const float* const qq = P.qv ? P.qv : S.q;
  const bool q_lds = qq && S.dim <= 2 * NT;
  float* const qf = reinterpret_cast<float*>(L.red);
  if (q_lds) {
    if (tid < S.dim) qf[tid] = a.q0;
    if (tid + NT < S.dim) qf[tid + NT] = a.q1;
  }
  __syncthreads();
  if (mode != A_CHAINED) {
    const bool has_row = (mode == A_FINAL || mode == A_CACHED);
    PM_G uint64_t* const orow = S.rows_h + (uint64_t)s * E;
    for (uint32_t w = (S.rows_partial ? S.pf_w0 : 0) + tid; w < (S.rows_partial ? S.pf_w1 : E); w += NT)
      row_store(orow + w, has_row ? row.w[w] : 0);
    if (mode == A_FINAL) {
      uint64_t* ar = P.arena + (uint64_t)r.slot * E;
      for (uint32_t w = tid; w < E; w += NT) {
        if (PM_EPI_NT) __builtin_nontemporal_store(row.w[w], ar + w);
        else ar[w] = row.w[w];
      }
    }
    float d = 0.0f;
    if (has_row && qq && tid < 8) d = l2_lds(row.f, q_lds ? qf : qq, S.dim);
    uint64_t cs = 0;
    if (tid < 64) cs = row_csum(S, row, has_row);
    publish_hdr(S, s, r.status, r.slot, d, cs);
  }
  // arrival of a refresh-chain member; the last one decodes the chained
  // sub-queries in order (answer_role)
  if (r.status == ST_OK && (r.flags & 3u)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      L.s_last = (uint32_t)chain_add(S, 1);
      if (L.s_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (L.s_last) finish_step<false>(S, row);
  }
  __syncthreads();   // row and red are the next sub-query's
}
template <int W, int NT>
__device__ __forceinline__ void ansp_record(const PmStep& S, uint32_t s, AnsQ& a, uint4& qpv) {
  const uint32_t tid = threadIdx.x;
  a.s = s;
  const PmSub sub = step_sub(S, s);
  a.part = sub.part;
  a.idx = sub.idx;
  a.r = S.res[s];
  qpv = make_uint4(0, 0, 0, 0);
  if (tid < S.qw / 8) qpv = *reinterpret_cast<const PM_G uint4*>(S.qset + (uint64_t)s * S.qw + 8 * tid);
  const PmPart& P = S.parts[a.part];
  const float* const qq = P.qv ? P.qv : S.q;
  a.q0 = a.q1 = 0.0f;
  if (qq && S.dim <= 2 * NT) {
    if (tid < S.dim) a.q0 = qq[tid];
    if (tid + NT < S.dim) a.q1 = qq[tid + NT];
  }
}
__device__ __forceinline__ bool ansp_gathers(const AnsQ& a) {
  return a.mode == A_FINAL || a.mode == A_CHAINED || a.mode == A_DUMMY;
}
// A workgroup owns sub-queries s_k = blockIdx.x + k * gridDim.x (grid =
// nsub / PM_ANSWER_PK on the host, 2 by default) in two operand slots: while
// slot c gathers, slot c ^ 1 holds the next sub-query's record and query set;
// the next one's first row batch is issued before slot c's reduction, decode
// and publication, and slot c is refilled (record + query set of s_{k+2})
// while that batch is in flight.
template <int W, int NT, int KG, int C>
__device__ __forceinline__ bool ansp_turn(const PmStep& S, AnswerPLds<NT>& L, AnsQ (&q)[2], uint4 (&qpv)[2],
                                          AnsGather<W, NT, KG> (&g)[2], uint32_t k, bool first) {
  constexpr int N = C ^ 1;
  const uint32_t ns = S.nsub, G = gridDim.x;
  const bool hasN = blockIdx.x + (k + 1) * G < ns;
  if (ansp_gathers(q[C])) {
    const PmPart& P = S.parts[q[C].part];
    const uint32_t nb = g[C].batches(P);
    uint32_t b = 0;
    if (!first) { g[C].fold(); b = 1; }   // batch 0 was issued under the previous turn's epilogue
    for (; b < nb; ++b) {
      g[C].load(S, P, L.qo[C], b);
      g[C].fold();
    }
  }
  const bool gathN = hasN && ansp_gathers(q[N]);
  if (gathN) {
    g[N].a0 = g[N].a1 = 0;
    g[N].load(S, S.parts[q[N].part], L.qo[N], 0);
  }
  if (ansp_gathers(q[C])) g[C].reduce(L, S.E);
  ansp_epilogue<W, NT>(S, q[C], L);   // ends with a barrier: L.qo[C] is free
  if (!hasN) return false;
  if (blockIdx.x + (k + 2) * G < ns) {
    ansp_record<W, NT>(S, blockIdx.x + (k + 2) * G, q[C], qpv[C]);
    q[C].mode = answer_mode(q[C].r);
    ansp_set(S, q[C], qpv[C], L.qo[C]);
    __syncthreads();   // L.qo[C] is read by the next turn's first batch of it
  }
  ansp_decode_ops<W, NT>(S, q[N]);
  return true;
}
#ifndef PM_ANSWER_PK_MAX
#define PM_ANSWER_PK_MAX 2   // sub-queries per k_answer_p workgroup the kernel is built for (the host's PM_ANSWER_PK is
                             // clamped to it); 3 spills ~150 VGPRs at 80
#endif
#ifndef PM_ANSWER_P_TAIL
#define PM_ANSWER_P_TAIL 0   // k_answer_p's grid capped at PM_ANSWER_P_TAIL workgroups; the sub-queries past two
                             // per workgroup are answered one at a time at the end (diagnostic build)
#endif
#ifndef PM_ANSWER_P_WAVES
#define PM_ANSWER_P_WAVES 6   // min waves per SIMD: <= 80 VGPRs (the next sub-query's row batch stays live through
                              // an epilogue); 12 two-wave workgroups per CU = the 3,072 of a 6,144-sub-query step
#endif
template <int W, int NT>
__global__ void __launch_bounds__(NT, PM_ANSWER_P_WAVES) k_answer_p(PmStep S) {
  __shared__ AnswerPLds<NT> L;
  constexpr int KG = PM_ANSWER_KG;
  AnsQ q[2];
  uint4 qpv[2];
  const uint32_t ns = S.nsub, G = gridDim.x;
  const bool has1 = blockIdx.x + G < ns;
  // ---- prologue: the first two records and query sets, one round trip
  ansp_record<W, NT>(S, blockIdx.x, q[0], qpv[0]);
  ansp_record<W, NT>(S, has1 ? blockIdx.x + G : blockIdx.x, q[1], qpv[1]);
  q[0].mode = answer_mode(q[0].r);
  q[1].mode = answer_mode(q[1].r);
  ansp_decode_ops<W, NT>(S, q[0]);
  ansp_set(S, q[0], qpv[0], L.qo[0]);
  if (has1) ansp_set(S, q[1], qpv[1], L.qo[1]);
  __syncthreads();
  AnsGather<W, NT, KG> g[2];
  g[0].init(S.E);
  g[1].init(S.E);
  // straight-line turns (a loop keeps every slot's state live across its
  // back edge and spills): at most PM_ANSWER_PK_MAX sub-queries per workgroup
  static_assert(PM_ANSWER_PK_MAX >= 2 && PM_ANSWER_PK_MAX <= 4, "k_answer_p turns");
  if (!ansp_turn<W, NT, KG, 0>(S, L, q, qpv, g, 0, true)) return;
  if (!ansp_turn<W, NT, KG, 1>(S, L, q, qpv, g, 1, false)) return;
  if (PM_ANSWER_PK_MAX > 2 && !ansp_turn<W, NT, KG, 0>(S, L, q, qpv, g, 2, false)) return;
  if (PM_ANSWER_PK_MAX > 3) ansp_turn<W, NT, KG, 1>(S, L, q, qpv, g, 3, false);
#if PM_ANSWER_P_TAIL
  // a grid of fewer workgroups than sub-query pairs (PM_ANSWER_P_TAIL: the
  // host caps it at the resident slots): the rest, one at a time, unpipelined
  for (uint32_t s = blockIdx.x + 2 * G; s < ns; s += G) {
    AnsQ t;
    uint4 tq;
    ansp_record<W, NT>(S, s, t, tq);
    t.mode = answer_mode(t.r);
    ansp_decode_ops<W, NT>(S, t);
    ansp_set(S, t, tq, L.qo[0]);
    __syncthreads();
    AnsGather<W, NT, KG> gt;
    gt.init(S.E);
    if (ansp_gathers(t)) {
      const PmPart& P = S.parts[t.part];
      const uint32_t nb = gt.batches(P);
      for (uint32_t b = 0; b < nb; ++b) {
        gt.load(S, P, L.qo[0], b);
        gt.fold();
      }
      gt.reduce(L, S.E);
    }
    ansp_epilogue<W, NT>(S, t, L);
  }
#endif
}

// ---- k_gather: the server's XOR gather of wide sets, split ----------------
// (HOT LOOP D + E for SetSize >= 256: BIGANN's 764 / 3,816 chunks.)  One
// workgroup per (sub-query s, chunk range j of nsplit); it expands its range
// of the query set from the resolution record (pir.go:424-444, dummy
// :363-371), XORs the rows (PrivateQuery pir.go:65-88) and writes one partial
// entry.  k_answer folds the nsplit partials, so a sub-query's 0.5-2.4 MB of
// rows are read by nsplit CUs instead of one.
constexpr int kGatherBlock = 256;
constexpr uint32_t kGatherMaxRange = 4096;   // chunks per workgroup (SetSize / nsplit; BIGANN-1B: 3,816 at nsplit 1)
#ifndef PM_GATHER_NT
#define PM_GATHER_NT 1   // k_gather's row loads nontemporal (BIGANN: a 32-64 GB DB, no Infinity Cache reuse):
                         // 100M +3.2 %, 1B +0.7 % (ABBA, profiles/r05/ab/bigann_gather_nt.log)
#endif
#ifndef PM_GATHER_KG
#define PM_GATHER_KG 8
#endif
#ifndef PM_GATHER_WAVES
#define PM_GATHER_WAVES 8   // min waves per SIMD: <= 64 VGPRs, eight 256-thread workgroups per CU
#endif
template <int W>
__global__ void __launch_bounds__(kGatherBlock, PM_GATHER_WAVES) k_gather(PmStep S) {
  __shared__ uint64_t red[kGatherBlock * 2];
  __shared__ uint32_t rows_l[kGatherMaxRange];   // the range's partition rows (set expansion), ~0u: none
  const uint32_t j = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
  const PmRes r = S.res[s];
  const uint32_t mode = answer_mode(r);
  if (mode != A_FINAL && mode != A_CHAINED && mode != A_DUMMY) return;   // block-uniform
  const PmSub sub = step_sub(S, s);
  const PmPart& P = S.parts[sub.part];
  const uint32_t E = S.E, EX = E & ~3u, NSEG = EX / W, mask = P.CS - 1, lg = P.log2CS;
  const uint32_t per = (P.SS + S.nsplit - 1) / S.nsplit, c0 = min(P.SS, j * per), c1 = min(P.SS, c0 + per);
  const bool real = mode != A_DUMMY;
  const uint32_t pchunk = real && r.pp != kDefaultProgramPoint ? (r.pp >> lg) : kNone;
  const uint32_t rchunk = real ? r.chunk : kNone;
  // the range's set first, every offset load in flight together, into LDS
  // (expanded inside the row batches, each batch waited for its offsets and then
  // for its rows: two round trips per batch)
  const uint32_t rep = real && rchunk - c0 < c1 - c0 ? (P.ridx[r.chunk * P.Qpc + r.ing] & mask) : 0;
  for (uint32_t i = c0 + tid; i < c1; i += kGatherBlock) {
    uint32_t o;
    if (real) {
      o = P.tabT[tabT_index(P.H, r.tag, i)];
      if (i == pchunk) o = r.pp & mask;
      if (i == rchunk) o = rep;
    } else {
      o = (uint32_t)(hash4(P.seed, DOM_DUMMY, P.idx, sub.idx, i) & mask);
    }
    const uint64_t row = (uint64_t)i * P.CS + o;
    rows_l[i - c0] = row < P.N ? (uint32_t)row : ~0u;
  }
  __syncthreads();

  const PM_G uint64_t* base = S.db + P.row0 * E;
  PM_G uint64_t* out = S.part_x + ((uint64_t)s * S.nsplit + j) * EX;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  const uint32_t nr = c1 - c0;
  for (uint32_t seg0 = 0; seg0 < NSEG; seg0 += kGatherBlock) {
    const uint32_t nseg = min(NSEG - seg0, (uint32_t)kGatherBlock);
    const uint32_t nsl = kGatherBlock / nseg;
    const uint32_t sl = tid / nseg, seg = seg0 + tid % nseg;
    uint64_t a0 = 0, a1 = 0;
    if (sl < nsl) {
      constexpr int kG = PM_GATHER_KG;   // every row load of a batch in flight together
      for (uint32_t i0 = sl; i0 < nr; i0 += kG * nsl) {
        uint32_t rr[kG];
#pragma unroll
        for (int u = 0; u < kG; ++u) rr[u] = rows_l[min(i0 + u * nsl, nr - 1)];
#pragma unroll
        for (int u = 0; u < kG; ++u)
          if (i0 + u * nsl >= nr) rr[u] = ~0u;
        u64x2 x[kG];
#pragma unroll
        for (int u = 0; u < kG; ++u) {
          x[u] = u64x2{0, 0};
          if (rr[u] != ~0u) {
            const PM_G uint64_t* q = base + (uint64_t)rr[u] * E + (uint64_t)seg * W;
            if (W == 2) x[u] = PM_GATHER_NT ? __builtin_nontemporal_load(reinterpret_cast<const PM_G u64x2*>(q))
                                         : *reinterpret_cast<const PM_G u64x2*>(q);
            else x[u].x = PM_GATHER_NT ? __builtin_nontemporal_load(q) : *q;
          }
        }
#pragma unroll
        for (int u = 0; u < kG; ++u) { a0 ^= x[u].x; a1 ^= x[u].y; }
      }
    }
    red[tid * 2] = a0;
    red[tid * 2 + 1] = a1;
    __syncthreads();
    if (tid < nseg) {
      uint64_t x0 = 0, x1 = 0;
      for (uint32_t k = 0; k < nsl; ++k) {
        x0 ^= red[(k * nseg + tid) * 2];
        x1 ^= red[(k * nseg + tid) * 2 + 1];
      }
      out[seg * W] = x0;
      if (W == 2) out[seg * W + 1] = x1;
    }
    __syncthreads();
  }
}

// ---- k_step: the step in one launch ---------------------------------------
// Workgroups [0, nsub) match one sub-query each (all its hints), the next np
// resolve one partition each, then nhelp x nsub gather helpers (helper_role:
// ranges 1..nhelp of each sub-query's guessed set), the last nsub answer one
// sub-query each.  Every hand-off is a set of granules (put_g / get_g): a
// resolver polls its partition's match records, an answer workgroup its
// helpers' partials and then its resolution record.  Dispatch is in
// workgroup order and a role only waits for lower-numbered ones (helpers wait
// for none), so the lowest unfinished workgroup can always run; at most 240
// workgroups of 1024 threads whose LDS admits one per CU, the envelope the
// hand-off forms are measured in (the host sizes nhelp to stay inside it).
constexpr int kStepBlock = 1024, kStepHPT = kLdsPH / kStepBlock;
union StepLds {
  uint32_t s_cand[kStepBlock / 64][6];
  ResolveLds<2> r;
  AnswerLds<kStepBlock> a;
  uint8_t one_per_cu[96 * 1024];
};

// A gather helper of sub-query s (k_step, S.nhelp > 0): the same guess as
// the answer workgroup's, then range j (1..nhelp) of its set: set expansion,
// rows, the partial XOR into granules (two per word), and the guess fields
// the answer checks before it merges the partial.
template <int W, int NT, class LDS>
__device__ __forceinline__ void helper_role(const PmStep& S, uint32_t s, uint32_t j, LDS& L) {
  const PmSub sub = step_sub(S, s);
  const PmPart& P = S.parts[sub.part];
  const uint32_t tid = threadIdx.x, EX = S.E & ~3u;
  PmRes g;
  const uint32_t gmode = step_guess<NT>(S, s, sub, P, L, g);
  PM_G uint64_t* const out = S.helpg + ((uint64_t)s * kStepHelpMax + (j - 1)) * kHelpGran;
  if (gmode == A_FINAL || gmode == A_DUMMY) {
    const uint32_t n = S.nhelp + 1, lo = P.SS * j / n, hi = P.SS * (j + 1) / n;
    set_range<NT>(P, sub, g, gmode, L.qo, lo, hi);
    __syncthreads();
    gather_range<W, NT, PM_STEP_KG>(S, P, L.qo, L.red, L.row, lo, hi);
    for (uint32_t w = tid; w < EX; w += NT) {
      const uint64_t x = L.row.w[w];
      put_g(out + 2 * w, (uint32_t)x, S.token);
      put_g(out + 2 * w + 1, (uint32_t)(x >> 32), S.token);
    }
  }
  if (tid < 6) {
    const uint32_t f = tid == 0 ? gmode : tid == 1 ? g.hit : tid == 2 ? g.chunk : tid == 3 ? g.ing : tid == 4 ? g.tag : g.pp;
    put_g(out + 2 * kHelpWords + tid, f, S.token);
  }
}

template <int W>
__global__ void __launch_bounds__(kStepBlock) k_step(PmStep S) {
  __shared__ StepLds L;
  const uint32_t b = blockIdx.x;
  TS(0);
  TS_HWID();
  if (b < S.nsub) {
    PmSub sub = S.subs_a[b];
    sub.part = __builtin_amdgcn_readfirstlane(sub.part);
    sub.kind = __builtin_amdgcn_readfirstlane(sub.kind);
    sub.idx = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(sub.idx >> 32)) << 32) |
              __builtin_amdgcn_readfirstlane((uint32_t)sub.idx);
    match_role<kStepBlock, kStepHPT, true>(S, b, 0, sub, L.s_cand);
    TS(1);
    return;
  }
  if (b < S.nsub + S.np) {
    const uint32_t p = b - S.nsub;
    if (S.sb_a[p + 1] == S.sb_a[p]) return;
    resolve_role<2, kStepBlock, true>(S, p, L.r);
    __syncthreads();
    TS(2);
    if (!L.r.fin) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();   // L.r is dead from here: its space holds the decode row
    finish_step<true>(S, L.a.row);
    return;
  }
  const uint32_t hb = S.nsub + S.np;   // then nhelp x nsub helpers, then the answers
  if (b < hb + S.nhelp * S.nsub) {
    const uint32_t k = b - hb;
    helper_role<W, kStepBlock>(S, k % S.nsub, 1 + k / S.nsub, L.a);
    TS(2);
    return;
  }
  answer_role<W, true, kStepBlock>(S, b - hb - S.nhelp * S.nsub, L.a);
  TS(2);
}

}  // namespace pm

namespace pmk {
static inline unsigned cdiv(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }
// Path selectors: the environment's choice (read once), unless pm_set_option
// overrides it (the tests drive every hint-search form through the same steps).
// value -2 (kOptUnset here) restores the environment's choice.
constexpr int kOptUnset = INT32_MIN;
static int env_int(const char* name, int def) { const char* e = getenv(name); return e ? atoi(e) : def; }
static const int env_match_part = env_int("PM_MATCH_PART", -1), env_match_part8 = env_int("PM_MATCH_PART8", 1),
                 env_match_resolve = env_int("PM_MATCH_RESOLVE", 1);
static std::atomic<int> ov_match_part{kOptUnset}, ov_match_part8{kOptUnset}, ov_match_resolve{kOptUnset};
static int opt(const std::atomic<int>& ov, int env) {
  const int v = ov.load(std::memory_order_relaxed);
  return v != kOptUnset ? v : env;
}
// One snapshot per step: every selector of the step reads the same values, so
// a pm_set_option on another thread cannot split a step between two paths
// (e.g. np_live = 0 with the general k_match_resolve).
StepOpts step_opts() {
  return StepOpts{opt(ov_match_part, env_match_part), opt(ov_match_part8, env_match_part8),
                  opt(ov_match_resolve, env_match_resolve)};
}
int set_option(const char* name, int value) {
  std::atomic<int>* o = !strcmp(name, "match_part") ? &ov_match_part
                      : !strcmp(name, "match_part8") ? &ov_match_part8
                      : !strcmp(name, "match_resolve") ? &ov_match_resolve : nullptr;
  if (!o) return -1;
  o->store(value <= -2 ? kOptUnset : value, std::memory_order_relaxed);
  return 0;
}
uint32_t step_match_blocks(uint32_t maxPH) { return cdiv(maxPH, kMatchHints); }
// With events, the launch carries them in its own dispatch packet
// (hipExtLaunchKernelGGL): the kernel's execution time as the profiler sees it.
#define PM_LAUNCH(ev, kern, grid, blk, st, ...)                                              \
  do {                                                                                       \
    if ((ev).a) hipExtLaunchKernelGGL(kern, grid, blk, 0, st, (ev).a, (ev).b, 0, __VA_ARGS__); \
    else hipLaunchKernelGGL(kern, grid, blk, 0, st, __VA_ARGS__);                             \
  } while (0)
int step_match(hipStream_t st, const PmStep& S, const StepOpts& O, bool ph8, uint32_t maxPH,
               uint32_t max_sub_per_part, PmEvents ev) {
  // many partitions with several sub-queries each (batched serving): one
  // workgroup per (partition, hint block); otherwise one per (sub-query, block)
  const int mode = O.match_part;
  const bool part = mode == 1 || (mode == -1 && S.np >= 128 && S.nsub >= 4 * S.np);
  // PM_MATCH_PART8=0: the LDS-merged form for every PH
  const int v8 = O.match_part8;
  // k_match_part8 from 64 partitions with 2+ sub-queries each (BIGANN teams of
  // 4-6 sessions: k_match's workgroup per (sub-query, block) took 85 us there)
  const bool part8 = ph8 && v8 && max_sub_per_part <= kPart8Subs && (part || (mode == -1 && S.np >= 64 && S.nsub >= 2 * S.np));
  if (part8) {
    PM_LAUNCH(ev, k_match_part8<PM_MATCHPART8_NW>, dim3(cdiv(step_match_blocks(maxPH), PM_MATCHPART8_NW), S.np),
              dim3(64 * PM_MATCHPART8_NW), st, S);
    return MATCH_PART8;
  }
  if (part) {
    PM_LAUNCH(ev, k_match_part<kMatchHints / kBlock>, dim3(step_match_blocks(maxPH), S.np), dim3(kBlock), st, S);
    return MATCH_PART;
  }
  PM_LAUNCH(ev, k_match, dim3(step_match_blocks(maxPH), S.nsub), dim3(kBlock), st, S);
  return MATCH_SUB;
}
bool step_match_resolve_ok(const PmStep& S, const StepOpts& O, bool lds) {
  const int mode = O.match_resolve;
  // one workgroup per partition matches every hint of it: search-sized hint
  // counts only (PH <= 16,384; BIGANN's 57,344 / 114,688 hints per partition
  // go to k_match_part's workgroup per (partition, hint block) instead)
  return mode && !lds && !S.args_valid && S.subs == S.subs_h && S.sb == S.sb_h && S.np >= 128 &&
         S.nsub >= 4 * S.np && S.words <= 256;
}
// k_match_resolve_s serves the step (its resolvers do not count in: PmStep::np_live = 0)
bool step_match_resolve_small(const StepOpts& O, bool ph8, uint32_t maxPH, uint32_t max_sub_per_part) {
  const int mode = O.match_resolve;
  return mode == 1 && max_sub_per_part <= kSpecSubs && ph8 && maxPH <= 16u * kResolveBlockG;
}
void step_match_resolve(hipStream_t st, const PmStep& S, const StepOpts& O, bool ph8, uint32_t maxPH,
                        uint32_t max_sub_per_part, PmEvents ev) {
  // the one-round-trip form where its shapes hold (PM_MATCH_RESOLVE=2: always the general one)
  const bool small = step_match_resolve_small(O, ph8, maxPH, max_sub_per_part);
  // workgroup size (PM_MR_NT): 256 leaves the GPU's wave slots to the other
  // groups' kernels while wave 0 runs the chain
  static const int nt = [] { const char* e = getenv("PM_MR_NT"); return e ? atoi(e) : 256; }();
  if (small && nt == 128 && maxPH <= 8u * 128 * 4)
    PM_LAUNCH(ev, (k_match_resolve_s<4, 128>), dim3(S.np), dim3(128), st, S);
  else if (small && nt == 128 && maxPH <= 8u * 128 * 8)
    PM_LAUNCH(ev, (k_match_resolve_s<8, 128>), dim3(S.np), dim3(128), st, S);
  else if (small && nt == 256 && maxPH <= 8u * 256 * 2)
    PM_LAUNCH(ev, (k_match_resolve_s<2, 256>), dim3(S.np), dim3(256), st, S);
  else if (small && nt == 256 && maxPH <= 8u * 256 * 4)
    PM_LAUNCH(ev, (k_match_resolve_s<4, 256>), dim3(S.np), dim3(256), st, S);
  else if (small && maxPH <= 8u * kResolveBlockG)
    PM_LAUNCH(ev, (k_match_resolve_s<1, kResolveBlockG>), dim3(S.np), dim3(kResolveBlockG), st, S);
  else if (small && maxPH <= 16u * kResolveBlockG)
    PM_LAUNCH(ev, (k_match_resolve_s<2, kResolveBlockG>), dim3(S.np), dim3(kResolveBlockG), st, S);
  else
    PM_LAUNCH(ev, k_match_resolve<kMatchHints / kBlock>, dim3(S.np), dim3(kResolveBlockG), st, S);
}
bool step_qset_ok(const PmStep& S, const StepOpts& O, bool lds, bool ph8, uint32_t maxPH,
                  uint32_t max_sub_per_part, uint32_t maxSS) {
  const int mode = O.match_resolve;
  static const int qs = [] { const char* e = getenv("PM_QSET"); return e ? atoi(e) : 1; }();
  return qs && mode == 1 && step_match_resolve_ok(S, O, lds) && max_sub_per_part <= kSpecSubs && ph8 &&
         maxPH <= 16u * kResolveBlockG && maxSS <= kSmallSS && S.nsplit <= 1;
}
void step_resolve(hipStream_t st, const PmStep& S, bool lds, PmEvents ev) {
  if (lds) PM_LAUNCH(ev, k_resolve<true>, dim3(S.np), dim3(kBlock), st, S);
  else PM_LAUNCH(ev, k_resolve<false>, dim3(S.np), dim3(kResolveBlockG), st, S);
}
bool step_resolve_lds_ok(uint32_t maxPH, uint32_t max_sub_per_part) {
  // the staged (LDS) resolver only for partitions with more sub-queries than
  // the fast prologue takes; otherwise the global-memory form, whose fast
  // prologue is the same and whose 36 KB of LDS (not 117) let four
  // workgroups share a CU
  return max_sub_per_part > kSpecSubs && maxPH <= kLdsPH &&
         max_sub_per_part * ((maxPH + 63) / 64) <= kLdsBitWords;
}
void step_answer(hipStream_t st, const PmStep& S, uint32_t maxSS, PmEvents ev) {
  // search-sized shapes: the small-LDS instance (PM_ANSWER_NT threads per
  // workgroup, 0 = the generic instance)
  static const int nt = [] { const char* e = getenv("PM_ANSWER_NT"); return e ? atoi(e) : 128; }();
  // the pipelined pair form (k_answer_p) where its shapes hold: pre-expanded
  // query sets, one gather segment per thread slice (E & ~3 <= 2 * 128 words)
  static const int pair = [] { const char* e = getenv("PM_ANSWER_PAIR"); return e ? atoi(e) : 1; }();
  // the pair form's decoded row lives in RowBufT<kSmallE>: E itself (not only
  // its gather part E & ~3) must fit, or the epilogue's tail words overrun it
  static_assert(2u * kAnsPNT >= kSmallE, "k_answer_p's gather slices must cover a kSmallE row");
  if (pair && S.qset && S.nsplit <= 1 && maxSS <= kSmallSS && S.E % 2 == 0 && S.E <= kSmallE &&
      (S.E & ~3u) <= 2u * kAnsPNT && S.nsub >= 2 * 256) {
    // sub-queries per workgroup (the grid is nsub / pk; 2: every workgroup of a
    // 6,144-sub-query step resident at once)
    static const uint32_t pk = [] { const char* e = getenv("PM_ANSWER_PK"); return std::min(e && atoi(e) > 1 ? (uint32_t)atoi(e) : (uint32_t)PM_ANSWER_PK_MAX, (uint32_t)PM_ANSWER_PK_MAX); }();
    uint32_t grid = (S.nsub + pk - 1) / pk;
    if (PM_ANSWER_P_TAIL) grid = std::min(grid, (uint32_t)PM_ANSWER_P_TAIL);
    PM_LAUNCH(ev, (k_answer_p<2, kAnsPNT>), dim3(grid), dim3(kAnsPNT), st, S);
    return;
  }
  if (nt && S.nsplit <= 1 && maxSS <= kSmallSS && S.E <= kSmallE) {
    const bool w2 = S.E % 2 == 0;
    if (nt == 128) {
      if (w2) PM_LAUNCH(ev, (k_answer_s<2, 128>), dim3(S.nsub), dim3(128), st, S);
      else PM_LAUNCH(ev, (k_answer_s<1, 128>), dim3(S.nsub), dim3(128), st, S);
    } else if (nt == 512) {
      if (w2) PM_LAUNCH(ev, (k_answer_s<2, 512>), dim3(S.nsub), dim3(512), st, S);
      else PM_LAUNCH(ev, (k_answer_s<1, 512>), dim3(S.nsub), dim3(512), st, S);
    } else {
      if (w2) PM_LAUNCH(ev, (k_answer_s<2, 256>), dim3(S.nsub), dim3(256), st, S);
      else PM_LAUNCH(ev, (k_answer_s<1, 256>), dim3(S.nsub), dim3(256), st, S);
    }
    return;
  }
  if (S.E % 2 == 0) PM_LAUNCH(ev, k_answer<2>, dim3(S.nsub), dim3(kAnsBlock), st, S);
  else PM_LAUNCH(ev, k_answer<1>, dim3(S.nsub), dim3(kAnsBlock), st, S);
}
uint32_t step_gather_split(uint32_t maxSS, uint32_t nsub) {
  if (maxSS < 256 || nsub == 0) return 1;
  static const int forced = [] { const char* e = getenv("PM_GATHER_SPLIT"); return e ? atoi(e) : 0; }();
  // >= 48 rows per workgroup, about 4,096 workgroups in all (two rounds of the
  // GPU's 2,048 resident 256-thread workgroups; BIGANN-100M's 960 sub-queries:
  // 5 ranges, 96-104 us, vs 3 ranges at ~2,048 workgroups, 124-143 us), at most
  // 64 per sub-query; PM_GATHER_SPLIT=n forces n
  uint32_t n = forced > 0 ? (uint32_t)forced : std::min(cdiv(maxSS, 48), cdiv(4096, nsub));
  n = std::max(1u, std::min(n, 64u));
  return n > 1 ? std::max(n, cdiv(maxSS, kGatherMaxRange)) : 1u;   // a range's set fits k_gather's LDS
}
void step_gather(hipStream_t st, const PmStep& S, PmEvents ev) {
  const dim3 grid(S.nsplit, S.nsub);
  if (S.E % 2 == 0) PM_LAUNCH(ev, k_gather<2>, grid, dim3(kGatherBlock), st, S);
  else PM_LAUNCH(ev, k_gather<1>, grid, dim3(kGatherBlock), st, S);
}
bool step_fused_ok(const PmStep& S, uint32_t maxPH, uint32_t max_sub_per_part) {
  return S.args_valid && S.recg && S.err_h && max_sub_per_part <= kSpecSubs && maxPH <= kLdsPH &&
         2 * S.nsub + S.np <= 256;
}
void step_fused(hipStream_t st, const PmStep& S, PmEvents ev) {
  // S.cblk must be 1 (one match record per sub-query)
  const dim3 grid(2 * S.nsub + S.np + S.nhelp * S.nsub);
  if (S.E % 2 == 0) PM_LAUNCH(ev, k_step<2>, grid, dim3(kStepBlock), st, S);
  else PM_LAUNCH(ev, k_step<1>, grid, dim3(kStepBlock), st, S);
}
uint32_t step_max_sub_per_part() { return kMaxSubPerPart; }
uint32_t step_max_ss() { return kMaxSSLds; }
uint32_t step_max_e() { return kMaxELds; }
}  // namespace pmk
