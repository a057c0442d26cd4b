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
#include "pm_aes.h"
#include "pm_internal.h"

namespace pm {

constexpr int kAnsBlock = 512;
constexpr uint32_t kNone = 0xffffffffu;

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_match(PmStep S) {
  __shared__ PmSub s_sub;
  const uint32_t s = blockIdx.y;
  if (threadIdx.x == 0) {
    const PmSub sub = S.subs_h[s];   // zero-copy read of the host descriptor
    s_sub = sub;
    if (blockIdx.x == 0) S.subs[s] = sub;
  }
  if (blockIdx.x == 0 && s == 0) {
    for (uint32_t i = threadIdx.x; i <= S.np; i += kBlock) S.sb[i] = S.sb_h[i];
    if (threadIdx.x < 3) S.done[threadIdx.x] = 0;
  }
  __syncthreads();
  const PmSub sub = s_sub;
  if (sub.kind != SUB_REAL) return;
  const PmPart& P = S.parts[sub.part];
  const uint32_t base = blockIdx.x * kBlock;
  if (base >= P.PH) return;
  const uint32_t mask = P.CS - 1, chunk = (uint32_t)(sub.idx >> P.log2CS),
                 offset = (uint32_t)(sub.idx & mask);
  const uint16_t* row = P.tab + (uint64_t)chunk * P.H;
  const uint32_t h = base + threadIdx.x;
  bool m = false;
  if (h < P.PH && sub.idx < P.N) {
    const uint32_t pp = P.pp[h];
    m = row[P.tag[h]] == offset && (pp == kDefaultProgramPoint || (pp >> P.log2CS) != chunk);
  }
  const uint64_t b = __ballot(m);
  if ((threadIdx.x & 63) == 0 && (h - (threadIdx.x & 63)) < P.PH) S.bits[(uint64_t)s * S.words + (h >> 6)] = b;
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

// Minimum over the wave of a per-lane candidate.
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor(x, o));
  return x;
}

constexpr int kMaxSubPerPart = 256;

__global__ void __launch_bounds__(kBlock) k_resolve(PmStep S) {
  __shared__ uint64_t s_idx[kMaxSubPerPart];
  __shared__ uint32_t s_kind[kMaxSubPerPart], s_chunk[kMaxSubPerPart], s_st[kMaxSubPerPart],
      s_hist0[kMaxSubPerPart], s_c1[kMaxSubPerPart], s_c2[kMaxSubPerPart], s_t1[kMaxSubPerPart],
      s_p1[kMaxSubPerPart], s_t2[kMaxSubPerPart], s_p2[kMaxSubPerPart];
  __shared__ uint32_t m_h[kMaxSubPerPart], m_tag[kMaxSubPerPart], m_pp[kMaxSubPerPart],
      m_sub[kMaxSubPerPart];
  __shared__ uint32_t s_fqn;
  const uint32_t p = blockIdx.x;
  const PmPart& P = S.parts[p];
  const uint32_t b0 = S.sb[p], n = S.sb[p + 1] - b0;
  if (n == 0) return;
  const uint32_t lg = P.log2CS, mask = P.CS - 1, nw = (P.PH + 63) / 64;
  // --- phase 0: prefetch the partition's sub-queries and counters -----------
  for (uint32_t j = threadIdx.x; j < n; j += kBlock) {
    const PmSub sub = S.subs[b0 + j];
    s_kind[j] = sub.kind;
    s_idx[j] = sub.idx;
    const uint32_t c = (uint32_t)(sub.idx >> lg);
    s_chunk[j] = c;
    s_hist0[j] = (sub.kind == SUB_REAL && sub.idx < P.N) ? P.hist[c] : 0;
    s_st[j] = kNone;
  }
  if (threadIdx.x == 0) s_fqn = *P.fqn;
  __syncthreads();
  // --- phase 1: first two stale candidates per real sub-query + their state --
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t j = wave; j < n; j += kBlock / 64) {
    if (s_kind[j] != SUB_REAL) continue;
    const uint64_t* bw = S.bits + (uint64_t)(b0 + j) * S.words;
    const uint32_t c1 = find_next(bw, nw, 0);
    const uint32_t c2 = c1 == kNone ? kNone : find_next(bw, nw, c1 + 1);
    if (lane == 0) {
      s_c1[j] = c1; s_c2[j] = c2;
      s_t1[j] = c1 == kNone ? 0 : P.tag[c1]; s_p1[j] = c1 == kNone ? 0 : P.pp[c1];
      s_t2[j] = c2 == kNone ? 0 : P.tag[c2]; s_p2[j] = c2 == kNone ? 0 : P.pp[c2];
    }
  }
  __syncthreads();
  if (wave != 0) return;
  // --- phase 2: the sequential chain of Client.Query calls, on wave 0 --------
  volatile uint32_t* vst = s_st;
  volatile uint32_t* vmh = m_h;
  volatile uint32_t* vmt = m_tag;
  volatile uint32_t* vmp = m_pp;
  volatile uint32_t* vms = m_sub;
  uint32_t fqn = s_fqn, nmod = 0;
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
          const bool d = k < j && s_kind[k] == SUB_REAL && s_idx[k] == idx && vst[k] == ST_OK;
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
              __ballot(k < j && vst[k] == ST_OK && s_chunk[k] == chunk));
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
            mod |= __ballot(k0 + lane < nmod && vmh[k0 + lane] == c) != 0;
          if (!mod) break;
          if (which == 1) { c = s_c2[j]; which = 2; }
          else { c = find_next(S.bits + (uint64_t)s * S.words, nw, c + 1); which = 3; }
        }
        // hints refreshed earlier in this step, with their current tag / program point
        uint32_t bm = kNone, bk = kNone;
        for (uint32_t k0 = 0; k0 < nmod; k0 += 64) {
          const uint32_t k = k0 + lane;
          uint32_t cand = kNone;
          if (k < nmod) {
            const uint32_t pp = vmp[k];
            if (P.tab[(uint64_t)chunk * P.H + vmt[k]] == off &&
                (pp == kDefaultProgramPoint || (pp >> lg) != chunk))
              cand = vmh[k];
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
          if (chained) { tag = vmt[bk]; pp = vmp[bk]; }
          else if (which == 1) { tag = s_t1[j]; pp = s_p1[j]; }
          else if (which == 2) { tag = s_t2[j]; pp = s_p2[j]; }
          else { tag = P.tag[hit]; pp = P.pp[hit]; }
          r = PmRes{ST_OK, hit, chunk, hist, tag, pp, fqn, chained ? 1u : 0u};
          // refresh (pir.go:460-470): backup hint (chunk, hist) has tag PH + chunk*Qpc + hist
          const uint32_t ntag = P.PH + chunk * P.Qpc + hist;
          if (lane == 0) {
            P.tag[hit] = ntag;
            P.pp[hit] = (uint32_t)idx;
            P.hist[chunk] = hist + 1;
            if (chained) {
              // the previous holder of this hint must publish its parity refresh
              const uint32_t prev = vms[bk];
              const uint32_t pf = S.res[prev].flags;
              // this chained sub-query counts itself; the chain head is counted once
              const uint32_t add = 1u + ((!(pf & 1u) && !(pf & 4u)) ? 1u : 0u);
              S.res[prev].flags = pf | 2u | 4u;
              const uint32_t pos = atomicAdd(&S.done[1], 1u);
              S.done[3 + pos] = s;
              atomicAdd(&S.done[2], add);
              vmt[bk] = ntag; vmp[bk] = (uint32_t)idx; vms[bk] = s;
            } else {
              vmh[nmod] = hit; vmt[nmod] = ntag; vmp[nmod] = (uint32_t)idx; vms[nmod] = s;
            }
          }
          if (!chained) ++nmod;
          ++fqn;
        }
      }
    }
    if (lane == 0) { vst[j] = r.status; S.res[s] = r; }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) *P.fqn = fqn;
}

// L2Dist of the first `dim` floats of an LDS row against q (device), one
// 8-lane group; bit-exact (see k_l2_rows).  Call with lanes 0..7 of a wave.
__device__ __forceinline__ float l2_lds(const float* row, const float* __restrict__ q, uint32_t dim) {
  const uint32_t k = threadIdx.x & 7;
  const uint32_t dimS = dim & ~7u;
  float acc = 0.0f;
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

union RowBuf {   // one decoded entry; the L2 reads its leading floats
  uint64_t w[kMaxELds];
  float f[2 * kMaxELds];
};

// What a k_answer workgroup does for its sub-query.
enum : uint32_t { A_ZERO = 0, A_FINAL = 1, A_CHAINED = 2, A_CACHED = 3, A_DUMMY = 4 };

// Decode one chained sub-query (its hint was refreshed earlier in this step)
// once every earlier refresh is visible; the whole workgroup participates.
__device__ void decode_chained(const PmStep& S, uint32_t s, RowBuf& row) {
  const PmSub sub = S.subs[s];
  const PmRes r = S.res[s];
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
  __syncthreads();
  uint64_t* orow = S.rows_h + (uint64_t)s * E;
  uint64_t* ar = P.arena + (uint64_t)r.slot * E;
  for (uint32_t w = tid; w < E; w += blockDim.x) { orow[w] = row.w[w]; ar[w] = row.w[w]; }
  if (tid < 64) {
    float d = 0.0f;
    if (S.q && tid < 8) d = l2_lds(row.f, S.q, S.dim);
    if (tid == 0) S.hdr_h[s] = PmOutHdr{r.status, r.slot, d, 0};
  }
  __syncthreads();
}

template <int W>
__global__ void __launch_bounds__(kAnsBlock) k_answer(PmStep S) {
  __shared__ uint32_t qo[kMaxSSLds];
  __shared__ uint64_t red[kAnsBlock * 2];
  __shared__ __attribute__((aligned(16))) RowBuf row;
  __shared__ uint32_t s_last;
  const uint32_t s = blockIdx.x, tid = threadIdx.x;
  const uint32_t E = S.E, EX = E & ~3u, NSEG = EX / W;
  const PmSub sub = S.subs[s];
  const PmRes r = S.res[s];
  const PmPart& P = S.parts[sub.part];
  uint64_t* const orow = S.rows_h + (uint64_t)s * E;
  const uint32_t mode = r.status == ST_OK ? ((r.flags & 1u) ? A_CHAINED : A_FINAL)
                      : r.status == ST_CACHED ? A_CACHED
                      : r.status == ST_DUMMY ? A_DUMMY : A_ZERO;
  const uint32_t mask = P.CS - 1, lg = P.log2CS;
  // decode operands: independent of the gather, issued first (pir.go:450-468)
  const uint64_t dslot = (uint64_t)r.chunk * P.Qpc + r.ing;
  const uint64_t* rv = P.rval + dslot * E;
  const uint64_t* bp = P.parity + ((uint64_t)P.PH + dslot) * E;
  uint64_t* pp = P.parity + (uint64_t)r.hit * E;
  uint64_t e_rv = 0, e_bp = 0, e_pp = 0;
  if (mode == A_FINAL && tid < E) { e_rv = rv[tid]; e_bp = bp[tid]; e_pp = pp[tid]; }
  // ---- query set (pir.go:363-371 dummy; :424-444 real) -------------------
  if (mode == A_FINAL || mode == A_CHAINED) {
    const uint32_t pchunk = r.pp != kDefaultProgramPoint ? (r.pp >> lg) : kNone;
    const uint16_t* trow = P.tabT + (uint64_t)r.tag * P.SS;
    for (uint32_t i = tid; i < P.SS; i += kAnsBlock) {
      uint32_t o = trow[i];
      if (i == pchunk) o = r.pp & mask;
      if (i == r.chunk) o = P.ridx[r.chunk * P.Qpc + r.ing] & mask;
      qo[i] = o;
    }
  } else if (mode == A_DUMMY) {
    for (uint32_t i = tid; i < P.SS; i += kAnsBlock)
      qo[i] = (uint32_t)(hash4(P.seed, DOM_DUMMY, P.idx, sub.idx, i) & mask);
  }
  __syncthreads();
  // ---- server XOR gather (HOT LOOP E) into row.w[0..EX) --------------------
  if (mode == A_FINAL || mode == A_CHAINED || mode == A_DUMMY) {
    const uint64_t* base = S.db + P.row0 * E;
    for (uint32_t seg0 = 0; seg0 < NSEG; seg0 += kAnsBlock) {
      const uint32_t nseg = min(NSEG - seg0, (uint32_t)kAnsBlock);
      const uint32_t nsl = kAnsBlock / nseg;
      const uint32_t sl = tid / nseg, seg = seg0 + tid % nseg;
      uint64_t a0 = 0, a1 = 0;
      if (sl < nsl) {
#pragma unroll 4
        for (uint32_t i = sl; i < P.SS; i += nsl) {
          const uint64_t rr = (uint64_t)i * P.CS + qo[i];
          if (rr < P.N) {
            const uint64_t* q = base + rr * E + (uint64_t)seg * W;
            if (W == 2) {
              const uint4 x = *reinterpret_cast<const uint4*>(q);
              a0 ^= ((uint64_t)x.y << 32) | x.x;
              a1 ^= ((uint64_t)x.w << 32) | x.z;
            } else {
              a0 ^= *q;
            }
          }
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
  // ---- decode + refresh, or the cached row -----------------------------
  if (mode == A_FINAL) {
    for (uint32_t w = tid; w < E; w += kAnsBlock) {
      const uint64_t rvw = w < kAnsBlock ? e_rv : rv[w], bpw = w < kAnsBlock ? e_bp : bp[w],
                     ppw = w < kAnsBlock ? e_pp : pp[w];
      uint64_t v = 0;
      if (w < EX) {
        v = row.w[w] ^ rvw ^ ppw;
        pp[w] = bpw ^ v;
      } else {
        pp[w] = bpw;
      }
      row.w[w] = v;
    }
  } else if (mode == A_CHAINED) {
    for (uint32_t w = tid; w < E; w += kAnsBlock) S.ans[(uint64_t)s * E + w] = w < EX ? row.w[w] : 0;
  } else if (mode == A_CACHED) {
    const uint64_t* a = P.arena + (uint64_t)r.slot * E;
    for (uint32_t w = tid; w < E; w += kAnsBlock) row.w[w] = a[w];
  }
  __syncthreads();
  // ---- results: row + header into pinned host memory, arena copy -----------
  if (mode != A_CHAINED) {
    const bool has_row = (mode == A_FINAL || mode == A_CACHED);
    for (uint32_t w = tid; w < E; w += kAnsBlock) orow[w] = has_row ? row.w[w] : 0;
    if (mode == A_FINAL) {
      uint64_t* ar = P.arena + (uint64_t)r.slot * E;
      for (uint32_t w = tid; w < E; w += kAnsBlock) ar[w] = row.w[w];
    }
    if (tid < 64) {
      float d = 0.0f;
      if (has_row && S.q && tid < 8) d = l2_lds(row.f, S.q, S.dim);
      if (tid == 0) S.hdr_h[s] = PmOutHdr{r.status, r.slot, d, 0};
    }
  }
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
    const uint32_t prev = __hip_atomic_fetch_add(&S.done[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev + 1 == S.done[2]);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  const uint32_t nchain = S.done[1];
  for (uint32_t k = 0; k < nchain; ++k) decode_chained(S, S.done[3 + k], row);
}

}  // namespace pm

namespace pmk {
static inline unsigned cdiv(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }
void step_match(hipStream_t st, const PmStep& S, uint32_t maxPH) {
  hipLaunchKernelGGL(k_match, dim3(cdiv(maxPH, kBlock), S.nsub), dim3(kBlock), 0, st, S);
}
void step_resolve(hipStream_t st, const PmStep& S) {
  hipLaunchKernelGGL(k_resolve, dim3(S.np), dim3(kBlock), 0, st, S);
}
void step_answer(hipStream_t st, const PmStep& S) {
  if (S.E % 2 == 0)
    hipLaunchKernelGGL(k_answer<2>, dim3(S.nsub), dim3(kAnsBlock), 0, st, S);
  else
    hipLaunchKernelGGL(k_answer<1>, dim3(S.nsub), dim3(kAnsBlock), 0, st, S);
}
uint32_t step_max_sub_per_part() { return kMaxSubPerPart; }
uint32_t step_max_ss() { return kMaxSSLds; }
uint32_t step_max_e() { return kMaxELds; }
}  // namespace pmk
