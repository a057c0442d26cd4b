// pm_kernels.hip — gfx950 kernels of the PianoPIR XOR fold / answer path and
// the graphann distance path.  See DESIGN.md §4 for the roofline of each.
#include "pm_aes.h"
#include "pm_internal.h"

namespace pm {

static constexpr AesTables kAesHost{};
__device__ const AesTables g_aes = kAesHost;

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// ---------------------------------------------------------------------------
// Client hint preprocessing (pir.go:267-352), split in two kernels:
//   prep_offsets: off[c][h] = PRF(tag_h, c) & (CS-1) for every hint h and
//                 chunk c (HOT LOOP A/B's PRF), kSkip for a backup hint's own
//                 chunk (pir.go:332-334).  AES-bound.
//   prep_fold:    parity[h] = XOR_c chunk_c[off[c][h]]  (HOT LOOP A/B's
//                 EntryXor), one lane per (hint, 16-B segment), parity held in
//                 a register for the whole chunk sweep.  Gather-bound.
// ---------------------------------------------------------------------------
constexpr int kOffsChunksPerBlock = 16;

__global__ void __launch_bounds__(kBlock) k_prep_offsets(const PmPart* __restrict__ parts,
                                                         uint16_t* __restrict__ offs,
                                                         uint64_t offs_stride) {
  __shared__ uint32_t te[kTeLdsWords];
  const PmPart& P = parts[blockIdx.z];
  const uint32_t H = P.H, SS = P.SS;
  const uint32_t c0 = blockIdx.y * kOffsChunksPerBlock;
  if (blockIdx.x * kBlock >= H || c0 >= SS) return;   // block-uniform
  aes_lds_init(te, g_aes.te0);
  __syncthreads();
  const AesLane A{te, threadIdx.x & 31u};
  const uint32_t h = blockIdx.x * kBlock + threadIdx.x;
  if (h >= H) return;
  const uint32_t mask = P.CS - 1;
  const uint32_t own = h >= P.PH ? (h - P.PH) / P.Qpc : 0xffffffffu;
  uint16_t* o = offs + blockIdx.z * offs_stride;
  const uint32_t c1 = min(SS, c0 + kOffsChunksPerBlock);
  for (uint32_t c = c0; c < c1; ++c) {
    uint16_t v = (uint16_t)(prf_lo32(A, P.rk, h, c) & mask);   // initial tag of hint h is h
    o[(uint64_t)c * H + h] = (c == own) ? kSkip : v;
  }
}

template <int W>   // 64-bit words per lane segment: 2 (16-B loads) or 1
__global__ void __launch_bounds__(kBlock) k_prep_fold(const PmPart* __restrict__ parts,
                                                      const uint16_t* __restrict__ offs,
                                                      uint64_t offs_stride,
                                                      const uint64_t* __restrict__ db, uint32_t E) {
  const PmPart& P = parts[blockIdx.y];
  const uint32_t EX = E & ~3u, NSEG = EX / W;
  const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t H = P.H;
  if (NSEG == 0) {   // xorSlices does nothing: every parity word stays zero
    if (e < (uint64_t)H * E) P.parity[e] = 0;
    return;
  }
  const uint32_t h = (uint32_t)(e / NSEG), seg = (uint32_t)(e % NSEG);
  if (h >= H) return;
  const uint16_t* o = offs + blockIdx.y * offs_stride + h;
  const uint64_t* base = db + (P.row0 * E) + (uint64_t)seg * W;
  const uint32_t CS = P.CS, SS = P.SS;
  const uint64_t N = P.N;
  uint64_t a0 = 0, a1 = 0;
  uint32_t c = 0;
  for (; c + 4 <= SS; c += 4) {
    uint16_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = o[(uint64_t)(c + u) * H];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t r = (uint64_t)(c + u) * CS + v[u];
      if (v[u] != kSkip && r < N) {
        const uint64_t* p = base + r * E;
        if (W == 2) {
          uint4 x = *reinterpret_cast<const uint4*>(p);
          a0 ^= ((uint64_t)x.y << 32) | x.x;
          a1 ^= ((uint64_t)x.w << 32) | x.z;
        } else {
          a0 ^= *p;
        }
      }
    }
  }
  for (; c < SS; ++c) {
    uint16_t v = o[(uint64_t)c * H];
    const uint64_t r = (uint64_t)c * CS + v;
    if (v != kSkip && r < N) {
      const uint64_t* p = base + r * E;
      a0 ^= p[0];
      if (W == 2) a1 ^= p[1];
    }
  }
  uint64_t* dst = P.parity + (uint64_t)h * E + (uint64_t)seg * W;
  dst[0] = a0;
  if (W == 2) dst[1] = a1;
  if (seg == 0)
    for (uint32_t w = EX; w < E; ++w) P.parity[(uint64_t)h * E + w] = 0;
}

// Replacement rows (pir.go:345-350): Qpc random offsets per chunk, idx + copy.
__global__ void __launch_bounds__(kBlock) k_prep_repl(const PmPart* __restrict__ parts,
                                                      const uint64_t* __restrict__ db, uint32_t E) {
  const PmPart& P = parts[blockIdx.y];
  const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nslot = (uint64_t)P.SS * P.Qpc;
  if (e >= nslot * E) return;
  const uint64_t slot = e / E;
  const uint32_t w = (uint32_t)(e % E);
  const uint32_t c = (uint32_t)(slot / P.Qpc);
  const uint64_t off = hash4(P.seed, DOM_REPL, P.idx, P.epoch, slot) & (P.CS - 1);
  const uint64_t r = (uint64_t)c * P.CS + off;
  if (w == 0) P.ridx[slot] = (uint32_t)r;
  P.rval[e] = r < P.N ? db[(P.row0 + r) * E + w] : 0;
}

// Initialization (pir.go:203-255): tags 0..H-1, program points, histogram.
__global__ void __launch_bounds__(kBlock) k_prep_init(const PmPart* __restrict__ parts) {
  const PmPart& P = parts[blockIdx.y];
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < P.H) P.tag[i] = i;
  if (i < P.PH) P.pp[i] = kDefaultProgramPoint;
  if (i < P.SS) P.hist[i] = 0;
  if (i < P.SS * P.Qpc) P.ridx[i] = kDefaultProgramPoint;
  if (i == 0) *P.fqn = 0;
}

// ---------------------------------------------------------------------------
// Online query, one batched step over every partition's sub-queries
// (batch-pir.go:189-216 -> pir.go:354-471).
// ---------------------------------------------------------------------------
constexpr int kMatchHintsPerThread = 8;

// HOT LOOP C (pir.go:404-414) against the state at the start of the step, for
// every (real sub-query, primary hint) pair: one bit per hint.
__global__ void __launch_bounds__(kBlock) k_hint_match(const PmPart* __restrict__ parts,
                                                       const PmSub* __restrict__ subs,
                                                       uint64_t* __restrict__ bits, uint32_t words) {
  __shared__ uint32_t te[kTeLdsWords];
  const PmSub sub = subs[blockIdx.y];
  if (sub.kind != SUB_REAL) return;
  const PmPart& P = parts[sub.part];
  const uint32_t base = blockIdx.x * kBlock * kMatchHintsPerThread;
  if (base >= P.PH) return;
  aes_lds_init(te, g_aes.te0);
  __syncthreads();
  const AesLane A{te, threadIdx.x & 31u};
  const uint32_t mask = P.CS - 1, chunk = (uint32_t)(sub.idx >> P.log2CS),
                 offset = (uint32_t)(sub.idx & mask);
  uint64_t* out = bits + (uint64_t)blockIdx.y * words;
#pragma unroll 1
  for (int k = 0; k < kMatchHintsPerThread; ++k) {
    const uint32_t h = base + k * kBlock + threadIdx.x;
    bool m = false;
    if (h < P.PH) {
      const uint32_t pp = P.pp[h];
      m = ((prf_lo32(A, P.rk, P.tag[h], chunk) & mask) == offset) &&
          (pp == kDefaultProgramPoint || (pp >> P.log2CS) != chunk);
    }
    const uint64_t b = __ballot(m);
    if ((threadIdx.x & 63) == 0 && (h - (threadIdx.x & 63)) < P.PH) out[h >> 6] = b;
  }
}

// Sequential part of Client.Query per partition: budget checks, first
// matching hint (stale bits + re-evaluation of hints refreshed earlier in
// this step), set expansion (HOT LOOP D, pir.go:424-427), programmed point and
// replacement substitution (:430-439), refresh of tag / program point /
// counters (:460-470).  Parities are refreshed by k_decode once the server
// answer is in.  One workgroup per partition.
constexpr int kMaxMod = 256;
__global__ void __launch_bounds__(kBlock) k_resolve(const PmPart* __restrict__ parts,
                                                    const PmSub* __restrict__ subs,
                                                    const uint32_t* __restrict__ sub_begin,
                                                    const uint64_t* __restrict__ bits, uint32_t words,
                                                    PmRes* __restrict__ res,
                                                    uint32_t* __restrict__ qoffs, uint32_t maxSS) {
  __shared__ uint32_t te[kTeLdsWords];
  __shared__ uint32_t mod_h[kMaxMod], mod_tag[kMaxMod], mod_pp[kMaxMod];
  __shared__ uint32_t s_nmod, s_best, s_go, s_chunk, s_off, s_tag, s_pp, s_repl;
  const uint32_t p = blockIdx.x;
  const PmPart& P = parts[p];
  const uint32_t b0 = sub_begin[p], b1 = sub_begin[p + 1];
  if (b0 == b1) return;
  aes_lds_init(te, g_aes.te0);
  if (threadIdx.x == 0) s_nmod = 0;
  __syncthreads();
  const AesLane A{te, threadIdx.x & 31u};
  const uint32_t mask = P.CS - 1, lg = P.log2CS;
  for (uint32_t s = b0; s < b1; ++s) {
    const PmSub sub = subs[s];
    uint32_t* qo = qoffs + (uint64_t)s * maxSS;
    if (sub.kind == SUB_DUMMY) {   // pir.go:363-371
      for (uint32_t i = threadIdx.x; i < P.SS; i += kBlock)
        qo[i] = (uint32_t)(hash4(P.seed, DOM_DUMMY, P.idx, sub.idx, i) & mask);
      if (threadIdx.x == 0) res[s] = PmRes{ST_DUMMY, 0, 0, 0, 0, 0, 0, 0};
      continue;
    }
    if (sub.kind != SUB_REAL) {
      if (threadIdx.x == 0) res[s] = PmRes{sub.kind == SUB_HOSTCACHE ? ST_CACHED : ST_SKIP, 0, 0, 0, 0, 0, 0, 0};
      continue;
    }
    // --- checks in reference order (thread 0), result broadcast via LDS ---
    if (threadIdx.x == 0) {
      uint32_t st = 0xffffffffu;
      if (sub.idx >= P.N) st = ST_ERANGE;
      if (st == 0xffffffffu)
        for (uint32_t t = b0; t < s; ++t)
          if (subs[t].kind == SUB_REAL && subs[t].idx == sub.idx && res[t].status == ST_OK) {
            res[s] = PmRes{ST_DUP, 0, 0, 0, t, 0, 0, 0};
            st = ST_DUP;
            break;
          }
      const uint32_t chunk = (uint32_t)(sub.idx >> lg);
      if (st == 0xffffffffu && *P.fqn >= P.MaxQ) st = ST_EBUDGET;
      if (st == 0xffffffffu && P.hist[chunk] >= P.Qpc) st = ST_ECHUNK;
      if (st != 0xffffffffu && st != ST_DUP) res[s] = PmRes{st, 0, 0, 0, 0, 0, 0, 0};
      s_go = (st == 0xffffffffu);
      s_chunk = chunk;
      s_off = (uint32_t)(sub.idx & mask);
      s_best = 0xffffffffu;
    }
    __syncthreads();
    if (!s_go) { __syncthreads(); continue; }
    const uint32_t chunk = s_chunk, offset = s_off, nmod = s_nmod;
    // --- first set stale bit, skipping refreshed hints ---
    const uint64_t* bw = bits + (uint64_t)s * words;
    const uint32_t nw = (P.PH + 63) / 64;
    for (uint32_t w = threadIdx.x; w < nw; w += kBlock) {
      uint64_t v = bw[w];
      if (v) {
        for (uint32_t k = 0; k < nmod; ++k)
          if ((mod_h[k] >> 6) == w) v &= ~(1ull << (mod_h[k] & 63));
        if (v) { atomicMin(&s_best, w * 64 + (uint32_t)__builtin_ctzll(v)); break; }
      }
    }
    // --- refreshed hints re-evaluated with their current tag / program point ---
    for (uint32_t k = threadIdx.x; k < nmod; k += kBlock) {
      const uint32_t pp = mod_pp[k];
      if ((prf_lo32(A, P.rk, mod_tag[k], chunk) & mask) == offset &&
          (pp == kDefaultProgramPoint || (pp >> lg) != chunk))
        atomicMin(&s_best, mod_h[k]);
    }
    __syncthreads();
    const uint32_t hit = s_best;
    if (hit == 0xffffffffu) {   // pir.go:416-419
      if (threadIdx.x == 0) res[s] = PmRes{ST_ENOHIT, 0, 0, 0, 0, 0, 0, 0};
      __syncthreads();
      continue;
    }
    if (threadIdx.x == 0) {
      uint32_t tag = P.tag[hit], pp = P.pp[hit];
      for (uint32_t k = 0; k < nmod; ++k)
        if (mod_h[k] == hit) { tag = mod_tag[k]; pp = mod_pp[k]; }
      const uint32_t ing = P.hist[chunk];
      s_tag = tag;
      s_pp = pp;
      s_repl = P.ridx[chunk * P.Qpc + ing];
      res[s] = PmRes{ST_OK, hit, chunk, ing, 0, 0, 0, 0};
      // refresh (pir.go:460-470); parity in k_decode
      const uint32_t ntag = P.tag[P.PH + chunk * P.Qpc + ing];
      P.tag[hit] = ntag;
      P.pp[hit] = (uint32_t)sub.idx;
      *P.fqn += 1;
      P.hist[chunk] = ing + 1;
      uint32_t k = 0;
      while (k < nmod && mod_h[k] != hit) ++k;
      if (k < kMaxMod) {
        mod_h[k] = hit; mod_tag[k] = ntag; mod_pp[k] = (uint32_t)sub.idx;
        if (k == nmod) s_nmod = nmod + 1;
      }
    }
    __syncthreads();
    const uint32_t tag = s_tag, pp = s_pp, repl = s_repl;
    for (uint32_t i = threadIdx.x; i < P.SS; i += kBlock) {
      uint32_t o = prf_lo32(A, P.rk, tag, i) & mask;
      if (pp != kDefaultProgramPoint && i == (pp >> lg)) o = pp & mask;
      if (i == chunk) o = repl & mask;
      qo[i] = o;
    }
    __syncthreads();
  }
}

// PianoPIRServer.PrivateQuery (pir.go:65-88) for every sub-query that sends
// one (real after resolution, and dummies): XOR of SetSize gathered rows.
// One workgroup per sub-query: lanes = (row slice, 16-B segment); slices are
// XOR-combined through LDS.
template <int W>
__global__ void __launch_bounds__(kBlock) k_answer(const PmPart* __restrict__ parts,
                                                   const PmSub* __restrict__ subs,
                                                   const PmRes* __restrict__ res,
                                                   const uint32_t* __restrict__ qoffs, uint32_t maxSS,
                                                   const uint64_t* __restrict__ db, uint32_t E,
                                                   uint64_t* __restrict__ ans) {
  __shared__ uint64_t red[kBlock * 2];
  const uint32_t s = blockIdx.x;
  if (res) {
    const uint32_t st = res[s].status;
    if (st != ST_OK && st != ST_DUMMY) return;
  }
  const PmPart& P = parts[subs ? subs[s].part : 0];
  const uint32_t EX = E & ~3u, NSEG = EX / W;
  const uint32_t* qo = qoffs + (uint64_t)s * maxSS;
  const uint64_t* base = db + P.row0 * E;
  uint64_t* out = ans + (uint64_t)s * E;
  for (uint32_t seg0 = 0; seg0 < NSEG; seg0 += kBlock) {
    const uint32_t nseg = min(NSEG - seg0, (uint32_t)kBlock);
    const uint32_t nsl = kBlock / nseg;
    const uint32_t sl = threadIdx.x / nseg, seg = seg0 + threadIdx.x % nseg;
    uint64_t a0 = 0, a1 = 0;
    if (sl < nsl) {
      for (uint32_t i = sl; i < P.SS; i += nsl) {
        const uint64_t r = (uint64_t)i * P.CS + qo[i];
        if (r < P.N) {
          const uint64_t* p = base + r * E + (uint64_t)seg * W;
          if (W == 2) {
            uint4 x = *reinterpret_cast<const uint4*>(p);
            a0 ^= ((uint64_t)x.y << 32) | x.x;
            a1 ^= ((uint64_t)x.w << 32) | x.z;
          } else {
            a0 ^= *p;
          }
        }
      }
    }
    red[threadIdx.x * 2] = a0;
    red[threadIdx.x * 2 + 1] = a1;
    __syncthreads();
    if (threadIdx.x < nseg) {
      uint64_t x0 = 0, x1 = 0;
      for (uint32_t k = 0; k < nsl; ++k) {
        x0 ^= red[(k * nseg + threadIdx.x) * 2];
        x1 ^= red[(k * nseg + threadIdx.x) * 2 + 1];
      }
      out[(uint64_t)seg * W] = x0;
      if (W == 2) out[(uint64_t)seg * W + 1] = x1;
    }
    __syncthreads();
  }
  for (uint32_t w = EX + threadIdx.x; w < E; w += kBlock) out[w] = 0;
}

// Decode + parity refresh, in sub-query order per partition (pir.go:450-468):
//   response = answer ^ replVal ^ primaryParity[hit]
//   primaryParity[hit] = backupParity[chunk][ing] ^ response
// Lane w owns word w of every entry, so consecutive sub-queries that hit the
// same hint need no barrier.
__global__ void __launch_bounds__(kBlock) k_decode(const PmPart* __restrict__ parts,
                                                   const PmSub* __restrict__ subs,
                                                   const uint32_t* __restrict__ sub_begin,
                                                   const PmRes* __restrict__ res,
                                                   const uint64_t* __restrict__ ans, uint32_t E,
                                                   uint64_t* __restrict__ out) {
  const uint32_t p = blockIdx.x;
  const PmPart& P = parts[p];
  const uint32_t b0 = sub_begin[p], b1 = sub_begin[p + 1];
  const uint32_t EX = E & ~3u;
  for (uint32_t s = b0; s < b1; ++s) {
    const PmRes r = res[s];
    uint64_t* o = out + (uint64_t)s * E;
    if (r.status == ST_OK) {
      const uint64_t slot = (uint64_t)r.chunk * P.Qpc + r.ing;
      const uint64_t* rv = P.rval + slot * E;
      const uint64_t* bp = P.parity + ((uint64_t)P.PH + slot) * E;
      uint64_t* pp = P.parity + (uint64_t)r.hit * E;
      const uint64_t* a = ans + (uint64_t)s * E;
      for (uint32_t w = threadIdx.x; w < E; w += kBlock) {
        if (w < EX) {
          const uint64_t resp = a[w] ^ rv[w] ^ pp[w];
          pp[w] = bp[w] ^ resp;
          o[w] = resp;
        } else {
          pp[w] = bp[w];
          o[w] = 0;
        }
      }
    } else if (r.status == ST_DUP) {
      const uint64_t* src = out + (uint64_t)r.ref * E;
      for (uint32_t w = threadIdx.x; w < E; w += kBlock) o[w] = src[w];
    } else if (r.status != ST_CACHED) {
      for (uint32_t w = threadIdx.x; w < E; w += kBlock) o[w] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Distance kernels (graphann/l2_distance_amd64.s).
// ---------------------------------------------------------------------------
// L2Dist, bit-exact: lane k of an 8-lane group owns running sum s_k over
// elements 8t+k (VSUBPS/VMULPS/VADDPS, each rounded: no FMA), then the
// VHADDPS tree ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)) as xor-1/2/4 shuffles, then
// the scalar tail of build_graph.go:123-125 on lane 0.
__global__ void __launch_bounds__(kBlock) k_l2_rows(const float* __restrict__ rows,
                                                    uint64_t stride, uint64_t nrows,
                                                    const uint32_t* __restrict__ ids,
                                                    const float* __restrict__ q, uint32_t dim,
                                                    float* __restrict__ out) {
  const uint64_t g = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 3;
  const uint32_t k = threadIdx.x & 7;
  const bool live = g < nrows;
  const float* r = rows + (live ? (ids ? (uint64_t)ids[g] : g) : 0) * stride;
  const uint32_t dimS = dim & ~7u;
  float acc = 0.0f;
  if (live)
    for (uint32_t t = k; t < dimS; t += 8) {
      const float d = __fsub_rn(r[t], q[t]);
      acc = __fadd_rn(acc, __fmul_rn(d, d));
    }
  acc = __fadd_rn(acc, __shfl_xor(acc, 1));
  acc = __fadd_rn(acc, __shfl_xor(acc, 2));
  acc = __fadd_rn(acc, __shfl_xor(acc, 4));
  if (live && k == 0) {
    float d = dimS ? acc : 0.0f;
    for (uint32_t i = dimS; i < dim; ++i) {
      const float t = __fsub_rn(r[i], q[i]);
      d = __fadd_rn(d, __fmul_rn(t, t));
    }
    out[g] = d;
  }
}

// InnerProduct per row (mod 2^32): 16 lanes per row, shuffle-reduced; the
// wrapping sum of all rows is atomically accumulated (order-independent).
__global__ void __launch_bounds__(kBlock) k_ip_rows(const uint32_t* __restrict__ rows, uint64_t nrows,
                                                    const uint32_t* __restrict__ q, uint32_t dim,
                                                    uint32_t* __restrict__ per_row,
                                                    uint32_t* __restrict__ sum) {
  const uint64_t g = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
  const uint32_t l = threadIdx.x & 15;
  uint32_t acc = 0;
  if (g < nrows) {
    const uint32_t* r = rows + g * dim;
    for (uint32_t j = l; j < dim; j += 16) acc += r[j] * q[j];
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) acc += __shfl_xor(acc, m);
  if (g < nrows && l == 0 && per_row) per_row[g] = acc;
  uint32_t w = (l == 0 && g < nrows) ? acc : 0;
#pragma unroll
  for (int m = 16; m < 64; m <<= 1) w += __shfl_xor(w, m);
  if ((threadIdx.x & 63) == 0) atomicAdd(sum, w);
}

// Streaming sum-only scan (the TestInnerProduct loop): 16-B loads, query
// element j = flat index mod dim from LDS, per-thread partial sums.
__global__ void __launch_bounds__(kBlock) k_ip_scan(const uint4* __restrict__ rows, uint64_t n4,
                                                    const uint32_t* __restrict__ q, uint32_t dim,
                                                    uint32_t* __restrict__ sum) {
  __shared__ uint32_t qs[4096];
  for (uint32_t j = threadIdx.x; j < dim; j += kBlock) qs[j] = q[j];
  __syncthreads();
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint32_t dim4 = dim / 4;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < n4; f += stride) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rows) + f);
    const uint4 v = make_uint4(t.x, t.y, t.z, t.w);
    const uint32_t j = (uint32_t)(f % dim4) * 4;
    acc += v.x * qs[j] + v.y * qs[j + 1] + v.z * qs[j + 2] + v.w * qs[j + 3];
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

__global__ void __launch_bounds__(kBlock) k_ip_fill(uint4* __restrict__ rows, uint64_t n4, uint32_t dim) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < n4; f += stride) {
    const uint64_t e = f * 4;
    const uint32_t i = (uint32_t)(e / dim), j = (uint32_t)(e % dim);
    rows[f] = make_uint4(i + j, i + j + 1, i + j + 2, i + j + 3);
  }
}

__global__ void __launch_bounds__(kBlock) k_prf_batch(const uint32_t* __restrict__ rk,
                                                      const uint64_t* __restrict__ tags,
                                                      const uint64_t* __restrict__ xs, uint64_t n,
                                                      uint64_t* __restrict__ out) {
  __shared__ uint32_t te[kTeLdsWords];
  __shared__ uint32_t srk[44];
  aes_lds_init(te, g_aes.te0);
  if (threadIdx.x < 44) srk[threadIdx.x] = rk[threadIdx.x];
  __syncthreads();
  const AesLane A{te, threadIdx.x & 31u};
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    out[i] = prf64(A, srk, tags[i], xs[i]);
}

}  // namespace pm

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
namespace pmk {
static inline unsigned cdiv(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }

void prep_init(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t maxRepl, uint32_t,
               bool) {
  const uint32_t n = maxH > maxRepl ? maxH : maxRepl;
  hipLaunchKernelGGL(k_prep_init, dim3(cdiv(n, kBlock), np), dim3(kBlock), 0, st, d);
}
void prep_offsets(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t maxSS,
                  uint16_t* offs, uint64_t stride) {
  hipLaunchKernelGGL(k_prep_offsets, dim3(cdiv(maxH, kBlock), cdiv(maxSS, kOffsChunksPerBlock), np),
                     dim3(kBlock), 0, st, d, offs, stride);
}
void prep_fold(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t, const uint16_t* offs,
               uint64_t stride, const uint64_t* db, uint32_t E) {
  const uint32_t EX = E & ~3u;
  if (EX == 0) {
    hipLaunchKernelGGL(k_prep_fold<2>, dim3(cdiv((uint64_t)maxH * E, kBlock), np), dim3(kBlock), 0,
                       st, d, offs, stride, db, E);
  } else if (E % 2 == 0) {
    hipLaunchKernelGGL(k_prep_fold<2>, dim3(cdiv((uint64_t)maxH * (EX / 2), kBlock), np),
                       dim3(kBlock), 0, st, d, offs, stride, db, E);
  } else {
    hipLaunchKernelGGL(k_prep_fold<1>, dim3(cdiv((uint64_t)maxH * EX, kBlock), np), dim3(kBlock), 0,
                       st, d, offs, stride, db, E);
  }
}
void prep_repl(hipStream_t st, const PmPart* d, int np, uint32_t maxRepl, const uint64_t* db,
               uint32_t E) {
  hipLaunchKernelGGL(k_prep_repl, dim3(cdiv((uint64_t)maxRepl * E, kBlock), np), dim3(kBlock), 0, st,
                     d, db, E);
}
void hint_match(hipStream_t st, const PmPart* d, const PmSub* subs, uint32_t nsub, uint32_t maxPH,
                uint64_t* bits, uint32_t words) {
  hipLaunchKernelGGL(k_hint_match, dim3(cdiv(maxPH, kBlock * kMatchHintsPerThread), nsub),
                     dim3(kBlock), 0, st, d, subs, bits, words);
}
void resolve(hipStream_t st, const PmPart* d, int np, const PmSub* subs, const uint32_t* sb,
             const uint64_t* bits, uint32_t words, PmRes* res, uint32_t* qoffs, uint32_t maxSS) {
  hipLaunchKernelGGL(k_resolve, dim3(np), dim3(kBlock), 0, st, d, subs, sb, bits, words, res, qoffs,
                     maxSS);
}
void answer(hipStream_t st, const PmPart* d, const PmSub* subs, const PmRes* res, uint32_t nsub,
            const uint32_t* qoffs, uint32_t maxSS, const uint64_t* db, uint32_t E, uint64_t* ans) {
  if (E % 2 == 0)
    hipLaunchKernelGGL(k_answer<2>, dim3(nsub), dim3(kBlock), 0, st, d, subs, res, qoffs, maxSS, db, E,
                       ans);
  else
    hipLaunchKernelGGL(k_answer<1>, dim3(nsub), dim3(kBlock), 0, st, d, subs, res, qoffs, maxSS, db, E,
                       ans);
}
void decode(hipStream_t st, const PmPart* d, int np, const PmSub* subs, const uint32_t* sb,
            const PmRes* res, const uint64_t* ans, uint32_t E, uint64_t* out) {
  hipLaunchKernelGGL(k_decode, dim3(np), dim3(kBlock), 0, st, d, subs, sb, res, ans, E, out);
}
void server_answer(hipStream_t st, const PmPart* d, const uint32_t* offs, uint32_t nq, uint32_t SS,
                   const uint64_t* db, uint32_t E, uint64_t* out) {
  answer(st, d, nullptr, nullptr, nq, offs, SS, db, E, out);
}
void l2_rows(hipStream_t st, const float* rows, uint64_t stride, uint64_t nrows, const uint32_t* ids,
             const float* q, uint32_t dim, float* out) {
  if (!nrows) return;
  hipLaunchKernelGGL(k_l2_rows, dim3(cdiv(nrows * 8, kBlock)), dim3(kBlock), 0, st, rows, stride, nrows,
                     ids, q, dim, out);
}
void ip_rows(hipStream_t st, const uint32_t* rows, uint64_t nrows, const uint32_t* q, uint32_t dim,
             uint32_t* per_row, uint32_t* sum) {
  if (!per_row && dim % 4 == 0 && dim <= 4096) {
    const uint64_t n4 = nrows * dim / 4;
    unsigned grid = cdiv(n4, kBlock);
    if (grid > 256 * 16) grid = 256 * 16;
    if (grid == 0) return;
    hipLaunchKernelGGL(k_ip_scan, dim3(grid), dim3(kBlock), 0, st, (const uint4*)rows, n4, q, dim, sum);
    return;
  }
  if (!nrows) return;
  hipLaunchKernelGGL(k_ip_rows, dim3(cdiv(nrows * 16, kBlock)), dim3(kBlock), 0, st, rows, nrows, q, dim,
                     per_row, sum);
}
void ip_fill(hipStream_t st, uint32_t* rows, uint64_t N, uint32_t D) {
  const uint64_t n4 = N * D / 4;
  unsigned grid = cdiv(n4, kBlock);
  if (grid > 256 * 16) grid = 256 * 16;
  hipLaunchKernelGGL(k_ip_fill, dim3(grid), dim3(kBlock), 0, st, (uint4*)rows, n4, D);
}
void prf_batch(hipStream_t st, const uint32_t* rk, const uint64_t* tags, const uint64_t* xs, uint64_t n,
               uint64_t* out) {
  unsigned grid = cdiv(n, kBlock * 16);
  if (grid == 0) return;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_prf_batch, dim3(grid), dim3(kBlock), 0, st, rk, tags, xs, n, out);
}
}  // namespace pmk
