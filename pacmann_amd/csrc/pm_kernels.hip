// pm_kernels.hip — gfx950 kernels of the PianoPIR XOR fold / answer path and
// the graphann distance path.  See DESIGN.md §5 for the roofline of each.
#include <atomic>
#include "pm_aes.h"
#include "pm_aes_bs.h"
#include "pm_internal.h"

namespace pm {
#ifndef PM_PREP_NT
#define PM_PREP_NT 0   // the maintenance's bulk stores (tabT tiles, the CS-512 fold's parities) nontemporal
#endif


__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// ---------------------------------------------------------------------------
// Client hint preprocessing (pir.go:267-352), split in two kernels:
//   prep_offsets: tab[c][h] = PRF(tag_h, c) & (CS-1) for every hint h and
//                 chunk c (HOT LOOP A/B's PRF), kSkip for a backup hint's own
//                 chunk (pir.go:332-334).  AES-bound.  The table stays resident
//                 and serves every online PRF (PmPart::tab).
//   prep_fold:    parity[h] = XOR_c chunk_c[off[c][h]]  (HOT LOOP A/B's
//                 EntryXor), one lane per (hint, 16-B segment), parity held in
//                 a register for the whole chunk sweep.  Gather-bound.
// ---------------------------------------------------------------------------
#ifndef PM_OFFS_CHUNKS
#define PM_OFFS_CHUNKS 8
#endif
constexpr int kOffsChunksPerBlock = PM_OFFS_CHUNKS;
constexpr int kOffsBlock = 1024;   // 64 KiB of replicated table per workgroup: 16 waves share it

// Initial PRF tables of every hint h < H (its tag is h) at 8 chunks per
// workgroup, written chunk-major (hint search) and hint-major (set
// expansion).  Bound by the AES T-table lookups in LDS: the hint-major stores
// are scattered 2-B writes (every lane on its own line, ~5x their bytes in
// HBM write traffic), yet staging them through LDS made the kernel 20-25 %
// slower (375 -> 450-470 us at SIFT1M shape), so they stay direct (without
// them the kernel is only 2 % faster).  1,024-thread workgroups share one 64 KiB
// table copy (the LDS init is 4 B per PRF, not 16) and keep 16 waves per CU
// for the lookups' latency: 0.370 -> 0.335 ms at SIFT1M shape.
#ifndef PM_OFFS_PAIR
#define PM_OFFS_PAIR 0   // k_prep_offsets: two chunks' PRFs per iteration (61 VGPRs at 8 waves: 56.5 vs 54.2 ms
                         // per 288-client launch, profiles/r05/ab/aes_chunk_pairs.log)
#endif
#ifndef PM_OFFS_TILES
#define PM_OFFS_TILES 1   // 8-chunk tiles per workgroup sharing one 64 KiB table fill (2 and 4 measured no faster: 244 / 268 vs 240 us per client alone)
#endif
constexpr int kOffsTiles = PM_OFFS_TILES;
__global__ void __launch_bounds__(kOffsBlock, PM_OFFS_PAIR ? 8 : 1) k_prep_offsets(const PmPart* __restrict__ parts) {
  __shared__ uint32_t te[kTeLdsWords];
  __shared__ R1Uniform r1u[kOffsTiles][kOffsChunksPerBlock];
  const PmPart& P = parts[blockIdx.z];
  const uint32_t H = P.H, SS = P.SS;
  const uint32_t cb = blockIdx.y * kOffsChunksPerBlock * kOffsTiles;
  if (blockIdx.x * kOffsBlock >= H || cb >= SS) return;   // block-uniform
  aes_lds_init(te, g_aes.te0);
  __syncthreads();
  const AesLane A(te, threadIdx.x);
  const uint32_t cend = min(SS, cb + kOffsChunksPerBlock * kOffsTiles);
  // round 1's chunk-dependent half, once per chunk for the workgroup (pm_aes.h)
  if (threadIdx.x < cend - cb)
    r1u[threadIdx.x / kOffsChunksPerBlock][threadIdx.x % kOffsChunksPerBlock] = r1_uniform(A, P.rk, cb + threadIdx.x);
  __syncthreads();
  const uint32_t h = blockIdx.x * kOffsBlock + threadIdx.x;
  if (h >= H) return;
  const uint32_t mask = P.CS - 1;
  const uint32_t own = h >= P.PH ? (h - P.PH) / P.Qpc : 0xffffffffu;
  uint16_t* o = P.tab;
  const R1Lane r1v = r1_lane(A, P.rk, h);   // initial tag of hint h is h
  // SetSize <= 256: round 2's hint-only part once per hint (pm_aes.h r2_hint)
  const bool r2 = SS <= 256;
  const R2Hint r2k = r2 ? r2_hint(A, P.rk, r1u[0][0], r1v) : R2Hint{0, 0, 0, 0};
  static_assert(kOffsChunksPerBlock == 8, "one 16-B tabT tile of 8 chunks per thread");
  for (int tl = 0; tl < kOffsTiles; ++tl) {
    const uint32_t c0 = cb + tl * kOffsChunksPerBlock;
    if (c0 >= SS) break;
    const uint32_t c1 = min(SS, c0 + kOffsChunksPerBlock);
    uint16_t tile[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[j] = kSkip;   // chunks past SetSize: padding
    auto put = [&](uint32_t c, uint32_t prf) {
      uint16_t v = (uint16_t)(prf & mask);
      v = (c == own) ? kSkip : v;
      if (o) o[(uint64_t)c * H + h] = v;   // chunk-major (only the folds that stage it read it)
      tile[c - c0] = v;
      if (h < P.PH) P.cur[cur_index(P.PH, P.curk, c, h)] = v;   // hint search (tags start at h)
    };
#if PM_OFFS_PAIR
    // two chunks' PRFs as independent chains side by side (twice the lookups in
    // flight per lane for the LDS latency)
    for (uint32_t c = c0; c < c1; c += 2) {
      const uint32_t cB = min(c + 1, c1 - 1);
      uint32_t pa, pb;
      if (r2) {
        pa = prf_lo16_r2(A, P.rk, r1u[tl][c - c0].u0, r1v, r2k, c);
        pb = prf_lo16_r2(A, P.rk, r1u[tl][cB - c0].u0, r1v, r2k, cB);
      } else {
        pa = prf_lo16_split(A, P.rk, r1u[tl][c - c0], r1v, c);
        pb = prf_lo16_split(A, P.rk, r1u[tl][cB - c0], r1v, cB);
      }
      put(c, pa);
      if (cB != c) put(cB, pb);
    }
#else
    for (uint32_t c = c0; c < c1; ++c)
      put(c, r2 ? prf_lo16_r2(A, P.rk, r1u[tl][c - c0].u0, r1v, r2k, c) : prf_lo16_split(A, P.rk, r1u[tl][c - c0], r1v, c));
#endif
    uint4 t4;   // tag-major tile (set expansion): one 16-B store
    t4.x = tile[0] | ((uint32_t)tile[1] << 16); t4.y = tile[2] | ((uint32_t)tile[3] << 16);
    t4.z = tile[4] | ((uint32_t)tile[5] << 16); t4.w = tile[6] | ((uint32_t)tile[7] << 16);
    if (PM_PREP_NT) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(u32x4{t4.x, t4.y, t4.z, t4.w}, reinterpret_cast<u32x4*>(P.tabT + tabT_index(H, h, c0)));
    } else {
      *reinterpret_cast<uint4*>(P.tabT + tabT_index(H, h, c0)) = t4;
    }
  }
}

// Bitsliced form of k_prep_offsets (round 6, pm_aes_bs.h): the same tables
// (tabT, cur, tab) bit for bit, the AES on the VALU instead of LDS T-table
// lookups.  A lane owns 32 consecutive hints (one bitsliced block set) and one
// tile group of 8 chunks; it evaluates the chunks in pairs, transposes each
// pair's 2 x 16 output planes into 32 words (hint j: chunk c | chunk c+1 << 16,
// i.e. one 4-B word of the hint's tabT tile) and stores them.  LDS holds only
// the per-key setup (Te0 for rounds 1-2, the folded round constants, W's
// planes): 2.7 KB.
constexpr int kBsThreads = 256;
#ifndef PM_BS_WAVES
#define PM_BS_WAVES 2
#endif
__global__ void __launch_bounds__(kBsThreads, PM_BS_WAVES) k_prep_offsets_bs(const PmPart* __restrict__ parts) {
  __shared__ uint32_t bs_te0[256];
  __shared__ uint32_t bs_kx[32];
  __shared__ uint32_t bs_wv[32][4];
  __shared__ __attribute__((aligned(16))) uint32_t bs_wp[128];
  __shared__ __attribute__((aligned(16))) uint32_t bs_stash[16 * kBsThreads];
  __shared__ __attribute__((aligned(16))) uint32_t bs_kpl[kBsKplWords];
  const PmPart& P = parts[blockIdx.y];
  const uint32_t H = P.H, SS = P.SS, PH = P.PH;
  const uint32_t nm = (H + 31) / 32, ng = (SS + 7) / 8;
  if (blockIdx.x * kBsThreads >= nm * ng) return;   // block-uniform
  bs_te0[threadIdx.x] = g_aes.te0[threadIdx.x];
  __syncthreads();
  bs_setup_a(bs_te0, P.rk, bs_kx, bs_wv);
  __syncthreads();
  bs_setup_b(bs_wv, bs_wp, bs_kx, bs_kpl);
  __syncthreads();
  const uint32_t task = blockIdx.x * kBsThreads + threadIdx.x;
  if (task >= nm * ng) return;
  const uint32_t m = task % nm, g = task / nm, h0 = 32 * m;
  const uint32_t nb = P.log2CS, Qpc = P.Qpc;
  const uint32_t keep = nb >= 16 ? 0xffffu : (1u << nb) - 1u;   // planes past log2(CS): masked off
  auto lowmask = [](int n) { return n <= 0 ? 0u : n >= 32 ? ~0u : (1u << n) - 1u; };
  // chunks in pairs: the first chunk's 16 planes wait in LDS (64 B per lane)
  // while the second is evaluated, so one copy of the AES code serves both and
  // no planes stay pinned in VGPRs across it
  uint4* stash = reinterpret_cast<uint4*>(bs_stash) + threadIdx.x;
#pragma unroll 1
  for (uint32_t q = 0; q < 8; ++q) {
    const uint32_t cc = 8 * g + q, c = cc & ~1u;
    uint32_t T[32];
    if (c < SS) {   // SetSize is a multiple of 4: a pair is whole
      uint32_t o[16];
      bs_prf16(bs_te0, P.rk, bs_kx, bs_wp, bs_kpl, m, cc, o);
      // backup hints whose own chunk is cc (pir.go:332-334): kSkip (all 16 bits set)
      const int lo = (int)(PH + cc * Qpc) - (int)h0, hi = lo + (int)Qpc;
      const uint32_t own = lowmask(hi) & ~lowmask(lo);
#pragma unroll
      for (int b = 0; b < 16; ++b) o[b] = (((keep >> b) & 1u) ? o[b] : 0u) | own;
      if ((q & 1) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) stash[i * kBsThreads] = make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 v = stash[i * kBsThreads];
        T[4 * i] = v.x; T[4 * i + 1] = v.y; T[4 * i + 2] = v.z; T[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int b = 0; b < 16; ++b) T[16 + b] = o[b];
      bs_transpose32(T);
    } else {
      if ((q & 1) == 0) continue;
#pragma unroll
      for (int j = 0; j < 32; ++j) T[j] = 0xffffffffu;   // tile padding past SetSize
    }
    // tag-major tiles: word (c & 7) / 2 of hint h0 + j's tile
    uint32_t* tt = reinterpret_cast<uint32_t*>(P.tabT + tabT_index(H, h0, c));
    if (h0 + 32 <= H) {
#pragma unroll
      for (int j = 0; j < 32; ++j) tt[4 * j] = T[j];
    } else {
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (h0 + j < H) tt[4 * j] = T[j];
    }
    if (c >= SS) continue;
    // 8-hint blocks of chunks c and c + 1 (cur: primary hints only; tab: every tag)
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const uint32_t hb = h0 + 8 * jb;
      uint4 wlo, whi;
      wlo.x = __builtin_amdgcn_perm(T[8 * jb + 1], T[8 * jb + 0], 0x05040100u);
      wlo.y = __builtin_amdgcn_perm(T[8 * jb + 3], T[8 * jb + 2], 0x05040100u);
      wlo.z = __builtin_amdgcn_perm(T[8 * jb + 5], T[8 * jb + 4], 0x05040100u);
      wlo.w = __builtin_amdgcn_perm(T[8 * jb + 7], T[8 * jb + 6], 0x05040100u);
      whi.x = __builtin_amdgcn_perm(T[8 * jb + 1], T[8 * jb + 0], 0x07060302u);
      whi.y = __builtin_amdgcn_perm(T[8 * jb + 3], T[8 * jb + 2], 0x07060302u);
      whi.z = __builtin_amdgcn_perm(T[8 * jb + 5], T[8 * jb + 4], 0x07060302u);
      whi.w = __builtin_amdgcn_perm(T[8 * jb + 7], T[8 * jb + 6], 0x07060302u);
      if (hb < PH) {
        *reinterpret_cast<uint4*>(P.cur + cur_index(PH, P.curk, c, hb)) = wlo;
        *reinterpret_cast<uint4*>(P.cur + cur_index(PH, P.curk, c + 1, hb)) = whi;
      }
      if (P.tab && hb < H) {
        *reinterpret_cast<uint4*>(P.tab + (uint64_t)c * H + hb) = wlo;
        *reinterpret_cast<uint4*>(P.tab + (uint64_t)(c + 1) * H + hb) = whi;
      }
    }
  }
}

#ifndef PM_FOLD_NT
#define PM_FOLD_NT 1   // k_prep_fold's (BIGANN's gather fold) row loads nontemporal: 221-222 -> 210-212 ms per
                       // 100M client = 0.83 of HBM peak (profiles/r05/ab/fold_nt_100m)
#endif
template <int W>   // 64-bit words per lane segment: 2 (16-B loads) or 1
__global__ void __launch_bounds__(kBlock) k_prep_fold(const PmPart* __restrict__ parts,
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
  const uint64_t* base = db + (P.row0 * E) + (uint64_t)seg * W;
  const uint32_t CS = P.CS, SS = P.SS;
  const uint64_t N = P.N;
  uint64_t a0 = 0, a1 = 0;
  uint32_t c = 0;
  for (; c + 4 <= SS; c += 4) {   // chunks c .. c+3 of hint h: 8 B of its tag-major tile (tabT)
    const uint64_t t4 = *reinterpret_cast<const uint64_t*>(P.tabT + tabT_index(H, h, c));
    uint16_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (uint16_t)(t4 >> (16 * u));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t r = (uint64_t)(c + u) * CS + v[u];
      if (v[u] != kSkip && r < N) {
        const uint64_t* p = base + r * E;
        if (W == 2) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 x = PM_FOLD_NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p))
                                     : *reinterpret_cast<const u32x4*>(p);
          a0 ^= ((uint64_t)x.y << 32) | x.x;
          a1 ^= ((uint64_t)x.w << 32) | x.z;
        } else {
          a0 ^= PM_FOLD_NT ? __builtin_nontemporal_load(p) : *p;
        }
      }
    }
  }
  for (; c < SS; ++c) {
    uint16_t v = P.tabT[tabT_index(H, h, c)];
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

// Cache-blocked fold (same result as k_prep_fold): a workgroup owns one
// partition, one SW-word column slice of every entry and one group of hints.
// For each chunk it stages the slice of all CS entries of the chunk into LDS
// with direct global->LDS loads (double-buffered, one barrier per chunk) and
// XORs the entry each of its hints selects into parity accumulators held in
// registers, so a DB byte is read from HBM once per hint group instead of once
// per hint that selects it.  Entry CS of a staged chunk is a zero row (kSkip
// selects it); rows past N are staged from a 16-byte zero source.
constexpr int kFoldThreads = 1024, kFoldHPT = 7;   // hints per thread: pipelined fold
constexpr int kFoldHPTBlk = 4;                      // hints per thread: double-buffered fold (up to 8-word slices)
constexpr uint32_t kFoldMaxItems = 4;   // 16-B staging items per thread per chunk
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_cvoid_t;

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4: lane l's bytes land at
// m0 + 16 l) issued by inline asm.  With __builtin_amdgcn_global_load_lds the
// compiler counts the DMA as a pending write to all of LDS and puts an
// s_waitcnt vmcnt(0) before the next ds_read of ANY buffer: a double buffer's
// staging of block b + 1 then completes before the fold of block b reads its
// first byte (k_prep_fold_rot's loop was serialised that way).  Issued here,
// the DMA is invisible to the compiler's wait insertion, so the caller waits
// for it (s_waitcnt vmcnt) before the buffer it fills is read.  The compiler's
// own counted waits for other loads stay correct: an extra operation in flight
// only makes a counted wait stricter.
__device__ __forceinline__ void lds_dma16(const void* src, const void* lds_wave_base) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)lds_wave_base);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(m) : "memory");
}

template <int SW>   // 64-bit words per column slice: 8, 4 or 2
__global__ void __launch_bounds__(kFoldThreads) k_prep_fold_blk(const PmPart* __restrict__ parts,
                                                                const uint64_t* __restrict__ db,
                                                                const uint64_t* __restrict__ zero16,
                                                                uint32_t E, uint32_t w0) {
  extern __shared__ __attribute__((aligned(16))) uint64_t fold_lds[];   // [2][(CS+1)*SW]
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t IPE = SW / 2;   // 16-B items per entry slice
  const PmPart& P = parts[blockIdx.z];
  const uint32_t H = P.H, CS = P.CS, SS = P.SS, tid = threadIdx.x;
  const uint32_t ng = (H + kFoldThreads * kFoldHPTBlk - 1) / (kFoldThreads * kFoldHPTBlk);
  if (blockIdx.x >= ng) return;   // block-uniform
  const uint32_t hb = (H + ng - 1) / ng, h0 = blockIdx.x * hb, h1 = min(H, h0 + hb);
  const uint32_t w = w0 + blockIdx.y * SW;
  const uint64_t N = P.N;
  const PM_G uint64_t* base = (const PM_G uint64_t*)db + P.row0 * E + w;
  const PM_G uint16_t* tab = P.tab;
  const uint32_t rowWords = (CS + 1) * SW, items = CS * IPE;
  const uint32_t wave_item0 = tid & ~63u;
  uint32_t hk[kFoldHPTBlk];
  uint64_t acc[kFoldHPTBlk][SW];
#pragma unroll
  for (int k = 0; k < kFoldHPTBlk; ++k) {
    hk[k] = h0 + tid + k * kFoldThreads;
#pragma unroll
    for (int x = 0; x < SW; ++x) acc[k][x] = 0;
  }
  uint32_t v[kFoldHPTBlk], nv[kFoldHPTBlk];
  // item it of chunk c: entry it / IPE, 16-B piece it % IPE, LDS byte offset it * 16
  auto stage = [&](uint32_t c, uint32_t buf) {
    uint64_t* L = fold_lds + buf * rowWords;
#pragma unroll
    for (uint32_t i = 0; i < kFoldMaxItems; ++i) {
      const uint32_t it = tid + i * kFoldThreads;
      if (i * kFoldThreads + wave_item0 < items && it < items) {
        const uint64_t r = (uint64_t)c * CS + it / IPE;
        const PM_G uint64_t* src = r < N ? base + r * E + (it % IPE) * 2 : (const PM_G uint64_t*)zero16;
        __builtin_amdgcn_global_load_lds((g_cvoid_t*)src, (lds_void_t*)(L + (i * kFoldThreads + wave_item0) * 2),
                                         16, 0, 0);
      }
    }
  };
  auto load_tab = [&](uint32_t c, uint32_t* out) {
#pragma unroll
    for (int k = 0; k < kFoldHPTBlk; ++k) out[k] = hk[k] < h1 ? tab[(uint64_t)c * H + hk[k]] : kSkip;
  };
  stage(0, 0);
  load_tab(0, v);
  for (uint32_t x = tid; x < 2 * SW; x += kFoldThreads) fold_lds[(x / SW) * rowWords + CS * SW + x % SW] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (uint32_t c = 0; c < SS; ++c) {
    const bool more = c + 1 < SS;
    if (more) { stage(c + 1, (c + 1) & 1); load_tab(c + 1, nv); }
    const uint64_t* L = fold_lds + (c & 1) * rowWords;
#pragma unroll
    for (int k = 0; k < kFoldHPTBlk; ++k) {
      const uint32_t o = v[k] == kSkip ? CS : v[k];
      const uint64_t* row = L + o * SW;
#pragma unroll
      for (int x = 0; x < SW; x += 2) {
        const u64x2 y = *reinterpret_cast<const u64x2*>(row + x);
        acc[k][x] ^= y.x;
        acc[k][x + 1] ^= y.y;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kFoldHPTBlk; ++k) v[k] = nv[k];
  }
#pragma unroll
  for (int k = 0; k < kFoldHPTBlk; ++k) {
    if (hk[k] >= h1) continue;
    PM_G uint64_t* dst = P.parity + (uint64_t)hk[k] * E + w;
#pragma unroll
    for (int x = 0; x < SW; x += 2) *reinterpret_cast<PM_G u64x2*>(dst + x) = u64x2{acc[k][x], acc[k][x + 1]};
    if (w == 0)   // xorSlices leaves the words past len&~3 zero
      for (uint32_t t = E & ~3u; t < E; ++t) P.parity[(uint64_t)hk[k] * E + t] = 0;
  }
}

// Pipelined form of k_prep_fold_blk for CS * SW == 2048 * G (every
// partition): three LDS buffers, two chunks in flight, and the PRF-table row
// of the chunk staged through LDS too, so every load of the loop is a direct
// global->LDS load and the waits are counted per wave (G or G+1 loads per
// chunk), never vmcnt(0).  One extern __shared__ array; raw s_barrier.
constexpr uint32_t kPipeTabWords = kFoldThreads * kFoldHPT / 4;   // the group's table row: one u16 per hint

// s_waitcnt vmcnt(n) for a runtime n, n <= 15.  n must be wave-uniform, and is
// made visibly so: s_waitcnt is a scalar instruction, and in a switch lowered
// as divergent (exec-masked) branches every case's wait would execute.
__device__ __forceinline__ void wait_vmcnt(uint32_t n) {
  switch (__builtin_amdgcn_readfirstlane(n)) {
#define PM_VMC(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    PM_VMC(1) PM_VMC(2) PM_VMC(3) PM_VMC(4) PM_VMC(5) PM_VMC(6) PM_VMC(7) PM_VMC(8)
    PM_VMC(9) PM_VMC(10) PM_VMC(11) PM_VMC(12) PM_VMC(13) PM_VMC(14) PM_VMC(15)
#undef PM_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

#ifndef PM_FOLD_FLIP
#define PM_FOLD_FLIP 1
#endif
// G = 16-B staging loads per thread per chunk; NB LDS buffers; D chunks folded
// between two workgroup barriers
template <int SW, int G, int NB, int D = 1>
__global__ void __launch_bounds__(kFoldThreads) k_prep_fold_pipe(const PmPart* __restrict__ parts,
                                                                 const uint64_t* __restrict__ db,
                                                                 const uint64_t* __restrict__ zero16,
                                                                 uint32_t E, uint32_t ngmax, uint32_t nsl,
                                                                 uint32_t npg, uint32_t K) {
  extern __shared__ __attribute__((aligned(16))) uint64_t fold_lds[];   // [NB][(CS+1)*SW + 1024]
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t IPE = SW / 2, CS = G * kFoldThreads / IPE;
  // XCD-aware order (workgroups b and b + 8 share an XCD, MI355X_MICROARCH.md
  // § Workgroup dispatch).  parts holds K clients of each partition, partition-
  // major; pg = (partition, hint group) runs on XCD pg % 8.  There, for each
  // group of LW column slices that split one 128-B line of every row, the
  // workgroups of all K clients follow each other, so the lines they stage are
  // fetched into that XCD's L2 once for K x LW workgroups instead of once per
  // client (the same DB, read by every client's fold).
  constexpr uint32_t LW = 16 / SW;   // slices per 128-B line
  const uint32_t ngl = (nsl + LW - 1) / LW, per_pg = K * ngl * LW;
  const uint32_t xcd = blockIdx.x % 8, k = blockIdx.x / 8;
  const uint32_t pg = xcd + 8 * (k / per_pg), r = k % per_pg;
  const uint32_t client = (r / LW) % K, slice = (r / (K * LW)) * LW + r % LW;
  if (pg >= npg || slice >= nsl) return;   // block-uniform
  const PmPart& P = parts[(pg / ngmax) * K + client];
  const uint32_t H = P.H, SS = P.SS, tid = threadIdx.x;
  const uint32_t ng = (H + kFoldThreads * kFoldHPT - 1) / (kFoldThreads * kFoldHPT);
  const uint32_t grp = pg % ngmax;
  if (grp >= ng) return;   // block-uniform
  const uint32_t hb = (((H + ng - 1) / ng) + 7) & ~7u, h0 = grp * hb, h1 = min(H, h0 + hb);
  const uint32_t w = slice * SW;
  const uint64_t N = P.N;
  const PM_G uint64_t* base = (const PM_G uint64_t*)db + P.row0 * E + w;
  const PM_G uint16_t* tab = P.tab;
  constexpr uint32_t TABW = (CS + 1) * SW, BUFW = TABW + kPipeTabWords;
  const uint32_t wave_item0 = tid & ~63u;
  const bool tab_wave = tid < kPipeTabWords / 2;   // these waves stage the table row (8 entries per lane)
  uint32_t hk[kFoldHPT];
  uint64_t acc[kFoldHPT][SW];
#pragma unroll
  for (int k = 0; k < kFoldHPT; ++k) {
    hk[k] = h0 + tid + k * kFoldThreads;
#pragma unroll
    for (int x = 0; x < SW; ++x) acc[k][x] = 0;
  }
  auto stage = [&](uint32_t c, uint32_t buf) {
    uint64_t* L = fold_lds + buf * BUFW;
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)G; ++i) {
      const uint32_t it = tid + i * kFoldThreads;
      const uint64_t r = (uint64_t)c * CS + it / IPE;
      const PM_G uint64_t* src = r < N ? base + r * E + (it % IPE) * 2 : (const PM_G uint64_t*)zero16;
      __builtin_amdgcn_global_load_lds((g_cvoid_t*)src, (lds_void_t*)(L + (i * kFoldThreads + wave_item0) * 2),
                                       16, 0, 0);
    }
    if (tab_wave) {   // 8 table entries (16 B) per lane; h0 and H are multiples of 8
      const uint32_t hh = h0 + tid * 8;
      const PM_G uint64_t* src = hh < h1 ? (const PM_G uint64_t*)(tab + (uint64_t)c * H + hh)
                                         : (const PM_G uint64_t*)zero16;
      __builtin_amdgcn_global_load_lds((g_cvoid_t*)src, (lds_void_t*)(L + TABW + wave_item0 * 2), 16, 0, 0);
    }
  };
  for (uint32_t x = tid; x < NB * SW; x += kFoldThreads) fold_lds[(x / SW) * BUFW + CS * SW + x % SW] = 0;
  // chunks 0 .. NB-D-1 in flight; chunks c+NB-D .. c+NB-1 are issued while
  // chunks c .. c+D-1 are folded
  static_assert(NB > D, "fold pipeline: more buffers than chunks per barrier");
  for (uint32_t c = 0; c + D < (uint32_t)NB && c < SS; ++c) stage(c, c);
  const uint32_t ops = G + (tab_wave ? 1 : 0);   // loads per chunk of this wave
  auto wait_chunks = [&](uint32_t next, uint32_t issued) {   // chunks next .. next+D-1 landed
    const uint32_t need = min(SS, next + D);
    wait_vmcnt(issued > need ? (issued - need) * ops : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  wait_chunks(0, min(SS, (uint32_t)(NB - D)));
  // LDS banking: a ds_read_b128 is served in 16-lane groups, and a SW = 4 row
  // (32 B) starts on one of 8 of the 16 16-B slots of the 256-B bank row, so 16
  // random rows pile up ~4.4-deep on 8 slots.  Odd lanes read the row's halves
  // in the other order (their accumulator holds words 2-3 first): each group's
  // 8 even and 8 odd lanes then fall on disjoint slot sets (~3.1-deep).
  const uint32_t fl = (SW == 4 && PM_FOLD_FLIP) ? ((tid & 1u) << 1) : 0u;
#ifndef PM_FOLD_ABL
#define PM_FOLD_ABL 0   // diagnostic builds: 1 = no LDS compute, 2 = no staging in the loop
#endif
  for (uint32_t c0 = 0; c0 < SS; c0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (PM_FOLD_ABL != 2 && c0 + NB - D + j < SS) stage(c0 + NB - D + j, (c0 + NB - D + j) % NB);
#pragma unroll
    for (int j = 0; j < D; ++j) {
    const uint32_t c = c0 + j;
    if (D > 1 && c >= SS) break;
    const uint64_t* L = fold_lds + (c % NB) * BUFW;
    const uint16_t* T = reinterpret_cast<const uint16_t*>(L + TABW);
#pragma unroll
    for (int k = 0; k < (PM_FOLD_ABL == 1 ? 0 : kFoldHPT); ++k) {
      const uint32_t t = hk[k] < h1 ? T[hk[k] - h0] : kSkip;
      const uint64_t* row = L + (t == kSkip ? CS : t) * SW;
#pragma unroll
      for (int x = 0; x < SW; x += 2) {
        const u64x2 y = *reinterpret_cast<const u64x2*>(row + (x ^ fl));
        acc[k][x] ^= y.x;
        acc[k][x + 1] ^= y.y;
      }
    }
    }
    if (c0 + D < SS) wait_chunks(c0 + D, min(SS, c0 + NB));
  }
#pragma unroll
  for (int k = 0; k < kFoldHPT; ++k) {
    if (hk[k] >= h1) continue;
    PM_G uint64_t* dst = P.parity + (uint64_t)hk[k] * E + w;
#pragma unroll
    for (int x = 0; x < SW; x += 2)
      *reinterpret_cast<PM_G u64x2*>(dst + (x ^ fl)) = u64x2{acc[k][x], acc[k][x + 1]};
    if (w == 0)   // xorSlices leaves the words past len&~3 zero
      for (uint32_t t = E & ~3u; t < E; ++t) P.parity[(uint64_t)hk[k] * E + t] = 0;
  }
}

// Bank-rotated fold for CS = 512 (same result as k_prep_fold): a workgroup
// owns (partition, 32-B column slice, group of <= 5,120 hints), one hint per
// lane slot (5 per lane), and folds the slice of every chunk into its hints'
// parities, like k_prep_fold_pipe.  What differs is how a chunk reaches LDS
// and is read there.  k_prep_fold_pipe has each lane read its hint's 32-B row
// with ds_read_b128: random rows land on random bank slots, ~3 rows pile up
// per slot in a 16-lane group, and the LDS array bounds the fold.  Here four
// chunks are staged side by side: LDS line k (128 B = the 32 banks of
// ds_read_b32) holds row k of chunks 4b..4b+3, one 32-B slot each.  In a
// 32-lane group, lane 8s + j reads chunk slot (s + phase) & 3 and, at step t,
// word (j + t) & 7 of its row (PM_ROT_B64 0): the 32 lanes touch 32 distinct
// banks whatever rows their hints select, so every ds_read_b32 takes its
// minimum 2 LDS cycles.  The default reads 8-B pairs ((j & 3) + t) & 3
// instead (PM_ROT_B64 below).  Accumulator t of a lane always holds the same
// word of its slice (XOR order does not matter) and is stored there at the end.
// The staged bytes come from the partition's fold image (PmPart::img: the
// same 64 KB LDS image per (slice, 4 chunks), contiguous, rows past N zero),
// a second, server-side copy of the DB laid out for this kernel (640 MB for
// SIFT1M: HBM capacity traded for whole-line sequential staging instead of
// 32-B pieces at 640-B stride).  Hint offsets come from the tag-major table
// (tabT: 8 chunks in 16 B per tag; hint h's initial tag is h).
// Two buffers of (CS + 1) lines (line CS is zero: kSkip), 128.3 KB.
// CS = 1,024 (MS-MARCO's 200K-row partitions): two chunks per block instead
// of four (64-B lines, the same 64 KB per block, nbuf = SS / 2), so the double
// buffer still fits (131.2 KB).  A 16-lane ds_read_b128 group then holds each
// (slot, half) four times and its lanes collide when their rows agree mod 4
// (about 2.6 instead of 2 LDS cycles per group for random rows).
#ifndef PM_ROT_HPL
#define PM_ROT_HPL 5
#endif
#ifndef PM_ROT_B64
#define PM_ROT_B64 1   // 8-B LDS reads: half the reads and address selects of the 4-B form, at the
                       // same LDS rate (lanes j and j + 4 share a bank pair when their rows have the
                       // same parity: 2 cycles per 32-lane group, like ds_read_b32's 2 x 128 B);
                       // 0.56-0.58 vs 0.68-0.69 ms per SIFT1M client, the fold being VALU-bound
#endif
#ifndef PM_ROT_B128
#define PM_ROT_B128 1   // 16-B reads of the two halves of a row's 32-B slot: half the reads of the 8-B form
                        // and one v_perm per (hint, chunk) for its offset instead of a 64-bit rotation
#endif
#ifndef PM_ROT_LW
#define PM_ROT_LW 2   // column slices of one (partition, group) pair dealt to an XCD back to back
                      // (64-client fold: 1 -> 31.5-31.7 ms, 2 -> 28.0-28.1, 4 -> 31.4-40.3, 5 -> 27.4-45.5)
#endif
#ifndef PM_ROT_ORDER
#define PM_ROT_ORDER 1   // 1: XCD tiles of GB pairs x SB slices (below); 0: round 2's order (PM_ROT_LW)
#endif                   // (64 clients, one box: 4 x 8 19.4 ms, 8 x 4 20.2, order 0 19.8, 16 x 2 +2 %)
#ifndef PM_ROT_GB
#define PM_ROT_GB 4
#endif
#ifndef PM_ROT_SB
#define PM_ROT_SB 8
#endif
#ifndef PM_ROT_PF
#define PM_ROT_PF 0   // L2 prefetch of the image block two buffers ahead (measured no gain once the
                      // staging overlaps the fold: 24.2-25.4 vs 24.8-25.0 ms per 64-client launch)
#endif
#ifndef PM_ROT_ABL
#define PM_ROT_ABL 0   // diagnostic builds: 1 = no LDS reads, 2 = no staging in the loop, 3 = one row per
                       // wave (no bank conflicts), 4 = 2 and 3, 5 = no fold work at all (B128 form), 6 = 4 without
                       // the tabT loads in the loop
#endif
#ifndef PM_ROT_PAIRS
#define PM_ROT_PAIRS 1   // the B128 fold XORs two phases' rows at a time (16 VGPRs of rows in flight, not 32)
#endif
#ifndef PM_ROT_HPL2
#define PM_ROT_HPL2 7   // hints per lane at CS 1,024 (2-B tiles; 128 VGPRs, no spills): 140 / 126 / 118 ms at 5 / 6 / 7
#endif
constexpr int kRotHPL = PM_ROT_HPL;   // hints per lane (SIFT1M's 12,512 hints: 3 groups of 4,171)
__host__ __device__ constexpr int rot_hpl(uint32_t cs) { return cs == 512 ? kRotHPL : PM_ROT_HPL2; }
constexpr uint32_t kRotBufBytes = 512 * 128;   // one image block per (slice, 4 chunks of 512 / 2 of 1,024 rows)
__host__ __device__ constexpr uint32_t rot_nch(uint32_t cs) { return cs == 512 ? 4 : 2; }   // chunks per block
template <int CS>
__global__ void __launch_bounds__(kFoldThreads) k_prep_fold_rot(const PmPart* __restrict__ parts, uint32_t E,
                                                                uint32_t nvg, uint32_t nsl, uint32_t npv,
                                                                uint32_t M, uint32_t K, uint32_t ngc) {
  constexpr uint32_t NCH = rot_nch(CS), LINE = NCH * 8, BUFW = (CS + 1) * LINE;
  constexpr int HPL = rot_hpl(CS);
  static_assert(CS == 512 || (CS == 1024 && PM_ROT_B128 && PM_ROT_PF == 0 && PM_ROT_ABL == 0),
                "CS 1,024: the 16-B read form only");
  static_assert(CS * LINE * 4 == kRotBufBytes, "64 KB blocks");
  // static (not extern) LDS: its address is a constant the reads fold into
  // their offsets
  __shared__ __attribute__((aligned(16))) uint32_t rot_lds[2 * BUFW];
  __shared__ uint32_t pf_lds[PM_ROT_PF ? kFoldThreads : 1];   // landing area of the L2 prefetch (never read)
  constexpr uint32_t ITEMS = CS * NCH * 2;   // 16-B staging items per buffer (NCH chunks x CS rows x 2)
  static_assert(ITEMS % kFoldThreads == 0, "whole staging items per thread");
  constexpr uint32_t G = ITEMS / kFoldThreads;
  // Virtual hint groups: the K clients' hint lists of a partition, concatenated
  // (client c's hint h is virtual hint c * H + h), cut into groups of HB =
  // 1,024 x HPL lane slots.  A group spans at most two clients (HB <= H),
  // and only the partition's last group has idle slots: 157 workgroups per
  // (partition, slice) for 64 SIFT1M clients instead of 3 per client (192),
  // each staging the slice's image once.  Order: XCD x takes the (partition,
  // group) pairs [x M, (x + 1) M); there, groups of PM_ROT_LW slices of consecutive
  // pairs follow each other (the pairs of one partition read the same image
  // blocks out of the XCD's L2).  (Round 1's order, (partition, group) on XCD
  // pg % 8 with groups of 4 slices of its K clients in turn, was measured
  // 10-15 % faster than all clients of one slice back to back.)  ngc != 0:
  // partitions with fewer than HB hints (small configs) keep ngc groups per
  // client instead (no mixing).
  constexpr uint32_t LW = PM_ROT_LW, HB = kFoldThreads * HPL;
  const uint32_t xcd = blockIdx.x % 8, kq = blockIdx.x / 8;
#if PM_ROT_ORDER == 1
  // Tiles of GB consecutive (partition, group) pairs x SB consecutive slices,
  // one tile per XCD at a time (GB * SB = its 32 CUs): a group's tabT rows are
  // read by SB workgroups and a slice's image blocks by GB workgroups out of
  // the XCD's L2.  The eight XCDs take eight consecutive pair blocks of the
  // SAME slice block, so the partition's image slices are shared through the
  // Infinity Cache; then the next slice block of the same pairs (their tabT
  // again, from the Infinity Cache).
  // Tile T = (its index on the XCD) * 8 + XCD; a last group of fewer than 8
  // pair blocks is dealt over the XCDs the same way (small launches, e.g. one
  // client's 48 pairs, keep every XCD busy).
  constexpr uint32_t GB = PM_ROT_GB, SB = PM_ROT_SB;
  const uint32_t nsb = (nsl + SB - 1) / SB, ngb = (npv + GB - 1) / GB;
  const uint32_t T = (kq / (GB * SB)) * 8 + xcd, wt = kq % (GB * SB);
  if (T >= ngb * nsb) return;   // block-uniform
  const uint32_t gsup = T / (8 * nsb), m = min(8u, ngb - gsup * 8), r = T - gsup * 8 * nsb;
  const uint32_t pgv = (gsup * 8 + r % m) * GB + wt % GB;
  const uint32_t slice = (r / m) * SB + wt / GB;
  (void)M; (void)LW;
#else
  const uint32_t loc = (kq / LW) % M, slice = (kq / (LW * M)) * LW + kq % LW;
  const uint32_t pgv = xcd * M + loc;
#endif
  if (pgv >= npv || slice >= nsl) return;   // block-uniform
  const uint32_t part = pgv / nvg, vg = pgv % nvg;
  const PmPart& P = parts[part * K];   // H, SS and the fold image are the same for every client
  const uint32_t H = P.H, SS = P.SS, tid = threadIdx.x;
  const uint32_t vend = K * H;
  uint32_t v0, v1;
  if (ngc == 0) {
    v0 = vg * HB;
    if (v0 >= vend) return;   // block-uniform (a partition with fewer hints than maxH)
    v1 = min(v0 + HB, vend);
  } else {
    const uint32_t c = vg / ngc, g = vg % ngc;
    if (c >= K || g * HB >= H) return;   // block-uniform
    v0 = c * H + g * HB;
    v1 = min(v0 + HB, (c + 1) * H);
  }
  const uint32_t cA = v0 / H, cB = min(cA + 1, K - 1), vb = (cA + 1) * H;
  const PmPart& PA = parts[part * K + cA];
  const PmPart& PB = parts[part * K + cB];
  const PM_G uint16_t* const tabA = PA.tabT;
  const PM_G uint16_t* const tabB = PB.tabT;
  const uint32_t hA = cA * H;
  const uint32_t w = slice * 4, nbuf = SS / NCH;   // SetSize is a multiple of 4 (pir.go:497)
  const PM_G char* img = (const PM_G char*)P.img + (uint64_t)slice * nbuf * kRotBufBytes;
#if PM_ROT_B128
  // 16-B reads: lane l reads chunk slot (s + phase) % NCH, halves f then f ^ 1
  // (s = l % NCH, f = (l / NCH) & 1: every ds_read_b128 lane group of 16 holds
  // each (slot, half) 8 / NCH times, MI355X_MICROARCH.md §LDS)
  const uint32_t lane = tid & 63, j = (lane / NCH) & 1, ks = lane & (NCH - 1);
#else
  const uint32_t lane = tid & 63, j = lane & 7, ks = (lane >> 3) & 3;
#endif
  const uint32_t vl = v0 + tid;   // virtual hint of lane slot k: vl + k * kFoldThreads
  uint32_t acc[HPL][8];
#pragma unroll
  for (int k = 0; k < HPL; ++k)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[k][t] = 0;
  const uint32_t wave_item0 = tid & ~63u;
  auto stage = [&](uint32_t b, uint32_t buf) {   // one contiguous 64 KB block of the image
    uint32_t* L = rot_lds + buf * BUFW;
    const PM_G char* src = img + (uint64_t)b * kRotBufBytes;
#pragma unroll
    for (uint32_t i = 0; i < G; ++i)
      lds_dma16(src + (tid + i * kFoldThreads) * 16u, L + (i * kFoldThreads + wave_item0) * 4);
  };
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  using Tile = std::conditional_t<NCH == 4, u32x2, uint32_t>;   // the NCH 2-B offsets of a hint's block
  auto load_tab = [&](uint32_t b, Tile* out) {   // chunks NCH b .. of each hint: 2 NCH B of its tabT tile
#pragma unroll
    for (int k = 0; k < HPL; ++k) {
      const uint32_t v = min(vl + k * kFoldThreads, vend - 1);
      const bool inB = v >= vb;
      const PM_G char* src = (const PM_G char*)(inB ? tabB : tabA) + (uint32_t)tabT_index(H, v - (inB ? vb : hA), NCH * b) * 2u;
      out[k] = *reinterpret_cast<const PM_G Tile*>(src);
    }
  };
  for (uint32_t x = tid; x < 2 * LINE; x += kFoldThreads) rot_lds[(x / LINE) * BUFW + CS * LINE + x % LINE] = 0;
  Tile tv[HPL], tn[HPL];
  stage(0, 0);
  // lane slots past the group read the zero line (kSkip).  Applied when a tile
  // is taken into use, not at its load: a select on the loaded value right
  // after the load made every iteration wait for its prefetched staging and
  // tabT loads before folding the current buffer (the double buffer's
  // overlap lost)
  auto skip_idle = [&](Tile* t) {
#pragma unroll
    for (int k = 0; k < HPL; ++k)
      if (PM_ROT_B128 && vl + k * kFoldThreads >= v1) t[k] = ~Tile{};
  };
  load_tab(0, tv);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  skip_idle(tv);
  const char* lds0 = reinterpret_cast<const char*>(rot_lds);
  for (uint32_t b = 0; b < nbuf; ++b) {
    if (b + 1 < nbuf) { if (PM_ROT_ABL != 2 && PM_ROT_ABL < 4) stage(b + 1, (b + 1) & 1); if (PM_ROT_ABL != 6) load_tab(b + 1, tn); }
    // L2 prefetch of block b + 2 (no third LDS buffer fits): one 4-B LDS-DMA load
    // per 128-B line by waves 0-7, issued after this iteration's staging and
    // tabT loads, so the counted wait below leaves only it in flight
    // (LDS-DMA intrinsics keep their order, so every staging load precedes it;
    // a tabT load the compiler places after it is covered by its own wait)
    // (issued by every thread, branch-free: two threads per line; past the last
    // block it re-reads the last one)
    if (PM_ROT_PF)
      __builtin_amdgcn_global_load_lds(
          (g_cvoid_t*)(img + (uint64_t)min(b + 2, nbuf - 1) * kRotBufBytes + (tid & (kFoldThreads / 2 - 1)) * 128u),
          (lds_void_t*)(pf_lds + (tid & ~63u)), 4, 0, 0);
    const uint32_t lb = (b & 1) * BUFW * 4;   // byte offset of this buffer
#if PM_ROT_B128
    {
      uint32_t cso[NCH], psel[NCH];
#pragma unroll
      for (uint32_t ph = 0; ph < NCH; ++ph) {
        const uint32_t sl = (ks + ph) & (NCH - 1);
        cso[ph] = lb + sl * 32 + 16 * j;
        psel[ph] = 0x0c0c0000u | ((2 * sl + 1) << 8) | (2 * sl);   // v_perm: tile word sl, zero-extended
      }
#pragma unroll
      for (int k = 0; k < (PM_ROT_ABL == 5 ? 0 : HPL); ++k) {
#if PM_ROT_PAIRS
#pragma unroll
       for (uint32_t p0 = 0; p0 < NCH; p0 += 2) {   // two phases' rows in flight, then their XOR
        uint32_t v[2][8];
#pragma unroll
        for (uint32_t pp = 0; pp < 2; ++pp) {
          const uint32_t ph = p0 + pp;
          uint32_t o;
          if constexpr (NCH == 4) o = __builtin_amdgcn_perm(tv[k].y, tv[k].x, psel[ph]);
          else o = __builtin_amdgcn_perm(0u, tv[k], psel[ph]);
          o = min(o, (uint32_t)CS);
          const uint32_t a = o * (LINE * 4) + cso[ph];
          const uint4 x0 = *reinterpret_cast<const uint4*>(lds0 + a);
          const uint4 x1 = *reinterpret_cast<const uint4*>(lds0 + (a ^ 16u));
          v[pp][0] = x0.x; v[pp][1] = x0.y; v[pp][2] = x0.z; v[pp][3] = x0.w;
          v[pp][4] = x1.x; v[pp][5] = x1.y; v[pp][6] = x1.z; v[pp][7] = x1.w;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[k][t] = xor3(acc[k][t], v[0][t], v[1][t]);
       }
       continue;
#endif
        uint32_t v[NCH][8];
#pragma unroll
        for (uint32_t ph = 0; ph < NCH; ++ph) {
          uint32_t o;
          if constexpr (NCH == 4) o = __builtin_amdgcn_perm(tv[k].y, tv[k].x, psel[ph]);
          else o = __builtin_amdgcn_perm(0u, tv[k], psel[ph]);
          o = min(o, (uint32_t)CS);   // kSkip -> zero line
          if (PM_ROT_ABL == 3 || PM_ROT_ABL == 4 || PM_ROT_ABL == 6) o = __builtin_amdgcn_readfirstlane(o);   // one row per wave: no conflicts
          const uint32_t a = o * (LINE * 4) + cso[ph];
          const uint4 x0 = *reinterpret_cast<const uint4*>(lds0 + a);
          const uint4 x1 = *reinterpret_cast<const uint4*>(lds0 + (a ^ 16u));
          v[ph][0] = x0.x; v[ph][1] = x0.y; v[ph][2] = x0.z; v[ph][3] = x0.w;
          v[ph][4] = x1.x; v[ph][5] = x1.y; v[ph][6] = x1.z; v[ph][7] = x1.w;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          if constexpr (NCH == 4) acc[k][t] = xor3(xor3(acc[k][t], v[0][t], v[1][t]), v[2][t], v[3][t]);
          else acc[k][t] = xor3(acc[k][t], v[0][t], v[1][t]);
        }
      }
    }
    if (false)
#endif
    if constexpr (NCH == 4) {
    // per phase: this lane's chunk slot and its word base in the line
    uint32_t cso[4];
#pragma unroll
    for (uint32_t ph = 0; ph < 4; ++ph) cso[ph] = lb + ((ks + ph) & 3) * 32 + (PM_ROT_B64 ? 8 * (j & 3) : 4 * j);
#pragma unroll
    for (int k = 0; k < (PM_ROT_ABL == 1 ? 0 : HPL); ++k) {
      const bool hv = vl + k * kFoldThreads < v1;   // lane slots past the group: zero line
      // the 4 offsets in phase order: rotate the 64-bit tile right by 16 ks
      const uint64_t t64 = ((uint64_t)tv[k].y << 32) | tv[k].x;
      const uint32_t sh = 16 * ks;
      const uint64_t rot = sh ? ((t64 >> sh) | (t64 << (64 - sh))) : t64;
      uint32_t v[4][8];
#pragma unroll
      for (uint32_t ph = 0; ph < 4; ++ph) {
        uint32_t o = (uint32_t)(rot >> (16 * ph)) & 0xffffu;
        o = hv ? min(o, (uint32_t)CS) : (uint32_t)CS;   // kSkip -> the zero line
        // word (j + t) & 7 of the slot: base + 4t, or base + 4t - 32 where
        // j + t >= 8 (a per-lane select; 4t is the instruction's offset)
        const uint32_t a = o * (LINE * 4) + cso[ph], a2 = a - 32;
        if (PM_ROT_B64) {   // word pair ((j & 3) + t) & 3: 8-B reads, lanes j and j + 4 2-way on a bank pair
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint64_t x = *reinterpret_cast<const uint64_t*>(lds0 + (((j & 3) < 4u - t) ? a : a2) + 8 * t);
            v[ph][2 * t] = (uint32_t)x;
            v[ph][2 * t + 1] = (uint32_t)(x >> 32);
          }
        } else {
#pragma unroll
          for (int t = 0; t < 8; ++t)
            v[ph][t] = *reinterpret_cast<const uint32_t*>(lds0 + ((j < 8u - t) ? a : a2) + 4 * t);
        }
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)   // v_bitop3_b32 0x96 = a ^ b ^ c (gfx950): two XORs per instruction
        acc[k][t] = xor3(xor3(acc[k][t], v[0][t], v[1][t]), v[2][t], v[3][t]);
    }
    }
    if (PM_ROT_PF) {
      // the prefetch may stay in flight: counted wait, then a raw barrier
      // (__syncthreads' fence would wait for every load, the prefetch included)
      asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < HPL; ++k) {
      if constexpr (NCH == 4) tv[k] = PM_ROT_ABL == 6 ? tv[k] + u32x2{1u, 3u} : tn[k];
      else tv[k] = tn[k];
    }
    skip_idle(tv);
  }
#pragma unroll
  for (int k = 0; k < HPL; ++k) {
    const uint32_t v = vl + k * kFoldThreads;
    if (v >= v1) continue;
    const bool inB = v >= vb;
    PM_G uint64_t* const par = (inB ? PB.parity : PA.parity) + (uint64_t)(v - (inB ? vb : hA)) * E;
    PM_G uint32_t* dst = reinterpret_cast<PM_G uint32_t*>(par + w);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      PM_G uint32_t* const d = dst + (PM_ROT_B128 ? 4 * (j ^ (t >> 2)) + (t & 3)
                                      : PM_ROT_B64 ? 2 * (((j & 3) + t / 2) & 3) + (t & 1) : (j + t) & 7);
      if (PM_PREP_NT) __builtin_nontemporal_store(acc[k][t], d);
      else *d = acc[k][t];
    }
    if (w == 0)   // xorSlices leaves the words past len&~3 zero
      for (uint32_t t = E & ~3u; t < E; ++t) par[t] = 0;
  }
}

// One partition's fold image: 16-B item it of block (slice s, chunks NCH b..)
// = line it / (2 NCH), chunk slot (it / 2) % NCH, half it % 2 of row
// (NCH b + slot) CS + line (NCH = rot_nch(CS); 4,096 items per block).
__global__ void __launch_bounds__(kBlock) k_fold_image(uint4* __restrict__ img, const uint64_t* __restrict__ rows,
                                                      uint64_t N, uint32_t nbuf, uint32_t E, uint64_t nitems,
                                                      uint32_t CS) {
  const uint32_t lg = CS == 512 ? 2 : 1;   // log2 NCH
  for (uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x; x < nitems; x += (uint64_t)gridDim.x * kBlock) {
    const uint32_t it = (uint32_t)(x % (kRotBufBytes / 16));
    const uint64_t blk = x / (kRotBufBytes / 16);
    const uint32_t b = (uint32_t)(blk % nbuf), s = (uint32_t)(blk / nbuf);
    const uint64_t r = (uint64_t)((b << lg) + ((it >> 1) & ((1u << lg) - 1))) * CS + (it >> (lg + 1));
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < N) v = *reinterpret_cast<const uint4*>(rows + r * E + 4 * s + (it & 1) * 2);
    img[x] = v;
  }
}

// Replacement rows (pir.go:345-350): Qpc random offsets per chunk, idx + copy.
// One workgroup per kReplRows slots: their offsets are hashed once per row
// (not once per word) into LDS, then the rows are copied in 16-B pieces with
// every piece of a thread in flight together (32-bit index math throughout).
constexpr uint32_t kReplRows = 32, kReplIt = (kReplRows * 1024 / 16 + kBlock - 1) / kBlock;   // E <= 128 words
template <int W>
__global__ void __launch_bounds__(kBlock) k_prep_repl(const PmPart* __restrict__ parts,
                                                      const uint64_t* __restrict__ db, uint32_t E) {
  typedef uint64_t vec __attribute__((ext_vector_type(W)));
  __shared__ uint32_t rrow[kReplRows];   // partition row of each slot, ~0u past the partition's end
  const PmPart& P = parts[blockIdx.y];
  const uint32_t nslot = P.SS * P.Qpc;
  const uint32_t s0 = blockIdx.x * kReplRows;
  if (s0 >= nslot) return;   // block-uniform
  const uint32_t ns = min(kReplRows, nslot - s0);
  if (threadIdx.x < ns) {
    const uint32_t slot = s0 + threadIdx.x, c = slot / P.Qpc;
    const uint64_t off = hash4(P.seed, DOM_REPL, P.idx, P.epoch, slot) & (P.CS - 1);
    const uint64_t r = (uint64_t)c * P.CS + off;
    P.ridx[slot] = (uint32_t)r;
    rrow[threadIdx.x] = r < P.N ? (uint32_t)r : ~0u;
  }
  __syncthreads();
  const uint32_t nseg = E / W, tot = ns * nseg;
  const uint64_t* const src = db + P.row0 * E;
  uint64_t* const dst = P.rval + (uint64_t)s0 * E;
  for (uint32_t x0 = 0; x0 < tot; x0 += kReplIt * kBlock) {
    vec v[kReplIt];
    uint32_t at[kReplIt];
#pragma unroll
    for (uint32_t u = 0; u < kReplIt; ++u) {
      const uint32_t x = x0 + u * kBlock + threadIdx.x;
      at[u] = ~0u;
      v[u] = vec{};
      if (x < tot) {
        const uint32_t i = x / nseg, sg = x - i * nseg, r = rrow[i];
        at[u] = i * E + sg * W;
        if (r != ~0u) v[u] = *reinterpret_cast<const vec*>(src + (uint64_t)r * E + sg * W);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kReplIt; ++u)
      if (at[u] != ~0u) *reinterpret_cast<vec*>(dst + at[u]) = v[u];
  }
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

// PianoPIRServer.PrivateQuery (pir.go:65-88) for nq client-supplied offset
// sets: XOR of SetSize gathered rows.  One workgroup per offset set: lanes =
// (row slice, 16-B segment); slices are XOR-combined through LDS.
template <int W>
__global__ void __launch_bounds__(kBlock) k_server_answer(const PmPart* __restrict__ parts,
                                                          const uint32_t* __restrict__ qoffs,
                                                          uint32_t maxSS,
                                                          const uint64_t* __restrict__ db, uint32_t E,
                                                          uint64_t* __restrict__ ans) {
  __shared__ uint64_t red[kBlock * 2];
  const uint32_t s = blockIdx.x;
  const PmPart& P = parts[0];
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

// ---------------------------------------------------------------------------
// Distance kernels (graphann/l2_distance_amd64.s).
// ---------------------------------------------------------------------------
// L2Dist, bit-exact: lane k of an 8-lane group owns running sum s_k over
// elements 8t+k (VSUBPS/VMULPS/VADDPS, each rounded: no FMA), then the
// VHADDPS tree ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)) as xor-1/2/4 shuffles, then
// the scalar tail of build_graph.go:123-125 on lane 0.
// seglen > 0: rows [j*seglen, (j+1)*seglen) are scored against query j at
// q + j*dim (several clients' start sets in one launch, pm_search_loop_batched)
__global__ void __launch_bounds__(kBlock) k_l2_rows(const float* __restrict__ rows,
                                                    uint64_t stride, uint64_t nrows,
                                                    const uint32_t* __restrict__ ids,
                                                    const float* __restrict__ q, uint32_t dim,
                                                    float* __restrict__ out, uint64_t seglen) {
  const uint64_t g = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 3;
  const uint32_t k = threadIdx.x & 7;
  const bool live = g < nrows;
  const float* r = rows + (live ? (ids ? (uint64_t)ids[g] : g) : 0) * stride;
  if (seglen && live) q += (g / seglen) * dim;
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
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* r4 = reinterpret_cast<const u32x4*>(rows);
  uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (stride % dim4 == 0) {
    // the grid stride is whole rows: a thread's column (and query slice) is
    // fixed, and kU 16-B nontemporal loads are in flight per thread
    const uint32_t j = (uint32_t)(f % dim4) * 4;
    const uint32_t q0 = qs[j], q1 = qs[j + 1], q2 = qs[j + 2], q3 = qs[j + 3];
    constexpr int kU = 8;
    for (; f + (kU - 1) * stride < n4; f += kU * stride) {
      u32x4 t[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) t[u] = __builtin_nontemporal_load(r4 + f + u * stride);
#pragma unroll
      for (int u = 0; u < kU; ++u) acc += t[u].x * q0 + t[u].y * q1 + t[u].z * q2 + t[u].w * q3;
    }
    for (; f < n4; f += stride) {
      const u32x4 t = __builtin_nontemporal_load(r4 + f);
      acc += t.x * q0 + t.y * q1 + t.z * q2 + t.w * q3;
    }
  } else {
    for (; f < n4; f += stride) {
      const u32x4 t = __builtin_nontemporal_load(r4 + f);
      const uint32_t j = (uint32_t)(f % dim4) * 4;
      acc += t.x * qs[j] + t.y * qs[j + 1] + t.z * qs[j + 2] + t.w * qs[j + 3];
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

__global__ void __launch_bounds__(kBlock) k_ip_fill(uint4* __restrict__ rows, uint64_t n4, uint32_t dim,
                                                    uint64_t r0) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < n4; f += stride) {
    const uint64_t e = f * 4;
    const uint32_t i = (uint32_t)(r0 + e / dim), j = (uint32_t)(e % dim);   // global row (uint32 as in Go)
    rows[f] = make_uint4(i + j, i + j + 1, i + j + 2, i + j + 3);
  }
}

// Synthetic DB fill (BIGANN-scale benchmarks: the rows never cross PCIe).
// Grid-stride over the words of rows [r0, r0 + rows) of the global DB.
__global__ void __launch_bounds__(kBlock) k_db_synth(uint64_t* __restrict__ dst, uint64_t r0, uint64_t nw,
                                                     uint32_t E, uint64_t k) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock, x0 = r0 * E;
  for (uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x; f < nw; f += stride)
    __builtin_nontemporal_store(sm64(k ^ (x0 + f)), dst + f);
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
  const AesLane A(te, threadIdx.x);
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    out[i] = prf64(A, srk, tags[i], xs[i]);
}

// Device-resident batch responses (pm_batchpir_query_dev): row i of out
// (E + 1 words) = the entry at src[i] (a row of a partition's localCache arena
// in HBM; the pointer list sits in pinned host memory) and the success flag,
// or zeros.  One workgroup per response; E <= 2048.
__global__ void __launch_bounds__(kBlock) k_gather_rows(const uint64_t* const* __restrict__ src, uint32_t E,
                                                         uint64_t* __restrict__ out) {
  const uint64_t i = blockIdx.x;
  const uint64_t* r = src[i];
  uint64_t* o = out + i * (E + 1);
  for (uint32_t w = threadIdx.x; w < E; w += kBlock) o[w] = r ? r[w] : 0;
  if (threadIdx.x == 0) o[E] = r ? 1 : 0;
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
void prep_offsets_tt(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t maxSS) {
  hipLaunchKernelGGL(k_prep_offsets, dim3(cdiv(maxH, kOffsBlock), cdiv(maxSS, kOffsChunksPerBlock * kOffsTiles), np),
                     dim3(kOffsBlock), 0, st, d);
}
void prep_offsets_bs(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t maxSS) {
  hipLaunchKernelGGL(k_prep_offsets_bs, dim3(cdiv((uint64_t)cdiv(maxH, 32) * cdiv(maxSS, 8), kBsThreads), np),
                     dim3(kBsThreads), 0, st, d);
}
static std::atomic<int> g_aes_bs{-1};
void set_aes_bs(int v) { g_aes_bs.store(v < 0 ? -1 : (v ? 1 : 0)); }
bool prep_offsets_bitsliced() {
  static const bool env = [] { const char* e = getenv("PM_AES_BS"); return e && e[0] == '1'; }();
  const int v = g_aes_bs.load();
  return v < 0 ? env : v == 1;
}
void prep_offsets(hipStream_t st, const PmPart* d, int np, uint32_t maxH, uint32_t maxSS) {
  if (prep_offsets_bitsliced()) prep_offsets_bs(st, d, np, maxH, maxSS);
  else prep_offsets_tt(st, d, np, maxH, maxSS);
}
bool fold_image_ok(uint32_t minCS, uint32_t maxCS, uint32_t E) {
  static const bool rot = [] { const char* e = getenv("PM_FOLD_ROT"); return !e || e[0] != '0'; }();
  return rot && minCS == maxCS && (maxCS == 512 || maxCS == 1024) && E % 2 == 0 && E >= 4;
}
bool fold_needs_tab(uint32_t minCS, uint32_t maxCS, uint32_t E, bool have_img) {
  // the folds that stage a chunk-major PRF table row through LDS (k_prep_fold_pipe
  // / _blk); the rotated fold and the unblocked gather read the tag-major one
  if ((E & ~3u) == 0) return false;
  if (have_img && fold_image_ok(minCS, maxCS, E)) return false;
  const bool pipe = minCS == maxCS && (maxCS == 512 || maxCS == 1024 || maxCS == 2048) && E % 2 == 0;
  if (pipe) return true;
  auto fits = [&](uint32_t sw) {   // prep_fold's choice of the double-buffered fold
    return 2ull * (maxCS + 1) * sw * 8 <= 150u * 1024 && (uint64_t)maxCS * (sw / 2) <= (uint64_t)kFoldMaxItems * kFoldThreads;
  };
  uint32_t sw = 8;
  while (sw > 2 && !fits(sw)) sw /= 2;
  return fits(sw) && E % 2 == 0;
}
uint64_t fold_image_words(uint32_t SS, uint32_t E, uint32_t CS) {
  return (uint64_t)(E / 4) * (SS / rot_nch(CS)) * (kRotBufBytes / 8);
}
void fold_image(hipStream_t st, uint64_t* img, const uint64_t* rows, uint64_t N, uint32_t SS, uint32_t E, uint32_t CS) {
  const uint64_t nitems = fold_image_words(SS, E, CS) / 2;
  unsigned grid = cdiv(nitems, kBlock);
  if (grid > 256 * 32) grid = 256 * 32;
  hipLaunchKernelGGL(k_fold_image, dim3(grid), dim3(kBlock), 0, st, (uint4*)img, rows, N, SS / rot_nch(CS), E, nitems,
                     CS);
}
int prep_fold(hipStream_t st, const PmPart* d, int np, uint32_t maxH, const uint64_t* db, uint32_t E,
              uint32_t minCS, uint32_t maxCS, const uint64_t* zero16, uint32_t clients, bool have_img,
               uint32_t minH) {
  const uint32_t EX = E & ~3u;
  if (EX == 0) {
    hipLaunchKernelGGL(k_prep_fold<2>, dim3(cdiv((uint64_t)maxH * E, kBlock), np), dim3(kBlock), 0,
                       st, d, db, E);
    return FOLD_OTHER;
  }
  // column-slice width: the widest whose double-buffered chunk fits in LDS and
  // whose staging fits kFoldMaxItems 16-B items per thread
  const uint32_t ng = cdiv(maxH, (uint64_t)kFoldThreads * kFoldHPT);      // pipelined fold
  const uint32_t ngb = cdiv(maxH, (uint64_t)kFoldThreads * kFoldHPTBlk);  // double-buffered fold
  auto fits = [&](uint32_t sw) {
    return 2ull * (maxCS + 1) * sw * 8 <= 150u * 1024 &&
           (uint64_t)maxCS * (sw / 2) <= (uint64_t)kFoldMaxItems * kFoldThreads;
  };
  auto launch = [&](uint32_t sw, uint32_t w0, uint32_t nsl) {
    const size_t lds = 2ull * (maxCS + 1) * sw * 8;
    const dim3 grid(ngb, nsl, np), blk(kFoldThreads);
    if (sw == 8) hipLaunchKernelGGL(k_prep_fold_blk<8>, grid, blk, lds, st, d, db, zero16, E, w0);
    else if (sw == 4) hipLaunchKernelGGL(k_prep_fold_blk<4>, grid, blk, lds, st, d, db, zero16, E, w0);
    else hipLaunchKernelGGL(k_prep_fold_blk<2>, grid, blk, lds, st, d, db, zero16, E, w0);
  };
  if (minCS == maxCS && (maxCS == 512 || maxCS == 1024 || maxCS == 2048) && E % 2 == 0) {
    // (SW, G): CS 512 -> (4, 1), 1024 -> (4, 2), 2048 -> (2, 2); EX % SW == 0
    const uint32_t psw = maxCS == 2048 ? 2 : 4, nsl = EX / psw;
    const uint32_t K = clients && np % clients == 0 ? clients : 1, npg = (np / K) * ng;
    const uint32_t lw = 16 / psw, per_pg = K * cdiv(nsl, lw) * lw;
#ifndef PM_FOLD_NB512
#define PM_FOLD_NB512 4
#endif
#ifndef PM_FOLD_D512
#define PM_FOLD_D512 1
#endif
    if (have_img && fold_image_ok(minCS, maxCS, E)) {   // the bank-rotated fold (same slices and block order)
      // virtual hint groups over the K clients of each partition (see the kernel)
      const uint64_t HB = (uint64_t)kFoldThreads * rot_hpl(maxCS);
      const uint32_t ngc = minH >= HB ? 0u : (uint32_t)cdiv(maxH, HB);
      const uint32_t nvg = ngc ? K * ngc : (uint32_t)cdiv((uint64_t)K * maxH, HB), npv = (np / K) * nvg;
      const uint32_t M = cdiv(npv, 8);
      const uint32_t grid = PM_ROT_ORDER == 1
                                ? 8 * cdiv((uint64_t)cdiv(npv, PM_ROT_GB) * cdiv(nsl, PM_ROT_SB), 8) * PM_ROT_GB * PM_ROT_SB
                                : 8 * M * cdiv(nsl, PM_ROT_LW) * PM_ROT_LW;
      if (maxCS == 512) {
        hipLaunchKernelGGL(k_prep_fold_rot<512>, dim3(grid), dim3(kFoldThreads), 0, st, d, E, nvg, nsl, npv, M, K, ngc);
        return FOLD_ROT512;
      }
      hipLaunchKernelGGL(k_prep_fold_rot<1024>, dim3(grid), dim3(kFoldThreads), 0, st, d, E, nvg, nsl, npv, M, K, ngc);
      return FOLD_ROT1024;
    }
    const uint32_t nb = maxCS == 512 ? PM_FOLD_NB512 : 3;   // LDS buffers: <= 150 KB
    const size_t lds = (size_t)nb * ((maxCS + 1) * psw + kPipeTabWords) * 8;
    const dim3 grid(cdiv(npg, 8) * 8 * per_pg), blk(kFoldThreads);
    if (maxCS == 512)
      hipLaunchKernelGGL((k_prep_fold_pipe<4, 1, PM_FOLD_NB512, PM_FOLD_D512>), grid, blk, lds, st, d, db, zero16, E, ng, nsl,
                         npg, K);
    else if (maxCS == 1024)
      hipLaunchKernelGGL((k_prep_fold_pipe<4, 2, 3>), grid, blk, lds, st, d, db, zero16, E, ng, nsl, npg, K);
    else
      hipLaunchKernelGGL((k_prep_fold_pipe<2, 2, 3>), grid, blk, lds, st, d, db, zero16, E, ng, nsl, npg, K);
    return FOLD_OTHER;
  }
  uint32_t sw = 8;
  while (sw > 2 && !fits(sw)) sw /= 2;
  if (!fits(sw) || E % 2) {   // very wide chunks or odd entries: the unblocked gather
    if (E % 2 == 0)
      hipLaunchKernelGGL(k_prep_fold<2>, dim3(cdiv((uint64_t)maxH * (EX / 2), kBlock), np),
                         dim3(kBlock), 0, st, d, db, E);
    else
      hipLaunchKernelGGL(k_prep_fold<1>, dim3(cdiv((uint64_t)maxH * EX, kBlock), np), dim3(kBlock), 0,
                         st, d, db, E);
    return FOLD_OTHER;
  }
  const uint32_t nfull = EX / sw, rem = EX % sw;   // EX is a multiple of 4
  if (nfull) launch(sw, 0, nfull);
  if (rem) launch(rem, nfull * sw, 1);
  return FOLD_OTHER;
}
void prep_repl(hipStream_t st, const PmPart* d, int np, uint32_t maxRepl, const uint64_t* db,
               uint32_t E) {
  if (E % 2 == 0)
    hipLaunchKernelGGL(k_prep_repl<2>, dim3(cdiv(maxRepl, kReplRows), np), dim3(kBlock), 0, st, d, db, E);
  else
    hipLaunchKernelGGL(k_prep_repl<1>, dim3(cdiv(maxRepl, kReplRows), np), dim3(kBlock), 0, st, d, db, E);
}
void server_answer(hipStream_t st, const PmPart* d, const uint32_t* offs, uint32_t nq, uint32_t SS,
                   const uint64_t* db, uint32_t E, uint64_t* out) {
  if (E % 2 == 0)
    hipLaunchKernelGGL(k_server_answer<2>, dim3(nq), dim3(kBlock), 0, st, d, offs, SS, db, E, out);
  else
    hipLaunchKernelGGL(k_server_answer<1>, dim3(nq), dim3(kBlock), 0, st, d, offs, SS, db, E, out);
}
void l2_rows(hipStream_t st, const float* rows, uint64_t stride, uint64_t nrows, const uint32_t* ids,
             const float* q, uint32_t dim, float* out, uint64_t seglen) {
  if (!nrows) return;
  hipLaunchKernelGGL(k_l2_rows, dim3(cdiv(nrows * 8, kBlock)), dim3(kBlock), 0, st, rows, stride, nrows,
                     ids, q, dim, out, seglen);
}
void ip_rows(hipStream_t st, const uint32_t* rows, uint64_t nrows, const uint32_t* q, uint32_t dim,
             uint32_t* per_row, uint32_t* sum) {
  if (!per_row && dim % 4 == 0 && dim <= 4096) {
    const uint64_t n4 = nrows * dim / 4;
    unsigned grid = cdiv(n4, kBlock);
    if (grid > 256 * 8) grid = 256 * 8;   // 8 workgroups per CU: 2,048 x 256 threads, 16 waves per CU
    if (grid == 0) return;
    hipLaunchKernelGGL(k_ip_scan, dim3(grid), dim3(kBlock), 0, st, (const uint4*)rows, n4, q, dim, sum);
    return;
  }
  if (!nrows) return;
  hipLaunchKernelGGL(k_ip_rows, dim3(cdiv(nrows * 16, kBlock)), dim3(kBlock), 0, st, rows, nrows, q, dim,
                     per_row, sum);
}
void ip_fill(hipStream_t st, uint32_t* rows, uint64_t N, uint32_t D, uint64_t r0) {
  const uint64_t n4 = N * D / 4;
  unsigned grid = cdiv(n4, kBlock);
  if (grid > 256 * 16) grid = 256 * 16;
  if (grid == 0) return;
  hipLaunchKernelGGL(k_ip_fill, dim3(grid), dim3(kBlock), 0, st, (uint4*)rows, n4, D, r0);
}
void db_synth(hipStream_t st, uint64_t* dst, uint64_t r0, uint64_t rows, uint32_t E, uint64_t db_seed) {
  const uint64_t nw = rows * E;
  unsigned grid = cdiv(nw, kBlock);
  if (grid > 256 * 32) grid = 256 * 32;
  if (grid == 0) return;
  hipLaunchKernelGGL(k_db_synth, dim3(grid), dim3(kBlock), 0, st, dst, r0, nw, E, sm64(db_seed + DOM_SYNTH_DB));
}
void gather_rows(hipStream_t st, const uint64_t* const* src, uint64_t n, uint32_t E, uint64_t* out) {
  if (n) hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)n), dim3(kBlock), 0, st, src, E, out);
}
void prf_batch(hipStream_t st, const uint32_t* rk, const uint64_t* tags, const uint64_t* xs, uint64_t n,
               uint64_t* out) {
  unsigned grid = cdiv(n, kBlock * 16);
  if (grid == 0) return;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_prf_batch, dim3(grid), dim3(kBlock), 0, st, rk, tags, xs, n, out);
}
}  // namespace pmk
