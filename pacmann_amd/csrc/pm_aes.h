// pm_aes.h — AES-128-MMO PRF for gfx950 VALU + LDS (no AES instructions on CDNA).
//
// Replaces aes128MMO / PRFEvalWithLongKeyAndTag (pianopir/aes_amd64.s:51-82,
// pianopir/util.go:157-165).  One block per lane, T-table formulation with two
// tables in LDS, Te0 and Te2 = rotl16(Te0), each replicated 32x so that lane l
// always reads bank (l & 31) of its 32-lane group: a random-index ds_read_b32
// is then conflict-free (bank = (addr/4) % 32, MI355X_MICROARCH.md §LDS).
// With Te2 a round column is Te0[a] ^ Te2[c] ^ rotl8(Te0[b] ^ Te2[d]) ^ rk:
// one rotation instead of three (the kernel is VALU-bound).  64 KiB of LDS per
// workgroup.  Bit-exact with AES-NI: the state is kept as
// four little-endian column words, exactly the byte order AESENC works on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pm {

struct AesTables {
  uint8_t sbox[256];
  uint32_t te0[256];   // LE column word {2S, S, S, 3S}
  constexpr AesTables() : sbox(), te0() {
    // S-box from the GF(2^8) inverse + affine map (FIPS-197 §5.1.1).
    for (int x = 0; x < 256; ++x) {
      uint8_t inv = 0;
      if (x) {
        // x^254 by square-and-multiply
        uint8_t r = 1, b = (uint8_t)x;
        int e = 254;
        while (e) {
          if (e & 1) r = gmul(r, b);
          b = gmul(b, b);
          e >>= 1;
        }
        inv = r;
      }
      uint8_t s = inv ^ rotl(inv, 1) ^ rotl(inv, 2) ^ rotl(inv, 3) ^ rotl(inv, 4) ^ 0x63;
      sbox[x] = s;
      uint32_t s2 = gmul(s, 2), s3 = gmul(s, 3);
      te0[x] = s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | (s3 << 24);
    }
  }
  static constexpr uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
      if (b & 1) p ^= a;
      bool hi = a & 0x80;
      a = (uint8_t)(a << 1);
      if (hi) a ^= 0x1b;
      b >>= 1;
    }
    return p;
  }
  static constexpr uint8_t rotl(uint8_t v, int n) { return (uint8_t)((v << n) | (v >> (8 - n))); }
};

// Entry b of lane l's copies: Te0 at byte (b << 8) | ((l & 31) << 2), Te2 at
// that | 0x80.  A lookup address is ONE v_perm_b32 (the state byte into byte
// 1, the lane offset with the table bit in byte 0), and a ds_read_b32 lane
// group (32 lanes, bank = (a/4) mod 32) reads 32 distinct banks.  64 KiB.
#ifndef PM_AES_4T
#define PM_AES_4T 0   // all four T-tables in LDS (Te1 = rotl8 Te0, Te3 = rotl24 Te0 in a second 64 KiB):
#endif                // no rotation or extra XOR per column, but 128 KiB per workgroup, i.e. 16 waves per CU
                      // instead of 32: 76 vs 53.6 ms per 288-client launch (profiles/r05/ab/aes_four_tables.log)
constexpr int kTeLdsWords = 256 * 64 * (PM_AES_4T ? 2 : 1);

// Device copy of the tables (one per translation unit; read only by aes_lds_init).
static constexpr AesTables kAesTablesHost{};
static __device__ const AesTables g_aes = kAesTablesHost;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t aes_x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Fill the replicated table.  Call with the whole block, then __syncthreads().
__device__ __forceinline__ void aes_lds_init(uint32_t* te, const uint32_t* __restrict__ g_te0) {
  for (int i = threadIdx.x; i < kTeLdsWords; i += blockDim.x) {
    const uint32_t t = g_te0[(i >> 6) & 255];
    te[i] = i < 256 * 64 ? ((i & 32) ? rotl32(t, 16) : t)     // Te0 | Te2
                         : ((i & 32) ? rotl32(t, 24) : rotl32(t, 8));   // Te1 | Te3
  }
}


struct AesLane {
  const uint32_t* te;
  uint32_t lane;    // (threadIdx.x & 31) << 2: this lane's byte offset within an entry row
  uint32_t lane2;   // lane | 0x80: its Te2 copy
  __device__ AesLane(const uint32_t* t, uint32_t tid) : te(t), lane((tid & 31u) << 2), lane2(((tid & 31u) << 2) | 0x80u) {}
  // Te0 / Te2 [byte k of s] from this lane's copy: address = (byte << 8) | lane, one v_perm_b32
  template <int K> __device__ __forceinline__ uint32_t Tk(uint32_t s) const {
    const uint32_t a = __builtin_amdgcn_perm(s, lane, 0x0c0c0000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(te) + a);
  }
  template <int K> __device__ __forceinline__ uint32_t T2k(uint32_t s) const {
    const uint32_t a = __builtin_amdgcn_perm(s, lane2, 0x0c0c0000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(te) + a);
  }
  template <int K> __device__ __forceinline__ uint32_t Sk(uint32_t s) const { return (Tk<K>(s) >> 8) & 0xffu; }
  // PM_AES_4T: Te1 / Te3 [byte k of s] in the second 64 KiB (byte 2 of the
  // address from the lane word: lane | 0x10000)
  template <int K> __device__ __forceinline__ uint32_t T1k(uint32_t s) const {
    const uint32_t a = __builtin_amdgcn_perm(s, lane | 0x10000u, 0x0c020000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(te) + a);
  }
  template <int K> __device__ __forceinline__ uint32_t T3k(uint32_t s) const {
    const uint32_t a = __builtin_amdgcn_perm(s, lane2 | 0x10000u, 0x0c020000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(te) + a);
  }
  // one round column: Te0[a.b0] ^ Te1[b.b1] ^ Te2[c.b2] ^ Te3[d.b3] ^ k
  __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
#if PM_AES_4T
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(Tk<0>(a), T1k<1>(b), T2k<2>(c), 0x96), T3k<3>(d), k, 0x96);
#else
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(Tk<0>(a), T2k<2>(c), k, 0x96),
                                       rotl32(Tk<1>(b) ^ T2k<3>(d), 8), 0u, 0x96);
#endif
  }
};

// Full rounds R0..R1-1 on state (s0..s3) with round keys rk[4*R0..4*R1-1].
template <int R0 = 1, int R1 = 10>
__device__ __forceinline__ void aes_rounds(const AesLane& A, const uint32_t* __restrict__ rk,
                                           uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3) {
#pragma unroll
  for (int r = R0; r < R1; ++r) {
    // Te0[a] ^ rotl8(Te0[b]) ^ rotl16(Te0[c]) ^ rotl24(Te0[d]) ^ rk
    //   = Te0[a] ^ Te2[c] ^ rotl8(Te0[b] ^ Te2[d]) ^ rk
    // (v_bitop3_b32 0x96 = three-input XOR on gfx950: 4 VALU per column instead of 5)
    uint32_t t0 = A.col(s0, s1, s2, s3, rk[4 * r + 0]);
    uint32_t t1 = A.col(s1, s2, s3, s0, rk[4 * r + 1]);
    uint32_t t2 = A.col(s2, s3, s0, s1, rk[4 * r + 2]);
    uint32_t t3 = A.col(s3, s0, s1, s2, rk[4 * r + 3]);
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
}

// Full 64-bit PRF(tag, x) = low64_LE(AES_k(B) ^ B), B = LE64((tag<<35)+x) || 0^8.
__device__ __forceinline__ uint64_t prf64(const AesLane& A, const uint32_t* __restrict__ rk,
                                          uint64_t tag, uint64_t x) {
  const uint64_t b = (tag << 35) + x;
  const uint32_t w0 = (uint32_t)b, w1 = (uint32_t)(b >> 32);
  uint32_t s0 = w0 ^ rk[0], s1 = w1 ^ rk[1], s2 = rk[2], s3 = rk[3];
  aes_rounds(A, rk, s0, s1, s2, s3);
  uint32_t c0 = (A.Sk<0>(s0) | (A.Sk<1>(s1) << 8) | (A.Sk<2>(s2) << 16) | (A.Sk<3>(s3) << 24)) ^ rk[40];
  uint32_t c1 = (A.Sk<0>(s1) | (A.Sk<1>(s2) << 8) | (A.Sk<2>(s3) << 16) | (A.Sk<3>(s0) << 24)) ^ rk[41];
  return ((uint64_t)(c1 ^ w1) << 32) | (uint64_t)(c0 ^ w0);
}

// Low 32 bits of the PRF (enough for an offset: ChunkSize <= 2^31).
__device__ __forceinline__ uint32_t prf_lo32(const AesLane& A, const uint32_t* __restrict__ rk,
                                             uint64_t tag, uint64_t x) {
  const uint64_t b = (tag << 35) + x;
  const uint32_t w0 = (uint32_t)b, w1 = (uint32_t)(b >> 32);
  uint32_t s0 = w0 ^ rk[0], s1 = w1 ^ rk[1], s2 = rk[2], s3 = rk[3];
  aes_rounds(A, rk, s0, s1, s2, s3);
  uint32_t c0 = (A.Sk<0>(s0) | (A.Sk<1>(s1) << 8) | (A.Sk<2>(s2) << 16) | (A.Sk<3>(s3) << 24)) ^ rk[40];
  return c0 ^ w0;
}

// PRF(tag, x) for a fixed tag over many x (the hint-table expansion, tag = the
// hint, x = the chunk): block words w0 = x, w1 = tag << 3 (x < 2^32), so after
// the whitening s0 = x ^ rk0 varies with x only, s1 = (tag << 3) ^ rk1 with the
// tag only, and s2 = rk2, s3 = rk3 not at all.  Round 1's columns split into a
// part of s0, s2, s3 (per x: R1Uniform, computed once per x for the whole
// workgroup) and a part of s1 (per lane: R1Lane, once per tag).
struct R1Uniform { uint32_t u0, u1, u2, u3; };
__device__ __forceinline__ R1Uniform r1_uniform(const AesLane& A, const uint32_t* __restrict__ rk, uint32_t x) {
  const uint32_t s0 = x ^ rk[0], s2 = rk[2], s3 = rk[3];
  // rotl24(Te0[v]) = rotl8(Te2[v])
  return R1Uniform{A.Tk<0>(s0) ^ A.T2k<2>(s2) ^ rotl32(A.T2k<3>(s3), 8) ^ rk[4],
                   A.T2k<2>(s3) ^ rotl32(A.Tk<1>(s2) ^ A.T2k<3>(s0), 8) ^ rk[5],
                   A.Tk<0>(s2) ^ A.T2k<2>(s0) ^ rotl32(A.Tk<1>(s3), 8) ^ rk[6],
                   A.Tk<0>(s3) ^ rotl32(A.Tk<1>(s0) ^ A.T2k<3>(s2), 8) ^ rk[7]};
}
struct R1Lane { uint32_t v0, v1, v2, v3; };
__device__ __forceinline__ R1Lane r1_lane(const AesLane& A, const uint32_t* __restrict__ rk, uint64_t tag) {
  const uint32_t s1 = (uint32_t)(tag << 3) ^ rk[1];
  return R1Lane{rotl32(A.Tk<1>(s1), 8), A.Tk<0>(s1), rotl32(A.T2k<3>(s1), 8), A.T2k<2>(s1)};
}
// = prf_lo32(A, rk, tag, x) given r1_uniform(x) and r1_lane(tag).
__device__ __forceinline__ uint32_t prf_lo32_split(const AesLane& A, const uint32_t* __restrict__ rk,
                                                   const R1Uniform& u, const R1Lane& v, uint32_t x) {
  uint32_t s0 = u.u0 ^ v.v0, s1 = u.u1 ^ v.v1, s2 = u.u2 ^ v.v2, s3 = u.u3 ^ v.v3;
  aes_rounds<2>(A, rk, s0, s1, s2, s3);
  const uint32_t c0 = (A.Sk<0>(s0) | (A.Sk<1>(s1) << 8) | (A.Sk<2>(s2) << 16) | (A.Sk<3>(s3) << 24)) ^ rk[40];
  return c0 ^ x;
}

// The low 16 bits of the same PRF (the hint tables keep PRF & (ChunkSize - 1),
// ChunkSize <= 2^15).  Output bytes 0 and 1 of the last round are S[s0 byte 0]
// and S[s1 byte 1], so round 9 computes only columns 0 and 1 and round 10 two
// S-box bytes: 122 lookups per PRF instead of 132.
__device__ __forceinline__ uint32_t prf_lo16_split(const AesLane& A, const uint32_t* __restrict__ rk,
                                                   const R1Uniform& u, const R1Lane& v, uint32_t x) {
  uint32_t s0 = u.u0 ^ v.v0, s1 = u.u1 ^ v.v1, s2 = u.u2 ^ v.v2, s3 = u.u3 ^ v.v3;
  aes_rounds<2, 9>(A, rk, s0, s1, s2, s3);
  const uint32_t t0 = A.col(s0, s1, s2, s3, rk[36]);
  const uint32_t t1 = A.col(s1, s2, s3, s0, rk[37]);
  return ((A.Sk<0>(t0) | (A.Sk<1>(t1) << 8)) ^ rk[40] ^ x) & 0xffffu;
}
// Chunks x < 256 (SetSize <= 256: SIFT1M's 124, MS-MARCO's 196): after the
// whitening only byte 0 of s0 depends on x, so of round 1's output only column
// 0 does (u0; u1..u3 see bytes 3, 2, 1 of s0).  Then every column of round 2
// takes exactly one byte of that column and three bytes fixed by the hint:
//   t0 = Te0[s0.b0]        ^ k0    t1 = rotl8(Te2[s0.b3]) ^ k1
//   t2 = Te2[s0.b2]        ^ k2    t3 = rotl8(Te0[s0.b1]) ^ k3
// (rotl8 is linear over XOR).  R2Hint holds k0..k3, 12 lookups once per hint;
// a PRF then costs 4 round-2 lookups instead of 16: 112 per PRF instead of
// 122.5, bit for bit the same function.
struct R2Hint { uint32_t k0, k1, k2, k3; };
__device__ __forceinline__ R2Hint r2_hint(const AesLane& A, const uint32_t* __restrict__ rk, const R1Uniform& u,
                                          const R1Lane& v) {
  const uint32_t s1 = u.u1 ^ v.v1, s2 = u.u2 ^ v.v2, s3 = u.u3 ^ v.v3;   // the same for every x < 256
  return R2Hint{A.T2k<2>(s2) ^ rk[8] ^ rotl32(A.Tk<1>(s1) ^ A.T2k<3>(s3), 8),
                A.Tk<0>(s1) ^ A.T2k<2>(s3) ^ rk[9] ^ rotl32(A.Tk<1>(s2), 8),
                A.Tk<0>(s2) ^ rk[10] ^ rotl32(A.Tk<1>(s3) ^ A.T2k<3>(s1), 8),
                A.Tk<0>(s3) ^ A.T2k<2>(s1) ^ rk[11] ^ rotl32(A.T2k<3>(s2), 8)};
}
// = prf_lo16_split(A, rk, u, v, x) for x < 256, given u0 = r1_uniform(x).u0 and r2_hint.
__device__ __forceinline__ uint32_t prf_lo16_r2(const AesLane& A, const uint32_t* __restrict__ rk, uint32_t u0,
                                                const R1Lane& v, const R2Hint& k, uint32_t x) {
  const uint32_t s = u0 ^ v.v0;
#if PM_AES_4T
  uint32_t s0 = A.Tk<0>(s) ^ k.k0, s1 = A.T3k<3>(s) ^ k.k1;   // rotl8(Te2) = Te3, rotl8(Te0) = Te1
  uint32_t s2 = A.T2k<2>(s) ^ k.k2, s3 = A.T1k<1>(s) ^ k.k3;
#else
  uint32_t s0 = A.Tk<0>(s) ^ k.k0, s1 = rotl32(A.T2k<3>(s), 8) ^ k.k1;
  uint32_t s2 = A.T2k<2>(s) ^ k.k2, s3 = rotl32(A.Tk<1>(s), 8) ^ k.k3;
#endif
  aes_rounds<3, 9>(A, rk, s0, s1, s2, s3);
  const uint32_t t0 = A.col(s0, s1, s2, s3, rk[36]);
  const uint32_t t1 = A.col(s1, s2, s3, s0, rk[37]);
  return ((A.Sk<0>(t0) | (A.Sk<1>(t1) << 8)) ^ rk[40] ^ x) & 0xffffu;
}
}  // namespace pm
