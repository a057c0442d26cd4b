// pm_aes.h — AES-128-MMO PRF for gfx950 VALU + LDS (no AES instructions on CDNA).
//
// Replaces aes128MMO / PRFEvalWithLongKeyAndTag (pianopir/aes_amd64.s:51-82,
// pianopir/util.go:157-165).  One block per lane, T-table formulation with a
// single table Te0 (rows 1-3 are byte rotations of it) held in LDS replicated
// 32x so that lane l always reads bank (l & 31): a random-index ds_read_b32 is
// then conflict-free (bank = (addr/4) % 32, MI355X_MICROARCH.md §LDS).
// 32 KiB of LDS per workgroup.  Bit-exact with AES-NI: the state is kept as
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

constexpr int kTeLdsWords = 256 * 32;   // 32 KiB replicated Te0

// Device copy of the tables (one per translation unit; read only by aes_lds_init).
static constexpr AesTables kAesTablesHost{};
static __device__ const AesTables g_aes = kAesTablesHost;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// Fill the replicated table.  Call with the whole block, then __syncthreads().
__device__ __forceinline__ void aes_lds_init(uint32_t* te, const uint32_t* __restrict__ g_te0) {
  for (int i = threadIdx.x; i < kTeLdsWords; i += blockDim.x) te[i] = g_te0[i >> 5];
}

struct AesLane {
  const uint32_t* te;
  uint32_t lane;   // (threadIdx.x & 31)
  __device__ __forceinline__ uint32_t T(uint32_t b) const { return te[(b << 5) | lane]; }
  __device__ __forceinline__ uint32_t S(uint32_t b) const { return (T(b) >> 8) & 0xffu; }
};

// Nine full rounds on state (s0..s3) with round keys rk[4..39].
__device__ __forceinline__ void aes_rounds(const AesLane& A, const uint32_t* __restrict__ rk,
                                           uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3) {
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t t0 = A.T(s0 & 0xff) ^ rotl32(A.T((s1 >> 8) & 0xff), 8) ^
                  rotl32(A.T((s2 >> 16) & 0xff), 16) ^ rotl32(A.T(s3 >> 24), 24) ^ rk[4 * r + 0];
    uint32_t t1 = A.T(s1 & 0xff) ^ rotl32(A.T((s2 >> 8) & 0xff), 8) ^
                  rotl32(A.T((s3 >> 16) & 0xff), 16) ^ rotl32(A.T(s0 >> 24), 24) ^ rk[4 * r + 1];
    uint32_t t2 = A.T(s2 & 0xff) ^ rotl32(A.T((s3 >> 8) & 0xff), 8) ^
                  rotl32(A.T((s0 >> 16) & 0xff), 16) ^ rotl32(A.T(s1 >> 24), 24) ^ rk[4 * r + 2];
    uint32_t t3 = A.T(s3 & 0xff) ^ rotl32(A.T((s0 >> 8) & 0xff), 8) ^
                  rotl32(A.T((s1 >> 16) & 0xff), 16) ^ rotl32(A.T(s2 >> 24), 24) ^ rk[4 * r + 3];
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
  uint32_t c0 = (A.S(s0 & 0xff) | (A.S((s1 >> 8) & 0xff) << 8) | (A.S((s2 >> 16) & 0xff) << 16) |
                 (A.S(s3 >> 24) << 24)) ^ rk[40];
  uint32_t c1 = (A.S(s1 & 0xff) | (A.S((s2 >> 8) & 0xff) << 8) | (A.S((s3 >> 16) & 0xff) << 16) |
                 (A.S(s0 >> 24) << 24)) ^ rk[41];
  return ((uint64_t)(c1 ^ w1) << 32) | (uint64_t)(c0 ^ w0);
}

// Low 32 bits of the PRF (enough for an offset: ChunkSize <= 2^31).
__device__ __forceinline__ uint32_t prf_lo32(const AesLane& A, const uint32_t* __restrict__ rk,
                                             uint64_t tag, uint64_t x) {
  const uint64_t b = (tag << 35) + x;
  const uint32_t w0 = (uint32_t)b, w1 = (uint32_t)(b >> 32);
  uint32_t s0 = w0 ^ rk[0], s1 = w1 ^ rk[1], s2 = rk[2], s3 = rk[3];
  aes_rounds(A, rk, s0, s1, s2, s3);
  uint32_t c0 = (A.S(s0 & 0xff) | (A.S((s1 >> 8) & 0xff) << 8) | (A.S((s2 >> 16) & 0xff) << 16) |
                 (A.S(s3 >> 24) << 24)) ^ rk[40];
  return c0 ^ w0;
}

}  // namespace pm
