// pm_aes_bs.h — bitsliced AES-128-MMO on the VALU (round 6): the PRF tables of
// client preprocessing (pir.go:316-339's PRF, pianopir/aes_amd64.s:51-82) with
// no table lookups in rounds 3-10.
//
// Layout: a lane holds 32 blocks as 128 bit planes, plane (byte p, bit b) =
// one uint32_t whose bit j is bit b of byte p of block j.  The 32 blocks of a
// lane are the tags 32m .. 32m + 31 (hints of one group) at one chunk x:
// B = LE64((tag << 35) + x) || 0^8, so only byte 4 (= tag bits 0..4 << 3)
// differs between them.  Through rounds 1 and 2 that byte stays separable:
// after round 1 only column 1 depends on j, and it depends on nothing else but
// the key (x < 2^24, bytes 9, 14, 3 are key bytes); round 2's columns each take
// one S-box of that column plus three bytes that do not depend on j.  So the
// state after round 2 is W(j) ^ U(m, x): W is a function of the key alone
// (computed once per workgroup, kept as 128 planes in LDS), U is one T-table
// evaluation per lane and chunk (j = 0).  Rounds 3..8 are bitsliced in full,
// round 9 only for the two output bytes the PRF keeps (offsets are
// PRF & (CS-1), CS <= 2^15), round 10 two S-boxes.
//
// S-box: Boyar-Peralta's 113-gate circuit (32 AND, 77 XOR, 4 XNOR), the XNORs
// as XORs: it then computes S(x) ^ 0x63.  AddRoundKey is folded into the
// S-box outputs: MC(SR(S ^ k')) = MC(SR(S)) ^ rk for k' = SR^-1(MC^-1(rk)), so
// round r adds k'_r ^ 0x63 per byte at the S-box output (wave-uniform planes
// from SGPRs, one v_xor3 operand), and MixColumns is pure XOR.
// Checked against AES-NI / OpenSSL through the T-table kernel bit for bit
// (tools/aes_bs_bench.hip, tests/test_gpu_parity.py::test_prep_offsets_bs*).
#pragma once
#include "pm_aes.h"

namespace pm {

// 0 or ~0: bit b of a wave-uniform byte (SALU when k is uniform)
__device__ __forceinline__ uint32_t bs_kp(uint32_t k, int b) { return (uint32_t)((int32_t)(k << (31 - b)) >> 31); }

// three-input forms (v_bitop3_b32; LUT = f(S0 = 0xf0, S1 = 0xcc, S2 = 0xaa))
__device__ __forceinline__ uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // a ^ b ^ c
}
__device__ __forceinline__ uint32_t bs_ax(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x6a);   // (a & b) ^ c
}

// S(x) ^ 0x63 ^ k on 8 planes (p[b] = bit b, LSB first): Boyar-Peralta's
// circuit with every AND that feeds one XOR fused into it ((a & b) ^ c) and
// XOR pairs merged into three-input XORs: 85 VALU instead of 113 gates, the
// round constant k (wave-uniform) riding in the output XORs.
#ifndef PM_BS_KMODE
#define PM_BS_KMODE 0   // round constants: 0 = planes made on the SALU from the byte (s_bfe), 1 = planes read
                        // from LDS (precomputed per workgroup), 2 = none (timing experiment only: wrong output)
#endif
// The constant byte as the S-box consumes it: plane b of q[b]'s constant is bit b
// of bs_kk(k) (q[3] = tc14 ^ q[4] needs k3 ^ k4, q[6] = q[4] ^ tc16 needs k6 ^ k4).
__device__ __host__ __forceinline__ uint32_t bs_kk(uint32_t k) {
  return k ^ ((k >> 1) & 0x08u) ^ ((k << 2) & 0x40u);
}
struct BsK { uint32_t v[8]; };
__device__ __forceinline__ BsK bs_kplanes(uint32_t kk) {
  BsK r;
#pragma unroll
  for (int b = 0; b < 8; ++b) r.v[b] = PM_BS_KMODE == 2 ? 0u : bs_kp(kk, b);
  return r;
}
__device__ __forceinline__ void bs_sbox(const uint32_t (&p)[8], uint32_t (&q)[8], const BsK& K) {
  const uint32_t U0 = p[7], U1 = p[6], U2 = p[5], U3 = p[4], U4 = p[3], U5 = p[2], U6 = p[1], U7 = p[0];
  // top linear layer (22)
  const uint32_t t0 = U1 ^ U2, y14 = U3 ^ U5, y13 = U0 ^ U6, y9 = U0 ^ U3, y8 = U0 ^ U5;
  const uint32_t y1 = t0 ^ U7, y4 = y1 ^ U3, y12 = y13 ^ y14, y2 = y1 ^ U0, y5 = y1 ^ U6, y3 = y5 ^ y8;
  const uint32_t y15 = bs_x3(y13, U3, U4), y20 = bs_x3(y15, U1, U5), y6 = y15 ^ U7, y10 = y15 ^ t0;
  const uint32_t y11 = y20 ^ y9, y7 = U7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8, y16 = t0 ^ y11;
  const uint32_t y21 = y13 ^ y16, y18 = U0 ^ y16;
  // middle, GF(2^4) inversion (29)
  const uint32_t t2 = y12 & y15, t4 = bs_ax(y3, y6, t2), t6 = bs_ax(y4, U7, t2);
  const uint32_t t7 = y13 & y16, t9 = bs_ax(y5, y1, t7), t11 = bs_ax(y2, y7, t7);
  const uint32_t t12 = y9 & y11, t14 = bs_ax(y14, y17, t12), t16 = bs_ax(y8, y10, t12);
  const uint32_t t21 = bs_x3(t4, t14, y20), t22 = bs_x3(t6, t16, y19);
  const uint32_t t23 = bs_x3(t9, t14, y21), t24 = bs_x3(t11, t16, y18);
  const uint32_t t25 = t21 ^ t22, t27 = bs_ax(t21, t23, t24), t31 = bs_ax(t21, t23, t22);
  const uint32_t t29 = bs_ax(t25, t27, t22), t30 = t23 ^ t24, t33 = bs_ax(t31, t30, t24);
  const uint32_t t34 = t23 ^ t33, t35 = t27 ^ t33, t37 = bs_ax(t24, t35, t34), t38 = bs_ax(t24, t35, t27);
  const uint32_t t40 = bs_ax(t29, t38, t25), t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40;
  const uint32_t t44 = t33 ^ t37, t45 = t42 ^ t41;
  // bottom linear layer with the 18 output ANDs folded in (34)
  const uint32_t z16 = t45 & y14, tc1 = bs_ax(t42, y9, z16), tc2 = bs_ax(t37, y3, tc1), tc3 = bs_ax(t44, y12, tc2);
  const uint32_t z0 = t44 & y15, z2 = t33 & U7, tc4 = z0 ^ z2, tc5 = bs_ax(t37, y6, z0);
  const uint32_t z4 = t40 & y1, tc6 = bs_ax(t43, y16, z4), z5 = t29 & y7, tc12 = bs_ax(t43, y16, z5);
  const uint32_t tc7 = bs_ax(t43, y13, tc4), tc8 = bs_ax(t45, y17, tc6), tc9 = bs_ax(t41, y10, tc7);
  const uint32_t tc10 = tc8 ^ tc9, tc11 = tc6 ^ tc5, tc13 = bs_ax(t40, y5, tc1), tc14 = tc4 ^ tc12;
  const uint32_t tc16 = bs_ax(t42, y11, tc8), tc17 = bs_ax(t29, y2, tc10), tc18 = tc13 ^ tc14;
  const uint32_t tc20 = bs_ax(t42, y9, tc16), tc21 = bs_ax(t33, y4, tc2);
  const uint32_t s3 = bs_x3(tc3, tc11, K.v[4]);                   // S3 ^ k4
  q[4] = s3;
  q[3] = bs_x3(tc14, s3, K.v[3]);                                  // S4 = tc14 ^ S3 (constant k3 ^ k4)
  q[6] = bs_x3(s3, tc16, K.v[6]);                                  // S1 = S3 ^ tc16 (constant k6 ^ k4)
  q[7] = bs_x3(tc3, tc16, K.v[7]);                                 // S0
  q[5] = bs_ax(t41, y8, bs_x3(tc17, tc20, K.v[5]));                // S2 = tc17 ^ tc20 ^ z17
  q[2] = bs_x3(tc21, tc17, K.v[2]);                                // S5
  q[1] = bs_x3(tc10, tc18, K.v[1]);                                // S6
  q[0] = bs_ax(t43, y13, tc18 ^ K.v[0]);                           // S7 = z12 ^ tc18
}

// MixColumns row i of column a[0..3] (8 planes each) into o:
// 2 (a_i ^ a_{i+1}) ^ a_{i+1} ^ (a_{i+2} ^ a_{i+3})
__device__ __forceinline__ void bs_mc_row(const uint32_t (&ai)[8], const uint32_t (&a1)[8], const uint32_t (&a2)[8],
                                          const uint32_t (&a3)[8], uint32_t (&o)[8]) {
  uint32_t d[8], e[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) { d[b] = ai[b] ^ a1[b]; e[b] = a2[b] ^ a3[b]; }
  o[0] = bs_x3(d[7], a1[0], e[0]);
  o[1] = bs_x3(d[0] ^ d[7], a1[1], e[1]);
  o[2] = bs_x3(d[1], a1[2], e[2]);
  o[3] = bs_x3(d[2] ^ d[7], a1[3], e[3]);
  o[4] = bs_x3(d[3] ^ d[7], a1[4], e[4]);
  o[5] = bs_x3(d[4], a1[5], e[5]);
  o[6] = bs_x3(d[5], a1[6], e[6]);
  o[7] = bs_x3(d[6], a1[7], e[7]);
}

// One full round on the state (S-box with the round's folded key, ShiftRows,
// MixColumns).  kw: the round's 16 constant bytes (k'_r ^ 0x63) as 4 words,
// byte p = 4 col + row, wave-uniform.
__device__ __forceinline__ BsK bs_kload(const uint32_t* kpl) {   // 8 planes from LDS (broadcast reads)
  const uint4 a = *reinterpret_cast<const uint4*>(kpl), b = *reinterpret_cast<const uint4*>(kpl + 4);
  return BsK{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}
__device__ __forceinline__ void bs_round(uint32_t (&s)[16][8], const uint32_t (&kw)[4], const uint32_t* kpl) {
  uint32_t t[16][8];
#pragma unroll
  for (int p = 0; p < 16; ++p)
    bs_sbox(s[p], t[p], PM_BS_KMODE == 1 ? bs_kload(kpl + 8 * p) : bs_kplanes((kw[p >> 2] >> (8 * (p & 3))) & 0xffu));
  // column c after ShiftRows: row r from byte 4 ((c + r) & 3) + r
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int p0 = 4 * c, p1 = 4 * ((c + 1) & 3) + 1, p2 = 4 * ((c + 2) & 3) + 2, p3 = 4 * ((c + 3) & 3) + 3;
    uint32_t d01[8], d12[8], d23[8], d30[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      d01[b] = t[p0][b] ^ t[p1][b]; d12[b] = t[p1][b] ^ t[p2][b];
      d23[b] = t[p2][b] ^ t[p3][b]; d30[b] = t[p3][b] ^ t[p0][b];
    }
    // row i: xtime(d_i) ^ a_{i+1} ^ d_{i+2}
    auto row = [&](const uint32_t (&di)[8], const uint32_t (&an)[8], const uint32_t (&dn)[8], uint32_t (&o)[8]) {
      o[0] = bs_x3(di[7], an[0], dn[0]);
      o[1] = bs_x3(di[0] ^ di[7], an[1], dn[1]);
      o[2] = bs_x3(di[1], an[2], dn[2]);
      o[3] = bs_x3(di[2] ^ di[7], an[3], dn[3]);
      o[4] = bs_x3(di[3] ^ di[7], an[4], dn[4]);
      o[5] = bs_x3(di[4], an[5], dn[5]);
      o[6] = bs_x3(di[5], an[6], dn[6]);
      o[7] = bs_x3(di[6], an[7], dn[7]);
    };
    row(d01, t[p1], d23, s[4 * c + 0]);
    row(d12, t[p2], d30, s[4 * c + 1]);
    row(d23, t[p3], d01, s[4 * c + 2]);
    row(d30, t[p0], d12, s[4 * c + 3]);
  }
}

// Rounds 1-2 of one block by T-table (te0: the 256-word Te0 in LDS), the
// state after round 2 as four LE column words.
__device__ __forceinline__ uint32_t bs_te(const uint32_t* te0, uint32_t s, int k) {
  return te0[(s >> (8 * k)) & 0xffu];
}
__device__ __forceinline__ void bs_r12(const uint32_t* te0, const uint32_t* __restrict__ rk, uint32_t w0, uint32_t w1,
                                       uint32_t (&u)[4]) {
  uint32_t s0 = w0 ^ rk[0], s1 = w1 ^ rk[1], s2 = rk[2], s3 = rk[3];
#pragma unroll
  for (int r = 1; r <= 2; ++r) {
    const uint32_t t0 = bs_te(te0, s0, 0) ^ rotl32(bs_te(te0, s1, 1), 8) ^ rotl32(bs_te(te0, s2, 2), 16) ^
                        rotl32(bs_te(te0, s3, 3), 24) ^ rk[4 * r + 0];
    const uint32_t t1 = bs_te(te0, s1, 0) ^ rotl32(bs_te(te0, s2, 1), 8) ^ rotl32(bs_te(te0, s3, 2), 16) ^
                        rotl32(bs_te(te0, s0, 3), 24) ^ rk[4 * r + 1];
    const uint32_t t2 = bs_te(te0, s2, 0) ^ rotl32(bs_te(te0, s3, 1), 8) ^ rotl32(bs_te(te0, s0, 2), 16) ^
                        rotl32(bs_te(te0, s1, 3), 24) ^ rk[4 * r + 2];
    const uint32_t t3 = bs_te(te0, s3, 0) ^ rotl32(bs_te(te0, s0, 1), 8) ^ rotl32(bs_te(te0, s1, 2), 16) ^
                        rotl32(bs_te(te0, s2, 3), 24) ^ rk[4 * r + 3];
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  u[0] = s0; u[1] = s1; u[2] = s2; u[3] = s3;
}

__device__ __forceinline__ uint32_t bs_gmul2(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1bu : 0u)) & 0xffu; }
__device__ __forceinline__ uint32_t bs_gmul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 4; ++i) {
    if (b & 1u) p ^= a;
    a = bs_gmul2(a);
    b >>= 1;
  }
  return p;
}

// Per-key setup of one workgroup (call with >= 128 threads, then the caller
// synchronises):
//   kx[4 (r-3) + w], r = 3..9: the S-box output constants of round r
//       (bs_kk of SR^-1 MC^-1 rk_r ^ 0x63), byte p = 4 w + row;
//   kx[28], kx[29]: round 10's bytes 0 and 5 (rk10 bytes 0 and 1 ^ 0x63);
//   wv[j][4]: round-2 state of tag j at chunk 0 (its XOR with j = 0's is W(j)).
__device__ __forceinline__ void bs_setup_a(const uint32_t* te0, const uint32_t* __restrict__ rk, uint32_t* kx,
                                           uint32_t (*wv)[4]) {
  const uint32_t t = threadIdx.x;
  if (t < 28) {
    const uint32_t r = 3 + t / 4, w = t & 3;
    uint32_t word = 0;
#pragma unroll
    for (uint32_t row = 0; row < 4; ++row) {
      const uint32_t c = (w + 4 - row) & 3;   // k' at (col w, row) = MC^-1(rk_r col c)[row], c = w - row
      const uint32_t kc = rk[4 * r + c];
      const uint32_t a0 = kc & 0xffu, a1 = (kc >> 8) & 0xffu, a2 = (kc >> 16) & 0xffu, a3 = kc >> 24;
      const uint32_t m0 = row == 0 ? 14u : row == 1 ? 9u : row == 2 ? 13u : 11u;
      const uint32_t m1 = row == 0 ? 11u : row == 1 ? 14u : row == 2 ? 9u : 13u;
      const uint32_t m2 = row == 0 ? 13u : row == 1 ? 11u : row == 2 ? 14u : 9u;
      const uint32_t m3 = row == 0 ? 9u : row == 1 ? 13u : row == 2 ? 11u : 14u;
      const uint32_t v = bs_gmul(a0, m0) ^ bs_gmul(a1, m1) ^ bs_gmul(a2, m2) ^ bs_gmul(a3, m3);
      word |= bs_kk(v ^ 0x63u) << (8 * row);
    }
    kx[t] = word;
  } else if (t == 28) {
    kx[28] = (rk[40] & 0xffu) ^ 0x63u;
    kx[29] = ((rk[40] >> 8) & 0xffu) ^ 0x63u;
  } else if (t >= 64 && t < 96) {
    uint32_t u[4];
    bs_r12(te0, rk, 0u, (t - 64) << 3, u);
    wv[t - 64][0] = u[0]; wv[t - 64][1] = u[1]; wv[t - 64][2] = u[2]; wv[t - 64][3] = u[3];
  }
}
// wp[8 p + b] = the plane (byte p, bit b) of W(j) = wv[j] ^ wv[0];
// PM_BS_KMODE 1: kpl[128 (r-3) + 8 p + b] = plane b of round r's constant byte p
constexpr int kBsKplWords = PM_BS_KMODE == 1 ? 7 * 128 : 1;
__device__ __forceinline__ void bs_setup_b(const uint32_t (*wv)[4], uint32_t* wp, const uint32_t* kx, uint32_t* kpl) {
  const uint32_t t = threadIdx.x;
  if (PM_BS_KMODE == 1)
    for (uint32_t i = t; i < 7 * 128; i += blockDim.x) {
      const uint32_t r = i >> 7, p = (i >> 3) & 15, b = i & 7;
      kpl[i] = bs_kp((kx[4 * r + (p >> 2)] >> (8 * (p & 3))) & 0xffu, b);
    }
  if (t < 128) {
    const uint32_t p = t >> 3, b = t & 7, sh = 8 * (p & 3) + b, w = p >> 2;
    const uint32_t z = (wv[0][w] >> sh) & 1u;
    uint32_t pl = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < 32; ++j) pl |= (((wv[j][w] >> sh) & 1u) ^ z) << j;
    wp[t] = pl;
  }
}

// 16 PRF-output planes (bits 0..15 of PRF(32 m + j, x) ^ ...): lo16 of the PRF
// for the lane's 32 tags at chunk x.  kx / wp from the setup (LDS).
__device__ __forceinline__ void bs_prf16(const uint32_t* te0, const uint32_t* __restrict__ rk, const uint32_t* kx,
                                         const uint32_t* wp, const uint32_t* kpl, uint32_t m, uint32_t x,
                                         uint32_t (&o)[16]) {
  // keep the W planes' LDS reads inside the caller's loop (hoisted, they would
  // pin 128 VGPRs for the whole kernel)
  asm volatile("" ::: "memory");
  uint32_t u[4];
  bs_r12(te0, rk, x, m << 8, u);   // tag 32 m: w1 = 32 m << 3
  uint32_t s[16][8];
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const uint4 w0 = *reinterpret_cast<const uint4*>(wp + 8 * p), w1 = *reinterpret_cast<const uint4*>(wp + 8 * p + 4);
    const uint32_t wl[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int b = 0; b < 8; ++b) s[p][b] = wl[b] ^ (uint32_t)((int32_t)(u[p >> 2] << (31 - (8 * (p & 3) + b))) >> 31);
  }
#pragma unroll 1
  for (int r = 0; r < 6; ++r) {   // rounds 3..8
    uint32_t kw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) kw[i] = __builtin_amdgcn_readfirstlane(kx[4 * r + i]);
    bs_round(s, kw, kpl + 128 * r);
  }
  // round 9: the S-boxes of columns 0 and 1 after ShiftRows, MixColumns rows 0 / 1
  uint32_t kw9[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) kw9[i] = __builtin_amdgcn_readfirstlane(kx[24 + i]);
  auto kb = [&](int p) {
    return PM_BS_KMODE == 1 ? bs_kload(kpl + 6 * 128 + 8 * p) : bs_kplanes((kw9[p >> 2] >> (8 * (p & 3))) & 0xffu);
  };
  uint32_t a0[8], a1[8], a2[8], a3[8], u00[8], u11[8];
  bs_sbox(s[0], a0, kb(0)); bs_sbox(s[5], a1, kb(5)); bs_sbox(s[10], a2, kb(10)); bs_sbox(s[15], a3, kb(15));
  bs_mc_row(a0, a1, a2, a3, u00);   // column 0 row 0
  bs_sbox(s[4], a0, kb(4)); bs_sbox(s[9], a1, kb(9)); bs_sbox(s[14], a2, kb(14)); bs_sbox(s[3], a3, kb(3));
  bs_mc_row(a1, a2, a3, a0, u11);   // column 1 row 1
  // round 10 (no MixColumns): output bytes 0 and 1, with B's bytes 0 and 1 (x) folded in
  const uint32_t k10a = __builtin_amdgcn_readfirstlane(kx[28]) ^ (x & 0xffu);
  const uint32_t k10b = __builtin_amdgcn_readfirstlane(kx[29]) ^ ((x >> 8) & 0xffu);
  uint32_t lo[8], hi[8];
  bs_sbox(u00, lo, bs_kplanes(bs_kk(k10a)));
  bs_sbox(u11, hi, bs_kplanes(bs_kk(k10b)));
#pragma unroll
  for (int b = 0; b < 8; ++b) { o[b] = lo[b]; o[8 + b] = hi[b]; }
}

// 32 x 32 bit transpose: a[i] bit j -> a[j] bit i.
__device__ __forceinline__ void bs_transpose32(uint32_t (&a)[32]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {   // 16-bit blocks: one v_perm each
    const uint32_t x = a[i], y = a[i + 16];
    a[i] = __builtin_amdgcn_perm(y, x, 0x05040100u);        // lo(x) | lo(y) << 16
    a[i + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);   // hi(x) | hi(y) << 16
  }
#pragma unroll
  for (int g = 0; g < 32; g += 16)
#pragma unroll
    for (int i = g; i < g + 8; ++i) {   // bytes
      const uint32_t x = a[i], y = a[i + 8];
      a[i] = __builtin_amdgcn_perm(y, x, 0x06020400u);       // x.b0, y.b0, x.b2, y.b2
      a[i + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);   // x.b1, y.b1, x.b3, y.b3
    }
  auto stage = [&](int s, uint32_t m) {
#pragma unroll
    for (int g = 0; g < 32; g += 2 * s)
#pragma unroll
      for (int i = g; i < g + s; ++i) {
        const uint32_t t = ((a[i] >> s) ^ a[i + s]) & m;
        a[i + s] ^= t;
        a[i] ^= t << s;
      }
  };
  stage(4, 0x0f0f0f0fu);
  stage(2, 0x33333333u);
  stage(1, 0x55555555u);
}


}  // namespace pm
