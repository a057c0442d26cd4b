// pm_oracle.cpp — TEST INFRASTRUCTURE ONLY (see pm_oracle.h header).
//
// CPU restatement of the reference hot path.  Single-threaded where the
// reference is (batch-pir.go:16 ThreadNum = 1).  AES-128-MMO uses AES-NI the
// way pianopir/aes_amd64.s does; xorSlices / L2DistanceSIMD / InnerProduct use
// the same AVX2 / AVX / AVX-512 lane structure as the Go assembly.
//
// Build: oracle/Makefile (g++ -O2 -maes -mavx2 -ffp-contract=off).
#include "pm_oracle.h"

#include <immintrin.h>
#include <wmmintrin.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

// ---------------------------------------------------------------------------
// Randomness seams.  Replace the reference's time-seeded
// math/rand sources: pir.go:132,208,305 (keys / replacement offsets),
// pir.go:366 (dummy offsets), private-search.go:517 / search.go:158 (ids).
// ---------------------------------------------------------------------------
static inline uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
extern "C" uint64_t or_hash4(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = sm64(seed + dom);
  h = sm64(h ^ a);
  h = sm64(h ^ b);
  h = sm64(h ^ c);
  return h;
}
enum : uint64_t { DOM_KEY = 1, DOM_REPL = 2, DOM_DUMMY = 3 };

struct SplitMix {  // the host-side "global rand" stream
  uint64_t s;
  uint64_t next() { s += 0x9e3779b97f4a7c15ULL; uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL; z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31); }
  uint64_t intn(uint64_t n) { return next() % n; }
};

// ---------------------------------------------------------------------------
// AES-128 (aes_amd64.s:87-126 expandKeyAsm, :51-82 aes128MMO)
// ---------------------------------------------------------------------------
static inline __m128i key_assist(__m128i k, __m128i t) {
  t = _mm_shuffle_epi32(t, 0xff);          // PSHUFD $0xff
  __m128i s = _mm_slli_si128(k, 4); k = _mm_xor_si128(k, s);
  s = _mm_slli_si128(s, 4); k = _mm_xor_si128(k, s);
  s = _mm_slli_si128(s, 4); k = _mm_xor_si128(k, s);
  return _mm_xor_si128(k, t);
}
extern "C" void or_expand_key(const uint8_t key[16], uint32_t rk[44]) {
  __m128i k = _mm_loadu_si128((const __m128i*)key);
  __m128i* o = (__m128i*)rk;
  _mm_storeu_si128(o + 0, k);
#define STEP(i, rc) k = key_assist(k, _mm_aeskeygenassist_si128(k, rc)); _mm_storeu_si128(o + i, k);
  STEP(1, 0x01) STEP(2, 0x02) STEP(3, 0x04) STEP(4, 0x08) STEP(5, 0x10)
  STEP(6, 0x20) STEP(7, 0x40) STEP(8, 0x80) STEP(9, 0x1b) STEP(10, 0x36)
#undef STEP
}
static inline __m128i aes_enc(const uint32_t rk[44], __m128i x) {
  const __m128i* k = (const __m128i*)rk;
  x = _mm_xor_si128(x, _mm_loadu_si128(k));
  for (int r = 1; r < 10; ++r) x = _mm_aesenc_si128(x, _mm_loadu_si128(k + r));
  return _mm_aesenclast_si128(x, _mm_loadu_si128(k + 10));
}
extern "C" void or_aes128_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  _mm_storeu_si128((__m128i*)out, aes_enc(rk, _mm_loadu_si128((const __m128i*)in)));
}
// PRFEvalWithLongKeyAndTag (util.go:157-165): block = LE64((tag<<35)+x) || 0^8,
// out = low64_LE(AES_k(block) ^ block)  (aes128MMO's final PXOR, aes_amd64.s:79-80).
static inline uint64_t prf(const uint32_t* rk, uint64_t tag, uint64_t x) {
  __m128i b = _mm_set_epi64x(0, (long long)((tag << 35) + x));
  __m128i c = _mm_xor_si128(aes_enc(rk, b), b);
  return (uint64_t)_mm_cvtsi128_si64(c);
}
extern "C" uint64_t or_prf(const uint32_t rk[44], uint64_t tag, uint64_t x) { return prf(rk, tag, x); }
extern "C" void or_prf_batch(const uint32_t rk[44], const uint64_t* t, const uint64_t* x, size_t n,
                             uint64_t* out) {
  for (size_t i = 0; i < n; ++i) out[i] = prf(rk, t[i], x[i]);
}
// RandKey128 (util.go:25-31): key bytes = LE64(r1) || LE64(r2)
extern "C" void or_derive_key(uint64_t seed, uint64_t partition, uint64_t epoch, uint8_t key[16]) {
  uint64_t r1 = or_hash4(seed, DOM_KEY, partition, epoch, 0);
  uint64_t r2 = or_hash4(seed, DOM_KEY, partition, epoch, 1);
  memcpy(key, &r1, 8); memcpy(key + 8, &r2, 8);
}

// xorSlices (aes_amd64.s:133-157): count comes from len(src), 4 words per step.
static inline void xor_slices(uint64_t* dst, const uint64_t* src, size_t src_len) {
  size_t groups = src_len >> 2;
  for (size_t g = 0; g < groups; ++g) {
    __m256i a = _mm256_loadu_si256((const __m256i*)(dst + 4 * g));
    __m256i b = _mm256_loadu_si256((const __m256i*)(src + 4 * g));
    _mm256_storeu_si256((__m256i*)(dst + 4 * g), _mm256_xor_si256(a, b));
  }
}
extern "C" void or_xor_slices(uint64_t* dst, const uint64_t* src, size_t n) { xor_slices(dst, src, n); }

// ---------------------------------------------------------------------------
// Distance (l2_distance_amd64.s:4-36, build_graph.go:119-134)
// ---------------------------------------------------------------------------
// L2DistanceSIMD: 8 running sums (VSUBPS, VMULPS, VADDPS separately rounded),
// do-while over 8-float groups, then VEXTRACTF128 + 3x VHADDPS.
extern "C" float or_l2dist_avx(const float* a, const float* b, size_t n) {
  __m256 acc = _mm256_setzero_ps();
  size_t dx = 0;
  do {
    __m256 d = _mm256_sub_ps(_mm256_loadu_ps(a + dx), _mm256_loadu_ps(b + dx));
    acc = _mm256_add_ps(acc, _mm256_mul_ps(d, d));
    dx += 8;
  } while (dx < n);
  __m128 lo = _mm256_castps256_ps128(acc), hi = _mm256_extractf128_ps(acc, 1);
  __m128 x = _mm_hadd_ps(lo, hi);   // VHADDPS X1, X0, X0
  x = _mm_hadd_ps(x, x);
  x = _mm_hadd_ps(x, x);
  return _mm_cvtss_f32(x);
}
static float l2_simd_scalar(const float* a, const float* b, size_t n) {
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t dx = 0;
  do {
    for (int k = 0; k < 8; ++k) { float d = a[dx + k] - b[dx + k]; float p = d * d; s[k] = s[k] + p; }
    dx += 8;
  } while (dx < n);
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}
// L2Dist (build_graph.go:119-127): SIMD on the multiple-of-8 prefix, scalar tail.
extern "C" float or_l2dist(const float* a, const float* b, size_t dim) {
  size_t rem = dim & 7;
  float d = (dim - rem) ? l2_simd_scalar(a, b, dim - rem) : 0.0f;  // Go panics at dim<8
  for (size_t i = dim - rem; i < dim; ++i) { float t = a[i] - b[i]; float p = t * t; d = d + p; }
  return d;
}
extern "C" void or_l2_batch(const float* q, const float* rows, size_t nrows, size_t dim, float* out) {
  for (size_t r = 0; r < nrows; ++r) out[r] = or_l2dist(rows + r * dim, q, dim);
}
// InnerProduct (l2_distance_amd64.s:39-68): sum a_i*b_i mod 2^32 (VPMULLD/VPADDD).
// Wrapping add is associative, so the lane order cannot change the result.
extern "C" uint32_t or_inner_product(const uint32_t* a, const uint32_t* b, size_t n) {
  __m256i acc = _mm256_setzero_si256();
  size_t i = 0;
  for (; i + 8 <= n; i += 8)
    acc = _mm256_add_epi32(acc, _mm256_mullo_epi32(_mm256_loadu_si256((const __m256i*)(a + i)),
                                                    _mm256_loadu_si256((const __m256i*)(b + i))));
  uint32_t l[8]; _mm256_storeu_si256((__m256i*)l, acc);
  uint32_t s = 0; for (int k = 0; k < 8; ++k) s += l[k];
  for (; i < n; ++i) s += a[i] * b[i];
  return s;
}
// TestInnerProduct (graphann_test.go:249-283) with the fill generated per row
// in cache (the reference materialises 51.2 GB; the per-row arithmetic is the same).
extern "C" uint32_t or_inner_product_bench(uint64_t N, uint64_t D, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  std::vector<uint32_t> q(D);
  for (uint64_t j = 0; j < D; ++j) q[j] = (uint32_t)j;
  std::vector<uint32_t> part(nthreads, 0);
  auto work = [&](int t) {
    std::vector<uint32_t> row(D);
    uint64_t lo = N * t / nthreads, hi = N * (t + 1) / nthreads;
    uint32_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) {
      for (uint64_t j = 0; j < D; ++j) row[j] = (uint32_t)(i + j);
      s += or_inner_product(row.data(), q.data(), D);
    }
    part[t] = s;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  uint32_t s = 0; for (auto v : part) s += v;
  return s;
}

// The benchmark's scan over materialised rows (graphann_test.go:249-283: the
// N x D array is allocated and filled first, then InnerProduct runs row by
// row), split over nthreads contiguous row ranges; sums wrap mod 2^32.
extern "C" uint32_t or_inner_product_scan(const uint32_t* rows, const uint32_t* q, uint64_t N, uint64_t D,
                                          int nthreads) {
  if (nthreads < 1) nthreads = 1;
  std::vector<uint32_t> part(nthreads, 0);
  auto work = [&](int t) {
    uint64_t lo = N * t / nthreads, hi = N * (t + 1) / nthreads;
    uint32_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += or_inner_product(rows + i * D, q, D);
    part[t] = s;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  uint32_t s = 0; for (auto v : part) s += v;
  return s;
}

// ---------------------------------------------------------------------------
// PianoPIR (pianopir/pir.go)
// ---------------------------------------------------------------------------
static const uint64_t kDefaultProgramPoint = 0x7fffffff;  // pir.go:15

struct or_pir {
  // PianoPIRConfig (pir.go:18-26)
  uint64_t E_bytes, E, N, CS, SS, ThreadNum, F;
  const uint64_t* rawDB;   // alias, like PianoPIRServer.rawDB (pir.go:28-31)
  // client (pir.go:91-121)
  uint64_t seed, partition, epoch = 0;
  bool skipPrep = false;
  uint32_t rk[44];
  uint64_t MaxQ, FQN = 0, Qpc, PH;
  std::vector<uint64_t> hist, ptag, parity, pp, btag, bparity, ridx, rval;
  std::unordered_map<uint64_t, std::vector<uint64_t>> cache;
  uint64_t dummy_ctr = 0;
};

// NewPianoPIR (pir.go:479-514) + NewPianoPIRClient (pir.go:130-175)
extern "C" or_pir* or_pir_new(uint64_t DBSize, uint64_t DBEntryByteNum, const uint64_t* rawDB,
                              uint64_t F, uint64_t seed, uint64_t partition) {
  or_pir* p = new or_pir();
  p->E_bytes = DBEntryByteNum; p->E = DBEntryByteNum / 8; p->N = DBSize;
  uint64_t target = (uint64_t)(2 * std::sqrt((double)DBSize));
  uint64_t cs = 1; while (cs < target) cs *= 2;
  p->CS = cs;
  uint64_t ss = (uint64_t)std::ceil((double)DBSize / (double)cs);
  p->SS = (ss + 3) / 4 * 4;
  p->ThreadNum = 8; p->F = F; p->rawDB = rawDB;
  p->seed = seed; p->partition = partition;
  p->MaxQ = (uint64_t)(std::sqrt((double)DBSize) * std::log((double)DBSize));
  uint64_t k = (uint64_t)std::ceil(std::log(2.0) * (double)(F + 1));   // primaryNumParam :124-127
  uint64_t ph = k * cs;
  p->PH = (ph + p->ThreadNum - 1) / p->ThreadNum * p->ThreadNum;
  uint64_t qpc = 3 * (uint64_t)((double)p->MaxQ / (double)p->SS);
  p->Qpc = (qpc + p->ThreadNum - 1) / p->ThreadNum * p->ThreadNum;
  p->hist.assign(p->SS, 0);
  return p;
}
extern "C" void or_pir_free(or_pir* p) { delete p; }

// Initialization (pir.go:203-255)
static void initialization(or_pir* c) {
  c->FQN = 0;
  uint8_t key[16];
  or_derive_key(c->seed, c->partition, c->epoch, key);
  c->epoch++;
  or_expand_key(key, c->rk);
  c->hist.assign(c->SS, 0);
  uint64_t tag = 0;
  c->ptag.resize(c->PH); c->parity.assign(c->PH * c->E, 0); c->pp.resize(c->PH);
  for (uint64_t i = 0; i < c->PH; ++i) { c->ptag[i] = tag++; c->pp[i] = kDefaultProgramPoint; }
  uint64_t nb = c->SS * c->Qpc;
  c->ridx.resize(nb); c->rval.assign(nb * c->E, 0); c->btag.resize(nb); c->bparity.assign(nb * c->E, 0);
  for (uint64_t i = 0; i < c->SS; ++i)
    for (uint64_t j = 0; j < c->Qpc; ++j) {
      c->ridx[i * c->Qpc + j] = kDefaultProgramPoint;
      c->btag[i * c->Qpc + j] = tag++;
    }
  c->cache.clear();
}

// UpdatePreprocessing (pir.go:303-352), split in two: the hint fold of one
// chunk restricted to hint indices [h0, h1) of the concatenated space
// (primary hints 0..PH-1, then backup hint (g, j) at PH + g*Qpc + j), and the
// replacement rows of that chunk.  Every hint's parity is its own XOR chain in
// chunk order, so splitting the hint space over threads (the reference's
// "TODO: using multiple threads", pir.go:282) gives bit-identical state.
static void fold_chunk(or_pir* c, uint64_t chunkId, const uint64_t* chunk, uint64_t h0, uint64_t h1) {
  const uint64_t E = c->E, mask = c->CS - 1;
  for (uint64_t i = h0; i < std::min(h1, c->PH); ++i) {
    uint64_t off = prf(c->rk, c->ptag[i], chunkId) & mask;
    xor_slices(&c->parity[i * E], chunk + off * E, E);
  }
  const uint64_t b0 = h0 > c->PH ? h0 - c->PH : 0, b1 = h1 > c->PH ? h1 - c->PH : 0;
  for (uint64_t h = b0; h < b1; ++h) {
    const uint64_t g = h / c->Qpc;
    if (g == chunkId) continue;   // backup hints skip their own chunk
    uint64_t off = prf(c->rk, c->btag[h], chunkId) & mask;
    xor_slices(&c->bparity[h * E], chunk + off * E, E);
  }
}
static void replacement_rows(or_pir* c, uint64_t chunkId, const uint64_t* chunk) {
  const uint64_t E = c->E, mask = c->CS - 1;
  for (uint64_t j = 0; j < c->Qpc; ++j) {
    uint64_t off = or_hash4(c->seed, DOM_REPL, c->partition, c->epoch - 1, chunkId * c->Qpc + j) & mask;
    c->ridx[chunkId * c->Qpc + j] = off + chunkId * c->CS;
    memcpy(&c->rval[(chunkId * c->Qpc + j) * E], chunk + off * E, E * 8);
  }
}

static int g_prep_threads = 1;   // 1: the reference's single-threaded loop (batch-pir.go:16)
extern "C" void or_set_prep_threads(int n) { g_prep_threads = n < 1 ? 1 : n; }

// Preprocessing (pir.go:267-301)
static void client_preprocessing(or_pir* c) {
  initialization(c);
  if (c->skipPrep) return;
  const uint64_t E = c->E, len = c->N * E, H = c->PH + c->SS * c->Qpc;
  // chunk i, zero-padded past the end of the DB (pir.go:285-295)
  std::vector<uint64_t> tail;
  auto chunk_ptr = [&](uint64_t i) -> const uint64_t* {
    uint64_t start = i * c->CS, end = (i + 1) * c->CS;
    if (end * E <= len) return c->rawDB + start * E;
    return tail.data() + (i - (len / E) / c->CS) * c->CS * E;
  };
  {   // every chunk that reaches past the end, padded once
    const uint64_t first = (len / E) / c->CS;
    if (first < c->SS) {
      tail.assign((c->SS - first) * c->CS * E, 0);
      for (uint64_t j = first * c->CS * E; j < len; ++j) tail[j - first * c->CS * E] = c->rawDB[j];
    }
  }
  const int T = (int)std::min<uint64_t>((uint64_t)g_prep_threads, std::max<uint64_t>(1, H / 64));
  auto work = [&](int t) {
    const uint64_t h0 = H * t / T, h1 = H * (t + 1) / T;
    for (uint64_t i = 0; i < c->SS; ++i) fold_chunk(c, i, chunk_ptr(i), h0, h1);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  for (uint64_t i = 0; i < c->SS; ++i) replacement_rows(c, i, chunk_ptr(i));
}

// PrivateQuery (pir.go:65-88)
static void private_query(const or_pir* s, const uint32_t* offsets, uint64_t* ret) {
  memset(ret, 0, s->E * 8);
  for (uint64_t i = 0; i < s->SS; ++i) {
    uint64_t idx = (uint64_t)offsets[i] + i * s->CS;
    if (idx >= s->N) continue;
    xor_slices(ret, s->rawDB + idx * s->E, s->E);
  }
}
extern "C" int or_server_private_query(or_pir* p, const uint32_t* offsets, uint64_t* out) {
  private_query(p, offsets, out); return 0;
}

// Client.Query (pir.go:354-471)
static int client_query(or_pir* c, uint64_t idx, bool real, uint64_t* out) {
  const uint64_t E = c->E, CS = c->CS, mask = CS - 1;
  memset(out, 0, E * 8);
  if (!real) {
    std::vector<uint32_t> offs(c->SS);
    uint64_t d = c->dummy_ctr++;
    for (uint64_t i = 0; i < c->SS; ++i)
      offs[i] = (uint32_t)(or_hash4(c->seed, DOM_DUMMY, c->partition, d, i) & mask);
    std::vector<uint64_t> junk(E);
    private_query(c, offs.data(), junk.data());
    return 0;
  }
  if (idx >= c->N) return 4;                      // log.Fatalf in the reference (:373-378)
  auto it = c->cache.find(idx);
  if (it != c->cache.end()) { memcpy(out, it->second.data(), E * 8); return 0; }
  if (c->FQN >= c->MaxQ) return 1;
  uint64_t chunkId = idx / CS, offset = idx % CS;
  if (c->hist[chunkId] >= c->Qpc) return 2;
  uint64_t hit = kDefaultProgramPoint;
  for (uint64_t i = 0; i < c->PH; ++i) {
    uint64_t ho = prf(c->rk, c->ptag[i], chunkId) & mask;
    if (ho == offset && (c->pp[i] == kDefaultProgramPoint || c->pp[i] / CS != chunkId)) { hit = i; break; }
  }
  if (hit == kDefaultProgramPoint) return 3;
  std::vector<uint64_t> qs(c->SS);
  for (uint64_t i = 0; i < c->SS; ++i) qs[i] = i * CS + (prf(c->rk, c->ptag[hit], i) & mask);
  if (c->pp[hit] != kDefaultProgramPoint) qs[c->pp[hit] / CS] = c->pp[hit];
  uint64_t g = c->hist[chunkId];
  uint64_t replIdx = c->ridx[chunkId * c->Qpc + g];
  const uint64_t* replVal = &c->rval[(chunkId * c->Qpc + g) * E];
  qs[chunkId] = replIdx;
  std::vector<uint32_t> offs(c->SS);
  for (uint64_t i = 0; i < c->SS; ++i) offs[i] = (uint32_t)(qs[i] & mask);
  std::vector<uint64_t> resp(E);
  private_query(c, offs.data(), resp.data());
  xor_slices(resp.data(), replVal, E);
  xor_slices(resp.data(), &c->parity[hit * E], E);
  // refresh (:460-468)
  c->ptag[hit] = c->btag[chunkId * c->Qpc + g];
  memcpy(&c->parity[hit * E], &c->bparity[(chunkId * c->Qpc + g) * E], E * 8);
  c->pp[hit] = idx;
  xor_slices(&c->parity[hit * E], resp.data(), E);
  c->FQN++;
  c->hist[chunkId]++;
  c->cache[idx] = resp;
  memcpy(out, resp.data(), E * 8);
  return 0;
}

extern "C" void or_pir_preprocessing(or_pir* p) { client_preprocessing(p); }     // pir.go:516-518
extern "C" void or_pir_dummy_preprocessing(or_pir* p) {                          // pir.go:520-523
  initialization(p); p->skipPrep = true;
}
// PianoPIR.Query (pir.go:525-533)
extern "C" int or_pir_query(or_pir* p, uint64_t idx, int real, uint64_t* out) {
  if (p->FQN == p->MaxQ) client_preprocessing(p);
  return client_query(p, idx, real != 0, out);
}
extern "C" void or_pir_config_get(const or_pir* p, or_pir_config* c) {
  c->DBEntryByteNum = p->E_bytes; c->DBEntrySize = p->E; c->DBSize = p->N; c->ChunkSize = p->CS;
  c->SetSize = p->SS; c->ThreadNum = p->ThreadNum; c->FailureProbLog2 = p->F;
  c->MaxQueryNum = p->MaxQ; c->PrimaryHintNum = p->PH; c->MaxQueryPerChunk = p->Qpc;
  c->FinishedQueryNum = p->FQN;
}
// LocalStorageSize (pir.go:178-190)
extern "C" double or_pir_local_storage(const or_pir* c) {
  double s = 0;
  s = s + (double)c->PH * 8;
  s = s + (double)c->PH * (double)c->E_bytes;
  s = s + (double)c->PH * 8;
  double tb = (double)c->SS * (double)c->Qpc;
  s = s + tb * 8;
  s = s + tb * (double)c->E_bytes;
  s = s + tb * 8;
  s = s + tb * (double)c->E_bytes;
  return s;
}
// CommCostPerQuery (pir.go:539-544)
extern "C" double or_pir_comm_per_query(const or_pir* p) { return (double)(p->SS * 4 + p->E * 8); }
extern "C" uint64_t or_pir_epoch(const or_pir* p) { return p->epoch; }
extern "C" void or_pir_export(const or_pir* c, uint32_t* rk, uint64_t* pt, uint64_t* par, uint64_t* pp,
                              uint64_t* bt, uint64_t* bpar, uint64_t* ri, uint64_t* rv, uint64_t* hist) {
  if (rk) memcpy(rk, c->rk, sizeof(c->rk));
  auto cp = [](uint64_t* dst, const std::vector<uint64_t>& v) {
    if (dst && !v.empty()) memcpy(dst, v.data(), v.size() * 8); };
  cp(pt, c->ptag); cp(par, c->parity); cp(pp, c->pp); cp(bt, c->btag); cp(bpar, c->bparity);
  cp(ri, c->ridx); cp(rv, c->rval); cp(hist, c->hist);
}

// ---------------------------------------------------------------------------
// SimpleBatchPianoPIR (pianopir/batch-pir.go)
// ---------------------------------------------------------------------------
static const uint64_t kQueryPerPartition = 2, kRealQueryPerPartition = 2;  // :13-14
static const uint64_t kDefaultValue = 0xdeadbeef;                           // :15

struct or_batch {
  uint64_t E_bytes, E, N, B, P, PS, F;
  std::vector<or_pir*> sub;
  uint64_t FBN = 0, QMIP = 0, Support = 0, prepCount = 0;
  double storage = 0, prepTime = 0, commOn = 0, commOff = 0;
  ~or_batch() { for (auto* s : sub) delete s; }
};

// NewSimpleBatchPianoPIR (batch-pir.go:55-93)
extern "C" or_batch* or_batch_new(uint64_t DBSize, uint64_t DBEntryByteNum, uint64_t BatchSize,
                                  const uint64_t* rawDB, uint64_t F, uint64_t seed) {
  or_batch* b = new or_batch();
  b->E_bytes = DBEntryByteNum; b->E = DBEntryByteNum / 8; b->N = DBSize; b->B = BatchSize; b->F = F;
  b->P = BatchSize / kRealQueryPerPartition;
  b->PS = (DBSize + b->P - 1) / b->P;
  for (uint64_t i = 0; i < b->P; ++i) {
    uint64_t start = i * b->PS, end = std::min((i + 1) * b->PS, DBSize);
    b->sub.push_back(or_pir_new(end - start, DBEntryByteNum, rawDB + start * b->E, F, seed, i));
  }
  return b;
}
extern "C" void or_batch_free(or_batch* b) { delete b; }

static double batch_storage(const or_batch* b) {
  double r = 0; for (auto* s : b->sub) r += or_pir_local_storage(s); return r; }
static double batch_comm_online(const or_batch* b) {    // :258-264
  double r = 0; for (auto* s : b->sub) r += or_pir_comm_per_query(s) * (double)kQueryPerPartition;
  return (double)(uint64_t)r; }
// RecordStats (batch-pir.go:110-117)
static void record_stats(or_batch* b, double t) {
  b->prepTime = t;
  b->storage = (double)(uint64_t)batch_storage(b);
  b->commOn = batch_comm_online(b);
  b->Support = b->sub[0]->MaxQ / kQueryPerPartition;
  double dbBytes = (double)b->N * (double)b->E_bytes;
  b->commOff = (double)(uint64_t)(dbBytes / (double)b->Support);
}
// Preprocessing (batch-pir.go:119-155)
extern "C" void or_batch_preprocessing(or_batch* b) {
  b->FBN = 0; b->QMIP = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (auto* s : b->sub) client_preprocessing(s);
  double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  b->prepCount++;
  record_stats(b, t);
}
// DummyPreprocessing (batch-pir.go:157-166)
extern "C" void or_batch_dummy_preprocessing(or_batch* b) {
  for (auto* s : b->sub) or_pir_dummy_preprocessing(s);
  record_stats(b, 0);
}
// Query (batch-pir.go:170-248)
extern "C" int or_batch_query(or_batch* b, const uint64_t* idx, size_t n, uint64_t* out) {
  const uint64_t E = b->E;
  uint64_t qn = n / b->P;
  std::vector<std::vector<uint64_t>> pq(b->P);
  for (size_t i = 0; i < n; ++i) {
    uint64_t p = idx[i] / b->PS;
    if (p >= b->P) return 4;   // Go: index out of range panic
    pq[p].push_back(idx[i]);
  }
  std::unordered_map<uint64_t, std::vector<uint64_t>> responses;
  std::vector<uint64_t> buf(E);
  for (uint64_t i = 0; i < b->P; ++i) {
    while (pq[i].size() < qn) pq[i].push_back(kDefaultValue);
    for (uint64_t j = 0; j < qn; ++j) {
      if (pq[i][j] == kDefaultValue) {
        or_pir_query(b->sub[i], 0, 0, buf.data());
      } else {
        or_pir_query(b->sub[i], pq[i][j] - i * b->PS, 1, buf.data());
        responses[pq[i][j]] = buf;
      }
    }
  }
  for (size_t i = 0; i < n; ++i) {
    auto it = responses.find(idx[i]);
    if (it != responses.end()) memcpy(out + i * E, it->second.data(), E * 8);
    else memset(out + i * E, 0, E * 8);
  }
  if (b->QMIP >= b->sub[0]->MaxQ - 2) {
    or_batch_preprocessing(b);
  } else {
    b->FBN += (uint64_t)(n / b->B);
    b->QMIP += qn;
  }
  return 0;
}
extern "C" void or_batch_stats_get(const or_batch* b, or_batch_stats* s) {
  s->DBEntryByteNum = b->E_bytes; s->DBEntrySize = b->E; s->DBSize = b->N; s->BatchSize = b->B;
  s->PartitionNum = b->P; s->PartitionSize = b->PS; s->ThreadNum = 1; s->FailureProbLog2 = b->F;
  s->FinishedBatchNum = b->FBN; s->QueriesMadeInPartition = b->QMIP; s->SupportBatchNum = b->Support;
  s->PrepCount = b->prepCount;
  s->LocalStorage = b->storage; s->PreprocessingTime = b->prepTime;
  s->CommOnline = b->commOn; s->CommOffline = b->commOff;
}
extern "C" or_pir* or_batch_subpir(or_batch* b, uint64_t i) { return i < b->sub.size() ? b->sub[i] : nullptr; }

// ---------------------------------------------------------------------------
// graphann search (graphann/search.go) over PIRGraphInfo (private-search.go)
// ---------------------------------------------------------------------------
struct Vtx { int64_t id; std::vector<int64_t> nb; std::vector<float> vec; };
struct VD { float dist; int64_t id; };

struct or_graph {
  uint64_t n, dim, m;
  const float* vectors; const uint32_t* graph;
  bool nonprivate, skipPrep;
  uint64_t pir_seed;
  SplitMix rng;
  std::vector<uint64_t> rawDB;
  or_batch* pir = nullptr;
  std::vector<Vtx> start;
  uint64_t total = 0, succ = 0;
  ~or_graph() { if (pir) or_batch_free(pir); }
};

extern "C" or_graph* or_graph_new(uint64_t n, uint64_t dim, uint64_t m, const float* vectors,
                                  const uint32_t* graph, int nonprivate, int skip_prep,
                                  uint64_t pir_seed, uint64_t search_seed) {
  or_graph* g = new or_graph();
  g->n = n; g->dim = dim; g->m = m; g->vectors = vectors; g->graph = graph;
  g->nonprivate = nonprivate; g->skipPrep = skip_prep; g->pir_seed = pir_seed;
  g->rng.s = search_seed;
  return g;
}
extern "C" void or_graph_free(or_graph* g) { delete g; }
extern "C" or_batch* or_graph_pir(or_graph* g) { return g->pir; }

// PIRGraphInfo.Preprocess (private-search.go:355-412) + GetStartVertex (:508-531)
extern "C" void or_graph_preprocess(or_graph* g) {
  const uint64_t ebytes = g->dim * 4 + g->m * 4, E = ebytes / 8;
  g->rawDB.assign(g->n * E, 0);
  for (uint64_t i = 0; i < g->n; ++i) {
    uint8_t* e = (uint8_t*)&g->rawDB[i * E];
    memcpy(e, g->vectors + i * g->dim, g->dim * 4);            // LE f32
    memcpy(e + g->dim * 4, g->graph + i * g->m, g->m * 4);      // LE u32
  }
  g->pir = or_batch_new(g->n, ebytes, g->m, g->rawDB.data(), 8, g->pir_seed);
  if (g->skipPrep) or_batch_dummy_preprocessing(g->pir); else or_batch_preprocessing(g->pir);
  // GetStartVertex: floor(sqrt(n)) distinct random ids, non-private
  uint64_t target = (uint64_t)std::sqrt((double)g->n);
  std::unordered_map<uint64_t, bool> added;
  g->start.clear();
  for (uint64_t i = 0; i < target; ++i) {
    uint64_t x = g->rng.intn(g->n);
    while (added.count(x)) x = g->rng.intn(g->n);
    added[x] = true;
    Vtx v; v.id = (int64_t)x;
    v.vec.assign(g->vectors + x * g->dim, g->vectors + (x + 1) * g->dim);
    v.nb.assign(g->graph + x * g->m, g->graph + (x + 1) * g->m);
    g->start.push_back(std::move(v));
  }
}

// GetVertexInfo (private-search.go:441-506)
static std::vector<Vtx> get_vertex_info(or_graph* g, const std::vector<int64_t>& ids) {
  g->total += ids.size();
  std::vector<Vtx> out(ids.size());
  if (g->nonprivate) {
    for (size_t i = 0; i < ids.size(); ++i) {
      uint64_t x = (uint64_t)ids[i];
      out[i].id = ids[i];
      out[i].vec.assign(g->vectors + x * g->dim, g->vectors + (x + 1) * g->dim);
      out[i].nb.assign(g->graph + x * g->m, g->graph + (x + 1) * g->m);
    }
    return out;
  }
  const uint64_t E = (g->dim * 4 + g->m * 4) / 8;
  std::vector<uint64_t> q(ids.begin(), ids.end()), resp(ids.size() * E);
  or_batch_query(g->pir, q.data(), q.size(), resp.data());
  for (size_t i = 0; i < ids.size(); ++i) {
    const uint8_t* e = (const uint8_t*)&resp[i * E];
    out[i].id = ids[i];
    out[i].vec.resize(g->dim); memcpy(out[i].vec.data(), e, g->dim * 4);
    out[i].nb.resize(g->m);
    bool correct = true;
    for (uint64_t j = 0; j < g->m; ++j) {
      uint32_t t; memcpy(&t, e + (g->dim + j) * 4, 4);
      out[i].nb[j] = (int64_t)t;
    }
    for (uint64_t j = 0; j < g->m; ++j)
      if (out[i].nb[j] != (int64_t)g->graph[(uint64_t)ids[i] * g->m + j]) { correct = false; break; }
    if (correct) g->succ++;
  }
  return out;
}

// The GetGraphInfo surface (graphann/search.go:20-25) of PIRGraphInfo, flat:
// GetVertexInfo of n ids (vecs n x dim, nbrs n x m as uint32; either NULL)
// and GetStartVertex (up to cap entries; returns the start set's size).
extern "C" void or_graph_get_vertex_info(or_graph* g, const int64_t* ids, uint64_t n, float* vecs, uint32_t* nbrs) {
  const std::vector<Vtx> out = get_vertex_info(g, std::vector<int64_t>(ids, ids + n));
  for (uint64_t i = 0; i < n; ++i) {
    if (vecs) memcpy(vecs + i * g->dim, out[i].vec.data(), g->dim * 4);
    if (nbrs) for (uint64_t j = 0; j < g->m; ++j) nbrs[i * g->m + j] = (uint32_t)out[i].nb[j];
  }
}
extern "C" uint64_t or_graph_get_start_vertex(const or_graph* g, uint64_t cap, int64_t* ids, float* vecs,
                                              uint32_t* nbrs) {
  for (uint64_t i = 0; i < g->start.size() && i < cap; ++i) {
    const Vtx& v = g->start[i];
    if (ids) ids[i] = v.id;
    if (vecs) memcpy(vecs + i * g->dim, v.vec.data(), g->dim * 4);
    if (nbrs) for (uint64_t j = 0; j < g->m; ++j) nbrs[i * g->m + j] = (uint32_t)v.nb[j];
  }
  return g->start.size();
}

// container/heap (Go stdlib) on a min-heap of VD keyed by dist.
static void heap_up(std::vector<VD>& h, int64_t j) {
  for (;;) { int64_t i = (j - 1) / 2; if (i == j || !(h[j].dist < h[i].dist)) break; std::swap(h[i], h[j]); j = i; }
}
static void heap_down(std::vector<VD>& h, int64_t i0, int64_t n) {
  int64_t i = i0;
  for (;;) {
    int64_t j1 = 2 * i + 1; if (j1 >= n || j1 < 0) break;
    int64_t j = j1, j2 = j1 + 1;
    if (j2 < n && h[j2].dist < h[j1].dist) j = j2;
    if (!(h[j].dist < h[i].dist)) break;
    std::swap(h[i], h[j]); i = j;
  }
}
static void heap_push(std::vector<VD>& h, VD x) { h.push_back(x); heap_up(h, (int64_t)h.size() - 1); }
static VD heap_pop(std::vector<VD>& h) {
  int64_t n = (int64_t)h.size() - 1; std::swap(h[0], h[n]); heap_down(h, 0, n);
  VD r = h.back(); h.pop_back(); return r;
}

// SearchKNN (graphann/search.go:114-234).  Tie order: stable by insertion for
// the start sort (Go's pdqsort tie order is unpinned), (dist, id) for the final sort
// (the reference iterates a Go map, whose order is random).
extern "C" void or_search_knn(or_graph* g, const float* query, int k, int max_step, int parallel,
                              int benchmarking, int64_t* ids_out, int64_t* steps_out) {
  const int64_t n = (int64_t)g->n, m = (int64_t)g->m;
  std::unordered_map<int64_t, int64_t> reach;
  std::unordered_map<int64_t, Vtx> known;
  std::unordered_map<int64_t, float> kdist;
  std::vector<VD> heap;
  if (!benchmarking) {
    std::vector<std::pair<VD, size_t>> fs;
    for (size_t i = 0; i < g->start.size(); ++i)
      fs.push_back({{or_l2dist(g->start[i].vec.data(), query, g->dim), g->start[i].id}, i});
    std::stable_sort(fs.begin(), fs.end(), [](const auto& a, const auto& b) { return a.first.dist < b.first.dist; });
    for (size_t i = 0; (int64_t)heap.size() < parallel && i < fs.size(); ++i) {
      int64_t id = fs[i].first.id;
      if (known.count(id)) continue;
      known[id] = g->start[fs[i].second];
      kdist[id] = fs[i].first.dist;
      heap_push(heap, fs[i].first);
      reach[id] = 0;
    }
  }
  for (int step = 0; step < max_step; ++step) {
    std::vector<int64_t> batch;
    for (int r = 0; r < parallel; ++r) {
      if (heap.empty() || benchmarking) {
        for (int64_t i = 0; i < m; ++i) batch.push_back((int64_t)g->rng.intn((uint64_t)n));
      } else {
        VD it = heap_pop(heap);
        const Vtx& v = known[it.id];
        batch.insert(batch.end(), v.nb.begin(), v.nb.end());
      }
    }
    std::vector<Vtx> res = get_vertex_info(g, batch);
    if (benchmarking) continue;
    for (auto& v : res) {
      if (known.count(v.id)) continue;
      bool ok = false;
      for (auto x : v.nb) if (x != 0) { ok = true; break; }
      if (ok) {
        float d = or_l2dist(v.vec.data(), query, g->dim);
        int64_t id = v.id;
        reach[id] = step;
        kdist[id] = d;
        known[id] = std::move(v);
        heap_push(heap, {d, id});
      }
    }
  }
  std::vector<VD> all;
  for (auto& kv : kdist) all.push_back({kv.second, kv.first});
  std::sort(all.begin(), all.end(), [](const VD& a, const VD& b) {
    return a.dist < b.dist || (a.dist == b.dist && a.id < b.id); });
  for (int i = 0; i < k; ++i) {
    if (i >= (int)all.size()) { ids_out[i] = -1; steps_out[i] = -1; }
    else { ids_out[i] = all[i].id; steps_out[i] = reach[all[i].id]; }
  }
}
extern "C" void or_graph_counts(const or_graph* g, uint64_t* total, uint64_t* succ) {
  *total = g->total; *succ = g->succ;
}

// private-search.go:216-240: query loop with the maintenance trigger (:226-232).
extern "C" void or_search_loop(or_graph* g, const float* queries, uint64_t q, int k, int step,
                               int parallel, int benchmarking, int64_t* answers,
                               double* online_s, double* maintenance_s) {
  std::vector<int64_t> steps(k);
  double maint = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 0; i < q; ++i) {
    or_search_knn(g, queries + i * g->dim, k, step, parallel, benchmarking, answers + i * k, steps.data());
    if (g->pir && g->pir->FBN + (uint64_t)step * (uint64_t)parallel + 10 >= g->pir->Support) {
      auto a = std::chrono::steady_clock::now();
      or_batch_preprocessing(g->pir);
      maint += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    }
  }
  double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *online_s = total - maint;
  *maintenance_s = maint;
}

// ---------------------------------------------------------------------------
// Graph construction (graphann/build_graph.go:169-236,314-523) with exact kNN
// candidates in place of NGT (absent here), and the exact kNN ground truth.
// Spec shared with the product:
//   candidates(u) = the K = int(1.5 m) smallest (L2Dist(x_u, x_v), v) over all
//                   v (u included), then u removed       (NGT.Search :398-410)
//   robustPrune     sort by (L2Dist, list position); greedy alpha test (:169-236)
//   biGraph, inbounds, edge sampling with U = hash4(seed,7,u,j,0)>>11 * 2^-53,
//   second robustPrune of lists > m, fill with hash4(seed,8,u,t,0) % n (:421-486)
// ---------------------------------------------------------------------------
static void knn_row(const float* base, uint64_t n, uint64_t dim, const float* q, uint32_t K,
                    std::vector<std::pair<uint64_t, uint32_t>>& tmp, uint32_t* out, float* dist, uint32_t* len) {
  tmp.resize(n);
  for (uint64_t v = 0; v < n; ++v) {
    float d = or_l2dist(base + v * dim, q, dim);
    uint32_t b;
    memcpy(&b, &d, 4);
    tmp[v] = {((uint64_t)b << 32) | v, (uint32_t)v};
  }
  const uint64_t k = std::min<uint64_t>(K, n);
  std::partial_sort(tmp.begin(), tmp.begin() + k, tmp.end());
  for (uint64_t i = 0; i < k; ++i) {
    out[i] = tmp[i].second;
    if (dist) { uint32_t b = (uint32_t)(tmp[i].first >> 32); memcpy(&dist[i], &b, 4); }
  }
  *len = (uint32_t)k;
}
extern "C" void or_knn(const float* base, uint64_t n, uint64_t dim, const float* queries, uint64_t nq, uint32_t k,
                       int64_t* ids, float* dists) {
  std::vector<std::pair<uint64_t, uint32_t>> tmp;
  std::vector<uint32_t> o(k);
  std::vector<float> d(k);
  for (uint64_t i = 0; i < nq; ++i) {
    uint32_t len = 0;
    knn_row(base, n, dim, queries + i * dim, k, tmp, o.data(), d.data(), &len);
    for (uint32_t j = 0; j < k; ++j) {
      ids[i * k + j] = j < len ? (int64_t)o[j] : -1;
      if (dists) dists[i * k + j] = j < len ? d[j] : INFINITY;
    }
  }
}
// robustPrune (build_graph.go:169-236); ties of sort.Slice broken by list position
static std::vector<uint32_t> robust_prune(const float* X, uint64_t dim, uint64_t u, const std::vector<uint32_t>& c,
                                          uint64_t m, float alpha) {
  if (c.size() <= m) return c;
  std::vector<std::pair<uint64_t, float>> d2u(c.size());
  for (size_t i = 0; i < c.size(); ++i) {
    float d = or_l2dist(X + u * dim, X + (uint64_t)c[i] * dim, dim);
    uint32_t b;
    memcpy(&b, &d, 4);
    d2u[i] = {((uint64_t)b << 32) | i, d};
  }
  std::sort(d2u.begin(), d2u.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<uint32_t> accept, discarded;
  for (size_t i = 0; i < d2u.size(); ++i) {
    const uint32_t v = c[(uint32_t)d2u[i].first];
    const float duv = d2u[i].second;
    bool ok = true;
    for (uint32_t a : accept)
      if (or_l2dist(X + (uint64_t)a * dim, X + (uint64_t)v * dim, dim) * alpha < duv) { ok = false; break; }
    if (ok) {
      accept.push_back(v);
      if (accept.size() == m) break;
    } else {
      discarded.push_back(v);
    }
  }
  for (size_t i = 0; accept.size() < m && i < discarded.size(); ++i) accept.push_back(discarded[i]);
  return accept;
}
extern "C" void or_robust_prune(const float* X, uint64_t dim, uint64_t u, const uint32_t* cand, uint64_t n,
                                uint64_t m, float alpha, uint32_t* out, uint32_t* len) {
  std::vector<uint32_t> c(cand, cand + n);
  std::vector<uint32_t> r = robust_prune(X, dim, u, c, m, alpha);
  std::copy(r.begin(), r.end(), out);
  *len = (uint32_t)r.size();
}
extern "C" int or_build_graph(const float* X, uint64_t n, uint64_t dim, uint64_t m, float alpha, uint64_t seed,
                              uint32_t* graph) {
  const uint32_t K = (uint32_t)((float)m * 1.5f);
  if (n <= m) return -1;
  std::vector<std::vector<uint32_t>> g1(n);
  {
    std::vector<std::pair<uint64_t, uint32_t>> tmp;
    std::vector<uint32_t> o(K);
    for (uint64_t u = 0; u < n; ++u) {
      uint32_t len = 0;
      knn_row(X, n, dim, X + u * dim, K, tmp, o.data(), nullptr, &len);
      std::vector<uint32_t> cand;
      for (uint32_t i = 0; i < len; ++i) if (o[i] != u) cand.push_back(o[i]);
      g1[u] = robust_prune(X, dim, u, cand, m, alpha);
    }
  }
  std::vector<std::vector<uint32_t>> bi(n);   // :421-430, literally
  for (uint64_t u = 0; u < n; ++u)
    for (uint32_t v : g1[u]) { bi[u].push_back(v); bi[v].push_back((uint32_t)u); }
  std::vector<uint64_t> inb(n);
  for (uint64_t i = 0; i < n; ++i) inb[i] = bi[i].size();
  for (uint64_t u = 0; u < n; ++u) {
    std::vector<uint32_t> conn;
    for (size_t j = 0; j < bi[u].size(); ++j) {
      const uint32_t v = bi[u][j];
      const double prob = std::min(1.5 * (double)m / (double)inb[v], 1.0);
      if ((double)(or_hash4(seed, 7, u, j, 0) >> 11) * 0x1.0p-53 < prob) conn.push_back(v);
    }
    if (conn.size() > m) conn = robust_prune(X, dim, u, conn, m, alpha);
    uint64_t t = 0;
    while (conn.size() < m) {
      const uint32_t v = (uint32_t)(or_hash4(seed, 8, u, t++, 0) % n);
      if (v == u) continue;
      if (std::find(conn.begin(), conn.end(), v) != conn.end()) continue;
      conn.push_back(v);
    }
    std::copy(conn.begin(), conn.end(), graph + u * m);
  }
  return 0;
}
