// Microbenchmark: can the maintenance (LDS-bound) and the answers (HBM-bound)
// share the GPU by CU partition?  Streams made with hipExtStreamCreateWithCUMask:
//   1. the answer's register gather (gather_bench's k_reg: 6,912 sub-queries x
//      124 random 640-B rows of a 640 MB table) on the first n CUs of every XCD
//      (n / 8 per XCD, "spread") or on the first n CUs in mask order ("contig");
//   2. an LDS-bound kernel shaped like k_prep_fold_rot (1,024 threads, 128 KB
//      of LDS, random 16-B reads with 2-way bank conflicts, XOR accumulate) on
//      a mask alone and beside the gather on the complementary mask.
//   hipcc -O3 --offload-arch=gfx950 -o build/cumask_bench tools/cumask_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t E = 80, SS = 124, CS = 512, PS = 62500, NPART = 16, SEGS = E / 2;
constexpr uint64_t NROWS = 1000000;

template <int NT, int KG>
__global__ void __launch_bounds__(NT) k_reg(const uint64_t* __restrict__ db, const uint16_t* __restrict__ offs,
                                            uint64_t* __restrict__ out) {
  __shared__ uint16_t qo[SS];
  __shared__ u64x2 red[NT];
  const uint32_t s = blockIdx.x, tid = threadIdx.x, p = s % NPART;
  for (uint32_t i = tid; i < SS; i += NT) qo[i] = offs[(uint64_t)s * SS + i];
  __syncthreads();
  const uint64_t* base = db + (uint64_t)p * PS * E;
  const uint32_t nsl = NT / SEGS, sl = tid / SEGS, seg = tid % SEGS;
  u64x2 a = {0, 0};
  if (sl < nsl) {
    for (uint32_t i0 = sl; i0 < SS; i0 += KG * nsl) {
      uint32_t rr[KG];
#pragma unroll
      for (int u = 0; u < KG; ++u) { const uint32_t i = i0 + u * nsl; rr[u] = i < SS ? i * CS + qo[i] : ~0u; }
      u64x2 x[KG];
#pragma unroll
      for (int u = 0; u < KG; ++u) {
        x[u] = u64x2{0, 0};
        if (rr[u] < PS) x[u] = *reinterpret_cast<const u64x2*>(base + (uint64_t)rr[u] * E + seg * 2);
      }
#pragma unroll
      for (int u = 0; u < KG; ++u) a ^= x[u];
    }
  }
  red[tid] = a;
  __syncthreads();
  if (tid < SEGS) {
    u64x2 x = {0, 0};
    for (uint32_t k = 0; k < nsl; ++k) x ^= red[k * SEGS + tid];
    out[(uint64_t)s * E + tid * 2] = x.x;
    out[(uint64_t)s * E + tid * 2 + 1] = x.y;
  }
}

// LDS-bound stand-in for the fold: each lane XORs `iters` random 16-B LDS
// reads (128-B lines, the fold's 2-way conflicts), one result store per lane
__global__ void __launch_bounds__(1024) k_lds(uint64_t* __restrict__ out, uint32_t iters) {
  __shared__ __attribute__((aligned(16))) uint4 buf[8192];   // 128 KB
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 8192; i += 1024) buf[i] = make_uint4(i, i * 3, i * 5, i * 7);
  __syncthreads();
  uint32_t x = tid * 2654435761u + blockIdx.x, a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const uint32_t slot = tid & 7;
  for (uint32_t k = 0; k < iters; ++k) {
    x = x * 1664525u + 1013904223u;
    const uint4 v = buf[((x >> 20) & 1023) * 8 + slot];
    a0 ^= v.x; a1 ^= v.y; a2 ^= v.z; a3 ^= v.w;
  }
  out[(uint64_t)blockIdx.x * 1024 + tid] = (uint64_t)(a0 ^ a1) << 32 | (a2 ^ a3);
}

// where a workgroup runs: XCC id and HW_ID's (se, sh, cu)
__global__ void k_where(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID, 32 bits
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // XCC_ID[3:0]
    const uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    out[blockIdx.x] = xcc << 16 | se << 8 | sh << 4 | cu;
  }
}

static hipStream_t masked(uint32_t n, bool spread, bool invert) {
  std::vector<uint32_t> m(8, 0);
  for (uint32_t i = 0; i < 256; ++i) {
    bool on = spread ? (i % 32) < n / 8 : i < n;
    if (invert) on = !on;
    if (on) m[i / 32] |= 1u << (i % 32);
  }
  hipStream_t s;
  CK(hipExtStreamCreateWithCUMask(&s, 8, m.data()));
  return s;
}

int main() {
  const uint32_t ns = 6912, reps = 20;
  uint64_t *db, *out, *lout;
  uint16_t* offs;
  CK(hipMalloc(&db, NROWS * E * 8));
  CK(hipMemset(db, 1, NROWS * E * 8));
  CK(hipMalloc(&out, (size_t)ns * E * 8));
  CK(hipMalloc(&lout, (size_t)4096 * 1024 * 8));
  constexpr int NSETS = 8;
  CK(hipMalloc(&offs, (size_t)NSETS * ns * SS * 2));
  std::vector<uint16_t> ho((size_t)NSETS * ns * SS);
  uint64_t x = 88172645463325252ull, inrange = 0;
  for (auto& o : ho) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; o = x % CS; }
  for (uint32_t s = 0; s < ns; ++s) for (uint32_t i = 0; i < SS; ++i) inrange += (i * CS + ho[(size_t)s * SS + i]) < PS;
  CK(hipMemcpy(offs, ho.data(), ho.size() * 2, hipMemcpyHostToDevice));
  const double bytes = inrange * 640.0;
  hipEvent_t a, b, c, d;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); CK(hipEventCreate(&c)); CK(hipEventCreate(&d));
  int ln = 0;
  auto gather = [&](hipStream_t s) {
    hipLaunchKernelGGL((k_reg<128, 6>), dim3(ns), dim3(128), 0, s, db, offs + (size_t)(ln++ % NSETS) * ns * SS, out);
  };
  const uint32_t lds_iters = 256, lds_grid = 2048;
  auto lds = [&](hipStream_t s) { hipLaunchKernelGGL(k_lds, dim3(lds_grid), dim3(1024), 0, s, lout, lds_iters); };
  const double lds_bytes = (double)lds_grid * 1024 * lds_iters * 16;
  {   // placement of 8 masks: which XCCs / CUs run the workgroups of a stream whose mask is one 32-bit word
    uint32_t* w; CK(hipMalloc(&w, 4096 * 4));
    std::vector<uint32_t> h(4096);
    for (int word = 0; word < 8; word += 7) {
      std::vector<uint32_t> m(8, 0);
      m[word] = 0xffffffffu;
      hipStream_t s; CK(hipExtStreamCreateWithCUMask(&s, 8, m.data()));
      hipLaunchKernelGGL(k_where, dim3(4096), dim3(64), 0, s, w);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(h.data(), w, 4096 * 4, hipMemcpyDeviceToHost));
      uint32_t xccs = 0; std::vector<uint32_t> seen;
      for (uint32_t v : h) { xccs |= 1u << (v >> 16); bool f = false; for (uint32_t q : seen) f |= q == v; if (!f) seen.push_back(v); }
      printf("mask word %d: XCC set 0x%02x, %zu distinct (xcc, se, sh, cu)\n", word, xccs, seen.size());
      m.assign(8, 0);
      for (int k = 0; k < 8; ++k) m[k] = 1u;   // bit 0 of every word
      fflush(stdout);
    }
    for (int variant = 0; variant < 2; ++variant) {
      std::vector<uint32_t> m(8, 0);
      if (variant == 0) for (int k = 0; k < 8; ++k) m[k] = 0xfu;   // bits 0-3 of every word
      else m[0] = 0xffffffffu, m[1] = 0;                            // first 32 bits
      hipStream_t s; CK(hipExtStreamCreateWithCUMask(&s, 8, m.data()));
      hipLaunchKernelGGL(k_where, dim3(4096), dim3(64), 0, s, w);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(h.data(), w, 4096 * 4, hipMemcpyDeviceToHost));
      uint32_t xccs = 0; std::vector<uint32_t> seen;
      for (uint32_t v : h) { xccs |= 1u << (v >> 16); bool f = false; for (uint32_t q : seen) f |= q == v; if (!f) seen.push_back(v); }
      printf("%s: XCC set 0x%02x, %zu distinct CUs\n", variant == 0 ? "bits 0-3 of each word" : "word 0", xccs, seen.size());
      fflush(stdout);
    }
  }
  printf("gather alone on n CUs (TB/s of in-range rows)\n");
  std::vector<hipStream_t> pool;
  for (int spread = 1; spread >= 0; --spread)
    for (uint32_t n : {32u, 64u, 96u, 128u, 256u}) {
      hipStream_t s = masked(n, spread, false);
      pool.push_back(s);
      gather(s); gather(s);
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (uint32_t r = 0; r < reps; ++r) gather(s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("  %-6s n=%3u  %8.1f us  %.3f TB/s\n", spread ? "spread" : "contig", n, ms * 1e3 / reps, bytes / (ms / reps) / 1e9);
      fflush(stdout);
    }
  printf("LDS kernel alone on n CUs (TB/s of LDS reads)\n");
  for (uint32_t n : {256u, 176u}) {
    hipStream_t s = masked(n, true, false);
    lds(s);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (uint32_t r = 0; r < 3; ++r) lds(s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("  n=%3u  %8.3f ms  %.1f TB/s\n", n, ms / 3, lds_bytes / (ms / 3) / 1e9);
    fflush(stdout);
  }
  printf("together: LDS kernel on n CUs, gathers on the other 256 - n\n");
  for (uint32_t n : {176u}) {
    hipStream_t sl = masked(n, true, false), sg = masked(n, true, true);
    lds(sl); gather(sg);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, sl));
    CK(hipEventRecord(c, sg));
    for (uint32_t r = 0; r < 3; ++r) lds(sl);
    CK(hipEventRecord(b, sl));
    uint32_t ng = 0;
    // gathers until the LDS kernels are done
    while (hipEventQuery(b) == hipErrorNotReady && ng < 100000) {
      for (int k = 0; k < 10; ++k) gather(sg);
      ng += 10;
      CK(hipStreamSynchronize(sg));
    }
    CK(hipEventRecord(d, sg));
    CK(hipDeviceSynchronize());
    float ml, mg; CK(hipEventElapsedTime(&ml, a, b)); CK(hipEventElapsedTime(&mg, c, d));
    printf("  n=%3u  LDS %8.3f ms (%.1f TB/s)   gathers %u in %.3f ms: %.1f us each, %.3f TB/s\n", n, ml / 3,
           lds_bytes / (ml / 3) / 1e9, ng, mg, mg * 1e3 / ng, bytes * ng / mg / 1e9);
    fflush(stdout);
  }
  return 0;
}
