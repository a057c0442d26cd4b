// Microbenchmark: the server answer's XOR gather at the SIFT1M batched shape
// (6,144 sub-queries x 124 random 640-B rows of a 640 MB table), in three forms:
//   R  rows gathered into registers (k_answer_s's loop: 16-B lanes, kG rows in flight)
//   D  rows gathered into an LDS ring by LDS-DMA (global_load_lds_dwordx4), XORed from LDS
//   W  whole sub-query staged by LDS-DMA (79 KB), then XORed
// Each prints the average kernel time over its launches and the result hash.
//   hipcc -O3 --offload-arch=gfx950 -o build/gather_bench tools/gather_bench.hip
//   build/gather_bench [sub-queries] [table copies]: copies > 1 spreads the rows over
//   that many 640 MB tables (16 copies = 10 GB: the Infinity Cache holds ~2.5 % of it)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_cvoid_t;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t E = 80, SS = 124, CS = 512, PS = 62500, NPART = 16;
constexpr uint64_t NROWS = 1000000;
static uint32_t g_copies = 1;   // argv[2]: the table is this many 640 MB copies; sub-query s reads copy (s / NPART) % copies
constexpr uint32_t SEGS = E / 2;   // 16-B pieces per row

template <int NT, int KG, bool NTL = false>
__global__ void __launch_bounds__(NT) k_reg(const uint64_t* __restrict__ db, const uint16_t* __restrict__ offs,
                                            uint64_t* __restrict__ out, uint32_t copies) {
  __shared__ uint16_t qo[SS];
  __shared__ u64x2 red[NT];
  const uint32_t s = blockIdx.x, tid = threadIdx.x, p = s % NPART;
  for (uint32_t i = tid; i < SS; i += NT) qo[i] = offs[(uint64_t)s * SS + i];
  __syncthreads();
  const uint64_t* base = db + ((uint64_t)(s / NPART % copies) * NROWS + (uint64_t)p * PS) * E;
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
        if (rr[u] < PS) {
          const u64x2* src = reinterpret_cast<const u64x2*>(base + (uint64_t)rr[u] * E + seg * 2);
          x[u] = NTL ? __builtin_nontemporal_load(src) : *src;
        }
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

// k_reg with the next batch in flight while the current one folds (2 x KG rows per lane)
template <int NT, int KG>
__global__ void __launch_bounds__(NT) k_regp(const uint64_t* __restrict__ db, const uint16_t* __restrict__ offs,
                                             uint64_t* __restrict__ out, uint32_t copies) {
  __shared__ uint16_t qo[SS];
  __shared__ u64x2 red[NT];
  const uint32_t s = blockIdx.x, tid = threadIdx.x, p = s % NPART;
  for (uint32_t i = tid; i < SS; i += NT) qo[i] = offs[(uint64_t)s * SS + i];
  __syncthreads();
  const uint64_t* base = db + ((uint64_t)(s / NPART % copies) * NROWS + (uint64_t)p * PS) * E;
  const uint32_t nsl = NT / SEGS, sl = tid / SEGS, seg = tid % SEGS;
  u64x2 a = {0, 0};
  auto ld = [&](uint32_t i0, u64x2* x) {
#pragma unroll
    for (int u = 0; u < KG; ++u) {
      const uint32_t i = i0 + u * nsl;
      const uint32_t r = i < SS ? i * CS + qo[i] : ~0u;
      x[u] = u64x2{0, 0};
      if (r < PS) x[u] = *reinterpret_cast<const u64x2*>(base + (uint64_t)r * E + seg * 2);
    }
  };
  if (sl < nsl) {
    u64x2 x[KG], y[KG];
    uint32_t i0 = sl;
    ld(i0, x);
    for (;;) {
      const uint32_t i1 = i0 + KG * nsl;
      if (i1 >= SS) {
#pragma unroll
        for (int u = 0; u < KG; ++u) a ^= x[u];
        break;
      }
      ld(i1, y);
#pragma unroll
      for (int u = 0; u < KG; ++u) a ^= x[u];
#pragma unroll
      for (int u = 0; u < KG; ++u) x[u] = y[u];
      i0 = i1;
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


// k_reg + the answer's hint refresh: 124 scattered 2-B stores per sub-query
// (cur[c][hit] for every chunk c of a [SS][PH] u16 table, one table per
// (client, partition)), to price the refresh's partial-line writes
constexpr uint32_t PH = 3584;
// MODE 0: plain 2-B stores; 1: the target's word loaded first (before the
// gather: the line is in L2 when the store lands); 2: a 4-B atomic OR per
// entry (done in L2); 3: nontemporal 2-B stores
template <int NT, int KG, int MODE = 0>
__global__ void __launch_bounds__(NT) k_regw(const uint64_t* __restrict__ db, const uint16_t* __restrict__ offs,
                                             uint64_t* __restrict__ out, uint32_t copies, uint16_t* __restrict__ cur,
                                             uint32_t ntab, uint32_t salt) {
  __shared__ uint16_t qo[SS];
  __shared__ u64x2 red[NT];
  const uint32_t s = blockIdx.x, tid = threadIdx.x, p = s % NPART;
  const uint32_t hit = ((s + salt * 7919u) * 2654435761u >> 7) % PH;   // salt: new hints every launch
  // layouts of the [SS][PH] table: 0-3 row-major (chunk rows of PH hints);
  // 4: [PH / 64][SS][64] (a hint group's 124 chunk lines contiguous, 15.9 KB);
  // 5: [SS / 16][PH / 64][16][64] (2-KB tiles of 16 chunk lines x 64 hints)
  uint64_t off;
  if (MODE == 4) off = ((uint64_t)(hit / 64) * SS + tid) * 64 + hit % 64;
  else if (MODE == 5) off = (((uint64_t)(tid / 16) * (PH / 64) + hit / 64) * 16 + tid % 16) * 64 + hit % 64;
  else off = (uint64_t)tid * PH + hit;
  uint16_t* const cw = cur + (uint64_t)(s % ntab) * SS * PH + off;
  uint16_t pre = 0;
  if (MODE == 1 && tid < SS) pre = *reinterpret_cast<volatile uint16_t*>(cw);
  if (MODE == 6 && tid < SS) *cw = (uint16_t)(s + tid);   // the refresh issued before the gather
  for (uint32_t i = tid; i < SS; i += NT) qo[i] = offs[(uint64_t)s * SS + i];
  __syncthreads();
  const uint64_t* base = db + ((uint64_t)(s / NPART % copies) * NROWS + (uint64_t)p * PS) * E;
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
  if (MODE == 7 || MODE == 8) {   // chunk-pair / chunk-quad tiles: SS / 2 (4) stores of 4 (8) B
    constexpr uint32_t K = MODE == 7 ? 2 : 4;
    if (tid < SS / K) {
      uint16_t* t = cur + (uint64_t)(s % ntab) * SS * PH + ((uint64_t)tid * PH + hit) * K;
      if (K == 2) *reinterpret_cast<uint32_t*>(t) = qo[tid] | (uint32_t)qo[tid + 1] << 16;
      else *reinterpret_cast<uint2*>(t) = make_uint2(qo[tid], qo[tid + 1]);
    }
  } else if (MODE != 6 && tid < SS) {
    if (MODE == 2) atomicOr(reinterpret_cast<uint32_t*>((uintptr_t)cw & ~(uintptr_t)3), (uint32_t)qo[tid] << (((uintptr_t)cw & 2) * 8));
    else if (MODE == 3) __builtin_nontemporal_store((uint16_t)(qo[tid] ^ pre), cw);
    else *cw = (uint16_t)(qo[tid] ^ pre);
  }
}

// MODE 0 / 1: 2-B stores (plain / nontemporal); 2: aligned 4-B; 3: aligned
// 32-B (a full sector: two 16-B stores); 4: aligned 128-B (a full line: 8 lanes)
template <int MODE>
__global__ void __launch_bounds__(128) k_wonly(uint16_t* __restrict__ cur, uint32_t ntab, uint32_t salt) {
  const uint32_t s = blockIdx.x, tid = threadIdx.x;
  const uint32_t hit = ((s + salt * 7919u) * 2654435761u >> 7) % PH;
  if (tid < SS) {
    uint16_t* cw = cur + (uint64_t)(s % ntab) * SS * PH + (uint64_t)tid * PH + hit;
    if (MODE == 1) __builtin_nontemporal_store((uint16_t)(s + tid), cw);
    else if (MODE == 2) *reinterpret_cast<uint32_t*>((uintptr_t)cw & ~(uintptr_t)3) = s + tid;
    else if (MODE == 3) {
      uint4* q = reinterpret_cast<uint4*>((uintptr_t)cw & ~(uintptr_t)31);
      q[0] = make_uint4(s, tid, 1, 2);
      q[1] = make_uint4(s, tid, 3, 4);
    } else if (MODE == 4) {
      uint4* q = reinterpret_cast<uint4*>((uintptr_t)cw & ~(uintptr_t)127);
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = make_uint4(s, tid, k, 2);
    } else *cw = (uint16_t)(s + tid);
  }
}

// LDS-DMA ring: B rows per stage, NB stages in flight.  Piece q of a stage =
// row q / 40, 16-B segment q % 40; wave-instruction k of the stage moves pieces
// 64k .. 64k + 63 (whole 128-B lines: rows are 5 lines).
template <int NT, int B, int NB>
__global__ void __launch_bounds__(NT) k_dma(const uint64_t* __restrict__ db, const uint16_t* __restrict__ offs,
                                            uint64_t* __restrict__ out, uint32_t copies) {
  constexpr uint32_t PIECES = B * SEGS, INSTR = (PIECES + 63) / 64, NW = NT / 64;
  __shared__ __attribute__((aligned(16))) u64x2 ring[NB][INSTR * 64];
  __shared__ uint32_t rows[SS];
  __shared__ u64x2 red[NT];
  const uint32_t s = blockIdx.x, tid = threadIdx.x, p = s % NPART, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < SS; i += NT) {
    const uint32_t r = i * CS + offs[(uint64_t)s * SS + i];
    rows[i] = r < PS ? r : PS;   // PS: a zero row (the table has one past every partition? use row 0 masked below)
  }
  __syncthreads();
  const char* base = reinterpret_cast<const char*>(db + ((uint64_t)(s / NPART % copies) * NROWS + (uint64_t)p * PS) * E);
  constexpr uint32_t NST = (SS + B - 1) / B;
  auto issue = [&](uint32_t st) {
    for (uint32_t k = wave; k < INSTR; k += NW) {
      const uint32_t q = k * 64 + lane, rl = q / SEGS, i = st * B + rl;
      uint32_t r = (q < PIECES && i < SS) ? rows[i] : PS;
      if (r >= PS) r = 0;   // out-of-range rows: loaded from row 0 and masked at the XOR
      __builtin_amdgcn_global_load_lds((g_cvoid_t*)(base + (uint64_t)r * (E * 8) + (q % SEGS) * 16),
                                       (lds_void_t*)&ring[st % NB][k * 64], 16, 0, 0);
    }
  };
  for (uint32_t st = 0; st < NB - 1 && st < NST; ++st) issue(st);
  const uint32_t nsl = NT / SEGS, sl = tid / SEGS, seg = tid % SEGS;
  u64x2 a = {0, 0};
  for (uint32_t st = 0; st < NST; ++st) {
    if (st + NB - 1 < NST) issue(st + NB - 1);
    // wait for stage st: at most (stages issued after it) x (its instructions per wave) outstanding
    const uint32_t later = min(NST - 1 - st, (uint32_t)NB - 1);
    constexpr uint32_t IPW = (INSTR + NW - 1) / NW;
    if (later == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(IPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * IPW) : "memory");
    __syncthreads();
    if (sl < nsl)
      for (uint32_t rl = sl; rl < B; rl += nsl) {
        const uint32_t i = st * B + rl;
        if (i < SS && rows[i] < PS) a ^= ring[st % NB][rl * SEGS + seg];
      }
    __syncthreads();
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

__global__ void k_fill(uint64_t* db, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9e3779b97f4a7c15ull + 0x1234567ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    db[i] = z ^ (z >> 31);
  }
}

static double g_bytes = 0;
template <class F>
static void run(const char* name, F launch, uint64_t* d_out, uint32_t ns, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipMemset(d_out, 0, (size_t)ns * E * 8));
  launch(); launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  std::vector<uint64_t> h((size_t)ns * E);
  CK(hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t hs = 0; for (size_t i = 0; i < h.size(); ++i) hs = hs * 31 + h[i];
  const double us = ms * 1000.0 / reps;
  // algorithmic bytes: in-range rows x 640 B
  printf("%-14s %8.2f us  %6.3f TB/s(in-range rows)  hash %016llx\n", name, us, g_bytes / us / 1e6, (unsigned long long)hs);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const uint32_t ns = argc > 1 ? atoi(argv[1]) : 6144;
  g_copies = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = 50;
  uint64_t *db, *out; uint16_t* offs;
  CK(hipMalloc(&db, g_copies * NROWS * E * 8));
  CK(hipMalloc(&out, (size_t)ns * E * 8));
  CK(hipMalloc(&offs, (size_t)ns * SS * 2));
  k_fill<<<4096, 256>>>(db, g_copies * NROWS * E);
  std::vector<uint16_t> ho((size_t)ns * SS);
  uint64_t x = 88172645463325252ull, inrange = 0;
  for (auto& o : ho) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; o = x % CS; }
  for (uint32_t s = 0; s < ns; ++s) for (uint32_t i = 0; i < SS; ++i) inrange += (i * CS + ho[(size_t)s * SS + i]) < PS;
  CK(hipMemcpy(offs, ho.data(), ho.size() * 2, hipMemcpyHostToDevice));
  const double bytes = inrange * 640.0;
  g_bytes = bytes;
  printf("table copies %u (%.1f GB)\n", g_copies, g_copies * NROWS * E * 8 / 1e9);
  printf("sub-queries %u, in-range rows %llu, %.1f MB per launch\n", ns, (unsigned long long)inrange, bytes / 1e6);
  // NSETS different offset sets, cycled launch by launch (every launch gathers
  // new rows, as the serving steps do; one set repeated back to back keeps
  // half of its 480 MB in the 256 MB Infinity Cache and reads too fast)
  constexpr int NSETS = 8;
  uint16_t* offs_all;
  CK(hipMalloc(&offs_all, (size_t)NSETS * ns * SS * 2));
  for (int k = 0; k < NSETS; ++k) {
    for (auto& o : ho) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; o = x % CS; }
    CK(hipMemcpy(offs_all + (size_t)k * ns * SS, ho.data(), ho.size() * 2, hipMemcpyHostToDevice));
  }
  int launch_no = 0;
  auto R = [&](const char* nm, auto kern, int nt) {
    run(nm, [&] {
      hipLaunchKernelGGL(kern, dim3(ns), dim3(nt), 0, 0, db, offs_all + (size_t)(launch_no++ % NSETS) * ns * SS, out, g_copies);
    }, out, ns, reps);
  };
  R("reg128k6", (k_reg<128, 6>), 128);
  {   // the refresh's scattered writes beside the gather: 4,608 tables = 288 clients x 16 partitions (4.1 GB)
    const uint32_t ntab = 4608;
    const bool salt_on = getenv("GB_SALT") != nullptr;   // new hints every launch (the serving pattern)
    uint16_t* cur;
    CK(hipMalloc(&cur, (size_t)ntab * SS * PH * 2));
    CK(hipMemset(cur, 0, (size_t)ntab * SS * PH * 2));
    run("reg128k6", [&] {
      hipLaunchKernelGGL((k_reg<128, 6>), dim3(ns), dim3(128), 0, 0, db, offs_all + (size_t)(launch_no++ % NSETS) * ns * SS, out, g_copies);
    }, out, ns, reps);
    auto W = [&](const char* nm, auto kern) {
      run(nm, [&] {
        const uint32_t ln = launch_no++;
        hipLaunchKernelGGL(kern, dim3(ns), dim3(128), 0, 0, db, offs_all + (size_t)(ln % NSETS) * ns * SS, out,
                           g_copies, cur, ntab, salt_on ? ln : 0u);
      }, out, ns, reps);
    };
    W("regw_plain", (k_regw<128, 6, 0>));
    W("regw_pair", (k_regw<128, 6, 7>));
    W("regw_quad", (k_regw<128, 6, 8>));
    W("regw_plain", (k_regw<128, 6, 0>));
    W("regw_pair", (k_regw<128, 6, 7>));
    W("regw_quad", (k_regw<128, 6, 8>));
    W("regw_plain", (k_regw<128, 6, 0>));
    W("regw_nt", (k_regw<128, 6, 3>));
    auto WO = [&](const char* nm, auto kern) {
      run(nm, [&] { hipLaunchKernelGGL(kern, dim3(ns), dim3(128), 0, 0, cur, ntab, salt_on ? launch_no++ : 0u); }, out, ns, reps);
    };
    WO("wonly_2B", k_wonly<0>);
    WO("wonly_2B_nt", k_wonly<1>);
    WO("wonly_4B", k_wonly<2>);
    WO("wonly_32B", k_wonly<3>);
    WO("wonly_128B", k_wonly<4>);
    WO("wonly_2B", k_wonly<0>);
    CK(hipFree(cur));
  }
  if (getenv("GB_ONLY_W")) return 0;
  R("regp128k6", (k_regp<128, 6>), 128);
  R("regp128k4", (k_regp<128, 4>), 128);
  R("regp128k8", (k_regp<128, 8>), 128);
  R("reg128k6nt", (k_reg<128, 6, true>), 128);
  R("reg128k8nt", (k_reg<128, 8, true>), 128);
  R("reg256k8nt", (k_reg<256, 8, true>), 256);
  R("reg128k8", (k_reg<128, 8>), 128);
  R("reg128k16", (k_reg<128, 16>), 128);
  R("reg256k8", (k_reg<256, 8>), 256);
  R("reg256k4", (k_reg<256, 4>), 256);
  R("reg64k8", (k_reg<64, 8>), 64);
  R("dma128b16n2", (k_dma<128, 16, 2>), 128);
  R("dma128b16n3", (k_dma<128, 16, 3>), 128);
  R("dma128b32n2", (k_dma<128, 32, 2>), 128);
  R("dma256b32n2", (k_dma<256, 32, 2>), 256);
  R("dma256b32n3", (k_dma<256, 32, 3>), 256);
  R("dma256b64n2", (k_dma<256, 64, 2>), 256);
  R("dma128b124n1", (k_dma<128, 124, 1>), 128);
  R("dma256b124n1", (k_dma<256, 124, 1>), 256);
  R("dma64b16n3", (k_dma<64, 16, 3>), 64);
  printf("bytes per launch %.0f\n", bytes);
  return 0;
}
