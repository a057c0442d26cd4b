// Diagnostic: host-observed latency of one kernel launch on MI355X.
//   hipcc --offload-arch=gfx950 -O2 -o tools/launch_latency tools/launch_latency.hip
// (a) launch -> the kernel's token visible in fine-grained pinned host memory
//     (host spin-polls), for a 1-workgroup and a 208 x 1024-thread grid;
// (b) the same with a device-side spin of ~10 us before the token, to check
//     that (a) is latency and not the kernel body;
// (c) a resident "doorbell" kernel: the host writes a token into pinned host
//     memory, the kernel (already running) polls it and answers: the host->
//     device->host round trip without a launch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_token(volatile uint32_t* out, uint32_t tok, uint32_t spin_ticks) {
  if (spin_ticks && threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __hip_atomic_store((uint32_t*)out, tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// resident: waits for door == k, answers ans = k, for k = 1..n; bounded spin
__global__ void k_door(const uint32_t* door, uint32_t* ans, uint32_t n) {
  if (threadIdx.x != 0) return;
  for (uint32_t k = 1; k <= n; ++k) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != k) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) return;   // 1 s: give up
    }
    __hip_atomic_store(ans, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// G workgroups resident; for k = 1..n: every workgroup waits for door == k
// (mode 0: every workgroup polls `door` itself; mode 1: workgroup 0 polls
// `door` and broadcasts through device memory `bc`), counts into `cnt`, and
// the last arrival answers ans = k.  Bounded spins.
__global__ void __launch_bounds__(1024) k_door_many(const uint32_t* door, uint32_t* ans, uint32_t* cnt, uint32_t* bc,
                                                   uint32_t n, int mode) {
  __shared__ int quit;
  for (uint32_t k = 1; k <= n; ++k) {
    if (threadIdx.x == 0) {
      quit = 0;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      if (mode == 0 || blockIdx.x == 0) {
        while (__hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != k)
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) { quit = 1; break; }
        if (mode == 1 && !quit) __hip_atomic_store(bc, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (__hip_atomic_load(bc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != k) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) { quit = 1; break; }
        }
      }
      if (!quit) {
        const uint32_t prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == gridDim.x * k) __hip_atomic_store(ans, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
    if (quit) return;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  printf("%-44s median %7.2f us  p10 %7.2f  p90 %7.2f\n", name, v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t* tok;
  CK(hipHostMalloc((void**)&tok, 4096, hipHostMallocCoherent));
  const int iters = 2000;
  struct Cfg { const char* name; dim3 grid, blk; uint32_t spin; } cfgs[] = {
      {"launch -> token, 1 x 64", dim3(1), dim3(64), 0},
      {"launch -> token, 208 x 1024", dim3(208), dim3(1024), 0},
      {"launch -> token, 208 x 1024, 10 us body", dim3(208), dim3(1024), 1000},
  };
  for (auto& c : cfgs) {
    std::vector<double> v;
    for (int i = 0; i < iters; ++i) {
      const uint32_t t = i + 1 + (uint32_t)(&c - cfgs) * 100000;
      const double t0 = now_us();
      hipLaunchKernelGGL(k_token, c.grid, c.blk, 0, st, (volatile uint32_t*)tok, t, c.spin);
      const double t1 = now_us();
      while (__atomic_load_n(tok, __ATOMIC_ACQUIRE) != t) {}
      const double t2 = now_us();
      if (i >= 100) v.push_back(t2 - t0);
      (void)t1;
      CK(hipStreamSynchronize(st));
    }
    report(c.name, v);
  }
  {   // launch call cost alone
    std::vector<double> v;
    for (int i = 0; i < iters; ++i) {
      const double t0 = now_us();
      hipLaunchKernelGGL(k_token, dim3(1), dim3(64), 0, st, (volatile uint32_t*)tok, 7u, 0u);
      v.push_back(now_us() - t0);
      CK(hipStreamSynchronize(st));
    }
    report("hipLaunchKernelGGL call (host)", v);
  }
  {   // resident doorbell
    uint32_t* door = tok + 256;
    uint32_t* ans = tok + 512;
    *door = 0; *ans = 0;
    const uint32_t n = 2000;
    hipLaunchKernelGGL(k_door, dim3(1), dim3(64), 0, st, door, ans, n);
    std::vector<double> v;
    // wait until the kernel runs: first round trip is excluded
    for (uint32_t k = 1; k <= n; ++k) {
      const double t0 = now_us();
      __atomic_store_n(door, k, __ATOMIC_RELEASE);
      while (__atomic_load_n(ans, __ATOMIC_ACQUIRE) != k) {}
      if (k > 100) v.push_back(now_us() - t0);
    }
    CK(hipStreamSynchronize(st));
    report("doorbell round trip (resident kernel)", v);
  }
  for (int mode = 0; mode < 2; ++mode) {
    for (int G : {16, 240}) {
      uint32_t* door = tok + 256;
      uint32_t* ans = tok + 512;
      *door = 0; *ans = 0;
      uint32_t *cnt, *bc;
      CK(hipMalloc((void**)&cnt, 4096));
      CK(hipMemset(cnt, 0, 4096));
      bc = cnt + 64;
      const uint32_t n = 1000;
      hipLaunchKernelGGL(k_door_many, dim3(G), dim3(1024), 0, st, door, ans, cnt, bc, n, mode);
      std::vector<double> v;
      for (uint32_t k = 1; k <= n; ++k) {
        const double t0 = now_us();
        __atomic_store_n(door, k, __ATOMIC_RELEASE);
        const double tl = now_us();
        while (__atomic_load_n(ans, __ATOMIC_ACQUIRE) != k) {
          if (now_us() - tl > 2e6) { fprintf(stderr, "timeout\n"); return 1; }
        }
        if (k > 50) v.push_back(now_us() - t0);
      }
      CK(hipStreamSynchronize(st));
      char name[96];
      snprintf(name, sizeof name, "doorbell to %d WGs + fan-in, %s", G, mode ? "1 poller + bcast" : "all poll host");
      report(name, v);
      CK(hipFree(cnt));
    }
  }
  {   // host writes fine-grained device memory?
    uint32_t* fg = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&fg, 4096, hipDeviceMallocFinegrained);
    printf("fine-grained device alloc: %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
      hipPointerAttribute_t at;
      if (hipPointerGetAttributes(&at, fg) == hipSuccess) printf("  host pointer %p\n", at.hostPointer);
      CK(hipFree(fg));
    }
  }
  CK(hipHostFree(tok));
  return 0;
}
