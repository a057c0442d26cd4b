// aes_bs_bench.hip — the maintenance's PRF-table kernel in its forms at the
// serving shapes: k_prep_offsets (T-table AES in LDS, rounds 1-5) against the
// bitsliced AES on the VALU (round 6, pm_aes_bs.h): k_prep_offsets_bs (32
// blocks per lane, 256 VGPRs, 2 waves per SIMD).  The packed 16-block form
// (k_prep_offsets_bs16, 128 VGPRs, 4 waves per SIMD) measured 0.85x and was
// removed; it is in commit a8645fe (profiles/r06/aes/README.md).
// All write every table (tabT, cur, and tab where given) for K clients x 16
// partitions with their own keys; the outputs are compared word for word and
// each launch is timed with HIP events (ABAB order, REPS rounds).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o build/aes_bs_bench tools/aes_bs_bench.hip
//   build/aes_bs_bench [sift1m|msmarco|bigann] [clients] [reps]
#include "../pacmann_amd/csrc/pm_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

static void expand_key(const uint8_t key[16], uint32_t rk[44]) {   // FIPS-197 §5.2
  static constexpr pm::AesTables T{};
  uint8_t w[176];
  memcpy(w, key, 16);
  uint8_t rcon = 1;
  for (int i = 16; i < 176; i += 4) {
    uint8_t t[4] = {w[i - 4], w[i - 3], w[i - 2], w[i - 1]};
    if (i % 16 == 0) {
      const uint8_t u = t[0];
      t[0] = T.sbox[t[1]] ^ rcon; t[1] = T.sbox[t[2]]; t[2] = T.sbox[t[3]]; t[3] = T.sbox[u];
      rcon = pm::AesTables::gmul(rcon, 2);
    }
    for (int k = 0; k < 4; ++k) w[i + k] = w[i - 16 + k] ^ t[k];
  }
  memcpy(rk, w, 176);
}

struct Shape { const char* name; uint32_t CS, log2CS, SS, PH, Qpc; bool tab; };

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "sift1m";
  Shape S{"sift1m", 512, 9, 124, 3584, 72, false};
  if (which == "msmarco") S = Shape{"msmarco", 1024, 10, 196, 7168, 88, true};
  if (which == "bigann") S = Shape{"bigann100m", 8192, 13, 764, 57344, 160, false};
  const int K = argc > 2 ? atoi(argv[2]) : 288, reps = argc > 3 ? atoi(argv[3]) : 3;
  const int np = K * 16;
  const uint32_t H = S.PH + S.SS * S.Qpc, curk = pm::cur_k(S.PH, S.SS);
  const uint64_t tTw = pm::tabT_words(H, S.SS), cw = pm::cur_words(S.PH, S.SS, curk);
  const uint64_t tw = S.tab ? (uint64_t)S.SS * H : 0;
  const uint64_t per = tTw + cw + tw;
  printf("{\"shape\": \"%s\", \"clients\": %d, \"parts\": %d, \"H\": %u, \"SS\": %u, \"CS\": %u, \"curk\": %u, "
         "\"table_GB_per_variant\": %.2f}\n", S.name, K, np, H, S.SS, S.CS, curk, per * 2.0 * np / 1e9);
  constexpr int NV = 2;
  static const char* kname[NV] = {"k_prep_offsets", "k_prep_offsets_bs"};
  uint16_t* buf[NV];
  for (int v = 0; v < NV; ++v) {
    CK(hipMalloc(&buf[v], per * 2 * np));
    CK(hipMemset(buf[v], 0x11 * (v + 3), per * 2 * np));
  }
  std::vector<pm::PmPart> hp[NV];
  for (int v = 0; v < NV; ++v) hp[v].resize(np);
  uint64_t st = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < np; ++i) {
    pm::PmPart p;
    memset(&p, 0, sizeof p);
    p.N = (uint64_t)S.SS * S.CS; p.CS = S.CS; p.log2CS = S.log2CS; p.SS = S.SS; p.PH = S.PH; p.Qpc = S.Qpc;
    p.H = H; p.curk = curk;
    uint8_t key[16];
    for (int b = 0; b < 16; b += 8) { const uint64_t r = pm::sm64(st += 0x9e3779b97f4a7c15ULL); memcpy(key + b, &r, 8); }
    expand_key(key, p.rk);
    for (int v = 0; v < NV; ++v) {
      hp[v][i] = p;
      PM_G uint16_t* a = (PM_G uint16_t*)(buf[v] + (uint64_t)i * per);
      hp[v][i].tabT = a; hp[v][i].cur = a + tTw; hp[v][i].tab = S.tab ? a + tTw + cw : nullptr;
    }
  }
  pm::PmPart* dp[NV];
  for (int v = 0; v < NV; ++v) {
    CK(hipMalloc(&dp[v], sizeof(pm::PmPart) * np));
    CK(hipMemcpy(dp[v], hp[v].data(), sizeof(pm::PmPart) * np, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double prfs = (double)np * H * S.SS;
  std::vector<float> tv[NV];
  for (int r = 0; r < reps + 1; ++r) {
    for (int v = 0; v < NV; ++v) {
      CK(hipEventRecord(e0, 0));
      if (v == 0) pmk::prep_offsets_tt(0, dp[0], np, H, S.SS);
      else pmk::prep_offsets_bs(0, dp[1], np, H, S.SS);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) tv[v].push_back(ms);   // the first round warms up
      printf("{\"round\": %d, \"kernel\": \"%s\", \"ms\": %.3f, \"G_PRF_per_s\": %.1f}\n", r, kname[v], ms,
             prfs / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  // Co-residency: the T-table kernel (LDS-bound) and the bitsliced one (VALU-bound) side by side on
  // two streams over disjoint client sets; the T-table workgroups padded with dynamic LDS so that
  // one fits per CU and a bitsliced workgroup (one wave per SIMD) fits beside it.
  if (getenv("AES_COSPLIT")) {
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea)); CK(hipEventCreate(&eb));
    for (int pad : {0, 24 * 1024}) {
      for (int pct : {100, 80, 70, 60, 50, 0}) {
        const int na = (int)((int64_t)K * pct / 100) * 16, nbp = np - na;
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0, 0));
          CK(hipStreamWaitEvent(sa, e0, 0)); CK(hipStreamWaitEvent(sb, e0, 0));
          if (na) hipLaunchKernelGGL(pm::k_prep_offsets, dim3(pmk::cdiv(H, pm::kOffsBlock), pmk::cdiv(S.SS, 8), na),
                                     dim3(pm::kOffsBlock), pad, sa, dp[0]);
          if (nbp) pmk::prep_offsets_bs(sb, dp[1] + na, nbp, H, S.SS);
          CK(hipEventRecord(ea, sa)); CK(hipEventRecord(eb, sb));
          CK(hipStreamWaitEvent(0, ea, 0)); CK(hipStreamWaitEvent(0, eb, 0));
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          CK(hipGetLastError());
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = std::min(best, ms);
        }
        printf("{\"cosplit\": {\"tt_pct\": %d, \"tt_lds_pad\": %d, \"ms\": %.3f, \"G_PRF_s\": %.1f}}\n", pct, pad, best,
               prfs / (best * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
  }
  // compare every table word (padding words of tabT tiles included) with the T-table kernel's
  std::vector<uint16_t> A(per), B(per);
  uint64_t bad[NV][3] = {};
  for (int i = 0; i < np; ++i) {
    CK(hipMemcpy(A.data(), buf[0] + (uint64_t)i * per, per * 2, hipMemcpyDeviceToHost));
    for (int v = 1; v < NV; ++v) {
      CK(hipMemcpy(B.data(), buf[v] + (uint64_t)i * per, per * 2, hipMemcpyDeviceToHost));
      for (uint64_t w = 0; w < per; ++w)
        if (A[w] != B[w]) {
          if (bad[v][0] + bad[v][1] + bad[v][2] < 3)
            fprintf(stderr, "%s part %d word %llu: tt %04x got %04x\n", kname[v], i, (unsigned long long)w, A[w], B[w]);
          ++bad[v][w < tTw ? 0 : w < tTw + cw ? 1 : 2];
        }
    }
    if (K > 64 && i >= 64 * 16) break;   // the first 64 clients' tables are enough for the check at full shape
  }
  auto avg = [](const std::vector<float>& v) { double s = 0; for (float x : v) s += x; return v.empty() ? 0.0 : s / v.size(); };
  const double a = avg(tv[0]);
  uint64_t total_bad = 0;
  printf("{\"shape\": \"%s\", \"clients\": %d, \"prfs\": %.0f, \"tt_ms\": %.3f, \"tt_G_PRF_s\": %.1f", S.name, K, prfs, a,
         prfs / (a * 1e-3) / 1e9);
  for (int v = 1; v < NV; ++v) {
    const double b = avg(tv[v]);
    printf(", \"%s\": {\"ms\": %.3f, \"G_PRF_s\": %.1f, \"over_tt\": %.3f, \"mismatch_tabT\": %llu, \"mismatch_cur\": %llu, "
           "\"mismatch_tab\": %llu}", kname[v], b, prfs / (b * 1e-3) / 1e9, a / b, (unsigned long long)bad[v][0],
           (unsigned long long)bad[v][1], (unsigned long long)bad[v][2]);
    total_bad += bad[v][0] + bad[v][1] + bad[v][2];
  }
  printf("}\n");
  return total_bad ? 1 : 0;
}
