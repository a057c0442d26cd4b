// pm_internal.h — shared host/device definitions for libpacmann.so (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

// Device code sees the state pointers of PmPart / PmStep in the global address
// space, so their accesses lower to global_* instead of flat_* instructions
// (a flat access counts on lgkmcnt too: every later LDS wait would also wait
// for the outstanding global stores of the resolve chain).  Same layout on
// host and device (64-bit pointers).  Host-only translation units (the engine)
// define PM_HOST_TU so their device pass sees the plain host types.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PM_HOST_TU)
#define PM_G __attribute__((address_space(1)))
#else
#define PM_G
#endif

namespace pm {

constexpr uint32_t kDefaultProgramPoint = 0x7fffffffu;   // pir.go:15
constexpr uint64_t kDefaultValue = 0xdeadbeefULL;        // batch-pir.go:15
constexpr uint16_t kSkip = 0xffffu;                      // prep offset sentinel: backup hint's own chunk
constexpr int kBlock = 256;

// Randomness streams; identical spec to oracle/pm_oracle.cpp.
enum : uint64_t { DOM_KEY = 1, DOM_REPL = 2, DOM_DUMMY = 3, DOM_SYNTH_DB = 9, DOM_SYNTH_VEC = 10, DOM_SYNTH_NB = 11 };
__host__ __device__ inline uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t hash4(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b,
                                          uint64_t c) {
  uint64_t h = sm64(seed + dom);
  h = sm64(h ^ a);
  h = sm64(h ^ b);
  return sm64(h ^ c);
}

// The synthetic graph DB (pm_graph_create_synth; BIGANN-scale configs[3]/[4],
// where no graph can be built or shipped): the reference's synthetic mode
// (private-search.go:114-117,168-170: genRandomMatrix's uniform [0,1) f32
// vectors, genRandomGraph's uniform neighbour ids without self loops,
// :42-69) as a pure function of (seed, vertex), so a shard generates only its
// own rows and anyone can recompute any row.  u32 element e of vertex v's
// PIRGraphInfo entry (private-search.go:363-397: f32[dim] || u32[m]):
//   e <  dim: float((sm64(kv ^ (v*dim + e)) >> 40) * 2^-24)        (24 random bits, rand.Float32)
//   e >= dim: x = sm64(kg ^ (v*m + k) ^ (a << 56)) % n for a = 0, 1, ... until
//             x != v (k = e - dim; genRandomGraph redraws a self loop, so the
//             neighbours are uniform over the other n - 1 vertices)
// with kv = sm64(seed + DOM_SYNTH_VEC), kg = sm64(seed + DOM_SYNTH_NB).
__host__ __device__ inline float graph_synth_vec(uint64_t kv, uint64_t v, uint32_t dim, uint32_t j) {
  return (float)(sm64(kv ^ (v * dim + j)) >> 40) * 0x1.0p-24f;
}
__host__ __device__ inline uint32_t graph_synth_nb(uint64_t kg, uint64_t n, uint64_t v, uint32_t m, uint32_t k) {
  const uint64_t c = v * m + k;
  uint64_t x = sm64(kg ^ c) % n;
  for (uint64_t a = 1; x == v; ++a) x = sm64(kg ^ c ^ (a << 56)) % n;   // n > 1 (pm_graph_create_synth)
  return (uint32_t)x;
}
__host__ __device__ inline uint32_t graph_synth_elem(uint64_t kv, uint64_t kg, uint64_t n, uint32_t dim, uint32_t m,
                                                     uint64_t v, uint32_t e) {
  if (e < dim) return __builtin_bit_cast(uint32_t, graph_synth_vec(kv, v, dim, e));
  return graph_synth_nb(kg, n, v, m, e - dim);
}

// One PianoPIR instance ("partition") as the device sees it.  Parameters
// follow NewPianoPIR / NewPianoPIRClient (pir.go:130-175, 479-514).
// Hint index space h in [0, H): h < PH primary hints, h >= PH backup hint
// (g, j) with h = PH + g*Qpc + j (backupShortTag[g][j], pir.go:244-251).
struct PmPart {
  uint64_t N;        // DBSize of this sub-PIR
  uint64_t row0;     // first global DB row of this partition
  uint64_t seed;     // randomness seed (keys, replacement, dummy)
  uint64_t epoch;    // preprocessing epoch in use
  uint64_t idx;      // partition index (stream domain)
  uint32_t CS, log2CS, SS, PH, Qpc, H, MaxQ, curk;   // curk: chunks per hint-search block (cur_index)
  uint32_t rk[44];   // expanded AES-128 key (expandKeyAsm layout)
  // client state, device-resident
  PM_G uint32_t* tag;     // [H]   short tags (primary tags mutate on refresh)
  PM_G uint32_t* pp;      // [PH]  primaryProgramPoint
  PM_G uint64_t* parity;  // [H*E] primary parities then backup parities
  PM_G uint32_t* ridx;    // [SS*Qpc] replacementIdx
  PM_G uint64_t* rval;    // [SS*Qpc*E] replacementVal
  PM_G uint32_t* hist;    // [SS]  QueryHistogram
  PM_G uint32_t* fqn;     // [1]   FinishedQueryNum
  PM_G uint64_t* arena;   // [MaxQ*E] localCache rows (pir.go:120), slot = FinishedQueryNum at answer time
  // PRF table (only where the fold reads it, pmk::fold_needs_tab; else null):
  // tab[c*H + t] = PRF(tag t, chunk c) & (CS-1) for every tag t in
  // [0, H) and chunk c in [0, SS) (kSkip at a backup tag's own chunk).  Every
  // tag a hint can carry is a hint index (primary tags start at h, a refresh
  // hands over backup tag PH+g*Qpc+j), so this table, built once per
  // preprocessing, holds every PRF value the online phase needs.
  PM_G uint16_t* tab;
  PM_G uint16_t* tabT;    // the same table tag-major in tiles of 8 chunks (tabT_at): set expansion
                          // reads one tag's row; k_prep_offsets writes whole 16-B tiles
  // The hint search's table: entry (c, h) = PRF(current tag of primary hint
  // h, chunk c) & (CS-1), i.e. tab[c][tag[h]] kept in hint order, so matching
  // a (chunk, offset) streams chunk c's row of PH u16 instead of gathering
  // through the tags.  k_prep_offsets seeds it (tags are h); the final refresh
  // of a hint in a step rewrites its column from tabT[new tag] (pm_query.hip
  // refresh_cur).  Layout cur_index: chunk pairs interleaved in 16-B blocks.
  PM_G uint16_t* cur;
  // the search query this client's decoded rows are scored against (L2) when
  // several clients' steps share one launch (pm_search_loop_batched); null:
  // the step's PmStep::q
  const PM_G float* qv;
  // The partition's fold image (server-side, built once with the DB; null
  // where k_prep_fold_rot does not apply): per 32-B column slice s and group
  // of NCH chunks b (4 at CS 512, 2 at CS 1,024), the 64 KB LDS image
  // k_prep_fold_rot stages, line k = row k of chunks NCH b .. (rows past N
  // zero).  pmk::fold_image_words.
  const PM_G uint64_t* img;
};

// tabT layout: chunk c of tag t at tile (c / 8, t), element c % 8 (16-B tiles of
// 8 chunks; SetSize padded to a multiple of 8 with kSkip), so the writer of 8
// chunks x consecutive tags stores full lines instead of one 2-B store per line.
__host__ __device__ inline uint64_t tabT_index(uint32_t H, uint32_t t, uint32_t c) {
  return ((uint64_t)(c >> 3) * H + t) * 8 + (c & 7);
}
__host__ __device__ inline uint64_t tabT_words(uint32_t H, uint32_t SS) { return (uint64_t)((SS + 7) / 8) * 8 * H; }

// Hint-search table layout: [SS / 2][PH8 / 8][2][8] u16 (PH8 = PH rounded up
// to 8): block b of chunk c's row (hints 8b .. 8b + 7, one 16-B load) sits
// beside the same block of chunk c ^ 1.  A refresh writes a hint's entry of
// every chunk, i.e. one column: paired, its SS entries touch SS / 2 cache lines
// instead of SS (random line writes cost ~2.6 random line reads on MI355X:
// tools/gather_bench.hip regw_*), while a row's reads stay whole 16-B blocks
// (every other one: twice the row's bytes through L2).
#ifndef PM_CUR_K
#define PM_CUR_K 0   // chunks interleaved per 16-B hint block: 0 = chosen per partition (cur_k), else forced
#endif
// K chunks interleaved: a refresh writes SS / K lines, a search reads K x its
// row.  K = 2 unless the row (PH x 2 B) outweighs the column's lines (SS x
// 128 B): BIGANN-100M's 57,344-hint rows read twice cost the hint search more
// than the halved refresh saves (k_match_part8 34 -> 55 us per team step)
__host__ __device__ inline uint32_t cur_k(uint32_t PH, uint32_t SS) {
  return PM_CUR_K ? PM_CUR_K : ((uint64_t)PH * 2 > (uint64_t)SS * 128 ? 1u : 2u);
}
__host__ __device__ inline uint32_t cur_blocks(uint32_t PH) { return (PH + 7) >> 3; }
__host__ __device__ inline uint64_t cur_index(uint32_t PH, uint32_t K, uint32_t c, uint32_t h) {
  return K == 2 ? (((uint64_t)(c >> 1) * cur_blocks(PH) + (h >> 3)) * 2 + (c & 1)) * 8 + (h & 7)
                : (((uint64_t)(c / K) * cur_blocks(PH) + (h >> 3)) * K + (c % K)) * 8 + (h & 7);
}
// chunk c's row: hint h at row[cur_row_off(K, h)], block b (8 hints) at row + 8 K b
__host__ __device__ inline uint64_t cur_row(uint32_t PH, uint32_t K, uint32_t c) { return cur_index(PH, K, c, 0); }
__host__ __device__ inline uint32_t cur_row_off(uint32_t K, uint32_t h) { return (h >> 3) * 8 * K + (h & 7); }
__host__ __device__ inline uint64_t cur_words(uint32_t PH, uint32_t SS, uint32_t K) {
  return (uint64_t)((SS + K - 1) / K) * cur_blocks(PH) * 8 * K;
}

// Sub-query kinds / statuses for one batched step.
enum : uint32_t { SUB_NONE = 0, SUB_REAL = 1, SUB_DUMMY = 2, SUB_HOSTCACHE = 3 };
enum : uint32_t {
  ST_OK = 0, ST_EBUDGET = 1, ST_ECHUNK = 2, ST_ENOHIT = 3, ST_ERANGE = 4,
  ST_DUMMY = 8, ST_CACHED = 9, ST_DUP = 10, ST_SKIP = 11
};
struct PmSub {
  uint32_t part, kind;
  uint64_t idx;   // REAL: local index; DUMMY: dummy counter; HOSTCACHE: arena slot
};
// Per-sub-query resolution record written by k_resolve.
struct PmRes {
  uint32_t status, hit, chunk, ing;   // ing = in-group index (QueryHistogram before)
  uint32_t tag, pp;                   // hit hint's tag / program point used for the expansion
  uint32_t slot;                      // OK: arena slot; CACHED: arena slot; DUP: earlier sub
  uint32_t flags;                     // bit 0: hint refreshed earlier in this step (chained);
                                      // bit 1: a later sub-query in this step re-hits this hint
};
// Per-sub-query result header, written by the GPU into pinned host memory
// after the sub-query's row.  Stores to fine-grained host memory reach the
// host in no guaranteed order (measured: ~3e-5 of rows not yet complete when
// their token is first seen), and ordering them inside the kernel costs
// 2.8-4.4x the answer kernel's time (a system-scope L2 write-back per
// workgroup, or write-through stores).  So the token only says "answered";
// the host takes a step's results after the step's completion event, recorded
// with a system-scope release after the last kernel (pm_engine.cpp
// wait_step), which orders every byte.  The header also carries a
// multilinear hash of the row words the host reads ([pf_w0, pf_w1) of PmStep):
//   csum = token * kCsumMix + sum_w row[w] * row_hash_mult(w)   (mod 2^64)
// with odd multipliers, checked after completion as an assertion (and, with
// PM_PUBLISH_WAIT=0, as the token-time acceptance test: one stale word changes
// the sum by (new - old) * odd != 0; a stale header never matches).
constexpr uint64_t kCsumMix = 0x9E3779B97F4A7C15ull;
__host__ __device__ inline uint64_t row_hash_mult(uint64_t w) { return sm64(w ^ 0x5851F42D4C957F2Dull) | 1ull; }
struct alignas(16) PmOutHdr {
  uint32_t status, ref;
  float dist;
  uint32_t token;
  uint64_t csum, pad;
};
// Arguments of the step kernels (pm_query.hip).
#ifndef PM_KARG_SUBS
#define PM_KARG_SUBS 112
#endif
constexpr uint32_t kArgSubs = PM_KARG_SUBS, kArgParts = PM_KARG_SUBS > 1 ? 32 : 1;
// k_step gather helpers (PmStep::nhelp): at most kStepHelpMax per sub-query,
// for entries of <= 256 gathered words; granules per helper: 2 x 256 partial
// words + 8 guess fields
constexpr uint32_t kStepHelpMax = 3, kHelpWords = 256, kHelpGran = 2 * kHelpWords + 8;
struct PmStep {
  const PM_G PmPart* parts;
  const PM_G PmSub* subs_h;    // pinned host descriptor, read zero-copy by k_match
  const PM_G uint32_t* sb_h;   // sub_begin[np+1] (pinned host)
  PM_G PmSub* subs;            // device copies
  PM_G uint32_t* sb;
  PM_G uint64_t* bits;         // [nsub][words] hint-match bits (k_match -> k_resolve)
  PM_G uint32_t* cand;         // [nsub][cblk][6]: per k_match block its first two matches
                               // {hint, tag, program point} x 2 (hint kNone: none)
  PM_G PmRes* res;             // [nsub]
  PM_G uint64_t* ans;          // [nsub][E] raw answers of chained sub-queries
  PM_G uint32_t* done;         // [0..1] step completion counter (chain_add, pm_query.hip),
                               // [2] chained sub-queries, [3..] their list (filled by the
                               // resolvers; re-armed by each step's finisher)
  const PM_G uint64_t* db;
  const PM_G float* q;         // search query (device) or null
  PM_G PmOutHdr* hdr_h;        // pinned host outputs
  PM_G uint64_t* rows_h;
  PM_G uint64_t* stamps;       // PM_STAMPS diagnostic builds only: s_memtime per phase
  PM_G uint32_t* meta;         // [nsub][2]: chunk QueryHistogram, predicted in-chunk index
  PM_G uint32_t* spec;         // [nsub][64]: predicted re-evaluation values (k_match -> k_resolve)
  // k_step hand-off granules {value, token} (pm_query.hip put_g / get_g)
  PM_G uint64_t* recg;         // [kArgSubs][8] match record + prediction per sub-query
  PM_G uint64_t* specg;        // [kArgSubs][64] predicted re-evaluation values
  PM_G uint64_t* bitsg;        // [kArgSubs][words][2] match bits
  PM_G uint64_t* resg;         // [kArgSubs][8] resolution records
  // k_step gather helpers: nhelp extra workgroups per sub-query each gather a
  // range of the guessed set and hand over its partial XOR (granules: 2 per
  // word of the partial, then the guess fields); 0 = none
  PM_G uint64_t* helpg;        // [kArgSubs][kStepHelpMax][kHelpGran]
  uint32_t nhelp;
  PM_G uint32_t* err_h;        // pinned host: set when a hand-off spin timed out        // [np] k_step: token of the step whose results the resolver published
  uint32_t words, E, dim, nsub, np, cblk;
  uint32_t np_live;            // partitions with at least one sub-query in this step
  uint32_t pf_w0, pf_w1;       // row words the host reads (PmOutHdr::csum covers them)
  uint32_t rows_partial;       // 1: only words [pf_w0, pf_w1) of each result row are written to the host
  uint32_t no_guess;           // k_step diagnostics: answers wait for their resolution (PM_NO_GUESS=1)
  // Split gather (three-kernel path, wide sets): k_gather writes nsplit partial
  // XORs of each sub-query's set, [nsub][nsplit][E&~3]; k_answer folds them.
  uint32_t nsplit;             // 0/1: k_answer gathers its set itself
  PM_G uint64_t* part_x;
  // Query sets expanded by k_match_resolve_s ([nsub][qw] u16 offsets; qw = SetSize
  // rounded up to 8), read by k_answer with the resolution record; null: the
  // answer expands its set from tabT itself.
  PM_G uint16_t* qset;
  uint32_t qw;
  // Small steps ship the descriptor inside the kernel arguments (no PCIe
  // round trip); larger ones use subs_h / sb_h.
  uint32_t args_valid;
  uint32_t token;              // written into every PmOutHdr of this step
  uint32_t sb_a[kArgParts + 1];
  PmSub subs_a[kArgSubs];
};

// ---- the device-resident team round (pm_drl.hip; pm_search_loop_batched's
// device loop): a lock-step team's 20 rounds of SearchKNN +
// SimpleBatchPianoPIR.Query bucketing run on the GPU, chained on the team's
// stream, with the host touching only a query's start and end.
// the device loop's open-addressing tables (pm_drl.hip; the host builds the
// localCache table with the same probe sequence)
__host__ __device__ inline uint32_t drl_hash(uint32_t k) {
  uint64_t x = k;
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
  return (uint32_t)x;
}
struct DrlSess {          // one session's search state between launches
  uint64_t rng;           // SplitMix state (the host's id stream, SplitMix::next)
  uint64_t succ;          // successQueryNum (private-search.go:483-497)
  uint32_t nknown, nheap; // knownVertices / the min-heap's sizes
  uint32_t pad0, pad1;
};
enum : uint32_t { DRL_BEGIN = 0, DRL_MID = 1, DRL_END = 2 };
struct DrlArgs {
  uint32_t S, P, qn, n, m, parallel, k, E, dim, kcap, cmask, ns, mode, q, qi, seq;
  uint32_t vec16;                 // rows and neighbour lists 16-B aligned, m / 4 a power of two (vector decode)
  uint64_t N, PS;
  const PmOutHdr* hdr;            // the last shared step's results [nsub] (device)
  const uint64_t* rows;           // ... and rows [nsub][E] (the neighbour words only)
  PmSub* subs;                    // the next shared step's descriptor [S][P][qn]
  uint64_t* gid;                  // ... each sub-query's global id (~0: dummy)
  const uint32_t* graph;          // [N][m] the true neighbour lists (success check, start set)
  const float* start_dist;        // [S][ns] the start set's L2 distances to the query
  const uint32_t* start_ids;      // [S][ns]
  DrlSess* sess;                  // [S]
  uint64_t* dummy;                // [S][P] dummy-query counters (PartHost::dummy_ctr)
  uint32_t* batch;                // [S][n] the round's ids
  uint64_t* heap;                 // [S][kcap] {dist f32 bits | known slot << 32}
  uint64_t* ktab;                 // [S][2 kcap] knownVertices: {id + 1 | slot << 32}, 0 empty
  uint32_t* knb;                  // [S][kcap][m] known vertices' neighbour lists
  float* kdist;                   // [S][kcap]
  uint32_t* kid;                  // [S][kcap]
  uint64_t* const* ctab;          // [S] -> [P][cmask + 1] localCache: {local idx + 1 | arena slot << 32}
  int64_t* answers;               // [S][q][k]
  const double* part_bytes;       // [P] algorithmic answer bytes of one sub-query
  double* step_bytes;             // [launch seq][S] (timing runs; null: not counted)
  uint32_t* step_real;            // [launch seq][S] real sub-queries (timing runs)
  uint64_t* stamps;               // diagnostics (PM_DRL_STAMPS): [16] summed shader clocks per phase of MID rounds
};

}  // namespace pm

// Kernel launchers (pm_kernels.hip).  All asynchronous on `st`.
namespace pmk {
using namespace pm;
void prep_init(hipStream_t st, const PmPart* dparts, int nparts, uint32_t maxH, uint32_t maxRepl,
               uint32_t E, bool zero_state);
void prep_offsets(hipStream_t st, const PmPart* dparts, int nparts, uint32_t maxH, uint32_t maxSS);
// the PRF tables' AES form: 0 = T-table (k_prep_offsets, default), 1 = bitsliced on the
// VALU (k_prep_offsets_bs, pm_aes_bs.h; profiles/r06/aes: 0.93x), -1 = PM_AES_BS's value
void set_aes_bs(int v);
// dparts: `clients` clients of each partition, partition-major (nparts = partitions x clients)
// returns the fold kernel launched (FOLD_*)
enum : int { FOLD_OTHER = 0, FOLD_ROT512 = 1, FOLD_ROT1024 = 2 };
int prep_fold(hipStream_t st, const PmPart* dparts, int nparts, uint32_t maxH, const uint64_t* db,
              uint32_t E, uint32_t minCS, uint32_t maxCS, const uint64_t* zero16, uint32_t clients = 1,
              bool have_img = false, uint32_t minH = 0);
void prep_repl(hipStream_t st, const PmPart* dparts, int nparts, uint32_t maxRepl,
               const uint64_t* db, uint32_t E);
// The bank-rotated fold's DB image (CS 512, even E, E >= 4): whether it applies,
// its size per partition (words) and the build of one partition's image.
bool fold_image_ok(uint32_t minCS, uint32_t maxCS, uint32_t E);
// whether the fold of these shapes reads the chunk-major PRF table PmPart::tab
// (otherwise it is not allocated: every other reader uses tabT)
bool fold_needs_tab(uint32_t minCS, uint32_t maxCS, uint32_t E, bool have_img);
uint64_t fold_image_words(uint32_t SS, uint32_t E, uint32_t CS);
void fold_image(hipStream_t st, uint64_t* img, const uint64_t* part_rows, uint64_t N, uint32_t SS, uint32_t E,
                uint32_t CS);
// Timing events carried by a launch's own dispatch packet (null: untimed)
struct PmEvents { hipEvent_t a = nullptr, b = nullptr; };
// pm_set_option: the hint-search path selectors ("match_part" -1 auto / 0 / 1,
// "match_part8" 0 / 1, "match_resolve" 0 / 1 / 2); -2 restores the environment's
// choice (PM_MATCH_PART, PM_MATCH_PART8, PM_MATCH_RESOLVE).  Returns -1 for an
// unknown name.
int set_option(const char* name, int value);
// The selectors' values for one step (read once per step and passed to every
// selector below, so one step never mixes two settings).
struct StepOpts { int match_part, match_part8, match_resolve; };
StepOpts step_opts();
// ph8: every partition's PH is a multiple of 8 (k_match_part8).  Returns the
// hint-search kernel launched.
enum : int { MATCH_SUB = 0, MATCH_PART = 1, MATCH_PART8 = 2 };
int step_match(hipStream_t st, const PmStep& S, const StepOpts& O, bool ph8, uint32_t maxPH,
               uint32_t max_sub_per_part, PmEvents ev = {});
uint32_t step_match_blocks(uint32_t maxPH);   // k_match workgroups per sub-query
void step_resolve(hipStream_t st, const PmStep& S, bool lds, PmEvents ev = {});
// k_match_part + k_resolve fused (batched serving; descriptor already in device memory)
bool step_match_resolve_ok(const PmStep& S, const StepOpts& O, bool lds);
bool step_match_resolve_small(const StepOpts& O, bool ph8, uint32_t maxPH, uint32_t max_sub_per_part);
// ph8: every partition's PH is a multiple of 8
void step_match_resolve(hipStream_t st, const PmStep& S, const StepOpts& O, bool ph8, uint32_t maxPH,
                        uint32_t max_sub_per_part, PmEvents ev = {});
// k_step: match, resolve and answer in one launch (descriptor in the kernel
// arguments, <= 64 sub-queries and <= 8192 hints per partition, <= 256 workgroups)
bool step_fused_ok(const PmStep& S, uint32_t maxPH, uint32_t max_sub_per_part);
void step_fused(hipStream_t st, const PmStep& S, PmEvents ev = {});
bool step_resolve_lds_ok(uint32_t maxPH, uint32_t max_sub_per_part);
// k_match_resolve_s writes the query sets for the answer (PmStep::qset); S.nsplit set
bool step_qset_ok(const PmStep& S, const StepOpts& O, bool lds, bool ph8, uint32_t maxPH,
                  uint32_t max_sub_per_part, uint32_t maxSS);
void step_answer(hipStream_t st, const PmStep& S, uint32_t maxSS, PmEvents ev = {});
// Split gather ahead of k_answer for wide query sets (SetSize >= 256, BIGANN
// scale): how many workgroups per sub-query (1: no split), and the launch.
uint32_t step_gather_split(uint32_t maxSS, uint32_t nsub);
void step_gather(hipStream_t st, const PmStep& S, PmEvents ev = {});
uint32_t step_max_sub_per_part();
uint32_t step_max_ss();
uint32_t step_max_e();
void server_answer(hipStream_t st, const PmPart* dpart, const uint32_t* offs, uint32_t nq,
                   uint32_t SS, const uint64_t* db, uint32_t E, uint64_t* out);
void l2_rows(hipStream_t st, const float* rows, uint64_t row_stride_floats, uint64_t nrows,
             const uint32_t* row_ids, const float* q, uint32_t dim, float* out, uint64_t seglen = 0);
void ip_rows(hipStream_t st, const uint32_t* rows, uint64_t nrows, const uint32_t* q, uint32_t dim,
             uint32_t* per_row, uint32_t* sum);
void ip_fill(hipStream_t st, uint32_t* rows, uint64_t N, uint32_t D, uint64_t r0 = 0);   // rows r0 .. r0 + N
// Synthetic DB rows (pm_batchpir_create_synth): dst row i = global row r0 + i,
// word w = sm64(sm64(db_seed + DOM_SYNTH_DB) ^ (r * E + w)).
void db_synth(hipStream_t st, uint64_t* dst, uint64_t r0, uint64_t rows, uint32_t E, uint64_t db_seed);
// out[i] = {E words at src[i] (or zeros when null), success flag}, src in pinned host memory
void gather_rows(hipStream_t st, const uint64_t* const* src, uint64_t n, uint32_t E, uint64_t* out);
// ---- sharded private search (pm_shard.hip) ----
// Synthetic graph DB rows (graph_synth_elem): dst row i = global vertex r0 + i,
// E = (dim + m) / 2 words per row.
void graph_synth(hipStream_t st, uint64_t* dst, uint64_t r0, uint64_t rows, uint64_t n, uint32_t dim, uint32_t m,
                 uint64_t seed);
// out[i*dim + j] = vector of vertex ids[i] (the start set, GetStartVertex)
void graph_synth_vecs(hipStream_t st, const uint64_t* ids, uint64_t nids, uint32_t dim, uint64_t seed, float* out);
// Per-id records of a shared step for the shards' combine.  Record r (session
// s = r / npos, position r % npos of its GetVertexInfo batch) = the W - 1 row
// words [w0, w0 + W - 1) of its answer (the neighbour list) and one word
// {dist f32 bits | ok << 32}; map[r] = the answering sub-query of the step
// (a DUP followed to its source) or < 0 (no local answer: zeros).  Also
// st2[j] = {status, ref} of every sub-query j < nsub (the host's mirrors), and
// the error word rec[nrec * W] = errw (0, or 1 from a failed rank: group_exchange).
void pack_records(hipStream_t st, const int32_t* map, uint32_t nrec, const PmOutHdr* hdr, const uint64_t* rows,
                  uint32_t E, uint32_t w0, uint32_t W, uint64_t* rec, uint32_t nsub, uint32_t* st2, uint64_t errw);
// Modelled peers (a shard layout wider than the job): records with map[r] ==
// -2 are those another shard of the layout answers; they are filled from the
// synthetic graph's spec, the distance to session r / npos's query (qbuf) in
// the reference's L2 order (l2_distance_amd64.s:4-36).
void synth_records(hipStream_t st, const int32_t* map, const uint64_t* ids, uint32_t nrec, uint32_t npos,
                   const float* qbuf, uint32_t dim, uint32_t m, uint64_t n, uint64_t seed, uint32_t w0, uint32_t W,
                   uint64_t* rec);
void prf_batch(hipStream_t st, const uint32_t* rk, const uint64_t* tags, const uint64_t* xs,
               uint64_t n, uint64_t* out);
// the device-resident team round (pm_drl.hip): one 64-lane workgroup per session
void team_round(hipStream_t st, const DrlArgs& A, PmEvents ev = {});
uint32_t team_round_lds(uint32_t kcap, uint32_t n, uint32_t m);   // bytes of dynamic LDS
constexpr uint32_t kDrlMaxKcap = 4096, kDrlMaxN = 256, kDrlMaxNM = 8192, kDrlMaxParallel = 8;
// graph construction and ground truth (pm_graph.hip)
uint32_t knn_pad_dim(uint32_t dim);   // bf16 row width for the prefilter (0: unsupported)
uint32_t knn_top();                   // prefilter candidates per query row
uint32_t prune_max_list();
uint32_t prune_max_dim();
uint32_t prune_max_m();
void to_bf16(hipStream_t st, const float* rows, uint64_t n, uint32_t dim, uint32_t dp, void* out, float* norms);
void knn_prefilter(hipStream_t st, const void* X, const float* xn, uint64_t N, const void* Q, const float* qn,
                   uint64_t M, uint32_t dp, uint32_t* out);
void knn_rerank(hipStream_t st, const float* X, uint64_t N, uint32_t dim, const float* Q, uint64_t M,
                const uint32_t* cand, uint32_t K, bool self_base, uint32_t* out, float* dist, uint32_t* len);
void prune(hipStream_t st, const float* X, uint32_t dim, const uint32_t* verts, uint64_t nverts,
           const uint64_t* offs, uint64_t stride, const uint32_t* lens, const uint32_t* ids, uint32_t m,
           float alpha, uint32_t* out, uint32_t* out_len, uint32_t* err, const uint32_t* sorted_pos = nullptr,
           const float* dist_g = nullptr);
// L2Dist of every candidate of the listed vertices (hub lists above prune_max_list())
void cand_dist(hipStream_t st, const float* X, uint32_t dim, const uint32_t* verts, uint64_t nverts,
               const uint64_t* offs, const uint32_t* lens, const uint32_t* ids, float* dist_g);
}  // namespace pmk
