/*
 * pm_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (wuwuz/Pacmann) hot path, used as the
 * parity checker for the MI355X product library (libpacmann.so).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  It is never linked into, or called by, the product path.
 *
 * Parity status: the reference is Go + Go assembly and no Go toolchain exists
 * in this image or on the GPU box, so the reference itself cannot be run.
 * This restatement is pinned by the reference's own known-answer tests and
 * properties (FIPS-197 AES KAT, OpenSSL AES, TestXORPerf KAT, the
 * TestInnerProduct closed-form sum, TestPIRBasic / TestBatchPIRBasic answer
 * properties incl. overflow-drop, and the parameter/accounting figures of
 * private-search-report.txt) — see tests/test_oracle_*.py and DESIGN.md §3.
 *
 * Randomness seams: the reference seeds keys and replacement offsets from
 * time.Now() and draws search randomness from Go's global math/rand.  Neither
 * stream is reproducible without Go, so both the oracle and the product use
 * the explicit counter-based streams specified in DESIGN.md §3.2
 * (pm_hash4 / splitmix64).  Everything else follows the reference
 * line by line (file:line cited at each function).
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- AES / PRF (pianopir/aes_amd64.s, pianopir/util.go) ---------------- */
void     or_expand_key(const uint8_t key[16], uint32_t rk[44]);
void     or_aes128_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]);
uint64_t or_prf(const uint32_t rk[44], uint64_t tag, uint64_t x);
void     or_prf_batch(const uint32_t rk[44], const uint64_t* tags, const uint64_t* xs,
                      size_t n, uint64_t* out);
void     or_xor_slices(uint64_t* dst, const uint64_t* src, size_t src_len);
void     or_derive_key(uint64_t seed, uint64_t partition, uint64_t epoch, uint8_t key[16]);
uint64_t or_hash4(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b, uint64_t c);

/* ---- distance (graphann/l2_distance_amd64.s, build_graph.go) ---------- */
float    or_l2dist(const float* a, const float* b, size_t dim);         /* L2Dist      */
float    or_l2dist_avx(const float* a, const float* b, size_t dim);     /* AVX restatement */
uint32_t or_inner_product(const uint32_t* a, const uint32_t* b, size_t n);
/* TestInnerProduct scan: vectors[i*D+j]=i+j, query[j]=j, sum over rows. */
uint32_t or_inner_product_bench(uint64_t N, uint64_t D, int nthreads);
uint32_t or_inner_product_scan(const uint32_t* rows, const uint32_t* q, uint64_t N, uint64_t D, int nthreads);
void     or_l2_batch(const float* q, const float* rows, size_t nrows, size_t dim, float* out);

/* ---- PianoPIR (pianopir/pir.go) ---------------------------------------- */
typedef struct or_pir or_pir;
typedef struct {
  uint64_t DBEntryByteNum, DBEntrySize, DBSize, ChunkSize, SetSize, ThreadNum, FailureProbLog2;
  uint64_t MaxQueryNum, PrimaryHintNum, MaxQueryPerChunk, FinishedQueryNum;
} or_pir_config;

or_pir*  or_pir_new(uint64_t DBSize, uint64_t DBEntryByteNum, const uint64_t* rawDB,
                    uint64_t FailureProbLog2, uint64_t seed, uint64_t partition);
void     or_pir_free(or_pir*);
void     or_pir_preprocessing(or_pir*);
/* hint-fold threads of Preprocessing (default 1): split over hints, identical state */
void     or_set_prep_threads(int n);
void     or_pir_dummy_preprocessing(or_pir*);
/* returns 0 ok, 1 budget exhausted, 2 chunk budget, 3 no hit hint, 4 idx out of range */
int      or_pir_query(or_pir*, uint64_t idx, int real, uint64_t* out);
int      or_server_private_query(or_pir*, const uint32_t* offsets, uint64_t* out);
void     or_pir_config_get(const or_pir*, or_pir_config*);
double   or_pir_local_storage(const or_pir*);
double   or_pir_comm_per_query(const or_pir*);
uint64_t or_pir_epoch(const or_pir*);
/* Export client state, buffers sized by the config (NULL to skip). */
void     or_pir_export(const or_pir*, uint32_t* round_keys,
                       uint64_t* primary_tag, uint64_t* primary_parity, uint64_t* primary_pp,
                       uint64_t* backup_tag, uint64_t* backup_parity,
                       uint64_t* repl_idx, uint64_t* repl_val, uint64_t* hist);

/* ---- SimpleBatchPianoPIR (pianopir/batch-pir.go) ---------------------- */
typedef struct or_batch or_batch;
typedef struct {
  uint64_t DBEntryByteNum, DBEntrySize, DBSize, BatchSize, PartitionNum, PartitionSize,
           ThreadNum, FailureProbLog2;
  uint64_t FinishedBatchNum, QueriesMadeInPartition, SupportBatchNum, PrepCount;
  double   LocalStorage, PreprocessingTime, CommOnline, CommOffline;
} or_batch_stats;

or_batch* or_batch_new(uint64_t DBSize, uint64_t DBEntryByteNum, uint64_t BatchSize,
                       const uint64_t* rawDB, uint64_t FailureProbLog2, uint64_t seed);
void     or_batch_free(or_batch*);
void     or_batch_preprocessing(or_batch*);
void     or_batch_dummy_preprocessing(or_batch*);
int      or_batch_query(or_batch*, const uint64_t* ids, size_t n, uint64_t* out);
void     or_batch_stats_get(const or_batch*, or_batch_stats*);
or_pir*  or_batch_subpir(or_batch*, uint64_t i);

/* ---- graphann search + PIRGraphInfo (search.go, private-search.go) ---- */
typedef struct or_graph or_graph;
or_graph* or_graph_new(uint64_t n, uint64_t dim, uint64_t m, const float* vectors,
                       const uint32_t* graph, int nonprivate, int skip_prep,
                       uint64_t pir_seed, uint64_t search_seed);
void     or_graph_free(or_graph*);
void     or_graph_preprocess(or_graph*);            /* GraphANNFrontend.Preprocess */
void     or_search_knn(or_graph*, const float* query, int k, int max_step, int parallel,
                       int benchmarking, int64_t* ids_out, int64_t* steps_out);
void     or_graph_counts(const or_graph*, uint64_t* total, uint64_t* succ);
or_batch* or_graph_pir(or_graph*);
/* private-search.go:220-233 query loop incl. maintenance trigger; times in s */
void     or_search_loop(or_graph*, const float* queries, uint64_t q, int k, int step,
                        int parallel, int benchmarking, int64_t* answers,
                        double* online_s, double* maintenance_s);

/* ---- graph construction (graphann/build_graph.go) --------------------- */
void or_knn(const float* base, uint64_t n, uint64_t dim, const float* queries, uint64_t nq, uint32_t k,
            int64_t* ids, float* dists);                 /* exact (L2Dist, id) top k */
void or_robust_prune(const float* X, uint64_t dim, uint64_t u, const uint32_t* cand, uint64_t n,
                     uint64_t m, float alpha, uint32_t* out, uint32_t* len);
int  or_build_graph(const float* X, uint64_t n, uint64_t dim, uint64_t m, float alpha, uint64_t seed,
                    uint32_t* graph);                    /* CreateGraphBasedOnNGT, exact kNN candidates */

#ifdef __cplusplus
}
#endif
