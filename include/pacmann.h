/*
 * pacmann.h — C ABI of libpacmann.so, the MI355X (gfx950) implementation of
 * Pacmann's two data-parallel inner loops (wuwuz/Pacmann):
 *
 *   1. PianoPIR: AES-128-MMO PRF set expansion + 64-bit XOR database fold
 *      (client hint preprocessing, server answer, online hint search and
 *      refresh, 16-way batch PIR), bit-exact with the pianopir Go code + aes_amd64.s.
 *   2. graphann: batched L2 / uint32 inner-product distance evaluation that
 *      drives the degree-m beam search, bit-exact with l2_distance_amd64.s.
 *
 * The entry points replace the reference's Go package surfaces at method /
 * batch granularity (never per PRF or per 640-B XOR: a launch per leaf would
 * cost more than the Go assembly it replaces).  Each function cites the
 * reference interface it stands in for.  All pointers are HOST pointers;
 * device memory is owned by the library behind opaque handles.  Input host
 * buffers are copied and never retained; output buffers are caller-allocated.
 * Every function returns 0 on success or a negative PM_E* code; the message
 * is in pm_last_error() (thread-local).  The library never aborts the process
 * (the reference's log.Fatalf paths return PM_EINVAL instead).
 *
 * Threading: one handle per host thread; handles are not thread-safe (the
 * reference's PianoPIRClient is not either, pir.go:91-121).
 */
#ifndef PACMANN_H
#define PACMANN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_OK 0
#define PM_EINVAL -1   /* bad argument / reference log.Fatalf condition   */
#define PM_EHIP -2     /* HIP runtime error                              */
#define PM_ENOMEM -3   /* device allocation failed                       */
#define PM_ETIMEDOUT -4 /* a bounded wait expired (RCCL peer never joined) */

/* Per-sub-query status codes (pianopir/pir.go:354-471 error returns). */
#define PM_Q_OK 0          /* answered through PIR                             */
#define PM_Q_EBUDGET 1     /* "exceed the maximum number of queries" :386-391  */
#define PM_Q_ECHUNK 2      /* "too many queries in chunk" :396-400             */
#define PM_Q_ENOHIT 3      /* "no hit hint in the primary hint table" :416-419 */
#define PM_Q_ERANGE 4      /* idx out of range (:373-378 log.Fatalf)           */

typedef struct pm_ctx pm_ctx;
typedef struct pm_pir pm_pir;           /* PianoPIR             (pir.go:473-477)       */
typedef struct pm_batchpir pm_batchpir; /* SimpleBatchPianoPIR  (batch-pir.go:40-53)   */
typedef struct pm_graph pm_graph;       /* GraphANNFrontend + PIRGraphInfo / BasicGraphInfo */

/* ---- context ----------------------------------------------------------- */
int         pm_ctx_create(int device, pm_ctx** out);
void        pm_ctx_destroy(pm_ctx* ctx);
const char* pm_last_error(void);
int         pm_ctx_sync(pm_ctx* ctx);
/* Free and total device memory of the context's GPU (bytes; sizing how many
 * client sessions a GPU holds next to its DB). */
int         pm_ctx_mem_info(pm_ctx* ctx, uint64_t* free_bytes, uint64_t* total_bytes);
/* Per-kernel timing.  Level 1: HIP events around the preprocessing and leaf
 * kernels on the stream they run on ("prep_offsets", "prep_fold",
 * "prep_repl", "l2_rows", "ip_scan", "prf", server "answer").  Level 2 also
 * times the kernels of every online step ("step", "hint_match", "resolve",
 * "gather", "answer") with events carried in their own dispatch packets
 * (hipExtLaunchKernelGGL); steps are not synchronised for it (the events are
 * read by pm_timing_get).  Level 3 is level 2 with the kernels of a lock-step
 * team's shared steps timed on every 7th step of its stream only (the serving
 * bench: a sample, at a fraction of the events' cost).  Host wall-clock
 * accumulators are always on: "host_step_launch", "host_step_wait",
 * "host_step_post", "host_batch_query", "host_gvi_parse", "host_search_knn",
 * "host_knn_init", "host_knn_batch", "host_knn_update", "host_knn_final". */
int pm_timing_enable(pm_ctx* ctx, int level);
/* "rccl_timeout_s": the bound (seconds) on RCCL communicator creation and
 * its probe (pm_rccl_create / pm_rccl_probe); "verify_records" (sharded loop):
 * check every value-th shared step's records on the host.
 * Process-wide choice among equivalent kernel paths (no reference counterpart:
 * the same results by every path; tests drive each one).  "match_part": the
 * hint search per (partition, block) instead of per (sub-query, block), -1
 * automatic / 0 / 1; "match_part8": its one-wave-per-block form where PH % 8 ==
 * 0, 0 / 1; "match_resolve": k_match_resolve* for search-sized steps, 0 / 1 /
 * 2 (the general form).  -2 restores the environment's choice (PM_MATCH_PART,
 * PM_MATCH_PART8, PM_MATCH_RESOLVE).  "aes_bs": the preprocessing's PRF tables
 * by the bitsliced VALU AES (1) or the T-table AES (0, default; -1: PM_AES_BS).
 * "device_loop": the batched serving loop on the device (1 / 0; -1 automatic).
 * "fault_drl_query" (tests): the device loop fails before queueing query
 * `value` (-1 off); its sessions are then unusable (every later call on them
 * returns PM_EINVAL: their host counters no longer match the device state).
 * PM_EINVAL for an unknown name. */
int pm_set_option(const char* name, int value);
int pm_timing_reset(pm_ctx* ctx);
/* Diagnostics: append one line "kernel,start_us,end_us,ctx" per timed launch
 * of ctx (level >= 2 timing) to the file at `path`, on one time axis for every
 * context of the process (the GPU timeline of a serving run). */
int pm_timing_timeline(pm_ctx* ctx, const char* path);
int pm_timing_get(pm_ctx* ctx, const char* kernel, uint64_t* launches, double* total_ms,
                  double* alg_bytes);

/* ---- leaf primitives, batched ----------------------------------------- */
/* expandKeyAsm (pianopir/aes_amd64.s:87-126): FIPS-197 AES-128 key schedule. */
int pm_expand_key(const uint8_t key[16], uint32_t round_keys[44]);
/* PRFEvalWithLongKeyAndTag (pianopir/util.go:157-165) over n (tag, x) pairs on
 * the GPU: out[i] = low64_LE(AES_k(B) ^ B), B = LE64((tag<<35)+x) || 0^8. */
int pm_prf_batch(pm_ctx* ctx, const uint32_t round_keys[44], const uint64_t* tags,
                 const uint64_t* xs, uint64_t n, uint64_t* out);
/* L2Dist (graphann/build_graph.go:119-127 -> l2_distance_amd64.s:4-36) of one
 * query against nrows rows (row-major nrows x dim), bit-exact. */
int pm_l2_batch(pm_ctx* ctx, const float* query, const float* rows, uint64_t nrows,
                uint64_t dim, float* out);
/* InnerProduct (l2_distance_amd64.s:39-68) of one query against nrows rows:
 * per-row uint32 dot products mod 2^32 (per_row may be NULL) and their
 * wrapping sum. */
int pm_ip_batch(pm_ctx* ctx, const uint32_t* query, const uint32_t* rows, uint64_t nrows,
                uint64_t dim, uint32_t* per_row, uint32_t* sum);
/* TestInnerProduct scan (graphann/graphann_test.go:249-283) fully on device:
 * fills vectors[i*D+j] = i+j in HBM, query[j] = j, then sums the N row dot
 * products mod 2^32.  scan_ms = device time of the scan kernel alone. */
int pm_ip_bench(pm_ctx* ctx, uint64_t N, uint64_t D, uint32_t* sum, double* scan_ms);
/* The same scan over rows [r0, r0 + rows) of the N-row fill: one GPU's shard
 * of the row-sharded scan (scans shard by rows, the mod-2^32
 * partial sums add up to TestInnerProduct's sum).  r0 + rows <= N. */
int pm_ip_bench_shard(pm_ctx* ctx, uint64_t N, uint64_t D, uint64_t r0, uint64_t rows, uint32_t* sum,
                      double* scan_ms);

/* ---- PianoPIR (pianopir/pir.go) --------------------------------------- */
typedef struct {
  uint64_t DBEntryByteNum, DBEntrySize, DBSize, ChunkSize, SetSize, ThreadNum, FailureProbLog2;
  uint64_t MaxQueryNum, PrimaryHintNum, MaxQueryPerChunk, FinishedQueryNum;
} pm_pir_config;

/* NewPianoPIR(DBSize, DBEntryByteNum, rawDB, FailureProbLog2) (pir.go:479-514).
 * seed drives the key / replacement / dummy streams that the
 * reference draws from time-seeded math/rand (pir.go:132,208,305,366). */
int    pm_pir_create(pm_ctx* ctx, uint64_t DBSize, uint64_t DBEntryByteNum, const uint64_t* rawDB,
                     uint64_t FailureProbLog2, uint64_t seed, pm_pir** out);
void   pm_pir_destroy(pm_pir* h);
int    pm_pir_preprocessing(pm_pir* h);          /* PianoPIR.Preprocessing      pir.go:516-518 */
int    pm_pir_dummy_preprocessing(pm_pir* h);    /* PianoPIR.DummyPreprocessing pir.go:520-523 */
/* PianoPIR.Query(idx, realQuery) (pir.go:525-533); *status = PM_Q_* */
int    pm_pir_query(pm_pir* h, uint64_t idx, int real, uint64_t* out, int* status);
int    pm_pir_config_get(pm_pir* h, pm_pir_config* cfg);   /* PianoPIR.Config  pir.go:546-548 */
double pm_pir_local_storage(pm_pir* h);                    /* LocalStorageSize pir.go:178-190 */
double pm_pir_comm_per_query(pm_pir* h);                   /* CommCostPerQuery pir.go:539-544 */
/* PianoPIRServer.PrivateQuery (pir.go:65-88), batched: nq offset sets of
 * SetSize uint32 each -> nq entries of DBEntrySize words. */
int    pm_pir_server_answer(pm_pir* h, const uint32_t* offsets, uint64_t nq, uint64_t* out);

/* ---- SimpleBatchPianoPIR (pianopir/batch-pir.go) ---------------------- */
typedef struct {
  uint64_t DBEntryByteNum, DBEntrySize, DBSize, BatchSize, PartitionNum, PartitionSize,
           ThreadNum, FailureProbLog2;
  uint64_t FinishedBatchNum, QueriesMadeInPartition, SupportBatchNum, PrepCount;
  double   LocalStorage, PreprocessingTime, CommOnline, CommOffline;
} pm_batchpir_stats;

/* NewSimpleBatchPianoPIR (batch-pir.go:55-93) */
int  pm_batchpir_create(pm_ctx* ctx, uint64_t DBSize, uint64_t DBEntryByteNum, uint64_t BatchSize,
                        const uint64_t* rawDB, uint64_t FailureProbLog2, uint64_t seed,
                        pm_batchpir** out);
/* One shard of the same batch PIR for multi-GPU use: this
 * handle keeps the DB slice, keys and hint state of the partitions p with
 * p % nshards == shard only (rawDB is still the whole DB; only those rows are
 * uploaded).  Bucketing, dummies, drops, counters and the re-preprocessing
 * trigger are the global ones, so every shard, fed the same batches, makes the
 * same decisions; pm_batchpir_query(_ok) fills the entries of its own
 * partitions and leaves the others zero (ok = 0).  Summing the entries (and
 * OR-ing ok) over all shards gives the unsharded answer bit for bit (keys
 * derive from the global partition index). */
int  pm_batchpir_create_shard(pm_ctx* ctx, uint64_t DBSize, uint64_t DBEntryByteNum, uint64_t BatchSize,
                              const uint64_t* rawDB, uint64_t FailureProbLog2, uint64_t seed,
                              uint32_t shard, uint32_t nshards, pm_batchpir** out);
/* The same shard over a synthetic DB generated on the device (BIGANN-scale
 * benchmarks, BASELINE.json configs[3]/[4]: tens of GB never cross PCIe).  It
 * replaces the reference's in-process random DB of TestBatchPIRPerf
 * (pir_test.go:204-275).  Word w of global row r is
 *   sm64(sm64(db_seed + 9) ^ (r * DBEntrySize + w)),
 * sm64 = the splitmix64 finalizer of (x + 0x9e3779b97f4a7c15),
 * so a caller can recompute any row to check an answer. */
int  pm_batchpir_create_synth(pm_ctx* ctx, uint64_t DBSize, uint64_t DBEntryByteNum, uint64_t BatchSize,
                              uint64_t FailureProbLog2, uint64_t seed, uint64_t db_seed, uint32_t shard,
                              uint32_t nshards, pm_batchpir** out);
/* Another client of the same server (multi-session serving, SURVEY.md §8f
 * rank 2): a new SimpleBatchPianoPIR client (own keys from `seed`, own hint
 * state, counters and local cache) whose server side reads the DB rows of
 * `server` in place (one device copy of the DB for all its clients; the
 * reference's server likewise keeps one rawDB alias, pir.go:34-39).  Same
 * DBSize, entry size, BatchSize, FailureProbLog2 and shard as `server`; same
 * device as `ctx`.  The DB stays alive while any client holds it. */
int  pm_batchpir_create_client(pm_ctx* ctx, pm_batchpir* server, uint64_t seed, pm_batchpir** out);
void pm_batchpir_destroy(pm_batchpir* h);
int  pm_batchpir_preprocessing(pm_batchpir* h);         /* batch-pir.go:119-155 */
int  pm_batchpir_dummy_preprocessing(pm_batchpir* h);   /* batch-pir.go:157-166 */
/* Query (batch-pir.go:170-248): out = n x DBEntrySize words; dropped or failed
 * ids get an all-zero entry exactly like the reference. */
int  pm_batchpir_query(pm_batchpir* h, const uint64_t* ids, uint64_t n, uint64_t* out);
/* The same query with a per-id success mask: ok[i] = 1 when entry i is the
 * answer of a successful sub-query (or its local-cache copy), 0 when the id
 * was dropped by the bucketing (batch-pir.go:195-200) or its sub-query failed
 * (the error batch-pir.go:205 swallows); those entries are zero. */
int  pm_batchpir_query_ok(pm_batchpir* h, const uint64_t* ids, uint64_t n, uint64_t* out, uint8_t* ok);
/* The same query with the responses left in DEVICE memory, for an in-place
 * collective over the shards (the multi-GPU combine, SURVEY.md §8e;
 * replaces the host round trip of Query's [][]uint64 result, batch-pir.go:
 * 216-236): dev_out is a device pointer on this handle's GPU of
 * n x (DBEntrySize + 1) uint64 words; row i holds id i's entry and, in word
 * DBEntrySize, 1 when it is a successful answer (pm_batchpir_query_ok's flag)
 * or 0 (entry zero).  Entries are copied HBM to HBM from the partitions'
 * local caches.  stream: a HIP stream (hipStream_t) of the consumer, made to
 * wait for the rows without a host synchronisation; NULL: the rows are written
 * when the call returns. */
int  pm_batchpir_query_dev(pm_batchpir* h, const uint64_t* ids, uint64_t n, uint64_t* dev_out, void* stream);
int  pm_batchpir_stats_get(pm_batchpir* h, pm_batchpir_stats* s);
/* Many clients of one server answered together (batched serving, SURVEY.md
 * §8f rank 2): every pm_batchpir_group_query call makes, for each client s,
 * exactly the SimpleBatchPianoPIR.Query (batch-pir.go:170-248) call of its batch
 * ids[s*n .. s*n+n), with all clients' sub-queries in ONE shared step over
 * S x 16 partitions (on clients[0]'s stream).  out: S x n x DBEntrySize words,
 * ok (nullable): S x n success flags, as pm_batchpir_query_ok.  Clients: the
 * server and/or pm_batchpir_create_client handles of one server. */
typedef struct pm_batchpir_group pm_batchpir_group;
int  pm_batchpir_group_create(pm_batchpir** clients, uint32_t S, pm_batchpir_group** out);
int  pm_batchpir_group_query(pm_batchpir_group* g, const uint64_t* ids, uint64_t n, uint64_t* out, uint8_t* ok);
/* SimpleBatchPianoPIR.Preprocessing (batch-pir.go:119-155) of every client of
 * the group as ONE launch set on clients[0]'s stream: each partition's clients
 * are folded side by side over the shared DB (the batched serving loop's
 * maintenance).  Every client's state equals its own pm_batchpir_preprocessing. */
int  pm_batchpir_group_preprocessing(pm_batchpir_group* g);
void pm_batchpir_group_destroy(pm_batchpir_group* g);
int  pm_batchpir_subconfig(pm_batchpir* h, uint64_t partition, pm_pir_config* cfg);

/* State export of one partition's client (test hook; sizes from the config):
 * round_keys[44], primary_tag[PH], primary_parity[PH*E], primary_pp[PH],
 * backup_tag[SS*Qpc], backup_parity[SS*Qpc*E], repl_idx[SS*Qpc],
 * repl_val[SS*Qpc*E], hist[SS].  Any pointer may be NULL. */
int pm_pir_export(pm_pir* h, uint32_t* round_keys, uint64_t* primary_tag, uint64_t* primary_parity,
                  uint64_t* primary_pp, uint64_t* backup_tag, uint64_t* backup_parity,
                  uint64_t* repl_idx, uint64_t* repl_val, uint64_t* hist);
int pm_batchpir_export(pm_batchpir* h, uint64_t partition, uint32_t* round_keys,
                       uint64_t* primary_tag, uint64_t* primary_parity, uint64_t* primary_pp,
                       uint64_t* backup_tag, uint64_t* backup_parity, uint64_t* repl_idx,
                       uint64_t* repl_val, uint64_t* hist);

/* ---- graphann (graphann/search.go) over PIRGraphInfo (private-search.go) */
/* PIRGraphInfo{N,Dim,M,graph,vectors,skipPrep,NonPrivateMode} (private-search.go:336-353)
 * wrapped in a GraphANNFrontend (search.go:69-72).  vectors: n x dim f32,
 * graph: n x m uint32.  nonprivate=1 gives BasicGraphInfo-style direct access
 * (private-search.go:445-455).  search_seed drives the host id stream that the
 * reference draws from global math/rand. */
int  pm_graph_create(pm_ctx* ctx, uint64_t n, uint64_t dim, uint64_t m, const float* vectors,
                     const uint32_t* graph, int nonprivate, int skip_prep, uint64_t pir_seed,
                     uint64_t search_seed, pm_graph** out);
void pm_graph_destroy(pm_graph* g);
int  pm_graph_preprocess(pm_graph* g);   /* GraphANNFrontend.Preprocess  search.go:74-81 */
/* GraphANNFrontend.SearchKNN (search.go:114-234); ids/steps: k entries, -1 padded */
int  pm_search_knn(pm_graph* g, const float* query, int k, int max_step, int parallel,
                   int benchmarking, int64_t* ids, int64_t* steps);
/* private-search.go:216-240 query loop incl. the maintenance trigger (:226-232) */
int  pm_search_loop(pm_graph* g, const float* queries, uint64_t q, int k, int step, int parallel,
                    int benchmarking, int64_t* answers, double* online_s, double* maintenance_s);
int  pm_graph_counts(pm_graph* g, uint64_t* total_queries, uint64_t* succ_queries);
/* A further client session over a preprocessed `base` (same graph, vectors and
 * server DB, shared on the device): own context/stream, PIR keys (pir_seed),
 * hint state, start set and id stream (search_seed).  Call pm_graph_preprocess
 * on it (client hint preprocessing + GetStartVertex) before searching. */
int  pm_graph_create_session(pm_ctx* ctx, pm_graph* base, uint64_t pir_seed, uint64_t search_seed,
                             pm_graph** out);
/* S sessions served concurrently on one GPU, one host thread each: session i
 * runs the private-search.go:216-240 loop (incl. its own maintenance trigger)
 * over queries[i*q*dim ...] into answers[i*q*k ...].  wall_s: wall time from the
 * common start to the last session's end; online_s / maintenance_s: S entries. */
int  pm_search_loop_sessions(pm_graph** sessions, uint32_t S, const float* queries, uint64_t q, int k,
                             int step, int parallel, int64_t* answers, double* wall_s, double* online_s,
                             double* maintenance_s);
/* The same sessions in lock-step with every batch-PIR round of all of them
 * fused into ONE shared step (k_match -> k_resolve ->
 * k_answer over S x 16 partitions, launched on sessions[0]'s stream): each
 * session keeps its own keys, hint state, cache, counters, search and
 * maintenance (private-search.go:216-240), and gets exactly the answers it
 * would get alone.  Sessions: clients of one server DB on one device (base +
 * pm_graph_create_session), distinct contexts.  ngroups (0: 1) lock-step
 * groups of consecutive sessions run concurrently, each with its own shared
 * steps on its first session's stream, so one group's step overlaps the
 * others' host work; nthreads host workers in all (0: min(S, 16)) run the
 * sessions' searches between the steps.  Outputs as pm_search_loop_sessions;
 * online_s[i] = wall_s - maintenance_s[i]. */
int  pm_search_loop_batched(pm_graph** sessions, uint32_t S, const float* queries, uint64_t q, int k, int step,
                            int parallel, uint32_t ngroups, uint32_t nthreads, int64_t* answers, double* wall_s,
                            double* online_s, double* maintenance_s);
pm_batchpir* pm_graph_pir(pm_graph* g);

/* ---- the GetGraphInfo plugin surface (graphann/search.go:20-25) ---------
 * PIRGraphInfo's methods as batch calls, for a caller that keeps its own beam
 * search (graphann.SearchKNN) and plugs the GPU in behind GetGraphInfo:
 *   pm_graph_preprocess       Preprocess()       private-search.go:355-412
 *   pm_graph_get_metadata     GetMetadata()      private-search.go (n, dim, m)
 *   pm_graph_get_vertex_info  GetVertexInfo(ids) private-search.go:441-506
 *   pm_graph_get_start_vertex GetStartVertex()   private-search.go:508-531
 * pm_graph_get_vertex_info fetches every id through the batch PIR
 * (SimpleBatchPianoPIR.Query, one call per batch) and decodes the entries
 * (Entry2VectorAndNeighbors, :418-439) into vecs (n x dim f32) and nbrs
 * (n x m u32); a failed or dropped id decodes as zeros (ok[i] = 0), as in the
 * reference.  With a query (dim f32), dist[i] = L2Dist(vector i, query)
 * (build_graph.go:119-127, l2_distance_amd64.s order, 0 for a failed id) is
 * computed on the GPU next to the decode.  Any output may be NULL (dist needs
 * query).  Counts totalQueryNum / succQueryNum as the reference does
 * (pm_graph_counts).  pm_graph_get_start_vertex: the ⌊√n⌋ start vertices
 * chosen by pm_graph_preprocess (non-private), *count = their number, the
 * first min(cap, count) written. */
int pm_graph_get_metadata(pm_graph* g, uint64_t* n, uint64_t* dim, uint64_t* m);
int pm_graph_get_vertex_info(pm_graph* g, const uint64_t* ids, uint64_t n, float* vecs, uint32_t* nbrs, uint8_t* ok,
                             const float* query, float* dist);
int pm_graph_get_start_vertex(pm_graph* g, uint64_t cap, uint64_t* ids, float* vecs, uint32_t* nbrs,
                              uint64_t* count);

/* ---- private search over a SHARDED graph DB (multi-GPU) --
 * The reference's PIRGraphInfo (private-search.go:336-531) fetches every
 * vertex record through SimpleBatchPianoPIR.Query (batch-pir.go:170-248),
 * whose 16 partitions are independent sub-PIRs (batch-pir.go:62-85): the
 * sharding axis.  Rank `shard` of `nshards` holds the partitions
 * p % nshards == shard (DB rows, keys, hint state) and runs the SAME sessions
 * (same seeds, same queries) as every other rank; each shared step's answers
 * are combined across the ranks so every rank continues identical searches.
 *
 * pm_graph_create_shard: host vectors (n x dim f32) and graph (n x m u32) as
 * pm_graph_create; only this shard's partitions are uploaded.
 * pm_graph_create_synth: the synthetic graph of the reference's
 * `-input synthetic` mode (private-search.go:42-69,114-117,168-170: uniform
 * [0,1) f32 vectors, uniform neighbour ids without self loops) as a pure
 * function of data_seed (pm_internal.h graph_synth_elem), generated on the
 * device: graph DBs of 10^8-10^9 entries that cannot be built or shipped.
 * pm_graph_synth_rows: the host restatement of those rows (vec / nb NULLable).
 * Sessions: pm_graph_create_session on a preprocessed base, as unsharded. */
int pm_graph_create_shard(pm_ctx* ctx, uint64_t n, uint64_t dim, uint64_t m, const float* vectors,
                          const uint32_t* graph, uint32_t shard, uint32_t nshards, uint64_t pir_seed,
                          uint64_t search_seed, pm_graph** out);
int pm_graph_create_synth(pm_ctx* ctx, uint64_t n, uint64_t dim, uint64_t m, uint64_t data_seed, uint32_t shard,
                          uint32_t nshards, uint64_t pir_seed, uint64_t search_seed, pm_graph** out);
int pm_graph_synth_rows(uint64_t n, uint64_t dim, uint64_t m, uint64_t data_seed, const uint64_t* ids, uint64_t k,
                        float* vec, uint32_t* nb);
/* The combine of one team's shared step: SUM-all-reduce (uint64, wrapping)
 * the nwords device words at dev_words in place across the ranks, ordered on
 * `stream` (a hipStream_t: the reduction waits for the stream's work and the
 * stream's later work waits for the reduction).  Every rank calls it for the
 * same (round, team) sequence.  0 = success. */
typedef int (*pm_combine_fn)(void* user, uint32_t team, uint64_t* dev_words, uint64_t nwords, void* stream);
/* Words of one team's records: sessions x parallel x m x W (W = the entry
 * words holding the neighbour list, + 1 for {dist, ok}), + 1 error word.  The
 * error word is 0 from a healthy rank and 1 from a rank whose team failed: such
 * a rank still takes the team's next combine turn (zero records, error word 1),
 * and every rank stops the team at that turn with PM_EHIP, so no rank is left
 * waiting inside a collective. */
uint64_t pm_sharded_record_words(pm_graph* g, uint32_t sessions, int parallel);

/* The library-native combine (replaces the per-step hop into the caller's
 * runtime, e.g. torch.distributed): RCCL communicators over xGMI, one per
 * lock-step team, created inside libpacmann.so from `nteams` ncclUniqueIds
 * that rank 0 makes (pm_rccl_unique_id) and the caller broadcasts over any
 * channel; pm_rccl_combine is a pm_combine_fn (user = the pm_rccl handle):
 * ncclAllReduce(ncclUint64, ncclSum) in place on the team's stream.  RCCL is
 * loaded on first use (dlopen of librccl.so.1, the copy already mapped into
 * the process if any).  The batch-pir.go:62-85 partitions are the shards; the
 * all-reduce is the north_star's final XOR-reduce (one rank answers each id,
 * so the integer sum is the XOR). */
#define PM_RCCL_ID_BYTES 128
typedef struct pm_rccl pm_rccl;
int  pm_rccl_unique_id(uint8_t id[PM_RCCL_ID_BYTES]);
int  pm_rccl_create(int device, int nranks, int rank, const uint8_t* ids /* nteams x PM_RCCL_ID_BYTES */,
                    uint32_t nteams, pm_rccl** out);
void pm_rccl_destroy(pm_rccl* r);
int  pm_rccl_combine(void* user, uint32_t team, uint64_t* dev_words, uint64_t nwords, void* stream);
/* Creation is bounded, by one path: the teams' communicators are created
 * nonblocking (ncclCommInitRankConfig, blocking = 0) inside ONE
 * ncclGroupStart / ncclGroupEnd group, and each one's state is polled (with a
 * sleep between polls) for at most pm_set_option("rccl_timeout_s") seconds
 * (else PM_RCCL_TIMEOUT_S, default 120).  A rank whose peer never joins gets
 * PM_ETIMEDOUT, not a hang.  Its communicators are aborted (ncclCommAbort), so
 * no thread of the library stays inside RCCL.  An RCCL without the nonblocking
 * API gives PM_EHIP.
 * pm_rccl_probe runs one 1-word all-reduce per team within the same bound and
 * checks that it sums to nranks; on failure the communicators are aborted.
 * Callers agree on the ranks' outcomes over another channel (a MIN of their
 * success flags) and fall back to another combine unless every rank
 * succeeded (pacmann_amd.shard.RcclCombiner.prepare). */
int  pm_rccl_probe(pm_rccl* r);
/* pm_search_loop_batched over a sharded graph DB: S sessions (clients of one
 * shard's server DB) in ngroups lock-step teams; every round of a team is one
 * shared step over this shard's partitions followed by ONE combine of the
 * team's per-id records {neighbour list, L2 distance to the session's query,
 * success flag} (zero where this shard holds no answer: exactly one shard
 * answers an id, so the sum is the unsharded answer bit for bit).  Teams issue
 * their combines in one global (round, team) order on every rank.
 * team_bufs: NULL (library buffers) or one device buffer per team of
 * pm_sharded_record_words(sessions of that team) words (the tensors a
 * torch.distributed combine reduces in place); team g = sessions
 * [S*g/ngroups, S*(g+1)/ngroups).  combine NULL: no exchange, valid when this
 * shard holds every partition, or with model_peers = 1 (synthetic graphs
 * only): the other shards' partitions are answered from the graph's spec on
 * the device (a wider shard layout measured one shard per GPU; modelled).
 * Outputs as pm_search_loop_batched; the answers are identical on every rank
 * and equal to the unsharded search's. */
int pm_search_loop_sharded(pm_graph** sessions, uint32_t S, const float* queries, uint64_t q, int k, int step,
                           int parallel, uint32_t ngroups, uint32_t nthreads, pm_combine_fn combine, void* user,
                           uint64_t* const* team_bufs, int model_peers, int64_t* answers, double* wall_s,
                           double* online_s, double* maintenance_s);

/* ---- graph construction + ground truth (graphann/build_graph.go) ------- */
/* Exact k nearest base rows of each query by (L2Dist, id), k <= 64: the
 * ground truth ComputeRecall (build_graph.go:821-863) scores against.  ids:
 * nq x k (-1 padded), dists: nq x k or NULL.  Exact for integer-valued rows
 * (e.g. SIFT's uint8 values); for general float rows the GPU keeps the 64 best
 * by bf16-rounded distance before the exact re-rank. */
int pm_knn(pm_ctx* ctx, const float* base, uint64_t n, uint64_t dim, const float* queries, uint64_t nq,
           uint32_t k, int64_t* ids, float* dists);
/* BuildGraph / CreateGraphBasedOnNGT (build_graph.go:97-105,314-523) with the
 * NGT candidate search (absent here) replaced by exact kNN: candidates =
 * int(1.5 m) nearest by (L2Dist, id) minus u; robustPrune (alpha); reverse
 * edges; edge sampling with probability min(1.5 m / inbounds, 1); second
 * robustPrune; random fill to exactly m.  Sampling and fill draw from
 * hash4(seed, ...).  graph: n x m.  times (NULL or 4
 * doubles): kNN, first prune, host edge work, second prune, in seconds.
 * dim <= 192, m <= 42. */
int pm_build_graph(pm_ctx* ctx, const float* vectors, uint64_t n, uint64_t dim, uint64_t m, float alpha,
                   uint64_t seed, uint32_t* graph, double* times);

#ifdef __cplusplus
}
#endif
#endif /* PACMANN_H */
