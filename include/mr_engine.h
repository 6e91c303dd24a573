/*
 * mr_engine.h — C ABI of the MI355X collaborative-filtering similarity engine.
 *
 * This is the drop-in boundary for the reference's scoring hot path
 * (alberto-paparella/MusicRecommendation, paths relative to the reference root;
 * MR = src/main/scala/music_recommandation/MusicRecommender.scala):
 *
 *   reference                                       replaced by
 *   ----------------------------------------------  -------------------------------------------
 *   extractData / songs / songsToUsersMap MR:26-62  mr_corpus_from_tsv, mr_corpus_dataset (host)
 *   importTestLabels MR:70-91                       mr_corpus_from_tsv (labels CSR)
 *   getModel(rank) MR:105-111, getModelP MR:119-125 mr_run / mr_score_dense (batched, all pairs)
 *   UBM cosineSimilarity+rank MR:140-166            model = MR_UBM
 *   IBM cosineSimilarity+rank MR:230-257            model = MR_IBM
 *   getUserBasedModel(P) MR:132-215                 mr_score_dense(ctx, MR_UBM, ...)
 *   getItemBasedModel(P) MR:222-307                 mr_score_dense(ctx, MR_IBM, ...)
 *   Spark song partition getItemBasedModel2        mr_options.song_lo/song_hi (song-range shard)
 *     distributed.scala:477-479
 *
 * The reference has no FFI: its only plug point is the private closure
 * `rank: (String,String) => Double` (MR:105). A per-pair foreign call is ruled
 * out (3.85e9 pairs at full scale), so the boundary is the batched model: the
 * caller hands over interned CSR arrays once (mr_load) and receives every
 * (test user, song) score of the model in one call.
 *
 * Conventions (all plain C; no C++ or torch types cross this boundary):
 *  - Ids are dense int32. Songs are numbered in lexicographic order of their
 *    string id, users likewise (the driver's sort key, main.scala:57-59).
 *  - Return value 0 = MR_OK; negative = error; mr_last_error() describes the
 *    last error of the calling thread. Nothing here calls exit()/abort()
 *    (the reference's System.exit at MR:326 etc. becomes an error code).
 *  - Ownership: the caller owns every host buffer it passes; mr_load COPIES.
 *    The context owns its device memory and its HIP stream.
 *  - Threading: one context is driven by one host thread at a time; calls on
 *    different contexts are independent. mr_run is asynchronous on the
 *    context's stream; every other compute call is synchronous.
 */
#ifndef MR_ENGINE_H
#define MR_ENGINE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define MR_OK          0
#define MR_E_INVALID  -1 /* bad shape, unsorted/duplicate CSR, train∩test users, bad option */
#define MR_E_HIP      -2 /* HIP runtime error (no device, launch failure, ...)           */
#define MR_E_OOM      -3 /* device or host allocation failed                               */
#define MR_E_STATE    -4 /* call out of order (e.g. mr_run before mr_load)                 */
#define MR_E_IO       -5 /* file could not be opened/read                                  */
#define MR_E_PARSE    -6 /* malformed TSV line (reference: scala.MatchError, MR:34)         */
#define MR_E_RCCL     -7 /* RCCL missing or a collective failed (multi-GPU groups)          */

/* ---- models ------------------------------------------------------------ */
#define MR_UBM 0 /* UserBasedModel: MR:140-166 */
#define MR_IBM 1 /* ItemBasedModel: MR:230-257 */

/* ---- dense output element type ------------------------------------------ */
#define MR_OUT_F32 0
#define MR_OUT_F64 1

/*
 * Interned dataset, the engine's input. Mirrors the maps built by
 * extractData (MR:26-62). All CSR column lists are sorted ascending and
 * duplicate-free; the *_len arrays keep the reference's duplicate-counting
 * `.length` semantics (MR:147, MR:237).
 *
 *  n_train_users  = |trainUsers|                                (MR:55)
 *  n_test_users   = |testUsers|                                 (MR:56)
 *  n_songs        = |songs| = distinct songs of train ∪ test    (MR:58)
 *  tr_off/tr_songs: train user v -> distinct songs S(v)         (trainUsersToSongsMap)
 *  te_off/te_songs: test user u  -> distinct visible songs T(u) (testUsersToSongsMap)
 *  song_count[s]  = songsToUsersMap(s).length: train AND test lines, dups counted (MR:60-62, MR:237)
 *  tr_len[v]      = trainUsersToSongsMap(v).length, dups counted (MR:147)
 *  te_len[u]      = testUsersToSongsMap(u).length, dups counted  (MR:147)
 * Train and test users must be disjoint (dataExtraction.ipynb:149,301); the
 * engine checks what it can (every test user has >=1 visible song, counts
 * are consistent with the CSR) and returns MR_E_INVALID otherwise.
 * The song -> train-users transpose is built by mr_load itself.
 */
typedef struct mr_dataset {
  int32_t n_train_users;
  int32_t n_test_users;
  int32_t n_songs;
  int32_t reserved0;
  const int64_t* tr_off;     /* [n_train_users + 1] */
  const int32_t* tr_songs;   /* [tr_off[n_train_users]] */
  const int64_t* te_off;     /* [n_test_users + 1] */
  const int32_t* te_songs;   /* [te_off[n_test_users]] */
  const int32_t* song_count; /* [n_songs] */
  const int32_t* tr_len;     /* [n_train_users] */
  const int32_t* te_len;     /* [n_test_users] */
} mr_dataset;

typedef struct mr_options {
  int32_t device;      /* HIP device ordinal (default 0) */
  int32_t frac_bits;   /* fixed-point fraction bits F of the int64 accumulators (default 32, 8..40) */
  int32_t song_lo;     /* first song id of this context's shard (default 0) */
  int32_t song_hi;     /* one past the last song id; <= 0 means n_songs (default 0) */
  int32_t block_songs; /* songs per LDS accumulator tile; 0 = auto
                          (multiple of 256, <= 16384) */
  int32_t out_dtype;   /* MR_OUT_F32 (default) or MR_OUT_F64 for the dense model */
  int32_t topk;        /* k of the per-test-user recommendation list (0 = off, <= 64; default 10) */
  int32_t dense;       /* 1 (default) = write the dense model; 0 = top-k only */
  int32_t time_kernels;/* 1 = per-launch HIP events around each kernel in mr_run (diagnostic; they
                          perturb back-to-back launches — see mr_kernel_times / mr_timing_begin) */
  int32_t stage1;      /* launch shape: 0 = auto, 1 = fused (one kernel; stage 1 recomputed per
                          song tile in LDS; n_train_users <= 4096), 2 = separate stage-1 kernel
                          (compact neighbour lists), 4 = wide (large train sets: chunked stage 1,
                          16k-song tiles scored by 1024-thread workgroups, separate top-k merge
                          launch; topk <= 16). (3 and 5 named round-2 shapes that were never
                          faster and are gone: MR_E_INVALID.) Auto (topk <= 16): wide when
                          n_train_users > 4096 or n_test_users x n_train_users >= 1e5, else
                          fused; topk > 16: fused when n_train_users <= 4096, else separate. */
  int32_t stage1_chunk;/* separate shape: train users per stage-1 LDS chunk; 0 = auto (all of them up
                          to 16384, else 4096); smaller values exercise the chunked path */
  int32_t train_order; /* 0 (default) = train users renumbered internally by distinct-song count
                          (descending) for load balance; 1 = as given. Results are identical. */
  int32_t topk_lists;  /* 1 = tile top-k of the wide shape by per-thread running lists only
                          (diagnostic); 0 (default) = a threshold pass first (about k candidates),
                          the lists only when ties overflow it. Results are identical. */
  int32_t ibm_route;   /* ItemBasedModel route of the wide shape (the cosine sum of MR:249-257):
                          0 = auto (co-listening index when it applies), 1 = two-hop (per test user,
                          the train neighbours' weights, then their songs), 2 = co-listening index:
                          each run first counts, for every test-visible song s2 and every song s of
                          the shard, the train users that heard both (C[s2][s] = |L_tr(s2) ∩ L_tr(s)|,
                          the numerator of MR:232-235), then scores u as Σ_{s2∈T(u)} q(s2)·C[s2][s].
                          The same integer sum as the two-hop route: results are identical. Route 2
                          needs the wide shape, tiles <= 32768 songs and train listener counts
                          < 131072 (else MR_E_INVALID; auto then falls back to route 1). */
  int32_t reserved[2];
} mr_options;

typedef struct mr_ctx mr_ctx;

/* Fill *opt with defaults. */
int mr_options_default(mr_options* opt);

/* Create a context on opt->device (its own HIP stream). */
int mr_create(const mr_options* opt, mr_ctx** out);
int mr_destroy(mr_ctx* ctx);

/* Validate, copy to the device and build the device-side indexes. */
int mr_load(mr_ctx* ctx, const mr_dataset* d);

/* Shard geometry after mr_load: [*song_lo, *song_hi) and the number of
 * test users. The dense model of this context is n_te x (song_hi - song_lo). */
int mr_shard_info(const mr_ctx* ctx, int32_t* song_lo, int32_t* song_hi, int32_t* n_test_users);

/* Launch shape chosen by mr_load: *shape = 0 separate, 1 fused, 3 wide (auto
 * picks fused or wide for topk <= 16, fused or separate above; see
 * mr_options.stage1); songs per LDS tile and tiles per test user. */
int mr_launch_info(const mr_ctx* ctx, int32_t* shape, int32_t* block_songs, int32_t* n_tiles);

/* Test-user batch of the separate / wide shapes (mr_run launches the stage-1 and
 * scoring kernels once per batch of *batch users, sized so the neighbour lists
 * fit 8 GiB; = n_test_users for the other shapes) and the stage-1 chunking of
 * the train users (*n_chunks chunks of *chunk users). */
int mr_batch_info(const mr_ctx* ctx, int32_t* batch, int32_t* chunk, int32_t* n_chunks);

/* ItemBasedModel route chosen by mr_load (mr_options.ibm_route): *route = 1
 * two-hop, 2 co-listening index; for route 2 the index's rows (distinct
 * test-visible songs with train listeners) and the entries its pool can hold
 * (a bound on the shard's non-zero counts; 4 B each). Any pointer may be NULL. */
int mr_route_info(const mr_ctx* ctx, int32_t* route, int32_t* n_rows, int64_t* pool_entries);

/* Tile top-k of the wide shape (the per-(test user, song tile) selection that
 * feeds the segmented top-k merge, MR:249-257's scores ranked): *candidate_only
 * = 1 when this context's top-k-only runs rank fp32 approximations of every
 * song first and compute the exact fp64 score (the oracle's operations) of the
 * candidates within a relative margin of the threshold only — lists, keys and
 * scores bit-identical to the all-songs path; 0 when every song's exact score
 * is computed. Candidate mode is on (mr_load's cand_on) only for the wide shape
 * with all of: no dense output (so no dense min / max either), no per-tile
 * lists (topk_lists = 0), 1 <= k <= 16 (the wide shape's own bound; the
 * selection's k <= scoring threads / 16 holds for either kernel width), a song tile of at most 20 x scoring threads, and
 * MR_WIDE_CAND unset or not "0" in the environment at mr_load. */
int mr_topk_mode(const mr_ctx* ctx, int32_t* candidate_only);

/* Sizes of the latest ibm run on the co-listening route (the byte model of
 * bench.py's roofline; synchronous): *index_nnz = non-zero counts C[s2][s]
 * over all index rows and the shard's songs, *consumed = Σ_u Σ_{s2 ∈ T(u)}
 * (non-zeros of s2's row), *build_reads = Σ_rows (c_tr(s2) + Σ_{v ∈ L_tr(s2)}
 * |S(v) ∩ shard|) (the listener lists and their songs the build reads).
 * MR_E_STATE unless the context is on route 2 and has run ibm since its load
 * (the counts are those of the latest ibm run). */
int mr_cooc_stats(mr_ctx* ctx, int64_t* index_nnz, int64_t* consumed, int64_t* build_reads);

/* Encoding-independent byte counts of the latest ibm run on the co-listening
 * route, split by kernel (bench.py's north-star roofline; synchronous). The
 * index segment of row r (song s2) in tile t is charged the cheaper of its two
 * exact encodings, min(4 * nnz(r, t), songs of t) bytes: 4-B (song, count)
 * entries or a count byte per song of the tile (whatever the build actually
 * wrote; a dense segment is charged its tile's songs, exact under the build's
 * rule nnz * 3 >= songs — a test override of that rule, MR_COOC_DENSE_DIV,
 * can make it an over-count). Reads are counted in 4-B ids: a row's listener list and each
 * listener's songs in the shard, once.
 *   heavy_*  rows built by k_cooc_build (one listener walk per tile),
 *   light_*  rows built by k_cooc_light / k_cooc_light_wave (one walk);
 *   *_reads         Σ_rows (c_tr(s2) + Σ_{v ∈ L_tr(s2)} |S(v) ∩ shard|) ids,
 *   *_index_bytes   Σ_rows Σ_t min(4 nnz(r, t), songs of t),
 *   heavy_visits    Σ_heavy rows c_tr(s2) · walks (listener visits: one walk per
 *                   tile, or per tile group of k_cooc_group),
 *   consumed_bytes  Σ_u Σ_{s2 ∈ T(u)} Σ_t min(4 nnz(r, t), songs of t): the
 *                   segments the scoring kernel reads,
 *   group_tiles, n_groups  the heavy build's tile grouping,
 *   index_* / consumed_*   the written encoding: sparse entries, dense songs.
 * MR_E_STATE unless the context is on route 2 and has run ibm since its load. */
typedef struct mr_cooc_bytes_t {
  int64_t heavy_rows, light_rows;
  int64_t heavy_reads, light_reads;
  int64_t heavy_index_bytes, light_index_bytes;
  int64_t heavy_visits;
  int64_t consumed_bytes;
  int64_t group_tiles;  /* tiles per k_cooc_group pass (0: heavy rows per tile) */
  int64_t n_groups;     /* walks per u16 heavy row: tile groups, or n_tiles */
  /* the encoding the build wrote: sparse entries (with the dense segments'
   * excess entries) and the songs of dense segments, over the index and over
   * the scoring's reads (each row's counts x the test users reading it) */
  int64_t index_sparse_entries, index_dense_songs;
  int64_t consumed_sparse_entries, consumed_dense_songs;
} mr_cooc_bytes_t;
int mr_cooc_bytes(mr_ctx* ctx, mr_cooc_bytes_t* out);

/* Host only, before any load: the song tile of the wide shape that a context
 * with these options would use for n_train_users x n_test_users (the widest
 * the LDS holds, or opt->block_songs when set; opt = NULL: the defaults), or
 * *tile_songs = 0 when mr_load would pick another shape. The wide kernel's
 * unit of work is one walk of a test user's neighbour list per tile, so song
 * shards cut at multiples of it (mr_song_shards_tiled) carry no partial
 * tile: the multi-GPU layouts' per-GPU work (distributed.scala:477-479). */
int mr_shard_tile_songs(const mr_options* opt, int32_t n_train_users, int32_t n_test_users,
                        int32_t* tile_songs);

/* The same for a layout of n_shards song shards over n_songs songs: the tile
 * narrowed so that the shards hold the same whole number of tiles (the tile
 * count rounded up to a multiple of n_shards; = mr_shard_tile_songs for one
 * shard or an explicit opt->block_songs). mr_group_load and the per-process
 * layouts (sharding.ShardScorer) cut their shards with it. */
int mr_shard_tile_songs_n(const mr_options* opt, int32_t n_train_users, int32_t n_test_users, int32_t n_songs,
                          int32_t n_shards, int32_t* tile_songs);

/*
 * Score every (test user, song) pair of the shard for `model`, leaving the
 * results in device buffers (asynchronous on the context stream):
 *  dense[u][s - song_lo] = rank(u, s) for s not in T(u), NaN for s in T(u)
 *      (the reference emits no pair for heard songs, MR:109);
 *  topk[u][0..k)  = the k unheard songs of the shard with the highest score,
 *      ordered by (score desc, song id asc); the fixed-point key makes this
 *      order identical for any shard count. Missing entries: song -1.
 */
int mr_run(mr_ctx* ctx, int model);
int mr_sync(mr_ctx* ctx);

/* HIP graph of n_steps back-to-back mr_run(model) of this context (stream
 * capture on the context stream; instantiated once, replaced by the next
 * capture, released by mr_load / mr_destroy). mr_graph_launch replays it,
 * asynchronous on the context stream: one launch for the n steps instead of n
 * host launches. Outputs as after mr_run. Not with time_kernels = 1. */
int mr_graph_capture(mr_ctx* ctx, int model, int32_t n_steps);
int mr_graph_launch(mr_ctx* ctx);

/* Device pointers of the last mr_run's outputs (valid until the next
 * mr_run/mr_load/mr_destroy). Any pointer may be NULL. */
int mr_device_outputs(const mr_ctx* ctx, void** dense, int32_t** topk_songs,
                      int64_t** topk_keys, double** topk_scores);

/* mr_run with the dense model written to a caller-owned DEVICE buffer of
 * n_te * (song_hi - song_lo) elements of the context's out_dtype (instead of
 * the context's own buffer); top-k as mr_run. Asynchronous on the context
 * stream. Lets a caller keep several models on the device (e.g. ubm and ibm
 * for the combination models below). */
int mr_run_into(mr_ctx* ctx, int model, void* dense_dev);

/* Device-side view of a loaded context, for companion calls and callers that
 * launch their own work on the same data (pointers valid until mr_load /
 * mr_destroy). */
typedef struct mr_view {
  int32_t n_test_users, n_songs, song_lo, song_hi, out_dtype, device;
  const int64_t* te_off;   /* device [n_test_users + 1] */
  const int32_t* te_songs; /* device, sorted per user (T(u)) */
  void* stream;            /* hipStream_t of the context */
} mr_view;
int mr_view_get(const mr_ctx* ctx, mr_view* view);

/* Top-k of a dense model on the device (e.g. a combination model): per test
 * user, the k unheard songs of the shard with the highest score, ordered by
 * (score desc, song id asc), into the context's top-k outputs (read them with
 * mr_copy_topk / mr_device_outputs). k must equal the context's topk and be
 * <= 16; scores must be >= 0 (else MR_E_INVALID). Synchronous. */
int mr_topk_dense_device(mr_ctx* ctx, const void* dense_dev, int32_t k);

/* Synchronous convenience calls: run + copy to caller-allocated host buffers.
 * out: n_te * (song_hi - song_lo) elements of the context's out_dtype. */
int mr_score_dense(mr_ctx* ctx, int model, void* out);
/* songs/scores: n_te * k; keys (may be NULL): fixed-point sort keys. */
int mr_topk(mr_ctx* ctx, int model, int k, int32_t* songs, double* scores, int64_t* keys);

/* Copy the last mr_run's outputs to host buffers (synchronous). */
int mr_copy_dense(mr_ctx* ctx, void* out);
int mr_copy_topk(mr_ctx* ctx, int32_t* songs, double* scores, int64_t* keys);
/* Same, into DEVICE buffers of the context's GPU (e.g. an all-gather send
 * buffer owned by the caller); stream-ordered, returns after completion. */
int mr_copy_topk_device(mr_ctx* ctx, int32_t* songs, int64_t* keys);
/* Same, enqueued on the context stream without waiting (stream-ordered after
 * the last mr_run; the caller orders its own stream after it, e.g. with an
 * event — the one-process-per-GPU exchange of sharding.py). */
int mr_copy_topk_device_async(mr_ctx* ctx, int32_t* songs, int64_t* keys);

/*
 * Merge per-shard top-k lists (G shards, each n_te x k, song ids global) into
 * one n_te x k list by (key desc, song asc) — the exchange step of a
 * song-sharded run after the all-gather. Host version (no GPU needed) and a
 * device version that runs on the context stream over device pointers.
 */
int mr_topk_merge_host(int32_t n_shards, int32_t n_te, int32_t k,
                       const int32_t* songs_in, const int64_t* keys_in, const double* scores_in,
                       int32_t* songs_out, int64_t* keys_out, double* scores_out);
int mr_topk_merge_device(mr_ctx* ctx, int32_t n_shards, int32_t n_te, int32_t k,
                         const int32_t* songs_in, const int64_t* keys_in, const double* scores_in,
                         int32_t* songs_out, int64_t* keys_out, double* scores_out);
/* The device merge enqueued on the context stream without waiting. */
int mr_topk_merge_device_async(mr_ctx* ctx, int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in,
                               const int64_t* keys_in, int32_t* songs_out, int64_t* keys_out, double* scores_out);

/*
 * The exchange as ONE collective: a shard's top-k lists travel as one record
 * block — n_te*k int64 keys at byte 0, then n_te*k int32 songs at byte
 * 8*n_te*k, padded to *rec_bytes (a multiple of 16) — so a song-sharded run
 * all-gathers G blocks in a single call (the north star's "single RCCL
 * all-gather", distributed.scala:477-479) instead of one per array.
 * mr_copy_topk_device(_async)(ctx, block + 8*n_te*k, block) fills such a block;
 * mr_topk_merge_records_async merges G gathered blocks (stride rec_bytes) on
 * the context stream, like mr_topk_merge_device_async.
 */
int mr_topk_record_bytes(int32_t n_te, int32_t k, int64_t* rec_bytes);
int mr_topk_merge_records_async(mr_ctx* ctx, int32_t n_shards, int32_t n_te, int32_t k, const void* records,
                                int64_t rec_bytes, int32_t* songs_out, int64_t* keys_out, double* scores_out);

/* ---- combination models and evaluation on the device (MR:317-481, MR:521-639) ----
 * Over dense models of the context's shard (device pointers, n_te x width of
 * the context's out_dtype, NaN = no pair), e.g. filled by mr_run_into. Pairs
 * are indexed in the driver's sorted order (main.scala:57-59: user, then song,
 * heard songs skipped); pair_base = index of this context's first pair in the
 * full model (0 unless the context holds a block of test users), n_pairs = the
 * full model's length. All three are synchronous. */
#define MR_COMB_LINEAR      0 /* getLinearCombinationModel MR:317-351: ubm*param + ibm*(1-param) */
#define MR_COMB_AGGREGATION 1 /* getAggregationModel MR:361-418: pairs < (int)(param*n_pairs) from ibm */
#define MR_COMB_STOCHASTIC  2 /* getStochasticCombinationModel MR:429-481: ibm where u(seed,pair) < param;
                                 u = 24-bit uniform of splitmix64(seed + (idx+1)*0x9E3779B97F4A7C15) */
int mr_combine_device(mr_ctx* ctx, int kind, double param, uint64_t seed, int64_t pair_base, int64_t n_pairs,
                      const void* ubm, const void* ibm, void* out);
/* The driver's three combinations (main.scala:57-89) in one pass over ubm and
 * ibm: out_linear (alpha), out_aggregation (ibm_percentage), out_stochastic
 * (ibm_probability, seed) — each bit-equal to mr_combine_device of its kind —
 * and, when minmax is non-null, each output's min / max over its pairs as
 * minmax[0..5] = {lin min, lin max, agg min, agg max, sto min, sto max} (what
 * mr_eval_minmax_device returns for it: +inf / -inf when the shard holds no
 * pair). Replaces MR:317-481 called three times, each reading both models. */
int mr_combine_all_device(mr_ctx* ctx, double alpha, double ibm_percentage, double ibm_probability, uint64_t seed,
                          int64_t pair_base, int64_t n_pairs, const void* ubm, const void* ibm, void* out_linear,
                          void* out_aggregation, void* out_stochastic, double* minmax);
/* evaluateModel (MR:636), device part: min / max over the model's scores
 * (MR:524-525; +inf / -inf when the shard holds no pair) ... */
int mr_eval_minmax_device(mr_ctx* ctx, const void* dense, double* mn, double* mx);
/* The same min / max for the dense model of the context's last mr_run /
 * mr_run_into, computed by the wide-shape scoring kernels while they store it
 * (per-user ordered-key atomics; no second pass over the model). MR_E_STATE
 * when the last run was not a wide-shape dense run (or was a graph replay). */
int mr_dense_minmax(mr_ctx* ctx, double* mn, double* mx);
/* ... and per song s of the shard and threshold t_i = i/10, i < n_thresholds:
 * pred_counts[s][i] = #test users with (x - mn)/(mx - mn) > t_i (MR:529),
 * tp_counts[s][i] = those of them whose labels hold s (MR:545). n_thresholds:
 * 10 (0.0..0.9, evaluateModel MR:590; 0 = 10) or 11 (0.0..1.0, the distributed
 * evaluation, distributed.scala:395). mn/mx are the GLOBAL extremes (reduce
 * over shards first). Labels: host CSR over the context's test users, global
 * song ids (label-only songs >= n_songs). Counts: [width][n_thresholds]. */
int mr_eval_counts_device(mr_ctx* ctx, const void* dense, double mn, double mx, const int64_t* lab_off,
                          const int32_t* lab_songs, int32_t* pred_counts, int32_t* tp_counts, int32_t n_thresholds);
/* Host part: AP per song class (MR:588-618, left folds as List.sum; with 11
 * thresholds distributed.scala:401-415) and mAP = sum / n_label_songs
 * (MR:625-627), classes summed in song-id order (the distributed version sums
 * with RDD.sum, in partition order). pos[s] = #test users whose labels hold s. */
int mr_eval_map(int32_t n_classes, const int32_t* pred_counts, const int32_t* tp_counts, const int32_t* pos,
                int32_t n_label_songs, double* map_out, int32_t n_thresholds);
/* The two above in one call for a context that holds every test user: counts
 * and the per-class AP on the device (the same double operations), only the
 * AP per class crosses PCIe, summed on the host in song-id order — bit-equal
 * to mr_eval_counts_device + mr_eval_map. pos: host [>= song_hi], global. */
int mr_eval_map_device(mr_ctx* ctx, const void* dense, double mn, double mx, const int64_t* lab_off,
                       const int32_t* lab_songs, const int32_t* pos, int32_t n_label_songs, double* map_out,
                       int32_t n_thresholds);
/* The multi-rank evaluation without the counts crossing PCIe (MR:541-627 over
 * models spread across ranks — song shards, test-user blocks or both), for
 * n_models dense models of the context at once (dense: host array of device
 * pointers; mn / mx: host arrays, the GLOBAL extremes of each model):
 * mr_eval_class_counts_device writes the counts of the label classes only into
 * a caller DEVICE buffer laid out by a class list every rank shares —
 * counts[m][0][c][t] = pred, counts[m][1][c][t] = tp of class c for model m
 * (n_models x 2 x n_classes x n_thresholds int32), 0 for classes outside the
 * context's song range — so one SUM all-reduce of the buffers over the ranks
 * (RCCL) gives the counts over every test user; classes: host, strictly
 * ascending global song ids (< n_songs; the songs with label count pos > 0:
 * label-only songs are never predicted and add 0 to the sum).
 * mr_eval_map_counts_device then computes every model's AP per class on the
 * device from such a (reduced) buffer (class_pos: host, each > 0) and the mean
 * over n_label_songs into maps_out[m], classes summed in song-id order —
 * bit-equal to mr_eval_map over the full counts. Both synchronous; one launch
 * sequence and one host synchronisation per call, whatever n_models. */
int mr_eval_class_counts_device(mr_ctx* ctx, int32_t n_models, const void* const* dense, const double* mn,
                                const double* mx, const int64_t* lab_off, const int32_t* lab_songs, int32_t n_classes,
                                const int32_t* classes, int32_t* counts, int32_t n_thresholds);
int mr_eval_map_counts_device(mr_ctx* ctx, int32_t n_models, int32_t n_classes, const int32_t* class_pos,
                              const int32_t* counts, int32_t n_label_songs, double* maps_out, int32_t n_thresholds);

/* Kernel timing of mr_run calls made with opt.time_kernels = 1: per kernel
 * (0 = separate stage-1 kernel — neighbour lists —, 1 = the
 * scoring kernels — stage 2, fused stage 1, the in-launch top-k merge, the wide
 * kernel and its top-k merge —, 2 = reserved) the number of
 * timed launches and their summed device milliseconds; reset=1 clears. */
int mr_kernel_times(mr_ctx* ctx, int32_t which, int64_t* launches, double* total_ms, int32_t reset);

/* Timing window: mr_timing_begin records an event on the context stream,
 * mr_timing_end records a second one, waits for it and returns the device
 * time between them and the number of scoring-kernel launches issued in
 * between (no per-launch events: the window does not perturb the launches).
 * mr_timing_stop records the closing event without waiting (a caller that
 * synchronises the device itself reads the window later with mr_timing_end,
 * which then records nothing). */
int mr_timing_begin(mr_ctx* ctx);
int mr_timing_stop(mr_ctx* ctx);
int mr_timing_end(mr_ctx* ctx, int64_t* launches, double* total_ms);

/* Diagnostic builds only (libmr_engine_stamps.so, -DMR_STAMPS): copy the
 * per-workgroup phase timestamps of the last scoring launch ([grid][8]
 * s_memrealtime values); MR_E_STATE in the production build. */
int mr_debug_stamps(mr_ctx* ctx, int64_t* out, int64_t n);

/* HIP stream of the context (as void* = hipStream_t). */
void* mr_stream(const mr_ctx* ctx);

/* Thread-local description of the last error (never NULL). */
const char* mr_last_error(void);

/* ---- multi-GPU: one handle over G contexts (distributed.scala:450-479) -------
 * The reference fans ONE driver call out over Spark partitions: by song
 * (getItemBasedModel2 = parallelize(songs, numberSlices).map(getRanks2)
 * .collect.flatten, distributed.scala:477-479; getUserBasedModel2 :459-461) or
 * by test user (getItemBasedModel1 :468-470). A group is the same single call
 * over G = n_song_shards x n_user_blocks engine contexts: context (b, g) scores
 * test-user block b (contiguous, sizes within one) over song-range shard g
 * (boundaries balance sum(c_tr(s) + 1), the stage-2 work) on its own GPU and
 * stream. The shards of a user block then exchange their per-user top-k lists
 * with ONE all-gather and merge them by (key desc, song asc): the results are
 * bit-identical to one context (fixed-point keys) for every layout.
 * Transports: MR_TRANSPORT_RCCL — every context on its own device, one RCCL
 * communicator per user block (ncclCommInitAll, owned by the group; librccl —
 * or the library named by the environment variable MR_RCCL_LIB — is loaded on
 * first use), ONE ncclAllGather of the top-k record blocks per context under
 * ncclGroupStart/End on the contexts' streams, the merge on every device;
 * MR_TRANSPORT_COPY — every context on ONE device (logical shards), the
 * block's first context gathers the record blocks with device copies and
 * merges. AUTO = RCCL when the contexts span >= 2 devices. RCCL needs one
 * distinct device per context (MR_E_INVALID otherwise) unless MR_RCCL_LIB
 * names a library that accepts shared devices (the test fake). A group is driven by one host thread; calls are synchronous unless
 * stated. */
#define MR_TRANSPORT_AUTO 0
#define MR_TRANSPORT_COPY 1
#define MR_TRANSPORT_RCCL 2

typedef struct mr_group_options {
  int32_t n_song_shards;  /* G_s >= 1 (default 1) */
  int32_t n_user_blocks;  /* G_u >= 1 (default 1) */
  int32_t transport;      /* MR_TRANSPORT_* (default AUTO) */
  int32_t n_devices;      /* entries of `devices`; 0 = every context on opt->device */
  const int32_t* devices; /* context i = b*G_s + g runs on devices[i % n_devices] (not retained) */
} mr_group_options;

typedef struct mr_group mr_group;

/* Host helper (no GPU): the group's song-range shard boundaries, bounds[0..n_shards]
 * (bounds[0] = 0, bounds[n_shards] = n_songs), balancing sum(c_tr(s) + 1). */
int mr_song_shards(const mr_dataset* d, int32_t n_shards, int32_t* bounds);
/* The same balance, then every shard narrowed to at most
 * ceil(ceil(n_songs / tile_songs) / n_shards) tiles of tile_songs (each
 * boundary moved the least from the balanced one); tile_songs <= 0: as
 * mr_song_shards. mr_group_load uses it with mr_shard_tile_songs. */
int mr_song_shards_tiled(const mr_dataset* d, int32_t n_shards, int32_t tile_songs, int32_t* bounds);

int mr_group_options_default(mr_group_options* gopt);
/* opt: the contexts' options (song_lo/song_hi must be 0: the group sets them). */
int mr_group_create(const mr_options* opt, const mr_group_options* gopt, mr_group** out);
int mr_group_destroy(mr_group* g);
/* Validate the dataset as mr_load does, split it (shards, user blocks) and load
 * every context (in parallel). A reload frees the previous load first. */
int mr_group_load(mr_group* g, const mr_dataset* d);
/* Geometry of context i after mr_group_load: songs [*song_lo, *song_hi), test
 * users [*user_lo, *user_hi), device. */
int mr_group_info(const mr_group* g, int32_t i, int32_t* song_lo, int32_t* song_hi, int32_t* user_lo,
                  int32_t* user_hi, int32_t* device);
int mr_group_transport(const mr_group* g, int32_t* transport);
/* Shape of a loaded group: contexts, test users and songs of the whole model
 * (the sizes of mr_group_copy_dense's n_test x n_songs and of the n_test x k
 * top-k outputs; the JNI shim checks Java array lengths against them). */
int mr_group_shape(const mr_group* g, int32_t* n_contexts, int32_t* n_test, int32_t* n_songs);
/* Borrowed context i (e.g. for mr_timing_begin/end on its stream); NULL on error. */
mr_ctx* mr_group_context(mr_group* g, int32_t i);
/* Score every pair on every context, then the top-k exchange (asynchronous on
 * the contexts' streams; mr_group_sync waits for all of them). */
int mr_group_run(mr_group* g, int model);
int mr_group_sync(mr_group* g);
/* Merged top-k of all test users (n_test x k, host), after mr_group_run / in one call. */
int mr_group_copy_topk(mr_group* g, int32_t* songs, double* scores, int64_t* keys);
int mr_group_topk(mr_group* g, int model, int k, int32_t* songs, double* scores, int64_t* keys);
/* Device pointers of the merged lists held by context i (rows of its user
 * block; COPY: the block's first context holds them). */
int mr_group_device_topk(mr_group* g, int32_t i, int32_t** songs, int64_t** keys, double** scores);
/* The dense model n_test x n_songs on the host (collect.flatten, distributed.scala:478). */
int mr_group_copy_dense(mr_group* g, void* out);
int mr_group_score_dense(mr_group* g, int model, void* out);
/* All-gather of the dense shards: dst[i] = device buffer on context i's device
 * of (user_hi - user_lo) x n_songs elements, filled with its block's full rows
 * (RCCL: ncclAllGather of equal padded shard blocks + strided on-device copies). */
int mr_group_allgather_dense(mr_group* g, void* const* dst);

/* ---- host ingest: TSV triplets -> interned corpus (extractData, MR:26-91) ---- */
typedef struct mr_corpus mr_corpus;

/*
 * Parse `user \t song \t playcount` files (playcount ignored, MR:35) into an
 * interned corpus. labels_path may be NULL. Songs = distinct songs of train ∪
 * test (labels do not add songs, MR:79); ids are lexicographic.
 * Malformed lines (not exactly 3 tab-separated fields) -> MR_E_PARSE.
 */
int mr_corpus_from_tsv(const char* train_path, const char* test_path,
                       const char* labels_path, mr_corpus** out);
/* Borrowed view of the corpus as an engine dataset (valid while the corpus lives). */
int mr_corpus_dataset(const mr_corpus* c, mr_dataset* out);
/* Test labels CSR over test users (songs of the labels file that are in
 * `songs` get their id; label songs outside `songs` get ids >= n_songs,
 * numbered lexicographically among themselves). n_label_songs counts the
 * distinct label songs (= newSongs, MR:79). */
int mr_corpus_labels(const mr_corpus* c, const int64_t** off, const int32_t** songs,
                     int32_t* n_label_songs, int32_t* n_extra_songs);
/* String ids (NUL-terminated, owned by the corpus). kind: 0 = song (ids
 * 0..n_songs+n_extra_songs), 1 = train user, 2 = test user. */
const char* mr_corpus_name(const mr_corpus* c, int32_t kind, int32_t id);
/* Every name of `kind` in id order, each followed by '\n' (names hold no tab or
 * newline: they are TSV fields), into buf[0..buf_size); *bytes_needed = the
 * total. buf = NULL (or too small): only *bytes_needed is set (and
 * MR_E_INVALID returned when buf is non-NULL). One call instead of one per
 * name: 1.4M names at full scale. */
int mr_corpus_names(const mr_corpus* c, int32_t kind, char* buf, int64_t buf_size, int64_t* bytes_needed);
int mr_corpus_free(mr_corpus* c);

/* ---- model files (MR:489-512) --------------------------------------------
 * writeModelOnFile (MR:489-497): one "user\tsong\tscore\n" line per pair of a
 * dense n_test x n_songs model (NaN = no pair), the score formatted as
 * java.lang.Double.toString (shortest round-trip digits, JDK 19+). order 0 =
 * getModel's emission order (song-major, MR:106-108), 1 = the driver's sorted
 * (user, song) order (main.scala:57-59, names sorted like their ids). */
int mr_model_write_tsv(const char* path, int32_t n_test, int32_t n_songs, const char* const* user_names,
                       const char* const* song_names, const double* dense, int32_t order);
/* importModelFromFile (MR:505-512) into a dense n_test x n_songs buffer over
 * the given names (NaN where the file has no line). Malformed line ->
 * MR_E_PARSE (the reference: MatchError / NumberFormatException); unknown
 * name or duplicate pair -> MR_E_INVALID. */
int mr_model_read_tsv(const char* path, int32_t n_test, int32_t n_songs, const char* const* user_names,
                      const char* const* song_names, double* dense);
/* java.lang.Double.toString(x) into buf; returns its length (or an error code). */
int mr_java_double_string(double x, char* buf, int32_t cap);

/* Library version string. */
const char* mr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MR_ENGINE_H */
