/*
 * fugu.h -- C ABI of libfugu: MI355X (gfx950) execution of fugu's query hot
 * path (conjunctive posting-list intersection + BM25 + top-k).
 *
 * Drop-in boundary.  In fugu the replaceable call is
 *     searcher.search(&base_query, &TopDocs::with_limit(offset + per_page))
 * inside Dataset::search (reference src/db/search.rs:74-218, the call at
 * :162), reached from perform_search (src/server/handlers/search.rs:350-402)
 * and search_endpoint (:152-207).  A host (Rust over `extern "C"`, or the C++
 * host in fugu_amd/csrc/host.cpp) keeps query parsing, the term dictionary and
 * doc fetch, and calls this library for step A.4 of SURVEY.md §3.  The Rust
 * binding a maintainer would add is written out in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes; 0 = FG_OK, negative = error (message
 * in fg_last_error(), thread-local).  The caller owns every host buffer; the
 * library copies inputs.  Handles own device memory.  An fg_index is an
 * immutable, refcounted snapshot (tantivy Searcher semantics: a reader keeps
 * the segments it opened, src/db/core.rs:290-297).  All entry points are
 * thread-safe per handle except fg_plan_* on the SAME plan.
 */
#ifndef FUGU_H
#define FUGU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision: bumped whenever a struct of this header changes layout or a
 * call's contract changes (4: fg_query_batch.occur; fg_model_out.  5:
 * fg_index_stats.n_sparse_rank_terms / reserved0 / rank_bytes (16 B more);
 * query-time scoring: fg_index_rescore[_many] do no device work, fg_index_term_kth
 * of a rescore is a lower bound).  A binding checks fg_abi_version() against the
 * value it was written for before passing any struct. */
#define FG_ABI_VERSION 5

#define FG_OK 0
#define FG_EINVAL (-1)        /* bad argument (e.g. k == 0: tantivy asserts limit >= 1) */
#define FG_ENODEV (-2)        /* no usable gfx950 device */
#define FG_EOOM (-3)          /* host or device allocation failed */
#define FG_EHIP (-4)          /* HIP runtime error */
#define FG_EUNSUPPORTED (-5)  /* query outside the device subset: the host runs its CPU path */

#define FG_MAX_TERMS 16        /* terms per query on the device path */
#define FG_MAX_FACET_CLAUSES 8 /* facet filter clauses per query on the device path */
#define FG_MAX_K 1024          /* largest k on the device path */
#define FG_MAX_SEGMENTS 64     /* snapshots of one multi-snapshot plan / shards of one fg_search_sharded call */
#define FG_TERM_MISSING 0xFFFFFFFFu /* a query term absent from the term dictionary */

#define FG_MODE_AND 0 /* `t1 AND t2 ...` / `+t1 +t2`: Must clauses (src/db/search.rs:112 parser) */
#define FG_MODE_OR 1  /* `t1 t2 ...`: the parser's default Should conjunction */

/* Per-term occur (tantivy Occur) of fg_query_batch.occur: `+t` / `t AND u` Must,
 * bare `t` / `t OR u` Should, `-t` MustNot (query parser over [text, name],
 * src/db/search.rs:108-127; scoring: SURVEY.md Appendix A.6). */
#define FG_OCCUR_MUST 0
#define FG_OCCUR_SHOULD 1
#define FG_OCCUR_MUST_NOT 2

#define FG_FIELD_TEXT 0
#define FG_FIELD_NAME 1
#define FG_FIELD_FACET 2 /* the docs index's Facet field (src/db/schemas.rs:20) */

typedef struct fg_ctx fg_ctx;
typedef struct fg_index fg_index;
typedef struct fg_plan fg_plan;

/* ---- context ------------------------------------------------------------ */
/* Replaces: nothing in fugu (single process, no devices); the per-process
 * state the Rust AppState (src/server/server_main.rs:16-19) would hold. */
int fg_device_count(int* out);
int fg_ctx_create(int ndev, const int* devs, fg_ctx** out);
int fg_ctx_destroy(fg_ctx* ctx);
/* *enabled = 1 when fg_ctx_create enabled direct (xGMI) access from device a
 * to device b's memory (every ordered pair of the context's devices). */
int fg_ctx_peer_access(const fg_ctx* ctx, int a, int b, int* enabled);
const char* fg_last_error(void);
const char* fg_version(void);
int fg_abi_version(void); /* FG_ABI_VERSION of the library */

/* ---- index snapshot ------------------------------------------------------ */
/* Documents as analyzed token streams: for each doc the term ids produced by
 * the "default" analyzer (SimpleTokenizer -> RemoveLong(40) -> LowerCaser) on
 * the `text` and `name` fields, in order.  This is what NamedIndex::upsert
 * feeds tantivy (src/db/document.rs:23-67, build_full_document :116-139).
 * Field lengths (token counts) become fieldnorms; tf = occurrences. */
typedef struct fg_docs_input {
  uint32_t n_docs;
  uint32_t n_terms;          /* vocabulary size: every token < n_terms */
  const uint64_t* text_off;  /* [n_docs+1] */
  const uint32_t* text_tok;  /* [text_off[n_docs]] */
  const uint64_t* name_off;  /* [n_docs+1] or NULL (no `name` values) */
  const uint32_t* name_tok;  /* or NULL */
  const uint8_t* deleted;    /* [n_docs] 1 = deleted-not-merged, or NULL */
  int threads;               /* host threads for the inversion (<= 0: all) */
  int keep_host_postings;    /* keep a host copy (needed by fg_bytes_model) */
  /* Facet field (add_facets_to_document, src/db/document.rs:310-330): per doc
   * the FacetTokenizer tokens of its facets -- for each facet the root, every
   * ancestor and the facet itself -- as ids < n_facet_terms of the host's
   * facet dictionary (encoded facet paths).  Duplicates are kept: they count
   * in total_num_tokens, not in doc_freq.  NULL = no facets. */
  uint32_t n_facet_terms;
  const uint64_t* facet_off; /* [n_docs+1] or NULL */
  const uint32_t* facet_tok;
} fg_docs_input;

/* Replaces: Index::open_or_create + IndexWriter commit + Searcher snapshot
 * (src/db/core.rs:229-267, :290-297).  Builds the HBM layout of DESIGN.md on
 * device `dev` of ctx. */
int fg_index_build_from_docs(fg_ctx* ctx, int dev, const fg_docs_input* in, fg_index** out);

/* Postings already inverted by the host (SURVEY.md §8b proposal): merged
 * text U name postings per term, CSR by term id, docs ascending. */
typedef struct fg_index_input {
  uint32_t n_docs;
  uint32_t n_terms;
  const uint64_t* term_off;  /* [n_terms+1] */
  const uint32_t* doc;       /* [term_off[n_terms]] */
  const uint16_t* tf_text;   /* 0 when the doc has the term only in `name` */
  const uint16_t* tf_name;   /* 0 when the doc has the term only in `text` */
  const uint8_t* fn_text;    /* [n_docs] fieldnorm ids (fieldnorm/code.rs) */
  const uint8_t* fn_name;    /* [n_docs] */
  uint64_t tot_tokens[2];    /* total_num_tokens of text / name, deleted docs included */
  const uint8_t* deleted;    /* [n_docs] or NULL */
  /* facet postings (doc ids, ascending) per facet term, or NULL */
  uint32_t n_facet_terms;
  const uint64_t* facet_term_off; /* [n_facet_terms+1] */
  const uint32_t* facet_doc;
  uint64_t tot_facet_tokens;      /* total_num_tokens of the facet field */
} fg_index_input;
int fg_index_build(fg_ctx* ctx, int dev, const fg_index_input* in, fg_index** out);
/* ... one segment of a namespace scored with the namespace's statistics g
 * (below): the per-segment build a tantivy host makes for each new segment. */
typedef struct fg_global_stats fg_global_stats;
int fg_index_build_global(fg_ctx* ctx, int dev, const fg_index_input* in, const fg_global_stats* g, fg_index** out);

/* ---- doc-sharded namespace --------------------- */
/* One namespace split into contiguous doc-id ranges, one shard per GPU, each
 * scoring with the namespace's GLOBAL statistics -- exactly tantivy's segment
 * model, where Bm25Weight reads N, total_num_tokens and doc_freq summed over
 * all segments (core/searcher.rs Bm25StatisticsProvider) while each segment
 * runs its own postings.  A shard computes its local statistics with
 * fg_docs_stats, the ranks sum them (one all-reduce), and every shard builds
 * with the sums.  Merging the shard top-k lists by (score desc, shard asc,
 * doc asc) with fg_merge_shards then equals (score desc, global doc asc). */
struct fg_global_stats {
  uint64_t n_docs;           /* N over all shards, deleted docs included */
  uint64_t tot_tokens[2];    /* total_num_tokens(text), (name) over all shards */
  const uint32_t* df_text;   /* [n_terms] doc_freq in `text` over all shards */
  const uint32_t* df_name;   /* [n_terms] doc_freq in `name`, or NULL (all 0) */
  const uint32_t* df_facet;  /* [n_facet_terms] doc_freq in `facet`, or NULL (no facets) */
  uint64_t tot_facet_tokens; /* total_num_tokens(facet) over all shards */
};
/* Local statistics of one shard (host only, no device): df per term and field
 * ([n_terms] each, caller-owned) and the two token totals. */
int fg_docs_stats(const fg_docs_input* in, uint32_t* df_text, uint32_t* df_name, uint64_t* tot_tokens2);
/* ... and of its facet field: df_facet [n_facet_terms], *tot_facet. */
int fg_docs_facet_stats(const fg_docs_input* in, uint32_t* df_facet, uint64_t* tot_facet);
/* fg_index_build_from_docs scored with global statistics (g may be NULL = local).
 * A build whose docs hold fewer than a quarter of the n_terms vocabulary's terms
 * (a commit's new docs) keeps its own term dictionary -- its work and device
 * arrays then scale with its own terms, as a tantivy segment's do -- and every
 * call on the snapshot still takes vocabulary ids (a term it lacks matches
 * nothing; fg_index_stats::n_terms, term_ladder and set_kth_floor speak the
 * vocabulary's size). */
int fg_index_build_from_docs_global(fg_ctx* ctx, int dev, const fg_docs_input* in, const fg_global_stats* g,
                                    fg_index** out);

/* A new snapshot of `base` with other statistics: after a commit added docs
 * elsewhere in the namespace (a new segment) or deleted some.  tantivy's
 * Bm25Weight reads the Searcher's statistics at query time, so every segment
 * scores with the namespace's current N, df and token totals
 * (core/searcher.rs Bm25StatisticsProvider; one segment per commit,
 * src/db/document.rs:65) -- and so does this library: the kernels form each
 * posting's score at query time from its tf and fieldnorm id, so a rescore is
 * host work only (the new weights and tf caches, read by the plans; an upload
 * of the alive bitset when deletions changed).  Every device array stays
 * shared with `base`; the bounds the kernels prune with (computed once when the
 * segment was built) are scaled per query by the ratio of the statistics.
 * `deleted` [n_docs of base] or NULL (none).  g must cover base's own doc
 * frequencies. */
int fg_index_rescore(const fg_index* base, const fg_global_stats* g, const uint8_t* deleted, fg_index** out);
/* n snapshots rescored with ONE set of statistics (a commit's older segments):
 * the BM25 weights computed once and shared.  deleted[i] as fg_index_rescore's
 * (deleted itself may be NULL: none anywhere).  On error no snapshot is made
 * (outs[] all NULL). */
int fg_index_rescore_many(const fg_index* const* bases, uint32_t n, const fg_global_stats* g,
                          const uint8_t* const* deleted, fg_index** outs);
/* on != 0: the calling thread's snapshot builds run on the device's
 * low-priority background stream with their kernels capped at FUGU_BG_GRID
 * workgroups per CU (default 2), so searches beside them -- on high-priority
 * streams -- find wave slots free (fugu's writer / merge threads beside its
 * searchers, src/db/core.rs:247-249).  fg_db's commits and merger use it.
 * Returns the previous setting. */
int fg_thread_background(int on);

int fg_index_retain(fg_index* ix);
int fg_index_release(fg_index* ix);

typedef struct fg_index_stats {
  uint32_t n_docs;
  uint32_t n_terms;
  uint64_t n_postings;
  uint64_t device_bytes;
  uint64_t tot_tokens[2];
  float avgdl[2];
  int has_name;
  int device;
  uint32_t n_facet_terms;
  uint64_t tot_facet_tokens;
  uint32_t n_dense_f32;      /* terms with an f32 score table */
  uint32_t n_rank_terms;     /* terms with rank words */
  uint32_t n_sparse_rank_terms;  /* ... of which sparse rank words (block entries + the words holding docs) */
  uint32_t reserved0;
  uint64_t rank_bytes;       /* device bytes of the rank words, plain and sparse */
} fg_index_stats;
int fg_index_stats_get(const fg_index* ix, fg_index_stats* out);
/* doc_freq of `term` in `field` (tantivy Searcher::doc_freq; FG_FIELD_FACET:
 * a facet term), and the merged (text U name) posting-list length when field < 0. */
uint64_t fg_index_df(const fg_index* ix, int field, uint32_t term);
/* Bm25Weight pieces the device uses, for host-side checks. */
int fg_index_bm25(const fg_index* ix, uint32_t term, float* w_text, float* w_name, float* cache512);
/* The snapshot's per-term K-th best alive posting scores for K = 1, 10, 20, 100,
 * 1000 (0 when the term has fewer alive postings): the starting thresholds of
 * its disjunctions.  out[5].  Exact for a snapshot built (or merged) under its
 * statistics; a snapshot from fg_index_rescore[_many] holds a lower bound
 * instead: the build's K'-th best for the smallest stored K' >= K + the docs
 * deleted since, times the term's smallest current / build posting-score ratio
 * (within ~0.2% for a commit that grows the namespace by 10%). */
int fg_index_term_kth(const fg_index* ix, uint32_t term, float* out);

/* ---- doc-sharded namespaces: namespace-wide starting thresholds ----------------
 * A shard of a doc-sharded namespace (tantivy's segments, config C5) only sees its
 * own docs, so its per-term K-th scores bound the namespace's K-th score far
 * below it (K = 1000 over 8 shards: the namespace's 1000th best is about each
 * shard's 125th).  Every shard's score LADDER -- the K-th best alive score at the
 * ranks FG_LADDER_KS -- is exchanged once at build (an all-gather), combined into
 * per-term lower bounds of the namespace-wide K-th scores, and set on every shard
 * as a floor of its starting thresholds.  Score-only: a doc scoring exactly the
 * floor is still kept (the merge breaks ties by shard).  Results are unchanged;
 * the shards' disjunctions and single-list queries start closer to their final
 * thresholds, as a multi-snapshot plan's shards do through their shared threshold
 * word on one device (reference: Searcher-global statistics, src/db/search.rs:162). */
#define FG_LADDER_LEVELS 14 /* K = 1, 2, 3, 5, 10, 13, 20, 25, 50, 100, 125, 250, 500, 1000 */
/* out[n_terms * FG_LADDER_LEVELS], term-major, ascending K; 0 where the term has
 * fewer alive postings.  Runs one k_ktop pass of the snapshot on the device into
 * temporaries (the calling thread's stream; ~10 ms for a 12.5M-doc shard). */
int fg_index_term_ladder(const fg_index* ix, float* out);
/* Host only: ladders[s] = shard s's fg_index_term_ladder output (n_terms terms
 * each, one vocabulary); out[n_terms * 5] = for K = 1, 10, 20, 100, 1000 the
 * largest score x with sum over shards of max{K_l : ladder_s(K_l) >= x} >= K,
 * i.e. at least K docs of the namespace score >= x: a lower bound of the term's
 * namespace-wide K-th best alive score. */
int fg_kth_floor_combine(uint32_t n_shards, uint32_t n_terms, const float* const* ladders, float* out);
/* Set (or replace; floor = NULL clears) the snapshot's floor of its per-term K-th
 * scores for K = 1, 10, 20, 100, 1000: plans created afterwards start their
 * thresholds from max(own K-th score, floor).  floor[n_terms * 5] is copied; a
 * floor that is not a valid lower bound of the namespace-wide K-th scores can drop
 * hits.  Safe against concurrent plan creation (plans see the old or new floor). */
int fg_index_set_kth_floor(fg_index* ix, const float* floor, uint32_t n_terms);

/* ---- query batches -------------------------------------------------------- */
typedef struct fg_query_batch {
  uint32_t n_queries;
  const uint32_t* q_off;  /* [n_queries+1] */
  const uint32_t* terms;  /* term ids in query order; FG_TERM_MISSING allowed */
  int mode;               /* FG_MODE_AND (Must clauses) or FG_MODE_OR (Should clauses), when occur is NULL */
  /* Facet filters (Dataset::search, src/db/search.rs:129-150), or NULL: per
   * query the flat Should clause list build_facet_query makes (:221-293) --
   * the exact facet terms in filter order, then the prefix terms -- as facet
   * term ids (FG_TERM_MISSING allowed: matches nothing), <= FG_MAX_FACET_CLAUSES.
   *   text terms + clauses : Bool[Must(text query), Must(Should(clauses))],
   *                          score = text score + facet union score;
   *   no text  + clauses   : the facet union alone (empty query + filters);
   *   no text, no clauses  : AllQuery (score 1.0 for every alive doc). */
  const uint32_t* f_off;  /* [n_queries+1] */
  const uint32_t* f_terms;
  /* Per-term occurs parallel to `terms` (FG_OCCUR_*), or NULL (every term is
   * `mode`'s).  tantivy BooleanWeight semantics per query: with a Must clause
   * the Musts intersect and the Shoulds only add score (RequiredOptionalScorer:
   * (0.0 + must score) + Should union); without one the Shoulds' union; MustNot
   * clauses exclude; no Must and no Should: no hits.  A batch may mix shapes. */
  const uint8_t* occur;
} fg_query_batch;

/* Plan a batch: host-side query planning (tantivy Weight creation: terms
 * ordered by cost, query/intersection.rs) and upload of the plan to HBM.
 * Returns FG_EUNSUPPORTED for queries outside the device subset
 * (> FG_MAX_TERMS terms, > FG_MAX_FACET_CLAUSES clauses, k > FG_MAX_K). */
int fg_plan_create(fg_index* ix, const fg_query_batch* q, uint32_t k, fg_plan** out);
/* Plan a batch over n_segs snapshots of ONE device (a namespace's segments,
 * doc shards scored with global statistics, or namespaces of a fan-out query)
 * run by one launch per kernel: query slot s * n_queries + q is query q on
 * ixs[s].  The slots of a query share its threshold score-only (as linked
 * plans do).  Results (fg_plan_execute / fg_plan_results, fg_plan_info's
 * n_queries) are per slot, layout [n_segs][n_queries][k] and [n_segs][n_queries]:
 * the input of fg_merge_shards.  n_segs = 1 is fg_plan_create. */
int fg_plan_create_multi(fg_index* const* ixs, uint32_t n_segs, const fg_query_batch* q, uint32_t k, fg_plan** out);
/* Run a multi-snapshot plan straight to the merged top-k of every batch query
 * (what fg_merge_shards makes of its per-slot lists): one final select over all
 * slots of a query.  Device outputs [n_queries*k] x 3 and [n_queries] (batch
 * queries); slots past d_out_n[q] hold score 0, doc 0, shard 0.  FG_EUNSUPPORTED
 * for a single-snapshot plan or snapshots holding >= 2^32 docs together. */
int fg_plan_execute_merged(fg_plan* p, void* stream, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_shard,
                           uint32_t* d_out_n);
/* Run a planned batch on `stream` (hipStream_t, NULL = default stream).
 * Outputs are device pointers [n_queries*k], [n_queries*k], [n_queries]; NULL
 * outputs use the plan's own buffers.  Asynchronous. */
int fg_plan_execute(fg_plan* p, void* stream, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_n);
/* Link plans of ONE query batch and k on one device (the shards, segments or
 * namespaces one merged result is drawn from) so they prune with one shared
 * per-query threshold and score histogram: a doc below the k-th best score
 * any of them has found cannot enter the merged top-k.  Thresholds are then
 * shared score-only (a doc tied with the k-th score is kept: the merge breaks
 * ties by shard).  plans[0] owns the shared state and zeroes it when executed:
 * execute plans[0] first in every round and the others after it on the same
 * stream (or ordered after it); destroy plans[0] last. */
int fg_plan_link(fg_plan* const* plans, uint32_t n);
/* ---- doc shards on several devices / processes (C5 over N GPUs) ----------
 * Linked plans share their per-query score histograms through memory on one
 * device.  Shards on different GPUs exchange them instead, between PARTS of the
 * k_disj sweep: every rank runs part [0, f) of its plan, the histograms are
 * summed over the ranks (one all-reduce of n_queries * FG_HIST_BINS u32), and
 * part [f, 1) then prunes with the counts of every shard's first part.  The
 * counted docs of different shards are distinct, so the summed histogram's
 * threshold is a lower bound of the namespace's k-th score and the merged
 * top-k is unchanged (a shard's own list may then hold fewer than k hits).
 * Reference: tantivy's Searcher-global statistics, src/db/search.rs:162. */
#define FG_HIST_BINS 512
/* lo[n_queries], hi[n_queries]: the f32 bit patterns the query's histogram bins
 * span (0, 0: no shard of this plan has work for the query).  Before the
 * exchange every rank sets the elementwise MAX over the ranks' spans
 * (fg_plan_set_hist_span), so a bin counts the same scores on every rank. */
int fg_plan_hist_span(const fg_plan* p, uint32_t* lo, uint32_t* hi);
int fg_plan_set_hist_span(fg_plan* p, const uint32_t* lo, const uint32_t* hi);
/* Run the k_disj items [from, to) of the plan's sweep (fractions, 0 <= from <
 * to <= 1; every query's first docs come first).  from = 0 also zeroes the
 * plan's state and runs the facet masks and k_conj; to = 1 also runs the scans
 * and the final select into the outputs (as fg_plan_execute; d_out_shard !=
 * NULL: fg_plan_execute_merged's merged select).  Asynchronous.  Parts run in
 * order, each from where the last ended (FG_EINVAL otherwise). */
int fg_plan_execute_part(fg_plan* p, void* stream, double from, double to, float* d_out_score, uint32_t* d_out_doc,
                         uint32_t* d_out_shard, uint32_t* d_out_n);
/* Copy the plan's histograms [n_queries][FG_HIST_BINS] u32 to (into_plan = 0)
 * or from (1) device memory d_buf of the plan's device, on `stream`. */
int fg_plan_hist_copy(fg_plan* p, void* stream, uint32_t* d_buf, int into_plan);
/* ---- peer plans: thresholds shared DURING a launch, across devices or
 * processes (C5's shards, one per GPU).  Each shard's plan keeps its own
 * per-query threshold and histogram; with peers set, every threshold it
 * publishes and every hit count it adds ALSO go, score-only, into the peers'
 * words of the same batch query (device atomics: in-process peer access, or
 * the peer's workspace mapped through HIP IPC), so every shard prunes with the
 * hits of all of them as they are found, not only between parts.  Peers plan
 * the same batch and k with one histogram span (fg_plan_set_hist_span).  With
 * peers set an execute no longer zeroes the plan's state: before each round
 * call fg_plan_reset on every peer and order all resets before any peer's
 * execute (a barrier across the devices or processes); destroy no plan while
 * a peer can still publish into it.  n = 0 clears the peers. */
#define FG_MAX_PEERS 15
int fg_plan_set_peers(fg_plan* p, fg_plan* const* peers, uint32_t n);
/* A plan's threshold / histogram words as another process maps them. */
typedef struct fg_plan_ipc {
  uint8_t handle[64]; /* hipIpcMemHandle_t of the plan's workspace */
  uint64_t thresh_off, hist_off;
  uint32_t n_queries, k;
  int device;
  uint32_t reserved;
} fg_plan_ipc;
int fg_plan_ipc_export(const fg_plan* p, fg_plan_ipc* out);
int fg_plan_set_ipc_peers(fg_plan* p, const fg_plan_ipc* peers, uint32_t n);
/* Zero the plan's thresholds, histograms and candidate counts on `stream`. */
int fg_plan_reset(fg_plan* p, void* stream);
/* Copy the plan's own result buffers to host (synchronises the plan's stream). */
int fg_plan_results(fg_plan* p, float* out_score, uint32_t* out_doc, uint32_t* out_n);
typedef struct fg_plan_info {
  uint32_t n_queries;
  uint32_t k;
  uint32_t total_chunks;
  uint64_t workspace_bytes;
} fg_plan_info;
int fg_plan_info_get(const fg_plan* p, fg_plan_info* out);
/* Per-kernel HIP-event timing of every execute while enabled.  ms_out[2] =
 * summed device time of (k_fmask + k_conj / k_disj + k_scan, k_final);
 * *n_out = executes.  Resets. */
int fg_plan_profile(fg_plan* p, int enable);
int fg_plan_kernel_ms(fg_plan* p, double* ms_out, uint32_t* n_out);
/* Diagnostics of the last execute: per-query candidate counts (cand_cnt
 * [n_queries], may be NULL) and, in -DFG_DIAG builds only, 8 u64 phase stamps
 * per workgroup (k_conj work items, then k_final queries); FG_EUNSUPPORTED
 * for the stamps in product builds. */
int fg_plan_diag(fg_plan* p, uint64_t* out, size_t n_words, uint32_t* cand_cnt);
int fg_plan_destroy(fg_plan* p);

/* Synchronous convenience: plan + execute + copy back.  Host buffers
 * out_score/out_doc [n_queries*k] in (score desc, doc asc) order, out_n
 * [n_queries] = min(k, hits).  This is the call Dataset::search would make in
 * place of searcher.search(..., TopDocs::with_limit(k)). */
int fg_search_batch(fg_index* ix, const fg_query_batch* q, uint32_t k, float* out_score, uint32_t* out_doc,
                    uint32_t* out_n);

/* Cross-shard merge: per-shard top-k lists gathered from
 * n_shards GPUs (RCCL all-gather) merged into the global top-k by (score
 * desc, shard asc, doc asc).  Device pointers, layout [n_shards][n_queries][k]
 * and [n_shards][n_queries].  Output slots past d_out_n[q] hold score 0, doc 0,
 * shard 0. */
int fg_merge_shards(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* d_score, const uint32_t* d_doc,
                    const uint32_t* d_n, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_shard,
                    uint32_t* d_out_n, void* stream);

/* One batch over the shards of one logical index (SURVEY.md §8b
 * fg_search_sharded, §8e): the segments of a namespace (tantivy's per-commit
 * segments, src/db/document.rs:65, searched and merged by
 * searcher.search(.., TopDocs), src/db/search.rs:162), the doc shards of a
 * namespace built with global statistics, or several namespaces of a fan-out
 * query.  The shards share one term / facet dictionary; a term id >= a shard's
 * n_terms matches nothing there.  Each shard runs on its own device (one
 * process driving the node's GPUs; the shards of one device run as ONE
 * multi-snapshot plan: fg_plan_create_multi), its per-shard top-k is copied
 * over xGMI to shards[0]'s device and merged there
 * into (score desc, shard asc, doc asc) -- merge_fruits over (segment_ord, doc).
 * Host outputs [n_queries*k] (out_shard may be NULL) and out_n [n_queries].
 * ctx, when given, must hold every shard's device.  Thread-safe like
 * fg_search_batch (the calling thread's per-thread streams). */
int fg_search_sharded(fg_ctx* ctx, fg_index* const* shards, uint32_t n_shards, const fg_query_batch* q, uint32_t k,
                      float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n);

/* ---- traffic models (roofline numerators; host analysis, model.cpp) --------- */
/* The loads k_conj / k_disj issue for a batch, replayed on the host over this
 * snapshot's layout (needs keep_host_postings, reads the score,
 * bound and directory tables back from the device).  thr_score[i] = query i's
 * final k-th best score: the replay prunes as an exact MaxScore kernel at that
 * threshold must at least (k_conj's bounds after each list and a single
 * list's block-max chunk skip; k_disj's tile split and both bounds); NULL =
 * k_conj's exhaustive cascade (k_disj at threshold 0).  Pure Must and pure
 * Should queries only (FG_EINVAL otherwise).  per_query[4*i..] (may be NULL) =
 * {stream, probe, output, total} bytes of query i. */
typedef struct fg_model_out {
  double stream_bytes;     /* lead / essential postings (doc + score); k_disj's per-(tile, clause) ranges + bounds */
  double probe_bytes;      /* other lists: rank words, posting scores, directory steps, bucket maxima */
  double output_bytes;     /* 8 B per kept key, <= k per query */
  double alg_bytes;        /* their sum: the algorithmic bytes of the launch */
  double line_bytes;       /* 128 B x the distinct 128-B lines those loads touch in the launch: the line floor */
  double query_line_bytes; /* 128 B x sum over queries of the distinct lines each touches (no cross-query reuse) */
  double loads;            /* modelled loads (lanes) */
  double candidates;       /* docs the replay keeps (at the threshold) */
} fg_model_out;
int fg_model_batch(const fg_index* ix, const fg_query_batch* q, uint32_t k, const float* thr_score, double* per_query,
                   fg_model_out* out);

/* SURVEY.md §8(d) algorithmic bytes of tantivy's CPU walk per query: out[4*i..]
 * = {B_merge, B_skip, B, |I|} (1 KiB block decode per probed 128-posting block;
 * not bytes the device layout reads). */
int fg_bytes_model(const fg_index* ix, const fg_query_batch* q, uint32_t k, double* out);
/* fg_model_batch's per-query bytes with no threshold (FG_MODE_AND: k_conj's
 * exhaustive cascade -- 8 B per lead posting, then per candidate still alive
 * 8 B rank word + 4 B score on a hit, or 8 B bucket bounds + 4 B per search
 * step + 4 B final compare + 4 B score on a hit; 8 B per kept key) or, for
 * FG_MODE_OR, k_disj at threshold 0. */
int fg_bytes_model_gpu(const fg_index* ix, const fg_query_batch* q, uint32_t k, double* out);
/* fg_model_batch's per-query bytes at thresholds thr_score (k_disj / k_conj). */
int fg_bytes_model_or(const fg_index* ix, const fg_query_batch* q, uint32_t k, const float* thr_score, double* out);

#ifdef __cplusplus
}
#endif
#endif /* FUGU_H */
