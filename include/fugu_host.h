/*
 * fugu_host.h -- the host side of fugu's search path above the device ABI
 * (include/fugu.h), written in C++ because the reference's toolchain (Rust)
 * is absent.  It mirrors, name for name, the reference pieces
 * around the replaced call:
 *
 *   fg_db_*            DatasetManager (src/db/config.rs:91-331): namespace
 *                      registry; create/delete are the routes the CLI speaks
 *                      but the server lacks (cli.rs:241-243, 280-282)
 *   fg_db_upsert_record NamedIndex::upsert for the docs index
 *                      (src/db/document.rs:23-67, build_full_document :116-184):
 *                      ObjectRecord::validate (src/object.rs:31-78), delete by
 *                      the RAW id term, index `text`, metadata["name"] and the
 *                      facets (get_all_facet_paths, document.rs:277-309)
 *   fg_db_upsert       the same with `name` given directly (no namespace facets)
 *   fg_db_commit       IndexWriter::commit + reader reload: rebuilds the
 *                      namespace's immutable device snapshot (fg_index)
 *   fg_db_add_file     POST /add/{namespace} (cli.rs:392-397, types.rs:71-75)
 *   fg_db_search_ex    Dataset::search (src/db/search.rs:74-218): QueryParser
 *                      over [text, name], facet filters (build_facet_query,
 *                      :221-324), TopDocs::with_limit(offset+per_page) on the
 *                      GPU, doc fetch, skip(offset).take(per_page)
 *   fg_db_search_json  perform_search (src/server/handlers/search.rs:350-402)
 *                      + the response shapes of the GET /search, POST /search
 *                      and POST /search/{namespace} handlers (Appendix B)
 *   fg_analyze         the "default" analyzer (SimpleTokenizer ->
 *                      RemoveLongFilter(40) -> LowerCaser)
 *   fg_parse_query     the QueryParser subset the device runs
 *
 * Queries outside the device subset (phrases, field:, -, boosts, a text
 * query with filters that parse to no facet term) return FG_EUNSUPPORTED: the
 * reference host then runs tantivy; this library never answers them on the CPU.
 * Empty queries (AllQuery), facet-only queries and text + facet filters run
 * on the device.
 */
#ifndef FUGU_HOST_H
#define FUGU_HOST_H

#include "fugu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fg_db fg_db;

#define FG_ENOTFOUND (-6) /* namespace not found: "Namespace '...' not found" */
#define FG_EEXIST (-7)    /* namespace already exists */

/* Response shapes. */
/* Every response is a serde_json Value in the reference, so object keys come out
 * in byte order (serde_json without preserve_order, Cargo.lock:4313-4322), and
 * stored metadata is re-serialized the same way (sorted keys, serde numbers). */
#define FG_SHAPE_GET_SEARCH 0  /* GET /search: {page, per_page, query, results, total}, text stripped unless asked */
#define FG_SHAPE_POST_SEARCH 1 /* POST /search, POST /search/{namespace}: {filters, page, per_page, query,
                                * results, status, total}, text kept, no per_page clamp */
#define FG_SHAPE_GET_SEARCH_PATH 2 /* GET /search/{query} (handlers/search.rs:79-139): `query` is the URL-encoded
                                    * path component (decoded here; bad UTF-8 -> 400 "Invalid URL encoding in
                                    * query", FG_EINVAL); page 0, per_page 20 */

/* ctx may be NULL: the registry, upserts and doc store then work on the host
 * alone and fg_db_commit fails with FG_ENODEV (CPU tests of the host logic). */
int fg_db_create(fg_ctx* ctx, int dev, const char* default_namespace, fg_db** out);
int fg_db_destroy(fg_db* db);
int fg_db_namespace_create(fg_db* db, const char* name);
int fg_db_namespace_delete(fg_db* db, const char* name);
/* {"namespaces":[...],"status":"success"} (handlers/namespaces.rs:24-30), names sorted */
int fg_db_namespaces_json(fg_db* db, char* out, size_t cap, size_t* len);

/* ObjectRecord (src/object.rs:8-27) as the upsert routes receive it. */
typedef struct fg_object_record {
  const char* id;
  const char* text;
  const char* metadata_json;    /* a JSON object, or NULL (metadata: None) */
  const char* namespace_;       /* ObjectRecord.namespace, or NULL */
  const char* organization;     /* or NULL */
  const char* conversation_id;  /* or NULL */
  const char* data_type;        /* or NULL */
  const char* const* facets;    /* ObjectRecord.facets: n_facets paths when has_facets */
  uint32_t n_facets;
  int has_facets;               /* Some(facets) (even empty) vs None */
} fg_object_record;
int fg_db_upsert_record(fg_db* db, const char* ns, const fg_object_record* rec);
/* POST /batch/upsert (src/server/handlers/ingest.rs:160-220, Dataset::
 * batch_upsert src/db/document.rs:70-73): n records {id, text} (no metadata,
 * namespace or facets) as two byte buffers with offsets [n+1]; every record is
 * validated before any is upserted, then one commit (one segment), as
 * NamedIndex::upsert commits once per call (src/db/document.rs:65). */
int fg_db_upsert_batch(fg_db* db, const char* ns, uint32_t n, const char* ids, const uint64_t* id_off,
                       const char* texts, const uint64_t* text_off);
int fg_db_upsert(fg_db* db, const char* ns, const char* id, const char* text, const char* name,
                 const char* metadata_json);
/* IndexWriter::commit (src/db/document.rs:65): the docs since the last commit
 * become a segment, the older segments are rescored with the new statistics
 * and pick up the deletes of the upserts since the last commit (a delete takes
 * effect at the commit, as delete_term does; a merge in between neither drops
 * nor flags the doc).  When 8 segments of one size level have accumulated
 * (tantivy's LogMergePolicy) the namespace is queued for the background merger:
 * the run becomes one segment, built and rescored off the commit path and
 * swapped in between commits; readers keep the snapshot they hold. */
int fg_db_commit(fg_db* db, const char* ns);
/* Block until no merge of the namespace is queued or running (tests, shutdown);
 * FG_EHIP with the message when a background merge failed. */
int fg_db_merge_wait(fg_db* db, const char* ns);
typedef struct fg_merge_info {
  uint64_t merges;           /* merges done */
  uint64_t merged_docs;      /* alive docs written by them */
  double merge_ms_total, merge_ms_last, merge_ms_max;
  uint32_t segments;         /* segments of the current snapshot */
  int pending;               /* a merge is queued or running */
  uint64_t n_docs_stats;     /* the namespace's BM25 statistics: N (deleted-not-merged included) */
  uint64_t tot_tokens[2];    /* total_num_tokens(text), (name) */
  uint64_t tot_facet_tokens; /* total_num_tokens(facet) */
} fg_merge_info;
int fg_db_merge_info_get(fg_db* db, const char* ns, fg_merge_info* out);
/* The merge policy alone (host only): given the namespace's segments in doc
 * order (their doc counts), the contiguous run [*j0, *j1) the merger merges
 * next, *j0 == *j1 when none (tantivy LogMergePolicy levels, contiguous runs;
 * FUGU_MERGE_MAX_DOCS = set_max_docs_before_merge, default 10M). */
int fg_merge_policy_pick(const uint64_t* seg_docs, uint32_t n_segs, uint32_t* j0, uint32_t* j1);
/* Global doc ids of segment `seg` of the current snapshot, in its doc order:
 * *n = its size, out[0..min(n, cap)) (out may be NULL). */
int fg_db_segment_docs(fg_db* db, const char* ns, uint32_t seg, uint32_t* out, uint32_t cap, uint32_t* n);
int fg_db_add_file(fg_db* db, const char* ns, const char* name, const char* body);
/* docs stored in the namespace (deleted included = tantivy max_doc) and alive ones */
int fg_db_doc_count(fg_db* db, const char* ns, uint64_t* total, uint64_t* alive);

typedef struct fg_hit {
  float score;
  uint32_t doc; /* global doc id in the namespace (insertion order) */
} fg_hit;
/* Dataset::search: hits of page `page` (per_page each), *n_out <= per_page.
 * filters: the request's `filters` strings (FuguSearchQuery / JsonQueryRequest). */
int fg_db_search_ex(fg_db* db, const char* ns, const char* query, const char* const* filters, uint32_t n_filters,
                    uint32_t page, uint32_t per_page, fg_hit* out, uint32_t cap, uint32_t* n_out);
int fg_db_search(fg_db* db, const char* ns, const char* query, uint32_t page, uint32_t per_page, fg_hit* out,
                 uint32_t cap, uint32_t* n_out);
/* Phase times of every search of the process while enabled (all threads):
 * out_ms[0..5] = parse + dictionary, host planning (+ upload queued), launches,
 * kernels + merge + D2H until the hits are on the host, JSON doc fetch +
 * serialization, the whole fg_db_search* call; *calls = fg_db_search* calls.
 * Reading resets the sums; enable: 1 on, 0 off, -1 unchanged.  Off by default
 * (one relaxed load per phase boundary). */
#define FG_SEARCH_PHASES 6
int fg_search_trace(int enable, double* out_ms, uint32_t n, uint64_t* calls);
/* perform_search + handler response JSON (per_page clamp 1..100 else 20). */
int fg_db_search_json_ex(fg_db* db, const char* ns, const char* query, const char* const* filters,
                         uint32_t n_filters, uint32_t page, uint32_t per_page, int include_text, int shape, char* out,
                         size_t cap, size_t* len);
int fg_db_search_json(fg_db* db, const char* ns, const char* query, uint32_t page, uint32_t per_page,
                      int include_text, int shape, char* out, size_t cap, size_t* len);
/* POST /search/json (query_json_post, handlers/search.rs:210-301): the
 * JsonQueryRequest fields and the ?text= / ?include_data= URL flags, each flag
 * tri-state (-1 absent, 0 false, 1 true); has_page = 0 means no `page` object
 * (page 0, per_page 20).  Text: the URL flag wins, a disagreeing body flag adds
 * "developer_message"; "includes_data_objects" = body flag, else URL flag, else
 * not targeting; "targeting_conversations_or_organizations" = a filter
 * containing /conversation or /organization (handlers/utils.rs:4-14). */
int fg_db_search_json_post(fg_db* db, const char* ns, const char* query, const char* const* filters,
                           uint32_t n_filters, int has_page, uint32_t page, uint32_t per_page, int url_text,
                           int body_text, int url_include_data, int body_include_data, char* out, size_t cap,
                           size_t* len);
/* Stored facets of doc `doc` as Facet Display strings, '\n'-separated. */
int fg_db_doc_facets(fg_db* db, const char* ns, uint32_t doc, char* out, size_t cap, size_t* len);

/* Analyzer / parser exposed for tests: tokens separated by '\n'. */
int fg_analyze(const char* text, char* out, size_t cap, size_t* len);
/* mode (FG_MODE_AND / FG_MODE_OR: every clause Must / Should; FG_MODE_MIXED
 * otherwise) and the analyzed terms ('\n'-separated). */
#define FG_MODE_MIXED 2
int fg_parse_query(const char* query, int* mode, char* out, size_t cap, size_t* len);
/* The terms with their occurs: one line per term, "<o>:<term>", o = FG_OCCUR_*
 * ('0' Must, '1' Should, '2' MustNot). */
int fg_parse_query_occur(const char* query, char* out, size_t cap, size_t* len);
/* FacetTokenizer tokens of Facet::from_text(path), '\n'-separated; the
 * encoded facets keep their U+0000 separators, so read *len bytes. */
int fg_facet_tokens(const char* path, char* out, size_t cap, size_t* len);
/* build_facet_query's clause list for `filters` (encoded facet terms,
 * '\n'-separated, *len bytes); *applies = some filter survives the wildcard
 * split; *all_query = none parsed into a term (facet_query = AllQuery). */
int fg_facet_clauses(const char* const* filters, uint32_t n_filters, int* applies, int* all_query, char* out,
                     size_t cap, size_t* len);

#ifdef __cplusplus
}
#endif
#endif /* FUGU_HOST_H */
