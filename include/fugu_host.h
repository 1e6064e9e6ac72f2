/*
 * fugu_host.h -- the host side of fugu's search path above the device ABI
 * (include/fugu.h), written in C++ because the reference's toolchain (Rust)
 * is absent.  It mirrors, name for name, the reference pieces
 * around the replaced call:
 *
 *   fg_db_*            DatasetManager (src/db/config.rs:91-331): namespace
 *                      registry; create/delete are the routes the CLI speaks
 *                      but the server lacks (cli.rs:241-243, 280-282)
 *   fg_db_upsert       NamedIndex::upsert for the docs index
 *                      (src/db/document.rs:23-67, build_full_document :116-139):
 *                      ObjectRecord::validate (src/object.rs:31-78), delete by
 *                      the RAW id term, index `text` and metadata["name"]
 *   fg_db_commit       IndexWriter::commit + reader reload: rebuilds the
 *                      namespace's immutable device snapshot (fg_index)
 *   fg_db_add_file     POST /add/{namespace} (cli.rs:392-397, types.rs:71-75)
 *   fg_db_search       Dataset::search (src/db/search.rs:74-218): QueryParser
 *                      over [text, name], TopDocs::with_limit(offset+per_page)
 *                      on the GPU, doc fetch, skip(offset).take(per_page)
 *   fg_db_search_json  perform_search (src/server/handlers/search.rs:350-402)
 *                      + the response shapes of the GET /search, POST /search
 *                      and POST /search/{namespace} handlers (Appendix B)
 *   fg_analyze         the "default" analyzer (SimpleTokenizer ->
 *                      RemoveLongFilter(40) -> LowerCaser)
 *   fg_parse_query     the QueryParser subset the device runs
 *
 * Queries outside the device subset (phrases, field:, -, boosts, empty =
 * AllQuery, facet filters) return FG_EUNSUPPORTED: the
 * reference host then runs tantivy; this library never answers them on the CPU.
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
#define FG_SHAPE_GET_SEARCH 0  /* GET /search, GET /search/{q}: SearchResponse, text stripped unless asked */
#define FG_SHAPE_POST_SEARCH 1 /* POST /search, POST /search/{namespace}: status/query/filters/page/... */

/* ctx may be NULL: the registry, upserts and doc store then work on the host
 * alone and fg_db_commit fails with FG_ENODEV (CPU tests of the host logic). */
int fg_db_create(fg_ctx* ctx, int dev, const char* default_namespace, fg_db** out);
int fg_db_destroy(fg_db* db);
int fg_db_namespace_create(fg_db* db, const char* name);
int fg_db_namespace_delete(fg_db* db, const char* name);
/* {"status":"success","namespaces":[...]} (handlers/namespaces.rs:24-30), names sorted */
int fg_db_namespaces_json(fg_db* db, char* out, size_t cap, size_t* len);

int fg_db_upsert(fg_db* db, const char* ns, const char* id, const char* text, const char* name,
                 const char* metadata_json);
int fg_db_commit(fg_db* db, const char* ns);
int fg_db_add_file(fg_db* db, const char* ns, const char* name, const char* body);
/* docs stored in the namespace (deleted included = tantivy max_doc) and alive ones */
int fg_db_doc_count(fg_db* db, const char* ns, uint64_t* total, uint64_t* alive);

typedef struct fg_hit {
  float score;
  uint32_t doc; /* global doc id in the namespace (insertion order) */
} fg_hit;
/* Dataset::search: hits of page `page` (per_page each), *n_out <= per_page. */
int fg_db_search(fg_db* db, const char* ns, const char* query, uint32_t page, uint32_t per_page, fg_hit* out,
                 uint32_t cap, uint32_t* n_out);
/* perform_search + handler response JSON (per_page clamp 1..100 else 20). */
int fg_db_search_json(fg_db* db, const char* ns, const char* query, uint32_t page, uint32_t per_page,
                      int include_text, int shape, char* out, size_t cap, size_t* len);

/* Analyzer / parser exposed for tests: tokens separated by '\n'. */
int fg_analyze(const char* text, char* out, size_t cap, size_t* len);
/* mode (FG_MODE_AND / FG_MODE_OR) and the analyzed terms ('\n'-separated). */
int fg_parse_query(const char* query, int* mode, char* out, size_t cap, size_t* len);

#ifdef __cplusplus
}
#endif
#endif /* FUGU_HOST_H */
