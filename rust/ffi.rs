//! Rust binding of libfugu's C ABI (`include/fugu.h`, `include/fugu_host.h`) as
//! fugu would declare it (`src/gpu/ffi.rs`).  The seam it
//! serves: `searcher.search(&base_query, &TopDocs::with_limit(n))` inside
//! `Dataset::search` (reference `src/db/search.rs:162`); the host-side entry
//! points (`fg_db_*`) mirror `Dataset` / `DatasetManager` and the `/search*`
//! handlers for hosts without tantivy (the C++ host in `fugu_amd/csrc/host.cpp`).
//!
//! No Rust toolchain exists in this build environment, so this file is not
//! compiled here.  `tests/test_rust_ffi.py` parses it and checks every function
//! (name, arity, argument and return types in order) and every `#[repr(C)]`
//! struct (field names and types in order) against the two headers, so it
//! fails on any header drift.  Types: `int` = `c_int`, `size_t` = `usize`,
//! `T*` = `*mut T`, `const T*` = `*const T`, `T* const*` = `*const *mut T`.
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

// ---- opaque handles
#[repr(C)] pub struct fg_ctx { _p: [u8; 0] }
#[repr(C)] pub struct fg_index { _p: [u8; 0] }
#[repr(C)] pub struct fg_plan { _p: [u8; 0] }
#[repr(C)] pub struct fg_db { _p: [u8; 0] }

// ---- constants (fugu.h)
pub const FG_ABI_VERSION: c_int = 5;  // checked against fg_abi_version() before any struct is passed
pub const FG_OK: c_int = 0;
pub const FG_EINVAL: c_int = -1;
pub const FG_ENODEV: c_int = -2;
pub const FG_EOOM: c_int = -3;
pub const FG_EHIP: c_int = -4;
pub const FG_EUNSUPPORTED: c_int = -5;  // outside the device subset: run tantivy's CPU path
pub const FG_MAX_TERMS: u32 = 16;
pub const FG_MAX_FACET_CLAUSES: u32 = 8;
pub const FG_MAX_K: u32 = 1024;
pub const FG_HIST_BINS: u32 = 512;
pub const FG_MAX_SEGMENTS: u32 = 64;
pub const FG_TERM_MISSING: u32 = 0xFFFF_FFFF;
pub const FG_MODE_AND: c_int = 0;
pub const FG_MODE_OR: c_int = 1;
pub const FG_OCCUR_MUST: u8 = 0;      // tantivy Occur, per term of a query
pub const FG_OCCUR_SHOULD: u8 = 1;
pub const FG_OCCUR_MUST_NOT: u8 = 2;
pub const FG_FIELD_TEXT: c_int = 0;
pub const FG_FIELD_NAME: c_int = 1;
pub const FG_FIELD_FACET: c_int = 2;

// ---- structs (fugu.h)
#[repr(C)]
pub struct fg_docs_input {
    pub n_docs: u32,
    pub n_terms: u32,
    pub text_off: *const u64,
    pub text_tok: *const u32,
    pub name_off: *const u64,
    pub name_tok: *const u32,
    pub deleted: *const u8,
    pub threads: c_int,
    pub keep_host_postings: c_int,
    pub n_facet_terms: u32,
    pub facet_off: *const u64,
    pub facet_tok: *const u32,
}

#[repr(C)]
pub struct fg_index_input {
    pub n_docs: u32,
    pub n_terms: u32,
    pub term_off: *const u64,       // [n_terms + 1]
    pub doc: *const u32,            // merged text ∪ name postings, ascending per term
    pub tf_text: *const u16,
    pub tf_name: *const u16,
    pub fn_text: *const u8,         // fieldnorm ids per doc
    pub fn_name: *const u8,
    pub tot_tokens: [u64; 2],       // total_num_tokens(text), (name), deleted docs included
    pub deleted: *const u8,
    pub n_facet_terms: u32,
    pub facet_term_off: *const u64,
    pub facet_doc: *const u32,
    pub tot_facet_tokens: u64,
}

#[repr(C)]
pub struct fg_global_stats {        // the Searcher's Bm25StatisticsProvider, summed over segments
    pub n_docs: u64,
    pub tot_tokens: [u64; 2],
    pub df_text: *const u32,
    pub df_name: *const u32,
    pub df_facet: *const u32,
    pub tot_facet_tokens: u64,
}

#[repr(C)]
pub struct fg_index_stats {
    pub n_docs: u32,
    pub n_terms: u32,
    pub n_postings: u64,
    pub device_bytes: u64,
    pub tot_tokens: [u64; 2],
    pub avgdl: [f32; 2],
    pub has_name: c_int,
    pub device: c_int,
    pub n_facet_terms: u32,
    pub tot_facet_tokens: u64,
    pub n_dense_f32: u32,
    pub n_rank_terms: u32,
    pub n_sparse_rank_terms: u32,
    pub reserved0: u32,
    pub rank_bytes: u64,
}

#[repr(C)]
pub struct fg_query_batch {
    pub n_queries: u32,
    pub q_off: *const u32,
    pub terms: *const u32,          // empty range = empty text query (AllQuery, or the filter alone)
    pub mode: c_int,
    pub f_off: *const u32,          // [n_queries + 1] facet clauses per query, or null
    pub f_terms: *const u32,
    pub occur: *const u8,           // per term FG_OCCUR_*, parallel to `terms`, or null
}

#[repr(C)]
pub struct fg_plan_ipc {
    pub handle: [u8; 64],           // hipIpcMemHandle_t of the plan's workspace
    pub thresh_off: u64,
    pub hist_off: u64,
    pub n_queries: u32,
    pub k: u32,
    pub device: c_int,
    pub reserved: u32,
}

#[repr(C)]
pub struct fg_plan_info {
    pub n_queries: u32,
    pub k: u32,
    pub total_chunks: u32,
    pub workspace_bytes: u64,
}

#[repr(C)]
pub struct fg_model_out {
    pub stream_bytes: f64,
    pub probe_bytes: f64,
    pub output_bytes: f64,
    pub alg_bytes: f64,
    pub line_bytes: f64,
    pub query_line_bytes: f64,
    pub loads: f64,
    pub candidates: f64,
}

// ---- structs (fugu_host.h)
#[repr(C)]
pub struct fg_object_record {       // ObjectRecord (src/object.rs:8-27)
    pub id: *const c_char,
    pub text: *const c_char,
    pub metadata_json: *const c_char,
    pub namespace_: *const c_char,
    pub organization: *const c_char,
    pub conversation_id: *const c_char,
    pub data_type: *const c_char,
    pub facets: *const *const c_char,
    pub n_facets: u32,
    pub has_facets: c_int,
}

#[repr(C)]
pub struct fg_merge_info {
    pub merges: u64,
    pub merged_docs: u64,
    pub merge_ms_total: f64,
    pub merge_ms_last: f64,
    pub merge_ms_max: f64,
    pub segments: u32,
    pub pending: c_int,
    pub n_docs_stats: u64,
    pub tot_tokens: [u64; 2],
    pub tot_facet_tokens: u64,
}

#[repr(C)]
pub struct fg_hit {
    pub score: f32,
    pub doc: u32,
}

extern "C" {
    // ---- context (fugu.h)
    pub fn fg_device_count(out: *mut c_int) -> c_int;
    pub fn fg_ctx_create(ndev: c_int, devs: *const c_int, out: *mut *mut fg_ctx) -> c_int;
    pub fn fg_ctx_destroy(ctx: *mut fg_ctx) -> c_int;
    pub fn fg_ctx_peer_access(ctx: *const fg_ctx, a: c_int, b: c_int, enabled: *mut c_int) -> c_int;
    pub fn fg_last_error() -> *const c_char;
    pub fn fg_version() -> *const c_char;
    pub fn fg_abi_version() -> c_int;

    // ---- index snapshots: one per tantivy segment (src/db/core.rs:229-297)
    pub fn fg_index_build_from_docs(ctx: *mut fg_ctx, dev: c_int, inp: *const fg_docs_input,
                                    out: *mut *mut fg_index) -> c_int;
    pub fn fg_index_build(ctx: *mut fg_ctx, dev: c_int, inp: *const fg_index_input, out: *mut *mut fg_index) -> c_int;
    pub fn fg_index_build_global(ctx: *mut fg_ctx, dev: c_int, inp: *const fg_index_input, g: *const fg_global_stats,
                                 out: *mut *mut fg_index) -> c_int;
    pub fn fg_docs_stats(inp: *const fg_docs_input, df_text: *mut u32, df_name: *mut u32, tot_tokens2: *mut u64)
                         -> c_int;
    pub fn fg_docs_facet_stats(inp: *const fg_docs_input, df_facet: *mut u32, tot_facet: *mut u64) -> c_int;
    pub fn fg_index_build_from_docs_global(ctx: *mut fg_ctx, dev: c_int, inp: *const fg_docs_input,
                                           g: *const fg_global_stats, out: *mut *mut fg_index) -> c_int;
    pub fn fg_index_rescore(base: *const fg_index, g: *const fg_global_stats, deleted: *const u8,
                            out: *mut *mut fg_index) -> c_int;
    pub fn fg_index_rescore_many(bases: *const *const fg_index, n: u32, g: *const fg_global_stats,
                                 deleted: *const *const u8, outs: *mut *mut fg_index) -> c_int;
    pub fn fg_thread_background(on: c_int) -> c_int;
    pub fn fg_index_retain(ix: *mut fg_index) -> c_int;
    pub fn fg_index_release(ix: *mut fg_index) -> c_int;
    pub fn fg_index_stats_get(ix: *const fg_index, out: *mut fg_index_stats) -> c_int;
    pub fn fg_index_df(ix: *const fg_index, field: c_int, term: u32) -> u64;
    pub fn fg_index_bm25(ix: *const fg_index, term: u32, w_text: *mut f32, w_name: *mut f32, cache512: *mut f32)
                         -> c_int;
    pub fn fg_index_term_kth(ix: *const fg_index, term: u32, out: *mut f32) -> c_int;  // K = 1, 10, 20, 100, 1000
    pub fn fg_index_term_ladder(ix: *const fg_index, out: *mut f32) -> c_int;  // [n_terms * FG_LADDER_LEVELS]
    pub fn fg_kth_floor_combine(n_shards: u32, n_terms: u32, ladders: *const *const f32, out: *mut f32) -> c_int;
    pub fn fg_index_set_kth_floor(ix: *mut fg_index, floor: *const f32, n_terms: u32) -> c_int;

    // ---- query batches: the searcher.search(.., TopDocs::with_limit(k)) replacement
    pub fn fg_plan_create(ix: *mut fg_index, q: *const fg_query_batch, k: u32, out: *mut *mut fg_plan) -> c_int;
    pub fn fg_plan_create_multi(ixs: *const *mut fg_index, n_segs: u32, q: *const fg_query_batch, k: u32,
                                out: *mut *mut fg_plan) -> c_int;
    pub fn fg_plan_execute_merged(p: *mut fg_plan, stream: *mut c_void, d_out_score: *mut f32, d_out_doc: *mut u32,
                                  d_out_shard: *mut u32, d_out_n: *mut u32) -> c_int;
    pub fn fg_plan_execute(p: *mut fg_plan, stream: *mut c_void, d_out_score: *mut f32, d_out_doc: *mut u32,
                           d_out_n: *mut u32) -> c_int;
    pub fn fg_plan_link(plans: *const *mut fg_plan, n: u32) -> c_int;
    pub fn fg_plan_hist_span(p: *const fg_plan, lo: *mut u32, hi: *mut u32) -> c_int;
    pub fn fg_plan_set_hist_span(p: *mut fg_plan, lo: *const u32, hi: *const u32) -> c_int;
    pub fn fg_plan_execute_part(p: *mut fg_plan, stream: *mut c_void, from: f64, to: f64, d_out_score: *mut f32,
                                d_out_doc: *mut u32, d_out_shard: *mut u32, d_out_n: *mut u32) -> c_int;
    pub fn fg_plan_hist_copy(p: *mut fg_plan, stream: *mut c_void, d_buf: *mut u32, into_plan: c_int) -> c_int;
    pub fn fg_plan_set_peers(p: *mut fg_plan, peers: *const *mut fg_plan, n: u32) -> c_int;
    pub fn fg_plan_ipc_export(p: *const fg_plan, out: *mut fg_plan_ipc) -> c_int;
    pub fn fg_plan_set_ipc_peers(p: *mut fg_plan, peers: *const fg_plan_ipc, n: u32) -> c_int;
    pub fn fg_plan_reset(p: *mut fg_plan, stream: *mut c_void) -> c_int;
    pub fn fg_plan_results(p: *mut fg_plan, out_score: *mut f32, out_doc: *mut u32, out_n: *mut u32) -> c_int;
    pub fn fg_plan_info_get(p: *const fg_plan, out: *mut fg_plan_info) -> c_int;
    pub fn fg_plan_profile(p: *mut fg_plan, enable: c_int) -> c_int;
    pub fn fg_plan_kernel_ms(p: *mut fg_plan, ms_out: *mut f64, n_out: *mut u32) -> c_int;
    pub fn fg_plan_diag(p: *mut fg_plan, out: *mut u64, n_words: usize, cand_cnt: *mut u32) -> c_int;
    pub fn fg_plan_destroy(p: *mut fg_plan) -> c_int;
    pub fn fg_search_batch(ix: *mut fg_index, q: *const fg_query_batch, k: u32, out_score: *mut f32,
                           out_doc: *mut u32, out_n: *mut u32) -> c_int;
    pub fn fg_merge_shards(n_shards: u32, n_queries: u32, k: u32, d_score: *const f32, d_doc: *const u32,
                           d_n: *const u32, d_out_score: *mut f32, d_out_doc: *mut u32, d_out_shard: *mut u32,
                           d_out_n: *mut u32, stream: *mut c_void) -> c_int;
    pub fn fg_search_sharded(ctx: *mut fg_ctx, shards: *const *mut fg_index, n_shards: u32, q: *const fg_query_batch,
                             k: u32, out_score: *mut f32, out_doc: *mut u32, out_shard: *mut u32, out_n: *mut u32)
                             -> c_int;

    // ---- traffic models (measurement only)
    pub fn fg_model_batch(ix: *const fg_index, q: *const fg_query_batch, k: u32, thr_score: *const f32,
                          per_query: *mut f64, out: *mut fg_model_out) -> c_int;
    pub fn fg_bytes_model(ix: *const fg_index, q: *const fg_query_batch, k: u32, out: *mut f64) -> c_int;
    pub fn fg_bytes_model_gpu(ix: *const fg_index, q: *const fg_query_batch, k: u32, out: *mut f64) -> c_int;
    pub fn fg_bytes_model_or(ix: *const fg_index, q: *const fg_query_batch, k: u32, thr_score: *const f32,
                             out: *mut f64) -> c_int;

    // ---- host mirror (fugu_host.h): DatasetManager / Dataset / the /search* handlers
    pub fn fg_db_create(ctx: *mut fg_ctx, dev: c_int, default_namespace: *const c_char, out: *mut *mut fg_db) -> c_int;
    pub fn fg_db_destroy(db: *mut fg_db) -> c_int;
    pub fn fg_db_namespace_create(db: *mut fg_db, name: *const c_char) -> c_int;
    pub fn fg_db_namespace_delete(db: *mut fg_db, name: *const c_char) -> c_int;
    pub fn fg_db_namespaces_json(db: *mut fg_db, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn fg_db_upsert_record(db: *mut fg_db, ns: *const c_char, rec: *const fg_object_record) -> c_int;
    pub fn fg_db_upsert_batch(db: *mut fg_db, ns: *const c_char, n: u32, ids: *const c_char, id_off: *const u64,
                              texts: *const c_char, text_off: *const u64) -> c_int;
    pub fn fg_db_upsert(db: *mut fg_db, ns: *const c_char, id: *const c_char, text: *const c_char,
                        name: *const c_char, metadata_json: *const c_char) -> c_int;
    pub fn fg_db_commit(db: *mut fg_db, ns: *const c_char) -> c_int;
    pub fn fg_db_merge_wait(db: *mut fg_db, ns: *const c_char) -> c_int;
    pub fn fg_db_merge_info_get(db: *mut fg_db, ns: *const c_char, out: *mut fg_merge_info) -> c_int;
    pub fn fg_merge_policy_pick(seg_docs: *const u64, n_segs: u32, j0: *mut u32, j1: *mut u32) -> c_int;
    pub fn fg_db_segment_docs(db: *mut fg_db, ns: *const c_char, seg: u32, out: *mut u32, cap: u32, n: *mut u32)
                              -> c_int;
    pub fn fg_db_add_file(db: *mut fg_db, ns: *const c_char, name: *const c_char, body: *const c_char) -> c_int;
    pub fn fg_db_doc_count(db: *mut fg_db, ns: *const c_char, total: *mut u64, alive: *mut u64) -> c_int;
    pub fn fg_db_search_ex(db: *mut fg_db, ns: *const c_char, query: *const c_char, filters: *const *const c_char,
                           n_filters: u32, page: u32, per_page: u32, out: *mut fg_hit, cap: u32, n_out: *mut u32)
                           -> c_int;
    pub fn fg_db_search(db: *mut fg_db, ns: *const c_char, query: *const c_char, page: u32, per_page: u32,
                        out: *mut fg_hit, cap: u32, n_out: *mut u32) -> c_int;
    pub fn fg_search_trace(enable: c_int, out_ms: *mut f64, n: u32, calls: *mut u64) -> c_int;
    pub fn fg_db_search_json_ex(db: *mut fg_db, ns: *const c_char, query: *const c_char,
                                filters: *const *const c_char, n_filters: u32, page: u32, per_page: u32,
                                include_text: c_int, shape: c_int, out: *mut c_char, cap: usize, len: *mut usize)
                                -> c_int;
    pub fn fg_db_search_json(db: *mut fg_db, ns: *const c_char, query: *const c_char, page: u32, per_page: u32,
                             include_text: c_int, shape: c_int, out: *mut c_char, cap: usize, len: *mut usize)
                             -> c_int;
    pub fn fg_db_search_json_post(db: *mut fg_db, ns: *const c_char, query: *const c_char,
                                  filters: *const *const c_char, n_filters: u32, has_page: c_int, page: u32,
                                  per_page: u32, url_text: c_int, body_text: c_int, url_include_data: c_int,
                                  body_include_data: c_int, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn fg_db_doc_facets(db: *mut fg_db, ns: *const c_char, doc: u32, out: *mut c_char, cap: usize,
                            len: *mut usize) -> c_int;
    pub fn fg_analyze(text: *const c_char, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn fg_parse_query(query: *const c_char, mode: *mut c_int, out: *mut c_char, cap: usize, len: *mut usize)
                          -> c_int;
    pub fn fg_parse_query_occur(query: *const c_char, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn fg_facet_tokens(path: *const c_char, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn fg_facet_clauses(filters: *const *const c_char, n_filters: u32, applies: *mut c_int,
                            all_query: *mut c_int, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
}

/// The check a host makes once before passing any struct: the library's layout
/// revision must be the one this file follows.
pub fn abi_ok() -> bool {
    unsafe { fg_abi_version() == FG_ABI_VERSION }
}
