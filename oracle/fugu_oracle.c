/*
 * fugu_oracle.c -- CPU ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the query path fugu delegates to tantivy 0.24.1
 * (crates.io, Cargo.lock:4609-4612; not vendored under /root/reference):
 *   fugu call site  : src/db/search.rs:108-127 (QueryParser over [text,name]),
 *                     src/db/search.rs:154-162 (TopDocs::with_limit(offset+per_page)),
 *                     src/db/schemas.rs:10,14 (text/name = TEXT|STORED),
 *                     src/db/document.rs:116-139 (what is indexed into text/name).
 *   upstream pieces restated:
 *     fieldnorm/code.rs      FIELD_NORMS_TABLE, fieldnorm_to_id      -> or_fieldnorm_*
 *     query/bm25.rs          idf, Bm25Weight, tf cache               -> or_idf, bm25_*
 *     postings/{segment_postings,skip}.rs: 128-doc blocks + last_doc skip    -> TermCur
 *     query/union/           Should(text:t, name:t), SumCombiner     -> UnionCur
 *     query/intersection.rs  leapfrog, children sorted by cost       -> conj_search
 *     collector/top_*.rs     TopNComputer (2K buffer, median cut)    -> TopN
 *
 * PARITY STATUS: "parity unpinned" -- the reference ships no test, fixture or
 * golden vector for this path and cannot be built or
 * imported here (no rustc/cargo, tantivy not vendored).  The restatement is
 * pinned to the hand-derived known-answer test of SURVEY.md Appendix C and
 * cross-checked against an independent numpy restatement
 * (tests/golden/gen_golden.py) on small corpora.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  It is the checker and the CPU baseline, never the
 * product path.  Deliberate simplification vs tantivy (documented in
 * DESIGN.md): blocks hold raw u32 doc ids / tfs instead of bitpacked deltas,
 * which makes this baseline FASTER than tantivy, never slower.
 *
 * Build: oracle/Makefile.  The portable test build uses -march=x86-64-v2 (the
 * container that builds it is not the GPU box's CPU); bench.py's CPU baseline
 * recompiles this file with -O3 -march=native -ffp-contract=off ON THE BOX
 * (`make -C oracle native OUT=<dir>`) and loads that copy (FUGU_ORACLE_LIB).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OR_BLOCK 128u
#define OR_TERMINATED 0x7FFFFFFFu /* tantivy: TERMINATED = i32::MAX as u32 */
#define OR_MAX_TERMS 64

static const float OR_K1 = 1.2f; /* query/bm25.rs K1 */
static const float OR_B = 0.75f; /* query/bm25.rs B */

/* ---------------------------------------------------------------- fieldnorm */
/* fieldnorm/code.rs: 0..=40 exact, then groups of 8 with step 2,4,8,...; 256 entries. */
static uint32_t g_table[256];
static int g_table_ready = 0;

static void table_init(void) {
  if (g_table_ready) return;
  uint32_t i = 0;
  for (; i <= 40; ++i) g_table[i] = i;
  uint64_t v = 40, step = 2;
  while (i < 256) {
    for (int j = 0; j < 8 && i < 256; ++j) { v += step; g_table[i++] = (uint32_t)v; }
    step <<= 1;
  }
  g_table_ready = 1;
}

void or_fieldnorm_table(uint32_t* out) { table_init(); memcpy(out, g_table, sizeof g_table); }

/* FIELD_NORMS_TABLE.binary_search(n).unwrap_or_else(|i| i - 1) */
uint8_t or_fieldnorm_to_id(uint32_t n) {
  table_init();
  uint32_t lo = 0, hi = 256; /* first index with table > n */
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (g_table[mid] <= n) lo = mid + 1; else hi = mid;
  }
  return (uint8_t)(lo - 1);
}

/* ---------------------------------------------------------------- bm25 */
/* bm25.rs idf(): ((N - df) as f32 + 0.5) / (df as f32 + 0.5), then (1 + x).ln() */
float or_idf(uint64_t df, uint64_t n) {
  float x = ((float)(n - df) + 0.5f) / ((float)df + 0.5f);
  return logf(1.0f + x);
}

/* Bm25Weight::new: idf * (1 + K1) (boost 1.0 multiplies exactly) */
float or_term_weight(uint64_t df, uint64_t n) { return or_idf(df, n) * (1.0f + OR_K1); }

/* compute_tf_cache: K1 * (1 - B + B * fieldnorm as f32 / avg) */
void or_bm25_cache(float avgdl, float* out) {
  table_init();
  for (int i = 0; i < 256; ++i) out[i] = OR_K1 * ((1.0f - OR_B) + (OR_B * (float)g_table[i]) / avgdl);
}

/* ---------------------------------------------------------------- index */
typedef struct {
  uint32_t n;        /* doc_freq in this field */
  uint32_t* doc;     /* sorted doc ids */
  uint32_t* tf;      /* term freqs */
  uint32_t* last;    /* skip list: last doc of each 128-doc block */
} Postings;

/* Field slots: 0 = text, 1 = name (TEXT, "default" analyzer), 2 = facet
 * (schemas.rs:20 add_facet_field("facet", INDEXED|STORED): IndexRecordOption
 * Basic, so tf = 1; no fieldnorms, so tantivy reads FieldNormReader::constant(
 * max_doc, 1) = id 1; total_num_tokens counts every FacetTokenizer token). */
#define OR_FIELDS 3
#define OR_FACET 2
typedef struct or_index {
  uint32_t n_docs, n_terms, n_fterms;
  int has_name;
  Postings* fld[OR_FIELDS];   /* [0]=text, [1]=name: [n_terms]; [2]=facet: [n_fterms] */
  uint32_t* store_doc[OR_FIELDS];
  uint32_t* store_tf[OR_FIELDS];
  uint32_t* store_last[OR_FIELDS];
  uint8_t* fn[OR_FIELDS];     /* fieldnorm ids [n_docs] (facet: constant 1) */
  uint8_t* deleted;           /* nullable [n_docs] */
  uint64_t tot[OR_FIELDS];    /* total_num_tokens per field (deleted docs included) */
  float avgdl[OR_FIELDS];
  float cache[OR_FIELDS][256];
} or_index;

typedef struct {
  const uint64_t* off;
  const uint32_t* tok;
  uint32_t n_docs, n_terms;
  uint32_t b, e;
  uint32_t* df;   /* per-thread counts [n_terms] */
  uint64_t* pos;  /* per-thread write cursors [n_terms] (fill pass) */
  Postings* post;
  int pass;
} BuildJob;

static int cmp_u32(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return (x > y) - (x < y);
}

static void* build_worker(void* arg) {
  BuildJob* j = (BuildJob*)arg;
  uint32_t buf[4096];
  for (uint32_t d = j->b; d < j->e; ++d) {
    uint64_t s = j->off[d], e = j->off[d + 1];
    uint32_t len = (uint32_t)(e - s);
    uint32_t* t = len <= 4096 ? buf : (uint32_t*)malloc(sizeof(uint32_t) * len);
    memcpy(t, j->tok + s, sizeof(uint32_t) * len);
    qsort(t, len, sizeof(uint32_t), cmp_u32);
    for (uint32_t i = 0; i < len;) {
      uint32_t k = i;
      while (k < len && t[k] == t[i]) ++k;
      uint32_t term = t[i];
      if (j->pass == 0) {
        j->df[term]++;
      } else {
        uint64_t p = j->pos[term]++;
        Postings* P = &j->post[term];
        P->doc[p] = d;
        P->tf[p] = k - i;
      }
      i = k;
    }
    if (t != buf) free(t);
  }
  return NULL;
}

static int build_field(or_index* ix, int f, const uint64_t* off, const uint32_t* tok, int threads, uint32_t nt) {
  uint32_t nd = ix->n_docs;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  BuildJob* jobs = (BuildJob*)calloc((size_t)threads, sizeof(BuildJob));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  uint32_t step = (nd + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    jobs[t].off = off; jobs[t].tok = tok; jobs[t].n_docs = nd; jobs[t].n_terms = nt;
    jobs[t].b = t * step < nd ? t * step : nd;
    jobs[t].e = (t + 1) * step < nd ? (t + 1) * step : nd;
    jobs[t].df = (uint32_t*)calloc(nt, sizeof(uint32_t));
    jobs[t].pos = (uint64_t*)calloc(nt, sizeof(uint64_t));
    jobs[t].pass = 0;
  }
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, build_worker, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  /* term df and per-thread start offsets */
  Postings* post = (Postings*)calloc(nt, sizeof(Postings));
  uint64_t total = 0, nblocks = 0;
  for (uint32_t term = 0; term < nt; ++term) {
    uint64_t df = 0;
    for (int t = 0; t < threads; ++t) { jobs[t].pos[term] = df; df += jobs[t].df[term]; }
    post[term].n = (uint32_t)df;
    total += df;
    nblocks += (df + OR_BLOCK - 1) / OR_BLOCK;
  }
  uint32_t* sdoc = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
  uint32_t* stf = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
  uint32_t* slast = (uint32_t*)malloc(sizeof(uint32_t) * (nblocks ? nblocks : 1));
  if (!sdoc || !stf || !slast) return -1;
  uint64_t o = 0, ob = 0;
  for (uint32_t term = 0; term < nt; ++term) {
    post[term].doc = sdoc + o; post[term].tf = stf + o; post[term].last = slast + ob;
    o += post[term].n;
    ob += (post[term].n + OR_BLOCK - 1) / OR_BLOCK;
  }
  for (int t = 0; t < threads; ++t) { jobs[t].post = post; jobs[t].pass = 1; }
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, build_worker, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  for (uint32_t term = 0; term < nt; ++term) {
    Postings* P = &post[term];
    uint32_t nb = (P->n + OR_BLOCK - 1) / OR_BLOCK;
    for (uint32_t b = 0; b < nb; ++b) {
      uint32_t end = (b + 1) * OR_BLOCK < P->n ? (b + 1) * OR_BLOCK : P->n;
      P->last[b] = P->doc[end - 1];
    }
  }
  for (int t = 0; t < threads; ++t) { free(jobs[t].df); free(jobs[t].pos); }
  free(jobs); free(th);
  ix->fld[f] = post; ix->store_doc[f] = sdoc; ix->store_tf[f] = stf; ix->store_last[f] = slast;
  /* fieldnorms: number of tokens that reached the index (post-filter count) */
  ix->fn[f] = (uint8_t*)malloc(nd ? nd : 1);
  uint64_t tot = 0;
  for (uint32_t d = 0; d < nd; ++d) {
    uint64_t len = off ? off[d + 1] - off[d] : 0;
    tot += len;
    ix->fn[f][d] = or_fieldnorm_to_id(len > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)len);
  }
  ix->tot[f] = tot;
  return 0;
}

void or_index_free(or_index* ix) {
  if (!ix) return;
  for (int f = 0; f < OR_FIELDS; ++f) {
    free(ix->fld[f]); free(ix->store_doc[f]); free(ix->store_tf[f]); free(ix->store_last[f]); free(ix->fn[f]);
  }
  free(ix->deleted);
  free(ix);
}

/*
 * text_off/text_tok: per-doc token term ids of the `text` field (after the
 * "default" analyzer), name_* likewise for `name` (nullable: no name field
 * values).  deleted: nullable, 1 = deleted-not-yet-merged (still counted in
 * N/df/total tokens, excluded from results: Appendix A.7).
 */
or_index* or_index_build(uint32_t n_docs, uint32_t n_terms, const uint64_t* text_off, const uint32_t* text_tok,
                         const uint64_t* name_off, const uint32_t* name_tok, const uint8_t* deleted, int threads) {
  table_init();
  or_index* ix = (or_index*)calloc(1, sizeof(or_index));
  ix->n_docs = n_docs; ix->n_terms = n_terms;
  static const uint64_t zero_off_dummy = 0;
  (void)zero_off_dummy;
  if (build_field(ix, 0, text_off, text_tok, threads, n_terms)) { or_index_free(ix); return NULL; }
  if (name_off && name_tok) {
    if (build_field(ix, 1, name_off, name_tok, threads, n_terms)) { or_index_free(ix); return NULL; }
    ix->has_name = 1;
  } else {
    /* empty name field: every doc has fieldnorm 0, no postings */
    ix->fld[1] = (Postings*)calloc(n_terms, sizeof(Postings));
    ix->fn[1] = (uint8_t*)calloc(n_docs ? n_docs : 1, 1);
    ix->tot[1] = 0;
  }
  if (deleted) {
    ix->deleted = (uint8_t*)malloc(n_docs ? n_docs : 1);
    memcpy(ix->deleted, deleted, n_docs);
  }
  for (int f = 0; f < 2; ++f) {
    ix->avgdl[f] = (float)ix->tot[f] / (float)n_docs; /* total_num_tokens as f32 / N as f32 */
    or_bm25_cache(ix->avgdl[f], ix->cache[f]);
  }
  return ix;
}

/* Facets of each doc as FacetTokenizer output (facet/facet_tokenizer.rs: the
 * root, then every ancestor, then the facet itself, for each stored facet
 * value; duplicates kept -- they count in total_num_tokens, not in df).
 * fugu indexes them through build_full_document -> add_facets_to_document
 * (src/db/document.rs:175-178, 310-330). */
int or_index_set_facets(or_index* ix, uint32_t n_fterms, const uint64_t* facet_off, const uint32_t* facet_tok,
                        int threads) {
  if (!ix || !facet_off || ix->fld[OR_FACET]) return -1;
  if (build_field(ix, OR_FACET, facet_off, facet_tok, threads, n_fterms)) return -1;
  ix->n_fterms = n_fterms;
  /* IndexRecordOption::Basic: term_freq() = 1; no fieldnorms: constant id 1 */
  uint64_t np = 0;
  for (uint32_t t = 0; t < n_fterms; ++t) np += ix->fld[OR_FACET][t].n;
  for (uint64_t p = 0; p < np; ++p) ix->store_tf[OR_FACET][p] = 1;
  memset(ix->fn[OR_FACET], 1, ix->n_docs ? ix->n_docs : 1);
  ix->avgdl[OR_FACET] = (float)ix->tot[OR_FACET] / (float)ix->n_docs;
  or_bm25_cache(ix->avgdl[OR_FACET], ix->cache[OR_FACET]);
  return 0;
}

/* total_num_tokens of `field` set from outside (a merged segment's total
 * follows tantivy's merger: per source segment with deletes the alive docs'
 * quantized lengths, merger.rs compute_total_num_tokens), then avgdl and the
 * tf cache recomputed from it as or_index_build does. */
int or_index_set_total_tokens(or_index* ix, int field, uint64_t tot) {
  if (!ix || field < 0 || field >= OR_FIELDS) return -1;
  ix->tot[field] = tot;
  ix->avgdl[field] = (float)tot / (float)ix->n_docs;
  or_bm25_cache(ix->avgdl[field], ix->cache[field]);
  return 0;
}

uint32_t or_df(const or_index* ix, int field, uint32_t term) {
  uint32_t nt = field == OR_FACET ? ix->n_fterms : ix->n_terms;
  return term < nt && ix->fld[field] ? ix->fld[field][term].n : 0;
}
uint64_t or_total_tokens(const or_index* ix, int field) { return ix->tot[field]; }
float or_avgdl(const or_index* ix, int field) { return ix->avgdl[field]; }
void or_cache(const or_index* ix, int field, float* out) { memcpy(out, ix->cache[field], sizeof(float) * 256); }
uint8_t or_fieldnorm_id_of(const or_index* ix, int field, uint32_t doc) { return ix->fn[field][doc]; }

/* ---------------------------------------------------------------- cursors */
typedef struct {
  const Postings* p;
  uint32_t cur;
  float weight;
  const float* cache;
  const uint8_t* fn;
} TermCur;

static inline uint32_t tc_doc(const TermCur* c) { return c->cur < c->p->n ? c->p->doc[c->cur] : OR_TERMINATED; }
static inline uint32_t tc_advance(TermCur* c) { if (c->cur < c->p->n) c->cur++; return tc_doc(c); }

/* SegmentPostings::seek: skip reader walks block last_doc entries forward, then
 * searches inside the block. */
static uint32_t tc_seek(TermCur* c, uint32_t target) {
  uint32_t d = tc_doc(c);
  if (d >= target) return d;
  const Postings* p = c->p;
  uint32_t nb = (p->n + OR_BLOCK - 1) / OR_BLOCK;
  uint32_t b = c->cur / OR_BLOCK;
  while (b < nb && p->last[b] < target) ++b;
  if (b == nb) { c->cur = p->n; return OR_TERMINATED; }
  uint32_t lo = b * OR_BLOCK > c->cur ? b * OR_BLOCK : c->cur;
  uint32_t hi = (b + 1) * OR_BLOCK < p->n ? (b + 1) * OR_BLOCK : p->n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (p->doc[mid] < target) lo = mid + 1; else hi = mid;
  }
  c->cur = lo;
  return tc_doc(c);
}

/* Bm25Weight::score(fieldnorm_id, tf) = weight * (tf / (tf + cache[id])) */
static inline float tc_score(const TermCur* c) {
  uint32_t d = c->p->doc[c->cur];
  float tf = (float)c->p->tf[c->cur];
  float norm = c->cache[c->fn[d]];
  return c->weight * (tf / (tf + norm));
}

/* One query term over default fields [text, name]: Should(text:t, name:t),
 * BufferedUnionScorer with SumCombiner (score starts at 0.0). */
typedef struct {
  TermCur f[2];
  uint32_t doc;
  uint64_t cost; /* DocSet::cost of a union = sum of children (df_text + df_name) */
} UnionCur;

static inline uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }

static void uc_init(UnionCur* u, const or_index* ix, uint32_t term) {
  uint64_t n = ix->n_docs;
  for (int f = 0; f < 2; ++f) {
    static const Postings empty = {0, NULL, NULL, NULL};
    u->f[f].p = term < ix->n_terms ? &ix->fld[f][term] : &empty;
    u->f[f].cur = 0;
    u->f[f].weight = or_term_weight(u->f[f].p->n, n);
    u->f[f].cache = ix->cache[f];
    u->f[f].fn = ix->fn[f];
  }
  u->doc = min_u32(tc_doc(&u->f[0]), tc_doc(&u->f[1]));
  u->cost = (uint64_t)u->f[0].p->n + u->f[1].p->n;
}
static inline uint32_t uc_advance(UnionCur* u) {
  for (int f = 0; f < 2; ++f) if (tc_doc(&u->f[f]) == u->doc) tc_advance(&u->f[f]);
  u->doc = min_u32(tc_doc(&u->f[0]), tc_doc(&u->f[1]));
  return u->doc;
}
static inline uint32_t uc_seek(UnionCur* u, uint32_t target) {
  if (u->doc >= target) return u->doc;
  tc_seek(&u->f[0], target);
  tc_seek(&u->f[1], target);
  u->doc = min_u32(tc_doc(&u->f[0]), tc_doc(&u->f[1]));
  return u->doc;
}
static inline float uc_score(const UnionCur* u) {
  float s = 0.0f;
  for (int f = 0; f < 2; ++f) if (tc_doc(&u->f[f]) == u->doc) s += tc_score(&u->f[f]);
  return s;
}

/* ---------------------------------------------------------------- TopN */
typedef struct { float score; uint32_t doc; } Hit;

/* ComparableDoc ordering with REVERSE_ORDER: score descending, then doc ascending */
static int hit_cmp(const void* a, const void* b) {
  const Hit* x = (const Hit*)a; const Hit* y = (const Hit*)b;
  if (x->score > y->score) return -1;
  if (x->score < y->score) return 1;
  return (x->doc > y->doc) - (x->doc < y->doc);
}

typedef struct {
  Hit* buf;
  uint32_t len, top_n, cap;
  int has_thr;
  float thr;
} TopN;

static void topn_init(TopN* t, uint32_t k) {
  t->top_n = k; t->cap = 2 * k; t->len = 0; t->has_thr = 0; t->thr = -3.40282347e+38f;
  t->buf = (Hit*)malloc(sizeof(Hit) * t->cap);
}
/* truncate_top_n: the element at sorted index top_n becomes the threshold */
static float topn_truncate(TopN* t) {
  qsort(t->buf, t->len, sizeof(Hit), hit_cmp);
  float median = t->buf[t->top_n].score;
  t->len = t->top_n;
  t->thr = median; t->has_thr = 1;
  return median;
}
static void topn_push(TopN* t, float score, uint32_t doc) {
  if (t->has_thr && score < t->thr) return;
  if (t->len == t->cap) topn_truncate(t);
  t->buf[t->len].score = score; t->buf[t->len].doc = doc; t->len++;
}
static uint32_t topn_finish(TopN* t, float* out_score, uint32_t* out_doc) {
  if (t->len > t->top_n) topn_truncate(t);
  qsort(t->buf, t->len, sizeof(Hit), hit_cmp);
  for (uint32_t i = 0; i < t->len; ++i) { out_score[i] = t->buf[i].score; out_doc[i] = t->buf[i].doc; }
  uint32_t n = t->len;
  free(t->buf);
  return n;
}
/* the callback of for_each_pruning: push, return the current threshold */
static inline float collect(TopN* t, const or_index* ix, uint32_t doc, float score) {
  if (!(ix->deleted && ix->deleted[doc])) topn_push(t, score, doc);
  return t->has_thr ? t->thr : -3.40282347e+38f;
}

/* ---------------------------------------------------------------- search */
typedef struct { UnionCur* c; uint64_t cost; uint32_t qpos; } Child;

static int child_cmp(const void* a, const void* b) {
  const Child* x = (const Child*)a; const Child* y = (const Child*)b;
  if (x->cost != y->cost) return x->cost < y->cost ? -1 : 1;
  return (x->qpos > y->qpos) - (x->qpos < y->qpos); /* sort_by_key is stable */
}

/* intersection.rs go_to_first_doc */
static uint32_t go_to_first_doc(UnionCur** ds, uint32_t n) {
  uint32_t cand = 0;
  for (uint32_t i = 0; i < n; ++i) if (ds[i]->doc > cand) cand = ds[i]->doc;
  for (;;) {
    int again = 0;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t s = uc_seek(ds[i], cand);
      if (s > cand) { cand = ds[i]->doc; again = 1; break; }
    }
    if (!again) return cand;
  }
}

/* Intersection::advance (leapfrog on the two rarest, then probe the others) */
static uint32_t isect_advance(UnionCur** ds, uint32_t n) {
  UnionCur* left = ds[0];
  UnionCur* right = ds[1];
  uint32_t cand = uc_advance(left);
  if (cand == OR_TERMINATED) return OR_TERMINATED;
  for (;;) {
    for (;;) {
      uint32_t rd = uc_seek(right, cand);
      cand = uc_seek(left, rd);
      if (cand == rd) break;
    }
    if (cand == OR_TERMINATED) return OR_TERMINATED;
    uint32_t next = cand;
    for (uint32_t i = 2; i < n; ++i) {
      uint32_t s = uc_seek(ds[i], cand);
      if (s > cand) { next = s; break; }
    }
    if (next == cand) return cand;
    cand = uc_seek(left, next);
    if (cand == OR_TERMINATED) return OR_TERMINATED;
  }
}

/* Intersection::score = left + right + others.sum() (fold from 0.0) */
static inline float isect_score(UnionCur** ds, uint32_t n) {
  float others = 0.0f;
  for (uint32_t i = 2; i < n; ++i) others += uc_score(ds[i]);
  return uc_score(ds[0]) + uc_score(ds[1]) + others;
}

/*
 * mode 0: conjunction  `t1 AND t2 AND ...` (Must clauses)
 * mode 1: disjunction  `t1 t2 ...`         (default operator: Should)
 * k >= 1 (TopDocs::with_limit asserts limit >= 1).
 * Returns number of hits written (<= k), or -1 on bad arguments.
 */
int or_search(const or_index* ix, const uint32_t* terms, uint32_t m, int mode, uint32_t k, float* out_score,
              uint32_t* out_doc) {
  if (k < 1 || m < 1 || m > OR_MAX_TERMS) return -1;
  UnionCur cur[OR_MAX_TERMS];
  Child ch[OR_MAX_TERMS];
  UnionCur* ds[OR_MAX_TERMS];
  for (uint32_t i = 0; i < m; ++i) {
    uc_init(&cur[i], ix, terms[i]);
    ch[i].c = &cur[i]; ch[i].cost = cur[i].cost; ch[i].qpos = i;
  }
  TopN top;
  topn_init(&top, k);
  float thr = -3.40282347e+38f;
  if (mode == 0 && m == 1) {
    /* a single term: the top-level query is the field union itself */
    UnionCur* u = &cur[0];
    for (uint32_t d = u->doc; d != OR_TERMINATED; d = uc_advance(u)) {
      float s = uc_score(u);
      if (s > thr) thr = collect(&top, ix, d, s);
    }
  } else if (mode == 0) {
    qsort(ch, m, sizeof(Child), child_cmp);
    for (uint32_t i = 0; i < m; ++i) ds[i] = ch[i].c;
    uint32_t d = go_to_first_doc(ds, m);
    while (d != OR_TERMINATED) {
      float s = isect_score(ds, m);
      if (s > thr) thr = collect(&top, ix, d, s);
      d = isect_advance(ds, m);
    }
  } else {
    /* pure disjunction over the per-term unions, SumCombiner in clause order */
    for (;;) {
      uint32_t d = OR_TERMINATED;
      for (uint32_t i = 0; i < m; ++i) d = min_u32(d, cur[i].doc);
      if (d == OR_TERMINATED) break;
      float s = 0.0f;
      for (uint32_t i = 0; i < m; ++i) if (cur[i].doc == d) s += uc_score(&cur[i]);
      if (s > thr) thr = collect(&top, ix, d, s);
      for (uint32_t i = 0; i < m; ++i) if (cur[i].doc == d) uc_advance(&cur[i]);
    }
  }
  return (int)topn_finish(&top, out_score, out_doc);
}

/* Postings of `p` with doc < d (lower bound). */
static uint32_t post_lb(const Postings* p, uint32_t d) {
  uint32_t lo = 0, hi = p->n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (p->doc[mid] < d) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/*
 * or_search over a multi-segment index: one segment per commit
 * (src/db/document.rs:65), seg[0..nseg] = the segments' doc-id boundaries.
 * Every segment runs its own scorer with the index-wide statistics
 * (Bm25StatisticsProvider of the Searcher), and BooleanWeight orders the
 * intersection's children by the SEGMENT's cost (its own doc_freq), so a
 * conjunction of >= 3 terms sums its scores in each segment's own order.  One
 * TopN collects all segments (merge_fruits of per-segment top-k gives the same
 * top-k: a later segment's doc loses every tie by DocAddress).  Disjunctions
 * and single terms do not depend on the segmentation.
 */
int or_search_seg(const or_index* ix, const uint32_t* terms, uint32_t m, int mode, uint32_t k, const uint32_t* seg,
                  uint32_t nseg, float* out_score, uint32_t* out_doc) {
  if (mode != 0 || m < 2 || nseg < 1) return or_search(ix, terms, m, mode, k, out_score, out_doc);
  if (k < 1 || m > OR_MAX_TERMS) return -1;
  UnionCur cur[OR_MAX_TERMS];
  Child ch[OR_MAX_TERMS];
  UnionCur* ds[OR_MAX_TERMS];
  TopN top;
  topn_init(&top, k);
  float thr = -3.40282347e+38f;
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint32_t lo = seg[s], hi = seg[s + 1];
    if (lo >= hi) continue;
    for (uint32_t i = 0; i < m; ++i) {
      uc_init(&cur[i], ix, terms[i]);
      uint64_t cost = 0;
      for (int f = 0; f < 2; ++f) cost += post_lb(cur[i].f[f].p, hi) - post_lb(cur[i].f[f].p, lo);
      ch[i].c = &cur[i]; ch[i].cost = cost; ch[i].qpos = i;
      uc_seek(&cur[i], lo);
    }
    qsort(ch, m, sizeof(Child), child_cmp);
    for (uint32_t i = 0; i < m; ++i) ds[i] = ch[i].c;
    uint32_t d = go_to_first_doc(ds, m);
    while (d < hi) {
      float sc = isect_score(ds, m);
      if (sc > thr) thr = collect(&top, ix, d, sc);
      d = isect_advance(ds, m);
    }
  }
  return (int)topn_finish(&top, out_score, out_doc);
}

/* ---------------------------------------------------------------- filtered search */
/*
 * Dataset::search with facet filters (src/db/search.rs:129-150):
 *   base_query = Bool[Must(text_query), Must(facet_query)]   text and filters
 *              = facet_query                                  empty text, filters
 *              = AllQuery                                     empty text, no filters
 * facet_query = build_facet_query (:221-293): Should over the exact facet
 * terms (new_multiterms_query), then one Should TermQuery per prefix filter;
 * the caller passes that flat clause list (exact terms first, then prefixes).
 * A union scores 0.0 + the matching clauses in clause order (SumCombiner);
 * an Intersection of two children scores left + right (+ 0.0 for no others),
 * which is commutative, so the order the children run in does not matter.
 * AllScorer scores 1.0 (query/all_query.rs).  Scorers are generic cursors here.
 */
typedef struct Cur {
  uint32_t (*doc)(struct Cur*);
  uint32_t (*advance)(struct Cur*);
  uint32_t (*seek)(struct Cur*, uint32_t);
  float (*score)(struct Cur*);
  uint64_t cost;
} Cur;

/* text AND over >= 2 terms: Intersection of the per-term unions */
typedef struct { Cur c; UnionCur* ds[OR_MAX_TERMS]; uint32_t n, d; } AndCur;
static uint32_t and_doc(Cur* c) { return ((AndCur*)c)->d; }
static uint32_t and_advance(Cur* c) { AndCur* a = (AndCur*)c; return a->d = isect_advance(a->ds, a->n); }
static uint32_t and_seek(Cur* c, uint32_t t) {
  AndCur* a = (AndCur*)c;
  if (a->d >= t) return a->d;
  uc_seek(a->ds[0], t);
  return a->d = go_to_first_doc(a->ds, a->n);
}
static float and_score(Cur* c) { AndCur* a = (AndCur*)c; return isect_score(a->ds, a->n); }

/* one text term: the field union itself */
typedef struct { Cur c; UnionCur* u; } OneCur;
static uint32_t one_doc(Cur* c) { return ((OneCur*)c)->u->doc; }
static uint32_t one_advance(Cur* c) { return uc_advance(((OneCur*)c)->u); }
static uint32_t one_seek(Cur* c, uint32_t t) { return uc_seek(((OneCur*)c)->u, t); }
static float one_score(Cur* c) { return uc_score(((OneCur*)c)->u); }

/* text OR: union of the per-term unions, SumCombiner in clause order */
typedef struct { Cur c; UnionCur* u; uint32_t n, d; } OrCur;
static uint32_t or_min(OrCur* o) {
  uint32_t d = OR_TERMINATED;
  for (uint32_t i = 0; i < o->n; ++i) d = min_u32(d, o->u[i].doc);
  return o->d = d;
}
static uint32_t orc_doc(Cur* c) { return ((OrCur*)c)->d; }
static uint32_t orc_advance(Cur* c) {
  OrCur* o = (OrCur*)c;
  for (uint32_t i = 0; i < o->n; ++i) if (o->u[i].doc == o->d) uc_advance(&o->u[i]);
  return or_min(o);
}
static uint32_t orc_seek(Cur* c, uint32_t t) {
  OrCur* o = (OrCur*)c;
  if (o->d >= t) return o->d;
  for (uint32_t i = 0; i < o->n; ++i) uc_seek(&o->u[i], t);
  return or_min(o);
}
static float orc_score(Cur* c) {
  OrCur* o = (OrCur*)c;
  float s = 0.0f;
  for (uint32_t i = 0; i < o->n; ++i) if (o->u[i].doc == o->d) s += uc_score(&o->u[i]);
  return s;
}

/* facet_query: union of facet TermScorers (tf 1, fieldnorm id 1), clause order */
#define OR_MAX_FACETS 64
typedef struct { Cur c; TermCur t[OR_MAX_FACETS]; uint32_t n, d; } FacetCur;
static uint32_t fc_min(FacetCur* f) {
  uint32_t d = OR_TERMINATED;
  for (uint32_t i = 0; i < f->n; ++i) d = min_u32(d, tc_doc(&f->t[i]));
  return f->d = d;
}
static uint32_t fc_doc(Cur* c) { return ((FacetCur*)c)->d; }
static uint32_t fc_advance(Cur* c) {
  FacetCur* f = (FacetCur*)c;
  for (uint32_t i = 0; i < f->n; ++i) if (tc_doc(&f->t[i]) == f->d) tc_advance(&f->t[i]);
  return fc_min(f);
}
static uint32_t fc_seek(Cur* c, uint32_t t) {
  FacetCur* f = (FacetCur*)c;
  if (f->d >= t) return f->d;
  for (uint32_t i = 0; i < f->n; ++i) tc_seek(&f->t[i], t);
  return fc_min(f);
}
static float fc_score(Cur* c) {
  FacetCur* f = (FacetCur*)c;
  float s = 0.0f;
  for (uint32_t i = 0; i < f->n; ++i) if (tc_doc(&f->t[i]) == f->d) s += tc_score(&f->t[i]);
  return s;
}

/* AllQuery: every doc, score 1.0 */
typedef struct { Cur c; uint32_t d, n; } AllCur;
static uint32_t all_doc(Cur* c) { return ((AllCur*)c)->d; }
static uint32_t all_advance(Cur* c) {
  AllCur* a = (AllCur*)c;
  a->d = a->d + 1 < a->n ? a->d + 1 : OR_TERMINATED;
  return a->d;
}
static uint32_t all_seek(Cur* c, uint32_t t) {
  AllCur* a = (AllCur*)c;
  if (a->d >= t) return a->d;
  a->d = t < a->n ? t : OR_TERMINATED;
  return a->d;
}
static float all_score(Cur* c) { (void)c; return 1.0f; }

/*
 * terms/m/mode: the text query (m = 0: empty text); fterms/nf: the facet
 * clauses (facet term ids, ids >= n_fterms match nothing; nf = 0: no filter).
 * Returns hits written (<= k) or -1 on bad arguments.
 */
int or_search_ex(const or_index* ix, const uint32_t* terms, uint32_t m, int mode, const uint32_t* fterms, uint32_t nf,
                 uint32_t k, float* out_score, uint32_t* out_doc) {
  if (k < 1 || m > OR_MAX_TERMS || nf > OR_MAX_FACETS) return -1;
  if (nf == 0 && m > 0) return or_search(ix, terms, m, mode, k, out_score, out_doc);
  UnionCur uc[OR_MAX_TERMS];
  Child ch[OR_MAX_TERMS];
  AndCur ac; OneCur oc; OrCur orc; FacetCur fc; AllCur al;
  Cur* text = NULL;
  for (uint32_t i = 0; i < m; ++i) {
    uc_init(&uc[i], ix, terms[i]);
    ch[i].c = &uc[i]; ch[i].cost = uc[i].cost; ch[i].qpos = i;
  }
  if (m == 0) {
    text = NULL;
  } else if (mode == 0 && m == 1) {
    oc.u = &uc[0];
    oc.c = (Cur){one_doc, one_advance, one_seek, one_score, uc[0].cost};
    text = &oc.c;
  } else if (mode == 0) {
    qsort(ch, m, sizeof(Child), child_cmp);
    for (uint32_t i = 0; i < m; ++i) ac.ds[i] = ch[i].c;
    ac.n = m;
    ac.d = go_to_first_doc(ac.ds, m);
    ac.c = (Cur){and_doc, and_advance, and_seek, and_score, ac.ds[0]->cost};
    text = &ac.c;
  } else {
    orc.u = uc; orc.n = m;
    uint64_t cost = 0;
    for (uint32_t i = 0; i < m; ++i) cost += uc[i].cost;
    or_min(&orc);
    orc.c = (Cur){orc_doc, orc_advance, orc_seek, orc_score, cost};
    text = &orc.c;
  }
  Cur* filt = NULL;
  if (nf > 0) {
    static const Postings empty = {0, NULL, NULL, NULL};
    uint64_t cost = 0;
    for (uint32_t i = 0; i < nf; ++i) {
      const Postings* p = (ix->fld[OR_FACET] && fterms[i] < ix->n_fterms) ? &ix->fld[OR_FACET][fterms[i]] : &empty;
      fc.t[i].p = p;
      fc.t[i].cur = 0;
      fc.t[i].weight = or_term_weight(p->n, ix->n_docs);
      fc.t[i].cache = ix->cache[OR_FACET];
      fc.t[i].fn = ix->fn[OR_FACET];
      cost += p->n;
    }
    fc.n = nf;
    fc_min(&fc);
    fc.c = (Cur){fc_doc, fc_advance, fc_seek, fc_score, cost};
    filt = &fc.c;
  } else {
    al.n = ix->n_docs;
    al.d = ix->n_docs ? 0 : OR_TERMINATED;
    al.c = (Cur){all_doc, all_advance, all_seek, all_score, ix->n_docs};
    filt = &al.c; /* m == 0 here: the query is AllQuery itself */
  }
  TopN top;
  topn_init(&top, k);
  float thr = -3.40282347e+38f;
  if (!text) {
    for (uint32_t d = filt->doc(filt); d != OR_TERMINATED; d = filt->advance(filt)) {
      float s = filt->score(filt);
      if (s > thr) thr = collect(&top, ix, d, s);
    }
  } else {
    /* Intersection of (text, facet): children by cost (stable), leapfrog */
    Cur* left = text->cost <= filt->cost ? text : filt;
    Cur* right = left == text ? filt : text;
    uint32_t cand = left->doc(left) > right->doc(right) ? left->doc(left) : right->doc(right);
    for (;;) {
      uint32_t a = left->seek(left, cand);
      uint32_t b = right->seek(right, a);
      if (b == a) { cand = a; break; }
      cand = b;
    }
    while (cand != OR_TERMINATED) {
      float s = left->score(left) + right->score(right) + 0.0f;
      if (s > thr) thr = collect(&top, ix, cand, s);
      cand = left->advance(left);
      if (cand == OR_TERMINATED) break;
      for (;;) {
        uint32_t r = right->seek(right, cand);
        if (r == cand) break;
        cand = left->seek(left, r);
        if (cand == OR_TERMINATED) break;
      }
    }
  }
  return (int)topn_finish(&top, out_score, out_doc);
}

/* ---------------------------------------------------------------- occurs: Must / Should / MustNot */
/*
 * The parser's BooleanQuery with per-clause occurs (src/db/search.rs:108-127:
 * `+a b -c`, `a OR b`, `a AND b`), each clause the per-term field union
 * Should(text:t, name:t).  tantivy 0.24.1 query/boolean_query/boolean_weight.rs
 * complex_scorer:
 *   Must clauses     -> the clause itself when one, else Intersection (children
 *                       by cost, leapfrog), score left + right + others;
 *   Should + Must    -> RequiredOptionalScorer (query/reqopt_scorer.rs): the
 *                       Must scorer drives; SumCombiner from 0.0 adds the
 *                       required score, then the optional union's score when it
 *                       is on the doc;
 *   Should only      -> the union (SumCombiner, clause order);
 *   MustNot          -> Exclude (query/exclude.rs) of the positive scorer by the
 *                       union of the excluded clauses; scores unchanged;
 *   no Must/Should   -> EmptyScorer (no hits).
 * The positive query then meets the facet filter as before (two-child
 * Intersection, text + facet).  Segments (seg != NULL): each runs its own
 * scorers over its doc range, the Must children ordered by the SEGMENT's cost
 * (BooleanWeight per SegmentReader), collected into one TopN.
 */
#define OR_OCC_MUST 0
#define OR_OCC_SHOULD 1
#define OR_OCC_MUST_NOT 2

typedef struct { Cur c; Cur* req; Cur* opt; } ReqOptCur;
static uint32_t ro_doc(Cur* c) { ReqOptCur* r = (ReqOptCur*)c; return r->req->doc(r->req); }
static uint32_t ro_advance(Cur* c) { ReqOptCur* r = (ReqOptCur*)c; return r->req->advance(r->req); }
static uint32_t ro_seek(Cur* c, uint32_t t) { ReqOptCur* r = (ReqOptCur*)c; return r->req->seek(r->req, t); }
static float ro_score(Cur* c) {
  ReqOptCur* r = (ReqOptCur*)c;
  float s = 0.0f;
  s += r->req->score(r->req);
  const uint32_t d = r->req->doc(r->req);
  if (r->opt && r->opt->doc(r->opt) <= d && r->opt->seek(r->opt, d) == d) s += r->opt->score(r->opt);
  return s;
}

typedef struct { Cur c; Cur* pos; Cur* ex; uint32_t d; } ExclCur;
static uint32_t ex_skip(ExclCur* e, uint32_t d) {
  while (d != OR_TERMINATED) {
    const uint32_t x = e->ex->doc(e->ex);
    if (x > d || e->ex->seek(e->ex, d) != d) break;  /* accept: not in the excluded set */
    d = e->pos->advance(e->pos);
  }
  return e->d = d;
}
static uint32_t exc_doc(Cur* c) { return ((ExclCur*)c)->d; }
static uint32_t exc_advance(Cur* c) { ExclCur* e = (ExclCur*)c; return ex_skip(e, e->pos->advance(e->pos)); }
static uint32_t exc_seek(Cur* c, uint32_t t) {
  ExclCur* e = (ExclCur*)c;
  if (e->d >= t) return e->d;
  return ex_skip(e, e->pos->seek(e->pos, t));
}
static float exc_score(Cur* c) { ExclCur* e = (ExclCur*)c; return e->pos->score(e->pos); }

typedef struct {
  UnionCur um[OR_MAX_TERMS], us[OR_MAX_TERMS], ux[OR_MAX_TERMS];
  Child ch[OR_MAX_TERMS];
  AndCur ac; OneCur oc, so; OrCur sor, xor_; ReqOptCur ro; ExclCur ex;
  FacetCur fc; AllCur al;
} QueryCurs;

/* The text cursor of one query over docs [lo, hi) (all cursors at or past lo),
 * or NULL: *empty = 1 when the query matches nothing, 0 when the text is empty
 * (m == 0: the facet union or AllQuery alone). */
static Cur* build_text(QueryCurs* Q, const or_index* ix, const uint32_t* terms, const uint8_t* occur, uint32_t m,
                       uint32_t lo, uint32_t hi, int* empty) {
  uint32_t nm = 0, ns = 0, nx = 0;
  *empty = 0;
  if (m == 0) return NULL;
  for (uint32_t i = 0; i < m; ++i) {
    UnionCur* u = occur[i] == OR_OCC_MUST ? &Q->um[nm++] : occur[i] == OR_OCC_SHOULD ? &Q->us[ns++] : &Q->ux[nx++];
    uc_init(u, ix, terms[i]);
    uc_seek(u, lo);
  }
  if (nm == 0 && ns == 0) { *empty = 1; return NULL; }
  Cur* req = NULL;
  if (nm == 1) {
    Q->oc.u = &Q->um[0];
    Q->oc.c = (Cur){one_doc, one_advance, one_seek, one_score, Q->um[0].cost};
    req = &Q->oc.c;
  } else if (nm > 1) {
    for (uint32_t i = 0; i < nm; ++i) {
      uint64_t cost = Q->um[i].cost;
      if (lo != 0 || hi != ix->n_docs) { /* the segment's own doc_freq */
        cost = 0;
        for (int f = 0; f < 2; ++f) cost += post_lb(Q->um[i].f[f].p, hi) - post_lb(Q->um[i].f[f].p, lo);
      }
      Q->ch[i].c = &Q->um[i]; Q->ch[i].cost = cost; Q->ch[i].qpos = i;
    }
    qsort(Q->ch, nm, sizeof(Child), child_cmp);
    for (uint32_t i = 0; i < nm; ++i) Q->ac.ds[i] = Q->ch[i].c;
    Q->ac.n = nm;
    Q->ac.d = go_to_first_doc(Q->ac.ds, nm);
    Q->ac.c = (Cur){and_doc, and_advance, and_seek, and_score, Q->ac.ds[0]->cost};
    req = &Q->ac.c;
  }
  Cur* opt = NULL;
  if (ns > 0) {
    Q->sor.u = Q->us; Q->sor.n = ns;
    uint64_t cost = 0;
    for (uint32_t i = 0; i < ns; ++i) cost += Q->us[i].cost;
    or_min(&Q->sor);
    Q->sor.c = (Cur){orc_doc, orc_advance, orc_seek, orc_score, cost};
    opt = &Q->sor.c;
  }
  Cur* pos;
  if (req && opt) {
    Q->ro.req = req; Q->ro.opt = opt;
    Q->ro.c = (Cur){ro_doc, ro_advance, ro_seek, ro_score, req->cost};
    pos = &Q->ro.c;
  } else {
    pos = req ? req : opt;
  }
  if (nx == 0) return pos;
  Q->xor_.u = Q->ux; Q->xor_.n = nx;
  or_min(&Q->xor_);
  Q->xor_.c = (Cur){orc_doc, orc_advance, orc_seek, orc_score, 0};
  Q->ex.pos = pos; Q->ex.ex = &Q->xor_.c;
  Q->ex.c = (Cur){exc_doc, exc_advance, exc_seek, exc_score, pos->cost};
  ex_skip(&Q->ex, pos->doc(pos));
  return &Q->ex.c;
}

static void run_range(const or_index* ix, const uint32_t* terms, const uint8_t* occur, uint32_t m,
                      const uint32_t* fterms, uint32_t nf, int filtered, uint32_t lo, uint32_t hi, TopN* top,
                      float* thr) {
  QueryCurs* Q = (QueryCurs*)malloc(sizeof(QueryCurs));
  int empty = 0;
  Cur* text = build_text(Q, ix, terms, occur, m, lo, hi, &empty);
  Cur* filt = NULL;
  if (!empty && filtered) {
    static const Postings emptyp = {0, NULL, NULL, NULL};
    uint64_t cost = 0;
    for (uint32_t i = 0; i < nf; ++i) {
      const Postings* p = (ix->fld[OR_FACET] && fterms[i] < ix->n_fterms) ? &ix->fld[OR_FACET][fterms[i]] : &emptyp;
      Q->fc.t[i].p = p;
      Q->fc.t[i].cur = 0;
      Q->fc.t[i].weight = or_term_weight(p->n, ix->n_docs);
      Q->fc.t[i].cache = ix->cache[OR_FACET];
      Q->fc.t[i].fn = ix->fn[OR_FACET];
      cost += p->n;
    }
    Q->fc.n = nf;
    fc_min(&Q->fc);
    Q->fc.c = (Cur){fc_doc, fc_advance, fc_seek, fc_score, cost};
    filt = &Q->fc.c;
    filt->seek(filt, lo);
  } else if (!empty && !text) {
    Q->al.n = ix->n_docs;
    Q->al.d = lo < ix->n_docs ? lo : OR_TERMINATED;
    Q->al.c = (Cur){all_doc, all_advance, all_seek, all_score, ix->n_docs};
    filt = &Q->al.c; /* m == 0, no filter: AllQuery */
  }
  if (empty) { free(Q); return; }
  if (!filt) {
    for (uint32_t d = text->doc(text); d < hi; d = text->advance(text)) {
      float s = text->score(text);
      if (s > *thr) *thr = collect(top, ix, d, s);
    }
  } else if (!text) {
    for (uint32_t d = filt->doc(filt); d < hi; d = filt->advance(filt)) {
      float s = filt->score(filt);
      if (s > *thr) *thr = collect(top, ix, d, s);
    }
  } else {
    /* Intersection of (text, facet): children by cost (stable), leapfrog */
    Cur* left = text->cost <= filt->cost ? text : filt;
    Cur* right = left == text ? filt : text;
    uint32_t cand = left->doc(left) > right->doc(right) ? left->doc(left) : right->doc(right);
    for (;;) {
      uint32_t a = left->seek(left, cand);
      uint32_t b = right->seek(right, a);
      if (b == a) { cand = a; break; }
      cand = b;
    }
    while (cand < hi) {
      float s = left->score(left) + right->score(right) + 0.0f;
      if (s > *thr) *thr = collect(top, ix, cand, s);
      cand = left->advance(left);
      if (cand == OR_TERMINATED) break;
      for (;;) {
        uint32_t r = right->seek(right, cand);
        if (r == cand) break;
        cand = left->seek(left, r);
        if (cand == OR_TERMINATED) break;
      }
    }
  }
  free(Q);
}

/*
 * The general entry: terms[m] with occur[m] (OR_OCC_*); fterms[nf] with
 * filtered != 0 = the facet clauses; seg[nseg+1] = segment doc-id bounds, or
 * NULL (one segment).  Returns hits written (<= k), or -1 on bad arguments.
 */
int or_search_q(const or_index* ix, const uint32_t* terms, const uint8_t* occur, uint32_t m, const uint32_t* fterms,
                uint32_t nf, int filtered, const uint32_t* seg, uint32_t nseg, uint32_t k, float* out_score,
                uint32_t* out_doc) {
  if (k < 1 || m > OR_MAX_TERMS || nf > OR_MAX_FACETS || (m && !occur)) return -1;
  for (uint32_t i = 0; i < m; ++i)
    if (occur[i] > OR_OCC_MUST_NOT) return -1;
  TopN top;
  topn_init(&top, k);
  float thr = -3.40282347e+38f;
  if (!seg) {
    run_range(ix, terms, occur, m, fterms, nf, filtered, 0, ix->n_docs, &top, &thr);
  } else {
    for (uint32_t s = 0; s < nseg; ++s)
      if (seg[s] < seg[s + 1]) run_range(ix, terms, occur, m, fterms, nf, filtered, seg[s], seg[s + 1], &top, &thr);
  }
  return (int)topn_finish(&top, out_score, out_doc);
}

/* ---------------------------------------------------------------- batch (CPU baseline) */
typedef struct {
  const or_index* ix;
  const uint32_t* q_off; const uint32_t* q_terms;
  const uint8_t* q_occur; /* nullable: every term is `mode`'s occur */
  const uint32_t* f_off; const uint32_t* f_terms; /* nullable: no facet filters */
  uint32_t nq; int mode; uint32_t k;
  float* out_score; uint32_t* out_doc; uint32_t* out_n;
  double* lat_ns;
  volatile uint32_t next;
  pthread_mutex_t mu;
} BatchCtx;

static double now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e9 + (double)ts.tv_nsec;
}

static void* batch_worker(void* arg) {
  BatchCtx* c = (BatchCtx*)arg;
  for (;;) {
    uint32_t q = __atomic_fetch_add(&c->next, 1u, __ATOMIC_RELAXED);
    if (q >= c->nq) break;
    double t0 = now_ns();
    int n = c->q_occur ? or_search_q(c->ix, c->q_terms + c->q_off[q], c->q_occur + c->q_off[q],
                                     c->q_off[q + 1] - c->q_off[q], c->f_off ? c->f_terms + c->f_off[q] : NULL,
                                     c->f_off ? c->f_off[q + 1] - c->f_off[q] : 0, c->f_off != NULL, NULL, 0, c->k,
                                     c->out_score + (size_t)q * c->k, c->out_doc + (size_t)q * c->k)
            : c->f_off ? or_search_ex(c->ix, c->q_terms + c->q_off[q], c->q_off[q + 1] - c->q_off[q], c->mode,
                                    c->f_terms + c->f_off[q], c->f_off[q + 1] - c->f_off[q], c->k,
                                    c->out_score + (size_t)q * c->k, c->out_doc + (size_t)q * c->k)
                     : or_search(c->ix, c->q_terms + c->q_off[q], c->q_off[q + 1] - c->q_off[q], c->mode, c->k,
                                 c->out_score + (size_t)q * c->k, c->out_doc + (size_t)q * c->k);
    double t1 = now_ns();
    c->out_n[q] = n < 0 ? 0 : (uint32_t)n;
    if (c->lat_ns) c->lat_ns[q] = t1 - t0;
  }
  return NULL;
}

/* Each thread runs whole queries (a tokio worker per request, tantivy's
 * single-threaded executor).  Returns the wall time in seconds. */
double or_search_batch_q(const or_index* ix, const uint32_t* q_off, const uint32_t* q_terms, const uint8_t* q_occur,
                         const uint32_t* f_off, const uint32_t* f_terms, uint32_t nq, int mode, uint32_t k,
                         float* out_score, uint32_t* out_doc, uint32_t* out_n, double* lat_ns, int threads) {
  BatchCtx c;
  memset(&c, 0, sizeof c);
  c.ix = ix; c.q_off = q_off; c.q_terms = q_terms; c.q_occur = q_occur; c.nq = nq; c.mode = mode; c.k = k;
  c.f_off = f_off; c.f_terms = f_terms;
  c.out_score = out_score; c.out_doc = out_doc; c.out_n = out_n; c.lat_ns = lat_ns; c.next = 0;
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  double t0 = now_ns();
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &c);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  double t1 = now_ns();
  free(th);
  return (t1 - t0) * 1e-9;
}

double or_search_batch_ex(const or_index* ix, const uint32_t* q_off, const uint32_t* q_terms, const uint32_t* f_off,
                          const uint32_t* f_terms, uint32_t nq, int mode, uint32_t k, float* out_score,
                          uint32_t* out_doc, uint32_t* out_n, double* lat_ns, int threads) {
  return or_search_batch_q(ix, q_off, q_terms, NULL, f_off, f_terms, nq, mode, k, out_score, out_doc, out_n, lat_ns,
                           threads);
}

double or_search_batch(const or_index* ix, const uint32_t* q_off, const uint32_t* q_terms, uint32_t nq, int mode,
                       uint32_t k, float* out_score, uint32_t* out_doc, uint32_t* out_n, double* lat_ns, int threads) {
  return or_search_batch_ex(ix, q_off, q_terms, NULL, NULL, nq, mode, k, out_score, out_doc, out_n, lat_ns, threads);
}

/* ---------------------------------------------------------------- bytes model */
/* per-query algorithmic bytes over the merged
 * (text U name) posting list of each term.
 *   B_merge = sum 8*df_t
 *   B_skip  = 8*df_min + sum_{t != min} (1024*blocks_t + 4*ceil(df_t/128))
 *   B       = min(B_merge, B_skip) + F*|I| + 8*min(K,|I|);  1-term: 8*df + 8*min(K,df)
 * out[0]=B_merge out[1]=B_skip out[2]=B out[3]=|I|
 */
static uint32_t* merged_docs(const or_index* ix, uint32_t term, uint32_t* n_out) {
  if (term >= ix->n_terms) { *n_out = 0; return NULL; }
  const Postings* a = &ix->fld[0][term];
  const Postings* b = &ix->fld[1][term];
  uint32_t* out = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)a->n + b->n + 1));
  uint32_t i = 0, j = 0, n = 0;
  while (i < a->n || j < b->n) {
    uint32_t x = i < a->n ? a->doc[i] : OR_TERMINATED;
    uint32_t y = j < b->n ? b->doc[j] : OR_TERMINATED;
    uint32_t d = x < y ? x : y;
    out[n++] = d;
    if (x == d) ++i;
    if (y == d) ++j;
  }
  *n_out = n;
  return out;
}

typedef struct { uint32_t* d; uint32_t n; uint32_t qpos; } MList;
static int mlist_cmp(const void* a, const void* b) {
  const MList* x = (const MList*)a; const MList* y = (const MList*)b;
  if (x->n != y->n) return x->n < y->n ? -1 : 1;
  return (x->qpos > y->qpos) - (x->qpos < y->qpos);
}

int or_bytes_model(const or_index* ix, const uint32_t* terms, uint32_t m, uint32_t k, double* out) {
  if (m < 1 || m > OR_MAX_TERMS) return -1;
  MList L[OR_MAX_TERMS];
  for (uint32_t i = 0; i < m; ++i) { L[i].d = merged_docs(ix, terms[i], &L[i].n); L[i].qpos = i; }
  double F = ix->has_name ? 2.0 : 1.0;
  if (m == 1) {
    double df = L[0].n;
    out[0] = out[1] = 8.0 * df;
    out[2] = 8.0 * df + 8.0 * (df < k ? df : k);
    out[3] = df;
    free(L[0].d);
    return 0;
  }
  qsort(L, m, sizeof(MList), mlist_cmp);
  double bmerge = 0;
  for (uint32_t i = 0; i < m; ++i) bmerge += 8.0 * L[i].n;
  double bskip = 8.0 * L[0].n;
  uint32_t ns = L[0].n;
  uint32_t* S = (uint32_t*)malloc(sizeof(uint32_t) * (ns + 1));
  if (ns) memcpy(S, L[0].d, sizeof(uint32_t) * ns);
  for (uint32_t t = 1; t < m; ++t) {
    const uint32_t* d = L[t].d;
    uint32_t n = L[t].n;
    uint64_t blocks = 0;
    int64_t last_block = -1;
    uint32_t keep = 0, lb = 0;
    for (uint32_t i = 0; i < ns; ++i) {
      uint32_t c = S[i];
      /* lower_bound(t, c); candidates ascend so lb moves forward */
      uint32_t lo = lb, hi = n;
      while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (d[mid] < c) lo = mid + 1; else hi = mid; }
      lb = lo;
      if (lb < n) {
        int64_t blk = lb / OR_BLOCK;
        if (blk != last_block) { ++blocks; last_block = blk; }
        if (d[lb] == c) S[keep++] = c;
      }
    }
    ns = keep;
    bskip += 1024.0 * (double)blocks + 4.0 * (double)((n + OR_BLOCK - 1) / OR_BLOCK);
  }
  double bmin = bmerge < bskip ? bmerge : bskip;
  out[0] = bmerge; out[1] = bskip;
  out[2] = bmin + F * ns + 8.0 * (ns < k ? ns : k);
  out[3] = ns;
  free(S);
  for (uint32_t i = 0; i < m; ++i) free(L[i].d);
  return 0;
}
