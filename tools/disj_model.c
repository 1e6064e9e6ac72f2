/*
 * disj_model.c -- CPU model of k_disj's work on the OR top-k bench batch
 * (design tool, not product code).  Builds the synthetic corpus
 * (libfugu_synth.so), scores every posting with tantivy's
 * Bm25Weight (the same f32 order as the device), and for each query reports
 * how many postings the MaxScore split leaves essential and how many survive
 * each bound, under three thresholds:
 *   thr0  : the planner's starting threshold (best per-clause K-th score),
 *   seed  : the K-th best exact score inside the S tiles of largest upper bound
 *           (sum of the clauses' tile maxima) -- a seed pass would set this,
 *   final : the query's true K-th best score.
 * Bounds per (tile, clause) are the clause's maximum posting score in the
 * 4096-doc tile.  Usage: disj_model N_DOCS N_QUERIES K [S_TILES] [ZIPF_S]
 *   gcc -O2 -o /tmp/disj_model tools/disj_model.c -L fugu_amd -lfugu_synth -lpthread -lm
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t fgs_doc_lengths(uint64_t, uint32_t, uint64_t, uint32_t, uint32_t, uint64_t*);
int fgs_fill_tokens(uint64_t, uint32_t, const uint64_t*, uint32_t, double, uint64_t, uint32_t*, int);
int fgs_queries(uint32_t, uint32_t, uint32_t, uint32_t, double, uint64_t, uint32_t*, uint32_t*);

#define V (1u << 20)
#define TS 12
#define TILE (1u << TS)

static uint32_t N, NQ, K, STILES;
static uint64_t* poff;   /* [V+1] */
static uint32_t* pdoc;   /* postings */
static float* psc;       /* posting scores */
static float* ktopk;     /* per term K-th best score (0 if fewer) */
static uint32_t *q_off, *q_terms;

typedef struct {
  double ess[5], b1[5], pres[5], hits_final, union_post, skip_tiles[5], filt_tiles[5];
  double thr_ratio_seed, n_seed_ok, thr_ratio_imp, n_imp;
} Acc;

static int cmpf_desc(const void* a, const void* b) {
  float x = *(const float*)a, y = *(const float*)b;
  return (x < y) - (x > y);
}

static float kth_best(float* v, uint32_t n, uint32_t k) {
  if (n < k) return 0.0f;
  /* partial select: nth_element by quickselect */
  uint32_t lo = 0, hi = n - 1, want = k - 1;
  while (lo < hi) {
    float p = v[(lo + hi) / 2];
    uint32_t i = lo, j = hi;
    while (i <= j) {
      while (v[i] > p) ++i;
      while (v[j] < p) --j;
      if (i <= j) { float t = v[i]; v[i] = v[j]; v[j] = t; ++i; if (j == 0) break; --j; }
    }
    if (want <= j) hi = j; else if (want >= i) lo = i; else break;
  }
  return v[want];
}

static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static volatile uint32_t next_q = 0;
static Acc tot;

static void* worker(void* arg) {
  (void)arg;
  const uint32_t nt = (N + TILE - 1) / TILE;
  float* acc = calloc(N, sizeof(float));
  uint8_t* mk = calloc(N, 1);     /* bit i: clause i present */
  float* tmx = malloc(sizeof(float) * nt * 16);
  uint32_t* tcnt = malloc(sizeof(uint32_t) * nt * 16);
  float* tub = malloc(sizeof(float) * nt);
  float* scratch = malloc(sizeof(float) * (size_t)N);
  uint32_t* order = malloc(sizeof(uint32_t) * nt);
  Acc a;
  memset(&a, 0, sizeof a);
  for (;;) {
    uint32_t q = __atomic_fetch_add(&next_q, 1u, __ATOMIC_RELAXED);
    if (q >= NQ) break;
    const uint32_t* t = q_terms + q_off[q];
    uint32_t m = q_off[q + 1] - q_off[q];
    memset(tmx, 0, sizeof(float) * nt * m);
    memset(tcnt, 0, sizeof(uint32_t) * nt * m);
    float thr0 = 0.0f;
    for (uint32_t i = 0; i < m; ++i) {
      uint32_t tt = t[i];
      if (ktopk[tt] > thr0) thr0 = ktopk[tt];
      for (uint64_t p = poff[tt]; p < poff[tt + 1]; ++p) {
        uint32_t d = pdoc[p];
        acc[d] += psc[p];
        mk[d] |= (uint8_t)(1u << i);
        uint32_t ti = d >> TS;
        if (psc[p] > tmx[ti * m + i]) tmx[ti * m + i] = psc[p];
        tcnt[ti * m + i]++;
      }
    }
    /* exact union scores -> final threshold */
    uint32_t nu = 0;
    for (uint32_t i = 0; i < m; ++i)
      for (uint64_t p = poff[t[i]]; p < poff[t[i] + 1]; ++p) {
        uint32_t d = pdoc[p];
        if (mk[d] & 0x80) continue;
        mk[d] |= 0x80;
        scratch[nu++] = acc[d];
      }
    a.union_post += nu;
    float thrF = kth_best(scratch, nu, K);
    for (uint32_t i = 0; i < m; ++i)
      for (uint64_t p = poff[t[i]]; p < poff[t[i] + 1]; ++p) mk[pdoc[p]] &= 0x7F;
    /* seed threshold: exact scores in the STILES tiles of largest bound */
    for (uint32_t ti = 0; ti < nt; ++ti) {
      float s = 0;
      for (uint32_t i = 0; i < m; ++i) s += tmx[ti * m + i];
      tub[ti] = s;
      order[ti] = ti;
    }
    /* partial sort of tiles by bound (selection of STILES largest) */
    uint32_t ns = STILES < nt ? STILES : nt;
    for (uint32_t x = 0; x < ns; ++x) {
      uint32_t best = x;
      for (uint32_t y = x + 1; y < nt; ++y) if (tub[order[y]] > tub[order[best]]) best = y;
      uint32_t tmp = order[x]; order[x] = order[best]; order[best] = tmp;
    }
    uint32_t nseed = 0;
    for (uint32_t x = 0; x < ns; ++x) {
      uint32_t ti = order[x];
      uint32_t d0 = ti << TS, d1 = d0 + TILE < N ? d0 + TILE : N;
      for (uint32_t d = d0; d < d1; ++d) if (mk[d]) scratch[nseed++] = acc[d];
    }
    float thrS = kth_best(scratch, nseed, K);
    /* impact seed: the union of every clause's K best-scoring docs, exact scores */
    uint32_t ni = 0;
    for (uint32_t i = 0; i < m; ++i) {
      uint64_t lo = poff[t[i]], hi = poff[t[i] + 1];
      if (hi - lo == 0) continue;
      float kt = ktopk[t[i]];
      for (uint64_t p = lo; p < hi; ++p)
        if (psc[p] >= kt && !(mk[pdoc[p]] & 0x40)) { mk[pdoc[p]] |= 0x40; scratch[ni++] = acc[pdoc[p]]; }
    }
    for (uint32_t i = 0; i < m; ++i)
      for (uint64_t p = poff[t[i]]; p < poff[t[i] + 1]; ++p) mk[pdoc[p]] &= 0xBF;
    float thrI = kth_best(scratch, ni, K);
    if (thrI < thr0) thrI = thr0;
    a.thr_ratio_imp += thrF > 0 ? thrI / thrF : 1.0;
    a.n_imp += ni;
    if (thrS > thr0) { a.n_seed_ok += 1; }
    if (thrS < thr0) thrS = thr0;
    a.thr_ratio_seed += thrF > 0 ? thrS / thrF : 1.0;
    float th[5] = {thr0, thrS, thrI, thrF, thr0};
    /* running threshold (v = 4): the K-th best exact score among the docs of the
     * tiles finished STILES tiles before this one (a min-heap of K scores) */
    float* heap = scratch;  /* reuse: K floats */
    uint32_t hn = 0, done_t = 0;
    for (int v = 0; v < 5; ++v) {
      float thr = th[v];
      for (uint32_t ti = 0; ti < nt; ++ti) {
        if (v == 4) {
          while (done_t + STILES <= ti) {
            uint32_t d0 = done_t << TS, d1 = d0 + TILE < N ? d0 + TILE : N;
            for (uint32_t d = d0; d < d1; ++d) {
              if (!mk[d]) continue;
              float x = acc[d];
              if (hn < K) {  /* sift up */
                uint32_t i = hn++;
                while (i > 0 && heap[(i - 1) / 2] > x) { heap[i] = heap[(i - 1) / 2]; i = (i - 1) / 2; }
                heap[i] = x;
              } else if (x > heap[0]) {  /* replace min, sift down */
                uint32_t i = 0;
                for (;;) {
                  uint32_t l = 2 * i + 1, r = l + 1, sm = i;
                  float smv = x;
                  if (l < K && heap[l] < smv) { sm = l; smv = heap[l]; }
                  if (r < K && heap[r] < smv) { sm = r; smv = heap[r]; }
                  if (sm == i) break;
                  heap[i] = heap[sm]; i = sm;
                }
                heap[i] = x;
              }
            }
            ++done_t;
          }
          thr = hn == K && heap[0] > thr0 ? heap[0] : thr0;
        }
        /* MaxScore split: sort clause bounds ascending, non-essential prefix below thr */
        float ub[16]; uint32_t ord[16];
        for (uint32_t i = 0; i < m; ++i) {
          ub[i] = tcnt[ti * m + i] ? tmx[ti * m + i] : 0.0f;
          uint32_t j = i;
          while (j > 0 && ub[ord[j - 1]] > ub[i]) { ord[j] = ord[j - 1]; --j; }
          ord[j] = i;
        }
        float s = 0; uint32_t P = 0;
        for (; P < m; ++P) { float s2 = s + ub[ord[P]]; if (s2 * 1.0000076f >= thr) break; s = s2; }
        if (P == m) { a.skip_tiles[v] += 1; continue; }
        a.filt_tiles[v] += 1;
        uint32_t ess = 0;
        for (uint32_t j = P; j < m; ++j) ess |= 1u << ord[j];
        float ubsum = 0;
        for (uint32_t i = 0; i < m; ++i) ubsum += ub[i];
        for (uint32_t i = 0; i < m; ++i) {
          if (!((ess >> i) & 1u)) continue;
          uint64_t lo = poff[t[i]], hi = poff[t[i] + 1];
          /* postings of clause i in tile ti: binary search */
          uint64_t l = lo, h = hi;
          while (l < h) { uint64_t md = (l + h) / 2; if (pdoc[md] < (ti << TS)) l = md + 1; else h = md; }
          for (uint64_t p = l; p < hi && (pdoc[p] >> TS) == ti; ++p) {
            uint32_t d = pdoc[p];
            a.ess[v] += 1;
            float b1 = psc[p] + (ubsum - ub[i]);
            if (b1 * 1.0000076f < thr) continue;
            a.b1[v] += 1;
            float pb = psc[p];
            for (uint32_t j = 0; j < m; ++j) if (j != i && ((mk[d] >> j) & 1u)) pb += ub[j];
            if (pb * 1.0000076f < thr) continue;
            a.pres[v] += 1;
            if (v == 3 && acc[d] >= thr) {
              /* count once: first essential clause the doc matches */
              uint32_t first = __builtin_ctz((uint32_t)mk[d] & ess);
              if (first == i) a.hits_final += 1;
            }
          }
        }
      }
    }
    for (uint32_t i = 0; i < m; ++i)
      for (uint64_t p = poff[t[i]]; p < poff[t[i] + 1]; ++p) { acc[pdoc[p]] = 0; mk[pdoc[p]] = 0; }
  }
  pthread_mutex_lock(&mu);
  tot.thr_ratio_imp += a.thr_ratio_imp; tot.n_imp += a.n_imp;
  for (int v = 0; v < 5; ++v) {
    tot.ess[v] += a.ess[v]; tot.b1[v] += a.b1[v]; tot.pres[v] += a.pres[v];
    tot.skip_tiles[v] += a.skip_tiles[v]; tot.filt_tiles[v] += a.filt_tiles[v];
  }
  tot.hits_final += a.hits_final; tot.union_post += a.union_post;
  tot.thr_ratio_seed += a.thr_ratio_seed; tot.n_seed_ok += a.n_seed_ok;
  pthread_mutex_unlock(&mu);
  free(acc); free(mk); free(tmx); free(tcnt); free(tub); free(scratch); free(order);
  return NULL;
}

int main(int argc, char** argv) {
  N = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  NQ = argc > 2 ? (uint32_t)atol(argv[2]) : 1024u;
  K = argc > 3 ? (uint32_t)atol(argv[3]) : 1000u;
  STILES = argc > 4 ? (uint32_t)atol(argv[4]) : 8u;
  double zs = argc > 5 ? atof(argv[5]) : 1.0;
  int T = 8;
  uint64_t* doff = malloc(sizeof(uint64_t) * (N + 1));
  uint64_t ntok = fgs_doc_lengths(0, N, 0x5EED1, 8, 113, doff);
  uint32_t* tok = malloc(sizeof(uint32_t) * ntok);
  fgs_fill_tokens(0, N, doff, V, zs, 20250808, tok, T);
  /* invert: per doc distinct terms with tf */
  uint64_t* cnt = calloc(V + 1, sizeof(uint64_t));
  uint8_t* fn = malloc(N);
  /* fieldnorm table */
  uint32_t tab[256];
  { uint32_t i = 0; for (; i <= 40; ++i) tab[i] = i; uint64_t x = 40, st = 2;
    while (i < 256) { for (int j = 0; j < 8 && i < 256; ++j) { x += st; tab[i++] = (uint32_t)x; } st <<= 1; } }
  uint32_t* sc = malloc(sizeof(uint32_t) * 256);
  for (uint32_t d = 0; d < N; ++d) {
    uint32_t L = (uint32_t)(doff[d + 1] - doff[d]);
    uint32_t id = 0; while (id < 255 && tab[id + 1] <= L) ++id;
    fn[d] = (uint8_t)id;
    uint32_t* tk = tok + doff[d];
    /* sort the doc's tokens (small) */
    for (uint32_t i = 1; i < L; ++i) { uint32_t v = tk[i], j = i; while (j > 0 && tk[j - 1] > v) { tk[j] = tk[j - 1]; --j; } tk[j] = v; }
    for (uint32_t i = 0; i < L; ++i) if (i == 0 || tk[i] != tk[i - 1]) cnt[tk[i] + 1]++;
  }
  free(sc);
  for (uint32_t v = 0; v < V; ++v) cnt[v + 1] += cnt[v];
  poff = cnt;
  uint64_t P = poff[V];
  pdoc = malloc(sizeof(uint32_t) * P);
  uint16_t* ptf = malloc(sizeof(uint16_t) * P);
  uint64_t* cur = malloc(sizeof(uint64_t) * V);
  memcpy(cur, poff, sizeof(uint64_t) * V);
  for (uint32_t d = 0; d < N; ++d) {
    uint32_t* tk = tok + doff[d];
    uint32_t L = (uint32_t)(doff[d + 1] - doff[d]);
    for (uint32_t i = 0; i < L;) {
      uint32_t j = i; while (j < L && tk[j] == tk[i]) ++j;
      uint64_t p = cur[tk[i]]++;
      pdoc[p] = d; ptf[p] = (uint16_t)(j - i);
      i = j;
    }
  }
  free(cur);
  float avgdl = (float)ntok / (float)N;
  float cache[256];
  for (int i = 0; i < 256; ++i) cache[i] = 1.2f * ((1.0f - 0.75f) + (0.75f * (float)tab[i]) / avgdl);
  psc = malloc(sizeof(float) * P);
  ktopk = calloc(V, sizeof(float));
  float* tmp = malloc(sizeof(float) * N);
  for (uint32_t v = 0; v < V; ++v) {
    uint64_t df = poff[v + 1] - poff[v];
    float w = logf(1.0f + ((float)(N - df) + 0.5f) / ((float)df + 0.5f)) * 2.2f;
    for (uint64_t p = poff[v]; p < poff[v + 1]; ++p) {
      float tf = (float)ptf[p];
      psc[p] = w * (tf / (tf + cache[fn[pdoc[p]]]));
    }
    if (df >= K) {
      memcpy(tmp, psc + poff[v], sizeof(float) * df);
      ktopk[v] = kth_best(tmp, (uint32_t)df, K);
    }
  }
  free(tmp);
  free(tok);
  fprintf(stderr, "corpus %u docs, %llu postings\n", N, (unsigned long long)P);
  q_off = malloc(sizeof(uint32_t) * (NQ + 1));
  q_terms = malloc(sizeof(uint32_t) * NQ * 5);
  fgs_queries(4096 > NQ ? NQ : NQ, 2, 5, 1u << 14, 1.0, 7, q_off, q_terms);
  pthread_t th[8];
  for (int i = 0; i < T; ++i) pthread_create(&th[i], NULL, worker, NULL);
  for (int i = 0; i < T; ++i) pthread_join(th[i], NULL);
  const char* nm[5] = {"thr0", "seed", "impact", "final", "running"};
  printf("{\"n_docs\": %u, \"queries\": %u, \"k\": %u, \"seed_tiles\": %u, \"union_docs\": %.0f,\n", N, NQ, K, STILES,
         tot.union_post);
  printf(" \"seed_over_final_thr_mean\": %.4f, \"seed_beats_thr0\": %.0f, \"hits_final\": %.0f,\n",
         tot.thr_ratio_seed / NQ, tot.n_seed_ok, tot.hits_final);
  printf(" \"impact_over_final_thr_mean\": %.4f, \"impact_docs_per_query\": %.0f,\n", tot.thr_ratio_imp / NQ, tot.n_imp / NQ);
  for (int v = 0; v < 5; ++v)
    printf(" \"%s\": {\"tiles_skip\": %.0f, \"tiles_work\": %.0f, \"essential\": %.0f, \"past_bound1\": %.0f, "
           "\"past_presence\": %.0f}%s\n",
           nm[v], tot.skip_tiles[v], tot.filt_tiles[v], tot.ess[v], tot.b1[v], tot.pres[v], v < 4 ? "," : "}");
  return 0;
}
