// Traffic models of the device kernels: the roofline numerators of bench.py
// (DESIGN.md §5).  A query batch is replayed on the host over one snapshot's
// layout -- the host posting copy (keep_host_postings) and the device's score,
// bound and directory tables read back -- issuing the loads k_conj / k_disj
// (kernels.hip) issue:
//   * the algorithmic bytes: the bytes each load needs (4 B or 8 B);
//   * the line floor: 128 B x the distinct 128-B lines those loads touch in
//     the launch -- a gather that needs 4 B moves a whole line from HBM
//     (tools/calib_fetch: 128 B of DRAM per scattered dword), so measured
//     traffic / line floor separates re-fetch (> 1) from granularity;
//   * the per-query line sum: the floor when no line is shared across queries.
// With a threshold (the query's final k-th best score) the replay prunes as
// an exact MaxScore kernel at that threshold must at least (bounds inflated
// by 2^-17 as in kernels.hip); without one, k_conj's cascade is exhaustive.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "../../include/fugu.h"
#include "fg_host.h"
#include "fg_internal.h"

using fgh::fail;
using fgh::hw_threads;
using fgh::parallel_dynamic;

namespace {

enum Arr : uint32_t { A_DOC, A_TFN, A_RANK, A_SRANK, A_SRANKW, A_DIR, A_BMAX, A_TMAX, A_TDIR, A_CMAX, A_TSUB, A_N };
constexpr uint64_t kLine = 128;
constexpr float kInflate = 1.00000762939453125f;  // kernels.hip inflate_bound: 1 + 2^-17

// host view of one snapshot: the postings (host copy) and the device tables the
// kernels read, copied back; psc: every posting's score under the snapshot's
// current statistics, formed on the host from the payloads as the kernels form
// it at query time; the bound tables scaled to the current statistics as the
// plans scale them (term_ratio)
struct Snap {
  const fg_index* ix = nullptr;
  const uint32_t* doc = nullptr;
  uint32_t pw = 2;  // payload bytes per posting the kernels load (tfn, + tfn_name)
  std::vector<float> psc, tmax, bmax, cmax;
  std::vector<uint64_t> tsub, srank;  // srank: the sparse rank block entries
  std::vector<uint32_t> dir_off, toff, coff;
  uint64_t bytes[A_N] = {0};
  int load(const fg_index* x) {
    ix = x;
    doc = x->h_doc ? x->h_doc->data() : nullptr;
    const uint64_t P = x->n_postings, V = x->n_terms;
    HIPCHK(hipSetDevice(x->dev));
    psc.resize(P);
    dir_off.resize(V);
    toff.resize(V);
    coff.resize(V);
    tmax.resize(x->tile_entries);
    tsub.assign(x->d.tsub ? x->tile_entries : 0, ~0ull);
    bmax.resize(x->dir_entries);
    cmax.resize(x->n_sc);
    auto rd = [](void* dst, const void* src, size_t n) -> hipError_t {
      return n && src ? hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) : hipSuccess;
    };
    {
      std::vector<uint16_t> tv(P), tn(x->d.tfn_name ? P : 0);
      std::vector<uint64_t> ep(x->d.n_esc);
      std::vector<uint32_t> et(x->d.n_esc);
      HIPCHK(rd(tv.data(), x->d.tfn, 2 * P));
      HIPCHK(rd(tn.data(), x->d.tfn_name, 2 * tn.size()));
      HIPCHK(rd(ep.data(), x->d.esc_pos, 8 * ep.size()));
      HIPCHK(rd(et.data(), x->d.esc_tf, 4 * et.size()));
      // the kernels read the build-time scores (4 B) while the statistics are the
      // build's, else the payloads (2 B; 4 B with names)
      pw = x->same_stats || x->d.tfn_name ? 4 : 2;
      parallel_dynamic(x->n_terms, hw_threads(0), 256, [&](int, uint32_t b, uint32_t e) {
        for (uint32_t t = b; t < e; ++t)
          for (uint64_t p = x->off[t]; p < x->off[t + 1]; ++p) {
            const uint32_t v = tv[p] | (tn.empty() ? 0u : (uint32_t)tn[p] << 16);
            uint32_t tt = v & 0xFFu, tm = (v >> 16) & 0xFFu;
            if (tt == fg::kTfEsc || tm == fg::kTfEsc) {
              const uint32_t ex = fg::tf_escaped(ep.data(), et.data(), ep.size(), p);
              if (tt == fg::kTfEsc) tt = ex & 0xFFFFu;
              if (tm == fg::kTfEsc) tm = ex >> 16;
            }
            float sc = 0.0f;
            if (tt) sc += fg::field_score(tt, (v >> 8) & 0xFFu, x->w_text[t], x->cache);
            if (tm) sc += fg::field_score(tm, v >> 24, x->w_name[t], x->cache + 256);
            psc[p] = sc;
          }
      });
    }
    HIPCHK(rd(dir_off.data(), x->d.dir_off, 4 * V));
    HIPCHK(rd(toff.data(), x->d.toff, 4 * V));
    HIPCHK(rd(coff.data(), x->d.coff, 4 * V));
    HIPCHK(rd(tmax.data(), x->d.tmax, 4 * tmax.size()));
    HIPCHK(rd(tsub.data(), x->d.tsub, 8 * tsub.size()));
    HIPCHK(rd(bmax.data(), x->d.bmax, 4 * bmax.size()));
    HIPCHK(rd(cmax.data(), x->d.cmax, 4 * cmax.size()));
    srank.resize((uint64_t)(x->n_rank - x->d.n_prank) * x->d.srank_blocks);
    HIPCHK(rd(srank.data(), x->d.srank, 8 * srank.size()));
    if (!x->same_stats)  // the bounds as a plan scales them (DevPlan::q_rup)
      parallel_dynamic(x->n_terms, hw_threads(0), 256, [&](int, uint32_t b, uint32_t e) {
        for (uint32_t t = b; t < e; ++t) {
          float rdn, rup;
          fgh::term_ratio(x, t, &rdn, &rup);
          if (rup == 1.0f) continue;
          const uint32_t d0 = dir_off[t], d1 = t + 1 < x->n_terms ? dir_off[t + 1] : (uint32_t)x->dir_entries;
          for (uint32_t i = d0; i < d1; ++i) bmax[i] *= rup;
          if (toff[t] != 0xFFFFFFFFu)
            for (uint64_t i = toff[t]; i <= toff[t] + (uint64_t)x->n_tiles; ++i) tmax[i] *= rup;
          const uint64_t nc = (len(t) + fg::kChunk - 1) / fg::kChunk;
          for (uint64_t i = 0; i < nc; ++i) cmax[coff[t] + i] *= rup;
        }
      });
    bytes[A_DOC] = 4 * P;
    bytes[A_TFN] = (uint64_t)pw * P;
    bytes[A_RANK] = 8ull * x->d.n_prank * x->d.rank_words;
    bytes[A_SRANK] = 8ull * srank.size();
    bytes[A_SRANKW] = 8ull * x->n_srank_words;
    bytes[A_DIR] = bytes[A_BMAX] = 4 * x->dir_entries;
    bytes[A_TMAX] = bytes[A_TDIR] = 4 * x->tile_entries;
    bytes[A_CMAX] = 4ull * x->n_sc;
    bytes[A_TSUB] = 8ull * tsub.size();
    return FG_OK;
  }
  // the loads of a rank-kind probe of doc d (plain: the word; sparse: the
  // block entry, then the word when the term holds any of its docs)
  template <class Acc>
  void rank_loads(Acc& A, uint32_t s, uint32_t slot, uint32_t d, double& cat) const {
    if (slot <= ix->d.n_prank) {
      A.gather(s, A_RANK, ((uint64_t)(slot - 1) * ix->d.rank_words + fg::rank_word(d)) * 8, 8, cat);
      return;
    }
    const uint64_t at = (uint64_t)(slot - 1 - ix->d.n_prank) * ix->d.srank_blocks + fg::srank_block(d);
    A.gather(s, A_SRANK, at * 8, 8, cat);
    const uint32_t w = fg::srank_index(srank[at], d);
    if (w != 0xFFFFFFFFu) A.gather(s, A_SRANKW, (uint64_t)w * 8, 8, cat);
  }
  uint64_t len(uint32_t t) const { return ix->off[t + 1] - ix->off[t]; }
  const uint32_t* list(uint32_t t) const { return doc + ix->off[t]; }
  // first position of term t's list with doc >= d (a bucket directory entry)
  uint32_t pos_ge(uint32_t t, uint64_t d) const {
    const uint32_t* l = list(t);
    const uint64_t n = len(t);
    if (d > 0xFFFFFFFFull) return (uint32_t)n;
    return (uint32_t)(std::lower_bound(l, l + n, (uint32_t)d) - l);
  }
};

// the loads of one query: bytes by category and the lines they touch.  Loads
// are issued per stream (one array of one term); a stream's consecutive loads
// of one line are recorded once (the set of lines is what counts)
struct Acc {
  std::vector<uint64_t> lines;
  uint64_t last[fg::kMaxTerms + 1][A_N];
  double stream = 0, probe = 0, loads = 0;
  void reset() {
    lines.clear();
    std::memset(last, 0xFF, sizeof last);
    stream = probe = loads = 0;
  }
  void line(uint32_t s, Arr a, uint64_t l) {
    if (last[s][a] == l) return;
    last[s][a] = l;
    lines.push_back(((uint64_t)a << 56) | l);
  }
  // one load of nb bytes at byte offset `at` of array a (stream s)
  void gather(uint32_t s, Arr a, uint64_t at, uint32_t nb, double& cat) {
    line(s, a, at / kLine);
    if ((at + nb - 1) / kLine != at / kLine) line(s, a, (at + nb - 1) / kLine);
    cat += nb;
    loads += 1;
  }
  // a coalesced stream of n elements of eb bytes from element e0
  void range(uint32_t s, Arr a, uint64_t e0, uint64_t n, uint32_t eb, double& cat) {
    if (!n) return;
    for (uint64_t l = e0 * eb / kLine; l <= ((e0 + n) * eb - 1) / kLine; ++l) line(s, a, l);
    cat += (double)n * eb;
    loads += (double)n;
  }
};

// union of the lines of every query of the launch
struct Union {
  std::vector<std::atomic<uint64_t>> bm[A_N];
  void init(const Snap& s) {
    for (uint32_t a = 0; a < A_N; ++a) {
      qlines[a].store(0, std::memory_order_relaxed);
      const uint64_t words = (s.bytes[a] / kLine + 2 + 63) / 64;
      std::vector<std::atomic<uint64_t>> v(words);
      for (auto& w : v) w.store(0, std::memory_order_relaxed);
      bm[a].swap(v);
    }
  }
  std::atomic<uint64_t> qlines[A_N];  // per-query distinct lines summed, by array
  // sorts / dedups the query's lines; returns how many are distinct
  uint64_t add(std::vector<uint64_t>& lines) {
    std::sort(lines.begin(), lines.end());
    lines.erase(std::unique(lines.begin(), lines.end()), lines.end());
    for (uint64_t x : lines) {
      qlines[x >> 56].fetch_add(1, std::memory_order_relaxed);
      const uint32_t a = (uint32_t)(x >> 56);
      const uint64_t l = x & ((1ull << 56) - 1);
      if ((l >> 6) < bm[a].size()) bm[a][l >> 6].fetch_or(1ull << (l & 63), std::memory_order_relaxed);
    }
    return lines.size();
  }
  uint64_t count(uint32_t a) const {
    uint64_t n = 0;
    for (const auto& w : bm[a]) n += (uint64_t)__builtin_popcountll(w.load(std::memory_order_relaxed));
    return n;
  }
  uint64_t count() const {
    uint64_t n = 0;
    for (uint32_t a = 0; a < A_N; ++a) n += count(a);
    return n;
  }
};

inline uint64_t key_of(float s, uint32_t d) { return fg::make_key(s, d); }

// Probe of term t at doc d as k_conj's probe_list / k_disj's rank probe and
// directory search issue it (stream s); returns the posting score or -1.
float probe_term(const Snap& S, Acc& A, uint32_t s, uint32_t t, uint32_t d, double& cat) {
  const uint32_t meta = S.ix->tmeta[t];
  const uint32_t slot = fg::meta_slot(meta);
  const uint32_t* l = S.list(t);
  const uint64_t n = S.len(t), base = S.ix->off[t];
  if (slot && fg::meta_rank(meta)) {
    S.rank_loads(A, s, slot, d, cat);
    const uint64_t p = std::lower_bound(l, l + n, d) - l;
    if (p < n && l[p] == d) {
      A.gather(s, A_TFN, (base + p) * S.pw, S.pw, cat);
      return S.psc[base + p];
    }
    return -1.0f;
  }
  const uint32_t B = meta & 0xFFu, St = (meta >> 8) & 0xFFu;
  const uint64_t b = d >> B;
  const uint64_t dirb = (uint64_t)S.dir_off[t] + b;
  A.gather(s, A_DIR, dirb * 4, 4, cat);
  A.gather(s, A_DIR, (dirb + 1) * 4, 4, cat);
  uint32_t pos = S.pos_ge(t, b << B);
  const uint32_t hi = S.pos_ge(t, (b + 1) << B);
  for (uint32_t st = St; st > 0; --st) {
    const uint32_t half = 1u << (st - 1), idx = pos + half - 1;
    if (idx < hi) {
      A.gather(s, A_DOC, (base + idx) * 4, 4, cat);
      if (l[idx] < d) pos += half;
    }
  }
  if (pos < hi) {
    A.gather(s, A_DOC, (base + pos) * 4, 4, cat);
    if (l[pos] == d) {
      A.gather(s, A_TFN, (base + pos) * S.pw, S.pw, cat);
      return S.psc[base + pos];
    }
  }
  return -1.0f;
}

// ---------------------------------------------------------------- k_conj
// One Must-driven query (pure conjunction, terms in cost order) as k_conj runs
// it: every lead chunk's postings (a single list skips the chunks whose
// block-max cannot reach the threshold), then per lead candidate the MaxScore
// bound and the other lists in order, each probe one rank word (+ the posting
// score on a hit) or one bucket-directory search; returns the docs that pass
// every list and the threshold.
uint64_t model_conj(const Snap& S, const uint32_t* terms, uint32_t m, bool has_thr, float thr, Acc& A) {
  const fg_index* ix = S.ix;
  const uint64_t thk = has_thr && thr > 0.0f ? key_of(thr, 0xFFFFFFFFu) : 0;  // lowest key with the score
  const uint32_t t0 = terms[0];
  const uint64_t base = ix->off[t0], df = S.len(t0);
  const uint32_t* ld = S.list(t0);
  uint64_t kept = 0;
  if (m == 1) {
    const uint64_t nch = (df + fg::kChunk - 1) / fg::kChunk;
    for (uint64_t c = 0; c < nch; ++c) {
      A.gather(0, A_CMAX, ((uint64_t)S.coff[t0] + c) * 4, 4, A.stream);
      if (thk && key_of(S.cmax[S.coff[t0] + c] * kInflate, 0u) < thk) continue;
      const uint64_t p0 = c * fg::kChunk, n = std::min<uint64_t>(fg::kChunk, df - p0);
      A.range(0, A_DOC, base + p0, n, 4, A.stream);
      A.range(0, A_TFN, base + p0, n, S.pw, A.stream);
      for (uint64_t p = p0; p < p0 + n; ++p) kept += key_of(S.psc[base + p], ld[p]) >= thk ? 1 : 0;
    }
    return kept;
  }
  // MaxScore suffix bounds (fg_plan_create's q_ub: f32 sums from the last list)
  float qub[fg::kMaxTerms + 1] = {0};
  {
    float acc = 0.0f;
    for (uint32_t j = m; j-- > 1;) {
      acc += fgh::term_max_now(ix, terms[j]);
      qub[j] = acc;
    }
  }
  A.range(0, A_DOC, base, df, 4, A.stream);
  A.range(0, A_TFN, base, df, S.pw, A.stream);
  for (uint64_t p = 0; p < df; ++p) {
    const uint32_t d = ld[p];
    float s0 = S.psc[base + p], acc = 0.0f;
    if (thk && key_of((s0 + qub[1]) * kInflate, d) < thk) continue;
    bool ok = true;
    for (uint32_t j = 1; j < m && ok; ++j) {
      const float sc = probe_term(S, A, j, terms[j], d, A.probe);
      if (sc < 0.0f) { ok = false; break; }
      if (j == 1) s0 = s0 + sc; else acc += sc;
      if (thk && j + 1 < m && key_of((s0 + acc + qub[j + 1]) * kInflate, d) < thk) ok = false;
    }
    if (ok && key_of(s0 + acc, d) >= thk) ++kept;
  }
  return kept;
}

// ---------------------------------------------------------------- k_disj
// One Should-only query (clauses in clause order, >= 2 present) as k_disj runs
// it at the threshold: per (tile, clause) the posting range and bound (R), the
// MaxScore split per tile (S), the essential clauses' postings (P) through
// bound 1 (the other clauses' tile bounds; a posting of a clause not essential
// in its 512-doc block -- the block split over the sub-tile maxima -- dropped) and bound 2 (every other clause at
// the doc: its rank word + posting score, or its bucket maximum); a doc whose
// other clauses are all dense is exact there, any other is rescored by probing
// every clause that may hold it.  Returns the keys formed at the threshold.
uint64_t model_disj(const Snap& S, const uint32_t* t, uint32_t m, float thr, Acc& A) {
  const fg_index* ix = S.ix;
  const uint32_t TS = fg::kDisjTileShift, N = ix->n_docs;
  const uint64_t thk = thr > 0.0f ? key_of(thr, 0xFFFFFFFFu) : 0;
  uint32_t dlo = 0xFFFFFFFFu, dhi = 0;
  for (uint32_t c = 0; c < m; ++c) {
    dlo = std::min(dlo, ix->first_doc[t[c]]);
    dhi = std::max(dhi, ix->last_doc[t[c]]);
  }
  uint32_t meta[fg::kMaxTerms], B[fg::kMaxTerms], St[fg::kMaxTerms];
  for (uint32_t c = 0; c < m; ++c) {
    meta[c] = ix->tmeta[t[c]];
    B[c] = meta[c] & 0xFFu;
    St[c] = (meta[c] >> 8) & 0xFFu;
  }
  uint64_t kept = 0;
  for (uint32_t ti = dlo >> TS; ti <= (dhi >> TS); ++ti) {
    const uint32_t d0 = ti << TS, d1 = std::min<uint64_t>((uint64_t)d0 + (1u << TS), N);
    uint32_t lo[fg::kMaxTerms], hi[fg::kMaxTerms];
    float ub[fg::kMaxTerms];
    // R: one thread per (tile, clause)
    for (uint32_t c = 0; c < m; ++c) {
      const uint32_t* l = S.list(t[c]);
      const uint64_t base = ix->off[t[c]], dob = S.dir_off[t[c]];
      float u;
      if (B[c] <= TS && S.toff[t[c]] != 0xFFFFFFFFu) {
        const uint64_t to = (uint64_t)S.toff[t[c]] + ti;
        A.gather(c, A_TDIR, to * 4, 4, A.stream);
        A.gather(c, A_TDIR, (to + 1) * 4, 4, A.stream);
        lo[c] = S.pos_ge(t[c], d0);
        hi[c] = S.pos_ge(t[c], d1);
        A.gather(c, A_TMAX, to * 4, 4, A.stream);
        u = S.tmax[to];
      } else if (B[c] <= TS) {
        A.gather(c, A_DIR, (dob + (d0 >> B[c])) * 4, 4, A.stream);
        A.gather(c, A_DIR, (dob + ((d1 - 1) >> B[c]) + 1) * 4, 4, A.stream);
        lo[c] = S.pos_ge(t[c], d0);
        hi[c] = S.pos_ge(t[c], d1);
        u = fgh::term_max_now(S.ix, t[c]);
      } else {
        const uint64_t b = d0 >> B[c];
        A.gather(c, A_DIR, (dob + b) * 4, 4, A.stream);
        A.gather(c, A_DIR, (dob + b + 1) * 4, 4, A.stream);
        const uint32_t p0 = S.pos_ge(t[c], b << B[c]), p1 = S.pos_ge(t[c], (b + 1) << B[c]);
        uint32_t a = p0, e = p0;
        for (uint32_t st = St[c]; st > 0; --st) {
          const uint32_t half = 1u << (st - 1), ia = a + half - 1, ie = e + half - 1;
          if (ia < p1) { A.gather(c, A_DOC, (base + ia) * 4, 4, A.stream); if (l[ia] < d0) a += half; }
          if (ie < p1) { A.gather(c, A_DOC, (base + ie) * 4, 4, A.stream); if (l[ie] < d1) e += half; }
        }
        if (a < p1) { A.gather(c, A_DOC, (base + a) * 4, 4, A.stream); if (l[a] < d0) ++a; }
        if (e < p1) { A.gather(c, A_DOC, (base + e) * 4, 4, A.stream); if (l[e] < d1) ++e; }
        lo[c] = a;
        hi[c] = e;
        A.gather(c, A_BMAX, (dob + b) * 4, 4, A.stream);
        u = S.bmax[dob + b];
      }
      ub[c] = lo[c] < hi[c] ? u : -0.0f;
    }
    // S: the longest prefix of clauses by ascending bound that cannot reach the threshold
    uint32_t ord[fg::kMaxTerms];
    for (uint32_t i = 0; i < m; ++i) {
      uint32_t j = i;
      while (j > 0 && ub[ord[j - 1]] > ub[i]) { ord[j] = ord[j - 1]; --j; }
      ord[j] = i;
    }
    float sacc = 0.0f;
    uint32_t P = 0;
    for (; P < m; ++P) {
      const float s2 = sacc + ub[ord[P]];
      if (key_of(s2 * kInflate, d0) >= thk) break;
      sacc = s2;
    }
    uint32_t ess = 0, any = 0;
    for (uint32_t j = P; j < m; ++j) {
      ess |= 1u << ord[j];
      any |= hi[ord[j]] > lo[ord[j]] ? 1u : 0u;
    }
    if (P == m || !any) continue;
    // the block split (k_disj's S phase, one thread per (tile, block)): the
    // tile's non-essential clauses plus essential ones, smallest tile bound
    // first, while their sub-tile bounds stay below the threshold together
    uint32_t bess[8];
    uint64_t subq[fg::kMaxTerms];  // each clause's sub-tile maxima (~0: its tile bound)
    {
      uint64_t* sub = subq;
      for (uint32_t c = 0; c < m; ++c) {
        sub[c] = ~0ull;
        if (B[c] <= TS && S.toff[t[c]] != 0xFFFFFFFFu && !S.tsub.empty()) {
          const uint64_t to = (uint64_t)S.toff[t[c]] + ti;
          A.gather(c, A_TSUB, to * 8, 8, A.stream);
          sub[c] = S.tsub[to];
        }
      }
      for (uint32_t z = 0; z < 8; ++z) {
        auto bound = [&](uint32_t i) { return fg::q8_bound((uint32_t)(sub[i] >> (8 * z)) & 0xFFu, ub[i]); };
        float sz = 0.0f;
        for (uint32_t i = 0; i < m; ++i)
          if (!((ess >> i) & 1u)) sz += bound(i);
        uint32_t ez = ess, left = ess;
        while (left) {
          uint32_t cc = (uint32_t)__builtin_ctz(left);
          for (uint32_t r = left & (left - 1); r; r &= r - 1) {
            const uint32_t i = (uint32_t)__builtin_ctz(r);
            if (ub[i] < ub[cc]) cc = i;
          }
          left &= ~(1u << cc);
          const float s2 = sz + bound(cc);
          if (key_of(s2 * kInflate, d0) >= thk) break;
          sz = s2;
          ez &= ~(1u << cc);
        }
        bess[z] = S.tsub.empty() ? ess : ez;
      }
    }
    // P: the essential clauses' postings, each segment trimmed to its first..last
    // essential block (the bucket directory's entries there: two 4-B loads)
    for (uint32_t c = 0; c < m; ++c) {
      if (!((ess >> c) & 1u) || lo[c] >= hi[c]) continue;
      uint32_t bm = 0, plo = lo[c], phi = hi[c];  // the streamed range (lo / hi stay the tile's: bound 2 walks them)
      for (uint32_t z = 0; z < 8; ++z) bm |= ((bess[z] >> c) & 1u) << z;
      if (bm != 0xFFu && B[c] <= TS) {
        uint32_t l2 = lo[c], h2 = lo[c];
        if (bm) {
          const uint32_t z0 = (uint32_t)__builtin_ctz(bm), z1 = 31u - (uint32_t)__builtin_clz(bm);
          const uint32_t da = d0 + (z0 << fg::kSubShift), db = std::min<uint32_t>(d0 + ((z1 + 1) << fg::kSubShift), N);
          if (da < db) {
            const uint64_t dob = S.dir_off[t[c]], ba = da >> B[c], bb = ((db - 1) >> B[c]) + 1;
            A.gather(c, A_DIR, (dob + ba) * 4, 4, A.stream);
            A.gather(c, A_DIR, (dob + bb) * 4, 4, A.stream);
            l2 = std::max(l2, S.pos_ge(t[c], ba << B[c]));
            h2 = std::max(l2, std::min(hi[c], S.pos_ge(t[c], bb << B[c])));
          }
        }
        plo = l2;
        phi = h2;
        if (plo >= phi) continue;
      }
      const uint64_t base = ix->off[t[c]];
      const uint32_t* l = S.list(t[c]);
      A.range(c, A_DOC, base + plo, phi - plo, 4, A.stream);
      A.range(c, A_TFN, base + plo, phi - plo, S.pw, A.stream);
      uint32_t cur[fg::kMaxTerms];
      for (uint32_t i = 0; i < m; ++i) cur[i] = lo[i];
      for (uint32_t p = plo; p < phi; ++p) {
        const uint32_t d = l[p];
        const float ps = S.psc[base + p];
        // bound 1: the other clauses' bounds over the doc's 512-doc block
        const uint32_t zb = ((d - d0) >> fg::kSubShift) & 7u;
        float b1 = ps;
        for (uint32_t i = 0; i < m; ++i)
          if (i != c) b1 += fg::q8_bound((uint32_t)(subq[i] >> (8 * zb)) & 0xFFu, ub[i]);
        if (key_of(b1 * kInflate, d) < thk) continue;
        const uint32_t bz = bess[((d - d0) >> fg::kSubShift) & 7u];
        if (!((bz >> c) & 1u)) continue;  // not essential in its block
        // bound 2, clause order; the own clause adds the streamed score
        float sum = 0.0f;
        uint32_t maybe = 0, first = 0xFFFFFFFFu;
        bool exact = true;
        float v[fg::kMaxTerms];
        for (uint32_t i = 0; i < m; ++i) {
          v[i] = -1.0f;
          if (i == c) { sum += ps; v[i] = ps; continue; }
          if (std::signbit(ub[i])) continue;  // no posting of clause i in the tile
          const uint32_t slot = fg::meta_slot(meta[i]);
          const uint32_t* li = S.list(t[i]);
          const uint64_t bi = ix->off[t[i]];
          while (cur[i] < hi[i] && li[cur[i]] < d) ++cur[i];
          const bool here = cur[i] < hi[i] && li[cur[i]] == d;
          if (slot && fg::meta_rank(meta[i])) {
            S.rank_loads(A, i, slot, d, A.probe);
            if (here) {
              A.gather(i, A_TFN, (bi + cur[i]) * S.pw, S.pw, A.probe);
              v[i] = S.psc[bi + cur[i]];
              maybe |= 1u << i;
              sum += v[i];
            }
          } else {
            exact = false;
            const uint64_t at = (uint64_t)S.dir_off[t[i]] + (d >> B[i]);
            A.gather(i, A_BMAX, at * 4, 4, A.probe);
            const float bm = S.bmax[at];
            if (!std::signbit(bm)) {
              maybe |= 1u << i;
              sum += bm;
            }
            if (here) v[i] = S.psc[bi + cur[i]];
          }
        }
        if (exact) {
          first = (uint32_t)__builtin_ctz((maybe | (1u << c)) & bz);
          if (first == c && key_of(sum, d) >= thk) ++kept;
          continue;
        }
        if (key_of(sum * kInflate, d) < thk) continue;
        // rescoring: every clause that may hold d, its own included
        float sc = 0.0f;
        uint32_t matched = 0;
        for (uint32_t i = 0; i < m; ++i) {
          if (i != c && !((maybe >> i) & 1u)) continue;
          const float x = probe_term(S, A, i, t[i], d, A.probe);
          if (x >= 0.0f) { sc += x; matched |= 1u << i; }
        }
        (void)v;
        first = (uint32_t)__builtin_ctz(matched & bz);
        if (first == c && key_of(sc, d) >= thk) ++kept;
      }
    }
  }
  return kept;
}

}  // namespace

extern "C" {

int fg_model_batch(const fg_index* ix, const fg_query_batch* q, uint32_t k, const float* thr_score, double* per_query,
                   fg_model_out* out) {
  if (!ix || !q || !out || (q->n_queries && !q->q_off) || k == 0) return fail(FG_EINVAL, "bad arguments");
  if (!ix->h_doc && ix->n_postings) return fail(FG_EINVAL, "index built without keep_host_postings");
  Snap S;
  if (int rc = S.load(ix)) return rc;
  Union U;
  U.init(S);
  const uint32_t nq = q->n_queries;
  std::vector<double> st(nq, 0.0), pr(nq, 0.0), ou(nq, 0.0), ld(nq, 0.0), ql(nq, 0.0), kp(nq, 0.0);
  std::atomic<bool> bad{false};
  parallel_dynamic(nq, hw_threads(0), 1, [&](int, uint32_t qb, uint32_t qe) {
    Acc A;
    for (uint32_t i = qb; i < qe; ++i) {
      A.reset();
      const uint32_t b = q->q_off[i], e = q->q_off[i + 1];
      if (e < b || e - b > fg::kMaxTerms) { bad = true; return; }
      // the query's clauses as fg_plan_create shapes them (pure Must / pure Should)
      uint32_t tm[fg::kMaxTerms], ts[fg::kMaxTerms], nm = 0, ns = 0;
      bool must_missing = false, other = false;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t t = fgh::local_term(ix, q->terms[j]);
        const uint8_t oc = q->occur ? q->occur[j] : (q->mode == FG_MODE_OR ? FG_OCCUR_SHOULD : FG_OCCUR_MUST);
        const bool present = t < ix->n_terms && ix->off[t + 1] > ix->off[t];
        if (oc == FG_OCCUR_MUST) { tm[nm++] = t; must_missing |= !present; }
        else if (oc == FG_OCCUR_SHOULD) { if (present) ts[ns++] = t; }
        else other = true;
      }
      if (other || (nm && ns)) { bad = true; return; }  // MustNot / mixed shapes: not modelled
      if (nm == 0 && ns == 1) { tm[nm++] = ts[0]; ns = 0; }
      uint64_t kept = 0;
      const bool has_thr = thr_score != nullptr;
      const float th = has_thr ? thr_score[i] : 0.0f;
      if (nm && !must_missing) {
        struct T { uint64_t cost; uint32_t term; };
        T tc[fg::kMaxTerms];
        for (uint32_t j = 0; j < nm; ++j) tc[j] = T{(uint64_t)ix->df_text[tm[j]] + ix->df_name[tm[j]], tm[j]};
        std::stable_sort(tc, tc + nm, [](const T& x, const T& y) { return x.cost < y.cost; });
        for (uint32_t j = 0; j < nm; ++j) tm[j] = tc[j].term;
        kept = model_conj(S, tm, nm, has_thr, th, A);
      } else if (ns >= 2) {
        kept = model_disj(S, ts, ns, th, A);
      }
      st[i] = A.stream;
      pr[i] = A.probe;
      ou[i] = 8.0 * (double)std::min<uint64_t>(kept, k);
      ld[i] = A.loads;
      kp[i] = (double)kept;
      ql[i] = (double)U.add(A.lines);
    }
  });
  if (bad) return fail(FG_EINVAL, "bad query batch (the model covers pure Must / pure Should queries)");
  std::memset(out, 0, sizeof *out);
  for (uint32_t i = 0; i < nq; ++i) {
    out->stream_bytes += st[i];
    out->probe_bytes += pr[i];
    out->output_bytes += ou[i];
    out->loads += ld[i];
    out->candidates += kp[i];
    out->query_line_bytes += (double)kLine * ql[i];
    if (per_query) {
      per_query[4ull * i] = st[i];
      per_query[4ull * i + 1] = pr[i];
      per_query[4ull * i + 2] = ou[i];
      per_query[4ull * i + 3] = st[i] + pr[i] + ou[i];
    }
  }
  out->alg_bytes = out->stream_bytes + out->probe_bytes + out->output_bytes;
  out->line_bytes = (double)kLine * (double)U.count();
  if (getenv("FUGU_MODEL_TRACE")) {  // the line floor and the per-query line sum, by array
    static const char* names[A_N] = {"doc", "tfn", "rank", "srank", "srankw", "dir", "bmax", "tmax", "tdir", "cmax", "tsub"};
    for (uint32_t a = 0; a < A_N; ++a)
      fprintf(stderr, "[fg model] %-6s floor %8.3f GB  per-query sum %8.3f GB\n", names[a],
              (double)kLine * (double)U.count(a) * 1e-9, (double)kLine * (double)U.qlines[a].load() * 1e-9);
  }
  return FG_OK;
}

// SURVEY.md §8(d) algorithmic bytes of tantivy's CPU walk (1 KiB block decode
// per probed 128-posting block), per query
int fg_bytes_model(const fg_index* ix, const fg_query_batch* q, uint32_t k, double* out) {
  if (!ix || !q || !out) return fail(FG_EINVAL, "bad arguments");
  if (!ix->h_doc && ix->n_postings) return fail(FG_EINVAL, "index built without keep_host_postings");
  const double F = ix->has_name ? 2.0 : 1.0;
  std::vector<uint32_t> S;
  for (uint32_t i = 0; i < q->n_queries; ++i) {
    const uint32_t b = q->q_off[i], m = q->q_off[i + 1] - b;
    double* o = out + 4ull * i;
    struct L { uint64_t n, off; uint32_t pos; };
    std::vector<L> ls;
    bool missing = false;
    for (uint32_t j = 0; j < m; ++j) {
      uint32_t t = fgh::local_term(ix, q->terms[b + j]);
      if (t >= ix->n_terms || ix->off[t + 1] == ix->off[t]) { missing = true; break; }
      ls.push_back(L{ix->off[t + 1] - ix->off[t], ix->off[t], j});
    }
    if (m == 0 || missing) { o[0] = o[1] = o[2] = o[3] = 0; continue; }
    if (m == 1) {
      double df = (double)ls[0].n;
      o[0] = o[1] = 8.0 * df;
      o[2] = 8.0 * df + 8.0 * std::min<double>(df, k);
      o[3] = df;
      continue;
    }
    std::stable_sort(ls.begin(), ls.end(), [](const L& x, const L& y) { return x.n < y.n; });
    double bmerge = 0;
    for (auto& l : ls) bmerge += 8.0 * (double)l.n;
    double bskip = 8.0 * (double)ls[0].n;
    S.assign(ix->h_doc->begin() + ls[0].off, ix->h_doc->begin() + ls[0].off + ls[0].n);
    for (size_t t = 1; t < ls.size(); ++t) {
      const uint32_t* d = ix->h_doc->data() + ls[t].off;
      const uint64_t n = ls[t].n;
      uint64_t blocks = 0, lb = 0;
      int64_t last_block = -1;
      size_t keep = 0;
      for (size_t x = 0; x < S.size(); ++x) {
        lb = std::lower_bound(d + lb, d + n, S[x]) - d;
        if (lb < n) {
          int64_t blk = (int64_t)(lb / fg::kBlock);
          if (blk != last_block) { ++blocks; last_block = blk; }
          if (d[lb] == S[x]) S[keep++] = S[x];
        }
      }
      S.resize(keep);
      bskip += 1024.0 * (double)blocks + 4.0 * (double)((n + fg::kBlock - 1) / fg::kBlock);
    }
    const double ns = (double)S.size();
    o[0] = bmerge;
    o[1] = bskip;
    o[2] = std::min(bmerge, bskip) + F * ns + 8.0 * std::min<double>(ns, k);
    o[3] = ns;
  }
  return FG_OK;
}

// Algorithmic bytes per query at the device layout (fugu.h): k_conj's
// exhaustive cascade (mode AND, no threshold) / k_disj at the thresholds
int fg_bytes_model_gpu(const fg_index* ix, const fg_query_batch* q, uint32_t k, double* out) {
  if (!out) return fail(FG_EINVAL, "bad arguments");
  fg_model_out o;
  if (q && q->mode == FG_MODE_OR) {
    std::vector<float> zero(q->n_queries, 0.0f);
    return fg_model_batch(ix, q, k, zero.data(), out, &o);
  }
  return fg_model_batch(ix, q, k, nullptr, out, &o);
}

int fg_bytes_model_or(const fg_index* ix, const fg_query_batch* q, uint32_t k, const float* thr, double* out) {
  if (!thr || !out) return fail(FG_EINVAL, "bad arguments");
  fg_model_out o;
  return fg_model_batch(ix, q, k, thr, out, &o);
}

}  // extern "C"
