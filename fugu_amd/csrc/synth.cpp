// Deterministic synthetic Zipf corpora and query streams.
//
// Test/bench infrastructure, not the product path: it produces the token
// streams that the product index builder (index.cpp) and the CPU oracle
// (oracle/fugu_oracle.c) both consume.  tools/synth_ref.py is a numpy mirror
// of this file used on small N to prove the two agree bit for bit.
//
// Spec (also written out in DESIGN.md §Corpus):
//   mix64     = SplitMix64 finaliser
//   h2(s,a)   = mix64(s + G*(a+1))            G = 0x9E3779B97F4A7C15
//   h3(s,a,b) = mix64(h2(s,a) + G*(b+1))
//   L_d       = len_min + h2(seed_L, d) % len_span          (8 + U{0..112})
//   u         = (h >> 11) * 2^-53
//   rank(u)   = 1 + #{ i < V-1 : cum[i] <= u*cum[V-1] },   cum = running sum of r^-s
//   token j of doc d: term id = rank(h3(seed_T, d, j)) - 1
//   query q: m = m_min + h2(seed_Q+1, q) % (m_max-m_min+1); terms drawn with
//            h3(seed_Q, q, i), i = 0,1,..., duplicates skipped, Zipf(s_q) on [1,max_rank]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr int kGuideBits = 20;

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t h2(uint64_t s, uint64_t a) { return mix64(s + kGolden * (a + 1)); }
inline uint64_t h3(uint64_t s, uint64_t a, uint64_t b) { return mix64(h2(s, a) + kGolden * (b + 1)); }

struct Zipf {
  uint32_t V = 0;
  double total = 0;
  std::vector<double> cum;       // cum[i] = sum_{r=1..i+1} r^-s, sequential double adds
  std::vector<uint32_t> guide;   // guide[g] = #{i < V-1 : cum[i] <= ((g / 2^20) * total)}

  Zipf(uint32_t v, double s) : V(v), cum(v) {
    double acc = 0;
    for (uint32_t i = 0; i < v; ++i) {
      double w = (s == 1.0) ? 1.0 / (double)(i + 1) : std::pow((double)(i + 1), -s);
      acc += w;
      cum[i] = acc;
    }
    total = cum[v - 1];
    const uint32_t G = 1u << kGuideBits;
    guide.resize(G + 1);
    uint32_t c = 0;
    for (uint32_t g = 0; g <= G; ++g) {
      double x = ((double)g * (1.0 / (double)G)) * total;
      while (c < v - 1 && cum[c] <= x) ++c;
      guide[g] = c;
    }
  }
  // count of cum[0..V-2] <= u*total, + 1
  uint32_t rank(uint64_t h) const {
    double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
    double x = u * total;
    uint64_t g = h >> (64 - kGuideBits);
    uint32_t lo = guide[g], hi = guide[g + 1];
    // upper_bound over cum[lo, hi): first index with cum > x
    while (lo < hi) {
      uint32_t mid = lo + ((hi - lo) >> 1);
      if (cum[mid] <= x) lo = mid + 1; else hi = mid;
    }
    return lo + 1;
  }
};

template <class F>
void parallel_for(uint32_t n, int threads, F&& f) {
  if (threads <= 1 || n < 4096) { f(0u, n); return; }
  std::vector<std::thread> ts;
  uint32_t step = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    uint32_t b = t * step, e = b + step < n ? b + step : n;
    if (b >= e) break;
    ts.emplace_back([&f, b, e] { f(b, e); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

uint64_t fgs_mix64(uint64_t z) { return mix64(z); }
uint64_t fgs_h2(uint64_t s, uint64_t a) { return h2(s, a); }
uint64_t fgs_h3(uint64_t s, uint64_t a, uint64_t b) { return h3(s, a, b); }

void* fgs_zipf_new(uint32_t V, double s) {
  if (V < 1) return nullptr;
  return new Zipf(V, s);
}
void fgs_zipf_free(void* z) { delete static_cast<Zipf*>(z); }
uint32_t fgs_zipf_rank(const void* z, uint64_t h) { return static_cast<const Zipf*>(z)->rank(h); }

// Document lengths for docs [doc_begin, doc_begin+n) and the exclusive prefix
// offsets (doc_off[0] = 0, doc_off[n] = total tokens).  Returns the total.
uint64_t fgs_doc_lengths(uint64_t doc_begin, uint32_t n, uint64_t seed_L, uint32_t len_min,
                         uint32_t len_span, uint64_t* doc_off) {
  uint64_t acc = 0;
  for (uint32_t i = 0; i < n; ++i) {
    doc_off[i] = acc;
    acc += len_min + (uint32_t)(h2(seed_L, doc_begin + i) % len_span);
  }
  doc_off[n] = acc;
  return acc;
}

// Fill tok[] (size doc_off[n]) with term ids for docs [doc_begin, doc_begin+n).
int fgs_fill_tokens(uint64_t doc_begin, uint32_t n, const uint64_t* doc_off, uint32_t V, double s,
                    uint64_t seed_T, uint32_t* tok, int threads) {
  Zipf z(V, s);
  parallel_for(n, threads, [&](uint32_t b, uint32_t e) {
    for (uint32_t i = b; i < e; ++i) {
      uint64_t d = doc_begin + i;
      uint64_t hd = h2(seed_T, d);
      uint32_t len = (uint32_t)(doc_off[i + 1] - doc_off[i]);
      uint32_t* out = tok + doc_off[i];
      for (uint32_t j = 0; j < len; ++j) out[j] = z.rank(mix64(hd + kGolden * (j + 1))) - 1;
    }
  });
  return 0;
}

// Decimal digits of x at out (no terminator); returns the length.
inline int put_u64(char* out, uint64_t x) {
  char t[24];
  int n = 0;
  do { t[n++] = (char)('0' + x % 10); x /= 10; } while (x);
  for (int i = 0; i < n; ++i) out[i] = t[n - 1 - i];
  return n;
}

// Docs as text for the host mirror's ingest path: token id t is the word
// "t<t>" (lowercase alphanumeric: the "default" analyzer keeps it as one token),
// words joined by ' '.  out == NULL: only the byte total; else out receives the
// texts back to back and out_off[n+1] their offsets.
uint64_t fgs_render_text(const uint64_t* doc_off, const uint32_t* tok, uint32_t n, char* out, uint64_t* out_off,
                         int threads) {
  auto word_len = [](uint32_t t) {
    int l = 2;
    while (t >= 10) { t /= 10; ++l; }
    return l;  // 't' + digits
  };
  std::vector<uint64_t> len(n + 1, 0);
  parallel_for(n, threads, [&](uint32_t b, uint32_t e) {
    for (uint32_t i = b; i < e; ++i) {
      uint64_t l = 0;
      for (uint64_t p = doc_off[i]; p < doc_off[i + 1]; ++p) l += word_len(tok[p]) + (p + 1 < doc_off[i + 1] ? 1 : 0);
      len[i] = l;
    }
  });
  uint64_t pos = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t l = len[i];
    len[i] = pos;
    pos += l;
  }
  len[n] = pos;
  if (out_off) std::memcpy(out_off, len.data(), 8ull * (n + 1));
  if (out)
    parallel_for(n, threads, [&](uint32_t b, uint32_t e) {
      for (uint32_t i = b; i < e; ++i) {
        char* o = out + len[i];
        for (uint64_t p = doc_off[i]; p < doc_off[i + 1]; ++p) {
          *o++ = 't';
          o += put_u64(o, tok[p]);
          if (p + 1 < doc_off[i + 1]) *o++ = ' ';
        }
      }
    });
  return pos;
}

// Doc id strings "d<doc_begin + i>" for i < n, as fgs_render_text lays texts out.
uint64_t fgs_render_ids(uint64_t doc_begin, uint32_t n, char* out, uint64_t* out_off) {
  uint64_t pos = 0;
  char buf[24];
  for (uint32_t i = 0; i < n; ++i) {
    if (out_off) out_off[i] = pos;
    int len = 0;
    buf[len++] = 'd';
    len += put_u64(buf + len, doc_begin + i);
    if (out) std::memcpy(out + pos, buf, (size_t)len);
    pos += (uint64_t)len;
  }
  if (out_off) out_off[n] = pos;
  return pos;
}

// Query stream: q_off[n_queries+1], q_terms[n_queries*m_max] (term ids).
int fgs_queries(uint32_t n_queries, uint32_t m_min, uint32_t m_max, uint32_t max_rank, double s,
                uint64_t seed_Q, uint32_t* q_off, uint32_t* q_terms) {
  if (m_min < 1 || m_max < m_min || max_rank < m_max) return -1;
  Zipf z(max_rank, s);
  uint32_t pos = 0;
  for (uint32_t q = 0; q < n_queries; ++q) {
    q_off[q] = pos;
    uint32_t m = m_min + (uint32_t)(h2(seed_Q + 1, q) % (m_max - m_min + 1));
    uint32_t got = 0;
    for (uint64_t i = 0; got < m; ++i) {
      uint32_t t = z.rank(h3(seed_Q, q, i)) - 1;
      bool dup = false;
      for (uint32_t k = 0; k < got; ++k) dup |= (q_terms[pos + k] == t);
      if (!dup) q_terms[pos + got++] = t;
    }
    pos += m;
  }
  q_off[n_queries] = pos;
  return 0;
}

}  // extern "C"
