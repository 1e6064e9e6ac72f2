// Host side above the device ABI (include/fugu_host.h): fugu's Dataset /
// DatasetManager glue, the "default" analyzer, the QueryParser subset the
// device runs, and the perform_search response shapes.  C++ because the
// reference's Rust toolchain is absent.  Reference citations
// are on each function.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cctype>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fugu.h"
#include "../../include/fugu_host.h"
#include "fg_pool.h"
#include "fg_trace.h"

void fg_set_last_error(const std::string& msg);  // fugu.cpp
int fg_host_threads();                           // fugu.cpp: FUGU_THREADS / the process's CPU share

namespace {

#include "unicode_tables.inc"

int hfail(int code, const std::string& msg) {
  fg_set_last_error(msg);
  return code;
}

// ---------------------------------------------------------------- UTF-8
// Decode one code point at s[i]; invalid bytes decode as U+FFFD (Rust strings
// are valid UTF-8 by construction; this only keeps bad input from crashing).
uint32_t utf8_next(std::string_view s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  auto cont = [&](size_t k) { return i + k < s.size() && ((unsigned char)s[i + k] & 0xC0) == 0x80; };
  if (c < 0x80) { i += 1; return c; }
  if ((c >> 5) == 6 && cont(1)) {
    uint32_t cp = ((c & 0x1Fu) << 6) | ((unsigned char)s[i + 1] & 0x3Fu);
    i += 2;
    return cp;
  }
  if ((c >> 4) == 14 && cont(1) && cont(2)) {
    uint32_t cp = ((c & 0x0Fu) << 12) | (((unsigned char)s[i + 1] & 0x3Fu) << 6) | ((unsigned char)s[i + 2] & 0x3Fu);
    i += 3;
    return cp;
  }
  if ((c >> 3) == 30 && cont(1) && cont(2) && cont(3)) {
    uint32_t cp = ((c & 0x07u) << 18) | (((unsigned char)s[i + 1] & 0x3Fu) << 12) |
                  (((unsigned char)s[i + 2] & 0x3Fu) << 6) | ((unsigned char)s[i + 3] & 0x3Fu);
    i += 4;
    return cp;
  }
  i += 1;
  return 0xFFFD;
}

void utf8_put(std::string& out, uint32_t cp) {
  if (cp < 0x80) out.push_back((char)cp);
  else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// char::is_alphanumeric (Alphabetic || Numeric); tables: tools/gen_unicode_tables.py
bool is_alnum(uint32_t cp) {
  if (cp < 0x80) return (cp >= '0' && cp <= '9') || (cp >= 'a' && cp <= 'z') || (cp >= 'A' && cp <= 'Z');
  size_t lo = 0, hi = sizeof(kAlnumRanges) / sizeof(kAlnumRanges[0]);
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (kAlnumRanges[mid][1] < cp) lo = mid + 1; else hi = mid;
  }
  return lo < sizeof(kAlnumRanges) / sizeof(kAlnumRanges[0]) && kAlnumRanges[lo][0] <= cp;
}

// char::to_lowercase (one or two code points)
void lower_put(std::string& out, uint32_t cp) {
  if (cp < 0x80) { out.push_back((char)((cp >= 'A' && cp <= 'Z') ? cp + 32 : cp)); return; }
  size_t lo = 0, hi = sizeof(kLower) / sizeof(kLower[0]);
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (kLower[mid][0] < cp) lo = mid + 1; else hi = mid;
  }
  if (lo < sizeof(kLower) / sizeof(kLower[0]) && kLower[lo][0] == cp) {
    utf8_put(out, kLower[lo][2]);
    if (kLower[lo][1] > 1) utf8_put(out, kLower[lo][3]);
    return;
  }
  utf8_put(out, cp);
}

// The "default" analyzer of TEXT fields (src/db/schemas.rs:10,14):
// SimpleTokenizer (runs of char::is_alphanumeric) -> RemoveLongFilter::limit(40)
// (keeps tokens with < 40 UTF-8 bytes, measured before lowercasing) -> LowerCaser.
void analyze(std::string_view s, std::vector<std::string>& out) {
  out.clear();
  size_t i = 0;
  while (i < s.size()) {
    size_t start = i;
    uint32_t cp = utf8_next(s, i);
    if (!is_alnum(cp)) continue;
    size_t end = i;
    while (end < s.size()) {
      size_t j = end;
      uint32_t c2 = utf8_next(s, j);
      if (!is_alnum(c2)) break;
      end = j;
    }
    i = end;
    if (end - start >= 40) continue;  // RemoveLongFilter
    std::string tok;
    size_t k = start;
    while (k < end) lower_put(tok, utf8_next(s, k));
    out.push_back(std::move(tok));
  }
}

// analyze() for bulk ingest: f(token) for each token as a string_view into a
// scratch buffer (valid until the next call).  Pure-ASCII text takes a byte
// loop (runs of [0-9A-Za-z], < 40 bytes, lowercased): the same tokens as
// analyze(), whose Unicode path handles everything else.
template <class F>
void analyze_each(std::string_view s, std::string& scratch, std::vector<std::string>& toks, F&& f) {
  bool ascii = true;
  for (unsigned char c : s) ascii = ascii && c < 0x80;
  if (!ascii) {
    analyze(s, toks);
    for (auto& t : toks) f(std::string_view(t));
    return;
  }
  auto alnum = [](unsigned char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); };
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && !alnum((unsigned char)s[i])) ++i;
    const size_t b = i;
    while (i < s.size() && alnum((unsigned char)s[i])) ++i;
    if (i == b || i - b >= 40) continue;  // RemoveLongFilter
    scratch.assign(s.data() + b, i - b);
    for (char& c : scratch)
      if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
    f(std::string_view(scratch));
  }
}

// A thread's term dictionary during bulk ingest: open addressing over an
// arena of the term bytes (no allocation per lookup).
struct LocalDict {
  std::string arena;
  std::vector<std::pair<uint64_t, uint32_t>> ent;  // (arena offset << 8 | length, hash low bits)
  std::vector<uint32_t> slot{std::vector<uint32_t>(1u << 16, 0)};  // entry + 1, 0 = empty
  static uint64_t hash(std::string_view w) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ w.size();
    for (unsigned char c : w) h = (h ^ c) * 0x100000001B3ull;
    return h ^ (h >> 29);
  }
  std::string_view key(uint32_t e) const { return std::string_view(arena.data() + (ent[e].first >> 8), ent[e].first & 0xFF); }
  uint32_t get(std::string_view w) {
    if (2 * (ent.size() + 1) > slot.size()) grow();
    const uint64_t h = hash(w);
    for (size_t m = slot.size() - 1, i = h & m;; i = (i + 1) & m) {
      if (!slot[i]) {
        ent.emplace_back(((uint64_t)arena.size() << 8) | w.size(), (uint32_t)h);
        arena.append(w.data(), w.size());
        slot[i] = (uint32_t)ent.size();
        return (uint32_t)ent.size() - 1;
      }
      const uint32_t e = slot[i] - 1;
      if (ent[e].second == (uint32_t)h && key(e) == w) return e;
    }
  }
  void grow() {
    std::vector<uint32_t> ns(slot.size() * 2, 0);
    for (uint32_t e = 0; e < ent.size(); ++e)
      for (size_t m = ns.size() - 1, i = hash(key(e)) & m;; i = (i + 1) & m)
        if (!ns[i]) { ns[i] = e + 1; break; }
    slot.swap(ns);
  }
};

// Storage that never moves once published: a directory of atomic pointers to
// chunks of GEOMETRIC sizes (chunk c holds 2^c << kFirstShift slots), so a small
// namespace costs a few KB and a large one still a few dozen chunks (ADVICE r05:
// fixed 2^18-entry directories and 4 MiB first chunks cost ~12 MiB per namespace).
// One writer appends; readers index any slot published before they looked
// (acquire on the chunk pointer) without a lock.
template <class T, uint32_t kFirstShift>
class ChunkDir {
  static constexpr uint32_t kMaxChunks = 48;
  std::atomic<T*> dir_[kMaxChunks] = {};
  std::vector<std::unique_ptr<T[]>> own_;  // writer side

 public:
  // chunk of slot i and i's offset in it: chunk c covers [(2^c - 1) << s, (2^(c+1) - 1) << s)
  static void locate(size_t i, uint32_t& c, size_t& o) {
    const size_t x = (i >> kFirstShift) + 1;
    c = 63u - (uint32_t)__builtin_clzll(x);
    o = i - (((size_t(1) << c) - 1) << kFirstShift);
  }
  static size_t chunk_begin(uint32_t c) { return ((size_t(1) << c) - 1) << kFirstShift; }
  static size_t chunk_size(uint32_t c) { return size_t(1) << (c + kFirstShift); }
  T& at(size_t i) const {
    uint32_t c;
    size_t o;
    locate(i, c, o);
    return dir_[c].load(std::memory_order_acquire)[o];
  }
  // the writer: slot i, its chunk allocated (and published) first if new
  T& slot(size_t i) {
    uint32_t c;
    size_t o;
    locate(i, c, o);
    if (c >= kMaxChunks) throw std::length_error("ChunkDir full");
    T* p = dir_[c].load(std::memory_order_relaxed);
    if (!p) {
      own_.emplace_back(new T[chunk_size(c)]());
      p = own_.back().get();
      dir_[c].store(p, std::memory_order_release);
    }
    return p[o];
  }
};

// A namespace's term dictionary (term -> id, ids in insertion order) whose
// lookups take no lock: the query path never waits on the IndexWriter, as in
// the reference (the searcher of each query reads committed segments,
// src/db/search.rs:86-87, while writers serialise on their own mutex,
// src/db/core.rs:211).  One writer (under Namespace::writer) inserts.  Term
// bytes and entries live in chunks that never move; the open-addressing table
// (hash's high half beside id + 1, one slot line per probe) is published by one
// release store per slot after the entry and bytes it points at, and replaced
// whole when it grows (old tables are kept: a reader may still probe one, and
// they add up to less than the current table).  A reader that finds no slot for
// a term interned after it looked reports it missing, which it also is in every
// snapshot the reader can hold.  (A node-based map chased two or three pointers
// per lookup; a 1000-doc upsert looks up ~20K distinct words in a dictionary of
// 10^6 terms.)
struct TermDict {
  static constexpr uint32_t kMissing = 0xFFFFFFFFu;
  static constexpr size_t kMaxKey = (1u << 20) - 1;  // bytes per term (tokens are < 40, facet paths short)
  struct Table {
    std::unique_ptr<std::atomic<uint64_t>[]> s;
    size_t mask;
    explicit Table(size_t n) : s(new std::atomic<uint64_t>[n]()), mask(n - 1) {}
  };
  // entry of id: byte offset of the term in the arena << 20 | length (a term
  // never straddles two arena chunks)
  ChunkDir<uint64_t, 10> ent;
  ChunkDir<char, 14> arena;
  size_t a_pos = 0;  // writer: where the next term's bytes go
  std::atomic<uint32_t> n{0};
  std::atomic<Table*> cur;
  std::vector<std::unique_ptr<Table>> tables;  // writer: current and retired
  TermDict() {
    tables.emplace_back(new Table(1u << 10));
    cur.store(tables.back().get(), std::memory_order_release);
  }
  uint32_t size() const { return n.load(std::memory_order_acquire); }
  static uint64_t hash(std::string_view w) { return LocalDict::hash(w); }
  std::string_view key(uint32_t id) const {
    const uint64_t e = ent.at(id);
    return std::string_view(&arena.at(e >> 20), e & kMaxKey);
  }
  void prefetch(uint64_t h) const {
    const Table* t = cur.load(std::memory_order_relaxed);
    __builtin_prefetch(&t->s[h & t->mask]);
  }
  uint32_t find(std::string_view w, uint64_t h) const {
    const Table* t = cur.load(std::memory_order_acquire);
    for (size_t i = h & t->mask;; i = (i + 1) & t->mask) {
      const uint64_t x = t->s[i].load(std::memory_order_acquire);
      if (!x) return kMissing;
      if ((x >> 32) == (h >> 32) && key((uint32_t)x - 1) == w) return (uint32_t)x - 1;
    }
  }
  uint32_t find(std::string_view w) const { return find(w, hash(w)); }
  static void put(Table& t, uint64_t h, uint32_t id) {
    for (size_t i = h & t.mask;; i = (i + 1) & t.mask)
      if (!t.s[i].load(std::memory_order_relaxed)) {
        t.s[i].store(((h >> 32) << 32) | (id + 1ull), std::memory_order_release);
        return;
      }
  }
  uint32_t get(std::string_view w, uint64_t h) {  // the writer: find, else insert with the next id
    const uint32_t f = find(w, h);
    if (f != kMissing) return f;
    if (w.size() > kMaxKey) throw std::length_error("term longer than 1 MiB");
    const uint32_t id = n.load(std::memory_order_relaxed);
    if (2 * (size_t(id) + 1) > cur.load(std::memory_order_relaxed)->mask + 1) grow();
    for (;;) {  // the term's bytes inside one chunk: skip to the next chunk start until they fit
      uint32_t c;
      size_t o;
      decltype(arena)::locate(a_pos, c, o);
      if (w.empty() || o + w.size() <= decltype(arena)::chunk_size(c)) break;
      a_pos = decltype(arena)::chunk_begin(c + 1);
    }
    char* dst = &arena.slot(a_pos);  // publishes the chunk when new
    if (!w.empty()) std::memcpy(dst, w.data(), w.size());
    ent.slot(id) = ((uint64_t)a_pos << 20) | w.size();
    a_pos += w.size();
    n.store(id + 1, std::memory_order_release);
    put(*cur.load(std::memory_order_relaxed), h, id);
    return id;
  }
  uint32_t get(std::string_view w) { return get(w, hash(w)); }
  void grow() {
    const Table* old = cur.load(std::memory_order_relaxed);
    auto t = std::make_unique<Table>((old->mask + 1) * 2);
    const uint32_t nn = n.load(std::memory_order_relaxed);
    for (uint32_t id = 0; id < nn; ++id) put(*t, hash(key(id)), id);
    cur.store(t.get(), std::memory_order_release);
    tables.push_back(std::move(t));
  }
};

// A namespace's docs by global id (insertion order): appended by the writer,
// read by searches' doc fetch without a lock (chunks never move; a search only
// reads docs of a committed snapshot, all appended before it was published).
// Only `deleted`, which the read path never touches, changes after an append.
template <class Doc>
class DocStore {
  ChunkDir<Doc, 8> c_;
  std::atomic<size_t> n_{0};

 public:
  size_t size() const { return n_.load(std::memory_order_acquire); }
  const Doc& operator[](size_t i) const { return c_.at(i); }
  Doc& operator[](size_t i) { return c_.at(i); }  // the writer
  void push_back(Doc&& d) {
    const size_t i = n_.load(std::memory_order_relaxed);
    c_.slot(i) = std::move(d);
    n_.store(i + 1, std::memory_order_release);
  }
};

// ---------------------------------------------------------------- query parser subset
// QueryParser::for_index(index, [text, name]).parse_query (src/db/search.rs:108-127)
// restricted to what the device runs (tantivy-query-grammar 0.24: the default
// conjunction is Should, `+` Must, `-` MustNot, binary AND / OR):
//   `t1 t2 -t3 +t4 ...`   each term's occur by its prefix (bare = Should)
//   `t1 AND t2 AND ...`   every term Must
//   `t1 OR t2 OR ...`     every term Should (the same query as `t1 t2 ...`)
// Every term must analyze to exactly one token (more = PhraseQuery).  Anything
// else (mixed AND / OR, parentheses, field:, phrases, boosts, ranges, a query
// of MustNot clauses only) is FG_EUNSUPPORTED: the reference host runs tantivy.
// An empty query is AllQuery (src/db/search.rs:115-116), handled by the caller.
bool is_special(char c) {
  switch (c) {
    case '+': case '-': case '(': case ')': case '[': case ']': case '{': case '}': case '"': case ':':
    case '^': case '~': case '*': case '?': case '\\': case '!': case '\'': case '`': case '<': case '>':
    case '=':
      return true;
    default:
      return false;
  }
}

int parse_query(std::string_view q, std::vector<std::string>& terms, std::vector<uint8_t>& occur, std::string& why) {
  terms.clear();
  occur.clear();
  std::vector<std::string_view> words;
  size_t i = 0;
  while (i < q.size()) {
    while (i < q.size() && (q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r')) ++i;
    size_t s = i;
    while (i < q.size() && !(q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r')) ++i;
    if (i > s) words.push_back(q.substr(s, i - s));
  }
  if (words.empty()) { why = "empty query (AllQuery)"; return FG_EUNSUPPORTED; }
  std::vector<std::pair<std::string_view, uint8_t>> raw;
  auto binary_form = [&](std::string_view op) {
    bool ok = words.size() >= 3 && words.size() % 2 == 1;
    for (size_t w = 1; ok && w < words.size(); w += 2) ok = words[w] == op;
    return ok;
  };
  if (binary_form("AND") || binary_form("OR")) {
    const uint8_t oc = words[1] == "AND" ? FG_OCCUR_MUST : FG_OCCUR_SHOULD;
    for (size_t w = 0; w < words.size(); w += 2) raw.emplace_back(words[w], oc);
  } else {
    for (auto w : words) {
      if (w.size() > 1 && (w[0] == '+' || w[0] == '-'))
        raw.emplace_back(w.substr(1), w[0] == '+' ? FG_OCCUR_MUST : FG_OCCUR_MUST_NOT);
      else
        raw.emplace_back(w, FG_OCCUR_SHOULD);
    }
  }
  bool positive = false;
  for (auto& [w, oc] : raw) {
    if (w == "AND" || w == "OR" || w == "NOT" || w == "IN" || w == "TO") {
      why = "operator outside the supported forms";
      return FG_EUNSUPPORTED;
    }
    for (char c : w)
      if (is_special(c)) {
        why = "query syntax beyond bare/+/-/AND/OR terms";
        return FG_EUNSUPPORTED;
      }
    std::vector<std::string> toks;
    analyze(w, toks);
    if (toks.size() != 1) {
      why = toks.empty() ? "a term analyzes to no token" : "a term analyzes to several tokens (PhraseQuery)";
      return FG_EUNSUPPORTED;
    }
    terms.push_back(std::move(toks[0]));
    occur.push_back(oc);
    positive |= oc != FG_OCCUR_MUST_NOT;
  }
  if (!positive) {
    why = "MustNot clauses only";
    return FG_EUNSUPPORTED;
  }
  return FG_OK;
}

// FG_MODE_AND / FG_MODE_OR when every clause is Must / Should, else FG_MODE_MIXED
int mode_of(const std::vector<uint8_t>& occur) {
  bool all_m = true, all_s = true;
  for (uint8_t o : occur) {
    all_m = all_m && o == FG_OCCUR_MUST;
    all_s = all_s && o == FG_OCCUR_SHOULD;
  }
  return occur.size() == 1 ? FG_MODE_AND : all_m ? FG_MODE_AND : all_s ? FG_MODE_OR : FG_MODE_MIXED;
}

// ---------------------------------------------------------------- JSON helpers
void json_str(std::string& o, std::string_view s) {
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

// serde_json writes an f32 with the shortest digits that round-trip as f32
// (ryu), keeping a ".0" on integral values.
void json_f32(std::string& o, float v) {
  char b[48];
  for (int p = 1; p <= 9; ++p) {
    snprintf(b, sizeof b, "%.*g", p, (double)v);
    if (strtof(b, nullptr) == v) break;
  }
  std::string s(b);
  if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
  o += s;
}

int copy_out(const std::string& s, char* out, size_t cap, size_t* len) {
  if (len) *len = s.size();
  if (!out) return FG_OK;
  if (cap < s.size() + 1) return hfail(FG_EINVAL, "output buffer too small");
  std::memcpy(out, s.data(), s.size());
  out[s.size()] = 0;
  return FG_OK;
}

// ---------------------------------------------------------------- JSON (metadata)
// ObjectRecord.metadata is Option<HashMap<String, serde_json::Value>>
// (src/object.rs:11): enough of a JSON reader to walk it.  Object members keep
// their input order (Rust's HashMap order is unspecified).
struct JVal {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;                                    // Bool
  std::string num;                                   // Num: the literal
  std::string str;                                   // Str
  std::vector<JVal> arr;                             // Arr
  std::vector<std::pair<std::string, JVal>> obj;     // Obj
};

struct JParser {
  std::string_view s;
  size_t i = 0;
  int depth = 0;
  void ws() { while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i; }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s.substr(i, n) != w) return false;
    i += n;
    return true;
  }
  bool hex4(uint32_t& v) {
    if (i + 4 > s.size()) return false;
    v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return false;
    }
    return true;
  }
  bool string(std::string& out) {
    if (i >= s.size() || s[i] != '"') return false;
    ++i;
    out.clear();
    while (i < s.size()) {
      char c = s[i++];
      if (c == '"') return true;
      if ((unsigned char)c < 0x20) return false;
      if (c != '\\') { out.push_back(c); continue; }
      if (i >= s.size()) return false;
      char e = s[i++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {
            uint32_t lo;
            if (!(lit("\\u") && hex4(lo) && lo >= 0xDC00 && lo < 0xE000)) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            return false;
          }
          utf8_put(out, cp);
          break;
        }
        default: return false;
      }
    }
    return false;
  }
  bool value(JVal& v) {
    if (++depth > 128) return false;
    ws();
    bool ok = false;
    if (i >= s.size()) ok = false;
    else if (s[i] == '{') {
      v.kind = JVal::Obj;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') { ++i; ok = true; }
      else
        for (;;) {
          ws();
          std::string k;
          JVal x;
          if (!string(k)) break;
          ws();
          if (i >= s.size() || s[i] != ':') break;
          ++i;
          if (!value(x)) break;
          // serde_json into a HashMap: a repeated key keeps the last value
          auto it = std::find_if(v.obj.begin(), v.obj.end(), [&](auto& m) { return m.first == k; });
          if (it != v.obj.end()) it->second = std::move(x); else v.obj.emplace_back(std::move(k), std::move(x));
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == '}') { ++i; ok = true; }
          break;
        }
    } else if (s[i] == '[') {
      v.kind = JVal::Arr;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') { ++i; ok = true; }
      else
        for (;;) {
          JVal x;
          if (!value(x)) break;
          v.arr.push_back(std::move(x));
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == ']') { ++i; ok = true; }
          break;
        }
    } else if (s[i] == '"') {
      v.kind = JVal::Str;
      ok = string(v.str);
    } else if (lit("null")) { v.kind = JVal::Null; ok = true; }
    else if (lit("true")) { v.kind = JVal::Bool; v.b = true; ok = true; }
    else if (lit("false")) { v.kind = JVal::Bool; v.b = false; ok = true; }
    else {
      size_t b = i;
      if (i < s.size() && s[i] == '-') ++i;
      while (i < s.size() && (std::isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                              s[i] == '+' || s[i] == '-'))
        ++i;
      v.kind = JVal::Num;
      v.num.assign(s.substr(b, i - b));
      ok = i > b && std::isdigit((unsigned char)s[i - 1]);
    }
    --depth;
    return ok;
  }
};

bool parse_json(std::string_view text, JVal& out) {
  JParser p{text};
  if (!p.value(out)) return false;
  p.ws();
  return p.i == text.size();
}

// serde_json's f64 output (ryu's shortest round-trip digits, ryu's layout:
// 1e16 -> "1e16", 1e15 -> "1000000000000000.0", 1e-5 -> "1e-5", 1e-4 -> "0.0001").
void json_f64(std::string& o, double v) {
  if (v == 0.0) { o += std::signbit(v) ? "-0.0" : "0.0"; return; }
  char b[48];
  int p = 1;
  for (; p <= 17; ++p) {
    snprintf(b, sizeof b, "%.*e", p - 1, v);
    if (strtod(b, nullptr) == v) break;
  }
  std::string m(b);
  const size_t epos = m.find('e');
  const int e10 = atoi(m.c_str() + epos + 1);
  std::string digits;
  for (size_t i = 0; i < epos; ++i)
    if (std::isdigit((unsigned char)m[i])) digits.push_back(m[i]);
  if (v < 0) o.push_back('-');
  const int len = (int)digits.size(), kk = e10 + 1, k = kk - len;
  if (k >= 0 && kk <= 16) {
    o += digits;
    o.append((size_t)k, '0');
    o += ".0";
  } else if (kk > 0 && kk <= 16) {
    o += digits.substr(0, (size_t)kk) + "." + digits.substr((size_t)kk);
  } else if (kk > -5 && kk <= 0) {
    o += "0.";
    o.append((size_t)-kk, '0');
    o += digits;
  } else {
    o += digits.substr(0, 1);
    if (len > 1) o += "." + digits.substr(1);
    o += "e" + std::to_string(kk - 1);
  }
}

// A number as serde_json re-serializes it (no arbitrary_precision): an integer
// literal that fits u64 (or i64 when negative) stays an integer, "-0" and
// everything else become f64.
void json_num(std::string& o, const std::string& lit) {
  const bool intlike = lit.find_first_of(".eE") == std::string::npos;
  if (intlike) {
    errno = 0;
    if (lit[0] != '-') {
      const unsigned long long u = strtoull(lit.c_str(), nullptr, 10);
      if (errno == 0) { o += std::to_string(u); return; }
    } else {
      const long long x = strtoll(lit.c_str(), nullptr, 10);
      if (errno == 0 && x != 0) { o += std::to_string(x); return; }
    }
  }
  json_f64(o, strtod(lit.c_str(), nullptr));
}

// serde_json::Value serialization: without the preserve_order feature (the
// reference's Cargo.lock builds serde_json 1.0.140 without indexmap) an object
// is a BTreeMap, so its keys come out in byte order.
void json_dump(std::string& o, const JVal& v) {
  switch (v.kind) {
    case JVal::Null: o += "null"; break;
    case JVal::Bool: o += v.b ? "true" : "false"; break;
    case JVal::Num: json_num(o, v.num); break;
    case JVal::Str: json_str(o, v.str); break;
    case JVal::Arr:
      o.push_back('[');
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) o.push_back(',');
        json_dump(o, v.arr[i]);
      }
      o.push_back(']');
      break;
    case JVal::Obj: {
      std::vector<const std::pair<std::string, JVal>*> m;
      for (auto& kv : v.obj) m.push_back(&kv);
      std::sort(m.begin(), m.end(), [](auto* a, auto* b) { return a->first < b->first; });
      o.push_back('{');
      for (size_t i = 0; i < m.size(); ++i) {
        if (i) o.push_back(',');
        json_str(o, m[i]->first);
        o.push_back(':');
        json_dump(o, m[i]->second);
      }
      o.push_back('}');
      break;
    }
  }
}

// ---------------------------------------------------------------- facets
// Facet::from_text (tantivy schema/facet.rs): the path must start with '/';
// '/' separates segments, stored as U+0000; '\' escapes the next char.
bool facet_from_text(std::string_view path, std::string& enc) {
  enc.clear();
  if (path.empty() || path[0] != '/') return false;
  bool escaped = false;
  size_t last = 1;
  for (size_t i = 1; i < path.size(); ++i) {
    const char c = path[i];
    if (escaped) {
      escaped = false;
    } else if (c == '\\') {
      enc.append(path.substr(last, i - last));
      last = i + 1;
      escaped = true;
    } else if (c == '/') {
      enc.append(path.substr(last, i - last));
      enc.push_back('\0');
      last = i + 1;
    }
  }
  enc.append(path.substr(last));
  return true;
}

// FacetTokenizer (tokenizer/facet_tokenizer.rs): the root (empty), every
// prefix ending before a separator after position 0, then the whole facet.
void facet_tokens(const std::string& enc, std::vector<std::string>& out) {
  out.clear();
  out.emplace_back();
  if (enc.empty()) return;
  size_t cur = 0;
  for (;;) {
    const size_t nxt = enc.find('\0', cur + 1);
    if (nxt == std::string::npos) {
      out.push_back(enc);
      return;
    }
    out.push_back(enc.substr(0, nxt));
    cur = nxt;
  }
}

// Facet's Display: '/' + segment per segment, '/' inside a segment as "\/"
// (convert_doc_to_search_result, src/db/search.rs:563-578)
std::string facet_display(const std::string& enc) {
  std::string o;
  size_t b = 0;
  for (;;) {
    const size_t e = enc.find('\0', b);
    o.push_back('/');
    for (char c : enc.substr(b, e == std::string::npos ? std::string::npos : e - b)) {
      if (c == '/') o.push_back('\\');
      o.push_back(c);
    }
    if (e == std::string::npos) return o;
    b = e + 1;
  }
}

std::string normalize_facet_path(std::string_view p) {  // src/db/search.rs:594-600
  return !p.empty() && p[0] == '/' ? std::string(p) : "/" + std::string(p);
}

// create_metadata_facets (src/db/utils.rs:11-56): one facet per non-empty
// string leaf, carrying only the top-level key (get_all_facet_paths takes
// facet_path.first(), src/db/document.rs:297-306)
void string_leaves(const JVal& v, size_t& n) {
  switch (v.kind) {
    case JVal::Obj: for (auto& m : v.obj) string_leaves(m.second, n); break;
    case JVal::Arr: for (auto& x : v.arr) string_leaves(x, n); break;
    case JVal::Str: n += v.str.empty() ? 0 : 1; break;
    default: break;
  }
}

// ---------------------------------------------------------------- datasets
struct Doc {
  std::string id, text, name, metadata;
  bool has_name = false;
  bool deleted = false;
  std::vector<uint32_t> text_tok, name_tok;
  std::vector<std::string> id_tokens;
  std::vector<std::string> facets;   // stored facet values, encoded (Facet), in document order
  std::vector<uint32_t> facet_tok;   // FacetTokenizer tokens of all of them (facet dictionary ids)
};

// One segment's share of the namespace statistics: tantivy's Searcher sums
// max_doc, total_num_tokens and doc_freq over the segments (deleted docs
// included until a merge drops them).  doc_freq as (term, count) pairs.
struct SegStats {
  uint64_t n = 0, tot[2] = {0, 0}, tot_f = 0;
  std::vector<std::pair<uint32_t, uint32_t>> df_t, df_n, df_f;
};

// A committed view of a namespace: tantivy's segments, one per commit
// (src/db/document.rs:65), in global doc order; the background merger
// (tantivy's merge threads, IndexWriter at src/db/core.rs:247-249) replaces
// contiguous runs of small segments by one.  Every segment scores with the
// namespace-wide statistics.
struct Segment {
  fg_index* ix = nullptr;
  uint32_t base = 0, n = 0;  // global doc ids [base, base + n) ...
  std::shared_ptr<const std::vector<uint32_t>> gid;  // ... or, for a merged segment, gid[local doc]
  uint64_t id = 0;                                   // stable across rescores (the merger finds its sources)
  std::shared_ptr<const SegStats> st;
  uint32_t global(uint32_t d) const { return gid ? (*gid)[d] : base + d; }
};
struct Snapshot {
  std::vector<Segment> segs;
  ~Snapshot() {
    for (auto& s : segs)
      if (s.ix) fg_index_release(s.ix);
  }
};
constexpr size_t kHardSegments = 48;  // a commit that would pass this many segments waits for a merge first

struct Namespace {
  std::string name;
  std::mutex writer;                                   // IndexWriter lock (src/db/core.rs:211)
  std::mutex committer;                                // serialises commits and merge swaps (snapshot order)
  std::mutex merging;                                  // one merge of this namespace at a time
  // global doc id = insertion order; chunked: appending never moves the ~250 B
  // Doc records (a vector's reallocation moved all 10M of them inside a commit),
  // and searches read them without the writer lock
  DocStore<Doc> docs;
  std::vector<uint8_t> del;                            // del[d] == docs[d].deleted (commits copy this, not the docs)
  // docs deleted by upserts since the last commit, in order: a delete takes
  // effect at the commit (IndexWriter::delete_term), so a merge in between
  // neither drops them nor flags them (committed_del)
  std::vector<uint32_t> pend_del;
  bool any_name = false;                               // some doc has a name field
  TermDict dict;                                       // term dictionary (text and name tokens)
  TermDict fdict;                                      // facet dictionary (encoded facet terms), same rules
  std::unordered_map<std::string, std::vector<uint32_t>> by_id_token;
  std::shared_ptr<Snapshot> snap;                      // committed device snapshot
  std::shared_mutex snap_mu;
  size_t committed_docs = 0;
  uint64_t next_seg = 1;
  // BM25 statistics of the committed segments (the sum of their SegStats),
  // deleted docs included: N, token totals, doc frequencies.  Written under the
  // writer AND committer locks together with the snapshot (so a committer reads
  // them without the writer lock); st_ver counts the changes.
  uint64_t st_n = 0, st_tot[2] = {0, 0}, st_tot_f = 0, st_ver = 0;
  std::vector<uint32_t> st_df_text, st_df_name, st_df_facet;
  // merger bookkeeping
  std::mutex mq;
  std::condition_variable mq_cv;
  bool queued = false, running = false;
  uint64_t merges = 0, merged_docs = 0;
  double merge_ms_total = 0, merge_ms_last = 0, merge_ms_max = 0;
  std::string merge_error;
};

}  // namespace

struct fg_db {
  fg_ctx* ctx = nullptr;
  int dev = 0;
  std::string default_ns;
  std::map<std::string, std::shared_ptr<Namespace>> ns;
  std::shared_mutex mu;
  // the background merger: one thread per db working through queued namespaces
  std::thread merger;
  std::mutex mq;
  std::condition_variable mq_cv;
  std::deque<std::weak_ptr<Namespace>> queue;
  bool stop = false;
  // Every snapshot is destroyed on the reaper thread, whoever drops its last
  // reference (new_snapshot's deleter): destroying one releases its segments'
  // scoring blocks, which waits for the device to drain (fgh::ScorePool), and
  // that must hold up neither the commit or merge that replaced it nor a search
  // that still held it when the swap came.
  std::thread reaper;
  std::mutex rq;
  std::condition_variable rq_cv;
  std::deque<Snapshot*> dead;
  bool rstop = false;
  void reap(Snapshot* p) {
    {
      std::lock_guard<std::mutex> l(rq);
      if (!rstop) {
        dead.push_back(p);
        if (!reaper.joinable())
          reaper = std::thread([this] {
            for (;;) {
              Snapshot* x = nullptr;
              {
                std::unique_lock<std::mutex> l2(rq);
                rq_cv.wait(l2, [&] { return rstop || !dead.empty(); });
                if (dead.empty()) return;  // stopping, drained
                x = dead.front();
                dead.pop_front();
              }
              delete x;
            }
          });
        rq_cv.notify_one();
        return;
      }
    }
    delete p;  // the db is being destroyed: its reaper has stopped
  }
  std::shared_ptr<Snapshot> new_snapshot() {
    return std::shared_ptr<Snapshot>(new Snapshot, [this](Snapshot* p) { reap(p); });
  }
  void retire(std::shared_ptr<Snapshot> s) { s.reset(); }  // the reaper destroys it once unreferenced
  ~fg_db() {
    {
      std::lock_guard<std::mutex> l(mq);
      stop = true;
    }
    mq_cv.notify_all();
    if (merger.joinable()) merger.join();
    {
      // the namespaces (and their snapshots) go while the reaper still runs
      std::map<std::string, std::shared_ptr<Namespace>> gone;
      {
        std::unique_lock<std::shared_mutex> l(mu);
        gone.swap(ns);
      }
    }
    {
      std::lock_guard<std::mutex> l(rq);
      rstop = true;
    }
    rq_cv.notify_all();
    if (reaper.joinable()) reaper.join();
  }
};

namespace {

std::shared_ptr<Namespace> find_ns(fg_db* db, const char* name) {
  std::shared_lock<std::shared_mutex> l(db->mu);
  auto it = db->ns.find(name ? name : db->default_ns);
  return it == db->ns.end() ? nullptr : it->second;
}

// validate_config's namespace-name rule (src/db/config.rs:302-315)
bool valid_ns_name(std::string_view n) {
  if (n.empty()) return false;
  for (char c : n)
    if (std::strchr("/\\:*?\"<>|", c)) return false;
  return true;
}

std::vector<uint32_t> intern(Namespace& ns, std::string_view text) {
  std::vector<std::string> toks;
  analyze(text, toks);
  std::vector<uint32_t> ids;
  ids.reserve(toks.size());
  for (auto& t : toks) ids.push_back(ns.dict.get(t));
  return ids;
}

// build_facet_query's clause list (src/db/search.rs:221-324) for the filters
// Dataset::search keeps (:98-103: not both starting and ending with '*'):
// parse_filters normalizes a path with a leading '/', "<path>/*" is a Prefix,
// "<key>=<value>" an Equals on <key> (the value is dropped), anything else an
// Equals.  Clauses: Facet::from_text of every Equals path (exact terms, one
// Should group), then of every Prefix path (one Should TermQuery each).
// *all_query: the filters are non-empty but no clause parsed (facet_query =
// AllQuery).  Returns whether facet filtering applies at all.
bool facet_clauses(const std::vector<std::string>& filters, std::vector<std::string>& clauses, bool* all_query) {
  clauses.clear();
  *all_query = false;
  std::vector<std::string> keep;
  for (auto& f : filters)
    if (!(!f.empty() && f.front() == '*' && f.back() == '*')) keep.push_back(f);
  if (keep.empty()) return false;
  std::vector<std::string> exact, prefix;
  for (auto& f : keep) {
    const std::string n = normalize_facet_path(f);
    std::string path;
    bool is_prefix = false;
    if (n.size() >= 2 && n.compare(n.size() - 2, 2, "/*") == 0) {
      path = n.substr(0, n.size() - 2);
      is_prefix = true;
    } else if (n.find('=') != std::string::npos) {
      path = n.substr(0, n.find('='));
    } else {
      path = n;
    }
    std::string enc;
    if (!facet_from_text(path, enc)) continue;  // `if let Ok(facet) = Facet::from_text(..)`
    (is_prefix ? prefix : exact).push_back(std::move(enc));
  }
  clauses = exact;
  clauses.insert(clauses.end(), prefix.begin(), prefix.end());
  *all_query = clauses.empty();
  return true;
}

bool blank(std::string_view q) {
  for (char c : q)
    if (!(c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v')) return false;
  return true;
}

// Dataset::search core: hits of the page in order, or an error code.
int search_hits(fg_db* db, Namespace& ns, const char* query, const std::vector<std::string>& filters, uint32_t page,
                uint32_t per_page, std::vector<fg_hit>& hits) {
  (void)db;
  hits.clear();
  fgh::SearchTrace& trace = fgh::search_trace();
  const uint64_t t_in = trace.enabled() ? fgh::now_ns() : 0;
  struct TotalOut {
    fgh::SearchTrace& t; uint64_t t0;
    ~TotalOut() {
      if (!t0) return;
      t.add(fgh::kPhTotal, fgh::now_ns() - t0);
      t.calls.fetch_add(1, std::memory_order_relaxed);
    }
  } total_out{trace, t_in};
  if (per_page == 0) return hfail(FG_EINVAL, "TopDocs::with_limit requires limit >= 1");
  const std::string_view qv = query ? query : "";
  std::vector<std::string> terms;
  std::vector<uint8_t> occur;
  std::string why;
  const bool empty_text = blank(qv);  // query.trim().is_empty() -> AllQuery (src/db/search.rs:115-116)
  if (!empty_text) {
    int rc = parse_query(qv, terms, occur, why);
    if (rc) return hfail(rc, "query outside the device subset: " + why);
  }
  std::vector<std::string> clauses;
  bool facet_all = false;
  const bool filtered = facet_clauses(filters, clauses, &facet_all);
  if (filtered && facet_all && !empty_text)
    return hfail(FG_EUNSUPPORTED, "query outside the device subset: text query AND an AllQuery facet filter");
  const uint64_t offset = (uint64_t)page * per_page, limit = offset + per_page;
  if (limit > FG_MAX_K) return hfail(FG_EUNSUPPORTED, "offset + per_page > FG_MAX_K");
  std::shared_ptr<Snapshot> snap;
  std::vector<uint32_t> ids, fids;
  {
    std::shared_lock<std::shared_mutex> l(ns.snap_mu);
    snap = ns.snap;
  }
  // no lock: term ids are stable once interned, and ids interned after the
  // snapshot are >= its n_terms (they match nothing there) -- a commit's gather,
  // an upsert's dictionary merge or a merge never holds up a search
  for (auto& t : terms) {
    const uint32_t id = ns.dict.find(t);
    ids.push_back(id == TermDict::kMissing ? FG_TERM_MISSING : id);
  }
  for (auto& c : clauses) {
    const uint32_t id = ns.fdict.find(c);
    fids.push_back(id == TermDict::kMissing ? FG_TERM_MISSING : id);
  }
  if (!snap) return FG_OK;  // nothing committed yet: no hits
  // every segment answers the query (TopDocs::with_limit(offset + per_page) per
  // segment), then merge_fruits on the device: (score desc, segment asc, doc
  // asc) = (score desc, global doc asc), since segments hold ascending doc-id
  // ranges.  Terms interned after a segment was built (ids >= its n_terms)
  // match nothing there.
  std::vector<fg_index*> segs;
  for (const Segment& seg : snap->segs) segs.push_back(seg.ix);
  const uint32_t q_off[2] = {0, (uint32_t)ids.size()};
  const uint32_t f_off[2] = {0, (uint32_t)fids.size()};
  fg_query_batch qb{1, q_off, ids.data(), FG_MODE_AND, fids.empty() ? nullptr : f_off, fids.data(), occur.data()};
  std::vector<float> sc(limit);
  std::vector<uint32_t> dc(limit), sh(limit);
  uint32_t n = 0;
  if (t_in) trace.add(fgh::kPhParse, fgh::now_ns() - t_in);
  int rc = fg_search_sharded(nullptr, segs.data(), (uint32_t)segs.size(), &qb, (uint32_t)limit, sc.data(), dc.data(),
                             sh.data(), &n);
  if (rc) return hfail(rc, fg_last_error());
  for (uint64_t i = offset; i < n; ++i)  // skip(offset).take(per_page)
    hits.push_back(fg_hit{sc[i], snap->segs[sh[i]].global(dc[i])});
  return FG_OK;
}

std::vector<std::string> filter_list(const char* const* filters, uint32_t n) {
  std::vector<std::string> v;
  for (uint32_t i = 0; i < n; ++i) v.emplace_back(filters && filters[i] ? filters[i] : "");
  return v;
}

// urlencoding::decode: %XX escapes become bytes (a malformed escape stays as
// it is); the result must be UTF-8, else "Invalid URL encoding in query"
bool url_decode(std::string& q) {
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  std::string o;
  for (size_t i = 0; i < q.size(); ++i) {
    if (q[i] == '%' && i + 2 < q.size() && hex(q[i + 1]) >= 0 && hex(q[i + 2]) >= 0) {
      o.push_back((char)(hex(q[i + 1]) * 16 + hex(q[i + 2])));
      i += 2;
    } else {
      o.push_back(q[i]);
    }
  }
  // UTF-8 validation (Rust String::from_utf8)
  for (size_t i = 0; i < o.size();) {
    const unsigned char c = (unsigned char)o[i];
    size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (!n || i + n > o.size()) return false;
    uint32_t cp = n == 1 ? c : c & (0x7F >> n);
    for (size_t k = 1; k < n; ++k) {
      const unsigned char x = (unsigned char)o[i + k];
      if ((x >> 6) != 2) return false;
      cp = (cp << 6) | (x & 0x3F);
    }
    if ((n == 2 && cp < 0x80) || (n == 3 && cp < 0x800) || (n == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
        (cp >= 0xD800 && cp < 0xE000))
      return false;
    i += n;
  }
  q.swap(o);
  return true;
}

// The POST /search/json additions (src/server/handlers/search.rs:273-285).
struct JsonExtras {
  bool include_data = true, targeting = false;
  std::string developer_message;  // empty: absent
};

// perform_search + the handlers' JSON (src/server/handlers/search.rs).  Every
// response is a serde_json Value, so object keys come out in byte order
// (BTreeMap: serde_json is built without preserve_order, Cargo.lock:4313-4322).
//   post_search   search_endpoint (POST /search, :152-207): no per_page clamp,
//                 text kept, {filters, page, per_page, query, results, status, total}
//   otherwise     perform_search (:350-402) shapes {page, per_page, query, results,
//                 total} (+ the POST /search/json extras), text stripped unless asked
int search_json(fg_db* db, const char* nsname, const std::string& q, const std::vector<std::string>& fl,
                uint32_t page, uint32_t per_page, bool include_text, bool post_search, const JsonExtras* ex,
                char* out, size_t cap, size_t* len) {
  auto ns = find_ns(db, nsname);
  const std::string nsn = nsname ? nsname : "";
  if (!ns) {
    std::string o;
    if (post_search && !nsname) {
      o = "{\"error\":\"Default dataset not found\",\"status\":\"error\"}";
    } else if (post_search) {
      // POST /search/{namespace} (CLI contract cli.rs:352-355): the POST shape, scoped
      o = "{\"error\":";
      json_str(o, "Namespace '" + nsn + "' not found");
      o += ",\"status\":\"error\"}";
    } else {
      o = "{\"error\":";
      json_str(o, "Search failed: Namespace '" + nsn + "' not found");
      o += "}";
    }
    copy_out(o, out, cap, len);
    return hfail(FG_ENOTFOUND, "Namespace '" + nsn + "' not found");
  }
  if (!post_search && (per_page == 0 || per_page > 100)) per_page = 20;
  std::vector<fg_hit> hits;
  int rc = search_hits(db, *ns, q.c_str(), fl, page, per_page, hits);
  fgh::SearchTrace& trace = fgh::search_trace();
  struct FetchOut {
    fgh::SearchTrace& t; uint64_t t0;
    ~FetchOut() { if (t0) t.add(fgh::kPhFetch, fgh::now_ns() - t0); }
  } fetch_out{trace, trace.enabled() ? fgh::now_ns() : 0};
  if (rc) {
    // perform_search wraps Dataset::search's error once, its handler again
    std::string o = "{\"error\":";
    json_str(o, std::string(post_search ? "Search failed: " : "Search failed: Search failed: ") + fg_last_error());
    o += post_search ? ",\"status\":\"error\"}" : "}";
    copy_out(o, out, cap, len);
    return rc;
  }
  const bool with_text = post_search || include_text;
  std::string res = "[";
  {
    // the stored fields of committed docs never change: no lock (searcher.doc
    // reads the committed segments' doc stores, src/db/search.rs:172-211)
    const DocStore<Doc>& docs = ns->docs;
    for (size_t i = 0; i < hits.size(); ++i) {
      const Doc& d = docs[hits[i].doc];
      if (i) res.push_back(',');
      // FuguSearchResult {id, score, text, metadata, facets} (src/db/search.rs:20-27, 534-590) as a Value
      res += "{\"facets\":";
      if (d.facets.empty()) {
        res += "null";
      } else {
        res.push_back('[');
        for (size_t j = 0; j < d.facets.size(); ++j) {
          if (j) res.push_back(',');
          json_str(res, facet_display(d.facets[j]));
        }
        res.push_back(']');
      }
      res += ",\"id\":";
      json_str(res, d.id);
      res += ",\"metadata\":";
      res += d.metadata.empty() ? "null" : d.metadata;
      res += ",\"score\":";
      json_f32(res, hits[i].score);
      if (with_text) {
        res += ",\"text\":";
        json_str(res, d.text);
      }
      res += "}";
    }
  }
  res += "]";
  std::string o = "{";
  char num[64];
  if (post_search) {
    o += "\"filters\":[";
    for (size_t j = 0; j < fl.size(); ++j) {
      if (j) o.push_back(',');
      json_str(o, fl[j]);
    }
    o += "],";
  }
  if (ex) {
    if (!ex->developer_message.empty()) {
      o += "\"developer_message\":";
      json_str(o, ex->developer_message);
      o += ",";
    }
    o += ex->include_data ? "\"includes_data_objects\":true," : "\"includes_data_objects\":false,";
  }
  snprintf(num, sizeof num, "\"page\":%u,\"per_page\":%u,\"query\":", page, per_page);
  o += num;
  json_str(o, q);
  o += ",\"results\":" + res;
  if (post_search) o += ",\"status\":\"success\"";
  if (ex) o += ex->targeting ? ",\"targeting_conversations_or_organizations\":true"
                             : ",\"targeting_conversations_or_organizations\":false";
  snprintf(num, sizeof num, ",\"total\":%zu}", hits.size());
  o += num;
  return copy_out(o, out, cap, len);
}

}  // namespace

extern "C" {

int fg_db_create(fg_ctx* ctx, int dev, const char* default_namespace, fg_db** out) {
  if (!out) return hfail(FG_EINVAL, "bad arguments");
  auto db = std::make_unique<fg_db>();
  db->ctx = ctx;
  db->dev = dev;
  db->default_ns = default_namespace && *default_namespace ? default_namespace : "fugu_db";  // main.rs:118-121
  auto ns = std::make_shared<Namespace>();
  ns->name = db->default_ns;
  db->ns.emplace(db->default_ns, ns);
  *out = db.release();
  return FG_OK;
}

int fg_db_destroy(fg_db* db) {
  delete db;
  return FG_OK;
}

int fg_db_namespace_create(fg_db* db, const char* name) {
  if (!db || !name) return hfail(FG_EINVAL, "bad arguments");
  if (!valid_ns_name(name)) return hfail(FG_EINVAL, std::string("Invalid characters in namespace name: ") + name);
  std::unique_lock<std::shared_mutex> l(db->mu);
  if (db->ns.count(name)) return hfail(FG_EEXIST, std::string("Namespace '") + name + "' already exists");
  auto ns = std::make_shared<Namespace>();
  ns->name = name;
  db->ns.emplace(name, ns);
  return FG_OK;
}

int fg_db_namespace_delete(fg_db* db, const char* name) {
  if (!db || !name) return hfail(FG_EINVAL, "bad arguments");
  std::unique_lock<std::shared_mutex> l(db->mu);
  if (!db->ns.erase(name)) return hfail(FG_ENOTFOUND, std::string("Namespace '") + name + "' not found");
  return FG_OK;  // in-flight searches keep the namespace's snapshot alive (shared_ptr)
}

int fg_db_namespaces_json(fg_db* db, char* out, size_t cap, size_t* len) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  // json!({"status", "namespaces"}) is a serde_json Value: keys in byte order
  std::string o = "{\"namespaces\":[";
  {
    std::shared_lock<std::shared_mutex> l(db->mu);
    bool first = true;
    for (auto& kv : db->ns) {
      if (!first) o.push_back(',');
      first = false;
      json_str(o, kv.first);
    }
  }
  o += "],\"status\":\"success\"}";
  return copy_out(o, out, cap, len);
}

}  // extern "C"

namespace {

std::vector<uint32_t> intern_facet(Namespace& ns, const std::vector<std::string>& enc) {
  std::vector<uint32_t> ids;
  std::vector<std::string> toks;
  for (auto& e : enc) {
    facet_tokens(e, toks);
    for (auto& t : toks) ids.push_back(ns.fdict.get(t));
  }
  return ids;
}

// NamedIndex::upsert of one ObjectRecord into the docs index
// (src/db/document.rs:23-67, build_full_document :116-184).  name_override:
// the legacy fg_db_upsert entry passes the `name` value directly.
int upsert_record(fg_db* db, const char* nsname, const fg_object_record* r, const char* name_override,
                  bool legacy) {
  if (!db || !r) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  // ObjectRecord::validate (src/object.rs:31-78)
  const std::string sid = r->id ? r->id : "", stext = r->text ? r->text : "";
  if (sid.empty()) return hfail(FG_EINVAL, "Object ID cannot be empty");
  if (sid.size() > 256) return hfail(FG_EINVAL, "Object ID too long (max 256 characters)");
  if (stext.empty()) return hfail(FG_EINVAL, "Object text cannot be empty");
  if (stext.size() > 10000) return hfail(FG_EINVAL, "Text too long (max 10000 characters)");
  const char* rns = legacy ? nsname : r->namespace_;
  if (rns) {
    std::string_view n(rns);
    if (n.empty() || n.find('/') != std::string_view::npos || n.find(' ') != std::string_view::npos)
      return hfail(FG_EINVAL, "Invalid namespace format");
    if (n.size() > 128) return hfail(FG_EINVAL, "Namespace too long (max 128 characters)");
  }
  if (r->has_facets) {
    if (r->n_facets > 100) return hfail(FG_EINVAL, "Too many facets (max 100 per object)");
    for (uint32_t i = 0; i < r->n_facets; ++i) {
      const size_t len = r->facets[i] ? std::strlen(r->facets[i]) : 0;
      if (!len) return hfail(FG_EINVAL, "Facet at index " + std::to_string(i) + " cannot be empty");
      if (len > 512) return hfail(FG_EINVAL, "Facet at index " + std::to_string(i) + " too long (max 512 characters)");
    }
  }
  JVal meta;
  const bool has_meta = r->metadata_json != nullptr;
  if (has_meta && (!parse_json(r->metadata_json, meta) || meta.kind != JVal::Obj))
    return hfail(FG_EINVAL, "metadata must be a JSON object");
  Doc doc;
  doc.id = sid;
  doc.text = stext;
  if (has_meta) json_dump(doc.metadata, meta);  // what the reference returns: serde_json::from_str(stored) re-serialized
  if (name_override) {
    doc.has_name = true;
    doc.name = name_override;
  } else if (has_meta) {
    // metadata["name"] when it is a string (build_full_document, document.rs:131-139)
    for (auto& m : meta.obj)
      if (m.first == "name" && m.second.kind == JVal::Str) { doc.has_name = true; doc.name = m.second.str; }
  }
  // get_all_facet_paths (document.rs:277-309): explicit facets, else the
  // namespace facets (object.rs:81-111) then the metadata facets
  std::vector<std::string> paths;
  if (r->has_facets) {
    for (uint32_t i = 0; i < r->n_facets; ++i) paths.push_back(normalize_facet_path(r->facets[i]));
  } else {
    if (r->namespace_ && !legacy) {
      const std::string base = std::string("/namespace/") + r->namespace_;
      paths.push_back(base);
      if (r->organization) paths.push_back(base + "/organization/" + r->organization);
      if (r->conversation_id) paths.push_back(base + "/conversation/" + r->conversation_id);
      if (r->data_type) paths.push_back(base + "/data/" + r->data_type);
    }
    if (has_meta)
      for (auto& m : meta.obj) {
        size_t n = 0;
        string_leaves(m.second, n);
        const std::string path = !m.first.empty() && m.first[0] == '/' ? m.first : "/metadata/" + m.first;
        for (size_t j = 0; j < n; ++j) paths.push_back(path);
      }
  }
  for (auto& pth : paths) {
    std::string enc;
    if (facet_from_text(pth, enc)) doc.facets.push_back(std::move(enc));  // add_facets_to_document skips failures
  }
  for (auto& e : doc.facets)  // (a facet token is a prefix of its path)
    if (e.size() > TermDict::kMaxKey) return hfail(FG_EINVAL, "facet path longer than 1 MiB");
  std::lock_guard<std::mutex> w(ns->writer);
  // w.delete_term(Term::from_field_text(id_field, &object.id)) (src/db/document.rs:38-42): the
  // RAW id is matched against the tokens of the tokenized `id` field, so ids with
  // uppercase or punctuation never match and are not replaced
  auto it = ns->by_id_token.find(sid);
  if (it != ns->by_id_token.end())
    for (uint32_t d : it->second) {
      if (!ns->del[d]) ns->pend_del.push_back(d);
      ns->docs[d].deleted = true;
      ns->del[d] = 1;
    }
  doc.text_tok = intern(*ns, doc.text);
  if (doc.has_name) doc.name_tok = intern(*ns, doc.name);
  doc.facet_tok = intern_facet(*ns, doc.facets);
  analyze(doc.id, doc.id_tokens);
  const uint32_t d = (uint32_t)ns->docs.size();
  for (auto& t : doc.id_tokens) ns->by_id_token[t].push_back(d);
  ns->any_name |= !doc.name_tok.empty();
  ns->del.push_back(0);
  ns->docs.push_back(std::move(doc));
  return FG_OK;
}

// ---------------------------------------------------------------- commits and merges
// FUGU_COMMIT_TRACE=1: per-phase wall time of upserts, commits and merges on stderr
struct PhaseTrace {
  const char* what;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit PhaseTrace(const char* w)
      : what(w), on(getenv("FUGU_COMMIT_TRACE") != nullptr), t(std::chrono::steady_clock::now()) {}
  void mark(const char* phase) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    // @: the phase's end on the steady clock (ms; Python's time.monotonic)
    fprintf(stderr, "[fg %s] %-28s %9.2f ms @%.3f\n", what, phase, std::chrono::duration<double, std::milli>(n - t).count(),
            std::chrono::duration<double, std::milli>(n.time_since_epoch()).count());
    t = n;
  }
};

// FIELD_NORMS_TABLE (fieldnorm/code.rs): 0..40 exactly, then groups of 8 with a
// doubling step; a length is stored as the largest entry <= it.
uint64_t quantized_len(uint64_t n) {
  static const std::vector<uint64_t> t = [] {
    std::vector<uint64_t> v;
    for (uint64_t i = 0; i <= 40; ++i) v.push_back(i);
    uint64_t x = 40, step = 2;
    while (v.size() < 256) {
      for (int j = 0; j < 8 && v.size() < 256; ++j) v.push_back(x += step);
      step <<= 1;
    }
    return v;
  }();
  return *(std::upper_bound(t.begin(), t.end(), n) - 1);
}

// (term, docs holding it) of a few docs' field, sparse: each doc's distinct
// terms gathered, then sorted and counted (a commit's 1000 docs: no
// vocabulary-sized arrays)
struct SparseDf {
  std::vector<uint32_t> all, scratch;
  void add(const std::vector<uint32_t>& toks) {
    scratch = toks;
    std::sort(scratch.begin(), scratch.end());
    scratch.erase(std::unique(scratch.begin(), scratch.end()), scratch.end());
    all.insert(all.end(), scratch.begin(), scratch.end());
  }
  std::vector<std::pair<uint32_t, uint32_t>> take() {
    std::sort(all.begin(), all.end());
    std::vector<std::pair<uint32_t, uint32_t>> v;
    for (size_t i = 0; i < all.size();) {
      size_t j = i;
      while (j < all.size() && all[j] == all[i]) ++j;
      v.emplace_back(all[i], (uint32_t)(j - i));
      i = j;
    }
    return v;
  }
};

// the distinct terms of a doc counted once into df
void count_distinct(const std::vector<uint32_t>& toks, std::vector<uint32_t>& scratch, std::vector<uint32_t>& df) {
  scratch = toks;
  std::sort(scratch.begin(), scratch.end());
  scratch.erase(std::unique(scratch.begin(), scratch.end()), scratch.end());
  for (uint32_t t : scratch) df[t]++;
}

std::vector<std::pair<uint32_t, uint32_t>> sparse_of(const std::vector<uint32_t>& df) {
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (uint32_t t = 0; t < df.size(); ++t)
    if (df[t]) v.emplace_back(t, df[t]);
  return v;
}

void df_add(std::vector<uint32_t>& df, const std::vector<std::pair<uint32_t, uint32_t>>& sp, bool sub) {
  for (auto& e : sp) {
    if (e.first >= df.size()) df.resize(e.first + 1, 0);
    df[e.first] = sub ? df[e.first] - e.second : df[e.first] + e.second;
  }
}

// Runs f(0..n-1) on up to `width` threads (this one and the helper pool's).
template <class F>
void run_threads(size_t n, size_t width, F&& f) {
  fgh::parallel_dynamic((uint32_t)n, (int)width, 1, [&](int, uint32_t b, uint32_t e) {
    for (uint32_t i = b; i < e; ++i) f(i);
  });
}

// Dense namespace statistics in local copies (fg_global_stats points into them).
struct Stats {
  uint64_t n = 0, tot[2] = {0, 0}, tot_f = 0;
  std::vector<uint32_t> df_t, df_n, df_f;
  void load(const Namespace& ns, uint32_t n_terms, uint32_t n_fterms) {
    n = ns.st_n;
    tot[0] = ns.st_tot[0];
    tot[1] = ns.st_tot[1];
    tot_f = ns.st_tot_f;
    // the vocabulary-sized arrays copied in 1 MiB pieces on the pool (~12 MB per commit)
    auto copy = [](std::vector<uint32_t>& dst, const std::vector<uint32_t>& src, uint32_t size) {
      dst.assign(size, 0);
      const size_t m = std::min<size_t>(size, src.size()), piece = 1u << 18;
      run_threads((m + piece - 1) / piece, 8, [&](size_t i) {
        const size_t b = i * piece, e = std::min(m, b + piece);
        std::memcpy(dst.data() + b, src.data() + b, 4 * (e - b));
      });
    };
    copy(df_t, ns.st_df_text, std::max<uint32_t>(n_terms, (uint32_t)ns.st_df_text.size()));
    copy(df_n, ns.st_df_name, std::max<uint32_t>(n_terms, (uint32_t)ns.st_df_name.size()));
    copy(df_f, ns.st_df_facet, std::max<uint32_t>(n_fterms, (uint32_t)ns.st_df_facet.size()));
  }
  void add(const SegStats& s, bool sub) {
    n = sub ? n - s.n : n + s.n;
    tot[0] = sub ? tot[0] - s.tot[0] : tot[0] + s.tot[0];
    tot[1] = sub ? tot[1] - s.tot[1] : tot[1] + s.tot[1];
    tot_f = sub ? tot_f - s.tot_f : tot_f + s.tot_f;
    df_add(df_t, s.df_t, sub);
    df_add(df_n, s.df_n, sub);
    df_add(df_f, s.df_f, sub);
  }
  fg_global_stats global() const {
    fg_global_stats g{};
    g.n_docs = n;
    g.tot_tokens[0] = tot[0];
    g.tot_tokens[1] = tot[1];
    g.df_text = df_t.data();
    g.df_name = df_n.data();
    g.df_facet = df_f.empty() ? nullptr : df_f.data();
    g.tot_facet_tokens = tot_f;
    return g;
  }
  void store(Namespace& ns) {  // under the writer and committer locks; the arrays move (S is spent)
    ns.st_n = n;
    ns.st_tot[0] = tot[0];
    ns.st_tot[1] = tot[1];
    ns.st_tot_f = tot_f;
    ns.st_df_text = std::move(df_t);
    ns.st_df_name = std::move(df_n);
    ns.st_df_facet = std::move(df_f);
    ns.st_ver++;
  }
};

// The docs `ids` (global, in order) as fg_docs_input arrays
struct DocsBuf {
  std::vector<uint64_t> toff{0}, noff{0}, foff{0};
  std::vector<uint32_t> ttok, ntok, ftok;
  std::vector<uint8_t> del;
  bool any_name = false, any_del = false;
  void add(const Doc& d, bool deleted) {
    ttok.insert(ttok.end(), d.text_tok.begin(), d.text_tok.end());
    ntok.insert(ntok.end(), d.name_tok.begin(), d.name_tok.end());
    ftok.insert(ftok.end(), d.facet_tok.begin(), d.facet_tok.end());
    toff.push_back(ttok.size());
    noff.push_back(ntok.size());
    foff.push_back(ftok.size());
    any_name |= !d.name_tok.empty();
    del.push_back(deleted ? 1 : 0);
    any_del |= deleted;
  }
  fg_docs_input input(uint32_t n_terms, uint32_t n_fterms, bool with_name) const {
    fg_docs_input in{};
    in.n_docs = (uint32_t)del.size();
    in.n_terms = n_terms;
    in.text_off = toff.data();
    in.text_tok = ttok.data();
    in.name_off = with_name ? noff.data() : nullptr;
    in.name_tok = with_name ? ntok.data() : nullptr;
    in.deleted = any_del ? del.data() : nullptr;
    in.threads = 0;
    in.keep_host_postings = 0;
    in.n_facet_terms = n_fterms;
    in.facet_off = n_fterms ? foff.data() : nullptr;
    in.facet_tok = n_fterms ? ftok.data() : nullptr;
    return in;
  }
};

// every segment of `segs` rescored with g and the current deleted flags
// (`del`, global); appended to out in order.  One fg_index_rescore_many: the
// weights once, the segments side by side on their own threads and streams.
// Returns an error code (out then owns nothing new).
int rescore_into(const std::vector<Segment>& segs, const fg_global_stats& g, const std::vector<uint8_t>& del,
                 std::vector<Segment>& out) {
  const size_t n = segs.size();
  std::vector<std::vector<uint8_t>> sdel(n);
  std::vector<const uint8_t*> dp(n, nullptr);
  std::vector<const fg_index*> bases(n);
  run_threads(n, 8, [&](size_t i) {
    const Segment& s0 = segs[i];
    bases[i] = s0.ix;
    // (a contiguous segment without deleted docs: one memchr)
    if (!s0.gid && !std::memchr(del.data() + s0.base, 1, s0.n)) return;
    sdel[i].assign(s0.n, 0);
    bool sany = false;
    for (uint32_t d = 0; d < s0.n; ++d) sany |= (sdel[i][d] = del[s0.global(d)]) != 0;
    dp[i] = sany ? sdel[i].data() : nullptr;
  });
  std::vector<fg_index*> re(n, nullptr);
  if (int rc = fg_index_rescore_many(bases.data(), (uint32_t)n, &g, dp.data(), re.data())) return hfail(rc, fg_last_error());
  for (size_t i = 0; i < n; ++i) {
    Segment x = segs[i];
    x.ix = re[i];
    out.push_back(std::move(x));
  }
  return FG_OK;
}

// A commit: the docs since the last one as a new segment (the first commit:
// every doc, deleted ones included), the older segments rescored with the new
// statistics.  The statistics and the snapshot change together, only when
// every step succeeded.
int commit_segment(fg_db* db, Namespace& ns) {
  PhaseTrace tr("commit");
  std::lock_guard<std::mutex> c(ns.committer);
  std::shared_ptr<Snapshot> cur;
  {
    std::shared_lock<std::shared_mutex> l(ns.snap_mu);
    cur = ns.snap;
  }
  // gather under the writer lock, build outside it so searches (doc fetch) and
  // upserts are not blocked by the device work
  std::unique_lock<std::mutex> w(ns.writer);
  const uint32_t N = (uint32_t)ns.docs.size();
  const uint32_t old = cur ? (uint32_t)ns.committed_docs : 0;
  if (N == 0 || (N == old && cur)) return FG_OK;
  const uint32_t n_terms = std::max<uint32_t>(1, (uint32_t)ns.dict.size());
  const uint32_t n_fterms = (uint32_t)ns.fdict.size();
  DocsBuf buf;
  auto st = std::make_shared<SegStats>();
  SparseDf dt, dn, dfc;
  for (uint32_t d = old; d < N; ++d) {
    const Doc& doc = ns.docs[d];
    buf.add(doc, doc.deleted);
    st->n++;
    st->tot[0] += doc.text_tok.size();
    st->tot[1] += doc.name_tok.size();
    st->tot_f += doc.facet_tok.size();
    dt.add(doc.text_tok);
    dn.add(doc.name_tok);
    dfc.add(doc.facet_tok);
  }
  const bool any_name = ns.any_name;
  const std::vector<uint8_t> del(ns.del.begin(), ns.del.begin() + N);
  const size_t n_pend = ns.pend_del.size();  // committed by this commit
  w.unlock();
  tr.mark("gather (writer lock)");
  st->df_t = dt.take();
  st->df_n = dn.take();
  st->df_f = dfc.take();
  // the statistics change only under the committer lock (held): read without the writer's
  Stats S;
  S.load(ns, n_terms, n_fterms);
  S.add(*st, false);
  tr.mark("statistics");
  const fg_global_stats g = S.global();
  const fg_docs_input in = buf.input(n_terms, n_fterms, any_name);
  auto snap = db->new_snapshot();
  // the new segment builds while the older ones rescore (their own threads and streams)
  fg_index* ix = nullptr;
  int brc = FG_OK;
  std::string berr;
  std::thread builder([&] {
    fg_thread_background(1);
    if (const char* f = getenv("FUGU_FAULT_INJECT"))  // tests only: a commit whose device build fails
      if (std::strcmp(f, "commit_build") == 0) {
        brc = FG_EHIP;
        berr = "injected fault: segment build";
        return;
      }
    if ((brc = fg_index_build_from_docs_global(db->ctx, db->dev, &in, &g, &ix))) berr = fg_last_error();
  });
  const int rrc = cur ? rescore_into(cur->segs, g, del, snap->segs) : FG_OK;  // snap releases the rescored ones
  const std::string rerr = rrc ? fg_last_error() : std::string();
  tr.mark("rescore older (beside the build)");
  builder.join();
  tr.mark("build new (rest)");
  if (rrc || brc) {
    if (ix) fg_index_release(ix);
    return rrc ? hfail(rrc, rerr) : hfail(brc, berr);
  }
  std::shared_ptr<Snapshot> prev;  // released after the locks (its blocks wait for the device to drain)
  {
    std::lock_guard<std::mutex> w2(ns.writer);  // the statistics are read under the writer lock
    snap->segs.push_back(Segment{ix, old, N - old, nullptr, ns.next_seg++, st});
    std::unique_lock<std::shared_mutex> l(ns.snap_mu);  // readers keep the old snapshot (refcount)
    prev = std::move(ns.snap);
    ns.snap = snap;
    ns.committed_docs = N;
    ns.pend_del.erase(ns.pend_del.begin(), ns.pend_del.begin() + n_pend);
    S.store(ns);
  }
  cur.reset();
  db->retire(std::move(prev));
  tr.mark("swap");
  return FG_OK;
}

// The merge policy: tantivy 0.24.1's LogMergePolicy with its defaults
// (indexer/log_merge_policy.rs): segments of more than max_docs_before_merge
// docs are left alone; the others, largest first, form levels -- a segment
// starts a new level when log2 of its size (clipped up to min_layer_size docs,
// so every small segment shares the smallest level) is below the current
// level's first by more than level_log_size -- and a level of at least
// min_num_segments segments is merged.  Kept contiguous here: the merged
// segment must keep global doc order (merge_fruits' (segment, doc) tie order),
// so a level merges as its contiguous runs of >= kMergeFactor segments (the
// newest such run first).  Levels that interleave in doc order could then
// stall, so past kBoundSegments segments the kMergeFactor contiguous mergeable
// segments with the fewest docs merge; from kHardSegments on (every segment
// past the cap) the two newest.  Returns [j0, j1) or j0 == j1 (nothing).
constexpr size_t kMergeFactor = 8;             // min_num_segments
constexpr uint64_t kMinLayerSize = 10000;      // min_layer_size
constexpr double kLevelLogSize = 0.75;         // level_log_size
constexpr uint64_t kMaxDocsBeforeMerge = 10000000;  // max_docs_before_merge
constexpr size_t kBoundSegments = 3 * kMergeFactor;
// FUGU_MERGE_MAX_DOCS: LogMergePolicy::set_max_docs_before_merge (bench.py holds
// its 8-segment namespace at 2^20 so the segmented search path stays measured)
uint64_t merge_max_docs() {
  const char* e = getenv("FUGU_MERGE_MAX_DOCS");
  return e && *e ? std::strtoull(e, nullptr, 10) : kMaxDocsBeforeMerge;
}
// level of every segment (-1: too large to merge), levels numbered from the largest
std::vector<int> merge_levels(const std::vector<uint64_t>& n, uint64_t max_docs) {
  std::vector<size_t> by;
  for (size_t i = 0; i < n.size(); ++i)
    if (n[i] <= max_docs) by.push_back(i);
  std::stable_sort(by.begin(), by.end(), [&](size_t a, size_t b) { return n[a] > n[b]; });
  std::vector<int> lev(n.size(), -1);
  double cur = std::numeric_limits<double>::max();
  int l = -1;
  for (size_t i : by) {
    const double ls = std::log2((double)std::max(n[i], kMinLayerSize));
    if (ls < cur - kLevelLogSize) {
      cur = ls;
      ++l;
    }
    lev[i] = l;
  }
  return lev;
}
std::pair<size_t, size_t> pick_merge(const std::vector<uint64_t>& n) {
  const size_t c = n.size();
  const std::vector<int> lev = merge_levels(n, merge_max_docs());
  for (size_t j1 = c; j1 > 0;) {  // contiguous runs of one level, newest first
    size_t j0 = j1 - 1;
    while (j0 > 0 && lev[j0 - 1] == lev[j1 - 1]) --j0;
    if (lev[j1 - 1] >= 0 && j1 - j0 >= kMergeFactor) return {j0, j1};
    j1 = j0;
  }
  if (c > kBoundSegments) {
    size_t best = c;
    uint64_t best_docs = ~0ull;
    for (size_t j = 0; j + kMergeFactor <= c; ++j) {
      uint64_t t = 0;
      bool ok = true;
      for (size_t i = j; i < j + kMergeFactor && ok; ++i) {
        ok = lev[i] >= 0;
        t += n[i];
      }
      if (ok && t < best_docs) {
        best_docs = t;
        best = j;
      }
    }
    if (best < c) return {best, best + kMergeFactor};
  }
  if (c >= kHardSegments) return {c - 2, c};
  return {c, c};
}

// One merge of a run of segments into one, as a tantivy merge does it: the
// deleted docs are dropped (N and doc_freq then count the alive docs), and the
// merged total_num_tokens is, per source segment, its own total when it has no
// deletes, else the sum over its alive docs of their quantized field lengths
// (FIELD_NORMS_TABLE[fieldnorm_id]; a field without fieldnorms -- the facet
// field -- counts 1 per alive doc) (merger.rs compute_total_num_tokens).
// The merged segment is built outside the locks; the swap re-checks what
// commits did meanwhile (new statistics, new deletions) and rescores.
int merge_once(fg_db* db, Namespace& ns, bool* did) {
  *did = false;
  PhaseTrace tr("merge");
  std::lock_guard<std::mutex> mg(ns.merging);
  const auto t0 = std::chrono::steady_clock::now();
  std::shared_ptr<Snapshot> cur;
  {
    std::shared_lock<std::shared_mutex> l(ns.snap_mu);
    cur = ns.snap;
  }
  if (!cur) return FG_OK;
  std::vector<uint64_t> sizes;
  for (auto& sg : cur->segs) sizes.push_back(sg.n);
  const auto run = pick_merge(sizes);
  if (run.first >= run.second) return FG_OK;
  const std::vector<Segment> src(cur->segs.begin() + run.first, cur->segs.begin() + run.second);
  // ---- gather the run's alive docs and the merged statistics
  DocsBuf buf;
  auto mst = std::make_shared<SegStats>();
  std::vector<uint32_t> ids;
  Stats S;
  uint64_t ver0 = 0;
  uint32_t n_terms = 0, n_fterms = 0;
  bool any_name = false;
  // under the writer lock only what upserts change (the deletion flags, the
  // statistics); the docs' tokens are read after it (appended docs never change
  // but for `deleted`), so upserts and commits go on while a large merge gathers
  std::vector<uint8_t> del0;
  {
    std::lock_guard<std::mutex> w(ns.writer);
    n_terms = std::max<uint32_t>(1, (uint32_t)ns.dict.size());
    n_fterms = (uint32_t)ns.fdict.size();
    del0 = ns.del;
    for (uint32_t g : ns.pend_del) del0[g] = 0;  // committed deletions only
    any_name = ns.any_name;
    S.load(ns, n_terms, n_fterms);
    ver0 = ns.st_ver;
  }
  tr.mark("gather (writer lock)");
  {
    std::vector<uint32_t> dt(n_terms, 0), dn(n_terms, 0), dfc(n_fterms, 0), scratch;
    for (const Segment& sg : src) {
      bool has_del = false;
      for (uint32_t d = 0; d < sg.n && !has_del; ++d) has_del = del0[sg.global(d)] != 0;
      if (!has_del) {
        mst->tot[0] += sg.st->tot[0];
        mst->tot[1] += sg.st->tot[1];
        mst->tot_f += sg.st->tot_f;
      }
      for (uint32_t d = 0; d < sg.n; ++d) {
        const uint32_t gd = sg.global(d);
        if (del0[gd]) continue;
        const Doc& doc = ns.docs[gd];
        ids.push_back(gd);
        buf.add(doc, false);
        mst->n++;
        if (has_del) {
          mst->tot[0] += quantized_len(doc.text_tok.size());
          mst->tot[1] += quantized_len(doc.name_tok.size());
          mst->tot_f += 1;
        }
        count_distinct(doc.text_tok, scratch, dt);
        count_distinct(doc.name_tok, scratch, dn);
        count_distinct(doc.facet_tok, scratch, dfc);
      }
    }
    mst->df_t = sparse_of(dt);
    mst->df_n = sparse_of(dn);
    mst->df_f = sparse_of(dfc);
    for (const Segment& sg : src) S.add(*sg.st, true);
    S.add(*mst, false);
  }
  tr.mark("gather docs");
  fg_index* mix = nullptr;
  if (!ids.empty()) {
    const fg_global_stats g = S.global();
    const fg_docs_input in = buf.input(n_terms, n_fterms, any_name);
    if (int rc = fg_index_build_from_docs_global(db->ctx, db->dev, &in, &g, &mix)) return hfail(rc, fg_last_error());
  }
  if (const char* e = getenv("FUGU_MERGE_DELAY_MS"))  // tests only: searches run while the merge is in flight
    std::this_thread::sleep_for(std::chrono::milliseconds(atoi(e)));
  tr.mark("build merged segment");
  // ---- the merged segment brought to the statistics and deletions of this
  // moment OUTSIDE the committer lock (commits go on meanwhile); under the lock
  // it is rescored again only if another commit slipped in
  uint64_t src_n = 0;
  for (const Segment& sg : src) src_n += sg.n;
  const bool stats_change = ids.size() != src_n;  // deleted docs dropped (their N, df and tokens go)
  uint64_t ver_used = ver0;
  std::vector<uint8_t> mdel_used(ids.size(), 0);
  auto refresh = [&](uint64_t& ver, std::vector<uint8_t>& md) {  // under the writer lock
    ver = ns.st_ver;
    if (ver != ver0) {
      const uint32_t nt = std::max<uint32_t>(1, (uint32_t)ns.dict.size()), nf = (uint32_t)ns.fdict.size();
      S = Stats();
      S.load(ns, nt, nf);
      for (const Segment& sg : src) S.add(*sg.st, true);
      S.add(*mst, false);
    }
    for (size_t i = 0; i < ids.size(); ++i) md[i] = ns.del[ids[i]];
    for (uint32_t g : ns.pend_del) {  // not committed yet
      const auto it = std::lower_bound(ids.begin(), ids.end(), g);
      if (it != ids.end() && *it == g) md[it - ids.begin()] = 0;
    }
  };
  if (mix) {
    {
      std::lock_guard<std::mutex> w(ns.writer);
      refresh(ver_used, mdel_used);
    }
    const bool any_del = std::find(mdel_used.begin(), mdel_used.end(), 1) != mdel_used.end();
    if (ver_used != ver0 || any_del || stats_change) {
      const fg_global_stats g0 = S.global();
      fg_index* re = nullptr;
      const int rc = fg_index_rescore(mix, &g0, any_del ? mdel_used.data() : nullptr, &re);
      fg_index_release(mix);
      if (rc) return hfail(rc, fg_last_error());
      mix = re;
    }
  }
  tr.mark("rescore merged segment");
  // ---- swap: no commit runs meanwhile.  A commit that landed since the last
  // rescore changed the statistics (or deleted docs): the merged segment is
  // rescored again OUTSIDE the committer lock and the swap retried, so a commit
  // waits on a merge only for the swap itself; after kSwapTries the rescore
  // runs under the lock (commits arriving faster than one rescore).
  constexpr int kSwapTries = 3;
  std::unique_lock<std::mutex> c(ns.committer);
  tr.mark("wait for the committer");
  std::shared_ptr<Snapshot> now;
  std::vector<uint8_t> del, mdel(ids.size(), 0);
  bool moved = false, new_del = false;
  for (int attempt = 1;; ++attempt) {
    {
      std::shared_lock<std::shared_mutex> l(ns.snap_mu);
      now = ns.snap;
    }
    {
      std::lock_guard<std::mutex> w(ns.writer);
      uint64_t ver = 0;
      refresh(ver, mdel);
      moved = ver != ver_used;  // a commit since the last rescore: other statistics
      new_del = mdel != mdel_used;
      del = ns.del;
      for (uint32_t g : ns.pend_del) del[g] = 0;  // committed deletions only
      if (mix && (moved || new_del) && attempt < kSwapTries) {
        ver_used = ver;
        mdel_used = mdel;
      }
    }
    if (!mix || !(moved || new_del) || attempt >= kSwapTries) break;
    c.unlock();
    const fg_global_stats g1 = S.global();
    const bool any_del = std::find(mdel_used.begin(), mdel_used.end(), 1) != mdel_used.end();
    fg_index* re = nullptr;
    const int rc = fg_index_rescore(mix, &g1, any_del ? mdel_used.data() : nullptr, &re);
    fg_index_release(mix);
    if (rc) return hfail(rc, fg_last_error());
    mix = re;
    tr.mark("rescore merged segment (a commit landed)");
    c.lock();
    tr.mark("wait for the committer");
  }
  size_t j0 = now->segs.size();
  for (size_t j = 0; j < now->segs.size(); ++j)
    if (now->segs[j].id == src[0].id) { j0 = j; break; }
  bool same = j0 + src.size() <= now->segs.size();
  for (size_t i = 0; same && i < src.size(); ++i) same = now->segs[j0 + i].id == src[i].id;
  if (!same) {  // only the merger removes segments: cannot happen
    if (mix) fg_index_release(mix);
    return hfail(FG_EINVAL, "merge sources vanished from the snapshot");
  }
  const fg_global_stats g = S.global();
  if (mix && (moved || new_del)) {
    fg_index* re = nullptr;
    const bool any_del = std::find(mdel.begin(), mdel.end(), 1) != mdel.end();  // every deletion, not just the new ones
    const int rc = fg_index_rescore(mix, &g, any_del ? mdel.data() : nullptr, &re);
    fg_index_release(mix);
    if (rc) return hfail(rc, fg_last_error());
    mix = re;
  }
  auto snap = db->new_snapshot();
  const std::vector<Segment> before(now->segs.begin(), now->segs.begin() + j0),
      after(now->segs.begin() + j0 + src.size(), now->segs.end());
  auto keep = [&](const std::vector<Segment>& v) -> int {
    if (stats_change) return rescore_into(v, g, del, snap->segs);  // N / df changed: every segment rescores
    for (const Segment& sg : v) {
      fg_index_retain(sg.ix);
      snap->segs.push_back(sg);
    }
    return FG_OK;
  };
  if (int rc = keep(before)) {
    if (mix) fg_index_release(mix);
    return rc;
  }
  if (mix) {
    Segment m{mix, 0, (uint32_t)ids.size(), nullptr, 0, mst};
    if (ids.back() - ids.front() + 1 == ids.size()) m.base = ids.front();  // contiguous: no id table
    else m.gid = std::make_shared<const std::vector<uint32_t>>(ids);
    snap->segs.push_back(std::move(m));
  }
  if (int rc = keep(after)) return rc;
  std::shared_ptr<Snapshot> prev;  // released after the locks
  {
    std::lock_guard<std::mutex> w(ns.writer);
    if (mix) snap->segs[before.size()].id = ns.next_seg++;
    std::unique_lock<std::shared_mutex> l(ns.snap_mu);
    prev = std::move(ns.snap);
    ns.snap = snap;
    if (stats_change || moved) S.store(ns);
  }
  now.reset();
  cur.reset();
  db->retire(std::move(prev));
  tr.mark("rescore + swap");
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  {
    std::lock_guard<std::mutex> l(ns.mq);
    ns.merges++;
    ns.merged_docs += ids.size();
    ns.merge_ms_total += ms;
    ns.merge_ms_last = ms;
    ns.merge_ms_max = std::max(ns.merge_ms_max, ms);
  }
  *did = true;
  return FG_OK;
}

void merger_main(fg_db* db) {
  fg_thread_background(1);  // merges build on the device's CU-masked background streams
  for (;;) {
    std::shared_ptr<Namespace> ns;
    {
      std::unique_lock<std::mutex> l(db->mq);
      db->mq_cv.wait(l, [&] { return db->stop || !db->queue.empty(); });
      if (db->stop) return;
      ns = db->queue.front().lock();
      db->queue.pop_front();
    }
    if (!ns) continue;
    {
      std::lock_guard<std::mutex> l(ns->mq);
      ns->queued = false;
      ns->running = true;
    }
    std::string err;
    for (;;) {
      bool did = false;
      if (merge_once(db, *ns, &did)) {
        err = fg_last_error();
        break;
      }
      std::lock_guard<std::mutex> l(db->mq);
      if (!did || db->stop) break;
    }
    {
      std::lock_guard<std::mutex> l(ns->mq);
      ns->running = false;
      if (!err.empty()) ns->merge_error = err;
    }
    ns->mq_cv.notify_all();
  }
}

void enqueue_merge(fg_db* db, const std::shared_ptr<Namespace>& ns) {
  {
    std::lock_guard<std::mutex> l(ns->mq);
    if (ns->queued) return;
    ns->queued = true;
  }
  {
    std::lock_guard<std::mutex> l(db->mq);
    db->queue.push_back(ns);
    if (!db->merger.joinable()) db->merger = std::thread(merger_main, db);
  }
  db->mq_cv.notify_one();
}

}  // namespace

extern "C" {

int fg_db_upsert(fg_db* db, const char* nsname, const char* id, const char* text, const char* name,
                 const char* metadata_json) {
  fg_object_record r{};
  r.id = id;
  r.text = text;
  r.metadata_json = metadata_json;
  return upsert_record(db, nsname, &r, name, true);
}

int fg_db_upsert_record(fg_db* db, const char* nsname, const fg_object_record* rec) {
  return upsert_record(db, nsname, rec, nullptr, false);
}

int fg_db_commit(fg_db* db, const char* nsname) {
  // IndexWriter::commit (src/db/document.rs:65): the docs upserted since the
  // last commit become a new segment; the namespace statistics change, so the
  // older segments are rescored on the device (fg_index_rescore: their postings
  // stay where they are) and pick up the new deletions.  Merges run on the
  // background merger (merge_once); a commit waits for one only when the
  // namespace holds kHardSegments segments.
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  if (!db->ctx) return hfail(FG_ENODEV, "fg_db created without a device context");
  // the commit's device work (new segment, rescores, an inline merge) on the
  // background streams, leaving CUs to the searches running beside it
  struct Background {
    int prev = fg_thread_background(1);
    ~Background() { fg_thread_background(prev); }
  } bg;
  size_t nseg = 0;
  {
    std::shared_lock<std::shared_mutex> l(ns->snap_mu);
    nseg = ns->snap ? ns->snap->segs.size() : 0;
  }
  if (nseg + 1 > kHardSegments) {
    bool did = false;
    if (int rc = merge_once(db, *ns, &did)) return rc;
  }
  if (int rc = commit_segment(db, *ns)) return rc;
  std::vector<uint64_t> sizes;
  {
    std::shared_lock<std::shared_mutex> l(ns->snap_mu);
    if (ns->snap)
      for (auto& sg : ns->snap->segs) sizes.push_back(sg.n);
  }
  const auto run = pick_merge(sizes);
  if (run.first < run.second) enqueue_merge(db, ns);
  return FG_OK;
}

int fg_merge_policy_pick(const uint64_t* seg_docs, uint32_t n_segs, uint32_t* j0, uint32_t* j1) {
  if ((n_segs && !seg_docs) || !j0 || !j1) return hfail(FG_EINVAL, "bad arguments");
  const auto run = pick_merge(std::vector<uint64_t>(seg_docs, seg_docs + n_segs));
  *j0 = (uint32_t)run.first;
  *j1 = (uint32_t)run.second;
  return FG_OK;
}

int fg_db_merge_wait(fg_db* db, const char* nsname) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::unique_lock<std::mutex> l(ns->mq);
  ns->mq_cv.wait(l, [&] { return !ns->queued && !ns->running; });
  if (!ns->merge_error.empty()) {
    const std::string e = ns->merge_error;
    ns->merge_error.clear();
    return hfail(FG_EHIP, "background merge failed: " + e);
  }
  return FG_OK;
}

int fg_db_merge_info_get(fg_db* db, const char* nsname, fg_merge_info* out) {
  if (!db || !out) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::memset(out, 0, sizeof *out);
  {
    std::lock_guard<std::mutex> l(ns->mq);
    out->merges = ns->merges;
    out->merged_docs = ns->merged_docs;
    out->merge_ms_total = ns->merge_ms_total;
    out->merge_ms_last = ns->merge_ms_last;
    out->merge_ms_max = ns->merge_ms_max;
    out->pending = (ns->queued || ns->running) ? 1 : 0;
  }
  std::shared_ptr<Snapshot> snap;
  {
    std::shared_lock<std::shared_mutex> l(ns->snap_mu);
    snap = ns->snap;
  }
  out->segments = snap ? (uint32_t)snap->segs.size() : 0;
  std::lock_guard<std::mutex> w(ns->writer);
  out->n_docs_stats = ns->st_n;
  out->tot_tokens[0] = ns->st_tot[0];
  out->tot_tokens[1] = ns->st_tot[1];
  out->tot_facet_tokens = ns->st_tot_f;
  return FG_OK;
}

int fg_db_segment_docs(fg_db* db, const char* nsname, uint32_t seg, uint32_t* out, uint32_t cap, uint32_t* n) {
  if (!db || !n) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::shared_ptr<Snapshot> snap;
  {
    std::shared_lock<std::shared_mutex> l(ns->snap_mu);
    snap = ns->snap;
  }
  if (!snap || seg >= snap->segs.size()) return hfail(FG_EINVAL, "no such segment");
  const Segment& s0 = snap->segs[seg];
  *n = s0.n;
  if (out)
    for (uint32_t d = 0; d < s0.n && d < cap; ++d) out[d] = s0.global(d);
  return FG_OK;
}

int fg_db_upsert_batch(fg_db* db, const char* nsname, uint32_t n, const char* ids, const uint64_t* id_off,
                       const char* texts, const uint64_t* text_off) {
  // batch_upsert_objects (src/server/handlers/ingest.rs:160-220) -> Dataset::
  // batch_upsert -> NamedIndex::upsert (src/db/document.rs:23-73): every record
  // validated first ("Validation failed for object at index i: ..."), then
  // upserted in order under the writer lock (raw-id delete, add), then ONE
  // commit (one segment).  Records are {id, text} (no metadata, namespace or facets).  The
  // "default" analyzer runs on the host threads before the lock (each thread
  // interns into its own dictionary; the dictionaries merge into the
  // namespace's under the lock), so a bulk load does not serialise on it.
  if (!db || (n && (!ids || !id_off || !texts || !text_off))) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  auto sv = [](const char* b, const uint64_t* off, uint32_t i) { return std::string_view(b + off[i], off[i + 1] - off[i]); };
  for (uint32_t i = 0; i < n; ++i) {  // ObjectRecord::validate (src/object.rs:31-78)
    const std::string_view id = sv(ids, id_off, i), tx = sv(texts, text_off, i);
    const char* e = id.empty() ? "Object ID cannot be empty"
                    : id.size() > 256 ? "Object ID too long (max 256 characters)"
                    : tx.empty() ? "Object text cannot be empty"
                    : tx.size() > 10000 ? "Text too long (max 10000 characters)" : nullptr;
    if (e) return hfail(FG_EINVAL, "Validation failed for object at index " + std::to_string(i) + ": " + e);
  }
  PhaseTrace tr("upsert");
  // ~256 docs per thread: a commit's 1000 docs analyze on 4 (the pool's)
  const int T = std::max(1, std::min<int>(fg_host_threads(), (int)(n / 256) + 1));
  std::vector<LocalDict> ldict(T);
  std::vector<Doc> docs(n);
  // per thread: its docs analyzed into its own dictionary, then its terms looked
  // up in the namespace's without a lock (ids never change once interned; a
  // term missing here is interned under the writer lock below)
  std::vector<std::vector<uint32_t>> remap(T);
  std::vector<std::vector<uint64_t>> hsh(T);
  run_threads((size_t)T, (size_t)T, [&](size_t t) {
    const uint32_t b = (uint32_t)((uint64_t)n * t / T), e = (uint32_t)((uint64_t)n * (t + 1) / T);
    std::vector<std::string> toks;
    std::string scratch;
    for (uint32_t i = b; i < e; ++i) {
      Doc& d = docs[i];
      d.id = std::string(sv(ids, id_off, i));
      d.text = std::string(sv(texts, text_off, i));
      // thread-local term ids until the merge
      analyze_each(d.text, scratch, toks, [&](std::string_view w) { d.text_tok.push_back(ldict[t].get(w)); });
      analyze(d.id, d.id_tokens);
    }
    const uint32_t ne = (uint32_t)ldict[t].ent.size();
    hsh[t].resize(ne);
    remap[t].resize(ne);
    for (uint32_t j = 0; j < ne; ++j) hsh[t][j] = TermDict::hash(ldict[t].key(j));
    constexpr uint32_t kAhead = 16;  // the slot lines of later lookups in flight
    for (uint32_t j = 0; j < std::min(ne, kAhead); ++j) ns->dict.prefetch(hsh[t][j]);
    for (uint32_t j = 0; j < ne; ++j) {
      if (j + kAhead < ne) ns->dict.prefetch(hsh[t][j + kAhead]);
      remap[t][j] = ns->dict.find(ldict[t].key(j), hsh[t][j]);
    }
  });
  tr.mark("analyze");
  {  // the writer lock: the new terms interned, the ordered upserts
    std::lock_guard<std::mutex> w(ns->writer);
    for (int t = 0; t < T; ++t)
      for (uint32_t j = 0; j < (uint32_t)remap[t].size(); ++j)
        if (remap[t][j] == TermDict::kMissing) remap[t][j] = ns->dict.get(ldict[t].key(j), hsh[t][j]);
    tr.mark("dictionary merge");
    run_threads((size_t)T, (size_t)T, [&](size_t t) {
      const uint32_t b = (uint32_t)((uint64_t)n * t / T), e = (uint32_t)((uint64_t)n * (t + 1) / T);
      for (uint32_t i = b; i < e; ++i)
        for (auto& x : docs[i].text_tok) x = remap[t][x];
    });
    tr.mark("remap");
    // a bulk load sizes the id map once; a small batch lets it grow geometrically
    // (reserving size + n on every call rehashed all 10M entries per commit)
    if (n > ns->by_id_token.size()) ns->by_id_token.reserve(ns->by_id_token.size() + n);
    for (uint32_t i = 0; i < n; ++i) {
      // delete_term(id_field, raw id) (src/db/document.rs:38-42), then add_document
      auto it = ns->by_id_token.find(docs[i].id);
      if (it != ns->by_id_token.end())
        for (uint32_t d : it->second) {
          if (!ns->del[d]) ns->pend_del.push_back(d);
          ns->docs[d].deleted = true;
          ns->del[d] = 1;
        }
      const uint32_t d = (uint32_t)ns->docs.size();
      for (auto& t : docs[i].id_tokens) ns->by_id_token[t].push_back(d);
      ns->del.push_back(0);
      ns->docs.push_back(std::move(docs[i]));
    }
  }
  tr.mark("dictionary + upserts");
  return fg_db_commit(db, nsname);  // NamedIndex::upsert commits once per call (src/db/document.rs:65)
}

int fg_db_add_file(fg_db* db, const char* ns, const char* name, const char* body) {
  // POST /add/{namespace} {"name","body"} -> ObjectRecord{id: name, text: body,
  // namespace: ns, metadata: {"name": name}} -> upsert + commit (one commit per call,
  // as NamedIndex::upsert commits per call, src/db/document.rs:65)
  if (!name) return hfail(FG_EINVAL, "name is required");
  std::string meta = "{\"name\":";
  json_str(meta, name);
  meta += "}";
  fg_object_record r{};
  r.id = name;
  r.text = body;
  r.metadata_json = meta.c_str();
  r.namespace_ = ns;
  int rc = fg_db_upsert_record(db, ns, &r);
  if (rc) return rc;
  return fg_db_commit(db, ns);
}

int fg_db_doc_count(fg_db* db, const char* nsname, uint64_t* total, uint64_t* alive) {
  if (!db || !total || !alive) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::lock_guard<std::mutex> w(ns->writer);
  *total = ns->docs.size();
  *alive = 0;
  for (uint8_t x : ns->del) *alive += x ? 0 : 1;
  return FG_OK;
}

int fg_db_search_ex(fg_db* db, const char* nsname, const char* query, const char* const* filters, uint32_t n_filters,
                    uint32_t page, uint32_t per_page, fg_hit* out, uint32_t cap, uint32_t* n_out) {
  if (!db || !n_out) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::vector<fg_hit> hits;
  int rc = search_hits(db, *ns, query, filter_list(filters, n_filters), page, per_page, hits);
  if (rc) return rc;
  *n_out = (uint32_t)std::min<size_t>(hits.size(), cap);
  if (out) std::copy(hits.begin(), hits.begin() + *n_out, out);
  return FG_OK;
}

int fg_db_search(fg_db* db, const char* nsname, const char* query, uint32_t page, uint32_t per_page, fg_hit* out,
                 uint32_t cap, uint32_t* n_out) {
  return fg_db_search_ex(db, nsname, query, nullptr, 0, page, per_page, out, cap, n_out);
}

int fg_db_search_json_ex(fg_db* db, const char* nsname, const char* query, const char* const* filters,
                         uint32_t n_filters, uint32_t page, uint32_t per_page, int include_text, int shape, char* out,
                         size_t cap, size_t* len) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  if (shape != FG_SHAPE_GET_SEARCH && shape != FG_SHAPE_POST_SEARCH && shape != FG_SHAPE_GET_SEARCH_PATH)
    return hfail(FG_EINVAL, "bad shape (POST /search/json: fg_db_search_json_post)");
  std::string q = query ? query : "";
  if (shape == FG_SHAPE_GET_SEARCH_PATH) {
    // query_text_path (src/server/handlers/search.rs:79-139): the path component
    // is URL-decoded; page 0, per_page 20
    if (!url_decode(q)) {
      copy_out("{\"error\":\"Invalid URL encoding in query\"}", out, cap, len);
      return hfail(FG_EINVAL, "Invalid URL encoding in query");
    }
    page = 0;
    per_page = 20;
  }
  return search_json(db, nsname, q, filter_list(filters, n_filters), page, per_page, include_text != 0,
                     shape == FG_SHAPE_POST_SEARCH, nullptr, out, cap, len);
}

int fg_db_search_json_post(fg_db* db, const char* nsname, const char* query, const char* const* filters,
                           uint32_t n_filters, int has_page, uint32_t page, uint32_t per_page, int url_text,
                           int body_text, int url_include_data, int body_include_data, char* out, size_t cap,
                           size_t* len) {
  // query_json_post (src/server/handlers/search.rs:210-301)
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  const std::vector<std::string> fl = filter_list(filters, n_filters);
  if (!has_page) { page = 0; per_page = 20; }
  // text: the URL flag wins when set; a disagreeing body flag adds a developer_message
  const bool include_text = url_text >= 0 ? url_text != 0 : body_text > 0;
  JsonExtras ex;
  if (url_text >= 0 && body_text >= 0 && (url_text != 0) != (body_text != 0))
    ex.developer_message = "url and request body are set to different values; using url:true/false";
  // is_targeting_conversations_or_organizations (handlers/utils.rs:4-14)
  ex.targeting = false;
  for (auto& f : fl) {
    const std::string n = !f.empty() && f[0] == '/' ? f : "/" + f;
    if (n.find("/conversation") != std::string::npos || n.find("/organization") != std::string::npos) ex.targeting = true;
  }
  // include_data: body, else URL, else !targeting
  ex.include_data = body_include_data >= 0 ? body_include_data != 0
                    : url_include_data >= 0 ? url_include_data != 0 : !ex.targeting;
  return search_json(db, nsname, query ? query : "", fl, page, per_page, include_text, false, &ex, out, cap, len);
}

int fg_db_search_json(fg_db* db, const char* nsname, const char* query, uint32_t page, uint32_t per_page,
                      int include_text, int shape, char* out, size_t cap, size_t* len) {
  return fg_db_search_json_ex(db, nsname, query, nullptr, 0, page, per_page, include_text, shape, out, cap, len);
}

int fg_db_doc_facets(fg_db* db, const char* nsname, uint32_t doc, char* out, size_t cap, size_t* len) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::lock_guard<std::mutex> w(ns->writer);
  if (doc >= ns->docs.size()) return hfail(FG_EINVAL, "doc out of range");
  std::string o;
  for (size_t j = 0; j < ns->docs[doc].facets.size(); ++j) {
    if (j) o.push_back('\n');
    o += facet_display(ns->docs[doc].facets[j]);
  }
  return copy_out(o, out, cap, len);
}

int fg_facet_tokens(const char* path, char* out, size_t cap, size_t* len) {
  if (!path) return hfail(FG_EINVAL, "bad arguments");
  std::string enc;
  if (!facet_from_text(path, enc)) return hfail(FG_EINVAL, "Facet::from_text: path must start with '/'");
  std::vector<std::string> toks;
  facet_tokens(enc, toks);
  std::string o;
  for (size_t i = 0; i < toks.size(); ++i) {
    if (i) o.push_back('\n');
    o += toks[i];  // U+0000 separators kept: read *len bytes
  }
  if (len) *len = o.size();
  if (!out) return FG_OK;
  if (cap < o.size() + 1) return hfail(FG_EINVAL, "output buffer too small");
  std::memcpy(out, o.data(), o.size());
  out[o.size()] = 0;
  return FG_OK;
}

int fg_facet_clauses(const char* const* filters, uint32_t n_filters, int* applies, int* all_query, char* out,
                     size_t cap, size_t* len) {
  if (!applies || !all_query) return hfail(FG_EINVAL, "bad arguments");
  std::vector<std::string> cl;
  bool all = false;
  *applies = facet_clauses(filter_list(filters, n_filters), cl, &all) ? 1 : 0;
  *all_query = all ? 1 : 0;
  std::string o;
  for (size_t i = 0; i < cl.size(); ++i) {
    if (i) o.push_back('\n');
    o += cl[i];
  }
  if (len) *len = o.size();
  if (!out) return FG_OK;
  if (cap < o.size() + 1) return hfail(FG_EINVAL, "output buffer too small");
  std::memcpy(out, o.data(), o.size());
  out[o.size()] = 0;
  return FG_OK;
}

int fg_analyze(const char* text, char* out, size_t cap, size_t* len) {
  if (!text) return hfail(FG_EINVAL, "bad arguments");
  std::vector<std::string> toks;
  analyze(text, toks);
  std::string o;
  for (size_t i = 0; i < toks.size(); ++i) {
    if (i) o.push_back('\n');
    o += toks[i];
  }
  return copy_out(o, out, cap, len);
}

int fg_parse_query(const char* query, int* mode, char* out, size_t cap, size_t* len) {
  if (!query || !mode) return hfail(FG_EINVAL, "bad arguments");
  std::vector<std::string> terms;
  std::vector<uint8_t> occur;
  std::string why;
  int rc = parse_query(query, terms, occur, why);
  if (rc) return hfail(rc, why);
  *mode = mode_of(occur);
  std::string o;
  for (size_t i = 0; i < terms.size(); ++i) {
    if (i) o.push_back('\n');
    o += terms[i];
  }
  return copy_out(o, out, cap, len);
}

int fg_parse_query_occur(const char* query, char* out, size_t cap, size_t* len) {
  if (!query) return hfail(FG_EINVAL, "bad arguments");
  std::vector<std::string> terms;
  std::vector<uint8_t> occur;
  std::string why;
  int rc = parse_query(query, terms, occur, why);
  if (rc) return hfail(rc, why);
  std::string o;
  for (size_t i = 0; i < terms.size(); ++i) {
    if (i) o.push_back('\n');
    o.push_back((char)('0' + occur[i]));
    o.push_back(':');
    o += terms[i];
  }
  return copy_out(o, out, cap, len);
}

}  // extern "C"
