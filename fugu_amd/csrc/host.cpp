// Host side above the device ABI (include/fugu_host.h): fugu's Dataset /
// DatasetManager glue, the "default" analyzer, the QueryParser subset the
// device runs, and the perform_search response shapes.  C++ because the
// reference's Rust toolchain is absent.  Reference citations
// are on each function.
#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "../../include/fugu.h"
#include "../../include/fugu_host.h"

void fg_set_last_error(const std::string& msg);  // fugu.cpp

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

// ---------------------------------------------------------------- query parser subset
// QueryParser::for_index(index, [text, name]).parse_query (src/db/search.rs:108-127)
// restricted to what the device runs:
//   `t1 t2 ...`                 default conjunction Should  -> FG_MODE_OR
//   `t1 AND t2 AND ...`, `+t1 +t2`                          -> FG_MODE_AND
//   `t1`                                                    -> single term
// Every term must analyze to exactly one token (more = PhraseQuery).  Anything
// else is FG_EUNSUPPORTED (the reference host runs tantivy).  An empty query is
// AllQuery (src/db/search.rs:115-116): unsupported on the device.
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

int parse_query(std::string_view q, int* mode, std::vector<std::string>& terms, std::string& why) {
  terms.clear();
  std::vector<std::string_view> words;
  size_t i = 0;
  while (i < q.size()) {
    while (i < q.size() && (q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r')) ++i;
    size_t s = i;
    while (i < q.size() && !(q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r')) ++i;
    if (i > s) words.push_back(q.substr(s, i - s));
  }
  if (words.empty()) { why = "empty query (AllQuery)"; return FG_EUNSUPPORTED; }
  std::vector<std::string_view> raw;
  bool and_form = words.size() >= 3 && words.size() % 2 == 1;
  for (size_t w = 1; and_form && w < words.size(); w += 2) and_form = words[w] == "AND";
  bool plus_form = true;
  for (auto w : words) plus_form = plus_form && w.size() > 1 && w[0] == '+';
  if (and_form) {
    *mode = FG_MODE_AND;
    for (size_t w = 0; w < words.size(); w += 2) raw.push_back(words[w]);
  } else if (plus_form) {
    *mode = FG_MODE_AND;
    for (auto w : words) raw.push_back(w.substr(1));
  } else {
    *mode = words.size() == 1 ? FG_MODE_AND : FG_MODE_OR;
    raw = words;
  }
  for (auto w : raw) {
    if (w == "AND" || w == "OR" || w == "NOT" || w == "IN" || w == "TO") {
      why = "operator outside the supported forms";
      return FG_EUNSUPPORTED;
    }
    for (char c : w)
      if (is_special(c)) {
        why = "query syntax beyond bare/+/AND terms";
        return FG_EUNSUPPORTED;
      }
    std::vector<std::string> toks;
    analyze(w, toks);
    if (toks.size() != 1) {
      why = toks.empty() ? "a term analyzes to no token" : "a term analyzes to several tokens (PhraseQuery)";
      return FG_EUNSUPPORTED;
    }
    terms.push_back(std::move(toks[0]));
  }
  return FG_OK;
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

// ---------------------------------------------------------------- datasets
struct Doc {
  std::string id, text, name, metadata;
  bool has_name = false;
  bool deleted = false;
  std::vector<uint32_t> text_tok, name_tok;
  std::vector<std::string> id_tokens;
};

struct Snapshot {
  fg_index* ix = nullptr;
  ~Snapshot() { if (ix) fg_index_release(ix); }
};

struct Namespace {
  std::string name;
  std::mutex writer;                                   // IndexWriter lock (src/db/core.rs:211)
  std::mutex committer;                                // serialises commits (snapshot order)
  std::vector<Doc> docs;                               // global doc id = insertion order
  std::unordered_map<std::string, uint32_t> dict;      // term dictionary (text and name tokens)
  std::unordered_map<std::string, std::vector<uint32_t>> by_id_token;
  std::shared_ptr<Snapshot> snap;                      // committed device snapshot
  std::shared_mutex snap_mu;
  size_t committed_docs = 0;
};

}  // namespace

struct fg_db {
  fg_ctx* ctx = nullptr;
  int dev = 0;
  std::string default_ns;
  std::map<std::string, std::shared_ptr<Namespace>> ns;
  std::shared_mutex mu;
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
  for (auto& t : toks) {
    auto it = ns.dict.find(t);
    if (it == ns.dict.end()) it = ns.dict.emplace(t, (uint32_t)ns.dict.size()).first;
    ids.push_back(it->second);
  }
  return ids;
}

// Dataset::search core: hits of the page in order, or an error code.
int search_hits(fg_db* db, Namespace& ns, const char* query, uint32_t page, uint32_t per_page,
                std::vector<fg_hit>& hits) {
  hits.clear();
  if (per_page == 0) return hfail(FG_EINVAL, "TopDocs::with_limit requires limit >= 1");
  int mode = FG_MODE_AND;
  std::vector<std::string> terms;
  std::string why;
  int rc = parse_query(query ? query : "", &mode, terms, why);
  if (rc) return hfail(rc, "query outside the device subset: " + why);
  const uint64_t offset = (uint64_t)page * per_page, limit = offset + per_page;
  if (limit > FG_MAX_K) return hfail(FG_EUNSUPPORTED, "offset + per_page > FG_MAX_K");
  std::shared_ptr<Snapshot> snap;
  std::vector<uint32_t> ids;
  {
    std::shared_lock<std::shared_mutex> l(ns.snap_mu);
    snap = ns.snap;
  }
  {
    // term ids are stable once interned; ids interned after the snapshot are >= its n_terms
    std::lock_guard<std::mutex> w(ns.writer);
    for (auto& t : terms) {
      auto it = ns.dict.find(t);
      ids.push_back(it == ns.dict.end() ? FG_TERM_MISSING : it->second);
    }
  }
  if (!snap) return FG_OK;  // nothing committed yet: no hits
  // terms added after the snapshot are unknown to it
  fg_index_stats st;
  fg_index_stats_get(snap->ix, &st);
  for (auto& t : ids)
    if (t != FG_TERM_MISSING && t >= st.n_terms) t = FG_TERM_MISSING;
  const uint32_t q_off[2] = {0, (uint32_t)ids.size()};
  fg_query_batch qb{1, q_off, ids.data(), mode};
  std::vector<float> sc(limit);
  std::vector<uint32_t> dc(limit);
  uint32_t n = 0;
  rc = fg_search_batch(snap->ix, &qb, (uint32_t)limit, sc.data(), dc.data(), &n);
  if (rc) return hfail(rc, fg_last_error());
  for (uint64_t i = offset; i < n; ++i) hits.push_back(fg_hit{sc[i], dc[i]});  // skip(offset).take(per_page)
  return FG_OK;
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
  std::string o = "{\"status\":\"success\",\"namespaces\":[";
  {
    std::shared_lock<std::shared_mutex> l(db->mu);
    bool first = true;
    for (auto& kv : db->ns) {
      if (!first) o.push_back(',');
      first = false;
      json_str(o, kv.first);
    }
  }
  o += "]}";
  return copy_out(o, out, cap, len);
}

int fg_db_upsert(fg_db* db, const char* nsname, const char* id, const char* text, const char* name,
                 const char* metadata_json) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  // ObjectRecord::validate (src/object.rs:31-78)
  const std::string sid = id ? id : "", stext = text ? text : "";
  if (sid.empty()) return hfail(FG_EINVAL, "Object ID cannot be empty");
  if (sid.size() > 256) return hfail(FG_EINVAL, "Object ID too long (max 256 characters)");
  if (stext.empty()) return hfail(FG_EINVAL, "Object text cannot be empty");
  if (stext.size() > 10000) return hfail(FG_EINVAL, "Text too long (max 10000 characters)");
  if (nsname) {
    std::string_view n(nsname);
    if (n.empty() || n.find('/') != std::string_view::npos || n.find(' ') != std::string_view::npos)
      return hfail(FG_EINVAL, "Invalid namespace format");
    if (n.size() > 128) return hfail(FG_EINVAL, "Namespace too long (max 128 characters)");
  }
  std::lock_guard<std::mutex> w(ns->writer);
  // w.delete_term(Term::from_field_text(id_field, &object.id)) (src/db/document.rs:38-42): the
  // RAW id is matched against the tokens of the tokenized `id` field, so ids with
  // uppercase or punctuation never match and are not replaced
  auto it = ns->by_id_token.find(sid);
  if (it != ns->by_id_token.end())
    for (uint32_t d : it->second) ns->docs[d].deleted = true;
  Doc doc;
  doc.id = sid;
  doc.text = stext;
  doc.has_name = name != nullptr;
  if (name) doc.name = name;
  if (metadata_json) doc.metadata = metadata_json;
  doc.text_tok = intern(*ns, doc.text);
  if (doc.has_name) doc.name_tok = intern(*ns, doc.name);
  analyze(doc.id, doc.id_tokens);
  const uint32_t d = (uint32_t)ns->docs.size();
  for (auto& t : doc.id_tokens) ns->by_id_token[t].push_back(d);
  ns->docs.push_back(std::move(doc));
  return FG_OK;
}

int fg_db_commit(fg_db* db, const char* nsname) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  if (!db->ctx) return hfail(FG_ENODEV, "fg_db created without a device context");
  std::lock_guard<std::mutex> c(ns->committer);
  // gather under the writer lock, build the device snapshot outside it so
  // searches (doc fetch) and upserts are not blocked by the upload
  std::unique_lock<std::mutex> w(ns->writer);
  if (ns->docs.empty()) return FG_OK;
  const uint32_t N = (uint32_t)ns->docs.size();
  const uint32_t n_terms = std::max<uint32_t>(1, (uint32_t)ns->dict.size());
  std::vector<uint64_t> toff(N + 1, 0), noff(N + 1, 0);
  std::vector<uint32_t> ttok, ntok;
  std::vector<uint8_t> del(N, 0);
  bool any_name = false, any_del = false;
  for (uint32_t d = 0; d < N; ++d) {
    const Doc& doc = ns->docs[d];
    ttok.insert(ttok.end(), doc.text_tok.begin(), doc.text_tok.end());
    ntok.insert(ntok.end(), doc.name_tok.begin(), doc.name_tok.end());
    toff[d + 1] = ttok.size();
    noff[d + 1] = ntok.size();
    any_name |= !doc.name_tok.empty();
    del[d] = doc.deleted ? 1 : 0;
    any_del |= doc.deleted;
  }
  w.unlock();
  fg_docs_input in{};
  in.n_docs = N;
  in.n_terms = n_terms;
  in.text_off = toff.data();
  in.text_tok = ttok.data();
  in.name_off = any_name ? noff.data() : nullptr;
  in.name_tok = any_name ? ntok.data() : nullptr;
  in.deleted = any_del ? del.data() : nullptr;
  in.threads = 0;
  in.keep_host_postings = 0;
  fg_index* ix = nullptr;
  int rc = fg_index_build_from_docs(db->ctx, db->dev, &in, &ix);
  if (rc) return hfail(rc, fg_last_error());
  auto snap = std::make_shared<Snapshot>();
  snap->ix = ix;
  {
    std::unique_lock<std::shared_mutex> l(ns->snap_mu);  // readers keep the old snapshot (refcount)
    ns->snap = snap;
    ns->committed_docs = N;
  }
  return FG_OK;
}

int fg_db_add_file(fg_db* db, const char* ns, const char* name, const char* body) {
  // POST /add/{namespace} {"name","body"} -> ObjectRecord{id: name, text: body,
  // namespace: ns, metadata: {"name": name}} -> upsert + commit (one commit per call,
  // as NamedIndex::upsert commits per call, src/db/document.rs:65)
  if (!name) return hfail(FG_EINVAL, "name is required");
  std::string meta = "{\"name\":";
  json_str(meta, name);
  meta += "}";
  int rc = fg_db_upsert(db, ns, name, body, name, meta.c_str());
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
  for (auto& d : ns->docs) *alive += d.deleted ? 0 : 1;
  return FG_OK;
}

int fg_db_search(fg_db* db, const char* nsname, const char* query, uint32_t page, uint32_t per_page, fg_hit* out,
                 uint32_t cap, uint32_t* n_out) {
  if (!db || !n_out) return hfail(FG_EINVAL, "bad arguments");
  auto ns = find_ns(db, nsname);
  if (!ns) return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  std::vector<fg_hit> hits;
  int rc = search_hits(db, *ns, query, page, per_page, hits);
  if (rc) return rc;
  *n_out = (uint32_t)std::min<size_t>(hits.size(), cap);
  if (out) std::copy(hits.begin(), hits.begin() + *n_out, out);
  return FG_OK;
}

int fg_db_search_json(fg_db* db, const char* nsname, const char* query, uint32_t page, uint32_t per_page,
                      int include_text, int shape, char* out, size_t cap, size_t* len) {
  if (!db) return hfail(FG_EINVAL, "bad arguments");
  const std::string q = query ? query : "";
  // perform_search (src/server/handlers/search.rs:350-402): namespace lookup, then
  // per_page 0 or > 100 -> 20; the POST /search shape has no clamp (:183)
  auto ns = find_ns(db, nsname);
  if (!ns) {
    std::string o = "{\"error\":";
    json_str(o, std::string("Search failed: Namespace '") + (nsname ? nsname : "") + "' not found");
    o += "}";
    copy_out(o, out, cap, len);
    return hfail(FG_ENOTFOUND, std::string("Namespace '") + (nsname ? nsname : "") + "' not found");
  }
  if (shape == FG_SHAPE_GET_SEARCH && (per_page == 0 || per_page > 100)) per_page = 20;
  std::vector<fg_hit> hits;
  int rc = search_hits(db, *ns, q.c_str(), page, per_page, hits);
  if (rc) {
    std::string o = "{\"error\":";
    json_str(o, std::string("Search failed: ") + fg_last_error());
    o += "}";
    copy_out(o, out, cap, len);
    return rc;
  }
  std::string res = "[";
  {
    std::lock_guard<std::mutex> w(ns->writer);
    for (size_t i = 0; i < hits.size(); ++i) {
      const Doc& d = ns->docs[hits[i].doc];
      if (i) res.push_back(',');
      // FuguSearchResult {id, score, text, metadata, facets} (src/db/search.rs:20-27)
      res += "{\"id\":";
      json_str(res, d.id);
      res += ",\"score\":";
      json_f32(res, hits[i].score);
      if (include_text) {
        res += ",\"text\":";
        json_str(res, d.text);
      }
      res += ",\"metadata\":";
      res += d.metadata.empty() ? "null" : d.metadata;
      res += ",\"facets\":null}";
    }
  }
  res += "]";
  std::string o;
  char num[64];
  if (shape == FG_SHAPE_POST_SEARCH) {
    // search_endpoint (src/server/handlers/search.rs:184-195)
    o = "{\"status\":\"success\",\"query\":";
    json_str(o, q);
    o += ",\"filters\":[]";
    snprintf(num, sizeof num, ",\"page\":%u,\"per_page\":%u,\"total\":%zu", page, per_page, hits.size());
    o += num;
    o += ",\"results\":" + res + "}";
  } else {
    // SearchResponse {results, total, page, per_page, query} (server/types.rs)
    o = "{\"results\":" + res;
    snprintf(num, sizeof num, ",\"total\":%zu,\"page\":%u,\"per_page\":%u", hits.size(), page, per_page);
    o += num;
    o += ",\"query\":";
    json_str(o, q);
    o += "}";
  }
  return copy_out(o, out, cap, len);
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
  std::string why;
  int rc = parse_query(query, mode, terms, why);
  if (rc) return hfail(rc, why);
  std::string o;
  for (size_t i = 0; i < terms.size(); ++i) {
    if (i) o.push_back('\n');
    o += terms[i];
  }
  return copy_out(o, out, cap, len);
}

}  // extern "C"
