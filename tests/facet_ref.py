"""Python restatement of tantivy's facet encoding and FacetTokenizer
(test infrastructure; independent of fugu_amd/csrc/host.cpp).

  Facet::from_text (schema/facet.rs): the path must start with '/'; '/'
  separates segments (stored as U+0000), '\\' escapes the next char.
  FacetTokenizer (tokenizer/facet_tokenizer.rs): the root facet (empty), then
  every prefix ending before a separator (not counting one at position 0),
  then the whole encoded facet.
  Display (schema/facet.rs): '/' + segments joined by '/', with '/' inside a
  segment written as '\\/'.
fugu normalizes facet paths with a leading '/' (src/db/document.rs:283-287,
src/db/search.rs:594-600).
"""
from __future__ import annotations

SEP = "\x00"


def from_text(path: str):
    if not path or not path.startswith("/"):
        return None
    out = []
    escaped = False
    last = 1
    i = 1
    while i < len(path):
        c = path[i]
        if escaped:
            escaped = False
        elif c == "\\":
            out.append(path[last:i])
            last = i + 1
            escaped = True
        elif c == "/":
            out.append(path[last:i])
            out.append(SEP)
            last = i + 1
        i += 1
    out.append(path[last:])
    return "".join(out)


def tokens(enc: str):
    toks = [""]
    if enc == "":
        return toks
    cur = 0
    b = enc.encode()
    while True:
        nxt = b.find(b"\x00", cur + 1)
        if nxt < 0:
            toks.append(enc)
            return toks
        toks.append(b[:nxt].decode())
        cur = nxt


def display(enc: str) -> str:
    return "".join("/" + seg.replace("/", "\\/") for seg in enc.split(SEP))


def normalize(path: str) -> str:
    return path if path.startswith("/") else "/" + path
