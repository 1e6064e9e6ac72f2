"""Batch-of-one GET /search latency (fg_db_search over a 10M namespace of 8
commit segments, OR top-20, bench.py's db_api line) for several builds of
libfugu, each in its own child process (one HIP runtime binding per process).

  python tools/db_latency_ab.py lib1.so lib2.so ...
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np
    from fugu_amd import db as fdb, native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(10_000_000, threads=16)
    d = fdb.Database(ctx)
    d.create_namespace("api")
    tb, to = synth.render_text(corp, 16)
    ib, io = synth.render_ids(corp.n_docs)
    bounds = [corp.n_docs * i // 8 for i in range(9)]
    for a, b in zip(bounds[:-1], bounds[1:]):
        d.upsert_batch("api", id_buf=ib[int(io[a]):int(io[b])], id_off=io[a:b + 1] - io[a],
                       text_buf=tb[int(to[a]):int(to[b])], text_off=to[a:b + 1] - to[a])
    q_off, terms = synth.queries(200, 2, 5, seed_q=333)
    qs = [" ".join(f"t{t}" for t in terms[q_off[i]:q_off[i + 1]]) for i in range(200)]
    for q in qs[:16]:
        d.search("api", q, 0, 20)
    out = []
    for _ in range(3):
        lat = []
        for q in qs:
            t1 = time.perf_counter()
            d.search("api", q, 0, 20)
            lat.append(time.perf_counter() - t1)
        out.append([round(float(np.percentile(lat, p) * 1e3), 4) for p in (50, 90, 99)])
    print(json.dumps({"lib": os.environ.get("FUGU_LIB"), "p50_p90_p99_ms": out}), flush=True)


def main():
    if sys.argv[1:] == ["--child"]:
        return child()
    for lib in sys.argv[1:]:
        env = dict(os.environ, FUGU_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=400)
        sys.stdout.write(r.stdout)
        if r.returncode:
            sys.stderr.write(r.stderr[-2000:])
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
