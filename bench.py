"""fugu query hot path on MI355X: queries/sec + p50 latency on a synthetic
10M-doc Zipf corpus, 3-term AND, BM25 top-100 (BASELINE.json `metric`).

A step = one batch of 1024 planned queries through the gfx950 pipeline
(k_conj -> k_final) with the plan and the index resident in HBM.
N > 1 (torchrun, one rank per GPU): rank r holds namespace r (its own 10M-doc
corpus, weak scaling); every step also all-gathers the per-shard top-100 over
RCCL and merges them on the device (fan-out query over all namespaces).

Prints ONE JSON line on rank 0.  See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "queries/sec + p50 latency, 10M-doc Zipf corpus, 3-term AND, top-100"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def host_cores():
    """The host CPU share this process may use (T = nproc on the box).
    nproc honours OMP_NUM_THREADS (16 on the GPU box = its CPU share per GPU);
    the affinity mask and the cgroup quota are reported beside it."""
    import subprocess
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout.strip())
    except Exception:
        nproc = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except Exception:
        pass
    return {"nproc": nproc, "affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "cgroup_cpus": quota}


def native_oracle():
    """Compile the CPU baseline (oracle/fugu_oracle.c) for THIS host with
    -march=native and point oracle.py at it; returns the flags."""
    import subprocess
    import tempfile
    d = tempfile.mkdtemp(prefix="fugu_oracle_")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"OUT={d}"],
                       capture_output=True, text=True)
    lib = os.path.join(d, "libfugu_oracle_native.so")
    if r.returncode == 0 and os.path.exists(lib):
        os.environ["FUGU_ORACLE_LIB"] = lib
        from oracle import oracle as orc
        return orc.NATIVE_FLAGS
    log(f"[bench] native oracle build failed ({r.stderr[-300:]}); using the portable build")
    return "-O3 -ffp-contract=off -march=x86-64-v2 (portable build: native compile failed)"


def timed_steps(step, steps, warmup, torch):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def commit_latency(ctx, ix, corp, native, synth, threads, n_new=1000):
    """fg_db_commit's device work on a 10M-doc namespace: the
    new docs become a segment built with the namespace statistics and the
    10M-doc segment is rescored with them (fg_index_rescore: posting scores,
    bounds, alive bitset recomputed on the device; postings, directory and rank
    words shared).  The namespace's running statistics are kept per commit
    (O(new docs)), so only the new docs' statistics are computed here."""
    base_stats = native.docs_stats(corp.off, corp.tok, synth.VOCAB, threads=threads)  # maintained incrementally
    new = synth.corpus(n_new, doc_begin=corp.n_docs)
    out = {}
    for rep in range(3):
        t0 = time.perf_counter()
        g = base_stats + native.docs_stats(new.off, new.tok, synth.VOCAB, threads=threads)
        t1 = time.perf_counter()
        re = ix.rescore(g)
        t2 = time.perf_counter()
        seg = native.Index.from_docs(ctx, new.off, new.tok, synth.VOCAB, threads=threads, keep_host=False,
                                     global_stats=g)
        t3 = time.perf_counter()
        out = {"commit_ms": round((t3 - t0) * 1e3, 1), "stats_ms": round((t1 - t0) * 1e3, 1),
               "rescore_10M_ms": round((t2 - t1) * 1e3, 1), "new_segment_ms": round((t3 - t2) * 1e3, 1),
               "new_docs": n_new, "base_docs": corp.n_docs}
        re.close()
        seg.close()
    out["note"] = ("device work of one commit of 1000 docs on a 10M-doc namespace: a new segment + the 10M "
                   "segment rescored with the new statistics (third of 3 runs); a full rebuild is the "
                   "'index built in' time")
    return out


def e2e_pipeline(ix, native, synth, torch, dev, nq, K, steps, workers):
    """End-to-end batch throughput: every step plans a DIFFERENT 1024-query batch
    on the host (fg_plan_create: cost order, work items, H2D), executes it and
    copies the hits back (D2H), with `workers` batches in flight on their own
    streams so host planning overlaps the kernels of the other batches."""
    import threading
    batches = [synth.queries(nq, 3, 3, seed_q=1000 + i) for i in range(steps + workers)]
    streams = [torch.cuda.Stream(dev) for _ in range(workers)]
    plan_ms, errors = [], []

    def work(w, idxs):
        try:
            for i in idxs:
                t1 = time.perf_counter()
                p = ix.plan(batches[i][0], batches[i][1], K)
                plan_ms.append((time.perf_counter() - t1) * 1e3)
                p.execute(streams[w].cuda_stream)
                p.results()
                p.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    def run(idxs_all):
        th = [threading.Thread(target=work, args=(w, idxs_all[w::workers])) for w in range(workers)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    run(list(range(steps, steps + workers)))  # warm the workspace pool and the streams
    plan_ms.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(list(range(steps)))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if errors:
        raise RuntimeError(errors[0])
    return {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_batch": round(el * 1e3 / steps, 3),
            "batches": steps, "batch": nq, "k": K, "workers": workers,
            "plan_ms_per_batch_p50": round(float(np.median(plan_ms)), 3),
            "note": "each step = a different 3-term AND batch: host planning + H2D + k_conj + k_final + D2H of the "
                    "hits, pipelined over the workers' streams (planning overlaps other batches' kernels)"}


def bench_db_api(ctx, corp, native, synth, ref, threads, nq=200, n_seg=8):
    """The default API shape end to end through the host mirror: a 10M-doc
    namespace ingested by n_seg POST /batch/upsert calls (one commit, one
    segment each: src/db/document.rs:65), then batch-of-one GET /search?q=a b
    (bare terms = Should, limit 20: src/server/handlers/search.rs:36, 370-374;
    src/db/search.rs:112) through fg_db_search: parse, dictionary, ONE
    fg_search_sharded over the 8 segments (shared thresholds, device merge),
    hits out; and the same query through the full handler (JSON with the 20
    docs fetched).  Parity sample: the oracle's top-20 (an OR does not depend
    on the segmentation)."""
    from fugu_amd import db as fdb
    t0 = time.time()
    d = fdb.Database(ctx)
    d.create_namespace("api")
    tb, to = synth.render_text(corp, threads)
    ib, io = synth.render_ids(corp.n_docs)
    bounds = [corp.n_docs * i // n_seg for i in range(n_seg + 1)]
    for a, b in zip(bounds[:-1], bounds[1:]):
        d.upsert_batch("api", id_buf=ib[int(io[a]):int(io[b])], id_off=io[a:b + 1] - io[a],
                       text_buf=tb[int(to[a]):int(to[b])], text_off=to[a:b + 1] - to[a])
    del tb, ib
    ingest_s = time.time() - t0
    q_off, terms = synth.queries(nq, 2, 5, seed_q=333)
    qs = [" ".join(f"t{t}" for t in terms[q_off[i]:q_off[i + 1]]) for i in range(nq)]
    for q in qs[:8]:
        d.search("api", q, 0, 20)
    lat, lat_json, mism = [], [], 0
    for i, q in enumerate(qs):
        t1 = time.perf_counter()
        got = d.search("api", q, 0, 20)
        lat.append(time.perf_counter() - t1)
        t1 = time.perf_counter()
        d.search_json("api", q, 0, 20)
        lat_json.append(time.perf_counter() - t1)
        if ref is not None:
            rs, rd = ref.search(terms[q_off[i]:q_off[i + 1]], 20, mode=1)
            if [g[1] for g in got] != rd.tolist() or not np.allclose([g[0] for g in got], rs, rtol=1e-5, atol=0):
                mism += 1
    pct = lambda v, p: round(float(np.percentile(v, p) * 1e3), 4)  # noqa: E731
    out = {"p50_ms": pct(lat, 50), "p90_ms": pct(lat, 90), "p99_ms": pct(lat, 99),
           "json_p50_ms": pct(lat_json, 50), "json_p99_ms": pct(lat_json, 99), "queries": nq, "segments": n_seg,
           "k": 20, "mode": "OR (bare terms)", "ingest_s": round(ingest_s, 1), "n_docs": corp.n_docs,
           "note": "batch of one through fg_db_search (parse + dictionary + fg_search_sharded over the namespace's "
                   "8 commit segments + device merge + hits out); json_*: the GET /search handler shape with the "
                   "20 docs fetched from the host doc store"}
    if ref is not None:
        out["parity"] = {"queries_checked": nq, "mismatches": mism}
    d.close()
    return out


def fanout(plans, gs, gd, gn, streams, torch, dev):
    """One fan-out step's shard executes: every shard's plan on its own stream
    (the shards are independent, so one shard's tail overlaps the next one's
    start), joined back into torch's current stream before the merge."""
    main = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    ev.record(main)
    for r, p in enumerate(plans):
        s = streams[r % len(streams)]
        s.wait_event(ev)
        p.execute(s.cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
    for s in streams:
        main.wait_stream(s)


def merge_ms(gs, gd, gn, nq, K, torch, reps=20):
    """Device time of one fg_merge_shards call on the gathered lists (torch's
    current stream, where merge_on_device launches it)."""
    from fugu_amd.shard import merge_on_device
    st = torch.cuda.current_stream(gs.device)
    merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
    e1.record(st)
    e1.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def bench_c4(ctx, corp, native, synth, torch, dev, nq, K, steps, warmup, threads):
    """C4 (BASELINE configs[3]) on one GPU: the 10M docs as 8 namespaces x
    1.25M, each its own index and statistics; a step = one fan-out 3-term AND
    top-100 batch on all 8 namespaces + the device merge of the 8 top-100 lists
    (what each GPU of the 8-GPU run does for its namespace, then the RCCL
    gather's merge)."""
    from fugu_amd.shard import merge_on_device, shard_ranges
    q_off, terms = synth.queries(nq, 3, 3)
    ranges = shard_ranges(corp.n_docs, 8)
    ixs, plans = [], []
    t0 = time.time()
    for b, e in ranges:
        off = corp.off[b:e + 1] - corp.off[b]
        ix = native.Index.from_docs(ctx, off, corp.tok[corp.off[b]:corp.off[e]], synth.VOCAB, threads=threads,
                                    keep_host=False)
        ixs.append(ix)
        plans.append(ix.plan(q_off, terms, K))
    build_s = time.time() - t0
    gs = torch.empty((8, nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((8, nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((8, nq), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    streams = [torch.cuda.Stream(dev) for _ in range(8)]

    def step_seq():
        for r, p in enumerate(plans):
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        merge_on_device(gs, gd, gn, nq, K, st)

    def step_fan():
        fanout(plans, gs, gd, gn, streams, torch, dev)
        merge_on_device(gs, gd, gn, nq, K, st)

    # per-namespace kernel times from back-to-back launches; then the 8
    # namespaces on 8 streams; then the step: ONE multi-snapshot plan over the 8
    # namespaces (one launch per kernel, shared score-only thresholds), the plan
    # fg_search_sharded runs for a device's namespaces
    for p in plans:
        p.profile(True)
    el_seq = timed_steps(step_seq, steps, warmup, torch)
    kms = [p.kernel_ms() for p in plans]
    per_ns = [round(m[0][0] / max(m[1], 1), 4) for m in kms]
    for p in plans:
        p.profile(False)
    el_fan = timed_steps(step_fan, steps, warmup, torch)
    mp = native.Plan(ixs, q_off, terms, K)
    os_, od_, osh_ = (torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32))
    on_ = torch.empty(nq, dtype=torch.int32, device=dev)

    def step():  # the merged select: the merged lists straight from k_final
        mp.execute_merged(st, os_.data_ptr(), od_.data_ptr(), osh_.data_ptr(), on_.data_ptr())

    mp.profile(True)
    el = timed_steps(step, steps, warmup, torch)
    mk, mkn = mp.kernel_ms()
    mms = merge_ms(gs, gd, gn, nq, K, torch)
    # the same fan-out through the ABI call a host makes: fg_search_sharded
    # (host batch in, merged host hits out: 8 plans, 8 executes, merge, D2H)
    ms_, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, st)
    torch.cuda.synchronize()
    native.search_sharded(ixs, q_off, terms, K)
    t0 = time.perf_counter()
    for _ in range(steps):
        s2, d2, sh2, n2 = native.search_sharded(ixs, q_off, terms, K)
    sharded_ms = (time.perf_counter() - t0) * 1e3 / steps
    mn = mn.cpu().numpy()
    same = bool(np.array_equal(n2, mn))
    ms_, md, msh = (x.cpu().numpy().reshape(nq, K) for x in (ms_, md, msh))
    for i in range(nq):
        m = int(mn[i])
        same = same and np.array_equal(s2[i, :m], ms_[i, :m]) and np.array_equal(
            d2[i, :m], md[i, :m].view(np.uint32)) and np.array_equal(sh2[i, :m], msh[i, :m].astype(np.uint32))
    del plans, mp
    for ix in ixs:
        ix.close()
    return {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_step": round(el * 1e3 / steps, 4),
            "batch": nq, "k": K, "terms": 3, "mode": "AND", "namespaces": 8, "docs_per_namespace": ranges[0][1],
            "step": "one multi-snapshot plan over the 8 namespaces (fg_plan_create_multi) and its merged select "
                    "(fg_plan_execute_merged)",
            "multi_plan_kernels_ms": [round(mk[0] / max(mkn, 1), 4), round(mk[1] / max(mkn, 1), 4)],
            "k_conj_ms_per_namespace": per_ns, "merge_ms": mms, "snapshot_build_s": round(build_s, 1),
            "ms_per_step_8_plans_8_streams": round(el_fan * 1e3 / steps, 4),
            "ms_per_step_8_plans_one_stream": round(el_seq * 1e3 / steps, 4),
            "fg_search_sharded": {"value": round(nq / sharded_ms * 1e3, 1), "ms_per_batch": round(sharded_ms, 4),
                                  "same_hits_as_step": same,
                                  "note": "one synchronous ABI call per batch: host planning of 8 namespaces "
                                          "(in parallel), one multi-snapshot plan, device merge, D2H"},
            "workload": "C4: 10M docs as 8 namespaces x 1.25M (own statistics each), fan-out 3-term AND top-100 "
                        "on all 8 + device merge, all 8 namespaces on this one GPU",
            "projected_8gpu": "each GPU runs one namespace: step ~ max(k_conj_ms_per_namespace) + k_final + gather"}


def bench_c5(ctx, native, synth, torch, dev, nq, steps, warmup, threads, cpu_seconds, do_cpu):
    """C5 (BASELINE configs[4]) on one GPU: 100M docs, Zipf s=1.1, as 8
    contiguous doc shards scored with the GLOBAL statistics (tantivy's segment
    model); a step = one 2-5-term OR top-1000 batch on all 8 shards + the device
    merge by (score desc, shard asc, doc asc)."""
    from fugu_amd.shard import merge_on_device, shard_ranges
    K, N, S = 1000, 100_000_000, 1.1
    t0 = time.time()
    c = synth.corpus(N, synth.VOCAB, S, threads=threads)
    ranges = shard_ranges(N, 8)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, synth.VOCAB, threads=threads)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=threads, keep_host=False, global_stats=g)
           for off, tok in parts]
    del parts
    build_s = time.time() - t0
    log(f"[bench] C5: 100M docs as 8 shards built in {build_s:.1f}s")
    q_off, terms = synth.queries(nq, 2, 5)
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    native.link_plans(plans)
    gs = torch.empty((8, nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((8, nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((8, nq), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    merged = {}

    # the round-2/3 step: 8 linked plans back to back on one stream (per-shard times)
    def step_linked():
        for r, p in enumerate(plans):
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        merge_on_device(gs, gd, gn, nq, K, st)

    for p in plans:
        p.profile(True)
    el_linked = timed_steps(step_linked, max(2, steps // 2), 1, torch)
    kms = [p.kernel_ms() for p in plans]
    per_shard = [round(m[0][0] / max(m[1], 1), 4) for m in kms]
    del plans
    # the step: ONE multi-snapshot plan over the 8 shards (one launch per kernel)
    mp = native.Plan(ixs, q_off, terms, K, native.MODE_OR)
    outs = tuple(torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)) + (
        torch.empty(nq, dtype=torch.int32, device=dev),)

    def step():  # the merged select: the merged lists straight from k_final
        mp.execute_merged(st, *[x.data_ptr() for x in outs])
        merged["out"] = outs

    mp.profile(True)
    el = timed_steps(step, steps, warmup, torch)
    mk, mkn = mp.kernel_ms()
    mms = merge_ms(gs, gd, gn, nq, K, torch)
    ent = {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_step": round(el * 1e3 / steps, 4),
           "batch": nq, "k": K, "terms": "2-5", "mode": "OR", "n_docs": N, "zipf_s": S, "shards": 8,
           "step": "one multi-snapshot plan over the 8 shards (fg_plan_create_multi) and its merged select "
                   "(fg_plan_execute_merged)",
           "multi_plan_kernels_ms": [round(mk[0] / max(mkn, 1), 4), round(mk[1] / max(mkn, 1), 4)],
           "ms_per_step_8_linked_plans": round(el_linked * 1e3 / max(2, steps // 2), 4),
           "k_disj_ms_per_shard_linked": per_shard, "merge_ms": mms, "snapshot_build_s": round(build_s, 1),
           "workload": "C5: 100M docs s=1.1 as 8 doc shards with global BM25 statistics, 2-5-term OR top-1000 on "
                       "all 8 + device merge, all 8 shards on this one GPU",
           "projected_8gpu": "each GPU runs one shard: step ~ max(k_disj_ms_per_shard) + k_final + gather"}
    del mp
    for ix in ixs:
        ix.close()
    if do_cpu:
        # CPU baseline + parity on a bounded sample: ONE 100M-doc oracle index
        from oracle import oracle as orc
        ms_, md, msh, mn = merged["out"]
        base = np.array([b for b, _ in ranges], np.uint64)
        ms_ = ms_.cpu().numpy().reshape(nq, K)
        gdoc = md.cpu().numpy().view(np.uint32).reshape(nq, K).astype(np.uint64) + base[
            msh.cpu().numpy().reshape(nq, K)]
        mn = mn.cpu().numpy()
        ref = orc.OracleIndex(synth.VOCAB, c.off, c.tok, threads=threads)
        done, wall, mism = 0, 0.0, 0
        while done < nq and wall < cpu_seconds:
            hi = min(nq, done + threads)
            so = (q_off[done:hi + 1] - q_off[done]).astype(np.uint32)
            rs, rd, rn, w, _ = ref.search_batch(so, terms[q_off[done]:q_off[hi]], K, mode=orc.OR, threads=threads)
            wall += w
            for j in range(hi - done):
                i, m = done + j, int(rn[j])
                if (int(mn[i]) != m or not np.array_equal(gdoc[i, :m], rd[j, :m].astype(np.uint64))
                        or not np.allclose(ms_[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                    mism += 1
            done = hi
        ent["cpu_baseline"] = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads, "kind": "port",
                               "sample": f"first {done} queries of the batch on ONE 100M-doc oracle index "
                                         "(exhaustive union, SumCombiner)"}
        ent["parity"] = {"queries_checked": done, "mismatches": mism}
        del ref
    return ent


def pmc_traffic(path, kname, workload):
    """(HBM bytes per launch of `kname`, source) from a committed rocprofv3 PMC summary when
    its lib_id is this build's and its workload matches, else None."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pmc = json.load(f)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from lib_id import lib_id
    wl = pmc.get("workload", {})
    if pmc.get("lib_id") != lib_id() or any(wl.get(k) != v for k, v in workload.items()):
        log(f"[bench] {path} does not match this build/workload: no measured traffic for {kname}")
        return None
    v = pmc.get(f"{kname}_hbm_bytes_per_launch")
    return (v, pmc.get("source")) if v else None


def run_config(args, cfg, rank, world, local, dev, backend, threads, torch, dist):
    """BASELINE configs[3] (c4) / configs[4] (c5) across the job's GPUs (strong
    scaling: the corpus is fixed, its 8 units are split over the ranks):
      c4: the 10M-doc corpus as 8 namespaces x 1.25M (own statistics each), a
          fan-out 3-term AND top-100 batch;
      c5: 100M docs, Zipf s = 1.1, as 8 doc shards scored with the namespace's
          global statistics (one all-reduce of the shard statistics at build),
          a 2-5-term OR top-1000 batch.
    Rank r holds units [8r/N, 8(r+1)/N) on its GPU, their plans linked (one
    shared threshold per query); a step = every unit's kernels, the rank's
    device merge, ONE all-gather of the rank lists (RCCL over xGMI) and the
    final device merge by (score desc, unit asc, doc asc).  Every rank prints
    nothing; rank 0 prints the JSON line, with a hash of the merged hits (equal
    for every N)."""
    import hashlib

    from fugu_amd import native, synth
    from fugu_amd.shard import allreduce_stats, gather_packed, merge_on_device, shard_ranges
    c4 = cfg == "c4"
    N, S, K = (10_000_000, 1.0, 100) if c4 else (100_000_000, 1.1, 1000)
    mode = native.MODE_AND if c4 else native.MODE_OR
    nq = args.batch
    units = 8
    if units % world:
        raise SystemExit(f"--config {cfg}: {units} units do not split over {world} ranks")
    ranges = shard_ranges(N, units)
    per = units // world
    mine = list(range(rank * per, (rank + 1) * per))
    t0 = time.time()
    parts = []
    for u in mine:
        b, e = ranges[u]
        c = synth.corpus(e - b, synth.VOCAB, S, doc_begin=b, threads=threads)
        parts.append((c.off, c.tok))
    ctx = native.Context((local,))
    g = None
    if not c4:  # global statistics: the rank's shards summed, then one all-reduce over the ranks
        for off, tok in parts:
            x = native.docs_stats(off, tok, synth.VOCAB, threads=threads)
            g = x if g is None else g + x
        if world > 1:
            g = allreduce_stats(g, device=dev if backend == "nccl" else None)
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=threads, keep_host=False, global_stats=g)
           for off, tok in parts]
    del parts
    build_s = time.time() - t0
    log(f"[bench] {cfg}: rank {rank} built units {mine} in {build_s:.1f}s")
    q_off, terms = synth.queries(nq, 3, 3) if c4 else synth.queries(nq, 2, 5)
    # a rank's units: ONE multi-snapshot plan (one launch per kernel, shared
    # score-only thresholds); FUGU_BENCH_LINKED=1: one linked plan per unit (A/B)
    if len(ixs) > 1 and os.environ.get("FUGU_BENCH_LINKED") != "1":
        plans = [native.Plan(ixs, q_off, terms, K, mode)]
    else:
        plans = [ix.plan(q_off, terms, K, mode) for ix in ixs]
        if len(plans) > 1:
            native.link_plans(plans)
    gs = torch.empty((len(ixs), nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((len(ixs), nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((len(ixs), nq), dtype=torch.int32, device=dev)
    # unit u's doc d as a global id: c5 the corpus doc id, c4 (namespace << 24) | doc
    off_u = torch.tensor([ranges[u][0] if not c4 else (u << 24) for u in mine], dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    out = {}

    merged_sel = len(plans) == 1 and len(ixs) > 1
    mouts = [torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)] + [
        torch.empty(nq, dtype=torch.int32, device=dev)]

    def step():
        if merged_sel:  # the rank's units merged by the plan's own final select
            plans[0].execute_merged(st.cuda_stream, *[x.data_ptr() for x in mouts])
            ms, md, msh, mn = mouts
        else:
            for r, p in enumerate(plans):  # plans[0] first: it zeroes the shared thresholds
                p.execute(st.cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
            ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
        # slots past a query's count hold no hit (undefined shard / doc): clamp the
        # gather index so it stays inside off_u; those slots are never read
        gdoc = (md.to(torch.int64) + off_u[msh.to(torch.int64).clamp_(0, len(mine) - 1)]).to(torch.int32)
        if world > 1:
            s2, d2, c2 = gather_packed(ms, gdoc, mn)
            out["m"] = merge_on_device(s2, d2, c2, nq, K, st.cuda_stream)
        else:
            out["m"] = (ms, gdoc, None, mn)

    for p in plans:
        p.profile(True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    for p in plans:
        p.kernel_ms()  # drop the warmup's events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    kms = [p.kernel_ms() for p in plans]
    kern = sum(m[0][0] for m in kms) / max(kms[0][1], 1)
    fin = sum(m[0][1] for m in kms) / max(kms[0][1], 1)
    if world > 1:
        t = torch.tensor([el, kern], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern = float(t[0].item()), float(t[1].item())
    ms, md, _, mn = out["m"]
    mn = mn.cpu().numpy()
    ms = ms.cpu().numpy().reshape(nq, K)
    md = md.cpu().numpy().view(np.uint32).reshape(nq, K)
    h = hashlib.sha1()
    for i in range(nq):
        h.update(md[i, :mn[i]].tobytes())
        h.update(ms[i, :mn[i]].tobytes())
    if rank == 0:
        kname = "k_conj" if c4 else "k_disj"
        line = {
            "metric": METRIC, "value": round(nq * args.steps / el, 1), "unit": "queries/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32+f32",
            "data": "synthetic",
            "config": {"workload": ("C4: 10M docs as 8 namespaces x 1.25M, fan-out 3-term AND top-100"
                                    if c4 else "C5: 100M docs Zipf s=1.1 as 8 doc shards (global BM25 statistics), "
                                               "2-5-term OR top-1000"),
                       "n_docs": N, "batch": nq, "k": K, "units": units, "units_per_gpu": per,
                       "parallelism": f"{'namespace' if c4 else 'doc'}-shard x{world}" + (
                           (" + RCCL all-gather top-k" if backend == "nccl" else f" + {backend} all-gather (rehearsal)")
                           if world > 1 else "")},
            "kernels_ms_per_step_max_rank": {kname: round(kern, 4), "k_final": round(fin, 4)},
            "rank_plan": ("one multi-snapshot plan over the rank's units, merged by its final select"
                          if merged_sel else f"{len(plans)} linked plan(s) + k_merge_rank"),
            "result_sha1": h.hexdigest()[:16],
            "hits": int(mn.sum()),
            "snapshot_build_s_rank0": round(build_s, 1),
            "cpu_baseline": None,
            "note": "strong scaling of one fixed corpus; the headline mode (no --config) carries the CPU baseline "
                    "and the roofline",
        }
        print(json.dumps(line), flush=True)
    del plans[1:]
    del plans


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--terms", type=int, default=3)
    ap.add_argument("--mixed", action="store_true", help="1-5 terms per query (config C3) instead of 3")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--p50-queries", type=int, default=200)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary workloads (C3, OR top-1000, end-to-end, C4, C5)")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--no-c5", action="store_true", help="skip the 100M-doc C5 secondary line")
    ap.add_argument("--e2e-workers", type=int, default=4,
                    help="batches in flight in the end-to-end line (tools/e2e_workers.py with the radix planner: "
                         "1 -> 697K, 2 -> 816K, 4 -> 934K, 8 -> 868K q/s)")
    ap.add_argument("--disj", action="store_true",
                    help="headline batch = 2-5-term OR (k_disj; profiling runs, pass --k 1000 --no-cpu)")
    ap.add_argument("--overlap", action="store_true",
                    help="N > 1: each step's gather + merge on a side stream behind the next batch (opt-in: a gloo "
                         "rehearsal on one GPU measured it slower, RCCL unmeasured)")
    ap.add_argument("--config", choices=["headline", "c4", "c5"], default="headline",
                    help="c4 / c5: BASELINE configs[3] / [4] split over the job's GPUs (strong scaling)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; FUGU_DIST_BACKEND=gloo rehearses the N>1 flow with
    # several ranks on fewer GPUs (the driver's runs use RCCL, one GPU each)
    backend = os.environ.get("FUGU_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from fugu_amd import native, synth

    cores = host_cores()
    threads = args.threads or cores["nproc"]
    if args.config != "headline":
        run_config(args, args.config, rank, world, local, dev, backend, threads, torch, dist)
        if world > 1:
            dist.destroy_process_group()
        return
    t0 = time.time()
    # namespace r: its own corpus (seeds offset by rank); rank 0 is the standard corpus
    corp = synth.corpus(args.docs, synth.VOCAB, 1.0, synth.SEED_L + rank, synth.SEED_T + rank, threads=threads)
    log(f"[bench] corpus {args.docs} docs, {len(corp.tok)} tokens in {time.time() - t0:.1f}s")
    t0 = time.time()
    ctx = native.Context((local,))
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=threads, keep_host=True)
    st = ix.stats()
    log(f"[bench] index: {st.n_postings} postings, {st.device_bytes / 2**30:.2f} GiB in HBM, built in "
        f"{time.time() - t0:.1f}s")

    m_min, m_max = (1, 5) if args.mixed else (2, 5) if args.disj else (args.terms, args.terms)
    qmode = native.MODE_OR if args.disj else native.MODE_AND
    kname = "k_disj" if args.disj else "k_conj"
    wl_terms = "1-5" if args.mixed else "2-5 OR" if args.disj else args.terms
    q_off_all, terms_all = synth.queries(4096, m_min, m_max)
    nq = args.batch
    q_off = q_off_all[: nq + 1].copy()
    terms = terms_all[: q_off[-1]].copy()
    K = args.k
    plan = ix.plan(q_off, terms, K, qmode)
    info = plan.info()
    log(f"[bench] plan: {info.total_chunks} work items, workspace {info.workspace_bytes / 2**20:.1f} MiB")

    out_s = torch.empty(nq * K, dtype=torch.float32, device=dev)
    out_d = torch.empty(nq * K, dtype=torch.int32, device=dev)
    out_n = torch.empty(nq, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    merged = {}  # N > 1: the last step's merged lists (result_sha1)

    def step():
        plan.execute(stream.cuda_stream, out_s.data_ptr(), out_d.data_ptr(), out_n.data_ptr())
        if world > 1:
            from fugu_amd.shard import gather_packed, merge_on_device
            s, d, c = gather_packed(out_s, out_d, out_n)
            merged["m"] = merge_on_device(s, d, c, nq, K, stream.cuda_stream)

    if world > 1 and args.overlap:
        # N > 1: a step's all-gather + merge run on a side stream while the next
        # step's batch runs (two output buffers in turn; a buffer is reused only
        # after its gather has read it), so the collective hides behind the kernels
        from fugu_amd.shard import gather_packed, merge_on_device
        side = torch.cuda.Stream(dev)
        bufs = [(torch.empty(nq * K, dtype=torch.float32, device=dev), torch.empty(nq * K, dtype=torch.int32, device=dev),
                 torch.empty(nq, dtype=torch.int32, device=dev)) for _ in range(2)]
        gathered = [None, None]
        turn = [0]

        def step():  # noqa: F811
            b = turn[0] % 2
            turn[0] += 1
            s_, d_, n_ = bufs[b]
            if gathered[b] is not None:
                stream.wait_event(gathered[b])
            plan.execute(stream.cuda_stream, s_.data_ptr(), d_.data_ptr(), n_.data_ptr())
            ran = torch.cuda.Event()
            ran.record(stream)
            side.wait_event(ran)
            with torch.cuda.stream(side):
                s, d, c = gather_packed(s_, d_, n_)
                merged["m"] = merge_on_device(s, d, c, nq, K, side.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(side)
                gathered[b] = ev

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    plan.profile(False)
    ms_k, n_prof = plan.kernel_ms()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_queries = nq * world * args.steps
    result_sha1 = None
    if world > 1 and "m" in merged:  # the merged lists of the last step (equal with and without --overlap)
        import hashlib
        ms_, md_, msh_, mn_ = (x.cpu().numpy() for x in merged["m"])
        h = hashlib.sha1()
        for i in range(nq):
            m = int(mn_[i])
            h.update(ms_[i * K:i * K + m].tobytes() + md_[i * K:i * K + m].tobytes() + msh_[i * K:i * K + m].tobytes())
        result_sha1 = h.hexdigest()[:16]
    qps = total_queries / elapsed

    # ---- p50 latency at batch = 1 (host query in, host hits out: plan + PCIe + kernels)
    lat = []
    for i in range(min(args.p50_queries, nq)):
        a, b = int(q_off[i]), int(q_off[i + 1])
        one_off = np.array([0, b - a], np.uint32)
        t1 = time.perf_counter()
        ix.search_batch(one_off, terms[a:b], K)
        lat.append(time.perf_counter() - t1)
    p50_ms = float(np.median(lat) * 1e3) if lat else None
    tail_ms = {f"p{q}": round(float(np.percentile(lat, q) * 1e3), 4) for q in (90, 99)} if lat else None

    # ---- roofline of the dominant kernel (k_conj): algorithmic bytes at the HBM
    # layout (fg_bytes_model_gpu: k_conj's exhaustive cascade) over
    # its HIP-event time on the launch stream.  The SURVEY 8(d) tantivy byte
    # model (1 KiB block decode per probed block) is reported beside it, labelled.
    if args.disj:
        # k_disj: MaxScore bytes at each query's final k-th score (fg_bytes_model_or)
        s_h = out_s.cpu().numpy().reshape(nq, K)
        n_h = out_n.cpu().numpy()
        bmg = ix.bytes_model_or(q_off, terms, K, np.where(n_h >= K, s_h[:, K - 1], 0.0).astype(np.float32))
    else:
        bmg = ix.bytes_model_gpu(q_off, terms, K, qmode)
    alg_bytes = float(bmg[:, 3].sum())
    # (FG_MODE_OR: the exhaustive union is both models)
    cpu_model_bytes = alg_bytes if args.disj else float(ix.bytes_model(q_off, terms, K)[:, 2].sum())
    conj_ms = ms_k[0] / max(n_prof, 1)
    achieved = alg_bytes / (conj_ms * 1e-3) / 1e9
    # HBM bytes per k_conj launch from rocprofv3 PMC (FETCH_SIZE with the
    # gather-calibrated gfx950 correction + WRITE_SIZE), collected by
    # tools/profile_bench.sh on this exact workload and build, committed under
    # profiles/ (profiles/latest.json)
    traffic, pmc = None, {}
    pmc_file = os.environ.get("FUGU_PMC_BYTES") or os.path.join(ROOT, "profiles", "latest.json")
    if os.path.exists(pmc_file):
        with open(pmc_file) as f:
            pmc = json.load(f)
        wl = pmc.get("workload", {})
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from lib_id import lib_id
        same_build = pmc.get("lib_id") == lib_id()
        if same_build and (not wl or (wl.get("n_docs") == args.docs and wl.get("batch") == nq and wl.get("k") == K
                                      and wl.get("terms") == wl_terms)):
            traffic = pmc.get(f"{kname}_hbm_bytes_per_launch")
        else:
            log(f"[bench] {pmc_file} does not match this build/workload: roofline.traffic = null")

    # ---- CPU baseline: the oracle (tantivy's algorithm restated in C, compiled
    # -march=native on this host) on T = nproc host threads, each running whole
    # queries (a tokio worker per request, tantivy's single-threaded executor),
    # plus a T = 1 row; rank 0, N = 1 only, bounded samples of the same batch
    cpu = None
    parity = None
    ref = None
    s_gpu = out_s.cpu().numpy().reshape(nq, K)
    d_gpu = out_d.cpu().numpy().view(np.uint32).reshape(nq, K)
    n_gpu = out_n.cpu().numpy()
    if rank == 0 and world == 1 and not args.no_cpu:
        flags = native_oracle()
        from oracle import oracle as orc
        t0 = time.time()
        ref = orc.OracleIndex(synth.VOCAB, corp.off, corp.tok, threads=threads)
        log(f"[bench] oracle index built in {time.time() - t0:.1f}s ({flags})")

        def cpu_run(T, budget, step):
            done, wall, lats, mism = 0, 0.0, [], 0
            while done < nq and wall < budget:
                hi = min(nq, done + step)
                sub_off = (q_off[done:hi + 1] - q_off[done]).astype(np.uint32)
                rs, rd, rn, w, l = ref.search_batch(sub_off, terms[q_off[done]:q_off[hi]], K, threads=T,
                                                    latencies=True)
                wall += w
                lats.append(l)
                for j in range(hi - done):
                    i, m = done + j, int(rn[j])
                    if (int(n_gpu[i]) != m or not np.array_equal(d_gpu[i, :m], rd[j, :m])
                            or not np.allclose(s_gpu[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                        mism += 1
                done = hi
            return done, wall, float(np.median(np.concatenate(lats))) * 1e-6, mism

        done, wall, p50_cpu, mism = cpu_run(threads, args.cpu_seconds, 128)
        d1, w1, p1, m1 = cpu_run(1, args.cpu_seconds / 4, 16)
        cpu = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads, "kind": "port",
               "sample": f"first {done} queries of the same 1024-query batch, {threads} threads x whole queries, "
                         f"warm in-RAM index (tantivy 0.24.1 algorithm restated in C: oracle/fugu_oracle.c)",
               "p50_ms": round(p50_cpu, 4), "compile": f"gcc {flags}", "host": cores,
               "t1": {"value": round(d1 / w1, 2), "unit": "queries/s", "cores": 1, "p50_ms": round(p1, 4),
                      "sample": f"first {d1} queries of the batch, 1 thread"}}
        parity = {"queries_checked": done, "mismatches": mism + m1, "rule": "doc ids exact, scores rtol 1e-5"}

    # ---- secondary workloads on the same index (rank 0, N=1): SURVEY §8(d) C3 and the
    # disjunctive C5 query shape (k_disj), each timed the same way and parity-sampled
    extra = None
    if rank == 0 and world == 1 and not args.no_extra:
        extra = {}
        specs = [("C3_mixed_and", 1, 5, 100, native.MODE_AND), ("OR_top1000_10M", 2, 5, 1000, native.MODE_OR),
                 ("OR_top20_default_api", 2, 5, 20, native.MODE_OR)]
        for name, a_min, a_max, kk, mode in specs:
            qo_all, qt_all = synth.queries(4096, a_min, a_max)
            qo = qo_all[: nq + 1].copy()
            qt = qt_all[: qo[-1]].copy()
            pl2 = ix.plan(qo, qt, kk, mode=mode)
            os2 = torch.empty(nq * kk, dtype=torch.float32, device=dev)
            od2 = torch.empty(nq * kk, dtype=torch.int32, device=dev)
            on2 = torch.empty(nq, dtype=torch.int32, device=dev)
            for _ in range(2):
                pl2.execute(stream.cuda_stream, os2.data_ptr(), od2.data_ptr(), on2.data_ptr())
            torch.cuda.synchronize()
            pl2.profile(True)
            t1 = time.perf_counter()
            for _ in range(args.extra_steps):
                pl2.execute(stream.cuda_stream, os2.data_ptr(), od2.data_ptr(), on2.data_ptr())
            torch.cuda.synchronize()
            el = time.perf_counter() - t1
            pl2.profile(False)
            kms, kn = pl2.kernel_ms()
            dfs = np.array([ix.df(int(t)) for t in qt], np.float64)
            merge_bytes = 8.0 * dfs.sum()  # every posting of every clause once (exhaustive merge/union)
            s2 = os2.cpu().numpy().reshape(nq, kk)
            d2 = od2.cpu().numpy().view(np.uint32).reshape(nq, kk)
            n2 = on2.cpu().numpy()
            ent = {"value": round(nq * args.extra_steps / el, 1), "unit": "queries/s",
                   "ms_per_step": round(el * 1e3 / args.extra_steps, 4), "batch": nq, "k": kk,
                   "terms": f"{a_min}-{a_max}", "mode": "AND" if mode == native.MODE_AND else "OR",
                   "kernel": "k_conj" if mode == native.MODE_AND else "k_disj",
                   "kernel_ms": round(kms[0] / max(kn, 1), 4), "k_final_ms": round(kms[1] / max(kn, 1), 4),
                   "merge_bytes_per_launch": merge_bytes,
                   "merge_equiv_gbs": round(merge_bytes / (kms[0] / max(kn, 1) * 1e-3) / 1e9, 1)}
            if mode == native.MODE_OR:
                # device-layout MaxScore bytes at each query's final k-th score (fg_bytes_model_or):
                # the least an exact k_disj reads, over the kernel's time
                thr = np.where(n2 >= kk, s2[:, kk - 1], 0.0).astype(np.float32)
                bo = ix.bytes_model_or(qo, qt, kk, thr)
                kms_ = kms[0] / max(kn, 1)
                ent["roofline"] = {"bound": "hbm", "kernel": "k_disj", "alg_bytes_per_launch": float(bo[:, 3].sum()),
                                   "alg_bytes_split": {"stream": float(bo[:, 0].sum()), "probe": float(bo[:, 1].sum()),
                                                       "output": float(bo[:, 2].sum())},
                                   "achieved": round(float(bo[:, 3].sum()) / (kms_ * 1e-3) / 1e9, 1),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(float(bo[:, 3].sum()) / (kms_ * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "alg_model": "fg_bytes_model_or: MaxScore over 4096-doc tiles at the final k-th "
                                                "score (12 B per tile-clause bound, 8 B per essential posting, rank "
                                                "word / bucket max per posting past the tile bound, 4 B score per "
                                                "present clause past the presence bound, 8 B per kept key)"}
                # measured DRAM bytes per k_disj launch (rocprofv3 PMC of `bench.py --disj --k 1000`,
                # profiles/latest_or.json) when it was taken on this build and workload
                tr = pmc_traffic(os.path.join(ROOT, "profiles", "latest_or.json"), "k_disj",
                                 {"n_docs": args.docs, "batch": nq, "k": kk, "terms": "2-5 OR"})
                if tr:
                    ent["roofline"].update({"traffic": tr[0], "traffic_source": tr[1],
                                            "traffic_over_alg": round(tr[0] / float(bo[:, 3].sum()), 3),
                                            "hbm_gbs_measured": round(tr[0] / (kms_ * 1e-3) / 1e9, 1)})
            if ref is not None:
                done, wall, mism = 0, 0.0, 0
                budget = args.cpu_seconds / 2
                while done < nq and wall < budget:
                    hi = min(nq, done + 32)
                    so = (qo[done:hi + 1] - qo[done]).astype(np.uint32)
                    rs, rd, rn, w, _ = ref.search_batch(so, qt[qo[done]:qo[hi]], kk, mode=mode, threads=threads)
                    wall += w
                    for j in range(hi - done):
                        i, m = done + j, int(rn[j])
                        if (int(n2[i]) != m or not np.array_equal(d2[i, :m], rd[j, :m])
                                or not np.allclose(s2[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                            mism += 1
                    done = hi
                ent["cpu_baseline"] = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads,
                                       "kind": "port",
                                       "sample": f"first {done} queries of the batch, oracle/fugu_oracle.c "
                                                 f"({'leapfrog intersection' if mode == native.MODE_AND else 'exhaustive union, SumCombiner'})"}
                ent["parity"] = {"queries_checked": done, "mismatches": mism}
            extra[name] = ent
            log(f"[bench] {name}: {ent['value']} q/s, {ent['kernel']} {ent['kernel_ms']} ms")
            del pl2

    # ---- end-to-end batches, then the fan-out configs C4 and C5 on this one GPU
    if rank == 0 and world == 1 and not args.no_extra:
        extra["e2e_pipelined"] = e2e_pipeline(ix, native, synth, torch, dev, nq, K, 24, args.e2e_workers)
        log(f"[bench] e2e pipelined: {extra['e2e_pipelined']['value']} q/s")
    if rank == 0 and world == 1 and not args.no_extra:
        extra["commit_10M"] = commit_latency(ctx, ix, corp, native, synth, threads)
        log(f"[bench] commit on the 10M namespace: {extra['commit_10M']['commit_ms']} ms")
        extra["db_api_default_search_10M_8seg"] = bench_db_api(ctx, corp, native, synth, ref, threads)
        log(f"[bench] GET /search (OR, limit 20) through fg_db_search on 8 segments: "
            f"p50 {extra['db_api_default_search_10M_8seg']['p50_ms']} ms")
    del plan
    ix.close()
    if rank == 0 and world == 1 and not args.no_extra:
        extra["C4_8ns_fanout"] = bench_c4(ctx, corp, native, synth, torch, dev, nq, K, args.extra_steps, 2, threads)
        log(f"[bench] C4: {extra['C4_8ns_fanout']['value']} q/s")
        if not args.no_c5:
            ref = None
            del corp
            extra["C5_or_top1000_100M"] = bench_c5(ctx, native, synth, torch, dev, nq, args.extra_steps, 2, threads,
                                                   args.cpu_seconds / 2, not args.no_cpu)
            log(f"[bench] C5: {extra['C5_or_top1000_100M']['value']} q/s")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(qps, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32+f32",
            "data": "synthetic",
            "config": {
                "workload": (f"{'C3 mixed 1-5' if args.mixed else '2-5-term OR' if args.disj else str(args.terms) + '-term'}"
                             f"{'' if args.disj else ' AND'}, BM25 top-{K}, "
                             f"{args.docs // 1_000_000}M-doc Zipf s=1.0 corpus per namespace, batch {nq}"),
                "n_docs": args.docs, "vocab": synth.VOCAB, "batch": nq, "k": K,
                "terms": wl_terms, "namespaces": world,
                "parallelism": f"namespace-shard x{world}" + (
                    (" + RCCL all-gather top-k" if backend == "nccl" else f" + {backend} all-gather top-k (rehearsal)")
                    + (", overlapped with the next batch" if args.overlap else "") if world > 1 else ""),
            },
            "p50_ms": round(p50_ms, 4) if p50_ms is not None else None,
            "latency_ms": tail_ms,  # batch-of-one p90 / p99 beside p50 (same sample)
            **({"result_sha1": result_sha1} if result_sha1 else {}),
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kname, "kernel_ms": round(conj_ms, 4),
                "alg_bytes_per_launch": alg_bytes,
                "alg_model": ("fg_bytes_model_or: k_disj's MaxScore at the final k-th score (DESIGN.md §5)"
                              if args.disj else
                              "fg_bytes_model_gpu: k_conj's exhaustive cascade at the HBM layout (8 B per lead "
                              "posting; per probe 8 B rank word + 4 B score on a hit, or 8 B bucket bounds + 4 B per "
                              "search step + 4 B compare + 4 B score on a hit; 8 B per kept key)"),
                "alg_bytes_split": {("stream" if args.disj else "lead"): float(bmg[:, 0].sum()),
                                    "probe": float(bmg[:, 1].sum()), "output": float(bmg[:, 2].sum())},
                "traffic_over_alg": round(traffic / alg_bytes, 3) if traffic else None,
                "traffic_source": pmc.get("source") if traffic else None,
                "hbm_gbs_measured": (round(traffic / (conj_ms * 1e-3) / 1e9, 1) if traffic else None),
                "hbm_frac_measured": (round(traffic / (conj_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None),
                "cpu_model_bytes_per_launch": cpu_model_bytes,
                "cpu_model": "SURVEY.md 8(d) B(q): tantivy's CPU walk (1 KiB block decode per probed 128-posting "
                             "block); not bytes this layout reads",
                "cpu_model_gbs": round(cpu_model_bytes / (conj_ms * 1e-3) / 1e9, 1),
            },
            "kernels_ms_per_step": {kname: round(ms_k[0] / max(n_prof, 1), 4),
                                    "k_final": round(ms_k[1] / max(n_prof, 1), 4)},
            "cpu_baseline": cpu,
            "parity": parity,
            "speedup_vs_cpu": round(qps / cpu["value"], 1) if cpu else None,
            "secondary": extra,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
