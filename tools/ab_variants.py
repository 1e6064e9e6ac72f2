"""A/B tuning builds of libfugu on the same batch, interleaved in one process
per variant round (cdna_hip_programming.md §5.4 rule 24: interleaved rounds,
report median and min).

  python tools/ab_variants.py [--docs N] [--rounds R] lib1.so lib2.so ...

Each variant is loaded in its own child process (one HIP runtime binding per
process); the child times k_conj/k_final with HIP events and hashes the
results so variants can be checked for identical output.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path.insert(0, ROOT)
    import numpy as np
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16, keep_host=False)
    m_min, m_max = (1, 5) if args.mixed else (args.terms, args.terms)
    mode = native.MODE_AND
    if args.disj:  # config C5 shape: 2-5 bare terms (Should), k = 1000
        m_min, m_max, mode = 2, 5, native.MODE_OR
    q_off, terms = synth.queries(args.batch, m_min, m_max)
    plan = ix.plan(q_off, terms, args.k, mode)
    for _ in range(2):
        plan.execute()
    plan.results()
    plan.profile(True)
    times = []
    for _ in range(args.steps):
        plan.execute()
        ms, n = plan.kernel_ms()
        times.append(ms.tolist())
    s, d, n = plan.results()
    h = hashlib.sha1()
    for i in range(len(n)):
        h.update(d[i, :n[i]].tobytes())
        h.update(s[i, :n[i]].tobytes())
    t = np.array(times)
    print(json.dumps({"lib": os.environ.get("FUGU_LIB"), "env": os.environ.get("FUGU_SWEEP_TERM"), "k_conj_ms_med": float(np.median(t[:, 0])),
                      "k_conj_ms_min": float(t[:, 0].min()), "k_final_ms_med": float(np.median(t[:, 1])),
                      "hash": h.hexdigest()[:16]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--terms", type=int, default=3)
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--disj", action="store_true", help="OR queries (k_disj), use with --k 1000")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    args = ap.parse_args()
    if args.child:
        return child(args)
    res = {}
    for r in range(args.rounds):
        for lib in args.libs:
            # "lib.so@NAME=VALUE,...": the variant is the library under that environment
            path, _, envs = lib.partition("@")
            env = dict(os.environ, FUGU_LIB=os.path.abspath(path))
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            cmd = [sys.executable, __file__, "--child", "--docs", str(args.docs), "--batch", str(args.batch),
                   "--terms", str(args.terms), "--k", str(args.k), "--steps", str(args.steps)]
            if args.mixed:
                cmd.append("--mixed")
            if args.disj:
                cmd.append("--disj")
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(json.dumps({"lib": lib, "error": out.stderr[-800:]}), flush=True)
                return 1
            line = json.loads(out.stdout.strip().splitlines()[-1])
            res.setdefault(lib, []).append(line)
            print(json.dumps({"round": r, **line}), flush=True)
    hashes = {l: v[0]["hash"] for l, v in res.items()}
    print(json.dumps({"summary": {l: min(x["k_conj_ms_med"] for x in v) for l, v in res.items()},
                      "identical_outputs": len(set(hashes.values())) == 1}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
