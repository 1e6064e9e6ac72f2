"""End-to-end batch throughput (bench.py's e2e line) against the number of
batches in flight, on the 10M-doc headline index: which worker count keeps the
GPU busy while the host plans.  python tools/e2e_workers.py [--workers 1,2,4,8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="1,2,4,8")
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--repeat", type=int, default=1)
    args = ap.parse_args()
    import torch

    import bench
    from fugu_amd import native, synth
    dev = torch.device("cuda:0")
    ctx = native.Context((0,))
    c = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, keep_host=False)
    out = {}
    for rep in range(args.repeat):
        for w in [int(x) for x in args.workers.split(",")]:
            r = bench.e2e_pipeline(ix, native, synth, torch, dev, 1024, 100, args.steps, w)
            out[w] = {k: r[k] for k in ("value", "ms_per_batch", "plan_ms_per_batch_p50", "breakdown_ms_p50",
                                        "breakdown_ms_p90")}
            print(json.dumps({"workers": w, "steps": args.steps, "rep": rep, **out[w]}), flush=True)


if __name__ == "__main__":
    main()
