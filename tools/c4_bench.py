"""bench.py's C4 line alone (bench_c4): the 10M corpus as 8 namespaces x 1.25M
on one GPU, one multi-snapshot plan per fan-out batch and its merged select.

  python tools/c4_bench.py [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    import torch

    import bench
    from fugu_amd import native, synth
    bench.NO_MODEL = True
    threads = bench.host_threads(bench.host_cores())
    dev = torch.device("cuda:0")
    ctx = native.Context((0,))
    corp = synth.corpus(10_000_000, synth.VOCAB, 1.0, threads=threads)
    ent = bench.bench_c4(ctx, corp, native, synth, torch, dev, args.batch, 100, args.steps, 2, threads)
    ent.pop("roofline", None)
    print(json.dumps(ent))


if __name__ == "__main__":
    main()
