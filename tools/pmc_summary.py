"""Per-dispatch averages of every counter in a tools/pmc_conj.sh output dir,
per kernel (k_conj, k_final, ...): {kernel: {counter: mean over dispatches}}."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ("k_conj", "k_disj", "k_scan", "k_fmask", "k_final", "k_merge"):
        if k in name:
            return k
    return name[:40]


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in acc.items()
           if k.startswith("k_")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
