"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        n = short(r["Kernel_Name"])
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
    return {n: {c: v / len(disp[n]) for c, v in d.items()} for n, d in agg.items()}


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for n, d in sorted(load(p).items()):
            if n.startswith("k_"):
                print(n, " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
