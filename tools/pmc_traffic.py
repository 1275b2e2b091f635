"""HBM traffic and rocprof duration per kernel launch -> the table bench.py reports its roofline evidence from.

usage: python tools/pmc_traffic.py <fetch_pass.csv> <write_pass.csv> <kernel_stats.csv> [--cmd "..."] \
           > code-structure-aware-transformer_amd/csa_amd/pmc_gfx950.json

bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB, average per dispatch): on gfx950 FETCH_SIZE tallies wide streaming
reads at half their bytes (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane stores.
rocprof_avg_ns: the average duration of the kernel in a rocprofv3 --kernel-trace --stats run of the same
command. Keyed by kernel base name (template arguments dropped). The table ships inside the package (the
profiles/ directory does not travel to the GPU box), stamped with the library source hash it was measured on.
"""
import argparse
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def base(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("stats")
    ap.add_argument("--cmd", default="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-bf16-leg")
    ap.add_argument("--source-hash", default="")
    ap.add_argument("--leg", action="append", default=[],
                    help="NAME=kernel_stats.csv of a side-leg run (bench.py's cse / dense / long_k* roofline legs)")
    a = ap.parse_args()
    fetch, write = load(a.fetch), load(a.write)
    dur = {}
    for r in csv.DictReader(open(a.stats)):
        n = base(r["Name"])
        if n.startswith("k_"):
            dur.setdefault(n, float(r["AverageNs"]))
    kernels = {}
    for n in sorted(set(fetch) | set(write)):
        if not n.startswith("k_"):
            continue
        b = base(n)
        f = fetch.get(n, {}).get("FETCH_SIZE", 0.0)
        w = write.get(n, {}).get("WRITE_SIZE", 0.0)
        kernels[b] = {"bytes": int(round((2.0 * f + w) * 1024)), "fetch_bytes_corrected": int(round(2.0 * f * 1024)),
                      "write_bytes": int(round(w * 1024)), "rocprof_avg_ns": dur.get(b)}
    legs = {}
    for spec in a.leg:
        name, path = spec.split("=", 1)
        legs[name] = {}
        for r in csv.DictReader(open(path)):
            n = base(r["Name"])
            if n.startswith("k_"):
                legs[name].setdefault(n, {"rocprof_avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"])})
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) + --kernel-trace --stats",
           "command": a.cmd, "csa_source_hash": a.source_hash, "kernels": kernels, "legs": legs}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
