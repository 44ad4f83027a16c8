"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py --kernel "cheb_step_kernel<4, true" DIR [DIR ...] [--out traffic.json]
(--kernel is a substring of the kernel name: make it specific enough to pick
one instantiation -- the bench's F = 1 companion runs cheb_step_kernel<1, ...>)

Each DIR is the -d output of one `rocprofv3 --pmc <counters> --output-format csv`
pass (FETCH_SIZE and WRITE_SIZE must be collected in separate passes on gfx950:
TCC slots, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Following
MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE are KiB from the L2's memory-side
request counters; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
(16 B/lane) read, so it is doubled (the step kernel's vector reads are all
16 B/lane float4; its 4 B index/value streams make this an upper-bound
correction).  Infinity-Cache hits are counted as well, so this is L2-miss
(fabric) traffic, an upper bound of true HBM bytes."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counters(d, kernel):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="cheb_step_kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    means, counts = {}, {}
    for d in a.dirs:
        m, c = read_counters(d, a.kernel)
        means.update(m)
        counts.update(c)
    res = {"kernel": a.kernel, "counters_per_dispatch": means, "dispatches": counts}
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        fetch = means["FETCH_SIZE"] * 1024.0
        write = means["WRITE_SIZE"] * 1024.0
        res["fetch_bytes_raw"] = fetch
        res["fetch_bytes_corrected"] = 2.0 * fetch
        res["write_bytes"] = write
        res["bytes_per_launch"] = 2.0 * fetch + write
    hit, miss = means.get("TCC_HIT_sum"), means.get("TCC_MISS_sum")
    if hit is not None and miss is not None and hit + miss > 0:
        res["l2_hit_rate"] = hit / (hit + miss)
    js = json.dumps(res, indent=1)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
