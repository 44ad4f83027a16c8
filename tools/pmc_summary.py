"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more pass
directories): {kernel: {counter: mean value per dispatch, "dispatches": n}}.

    python tools/pmc_summary.py gpurun_out/s/pmc_1 gpurun_out/s/pmc_2 --match cheb_ --out s.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="", help="keep kernels whose name contains this")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r.get("Kernel_Name", "")
                    if a.match and a.match not in name:
                        continue
                    short = name.replace("void ", "").replace("wg::(anonymous namespace)::", "").split("(")[0]
                    acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
        # per counter: FETCH_SIZE and WRITE_SIZE (separate passes) must cover the same dispatch set
        out[k]["dispatches_per_counter"] = {c: len(v) for c, v in cs.items()}
    text = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
