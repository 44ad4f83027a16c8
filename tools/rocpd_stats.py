"""Per-kernel statistics from a rocprofv3 rocpd database (ROCm 7 writes
`<dir>/<name>_results.db` by default instead of the CSV summaries).

    python tools/rocpd_stats.py gpurun_out/x/prof/run_results.db [--by-grid] [--csv out.csv] [--seq] [--like name]

Prints name, calls, average / min / max / total duration (ns), sorted by total;
--by-grid splits each kernel by its grid size (a proxy for the plan / workload).
"""
import argparse
import csv
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace(".kd", "")
    return name.split("(")[0].replace("void ", "").replace("wg::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--csv")
    ap.add_argument("--like", default=None, help="only kernels whose name contains this")
    ap.add_argument("--seq", action="store_true", help="every dispatch in launch order: name grid_x grid_y ns")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = {}
    names = {kid: (disp or kname) for kid, kname, disp in
             c.execute("select kernel_id, kernel_name, display_name from kernel_symbols")}
    if a.seq:
        q = "select kernel_id, duration, grid_x, grid_y, workgroup_x from kernels order by start"
        for kid, dur, gx, gy, wx in c.execute(q):
            name = names.get(kid, str(kid))
            if a.like is None or a.like in name:
                print(short(name).replace(" ", ""), gx // max(wx, 1), gy, dur)
        return
    for kid, dur, gx, gy, wx in c.execute("select kernel_id, duration, grid_x, grid_y, workgroup_x from kernels"):
        name = names.get(kid, str(kid))
        if a.like and a.like not in name:
            continue
        key = (short(name), f"{gx}x{gy}/{wx}" if a.by_grid else "")
        s = agg.setdefault(key, [0, 0, 1 << 62, 0])
        s[0] += 1
        s[1] += dur
        s[2] = min(s[2], dur)
        s[3] = max(s[3], dur)
    rows = sorted(((k[0], k[1], v[0], v[1] / v[0], v[2], v[3], v[1]) for k, v in agg.items()), key=lambda r: -r[6])
    w = csv.writer(open(a.csv, "w", newline="") if a.csv else sys.stdout)
    w.writerow(["Name", "Grid", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalNs"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.0f}", r[4], r[5], r[6]])


if __name__ == "__main__":
    main()
