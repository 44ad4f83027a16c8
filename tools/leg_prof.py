"""One row-sharded bench leg alone (run on the GPU box, under rocprofv3), so that a kernel
summary holds that leg's kernels only (the extras' frac reproduced
from profiles/):

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/leg_prof.py reddit-f41 [steps]
    python3 tools/leg_prof.py --report DIR/..._kernel_stats.csv leg.json

The leg is bench.run_sharded at one rank (IPC exchange object, no peers), its parity check
off (the check runs an unsharded chain whose kernels would mix into the summary).  --report
sums the step kernels' average durations per Chebyshev step and recomputes the line's frac
from them."""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

STEP_KERNELS = ("cheb_team4_kernel", "cheb_step_kernel", "cheb_tiles_kernel", "cheb_tiles32_kernel",
                "tiles_combine_kernel", "cheb_hub1_kernel", "cheb_lds1_kernel", "cheb_lds3_kernel",
                "combine_lds2_kernel", "cheb_windows")


def report(stats_csv, leg_json):
    line = json.loads(open(leg_json).read().strip().splitlines()[-1])
    r = line["roofline"]
    K = line["config"]["K"]
    per_step = 0.0
    rows = []
    for row in csv.DictReader(open(stats_csv)):
        name = row["Name"]
        if any(k in name for k in STEP_KERNELS):
            calls, tot = int(row["Calls"]), float(row["TotalDurationNs"])
            short = name.replace("void ", "").replace("wg::(anonymous namespace)::", "").split("(")[0]
            rows.append((short, calls, tot / calls / 1e3))
            per_step += tot / 1e3
    steps = None
    # calls of the most frequent step kernel = Chebyshev steps launched (one per step)
    if rows:
        steps = max(c for _, c, _ in rows)
        per_step /= steps
    out = {"leg": line["metric"], "K": K, "line_avg_step_us": r["avg_launch_us"], "line_frac": r["frac"],
           "rocprof_step_us": per_step, "rocprof_frac": r["algorithmic_bytes_per_launch"] / (per_step * 1e-6) / 8e12,
           "kernels": [{"kernel": n, "calls": c, "avg_us": a} for n, c, a in rows],
           "ms_per_step": line["ms_per_step"], "K_x_rocprof_step_ms": K * per_step / 1e3}
    print(json.dumps(out, indent=1))


def main():
    if sys.argv[1] == "--report":
        report(sys.argv[2], sys.argv[3])
        return
    import torch
    import bench
    cfg = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    line = bench.run_sharded(cfg, None, None, steps, 1, 0, 0.8, 1, 0, dev, "ipc", check=False)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
