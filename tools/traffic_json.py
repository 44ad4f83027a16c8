"""bytes per launch of one kernel from a pmc_summary.json (tools/pmc_legs.sh): FETCH_SIZE x 2 (gfx950
counts a 128-B fabric read as 64 B: MI355X_MICROARCH.md "HBM") + WRITE_SIZE, cross-checked against
TCC_EA0_RDREQ_128B x 128 B, with the dispatch count of every counter (they must match).

    python tools/traffic_json.py gpurun_out/x/arxiv/pmc_summary.json "cheb_team4_kernel<6, false, 2>" out.json
"""
import json
import sys


def main():
    src, kernel, out = sys.argv[1], sys.argv[2], sys.argv[3]
    d = json.load(open(src))[kernel]
    per = d.get("dispatches_per_counter", {})
    fetch = d["FETCH_SIZE"] * 1024.0
    write = d["WRITE_SIZE"] * 1024.0
    r = {
        "kernel": kernel,
        "source": src,
        "counters_per_dispatch": {k: v for k, v in d.items() if not k.startswith("dispatches")},
        "dispatches": per or d.get("dispatches"),
        "dispatch_counts_match": (len(set(per.values())) == 1) if per else None,
        "fetch_bytes_raw": fetch,
        "fetch_bytes_corrected": 2.0 * fetch,
        "rdreq_128b_bytes": d.get("TCC_EA0_RDREQ_128B_sum", 0.0) * 128.0 + d.get("TCC_EA0_RDREQ_64B_sum", 0.0) * 64.0,
        "write_bytes": write,
        "bytes_per_launch": 2.0 * fetch + write,
        "l2_hit_rate": d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]) if "TCC_HIT_sum" in d else None,
    }
    with open(out, "w") as fh:
        json.dump(r, fh, indent=1)
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
