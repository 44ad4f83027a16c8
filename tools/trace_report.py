"""Offline report of a step-launch timeline recorded by tools/trace_probe.py.

python tools/trace_report.py gpurun_out/<session>/trace_*.npz"""
import re
import sys

import numpy as np


def segments(plan: str):
    """[(kind, first block, end block)] in block order, from wg_laplacian_describe's text."""
    segs = []
    blk = 0
    for ln in plan.splitlines():
        m = re.match(r"split rows\[(\d+),(\d+)\) chunks=(\d+)", ln)
        if m:
            segs.append(("split", blk, blk + int(m.group(3))))
            blk += int(m.group(3))
            continue
        m = re.match(r"block rows\[(\d+),(\d+)\)", ln)
        if m:
            cnt = int(m.group(2)) - int(m.group(1))
            segs.append(("block", blk, blk + cnt))
            blk += cnt
            continue
        m = re.match(r"team rows\[(\d+),(\d+)\) ln=(\d+) blocks=(\d+)", ln)
        if m:
            segs.append((f"team[{m.group(1)},{m.group(2)}) ln={m.group(3)}", blk, blk + int(m.group(4))))
            blk += int(m.group(4))
    return segs


def report(path):
    z = np.load(path)
    plan = str(z["plan"])
    segs = segments(plan)
    for key in sorted(k for k in z.files if k.startswith("trace")):
        tr = z[key]
        tr = tr[tr[:, 1] > 0]
        block = (tr[:, 0] & 0xFFFFFF).astype(np.int64)
        xcc = ((tr[:, 0] >> 28) & 15).astype(np.int64)
        t0 = (tr[:, 1] - tr[:, 1].min()).astype(np.int64) * 10   # ns
        t1 = (tr[:, 2] - tr[:, 1].min()).astype(np.int64) * 10
        cyc = tr[:, 3].astype(np.int64)
        span = t1.max()
        print(f"== {path} {key}: {len(tr)} waves, span {span / 1e3:.2f} us, wave time sum {(t1 - t0).sum() / 1e6:.1f} ms, "
              f"mean concurrency {(t1 - t0).sum() / span:.0f} waves ({(t1 - t0).sum() / span / 256:.1f} per CU), "
              f"clock {cyc.sum() / max(1, (t1 - t0).sum()):.2f} GHz")
        for kind, b0, b1 in segs:
            m = (block >= b0) & (block < b1)
            if not m.any():
                continue
            d = t1[m] - t0[m]
            print(f"  {kind:28s} blocks {b1 - b0:5d}: start {t0[m].min() / 1e3:6.2f}-{t0[m].max() / 1e3:6.2f} us, "
                  f"end <= {t1[m].max() / 1e3:6.2f}, wave mean {d.mean() / 1e3:5.2f} max {d.max() / 1e3:5.2f} us, "
                  f"share of wave time {d.sum() / (t1 - t0).sum():.3f}")
        bins = np.arange(0, span + 1000, 1000)
        conc = [int(((t0 < hi) & (t1 > lo)).sum()) for lo, hi in zip(bins[:-1], bins[1:])]
        print("  active waves per us:", " ".join(str(c) for c in conc))
        per_x = [int(((xcc == x)).sum()) for x in range(8)]
        end_x = [round(t1[xcc == x].max() / 1e3, 2) if (xcc == x).any() else 0 for x in range(8)]
        print(f"  waves per XCD {per_x}; last end per XCD (us) {end_x}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        report(p)
