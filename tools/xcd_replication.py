"""How many XCD L2s must fetch each gathered u row in one step (CPU, plan-time analysis).

A step gathers u[c] for every entry (r, c); a row r runs on one XCD, so u[c] is fetched by every
XCD that runs a row referencing c: with rows dealt round-robin (the hardware's workgroup
placement) a column of degree d is fetched by ~8 (1 - (7/8)^d) XCDs.  This prints that
replication for the arxiv-size R-MAT graph under round-robin placement and under a greedy
column-affine assignment of waves (G rows each) to XCDs (each wave to the XCD already holding
most of its columns, loads capped at +3 %) -- the XCD-affine scheduling lever of VERDICT r3 item
1(b).  r04: 366 953 vs 365 061 (column, XCD) pairs = 58.7 vs 58.4 MB of u rows at F = 40:
R-MAT has no column locality to exploit, so the replicated L2 fills are a floor of the graph,
not of the kernel.

    python tools/xcd_replication.py [--config ogbn-arxiv] [--rows-per-wave 6]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "efficient-gnn_amd"))
from wats_hip.graphgen import named_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ogbn-arxiv")
    ap.add_argument("--rows-per-wave", type=int, default=6)
    ap.add_argument("--F", type=int, default=40)
    a = ap.parse_args()
    A = named_graph(a.config).to_scipy().tocsr()
    deg = np.diff(A.indptr)
    rows = np.argsort(-deg, kind="stable")
    rows = rows[deg[rows] > 0]
    P, G = 8, a.rows_per_wave
    ind, ip = A.indices, A.indptr
    waves = [np.concatenate([ind[ip[r]:ip[r + 1]] for r in rows[s:s + G]]) for s in range(0, len(rows), G)]
    row_bytes = 4 * a.F
    d = deg[deg > 0]
    print(f"{a.config}: {len(rows)} active rows, {int(deg.sum())} entries; u fetched once: "
          f"{d.size * row_bytes / 1e6:.1f} MB; expected round-robin pairs {(P * (1 - (1 - 1 / P) ** d)).sum():.0f}")
    present = np.zeros((P, A.shape[0]), bool)
    for i, cols in enumerate(waves):
        present[i % P, cols] = True
    rr = int(present.sum())
    present[:] = False
    load = np.zeros(P)
    cap = deg.sum() / P * 1.03
    for cols in waves:
        ov = present[:, cols].sum(1).astype(float)
        ok = load + len(cols) <= cap
        if not ok.any():
            ok[:] = True
        ov[~ok] = -1
        best = np.flatnonzero(ov == ov.max())
        p = best[np.argmin(load[best])]
        present[p, cols] = True
        load[p] += len(cols)
    gr = int(present.sum())
    print(f"(column, XCD) pairs: round-robin {rr} ({rr * row_bytes / 1e6:.1f} MB), greedy column-affine {gr} "
          f"({gr * row_bytes / 1e6:.1f} MB; loads {load.min():.0f} .. {load.max():.0f})")


if __name__ == "__main__":
    main()
