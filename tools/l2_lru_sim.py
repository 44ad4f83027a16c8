"""Per-XCD L2 line fetches of one arxiv-size F = 40 step's gathers (CPU model).

Rows in internal (descending-degree) order, G = 6 rows per team wave, waves dispatched alternately
from the long and the short end (team_order 2), workgroups of 4 waves dealt round-robin to the 8
XCDs; every gathered u row is 160 B at a 160-B stride (so 2 lines of 128 B).  Prints, per XCD L2
capacity (gather lines only; the step's own-row streams take the rest of the 4 MiB): the
compulsory line fetches (every (line, XCD) pair once: the replication floor) and the LRU misses.
r05: compulsory 538 277 lines = 68.9 MB; LRU 4.2 MB 801 021 (102.5 MB), 3.1 MB 1 014 993
(129.9 MB; any wave order: 129.9-130.1 MB), 2.1 MB 1 374 604 (175.9 MB) -- against the PMC's
~960 k gather lines per launch (TCC_EA0_RDREQ_128B 1.28 M minus the streams' ~0.33 M).

    python tools/l2_lru_sim.py [cap_lines ...]
"""
import os
import sys
from collections import OrderedDict

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "efficient-gnn_amd"))
from wats_hip.graphgen import named_graph  # noqa: E402


def main():
    caps = [int(x) for x in sys.argv[1:]] or [32768, 24576, 16384]
    A = named_graph("ogbn-arxiv").to_scipy().tocsr()
    deg = np.diff(A.indptr)
    order = np.argsort(-deg, kind="stable")
    order = order[deg[order] > 0]
    rank = np.empty(A.shape[0], np.int64)
    rank[order] = np.arange(len(order))
    G, RB, P = 6, 160, 8
    ind, ip = A.indices, A.indptr
    nw = (len(order) + G - 1) // G
    seq, lo, hi = [], 0, nw
    while lo < hi:
        seq.append(lo)
        lo += 1
        if lo < hi:
            hi -= 1
            seq.append(hi)
    for cap in caps:
        caches = [OrderedDict() for _ in range(P)]
        comp = [set() for _ in range(P)]
        miss = acc = 0
        for pos, w in enumerate(seq):
            x = (pos // 4) % P
            c = caches[x]
            for r in order[w * G:(w + 1) * G]:
                for j in ind[ip[r]:ip[r + 1]]:
                    b0 = rank[j] * RB
                    for line in range(b0 // 128, (b0 + RB - 1) // 128 + 1):
                        acc += 1
                        comp[x].add(line)
                        if line in c:
                            c.move_to_end(line)
                        else:
                            miss += 1
                            c[line] = 1
                            if len(c) > cap:
                                c.popitem(last=False)
        nc = sum(len(s) for s in comp)
        print(f"L2 {cap * 128 / 1e6:.1f} MB: line accesses {acc}, LRU misses {miss} ({miss * 128 / 1e6:.1f} MB), "
              f"compulsory {nc} ({nc * 128 / 1e6:.1f} MB)", flush=True)


if __name__ == "__main__":
    main()
