"""Per-pass time of graph_wavelet_features with and without the per-step HIP
events of wg_profile_enable (run on the GPU box): how much of a pass is
kernel time and how much the gaps between launches."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import named_graph  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "ogbn-arxiv"
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    K = 16
    g = named_graph(cfg)
    L = wats_hip.NormalizedLaplacian.from_graph(g)
    X = torch.from_numpy(np.random.default_rng(1).standard_normal((g.n, F)).astype(np.float32)).cuda() if F > 1 \
        else L.log1p_degree()
    S = torch.empty(g.n, F, device="cuda")
    H = torch.empty(g.n, F, device="cuda")
    lib = wats_hip._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    run = lambda: wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, 0.8, S.data_ptr(),
                                                               H.data_ptr(), st))
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    reps = 50
    for prof in (False, True, False, True):
        L.profile_enable(prof)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for _ in range(reps):
            run()
        b.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps * 1e3
        line = f"profile={prof}: pass {a.elapsed_time(b) / reps:.4f} ms (wall {wall:.4f})"
        if prof:
            p = L.profile_collect()
            line += f"; step kernels {p['sum_ms'] / reps:.4f} ms ({p['sum_ms'] / p['launches'] * 1e3:.2f} us each)"
        print(line, flush=True)
    L.profile_enable(False)


if __name__ == "__main__":
    main()
