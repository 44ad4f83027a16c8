"""Does a kernel slow down after large allocations were freed in the same process?
(run on the GPU box)

Times the Reddit-size F = 1 chain (LDS windows kernel) fresh, again after a
re-create, after an F = 41 chain on the same graph (several GB allocated and
freed), and after that with torch's cache emptied / a 4 GiB scratch buffer
held, printing the per-step kernel time each time.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def chain_us(L, F, K=16, reps=20):
    lib = wats_hip._lib.load()
    X = L.log1p_degree() if F == 1 else torch.randn(L.n, F, device="cuda")
    S = torch.empty(L.n, F, device="cuda")
    H = torch.empty(L.n, F, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    run = lambda: wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, 0.8, S.data_ptr(),
                                                               H.data_ptr(), st))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    L.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    p = L.profile_collect()
    L.profile_enable(False)
    return p["sum_ms"] / max(1, p["launches"]) * 1e3, wall


def main():
    n, nnz, _, _ = NAMED_CONFIGS["reddit"]
    ip, ix = rmat_graph_device(n, nnz, seed=0)

    def f1(tag):
        L = wats_hip.NormalizedLaplacian(n, ip, ix)
        us, ms = chain_us(L, 1)
        print(f"{tag}: F=1 step kernel {us:.1f} us, chain {ms:.3f} ms", flush=True)
        L.close()

    f1("fresh")
    f1("re-created")
    L = wats_hip.NormalizedLaplacian(n, ip, ix)
    us, ms = chain_us(L, 41, reps=5)
    print(f"F=41 step kernel {us:.1f} us, chain {ms:.3f} ms", flush=True)
    L.close()
    torch.cuda.synchronize()
    f1("after F=41 (torch cache kept)")
    torch.cuda.empty_cache()
    f1("after F=41, torch cache emptied")
    scratch = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    f1("4 GiB torch scratch held")
    del scratch
    torch.cuda.empty_cache()
    f1("scratch freed")


if __name__ == "__main__" and not os.environ.get("ALLOC_PROBE_SHARDED"):
    main()


def sharded_main():
    """The same question for the native sharded chain at world 1 (wats_hip.dist)."""
    import numpy as np
    from wats_hip.dist import ShardedWavelet
    n, nnz, _, _ = NAMED_CONFIGS["reddit"]
    ip, ix = rmat_graph_device(n, nnz, seed=0)
    indptr = ip.cpu().numpy()
    cols = ix.cpu().numpy()
    bounds = np.array([0, n])

    def run(tag, F, exchange="rccl", reps=20):
        sw = ShardedWavelet(indptr, cols, None, n, bounds, exchange=exchange, device="cuda:0", max_features=F)
        X = sw.L.log1p_degree() if F == 1 else torch.randn(n, F, device="cuda")
        out = (torch.empty(n, F, device="cuda"), torch.empty(n, F, device="cuda"))
        for _ in range(3):
            sw.wavelet_features(X, k=16, s=0.8, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            sw.wavelet_features(X, k=16, s=0.8, out=out)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"{tag}: F={F} {exchange} chain {ms:.3f} ms, info {sw.info()}", flush=True)
        sw.close()
        del sw
        torch.cuda.empty_cache()

    run("sharded fresh", 1)
    run("sharded again", 1)
    run("sharded F=41", 41, reps=5)
    run("sharded F=1 after F=41", 1)
    run("sharded F=41 ipc", 41, "ipc", reps=5)
    run("sharded F=1 after ipc", 1)
    run("sharded F=1 ipc", 1, "ipc")


if __name__ == "__main__" and os.environ.get("ALLOC_PROBE_SHARDED"):
    sharded_main()
