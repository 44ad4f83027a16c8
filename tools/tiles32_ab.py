"""A/B of the hybrid step's two MFMA shapes on Reddit-size F = 41 (run on the GPU box).

tile_mfma 16 (cheb_tiles_kernel, v_mfma_f32_16x16x32_bf16) against 32
(cheb_tiles32_kernel, v_mfma_f32_32x32x16_bf16), alternated so clocks and
caches are shared; prints the chain time per step of each and the norm-wise
difference of their S.  Under `rocprofv3 --kernel-trace --stats` the two tile
kernels show up under their own names.

    python tools/tiles32_ab.py --config reddit-f41 --rounds 3
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip import _lib  # noqa: E402
from wats_hip._lib import check, ptr  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="reddit-f41")
    ap.add_argument("--F", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="16,32")
    ap.add_argument("--variants", default=None,
                    help="knob sets instead of --shapes, e.g. 'tile_max=64|tile_max=256,tile_th=64' (plan knobs rebuild)")
    a = ap.parse_args()
    n, nnz_t, K, F = NAMED_CONFIGS[a.config]
    F = a.F or F
    dev = torch.device("cuda", 0)
    ip, ix = rmat_graph_device(n, nnz_t, seed=0, device=dev)
    L = wats_hip.NormalizedLaplacian(n, ip, ix, None, device=dev)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    X = torch.randn(n, F, device=dev)
    out = {}
    if a.variants:
        shapes = a.variants.split("|")
        knobs = {v: {kv.split("=")[0]: int(kv.split("=")[1]) for kv in v.split(",")} for v in shapes}
    else:
        shapes = [int(s) for s in a.shapes.split(",")]
        knobs = {m: {"tile_mfma": m} for m in shapes}
    for r in range(a.rounds):
        for m in shapes:
            L.tune(**knobs[m])
            S = torch.empty_like(X)
            H = torch.empty_like(X)
            run = lambda: check(lib.wg_wavelet_features(L.handle, ptr(X), F, K, 0.8, ptr(S), ptr(H), st), "wavelet_features")
            run()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record()
            for i in range(a.reps):
                run()
                ev[i + 1].record()
            torch.cuda.synchronize()
            ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps))[a.reps // 2]
            out.setdefault(m, []).append(ms * 1e3 / K)
            if r == 0:
                out[f"S{m}"] = S.clone()
            print(f"round {r} {knobs[m]}: {ms * 1e3 / K:8.1f} us per step", flush=True)
    print(L.describe(F).strip())
    for m in shapes:
        print(f"{knobs[m]}: median {sorted(out[m])[len(out[m]) // 2]:8.1f} us per step")
    if len(shapes) == 2:
        s0, s1 = out[f"S{shapes[0]}"].double(), out[f"S{shapes[1]}"].double()
        err = ((s0 - s1).abs().amax(0) / (s0.abs().amax(0) + 1e-30)).max().item()
        print(f"S norm-wise difference between the shapes: {err:.3e}")


if __name__ == "__main__":
    main()
