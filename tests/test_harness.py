"""GPU test: the WATS block of the reference harness end to end (SURVEY.md
8(c), caller harness counterpart).

Reproduces ``benchmark_calibration_methods.py``: seeds 42 (:166-167); a
CompatibleGCN (nhid 64, dropout .5) trained 200 epochs with Adam (lr .01, wd
5e-4) on the train mask (:58-84, :178-179); then WATS constructed on the val
mask and timed (:317-327); everything scored by ``evaluate_calibration``
(acc, mean confidence, per-class 10-bin ECE; :87-127, utils/ece.py).

Planetoid Cora cannot be downloaded here (no network), so the data is a
synthetic Cora-shaped graph: N = 2708, 1433 sparse binary features
(row-normalised as NormalizeFeatures does), 7 classes planted as a stochastic
block model, the Planetoid split (20 train per class, 500 val, 1000 test), and
a dense float32 adjacency without self loops (:53).

Two runs over the same trained base model:
  reference execution -- features on the CPU (the oracle: scipy on
      csr_matrix(adj.cpu().numpy()), as WATS.py:99), dense torch CompatibleGCN,
      torch temperature head;
  MI355X drop-in -- features on the GPU from the dense adj (HIP), the base
      model's propagation as HIP SpMM (SparseCompatibleGCN, same weights), the
      fused HIP temperature head.
Asserted: the features agree (<= 1e-5), the node-wise temperature keeps the
base model's argmax (same accuracy), and both runs calibrate alike (ECE within
0.02; training is stochastic only through float rounding).  The JSON lines
(run `pytest -s`) carry the timings.
"""
import json
import time

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import wats_hip  # noqa: E402
from models import CompatibleGCN  # noqa: E402
from wats_hip.metrics import calculate_average_ece  # noqa: E402


def cora_like(seed=42, n=2708, nfeat=1433, ncls=7, avg_deg=3.9):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, ncls, n)
    # SBM: 85 % of edges inside a class
    m = int(n * avg_deg / 2)
    src = rng.integers(0, n, m)
    same = rng.random(m) < 0.85
    by_cls = [np.flatnonzero(y == c) for c in range(ncls)]
    dst = np.where(same, [by_cls[y[s]][rng.integers(0, len(by_cls[y[s]]))] for s in src], rng.integers(0, n, m))
    keep = src != dst
    adj = np.zeros((n, n), np.float32)
    adj[src[keep], dst[keep]] = 1.0
    adj[dst[keep], src[keep]] = 1.0
    # class-dependent sparse binary features, row-normalised (NormalizeFeatures)
    proto = rng.random((ncls, nfeat)) < 0.02
    x = (rng.random((n, nfeat)) < 0.004) | (proto[y] & (rng.random((n, nfeat)) < 0.5))
    x = x.astype(np.float32)
    x /= np.maximum(x.sum(1, keepdims=True), 1)
    train = np.zeros(n, bool)
    for c in range(ncls):
        train[np.flatnonzero(y == c)[:20]] = True
    rest = np.flatnonzero(~train)
    rng.shuffle(rest)
    val = np.zeros(n, bool)
    val[rest[:500]] = True
    test = np.zeros(n, bool)
    test[rest[500:1500]] = True
    t = lambda a: torch.from_numpy(a)
    return t(x), t(y.astype(np.int64)), t(adj), t(train), t(val), t(test)


def train_base(model, x, y, adj, train_mask, epochs=200):
    """benchmark_calibration_methods.py:58-84."""
    opt = torch.optim.Adam(model.parameters(), lr=0.01, weight_decay=5e-4)
    model.train()
    for _ in range(epochs):
        opt.zero_grad()
        out = model(x, adj)
        loss = F.nll_loss(F.log_softmax(out[train_mask], dim=1), y[train_mask])
        loss.backward()
        opt.step()
    return model


def evaluate(model, x, y, adj, test_mask):
    """benchmark_calibration_methods.py:87-127 (ECE on the device)."""
    model.eval()
    with torch.no_grad():
        out = model(x, adj)
        probs = out.exp() if isinstance(model, wats_hip.WATS) else F.softmax(out, dim=1)
        tp, tl = probs[test_mask], y[test_mask]
        acc = (tp.argmax(1) == tl).float().mean().item()
        conf = tp.max(1)[0].mean().item()
        ece = calculate_average_ece(tp, tl, tp.shape[1], logits=False)
    return acc, conf, ece


def test_harness_wats_block():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(42)
    np.random.seed(42)
    dev = torch.device("cuda")
    x, y, adj, train_mask, val_mask, test_mask = (t.to(dev) for t in cora_like())
    base = CompatibleGCN(x.shape[1], 7, nhid=64, dropout=0.5).to(dev)
    train_base(base, x, y, adj, train_mask)
    base.eval()
    for p in base.parameters():
        p.requires_grad = False
    base_acc, conf, base_ece = evaluate(base, x, y, adj, test_mask)
    print(json.dumps(dict(run="base model", acc=base_acc, conf=conf, ece=base_ece)), flush=True)

    # reference execution: CPU features (the oracle restatement of WATS.py:39-74 on
    # csr_matrix(adj.cpu().numpy()), WATS.py:99), dense base model, torch head
    import scipy.sparse as sp
    from oracle import wats_oracle as O
    t0 = time.perf_counter()
    feats_cpu = O.graph_wavelet_features(sp.csr_matrix(adj.cpu().numpy()), k=3, s=0.8)
    t_feat_cpu = time.perf_counter() - t0
    torch.manual_seed(0)
    t0 = time.perf_counter()
    w_ref = wats_hip.WATS(base, x, y, adj, val_mask, wavelet_feats=np.asarray(feats_cpu, np.float32),
                          fused_head=False, verbose=False)
    torch.cuda.synchronize()
    t_ref = time.perf_counter() - t0 + t_feat_cpu
    acc, conf, ref_ece = evaluate(w_ref, x, y, adj, test_mask)
    assert acc == base_acc
    print(json.dumps(dict(run="WATS reference execution (CPU scipy features, dense GCN, torch head)", acc=acc,
                          conf=conf, ece=ref_ece, construct_s=t_ref, features_s=t_feat_cpu)), flush=True)

    # the drop-in: GPU features, sparse propagation, fused head
    sbase = wats_hip.SparseCompatibleGCN(x.shape[1], nclass=7, nhid=64).to(dev)
    sbase.load_state_dict(base.state_dict())
    sbase.eval()
    for p in sbase.parameters():
        p.requires_grad = False
    torch.manual_seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feats_gpu = wats_hip.graph_wavelet_features(adj, k=3, s=0.8)
    torch.cuda.synchronize()
    t_feat_gpu = time.perf_counter() - t0
    torch.manual_seed(0)
    t0 = time.perf_counter()
    w = wats_hip.WATS(sbase, x, y, adj, val_mask, verbose=False)
    torch.cuda.synchronize()
    t_gpu = time.perf_counter() - t0
    acc, conf, ece = evaluate(w, x, y, adj, test_mask)
    assert acc == base_acc
    assert abs(ece - ref_ece) <= 0.02
    print(json.dumps(dict(run="WATS MI355X drop-in (HIP features, HIP SpMM GCN, fused head)", acc=acc, conf=conf,
                          ece=ece, construct_s=t_gpu, features_s=t_feat_gpu)), flush=True)
    f_ref = np.asarray(feats_cpu, np.float64).reshape(-1)
    err = float(np.abs(feats_gpu.cpu().numpy().reshape(-1) - f_ref).max() / max(np.abs(f_ref).max(), 1e-30))
    print(json.dumps(dict(check="wavelet features GPU vs CPU oracle", max_rel_err=err)), flush=True)
    assert err <= 1e-5
