"""Drop-in WATS calibrator whose wavelet features come from the HIP path.

Same class name, constructor signature / positional order and ``forward``
contract as the reference ``calibration/WATS.py:76-170``:

* ``WATS(base_model, features, labels, adj, val_mask)`` trains in the
  constructor (WATS.py:110) and caches the wavelet features (WATS.py:99-100);
* ``forward(x, adj)`` returns ``log_softmax(base_model(x, adj) / T)`` with the
  node-wise temperature ``T = log(exp(net(H)) + 1.1)`` (WATS.py:112-130); the
  features are NOT recomputed from ``adj`` (WATS.py:123), so gradients w.r.t.
  ``adj`` flow only through the base model, as the attack code expects.

Differences: the features are computed on the GPU from the dense ``adj``
(no ``adj.cpu().numpy()`` round trip, WATS.py:99); keyword-only extras
``k``/``s`` (defaults 3 / 0.8 as hard-coded at WATS.py:99), ``X0`` (signal),
``graph`` (a sparse graph to use instead of the dense ``adj`` for the
features), ``wavelet_feats`` (precomputed features, e.g. a cache),
``fused_head`` (default off: the reference's torch ops; on: the temperature
head + log_softmax as the fused HIP kernels of ``head.py``) and
``verbose``; ``fit()`` is an alias of ``calib_train``.
"""
from __future__ import annotations

import time

import torch
import torch.nn as nn
import torch.nn.functional as F

from .wavelet import graph_wavelet_features


def accuracy(outputs: torch.Tensor, labels: torch.Tensor) -> float:
    """``calibration/utils.py:139-167``: argmax accuracy as a Python float."""
    if not isinstance(outputs, torch.Tensor) or not isinstance(labels, torch.Tensor):
        raise ValueError("Input arrays must be of type torch.Tensor.")
    if outputs.shape[0] != labels.shape[0]:
        raise ValueError("Input arrays must have the same number of elements.")
    predicted = torch.argmax(outputs, dim=1)
    correct = torch.sum(predicted == labels)
    return (correct / labels.shape[0]).item()


class WATS(torch.nn.Module):
    def __init__(self, base_model, features, labels, adj, val_mask, *, k: int = 3, s: float = 0.8, X0=None,
                 graph=None, wavelet_feats=None, verbose: bool = True, fused_head: bool = False):
        super().__init__()
        self.fused_head = bool(fused_head) and torch.cuda.is_available()
        # WATS.py:91 picks cuda when available; the HIP feature path requires it.
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.base_model = base_model.to(self.device)
        self.x = features.to(self.device)
        self.y = labels.to(self.device)
        self.adj = adj.to(self.device)
        self.val_idx = val_mask.to(self.device)
        self.k, self.s, self.verbose = int(k), float(s), verbose

        if wavelet_feats is None:
            # WATS.py:99-100 -- computed once, cached, float32 on the device
            src = graph if graph is not None else self.adj
            feats = graph_wavelet_features(src, k=self.k, s=self.s, X0=X0)
        else:
            feats = torch.as_tensor(wavelet_feats)
            if feats.dim() == 1:
                feats = feats.reshape(-1, 1)
        self.wavelet_feats = feats.to(device=self.device, dtype=torch.float32)
        self.net = nn.Sequential(                                   # WATS.py:101-105
            nn.Linear(self.wavelet_feats.shape[1], 16),
            nn.ReLU(),
            nn.Linear(16, 1),
        ).to(self.device)
        for para in self.net.parameters():
            para.requires_grad = True
        self.calib_train()

    def temperatures(self) -> torch.Tensor:
        """Node-wise temperature ``log(exp(net(H)) + 1.1)`` (WATS.py:124-125)."""
        t = self.net(self.wavelet_feats.to(self.device)).squeeze()
        return torch.log(torch.exp(t) + torch.tensor(1.1, device=self.device)).to(self.device)

    def forward(self, x, adj):
        """WATS.py:112-130."""
        x, adj = x.to(self.device), adj.to(self.device)
        if self.fused_head:
            from .head import wats_head
            return wats_head(self.wavelet_feats, self.base_model(x, adj), self.net)
        temperatures = self.temperatures()
        logits = self.base_model(x, adj)
        calibrated_logits = logits / temperatures.unsqueeze(1)
        return F.log_softmax(calibrated_logits, dim=1)

    def calib_train(self, patience: int = 10):
        """WATS.py:132-170: Adam(lr .01, wd 5e-4) on the temperature head only,
        NLL on the calibration nodes, <= 250 epochs, early stop after
        ``patience`` non-improving epochs."""
        t = time.time()
        best_loss = float("inf")
        patience_counter = patience
        optimizer = torch.optim.Adam(self.net.parameters(), lr=0.01, weight_decay=5e-4)
        for epoch in range(250):
            self.train()
            optimizer.zero_grad()
            output = self(self.x, self.adj)
            loss = F.nll_loss(output[self.val_idx], self.y[self.val_idx])
            loss.backward()
            optimizer.step()
            with torch.no_grad():
                self.eval()
                acc = accuracy(output[self.val_idx], self.y[self.val_idx])
                if self.verbose:
                    print(f"epoch: {epoch}", f"loss_calibration: {loss.item():.4f}",
                          f"acc_calibration: {acc:.4f}", f"time: {time.time() - t:.4f}s")
            if loss < best_loss:
                best_loss = loss
                patience_counter = patience
            else:
                patience_counter -= 1
            if patience_counter <= 0:
                if self.verbose:
                    print(f"Early stopping at epoch {epoch}, best loss: {best_loss:.4f}")
                break
        return self

    fit = calib_train
