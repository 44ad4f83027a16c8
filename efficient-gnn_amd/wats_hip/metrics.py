"""Expected Calibration Error on the device.

Torch restatement of the reference's ``utils/ece.py:8-89`` (what the harness
scores every calibrator with, ``benchmark_calibration_methods.py:122``), so
the WATS evaluation needs no host copy.  Same binning quirks:

* ``np.digitize(p, linspace(0,1,n_bins+1), right=True) - 1`` (ece.py:40): bin i
  holds ``edges[i] < p <= edges[i+1]``; a probability of exactly 0 falls in no bin;
* bins with fewer than 4 samples are skipped (ece.py:49);
* ECE = sum |mean(p) - mean(label)| * bin_fraction (ece.py:60);
  ``calculate_average_ece`` = mean over classes (ece.py:64-89).

Inputs may be numpy arrays or torch tensors (any device); the result is a
Python float.  (This evaluation is plain torch: it is not on the wavelet hot
path.)
"""
from __future__ import annotations

import torch


def _as_tensor(x, device=None):
    t = torch.as_tensor(x)
    return t.to(device) if device is not None else t


def calculate_ece(model_outputs, labels, pos_class: int, logits: bool = True, n_bins: int = 10) -> float:
    out = _as_tensor(model_outputs)
    lab = _as_tensor(labels, out.device)
    if out.shape[0] != lab.shape[0]:
        raise ValueError("Input arrays must have the same number of elements.")
    return float(_ece_all(out, lab, logits, n_bins, classes=[pos_class])[0])


def calculate_average_ece(model_outputs, labels, n_classes: int, logits: bool = True, n_bins: int = 10) -> float:
    out = _as_tensor(model_outputs)
    lab = _as_tensor(labels, out.device)
    if out.shape[0] != lab.shape[0]:
        raise ValueError("Input arrays must have the same number of elements.")
    return float(_ece_all(out, lab, logits, n_bins, classes=list(range(n_classes))).mean())


def _ece_all(out: torch.Tensor, lab: torch.Tensor, logits: bool, n_bins: int, classes) -> torch.Tensor:
    """Per-class ECE for the given classes, all classes in one pass (float64)."""
    probs = torch.softmax(out.double(), dim=1) if logits else out.double()
    p = probs[:, classes]                                        # (N, C)
    y = (lab.reshape(-1, 1) == torch.as_tensor(classes, device=lab.device).reshape(1, -1)).double()
    edges = torch.linspace(0, 1, n_bins + 1, dtype=torch.float64, device=p.device)
    b = torch.bucketize(p, edges, right=False) - 1               # == np.digitize(right=True) - 1
    n, C = p.shape
    valid = (b >= 0) & (b < n_bins)
    b = torch.where(valid, b, torch.zeros_like(b))
    idx = b + n_bins * torch.arange(C, device=p.device).reshape(1, -1)
    w = valid.double()
    cnt = torch.zeros(C * n_bins, dtype=torch.float64, device=p.device).index_add_(0, idx.flatten(), w.flatten())
    sp = torch.zeros_like(cnt).index_add_(0, idx.flatten(), (p * w).flatten())
    sy = torch.zeros_like(cnt).index_add_(0, idx.flatten(), (y * w).flatten())
    ok = cnt >= 4
    safe = torch.where(ok, cnt, torch.ones_like(cnt))
    term = torch.where(ok, (sp / safe - sy / safe).abs() * (cnt / n), torch.zeros_like(cnt))
    return term.reshape(C, n_bins).sum(dim=1)
