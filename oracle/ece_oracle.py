"""CPU oracle for the ECE evaluation -- TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's ``utils/ece.py:8-89``
(``calculate_ece`` / ``calculate_average_ece``), used only by tests to check
``wats_hip.metrics``.  PINNED to the reference: ``tools/gen_ece_golden.py``
imports the reference module itself (a stub stands in for its unused seaborn
import, ``utils/ece.py:6``) and writes its outputs on logits, probabilities
and binning edge cases to ``tests/golden/ece_cases.npz``;
``tests/test_oracle.py::test_ece_oracle_bitwise_vs_reference_fixtures``
checks this restatement against every case bit for bit.
"""
import numpy as np
from scipy.special import softmax


def calculate_ece(model_outputs, labels, pos_class, logits=True, n_bins=10):
    """utils/ece.py:8-62."""
    if not isinstance(model_outputs, np.ndarray) or not isinstance(labels, np.ndarray):
        raise ValueError("Input arrays must be of type numpy.ndarray.")
    if model_outputs.shape[0] != labels.shape[0]:
        raise ValueError("Input arrays must have the same number of elements.")
    if logits:
        predictions = softmax(model_outputs, axis=1)[:, pos_class]           # :30-31
    else:
        predictions = model_outputs[:, pos_class]                            # :33
    labels = (labels == pos_class)                                          # :36
    bin_edges = np.linspace(0, 1, n_bins + 1)                               # :39
    bin_indices = np.digitize(predictions, bin_edges, right=True) - 1       # :40
    ece = 0.0
    for i in range(n_bins):                                                 # :44
        bin_mask = bin_indices == i
        if np.sum(bin_mask) < 4:                                            # :49 skip small bins
            continue
        bin_accuracy = np.mean(labels[bin_mask])
        bin_confidence = np.mean(predictions[bin_mask])
        bin_weight = np.mean(bin_mask)
        ece += np.abs(bin_confidence - bin_accuracy) * bin_weight           # :60
    return ece


def calculate_average_ece(model_outputs, labels, n_classes, logits=True, n_bins=10):
    """utils/ece.py:64-89."""
    return np.mean([calculate_ece(model_outputs, labels, c, logits=logits, n_bins=n_bins)
                    for c in range(n_classes)])
