"""Generate golden vectors for the ECE evaluation FROM THE REFERENCE.

Run only in the build container, where the reference is mounted read-only at
/root/reference:

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_ece_golden.py

It imports the reference's ``utils/ece.py`` (``calculate_ece`` /
``calculate_average_ece``, ``utils/ece.py:8-89``: what the harness scores
every calibrator with, ``benchmark_calibration_methods.py:122``) as a
standalone module.  Its only missing dependency is ``seaborn``
(``utils/ece.py:6``), imported but never used by those two functions: a stub
module stands in for it; numpy, scipy, sklearn and
matplotlib (Agg backend) are the installed ones.

Outputs are DATA only -- the inputs (logits or probabilities, labels) and the
reference's outputs (per-class ECE, average ECE) -- written to
``tests/golden/ece_cases.npz`` plus ``tests/golden/ece_manifest.json``
(versions, seeds, sha256).  Nothing of the reference's source travels.

Cases cover the binning quirks the restatements must reproduce: probabilities
exactly 0 (no bin: ``np.digitize(right=True) - 1 == -1``), exactly on bin
edges (0.1, 0.5, 1.0: right-closed bins), bins with fewer than 4 samples
(skipped), one-sample / empty classes, logits and probabilities, 2 to 41
classes, 7 to 5 000 samples.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")


def import_reference_ece():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))   # unused by calculate_ece
    spec = importlib.util.spec_from_file_location("ref_utils_ece", os.path.join(REF, "utils", "ece.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cases():
    """(name, model_outputs, labels, n_classes, logits) -- deterministic."""
    rng = np.random.default_rng(2024)
    out = []
    # logits, typical sizes (the harness passes probabilities; WATS.forward gives log-probs)
    for n, c in ((7, 2), (50, 3), (1000, 7), (2708, 7), (3000, 41)):
        z = (rng.standard_normal((n, c)) * 2.0).astype(np.float32)
        y = rng.integers(0, c, n)
        out.append((f"logits_n{n}_c{c}", z, y, c, True))
    # probabilities (the harness: exp(log_softmax), benchmark_calibration_methods.py:98-101)
    for n, c in ((300, 5), (5000, 10)):
        z = rng.standard_normal((n, c)) * 3.0
        p = np.exp(z - z.max(axis=1, keepdims=True))
        p = (p / p.sum(axis=1, keepdims=True)).astype(np.float32)
        y = rng.integers(0, c, n)
        out.append((f"probs_n{n}_c{c}", p, y, c, False))
    # edge cases: exact zeros (no bin), exact bin edges, 1.0, bins with < 4 samples
    c = 4
    p = np.zeros((40, c), np.float64)
    vals = [0.0, 0.1, 0.2, 0.5, 1.0, 0.1000001, 0.35, 0.95]
    for i in range(40):
        p[i, 0] = vals[i % len(vals)]
        p[i, 1] = 1.0 - p[i, 0]
    y = rng.integers(0, c, 40)
    out.append(("probs_edges_c4", p, y, c, False))
    # a class never predicted and never labelled; few samples per bin
    p = rng.dirichlet(np.ones(3), 11)
    p = np.concatenate([p, np.zeros((11, 1))], axis=1)
    y = rng.integers(0, 3, 11)
    out.append(("probs_sparse_bins_c4", p, y, 4, False))
    # confident logits: most mass in the top bin, many bins below 4 samples
    z = rng.standard_normal((64, 6)) * 0.5
    z[np.arange(64), rng.integers(0, 6, 64)] += 9.0
    out.append(("logits_confident_c6", z.astype(np.float64), rng.integers(0, 6, 64), 6, True))
    return out


def main():
    E = import_reference_ece()
    import matplotlib
    import scipy
    import sklearn
    manifest = {"source": "reference utils/ece.py:8-89 (calculate_ece, calculate_average_ece), imported with a "
                          "stub seaborn module", "numpy": np.__version__, "scipy": scipy.__version__,
                "sklearn": sklearn.__version__, "matplotlib": matplotlib.__version__, "seed": 2024, "cases": []}
    arrays = {}
    for name, mo, y, c, logits in cases():
        per = np.array([E.calculate_ece(mo, y, k, logits=logits, n_bins=10) for k in range(c)], np.float64)
        avg = float(E.calculate_average_ece(mo, y, c, logits=logits, n_bins=10))
        arrays[name + "__outputs"] = mo
        arrays[name + "__labels"] = y.astype(np.int64)
        arrays[name + "__per_class"] = per
        arrays[name + "__average"] = np.array([avg])
        arrays[name + "__meta"] = np.array([c, int(logits)], np.int64)
        manifest["cases"].append(name)
        print(f"{name}: average ECE {avg:.6f}")
    path = os.path.join(OUT, "ece_cases.npz")
    np.savez_compressed(path, **arrays)
    with open(path, "rb") as f:
        manifest["sha256"] = hashlib.sha256(f.read()).hexdigest()
    with open(os.path.join(OUT, "ece_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


if __name__ == "__main__":
    main()
