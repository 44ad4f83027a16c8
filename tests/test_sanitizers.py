"""Host sanitizers on the CPU code paths: the C restatement of the
oracle (oracle/wats_chain.c, the full-size parity checker) built with
AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`) and run on
every golden fixture -- empty, single-node, self-loop-only, directed weighted
graphs with isolated nodes -- and on wider random inputs, bit for bit against
the fixtures; and the C99 consumer of include/wats_hip.h instrumented the same
way against the shipped library's argument-validation paths.  CPU only (the GPU
kernels have their own bounds-checked variant, tools/debug_suite.sh)."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")


def _asan_env(extra=None):
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("no libasan")
    env = dict(os.environ)
    env.update({"LD_PRELOAD": libasan, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "OMP_NUM_THREADS": "3"})
    env.update(extra or {})
    return env


_SCRIPT = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
sys.path.insert(0, os.path.join(os.environ["REPO"], "efficient-gnn_amd"))
from conftest import golden_csr, golden_names, load_golden
from oracle import wats_oracle as O
from oracle import wats_oracle_c as C
assert C.LIB_PATH.endswith("libwats_oracle_asan.so"), C.LIB_PATH
n = 0
for name in golden_names():
    d = load_golden(name)
    A = golden_csr(d)
    A.sort_indices()
    S, H = C.graph_wavelet_features(A.indptr, A.indices, A.data, d["X0"].astype(np.float32), int(d["k"]),
                                    float(d["s"]), threads=3)
    np.testing.assert_array_equal(S, d["S"])
    n += 1
from wats_hip.graphgen import random_graph, rmat_graph
for g, F, k in ((rmat_graph(1500, 20000, seed=3), 5, 16),
                (random_graph(300, 0.03, seed=4, directed=True, weighted=True, self_loop_frac=0.1,
                              isolated_frac=0.05), 3, 7)):
    X0 = np.random.default_rng(0).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=k, s=0.8, X0=X0, return_all=True)
    S, H = C.graph_wavelet_features(g.indptr, g.indices, g.values, X0, k, 0.8, threads=3)
    np.testing.assert_array_equal(S, ref["S"])
    n += 1
print("sanitized ok", n)
"""


def test_c_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True)
    lib = os.path.join(REPO, "oracle", "build", "libwats_oracle_asan.so")
    env = _asan_env({"WATS_ORACLE_LIB": lib, "REPO": REPO})
    out = subprocess.run([sys.executable, "-c", _SCRIPT], env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "sanitized ok" in out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-4000:]


def test_c_abi_consumer_under_asan_ubsan(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
    from wats_hip import _lib
    src = os.path.join(REPO, "tests", "c", "abi_check.c")
    exe = str(tmp_path / "abi_check_asan")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), src, "-L",
                    libdir, "-lwats_hip", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    assert out.stdout.startswith("ok")
