"""The bench.py contract the driver parses: one JSON line on stdout with the
required keys, a roofline object (bound, achieved, peak, unit, frac,
traffic) and, at N = 1, a cpu_baseline object -- run on a small workload."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


def _run(args, timeout=600):
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                         timeout=timeout, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must be exactly one JSON line, got {len(lines)}: {out.stdout[:2000]}"
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_line_schema_small():
    d = _run(["--config", "pubmed", "--F", "8", "--steps", "3", "--warmup", "1", "--cpu-seconds", "1",
              "--sharded-extra", "pubmed", "--sharded-steps", "2", "--exchange", "ipc,rccl", "--cold-reps", "1"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["higher_is_better"] is True and d["value"] > 0
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1.5
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["check"]["ok"], c["check"]          # the benchmarked S vs the C oracle (all columns)
    assert "connected_companion" not in d          # only for the ogbn-arxiv headline
    assert d["prologue"]["create_ms"] > 0 and d["prologue"]["log1p_degree_ms"] > 0
    assert d["cpu_baseline"]["prologue_s"] > 0
    for key in ("sharded", "sharded_pubmed_rccl"):
        sh = d[key]
        assert "error" not in sh, sh
        assert sh["value"] > 0 and sh["check"]["ok"], sh["check"]


@pytest.mark.gpu
def test_bench_multi_rank_headline_rehearsal():
    """The N > 1 code path (headline = one graph row-sharded over the ranks,
    strong scaling; replicas as an extra) with 2 ranks sharing the one GPU:
    gloo process group, IPC exchange (RCCL refuses two ranks per device)."""
    env = dict(os.environ, WATS_BENCH_PG="gloo", WATS_BENCH_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={29500 + os.getpid() % 1000}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--scale-config", "pubmed", "--F", "8",
           "--exchange", "ipc", "--sharded-extra", "none", "--config", "pubmed"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["parallelism"] == "rows x2" and d["check"]["ok"], d.get("check")
    assert d["replicas"]["value"] > 0


@pytest.mark.gpu
def test_bench_multi_rank_picks_the_faster_exchange():
    """N > 1 with two exchanges: the headline is timed with both and the line is
    the faster one whose check passed; the other is attached in full."""
    env = dict(os.environ, WATS_BENCH_PG="gloo", WATS_BENCH_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={30500 + os.getpid() % 1000}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--scale-config", "pubmed", "--F", "8",
           "--exchange", "ipc,host", "--sharded-extra", "none", "--config", "pubmed", "--replicas", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    cmp = d["exchange_compare"]
    assert set(cmp) == {"ipc", "host"} and all(v["check_ok"] for v in cmp.values()), cmp
    best = max(cmp, key=lambda x: cmp[x]["value"])
    assert d["config"]["exchange"] == best and d["value"] == cmp[best]["value"]
    other = "host" if best == "ipc" else "ipc"
    assert d[f"sharded_pubmed_{other}"]["value"] == cmp[other]["value"]


def test_byte_models_cpu():
    """bench.py's byte models (no GPU): SURVEY 8(d)'s forward-recurrence B_step
    and the Clenshaw form, which drops the S read + write (8 B) and adds the
    X0 read (4 B) per row and column."""
    sys.path.insert(0, REPO)
    import bench
    n, nnz, F = 93_861, 2_315_600, 40
    assert bench.algorithmic_bytes(n, nnz, F) == 8 * nnz + 4 * (n + 1) + 20 * n * F
    assert bench.algorithmic_bytes(n, nnz, F) - bench.clenshaw_bytes(n, nnz, F) == 4 * n * F
    assert bench.algorithmic_bytes(n, nnz, F) == 93_989_048   # the active-row B_step quoted in DESIGN.md 4.1
    # unweighted: no CSR values (4 B/nnz), plus the float64 dinv of each row
    assert bench.clenshaw_bytes(n, nnz, F) - bench.clenshaw_bytes(n, nnz, F, unit=True) == 4 * nnz - 8 * n
