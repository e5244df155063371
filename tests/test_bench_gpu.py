"""bench.py through the single-process C-ABI context (`--driver ctx`): the
path `python bench.py --gpus N` takes without a launcher.  At N = 1 on this
pool: allgather over cyclic chunks (xsort, row split) and BASELINE
configs[2]'s literal form (CSR5 kernel, nnz-balanced rows, ncclAllReduce of
the zero-padded y).  --check compares device 0's y with the oracle under the
per-row fp64 bound and requires every device's y to be
bit-identical."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CONFIG3_KEYS = ("kernel_ms_max", "exchange_ms_max", "step_ms", "gflops", "roofline", "check")


@pytest.mark.parametrize("algo,partition,exchange", [
    ("xsort", "cyclic", "allgather"),
    ("rowsplit", "nnz", "allgather"),
    ("csr5", "nnz", "allreduce"),
    ("panel", "cyclic", "allgather"),
])
def test_bench_ctx_driver(algo, partition, exchange):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--driver", "ctx", "--check",
           "--nrows", "200000", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--algo", algo,
           "--partition", partition, "--exchange", exchange]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout  # the contract: ONE JSON line on stdout
    line = json.loads(lines[0])
    assert line["check_vs_oracle"] is True
    assert line["n_gpus"] == 1
    assert line["config"]["driver"].startswith("ctx")
    assert line["topology"]["comm_ranks"] == 1 and line["topology"]["device_ordinals"] == [0]
    assert line["config"]["exchange"] == exchange
    assert line["ms_per_step"] > 0 and line["kernel_ms_max_over_ranks"] > 0
    assert line["ms_per_step"] >= line["kernel_ms_max_over_ranks"]
    # BASELINE configs[2] rides on every line
    c3 = line["config3"]
    assert set(CONFIG3_KEYS) <= set(c3), c3
    assert c3["check"] is True and c3["algo"] == "csr5" and c3["n_gpus"] == 1
    # the north star's SuiteSparse-class stand-ins ride on every N = 1 line
    st = line["structured"]
    for kind in ("stencil27", "stencil7", "rmat"):
        assert "error" not in st[kind] and 0.0 < st[kind]["roofline_frac"] < 1.0, st[kind]


@pytest.mark.parametrize("gpus,algo,partition,exchange", [
    (2, "xsort", "cyclic", "allgather"),
    (3, "csr5", "nnz", "allreduce"),
    (8, "xsort", "cyclic", "allgather"),
    (8, "rowsplit", "nnz", "allgather"),
    (8, "csr5", "nnz", "allreduce"),
    (4, "panel", "nnz", "allreduce"),
])
def test_bench_ctx_loopback(gpus, algo, partition, exchange):
    """`bench.py --gpus N` through the ctx driver with N > 1 context ranks
    wrapped onto the box's GPU (SBLAS_CTX_LOOPBACK: the collectives become
    stream-ordered device copies / a rank-order sum instead of RCCL), so the
    N > 1 partitions, split-row carries, cyclic placement, re-priming of the
    next step's y and the per-device timing all run and are checked against
    the oracle; every rank's y must be bit-identical."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--ctx-loopback", "--check",
           "--nrows", "200000", "--steps", "2", "--warmup", "2", "--no-cpu-baseline", "--algo", algo,
           "--partition", partition, "--exchange", exchange]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["check_vs_oracle"] is True, line
    assert line["n_gpus"] == gpus and "loopback" in line["note"]
    assert len(line["kernel_ms_per_device"]) == gpus
    # first-contact readiness: what the line ran on
    topo = line["topology"]
    assert topo["comm_ranks"] == 0 and topo["backend"].startswith("loopback")
    assert len(topo["device_ordinals"]) == gpus and len(topo["pci_bus"]) == gpus
    nd = topo["visible_devices"]
    assert topo["device_ordinals"] == [d % nd for d in range(gpus)]
    assert len(topo["peer_access"]) == nd and all(len(r) == nd for r in topo["peer_access"])
    assert sum(line["nnz_per_device"]) == line["config"]["nnz"]
    c3 = line["config3"]
    assert c3["check"] is True and c3["n_gpus"] == gpus and c3["exchange"] == "allreduce", c3
    assert sum(c3["nnz_per_device"]) == line["config"]["nnz"]


def test_bench_ctx_loopback_full_config3():
    """`bench.py --gpus 8 --ctx-loopback --check` on the
    FULL n = 2e6 matrix (39.75M nnz): the default leg (cyclic chunks, the
    library's kernel per slice, all-gather + placement) and the configs[2]
    leg (CSR5 on the nnz split, all-reduce of the zero-padded y) both checked
    against the oracle under the per-row fp64 bound, every rank's y
    bit-identical.  8 context ranks share the box's GPU (loopback
    collectives); the first 8-GPU run executes the same code with RCCL."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--ctx-loopback", "--check",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["nnz"] == 39_750_000 and line["n_gpus"] == 8
    assert line["check_vs_oracle"] is True, line
    c3 = line["config3"]
    assert set(CONFIG3_KEYS) <= set(c3), c3
    assert c3["check"] is True and c3["n_gpus"] == 8 and c3["exchange"] == "allreduce", c3
    assert len(c3["kernel_ms_per_device"]) == 8 and sum(c3["nnz_per_device"]) == 39_750_000


@pytest.mark.parametrize("gpus,parts", [(2, 2), (4, 4), (8, 2), (8, 4)])
def test_bench_ctx_loopback_overlap(gpus, parts):
    """`bench.py --gpus N --overlap K` through the ctx driver (loopback): the
    exchange overlapped over K parts of every rank's chunks, checked."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--ctx-loopback", "--check",
           "--nrows", "200000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-config3",
           "--overlap", str(parts)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["check_vs_oracle"] is True, line
    assert line["config"]["overlap_parts"] == parts
