"""CLI stdout contract and multi-rank runs, each as a fresh child process.

* The four CLIs (s-blas_amd/bin/test_spmv, test_spmm, test_sptrsv,
  test_sptrans) are run with the reference harness's argv and their stdout is
  parsed exactly as run_test.py:29-43 (spmv), :69-80 (sptrsv), :114-126
  (sptrans) and :146-160 (spmm) do; the pass markers each prints are
  asserted.
* BASELINE configs[2] (CSR5 kernel, nnz-balanced rows, literal allreduce of
  y) and the cyclic allgather are run as 2 ranks on the box's GPU through
  bench.py -> sblas_dist (the real multi-rank classes, HIP kernels), over
  gloo so both ranks can share one GPU, at the full config-2 size; bench.py
  --check compares the assembled y with the oracle.  torch.distributed.run
  starts the ranks as new processes (no GPU call precedes them in the child).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "s-blas_amd", "bin")
QH = os.path.join(GOLDEN, "qh768.mtx")
ASH = os.path.join(GOLDEN, "ash85.mtx")


def run(args, timeout=120):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    return r.returncode, r.stdout, r.stderr


# --- run_test.py parsers (same tokenisation) --------------------------------
def parse_spmv(result):
    m = n = nnz = None
    times = None
    rows = []
    for line in result.strip().split("\n"):
        l = line.strip()
        if l.startswith("m:"):
            words = l.strip("\n").split(" ")
            m, n, nnz = int(words[1]), int(words[3]), int(words[5])
        if l.startswith("Average"):
            words = [i for i in l.strip("\n").split(" ") if i]
            times = (float(words[1]), float(words[2]), float(words[3]))
        elif l and l[0].isdigit() and l.split()[-1] in ("Y", "N", "N/A"):
            rows.append(l.split())
    return m, n, nnz, times, rows


def parse_sptrsv(result):
    m = n = nnz = t = None
    for line in result.strip().split("\n"):
        l = line.strip()
        if l.startswith("input matrix A:"):
            words = l.strip("\n").split(" ")
            m, n, nnz = int(words[4][:-1]), int(words[5]), int(words[9])
        if l.startswith("cuda syncfree SpTRSV solve used"):
            t = float(l.strip("\n").split(" ")[5])
    return m, n, nnz, t


def parse_sptrans(result):
    m = n = nnz = t = None
    for line in result.strip().split("\n"):
        l = line.strip()
        if l.startswith("input matrix A:"):
            words = l.strip("\n").split(" ")
            m, n, nnz = int(words[4][:-1]), int(words[5]), int(words[9])
        if l.startswith("SpTrans computation time:"):
            t = float(l.strip("\n").split(" ")[3])
    return m, n, nnz, t


def parse_spmm(result):
    m = n = k = nnz = t = None
    for line in result.strip().split("\n"):
        l = line.strip()
        if l.startswith("Matrix A --"):
            words = l.strip("\n").split(" ")
            m, n, nnz = int(words[4]), int(words[6]), int(words[8])
        if l.startswith("Matrix B --"):
            k = int(l.strip("\n").split(" ")[6])
        if l.startswith("SPMM:"):
            t = float(l.strip("\n").split(" ")[5])
    return m, n, k, nnz, t


def flags(row):
    """The two Pass columns of a test row (the test number and the baseline
    time can touch, as setw(10)/setw(11) print them, so count from the flags)."""
    return [w for w in row if w in ("Y", "N", "N/A")]


# --- CLIs ---------------------------------------------------------------------
@pytest.mark.parametrize("ngpu", [1, 2, 3])
@pytest.mark.parametrize("kernel", [1, 2, 3])
@pytest.mark.parametrize("loader", ["default", "ref"])
def test_cli_spmv(ngpu, kernel, loader):
    args = [os.path.join(BIN, "test_spmv"), "f", QH, str(ngpu), "3", str(kernel), "f"]
    if loader == "ref":
        args.append("--ref-loader")
    rc, out, err = run(args)
    assert rc == 0, out + err
    m, n, nnz, times, rows = parse_spmv(out)
    assert (m, n, nnz) == (768, 768, 2934)
    assert times is not None and all(t > 0 for t in times)
    assert len(rows) == 3 and all(flags(r) == ["Y", "Y"] for r in rows), out


def test_cli_spmv_generator_and_binary():
    rc, out, err = run([os.path.join(BIN, "test_spmv"), "g", "1000", "2", "1", "1"])
    assert rc == 0, out + err
    m, n, nnz, times, rows = parse_spmv(out)
    assert (m, n) == (1000, 1000) and nnz > 0 and rows and flags(rows[0]) == ["Y", "Y"]
    rc, out, err = run([os.path.join(BIN, "test_spmv"), "f", ASH, "2", "1", "2", "b"])
    assert rc == 0, out + err
    m, n, nnz, times, rows = parse_spmv(out)
    assert m == 85 and rows and flags(rows[0]) == ["Y", "Y"]


@pytest.mark.parametrize("ngpu", [1, 2])
def test_cli_spmm(ngpu):
    rc, out, err = run([os.path.join(BIN, "test_spmm"), QH, "128", str(ngpu), "1"])
    assert rc == 0, out + err
    m, n, k, nnz, t = parse_spmm(out)
    assert (m, n, nnz, k) == (768, 768, 2934, 128) and t > 0
    assert "mgpu check: PASS" in out


@pytest.mark.parametrize("mtx", [QH, ASH], ids=["qh768", "ash85"])
@pytest.mark.parametrize("ngpu", [1, 2])
@pytest.mark.parametrize("rhs", [1, 5])
@pytest.mark.parametrize("sub", ["-forward", "-backward"])
def test_cli_sptrsv(mtx, ngpu, rhs, sub):
    rc, out, err = run([os.path.join(BIN, "test_sptrsv"), "-n", str(ngpu), "-rhs", str(rhs), sub,
                        "-mtx", mtx])
    assert rc == 0, out + err
    m, n, nnz, t = parse_sptrsv(out)
    assert m == n and nnz > 0 and t is not None and t >= 0
    assert "cuda syncfree SpTRSV executor passed!" in out


@pytest.mark.parametrize("ngpu,task", [(1, 4), (2, 2)])
def test_cli_sptrsv_v3_tasks(ngpu, task):
    """test_sptrsv -k <task>: sptrsv_v3's ngpu*task round-robin tasks."""
    rc, out, err = run([os.path.join(BIN, "test_sptrsv"), "-n", str(ngpu), "-rhs", "1", "-forward",
                        "-mtx", QH, "-k", str(task)])
    assert rc == 0, out + err
    m, n, nnz, t = parse_sptrsv(out)
    assert m == 768 and t is not None
    assert out.count("nnz for device") == ngpu * task
    assert "cuda syncfree SpTRSV executor passed!" in out


@pytest.mark.parametrize("ngpu", [1, 3])
def test_cli_sptrans(ngpu):
    rc, out, err = run([os.path.join(BIN, "test_sptrans"), "-n", str(ngpu), "-csr", "-mtx", QH])
    assert rc == 0, out + err
    m, n, nnz, t = parse_sptrans(out)
    assert (m, n, nnz) == (768, 768, 2934) and t is not None
    for what in ("value", "pointer", "row index"):
        assert f"sptrans {what} test on multiple GPU: passed!" in out


# --- 2 ranks on one GPU through sblas_dist ------------------------------------
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def bench_2rank(extra, nrows=2_000_000):
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
            os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
            "--dist-backend", "gloo", "--check", "--no-cpu-baseline", "--nrows", str(nrows)] + extra
    rc, out, err = run(args, timeout=110)
    assert rc == 0, out[-3000:] + err[-3000:]
    line = [l for l in out.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("extra", [
    ["--algo", "csr5", "--partition", "nnz", "--exchange", "allreduce"],
    ["--algo", "csr5"],
    ["--algo", "xsort"],
    ["--algo", "panel", "--partition", "nnz"],
    ["--algo", "xsort", "--overlap"]],
    ids=["cfg3_csr5_nnz_allreduce", "csr5_cyclic_allgather", "xsort_cyclic_allgather",
         "panel_nnz_allgather", "xsort_cyclic_overlap_halves"])
def test_config3_two_ranks(extra):
    """BASELINE configs[2]'s dataflow on 2 ranks at full size, checked."""
    cfg3 = extra[1] == "csr5" and "allreduce" in extra
    out = bench_2rank(extra if cfg3 else extra + ["--no-config3"])
    assert out["n_gpus"] == 2 and out["check_vs_oracle"] is True, out
    assert out["config"]["nnz"] == 39_750_000
    if cfg3:  # the line's configs[2] leg (torch path: one process per rank)
        c3 = out["config3"]
        assert c3["check"] is True and c3["n_gpus"] == 2 and c3["exchange"] == "allreduce", c3
        assert sum(c3["nnz_per_device"]) == 39_750_000


@pytest.mark.parametrize("split,ranks,ncols", [("rows", 2, 64), ("rows", 3, 64), ("cols", 2, 64), ("cols", 3, 64),
                                               ("grid", 2, 64), ("grid", 4, 32)])
def test_spmm_multi_rank_config4(split, ranks, ncols):
    """sblas_dist.DistSpMM on 2-4 ranks (torchrun children, gloo exchange,
    HIP kernels) at BASELINE configs[3]'s full size (rail4284-shaped, 4,284 x
    1,092,610, 11.28M nnz, 64 columns): the north star's row blocks, the
    reference's column split, and the 2-D grid (2 ranks: 2 column groups; 4
    ranks at 32 columns: 2 row blocks x 2 column groups).  Rank 0 compares
    EVERY entry of the assembled C with the oracle (orc_spmm_omp) under the
    per-entry fp64 bound, as dspmm_baseline_test.cu:544-549 checks every
    entry."""
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
            os.path.join(ROOT, "s-blas_amd", "tools", "bench_spmm.py"), "--steps", "2", "--warmup", "1",
            "--dist-backend", "gloo", "--split", split, "--check", "--no-cpu-baseline", "--ncols", str(ncols)]
    rc, out, err = run(args, timeout=115)
    assert rc == 0, out[-3000:] + err[-3000:]
    res = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == ranks and res["config"]["nnz"] == 11_279_748, res
    chk = res["check_vs_oracle"]
    assert chk["entries"] == 4284 * ncols and chk["pass"] and chk["abs_1e-3"], chk


def test_torchrun_8_ranks_full_size():
    """The path the driver's 8-GPU scaling run takes (torch.distributed.run,
    one process per rank, `bench.py --gpus 8`), rehearsed with 8 ranks sharing
    the box's GPU over gloo at the full config-2 size: the default leg
    (cyclic chunks, all-gather + placement) and the configs[2] leg (CSR5 on
    the nnz split, all-reduce of y) both checked against the oracle, every
    rank's configs[2] y bit-identical."""
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
            os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
            "--dist-backend", "gloo", "--check", "--no-cpu-baseline"]
    rc, out, err = run(args, timeout=115)
    assert rc == 0, out[-3000:] + err[-3000:]
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["check_vs_oracle"] is True, line
    assert line["config"]["nnz"] == 39_750_000
    c3 = line["config3"]
    assert c3["check"] is True and c3["n_gpus"] == 8 and c3["exchange"] == "allreduce", c3
    assert len(c3["kernel_ms_per_device"]) == 8 and sum(c3["nnz_per_device"]) == 39_750_000
    # first contact: the communicator and devices the line ran on
    topo = line["topology"]
    assert topo["comm_ranks"] == 8 and topo["backend"] == "gloo", topo
    nd = topo["visible_devices"]
    assert topo["device_ordinals"] == [r % nd for r in range(8)] and len(topo["pci_bus"]) == 8, topo
    assert len(topo["peer_access"]) == nd
    b4 = line["config5"]["blocks4"]
    assert b4["check_exact_vs_xref"] and len(b4["block_devices"]) == 4 and sum(b4["block_rows"]) == 5_558_326, b4
