"""SpMV parity on the GPU: HIP kernels (via libsblas C-ABI) vs the oracle.

Tolerance (DESIGN.md "Parity"): per row
  |y_gpu - y_ref| <= 4*gamma_k*sum_j |alpha*a_ij*x_j| + 4u*|beta*y0|,
gamma_k = k*u/(1-k*u), u = 2^-53, k = row length.  The reference's own abs
1e-3 check (spmv/test/dspmv_test.cu:390-401) is asserted as well.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

# (algorithm, planner test options -- sblas.test_options, never the
# environment).  The panel algorithm (4) picks ~4 MiB of x per panel, i.e.
# one panel for these small matrices; 3 and 8 panels are forced too so the
# multi-panel path (interleaved grid + partial reduce) runs.  The
# column-sorted algorithm (5) makes every range wide (one sub-item per XCD +
# the partial reduce) on matrices of <= 6M entries, so these small cases run
# the all-wide layout by default; xs_allwide=0 restores the planner's narrow
# ranges (few, for small matrices; a tiny work cap, xs_cap, forces many, most
# of them wide and paired with narrow ones, claimed dynamically); xs_solo=1
# the solo narrow items of power-law plans.  "det" runs the handle in
# deterministic mode (xsort's ordered form).
ALGOS = [(0, {}), (1, {}), (2, {}), (2, {"csr5_hostplan": 1}),
         (2, {"csr5_panel": 1, "panels": 3}), (2, {"csr5_panel": 1, "panels": 8}),
         (4, {}), (4, {"panels": 3}), (4, {"panels": 8}),
         (5, {}), (5, {"xs_cap": 50}), (5, {"xs_allwide": 1}),
         (5, {"xs_allwide": 0}), (5, {"xs_allwide": 0, "xs_cap": 50}),
         (5, {"xs_solo": 1}), (5, {"xs_solo": 1, "xs_cap": 50}),
         (2, {"csr5_panel": 1, "panels": 2}), (1, {"rs_panel": 1, "panels": 3}),
         (5, {"det": 1}), (5, {"det": 1, "xs_cap": 50}), (5, {"det": 1, "xs_allwide": 0}),
         (5, {"det": 1, "xs_solo": 1, "xs_cap": 50}), (0, {"det": 1})]
ALGO_IDS = ["auto", "rowsplit", "csr5", "csr5_hostplan", "csr5_panel3", "csr5_panel8", "panel", "panel3",
            "panel8", "xsort", "xsort_cap50", "xsort_allwide", "xsort_narrow", "xsort_narrow_cap50",
            "xsort_solo", "xsort_solo_cap50", "csr5_panel2", "rowsplit_panel3", "xsort_det",
            "xsort_det_cap50", "xsort_det_narrow", "xsort_det_solo_cap50", "auto_det"]
DET = {"on": False}


@pytest.fixture(params=ALGOS, ids=ALGO_IDS)
def algo(request, sb):
    a, opts = request.param
    opts = dict(opts)
    DET["on"] = bool(opts.pop("det", 0))
    with sb.test_options(**opts):
        yield a
    DET["on"] = False


def random_csr(rng, m, n, density_rows, long_rows=(), empty_frac=0.1):
    lens = rng.integers(0, density_rows, size=m)
    lens[rng.random(m) < empty_frac] = 0
    for r, L in long_rows:
        lens[r] = L
    lens = np.minimum(lens, n)
    rp = np.zeros(m + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    col = np.concatenate([np.sort(rng.choice(n, size=L, replace=False)) for L in lens]
                         ).astype(np.int32) if rp[-1] else np.zeros(0, np.int32)
    val = rng.standard_normal(int(rp[-1]))
    return rp, col, val


def run_gpu(torch, sb, algo, n, rp, col, val, x, alpha, beta, y0, det=None):
    A = sb.DeviceCSR.upload(0, n, rp, col, val)
    A.deterministic = DET["on"] if det is None else det
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    yd = torch.from_numpy(np.ascontiguousarray(y0)).cuda()
    A.analyse(algo)
    A.spmv(algo, alpha, xd.data_ptr(), beta, yd.data_ptr())
    torch.cuda.synchronize()
    out = yd.cpu().numpy()
    A.close()
    return out


def check(orc, rp, col, val, x, alpha, beta, y0, got):
    want = orc.csr_spmv(rp, col, val, x, alpha, beta, y0)
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y0)
    err = np.abs(got - want)
    assert np.all(err <= bound), f"max excess {np.max(err - bound)} at {np.argmax(err - bound)}"
    assert np.all(np.abs(got - want) <= 1e-3 * np.maximum(1.0, np.abs(want)))


@pytest.mark.parametrize("mode", [0, 1])
def test_qh768(torch_cuda, sb, orc, algo, mode):
    path = os.path.join(GOLDEN, "qh768.mtx")
    m, n, rp, col, val = sb.mm_read(path, mode)
    alpha, beta = orc.alpha_beta()
    x = np.ones(n)
    y0 = np.zeros(m)
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, alpha, beta, y0)
    check(orc, rp, col, val, x, alpha, beta, y0, got)


@pytest.mark.parametrize("prefix", [False, True])
def test_synthetic(torch_cuda, sb, orc, algo, prefix):
    n = 20000
    rp, col, val = orc.gen_synth(n, prefix=prefix)
    x = orc.gen_vector(n, 43)
    alpha, beta = orc.alpha_beta()
    y0 = orc.gen_vector(n, 44)
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, alpha, beta, y0)
    check(orc, rp, col, val, x, alpha, beta, y0, got)


@pytest.mark.parametrize("beta", [0.0, 0.75])
def test_ragged_long_empty(torch_cuda, sb, orc, algo, beta):
    rng = np.random.default_rng(7)
    m, n = 3000, 40000
    rp, col, val = random_csr(rng, m, n, 60, long_rows=[(5, 2049), (17, 8192), (900, 30000),
                                                          (2999, 9000), (1500, 20000)])
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    if beta == 0.0:
        y0[::7] = np.nan  # beta == 0 must not read y
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, 1.25, beta, y0)
    y0c = np.where(np.isnan(y0), 0.0, y0)
    check(orc, rp, col, val, x, 1.25, beta, y0c, got)


@pytest.mark.parametrize("beta", [0.0, 0.75])
def test_mostly_empty_rows(torch_cuda, sb, orc, algo, beta):
    """60% empty rows (a power-law graph's share): xsort takes its solo layout
    by default (>= 40% empty), the other algorithms their usual one."""
    rng = np.random.default_rng(11)
    m, n = 60000, 70000
    rp, col, val = random_csr(rng, m, n, 40, long_rows=[(3, 3000), (31000, 12000)], empty_frac=0.6)
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, 0.5, beta, y0)
    check(orc, rp, col, val, x, 0.5, beta, y0, got)


def test_edge_shapes(torch_cuda, sb, orc, algo):
    rng = np.random.default_rng(3)
    # all rows empty
    m, n = 100, 50
    rp = np.zeros(m + 1, np.int64)
    got = run_gpu(torch_cuda, sb, algo, n, rp, np.zeros(0, np.int32), np.zeros(0), np.ones(n),
                  2.0, 0.5, np.ones(m))
    assert np.array_equal(got, np.full(m, 0.5))
    # one dense row; many leading empty rows
    for m, n in [(1, 1000), (5000, 1000)]:
        rp = np.zeros(m + 1, np.int64)
        rp[-1] = n
        col = np.arange(n, dtype=np.int32)
        val = rng.standard_normal(n)
        x = rng.standard_normal(n)
        y0 = rng.standard_normal(m)
        got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, 0.5, -1.0, y0)
        check(orc, rp, col, val, x, 0.5, -1.0, y0, got)
    # rows of length 1 (tile boundaries everywhere), nnz not a multiple of 4
    m = n = 4099
    rp = np.arange(m + 1, dtype=np.int64)
    col = rng.integers(0, n, size=m).astype(np.int32)
    val = rng.standard_normal(m)
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, 1.0, 1.0, y0)
    check(orc, rp, col, val, x, 1.0, 1.0, y0, got)


@pytest.mark.parametrize("case", ["ragged", "empty_runs", "tile_rows", "synth"])
def test_csr5_device_plan_matches_host_plan(torch_cuda, sb, orc, monkeypatch, case):
    """CSR5 tile descriptors built on the device (row-start bits, tile rows,
    empty-row segment lists; format_cuda.h:21-300's job) give the same y, bit
    for bit, as the host-built descriptors (test option csr5_hostplan)."""
    rng = np.random.default_rng(11)
    if case == "ragged":
        m, n = 3000, 40000
        rp, col, val = random_csr(rng, m, n, 60, long_rows=[(5, 2049), (17, 8192), (900, 30000)])
    elif case == "empty_runs":  # long runs of empty rows inside and across tiles
        m, n = 20000, 5000
        lens = np.zeros(m, np.int64)
        live = rng.choice(m, 900, replace=False)
        lens[live] = rng.integers(1, 40, 900)
        lens[-1] = 3000
        rp = np.concatenate([[0], np.cumsum(lens)])
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    elif case == "tile_rows":  # rows of exactly one tile, and of 1 / 16 entries
        m, n = 600, 3000
        lens = rng.choice([1, 16, 1024, 0], m)
        rp = np.concatenate([[0], np.cumsum(lens)])
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    else:
        m = n = 20000
        rp, col, val = orc.gen_synth(n)
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    got = run_gpu(torch_cuda, sb, 2, n, rp, col, val, x, 1.5, 0.5, y0)
    with sb.test_options(csr5_hostplan=1):
        want = run_gpu(torch_cuda, sb, 2, n, rp, col, val, x, 1.5, 0.5, y0)
    assert np.array_equal(got, want)
    check(orc, rp, col, val, x, 1.5, 0.5, y0, got)


def test_repeat_deterministic(torch_cuda, sb, orc):
    n = 5000
    rp, col, val = orc.gen_synth(n)
    x = orc.gen_vector(n, 43)
    outs = [run_gpu(torch_cuda, sb, a, n, rp, col, val, x, 1.0, 0.0, np.zeros(n))
            for a in (1, 1, 2, 2, 4, 4)]
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[2], outs[3])
    assert np.array_equal(outs[4], outs[5])


@pytest.mark.parametrize("opts", [{}, {"xs_allwide": 0}, {"xs_allwide": 0, "xs_cap": 50},
                                  {"xs_solo": 1, "xs_cap": 50}])
def test_xsort_deterministic_mode(torch_cuda, sb, orc, opts):
    """a deterministic handle's xsort launches give the
    same y bit for bit (chunk-ordered adds, fixed narrow walk), within the
    per-row bound; the reference compares repeated runs the same way
    (spmv/test/dspmv_test.cu:390-401)."""
    n = 60000
    rp, col, val = orc.gen_synth(n)
    x = orc.gen_vector(n, 43)
    y0 = orc.gen_vector(n, 44)
    with sb.test_options(**opts):
        A = sb.DeviceCSR.upload(0, n, rp, col, val)
        A.deterministic = True
        A.analyse(5)
    xd = torch_cuda.from_numpy(x).cuda()
    outs = []
    for _ in range(6):
        yd = torch_cuda.from_numpy(y0.copy()).cuda()
        A.spmv(5, 0.75, xd.data_ptr(), -1.5, yd.data_ptr())
        torch_cuda.cuda.synchronize()
        outs.append(yd.cpu().numpy())
    A.close()
    for o in outs[1:]:
        assert np.array_equal(outs[0], o), f"{np.sum(outs[0] != o)} rows differ"
    check(orc, rp, col, val, x, 0.75, -1.5, y0, outs[0])


@pytest.mark.parametrize("opts", [{}, {"xs_cap": 50}, {"xs_allwide": 0}, {"xs_allwide": 0, "xs_cap": 50},
                                  {"xs_solo": 1, "xs_cap": 50}])
def test_xsort_relaunch(torch_cuda, sb, orc, opts):
    """The column-sorted kernel's work queues re-arm themselves at the end of
    each launch (no memset): five launches on one plan, each checked."""
    n = 20000
    rp, col, val = orc.gen_synth(n)
    x = orc.gen_vector(n, 43)
    with sb.test_options(**opts):
        A = sb.DeviceCSR.upload(0, n, rp, col, val)
        A.analyse(5)
    xd = torch_cuda.from_numpy(x).cuda()
    want = orc.csr_spmv(rp, col, val, x, 1.5, 0.0, np.zeros(n))
    bound = orc.spmv_bound(rp, col, val, x, 1.5, 0.0, np.zeros(n))
    for it in range(5):
        yd = torch_cuda.full((n,), np.nan, dtype=torch_cuda.float64, device="cuda")
        A.spmv(5, 1.5, xd.data_ptr(), 0.0, yd.data_ptr())
        torch_cuda.cuda.synchronize()
        got = yd.cpu().numpy()
        assert np.all(np.abs(got - want) <= bound), f"launch {it}"
    A.close()


@pytest.mark.parametrize("version", ["baseline", "v1", "v2"])
@pytest.mark.parametrize("ngpu", [1, 2, 3, 8])
def test_reference_api(torch_cuda, sb, orc, version, ngpu):
    """spMV_mgpu_* drop-in (host pointers); ordinals wrap onto the box's GPU."""
    rng = np.random.default_rng(11)
    m, n = 2500, 3000
    rp, col, val = random_csr(rng, m, n, 40, long_rows=[(10, 2500)])
    x = rng.standard_normal(n)
    alpha, beta = orc.alpha_beta()
    y0 = rng.standard_normal(m)
    for kernel in ([1] if version == "baseline" else [1, 2, 3]):
        y = y0.copy()
        nb = max(int(rp[-1]) // 5, 1) if version == "v2" else None
        rc = sb.spmv_mgpu(version, m, n, rp, col, val, x, y, alpha, beta, ngpu=ngpu,
                          kernel=kernel, nb=nb, q=2)
        assert rc == 0
        check(orc, rp, col, val, x, alpha, beta, y0, y)
        if version != "v2":
            y_ref_flow = orc.spmv_mgpu(version, m, n, rp, col, val, x, alpha, beta, y0, ngpu)
            assert np.all(np.abs(y - y_ref_flow) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y0))


@pytest.mark.parametrize("chunk", [37, 1000, 20000, 1 << 30])
@pytest.mark.parametrize("nstreams", [1, 3])
@pytest.mark.parametrize("ngpu", [1, 2])
@pytest.mark.parametrize("beta_zero", [False, True])
def test_spmv_out_of_core(torch_cuda, sb, orc, chunk, nstreams, ngpu, beta_zero):
    """Out-of-core executor: host CSR streamed in chunks; tiny
    chunks make rows span many chunks (continuations), a 9000-nnz row spans
    chunks and the 8192-nnz long-row path, empty rows stay beta*y0."""
    rng = np.random.default_rng(chunk + 7 * nstreams)
    m, n = 3000, 12000
    rp, col, val = random_csr(rng, m, n, 30, long_rows=[(17, 9000)], empty_frac=0.2)
    x = rng.standard_normal(n)
    alpha, beta = orc.alpha_beta()
    if beta_zero:
        beta = 0.0
    y0 = rng.standard_normal(m)
    y = y0.copy()
    st = sb.spmv_ooc(m, n, rp, col, val, x, alpha, beta, y, ngpu=ngpu, chunk_nnz=chunk,
                     nstreams=nstreams)
    assert st["chunks"] == max(1, -(-int(rp[-1]) // min(chunk, 1 << 30)))
    check(orc, rp, col, val, x, alpha, beta, y0, y)


@pytest.mark.parametrize("kind", ["stencil7", "stencil27", "rmat"])
def test_suitesparse_class(torch_cuda, sb, orc, algo, kind):
    """Every kernel on the SuiteSparse-class generators bench.py --matrix
    offers: 3-D 7- and 27-point stencils (banded, structured) and an R-MAT
    power-law graph (rows of 0 to ~1,000 entries, hot columns)."""
    if kind == "rmat":
        rp, col, val = sb.gen_rmat(11, 16, seed=5)
    else:
        rp, col, val = sb.gen_stencil3d(13, 11, 9, int(kind[7:]), seed=6)
    n = len(rp) - 1
    x = orc.gen_vector(n, 43)
    y0 = orc.gen_vector(n, 45)
    alpha, beta = orc.alpha_beta()
    got = run_gpu(torch_cuda, sb, algo, n, rp, col, val, x, alpha, beta, y0)
    check(orc, rp, col, val, x, alpha, beta, y0, got)


@pytest.mark.parametrize("case", ["random_small", "prefix", "banded_runs", "diagonal", "override", "stencil27"])
def test_auto_pick(torch_cuda, sb, orc, monkeypatch, case):
    """SBLAS_SPMV_AUTO (sblas_csr_pick): coalescing columns -> row split;
    scattered columns under 2M nonzeros -> panel; SBLAS_AUTO overrides.  The
    resolved algorithm's analysis is built by analyse(AUTO) and spmv(AUTO)
    matches the oracle."""
    rng = np.random.default_rng(5)
    n = 20000
    if case == "prefix":
        rp, col, val = orc.gen_synth(n, prefix=True)
        want_algo = sb.ROWSPLIT
    elif case == "banded_runs":
        # rows of 3 runs of 8 consecutive columns in three disjoint bands
        lens = np.full(n, 24, np.int64)
        rp = np.zeros(n + 1, np.int64)
        rp[1:] = np.cumsum(lens)
        starts = np.stack([np.arange(n) % 5990, 6000 + np.arange(n) % 5990, 12000 + np.arange(n) % 7990], 1)
        col = (starts[:, :, None] + np.arange(8)[None, None, :]).reshape(-1).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
        want_algo = sb.ROWSPLIT
    elif case == "stencil27":  # 3-D FEM-block pattern: neighbouring rows share x lines
        rp, col, val = sb.gen_stencil3d(30, 30, 22, 27, seed=6)
        n = len(rp) - 1
        want_algo = sb.ROWSPLIT
    elif case == "diagonal":  # one entry per row: locality across rows
        rp = np.arange(n + 1, dtype=np.int64)
        col = np.arange(n, dtype=np.int32)
        val = rng.standard_normal(n)
        want_algo = sb.ROWSPLIT
    else:
        rp, col, val = orc.gen_synth(n)
        want_algo = sb.PANEL
    if case == "override":
        monkeypatch.setenv("SBLAS_AUTO", "2")
        want_algo = sb.CSR5
    x = orc.gen_vector(n, 43)
    alpha, beta = orc.alpha_beta()
    y0 = orc.gen_vector(n, 44)
    A = sb.DeviceCSR.upload(0, n, rp, col, val)
    try:
        assert A.pick() == want_algo
        xd = torch_cuda.from_numpy(x).cuda()
        yd = torch_cuda.from_numpy(y0.copy()).cuda()
        A.spmv(sb.AUTO, alpha, xd.data_ptr(), beta, yd.data_ptr())  # analyses on first use
        torch_cuda.cuda.synchronize()
        assert A.plan_bytes(want_algo) >= 0
        check(orc, rp, col, val, x, alpha, beta, y0, yd.cpu().numpy())
        yd2 = torch_cuda.from_numpy(y0.copy()).cuda()
        ms = A.spmv_timed(sb.AUTO, alpha, xd.data_ptr(), beta, yd2.data_ptr())
        assert ms > 0
        check(orc, rp, col, val, x, alpha, beta, y0, yd2.cpu().numpy())
    finally:
        A.close()
