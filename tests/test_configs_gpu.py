"""Full-size parity on BASELINE.json configs[1..4] ("next round" 1).

Every case runs the HIP kernels through libsblas's C-ABI at the size the
config names and checks every output against the oracle (tests/orc.py):

* config 2: synthetic non-uniform n = 2e6, 39.75M nnz (bench.py's matrix),
  every SpMV algorithm, per-row fp64 bound of DESIGN.md §3 (reference
  check site spmv/test/dspmv_test.cu:390-401 uses abs 1e-3, asserted too);
  the default column-sorted plan (G = 16 column groups at this n) is
  relaunched 25 times on one plan so the self-rearming queues are covered;
* config 4: rail4284-shaped SpMM (4284 x 1,092,610, 11.28M nnz, 64 columns
  of B), every entry of C against orc_spmm's arithmetic with its bound;
* config 5: circuit5M-class forward solve (n = 5,558,326, 33.35M nnz):
  an integer KAT (unit diagonal, off-diagonals 1..10, x_ref in 1..10 -- the
  structure of sptrsv_v1/src/main.cu:150-355, exact in fp64 whatever the
  summation order) that must come back bit-exact on one device and on 4
  blocks, and the bench's real-valued system against the reference's
  serial executor (orc_sptrsv_serial, pinned to sptrsv_syncfree_serialref.h)
  with rel-L1 <= 1e-12.
The 2-rank config-3 run lives in tests/test_cli_gpu.py (child processes).
"""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(ROOT, "s-blas_amd", "tools"))

N2 = 2_000_000


def _check_spmv(want, bound, got, what):
    err = np.abs(got - want)
    bad = ~(err <= bound)
    assert not bad.any(), f"{what}: {bad.sum()} rows over the bound, max excess {np.max(err - bound)}"
    assert np.all(err <= 1e-3 * np.maximum(1.0, np.abs(want))), what


@pytest.fixture(scope="module", params=["random", "prefix"])
def cfg2(request, sb, orc, torch_cuda):
    torch = torch_cuda
    prefix = request.param == "prefix"
    rp = sb.gen_synth_rowptr(N2)
    col, val = sb.gen_synth_rows(N2, rp, 0, N2, prefix=prefix, seed=42)
    assert int(rp[-1]) == 39_750_000
    x = sb.gen_vector(N2, 43)
    y0 = sb.gen_vector(N2, 44)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y0)
    d = dict(rp=rp, col=col, val=val, alpha=alpha, beta=beta, want=want, bound=bound,
             prefix=prefix, xd=torch.from_numpy(x).cuda(), y0d=torch.from_numpy(y0).cuda())
    yield d


def _run_cfg2(torch, sb, c, algo, launches=1, det=False):
    """launches of one plan, each against the oracle; returns the y's."""
    A = sb.DeviceCSR.upload(0, N2, c["rp"], c["col"], c["val"])
    A.deterministic = det
    ys = []
    try:
        A.analyse(algo)
        yd = torch.empty_like(c["y0d"])
        for it in range(launches):
            yd.copy_(c["y0d"])
            A.spmv(algo, c["alpha"], c["xd"].data_ptr(), c["beta"], yd.data_ptr())
            torch.cuda.synchronize()
            ys.append(yd.cpu().numpy())
            _check_spmv(c["want"], c["bound"], ys[-1], f"algo {algo} launch {it}")
    finally:
        A.close()
    return ys


@pytest.mark.parametrize("algo,opts", [
    (1, {}), (2, {}), (3, {}), (2, {"csr5_panel": 0}), (1, {"rs_panel": 0}), (4, {}), (5, {}),
    (5, {"xs_allwide": 1}), (5, {"xs_solo": 1})],
    ids=["rowsplit", "csr5", "csr5_alt", "csr5_plain", "rowsplit_plain", "panel", "xsort", "xsort_allwide",
         "xsort_solo"])
def test_config2_full_size(torch_cuda, sb, cfg2, algo, opts):
    """BASELINE configs[1] at full size, every algorithm against the oracle
    (planner test options force the non-default layouts)."""
    launches = 25 if (algo == 5 and opts in ({}, {"xs_solo": 1}) and not cfg2["prefix"]) else 1
    with sb.test_options(**opts):
        _run_cfg2(torch_cuda, sb, cfg2, algo, launches)


def test_config2_auto_deterministic(torch_cuda, sb, cfg2):
    """on a deterministic handle (SBLAS_DETERMINISTIC /
    sblas_csr_set_deterministic) AUTO's launches on config 2 are bitwise
    equal and within the per-row bound; AUTO still picks xsort (its ordered
    form).  Without the flag xsort's LDS-atomic order varies."""
    A = sb.DeviceCSR.upload(0, N2, cfg2["rp"], cfg2["col"], cfg2["val"])
    try:
        want = sb.ROWSPLIT if cfg2["prefix"] else sb.XSORT
        assert A.pick() == want
    finally:
        A.close()
    ys = _run_cfg2(torch_cuda, sb, cfg2, sb.AUTO, launches=4, det=True)
    for it, y in enumerate(ys[1:], 1):
        assert np.array_equal(ys[0], y), f"launch {it}: {np.sum(ys[0] != y)} rows differ"


@pytest.fixture(scope="module")
def rmat21(sb, orc, torch_cuda):
    """bench.py's structured R-MAT leg: 2^21 vertices, edge factor 16, seed 50."""
    rp, col, val = sb.gen_rmat(21, 16, seed=50)
    n = len(rp) - 1
    x = sb.gen_vector(n, 43)
    y0 = sb.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y0)
    yield dict(n=n, rp=rp, col=col, val=val, alpha=alpha, beta=beta, want=want, bound=bound,
               xd=torch_cuda.from_numpy(x).cuda(), y0d=torch_cuda.from_numpy(y0).cuda())


@pytest.mark.parametrize("opts", [{}, {"det": 1}, {"xs_cap": 2000}])
def test_rmat21_xsort(torch_cuda, sb, rmat21, opts):
    """the R-MAT scale-21 stand-in at full size (the
    bench's structured leg) through AUTO's xsort plan (solo narrow items),
    every row within the per-row bound; relaunched so the self-rearming
    queues run; a deterministic handle's launches bitwise equal; a small
    sub-item cap (many more items than workgroups: the dynamic claims)."""
    c = rmat21
    opts = dict(opts)
    det = bool(opts.pop("det", 0))
    with sb.test_options(**opts):
        A = sb.DeviceCSR.upload(0, c["n"], c["rp"], c["col"], c["val"])
    A.deterministic = det
    try:
        with sb.test_options(**opts):
            assert A.pick() == sb.XSORT
            A.analyse(sb.XSORT)
        info = A.xsort_info()
        assert info["solo"] == 1
        ys = []
        yd = torch_cuda.empty_like(c["y0d"])
        for it in range(3):
            yd.copy_(c["y0d"])
            A.spmv(sb.XSORT, c["alpha"], c["xd"].data_ptr(), c["beta"], yd.data_ptr())
            torch_cuda.cuda.synchronize()
            ys.append(yd.cpu().numpy())
            _check_spmv(c["want"], c["bound"], ys[-1], f"rmat21 {opts} det={det} launch {it}")
        if det:
            assert all(np.array_equal(ys[0], y) for y in ys[1:])
    finally:
        A.close()


def test_config2_xcd_panel_choice(torch_cuda, sb, cfg2):
    """Row split and CSR5 run over XCD column panels on config 2's random
    columns (x = 16 MB > 8 MiB, 39.75M nnz, rows spanning most of x): 4 for
    the row split, 8 for CSR5 from 32M entries; both keep the plain layout on
    the reference generator's prefix columns; PANEL always uses panels
    (sblas_csr_panels, spmv.hip xcd_panels_pay)."""
    A = sb.DeviceCSR.upload(0, N2, cfg2["rp"], cfg2["col"], cfg2["val"])
    try:
        for algo in (sb.ROWSPLIT, sb.CSR5, sb.PANEL):
            A.analyse(algo)
        want = 0 if cfg2["prefix"] else 4
        assert A.panels(sb.ROWSPLIT) == want and A.panels(sb.CSR5) == 2 * want
        assert A.panels(sb.PANEL) == 4 or cfg2["prefix"]
    finally:
        A.close()


@pytest.mark.parametrize("world", [4, 8])
def test_config2_slice_xcd_panel_choice(torch_cuda, sb, orc, cfg2, world):
    """Rank 0's cyclic slice at N = 4 (9.9M nnz) and N = 8 (5M): the row split
    and CSR5 take 4 panels from 2M entries (profiles/r05/c5P/); both stay
    within the bound against the oracle on the slice."""
    import sblas_dist
    rp = cfg2["rp"]
    plan = sblas_dist.make_cyclic_plan(rp, N2, world)
    lrp, col, val = sblas_dist.cyclic_local_csr(rp, plan, 0, lambda a, b: (cfg2["col"][rp[a]:rp[b]],
                                                                         cfg2["val"][rp[a]:rp[b]]))
    m = len(lrp) - 1
    x = cfg2["xd"]
    y0 = sb.gen_vector(m, 45)
    want = orc.csr_spmv(lrp, col, val, x.cpu().numpy(), cfg2["alpha"], cfg2["beta"], y0.copy())
    bound = orc.spmv_bound(lrp, col, val, x.cpu().numpy(), cfg2["alpha"], cfg2["beta"], y0)
    A = sb.DeviceCSR.upload(0, N2, lrp, col, val)
    try:
        for algo, thr in ((sb.ROWSPLIT, 2_000_000), (sb.CSR5, 2_000_000)):
            A.analyse(algo)
            want_p = 0 if cfg2["prefix"] or int(lrp[-1]) < thr else 4
            assert A.panels(algo) == want_p, (world, algo)
            y = torch_cuda.from_numpy(y0.copy()).cuda()
            A.spmv(algo, cfg2["alpha"], x.data_ptr(), cfg2["beta"], y.data_ptr(), 0)
            torch_cuda.cuda.synchronize()
            _check_spmv(want, bound, y.cpu().numpy(), f"slice N={world} algo {algo}")
    finally:
        A.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config2_nnz_split_light_rank_csr5(torch_cuda, sb, orc, cfg2, world):
    """configs[2]'s nnz split puts the light rows on the last rank (9-entry
    rows): CSR5 takes 4 XCD panels there, as on longer rows, from 2M entries;
    within the bound against the oracle on that slice."""
    rp = cfg2["rp"]
    _, _, sr, er, _ = sb.partition_nnz(rp, world)
    a, b = int(sr[world - 1]), int(er[world - 1]) + 1
    lrp = np.asarray(rp[a:b + 1], np.int64) - int(rp[a])
    col, val = cfg2["col"][rp[a]:rp[b]], cfg2["val"][rp[a]:rp[b]]
    m = len(lrp) - 1
    assert int(lrp[-1]) < 12 * m  # short rows
    x = cfg2["xd"]
    y0 = sb.gen_vector(m, 46)
    xh = x.cpu().numpy()
    want = orc.csr_spmv(lrp, col, val, xh, cfg2["alpha"], cfg2["beta"], y0.copy())
    bound = orc.spmv_bound(lrp, col, val, xh, cfg2["alpha"], cfg2["beta"], y0)
    A = sb.DeviceCSR.upload(0, N2, lrp, col, val)
    try:
        A.analyse(sb.CSR5)
        assert A.panels(sb.CSR5) == (0 if cfg2["prefix"] else 4)
        y = torch_cuda.from_numpy(y0.copy()).cuda()
        A.spmv(sb.CSR5, cfg2["alpha"], x.data_ptr(), cfg2["beta"], y.data_ptr(), 0)
        torch_cuda.cuda.synchronize()
        _check_spmv(want, bound, y.cpu().numpy(), f"nnz split N={world} last rank, CSR5")
    finally:
        A.close()


@pytest.mark.parametrize("world,rank", [(2, 1), (4, 0), (8, 0), (8, 7)])
@pytest.mark.parametrize("opts", [{}, {"xs_solo": 1}, {"det": 1}], ids=["default", "solo", "det"])
def test_config2_rank_slice_xsort(torch_cuda, sb, orc, cfg2, world, rank, opts):
    """A rank's cyclic slice of config 2 (bench.py's N > 1 share) with the
    persistent column-sorted kernel (and its solo-item layout), three launches
    on one plan against the oracle, and the beta = 0 form on a NaN-filled y."""
    import sblas_dist
    torch = torch_cuda
    opts = dict(opts)
    det = bool(opts.pop("det", 0))
    rp, col, val = cfg2["rp"], cfg2["col"], cfg2["val"]
    plan = sblas_dist.make_cyclic_plan(rp, N2, world)
    lrp, lcol, lval = sblas_dist.cyclic_local_csr(rp, plan, rank, lambda a, b: (col[rp[a]:rp[b]], val[rp[a]:rp[b]]))
    m = len(lrp) - 1
    x = cfg2["xd"].cpu().numpy()
    y0 = sb.gen_vector(m, 45)
    alpha, beta = cfg2["alpha"], cfg2["beta"]
    A = sb.DeviceCSR.upload(0, N2, lrp, lcol, lval)
    A.deterministic = det
    try:
        with sb.test_options(**opts):
            A.analyse(5)
        for b in (beta, 0.0):
            want = orc.csr_spmv_omp(lrp, lcol, lval, x, alpha, b, y0.copy())
            bound = orc.spmv_bound(lrp, lcol, lval, x, alpha, b, y0)
            for it in range(3 if b else 1):
                yd = torch.from_numpy(y0).cuda() if b else torch.full((m,), float("nan"), dtype=torch.float64,
                                                                      device="cuda")
                A.spmv(5, alpha, cfg2["xd"].data_ptr(), b, yd.data_ptr())
                torch.cuda.synchronize()
                _check_spmv(want, bound, yd.cpu().numpy(), f"world {world} rank {rank} beta {b} launch {it}")
    finally:
        A.close()


def test_config2_auto(torch_cuda, sb, cfg2):
    """SBLAS_SPMV_AUTO on config 2: xsort for random columns, the row split
    for the reference generator's contiguous (prefix) columns; y against the
    oracle."""
    A = sb.DeviceCSR.upload(0, N2, cfg2["rp"], cfg2["col"], cfg2["val"])
    try:
        assert A.pick() == (sb.ROWSPLIT if cfg2["prefix"] else sb.XSORT)
    finally:
        A.close()
    _run_cfg2(torch_cuda, sb, cfg2, sb.AUTO)


def test_config2_alpha_beta_zero(torch_cuda, sb, orc, cfg2):
    """beta = 0 must not read y (y pre-filled with NaN): xsort, row split and
    CSR5."""
    torch = torch_cuda
    if cfg2["prefix"]:
        pytest.skip("random columns only")
    want = orc.csr_spmv_omp(cfg2["rp"], cfg2["col"], cfg2["val"], cfg2["xd"].cpu().numpy(), 1.5,
                            0.0, np.zeros(N2))
    bound = orc.spmv_bound(cfg2["rp"], cfg2["col"], cfg2["val"], cfg2["xd"].cpu().numpy(), 1.5,
                           0.0, np.zeros(N2))
    A = sb.DeviceCSR.upload(0, N2, cfg2["rp"], cfg2["col"], cfg2["val"])
    for algo in (1, 5, 2):
        A.analyse(algo)
        yd = torch.full((N2,), float("nan"), dtype=torch.float64, device="cuda")
        A.spmv(algo, 1.5, cfg2["xd"].data_ptr(), 0.0, yd.data_ptr())
        torch.cuda.synchronize()
        _check_spmv(want, bound, yd.cpu().numpy(), f"algo {algo} beta 0")
    A.close()


def test_config2_transpose_full_size(torch_cuda, sb, orc, cfg2):
    """CSR -> CSC of the config-2 matrix (the size tools/bench_transpose.py
    times): colptr, row indices and values bit-exact against orc_transpose
    (tranpose.h:6-43's stable scatter)."""
    torch = torch_cuda
    if cfg2["prefix"]:
        pytest.skip("random columns only")
    rp, col, val = cfg2["rp"], cfg2["col"], cfg2["val"]
    nnz = int(rp[-1])
    cp, ri, cv = orc.transpose(N2, N2, rp, col, val)
    A = sb.DeviceCSR.upload(0, N2, rp, col, val)
    try:
        dcp = torch.zeros(N2 + 1, dtype=torch.int32, device="cuda")
        dri = torch.zeros(nnz, dtype=torch.int32, device="cuda")
        dcv = torch.zeros(nnz, dtype=torch.float64, device="cuda")
        for _ in range(2):  # the second call reuses the grown scratch
            A.transpose(dcp.data_ptr(), dri.data_ptr(), dcv.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(dcp.cpu().numpy(), cp)
            assert np.array_equal(dri.cpu().numpy(), ri)
            assert np.array_equal(dcv.cpu().numpy(), cv)
    finally:
        A.close()


# ------------------------------------------------------------- config 4 ----
@pytest.fixture(scope="module")
def cfg4(orc):
    from bench_spmm import rail_like
    m, k, nnz, n = 4284, 1_092_610, 11_279_748, 64
    rp, col = rail_like(m, k, nnz, 44)
    val = np.random.default_rng(45).random(nnz)
    B = np.random.default_rng(46).random((k, n))
    C0 = np.random.default_rng(47).random((m, n))
    alpha, beta = -0.7, 0.8  # dspmm_baseline_test.cu:518-519
    want, bound = orc.spmm_checked(m, n, alpha, rp, col, val, B, beta, C0)
    return dict(m=m, k=k, n=n, rp=rp, col=col, val=val, B=B, C0=C0, alpha=alpha, beta=beta,
                want=want, bound=bound)


@pytest.mark.parametrize("layout,form", [("row", "ctile"), ("col", "ctile"), ("row", "rowwave")])
def test_config4_spmm_full_size(torch_cuda, sb, cfg4, layout, form):
    """BASELINE configs[3]: C = -0.7 A B + 0.8 C on the rail4284-shaped matrix,
    all 4284 x 64 entries of C checked (B row-major as resident in HBM, and
    the reference's column-major host layout), with the default column-sorted
    C-tile form and the row kernels (test option spmm_ctile=0)."""
    torch = torch_cuda
    c = cfg4
    m, k, n = c["m"], c["k"], c["n"]
    A = sb.DeviceCSR.upload(0, k, c["rp"], c["col"], c["val"])
    if layout == "row":
        Bd, ldb, lay = torch.from_numpy(c["B"]).cuda(), n, 1
    else:
        Bd, ldb, lay = torch.from_numpy(np.asfortranarray(c["B"]).ravel(order="F")).cuda(), k, 0
    Cd = torch.from_numpy(np.asfortranarray(c["C0"]).ravel(order="F")).cuda()
    with sb.test_options(**({"spmm_ctile": 0} if form == "rowwave" else {})):  # the plan builds on this call
        A.spmm(n, c["alpha"], Bd.data_ptr(), ldb, lay, c["beta"], Cd.data_ptr(), m)
    torch.cuda.synchronize()
    got = Cd.cpu().numpy().reshape((n, m)).T
    A.close()
    err = np.abs(got - c["want"])
    assert np.all(err <= c["bound"]), f"max excess {np.max(err - c['bound'])}"


# ------------------------------------------------------------- config 5 ----
N5, OFFD5, BAND5 = 5_558_326, 5, 80_000


@pytest.fixture(scope="module")
def cfg5(sb):
    cp, ri, v = sb.gen_lower_banded(N5, OFFD5, BAND5, 47)
    cols = np.repeat(np.arange(N5, dtype=np.int64), np.diff(cp))
    # integer KAT on the same pattern: unit diagonal, off-diagonals 1..10
    vi = np.random.default_rng(5).integers(1, 11, len(ri)).astype(np.float64)
    vi[cp[:-1]] = 1.0
    xref = np.floor(sb.gen_vector(N5, 48) * 10.0) + 1.0
    bi = np.bincount(ri, weights=vi * xref[cols], minlength=N5)  # exact: integers < 2^53
    b = np.bincount(ri, weights=v * xref[cols], minlength=N5)
    return dict(cp=cp, ri=ri, v=v, vi=vi, xref=xref, bi=bi, b=b)


def test_config5_kat_serial_oracle(orc, cfg5):
    """The reference's serial executor (restated) solves the KAT exactly."""
    c = cfg5
    x = orc.sptrsv_serial(c["cp"], c["ri"], c["vi"], c["bi"], 0)
    assert np.array_equal(x, c["xref"])
    assert orc.levels_lower(c["cp"], c["ri"]) > 100


@pytest.mark.parametrize("algo", [1, 0, 2, 3], ids=["pull", "push", "levelset", "pull_level_order"])
def test_config5_single_device_exact(torch_cuda, sb, cfg5, algo):
    torch = torch_cuda
    c = cfg5
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (c["cp"], c["ri"], c["vi"], c["bi"])]
    xd = torch.zeros(N5, dtype=torch.float64, device="cuda")
    T = sb.DeviceTRSV(0, N5, len(c["ri"]), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 0)
    T.solve(algo, d[3].data_ptr(), xd.data_ptr())
    torch.cuda.synchronize()
    T.close()
    assert np.array_equal(xd.cpu().numpy(), c["xref"])


@pytest.mark.parametrize("ngpu", [4])
def test_config5_blocks_exact(torch_cuda, sb, cfg5, ngpu):
    """BASELINE configs[4]'s 4-way partition (blocks running concurrently):
    exact on the KAT; and sptrsv_v3's decomposition, 4 devices x 2 tasks."""
    c = cfg5
    x, ms = sb.trsv_mgpu_solve(c["cp"], c["ri"], c["vi"], N5, c["bi"], ngpu, 0)
    assert np.array_equal(x, c["xref"]) and ms > 0.0
    x, ms = sb.trsv_mgpu_solve_tasks(c["cp"], c["ri"], c["vi"], N5, c["bi"], ngpu, 2)
    assert np.array_equal(x, c["xref"]) and ms > 0.0


@pytest.mark.parametrize("ngpu", [1, 4])
def test_config5_real_vs_serial_oracle(torch_cuda, sb, orc, cfg5, ngpu):
    """The bench's real-valued system against the reference's serial executor."""
    c = cfg5
    want = orc.sptrsv_serial(c["cp"], c["ri"], c["v"], c["b"], 0)
    x, _ = sb.trsv_mgpu_solve(c["cp"], c["ri"], c["v"], N5, c["b"], ngpu, 0)
    rel = np.abs(x - want).sum() / np.abs(want).sum()
    assert rel <= 1e-12, rel
    assert np.abs(x - c["xref"]).sum() / np.abs(c["xref"]).sum() < 1e-10
