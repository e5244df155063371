"""SpMM, CSR->CSC transpose, SpTRSV and y-assembly kernels vs the oracle."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def rand_csr(rng, m, n, maxlen, empty_frac=0.1, long_rows=()):
    lens = rng.integers(0, maxlen, m)
    lens[rng.random(m) < empty_frac] = 0
    for r, L in long_rows:
        lens[r] = L
    lens = np.minimum(lens, n)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = (np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
           if rp[-1] else np.zeros(0, np.int32))
    return rp, col, rng.standard_normal(int(rp[-1]))


# ---------------------------------------------------------------- SpMM ----
def spmm_bound(rp, col, val, B, alpha, beta, C0):
    u = 2.0 ** -53
    m = len(rp) - 1
    k = np.diff(rp).astype(np.float64)
    gam = (k * u / (1 - k * u))[:, None]
    rows = np.repeat(np.arange(m), np.diff(rp))
    S = np.zeros((m, B.shape[1]))
    np.add.at(S, rows, np.abs(alpha * val[:, None] * B[col, :]))
    return 4 * gam * S + 4 * u * np.abs(beta * C0) + 1e-300


@pytest.mark.parametrize("form", ["rowwave", "splitk", "ct", "ctrows"])
@pytest.mark.parametrize("ncols", [1, 16, 64, 100])
@pytest.mark.parametrize("layout", [0, 1])
def test_spmm(torch_cuda, sb, orc, ncols, layout, form):
    """Both row kernels: wave per row ("rowwave") and workgroup per row split
    over its nonzeros (picked for rows of >= 256 entries on average:
    "splitk", 60 rows of ~1,000), and the column-sorted C-tile form (test
    option spmm_ctile=1: "ct" = 3 slabs of 2048 columns, one slab set;
    "ctrows" = 2,500 rows, i.e. 3 row blocks of 834)."""
    torch = torch_cuda
    rng = np.random.default_rng(ncols + 10 * layout)
    m, k = {"ctrows": 2500, "splitk": 60}.get(form, 700), 5000
    rp, col, val = rand_csr(rng, m, k, 2000 if form == "splitk" else 50, long_rows=[(3, 3000)])
    B = rng.standard_normal((k, ncols))
    C0 = rng.standard_normal((m, ncols))
    alpha, beta = -0.7, 0.8  # dspmm_baseline_test.cu:518-519
    want = orc.spmm(m, ncols, k, alpha, rp, col, val, B, beta, C0)
    A = sb.DeviceCSR.upload(0, k, rp, col, val)
    if layout == 0:  # column-major B (ld = k)
        Bd = torch.from_numpy(np.asfortranarray(B).ravel(order="F")).cuda()
        ldb = k
    else:            # row-major B (ld = ncols)
        Bd = torch.from_numpy(np.ascontiguousarray(B).ravel()).cuda()
        ldb = ncols
    Cd = torch.from_numpy(np.asfortranarray(C0).ravel(order="F")).cuda()
    with sb.test_options(**({"spmm_ctile": 1} if form.startswith("ct") else {})):  # the plan builds here
        A.spmm(ncols, alpha, Bd.data_ptr(), ldb, layout, beta, Cd.data_ptr(), m)
    torch.cuda.synchronize()
    got = Cd.cpu().numpy().reshape((ncols, m)).T
    assert np.all(np.abs(got - want) <= spmm_bound(rp, col, val, B, alpha, beta, C0))
    A.close()


@pytest.mark.parametrize("form", ["ctile"])
@pytest.mark.parametrize("layout", [0, 1])
def test_spmm_two_handles_two_streams(torch_cuda, sb, orc, layout, form):
    """Two handles of different matrices on two streams of one device, launched
    back to back without synchronising: each keeps its own scratch (B copy,
    C-tile partials: sblas_csr_s::spmm_*), so both C match the oracle."""
    torch = torch_cuda
    ncols, k = 64, 6000
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i, m in enumerate((900, 1300)):
        rng = np.random.default_rng(50 + i)
        rp, col, val = rand_csr(rng, m, k, 60)
        B = rng.standard_normal((k, ncols))
        C0 = rng.standard_normal((m, ncols))
        A = sb.DeviceCSR.upload(0, k, rp, col, val)
        if layout == 0:
            Bd = torch.from_numpy(np.asfortranarray(B).ravel(order="F")).cuda()
            ldb = k
        else:
            Bd = torch.from_numpy(np.ascontiguousarray(B).ravel()).cuda()
            ldb = ncols
        Cd = torch.from_numpy(np.asfortranarray(C0).ravel(order="F")).cuda()
        outs.append((A, Bd, ldb, Cd, rp, col, val, B, C0, m))
    torch.cuda.synchronize()
    with sb.test_options(spmm_ctile=1):  # the plans build on the first calls
        for rep in range(3):  # C <- alpha*A*B + beta*C, three times on each stream
            for (A, Bd, ldb, Cd, *_), st in zip(outs, streams):
                A.spmm(ncols, 0.5, Bd.data_ptr(), ldb, layout, 0.0 if rep else 1.0, Cd.data_ptr(),
                       Cd.numel() // ncols, st.cuda_stream)
    torch.cuda.synchronize()
    for A, Bd, ldb, Cd, rp, col, val, B, C0, m in outs:
        want = orc.spmm(m, ncols, k, 0.5, rp, col, val, B, 0.0, C0)
        got = Cd.cpu().numpy().reshape((ncols, m)).T
        assert np.all(np.abs(got - want) <= spmm_bound(rp, col, val, B, 0.5, 0.0, C0))
        A.close()


@pytest.mark.parametrize("split", ["rows", "cols"])
@pytest.mark.parametrize("ngpu", [1, 2, 3])
def test_csrmm_reference_api(torch_cuda, sb, orc, ngpu, split):
    """cusparse_mgpu_csrmm drop-in on qh768 x 128 (run_test.py's spmm case),
    with the north star's row partition and the reference's own column split
    (A replicated, B/C split by columns, dspmm_mgpu_baseline.cu:147-150)."""
    path = os.path.join(GOLDEN, "qh768.mtx")
    m, k, rp, col, val = sb.mm_read(path, 0)
    ncols = 128
    rng = np.random.default_rng(1)
    B = rng.random((k, ncols))
    C0 = rng.random((m, ncols))
    Cf = np.array(C0, order="F", copy=True)
    Bf = np.asfortranarray(B)
    rp32 = rp.astype(np.int32)
    a = np.array([-0.7]); b = np.array([0.8])
    fn = sb.lib.sblas_csrmm_mgpu if split == "rows" else sb.lib.sblas_csrmm_mgpu_colsplit
    rc = fn(m, ncols, k, sb.ptr(a), int(rp[-1]), sb.ptr(rp32), sb.ptr(col),
            sb.ptr(val), sb.ptr(b), Bf.ctypes.data, Cf.ctypes.data, ngpu)
    assert rc == 0
    want = orc.spmm(m, ncols, k, -0.7, rp32, col, val, B, 0.8, C0)
    assert np.all(np.abs(Cf - want) <= spmm_bound(rp, col, val, B, -0.7, 0.8, C0))
    # the reference's own check (:544-549) is abs 1e-3 between two cuSPARSE runs of the
    # same algorithm; against an independent summation order it is applied relatively
    assert np.all(np.abs(Cf - want) < 1e-3 * np.maximum(1.0, np.abs(want)))


# ----------------------------------------------------------- transpose ----
@pytest.mark.parametrize("case", ["qh768", "ash85", "random", "longcols", "wide", "big", "shortrows", "sparserows"])
def test_transpose_bit_exact(torch_cuda, sb, orc, case):
    """Stable transpose, every path the default build takes: the MSD
    partition passes + per-bucket final pass where n > 512 (pass A derives
    each entry's row from rowptr and hands pass B one word of key bits and
    row offset when the segments' row spans allow -- "sparserows" spans too
    many rows, the device falls back; pass B hands the last pass one word of
    row and low column bits; "longcols" gives few, long buckets; "big" 3M
    columns), and the LSD passes on narrow matrices (qh768, ash85, "wide" is
    n = 1e5 over 50 rows, "longcols" n = 40).  Colptr, row indices and values
    bit-exact against orc_transpose (tranpose.h:6-43's stable scatter)."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    if case in ("qh768", "ash85"):
        m, n, rp, col, val = sb.mm_read(os.path.join(GOLDEN, f"{case}.mtx"), 0)
    elif case == "random":
        m, n = 3000, 2500
        rp, col, val = rand_csr(rng, m, n, 30)
    elif case == "big":  # 2.2M nonzeros over 3M columns: 2 passes x 11 bits, 2 tiles per workgroup
        m, n = 110000, 3_000_000
        lens = rng.integers(0, 40, m)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    elif case == "shortrows":  # 0-3 entries per row, half the rows empty: a 4096-entry tile
        # holds thousands of row starts (pass A's row derivation takes several windows)
        m, n = 200000, 5000
        lens = rng.integers(0, 4, m) * (rng.random(m) < 0.5)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    elif case == "sparserows":  # 2^24 columns (16 key bits past pass A) and one row in 100
        # non-empty: a segment spans > 2^16 rows, so pass A cannot pack the row offset
        m, n = 300000, 1 << 24
        lens = np.where(rng.random(m) < 0.01, 5, 0)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    elif case == "wide":  # more columns than rows, many empty columns
        m, n = 50, 100000
        rp, col, val = rand_csr(rng, m, n, 400, empty_frac=0.3)
    else:  # columns longer than 32 / 4096 (medium and big sort paths)
        m, n = 9000, 40
        rp, col, val = rand_csr(rng, m, n, 40, empty_frac=0.2)
    nnz = int(rp[-1])
    cp, ri, cv = orc.transpose(m, n, rp, col, val)
    A = sb.DeviceCSR.upload(0, n, rp, col, val)
    dcp = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    dri = torch.zeros(max(nnz, 1), dtype=torch.int32, device="cuda")
    dcv = torch.zeros(max(nnz, 1), dtype=torch.float64, device="cuda")
    A.transpose(dcp.data_ptr(), dri.data_ptr(), dcv.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(dcp.cpu().numpy(), cp)
    assert np.array_equal(dri.cpu().numpy()[:nnz], ri)
    assert np.array_equal(dcv.cpu().numpy()[:nnz], cv)
    A.close()


@pytest.mark.parametrize("shape", ["one_entry", "one_row", "one_col_tall", "last_col", "tile_edge",
                                   "dup_free_dense_row", "empty_tail_rows"])
def test_transpose_edges(torch_cuda, sb, orc, shape):
    """Edge shapes on the default MSD path (n > 512): a single nonzero, every
    entry in one row, one populated column over many rows, entries only in the
    last column, nnz exactly one tile / one past it, rows empty at the end."""
    torch = torch_cuda
    rng = np.random.default_rng(7)
    n = 5000
    if shape == "one_entry":
        m = 3
        rp = np.array([0, 0, 1, 1], np.int64)
        col = np.array([4321], np.int32)
    elif shape == "one_row":
        m = 1
        col = np.sort(rng.choice(n, 3000, replace=False)).astype(np.int32)
        rp = np.array([0, len(col)], np.int64)
    elif shape == "one_col_tall":
        m = 20000
        rp = np.arange(m + 1, dtype=np.int64)
        col = np.full(m, 777, np.int32)
    elif shape == "last_col":
        m = 4096
        rp = np.arange(m + 1, dtype=np.int64)
        col = np.full(m, n - 1, np.int32)
    elif shape == "tile_edge":  # 4097 nonzeros: one full tile and one entry
        m = 4097
        rp = np.arange(m + 1, dtype=np.int64)
        col = rng.integers(0, n, m).astype(np.int32)
    elif shape == "dup_free_dense_row":  # every column of one row, then sparse rows
        m = 700
        lens = np.concatenate([[n], rng.integers(0, 5, m - 1)])
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.arange(n)] + [np.sort(rng.choice(n, L, replace=False)) for L in lens[1:]]).astype(np.int32)
    else:  # empty_tail_rows
        m = 50000
        lens = np.concatenate([rng.integers(1, 6, 1000), np.zeros(m - 1000, np.int64)])
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens[:1000]]).astype(np.int32)
    val = rng.standard_normal(len(col))
    nnz = int(rp[-1])
    cp, ri, cv = orc.transpose(m, n, rp, col, val)
    A = sb.DeviceCSR.upload(0, n, rp, col, val)
    dcp = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    dri = torch.zeros(max(nnz, 1), dtype=torch.int32, device="cuda")
    dcv = torch.zeros(max(nnz, 1), dtype=torch.float64, device="cuda")
    A.transpose(dcp.data_ptr(), dri.data_ptr(), dcv.data_ptr())
    torch.cuda.synchronize()
    A.close()
    assert np.array_equal(dcp.cpu().numpy(), cp)
    assert np.array_equal(dri.cpu().numpy()[:nnz], ri)
    assert np.array_equal(dcv.cpu().numpy()[:nnz], cv)


@pytest.mark.parametrize("case", ["qh768", "ash85", "random", "longcols", "wide"])
@pytest.mark.parametrize("ngpu", [1, 2, 3, 5])
def test_transpose_mgpu_bit_exact(torch_cuda, sb, orc, case, ngpu):
    """Multi-device CSR -> CSC: blocks of whole rows, composed
    on device 0; indices and values bit-exact against the stable transpose."""
    rng = np.random.default_rng(11)
    if case in ("qh768", "ash85"):
        m, n, rp, col, val = sb.mm_read(os.path.join(GOLDEN, f"{case}.mtx"), 0)
    elif case == "random":
        m, n = 3000, 2500
        rp, col, val = rand_csr(rng, m, n, 30)
    elif case == "longcols":
        m, n = 9000, 40
        rp, col, val = rand_csr(rng, m, n, 40, empty_frac=0.2)
    else:  # more columns than rows, many empty columns
        m, n = 50, 100000
        rp, col, val = rand_csr(rng, m, n, 400, empty_frac=0.3)
    cp, ri, cv = orc.transpose(m, n, rp, col, val)
    gcp, gri, gcv, t1, t2 = sb.csr2csc_mgpu(m, n, rp, col, val, ngpu)
    assert np.array_equal(gcp, cp) and np.array_equal(gri, ri) and np.array_equal(gcv, cv)
    assert t1 >= 0 and t2 >= 0


def test_sptrans_reference_api(torch_cuda, sb, orc, capfd):
    m, n, rp, col, val = sb.mm_read(os.path.join(GOLDEN, "qh768.mtx"), 0)
    rp32 = rp.astype(np.int32)
    cp, ri, cv = orc.transpose(m, n, rp, col, val)
    nnz = len(ri)
    ocp, ori, ocv = np.zeros(n + 1, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
    for ngpu in (1, 3):
        rc = sb.lib.sblas_sptrans(m, n, nnz, ngpu, sb.ptr(rp32), sb.ptr(col), sb.ptr(val),
                                  sb.ptr(ori), sb.ptr(ocp), sb.ptr(ocv), sb.ptr(ri), sb.ptr(cp),
                                  sb.ptr(cv))
        assert rc == 0
        assert np.array_equal(ocp, cp) and np.array_equal(ori, ri) and np.array_equal(ocv, cv)
    out = capfd.readouterr().out
    assert "sptrans value test on single GPU: passed!" in out
    assert "sptrans pointer test on multiple GPU: passed!" in out
    assert "row index test on multiple GPU: passed!" in out


# -------------------------------------------------------------- SpTRSV ----
@pytest.mark.parametrize("name", ["qh768", "ash85"])
@pytest.mark.parametrize("sub", ["fwd", "bwd"])
@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_sptrsv_kat(torch_cuda, sb, orc, name, sub, algo):
    torch = torch_cuda
    g = np.load(os.path.join(GOLDEN, f"trsv_{name}_{sub}.npz"))
    cp, ri, cv, b = g["colptr"], g["rowidx"], g["val"], g["b"]
    n, nnz = len(cp) - 1, len(ri)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, cv, b)]
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    T = sb.DeviceTRSV(0, n, nnz, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                      0 if sub == "fwd" else 1)
    for _ in range(3):
        xd.zero_()
        T.solve(algo, d[3].data_ptr(), xd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(xd.cpu().numpy(), g["x_ref"])  # exact KAT
    if sub == "fwd":
        assert T.levels() == orc.levels_lower(cp, ri)
    T.close()


@pytest.mark.parametrize("kind", ["stencil27", "stencil7", "banded"])
def test_sptrsv_auto_order(torch_cuda, sb, orc, kind):
    """algo 4 (AUTO): level-ordered tickets for a stencil's lower triangle
    (row i depends on row i - 1, a chain through every wave), natural order
    for a banded random triangle; x bit-identical to algo 1 and within the
    bound of the exact solution."""
    torch = torch_cuda
    if kind == "banded":
        cp, ri, v = sb.gen_lower_banded(30000, 4, 5000, 11)
        n = len(cp) - 1
        want = 1
    else:
        g = 24
        srp, scol, sval = sb.gen_stencil3d(g, g, g, int(kind[7:]), seed=49)
        n = len(srp) - 1
        srow = np.repeat(np.arange(n), np.diff(srp))
        keep = scol >= srow
        cp = np.zeros(n + 1, np.int32)
        cp[1:] = np.cumsum(np.bincount(srow[keep], minlength=n))
        ri = np.ascontiguousarray(scol[keep]).astype(np.int32)
        v = np.ascontiguousarray(sval[keep])
        want = 3
    xref = np.floor(sb.gen_vector(n, 48) * 10.0) + 1.0
    cols = np.repeat(np.arange(n), np.diff(cp))
    b = np.bincount(ri, weights=v * xref[cols], minlength=n)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, v, b)]
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 0)
    try:
        assert T.pick() == want
        xs = []
        for algo in (4, 1):
            xd = torch.zeros(n, dtype=torch.float64, device="cuda")
            T.solve(algo, d[3].data_ptr(), xd.data_ptr())
            torch.cuda.synchronize()
            xs.append(xd.cpu().numpy())
        assert np.array_equal(xs[0], xs[1])
        assert np.abs(xs[0] - xref).sum() / np.abs(xref).sum() < 1e-12
        # SpTRSM: algo 3 (level-ordered tickets) and 4 bit-identical to the
        # natural-order pull, every right-hand side within the bound
        rhs = 5
        xr = np.stack([xref * (k + 1) for k in range(rhs)], axis=1)
        bm = np.stack([b * (k + 1) for k in range(rhs)], axis=1)
        db = torch.from_numpy(np.ascontiguousarray(bm)).cuda()
        xm = []
        for algo in (1, 3, 4):
            xd = torch.zeros(n * rhs, dtype=torch.float64, device="cuda")
            T.solve_rhs_opt(algo, 3, rhs, db.data_ptr(), xd.data_ptr())
            torch.cuda.synchronize()
            xm.append(xd.cpu().numpy().reshape(n, rhs))
        assert np.array_equal(xm[0], xm[1]) and np.array_equal(xm[0], xm[2])
        assert np.abs(xm[0] - xr).sum() / np.abs(xr).sum() < 1e-12
        with pytest.raises(RuntimeError):
            T.solve_rhs_opt(2, 3, rhs, db.data_ptr(), xd.data_ptr())
    finally:
        T.close()


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_sptrsv_random_wellconditioned(torch_cuda, sb, orc, algo):
    """Random lower-triangular with long chains and a long column/row."""
    torch = torch_cuda
    rng = np.random.default_rng(9)
    n = 20000
    rp, col, _ = rand_csr(rng, n, n, 8, empty_frac=0.0)
    (trp, tc, tv), (cp, ri, cv), xref, b = orc.build_tri(rp.astype(np.int32), col, 0, seed=3)
    # scale to keep the solve well conditioned
    lens = np.diff(cp)
    rows = ri
    cv = cv.copy()
    off = np.ones(len(cv), bool)
    off[cp[:-1]] = False
    rl = np.bincount(ri, minlength=n)
    cv[off] = cv[off] / (2.0 * rl[rows[off]])
    b = np.zeros(n)
    for c in range(n):
        b[ri[cp[c]:cp[c + 1]]] += cv[cp[c]:cp[c + 1]] * xref[c]
    want = orc.sptrsv_serial(cp, ri, cv, b, 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, cv, b)]
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 0)
    T.solve(algo, d[3].data_ptr(), xd.data_ptr())
    torch.cuda.synchronize()
    x = xd.cpu().numpy()
    rel = np.abs(x - want).sum() / np.abs(want).sum()
    assert rel <= 1e-12, rel
    if algo in (2, 3):  # level-set / level-ordered pull sum in the pull executor's order: bit-identical
        xp = torch.zeros(n, dtype=torch.float64, device="cuda")
        T.solve(1, d[3].data_ptr(), xp.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(xp.cpu().numpy(), x)
    T.close()


@pytest.mark.parametrize("sub", [0, 1])
@pytest.mark.parametrize("shape", ["chain", "wide"])
def test_sptrsv_levelset_schedule(torch_cuda, sb, orc, sub, shape):
    """Level-set executor over both schedule kinds: "chain" = a bidiagonal
    system (n levels of one row: one narrow run in one workgroup), "wide" = a
    diagonal-heavy system with a few long dependency columns (levels of more
    than 2,048 rows: one grid launch per level), forward and backward; exact
    integer KATs (x integer, values small integers)."""
    torch = torch_cuda
    rng = np.random.default_rng(17 + sub)
    n = 5000 if shape == "chain" else 60000
    cols, rows = [], []
    for c in range(n):
        deps = []
        if shape == "chain":
            if (sub == 0 and c + 1 < n) or (sub == 1 and c > 0):
                deps = [c + 1 if sub == 0 else c - 1]
        else:
            lo, hi = (c + 1, min(n, c + 4000)) if sub == 0 else (max(0, c - 4000), c)
            if hi > lo and rng.random() < 0.3:
                deps = sorted(set(rng.integers(lo, hi, 2).tolist()))
        rr = [c] + deps if sub == 0 else deps + [c]
        rows.append(rr)
    cp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ri = np.concatenate(rows).astype(np.int32)
    cv = rng.integers(1, 4, len(ri)).astype(np.float64)
    diag_pos = cp[:-1] if sub == 0 else cp[1:] - 1
    cv[diag_pos] = 1.0
    xref = rng.integers(-3, 4, n).astype(np.float64)
    colidx = np.repeat(np.arange(n), np.diff(cp))
    b = np.bincount(ri, weights=cv * xref[colidx], minlength=n)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, cv, b)]
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sub)
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    for _ in range(2):  # second solve reuses the level schedule
        xd.zero_()
        T.solve(2, d[3].data_ptr(), xd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(xd.cpu().numpy(), xref)
    if shape == "chain":
        assert T.levels() == n
    T.close()


def test_sptrsv_reference_api(torch_cuda, sb, capfd):
    g = np.load(os.path.join(GOLDEN, "trsv_qh768_fwd.npz"))
    cp, ri, cv, b, xref = g["colptr"], g["rowidx"], g["val"], g["b"], g["x_ref"]
    n = len(cp) - 1
    x = np.zeros(n)
    gf = np.zeros(1)
    for opt in (1, 3):
        rc = sb.lib.sblas_sptrsv_syncfree(sb.ptr(cp), sb.ptr(ri), sb.ptr(cv), n, n, len(ri), 0, 1,
                                          opt, sb.ptr(x), sb.ptr(b), sb.ptr(xref), sb.ptr(gf), 1)
        assert rc == 0 and np.array_equal(x, xref)
    out = capfd.readouterr().out
    assert "cuda syncfree SpTRSV solve used" in out and "executor passed!" in out


@pytest.mark.parametrize("name", ["qh768", "ash85"])
@pytest.mark.parametrize("sub", ["fwd", "bwd"])
@pytest.mark.parametrize("ngpu", [2, 3, 4])
def test_sptrsv_mgpu_kat(torch_cuda, sb, name, sub, ngpu):
    """Multi-device executor: blocks of the solve order, x
    pushed to later blocks; exact against the reference's KAT.  On a one-GPU
    box the blocks wrap onto device 0 and run in order."""
    g = np.load(os.path.join(GOLDEN, f"trsv_{name}_{sub}.npz"))
    n = len(g["colptr"]) - 1
    x, ms = sb.trsv_mgpu_solve(g["colptr"], g["rowidx"], g["val"], n, g["b"], ngpu,
                               0 if sub == "fwd" else 1)
    assert np.array_equal(x, g["x_ref"]) and ms >= 0.0


@pytest.mark.parametrize("ngpu", [1, 2, 4, 7])
def test_sptrsv_mgpu_banded_matches_single(torch_cuda, sb, ngpu):
    """Partitioned solve == single-device pull solve, bit for bit (each row
    sums its dependencies in the same CSR order)."""
    torch = torch_cuda
    n = 300_000
    cp, ri, v = sb.gen_lower_banded(n, 4, 5000, 11)
    xref = np.floor(sb.gen_vector(n, 12) * 10.0) + 1.0
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(cp))
    b = np.bincount(ri, weights=v * xref[cols], minlength=n)
    d = [torch.from_numpy(a).cuda() for a in (cp, ri, v, b)]
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 0)
    T.solve(1, d[3].data_ptr(), xd.data_ptr())
    torch.cuda.synchronize()
    T.close()
    want = xd.cpu().numpy()
    x, _ = sb.trsv_mgpu_solve(cp, ri, v, n, b, ngpu, 0)
    assert np.array_equal(x, want)
    assert np.abs(x - xref).sum() / np.abs(xref).sum() < 1e-10


def _banded_system(sb, n, seed=11):
    cp, ri, v = sb.gen_lower_banded(n, 4, 5000, seed)
    xref = np.floor(sb.gen_vector(n, seed + 1) * 10.0) + 1.0
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(cp))
    b = np.bincount(ri, weights=v * xref[cols], minlength=n)
    return cp, ri, v, b, xref


@pytest.mark.parametrize("blocks,rhs,sub", [(1, 1, 0), (4, 1, 0), (3, 1, 1), (4, 3, 0), (2, 5, 1)])
def test_sptrsv_mgpu_persistent_handle(torch_cuda, sb, orc, blocks, rhs, sub):
    """sblas_trsv_mgpu_create / run / destroy: blocks built once, then several
    right-hand sides solved on the same handle; each x bit-identical to the
    one-shot sblas_trsv_mgpu_solve and within 1e-12 of the reference's serial
    executor (rhs 1)."""
    n = 120_000
    cp, ri, v, b0, xref = _banded_system(sb, n)
    if sub == 1:  # the upper triangle: U = L^T (CSC of U = CSR of L), diagonal last
        cp, ri, v = orc.transpose(n, n, cp, ri, v)
    H = sb.TrsvMgpu(cp, ri, v, n, blocks, substitution=sub, rhs=rhs)
    rng = np.random.default_rng(blocks * 10 + rhs)
    for k in range(3):
        b = rng.standard_normal(n * rhs) if k else np.tile(b0[:, None], (1, rhs)).ravel()
        x, ms = H.run(b)
        want, _ = sb.trsv_mgpu_solve(cp, ri, v, n, b, blocks, sub, rhs)
        assert np.array_equal(x, want) and ms > 0.0
        if rhs == 1:
            ser = orc.sptrsv_serial(cp, ri, v, b, sub)
            assert np.abs(x - ser).sum() / np.abs(ser).sum() <= 1e-12
    H.close()


@pytest.mark.parametrize("ngpu,tasks", [(1, 4), (2, 3), (3, 2), (4, 2)])
@pytest.mark.parametrize("balance", [0, 1])
def test_sptrsv_tasks_kat(torch_cuda, sb, ngpu, tasks, balance):
    """sptrsv_v3's task decomposition: ngpu*tasks blocks, block d on device
    d % ngpu, all running concurrently; exact on the KATs, and equal to the
    single-block solve on the banded system."""
    for name, sub in (("qh768", "fwd"), ("ash85", "bwd")):
        g = np.load(os.path.join(GOLDEN, f"trsv_{name}_{sub}.npz"))
        n = len(g["colptr"]) - 1
        x, _ = sb.trsv_mgpu_solve_tasks(g["colptr"], g["rowidx"], g["val"], n, g["b"], ngpu, tasks,
                                        0 if sub == "fwd" else 1, balance=balance)
        assert np.array_equal(x, g["x_ref"])
    n = 300_000
    cp, ri, v, b, _ = _banded_system(sb, n)
    want, _ = sb.trsv_mgpu_solve(cp, ri, v, n, b, 1, 0)
    x, _ = sb.trsv_mgpu_solve_tasks(cp, ri, v, n, b, ngpu, tasks, balance=balance)
    assert np.array_equal(x, want)


def test_sptrsv_v3_reference_api(torch_cuda, sb, capfd):
    """sptrsv_syncfree_cuda(..., ngpu, task) (sptrsv_v3): prints v3's lines."""
    g = np.load(os.path.join(GOLDEN, "trsv_qh768_fwd.npz"))
    cp, ri, cv, b, xref = g["colptr"], g["rowidx"], g["val"], g["b"], g["x_ref"]
    n = len(cp) - 1
    x = np.zeros(n)
    gf = np.zeros(1)
    rc = sb.lib.sblas_sptrsv_syncfree_v3(sb.ptr(cp), sb.ptr(ri), sb.ptr(cv), n, n, len(ri), 0, 1, 3,
                                         sb.ptr(x), sb.ptr(b), sb.ptr(xref), sb.ptr(gf), 2, 3)
    assert rc == 0 and np.array_equal(x, xref) and gf[0] > 0
    out = capfd.readouterr().out
    assert out.count("nnz for device") == 6
    assert "cuda syncfree SpTRSV solve used" in out
    assert "device:0 cuda syncfree SpTRSV executor passed!" in out


def test_sptrsv_reference_api_mgpu(torch_cuda, sb, capfd):
    g = np.load(os.path.join(GOLDEN, "trsv_ash85_bwd.npz"))
    cp, ri, cv, b, xref = g["colptr"], g["rowidx"], g["val"], g["b"], g["x_ref"]
    n = len(cp) - 1
    x = np.zeros(n)
    gf = np.zeros(1)
    rc = sb.lib.sblas_sptrsv_syncfree(sb.ptr(cp), sb.ptr(ri), sb.ptr(cv), n, n, len(ri), 1, 1,
                                      3, sb.ptr(x), sb.ptr(b), sb.ptr(xref), sb.ptr(gf), 3)
    assert rc == 0 and np.array_equal(x, xref)
    assert "executor passed!" in capfd.readouterr().out


def csc_matmat(cp, ri, cv, X):
    """B = L X for CSC L (exact for the integer KAT systems)."""
    B = np.zeros_like(X)
    for c in range(len(cp) - 1):
        s, e = cp[c], cp[c + 1]
        B[ri[s:e]] += cv[s:e, None] * X[c][None, :]
    return B


@pytest.mark.parametrize("name", ["qh768", "ash85"])
@pytest.mark.parametrize("sub", ["fwd", "bwd"])
@pytest.mark.parametrize("rhs", [2, 3, 8, 64, 100])
def test_sptrsm_kat(torch_cuda, sb, name, sub, rhs):
    """SpTRSM (rhs > 1): integer L (unit diagonal) and integer
    X, so B = L X and the solve are exact in fp64."""
    torch = torch_cuda
    g = np.load(os.path.join(GOLDEN, f"trsv_{name}_{sub}.npz"))
    cp, ri, cv = g["colptr"], g["rowidx"], g["val"]
    n = len(cp) - 1
    X = np.random.default_rng(rhs).integers(1, 11, (n, rhs)).astype(np.float64)
    B = csc_matmat(cp, ri, cv, X)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, cv, B)]
    xd = torch.zeros((n, rhs), dtype=torch.float64, device="cuda")
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                      0 if sub == "fwd" else 1)
    for _ in range(2):
        xd.zero_()
        T.solve_rhs(rhs, d[3].data_ptr(), xd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(xd.cpu().numpy(), X)
    T.close()
    for ngpu in (1, 3):
        x, _ = sb.trsv_mgpu_solve(cp, ri, cv, n, B, ngpu, 0 if sub == "fwd" else 1, rhs)
        assert np.array_equal(x, X)


@pytest.mark.parametrize("opt", [1, 2, 3], ids=["warp_nnz", "warp_rhs", "warp_auto"])
@pytest.mark.parametrize("rhs", [1, 3, 17, 64, 100])
def test_sptrsm_push_lane_mappings(torch_cuda, sb, opt, rhs):
    """The reference's SpTRSM push dataflow with each `opt` lane mapping
    (sptrsv_syncfree_cuda.h:229-281) on the KAT matrices (integer systems:
    exact whatever the atomic order) and on a 300k banded system (against the
    pull executor, fp64 bound)."""
    torch = torch_cuda
    for name, sub in (("qh768", "fwd"), ("ash85", "bwd"), ("qh768", "bwd")):
        g = np.load(os.path.join(GOLDEN, f"trsv_{name}_{sub}.npz"))
        cp, ri, cv = g["colptr"], g["rowidx"], g["val"]
        n = len(cp) - 1
        X = np.random.default_rng(rhs + opt).integers(1, 11, (n, rhs)).astype(np.float64)
        B = csc_matmat(cp, ri, cv, X)
        d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, cv, B)]
        xd = torch.zeros((n, rhs), dtype=torch.float64, device="cuda")
        T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                          0 if sub == "fwd" else 1)
        for _ in range(2):  # scratch reuse
            xd.fill_(-1.0)
            T.solve_rhs_opt(0, opt, rhs, d[3].data_ptr(), xd.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(xd.cpu().numpy(), X), (name, sub)
        T.close()
    n, k = 300_000, 4 if rhs > 4 else rhs
    cp, ri, v, b1, _ = _banded_system(sb, n)
    Bk = np.repeat(b1[:, None], k, axis=1) * (1.0 + np.arange(k))[None, :]
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (cp, ri, v, Bk)]
    T = sb.DeviceTRSV(0, n, len(ri), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 0)
    xp = torch.zeros((n, k), dtype=torch.float64, device="cuda")
    xq = torch.zeros((n, k), dtype=torch.float64, device="cuda")
    T.solve_rhs_opt(0, opt, k, d[3].data_ptr(), xp.data_ptr())
    T.solve_rhs_opt(1, opt, k, d[3].data_ptr(), xq.data_ptr())
    torch.cuda.synchronize()
    T.close()
    p, q = xp.cpu().numpy(), xq.cpu().numpy()
    assert np.abs(p - q).sum() / np.abs(q).sum() < 1e-12


@pytest.mark.parametrize("opt", [1, 2])
def test_sptrsm_reference_api_push(torch_cuda, sb, capfd, opt):
    """sptrsv_syncfree_cuda with rhs > 1 and an explicit lane mapping runs the
    reference's push executor; exact on the integer KAT system."""
    g = np.load(os.path.join(GOLDEN, "trsv_ash85_fwd.npz"))
    cp, ri, cv = g["colptr"], g["rowidx"], g["val"]
    n, rhs = len(cp) - 1, 6
    X = np.random.default_rng(2).integers(1, 11, (n, rhs)).astype(np.float64)
    B = csc_matmat(cp, ri, cv, X)
    x = np.zeros((n, rhs))
    gf = np.zeros(1)
    rc = sb.lib.sblas_sptrsv_syncfree(sb.ptr(cp), sb.ptr(ri), sb.ptr(cv), n, n, len(ri), 0,
                                      rhs, opt, sb.ptr(x), sb.ptr(B), sb.ptr(X), sb.ptr(gf), 1)
    assert rc == 0 and np.array_equal(x, X)
    assert "executor passed!" in capfd.readouterr().out


def test_sptrsm_reference_api(torch_cuda, sb, capfd):
    g = np.load(os.path.join(GOLDEN, "trsv_qh768_fwd.npz"))
    cp, ri, cv = g["colptr"], g["rowidx"], g["val"]
    n, rhs = len(cp) - 1, 5
    X = np.random.default_rng(1).integers(1, 11, (n, rhs)).astype(np.float64)
    B = csc_matmat(cp, ri, cv, X)
    x = np.zeros((n, rhs))
    gf = np.zeros(1)
    for ngpu in (1, 2):
        x[:] = 0
        rc = sb.lib.sblas_sptrsv_syncfree(sb.ptr(cp), sb.ptr(ri), sb.ptr(cv), n, n, len(ri), 0,
                                          rhs, 3, sb.ptr(x), sb.ptr(B), sb.ptr(X), sb.ptr(gf), ngpu)
        assert rc == 0 and np.array_equal(x, X)
    assert "executor passed!" in capfd.readouterr().out


# ------------------------------------------------------------ assembly ----
def test_assemble_slices(torch_cuda, sb):
    torch = torch_cuda
    # 4 partitions; rank 2 and 3 continue a row of the previous one
    meta = np.array([0, 3, 0, 3, 2, 0, 4, 2, 1, 5, 1, 1], np.int32)  # rows 0-2 | 3-4 | 4-5 | 5
    stride = 3
    gathered = np.array([1, 2, 3, 4, 5, 0, 6, 7, 0, 8, 0, 0], np.float64)
    want = np.array([1, 2, 3, 4, 5 + 6, 7 + 8])
    gd = torch.from_numpy(gathered).cuda()
    md = torch.from_numpy(meta).cuda()
    y = torch.full((6,), -1.0, dtype=torch.float64, device="cuda")
    yl = torch.from_numpy(np.array([6.0, 7.0, 0.0])).cuda()  # rank 2's slice
    sb.check(sb.lib.sblas_assemble_slices(gd.data_ptr(), 4, stride, md.data_ptr(), y.data_ptr(),
                                          2, yl.data_ptr(), None), "assemble")
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), want)
    assert np.array_equal(yl.cpu().numpy(), [0.0, 15.0, 0.0])


# ------------------------------------------------------- SpMM MFMA tiles ----
def block_dense_csr(rng, nblk, width, k, sparse_tail=0):
    """16-row blocks, each dense over `width` random columns (MFMA path), plus
    `sparse_tail` random sparse rows (row-wave path)."""
    rows = []
    for _ in range(nblk):
        cols = np.sort(rng.choice(k, width, replace=False))
        for _ in range(16):
            keep = cols[rng.random(width) < 0.9]  # ~90% fill
            rows.append(keep)
    for _ in range(sparse_tail):
        rows.append(np.sort(rng.choice(k, 20, replace=False)))
    lens = np.array([len(r) for r in rows])
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate(rows).astype(np.int32)
    return rp, col, rng.standard_normal(int(rp[-1]))


@pytest.mark.parametrize("fill", ["default", "0", "2"])
@pytest.mark.parametrize("ncols", [64, 40, 130])
def test_spmm_mfma_tiles(torch_cuda, sb, orc, fill, ncols):
    """The v_mfma_f64_16x16x4f64 B-panel tile on block-dense rows (test
    option spmm_mfma_fill: 0 = every 16-row block on MFMA, 2 = none)."""
    torch = torch_cuda
    rng = np.random.default_rng(ncols)
    k = 3000
    rp, col, val = block_dense_csr(rng, 12, 37, k, sparse_tail=21)  # m = 213: partial last block
    m = len(rp) - 1
    B = rng.standard_normal((k, ncols))
    C0 = rng.standard_normal((m, ncols))
    want = orc.spmm(m, ncols, k, 0.75, rp, col, val, B, -0.5, C0)
    A = sb.DeviceCSR.upload(0, k, rp, col, val)
    Bd = torch.from_numpy(np.ascontiguousarray(B).ravel()).cuda()
    Cd = torch.from_numpy(np.asfortranarray(C0).ravel(order="F")).cuda()
    with sb.test_options(**({} if fill == "default" else {"spmm_mfma_fill": float(fill)})):
        A.spmm(ncols, 0.75, Bd.data_ptr(), ncols, 1, -0.5, Cd.data_ptr(), m)
    torch.cuda.synchronize()
    got = Cd.cpu().numpy().reshape((ncols, m)).T
    # MFMA sums the dense tile in union-column order (the rows' own order here,
    # columns are sorted) with exact zeros for the holes: same bound applies
    assert np.all(np.abs(got - want) <= spmm_bound(rp, col, val, B, 0.75, -0.5, C0))
    A.close()


@pytest.mark.parametrize("blocks", [1, 4])
def test_sptrsv_mgpu_block_devices(torch_cuda, sb, blocks):
    """sblas_trsv_mgpu_info: the device each block runs on and its rows (the
    `config5.blocks4.block_devices` of every bench line): block d on device
    d % visible, rows summing to n."""
    n = 50_000
    cp, ri, v, b0, xref = _banded_system(sb, n)
    ngpu = min(blocks, torch_cuda.cuda.device_count())
    H = sb.TrsvMgpu(cp, ri, v, n, ngpu, tasks=blocks // ngpu)
    info = H.info()
    assert len(info) == blocks and sum(r for _, r in info) == n
    assert [d for d, _ in info] == [d % ngpu for d in range(blocks)]
    x, _ = H.run(b0)
    assert np.abs(x - xref).sum() / np.abs(xref).sum() <= 1e-12
    H.close()


def test_sptrsv_mgpu_peer_refusal_is_bounded(torch_cuda, sb):
    """a multi-block solve whose peer links cannot be
    enabled fails at create with SBLAS_ERR_* before launching anything (no
    block spins on stores that can never arrive), in bounded time; the hook
    (sblas_test_deny_peer_access) treats blocks sharing the GPU as distinct
    devices so the refusal runs here.  After the hook is cleared the same
    solve runs and is exact."""
    import time
    n = 50_000
    cp, ri, v, b0, xref = _banded_system(sb, n)
    sb.test_deny_peer_access(True)
    try:
        t0 = time.perf_counter()
        with pytest.raises(sb.SblasError, match="peer"):
            sb.TrsvMgpu(cp, ri, v, n, 1, tasks=4)
        with pytest.raises(sb.SblasError, match="peer"):
            sb.trsv_mgpu_solve_tasks(cp, ri, v, n, b0, 1, 4)
        assert time.perf_counter() - t0 < 30.0
        H1 = sb.TrsvMgpu(cp, ri, v, n, 1, tasks=1)  # one block: no peer link needed
        x1, _ = H1.run(b0)
        H1.close()
    finally:
        sb.test_deny_peer_access(False)
    assert np.abs(x1 - xref).sum() / np.abs(xref).sum() <= 1e-12
    H = sb.TrsvMgpu(cp, ri, v, n, 1, tasks=4)
    x, _ = H.run(b0)
    H.close()
    assert np.abs(x - xref).sum() / np.abs(xref).sum() <= 1e-12
