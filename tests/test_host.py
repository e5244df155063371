"""Host-side product code (libsblas, no GPU needed) vs the oracle."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.mark.parametrize("name", ["qh768", "ash85"])
def test_mm_read_mmio_mode(sb, orc, name):
    path = os.path.join(GOLDEN, f"{name}.mtx")
    m, n, rp, col, val = sb.mm_read(path, 0)
    m2, n2, rp2, col2, val2, _ = orc.load_mmio(path)
    assert (m, n) == (m2, n2)
    assert np.array_equal(rp, rp2.astype(np.int64))
    assert np.array_equal(col, col2) and np.array_equal(val, val2)


@pytest.mark.parametrize("mode,dt,name", [(1, "f", "qh768"), (2, "b", "ash85")])
def test_mm_read_testspmv_modes(sb, orc, mode, dt, name):
    path = os.path.join(GOLDEN, f"{name}.mtx")
    m, n, rp, col, val = sb.mm_read(path, mode)
    m2, n2, rp2, col2, val2 = orc.load_testspmv(path, dt)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)


def test_mm_read_errors(sb, tmp_path):
    bad = tmp_path / "bad.mtx"
    bad.write_text("not a matrix\n")
    with pytest.raises(sb.SblasError):
        sb.mm_read(str(bad))
    with pytest.raises(sb.SblasError):
        sb.mm_read(str(tmp_path / "missing.mtx"))
    oob = tmp_path / "oob.mtx"
    oob.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")
    with pytest.raises(sb.SblasError):
        sb.mm_read(str(oob))


def test_mm_read_integer_complex(sb, orc, tmp_path):
    p = tmp_path / "ic.mtx"
    p.write_text("%%MatrixMarket matrix coordinate integer symmetric\n% c\n3 3 3\n1 1 4\n3 1 -2\n3 2 7\n")
    m, n, rp, col, val = sb.mm_read(str(p), 0)
    m2, n2, rp2, col2, val2, _ = orc.load_mmio(str(p))
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
    p2 = tmp_path / "cx.mtx"
    p2.write_text("%%MatrixMarket matrix coordinate complex general\n2 2 2\n1 2 1.5 9\n2 1 -3 1\n")
    m, n, rp, col, val = sb.mm_read(str(p2), 0)
    assert list(val) == [1.5, -3.0]


def _rand_rowptr(rng, m, maxlen, empty_frac):
    lens = rng.integers(0, maxlen, m)
    lens[rng.random(m) < empty_frac] = 0
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)


@pytest.mark.parametrize("seed", range(6))
def test_partition_nnz_matches_oracle(sb, orc, seed):
    rng = np.random.default_rng(seed)
    m = int(rng.integers(1, 500))
    rp = _rand_rowptr(rng, m, int(rng.integers(1, 50)), [0.0, 0.3, 0.9][seed % 3])
    if seed == 5:
        rp[1:] += 5000  # a single giant first row spanning partitions
    for g in (1, 2, 3, 5, 8, 13):
        a = sb.partition_nnz(rp, g)
        b = orc.partition_nnz(rp, g)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
        si, ei, sr, er, sf = a
        # every row covered, in order; continuation only when the row is split
        covered = []
        for d in range(g):
            rows = list(range(sr[d], er[d] + 1))
            if sf[d]:
                assert covered and covered[-1] == sr[d]
                rows = rows[1:]
            covered += rows
        assert covered == list(range(m))


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("w", [0.0, 6.0, 100.0])
def test_partition_cost_whole_rows_balanced(sb, seed, w):
    """The cost-weighted split (sblas_partition_cost): contiguous whole-row
    ranges covering every row once, no carries, index ranges matching the
    rows, and each range's cost sum(nnz_r + w) within one row's cost of the
    ideal share."""
    rng = np.random.default_rng(seed)
    m = int(rng.integers(1, 600))
    rp = _rand_rowptr(rng, m, int(rng.integers(1, 50)), [0.0, 0.3, 0.9][seed % 3])
    cost = rp[1:] - rp[:-1] + w
    for g in (1, 2, 3, 5, 8, 13):
        si, ei, sr, er, sf = sb.partition_cost(rp, g, w)
        assert not sf.any() and sr[0] == 0 and er[-1] == m - 1
        assert np.all(sr[1:] == er[:-1] + 1)
        assert np.array_equal(si, rp[sr]) and np.array_equal(ei, rp[er + 1] - 1)
        share = cost.sum() / g
        for d in range(g):
            c = cost[sr[d]:er[d] + 1].sum()
            assert c <= share + cost.max() + 1e-9, (g, d, c, share)


def test_partition_cost_config2_shape(sb):
    """On config 2's shape (rows < n/8: 96 entries, others 9) the cost split
    gives the light ranks fewer entries than the nnz split does."""
    rp = sb.gen_synth_rowptr(2_000_000)
    si, ei, sr, er, _ = sb.partition_cost(rp, 8, 6.0)
    nnz = ei - si + 1
    assert nnz[-1] < rp[-1] / 8 < nnz[0]
    costs = [(rp[er[d] + 1] - rp[sr[d]]) + 6.0 * (er[d] - sr[d] + 1) for d in range(8)]
    assert max(costs) / min(costs) < 1.001


def test_partition_rowblock(sb, orc):
    for m, g in [(10, 3), (2000000, 8), (5, 8), (0, 2)]:
        rs = sb.partition_rowblock(m, g)
        assert rs[0] == 0 and rs[-1] == m and np.all(np.diff(rs) >= 0)


@pytest.mark.parametrize("prefix", [False, True])
def test_generator_bit_exact(sb, orc, prefix):
    n = 6000
    rp = sb.gen_synth_rowptr(n)
    rp2, col2, val2 = orc.gen_synth(n, prefix=prefix)
    assert np.array_equal(rp, rp2)
    col, val = sb.gen_synth_rows(n, rp, 0, n, prefix=prefix)
    assert np.array_equal(col, col2) and np.array_equal(val, val2)
    # slices generate the same rows
    c1, v1 = sb.gen_synth_rows(n, rp, 700, 3100, prefix=prefix)
    assert np.array_equal(c1, col2[rp[700]:rp[3100]]) and np.array_equal(v1, val2[rp[700]:rp[3100]])
    if not prefix:
        for r in (0, 5, n // 8 - 1, n // 8, n - 1):
            seg = col[rp[r]:rp[r + 1]]
            assert np.all(np.diff(seg) > 0) and seg.min() >= 0 and seg.max() < n


def test_generator_rows_independent(sb):
    """Rows draw independent uniform columns (round 5: rounds 1-4 started row
    i+1's stream where row i's left off after one draw, so runs of rows
    shared their column sets; profiles/r05/gen/).  On config 2's first 20k
    heavy rows and 20k light rows the distinct-column fraction matches
    uniform draws and consecutive rows share ~nothing."""
    n = 2_000_000
    rp = sb.gen_synth_rowptr(n)
    for a, L in ((0, 96), (1_000_000, 9)):
        col, _ = sb.gen_synth_rows(n, rp, a, a + 20000)
        c = col.reshape(-1, L)
        want = n * (1 - np.exp(-col.size / n)) / col.size
        assert abs(len(np.unique(col)) / col.size - want) < 0.01
        shared = [len(np.intersect1d(c[i], c[i + 1])) for i in range(0, len(c) - 1, 7)]
        assert np.mean(shared) < 0.05 * L and max(shared) <= 3
    # the SpTRSV stand-in's columns likewise (per-column streams)
    cp, ri, _ = sb.gen_lower_banded(200000, 5, 80000, 47)
    both = [len(np.intersect1d(ri[cp[j] + 1:cp[j + 1]], ri[cp[j + 1] + 1:cp[j + 2]])) for j in range(1000, 5000)]
    assert sum(both) <= 10  # ~25 / 80000 per pair expected


def test_config2_shape(sb):
    rp = sb.gen_synth_rowptr(2_000_000)
    assert int(rp[-1]) == 39_750_000
    assert np.array_equal(sb.gen_vector(1000, 43), __import__("orc").gen_vector(1000, 43))


def test_get_row_from_index_fixed(sb):
    rp = np.array([0, 2, 2, 2, 5, 7], np.int64)
    assert sb.lib.sblas_get_row_from_index(5, sb.ptr(rp), 2) == 3
    assert sb.lib.sblas_get_row_from_index(5, sb.ptr(rp), 6) == 4


def write_mtx(path, m, n, r, c, v, field="real", symm="general"):
    with open(path, "w") as fh:
        fh.write(f"%%MatrixMarket matrix coordinate {field} {symm}\n% generated\n")
        fh.write(f"{m} {n} {len(r)}\n")
        if field == "pattern":
            fh.writelines(f"{a + 1} {b + 1}\n" for a, b in zip(r, c))
        elif field == "integer":
            fh.writelines(f"{a + 1} {b + 1} {int(x)}\n" for a, b, x in zip(r, c, v))
        else:
            fh.writelines(f"{a + 1} {b + 1} {float(x)!r}\n" for a, b, x in zip(r, c, v))


@pytest.mark.parametrize("field,symm", [("real", "general"), ("real", "symmetric"),
                                        ("integer", "general"), ("pattern", "symmetric")])
def test_mm_read_parallel_matches_oracle(sb, orc, tmp_path, field, symm):
    """> 1 MB of entries, so the parser splits the file across
    threads; the CSR must equal the sequential oracle loader exactly."""
    rng = np.random.default_rng(5)
    m = n = 30000
    k = 120000
    r = rng.integers(0, m, k)
    c = rng.integers(0, n, k)
    if symm == "symmetric":
        r, c = np.maximum(r, c), np.minimum(r, c)
    v = rng.integers(-50, 50, k) if field == "integer" else rng.standard_normal(k)
    path = str(tmp_path / "big.mtx")
    write_mtx(path, m, n, r, c, v, field, symm)
    assert os.path.getsize(path) > (1 << 20)
    got = sb.mm_read(path, 0)
    want = orc.load_mmio(path)
    assert got[:2] == want[:2]
    assert np.array_equal(got[2], want[2].astype(np.int64))
    assert np.array_equal(got[3], want[3]) and np.array_equal(got[4], want[4])
    if field == "real":
        got1 = sb.mm_read(path, 1)
        want1 = orc.load_testspmv(path, "f")
        assert all(np.array_equal(a, b) for a, b in zip(got1[2:], want1[2:]))


def test_mm_cache_roundtrip_and_staleness(sb, orc, tmp_path, monkeypatch):
    rng = np.random.default_rng(6)
    m, n, k = 500, 400, 3000
    r, c, v = rng.integers(0, m, k), rng.integers(0, n, k), rng.standard_normal(k)
    path = str(tmp_path / "a.mtx")
    write_mtx(path, m, n, r, c, v)
    cache = tmp_path / "cache"
    cache.mkdir()
    monkeypatch.setenv("SBLAS_MM_CACHE", str(cache))
    first = sb.mm_read(path, 0)
    assert (cache / "a.mtx.m0.csrbin").exists()
    second = sb.mm_read(path, 0)  # served from the cache
    for a, b in zip(first[2:], second[2:]):
        assert np.array_equal(a, b)
    # a changed source invalidates the cache entry
    write_mtx(path, m, n, r[:-10], c[:-10], v[:-10])
    os.utime(path, ns=(1, 1))
    third = sb.mm_read(path, 0)
    assert third[2][-1] == k - 10
    want = orc.load_mmio(path)
    assert np.array_equal(third[3], want[3]) and np.array_equal(third[4], want[4])


def test_csrbin_write_read(sb, tmp_path):
    rp = np.array([0, 2, 2, 5], np.int64)
    col = np.array([0, 3, 1, 2, 3], np.int32)
    val = np.arange(5, dtype=np.float64) / 3
    p = str(tmp_path / "x.csrbin")
    sb.csrbin_write(p, 3, 4, rp, col, val)
    m, n, rp2, col2, val2 = sb.csrbin_read(p)
    assert (m, n) == (3, 4)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
    with open(p, "r+b") as fh:
        fh.write(b"X")
    with pytest.raises(sb.SblasError):
        sb.csrbin_read(p)


def test_mm_read_truncated(sb, tmp_path):
    p = tmp_path / "t.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real general\n3 3 4\n1 1 1.0\n2 2 2.0\n")
    with pytest.raises(sb.SblasError, match="entries"):
        sb.mm_read(str(p))


@pytest.mark.parametrize("seed", [0, 1])
def test_coo_sortbyrow_matches_oracle(sb, orc, seed):
    """sortbyrow + COO -> CSR (dspmm_baseline_test.cu:41-55,
    461-493): distinct (row, col) entries in random order sort bit-exactly
    as the reference's qsort by (row, col); empty rows get empty ranges."""
    rng = np.random.default_rng(seed)
    m, k, nnz = 500, 300, 6000
    flat = rng.choice(m * k, nnz, replace=False)
    row = (flat // k).astype(np.int32)
    col = (flat % k).astype(np.int32)
    row[row == 7] = 8  # one empty row
    flat = np.unique(row.astype(np.int64) * k + col)
    rng.shuffle(flat)
    row, col = (flat // k).astype(np.int32), (flat % k).astype(np.int32)
    val = rng.standard_normal(len(row))
    r1, c1, v1, rp1 = sb.coo_sortbyrow(m, row, col, val)
    r2, c2, v2 = row.copy(), col.copy(), val.copy()
    rp2 = np.zeros(m + 1, np.int32)
    orc.lib.orc_coo_sort_to_csr(m, len(r2), orc.P(r2), orc.P(c2), orc.P(v2), orc.P(rp2))
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2) and np.array_equal(v1, v2)
    assert np.array_equal(rp1, rp2) and rp1[8] == rp1[7 + 1]


def test_coo_sortbyrow_test_spmm_loader(sb, orc):
    """test_spmm's loader (mode 3) + sortbyrow on qh768 gives the CSR that the
    mmio_data loader gives for a general (non-symmetric) file, once each row
    is ordered by column; duplicates keep file order; bad rows rejected."""
    path = os.path.join(GOLDEN, "qh768.mtx")
    m, n, rp, col, val = sb.mm_read(path, 3)
    row = np.repeat(np.arange(m, dtype=np.int32), np.diff(rp))
    r, c, v, rp32 = sb.coo_sortbyrow(m, row, col, val)
    assert np.array_equal(rp32, rp)
    key = r.astype(np.int64) * n + c
    assert np.all(np.diff(key) >= 0)
    # same multiset of entries as the file
    _, _, rp0, col0, val0 = sb.mm_read(path, 1)
    assert sorted(zip(col0.tolist(), val0.tolist())) == sorted(zip(c.tolist(), v.tolist()))
    # duplicates: stable
    rr, cc, vv, _ = sb.coo_sortbyrow(2, np.array([1, 0, 1, 1], np.int32), np.array([5, 1, 5, 2], np.int32),
                                     np.array([1.0, 2.0, 3.0, 4.0]))
    assert rr.tolist() == [0, 1, 1, 1] and cc.tolist() == [1, 2, 5, 5] and vv.tolist() == [2.0, 4.0, 1.0, 3.0]
    with pytest.raises(sb.SblasError):
        sb.coo_sortbyrow(2, np.array([2], np.int32), np.array([0], np.int32), np.array([1.0]))


@pytest.mark.parametrize("m,g", [(0, 1), (1, 3), (1000, 1), (1003, 2), (2_000_00, 8), (77, 5)])
def test_cyclic_partition_matches_dist_plan(sb, m, g):
    """The C-ABI context's cyclic distribution (sblas_cyclic_plan /
    sblas_cyclic_local_csr, used by sblas_ctx) is the one sblas_dist's
    CyclicPlan deals to torch.distributed ranks: same chunk size, slice
    stride and local CSR, bit for bit, and the slices tile the matrix."""
    import sblas_dist
    rng = np.random.default_rng(m + g)
    lens = rng.integers(0, 7, m)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = rng.integers(0, max(m, 1), int(rp[-1])).astype(np.int32)
    val = rng.standard_normal(int(rp[-1]))
    plan = sblas_dist.make_cyclic_plan(rp, m, g)
    R, S = sb.cyclic_plan(m, g)
    assert (R, S) == (plan.chunk_rows, plan.stride)
    total_rows = total_nnz = 0
    for d in range(g):
        lrp, lc, lv = sb.cyclic_local_csr(rp, col, val, g, R, d)
        wrp, wc, wv = sblas_dist.cyclic_local_csr(rp, plan, d, lambda a, b: (col[rp[a]:rp[b]], val[rp[a]:rp[b]]))
        assert np.array_equal(lrp, wrp) and np.array_equal(lc, wc) and np.array_equal(lv, wv)
        assert len(lrp) - 1 == plan.local_rows(d) <= S
        total_rows += len(lrp) - 1
        total_nnz += int(lrp[-1])
    assert total_rows == m and total_nnz == int(rp[-1])


@pytest.mark.parametrize("m,g", [(1, 2), (77, 5), (1003, 2), (1003, 3), (200_003, 8), (9, 4)])
def test_overlap_halves_place_every_row_once(m, g):
    """DistSpMVCyclic(overlap=True) splits each rank's slice at hA chunks
    and places the halves with two assemble_cyclic calls (rows [0, rows_a)
    and [rows_a, m)).  With each rank's slice filled by its global row ids,
    the two placements reproduce 0..m-1 (ragged last chunk, ranks with fewer
    chunks included)."""
    import sblas_dist
    rp = np.zeros(m + 1, np.int64)
    plan = sblas_dist.make_cyclic_plan(rp, m, g)
    hA, sA, sB, rows_a = sblas_dist.overlap_halves(plan)
    assert sA + sB == plan.stride or (sA == plan.stride and sB == 1)
    R = plan.chunk_rows
    slices = []
    for d in range(g):
        ids = np.concatenate([np.arange(a, b) for a, b in plan.chunks(d)] or [np.zeros(0, np.int64)])
        buf = np.full(plan.stride + 1, -1, np.int64)
        buf[:len(ids)] = ids
        slices.append(buf)

    def place(gathered, stride, rows):
        r = np.arange(rows)
        j = r // R
        return gathered[(j % g) * stride + (j // g) * R + (r - j * R)]

    gA = np.concatenate([s[:sA] for s in slices])
    gB = np.concatenate([s[sA:sA + sB] for s in slices])
    y = np.concatenate([place(gA, sA, rows_a), place(gB, sB, m - rows_a)])
    assert np.array_equal(y, np.arange(m))


@pytest.mark.parametrize("points", [7, 27])
def test_stencil3d_generator(sb, points):
    """sblas_gen_stencil3d: natural-order 3-D stencil, every neighbour inside
    the grid present exactly once, columns ascending, symmetric pattern,
    diagonally dominant, deterministic."""
    nx, ny, nz = 5, 4, 3
    rp, col, val = sb.gen_stencil3d(nx, ny, nz, points, seed=7)
    n = nx * ny * nz
    assert len(rp) == n + 1
    A = np.zeros((n, n))
    for r in range(n):
        c = col[rp[r]:rp[r + 1]]
        assert np.all(np.diff(c) > 0)
        A[r, c] = val[rp[r]:rp[r + 1]]
        i, j, k = r % nx, (r // nx) % ny, r // (nx * ny)
        want = []
        for dk in (-1, 0, 1):
            for dj in (-1, 0, 1):
                for di in (-1, 0, 1):
                    if points == 7 and abs(di) + abs(dj) + abs(dk) > 1:
                        continue
                    if 0 <= i + di < nx and 0 <= j + dj < ny and 0 <= k + dk < nz:
                        want.append(r + (dk * ny + dj) * nx + di)
        assert list(c) == want
    assert np.array_equal(A != 0, (A != 0).T)
    off = np.abs(A).sum(axis=1) - np.abs(np.diag(A))
    assert np.allclose(np.diag(A), 1.0 + off)
    rp2, col2, val2 = sb.gen_stencil3d(nx, ny, nz, points, seed=7)
    assert np.array_equal(col, col2) and np.array_equal(val, val2)


def test_rmat_generator(sb):
    """sblas_gen_rmat: 2^scale rows, sorted distinct columns per row, at most
    edge_factor * 2^scale entries after merging duplicates, a power-law row
    length spread, deterministic for a seed."""
    scale, ef = 12, 16
    rp, col, val = sb.gen_rmat(scale, ef, seed=3)
    n = 1 << scale
    assert len(rp) == n + 1 and 0 < rp[-1] <= ef * n
    assert np.all((col >= 0) & (col < n))
    for r in range(n):
        assert np.all(np.diff(col[rp[r]:rp[r + 1]]) > 0)
    lens = np.diff(rp)
    assert lens.max() > 20 * lens.mean()          # heavy rows exist
    assert (lens == 0).sum() > 0                    # and empty ones
    assert np.all(val > 0)                          # U[0,1) draws, merged by summing
    rp2, col2, val2 = sb.gen_rmat(scale, ef, seed=3)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
