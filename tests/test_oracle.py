"""Pin the oracle (CPU restatement) before trusting it.

* against the reference's own host code compiled in place (oracle/_ref),
  when that build exists (build container);
* against the committed golden fixtures (always; made by
  tests/golden/make_golden.py from the same reference build);
* against the reference facts recorded in SURVEY.md [probe] rows.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def gold(name):
    return np.load(os.path.join(GOLDEN, name))


def test_alpha_beta_constants(orc):
    # SURVEY §3.1 [probe]: test_spmv f draws ALPHA/BETA = 0.8401877172 / 0.3943829268
    a, b = orc.alpha_beta()
    assert abs(a - 0.8401877172) < 1e-10 and abs(b - 0.3943829268) < 1e-10
    g = gold("spmv_qh768_testspmv.npz")
    assert a == float(g["alpha"]) and b == float(g["beta"])


@pytest.mark.parametrize("name", ["qh768", "ash85"])
def test_mmio_loader_vs_golden(orc, name):
    m, n, rp, col, val, sym = orc.load_mmio(os.path.join(GOLDEN, f"{name}.mtx"))
    g = gold(f"{name}_mmio.npz")
    assert (m, n, sym) == (int(g["m"]), int(g["n"]), int(g["sym"]))
    assert np.array_equal(rp, g["rowptr"]) and np.array_equal(col, g["col"])
    assert np.array_equal(val, g["val"])


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref",
                                                    "libsblas_ref.so")),
                    reason="oracle/_ref not built (no /root/reference here)")
@pytest.mark.parametrize("name", ["qh768", "ash85"])
def test_mmio_loader_vs_reference_build(orc, name):
    import ctypes as C
    path = os.path.join(GOLDEN, f"{name}.mtx")
    m, n, nnz, sym = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    assert orc.ref.ref_mmio_info(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(sym)) == 0
    rp = np.zeros(m.value + 1, np.int32)
    col = np.zeros(nnz.value, np.int32)
    val = np.zeros(nnz.value)
    assert orc.ref.ref_mmio_data(path.encode(), orc.P(rp), orc.P(col), orc.P(val)) == 0
    m2, n2, rp2, col2, val2, sym2 = orc.load_mmio(path)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
    hm, hn, hz, hf = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    assert orc.ref.ref_mm_header(path.encode(), C.byref(hm), C.byref(hn), C.byref(hz), C.byref(hf)) == 0
    om, on, oz, of = orc.mm_info(path)
    assert (hm.value, hn.value, hz.value, hf.value) == (om, on, oz, of)


@pytest.mark.parametrize("name", ["qh768", "ash85"])
@pytest.mark.parametrize("sub", ["fwd", "bwd"])
def test_sptrsv_serial_vs_golden(orc, name, sub):
    g = gold(f"trsv_{name}_{sub}.npz")
    x = orc.sptrsv_serial(g["colptr"], g["rowidx"], g["val"], g["b"], 0 if sub == "fwd" else 1)
    # KAT: integer L, unit diagonal, x_ref in 1..10 -> exact in fp64
    assert np.array_equal(x, g["x_ref"])
    assert np.array_equal(x, g["x_refsolve"])  # the reference's own executor


@pytest.mark.parametrize("name", ["qh768", "ash85"])
def test_build_tri_matches_golden(orc, name):
    g = gold(f"{name}_mmio.npz")
    for sub in (0, 1):
        _, (cp, ri, cv), xref, b = orc.build_tri(g["rowptr"], g["col"], sub, seed=1)
        t = gold(f"trsv_{name}_{'fwd' if sub == 0 else 'bwd'}.npz")
        assert np.array_equal(cp, t["colptr"]) and np.array_equal(ri, t["rowidx"])
        assert np.array_equal(cv, t["val"]) and np.array_equal(b, t["b"])


def test_tri_sizes_and_levels(orc):
    # SURVEY §8 H12 [probe]: qh768-L nnz 2066 / 14 levels, ash85-L nnz 304 / 43 levels
    for name, nnz, nlev in (("qh768", 2066, 14), ("ash85", 304, 43)):
        t = gold(f"trsv_{name}_fwd.npz")
        assert len(t["rowidx"]) == nnz
        assert orc.levels_lower(t["colptr"], t["rowidx"]) == nlev


def test_transpose_stable(orc):
    g = gold("qh768_mmio.npz")
    m, n = int(g["m"]), int(g["n"])
    cp, ri, cv = orc.transpose(m, n, g["rowptr"], g["col"], g["val"])
    for c in range(n):
        seg = ri[cp[c]:cp[c + 1]]
        assert np.all(np.diff(seg) > 0)
    # round trip CSR -> CSC -> CSR
    rp2, ci2, v2 = orc.transpose(n, m, cp, ri, cv)
    dense = np.zeros((m, n))
    for r in range(m):
        dense[r, g["col"][g["rowptr"][r]:g["rowptr"][r + 1]]] += g["val"][g["rowptr"][r]:g["rowptr"][r + 1]]
    dense2 = np.zeros((m, n))
    for r in range(m):
        dense2[r, ci2[rp2[r]:rp2[r + 1]]] += v2[rp2[r]:rp2[r + 1]]
    assert np.array_equal(dense, dense2)


def test_testspmv_loader_quirk_q1(orc):
    """test_spmv 'f' keeps col/val in file order (Q1): 766/768 rows of qh768
    differ from the true A*x ([probe])."""
    path = os.path.join(GOLDEN, "qh768.mtx")
    m, n, rp, col, val = orc.load_testspmv(path, "f")
    g = gold("spmv_qh768_testspmv.npz")
    assert np.array_equal(rp, g["rowptr"]) and np.array_equal(col, g["col"])
    y = orc.csr_spmv(rp, col, val, np.ones(n), float(g["alpha"]), float(g["beta"]), np.zeros(m))
    assert np.array_equal(y, g["y"])
    _, _, rp0, col0, val0, _ = orc.load_mmio(path)
    ytrue = orc.csr_spmv(rp0, col0, val0, np.ones(n), float(g["alpha"]), 0.0, np.zeros(m))
    differ = np.sum(np.abs(y - ytrue) > 1e-6 * np.maximum(1, np.abs(ytrue)))
    assert differ == 766
    assert abs(y.sum() - ytrue.sum()) <= 1e-9 * np.abs(ytrue).sum()


def test_reference_binary_search_q5(orc):
    """get_row_from_index returns *a* row whose rowptr equals idx (Q5);
    the fixed search returns the last such row (the non-empty one)."""
    rp = np.array([0, 2, 2, 2, 5, 7], np.int64)  # rows 1,2 empty
    assert orc.lib.orc_row_of_index(5, orc.P(rp), 2) == 3
    r = orc.lib.orc_get_row_from_index_ref(5, orc.P(rp), 2)
    assert rp[r] == 2


@pytest.mark.parametrize("g", [1, 2, 3, 4, 7, 8])
def test_v1_flow_matches_plain_spmv(orc, g):
    """orc_spmv_mgpu_v1 (partition + host fix-up, dspmv_mgpu_v1.cu) equals a
    single csrmv within the fp64 bound, including empty rows at splits."""
    rng = np.random.default_rng(g)
    m, n = 400, 300
    lens = rng.integers(0, 12, m)
    lens[rng.random(m) < 0.3] = 0
    lens[50] = 700 if n >= 700 else n
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
    val = rng.standard_normal(int(rp[-1]))
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    a, b = orc.alpha_beta()
    want = orc.csr_spmv(rp, col, val, x, a, b, y0)
    for version in ("v1", "baseline"):
        got = orc.spmv_mgpu(version, m, n, rp, col, val, x, a, b, y0, g)
        assert np.all(np.abs(got - want) <= orc.spmv_bound(rp, col, val, x, a, b, y0))


def test_gen_ref_shape(orc):
    # dspmv_test.cu 'g n': first n/8 rows ceil(0.9n) cols, others ceil(0.01n)
    r, c, v = orc.gen_ref(800)
    assert len(r) == 100 * 720 + 700 * 8
    assert r[0] == 0 and c[719] == 719 and r[720] == 1
    assert np.all((v >= 0) & (v <= 1))
