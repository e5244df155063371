"""Regenerate the committed golden fixtures (tests/golden/*.npz).

Run in the build container, where /root/reference exists:
    make -C oracle && python tests/golden/make_golden.py

Sources of truth, per fixture:
  * *_mmio.npz    : CSR from the reference's own mmio_data
                    (sptrsv/sptrsv_v1/src/mmio_highlevel.h:137-296) compiled in
                    place into oracle/_ref/libsblas_ref.so.
  * trsv_*.npz    : unit-triangular KAT built as sptrsv_v1/src/main.cu:150-355
                    does (fixed seed instead of time(NULL), quirk Q8), solved by
                    the reference's sptrsv_syncfree_analyser/_executor
                    (sptrsv_syncfree_serialref.h:6-108) from the same build.
  * spmv_*.npz    : y of test_spmv's dataflow (loader Q1, alpha/beta from
                    unseeded glibc rand(), x = 1) from the oracle restatement --
                    cuSPARSE is absent, so these are regression vectors of the
                    restatement ("parity unpinned" for the arithmetic itself,
                    pinned only through loader + alpha/beta + the ref test's
                    own abs 1e-3 criterion).
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import orc  # noqa: E402

if orc.ref is None:
    sys.exit("oracle/_ref/libsblas_ref.so missing: run `make -C oracle` with /root/reference present")

P = orc.P


def ref_mmio(path):
    m, n, nnz, sym = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    assert orc.ref.ref_mmio_info(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(sym)) == 0
    rp = np.zeros(m.value + 1, np.int32)
    col = np.zeros(nnz.value, np.int32)
    val = np.zeros(nnz.value)
    assert orc.ref.ref_mmio_data(path.encode(), P(rp), P(col), P(val)) == 0
    return m.value, n.value, rp, col, val, sym.value


def ref_trsv(cp, ri, cv, b, substitution):
    n = len(cp) - 1
    x = np.zeros(n)
    assert orc.ref.ref_sptrsv_serial(P(cp), P(ri), P(cv), n, len(ri), substitution, 1, P(b), P(x)) == 0
    return x


def main():
    for name in ("qh768", "ash85"):
        path = os.path.join(HERE, f"{name}.mtx")
        m, n, rp, col, val, sym = ref_mmio(path)
        np.savez_compressed(os.path.join(HERE, f"{name}_mmio.npz"), m=m, n=n, rowptr=rp,
                            col=col, val=val, sym=sym)
        for sub in (0, 1):
            (trp, tc, tv), (cp, ri, cv), xref, b = orc.build_tri(rp, col, sub, seed=1)
            x = ref_trsv(cp, ri, cv, b, sub)
            np.savez_compressed(os.path.join(HERE, f"trsv_{name}_{'fwd' if sub == 0 else 'bwd'}.npz"),
                                colptr=cp, rowidx=ri, val=cv, b=b, x_ref=xref, x_refsolve=x)
    # test_spmv 'f' dataflow on qh768
    alpha, beta = orc.alpha_beta()
    m, n, rp, col, val = orc.load_testspmv(os.path.join(HERE, "qh768.mtx"), "f")
    y = orc.csr_spmv(rp, col, val, np.ones(n), alpha, beta, np.zeros(m))
    np.savez_compressed(os.path.join(HERE, "spmv_qh768_testspmv.npz"), alpha=alpha, beta=beta,
                        rowptr=rp, col=col, val=val, y=y)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
