"""Single-process multi-GPU context over RCCL (sblas_ctx, include/sblas.h §3).

The context is the C-ABI's multi-GPU SpMV: ncclCommInitAll over distinct
devices, resident slices, ncclBroadcast of x, ONE ncclAllGather of the y
slices and device placement (or configs[2]'s ncclAllReduce of the
zero-padded y).  On the one-GPU box the communicator has one rank:
ncclBroadcast and the timing protocol's aligning ncclAllReduce run on every
context; a plain one-device context aliases y and skips the y exchange, so
the y collectives (ncclAllGather, ncclAllReduce of y) run only where the
tests set SBLAS_CTX_NOALIAS=1 (test_ctx_noalias_exchange_rccl) and in the
overlapped form (test_ctx_overlap_parts, g = 1).  The g > 1 partition /
exchange / placement logic runs in loopback (SBLAS_CTX_LOOPBACK=1: ranks on
one GPU, collectives as stream-ordered device copies) and on the CPU in
tests/test_host.py and tests/test_dist_cpu.py.  Parity: the oracle's CSR
SpMV with the per-row fp64 bound.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def rand_csr(rng, m, n, maxlen, long_rows=()):
    lens = rng.integers(0, maxlen, m)
    lens[rng.random(m) < 0.1] = 0
    for r, L in long_rows:
        lens[r] = L
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(n, L, replace=False)) for L in lens]).astype(np.int32)
    return rp, col, rng.standard_normal(int(rp[-1]))


@pytest.mark.parametrize("algo", [0, 1, 2, 4, 5])
@pytest.mark.parametrize("partition,exchange", [(0, 0), (1, 0), (1, 1), (2, 1)])
def test_ctx_spmv_chain(torch_cuda, sb, orc, algo, partition, exchange):
    """Two chained steps (the second's beta input is the first's y, kept on
    the devices by the context) against the oracle; exchange 1 is the
    literal all-reduce of the zero-padded y (BASELINE configs[2])."""
    rng = np.random.default_rng(algo + 10 * partition)
    m, n = 5000, 7000
    rp, col, val = rand_csr(rng, m, n, 40, long_rows=[(3, 6000), (4000, 2500)])
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(1)
    ctx.upload(m, n, rp, col, val, algo, partition, exchange)
    # AUTO resolves per slice (scattered columns, < 2M nonzeros: panel)
    assert ctx.slice_algo(0) == (algo if algo else sb.PANEL)
    ctx.set_x(x)
    ctx.set_y(y0)
    k, xch, tot = ctx.spmv(alpha, beta)
    assert k >= 0 and xch >= 0 and tot >= k
    y1 = ctx.get_y()
    want1 = orc.csr_spmv(rp, col, val, x, alpha, beta, y0)
    assert np.all(np.abs(y1 - want1) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y0))
    ctx.spmv(alpha, beta)
    y2 = ctx.get_y()
    want2 = orc.csr_spmv(rp, col, val, x, alpha, beta, y1)
    assert np.all(np.abs(y2 - want2) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y1))
    ctx.close()


@pytest.mark.parametrize("algo", [0, 2, 5])
def test_ctx_config2_full_size(torch_cuda, sb, orc, algo):
    n = 2_000_000
    rp = sb.gen_synth_rowptr(n)
    col, val = sb.gen_synth_rows(n, rp, 0, n)
    x = sb.gen_vector(n, 43)
    y0 = sb.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(1)
    ctx.upload(n, n, rp, col, val, algo, 0)
    assert ctx.slice_algo(0) == (algo if algo else sb.XSORT)
    ctx.set_x(x)
    ctx.set_y(y0)
    ctx.spmv(alpha, beta)
    got = ctx.get_y()
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    assert np.all(np.abs(got - want) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y0))
    ctx.close()


def test_ctx_timed_steps_and_slice_info(torch_cuda, sb, orc):
    """sblas_ctx_spmv_ex's timing protocol (device-side hold + aligning
    all-reduce), the non-waiting form + sblas_ctx_sync, and slice_info."""
    rng = np.random.default_rng(7)
    m, n = 3000, 4000
    rp, col, val = rand_csr(rng, m, n, 30)
    x = rng.standard_normal(n)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(1)
    ctx.upload(m, n, rp, col, val, 5, 1, sb.CTX_ALLREDUCE)
    rows, nnz, byts = ctx.slice_info(0)
    assert (rows, nnz) == (m, int(rp[-1]))
    assert byts == 12 * nnz + 4 * (m + 1) + 8 * n + 16 * m
    ctx.set_x(x)
    y = np.zeros(m)
    ctx.set_y(y)
    st = ctx.spmv_ex(alpha, beta, delay_us=200.0)
    assert st.shape == (6,) and st[0] > 0 and st[2] >= st[0] and st[2] < 50.0
    assert st[3] == st[0] and st[5] == st[2]
    assert st[1] < 0.02  # one device: the kernel writes y in place, nothing to exchange
    y = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
    for _ in range(3):
        assert ctx.spmv_ex(alpha, beta, wait=False) is None
        y_prev = y
        y = orc.csr_spmv(rp, col, val, x, alpha, beta, y_prev)
    last = ctx.sync()
    assert last[2] > 0
    got = ctx.get_y()
    assert np.allclose(got, y, rtol=1e-12, atol=1e-12)
    ctx.close()


def test_ctx_allreduce_needs_contiguous_partition(torch_cuda, sb):
    rng = np.random.default_rng(8)
    rp, col, val = rand_csr(rng, 100, 100, 5)
    ctx = sb.DeviceCtx(1)
    with pytest.raises(sb.SblasError):
        ctx.upload(100, 100, rp, col, val, 2, 0, sb.CTX_ALLREDUCE)
    ctx.close()


def test_ctx_bound_reference_api(torch_cuda, sb, orc):
    """spMV_mgpu_v1 with a bound context of the same size runs the RCCL path;
    other ngpu values keep the host-merge path; both match the oracle."""
    rng = np.random.default_rng(4)
    m, n = 2500, 3000
    rp, col, val = rand_csr(rng, m, n, 40, long_rows=[(10, 2500)])
    x = rng.standard_normal(n)
    y0 = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv(rp, col, val, x, alpha, beta, y0)
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y0)
    ctx = sb.DeviceCtx(1)
    ctx.bind()
    try:
        for ngpu, kernel in ((1, 1), (1, 2), (2, 1), (3, 3)):
            y = y0.copy()
            assert sb.spmv_mgpu("v1", m, n, rp, col, val, x, y, alpha, beta, ngpu=ngpu, kernel=kernel) == 0
            assert np.all(np.abs(y - want) <= bound), (ngpu, kernel)
    finally:
        sb.DeviceCtx.unbind()
        ctx.close()


def test_ctx_rejects_shared_devices(torch_cuda, sb):
    """One RCCL rank per GPU: no ordinal wrapping, no duplicates."""
    count = sb.device_count()
    with pytest.raises(sb.SblasError):
        sb.DeviceCtx(count + 1)
    with pytest.raises(sb.SblasError):
        sb.DeviceCtx(2, devices=[0, 0])


@pytest.mark.parametrize("algo,partition,exchange,parts", [(5, 0, 0, 1), (2, 1, 0, 1), (1, 0, 0, 1), (2, 1, 1, 1),
                                                           (5, 0, 0, 4), (1, 0, 0, 2)])
def test_cli_spmv_ctx(algo, partition, exchange, parts):
    """The C++ driver (tools/spmv_ctx.cpp): a C caller reaching the RCCL path
    with no Python; it checks device agreement, the host-merge reference API
    and the bound reference API."""
    exe = os.path.join(ROOT, "s-blas_amd", "bin", "spmv_ctx")
    r = subprocess.run([exe, "1", "2000000", str(algo), str(partition), "5", str(exchange), str(parts)],
                       capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ctx devices agree: PASS" in r.stdout
    assert "(RCCL): PASS" in r.stdout
    assert "ctx spmv: kernel" in r.stdout


@pytest.mark.parametrize("g", [2, 3, 5])
@pytest.mark.parametrize("algo", [1, 2, 5])
@pytest.mark.parametrize("partition,exchange", [(0, 0), (1, 0), (1, 1), (2, 0), (2, 1)])
def test_ctx_loopback_multi_rank(torch_cuda, sb, orc, monkeypatch, g, algo, partition, exchange):
    """g > 1 context ranks on the one GPU (SBLAS_CTX_LOOPBACK=1: no RCCL, the
    collectives are stream-ordered device copies): three chained steps, long
    rows split across ranks by the nnz partition, every rank's y compared with
    the oracle and with rank 0's bit for bit."""
    monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    rng = np.random.default_rng(100 * g + 10 * algo + partition)
    m, n = 6000, 9000
    rp, col, val = rand_csr(rng, m, n, 40, long_rows=[(2, 7000), (3000, 8000), (5999, 3000)])
    x = rng.standard_normal(n)
    y = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(g)
    ctx.upload(m, n, rp, col, val, algo, partition, exchange)
    ctx.set_x(x)
    ctx.set_y(y)
    for step in range(3):
        st = ctx.spmv_ex(alpha, beta, delay_us=100.0 if step == 1 else 0.0)
        assert st.shape == (3 + 3 * g,)
        want = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
        bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y)
        got = [ctx.get_y(d) for d in range(g)]
        assert np.all(np.abs(got[0] - want) <= bound), (step, np.max(np.abs(got[0] - want) - bound))
        for d in range(1, g):
            assert np.array_equal(got[0], got[d]), (step, d)
        y = got[0]
    assert sum(ctx.slice_info(d)[1] for d in range(g)) == int(rp[-1])
    ctx.close()


@pytest.mark.parametrize("g", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("parts", [2, 4])
@pytest.mark.parametrize("algo", [0, 1, 2, 5])
def test_ctx_overlap_parts(torch_cuda, sb, orc, monkeypatch, g, parts, algo):
    """The overlapped exchange (sblas_ctx_matrix_upload_parts; VERDICT r03
    item 2): each rank's cyclic chunks in `parts` groups, part p all-gathered
    and placed on the comm stream while part p + 1's kernel runs.  g > 1 in
    loopback (collectives = stream-ordered copies); g = 1 through a one-rank
    RCCL communicator.  Three chained steps, every rank's y within the fp64
    bound of the oracle and bit-identical to rank 0's."""
    if g > 1:
        monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    rng = np.random.default_rng(1000 * g + 10 * parts + algo)
    m, n = 7000, 9000
    rp, col, val = rand_csr(rng, m, n, 40, long_rows=[(2, 7000), (3000, 8000), (6999, 3000)])
    x = rng.standard_normal(n)
    y = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(g)
    ctx.upload_parts(m, n, rp, col, val, algo, parts)
    assert ctx.parts() == parts
    ctx.set_x(x)
    ctx.set_y(y)
    for step in range(3):
        st = ctx.spmv_ex(alpha, beta, delay_us=100.0 if step == 1 else 0.0)
        assert st.shape == (3 + 3 * g,) and st[2] >= st[0] > 0
        want = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
        bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y)
        got = [ctx.get_y(d) for d in range(g)]
        assert np.all(np.abs(got[0] - want) <= bound), (step, np.max(np.abs(got[0] - want) - bound))
        for d in range(1, g):
            assert np.array_equal(got[0], got[d]), (step, d)
        y = got[0]
    ctx.close()


def test_ctx_overlap_config2_full_size_g8(torch_cuda, sb, orc, monkeypatch):
    """Config 2 at full size (n = 2e6, 39.75M nnz) over 8 loopback ranks with
    the exchange overlapped in 2 and 4 parts: y within the bound, every rank
    bit-identical."""
    monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    n = 2_000_000
    rp = sb.gen_synth_rowptr(n)
    col, val = sb.gen_synth_rows(n, rp, 0, n)
    x = sb.gen_vector(n, 43)
    y0 = sb.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y0)
    for parts in (2, 4):
        ctx = sb.DeviceCtx(8)
        ctx.upload_parts(n, n, rp, col, val, 0, parts)
        assert ctx.parts() == parts
        ctx.set_x(x)
        ctx.set_y(y0)
        ctx.spmv_ex(alpha, beta)
        got = [ctx.get_y(d) for d in range(8)]
        assert np.all(np.abs(got[0] - want) <= bound), parts
        for d in range(1, 8):
            assert np.array_equal(got[0], got[d]), (parts, d)
        ctx.close()


@pytest.mark.parametrize("algo", [1, 2, 5])
@pytest.mark.parametrize("partition,exchange", [(0, 0), (1, 0), (1, 1)])
def test_ctx_noalias_exchange_rccl(torch_cuda, sb, orc, monkeypatch, algo, partition, exchange):
    """SBLAS_CTX_NOALIAS=1: a one-device context keeps
    its y exchange, so xchg_spmv's ncclAllGather (exchange 0) and the literal
    ncclAllReduce of the zero-padded y (exchange 1, BASELINE configs[2]) run
    on the 1-rank communicator, followed by the placement / re-prime kernels.
    Three chained steps against the oracle; the exchange takes device time."""
    monkeypatch.setenv("SBLAS_CTX_NOALIAS", "1")
    rng = np.random.default_rng(500 + 10 * algo + 3 * partition + exchange)
    m, n = 6000, 8000
    rp, col, val = rand_csr(rng, m, n, 40, long_rows=[(5, 7000), (5999, 2000)])
    x = rng.standard_normal(n)
    y = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(1)
    ctx.upload(m, n, rp, col, val, algo, partition, exchange)
    ctx.set_x(x)
    ctx.set_y(y)
    for step in range(3):
        st = ctx.spmv_ex(alpha, beta, delay_us=100.0 if step == 1 else 0.0)
        assert st[1] > 0.0, st  # the collective + placement ran after the kernel
        want = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
        got = ctx.get_y()
        assert np.all(np.abs(got - want) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y)), step
        y = got
    ctx.close()


def test_ctx_noalias_config3_full_size(torch_cuda, sb, orc, monkeypatch):
    """configs[2]'s dataflow at full size on one device with the y exchange
    kept: CSR5, nnz partition, ncclAllReduce of the 2e6-row zero-padded y."""
    monkeypatch.setenv("SBLAS_CTX_NOALIAS", "1")
    n = 2_000_000
    rp = sb.gen_synth_rowptr(n)
    col, val = sb.gen_synth_rows(n, rp, 0, n)
    x = sb.gen_vector(n, 43)
    y0 = sb.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(1)
    ctx.upload(n, n, rp, col, val, sb.CSR5, 1, sb.CTX_ALLREDUCE)
    ctx.set_x(x)
    ctx.set_y(y0)
    st = ctx.spmv_ex(alpha, beta, delay_us=200.0)
    assert st[1] > 0.0
    got = ctx.get_y()
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    assert np.all(np.abs(got - want) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y0))
    ctx.close()


@pytest.mark.parametrize("g", [1, 2])
def test_ctx_reupload_fewer_parts(torch_cuda, sb, orc, monkeypatch, g):
    """one context re-uploaded with 4 parts, then 2, then 3; the
    part events are rebuilt for each part count (each on its own device),
    and every step matches the oracle."""
    if g > 1:
        monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    rng = np.random.default_rng(77 + g)
    m, n = 7000, 9000
    rp, col, val = rand_csr(rng, m, n, 30)
    x = rng.standard_normal(n)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(g)
    for parts in (4, 2, 3):
        ctx.upload_parts(m, n, rp, col, val, 0, parts)
        assert ctx.parts() == parts
        y = rng.standard_normal(m)
        ctx.set_x(x)
        ctx.set_y(y)
        ctx.spmv_ex(alpha, beta)
        want = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
        got = [ctx.get_y(d) for d in range(g)]
        assert np.all(np.abs(got[0] - want) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y)), parts
        for d in range(1, g):
            assert np.array_equal(got[0], got[d])
    ctx.close()


def test_ctx_loopback_cost_partition_config2_g8(torch_cuda, sb, orc, monkeypatch):
    """configs[2]'s dataflow at full size over 8 loopback ranks with the
    cost-weighted whole-row split (partition 2) and the all-reduce of the
    zero-padded y: every rank's y within the bound and bit-identical; the
    light ranks hold fewer entries than the heavy ones."""
    monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    n = 2_000_000
    rp = sb.gen_synth_rowptr(n)
    col, val = sb.gen_synth_rows(n, rp, 0, n)
    x = sb.gen_vector(n, 43)
    y0 = sb.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    ctx = sb.DeviceCtx(8)
    ctx.upload(n, n, rp, col, val, sb.CSR5, 2, sb.CTX_ALLREDUCE)
    nnz = [ctx.slice_info(d)[1] for d in range(8)]
    assert sum(nnz) == int(rp[-1]) and nnz[-1] < nnz[0]
    ctx.set_x(x)
    ctx.set_y(y0)
    ctx.spmv_ex(alpha, beta)
    want = orc.csr_spmv_omp(rp, col, val, x, alpha, beta, y0.copy())
    got = [ctx.get_y(d) for d in range(8)]
    assert np.all(np.abs(got[0] - want) <= orc.spmv_bound(rp, col, val, x, alpha, beta, y0))
    for d in range(1, 8):
        assert np.array_equal(got[0], got[d])
    ctx.close()


def test_ctx_two_contexts_peer_refcount(torch_cuda, sb, orc, monkeypatch):
    """peer links are reference-counted per process.  Two loopback
    all-reduce contexts over the same device pair (distinct GPUs where the
    box has two, else both ranks on one GPU, which needs no link), the first
    destroyed, the second still runs and matches the oracle; a trsv_mgpu
    handle on the same pair holds its own reference."""
    monkeypatch.setenv("SBLAS_CTX_LOOPBACK", "1")
    ndev = torch_cuda.cuda.device_count()
    rng = np.random.default_rng(7)
    m, n = 4000, 4000
    rp, col, val = rand_csr(rng, m, n, 30)
    x = rng.standard_normal(n)
    y = rng.standard_normal(m)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv(rp, col, val, x, alpha, beta, y)
    bound = orc.spmv_bound(rp, col, val, x, alpha, beta, y)
    link = 1 if ndev >= 2 else 0
    ctxs = []
    for _ in range(2):
        c = sb.DeviceCtx(2)
        c.upload(m, n, rp, col, val, 2, 1, 1)  # CSR5, nnz split, all-reduce
        c.set_x(x)
        c.set_y(y)
        ctxs.append(c)
    assert sb.peer_refs(0, 1) == 2 * link
    nr, ords = ctxs[0].comm_info()
    assert nr == 0 and ords == [d % ndev for d in range(2)]  # loopback: no communicator
    ctxs[0].close()
    assert sb.peer_refs(0, 1) == link
    ctxs[1].spmv(alpha, beta)
    assert np.all(np.abs(ctxs[1].get_y(0) - want) <= bound)
    ctxs[1].close()
    assert sb.peer_refs(0, 1) == 0


def test_ctx_comm_info_rccl(torch_cuda, sb):
    """A real (one-rank) RCCL communicator reports its rank count and device
    through sblas_ctx_comm_info (the `topology` of every bench line)."""
    ctx = sb.DeviceCtx(1)
    assert ctx.comm_info() == (1, [0])
    ctx.close()
