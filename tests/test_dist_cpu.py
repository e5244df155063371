"""World-size-2 gloo run of the multi-rank SpMV protocol (CPU): each rank
takes its nnz-balanced slice from sblas_dist.make_plan, computes its partial
with the oracle (checker), the slices travel through a real collective and
are merged with the {row0, nrows, cont} metadata sblas_assemble_slices
consumes on the GPU.  The merged y must equal the single-process oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def merge(gathered, meta, stride, m):
    """numpy restatement of k_assemble_copy + k_assemble_carry (checker)."""
    y = np.full(m, np.nan)
    g = len(meta) // 3
    for r in range(g):
        row0, nrows, cont = meta[3 * r:3 * r + 3]
        for k in range(nrows):
            if not (k == 0 and cont):
                y[row0 + k] = gathered[r * stride + k]
    for r in range(g):
        row0, nrows, cont = meta[3 * r:3 * r + 3]
        if cont and nrows > 0:
            y[row0] += gathered[r * stride]
    return y


def _worker(rank, world, port, n, result_q, row_cost=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    import sblas_dist
    rp, col, val = orc.gen_synth(n, heavy=40, light=3)
    x = orc.gen_vector(n, 43)
    y0 = orc.gen_vector(n, 44)
    a, b = orc.alpha_beta()
    plan = sblas_dist.make_plan(rp, n, world, row_cost=row_cost)
    r0, r1, i0, i1, cont = plan.local(rank)
    # local slice exactly as the GPU path uploads it (dspmv_mgpu_v1.cu:125-133)
    dm = r1 - r0
    lrp = np.zeros(dm + 1, np.int64)
    if dm:
        lrp[1:dm] = rp[r0 + 1:r1] - i0
        lrp[dm] = i1 - i0
    yl = y0[r0:r1].copy()
    if cont and dm:
        yl[0] = 0.0
    part = orc.csr_spmv(lrp, col[i0:i1], val[i0:i1], x, a, b, yl)
    if row_cost is not None:
        # cost-weighted whole rows + configs[2]'s exchange: the rank writes
        # its rows into a zero-padded full y, one all-reduce sums them
        yfull = torch.zeros(plan.m, dtype=torch.float64)
        yfull[r0:r1] = torch.from_numpy(part)
        dist.all_reduce(yfull)
        y = yfull.numpy()
    else:
        buf = torch.zeros(plan.stride, dtype=torch.float64)
        buf[:dm] = torch.from_numpy(part)
        out = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        y = merge(torch.cat(out).numpy(), plan.meta(), plan.stride, plan.m)
    want = orc.csr_spmv(rp, col, val, x, a, b, y0)
    ok = bool(np.all(np.abs(y - want) <= orc.spmv_bound(rp, col, val, x, a, b, y0)))
    result_q.put((rank, ok, int(cont)))
    dist.destroy_process_group()


@pytest.mark.parametrize("row_cost", [None, 6.0], ids=["nnz_split_allgather", "cost_rows_allreduce"])
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_protocol(world, row_cost):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 997, q, row_cost)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    if row_cost is None:
        assert any(c for _, _, c in res)  # the split actually crossed a row
    else:
        assert not any(c for _, _, c in res)  # whole rows: no carries


def assemble_cyclic(gathered, world, stride, R, m):
    """numpy restatement of k_assemble_cyclic (checker)."""
    r = np.arange(m)
    j = r // R
    return gathered[(j % world) * stride + (j // world) * R + (r - j * R)]


def _cyclic_worker(rank, world, port, n, result_q, halves=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    import sblas_dist
    rp, col, val = orc.gen_synth(n, heavy=40, light=3)
    x = orc.gen_vector(n, 43)
    y0 = orc.gen_vector(n, 44)
    a, b = orc.alpha_beta()
    plan = sblas_dist.make_cyclic_plan(rp, n, world)
    lrp, lcol, lval = sblas_dist.cyclic_local_csr(rp, plan, rank,
                                                  lambda r0, r1: (col[rp[r0]:rp[r1]],
                                                                  val[rp[r0]:rp[r1]]))
    yl = np.concatenate([y0[r0:r1] for r0, r1 in plan.chunks(rank)] or [np.zeros(0)])
    part = orc.csr_spmv(lrp, lcol, lval, x, a, b, yl)
    buf = torch.zeros(plan.stride, dtype=torch.float64)
    buf[:len(part)] = torch.from_numpy(part)
    if halves:
        # DistSpMVCyclic(overlap=True): the slice's first hA chunks and the
        # rest are all-gathered separately and each half placed on its own
        hA, sA, sB, rows_a = sblas_dist.overlap_halves(plan)
        outA = [torch.zeros(sA, dtype=torch.float64) for _ in range(world)]
        outB = [torch.zeros(sB, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(outA, buf[:sA].contiguous())
        dist.all_gather(outB, buf[sA:sA + sB].contiguous())
        y = np.concatenate([
            assemble_cyclic(torch.cat(outA).numpy(), world, sA, plan.chunk_rows, rows_a),
            assemble_cyclic(torch.cat(outB).numpy(), world, sB, plan.chunk_rows, plan.m - rows_a)])
    else:
        out = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        y = assemble_cyclic(torch.cat(out).numpy(), world, plan.stride, plan.chunk_rows, plan.m)
    want = orc.csr_spmv(rp, col, val, x, a, b, y0)
    ok = bool(np.all(np.abs(y - want) <= orc.spmv_bound(rp, col, val, x, a, b, y0)))
    # every rank holds the same number of rows (up to the last chunk) and
    # the heavy first eighth of the rows is spread over the ranks
    rows = [plan.local_rows(d) for d in range(world)]
    nnzs = [int(sum(rp[r1] - rp[r0] for r0, r1 in plan.chunks(d))) for d in range(world)]
    balanced = max(rows) - min(rows) <= plan.chunk_rows and max(nnzs) <= 1.5 * (plan.nnz / world)
    result_q.put((rank, ok and balanced and len(part) == plan.local_rows(rank)))
    dist.destroy_process_group()


@pytest.mark.parametrize("halves", [False, True], ids=["one_gather", "overlap_halves"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_cyclic_protocol(world, halves):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cyclic_worker, args=(r, world, port, 1003, q, halves))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def _spmm_worker(rank, world, port, result_q):
    """SpMM row-block protocol: whole-row blocks by nnz, B
    replicated, each rank's C slice (ncols x stride, ld = stride) all-gathered
    and placed back by the block boundaries -- as sblas_dist.DistSpMM does on
    the GPU.  The rank-local product is the oracle (checker)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    import sblas_dist
    rng = np.random.default_rng(3)
    m, k, ncols = 301, 450, 7
    lens = rng.integers(0, 40, m)
    lens[5] = 400  # one heavy row
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(k, L, replace=False)) for L in lens]).astype(np.int32)
    val = rng.standard_normal(int(rp[-1]))
    B = rng.standard_normal((k, ncols))
    C0 = rng.standard_normal((m, ncols))
    rb = sblas_dist.row_blocks_by_nnz(rp, world)
    stride = int(max(1, np.diff(rb).max()))
    r0, r1 = int(rb[rank]), int(rb[rank + 1])
    lrp = rp[r0:r1 + 1] - rp[r0]
    part = orc.spmm(r1 - r0, ncols, k, -0.7, lrp, col[rp[r0]:rp[r1]], val[rp[r0]:rp[r1]], B, 0.8,
                    C0[r0:r1]) if r1 > r0 else np.zeros((0, ncols))
    buf = torch.zeros((ncols, stride), dtype=torch.float64)
    buf[:, : r1 - r0] = torch.from_numpy(np.ascontiguousarray(part.T))
    out = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    C = np.zeros((ncols, m))
    for d in range(world):
        a, b = int(rb[d]), int(rb[d + 1])
        C[:, a:b] = out[d].numpy()[:, : b - a]
    want = orc.spmm(m, ncols, k, -0.7, rp, col, val, B, 0.8, C0).T
    ok = bool(np.allclose(C, want, rtol=1e-12, atol=1e-12))
    balanced = bool(np.all(np.diff(rb) >= 0) and rb[0] == 0 and rb[-1] == m)
    result_q.put((rank, ok and balanced))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_spmm_protocol(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spmm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def test_spmm_grid_shape():
    """DistSpMM split "grid": the most column groups that keep a multiple of
    16 C columns per rank, the rest as row blocks."""
    import sblas_dist
    g = sblas_dist.spmm_grid_shape
    assert [g(w, 64) for w in (1, 2, 3, 4, 6, 8, 16)] == [(1, 1), (1, 2), (3, 1), (1, 4), (3, 2), (2, 4), (4, 4)]
    assert g(8, 100) == (8, 1) and g(8, 128) == (1, 8) and g(2, 16) == (2, 1)


def _spmm_grid_worker(rank, world, port, result_q):
    """SpMM grid protocol: rank d owns the C block (row block d // Cg by nnz)
    x (column group d % Cg), computed from its rows of A and its columns of
    B, all-gathered as equal-shape (wc x stride) buffers and placed -- as
    sblas_dist.DistSpMM(split="grid") does on the GPU.  The rank-local
    product is the oracle (checker)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    import sblas_dist
    rng = np.random.default_rng(4)
    m, k = 257, 390
    ncols = 64 if world == 2 else 32  # (1, 2) at 2 ranks; (2, 2) at 4: row blocks AND column groups
    lens = rng.integers(0, 30, m)
    lens[7] = 300
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(k, L, replace=False)) for L in lens]).astype(np.int32)
    val = rng.standard_normal(int(rp[-1]))
    B = rng.standard_normal((k, ncols))
    C0 = rng.standard_normal((m, ncols))
    R, Cg = sblas_dist.spmm_grid_shape(world, ncols)
    rb = sblas_dist.row_blocks_by_nnz(rp, R)
    cb = [c * ncols // Cg for c in range(Cg + 1)]
    wc, stride = ncols // Cg, int(max(1, np.diff(rb).max()))
    blk = lambda d: (int(rb[d // Cg]), int(rb[d // Cg + 1]), cb[d % Cg], cb[d % Cg + 1])  # noqa: E731
    r0, r1, c0, c1 = blk(rank)
    lrp = rp[r0:r1 + 1] - rp[r0]
    part = orc.spmm(r1 - r0, wc, k, -0.7, lrp, col[rp[r0]:rp[r1]], val[rp[r0]:rp[r1]],
                    np.ascontiguousarray(B[:, c0:c1]), 0.8,
                    np.ascontiguousarray(C0[r0:r1, c0:c1])) if r1 > r0 else np.zeros((0, wc))
    buf = torch.zeros((wc, stride), dtype=torch.float64)
    buf[:, : r1 - r0] = torch.from_numpy(np.ascontiguousarray(part.T))
    out = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    C = np.zeros((ncols, m))
    for d in range(world):
        a, b, ca, cb_ = blk(d)
        C[ca:cb_, a:b] = out[d].numpy()[:, : b - a]
    want = orc.spmm(m, ncols, k, -0.7, rp, col, val, B, 0.8, C0).T
    result_q.put((rank, bool(np.allclose(C, want, rtol=1e-12, atol=1e-12))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_spmm_grid_protocol(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spmm_grid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)
