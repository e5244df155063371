"""bench.py's driver routing (no GPU): `python bench.py --gpus N` must measure
N GPUs or exit non-zero -- one process per GPU under a launcher (WORLD_SIZE
set), else one process driving N GPUs through the C-ABI context (sblas_ctx),
mirroring the reference's single host call over every GPU
(spmv/test/dspmv_test.cu:355-383 -> spmv/src/dspmv_mgpu_v1.cu:16-280)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,ndev,req,want", [
    (1, {}, 1, "auto", "single"),
    (1, {}, 8, "ctx", "ctx"),
    (2, {}, 8, "auto", "ctx"),
    (8, {}, 8, "auto", "ctx"),
    (8, {"WORLD_SIZE": "8"}, 8, "auto", "torch"),
    (1, {"WORLD_SIZE": "1"}, 1, "auto", "torch"),
    (1, {"WORLD_SIZE": "1"}, 1, "ctx", "ctx"),
])
def test_choose_driver(gpus, env, ndev, req, want):
    assert bench.choose_driver(gpus, env, ndev, req) == want


@pytest.mark.parametrize("gpus,env,ndev,req", [
    (9, {}, 8, "auto"),                   # more GPUs than visible
    (2, {}, 1, "auto"),
    (1, {}, 0, "auto"),
    (0, {}, 8, "auto"),
    (4, {"WORLD_SIZE": "2"}, 8, "auto"),  # launcher disagrees with --gpus
    (8, {"WORLD_SIZE": "8"}, 8, "ctx"),   # ctx is one process: no launcher
    (4, {}, 8, "torch"),                  # torch ranks need a launcher
])
def test_choose_driver_refuses(gpus, env, ndev, req):
    with pytest.raises(ValueError):
        bench.choose_driver(gpus, env, ndev, req)


def test_choose_driver_loopback():
    """the ctx rehearsal wraps N ranks onto the visible GPUs (never measures)"""
    assert bench.choose_driver(8, {}, 1, "auto", loopback=True) == "ctx"
    with pytest.raises(ValueError):
        bench.choose_driver(8, {}, 0, "auto", loopback=True)


def test_bench_exits_nonzero_when_gpus_exceed_devices():
    """--gpus above the visible device count exits 2 with a message before
    any data is generated (here: no GPU at all, or one on the box)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "refusing to measure fewer GPUs" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.parametrize("matrix", ["stencil7", "stencil27", "rmat"])
def test_workload_rows_match_generators(matrix):
    """bench.py's Workload hands out the generator's rows for any [a, b) (the
    torch path slices them per rank)."""
    sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))
    import argparse
    import sblas
    args = argparse.Namespace(matrix=matrix, grid=6, scale=10, nrows=0, heavy=96, light=9, cols="random")
    W = bench.Workload(args, sblas)
    if matrix == "rmat":
        rp, col, val = sblas.gen_rmat(10, 16, seed=50)
    else:
        rp, col, val = sblas.gen_stencil3d(6, 6, 6, int(matrix[7:]), seed=49)
    assert W.n == len(rp) - 1 and W.nnz == rp[-1] and not W.default
    for a, b in ((0, W.n), (3, 17), (W.n - 5, W.n)):
        c, v = W.rows(a, b)
        assert (c == col[rp[a]:rp[b]]).all() and (v == val[rp[a]:rp[b]]).all()
    assert matrix[:4] in W.describe("auto").lower() or "r-mat" in W.describe("auto").lower()


def test_config3_object_keys():
    """Every bench line carries BASELINE configs[2] under `config3`
    (kernel-only, exchange-only and total, max over devices):
    the object both drivers attach (bench.config3_object), at N > 1 and 1."""
    for N in (8, 2, 1):
        c3 = bench.config3_object(N, 0.05, 0.03, 0.08, 39_750_000, [6.7e7] * N, [0.05] * N, True, "cold")
        for k in ("kernel_ms_max", "exchange_ms_max", "step_ms", "gflops", "roofline", "check",
                  "kernel_ms_per_device", "algo", "partition", "exchange"):
            assert k in c3, k
        assert c3["algo"] == "csr5" and c3["exchange"] == ("allreduce" if N > 1 else "none (one device)")
        assert abs(c3["gflops"] - 2 * 39_750_000 / 0.08e-3 / 1e9) < 1e-3
        assert 0 < c3["roofline"]["frac"] < 1


def test_config3_is_on_by_default():
    """Both drivers add the configs[2] leg unless --no-config3 is given."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('out["config3"] = config3') == 2
    assert src.count("if not args.no_config3:") == 2


def test_config4_config5_object_keys():
    """Every bench line carries BASELINE configs[3] (SpMM) and configs[4]
    (SpTRSV) under `config4` / `config5`: the objects
    both drivers attach, built from per-rank stats rows."""
    per = [[0.36, 0.0, 0.36, 699e6, 11_279_748]]
    c4 = bench.config4_object(1, per, 1.5, 0.7, {"pass": True, "entries": 4284 * 64}, None)
    for k in ("kernel_ms_max", "exchange_ms_max", "step_ms", "gflops", "kernel_only_gflops", "roofline",
              "algorithmic_bytes_per_rank", "kernel_ms_per_rank", "nnz_per_rank", "check", "timing", "what"):
        assert k in c4, k
    assert abs(c4["gflops"] - 2 * 11_279_748 * 64 / 0.36e-3 / 1e9) < 1e-3
    assert abs(c4["roofline"]["achieved"] - 699e6 / 0.36e-3 / 1e9) < 0.1
    per8 = [[0.05 + 0.001 * r, 0.02, 0.07 + 0.001 * r, 90e6, 11_279_748 // 8] for r in range(8)]
    c48 = bench.config4_object(8, per8, 1.0, 0.7, None, None)
    assert c48["n_gpus"] == 8 and c48["kernel_ms_max"] == 0.057 and len(c48["kernel_ms_per_rank"]) == 8
    c5 = bench.config5_single(33_350_000, 985, 1, 2.45, True, 1.0, 0.5)
    for k in ("ms", "gflops", "algorithmic_bytes", "roofline", "levels", "check_exact_vs_xref", "us_per_level",
              "executor", "timing"):
        assert k in c5, k
    assert c5["algorithmic_bytes"] == 12 * 33_350_000 + 4 * (5_558_326 + 1) + 16 * 5_558_326
    b4 = bench.config5_blocks(33_350_000, 1, 2.6, True, 2.0)
    assert b4["blocks"] == 4 and b4["blocks_per_gpu"] == 4 and b4["check_exact_vs_xref"]


def test_config4_config5_on_by_default():
    """Both drivers add the configs[3] / configs[4] legs unless switched off."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('out["config4"] = config4') == 2 and src.count('out["config5"] = config5') == 2
    assert src.count("if not args.no_config4:") == 2 and src.count("if not args.no_config5:") == 2


def test_config4_grid_object_and_call():
    """At N > 1 the SpMM leg reports the 2-D grid split beside the row split
    (`config4.grid`), from the same per-rank rows as config4_object."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'config4["grid"] = config4_leg(' in src and 'split="grid"' in src
    per = [[0.08, 0.01, 0.09, 2.0e8, 5_639_874], [0.07, 0.01, 0.08, 2.0e8, 5_639_874]]
    g = bench.config4_grid_object(per, (1, 2), {"pass": True, "entries": 4284 * 64})
    assert g["row_blocks"] == 1 and g["column_groups"] == 2
    assert g["kernel_ms_max"] == 0.08 and g["step_ms"] == 0.09 and g["check"]["pass"]
    assert g["gflops"] > 0 and len(g["kernel_ms_per_rank"]) == 2


def test_structured_leg_on_by_default():
    """Both drivers add the SuiteSparse-class stand-ins (north star's >= 60%
    target) at N = 1 unless --no-structured is given; three matrices."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('out["structured"] = structured') == 2
    assert src.count("not args.no_structured") == 2
    assert [k for k, _, _ in bench.STRUCTURED] == ["stencil27", "stencil7", "rmat"]


def test_traffic_requires_matching_library_hash(tmp_path, monkeypatch):
    """roofline.traffic comes from a committed PMC summary only while its
    lib_sha256 stamp equals the loaded libsblas.so's hash."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    (prof / "pmc_x.json").write_text(json.dumps({"hbm_bytes_per_launch": 7.0e8, "lib_sha256": bench.lib_sha256()}))
    assert bench._stamped_traffic("x") == 7.0e8
    (prof / "pmc_y.json").write_text(json.dumps({"hbm_bytes_per_launch": 7.0e8, "lib_sha256": "0" * 64}))
    assert bench._stamped_traffic("y") is None and "not reported" in bench.TRAFFIC_NOTES["y"]
    (prof / "pmc_z.json").write_text(json.dumps({"hbm_bytes_per_launch": 7.0e8}))
    assert bench._stamped_traffic("z") is None
    assert bench._stamped_traffic("absent") is None


def _child(leg, budget):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_PROC_BIND="close", OMP_PLACES="cores")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-baseline-only", "--cpu-leg", leg,
                        "--cpu-budget", str(budget)], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_cpu_baseline_sptrsv_child_is_the_reference_serialref():
    """configs[4]'s CPU baseline: the reference's own
    serial analyser + executor (sptrsv_syncfree_serialref.h, compiled in place
    into oracle/_ref) on the full known-answer system, one core, x exact."""
    b = _child("sptrsv", 1)
    for k in ("value", "unit", "cores", "kind", "sample", "executor_ms", "analyser_ms", "check_exact_vs_xref"):
        assert k in b, k
    assert b["cores"] == 1 and b["check_exact_vs_xref"] is True and b["value"] > 0
    ref_built = os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsblas_ref.so"))
    assert b["kind"] == ("reference" if ref_built else "port")


def test_cpu_baseline_spmm_child_sweeps_threads():
    """configs[3]'s CPU baseline: orc_spmm_omp over the full rail4284-shaped
    product, thread count swept like the SpMV baseline."""
    b = _child("spmm", 1)
    for k in ("value", "unit", "cores", "kind", "sample", "thread_sweep_gflops", "ms_per_call"):
        assert k in b, k
    assert b["kind"] == "port" and b["value"] > 0 and str(b["cores"]) in b["thread_sweep_gflops"]


def test_every_leg_carries_cpu_baseline_and_check(monkeypatch):
    """attach_cpu_baselines puts a CPU baseline on the headline AND on the
    config4 / config5 legs; the headline's post-timing oracle check is on by
    default in both drivers (`check_vs_oracle`)."""
    seen = []
    monkeypatch.setattr(bench, "cpu_baseline", lambda args, leg="spmv": seen.append(leg) or {"leg": leg})
    out = {"config4": {}, "config5": {}}
    bench.attach_cpu_baselines(out, None)
    assert out["cpu_baseline"] == {"leg": "spmv"}
    assert out["config4"]["cpu_baseline"] == {"leg": "spmm"}
    assert out["config5"]["cpu_baseline"] == {"leg": "sptrsv"}
    out = {}
    bench.attach_cpu_baselines(out, None)
    assert "config4" not in out and "config5" not in out
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "args.check = not args.no_check" in src
    assert src.count('out["check_vs_oracle"] = check') == 2
    assert src.count("        attach_cpu_baselines(out, args)") == 2


def test_topology_object_keys():
    """Every line says what it ran on: communicator rank
    count, per-rank device ordinal and PCI address, peer-access matrix."""
    t = bench.topology_object("torch (one process per GPU)", "nccl", 8, list(range(8)),
                              [f"0000:{b:02x}:00" for b in range(8)], [[1] * 8 for _ in range(8)])
    for k in ("driver", "backend", "comm_ranks", "device_ordinals", "pci_bus", "visible_devices",
              "peer_access", "all_pairs_peer"):
        assert k in t, k
    assert t["comm_ranks"] == 8 and t["all_pairs_peer"] and t["visible_devices"] == 8
    t2 = bench.topology_object("ctx", "loopback (no communicator)", 0, [0, 0], [None, None], [[1]], note="x")
    assert t2["comm_ranks"] == 0 and t2["note"] == "x"
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('out["topology"] = ') == 2
    assert 'out["block_devices"] = ' in src
