"""The C-ABI library loads without a GPU and exports every symbol that
include/*.h declares (extern "C" names and the reference's C++ names)."""
import os
import re
import subprocess

from conftest import ROOT

LIB = os.path.join(ROOT, "s-blas_amd", "libsblas.so")


def declared(header, pattern):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(pattern, text)))


def exported(demangle):
    out = subprocess.run(["nm", "-D", "--defined-only"] + (["-C"] if demangle else []) + [LIB],
                         check=True, capture_output=True, text=True).stdout
    return {line.split(" ", 2)[2] for line in out.splitlines() if " T " in line}


def test_c_abi_symbols(sb):
    names = declared("sblas.h", r"\b(sblas_\w+)\s*\(")
    assert len(names) >= 30
    syms = exported(False)
    missing = [n for n in names if n not in syms]
    assert not missing, missing
    for n in names:  # resolvable through the loader too
        getattr(sb.lib, n)


def test_reference_cxx_names():
    names = declared("sblas_refapi.h", r"\b(\w+)\s*\([^;]*\);")
    assert {"spMV_mgpu_baseline", "spMV_mgpu_v1", "spMV_mgpu_v2", "cusparse_mgpu_csrmm",
            "cusparse_mgpu_csrmm_omp", "sptrsv_syncfree_cuda", "get_row_from_index",
            "get_time", "get_gpu_availble_mem"} <= set(names)
    syms = {s.split("(")[0] for s in exported(True)}
    assert not [n for n in names if n not in syms]


def test_no_gpu_host_calls(sb):
    import numpy as np
    assert sb.lib.sblas_version() == 100
    assert sb.lib.sblas_status_string(2) == b"HIP runtime error"
    rp = np.array([0, 1, 3], np.int64)
    assert sb.lib.sblas_get_row_from_index(2, sb.ptr(rp), 2) == 1
