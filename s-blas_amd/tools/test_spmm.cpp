// test_spmm -- CLI clone of spmm/test/dspmm_baseline_test.cu:
//
//   test_spmm <matrix.mtx> <ncols of B> <ngpu> <repeat (unused)>
//
// Loader: banner + "%d %d %lg" entries in file order (no symmetric
// expansion; sblas_mm_read mode 3), then sorted by (row, col) with
// sblas_coo_sortbyrow as sortbyrow does (:41-55).  B and C
// are rand()/RAND_MAX (unseeded), alpha = -0.7, beta = 0.8 (:518-519).  The
// single-device run is the check target (the reference used single-GPU
// cuSPARSE); the multi-device run is compared with abs 0.001 (:544-549).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <vector>

#include "../../include/sblas.h"
#include "../../include/sblas_refapi.h"

using namespace std;

int main(int argc, char *argv[])
{
    if (argc < 5) {
        std::cout << "Usage: ./spmm [input sparse matrix A file] [output row number] [number of "
                     "GPU(s)] [number of test(s)]\n";
        return -1;
    }
    char *filename_A = argv[1];
    const int n = atoi(argv[2]);
    const int ngpu = atoi(argv[3]);
    int deviceCount = 0;
    sblas_device_count(&deviceCount);
    if (deviceCount <= 0) {
        cout << "Error: Not enough number of GPUs. Only " << deviceCount << "available." << endl;
        return -1;
    }
    if (ngpu <= 0) {
        cout << "Error: Number of GPU(s) needs to be greater than 0." << endl;
        return -1;
    }
    cout << "Using " << ngpu << " GPU(s)." << endl;

    int m = 0, k = 0;
    long long nnz64 = 0;
    // mode 3: the test's own "%d %d %lg" loader (no symmetric expansion)
    if (sblas_mm_read(filename_A, 3, &m, &k, &nnz64, nullptr, nullptr, nullptr) != SBLAS_OK) {
        cout << "Could not open matrix A file.\n";
        return -1;
    }
    vector<long long> rp64((size_t)m + 1);
    vector<int> col((size_t)max(nnz64, 1LL)), row((size_t)max(nnz64, 1LL));
    vector<double> val((size_t)max(nnz64, 1LL));
    sblas_mm_read(filename_A, 3, &m, &k, &nnz64, rp64.data(), col.data(), val.data());
    const int nnz = (int)nnz64;
    cout << "Matrix A -- #row: " << m << " #col: " << k << " nnz: " << nnz << endl;
    cout << "Loading input matrix A from " << filename_A << "\n";
    // sortbyrow + COO -> CSR (dspmm_baseline_test.cu:41-55, 461-493)
    for (int r = 0; r < m; ++r)
        for (long long e = rp64[(size_t)r]; e < rp64[(size_t)r + 1]; ++e) row[(size_t)e] = r;
    vector<int> csrRowPtr((size_t)m + 1);
    if (sblas_coo_sortbyrow(m, nnz64, row.data(), col.data(), val.data(), csrRowPtr.data()) != SBLAS_OK) {
        cout << "sortbyrow failed: " << sblas_last_error() << "\n";
        return -1;
    }
    cout << "Matrix B -- #row: " << k << " #col: " << n << " (dense)" << endl;
    cout << "Start generating data for Matrix B\n" << std::flush;
    vector<double> B((size_t)k * n), C((size_t)m * n), C_mgpu;
    for (auto &v : B) v = (double)rand() / (RAND_MAX);
    for (auto &v : C) v = (double)rand() / (RAND_MAX);
    C_mgpu = C;
    double alpha = -0.7, beta = 0.8;

    cout << "Start computing SpMM on a single GPU (sblas).\n" << std::flush;
    double t0 = get_time();
    int rc = cusparse_mgpu_csrmm(m, n, k, &alpha, nnz, csrRowPtr.data(), col.data(), val.data(),
                                 &beta, B.data(), C.data(), 1);
    const double single = get_time() - t0;
    if (rc != 0) {
        cout << "single gpu csrmm failed: " << sblas_last_error() << "\n";
        return -1;
    }
    cout << "sblas single gpu processing time(s): " << single << "\n";
    cout << "Matrix C -- #row: " << m << " #col: " << n << " (dense)" << endl;
    t0 = get_time();
    rc = cusparse_mgpu_csrmm_omp(m, n, k, &alpha, nnz, csrRowPtr.data(), col.data(), val.data(),
                                 &beta, B.data(), C_mgpu.data(), ngpu);
    const double mgpu = get_time() - t0;
    cout << "SPMM: " << ngpu << " GPUs processing time(s): " << mgpu << "\n";
    bool ok = rc == 0;
    for (size_t i = 0; i < C.size() && ok; ++i) ok = std::fabs(C_mgpu[i] - C[i]) < 0.001;
    cout << "mgpu check: " << (ok ? "PASS" : "FAILED") << endl;
    return ok ? 0 : 1;
}
