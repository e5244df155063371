// test_sptrans -- CLI clone of sptrans/sptrans_v1/src/main.cu:
//
//   test_sptrans -n <ngpu> -csr -mtx <A.mtx>
//
// Loads A (mmio_data semantics), builds the reference CSC on the host with a
// stable counting transpose (tranpose.h matrix_transposition), checks the
// CPU round trip, then runs cuda_sptrans (one GPU) and kernal_sptrans
// (ngpu GPUs) and prints the reference's lines.  "-csc" is accepted and,
// as in the reference, only echoed.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/sblas.h"
#include "../../include/sblas_refapi.h"

using namespace std;

static void host_transpose(int m, int n, int nnz, const int *rp, const int *ci, const double *v,
                           vector<int> &cp, vector<int> &ri, vector<double> &cv)
{
    cp.assign((size_t)n + 1, 0);
    ri.assign((size_t)nnz, 0);
    cv.assign((size_t)nnz, 0.0);
    for (int e = 0; e < nnz; ++e) cp[(size_t)ci[e] + 1]++;
    for (int c = 0; c < n; ++c) cp[(size_t)c + 1] += cp[(size_t)c];
    vector<int> next(cp.begin(), cp.end() - 1);
    for (int r = 0; r < m; ++r)
        for (int e = rp[r]; e < rp[r + 1]; ++e) {
            const int o = next[(size_t)ci[e]]++;
            ri[(size_t)o] = r;
            cv[(size_t)o] = v[e];
        }
}

int main(int argc, char **argv)
{
    int ngpu = 0;
    const char *fmt = "-csr", *filename = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) ngpu = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-csr") || !strcmp(argv[i], "-csc")) fmt = argv[i];
        else if (!strcmp(argv[i], "-mtx") && i + 1 < argc) filename = argv[++i];
    }
    if (!filename) {
        printf("Usage: ./test_sptrans -n [number of GPU(s)] -csr -mtx [input sparse matrix A file]\n");
        return -1;
    }
    int count = 0;
    sblas_device_count(&count);
    if (ngpu <= 0) {
        printf("Error: Number of GPU(s) needs to be greater than 0.\n");
        return -1;
    }
    if (count < ngpu) printf("Note: %i GPU(s) visible; blocks wrap onto them.\n", count);
    printf("Using %i GPU(s).\n", ngpu);
    printf("input data format = %s\n", fmt);
    printf("-------------- %s --------------\n", filename);
    int m = 0, n = 0;
    long long nnz64 = 0;
    if (sblas_mm_read(filename, 0, &m, &n, &nnz64, nullptr, nullptr, nullptr) != SBLAS_OK) {
        printf("%s\n", sblas_last_error());
        return -1;
    }
    vector<long long> rp64((size_t)m + 1);
    vector<int> col((size_t)max(nnz64, 1LL));
    vector<double> val((size_t)max(nnz64, 1LL));
    sblas_mm_read(filename, 0, &m, &n, &nnz64, rp64.data(), col.data(), val.data());
    const int nnz = (int)nnz64;
    vector<int> rp(rp64.begin(), rp64.end());
    printf("input matrix A: ( %i, %i ) nnz = %i\n", m, n, nnz);
    vector<int> cpA, riA, cpB, riB;
    vector<double> cvA, cvB;
    host_transpose(m, n, nnz, rp.data(), col.data(), val.data(), cpA, riA, cvA);
    host_transpose(n, m, nnz, cpA.data(), riA.data(), cvA.data(), cpB, riB, cvB);  // back to CSR
    double ref = 0.0, res = 0.0;
    for (int i = 0; i < nnz; ++i) {
        ref += fabs(val[(size_t)i]);
        res += fabs(cvB[(size_t)i] - val[(size_t)i]);
    }
    res = ref == 0 ? res : res / ref;
    printf("matrix transposition in cpu: %s |x-xref|/|xref| = %8.2e\n",
           res < 1e-4 ? "passed!" : "_NOT_ passed!", res);
    vector<int> cp((size_t)n + 1), ri((size_t)max(nnz, 1));
    vector<double> cv((size_t)max(nnz, 1));
    printf("---------------------------------------------------------------------------------------------\n");
    int rc = cuda_sptrans(m, n, nnz, rp.data(), col.data(), val.data(), ri.data(), cp.data(), cv.data(),
                          riA.data(), cpA.data(), cvA.data());
    printf("---------------------------------------------------------------------------------------------\n");
    if (rc == 0)
        rc = kernal_sptrans(m, n, nnz, ngpu, rp.data(), col.data(), val.data(), ri.data(), cp.data(),
                            cv.data(), riA.data(), cpA.data(), cvA.data());
    printf("---------------------------------------------------------------------------------------------\n");
    return rc == 0 ? 0 : 1;
}
