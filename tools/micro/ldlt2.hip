// Development harness for the reduced-camera solve (one workgroup, dense LDL^T of S (n <= 128) +
// both triangular solves), standalone so a layout change can be checked and timed in one gpurun:
// random SPD systems, a CPU unblocked LDL^T in double as the reference, max relative error of x,
// average launch time over repeated launches and an in-kernel clock split.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/micro/ldlt2.hip -o tools/micro/ldlt2
// run:   tools/micro/ldlt2 [n] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHK(x)                                                                               \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

#include "ldlt2_kernel.inc"

// ---------------------------------------------------------------- host reference
static bool ldlt_solve_cpu(std::vector<double> A, std::vector<double> b, int n, std::vector<double>& x) {
    std::vector<double> d(n);
    for (int j = 0; j < n; j++) {   // column recurrence (oracle/lba_oracle.c style), W kept in A
        double dj = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) dj -= A[(size_t)j * n + k] * A[(size_t)j * n + k] / d[k];
        if (dj == 0.0 || !std::isfinite(dj)) return false;
        d[j] = dj;
        for (int i = j + 1; i < n; i++) {
            double w = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) w -= A[(size_t)i * n + k] * A[(size_t)j * n + k] / d[k];
            A[(size_t)i * n + j] = w;
        }
    }
    // L = W / d
    x = b;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < i; k++) x[i] -= A[(size_t)i * n + k] / d[k] * x[k];
    for (int i = 0; i < n; i++) x[i] /= d[i];
    for (int i = n - 1; i >= 0; i--)
        for (int k = i + 1; k < n; k++) x[i] -= A[(size_t)k * n + i] / d[i] * x[k];
    return true;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 114;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 400;
    const int kind = argc > 3 ? std::atoi(argv[3]) : 0;
    const int mode = argc > 4 ? std::atoi(argv[4]) : 0;
    {   // lane primitives
        double* d;
        CHK(hipMalloc(&d, 8 * 7 * 64));
        hipLaunchKernelGGL(k_prim_test, dim3(1), dim3(64), 0, 0, d);
        double h[7 * 64];
        CHK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
        int bad = 0;
        for (int l = 0; l < 64; l++) {
            for (int R = 0; R < 4; R++) bad += h[R * 64 + l] != (double)(16 * R + (l & 15));
            bad += h[4 * 64 + l] != (double)((l & ~15) + 0);
            bad += h[5 * 64 + l] != (double)((l & ~15) + 5);
            bad += h[6 * 64 + l] != (double)((l & ~15) + 15);
        }
        std::printf("lane primitives: %s\n", bad ? "FAIL" : "ok");
        if (bad) {
            for (int r = 0; r < 7; r++) {
                for (int l = 0; l < 64; l++) std::printf("%d ", (int)h[r * 64 + l]);
                std::printf("\n");
            }
            return 1;
        }
    }
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd;
    std::vector<double> S((size_t)n * n), b(n);
    {
        const int m = n + 8;
        std::vector<double> G((size_t)n * m);
        for (auto& g : G) g = nd(rng);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = 0;
                for (int k = 0; k < m; k++) s += G[(size_t)i * m + k] * G[(size_t)j * m + k];
                S[(size_t)i * n + j] = s + (i == j ? (kind == 1 ? 1e-6 : (double)n) : 0.0);
            }
        for (auto& v : b) v = nd(rng);
    }
    std::vector<double> xr;
    if (!ldlt_solve_cpu(S, b, n, xr)) { std::printf("cpu: zero pivot\n"); return 1; }
    double *dS, *db, *dx;
    int* df;
    long long* dt;
    CHK(hipMalloc(&dS, 8 * (size_t)n * n));
    CHK(hipMalloc(&db, 8 * (size_t)n));
    CHK(hipMalloc(&dx, 8 * (size_t)n));
    CHK(hipMalloc(&df, 4));
    CHK(hipMalloc(&dt, 8 * 64));
    CHK(hipMemset(dt, 0, 8 * 64));
    CHK(hipMemcpy(dS, S.data(), 8 * (size_t)n * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(db, b.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    const size_t lds = ldlt2_lds_bytes(n);
    CHK(hipFuncSetAttribute((const void*)k_ldlt2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_ldlt2, dim3(1), dim3(kLdlT), lds, 0, dS, db, n, dx, df, dt, mode);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    std::vector<double> x(n);
    int fail = -1;
    CHK(hipMemcpy(x.data(), dx, 8 * (size_t)n, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&fail, df, 4, hipMemcpyDeviceToHost));
    double err = 0, xmax = 0;
    for (int i = 0; i < n; i++) {
        err = std::max(err, std::fabs(x[i] - xr[i]));
        xmax = std::max(xmax, std::fabs(xr[i]));
    }
    double res = 0;
    for (int i = 0; i < n; i++) {
        double r = -b[i];
        for (int j = 0; j < n; j++) r += S[(size_t)i * n + j] * x[j];
        res = std::max(res, std::fabs(r));
    }
    std::printf("mode %d n %d kind %d: fail %d  max|x - x_cpu| / max|x| = %.3e  residual %.3e\n", mode, n, kind, fail, err / xmax, res);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k_ldlt2, dim3(1), dim3(kLdlT), lds, 0, dS, db, n, dx, df, nullptr, mode);
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_ldlt2, dim3(1), dim3(kLdlT), lds, 0, dS, db, n, dx, df, nullptr, mode);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    hipLaunchKernelGGL(k_ldlt2, dim3(1), dim3(kLdlT), lds, 0, dS, db, n, dx, df, dt, mode);
    CHK(hipDeviceSynchronize());
    long long t[64];
    CHK(hipMemcpy(t, dt, sizeof(t), hipMemcpyDeviceToHost));
    std::printf("avg per launch (back to back, %d reps): %.2f us | clock split: stage %lld factor %lld solve %lld total %lld cycles",
                reps, 1000.0 * ms / reps, t[1] - t[0], t[2] - t[1], t[3] - t[2], t[3] - t[0]);
    if (mode == 1) std::printf(" (tri-inv %lld, P tiles %lld, bsolve %lld)", t[4] - t[2], t[5] - t[4], t[3] - t[5]);
    std::printf(" | panel/trailing:");
    for (int i = 0; i < 8 && 16 * i < n; i++) std::printf(" %lld/%lld", t[8 + i] - (i ? t[16 + i - 1] : t[1]), t[16 + i] - t[8 + i]);
    std::printf("\n  pivot: epilogue(kb-1) / wait / prologue:");
    for (int i = 1; i < 8 && 16 * i < n; i++) std::printf(" %lld/%lld/%lld", t[40 + i] - t[8 + i - 1], t[48 + i] - t[40 + i], t[56 + i] - t[48 + i]);
    std::printf("\n  pivot loop / last follower loop:");
    for (int i = 0; i < 8 && 16 * i < n; i++) std::printf(" %lld/%lld", t[24 + i], t[32 + i]);
    std::printf("\n");
    return 0;
}
