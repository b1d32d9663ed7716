// Latency microbenchmarks for the LDL^T design (one wave, clock64 deltas).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double shfl_d(double v, int src) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__global__ void k_lat(const double* in, double* out, long long* t, const double* big) {
    const int lane = threadIdx.x;
    double a = in[lane], b = in[lane + 64];
    long long t0 = clock64();
    for (int i = 0; i < 256; i++) a = __builtin_fma(a, b, 1e-300);          // dependent fma chain
    long long t1 = clock64();
    for (int i = 0; i < 256; i++) a = __builtin_amdgcn_rcp(a);             // dependent rcp chain
    long long t2 = clock64();
    for (int i = 0; i < 256; i++) a = shfl_d(a, (i & 7)) * b;              // readlane -> mul chain
    long long t3 = clock64();
    for (int i = 0; i < 256; i++) a = a / b;                                // IEEE division chain
    long long t4 = clock64();
    __shared__ double sh[64];
    for (int i = 0; i < 256; i++) { sh[lane] = a; __builtin_amdgcn_wave_barrier(); a = sh[(lane + 1) & 63] * b; }  // LDS round trip
    long long t5 = clock64();
    double s = 0;
    for (int i = 0; i < 64; i++) s += big[(size_t)(i * 4099 + lane * 16) % (1 << 20)];   // independent loads
    long long t6 = clock64();
    int idx = lane;
    for (int i = 0; i < 64; i++) { double v = big[idx]; idx = ((int)v + i * 131071 + lane) & ((1 << 20) - 1); s += v; }   // dependent loads
    long long t7 = clock64();
    double c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a + 2, c5 = b + 2, c6 = a + 3, c7 = b + 3;
    for (int i = 0; i < 256; i++) {   // 8 independent fma chains: issue rate
        c0 = __builtin_fma(c0, b, 1e-300); c1 = __builtin_fma(c1, b, 1e-300); c2 = __builtin_fma(c2, b, 1e-300);
        c3 = __builtin_fma(c3, b, 1e-300); c4 = __builtin_fma(c4, b, 1e-300); c5 = __builtin_fma(c5, b, 1e-300);
        c6 = __builtin_fma(c6, b, 1e-300); c7 = __builtin_fma(c7, b, 1e-300);
    }
    long long t8 = clock64();
    unsigned r0 = 0;
    for (int i = 0; i < 256; i++) {   // independent readlanes: issue rate
        r0 += __builtin_amdgcn_readlane((int)__double2loint(c0), i & 7) + __builtin_amdgcn_readlane((int)__double2loint(c1), (i + 1) & 7) +
              __builtin_amdgcn_readlane((int)__double2loint(c2), (i + 2) & 7) + __builtin_amdgcn_readlane((int)__double2loint(c3), (i + 3) & 7);
    }
    long long t9 = clock64();
    out[lane] = a + s + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + r0;
    if (lane == 0) { t[7] = t8 - t7; t[8] = t9 - t8; t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; t[3] = t4 - t3; t[4] = t5 - t4; t[5] = t6 - t5; t[6] = t7 - t6; }
}
__global__ void k_fill(double* big, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) big[i] = (double)(i % 7);
}
int main() {
    double *in, *out, *big; long long* t;
    hipMalloc(&in, 128 * 8); hipMalloc(&out, 64 * 8); hipMalloc(&t, 16 * 8); hipMalloc(&big, (1 << 20) * 8);
    double h[128]; for (int i = 0; i < 128; i++) h[i] = 1.0 + i * 1e-3;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, big, 1 << 20);
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, in, out, t, big);
        long long ht[16]; hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        printf("per op cycles: fma %.1f rcp %.1f readlane+mul %.1f div %.1f lds-rt %.1f | 64 indep loads %lld, per dep load %.1f\n",
               ht[0] / 256.0, ht[1] / 256.0, ht[2] / 256.0, ht[3] / 256.0, ht[4] / 256.0, ht[5], ht[6] / 64.0);
        printf("independent fma: %.2f cycles per wave-instruction; readlane: %.2f per instruction\n", ht[7] / 2048.0, ht[8] / 1024.0);
    }
    return 0;
}
