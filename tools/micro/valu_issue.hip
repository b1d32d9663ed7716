// VALU issue rate vs waves per SIMD: every lane runs 8 independent v_fma_f32
// chains (or v_pk_fma_f32 / v_xad_u32 chains), k workgroups of 256 threads per CU = k waves per
// SIMD.  Each workgroup's wave 0 stamps s_memtime (shader clock) and s_memrealtime (100 MHz
// constant) around its loop, so the run reports the clock the SIMDs actually ran at and the
// cycles per wave64 instruction per SIMD, next to MI355X_MICROARCH.md's "2 cycles (SIMD-32),
// one wave alone 4".  Usage: valu_issue [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int OP>
__global__ __launch_bounds__(256) void k_issue(const float* in, float* out, unsigned long long* stamps, int iters) {
    float a[8];
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p[8];
    unsigned u[8];
    const int t = threadIdx.x + blockIdx.x * 256;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        a[k] = in[(t + k) & 1023];
        p[k] = f2{a[k], a[k] + 1.0f};
        u[k] = __float_as_uint(a[k]);
    }
    const float c = in[1000], d = in[1001];
    const f2 pc = {c, c}, pd = {d, d};
    const unsigned uc = __float_as_uint(c), ud = __float_as_uint(d);
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            // inline asm: exactly one instruction of the measured kind per step (the compiler would
            // otherwise SLP-pack the f32 chains or split the xad)
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "v"(d));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[k]) : "v"(pc), "v"(pd));
            if (OP == 2) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
        }
    }
    if (threadIdx.x == 0) {
        stamps[4 * blockIdx.x + 0] = __builtin_amdgcn_s_memtime() - t0;
        stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k] + p[k].x + p[k].y + __uint_as_float(u[k]);
    out[t] = s;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 8192;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *in, *out;
    unsigned long long* st;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&st, (size_t)cus * 8 * 4 * 8);
    std::vector<float> h(4096, 1.0f);
    h[1000] = 0.999f;
    h[1001] = 0.001f;
    hipMemcpy(in, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_xad_u32"};
    printf("CUs %d, iters %d, 8 independent chains per lane\n", cus, iters);
    printf("%-13s %5s %10s %12s %10s %14s %12s\n", "op", "w/SIMD", "ms", "wave-inst/s", "clock GHz", "cyc/inst/SIMD",
           "lane-ops/s");
    for (int op = 0; op < 3; op++)
        for (int k : {1, 2, 4, 8}) {
            const int blocks = cus * k;
            float ms = 0.f;
            for (int rep = 0; rep < 3; rep++) {
                hipEventRecord(e0);
                if (op == 0) hipLaunchKernelGGL(k_issue<0>, dim3(blocks), dim3(256), 0, 0, in, out, st, iters);
                if (op == 1) hipLaunchKernelGGL(k_issue<1>, dim3(blocks), dim3(256), 0, 0, in, out, st, iters);
                if (op == 2) hipLaunchKernelGGL(k_issue<2>, dim3(blocks), dim3(256), 0, 0, in, out, st, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            std::vector<unsigned long long> s((size_t)blocks * 4);
            hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0;
            for (int b = 0; b < blocks; b++) { cyc += (double)s[4 * b]; rt += (double)s[4 * b + 1]; }
            const double ghz = cyc / (rt / 100e6) / 1e9;           // shader cycles per second of realtime
            const double winst = (double)blocks * 4 * iters * 8;   // wave-instructions of the loop
            const double perSimd = winst / (cus * 4.0);
            const double loopSec = rt / blocks / 100e6;            // a workgroup's loop time (realtime)
            const double cycPerInst = loopSec * ghz * 1e9 / perSimd;
            const double lanes = op == 1 ? 128.0 : 64.0;           // a packed f32 instruction does two per lane
            printf("%-13s %5d %10.3f %12.4g %10.3f %14.3f %12.4g\n", names[op], k, ms, winst / (ms * 1e-3), ghz,
                   cycPerInst, winst * lanes / (ms * 1e-3));
        }
    return 0;
}
