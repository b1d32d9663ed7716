// Integer / f32 VALU issue-rate microbenchmark on the whole chip: every lane runs 8 independent
// dependency chains; wave-instructions per second against 256 CU x 4 SIMD x (1 / 2 or 1 / 4 cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ __launch_bounds__(256) void k_valu(const unsigned* in, unsigned* out, int iters) {
    unsigned a[8];
    const unsigned t = threadIdx.x + blockIdx.x * 256;
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = in[(t + k) & 1023];
    const unsigned c = in[1000], d = in[1001];
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (OP == 0) a[k] = (a[k] ^ c) + d;                                   // v_xad / v_xor + v_add
            if (OP == 1) a[k] = __builtin_amdgcn_alignbyte(a[k], c, d & 3);       // v_alignbyte_b32
            if (OP == 2) a[k] = __builtin_amdgcn_perm(a[k], c, 0x05040100u ^ d);  // v_perm_b32
            if (OP == 3) a[k] = min(min(a[k], c), d) + 1u;                        // v_min3 + v_add
            if (OP == 4) a[k] = __float_as_uint(__builtin_fmaf(__uint_as_float(a[k]), 1.0001f, __uint_as_float(c)));
        }
    }
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s ^= a[k];
    out[t] = s;
}
int main() {
    unsigned *in, *out;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, 256 * 2048 * 4 * 8);
    hipMemset(in, 1, 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 8;   // 8 workgroups (32 waves) per CU
    const char* names[] = {"xor+add", "alignbyte", "perm", "min3+add", "fma_f32"};
    for (int op = 0; op < 5; op++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            switch (op) {
                case 0: hipLaunchKernelGGL(k_valu<0>, dim3(blocks), dim3(256), 0, 0, in, out, iters); break;
                case 1: hipLaunchKernelGGL(k_valu<1>, dim3(blocks), dim3(256), 0, 0, in, out, iters); break;
                case 2: hipLaunchKernelGGL(k_valu<2>, dim3(blocks), dim3(256), 0, 0, in, out, iters); break;
                case 3: hipLaunchKernelGGL(k_valu<3>, dim3(blocks), dim3(256), 0, 0, in, out, iters); break;
                case 4: hipLaunchKernelGGL(k_valu<4>, dim3(blocks), dim3(256), 0, 0, in, out, iters); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) {
                // instructions per chain step counted from the ISA (tools/micro/valu_peak.s): printed by the caller
                const double waves = blocks * 4.0, steps = (double)iters * 8;
                printf("%-10s %.3f ms  chain-steps/s per wave-slot: %.4g  (x waves %.0f)\n", names[op], ms,
                       waves * steps / (ms * 1e-3), waves);
            }
        }
    }
    return 0;
}
