// Checks the lane maps of v_mfma_i32_16x16x64_i8 as k_orient_desc uses them: lane l holds
// A[l & 15][16 (l >> 4) + j] and B[16 (l >> 4) + j][l & 15] (j = byte 0..15), D[4 (l >> 4) + i][l & 15].
// Integer data, exact comparison against the host product.  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int* D) {   // A 16x64 row-major, B 64x16 row-major
    const int l = threadIdx.x, r = l & 15, g = l >> 4;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; j++) { a[j] = A[r * 64 + 16 * g + j]; b[j] = B[(16 * g + j) * 16 + r]; }
    i32x4 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    const i32x4 c = {1000, 1000, 1000, 1000};
    const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int i = 0; i < 4; i++) D[(4 * g + i) * 16 + r] = d[i];
}
int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    srand(7);
    for (auto& v : hA) v = (int8_t)(rand() % 256 - 128);
    for (auto& v : hB) v = (int8_t)(rand() % 256 - 128);
    int8_t *dA, *dB;
    int* dD;
    hipMalloc(&dA, sizeof(hA)); hipMalloc(&dB, sizeof(hB)); hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int hD[256];
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            int ref = 1000;
            for (int k = 0; k < 64; k++) ref += hA[i * 64 + k] * hB[k * 16 + j];
            if (ref != hD[i * 16 + j]) { if (bad < 5) printf("D[%d][%d] = %d, host %d\n", i, j, hD[i * 16 + j], ref); bad++; }
        }
    printf("mfma_i32_16x16x64_i8 lane maps: %d of 256 mismatches\n", bad);
    return bad != 0;
}
