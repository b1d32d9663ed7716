// Checks k_orient_desc's matrix-core horizontal Gaussian pass in isolation: a random 43 x 48 window
// in LDS, the host-built tap fragments, nine v_mfma_i32_16x16x64_i8, 16-bit row-sum stores; compared
// exactly with the direct 7-tap sums.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kOdPW = 48, kOdRows = 43, kOdRsCols = 37, kOdRsW = 42;
constexpr int kOdWaveBytes = (kOdRows * kOdPW + kOdRows * kOdRsW * 2 + 15) & ~15;
__global__ void hpass(const uint8_t* win_g, const uint4* ghFrag, uint32_t kA, uint32_t kB, uint16_t* rs_out) {
    __shared__ __attribute__((aligned(16))) unsigned char od_sm[4][kOdWaveBytes];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int t = lane; t < kOdRows * kOdPW; t += 64) od_sm[wid][t] = win_g[t];
    __builtin_amdgcn_wave_barrier();
    uint16_t* RS = reinterpret_cast<uint16_t*>(od_sm[wid] + kOdRows * kOdPW);
    uint4 ghB[3];
    for (int n = 0; n < 3; n++) ghB[n] = ghFrag[n * 64 + lane];
    {
        const unsigned char* win = od_sm[wid];
        const int ci = lane & 15, gq = lane >> 4;
        uint4 aP[3];
#pragma unroll
        for (int m = 0; m < 3; m++) {
            aP[m] = *reinterpret_cast<const uint4*>(win + (16 * m + ci) * kOdPW + 16 * gq);
            aP[m].x ^= 0x80808080u;
            aP[m].y ^= 0x80808080u;
            aP[m].z ^= 0x80808080u;
            aP[m].w ^= 0x80808080u;
        }
        const int c0i = 128 * (int)(__builtin_amdgcn_udot4(kA, 0x01010101u, 0u, false) +
                                    __builtin_amdgcn_udot4(kB, 0x01010101u, 0u, false));
        const i32x4 cinit = {c0i, c0i, c0i, c0i};
        uint16_t* const rsl = RS + 4 * gq * kOdRsW + ci;
#pragma unroll
        for (int n = 0; n < 3; n++) {
#pragma unroll
            for (int m = 0; m < 3; m++) {
                const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, aP[m]),
                                                                      __builtin_bit_cast(i32x4, ghB[n]), cinit, 0, 0, 0);
                if (n < 2 || 16 * n + ci < kOdRsCols) {
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if (m < 2 || 16 * m + 4 * gq + i < kOdRows) rsl[(16 * m + i) * kOdRsW + 16 * n] = (uint16_t)d[i];
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (wid == 1)
        for (int t = lane; t < kOdRows * kOdRsW; t += 64) rs_out[t] = RS[t];
}
int main() {
    int k[7];
    {   // gauss7_int (the extractor's 8-bit kernel)
        float cf[7];
        double sum = 0;
        for (int i = 0; i < 7; i++) { const double x = i - 3.0; cf[i] = (float)std::exp(-0.125 * x * x); sum += cf[i]; }
        sum = 1. / sum;
        for (int i = 0; i < 7; i++) { cf[i] = (float)(cf[i] * sum); k[i] = (int)std::nearbyint(cf[i] * 256.0f); }
    }
    const uint32_t kA = (uint32_t)k[0] | ((uint32_t)k[1] << 8) | ((uint32_t)k[2] << 16) | ((uint32_t)k[3] << 24);
    const uint32_t kB = (uint32_t)k[4] | ((uint32_t)k[5] << 8) | ((uint32_t)k[6] << 16);
    uint8_t frag[3 * 64 * 16];
    for (int n = 0; n < 3; n++)
        for (int l = 0; l < 64; l++)
            for (int j = 0; j < 16; j++) {
                const int t = 16 * (l >> 4) + j - (16 * n + (l & 15)) - 3;
                frag[(n * 64 + l) * 16 + j] = (uint8_t)(t >= 0 && t <= 6 ? k[t] : 0);
            }
    uint8_t win[kOdRows * kOdPW];
    srand(3);
    for (auto& v : win) v = (uint8_t)(rand() & 255);
    uint8_t* dW; uint4* dF; uint16_t* dR;
    (void)hipMalloc(&dW, sizeof(win)); (void)hipMalloc(&dF, sizeof(frag)); (void)hipMalloc(&dR, kOdRows * kOdRsW * 2);
    (void)hipMemcpy(dW, win, sizeof(win), hipMemcpyHostToDevice);
    (void)hipMemcpy(dF, frag, sizeof(frag), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(hpass, dim3(1), dim3(256), 0, 0, dW, dF, kA, kB, dR);
    uint16_t rs[kOdRows * kOdRsW];
    (void)hipMemcpy(rs, dR, sizeof(rs), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < kOdRows; r++)
        for (int c = 0; c < kOdRsCols; c++) {
            int ref = 0;
            for (int q = 0; q < 7; q++) ref += k[q] * win[r * kOdPW + c + 3 + q];
            if (ref != rs[r * kOdRsW + c]) { if (bad < 8) printf("RS[%d][%d] = %d, host %d\n", r, c, rs[r * kOdRsW + c], ref); bad++; }
        }
    printf("taps %d %d %d %d %d %d %d; row sums: %d of %d mismatches\n", k[0], k[1], k[2], k[3], k[4], k[5], k[6], bad, kOdRows * kOdRsCols);
    return bad != 0;
}
