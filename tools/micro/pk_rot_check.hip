// Checks the packed-f32 rotation of k_orient_desc's BRIEF pairs against scalar IEEE arithmetic on the
// host (x a - y b, x b + y a, each product rounded, no fma) and the magic-add rounding.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <cstring>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void rot(const float4* pp4, float a, float bb, uint32_t* out) {
    const int lane = threadIdx.x;
    const float4 pp = pp4[lane];   // (x0, x1, y0, y1)
    const f2 av = {a, a}, bv = {bb, bb}, magic = {12582912.0f, 12582912.0f};
    const f2 px = {pp.x, pp.y}, py = {pp.z, pp.w};
    const f2 xf = px * av - py * bv, yf = px * bv + py * av;
    const f2 xm = xf + magic, ym = yf + magic;
    out[4 * lane + 0] = __float_as_uint(xm.x);
    out[4 * lane + 1] = __float_as_uint(ym.x);
    out[4 * lane + 2] = __float_as_uint(xm.y);
    out[4 * lane + 3] = __float_as_uint(ym.y);
}
int main() {
    float h[64 * 4];
    for (int i = 0; i < 64; i++) { h[4 * i] = (float)(i % 27 - 13); h[4 * i + 1] = (float)((i * 7) % 27 - 13); h[4 * i + 2] = (float)((i * 5) % 27 - 13); h[4 * i + 3] = (float)((i * 11) % 27 - 13); }
    const float a = 0.8775825500488281f, b = 0.4794255495071411f;
    float4* d; uint32_t* o;
    (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&o, 64 * 16);
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(rot, dim3(1), dim3(64), 0, 0, d, a, b, o);
    uint32_t g[256];
    (void)hipMemcpy(g, o, sizeof(g), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; i++)
        for (int p = 0; p < 2; p++) {
            const float x = h[4 * i + p], y = h[4 * i + 2 + p];
            volatile float t1 = x * a, t2 = y * b, t3 = x * b, t4 = y * a;
            volatile float xf = t1 - t2, yf = t3 + t4;
            volatile float xm = xf + 12582912.0f, ym = yf + 12582912.0f;
            uint32_t ex, ey;
            float fx = xm, fy = ym;
            std::memcpy(&ex, &fx, 4); std::memcpy(&ey, &fy, 4);
            if (ex != g[4 * i + 2 * p] || ey != g[4 * i + 2 * p + 1]) {
                if (bad < 6) printf("pair %d pt %d: gpu %08x %08x host %08x %08x\n", i, p, g[4 * i + 2 * p], g[4 * i + 2 * p + 1], ex, ey);
                bad++;
            }
        }
    printf("packed rotation: %d of 128 mismatches\n", bad);
    return bad != 0;
}
