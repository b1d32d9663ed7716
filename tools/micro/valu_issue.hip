// VALU issue rate per instruction kind vs waves per SIMD: every lane
// runs 8 independent chains of ONE instruction (inline asm, so exactly that instruction), k
// workgroups of 256 threads per CU = k waves per SIMD.  Each workgroup's wave 0 stamps s_memtime
// (shader clock) and s_memrealtime (100 MHz constant) at its start and end and reads HW_ID (the CU
// it ran on), so the run can check what the wall clock alone cannot:
//   * co-residency: per CU, the largest number of its workgroups whose [start, end] overlap at one
//     instant (k means all k ran together);
//   * the all-running window [max start, min end] over every workgroup of the launch: inside it
//     every workgroup runs; each workgroup stamps s_memrealtime at 17 checkpoints (every 1/16 of its
//     loop), so the instructions it executed inside the window are interpolated from its own
//     checkpoints and the chip's steady-state rate is their sum over the window (no dispatch ramp or
//     tail, and no workgroup credited for time it ran with fewer neighbours);
//   * the wall-clock rate (instructions / event time) beside it; the two agree when the kernel is
//     long enough and the workgroups are co-resident.
// The ops are the extraction kernels' integer mix (v_perm, v_alignbyte, v_lerp_u8, v_dot4_u32_u8,
// v_bcnt, v_pk_minimum3_f16, v_xad_u32) and the f32 references (v_fma_f32, v_pk_fma_f32).
// Each op runs with 8 U instructions per loop trip, U = 1, 4, 16 (64 / 256 / 1024 bytes of VOP3 per
// trip): a rate that falls with U is bound by instruction fetch, not by the SIMD's issue.
// Usage: valu_issue [iters]   (default 65536: ~8x round 4's loop, >= 4 ms per launch at 8 waves/SIMD)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kOps = 9;
constexpr int kStride = 24;   // per workgroup: memtime start / end, realtime start / end, HW_ID, -, 17 checkpoints
static const char* kNames[kOps] = {"v_fma_f32",      "v_pk_fma_f32",  "v_xad_u32",       "v_perm_b32",        "v_alignbyte_b32",
                                   "v_lerp_u8",      "v_dot4_u32_u8", "v_bcnt_u32_b32",  "v_pk_minimum3_f16"};

template <int OP, int U>
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
        u[k] = __float_as_uint(a[k]) + k;
    }
    const float c = in[1000], d = in[1001];
    const f2 pc = {c, c}, pd = {d, d};
    const unsigned uc = __float_as_uint(c), ud = __float_as_uint(d) | 0x0c0c0c0cu;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
        stamps[kStride * blockIdx.x + 6] = r0;
    }
    const int chunk = iters / 16;   // iters is a multiple of 64
    for (int c = 0; c < 16; c++) {
        if (c > 0 && threadIdx.x == 0) stamps[kStride * blockIdx.x + 6 + c] = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < chunk; i += U) {   // 8 U instructions of the op per trip, 3 loop SALU
#pragma unroll
        for (int kk = 0; kk < 8 * U; kk++) {
            const int k = kk & 7;
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "v"(d));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[k]) : "v"(pc), "v"(pd));
            if (OP == 2) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
            if (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
            if (OP == 4) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
            if (OP == 5) asm volatile("v_lerp_u8 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
            if (OP == 6) asm volatile("v_dot4_u32_u8 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
            if (OP == 7) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(u[k]) : "v"(uc));
            if (OP == 8) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(u[k]) : "v"(uc), "v"(ud));
        }
    }
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        stamps[kStride * blockIdx.x + 0] = t0;
        stamps[kStride * blockIdx.x + 1] = t1;
        stamps[kStride * blockIdx.x + 2] = r0;
        stamps[kStride * blockIdx.x + 3] = r1;
        stamps[kStride * blockIdx.x + 4] = hw;
        stamps[kStride * blockIdx.x + 5] = 0;
        stamps[kStride * blockIdx.x + 22] = r1;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k] + p[k].x + p[k].y + __uint_as_float(u[k]);
    out[t] = s;
}

typedef void (*KFn)(const float*, float*, unsigned long long*, int);
template <int U>
static KFn kfn_u(int op) {
    switch (op) {
        case 0: return k_issue<0, U>;
        case 1: return k_issue<1, U>;
        case 2: return k_issue<2, U>;
        case 3: return k_issue<3, U>;
        case 4: return k_issue<4, U>;
        case 5: return k_issue<5, U>;
        case 6: return k_issue<6, U>;
        case 7: return k_issue<7, U>;
        default: return k_issue<8, U>;
    }
}
static KFn kfn(int op, int u) { return u == 1 ? kfn_u<1>(op) : u == 4 ? kfn_u<4>(op) : kfn_u<16>(op); }

int main(int argc, char** argv) {
    const int iters = (argc > 1 ? std::atoi(argv[1]) : 65536) & ~255;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *in, *out;
    unsigned long long* st;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    (void)hipMalloc(&st, (size_t)cus * 8 * kStride * 8);
    std::vector<float> h(4096, 1.0f);
    h[1000] = 0.999f;
    h[1001] = 0.001f;
    (void)hipMemcpy(in, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::printf("CUs %d, iters %d, 8 independent chains per lane; rates in wave64 instructions\n", cus, iters);
    std::printf("%-18s %3s %3s %8s %7s %9s | %9s %9s %6s | %11s %11s %6s | %12s %12s\n", "op", "U", "w/S", "wall ms", "GHz",
                "coresid", "win ms", "loop ms", "win%", "wall inst/s", "win inst/s", "ratio", "cyc/inst/SIMD",
                "lane-ops/s");
    for (int op = 0; op < kOps; op++)
        for (int u : {1, 4, 16})
        for (int k : {1, 2, 4, 8}) {
            const int blocks = cus * k;
            float ms = 0.f;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(e0);
                hipLaunchKernelGGL(kfn(op, u), dim3(blocks), dim3(256), 0, 0, in, out, st, iters);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            std::vector<unsigned long long> s((size_t)blocks * kStride);
            (void)hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
            // co-residency per CU (HW_ID: CU_ID bits 11:8, SH_ID 12, SE_ID 15:13 on gfx9; XCC from the
            // dispatch order is not in HW_ID, so CUs are keyed by (block % 8 XCD, SE, SH, CU))
            std::vector<std::vector<std::pair<unsigned long long, int>>> ev(8 * 256);
            unsigned long long winStart = 0, winEnd = ~0ull;
            double cyc = 0, rt = 0, rateSum = 0;
            for (int b = 0; b < blocks; b++) {
                const unsigned long long t0 = s[kStride * b], t1 = s[kStride * b + 1], r0 = s[kStride * b + 2], r1 = s[kStride * b + 3];
                const unsigned hw = (unsigned)s[kStride * b + 4];
                const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
                const int key = ((b % 8) * 8 + se) * 32 + sh * 16 + cu;
                ev[(size_t)key % ev.size()].push_back({r0, +1});
                ev[(size_t)key % ev.size()].push_back({r1, -1});
                winStart = std::max(winStart, r0);
                winEnd = std::min(winEnd, r1);
                cyc += (double)(t1 - t0);
                rt += (double)(r1 - r0);
                rateSum += 4.0 * iters * 8 / ((double)(r1 - r0) / 100e6);   // this workgroup's wave-inst/s
            }
            int minPeak = 1 << 30, used = 0;
            for (auto& e : ev) {
                if (e.empty()) continue;
                std::sort(e.begin(), e.end(), [](auto& x, auto& y) { return x.first != y.first ? x.first < y.first : x.second < y.second; });
                int cur = 0, peak = 0;
                for (auto& x : e) { cur += x.second; peak = std::max(peak, cur); }
                minPeak = std::min(minPeak, peak);
                used++;
            }
            const double ghz = cyc / (rt / 100e6) / 1e9;
            const double winst = (double)blocks * 4 * iters * 8;
            const double wallRate = winst / (ms * 1e-3);
            const double winMs = winEnd > winStart ? (double)(winEnd - winStart) / 1e5 : 0.0;
            const double loopMs = rt / blocks / 1e5;
            // instructions each workgroup executed inside the all-running window, interpolated from its
            // 17 checkpoints (1/16 of its loop apart)
            double winInst = 0.0;
            if (winEnd > winStart)
                for (int b = 0; b < blocks; b++) {
                    const unsigned long long* c = &s[(size_t)kStride * b + 6];
                    auto progress = [&](unsigned long long t) {   // fraction of the loop done at realtime t
                        if (t <= c[0]) return 0.0;
                        for (int j = 0; j < 16; j++)
                            if (t <= c[j + 1]) return (j + (double)(t - c[j]) / (double)(c[j + 1] - c[j] ? c[j + 1] - c[j] : 1)) / 16.0;
                        return 1.0;
                    };
                    winInst += (progress(winEnd) - progress(winStart)) * 4.0 * iters * 8;
                }
            const double winRate = winEnd > winStart ? winInst / ((double)(winEnd - winStart) / 100e6) : 0.0;
            (void)rateSum;
            const double cycPerInst = winRate > 0 ? cus * 4.0 * ghz * 1e9 / winRate : 0.0;
            const double lanes = op == 1 ? 128.0 : 64.0;
            std::printf("%-18s %3d %3d %8.3f %7.3f %4d/%-4d | %9.3f %9.3f %5.1f%% | %11.4g %11.4g %6.3f | %12.3f %12.4g\n",
                        kNames[op], u, k, ms, ghz, minPeak, used, winMs, loopMs, 100.0 * winMs / ms, wallRate, winRate,
                        winRate > 0 ? wallRate / winRate : 0.0, cycPerInst, winRate * lanes);
        }
    return 0;
}
