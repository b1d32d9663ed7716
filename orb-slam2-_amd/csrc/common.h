// Shared host/device helpers for liborbslam2_amd (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/orbslam2_amd.h"

namespace orbamd {
// One process-wide lock between a handle's legacy-stream setup calls (synchronous hipMemcpy /
// hipMemset / hipMalloc / hipFree) and the local BA's HIP graph capture: a legacy-stream call that
// meets another thread's capture fails the call and invalidates the capture (Tracking
// and LocalMapping threads call into the library at once).  Steady-state launches do not take it.
inline std::mutex& legacy_capture_mutex() {
    static std::mutex m;
    return m;
}
}   // namespace orbamd

// The C-ABI's exception barrier (include/orbslam2_amd.h: no C++ exception crosses it): every
// extern "C" definition is a function-try-block ending in one of these handlers.
namespace orbamd {
inline int abi_exception_status() noexcept {   // called inside a catch (...) handler
    try {
        throw;
    } catch (const std::bad_alloc&) {
        return ORB_ENOMEM;
    } catch (...) {
        return ORB_EINTERNAL;
    }
}
}   // namespace orbamd
#define ORB_ABI_CATCH \
    catch (...) { return orbamd::abi_exception_status(); }
#define ORB_ABI_CATCH_VOID \
    catch (...) {}

#define ORB_HIP_TRY(expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "[orbslam2_amd] %s failed: %s (%s:%d)\n", #expr,           \
                         hipGetErrorString(e_), __FILE__, __LINE__);                        \
            return ORB_EGPU;                                                                \
        }                                                                                   \
    } while (0)

namespace orbamd {

constexpr int kMaxLevels = 16;
constexpr int kWave = 64;

// Returns ORB_OK when a gfx950 device `dev` is usable, else ORB_ENODEV.
int check_device(int dev);

// Per-thread, per-device scratch of the handle-less host entry points (the LocalMapping,
// LoopClosing and Tracking threads call the matchers and PoseOptimization concurrently): one
// non-blocking stream and one grow-only device buffer per (host thread, device), so a call
// allocates nothing, never hipFree-synchronises the device, and two threads never share a
// buffer.  Kept for the thread's lifetime (no HIP calls from thread-exit destructors).
struct HostScratch {
    int device = -1;
    hipStream_t stream = nullptr;
    char* base = nullptr;   // device
    char* pin = nullptr;    // pinned host staging of the same size (Staging below)
    char* pinDev = nullptr; // its device-side address (the pull kernel reads the inputs through it)
    char* pout = nullptr;   // host-mapped coherent outputs: kernels store results straight into host memory
    char* poutDev = nullptr;
    size_t cap = 0;
};
// grow-only (rare; the caller's stream is idle between its calls), under the capture lock
inline int grow_scratch(HostScratch* h, size_t bytes) {
    if (h->cap >= bytes) return ORB_OK;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());
    if (h->base) (void)hipFree(h->base);
    if (h->pin) (void)hipHostFree(h->pin);
    if (h->pout) (void)hipHostFree(h->pout);
    h->base = h->pin = h->pinDev = h->pout = h->poutDev = nullptr;
    h->cap = 0;
    const size_t cap = std::max(bytes + bytes / 2, (size_t)1 << 20);
    if (hipMalloc((void**)&h->base, cap) != hipSuccess) return ORB_ENOMEM;
    if (hipHostMalloc((void**)&h->pin, cap, hipHostMallocMapped) != hipSuccess) return ORB_ENOMEM;
    if (hipHostGetDevicePointer((void**)&h->pinDev, h->pin, 0) != hipSuccess) return ORB_EGPU;
    if (hipHostMalloc((void**)&h->pout, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return ORB_ENOMEM;
    if (hipHostGetDevicePointer((void**)&h->poutDev, h->pout, 0) != hipSuccess) return ORB_EGPU;
    h->cap = cap;
    return ORB_OK;
}
inline int host_scratch(int device, size_t bytes, HostScratch** out) {
    thread_local std::vector<HostScratch*> pool;
    HostScratch* h = nullptr;
    for (HostScratch* p : pool)
        if (p->device == device) h = p;
    // creation and growth (first use, a larger call) take the capture lock: they may run on the
    // Tracking / LoopClosing threads while LocalMapping captures its LM graph
    if (!h) {
        std::lock_guard<std::mutex> lk(legacy_capture_mutex());
        h = new HostScratch();
        h->device = device;
        if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
            delete h;
            return ORB_EGPU;
        }
        pool.push_back(h);
    }
    if (int e = grow_scratch(h, bytes)) return e;
    *out = h;
    return ORB_OK;
}

// One PCIe crossing each way for a handle-less host call: its host inputs are packed into the
// thread's pinned staging at the offsets they take in the device scratch and go over in ONE copy
// (a pageable hipMemcpyAsync per array costs ~10 us each); outputs are reserved after them in one
// contiguous range that comes back in one copy, and the host reads them from the staging after
// the stream sync.  Offsets advance in 256-byte steps; running past the scratch is an error.
// The inputs' copy to the device as a kernel (Staging::upload_pull): 16-byte loads of the pinned
// staging through its device address, coalesced over the grid — for the few-tens-of-KB inputs of a
// matcher call the SDMA copy command's start-up (~8 us, then ~6 us before the dependent kernel
// starts) is most of its cost; a kernel's dependent successor starts within ~1-2 us.
static __global__ __launch_bounds__(256) void k_pull_staging(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                             size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

struct Staging {
    HostScratch* h;
    size_t off = 0, inEnd = 0, ooff = 0;
    bool over = false;
    explicit Staging(HostScratch* hs) : h(hs) {}
    static size_t al(size_t b) { return (b + 255) & ~(size_t)255; }
    char* take(size_t bytes) {
        const size_t a = al(bytes + 1);
        if (off + a > h->cap) { over = true; return h->base; }
        char* d = h->base + off;
        off += a;
        return d;
    }
    // an input: copied into the staging now, on the device after upload()
    char* in(const void* src, size_t bytes) {
        const size_t at = off;
        char* d = take(bytes);
        if (!over && src && bytes) std::memcpy(h->pin + at, src, bytes);
        return d;
    }
    // an input the caller writes into the staging itself (*hostp; nullptr once the staging overflowed)
    char* in_place(size_t bytes, char** hostp) {
        const size_t at = off;
        char* d = take(bytes);
        *hostp = over ? nullptr : h->pin + at;
        return d;
    }
    // staging bytes for arrays of these sizes (256-byte steps, one guard byte each)
    static size_t bytes_for(std::initializer_list<size_t> sizes) {
        size_t t = 4096;
        for (size_t b : sizes) t += al(b + 1);
        return t;
    }
    int upload(hipStream_t s) {
        if (over) return ORB_EINTERNAL;
        inEnd = off;
        if (off && hipMemcpyAsync(h->base, h->pin, off, hipMemcpyHostToDevice, s) != hipSuccess) return ORB_EGPU;
        return ORB_OK;
    }
    // the inputs to the device by a kernel instead of a copy command (same bytes, same offsets)
    int upload_pull(hipStream_t s) {
        if (over) return ORB_EINTERNAL;
        inEnd = off;
        if (off) {
            const size_t n16 = (off + 15) / 16;
            const unsigned nb = (unsigned)std::min<size_t>((n16 + 255) / 256, 1024);
            hipLaunchKernelGGL(k_pull_staging, dim3(nb), dim3(256), 0, s, reinterpret_cast<const uint4*>(h->pinDev),
                               reinterpret_cast<uint4*>(h->base), n16);
            if (hipGetLastError() != hipSuccess) return ORB_EGPU;
        }
        return ORB_OK;
    }
    // a write-once result stored by the kernel straight into host-mapped memory (no copy back):
    // the device address to pass to the kernel; read it with host_out() after the stream sync
    char* out_host(size_t bytes) {
        const size_t a = al(bytes + 1);
        if (ooff + a > h->cap) { over = true; return h->poutDev; }
        char* d = h->poutDev + ooff;
        ooff += a;
        return d;
    }
    template <class T>
    T* host_out(T* dptr) const { return (T*)(h->pout + ((const char*)dptr - h->poutDev)); }
    // device space after the inputs (outputs, work); `from` .. the end comes back in download()
    char* out(size_t bytes) { return take(bytes); }
    int download(hipStream_t s, const void* from) {
        if (over) return ORB_EINTERNAL;
        const size_t a = (size_t)((const char*)from - h->base);
        if (a < off && hipMemcpyAsync(h->pin + a, from, off - a, hipMemcpyDeviceToHost, s) != hipSuccess) return ORB_EGPU;
        return ORB_OK;
    }
    template <class T>
    T* host(T* dptr) const { return (T*)(h->pin + ((const char*)dptr - h->base)); }
};

// 8-bit row pitch used for every device image (multiple of 64 bytes).
inline int pitch_of(int w) { return (w + 63) & ~63; }

__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }

// Inclusive wave64 scan of a 64-bit value.
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Inclusive wave64 prefix sum with DPP row shifts and row broadcasts (gfx9: row_shr:1/2/4/8,
// row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3) — VALU only, no LDS.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

__device__ __forceinline__ int wave_incl_scan_i32(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Sum over a fully active wave: the DPP inclusive scan's total, read from lane 63 (no LDS
// crossbar round trips, unlike the __shfl_xor butterfly below)
__device__ __forceinline__ int wave_sum_dpp(int v) {
    return __builtin_amdgcn_readlane(wave_incl_scan_dpp(v), 63);
}

__device__ __forceinline__ int wave_reduce_sum_i32(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Raw buffer resource over `bytes` bytes at `base` (gfx9 dword 3: 32-bit data format) and a
// 64-bit load through it.  A byte offset at or past `bytes` reads 0 with no fault, so a guarded
// gather can issue its loads unconditionally (an out-of-range offset instead of a branch): the
// compiler then keeps them all in flight rather than waiting on each one behind an exec mask.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
constexpr int kBufOob = 0x7ffffff0;   // an offset past any buffer this library builds
__device__ __forceinline__ double buf_ld_f64(__amdgpu_buffer_rsrc_t r, int byteoff) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, byteoff, 0, 0);
    return __longlong_as_double((long long)(((unsigned long long)x.y << 32) | x.x));
}

// XCD-aware 2-D block index.  Workgroups are dealt round-robin over the 8 XCDs (dispatch id d
// lands on XCD d % 8; observed placement, MI355X_MICROARCH.md "Workgroup dispatch"), so blocks
// that are neighbours in (x, y) order land on different L2s and each XCD re-fetches the lines the
// neighbours share.  Remap so each XCD walks one contiguous range of logical blocks (frames and
// image rows stay on one L2).  Speed only: the map is a bijection on [0, gx*gy) whatever the
// placement (the tail beyond the last multiple of 8 keeps its own index).
__device__ __forceinline__ void xcd_block_2d(int& bx, int& by) {
    const int gx = gridDim.x, G = gx * gridDim.y;
    int d = blockIdx.y * gx + blockIdx.x;
    const int q = G >> 3;
    if (d < (q << 3)) d = (d & 7) * q + (d >> 3);
    by = d / gx;
    bx = d - by * gx;
}

}  // namespace orbamd
