// MI355X-native ORB extractor: ORBextractor::operator() (R/src/ORBextractor.cpp:1120-1188)
// as five gfx950 kernels over a batch of frames:
//   k_resize      A2  pyramid level l from level l-1 (INTER_LINEAR 8U fixed point)
//   k_fast_cell   A3  one wave per FAST cell: SWAR pre-test, FAST-9/16 score, cell-local NMS,
//                     iniThFAST / minThFAST retry, raster-order keys (R/src/ORBextractor.cpp:851-896)
//   k_octree      A4  DistributeOctTree, phase-parallel emulation of the std::list algorithm
//                     (R/src/ORBextractor.cpp:571-817), one workgroup per (frame, level)
//   k_orient_desc A5+A6+A7+A8  IC_Angle, 7x7 Gaussian where the descriptor samples, steered
//                     BRIEF, output assembly, one wave per keypoint
//   k_blur        A6  full blurred pyramid, only on demand (orb_pyramid_level_device)
// R/ = /root/reference/ORB-SLAM2注释版/.  All arithmetic follows the oracle's pinned
// semantics (oracle/orb_oracle.c); this file is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <array>
#include <mutex>
#include <vector>

#include "common.h"

#ifdef ORB_TIMING   // instrumented variant (tools/build_variant.py)
#define TSTAMP(v) const long long v = clock64()
#define TACC(acc, a) acc += clock64() - (a)
#else
#define TSTAMP(v)
#define TACC(acc, a)
#endif


namespace orbamd {

constexpr int kEdge = 19;          // EDGE_THRESHOLD
constexpr int kMinBorder = kEdge - 3;
constexpr int kPatch = 31;
constexpr int kHalfPatch = 15;

// bit_pattern_31_ (x0, y0, x1, y1 per pair) as floats (exact small integers), stored per pair as
// (x0, x1, y0, y1): one 16-byte load per point pair in the descriptor loop, and the two points'
// x and y coordinates land in register pairs for the packed-f32 rotation
constexpr int kPatternI[256 * 4] = {
#include "orb_pattern.inc"
};
struct PatternF {
    float v[256 * 4];
};
constexpr PatternF pattern_xxyy() {
    PatternF p{};
    for (int i = 0; i < 256; i++) {
        p.v[4 * i] = (float)kPatternI[4 * i];
        p.v[4 * i + 1] = (float)kPatternI[4 * i + 2];
        p.v[4 * i + 2] = (float)kPatternI[4 * i + 1];
        p.v[4 * i + 3] = (float)kPatternI[4 * i + 3];
    }
    return p;
}
__constant__ __attribute__((aligned(16))) PatternF c_patternf = pattern_xxyy();

struct LevelGeom {
    int w, h, pitch;
    long long off;        // byte offset of this level in a frame's pyramid slab
    int nCols, nRows, wCell, hCell;
    uint32_t nColsMag;    // floor(2^32 / nCols) + 1 (nCols > 1): cell row = umulhi(cell, nColsMag)
    int maxBX, maxBY;     // maxBorderX / maxBorderY (minBorder = 16)
    int cellBase;         // first cell of this level in the frame's cell array
    int slotBase;         // first FAST key slot of this level in the frame's slot array
    int cellCap;          // key slots per cell
    int N;                // DistributeOctTree quota (mnFeaturesPerLevel)
    int nIni;
    float hX;
    int nodeCap;          // node-table capacity == max keypoints out of this level
    int outBase;          // first retained-key slot of this level (per frame)
    float scale;          // mvScaleFactor[level]
    float size;           // (float)(int)(PATCH_SIZE * scale)
    double rsx, rsy;      // 1/((double)dst/src) for the resize producing this level
    int rzX, rzY;         // offsets (uint2 units) of this level's resize column / row tables
    int tileBase, tilesX; // 64x16 tiles (score / blur kernels)
};

struct Geom {
    int nlevels;
    int w, h;
    long long frameBytes;
    int cellsPerFrame, slotsPerFrame, outPerFrame, tilesPerFrame, maxNodeCap, maxLevelSlots;
    int maxCellW, maxCellH;   // largest FAST cell detection region
    int iniTh, minTh, tmin;
    float factorPI;
    int umax[16];
    LevelGeom lv[kMaxLevels];
};

// Level 0 as every consumer reads it.  R/src/ORBextractor.cpp:1223 rebinds mvImagePyramid[0] to the
// input image rather than copying it; so do the kernels: frame b's level 0 is the caller's frame
// p + b * frameStride (rows `pitch` bytes apart) whenever its rows are dword-aligned, else (odd
// widths, the k_resize fallback) the slab's pitched level 0 that a copy kernel fills.  `bytes` =
// the readable bytes from a frame's start (the bound of the consumers' buffer loads).  The frames
// must stay valid and unchanged while a later call reads level 0 (orb_pyramid_level*, the stereo
// matcher), as the reference's Mat header keeps the caller's image.
struct L0Src {
    const uint8_t* p;
    long long frameStride;
    int pitch;
    uint32_t bytes;
};

// ------------------------------------------------------------------ host geometry

static void host_tables(const orb_extractor_params& p, float* scale, float* inv_scale, float* sigma2,
                        float* inv_sigma2, int* fpl) {
    const int n = p.nlevels;
    const double sf = (double)p.scaleFactor;     // `double scaleFactor` member
    float s[kMaxLevels], s2[kMaxLevels];
    s[0] = 1.0f;
    s2[0] = 1.0f;
    for (int i = 1; i < n; i++) {
        s[i] = (float)((double)s[i - 1] * sf);
        s2[i] = s[i] * s[i];
    }
    for (int i = 0; i < n; i++) {
        if (scale) scale[i] = s[i];
        if (sigma2) sigma2[i] = s2[i];
        if (inv_scale) inv_scale[i] = 1.0f / s[i];
        if (inv_sigma2) inv_sigma2[i] = 1.0f / s2[i];
    }
    if (fpl) {
        float factor = (float)(1.0 / sf);
        float nDesired = (float)p.nfeatures * (1.0f - factor) / (1.0f - (float)std::pow((double)factor, (double)n));
        int sum = 0;
        for (int l = 0; l < n - 1; l++) {
            fpl[l] = (int)std::nearbyint(nDesired);
            sum += fpl[l];
            nDesired *= factor;
        }
        fpl[n - 1] = std::max(p.nfeatures - sum, 0);
    }
}

static void host_umax(int* umax) {
    int v, v0;
    int vmax = (int)std::floor((float)kHalfPatch * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil((float)kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (v = 0; v <= vmax; ++v) umax[v] = (int)std::nearbyint(std::sqrt(hp2 - v * v));
    for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

static int build_geom(const orb_extractor_params& p, int w, int h, Geom* g) {
    if (p.nlevels < 1 || p.nlevels > kMaxLevels) return ORB_EINVAL;
    std::memset(g, 0, sizeof(*g));
    g->nlevels = p.nlevels;
    g->w = w;
    g->h = h;
    float scale[kMaxLevels], inv[kMaxLevels];
    int fpl[kMaxLevels];
    host_tables(p, scale, inv, nullptr, nullptr, fpl);
    host_umax(g->umax);
    g->iniTh = std::min(std::max(p.iniThFAST, 0), 255);
    g->minTh = std::min(std::max(p.minThFAST, 0), 255);
    g->tmin = std::min(g->iniTh, g->minTh);
    g->factorPI = (float)(3.14159265358979323846 / 180.f);
    long long off = 0;
    int cells = 0, slots = 0, outs = 0, tiles = 0, maxNC = 0;
    for (int l = 0; l < p.nlevels; l++) {
        LevelGeom& L = g->lv[l];
        L.w = (int)std::nearbyint((float)w * inv[l]);
        L.h = (int)std::nearbyint((float)h * inv[l]);
        if (L.w < 2 * kEdge + 8 || L.h < 2 * kEdge + 8) return ORB_EINVAL;
        if (L.w - 2 * kMinBorder >= 4096 || L.h - 2 * kMinBorder >= 4096) return ORB_EINVAL;
        L.pitch = pitch_of(L.w);
        L.off = off;
        off += (long long)L.pitch * (L.h + 1);   // +1 row of slack for 4-byte tails
        L.maxBX = L.w - kEdge + 3;
        L.maxBY = L.h - kEdge + 3;
        const float width = (float)(L.maxBX - kMinBorder);
        const float height = (float)(L.maxBY - kMinBorder);
        L.nCols = (int)(width / 30.f);
        L.nRows = (int)(height / 30.f);
        if (L.nCols < 1 || L.nRows < 1) return ORB_EINVAL;
        L.nColsMag = L.nCols > 1 ? (uint32_t)((1ull << 32) / (unsigned)L.nCols + 1u) : 0u;
        L.wCell = (int)std::ceil(width / (float)L.nCols);
        L.hCell = (int)std::ceil(height / (float)L.nRows);
        L.cellBase = cells;
        cells += L.nCols * L.nRows;
        L.cellCap = ((L.wCell + 1) / 2) * ((L.hCell + 1) / 2) + 1;
        L.slotBase = slots;
        slots += L.nCols * L.nRows * L.cellCap;
        g->maxLevelSlots = std::max(g->maxLevelSlots, L.nCols * L.nRows * L.cellCap);
        g->maxCellW = std::max(g->maxCellW, L.wCell);
        g->maxCellH = std::max(g->maxCellH, L.hCell);
        if (L.wCell > 64) return ORB_EINVAL;   // a region row must fit the 64 lanes of a wave
        L.N = fpl[l];
        L.nIni = (int)std::round((float)(L.maxBX - kMinBorder) / (float)(L.maxBY - kMinBorder));
        if (L.nIni < 1) return ORB_EINVAL;
        L.hX = (float)(L.maxBX - kMinBorder) / (float)L.nIni;
        L.nodeCap = std::max(L.N, 4 * L.nIni) + 8;
        maxNC = std::max(maxNC, L.nodeCap);
        L.outBase = outs;
        outs += L.nodeCap;
        L.scale = scale[l];
        L.size = (float)(int)((float)kPatch * scale[l]);
        if (l > 0) {
            const LevelGeom& S = g->lv[l - 1];
            L.rsx = 1. / ((double)L.w / S.w);
            L.rsy = 1. / ((double)L.h / S.h);
        }
        L.tilesX = (L.w + 63) / 64;
        L.tileBase = tiles;
        tiles += L.tilesX * ((L.h + 15) / 16);
    }
    g->frameBytes = (off + 255) & ~255LL;
    g->cellsPerFrame = cells;
    g->slotsPerFrame = slots;
    g->outPerFrame = outs;
    g->tilesPerFrame = tiles;
    g->maxNodeCap = maxNC;
    return ORB_OK;
}

// ------------------------------------------------------------------ device helpers

// n / d for n <= 64 and 1 <= d <= 64 without a division: (n * m) >> 16 with m = floor(2^16 * rcp(d))
// + 1, which lies in [2^16 / d, 2^16 / d + 2) (v_rcp_f32 is within 1 ulp, so 2^16 rcp(d) is within
// 0.008 of 2^16 / d, itself an integer or at least 1/64 above one): e = m d - 2^16 < 2d and
// n e < 2^13 < 2^16, so the quotient is exact.  No table load in the chain to the window loads.
__device__ __forceinline__ uint32_t rcp16(int d) {
    return (uint32_t)(65536.0f * __builtin_amdgcn_rcpf((float)d)) + 1u;
}

// level l of frame b: base pointer, row pitch and readable bytes (level 0 per L0Src)
__device__ __forceinline__ const uint8_t* level_img(const Geom& g, const L0Src& z, const uint8_t* pyr, int b, int l,
                                                   int& pitch, uint32_t& bytes) {
    if (l == 0) {
        pitch = z.pitch;
        bytes = z.bytes;
        return z.p + (size_t)b * z.frameStride;
    }
    const LevelGeom& L = g.lv[l];
    pitch = L.pitch;
    bytes = (uint32_t)(g.frameBytes - L.off);
    return pyr + (size_t)b * g.frameBytes + L.off;
}

__device__ __forceinline__ int level_of_tile(const Geom& g, int tile) {
    int l = 0;
    while (l + 1 < g.nlevels && tile >= g.lv[l + 1].tileBase) l++;
    return l;
}
__device__ __forceinline__ int level_of_cell(const Geom& g, int c) {
    int l = 0;
    while (l + 1 < g.nlevels && c >= g.lv[l + 1].cellBase) l++;
    return l;
}
__device__ __forceinline__ int reflect101(int i, int n) {
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// ------------------------------------------------------------------ A2: resize

// One workgroup = 256 output columns x 16 output rows of level l; the source window is staged
// in LDS with dword loads; each thread computes 4 columns x 4 rows, so the x coefficients
// (cv::resize's fixed-point alpha, 11 fractional bits) are computed once per column.
constexpr int kRzCols = 256, kRzRows = 16;

// cv::resize INTER_LINEAR 8U coefficients of one destination column (x) or row (y): source
// index pair and 11-bit weights, {i0 | i1 << 16, w0 | w1 << 16}.  Computed on the host with
// the same IEEE float / double operations (build flags pin -ffp-contract=off on both sides).
static void rz_coef_host(double rs, int d, int srcN, bool clampFrac, uint32_t out[2]) {
    float f = (float)(((double)d + 0.5) * rs - 0.5);
    int s0 = (int)std::floor(f);
    f -= (float)s0;
    if (clampFrac) {   // columns: cv::resize clamps the x index and zeroes the fraction
        if (s0 < 0) { f = 0.f; s0 = 0; }
        if (s0 >= srcN - 1) { f = 0.f; s0 = srcN - 1; }
    }
    const int w0 = (int)std::nearbyint((1.f - f) * 2048.f), w1 = (int)std::nearbyint(f * 2048.f);
    int i0, i1;
    if (clampFrac) {
        i0 = s0;
        i1 = std::min(s0 + 1, srcN - 1);
    } else {           // rows: indices clamped, weights kept
        i0 = std::min(std::max(s0, 0), srcN - 1);
        i1 = std::min(std::max(s0 + 1, 0), srcN - 1);
    }
    out[0] = (uint32_t)i0 | ((uint32_t)i1 << 16);
    out[1] = (uint32_t)w0 | ((uint32_t)w1 << 16);
}

__global__ __launch_bounds__(256) void k_resize(Geom g, int l, uint8_t* __restrict__ pyr, const uint2* __restrict__ rztab,
                                                int srcW32, int srcRows) {
    extern __shared__ uint32_t rz[];   // [srcRows][srcW32] source window
    const LevelGeom& D = g.lv[l];
    const LevelGeom& S = g.lv[l - 1];
    const int b = blockIdx.z, tid = threadIdx.x;
    const int X0 = blockIdx.x * kRzCols, Y0 = blockIdx.y * kRzRows;
    const uint8_t* src = pyr + (size_t)b * g.frameBytes + S.off;
    uint8_t* dst = pyr + (size_t)b * g.frameBytes + D.off;
    const uint2* XT = rztab + D.rzX;
    const uint2* YT = rztab + D.rzY;
    // source window of the block (indices are monotonic in the destination coordinate)
    const int sxLo = (int)(XT[X0].x & 0xFFFF), sxHi = (int)(XT[min(X0 + kRzCols - 1, D.w - 1)].x >> 16);
    const int yLo = (int)(YT[Y0].x & 0xFFFF), yHi = (int)(YT[min(Y0 + kRzRows - 1, D.h - 1)].x >> 16);
    const int cA = sxLo & ~3;
    const int words = (sxHi - cA) / 4 + 1, rows = yHi - yLo + 1;
    const bool staged = words <= srcW32 && rows <= srcRows;
    if (staged) {
        // (row, word) walk without per-element division: step 256 = dq rows + dr words
        const int dq = 256 / words, dr = 256 - dq * words;
        int r = tid / words, wq = tid - r * words;
        while (r < rows) {   // 8 loads in flight per thread before the LDS stores
            uint32_t v[8];
            int rr[8], ww[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                rr[u] = r;
                ww[u] = wq;
                // unconditional (row clamped into the window): the eight loads stay in flight together
                v[u] = *reinterpret_cast<const uint32_t*>(src + (yLo + min(r, rows - 1)) * S.pitch + cA + 4 * wq);
                r += dq;
                wq += dr;
                if (wq >= words) { wq -= words; r++; }
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (rr[u] < rows) rz[rr[u] * srcW32 + ww[u]] = v[u];
        }
    }
    __syncthreads();
    const int cx = tid & 63, ry = tid >> 6;
    const int dx0 = X0 + 4 * cx;
    if (dx0 >= D.w) return;
    int lx0[4], lx1[4], a0[4], a1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint2 c = XT[min(dx0 + k, D.w - 1)];
        lx0[k] = (int)(c.x & 0xFFFF) - cA;
        lx1[k] = (int)(c.x >> 16) - cA;
        a0[k] = (int)(c.y & 0xFFFF);
        a1[k] = (int)(c.y >> 16);
    }
    const uint8_t* win = reinterpret_cast<const uint8_t*>(rz);
    for (int r = 0; r < 4; r++) {
        const int dy = Y0 + ry * 4 + r;
        if (dy >= D.h) break;
        const uint2 c = YT[dy];
        const int y0 = (int)(c.x & 0xFFFF), y1 = (int)(c.x >> 16), b0 = (int)(c.y & 0xFFFF), b1 = (int)(c.y >> 16);
        const uint8_t *R0, *R1;
        int o0 = 0;
        if (staged) {
            R0 = win + (size_t)(y0 - yLo) * srcW32 * 4;
            R1 = win + (size_t)(y1 - yLo) * srcW32 * 4;
        } else {
            R0 = src + (size_t)y0 * S.pitch;
            R1 = src + (size_t)y1 * S.pitch;
            o0 = cA;
        }
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int v0 = R0[o0 + lx0[k]] * a0[k] + R0[o0 + lx1[k]] * a1[k];
            const int v1 = R1[o0 + lx0[k]] * a0[k] + R1[o0 + lx1[k]] * a1[k];
            const uint32_t v = min((uint32_t)(v0 * b0 + v1 * b1 + (1 << 21)) >> 22, 255u);
            packed |= v << (8 * k);
        }
        const int valid = D.w - dx0;   // pitch padding stays 0
        if (valid < 4) packed &= (1u << (8 * valid)) - 1u;
        *reinterpret_cast<uint32_t*>(dst + (size_t)dy * D.pitch + dx0) = packed;
    }
}

// ------------------------------------------------------------------ A2: whole pyramid in one launch
//
// ComputePyramid (R/src/ORBextractor.cpp:1197-1229) for all levels in one launch: a workgroup owns
// one band of one frame.  Bands partition the rows of the last level; going down the pyramid, a
// band's range at level l-1 is exactly the source rows its level-l range reads (cv::resize's row
// pair of the first and last row), so a workgroup computes every level of its band from its own
// LDS copy of the level below.  Neighbouring bands recompute the few rows where their ranges
// overlap (the same arithmetic on the same source bytes, so both write identical values), and the
// ranges of all bands cover every row of every level (checked on the host; otherwise the per-level
// k_resize launches are used).  Level 0 is not copied (the reference rebinds mvImagePyramid[0] to
// the input, :1223): level 1 is computed straight from the caller's frame (L0Src, L2-resident
// buffer loads), so the LDS holds levels 1..7 only — the odd levels in one buffer, the even ones in
// the other.
// LDS budget of one k_pyramid workgroup (both level buffers + the coefficient tables)
#ifndef ORB_PYR_LDS_BUDGET_KB
#define ORB_PYR_LDS_BUDGET_KB 32
#endif
constexpr int kPyrLdsBudget = ORB_PYR_LDS_BUDGET_KB * 1024;

// output rows per k_pyramid thread iteration (rows r, r + 4, ..: their source-row loads in flight together)
constexpr int kPyrRows = 2;

struct PyrBand {
    int s0, n;   // rows [s0, s0 + n) of a level computed by a band
};

// One level of a band: output rows db of level l (D) from source rows sb of level l-1 (S), read
// from LDS (`cur`, row pitch sp) or, for level 1, from the caller's level 0 through `rs`.
template <bool FromGlobal>
__device__ __forceinline__ void pyr_band_level(const LevelGeom& D, const LevelGeom& S, const PyrBand sb, const PyrBand db,
                                               const uint2* XT, const uint2* YT, const uint8_t* cur,
                                               __amdgpu_buffer_rsrc_t rs, int srcPitch, uint8_t* nxt, uint8_t* out,
                                               int tid) {
    const int sp = ((S.w + 3) >> 2) << 2, dp = ((D.w + 3) >> 2) << 2;   // LDS row pitches
    const int G = (D.w + 3) >> 2;   // column groups
    // thread = (column group cg, row phase rp): the group's column coefficients stay in registers
    // while the thread walks rows rp, rp + 4, ... kPyrRows at a time (2; 3 and 4 measured the same
    // in a same-box A/B)
    for (int pr = tid; pr < 4 * G; pr += 256) {
        const int rp = pr / G, cg = pr - rp * G;
        const int dx0 = 4 * cg;
        // the group's source bytes x0[j], x1[j] lie in an 8-byte window starting at x0[0]
        // (host-checked span): per row three aligned dwords, two alignbytes re-base the window at
        // x0[0], one v_perm per column places x0[j] and x1[j] in the two u16 halves, and one
        // v_dot2_u32_u16 against (a0[j], a1[j]) gives the column's horizontal sum a0 x0 + a1 x1
        // (<= 255 * 2048, exact)
        uint32_t sel[4], wt[4];
        const int xb = (int)(XT[min(dx0, D.w - 1)].x & 0xFFFF);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint2 c = XT[min(dx0 + j, D.w - 1)];
            sel[j] = (uint32_t)((int)(c.x & 0xFFFF) - xb) | 0x0c00u | ((uint32_t)((int)(c.x >> 16) - xb) << 16) | 0x0c000000u;
            wt[j] = c.y;   // a0 | a1 << 16
        }
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const int dw = xb >> 2;
        const uint32_t sh = (uint32_t)(xb & 3);
        const int valid = D.w - dx0;   // pitch padding stays 0
        const uint32_t keep = valid < 4 ? (1u << (8 * valid)) - 1u : 0xFFFFFFFFu;
        // (tried: a thread walking its rows in order, reusing the horizontal sums of a source row
        // shared with the previous output row — 1.2 source rows per output row instead of 2 — was
        // slower: one row of loads in flight instead of two rows' four)
        const __amdgpu_buffer_rsrc_t ro = buf_rsrc(out, (uint32_t)(D.pitch * (db.s0 + db.n)));
        // one thread iteration: output rows r, r + 4, .. (kPyrRows of them, clamped to the band) —
        // their row coefficients and source dwords (fetch), then the sums and stores (compute)
        struct Rows {
            int rr[kPyrRows];
            uint2 cy[kPyrRows];
            uint32_t dd[kPyrRows][2][3];
        };
        auto fetch = [&](int r, Rows& f) {
#pragma unroll
            for (int u = 0; u < kPyrRows; u++) {
                f.rr[u] = min(r + 4 * u, db.n - 1);
                f.cy[u] = YT[f.rr[u]];
            }
#pragma unroll
            for (int u = 0; u < kPyrRows; u++) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t sy = h ? (f.cy[u].x >> 16) : (f.cy[u].x & 0xFFFF);
                    if (FromGlobal) {   // dword-aligned rows: the three dwords of the window (a dword
                                        // past the frame reads 0 and is never selected)
                        const int off = (int)__umul24(sy, (uint32_t)srcPitch) + 4 * dw;
                        f.dd[u][h][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
                        f.dd[u][h][1] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4, 0, 0);
                        f.dd[u][h][2] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 8, 0, 0);
                    } else {
                        const uint32_t* R = reinterpret_cast<const uint32_t*>(cur + __umul24(sy - (uint32_t)sb.s0, (uint32_t)sp)) + dw;
                        f.dd[u][h][0] = R[0];
                        f.dd[u][h][1] = R[1];
                        f.dd[u][h][2] = R[2];
                    }
                }
            }
        };
        auto compute = [&](int r, const Rows& f) {
            uint32_t hs[kPyrRows][2][4];   // [row u][source row 0/1][column]: horizontal sums
#pragma unroll
            for (int u = 0; u < kPyrRows; u++) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t w0 = __builtin_amdgcn_alignbyte(f.dd[u][h][1], f.dd[u][h][0], sh);
                    const uint32_t w1 = __builtin_amdgcn_alignbyte(f.dd[u][h][2], f.dd[u][h][1], sh);
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        hs[u][h][j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(w1, w0, sel[j])),
                                                             __builtin_bit_cast(u16x2, wt[j]), 0u, false);
                }
            }
#pragma unroll
            for (int u = 0; u < kPyrRows; u++) {
                // cv's (h0 b0 + h1 b1 + 2^21) >> 22 with the row weights scaled by 4 (the LDS table
                // holds them so): the result is byte 3 of the 32-bit sum — h <= 255 * 2049 (19 bits)
                // and 4 b <= 8196 fit v_mad_u32_u24, the sum stays below 2^32 (255 * 2049^2 * 4 + 2^23)
                // and its top byte never exceeds 255, so no shift and no clamp; two v_perm + one or
                // pack the four
                const uint32_t b0 = f.cy[u].y & 0xFFFF, b1 = f.cy[u].y >> 16;
                uint32_t v[4];
#pragma unroll
                for (int j = 0; j < 4; j++) v[j] = __umul24(hs[u][1][j], b1) + (__umul24(hs[u][0][j], b0) + (1u << 23));
                if (u > 0 && r + 4 * u >= db.n) break;
                const uint32_t pv = (__builtin_amdgcn_perm(v[1], v[0], 0x0c0c0703u) |
                                     __builtin_amdgcn_perm(v[3], v[2], 0x07030c0cu)) & keep;
                *reinterpret_cast<uint32_t*>(nxt + f.rr[u] * dp + dx0) = pv;
                __builtin_amdgcn_raw_buffer_store_b32(pv, ro, (int)__umul24((uint32_t)(db.s0 + f.rr[u]), (uint32_t)D.pitch) + dx0, 0, 0);
            }
        };
        constexpr int kStep = 4 * kPyrRows;
        if (FromGlobal) {
            // level 1 reads the caller's frame from L2 / HBM: the next iteration's rows are fetched
            // before this one's are computed (two register sets in turn; a fetch past the band reads
            // its last row again, unconditionally, so no load is exec-masked), so a thread waits one
            // load latency per band instead of one per iteration
            Rows fa, fb;
            if (rp < db.n) fetch(rp, fa);
            for (int r = rp; r < db.n; r += 2 * kStep) {
                fetch(r + kStep, fb);
                compute(r, fa);
                if (r + kStep >= db.n) break;
                fetch(r + 2 * kStep, fa);
                compute(r + kStep, fb);
            }
        } else {
            for (int r = rp; r < db.n; r += kStep) {
                Rows f;
                fetch(r, f);
                compute(r, f);
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_pyramid(Geom g, L0Src z, uint8_t* __restrict__ pyr,
                                                 const uint2* __restrict__ rztab, const PyrBand* __restrict__ bands,
                                                 int nBands, int bufABytes, int bufBBytes, int* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint32_t pyr_sm[];
    const int tid = threadIdx.x;
    int k, b;
    xcd_block_2d(k, b);
    uint8_t* bufOdd = reinterpret_cast<uint8_t*>(pyr_sm);
    uint8_t* bufEven = bufOdd + bufBBytes;   // odd levels (1, 3, 5, 7) in B, even (2, 4, 6) in A
    uint2* tabL = reinterpret_cast<uint2*>(bufEven + bufABytes);   // this level's column then row coefficients
    uint8_t* slab = pyr + (size_t)b * g.frameBytes;
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *status = 0;   // this call's status word
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(z.p + (size_t)b * z.frameStride, z.bytes);
#ifdef ORB_TIMING
    long long tl[9];
    tl[0] = tl[1] = clock64();
#endif
    for (int l = 1; l < g.nlevels; l++) {
        const LevelGeom& D = g.lv[l];
        const LevelGeom& S = g.lv[l - 1];
        const PyrBand sb = bands[(l - 1) * nBands + k], db = bands[l * nBands + k];
        // the level's column coefficients and the band's row coefficients -> LDS
        uint2* XT = tabL;
        uint2* YT = tabL + D.w;
        // (row weights scaled by 4 here: w0 <= 2049, so the shift carries nothing into w1's half)
        for (int i = tid; i < D.w + db.n; i += 256) {
            uint2 c = i < D.w ? rztab[D.rzX + i] : rztab[D.rzY + db.s0 + (i - D.w)];
            if (i >= D.w) c.y <<= 2;
            tabL[i] = c;
        }
        __syncthreads();
        uint8_t* nxt = (l & 1) ? bufOdd : bufEven;
        const uint8_t* cur = (l & 1) ? bufEven : bufOdd;
        if (l == 1)
            pyr_band_level<true>(D, S, sb, db, XT, YT, nullptr, rs, z.pitch, nxt, slab + D.off, tid);
        else
            pyr_band_level<false>(D, S, sb, db, XT, YT, cur, rs, 0, nxt, slab + D.off, tid);
        __syncthreads();   // (also: the coefficient tables are rewritten by the next level)
#ifdef ORB_TIMING
        tl[l + 1] = clock64();
#endif
    }
#ifdef ORB_TIMING
    if (tid == 0 && b == 0 && (k == 0 || k == 7))
        printf("pyramid band %d: L0 %lld L1 %lld L2 %lld L3 %lld L4 %lld L5 %lld L6 %lld L7 %lld\n", k, tl[1] - tl[0],
               tl[2] - tl[1], tl[3] - tl[2], tl[4] - tl[3], tl[5] - tl[4], tl[6] - tl[5], tl[7] - tl[6], tl[8] - tl[7]);
#endif
}

// ------------------------------------------------------------------ A3: FAST score

// S = max over the 16 circular 9-arcs of min(v - p) (dark) or min(p - v) (bright), minus 1.
// OpenCV's cornerScore<16>(threshold t) == S for every pixel that is a corner at t, and a
// pixel is a corner at t iff S >= t.  Stored as S if S >= tmin else 0.
// (Before gfx950's packed 3-input minimum: the 9-arc minima / maxima as min3 / max3 of three
// 3-arcs in 32-bit integers, one chain per polarity — 114 VALU operations per survivor.)
// Both polarities run in one packed-f16 register (gfx950 v_pk_minimum3_f16 /
// v_pk_maximum3_f16): lane pair k = (v - p_k, p_k - v).  The low half runs the dark chain (max over
// arcs of the arc minimum of v - p), the high half the bright one (max over arcs of the arc minimum
// of p - v); S = max(lo, hi) - 1.  Integers up to
// 2048 are exact in f16.  (1024 + x, -(1024 + x)) is one multiply-add on the f16 bit patterns
// (x * 0x10001 + 0xE4006400: 0x6400 + x is 1024 + x for x < 1024, no carry between the halves), and
// their difference gives each pair exactly.
__device__ __forceinline__ int fast_score_pk(const int v, const int p[16]) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 vn = __builtin_bit_cast(h2, (uint32_t)v * 0x10001u + 0xE4006400u);
    h2 d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = vn - __builtin_bit_cast(h2, (uint32_t)p[k] * 0x10001u + 0xE4006400u);
    h2 m3[16], a9[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++)
        a9[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
    h2 s = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a9[0], a9[1]), a9[2]);
#pragma unroll
    for (int k = 3; k < 15; k += 2) s = __builtin_elementwise_maximum(__builtin_elementwise_maximum(s, a9[k]), a9[k + 1]);
    s = __builtin_elementwise_maximum(s, a9[15]);
    return (int)(s.x > s.y ? s.x : s.y) - 1;
}

constexpr int kTileW = 64, kTileH = 16;   // blur tiles

// ------------------------------------------------------------------ A3: FAST per cell (fused)

// Per-wave LDS of k_fast_cell for regions up to maxW x maxH (host and device agree on it).
__host__ __device__ inline int fc_patch_stride(int maxW) { return ((maxW + 8 + 3) & ~3) + 4; }
__host__ __device__ inline int fc_score_stride(int maxW) { return (maxW + 3) & ~3; }
// patch (window bytes; after scoring it holds the u8 suppressed score per survivor), score map,
// u16 y*64+x list of the pre-test survivors, 64 u16 sinks.  ~6.0 KB per wave for 36 x 36
// regions: six 4-wave workgroups per CU.
__host__ __device__ inline int fc_wave_bytes(int maxW, int maxH) {
    int patch = ((maxH + 6) * fc_patch_stride(maxW) + 15) & ~15;
    const int keep = (maxW * maxH + 15) & ~15;
    if (patch < keep) patch = keep;
    const int sc = ((maxH + 2) * fc_score_stride(maxW + 2) + 15) & ~15;   // 1-px zero border
    const int list = (maxW * maxH * 2 + 15) & ~15;
    return patch + sc + list + 128;   // + one u16 sink per lane (branch-free list emission)
}

// One wave per FAST cell (R/src/ORBextractor.cpp:851-896): cv::FAST on the cell's window,
// restated without an intermediate score map.
//  1. the window (detection region + 3-px ring margin) is staged in LDS, rows realigned so
//     that region column 0 sits on a dword boundary;
//  2. SWAR pre-test, 4 pixels per lane-task: ring pixels 0/4/8/12 (any 9-arc holds two adjacent
//     ones) against the centre for 4 pixels at once, in 16-bit lanes (even / odd bytes) with a
//     512 bias so no lane borrows from its neighbour; survivors are compacted (wave prefix);
//  3. full score S (max over the 16 circular 9-arcs, min3/max3 form) for survivors only; the
//     score buffer holds S >= tmin, 0 elsewhere (cv::FAST's non-corners);
//  4. NMS of the scored pixels against their 8 neighbours; outside the region the window's
//     FAST sees 0.  With non-corners at threshold t scoring 0, "S > every neighbour"
//     does not depend on t (a neighbour >= S is a corner at t whenever S is), so both passes
//     (iniThFAST, then minThFAST if the cell is empty, :879-883) read the same maxima;
//  5. keys emitted in raster order, as cv::FAST returns them.
// MW > 0: the region width bound maxW is the compile-time MW (the host passes the same value), so
// the window / score-map row strides are constants and every ring / neighbour load takes an
// immediate offset from one address; MW = 0: strides at run time (any cell width).
template <int MW>
__global__ __launch_bounds__(256) void k_fast_cell(Geom g, const uint8_t* __restrict__ pyr, L0Src z,
                                                   uint32_t* __restrict__ slots, int* __restrict__ cellCount,
                                                   int* __restrict__ status, int maxWarg, int maxH) {
    const int maxW = MW > 0 ? MW : maxWarg;
    TSTAMP(t_fc0);
    extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
    // the wave index is uniform: readfirstlane keeps it (and the level / cell / geometry derived
    // from it) in SGPRs, so g.lv[l] fields are scalar loads instead of per-lane flat loads
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int bx, b;
    xcd_block_2d(bx, b);
    const int c = bx * 4 + wid;
    // the four cells' survivor counts (phases 3-4 are pooled over the workgroup) and their
    // "a key at iniThFAST" flags
    __shared__ int poolN[4], anyS[4];
    // a wave without a cell (past the frame's cells, or an empty / oversized region) keeps n = 0
    // and still takes part in the pooled phases' barriers
    bool act = c < g.cellsPerFrame;
    const int l = level_of_cell(g, act ? c : g.cellsPerFrame - 1);
    const LevelGeom& L = g.lv[l];
    const int ci = c - L.cellBase;
    // ci / nCols by a multiply-high on the scalar unit (exact: ci * (nColsMag * nCols - 2^32) < 2^32)
    const int i = L.nCols > 1 ? (int)__umulhi((uint32_t)ci, L.nColsMag) : ci, j = ci - i * L.nCols;
    int* cnt_out = cellCount + (size_t)b * g.cellsPerFrame + c;
    const int iniY = kMinBorder + i * L.hCell;
    int maxY = iniY + L.hCell + 6;
    const int iniX = kMinBorder + j * L.wCell;
    int maxX = iniX + L.wCell + 6;
    if (act && (iniY >= L.maxBY - 3 || iniX >= L.maxBX - 6)) {
        if (lane == 0) *cnt_out = 0;
        act = false;
    }
    if (maxY > L.maxBY) maxY = L.maxBY;
    if (maxX > L.maxBX) maxX = L.maxBX;
    const int rw = maxX - iniX - 6, rh = maxY - iniY - 6;   // detection region
    if (act && (rw <= 0 || rh <= 0)) {
        if (lane == 0) *cnt_out = 0;
        act = false;
    }
    if (act && (rw > maxW || rh > maxH || rw > 64)) {
        if (lane == 0) { *cnt_out = 0; atomicOr(status, 1); }
        act = false;
    }
    const int PWS = fc_patch_stride(maxW), W32 = PWS >> 2, SCS = fc_score_stride(maxW + 2);
    const int waveBytes = fc_wave_bytes(maxW, maxH);
    const int patchBytes = max(((maxH + 6) * PWS + 15) & ~15, (maxW * maxH + 15) & ~15);
    const int listOff = patchBytes + (((maxH + 2) * SCS + 15) & ~15);
    unsigned char* base = dsm + (size_t)wid * waveBytes;
    uint32_t* patch32 = reinterpret_cast<uint32_t*>(base);
    uint8_t* sc = base + patchBytes;
    uint16_t* list = reinterpret_cast<uint16_t*>(base + listOff);
    uint8_t* kp = base;   // the window is dead once every survivor is scored (phase 3)
    int pitch;
    uint32_t imgBytes;
    const uint8_t* img = level_img(g, z, pyr, b, l, pitch, imgBytes);
    const int rx0 = iniX + 3, ry0 = iniY + 3;
    int n = 0;
    if (act) {

    // 1. window rows ry0-3 .. ry0+rh+2, columns from rx0-4 (patch column 4 = region column 0):
    //    lane (row r0 + R*u, dword k) loads one aligned dword, all loads in flight at once; the
    //    realigned dword takes its upper bytes from the next lane (next dword of the row)
    {
        const int gx0 = rx0 - 4, sh = gx0 & 3, ga = gx0 - sh;
        const int NW = (rw + 8 + 3) >> 2;           // dwords per patch row
        const int NW1 = NW + 1;                     // aligned source dwords per row
        const uint32_t mW = rcp16(NW1);
        const int r0 = (int)(((uint32_t)lane * mW) >> 16), k = lane - r0 * NW1, R = (int)((64u * mW) >> 16);
        const int rows = rh + 6;
        // buffer loads over the rest of the level image: a row past the window (or past the
        // image: reads 0) is loaded but never stored, so no clamp and no exec mask; the row step
        // is a scalar offset, the lane's part one 24-bit multiply-add
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(img, imgBytes);
        const uint32_t laneOff = __umul24((uint32_t)(ry0 - 3 + r0), (uint32_t)pitch) + (uint32_t)(ga + 4 * k);
        uint32_t* const sink = reinterpret_cast<uint32_t*>(list) + lane;   // the list is written only later
        for (int rb = 0; rb < rows; rb += 8 * R) {
            uint32_t a[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                a[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)laneOff, (rb + u * R) * pitch, 0);
#pragma unroll
            for (int u = 0; u < 8; u++) {
                // the next dword of the row sits in the next lane (DPP wave_shl:1, no LDS round trip)
                const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a[u], 0x130, 0xF, 0xF, false);
                const int r = rb + u * R + r0;
                const bool st = r0 < R && r < rows && k < NW;
                *(st ? patch32 + r * W32 + k : sink) = __builtin_amdgcn_alignbyte(nx, a[u], sh);
            }
        }
        for (int q = lane; q < (rh + 2) * SCS / 4; q += 64) reinterpret_cast<uint32_t*>(sc)[q] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    // 2. pre-test, byte-SWAR over four pixels per dword: any 9-arc holds four cyclically
    //    consecutive even ring pixels (0, 2, .., 14), so they must all be dark (p < v - t) or all
    //    bright (p > v + t) at the strict threshold tmin — a necessary condition for both passes.
    //    Per byte, x > y is the top bit of the carry-free byte average v_lerp_u8(x, ~y), with the
    //    saturated A = max(v - t, 0) and B = min(v + t, 255) of the centre bytes: dark = A > p,
    //    bright = p > B (three operations per ring dword).
    //    Task (row y, column group gq) covers region columns 8gq .. 8gq+7 (two dwords: the loads,
    //    the scan and the index math shared by eight pixels); survivors (~8 % of the pixels) are
    //    appended in raster order by a loop over the task's set bits.
    const uint32_t tpre = (uint32_t)max(g.tmin, 1);
    {
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const u16x2 tt = {(unsigned short)tpre, (unsigned short)tpre};
        const u16x2 m255 = {255, 255};
        constexpr uint32_t H = 0x80808080u;
        auto pk = [](uint32_t u) { return __builtin_bit_cast(u16x2, u); };
        auto upk = [](u16x2 u) { return __builtin_bit_cast(uint32_t, u); };
        // bit k of the result = pixel k of dword cC may be a corner.  Ring pixels by (dy, dx):
        // 0 (+3, 0), 2 (+2, +2), 4 (0, +3), 6 (-2, +2), 8 (-3, 0), 10 (-2, -2), 12 (0, -3), 14 (+2, -2);
        // rows above / below as u3 / d3 (the dword itself) and u2L.. / d2L.. (with neighbours).
        auto even_ring4 = [&](uint32_t cL, uint32_t cC, uint32_t cR, uint32_t u3, uint32_t d3, uint32_t u2L,
                              uint32_t u2C, uint32_t u2R, uint32_t d2L, uint32_t d2C, uint32_t d2R) -> uint32_t {
            const uint32_t vE = cC & 0x00ff00ffu, vO = (cC >> 8) & 0x00ff00ffu;
            const uint32_t nA = ~(upk(__builtin_elementwise_sub_sat(pk(vE), tt)) |
                                  (upk(__builtin_elementwise_sub_sat(pk(vO), tt)) << 8));
            const uint32_t nB = ~(upk(__builtin_elementwise_min(pk(vE) + tt, m255)) |
                                  (upk(__builtin_elementwise_min(pk(vO) + tt, m255)) << 8));
            uint32_t ndk[8], br[8];
            // v_lerp_u8 averages bytes without carries between them: (x + y + r) >> 1 per byte, r the
            // byte's rounding bit.  Bright: (p + ~B) >> 1 has its top bit set iff p + 255 - B >= 256,
            // i.e. p > B.  Dark, complemented so no ~p is needed: (~A + p + 1) >> 1 has its top bit
            // set iff 255 - A + p + 1 >= 256, i.e. p >= A — NOT dark (A > p)
            auto flags = [&](uint32_t p, int u) {
                ndk[u] = __builtin_amdgcn_lerp(nA, p, 0x01010101u);   // !(A > p)
                br[u] = __builtin_amdgcn_lerp(p, nB, 0u);            // p > B: bright
            };
            flags(d3, 0);
            flags(__builtin_amdgcn_alignbyte(d2R, d2C, 2), 1);
            flags(__builtin_amdgcn_alignbyte(cR, cC, 3), 2);
            flags(__builtin_amdgcn_alignbyte(u2R, u2C, 2), 3);
            flags(u3, 4);
            flags(__builtin_amdgcn_alignbyte(u2C, u2L, 2), 5);
            flags(__builtin_amdgcn_alignbyte(cC, cL, 1), 6);
            flags(__builtin_amdgcn_alignbyte(d2C, d2L, 2), 7);
            // a run of four at u is P_u & P_{u+2} with P_u = D_u & D_{u+1}; over the four even (odd)
            // starts the OR of adjacent products on a 4-cycle factors as
            // P0 P2 | P2 P4 | P4 P6 | P6 P0 = (P0 | P4) & (P2 | P6)   (ten operations per polarity)
            // as 3-input v_bitop3 steps (truth table bit (a << 2 | b << 1 | c)): (a & b) | c = 0xEA,
            // (a | b) & c = 0xA8, (~a | b) & c = 0x8A — ten operations per polarity, one to combine
            // (the compiler's own form took 26.5 per dword)
            auto and_or = [](uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xEA); };
            auto or_and = [](uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xA8); };
            auto runs = [&](const uint32_t D[8]) {
                const uint32_t x = and_or(D[0], D[1], D[4] & D[5]), y = and_or(D[2], D[3], D[6] & D[7]);
                const uint32_t z = and_or(D[1], D[2], D[5] & D[6]), w = and_or(D[3], D[4], D[7] & D[0]);
                return and_or(x, y, z & w);
            };
            // the same on complemented flags N = ~D (De Morgan): ~runs(D)
            auto no_runs = [&](const uint32_t N[8]) {
                const uint32_t x = or_and(N[0], N[1], N[4] | N[5]), y = or_and(N[2], N[3], N[6] | N[7]);
                const uint32_t z = or_and(N[1], N[2], N[5] | N[6]), w = or_and(N[3], N[4], N[7] | N[0]);
                return or_and(x, y, z | w);
            };
            // pixel k's flag in bit 8k + 7: (~no_runs(dark) | runs(bright)) & H
            return __builtin_amdgcn_bitop3_b32(no_runs(ndk), runs(br), H, 0x8A);

        };
        const int NG = (rw + 7) >> 3;
        const uint32_t mG = rcp16(NG);
        const int r0 = (int)(((uint32_t)lane * mG) >> 16), gq = lane - r0 * NG, R = (int)((64u * mG) >> 16);
        for (int yb = 0; yb < rh; yb += R) {
            const int y = yb + r0;
            uint32_t want = 0;
            if (r0 < R && y < rh) {
                const int rowC = (y + 3) * W32 + 2 * gq + 1;   // dwords holding region columns 8gq..8gq+7
                const uint32_t cL = patch32[rowC - 1], c0 = patch32[rowC], c1 = patch32[rowC + 1], cR = patch32[rowC + 2];
                const int ru = rowC - 2 * W32, rd = rowC + 2 * W32;
                const uint32_t uL = patch32[ru - 1], uA = patch32[ru], uB = patch32[ru + 1], uR = patch32[ru + 2];
                const uint32_t dL = patch32[rd - 1], dA = patch32[rd], dB = patch32[rd + 1], dR = patch32[rd + 2];
                const uint32_t u30 = patch32[rowC - 3 * W32], u31 = patch32[rowC - 3 * W32 + 1];
                const uint32_t d30 = patch32[rowC + 3 * W32], d31 = patch32[rowC + 3 * W32 + 1];
                // flags of pixels 0-3 in bits 0, 8, 16, 24 and of pixels 4-7 in bits 4, 12, 20, 28;
                // one multiply moves bit 8k (+4) to bit 21 + k (+4): no two partial products collide
                const uint32_t f = (even_ring4(cL, c0, c1, u30, d30, uL, uA, uB, dL, dA, dB) >> 7) |
                                   (even_ring4(c0, c1, cR, u31, d31, uA, uB, uR, dA, dB, dR) >> 3);
                want = ((f * 0x00204081u) >> 21) & 0xFFu;
                const int valid = rw - 8 * gq;   // columns of this group inside the region
                if (valid < 8) want &= (1u << valid) - 1u;
            }
            const int cntW = __popc(want);
            const int incl = wave_incl_scan_dpp(cntW);
            int at = n + incl - cntW;
            const uint16_t e0 = (uint16_t)(y * 64 + 8 * gq);
            for (uint32_t m = want; m != 0u; m &= m - 1u) list[at++] = (uint16_t)(e0 + __builtin_ctz(m));
            n += __builtin_amdgcn_readlane(incl, 63);   // the wave total (scalar)
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    }   // act
    TSTAMP(t_fc1);
    if (lane == 0) { poolN[wid] = n; anyS[wid] = 0; }
    __syncthreads();
    TSTAMP(t_fc2);
    // Phases 3-4 run over the workgroup's pooled survivors (the four cells' lists back to back,
    // thread k on entry k): a cell's ~70 survivors no longer leave most of a wave's second pass
    // idle.  Entry k of cell w lives in wave w's LDS (same layout per wave).
    const int o1 = poolN[0], o2 = o1 + poolN[1], o3 = o2 + poolN[2], tot = o3 + poolN[3];
    auto cell_of = [&](int k, int& kk, int& w) -> unsigned char* {
        w = (int)(k >= o1) + (int)(k >= o2) + (int)(k >= o3);
        kk = k - (w == 0 ? 0 : w == 1 ? o1 : w == 2 ? o2 : o3);
        return dsm + __umul24((uint32_t)w, (uint32_t)waveBytes);
    };

    // 3. full score of the survivors.  The list is in raster order: lanes are row-major over
    //    (row, column group) and each lane appends its group's columns in order.
    for (int k = threadIdx.x; k < tot; k += 256) {
        int kk, w;
        unsigned char* bw = cell_of(k, kk, w);
        const uint8_t* pw = bw;
        const int p = reinterpret_cast<const uint16_t*>(bw + listOff)[kk];
        const int y = p >> 6, x = p & 63;
        const int cc = (y + 3) * PWS + x + 4;
        int q[16];
        q[0] = pw[cc + 3 * PWS];      q[1] = pw[cc + 3 * PWS + 1];
        q[2] = pw[cc + 2 * PWS + 2];  q[3] = pw[cc + PWS + 3];
        q[4] = pw[cc + 3];            q[5] = pw[cc - PWS + 3];
        q[6] = pw[cc - 2 * PWS + 2];  q[7] = pw[cc - 3 * PWS + 1];
        q[8] = pw[cc - 3 * PWS];      q[9] = pw[cc - 3 * PWS - 1];
        q[10] = pw[cc - 2 * PWS - 2]; q[11] = pw[cc - PWS - 3];
        q[12] = pw[cc - 3];           q[13] = pw[cc + PWS - 3];
        q[14] = pw[cc + 2 * PWS - 2]; q[15] = pw[cc + 3 * PWS - 1];
        const int S = fast_score_pk(pw[cc], q);
        if (S >= g.tmin && S > 0) bw[patchBytes + (y + 1) * SCS + x + 1] = (uint8_t)S;
    }
    __syncthreads();

    TSTAMP(t_fc3);
    // 4. local maxima among the scored pixels (neighbours outside the region count as 0)
    for (int k = threadIdx.x; k < tot; k += 256) {
        int kk, w;
        unsigned char* bw = cell_of(k, kk, w);
        const int p = reinterpret_cast<const uint16_t*>(bw + listOff)[kk];
        const int y = p >> 6, x = p & 63;
        const uint8_t* scw = bw + patchBytes;
        const int si = (y + 1) * SCS + x + 1;   // the zero border stands for "outside the region"
        const int s = scw[si];
        int nb = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++) {
#pragma unroll
            for (int dx = -1; dx <= 1; dx++) {
                if (dx == 0 && dy == 0) continue;
                nb = max(nb, (int)scw[si + dy * SCS + dx]);
            }
        }
        const int keep = s > 0 && s > nb ? s : 0;
        bw[kk] = (uint8_t)keep;   // kp of cell w
        if (keep > 0 && keep >= g.iniTh) anyS[w] = 1;
    }
    __syncthreads();
    if (!act) return;
    const bool anyIni = anyS[wid] != 0;

    TSTAMP(t_fc4);
    // 5. keys at the cell's threshold, in raster order
    const int t = anyIni ? g.iniTh : g.minTh;
    uint32_t* out = slots + (size_t)b * g.slotsPerFrame + L.slotBase + (size_t)ci * L.cellCap;
    int nk = 0;
    for (int k0 = 0; k0 < n; k0 += 64) {
        const int k = k0 + lane;
        const int keep = k < n ? (int)kp[k] : 0;
        const bool emit = keep > 0 && keep >= t;
        const uint64_t mask = __ballot(emit);
        const int before = __popcll(mask & ((1ull << lane) - 1ull));
        if (emit && nk + before < L.cellCap) {
            // DistributeOctTree coordinates: absolute - minBorder (R/src/ORBextractor.cpp:889-890)
            const int p = list[k];
            const uint32_t kx = (uint32_t)(rx0 + (p & 63) - kMinBorder), ky = (uint32_t)(ry0 + (p >> 6) - kMinBorder);
            out[nk + before] = kx | (ky << 12) | ((uint32_t)keep << 24);
        }
        nk += __popcll(mask);
    }
    if (lane == 0) {
        if (nk > L.cellCap) { atomicOr(status, 2); nk = L.cellCap; }
        *cnt_out = nk;
    }
#ifdef ORB_TIMING
    if (lane == 0 && b == 0 && (c == 0 || c == 100 || c == 500))
        printf("fast_cell c%d rw %d rh %d n %d keys %d: load+pretest %lld barrier %lld score %lld nms %lld emit %lld\n", c,
               rw, rh, n, nk, t_fc1 - t_fc0, t_fc2 - t_fc1, t_fc3 - t_fc2, t_fc4 - t_fc3, clock64() - t_fc4);
#endif
}

// ------------------------------------------------------------------ A4: octree

constexpr int OT_T = 256;

__device__ __forceinline__ int kx_of(uint32_t k) { return (int)(k & 0xFFFu); }
__device__ __forceinline__ int ky_of(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__device__ __forceinline__ int kr_of(uint32_t k) { return (int)(k >> 24); }

struct NodeTab {     // one table set in LDS (SoA)
    int* start;      // [cap+1]
    int* cnt;
    uint32_t* b0;    // x0 | y0 << 16
    uint32_t* b1;    // x1 | y1 << 16
    int* seq;
    int* flag;       // bit0 nomore, bit1 candidate
};

// Block-wide exclusive scan of an int array in LDS (length m), in place; returns the total.
__device__ int block_scan_lds(int* a, int m, int* wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int chunk = (m + OT_T - 1) / OT_T;
    const int s0 = min(tid * chunk, m), s1 = min(s0 + chunk, m);
    int local = 0;
    for (int i = s0; i < s1; i++) local += a[i];
    int incl = wave_incl_scan_dpp(local);   // (every thread of the workgroup calls it)
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int wofs = 0, total = 0;
    for (int w = 0; w < OT_T / 64; w++) {
        if (w < wid) wofs += wsum[w];
        total += wsum[w];
    }
    int run = wofs + incl - local;
    for (int i = s0; i < s1; i++) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// Splits the node rectangle like ExtractorNode::DivideNode (R/src/ORBextractor.cpp:515-541).
__device__ __forceinline__ void node_split(uint32_t b0, uint32_t b1, int& mx, int& my) {
    const int x0 = (int)(b0 & 0xFFFF), y0 = (int)(b0 >> 16);
    const int x1 = (int)(b1 & 0xFFFF), y1 = (int)(b1 >> 16);
    const int halfX = (int)ceilf((float)(x1 - x0) / 2);
    const int halfY = (int)ceilf((float)(y1 - y0) / 2);
    mx = x0 + halfX;
    my = y0 + halfY;
}
__device__ __forceinline__ void child_bounds(uint32_t b0, uint32_t b1, int q, uint32_t& c0, uint32_t& c1) {
    const int x0 = (int)(b0 & 0xFFFF), y0 = (int)(b0 >> 16);
    const int x1 = (int)(b1 & 0xFFFF), y1 = (int)(b1 >> 16);
    int mx, my;
    node_split(b0, b1, mx, my);
    const int cx0 = (q & 1) ? mx : x0, cx1 = (q & 1) ? x1 : mx;
    const int cy0 = (q & 2) ? my : y0, cy1 = (q & 2) ? y1 : my;
    c0 = (uint32_t)cx0 | ((uint32_t)cy0 << 16);
    c1 = (uint32_t)cx1 | ((uint32_t)cy1 << 16);
}
// quadrant of a key: n1=0 (x<mx,y<my), n2=1 (x>=mx,y<my), n3=2 (x<mx,y>=my), n4=3
__device__ __forceinline__ int key_quadrant(uint32_t key, int mx, int my) {
    return (kx_of(key) < mx ? 0 : 1) | (ky_of(key) < my ? 0 : 2);
}

__device__ __forceinline__ int node_of(const int* start, int m, int k) {
    int lo = 0, hi = m - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (start[mid] <= k) lo = mid; else hi = mid - 1;
    }
    return lo;
}

struct OctScratch {
    uint4* qc;      // [cap+1] per node: key counts of the four children (n1, n2, n3, n4)
    int* ne;        // nonempty children of a processed node (-1: not split this pass)
    int* push;      // push base of a processed node
    int* newpos;    // new list position of an unprocessed node
    int* rank;      // processing rank (final phase)
    int* order;     // node at rank
    int* proc;      // processed flag
    int* tmp;       // scan scratch
    long long* rk;  // [cap] final-phase sort key (count, creation sequence); -1 = not a candidate
};

struct OctCtx {          // LDS carve-up shared by both key-storage variants
    unsigned char* tabBase;
    size_t tabStride;
    int cap;
    __device__ NodeTab tab(int s) const {
        unsigned char* q = tabBase + (size_t)s * tabStride;
        auto r16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
        NodeTab t;
        t.start = (int*)q; q += r16(4 * (size_t)(cap + 1));
        t.cnt = (int*)q; q += r16(4 * (size_t)cap);
        t.b0 = (uint32_t*)q; q += r16(4 * (size_t)cap);
        t.b1 = (uint32_t*)q; q += r16(4 * (size_t)cap);
        t.seq = (int*)q; q += r16(4 * (size_t)cap);
        t.flag = (int*)q;
        return t;
    }
};

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) unsigned long long lds_u64;

__device__ __forceinline__ int quad_field(const uint4& c, int q) {
    return q == 0 ? (int)c.x : q == 1 ? (int)c.y : q == 2 ? (int)c.z : (int)c.w;
}
__device__ __forceinline__ unsigned nonempty_mask(const uint4& c) {
    return (unsigned)(c.x != 0) | ((unsigned)(c.y != 0) << 1) | ((unsigned)(c.z != 0) << 2) | ((unsigned)(c.w != 0) << 3);
}

// DistributeOctTree (R/src/ORBextractor.cpp:571-817) on n keys held in kA, in place: keys never
// move; each key carries the list index of the node that holds it (nid, same storage as kA: LDS
// for the common levels, global memory for very dense ones).  The std::list is emulated at node
// level (ping-pong SoA tables in list order); a pass is
//   1. each key of an active node adds itself to its child quadrant's count (LDS atomics),
//   2. per node: nonempty children, processing order (list order in the breadth-wise passes;
//      (count, creation sequence) descending in the final size-ordered phase, :736), push_front
//      positions, new positions of the nodes left in place,
//   3. each key takes its new node index (child of its node, or the node's new position).
// Within a node the reference keeps vToDistributeKeys order (every DivideNode partition is
// stable), so "first maximum wins" (:796-814) is the maximum response at the smallest original
// index: one 64-bit LDS atomicMax of (response, ~index) per node.
template <typename KP>
__device__ __forceinline__ void octree_run(const Geom& g, const LevelGeom& L, int l, int b, int n, const KP* kA, KP* nid,
                                           const OctCtx& C_, OctScratch& S, int* wsum, int* sc, lds_u64* best,
                                           uint32_t* outK, int* outCount, int* status) {
    const int tid = threadIdx.x;
    const int cap = C_.cap;
    TSTAMP(t_begin);
    long long tK = 0, tN = 0, tO0 = 0, tO1 = 0, tF = 0, tU = 0;
    int np0 = 0, np1 = 0;
    (void)tK; (void)tN; (void)tO0; (void)tO1; (void)tF; (void)tU; (void)np0; (void)np1; (void)l; (void)b;
    // ---- initial nodes (:577-627): part = x / hX; nodes pushed back in part order, empty ones erased
    const int nIni = L.nIni;
    const float hX = L.hX;
    const int H = L.maxBY - kMinBorder;
    for (int i = tid; i < nIni; i += OT_T) S.tmp[i] = 0;
    __syncthreads();
    for (int k = tid; k < n; k += OT_T) atomicAdd(&S.tmp[min((int)((float)kx_of(kA[k]) / hX), nIni - 1)], 1);
    __syncthreads();
    if (tid == 0) {
        const NodeTab T0 = C_.tab(0);
        int idx = 0;
        for (int part = 0; part < nIni; part++) {
            const int c = S.tmp[part];
            S.newpos[part] = idx;
            if (c == 0) continue;
            T0.cnt[idx] = c;
            T0.b0[idx] = (uint32_t)(int)(hX * (float)part);
            T0.b1[idx] = (uint32_t)(int)(hX * (float)(part + 1)) | ((uint32_t)H << 16);
            T0.seq[idx] = idx;
            T0.flag[idx] = c == 1 ? 1 : 0;
            idx++;
        }
        sc[0] = idx;
    }
    __syncthreads();
    // keys k = v * OT_T + tid, v < KV (2,048: most levels' every key) keep the key and its node index
    // in registers for the whole distribution (keys never move): a pass touches memory only for the
    // keys beyond them, where nid / kA live in LDS or, for batches, HBM (L2)
    constexpr int KV = 8;
    uint32_t keyr[KV];
    int nidr[KV];
#pragma unroll
    for (int v = 0; v < KV; v++) {
        const int k = v * OT_T + tid;
        keyr[v] = k < n ? (uint32_t)kA[k] : 0u;
        nidr[v] = k < n ? S.newpos[min((int)((float)kx_of(keyr[v]) / hX), nIni - 1)] : 0;
    }
    for (int k = KV * OT_T + tid; k < n; k += OT_T) nid[k] = (uint32_t)S.newpos[min((int)((float)kx_of(kA[k]) / hX), nIni - 1)];
    TSTAMP(t_init);
    int m = sc[0];   // list size (uniform)
    __syncthreads();
    int cur = 0;     // table holding the current list
    int phase = 0;   // 0 = breadth-wise passes, 1 = size-ordered passes
    int nIter = 0;
    while (true) {
        if (++nIter > 4096) { if (tid == 0) atomicOr(status, 4); break; }
        const NodeTab O = C_.tab(cur);
        const NodeTab Nw = C_.tab(cur ^ 1);
        const int prevSize = m;
#ifdef ORB_TIMING
        if (phase == 0) np0++; else np1++;
#endif
        TSTAMP(t_k);
        // 1. child counts of the active nodes (outer pass: every node with > 1 keys, i.e.
        //    !bNoMore; final phase: the candidates, i.e. children created with > 1 keys)
        for (int i = tid; i < m; i += OT_T) S.qc[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        int ndr[KV];
        uint32_t qr = 0;   // 2 bits per cached key; bit 16 + v: active
#pragma unroll
        for (int v = 0; v < KV; v++) {
            const int k = v * OT_T + tid;
            ndr[v] = 0;
            if (k < n) {
                const int nd = nidr[v];
                ndr[v] = nd;
                const bool act = phase == 0 ? (O.cnt[nd] > 1) : ((O.flag[nd] & 2) != 0);
                if (act) {
                    int mx, my;
                    node_split(O.b0[nd], O.b1[nd], mx, my);
                    const int q = key_quadrant(keyr[v], mx, my);
                    qr |= ((uint32_t)q << (2 * v)) | (1u << (16 + v));
                    atomicAdd(reinterpret_cast<unsigned*>(&S.qc[nd]) + q, 1u);
                }
            }
        }
        for (int k = KV * OT_T + tid; k < n; k += OT_T) {
            const int nd = (int)nid[k];
            const bool act = phase == 0 ? (O.cnt[nd] > 1) : ((O.flag[nd] & 2) != 0);
            if (act) {
                int mx, my;
                node_split(O.b0[nd], O.b1[nd], mx, my);
                atomicAdd(reinterpret_cast<unsigned*>(&S.qc[nd]) + key_quadrant(kA[k], mx, my), 1u);
            }
        }
        __syncthreads();
        TACC(tK, t_k);
        TSTAMP(t_nl);
        // 2. node level: nonempty children of the active nodes
        for (int i = tid; i < m; i += OT_T) {
            const bool act = phase == 0 ? (O.cnt[i] > 1) : ((O.flag[i] & 2) != 0);
            S.ne[i] = act ? __popc(nonempty_mask(S.qc[i])) : -1;
        }
        __syncthreads();
        TACC(tN, t_nl);
        TSTAMP(t_or);
        // processing order + push bases
        if (phase == 0) {
            for (int i = tid; i < m; i += OT_T) S.tmp[i] = S.ne[i] > 0 ? S.ne[i] : 0;
            __syncthreads();
            const int C = block_scan_lds(S.tmp, m, wsum);
            for (int i = tid; i < m; i += OT_T) {
                S.push[i] = S.tmp[i];
                S.proc[i] = S.ne[i] >= 0 ? 1 : 0;
            }
            if (tid == 0) sc[1] = C;
            __syncthreads();
        } else {
            // candidates sorted by (size, pointer) ascending and split from the back (:736-739):
            // rank = number of candidates with a larger (count, creation sequence)
            for (int i = tid; i < m; i += OT_T)
                S.rk[i] = S.ne[i] < 0 ? -1ll : (((long long)O.cnt[i] << 24) | (long long)O.seq[i]);
            if (tid == 0) sc[2] = 0;
            __syncthreads();
            for (int i = tid; i < m; i += OT_T) {
                const long long ki = S.rk[i];
                if (ki < 0) { S.rank[i] = -1; continue; }
                int r = 0, j2 = 0;
                for (; j2 + 8 <= m; j2 += 8) {
#pragma unroll
                    for (int u = 0; u < 8; u++) r += S.rk[j2 + u] > ki ? 1 : 0;
                }
                for (; j2 < m; j2++) r += S.rk[j2] > ki ? 1 : 0;
                S.rank[i] = r;
                S.order[r] = i;
                atomicAdd(&sc[2], 1);
            }
            __syncthreads();
            const int nc = sc[2];
            for (int r = tid; r < nc; r += OT_T) S.tmp[r] = S.ne[S.order[r]];
            __syncthreads();
            block_scan_lds(S.tmp, nc, wsum);
            if (tid == 0) sc[3] = 0x7fffffff;
            __syncthreads();
            // the loop stops after the first split that brings the list to N nodes (:783-784)
            for (int r = tid; r < nc; r += OT_T) {
                const int i = S.order[r];
                S.push[i] = S.tmp[r];
                const int inclNe = S.tmp[r] + S.ne[i];
                if (prevSize + inclNe - (r + 1) >= L.N) atomicMin(&sc[3], r);
            }
            __syncthreads();
            const int jstop = sc[3];
            for (int i = tid; i < m; i += OT_T) S.proc[i] = (S.ne[i] >= 0 && S.rank[i] <= jstop) ? 1 : 0;
            if (tid == 0) {
                int C = 0;
                if (jstop != 0x7fffffff) {
                    const int i = S.order[jstop];
                    C = S.push[i] + S.ne[i];
                } else if (nc > 0) {
                    const int i = S.order[nc - 1];
                    C = S.push[i] + S.ne[i];
                }
                sc[1] = C;
            }
            __syncthreads();
        }
        if (phase == 0) { TACC(tO0, t_or); } else { TACC(tO1, t_or); }
        TSTAMP(t_fi);
        const int C = sc[1];
        // new positions of the nodes left in place (they follow the C pushed children)
        for (int i = tid; i < m; i += OT_T) S.tmp[i] = S.proc[i] ? 0 : 1;
        __syncthreads();
        const int nUnproc = block_scan_lds(S.tmp, m, wsum);
        const int newM = C + nUnproc;
        if (newM > cap) {
            if (tid == 0) atomicOr(status, 8);
            break;
        }
        for (int i = tid; i < m; i += OT_T) S.newpos[i] = S.proc[i] ? -1 : C + S.tmp[i];
        if (tid == 0) sc[4] = 0;
        __syncthreads();
        // fill the new table: children of a processed node at C-1-(push + r) (push_front order)
        for (int i = tid; i < m; i += OT_T) {
            if (!S.proc[i]) {
                const int j2 = S.newpos[i];
                Nw.cnt[j2] = O.cnt[i];
                Nw.b0[j2] = O.b0[i];
                Nw.b1[j2] = O.b1[i];
                Nw.seq[j2] = 0;
                Nw.flag[j2] = O.cnt[i] == 1 ? 1 : 0;
            } else {
                const uint4 cq = S.qc[i];
                int r = 0;
                for (int q = 0; q < 4; q++) {
                    const int cc = quad_field(cq, q);
                    if (cc == 0) continue;
                    const int push = S.push[i] + r;
                    const int j2 = C - 1 - push;
                    uint32_t c0, c1;
                    child_bounds(O.b0[i], O.b1[i], q, c0, c1);
                    Nw.cnt[j2] = cc;
                    Nw.b0[j2] = c0;
                    Nw.b1[j2] = c1;
                    Nw.seq[j2] = push;
                    Nw.flag[j2] = cc == 1 ? 1 : 2;
                    if (cc > 1) atomicAdd(&sc[4], 1);
                    r++;
                }
            }
        }
        TACC(tF, t_fi);
        TSTAMP(t_u);
        // 3. every key takes its node's new index
#pragma unroll
        for (int v = 0; v < KV; v++) {
            const int k = v * OT_T + tid;
            if (k < n) {
                const int nd = ndr[v];
                int nn;
                if (S.proc[nd] && ((qr >> (16 + v)) & 1u)) {
                    const int q = (int)((qr >> (2 * v)) & 3u);
                    const int r = __popc(nonempty_mask(S.qc[nd]) & ((1u << q) - 1u));
                    nn = C - 1 - (S.push[nd] + r);
                } else {
                    nn = S.newpos[nd];
                }
                nidr[v] = nn;
            }
        }
        for (int k = KV * OT_T + tid; k < n; k += OT_T) {
            const int nd = (int)nid[k];
            int nn;
            if (S.proc[nd]) {
                int mx, my;
                node_split(O.b0[nd], O.b1[nd], mx, my);
                const int q = key_quadrant(kA[k], mx, my);
                const int r = __popc(nonempty_mask(S.qc[nd]) & ((1u << q) - 1u));
                nn = C - 1 - (S.push[nd] + r);
            } else {
                nn = S.newpos[nd];
            }
            nid[k] = (uint32_t)nn;
        }
        __syncthreads();
        TACC(tU, t_u);
        const int nToExpand = sc[4];
        cur ^= 1;
        m = newM;
        // termination logic of R/src/ORBextractor.cpp:722-791
        if (m >= L.N || m == prevSize) break;
        if (phase == 0) {
            if (m + nToExpand * 3 > L.N) phase = 1;
        }
        __syncthreads();
    }
    __syncthreads();
    // retain the best point in each node (first max wins, R/src/ORBextractor.cpp:796-814)
    for (int i = tid; i < m; i += OT_T) best[i] = 0ull;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < KV; v++) {
        const int k = v * OT_T + tid;
        if (k < n) {
            const unsigned long long bv = ((unsigned long long)kr_of(keyr[v]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k);
            __hip_atomic_fetch_max(&best[nidr[v]], bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    for (int k = KV * OT_T + tid; k < n; k += OT_T) {
        const unsigned long long v = ((unsigned long long)kr_of(kA[k]) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)k);
        __hip_atomic_fetch_max(&best[(int)nid[k]], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    for (int i = tid; i < m; i += OT_T) {
        const uint32_t k = 0xFFFFFFFFu - (uint32_t)(best[i] & 0xFFFFFFFFull);
        if (i < L.nodeCap) outK[i] = kA[k];
    }
    if (tid == 0) {
        if (m > L.nodeCap) atomicOr(status, 16);
        *outCount = min(m, L.nodeCap);
    }
#ifdef ORB_TIMING
    if (tid == 0 && b == 0 && (l == 0 || l == 7))
        printf("octree l%d n %d m %d: init %lld passes %d+%d K %lld N %lld O0 %lld O1 %lld F %lld U %lld total %lld\n", l, n,
               m, t_init - t_begin, np0, np1, tK, tN, tO0, tO1, tF, tU, clock64() - t_begin);
#endif
}

__global__ __launch_bounds__(OT_T) void k_octree(Geom g, const uint32_t* __restrict__ slots,
                                                 const int* __restrict__ cellCount, uint32_t* __restrict__ keyA,
                                                 uint32_t* __restrict__ keyB, uint32_t* __restrict__ outKeys,
                                                 int* __restrict__ levelCount, int* __restrict__ status,
                                                 int ldsKeyCap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const LevelGeom& L = g.lv[l];
    const int cap = g.maxNodeCap;
    // carve LDS (layout mirrored by octree_lds_bytes on the host)
    unsigned char* p = smem;
    auto carve = [&](size_t bytes) { unsigned char* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    OctScratch S;
    S.qc = (uint4*)carve(sizeof(uint4) * (cap + 1));
    OctCtx C_;
    C_.cap = cap;
    C_.tabStride = ((4 * (size_t)(cap + 1) + 15) & ~(size_t)15) + 5 * ((4 * (size_t)cap + 15) & ~(size_t)15);
    C_.tabBase = carve(2 * C_.tabStride);
    S.ne = (int*)carve(sizeof(int) * cap);
    S.push = (int*)carve(sizeof(int) * cap);
    S.newpos = (int*)carve(sizeof(int) * cap);
    S.rank = (int*)carve(sizeof(int) * cap);
    S.order = (int*)carve(sizeof(int) * cap);
    S.proc = (int*)carve(sizeof(int) * cap);
    S.tmp = (int*)carve(sizeof(int) * (cap + 1));
    S.rk = (long long*)carve(sizeof(long long) * cap);
    lds_u64* best = (lds_u64*)carve(sizeof(unsigned long long) * cap);
    int* cellOff = (int*)carve(sizeof(int) * (L.nCols * L.nRows + 1 + 64));
    int* wsum = (int*)carve(sizeof(int) * 8);
    int* sc = (int*)carve(sizeof(int) * 32);    // uniform scalars
    lds_u32* keysL = (lds_u32*)carve(sizeof(uint32_t) * ldsKeyCap);   // LDS keys + node ids

    const size_t kbase = (size_t)b * g.slotsPerFrame + L.slotBase;
    const int ncell = L.nCols * L.nRows;

    // ---- cell lists -> one contiguous key array (cell order i-major, j-minor)
    for (int c = tid; c < ncell; c += OT_T) cellOff[c] = cellCount[(size_t)b * g.cellsPerFrame + L.cellBase + c];
    __syncthreads();
    const int n = block_scan_lds(cellOff, ncell, wsum);
    if (tid == 0) cellOff[ncell] = n;
    __syncthreads();
    int* outCount = levelCount + (size_t)b * g.nlevels + l;
    uint32_t* outK = outKeys + (size_t)b * g.outPerFrame + L.outBase;
    if (n == 0) {
        if (tid == 0) *outCount = 0;
        return;
    }
    const bool inLds = 2 * n <= ldsKeyCap;   // typical levels hold a few thousand keys
    {
        // one thread per key (independent loads, all in flight): cell by binary search
        const uint32_t* src = slots + kbase;
        uint32_t* kg = keyA + kbase;
        for (int k0 = 0; k0 < n; k0 += OT_T * 4) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int k = k0 + u * OT_T + tid;
                v[u] = 0;
                if (k < n) {
                    int lo = 0, hi = ncell - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (cellOff[mid] <= k) lo = mid; else hi = mid - 1;
                    }
                    v[u] = src[(size_t)lo * L.cellCap + (k - cellOff[lo])];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int k = k0 + u * OT_T + tid;
                if (k < n) {
                    if (inLds) keysL[k] = v[u];
                    else kg[k] = v[u];
                }
            }
        }
    }
    __syncthreads();
    if (inLds)
        octree_run<lds_u32>(g, L, l, b, n, keysL, keysL + n, C_, S, wsum, sc, best, outK, outCount, status);
    else
        octree_run<uint32_t>(g, L, l, b, n, keyA + kbase, keyB + kbase, C_, S, wsum, sc, best, outK, outCount, status);
}

// ------------------------------------------------------------------ A6: blur

// Separable 7-tap integer blur; every LDS access is dword-aligned (the compiler otherwise
// merges neighbouring byte reads into ds_read_u16 at odd addresses, which mis-read on gfx950).
constexpr int kHalo = 3;   // blur radius
constexpr int kLdsW = kTileW + 2 * kHalo, kLdsH = kTileH + 2 * kHalo;
constexpr int kRowSumW = kTileW + 4;
__global__ __launch_bounds__(256) void k_blur(Geom g, const uint8_t* __restrict__ pyr, L0Src z,
                                              uint8_t* __restrict__ blurred, int k0, int k1, int k2, int k3) {
    __shared__ __attribute__((aligned(16))) uint32_t tile32[kLdsH][(kLdsW + 2) / 4];
    __shared__ __attribute__((aligned(16))) int rowsum[kLdsH][kRowSumW];
    const int b = blockIdx.y;
    const int l = level_of_tile(g, blockIdx.x);
    const LevelGeom& L = g.lv[l];
    const int t = blockIdx.x - L.tileBase;
    const int tx0 = (t % L.tilesX) * kTileW, ty0 = (t / L.tilesX) * kTileH;
    int ipitch;
    uint32_t ibytes;
    const uint8_t* img = level_img(g, z, pyr, b, l, ipitch, ibytes);
    uint8_t* out = blurred + (size_t)b * g.frameBytes + L.off;
    const int tid = threadIdx.x;
    constexpr int kWords = (kLdsW + 2) / 4;   // 18 words = 72 bytes per row, from column tx0 - 4
    // interior tiles read aligned dwords; tiles touching a level edge apply BORDER_REFLECT_101 per byte
    const bool interior = tx0 >= 4 && tx0 + kTileW + kHalo < L.w && ty0 >= kHalo && ty0 + kTileH + kHalo <= L.h;
    for (int i = tid; i < kLdsH * kWords; i += 256) {
        const int r = i / kWords, wd = i % kWords;
        uint32_t v = 0;
        if (interior) {
            v = *reinterpret_cast<const uint32_t*>(img + (size_t)(ty0 - kHalo + r) * ipitch + tx0 - 4 + 4 * wd);
        } else {
            const int y = reflect101(ty0 - kHalo + r, L.h);
            const uint8_t* row = img + (size_t)y * ipitch;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int x = reflect101(tx0 - 4 + 4 * wd + k, L.w);
                v |= (uint32_t)row[x] << (8 * k);
            }
        }
        tile32[r][wd] = v;
    }
    __syncthreads();
    const int kk[7] = {k3, k2, k1, k0, k1, k2, k3};
    for (int i = tid; i < kLdsH * (kTileW / 4); i += 256) {
        const int r = i / (kTileW / 4), gq = i % (kTileW / 4);
        const uint32_t w0 = tile32[r][gq], w1 = tile32[r][gq + 1], w2 = tile32[r][gq + 2];
        int px[12];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            px[k] = (w0 >> (8 * k)) & 0xff;
            px[4 + k] = (w1 >> (8 * k)) & 0xff;
            px[8 + k] = (w2 >> (8 * k)) & 0xff;
        }
    int4 s4;
        int sv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int s = 0;
#pragma unroll
            for (int q = 0; q < 7; q++) s += kk[q] * px[k + 1 + q];
            sv[k] = s;
        }
        s4.x = sv[0]; s4.y = sv[1]; s4.z = sv[2]; s4.w = sv[3];
        *reinterpret_cast<int4*>(&rowsum[r][gq * 4]) = s4;
    }
    __syncthreads();
    const int ly = tid / 16, lx0 = (tid % 16) * 4;
    const int y = ty0 + ly;
    if (y >= L.h) return;
    int acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 7; q++) {
        const int4 v = *reinterpret_cast<const int4*>(&rowsum[ly + q][lx0]);
        acc[0] += kk[q] * v.x;
        acc[1] += kk[q] * v.y;
        acc[2] += kk[q] * v.z;
        acc[3] += kk[q] * v.w;
    }
    // acc >= 0: unsigned shift + min.  (A signed clamp-of-ashr pair is lowered by ROCm 7.2 to
    // v_ashr_pk_u8_i32, whose untouched high half then leaks into the packed word.)
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t v = min(((uint32_t)acc[k] + (1u << 15)) >> 16, 255u);
        packed |= v << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(out + (size_t)y * L.pitch + tx0 + lx0) = packed;
}

// ------------------------------------------------------------------ A5/A7: orientation + descriptor

__device__ float fast_atan2_dev(float y, float x) {
    const double RAD2DEG = 180.0 / 3.14159265358979323846;
    const float p1 = 0.9997878412794807f * (float)RAD2DEG;
    const float p3 = -0.3258083974640975f * (float)RAD2DEG;
    const float p5 = 0.1555786518463281f * (float)RAD2DEG;
    const float p7 = -0.04432655554792128f * (float)RAD2DEG;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313080847e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313080847e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// glibc 2.35 x86_64 sinf/cosf (FMA variant) restated for |y| < 120 — see DESIGN.md §sincosf.
struct SinCosTab { double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4; };
__constant__ SinCosTab c_sct[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
};
__device__ __forceinline__ float sin_poly(double x, double x2, const SinCosTab& p) {
    const double x3 = x * x2;
    const double s1 = __fma_rn(x2, p.s3, p.s2);
    const double x5 = x2 * x3;
    const double s = __fma_rn(x3, p.s1, x);
    return (float)__fma_rn(s1, x5, s);
}
__device__ __forceinline__ float cos_poly(double x2, const SinCosTab& p) {
    const double x4 = x2 * x2;
    const double c1 = __fma_rn(x2, p.c1, p.c0);
    const double c2 = __fma_rn(x2, p.c4, p.c3);
    const double x6 = x2 * x4;
    const double c = __fma_rn(x4, p.c2, c1);
    return (float)__fma_rn(c2, x6, c);
}
__device__ void glibc_sincosf(float y, float& s, float& c) {
    const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ff;
    const double x = (double)y;
    if (top < 0x3f4) {
        if (top < 0x398) { s = y; c = 1.0f; return; }
        const double x2 = x * x;
        s = sin_poly(x, x2, c_sct[0]);
        c = cos_poly(x2, c_sct[0]);
        return;
    }
    const double r = x * c_sct[0].hpi_inv;
    const int n = (((int)r) + 0x800000) >> 24;
    const double xr = __fma_rn(-(double)n, c_sct[0].hpi, x);
    const double x2 = xr * xr;
    const SinCosTab& q = c_sct[(n & 2) ? 1 : 0];
    const double xs = xr * c_sct[0].sign[n & 3];
    if ((n & 1) == 0) {
        s = sin_poly(xs, x2, q);
        c = cos_poly(x2, q);
    } else {
        s = cos_poly(x2, q);
        c = sin_poly(xs, x2, q);
    }
}

// Fused A5 + A6 + A7 + A8, one wave per retained keypoint (4 per workgroup):
//  1. the raw level patch rows y-21..y+21, columns x-24..x+23 is staged in LDS (dword loads,
//     realigned; BORDER_REFLECT_101 per byte for the few keypoints within 21 px of an edge);
//  2. IC_Angle (R/src/ORBextractor.cpp:79-108) from the patch: per row and dword,
//     v_dot4_u32_u8 against (u + 16) and 1 weights masked to |u| <= umax[|v|];
//  3. the 7x7 Gaussian (8-bit kernel, R :1166-1167) only where the descriptor samples: the
//     horizontal pass over the 43 x 37 window (two dot4 per output, u16 row sums <= 65535),
//     the vertical pass per sample point — the same integer sums as the full-image filter;
//  4. steered BRIEF (R :113-155) with glibc sincosf, 4 ballots -> 32 bytes.
constexpr int kOdPW = 48;                // patch row stride (bytes): columns x-24 .. x+23
constexpr int kOdRows = 43;              // rows y-21 .. y+21
constexpr int kOdRsW = 42;               // row-sum stride (u16): columns x-18 .. x+18 (37 used; 8-column tasks end at 41)
// The horizontal pass's tasks: row r (<< 8) and the first of 8 output columns c0 (even), covering
// per row the columns a rotated pattern sample can need: a sample (X, Y) = the rounded rotation of a
// pattern point lies within R = max pattern radius (18.38) + 0.75 of the keypoint (rounding moves
// each coordinate by <= 0.5), and RS row r feeds the samples with |Y - (r - 21)| <= 3, so row r needs
// |X| <= sqrt(R^2 - max(0, |r - 21| - 3)^2).  189 tasks (3 per lane; the full 43 x 37 grid in 4-column
// tasks was 430, 7 per lane); 0xffff pads.  Generated from orb_pattern.inc.
__constant__ uint16_t c_htask[192] = {
    0x000c, 0x0014, 0x010a, 0x0112, 0x011a, 0x0208, 0x0210, 0x0218, 0x0306, 0x030e, 0x0316, 0x0404,
    0x040c, 0x0414, 0x041c, 0x0504, 0x050c, 0x0514, 0x051c, 0x0604, 0x060c, 0x0614, 0x061c, 0x0702,
    0x070a, 0x0712, 0x071a, 0x0802, 0x080a, 0x0812, 0x081a, 0x0822, 0x0902, 0x090a, 0x0912, 0x091a,
    0x0922, 0x0a00, 0x0a08, 0x0a10, 0x0a18, 0x0a20, 0x0b00, 0x0b08, 0x0b10, 0x0b18, 0x0b20, 0x0c00,
    0x0c08, 0x0c10, 0x0c18, 0x0c20, 0x0d00, 0x0d08, 0x0d10, 0x0d18, 0x0d20, 0x0e00, 0x0e08, 0x0e10,
    0x0e18, 0x0e20, 0x0f00, 0x0f08, 0x0f10, 0x0f18, 0x0f20, 0x1000, 0x1008, 0x1010, 0x1018, 0x1020,
    0x1100, 0x1108, 0x1110, 0x1118, 0x1120, 0x1200, 0x1208, 0x1210, 0x1218, 0x1220, 0x1300, 0x1308,
    0x1310, 0x1318, 0x1320, 0x1400, 0x1408, 0x1410, 0x1418, 0x1420, 0x1500, 0x1508, 0x1510, 0x1518,
    0x1520, 0x1600, 0x1608, 0x1610, 0x1618, 0x1620, 0x1700, 0x1708, 0x1710, 0x1718, 0x1720, 0x1800,
    0x1808, 0x1810, 0x1818, 0x1820, 0x1900, 0x1908, 0x1910, 0x1918, 0x1920, 0x1a00, 0x1a08, 0x1a10,
    0x1a18, 0x1a20, 0x1b00, 0x1b08, 0x1b10, 0x1b18, 0x1b20, 0x1c00, 0x1c08, 0x1c10, 0x1c18, 0x1c20,
    0x1d00, 0x1d08, 0x1d10, 0x1d18, 0x1d20, 0x1e00, 0x1e08, 0x1e10, 0x1e18, 0x1e20, 0x1f00, 0x1f08,
    0x1f10, 0x1f18, 0x1f20, 0x2000, 0x2008, 0x2010, 0x2018, 0x2020, 0x2102, 0x210a, 0x2112, 0x211a,
    0x2122, 0x2202, 0x220a, 0x2212, 0x221a, 0x2222, 0x2302, 0x230a, 0x2312, 0x231a, 0x2404, 0x240c,
    0x2414, 0x241c, 0x2504, 0x250c, 0x2514, 0x251c, 0x2604, 0x260c, 0x2614, 0x261c, 0x2706, 0x270e,
    0x2716, 0x2808, 0x2810, 0x2818, 0x290a, 0x2912, 0x291a, 0x2a0c, 0x2a14, 0xffff, 0xffff, 0xffff,
};
constexpr int kOdWaveBytes = kOdRows * kOdPW + kOdRows * kOdRsW * 2;
#ifndef ORB_OD_KPW
#define ORB_OD_KPW 2
#endif
// keypoint slots per wave (even): a slot's window loads overlap the previous slot's work
constexpr int kOdKpw = ORB_OD_KPW;
static_assert(kOdKpw % 2 == 0, "two register sets in turn");

// (six waves per SIMD: 80 VGPRs instead of 82, no spills; the LDS of six workgroups fits; the
// kernel is latency-bound, +0.6 % on the step, same-box A/B)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_orient_desc(Geom g, const uint8_t* __restrict__ pyr, L0Src z,
                                                     const uint32_t* __restrict__ outKeys,
                                                     const int* __restrict__ levelCount, orb_keypoint* __restrict__ kps,
                                                     uint8_t* __restrict__ desc, int cap, int32_t* __restrict__ counts,
                                                     uint32_t kA, uint32_t kB) {
    __shared__ __attribute__((aligned(16))) unsigned char od_sm[4][kOdWaveBytes];
    // IC_Angle's per-(row v, dword d) byte masks |4d + j - 16| <= umax[|v|] (step 2), built once
    // per workgroup before any wave can leave
    __shared__ uint32_t momMask[31 * 8];
    if (threadIdx.x < 31 * 8) {
        const int v = (int)(threadIdx.x >> 3) - 15, d = threadIdx.x & 7;
        const int um = g.umax[abs(v)];
        const int ja = max(0, 16 - um - 4 * d), jb = min(3, 16 + um - 4 * d);
        momMask[threadIdx.x] =
            ja > jb ? 0u : (0xFFFFFFFFu << (8 * min(ja, 3))) & (0xFFFFFFFFu >> (8 * (3 - max(jb, 0))));
    }
    __syncthreads();
    // the wave index is uniform: readfirstlane keeps it (and the level / cell / geometry derived
    // from it) in SGPRs, so g.lv[l] fields are scalar loads instead of per-lane flat loads
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int bx, b;
    xcd_block_2d(bx, b);
    const int q0 = (bx * 4 + wid) * kOdKpw;
    const int* lc = levelCount + (size_t)b * g.nlevels;
    if (q0 == 0 && lane == 0) {
        int tot = 0;
        for (int l = 0; l < g.nlevels; l++) tot += lc[l];
        counts[b] = tot;
    }
    uint32_t* P32 = reinterpret_cast<uint32_t*>(od_sm[wid]);
    uint16_t* RS = reinterpret_cast<uint16_t*>(od_sm[wid] + kOdRows * kOdPW);
    TSTAMP(t_od0);

    // the horizontal pass's task words and this lane's BRIEF point pairs: loaded first, so their
    // latency hides under the window load and the moments (neither depends on the angle); both
    // keypoints of the wave use them
    uint32_t task[3];
#pragma unroll
    for (int it = 0; it < 3; it++) task[it] = c_htask[lane + 64 * it];
    float4 ppair[4];
#pragma unroll
    for (int r = 0; r < 4; r++) ppair[r] = reinterpret_cast<const float4*>(c_patternf.v)[r * 64 + lane];

    // A keypoint slot: its level, output index and position, and (interior windows) the lane's
    // eleven window dwords, loaded as soon as the slot is known - the second keypoint's loads are
    // in flight while the first one is processed
    struct OdKey {
        int valid, l, outIdx, x, y, resp, pitch, interior, sh;
        uint32_t imgBytes;
        const uint8_t* img;
        uint32_t a[(kOdRows + 3) / 4];
    };
    const int r0 = lane / 13, kd = lane - 13 * r0;   // lane = (row r0 of 4 per pass, source dword kd of 13)
    auto setup = [&](int q, OdKey& k) {
        k.valid = 0;
        if (q >= g.outPerFrame) return;
        int l = 0;
        while (l + 1 < g.nlevels && q >= g.lv[l + 1].outBase) l++;
        const LevelGeom& L = g.lv[l];
        const int local = q - L.outBase;
        if (local >= lc[l]) return;
        int outIdx = local;
        for (int l2 = 0; l2 < l; l2++) outIdx += lc[l2];
        if (outIdx >= cap) return;
        const uint32_t key = outKeys[(size_t)b * g.outPerFrame + q];
        k.l = l;
        k.outIdx = outIdx;
        k.x = kx_of(key) + kMinBorder;
        k.y = ky_of(key) + kMinBorder;
        k.resp = kr_of(key);
        k.img = level_img(g, z, pyr, b, l, k.pitch, k.imgBytes);
        k.interior = k.x - 24 >= 0 && k.x + 24 <= L.w && k.y - 21 >= 0 && k.y + 21 < L.h;
        k.sh = 0;
        if (k.interior) {
            // one buffer load per pass at a scalar row offset (rows past the window, or past the
            // slab, read harmlessly and are never stored)
            const int gx0 = k.x - 24, ga = gx0 & ~3;
            k.sh = gx0 - ga;
            const uint32_t winOff = (uint32_t)(k.y - 21) * (uint32_t)k.pitch + (uint32_t)ga;
            const __amdgpu_buffer_rsrc_t rs = buf_rsrc(k.img + winOff, k.imgBytes - winOff);
            const uint32_t laneOff = __umul24((uint32_t)r0, (uint32_t)k.pitch) + 4u * (uint32_t)kd;
#pragma unroll
            for (int u = 0; u < (kOdRows + 3) / 4; u++)
                k.a[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)laneOff, 4 * u * k.pitch, 0);
        }
        k.valid = 1;
    };
    auto process = [&](const OdKey& k) {
        if (!k.valid) return;
        const int l = k.l, x = k.x, y = k.y, resp = k.resp, outIdx = k.outIdx, pitch = k.pitch;
        const uint8_t* img = k.img;
        const LevelGeom& L = g.lv[l];
        // 1. patch: the next dword of the row from the next lane by DPP wave_shl:1, the realigned
        //    dword stored (lanes with no patch dword write into the row-sum area, which step 3a
        //    overwrites)
        if (k.interior) {
            uint32_t* const sink = reinterpret_cast<uint32_t*>(RS) + lane;
    #pragma unroll
            for (int u = 0; u < (kOdRows + 3) / 4; u++) {
                const uint32_t a = k.a[u];
                const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x130, 0xF, 0xF, false);
                const int r = 4 * u + r0;
                const bool st = r0 < 4 && kd < 12 && r < kOdRows;
                *(st ? P32 + r * 12 + kd : sink) = __builtin_amdgcn_alignbyte(nx, a, (uint32_t)k.sh);
            }
        } else {   // within 21 / 24 px of an edge: BORDER_REFLECT_101 per byte
            uint8_t* P8w = od_sm[wid];
            for (int t = lane; t < kOdRows * kOdPW; t += 64) {
                const int r = t / kOdPW, cc = t % kOdPW;
                P8w[t] = img[(size_t)reflect101(y - 21 + r, L.h) * pitch + reflect101(x - 24 + cc, L.w)];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

        TSTAMP(t_od1);
        // 2. moments: lane = (row group vr, dword d); patch dword 2+d holds u = 4d-16 .. 4d-13
        int m10 = 0, m01 = 0;
        {
            const int d = lane & 7, vr = lane >> 3;
            for (int it = 0; it < 4; it++) {
                const int v = it * 8 + vr - 15;
                if (v > 15) continue;
                // bytes j with |4d + j - 16| <= umax[|v|], i.e. j in [16 - um - 4d, 16 + um - 4d] ∩ [0, 3]
                const uint32_t m = momMask[(v + 15) * 8 + d];
                const uint32_t w1 = m & 0x01010101u;
                const uint32_t wu = m & (0x03020100u + (uint32_t)(4 * d) * 0x01010101u);   // bytes u + 16 = 4d + j
                const uint32_t pw = P32[(21 + v) * 12 + 2 + d];
                const int s1 = (int)__builtin_amdgcn_udot4(pw, w1, 0u, false);
                m10 += (int)__builtin_amdgcn_udot4(pw, wu, 0u, false) - 16 * s1;
                m01 += v * s1;
            }
        }
        m10 = wave_sum_dpp(m10);
        m01 = wave_sum_dpp(m01);
        const float angle = fast_atan2_dev((float)m01, (float)m10);

        TSTAMP(t_od2);
        // 3a. horizontal Gaussian pass: RS[r][c] = sum_q k_q * raw(y-21+r, x-18+c-3+q) on the columns
        //     the pattern can reach (c_htask).  Task (r, c0) computes columns c0 .. c0+7 from the 16
        //     patch bytes c0+3 .. c0+18, re-based by four alignbytes at the task's byte offset; output i
        //     takes bytes c0+3+i .. +6 (taps -3 .. 0, kA) and c0+7+i .. +10 (taps +1 .. +3, kB).
        //     (Tried: the whole 43 x 37 pass on the matrix cores, RS^T = Gh^T P^T by nine
        //     v_mfma_i32_16x16x64_i8 over the i8-biased window and a host-built banded tap matrix —
        //     bit-exact, 17 % fewer VALU per keypoint, but the extraction step 3-5 % slower in
        //     same-box A/B runs, with 16-bit or 8-byte row-sum stores alike; kept out.)
        {
    #pragma unroll
            for (int it = 0; it < 3; it++) {
                if (task[it] == 0xFFFFu) continue;
                const int r = (int)(task[it] >> 8), c0 = (int)(task[it] & 0xFFu);
                const int o = c0 + 3;
                const uint32_t* row = P32 + r * 12 + (o >> 2);
                const uint32_t sh = (uint32_t)(o & 3);
                uint32_t d[5];
    #pragma unroll
                for (int k = 0; k < 5; k++) d[k] = row[k];   // (past the row: bytes of unused columns)
                uint32_t w[4];
    #pragma unroll
                for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
                uint32_t out[4] = {0u, 0u, 0u, 0u};
    #pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t A = (i & 3) == 0 ? w[i >> 2] : __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], i & 3);
                    const int j = i + 4;
                    const uint32_t B = (j & 3) == 0 ? w[j >> 2] : __builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], j & 3);
                    const uint32_t sum = __builtin_amdgcn_udot4(B, kB, __builtin_amdgcn_udot4(A, kA, 0u, false), false);
                    out[i >> 1] |= sum << (16 * (i & 1));
                }
                uint32_t* rs32 = reinterpret_cast<uint32_t*>(RS + r * kOdRsW + c0);
    #pragma unroll
                for (int k = 0; k < 4; k++) rs32[k] = out[k];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

        TSTAMP(t_od3);
        // 3b + 4. steered BRIEF: blurred(y+Y, x+X) = (sum_q k_q RS[Y+18+q][X+18] + 2^15) >> 16
        float bs, ac;
        glibc_sincosf(angle * g.factorPI, bs, ac);
        const float a = ac, bb = bs;
        const int k0 = (int)(kA & 0xff), k1 = (int)((kA >> 8) & 0xff), k2 = (int)((kA >> 16) & 0xff),
                  k3 = (int)(kA >> 24);   // taps 0..3 (3 = centre); taps 4..6 mirror 2..0
        // The rotated offsets of a pair's two points at once in packed f32 (v_pk_mul_f32 / v_pk_add_f32:
        // the same IEEE products and sums as the scalar form x a - y b, x b + y a, fp-contract off),
        // cvRound by the 1.5 * 2^23 magic add (round-half-even for |x| < 2^22), and the row-sum address
        // from the magic-biased bit patterns directly: __umul24 reads Y + 2^22 from the low 24 bits and
        // the biases fold into one constant (mod 2^32).  The vertical taps pair up (0, 6), (1, 5),
        // (2, 4) for v_dot2_u32_u16; the integer sum is the same.
        typedef float f2 __attribute__((ext_vector_type(2)));
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const f2 av = {a, a}, bv = {bb, bb};
        const uint32_t kk0 = (uint32_t)k0 * 0x10001u, kk1 = (uint32_t)k1 * 0x10001u, kk2 = (uint32_t)k2 * 0x10001u;
        constexpr uint32_t kMagicBits = 0x4B400000u;   // bits of 1.5 * 2^23
        constexpr uint32_t kRsOff = 2u * (18u * kOdRsW + 18u) - 2u * kOdRsW * (kMagicBits & 0xFFFFFFu) - 2u * kMagicBits;
        const f2 magic = {12582912.0f, 12582912.0f};
        // acc of one point, clamped so that acc >> 16 is the saturated blurred value (the 8-bit taps
        // sum to 257, so an unclamped sum can reach 257 << 16)
        auto sample = [&](uint32_t xb, uint32_t yb) -> uint32_t {
            const uint32_t off = __umul24(yb, 2u * kOdRsW) + (2u * xb + kRsOff);   // 2 ((Y + 18) kOdRsW + X + 18)
            const uint16_t* c0 = reinterpret_cast<const uint16_t*>(reinterpret_cast<const unsigned char*>(RS) + off);
            const uint32_t p06 = (uint32_t)c0[0] | ((uint32_t)c0[6 * kOdRsW] << 16);
            const uint32_t p15 = (uint32_t)c0[kOdRsW] | ((uint32_t)c0[5 * kOdRsW] << 16);
            const uint32_t p24 = (uint32_t)c0[2 * kOdRsW] | ((uint32_t)c0[4 * kOdRsW] << 16);
            uint32_t acc = __umul24((uint32_t)k3, (uint32_t)c0[3 * kOdRsW]) + (1u << 15);
            acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p06), __builtin_bit_cast(u16x2, kk0), acc, false);
            acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p15), __builtin_bit_cast(u16x2, kk1), acc, false);
            acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p24), __builtin_bit_cast(u16x2, kk2), acc, false);
            return min(acc, 0x00FFFFFFu);
        };
        uint64_t words[4];
    #pragma unroll
        for (int r = 0; r < 4; r++) {
            const float4 pp = ppair[r];   // pair r * 64 + lane (byte pi/8, bit pi%8): (x0, x1, y0, y1)
            const f2 px = {pp.x, pp.y}, py = {pp.z, pp.w};
            const f2 xf = px * av - py * bv, yf = px * bv + py * av;
            const f2 xm = xf + magic, ym = yf + magic;
            const uint32_t s0 = sample(__float_as_uint(xm.x), __float_as_uint(ym.x));
            const uint32_t s1 = sample(__float_as_uint(xm.y), __float_as_uint(ym.y));
            // blurred(p0) < blurred(p1) <=> acc0 < (acc1 with its low 16 bits cleared)
            words[r] = __ballot(s0 < (s1 & 0xFFFF0000u));
        }
    #ifdef ORB_TIMING
        if (lane == 0 && b == 0 && (k.outIdx == 0 || k.outIdx == 300 || k.outIdx == 700))
            printf("orient_desc q%d: patch %lld moments %lld hpass %lld brief %lld\n", k.outIdx, t_od1 - t_od0, t_od2 - t_od1,
                   t_od3 - t_od2, clock64() - t_od3);
    #endif
        if (lane < 4) {
            uint64_t wv = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
            reinterpret_cast<uint64_t*>(desc + ((size_t)b * cap + outIdx) * 32)[lane] = wv;
        }
        if (lane == 0) {
            orb_keypoint kp;
            kp.x = (float)x;
            kp.y = (float)y;
            if (l != 0) {
                kp.x = kp.x * L.scale;
                kp.y = kp.y * L.scale;
            }
            kp.size = L.size;
            kp.angle = angle;
            kp.response = (float)resp;
            kp.octave = l;
            kp.class_id = -1;
            kps[(size_t)b * cap + outIdx] = kp;
        }
    };
    // two register sets in turn: a slot's window loads are issued one slot ahead; each slot
    // reuses the wave's LDS (its window stores follow the previous slot's reads)
    OdKey k0, k1;
    setup(__builtin_amdgcn_readfirstlane(q0), k0);
    setup(__builtin_amdgcn_readfirstlane(q0 + 1), k1);
    for (int t = 0; t < kOdKpw; t += 2) {
        process(k0);
        if (t + 2 < kOdKpw) setup(__builtin_amdgcn_readfirstlane(q0 + t + 2), k0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        process(k1);
        if (t + 3 < kOdKpw) setup(__builtin_amdgcn_readfirstlane(q0 + t + 3), k1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// Compaction of per-frame rows stored at a capacity stride (keypoints 28 B, descriptors 32 B,
// matches12 4 B) into one contiguous run: workgroup b copies min(counts[b], cap) rows of frame b
// to the exclusive prefix of the clamped counts of frames < b (every workgroup sums them itself:
// no second launch, no inter-workgroup order).  Rows are whole dwords.
__global__ __launch_bounds__(256) void k_pack_rows(const uint32_t* __restrict__ src, int rowWords, int cap,
                                                   const int32_t* __restrict__ counts, int B, uint32_t* __restrict__ dst,
                                                   int32_t* __restrict__ offsets) {
    __shared__ int sOff;
    const int b = blockIdx.x;
    if (threadIdx.x == 0) sOff = 0;
    __syncthreads();
    int part = 0;
    for (int i = threadIdx.x; i < b; i += 256) part += min(max(counts[i], 0), cap);
    part = wave_sum_dpp(part);
    if ((threadIdx.x & 63) == 0 && part) atomicAdd(&sOff, part);
    __syncthreads();
    const int off = sOff, n = min(max(counts[b], 0), cap);
    if (threadIdx.x == 0) {
        offsets[b] = off;
        if (b == B - 1) offsets[B] = off + n;
    }
    const uint32_t* s = src + (size_t)b * cap * rowWords;
    uint32_t* d = dst + (size_t)off * rowWords;
    for (int t = threadIdx.x; t < n * rowWords; t += 256) d[t] = s[t];
}

// Copies B packed w x h frames into the pitched level-0 slots of the pyramid slab: 16 bytes
// per thread when rows are 16-byte aligned (w % 16 == 0 and an aligned source), else bytes.
__global__ __launch_bounds__(256) void k_load_frames(Geom g, const uint8_t* __restrict__ src, size_t frameStride,
                                                     uint8_t* __restrict__ pyr, int vec16) {
    const int b = blockIdx.y;
    const LevelGeom& L = g.lv[0];
    const uint8_t* s = src + (size_t)b * frameStride;
    uint8_t* d = pyr + (size_t)b * g.frameBytes + L.off;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (vec16) {
        const int perRow = L.w / 16;
        if (i >= perRow * L.h) return;
        const int y = i / perRow, x = (i % perRow) * 16;
        *reinterpret_cast<uint4*>(d + (size_t)y * L.pitch + x) = *reinterpret_cast<const uint4*>(s + (size_t)y * L.w + x);
    } else {
        const int perRow = (L.w + 3) / 4;
        if (i >= perRow * L.h) return;
        const int y = i / perRow, x = (i % perRow) * 4;
        uint32_t v = 0;
        for (int k = 0; k < 4; k++)
            if (x + k < L.w) v |= (uint32_t)s[(size_t)y * L.w + x + k] << (8 * k);
        *reinterpret_cast<uint32_t*>(d + (size_t)y * L.pitch + x) = v;
    }
}

// ------------------------------------------------------------------ stereo: Frame::ComputeStereoMatches

struct StereoTabs {
    float scale[kMaxLevels], inv[kMaxLevels];
};

// One wave per left keypoint (R/src/Frame.cpp:551-747): right keypoints of the row band
// [floor(y - 2s), ceil(y + 2s)] (vRowIndices, ascending index), octave within +-1 and
// uL - maxD <= uR <= uL; best Hamming distance (strict <, below TH_HIGH); if below
// (TH_HIGH+TH_LOW)/2, the 11 x 11 SAD (centre-normalised windows, cv::norm L1 of integer-valued
// floats = exact integer sums) at 11 offsets on the keypoint's level, parabola fit and the
// disparity gate.  Pair p's left / right data: kL + p*kStride etc.; pyramids pyrL + p*pyStride.
__global__ __launch_bounds__(256) void k_stereo_match(Geom g, StereoTabs tb, const uint8_t* __restrict__ pyrL,
                                                      const uint8_t* __restrict__ pyrR, size_t pyStride, L0Src zL,
                                                      L0Src zR,
                                                      const orb_keypoint* __restrict__ kL, const uint8_t* __restrict__ dL,
                                                      const int32_t* __restrict__ nLs, const orb_keypoint* __restrict__ kR,
                                                      const uint8_t* __restrict__ dR, const int32_t* __restrict__ nRs,
                                                      int kStride, int cntStride, int kCap, float mbf, float maxD,
                                                      float* __restrict__ ur, float* __restrict__ depth,
                                                      int32_t* __restrict__ sad, int outStride) {
    __shared__ int rowsad[4][128];
    // the wave index is uniform: readfirstlane keeps it (and the level / cell / geometry derived
    // from it) in SGPRs, so g.lv[l] fields are scalar loads instead of per-lane flat loads
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int p = blockIdx.y;
    const int iL = blockIdx.x * 4 + wid;
    const int nl = nLs[(size_t)p * cntStride], nr = nRs[(size_t)p * cntStride];
    if (iL >= min(nl, kCap)) return;
    const orb_keypoint* KL = kL + (size_t)p * kStride;
    const orb_keypoint* KR = kR + (size_t)p * kStride;
    float* UR = ur + (size_t)p * outStride;
    float* DP = depth + (size_t)p * outStride;
    int32_t* SD = sad + (size_t)p * outStride;
    const orb_keypoint kp = KL[iL];
    const int levelL = kp.octave;
    const float uL = kp.x, vL = kp.y;
    const int row = (int)vL;   // vRowIndices[vL]: float -> size_t
    const float minU = uL - maxD, maxU = uL;   // minD = 0
    bool done = maxU < 0 || row < 0 || row >= g.lv[0].h || levelL < 0 || levelL >= g.nlevels;
    unsigned long long best = ~0ull;
    if (!done) {
        const uint4* q4 = reinterpret_cast<const uint4*>(dL + ((size_t)p * kStride + iL) * 32);
        const uint4 qa = q4[0], qb = q4[1];
        for (int j0 = 0; j0 < min(nr, kCap); j0 += 64) {
            const int j = j0 + lane;
            unsigned long long key = ~0ull;
            if (j < min(nr, kCap)) {
                const orb_keypoint k2 = KR[j];
                const float r = 2.0f * tb.scale[k2.octave];
                const int maxr = (int)ceilf(k2.y + r), minr = (int)floorf(k2.y - r);
                if (row >= minr && row <= maxr && k2.octave >= levelL - 1 && k2.octave <= levelL + 1 && k2.x >= minU &&
                    k2.x <= maxU) {
                    const uint4* d4 = reinterpret_cast<const uint4*>(dR + ((size_t)p * kStride + j) * 32);
                    const uint4 a0 = d4[0], a1 = d4[1];
                    const int dist = __popc(a0.x ^ qa.x) + __popc(a0.y ^ qa.y) + __popc(a0.z ^ qa.z) +
                                     __popc(a0.w ^ qa.w) + __popc(a1.x ^ qb.x) + __popc(a1.y ^ qb.y) +
                                     __popc(a1.z ^ qb.z) + __popc(a1.w ^ qb.w);
                    if (dist < 100) key = ((unsigned long long)(unsigned)dist << 32) | (unsigned)j;   // TH_HIGH
                }
            }
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned long long v = __shfl_xor(key, o, 64);
                key = v < key ? v : key;
            }
            best = key < best ? key : best;
        }
        done = best == ~0ull || (int)(best >> 32) >= 75;   // thOrbDist = (TH_HIGH+TH_LOW)/2
    }
    float outU = -1.0f, outD = -1.0f;
    int outS = -1;
    if (!done) {
        const int bestIdxR = (int)(best & 0xFFFFFFFFull);
        const float uR0 = KR[bestIdxR].x;
        const float sf = tb.inv[levelL];
        const int cx = (int)roundf(uL * sf), cy = (int)roundf(vL * sf), cr = (int)roundf(uR0 * sf);
        const LevelGeom& Lg = g.lv[levelL];
        // iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1 (R :705-708); the windows must also lie
        // inside the level (the reference's cv::Mat ranges would assert otherwise)
        const bool ok = cr >= 0 && cr + 11 < Lg.w && cr - 10 >= 0 && cx - 5 >= 0 && cx + 5 < Lg.w && cy - 5 >= 0 &&
                        cy + 5 < Lg.h;
        if (ok) {
            // pair p's pyramids: pyrL / pyrR + p * pyStride (level 0 per zL / zR, pair p = frame p)
            int P, P2;
            uint32_t nb;
            const uint8_t* IL = level_img(g, zL, pyrL + (size_t)p * pyStride - (size_t)p * g.frameBytes, p, levelL, P, nb);
            const uint8_t* IR = level_img(g, zR, pyrR + (size_t)p * pyStride - (size_t)p * g.frameBytes, p, levelL, P2, nb);
            const int cL = IL[(size_t)cy * P + cx];
            for (int c = lane; c < 121; c += 64) {
                const int inc = c / 11 - 5, dy = c % 11 - 5;
                const int cR = IR[(size_t)cy * P2 + cr + inc];
                const uint8_t* rl = IL + (size_t)(cy + dy) * P + cx - 5;
                const uint8_t* rr = IR + (size_t)(cy + dy) * P2 + cr + inc - 5;
                int acc = 0;
#pragma unroll
                for (int dx = 0; dx < 11; dx++) acc += abs(((int)rl[dx] - cL) - ((int)rr[dx] - cR));
                rowsad[wid][c] = acc;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            int vD[11];
#pragma unroll
            for (int i = 0; i < 11; i++) {
                int sacc = 0;
#pragma unroll
                for (int dy = 0; dy < 11; dy++) sacc += rowsad[wid][i * 11 + dy];
                vD[i] = sacc;
            }
            int bestSad = INT_MAX, bestinc = 0;
#pragma unroll
            for (int i = 0; i < 11; i++)
                if ((float)vD[i] < (float)bestSad) { bestSad = vD[i]; bestinc = i - 5; }
            if (bestinc != -5 && bestinc != 5) {
                const float d1 = (float)vD[bestinc + 4], d2 = (float)vD[bestinc + 5], d3 = (float)vD[bestinc + 6];
                const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
                if (!(deltaR < -1 || deltaR > 1)) {
                    float bestuR = tb.scale[levelL] * (((float)cr + (float)bestinc) + deltaR);
                    float disparity = uL - bestuR;
                    if (disparity >= 0 && disparity < maxD) {
                        if (disparity <= 0) {
                            disparity = 0.01f;
                            bestuR = (float)((double)uL - 0.01);
                        }
                        outD = mbf / disparity;
                        outU = bestuR;
                        outS = bestSad;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        UR[iL] = outU;
        DP[iL] = outD;
        SD[iL] = outS;
    }
}

// The 2.1 x median SAD cut (R/src/Frame.cpp:749-769), one workgroup per stereo pair: the
// median of the kept (SAD, index) pairs in ascending order, then every entry at or above
// 1.5f*1.4f*median is dropped.  n_kept[p] receives the surviving count.
__global__ __launch_bounds__(1024) void k_stereo_median(const int32_t* __restrict__ nLs, int cntStride, int kCap,
                                                        float* __restrict__ ur, float* __restrict__ depth,
                                                        const int32_t* __restrict__ sad, int outStride,
                                                        int32_t* __restrict__ nKept, unsigned long long* __restrict__ keys) {
    __shared__ int cnt, med, kept;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = min((int)nLs[(size_t)p * cntStride], kCap);
    float* UR = ur + (size_t)p * outStride;
    float* DP = depth + (size_t)p * outStride;
    const int32_t* SD = sad + (size_t)p * outStride;
    unsigned long long* K = keys + (size_t)p * outStride;
    if (tid == 0) { cnt = 0; med = -1; kept = 0; }
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int s = SD[i];
        if (s >= 0) K[atomicAdd(&cnt, 1)] = ((unsigned long long)(unsigned)s << 32) | (unsigned)i;
    }
    __syncthreads();
    const int m = cnt;
    if (m == 0) {
        if (tid == 0) nKept[p] = 0;
        return;
    }
    for (int i = tid; i < m; i += 1024) {
        const unsigned long long k = K[i];
        int rank = 0;
        for (int j = 0; j < m; j++) rank += K[j] < k;
        if (rank == m / 2) med = (int)(k >> 32);
    }
    __syncthreads();
    const float thDist = 1.5f * 1.4f * (float)med;
    int mine = 0;
    for (int i = tid; i < m; i += 1024) {
        const unsigned long long k = K[i];
        const int idx = (int)(k & 0xFFFFFFFFull);
        if ((float)(int)(k >> 32) < thDist) {
            mine++;
        } else {
            UR[idx] = -1.0f;
            DP[idx] = -1.0f;
        }
    }
    atomicAdd(&kept, mine);
    __syncthreads();
    if (tid == 0) nKept[p] = kept;
}

// ------------------------------------------------------------------ host handle

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || dev < 0 || dev >= n) return ORB_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return ORB_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::fprintf(stderr, "[orbslam2_amd] device %d is %s, this build targets gfx950 only\n", dev, prop.gcnArchName);
        return ORB_ENODEV;
    }
    return ORB_OK;
}

}  // namespace orbamd

using namespace orbamd;

// Pipeline stages timed by orb_extractor_stage_times(): resize, fast (k_fast_cell), reserved (0),
// octree, reserved (0: the Gaussian runs inside k_orient_desc), orient_desc.
constexpr int kStages = 6;

struct orb_extractor {
    orb_extractor_params p;
    int device = 0;
    int maxW = 0, maxH = 0, maxB = 0;
    hipStream_t stream = nullptr;
    Geom g;                     // geometry of the last call
    int gw = -1, gh = -1;
    int blurK[4];
    uint2* d_rztab = nullptr;        // resize coefficient tables of the current geometry
    PyrBand* d_bands = nullptr;      // k_pyramid band table [level][band] (nullptr: per-level k_resize)
    int nBands = 0, pyrBufA = 0, pyrBufB = 0, pyrTab = 0;
    // stereo scratch (orb_compute_stereo_matches*)
    void* d_st = nullptr;
    size_t st_bytes = 0;
    void* h_st = nullptr;
    size_t h_st_bytes = 0;
    bool blurValid = false;          // d_blur holds the blurred pyramid of the last extraction
    hipStream_t lastStream = nullptr;
    L0Src l0{nullptr, 0, 0, 0};     // level 0 of the last extraction (the caller's frames or the slab)
    // copy level 0 into the slab even when it could be read in place: orb_extractor_set_level0_copy
    // (the caller refills its frames before the later level-0 readers run), or ORB_L0_COPY=1 (A/B)
    bool forceL0Copy = [] { const char* e = std::getenv("ORB_L0_COPY"); return e && e[0] == '1'; }();
    size_t capFrames = 0, capFrameBytes = 0, capSlots = 0, capOut = 0, capCells = 0;
    uint8_t *d_pyr = nullptr, *d_blur = nullptr;
    uint32_t *d_slots = nullptr, *d_keyA = nullptr, *d_keyB = nullptr, *d_outKeys = nullptr;
    int *d_cellCount = nullptr, *d_levelCount = nullptr, *d_status = nullptr;
    // host-path outputs
    orb_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int32_t* d_counts = nullptr;
    size_t capHostOut = 0;
    uint8_t* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    void* h_out = nullptr;
    size_t h_out_bytes = 0;
    // pyramid download cache
    std::vector<uint8_t> h_levels;
    std::vector<char> h_level_valid;
    int lastB = 0;
    // stage profiling (HIP events on the launch stream)
    int profile = 0;   // 0 off, 1 every stage boundary, 2 only around k_fast_cell (stage 1)
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, kStages + 1>> ev_sets;
    double stage_ms[kStages] = {0};
    int stage_calls = 0;
};

static void free_dev(void* p) {
    if (p) (void)hipFree(p);
}

static void release_buffers(orb_extractor* ex) {
    free_dev(ex->d_pyr); free_dev(ex->d_blur);
    free_dev(ex->d_slots); free_dev(ex->d_keyA); free_dev(ex->d_keyB); free_dev(ex->d_outKeys);
    free_dev(ex->d_cellCount); free_dev(ex->d_levelCount); free_dev(ex->d_status);
    free_dev(ex->d_kps); free_dev(ex->d_desc); free_dev(ex->d_counts);
    ex->d_pyr = ex->d_blur = nullptr;
    ex->d_slots = ex->d_keyA = ex->d_keyB = ex->d_outKeys = nullptr;
    ex->d_cellCount = ex->d_levelCount = ex->d_status = nullptr;
    ex->d_kps = nullptr; ex->d_desc = nullptr; ex->d_counts = nullptr;
    ex->capFrames = ex->capFrameBytes = ex->capSlots = ex->capOut = ex->capCells = ex->capHostOut = 0;
}

static int ensure_geom(orb_extractor* ex, int w, int h) {
    if (w == ex->gw && h == ex->gh) return ORB_OK;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // legacy-stream setup calls (common.h)
    Geom g;
    int st = build_geom(ex->p, w, h, &g);
    if (st) return st;
    // resize coefficient tables (per level: destination columns, then rows)
    std::vector<uint2> tab;
    for (int l = 1; l < g.nlevels; l++) {
        LevelGeom& L = g.lv[l];
        const LevelGeom& S = g.lv[l - 1];
        L.rzX = (int)tab.size();
        for (int x = 0; x < L.w; x++) {
            uint32_t c[2];
            rz_coef_host(L.rsx, x, S.w, true, c);
            tab.push_back(make_uint2(c[0], c[1]));
        }
        L.rzY = (int)tab.size();
        for (int y = 0; y < L.h; y++) {
            uint32_t c[2];
            rz_coef_host(L.rsy, y, S.h, false, c);
            tab.push_back(make_uint2(c[0], c[1]));
        }
    }
    ORB_HIP_TRY(hipSetDevice(ex->device));
    if (ex->d_rztab) (void)hipFree(ex->d_rztab);
    ex->d_rztab = nullptr;
    if (hipMalloc((void**)&ex->d_rztab, std::max<size_t>(tab.size(), 1) * sizeof(uint2)) != hipSuccess) return ORB_ENOMEM;
    ORB_HIP_TRY(hipMemcpy(ex->d_rztab, tab.data(), tab.size() * sizeof(uint2), hipMemcpyHostToDevice));
    // k_pyramid bands: the fewest bands whose two LDS level buffers (levels 1..7; level 0 is read
    // from the caller's frame) fit the budget, with every row of every level covered; none -> the
    // per-level k_resize launches
    if (ex->d_bands) (void)hipFree(ex->d_bands);
    ex->d_bands = nullptr;
    ex->nBands = 0;
    {
        const int nl = g.nlevels, Hl = g.lv[nl - 1].h;
        std::vector<PyrBand> best;
        int bestK = 0, bestA = 0, bestB = 0, bestT = 0;
        // k_pyramid gathers a 4-column group's source bytes from an 8-byte window at its first
        // column (scale factors up to ~1.9); wider spans keep the per-level launches
        bool spanOk = true;
        for (int l = 1; l < nl; l++) {
            const uint2* XT = tab.data() + g.lv[l].rzX;
            for (int x = 0; x < g.lv[l].w; x += 4) {
                const int xb = (int)(XT[x].x & 0xFFFF);
                for (int j = 0; j < 4; j++) {
                    const uint2 c = XT[std::min(x + j, g.lv[l].w - 1)];
                    if ((int)(c.x & 0xFFFF) - xb > 7 || (int)(c.x >> 16) - xb > 7 || (int)(c.x & 0xFFFF) < xb) spanOk = false;
                }
            }
        }
        // (ORB_PYR_LDS_KB: diagnostic override of the budget)
        const char* ev = std::getenv("ORB_PYR_LDS_KB");
        const int budget0 = (ev && std::atoi(ev) >= 8 && std::atoi(ev) <= 160) ? std::atoi(ev) * 1024 : kPyrLdsBudget;
        // the budget grows (to 96 KB) for geometries whose bands cannot fit it (wide levels:
        // KITTI's 1034-column level 1), rather than falling back to the per-level launches
        for (int budget = budget0; spanOk && bestK == 0 && budget <= 96 * 1024; budget += 8 * 1024)
        for (int K = 8; K <= std::min(64, Hl) && bestK == 0; K++) {
            std::vector<PyrBand> bt((size_t)nl * K);
            for (int k = 0; k < K; k++) {
                int a = (int)((long long)k * Hl / K), e = (int)((long long)(k + 1) * Hl / K);
                bt[(size_t)(nl - 1) * K + k] = {a, e - a};
                for (int l = nl - 1; l >= 1; l--) {   // source rows of [a, e) at level l
                    const uint2* YT = tab.data() + g.lv[l].rzY;
                    const int lo = (int)(YT[a].x & 0xFFFF), hi = (int)(YT[e - 1].x >> 16);
                    a = lo;
                    e = hi + 1;
                    bt[(size_t)(l - 1) * K + k] = {a, e - a};
                }
            }
            bool ok = true;
            int bufA = 0, bufB = 0;
            for (int l = 0; l < nl && ok; l++) {
                int end = 0;
                for (int k = 0; k < K; k++) {
                    const PyrBand& p = bt[(size_t)l * K + k];
                    if (p.n <= 0 || p.s0 > end) ok = false;
                    end = std::max(end, p.s0 + p.n);
                    const int bytes = p.n * (((g.lv[l].w + 3) >> 2) << 2);
                    if (l == 0) continue;   // level 0: the caller's frame, not staged
                    if (l % 2 == 0) bufA = std::max(bufA, bytes); else bufB = std::max(bufB, bytes);
                }
                if (end != g.lv[l].h || bt[(size_t)l * K].s0 != 0) ok = false;
            }
            bufA = (bufA + 15 + 16) & ~15;   // +16: the last row's third dword read may pass the row
            bufB = (bufB + 15 + 16) & ~15;
            int tabBytes = 0;   // per-level coefficient tables staged next to the buffers
            for (int l = 1; l < nl; l++) {
                int maxN = 0;
                for (int k = 0; k < K; k++) maxN = std::max(maxN, bt[(size_t)l * K + k].n);
                tabBytes = std::max(tabBytes, 8 * (g.lv[l].w + maxN));
            }
            if (ok && bufA + bufB + tabBytes <= budget) {
                best = bt; bestK = K; bestA = bufA; bestB = bufB; bestT = tabBytes;
            }
        }
        if (bestK > 0) {
            if (hipMalloc((void**)&ex->d_bands, best.size() * sizeof(PyrBand)) != hipSuccess) return ORB_ENOMEM;
            ORB_HIP_TRY(hipMemcpy(ex->d_bands, best.data(), best.size() * sizeof(PyrBand), hipMemcpyHostToDevice));
            ex->nBands = bestK;
            ex->pyrBufA = bestA;
            ex->pyrBufB = bestB;
            ex->pyrTab = bestT;
        }
    }
    ex->g = g;
    ex->gw = w;
    ex->gh = h;
    return ORB_OK;
}

static int ensure_capacity(orb_extractor* ex, int B) {
    const Geom& g = ex->g;
    const size_t fb = (size_t)g.frameBytes, sl = (size_t)g.slotsPerFrame, ou = (size_t)g.outPerFrame,
                 ce = (size_t)g.cellsPerFrame;
    if ((size_t)B <= ex->capFrames && fb <= ex->capFrameBytes && sl <= ex->capSlots && ou <= ex->capOut &&
        ce <= ex->capCells)
        return ORB_OK;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // legacy-stream setup calls (common.h)
    ORB_HIP_TRY(hipStreamSynchronize(ex->stream));
    release_buffers(ex);
    const size_t nb = std::max<size_t>(B, 1);
#define ALLOC(ptr, bytes) \
    if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess) { release_buffers(ex); return ORB_ENOMEM; }
    ALLOC(ex->d_pyr, nb * fb);
    ALLOC(ex->d_blur, nb * fb);
    ALLOC(ex->d_slots, nb * sl * 4);
    ALLOC(ex->d_keyA, nb * sl * 4);
    ALLOC(ex->d_keyB, nb * sl * 4);
    ALLOC(ex->d_outKeys, nb * ou * 4);
    ALLOC(ex->d_cellCount, nb * ce * 4);
    ALLOC(ex->d_levelCount, nb * kMaxLevels * 4);
    ALLOC(ex->d_status, 64);
    ALLOC(ex->d_kps, nb * ou * sizeof(orb_keypoint));
    ALLOC(ex->d_desc, nb * ou * 32);
    ALLOC(ex->d_counts, nb * 4 + 64);
#undef ALLOC
    ex->capFrames = nb;
    ex->capFrameBytes = fb;
    ex->capSlots = sl;
    ex->capOut = ou;
    ex->capCells = ce;
    ex->capHostOut = ou;
    ORB_HIP_TRY(hipMemset(ex->d_pyr, 0, nb * fb));
    ORB_HIP_TRY(hipMemset(ex->d_blur, 0, nb * fb));
    return ORB_OK;
}

static size_t octree_lds_bytes(const Geom& g) {
    const size_t cap = (size_t)g.maxNodeCap;
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t s = r16(sizeof(uint4) * (cap + 1));
    s += 2 * (r16(4 * (cap + 1)) + 5 * r16(4 * cap));
    s += 6 * r16(4 * cap) + r16(4 * (cap + 1));
    s += 2 * r16(8 * cap);
    int maxCells = 0;
    for (int l = 0; l < g.nlevels; l++) maxCells = std::max(maxCells, g.lv[l].nCols * g.lv[l].nRows);
    s += r16(4 * (maxCells + 1 + 64));
    s += r16(4 * 8) + r16(4 * 32);
    return s;
}

// Enqueues the full pipeline for B frames already resident in d_pyr level 0.
static hipEvent_t ev_get(orb_extractor* ex) {
    if (!ex->ev_pool.empty()) {
        hipEvent_t e = ex->ev_pool.back();
        ex->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Enqueues the full pipeline for B frames.  Level 0 of frame b is src + b * srcFrameStride (dense
// rows srcRowStride bytes apart); `inSlab` = it already is the slab's pitched level 0 (orb_extract's
// upload).  Dword-aligned frames are read in place by every consumer (L0Src, no copy); other frames
// (odd widths) and the per-level k_resize fallback are first copied into the slab.  The level-0
// source is kept in ex->l0 for the later readers (orb_pyramid_level*, the stereo matchers).
static int run_pipeline(orb_extractor* ex, int B, const uint8_t* src, long long srcFrameStride, int srcRowStride,
                        int inSlab, orb_keypoint* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts, hipStream_t st) {
    const Geom& g = ex->g;
    const LevelGeom& L0 = g.lv[0];
    const bool inPlace = inSlab || (ex->d_bands && (srcRowStride & 3) == 0 && (srcFrameStride & 3) == 0 &&
                                    ((uintptr_t)src & 3) == 0 && !ex->forceL0Copy);
    const bool copyL0 = !inPlace;
    L0Src z;
    if (inPlace && !inSlab) {
        z.p = src;
        z.frameStride = srcFrameStride;
        z.pitch = srcRowStride;
        z.bytes = (uint32_t)((size_t)(L0.h - 1) * srcRowStride + L0.w);
    } else {
        z.p = ex->d_pyr + L0.off;
        z.frameStride = g.frameBytes;
        z.pitch = L0.pitch;
        z.bytes = (uint32_t)(g.frameBytes - L0.off);
    }
    ex->l0 = z;
    std::array<hipEvent_t, kStages + 1> ev{};
    const int prof = ex->profile;
    if (prof) {
        for (int i = 0; i <= kStages; i++) {
            if (prof == 2 && i != 1 && i != 2) continue;   // two events bracketing k_fast_cell only
            if (prof == 3 && (i == 3 || i == 5)) continue;  // the four kernels' boundaries only
            ev[i] = ev_get(ex);
            if (!ev[i]) return ORB_EGPU;
        }
    }
    auto mark = [&](int i) {
        if (prof && ev[i]) (void)hipEventRecord(ev[i], st);
    };
    mark(0);
    if (copyL0) {   // odd widths / the fallback: level 0 into the slab first
        const int w = L0.w, h = L0.h;
        const int vec16 = (w % 16 == 0) && (srcRowStride == w) && (srcFrameStride % 16 == 0) && ((uintptr_t)src % 16 == 0);
        const int items = vec16 ? (w / 16) * h : ((w + 3) / 4) * h;
        hipLaunchKernelGGL(k_load_frames, dim3((items + 255) / 256, B), dim3(256), 0, st, g, src, (size_t)srcFrameStride,
                           ex->d_pyr, vec16);
    }
    if (ex->d_bands) {
        // levels 1..7 in one launch; it also clears the status word
        hipLaunchKernelGGL(k_pyramid, dim3(ex->nBands, B), dim3(256), (size_t)(ex->pyrBufA + ex->pyrBufB + ex->pyrTab),
                           st, g, z, ex->d_pyr, ex->d_rztab, ex->d_bands, ex->nBands, ex->pyrBufA, ex->pyrBufB,
                           ex->d_status);
    } else {
        ORB_HIP_TRY(hipMemsetAsync(ex->d_status, 0, 4, st));
        for (int l = 1; l < g.nlevels; l++) {
            const LevelGeom& L = g.lv[l];
            // source window bound of one 256 x 16 block: ceil(256 * rsx) + 2 columns (+3 for dword
            // alignment), ceil(16 * rsy) + 2 rows
            const int srcW32 = (int)std::ceil(kRzCols * L.rsx) / 4 + 3;
            const int srcRows = (int)std::ceil(kRzRows * L.rsy) + 3;
            dim3 grid((L.w + kRzCols - 1) / kRzCols, (L.h + kRzRows - 1) / kRzRows, B);
            hipLaunchKernelGGL(k_resize, grid, dim3(256), (size_t)srcW32 * srcRows * 4, st, g, l, ex->d_pyr,
                               ex->d_rztab, srcW32, srcRows);
        }
    }
    mark(1);
    {
        // FAST + NMS + cell retry fused per cell (stage 1); stage 2 (the former separate
        // cell pass) is empty
        // the width bound rounded up to 4 (a layout with room for it); the common cell widths of
        // ORB-SLAM2's 30-px grid get a compile-time instantiation
        const int mw = (g.maxCellW + 3) & ~3;
        const size_t lds = 4 * (size_t)fc_wave_bytes(mw, g.maxCellH);
        const dim3 grid((g.cellsPerFrame + 3) / 4, B);
        if (mw == 32)
            hipLaunchKernelGGL(k_fast_cell<32>, grid, dim3(256), lds, st, g, ex->d_pyr, z, ex->d_slots, ex->d_cellCount,
                               ex->d_status, mw, g.maxCellH);
        else if (mw == 36)
            hipLaunchKernelGGL(k_fast_cell<36>, grid, dim3(256), lds, st, g, ex->d_pyr, z, ex->d_slots, ex->d_cellCount,
                               ex->d_status, mw, g.maxCellH);
        else if (mw == 40)
            hipLaunchKernelGGL(k_fast_cell<40>, grid, dim3(256), lds, st, g, ex->d_pyr, z, ex->d_slots, ex->d_cellCount,
                               ex->d_status, mw, g.maxCellH);
        else if (mw == 44)
            hipLaunchKernelGGL(k_fast_cell<44>, grid, dim3(256), lds, st, g, ex->d_pyr, z, ex->d_slots, ex->d_cellCount,
                               ex->d_status, mw, g.maxCellH);
        else
            hipLaunchKernelGGL(k_fast_cell<0>, grid, dim3(256), lds, st, g, ex->d_pyr, z, ex->d_slots, ex->d_cellCount,
                               ex->d_status, mw, g.maxCellH);
    }
    mark(2);
    mark(3);
    // LDS key buffers: small batches (latency) keep a level's keys in LDS when they fit, with the
    // buffers sized so that two workgroups still fit a CU (<= 80 KB each); batches of 32 frames or
    // more keep them in their HBM arrays (L2-resident) and the launch takes only the node tables'
    // LDS — measured on the bench step (3 x 128 frames): 80 KB -> 248 k frames/s, node tables only
    // -> 259 k, as the octree's low-VALU workgroups no longer hold LDS that the other streams'
    // FAST / descriptor workgroups could use.  ORB_OT_LDS_KB overrides the budget (diagnostics).
    const size_t ldsBase = octree_lds_bytes(g);
    static const int otEnvKb = [] {
        const char* e = std::getenv("ORB_OT_LDS_KB");
        const int kb = e ? std::atoi(e) : 0;
        return kb >= 16 && kb <= 160 ? kb : 0;
    }();
    const long long otBudget = otEnvKb ? otEnvKb * 1024LL : B >= 32 ? 0LL : 80 * 1024LL;
    const int keyCap = (int)std::max<long long>(0, std::min<long long>(2LL * g.maxLevelSlots,
                                                                          (otBudget - (long long)ldsBase) / 4 - 8));
    const size_t lds = ldsBase + 16 + 4 * (size_t)keyCap;
    hipLaunchKernelGGL(k_octree, dim3(g.nlevels, B), dim3(OT_T), lds, st, g, ex->d_slots, ex->d_cellCount,
                       ex->d_keyA, ex->d_keyB, ex->d_outKeys, ex->d_levelCount, ex->d_status, keyCap);
    mark(4);
    // the Gaussian is evaluated inside k_orient_desc where the descriptor samples (stage 4 empty);
    // the full blurred pyramid is produced on demand by orb_pyramid_level_device(blurred = 1)
    mark(5);
    {
        const int* k = ex->blurK;   // centre, +-1, +-2, +-3
        const uint32_t kA = (uint32_t)k[3] | ((uint32_t)k[2] << 8) | ((uint32_t)k[1] << 16) | ((uint32_t)k[0] << 24);
        const uint32_t kB = (uint32_t)k[1] | ((uint32_t)k[2] << 8) | ((uint32_t)k[3] << 16);
        hipLaunchKernelGGL(k_orient_desc, dim3((g.outPerFrame + 4 * kOdKpw - 1) / (4 * kOdKpw), B), dim3(256), 0, st, g, ex->d_pyr, z,
                           ex->d_outKeys, ex->d_levelCount, d_kps, d_desc, cap, d_counts, kA, kB);
    }
    mark(6);
    ex->blurValid = false;
    ex->lastStream = st;
    ORB_HIP_TRY(hipGetLastError());
    if (prof) ex->ev_sets.push_back(ev);
    return ORB_OK;
}

static void gauss7_int(int k[7]) {
    float cf[7];
    const double sigma = 2.0, scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < 7; i++) {
        const double x = i - 3.0;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) {
        cf[i] = (float)(cf[i] * sum);
        k[i] = (int)std::nearbyint(cf[i] * 256.0f);
    }
}

extern "C" {

int orb_extractor_create(const orb_extractor_params* params, int device, int max_w, int max_h, int max_batch,
                         orb_extractor** out) try {
    if (!params || !out || max_w <= 0 || max_h <= 0 || max_batch <= 0) return ORB_EINVAL;
    if (params->nlevels < 1 || params->nlevels > kMaxLevels || params->nfeatures < 0 || !(params->scaleFactor > 1.0f))
        return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    ORB_HIP_TRY(hipSetDevice(device));
    orb_extractor* ex = new orb_extractor();
    ex->p = *params;
    ex->device = device;
    ex->maxW = max_w;
    ex->maxH = max_h;
    ex->maxB = max_batch;
    int k[7];
    gauss7_int(k);
    ex->blurK[0] = k[3]; ex->blurK[1] = k[2]; ex->blurK[2] = k[1]; ex->blurK[3] = k[0];
    {
        std::lock_guard<std::mutex> lk(legacy_capture_mutex());
        if (hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking) != hipSuccess) { delete ex; return ORB_EGPU; }
    }
    st = ensure_geom(ex, max_w, max_h);
    if (!st) st = ensure_capacity(ex, max_batch);
    if (st) { orb_extractor_destroy(ex); return st; }
    *out = ex;
    return ORB_OK;
} ORB_ABI_CATCH

void orb_extractor_destroy(orb_extractor* ex) try {
    if (!ex) return;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // hipFree (common.h)
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    release_buffers(ex);
    if (ex->d_rztab) (void)hipFree(ex->d_rztab);
    if (ex->d_bands) (void)hipFree(ex->d_bands);
    if (ex->d_st) (void)hipFree(ex->d_st);
    if (ex->h_st) (void)hipHostFree(ex->h_st);
    for (auto& set : ex->ev_sets)
        for (auto e : set) ex->ev_pool.push_back(e);
    for (auto e : ex->ev_pool) (void)hipEventDestroy(e);
    if (ex->h_stage) (void)hipHostFree(ex->h_stage);
    if (ex->h_out) (void)hipHostFree(ex->h_out);
    if (ex->stream) (void)hipStreamDestroy(ex->stream);
    delete ex;
} ORB_ABI_CATCH_VOID

int orb_extractor_levels(const orb_extractor* ex) try { return ex ? ex->p.nlevels : ORB_EINVAL; } ORB_ABI_CATCH

int orb_extractor_scale_tables(const orb_extractor* ex, float* scale, float* inv_scale, float* sigma2,
                               float* inv_sigma2) try {
    if (!ex) return ORB_EINVAL;
    host_tables(ex->p, scale, inv_scale, sigma2, inv_sigma2, nullptr);
    return ORB_OK;
} ORB_ABI_CATCH

int orb_extractor_features_per_level(const orb_extractor* ex, int* per_level) try {
    if (!ex || !per_level) return ORB_EINVAL;
    host_tables(ex->p, nullptr, nullptr, nullptr, nullptr, per_level);
    return ORB_OK;
} ORB_ABI_CATCH

static int ensure_pinned(void** p, size_t* cur, size_t need) {
    if (*cur >= need) return ORB_OK;
    // growth (first use, a larger frame) frees and allocates pinned memory: under the capture lock,
    // as the matcher's pinned staging does (common.h) — never called with the lock held
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cur = 0;
    if (hipHostMalloc(p, need, hipHostMallocDefault) != hipSuccess) return ORB_ENOMEM;
    *cur = need;
    return ORB_OK;
}

int orb_extract(orb_extractor* ex, const uint8_t* img, int w, int h, size_t stride, orb_keypoint* kps, uint8_t* desc,
                int capacity, int* n_out) try {
    if (!ex) return ORB_EINVAL;
    if (!img || w <= 0 || h <= 0) return ORB_OK;   // R/src/ORBextractor.cpp:1123-1124
    if (stride < (size_t)w || capacity < 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    int st = ensure_geom(ex, w, h);
    if (st) return st;
    st = ensure_capacity(ex, 1);
    if (st) return st;
    const Geom& g = ex->g;
    const LevelGeom& L0 = g.lv[0];
    const size_t imgBytes = (size_t)L0.pitch * h;
    st = ensure_pinned((void**)&ex->h_stage, &ex->h_stage_bytes, imgBytes);
    if (st) return st;
    for (int y = 0; y < h; y++) std::memcpy(ex->h_stage + (size_t)y * L0.pitch, img + (size_t)y * stride, (size_t)w);
    ORB_HIP_TRY(hipMemcpyAsync(ex->d_pyr + L0.off, ex->h_stage, imgBytes, hipMemcpyHostToDevice, ex->stream));
    const int cap = (int)ex->capHostOut;
    st = run_pipeline(ex, 1, ex->d_pyr + L0.off, g.frameBytes, L0.pitch, 1, ex->d_kps, ex->d_desc, cap, ex->d_counts,
                      ex->stream);
    if (st) return st;
    st = ensure_pinned(&ex->h_out, &ex->h_out_bytes, 64 + (size_t)cap * (sizeof(orb_keypoint) + 32));
    if (st) return st;
    int32_t* h_cnt = (int32_t*)ex->h_out;
    ORB_HIP_TRY(hipMemcpyAsync(h_cnt, ex->d_counts, 4, hipMemcpyDeviceToHost, ex->stream));
    ORB_HIP_TRY(hipMemcpyAsync(h_cnt + 1, ex->d_status, 4, hipMemcpyDeviceToHost, ex->stream));
    ORB_HIP_TRY(hipStreamSynchronize(ex->stream));
    ex->lastB = 1;
    ex->h_level_valid.assign(g.nlevels, 0);
    if (h_cnt[1] != 0) {
        std::fprintf(stderr, "[orbslam2_amd] extractor status 0x%x\n", h_cnt[1]);
        return ORB_EOVERFLOW;
    }
    const int N = h_cnt[0];
    if (n_out) *n_out = N;
    if (N > capacity) return ORB_E2BIG;
    if (N > 0) {
        orb_keypoint* hk = (orb_keypoint*)((char*)ex->h_out + 64);
        uint8_t* hd = (uint8_t*)(hk + cap);
        ORB_HIP_TRY(hipMemcpyAsync(hk, ex->d_kps, (size_t)N * sizeof(orb_keypoint), hipMemcpyDeviceToHost, ex->stream));
        ORB_HIP_TRY(hipMemcpyAsync(hd, ex->d_desc, (size_t)N * 32, hipMemcpyDeviceToHost, ex->stream));
        ORB_HIP_TRY(hipStreamSynchronize(ex->stream));
        if (kps) std::memcpy(kps, hk, (size_t)N * sizeof(orb_keypoint));
        if (desc) std::memcpy(desc, hd, (size_t)N * 32);
    }
    return N;
} ORB_ABI_CATCH

int orb_extract_batch_device(orb_extractor* ex, const uint8_t* d_imgs, size_t img_stride_frame, int B, int w, int h,
                             orb_keypoint* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts, void* stream) try {
    if (!ex || !d_imgs || B <= 0 || w <= 0 || h <= 0 || !d_kps || !d_desc || !d_counts || cap < 0) return ORB_EINVAL;
    if (img_stride_frame < (size_t)w * h) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    int st = ensure_geom(ex, w, h);
    if (st) return st;
    st = ensure_capacity(ex, B);
    if (st) return st;
    hipStream_t s = stream ? (hipStream_t)stream : ex->stream;
    const Geom& g = ex->g;
    ex->lastB = B;
    ex->h_level_valid.assign((size_t)B * g.nlevels, 0);
    return run_pipeline(ex, B, d_imgs, (long long)img_stride_frame, w, 0, d_kps, d_desc, cap, d_counts, s);
} ORB_ABI_CATCH

int orb_extractor_set_level0_copy(orb_extractor* ex, int copy) try {
    if (!ex || (copy != 0 && copy != 1)) return ORB_EINVAL;
    ex->forceL0Copy = copy != 0;
    return ORB_OK;
} ORB_ABI_CATCH

int orb_extractor_batch_status(orb_extractor* ex, int32_t* status) try {
    if (!ex || !status) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    hipStream_t st = ex->lastStream ? ex->lastStream : ex->stream;
    int32_t* h = nullptr;
    if (ensure_pinned(&ex->h_out, &ex->h_out_bytes, 64)) return ORB_ENOMEM;
    h = (int32_t*)ex->h_out + 15;   // the last word of the 64-byte header (orb_extract uses words 0-1)
    ORB_HIP_TRY(hipMemcpyAsync(h, ex->d_status, 4, hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipStreamSynchronize(st));
    *status = *h;
    return *h ? ORB_EOVERFLOW : ORB_OK;
} ORB_ABI_CATCH

int orb_pyramid_level(orb_extractor* ex, int frame, int level, const uint8_t** host, int* w, int* h, size_t* stride) try {
    if (!ex || level < 0 || level >= ex->p.nlevels || frame < 0 || frame >= ex->lastB || ex->gw < 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    const Geom& g = ex->g;
    const size_t per = (size_t)g.frameBytes;
    if (ex->h_levels.size() < per * ex->lastB) ex->h_levels.resize(per * ex->lastB);
    if (ex->h_level_valid.size() < (size_t)ex->lastB * g.nlevels) ex->h_level_valid.assign((size_t)ex->lastB * g.nlevels, 0);
    const LevelGeom& L = g.lv[level];
    uint8_t* dst = ex->h_levels.data() + per * frame + L.off;
    char& valid = ex->h_level_valid[(size_t)frame * g.nlevels + level];
    if (!valid) {   // ordered after the extraction on the stream it ran on (a caller stream for the batch path)
        hipStream_t st = ex->lastStream ? ex->lastStream : ex->stream;
        if (level == 0)   // the caller's frame (read in place) or the slab's copy
            ORB_HIP_TRY(hipMemcpy2DAsync(dst, (size_t)L.pitch, ex->l0.p + (size_t)frame * ex->l0.frameStride,
                                         (size_t)ex->l0.pitch, (size_t)L.w, (size_t)L.h, hipMemcpyDeviceToHost, st));
        else
            ORB_HIP_TRY(hipMemcpyAsync(dst, ex->d_pyr + per * frame + L.off, (size_t)L.pitch * L.h,
                                       hipMemcpyDeviceToHost, st));
        ORB_HIP_TRY(hipStreamSynchronize(st));
        valid = 1;
    }
    if (host) *host = dst;
    if (w) *w = L.w;
    if (h) *h = L.h;
    if (stride) *stride = (size_t)L.pitch;
    return ORB_OK;
} ORB_ABI_CATCH

int orb_pyramid_level_device(orb_extractor* ex, int frame, int level, int blurred, const uint8_t** dptr, int* w,
                             int* h, size_t* pitch) try {
    if (!ex || level < 0 || level >= ex->p.nlevels || frame < 0 || frame >= (int)ex->capFrames || ex->gw < 0)
        return ORB_EINVAL;
    const Geom& g = ex->g;
    const LevelGeom& L = g.lv[level];
    if (blurred && !ex->blurValid && ex->lastB > 0) {
        ORB_HIP_TRY(hipSetDevice(ex->device));
        hipStream_t st = ex->lastStream ? ex->lastStream : ex->stream;
        hipLaunchKernelGGL(k_blur, dim3(g.tilesPerFrame, ex->lastB), dim3(256), 0, st, g, ex->d_pyr, ex->l0,
                           ex->d_blur, ex->blurK[0], ex->blurK[1], ex->blurK[2], ex->blurK[3]);
        ORB_HIP_TRY(hipGetLastError());
        ORB_HIP_TRY(hipStreamSynchronize(st));
        ex->blurValid = true;
    }
    const uint8_t* base = blurred ? ex->d_blur : ex->d_pyr;
    const bool raw0 = !blurred && level == 0;   // level 0 as the consumers read it (L0Src)
    if (dptr) *dptr = raw0 ? ex->l0.p + (size_t)frame * ex->l0.frameStride : base + (size_t)frame * g.frameBytes + L.off;
    if (w) *w = L.w;
    if (h) *h = L.h;
    if (pitch) *pitch = raw0 ? (size_t)ex->l0.pitch : (size_t)L.pitch;
    return ORB_OK;
} ORB_ABI_CATCH

int orb_extractor_profile(orb_extractor* ex, int enable) try {
    if (!ex) return ORB_EINVAL;
    if (enable < 0 || enable > 3) return ORB_EINVAL;
    ex->profile = enable;
    return ORB_OK;
} ORB_ABI_CATCH

int orb_extractor_stage_times(orb_extractor* ex, double* ms, int n_stages, int* n_calls) try {
    if (!ex || (n_stages > 0 && !ms)) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    for (auto& set : ex->ev_sets) {
        for (int i = kStages; i >= 0; i--)
            if (set[i]) { ORB_HIP_TRY(hipEventSynchronize(set[i])); break; }
        // consecutive recorded events a < b bracket the kernel of stage b - 1 (the stages between
        // them launch nothing): mode 1 records every boundary, 2 the two around stage 1, 3 the
        // kernel boundaries 0, 1, 2, 4, 6
        for (int a = 0; a < kStages; a++) {
            if (!set[a]) continue;
            int b = a + 1;
            while (b <= kStages && !set[b]) b++;
            if (b > kStages) break;
            float t = 0.f;
            ORB_HIP_TRY(hipEventElapsedTime(&t, set[a], set[b]));
            ex->stage_ms[b - 1] += t;
            a = b - 1;
        }
        ex->stage_calls++;
        for (auto e : set)
            if (e) ex->ev_pool.push_back(e);
    }
    ex->ev_sets.clear();
    for (int i = 0; i < n_stages && i < kStages; i++) ms[i] = ex->stage_ms[i];
    if (n_calls) *n_calls = ex->stage_calls;
    for (int i = 0; i < kStages; i++) ex->stage_ms[i] = 0;
    ex->stage_calls = 0;
    return kStages;
} ORB_ABI_CATCH

int orb_extractor_geometry(orb_extractor* ex, int w, int h, int* level_w, int* level_h, int* cells_per_level,
                           int* max_keypoints_per_frame) try {
    if (!ex || w <= 0 || h <= 0) return ORB_EINVAL;
    int st = ensure_geom(ex, w, h);
    if (st) return st;
    const Geom& g = ex->g;
    for (int l = 0; l < g.nlevels; l++) {
        if (level_w) level_w[l] = g.lv[l].w;
        if (level_h) level_h[l] = g.lv[l].h;
        if (cells_per_level) cells_per_level[l] = g.lv[l].nCols * g.lv[l].nRows;
    }
    if (max_keypoints_per_frame) *max_keypoints_per_frame = g.outPerFrame;
    return ORB_OK;
} ORB_ABI_CATCH

int orb_extractor_last_counts(orb_extractor* ex, int frame, int* pre_counts, int* level_counts) try {
    if (!ex || frame < 0 || frame >= ex->lastB || ex->gw < 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(ex->device));
    const Geom& g = ex->g;
    std::vector<int> cc(g.cellsPerFrame), lc(g.nlevels);
    ORB_HIP_TRY(hipStreamSynchronize(ex->lastStream ? ex->lastStream : ex->stream));
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // legacy-stream copies (common.h)
    ORB_HIP_TRY(hipMemcpy(cc.data(), ex->d_cellCount + (size_t)frame * g.cellsPerFrame, cc.size() * 4,
                          hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(lc.data(), ex->d_levelCount + (size_t)frame * g.nlevels, lc.size() * 4,
                          hipMemcpyDeviceToHost));
    for (int l = 0; l < g.nlevels; l++) {
        int s = 0;
        for (int c = 0; c < g.lv[l].nCols * g.lv[l].nRows; c++) s += cc[g.lv[l].cellBase + c];
        if (pre_counts) pre_counts[l] = s;
        if (level_counts) level_counts[l] = lc[l];
    }
    return ORB_OK;
} ORB_ABI_CATCH

static int stereo_scratch(orb_extractor* ex, size_t bytes) {
    if (ex->st_bytes >= bytes) return ORB_OK;
    if (ex->d_st) (void)hipFree(ex->d_st);
    ex->d_st = nullptr;
    ex->st_bytes = 0;
    if (hipMalloc(&ex->d_st, bytes) != hipSuccess) return ORB_ENOMEM;
    ex->st_bytes = bytes;
    return ORB_OK;
}

static StereoTabs stereo_tabs(const orb_extractor* ex) {
    StereoTabs tb;
    std::memset(&tb, 0, sizeof(tb));
    host_tables(ex->p, tb.scale, tb.inv, nullptr, nullptr, nullptr);
    return tb;
}

int orb_compute_stereo_matches(orb_extractor* left, orb_extractor* right, const orb_keypoint* kps_l,
                               const uint8_t* desc_l, int n_l, const orb_keypoint* kps_r, const uint8_t* desc_r,
                               int n_r, float mbf, float mb, float* uright, float* depth) try {
    if (!left || !right || n_l < 0 || n_r < 0 || (n_l && (!kps_l || !desc_l || !uright || !depth)) || (n_r && (!kps_r || !desc_r)))
        return ORB_EINVAL;
    for (int i = 0; i < n_l; i++) { uright[i] = -1.0f; depth[i] = -1.0f; }
    if (n_l == 0) return 0;
    if (left->gw < 0 || left->gw != right->gw || left->gh != right->gh || left->lastB < 1 || right->lastB < 1 ||
        left->p.nlevels != right->p.nlevels || left->device != right->device)
        return ORB_EINVAL;   // both extractors must hold an extraction of the same geometry
    ORB_HIP_TRY(hipSetDevice(left->device));
    const int cap = std::max(n_l, n_r);
    const size_t kb = (size_t)cap * sizeof(orb_keypoint), db = (size_t)cap * 32, ob = (size_t)cap * 4;
    const size_t bytes = 2 * kb + 2 * db + 3 * ob + (size_t)cap * 8 + 64;
    int st = stereo_scratch(left, bytes);
    if (st) return st;
    st = ensure_pinned(&left->h_st, &left->h_st_bytes, bytes);
    if (st) return st;
    char* d = (char*)left->d_st;
    orb_keypoint* dkl = (orb_keypoint*)d;
    orb_keypoint* dkr = (orb_keypoint*)(d + kb);
    uint8_t* ddl = (uint8_t*)(d + 2 * kb);
    uint8_t* ddr = ddl + db;
    float* dur = (float*)(ddr + db);
    float* ddp = dur + cap;
    int32_t* dsd = (int32_t*)(ddp + cap);
    unsigned long long* dkeys = (unsigned long long*)(((uintptr_t)(dsd + cap) + 7) & ~(uintptr_t)7);
    int32_t* dn = (int32_t*)(dkeys + cap);
    char* h = (char*)left->h_st;
    int32_t* hn = (int32_t*)(h + bytes - 16);
    hn[0] = n_l;
    hn[1] = n_r;
    hipStream_t s = left->stream;
    // the right extractor's pyramid must be complete before this stream reads it
    ORB_HIP_TRY(hipStreamSynchronize(right->lastStream ? right->lastStream : right->stream));
    ORB_HIP_TRY(hipMemcpyAsync(dkl, kps_l, (size_t)n_l * sizeof(orb_keypoint), hipMemcpyHostToDevice, s));
    if (n_r) ORB_HIP_TRY(hipMemcpyAsync(dkr, kps_r, (size_t)n_r * sizeof(orb_keypoint), hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(ddl, desc_l, (size_t)n_l * 32, hipMemcpyHostToDevice, s));
    if (n_r) ORB_HIP_TRY(hipMemcpyAsync(ddr, desc_r, (size_t)n_r * 32, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(dn, hn, 8, hipMemcpyHostToDevice, s));
    const float maxD = mbf / mb;   // mb = 0 in the reference: +inf
    hipLaunchKernelGGL(k_stereo_match, dim3((n_l + 3) / 4, 1), dim3(256), 0, s, left->g, stereo_tabs(left),
                       left->d_pyr, right->d_pyr, (size_t)0, left->l0, right->l0, dkl, ddl, dn, dkr, ddr, dn + 1, cap, 1, cap, mbf, maxD, dur,
                       ddp, dsd, cap);
    hipLaunchKernelGGL(k_stereo_median, dim3(1), dim3(1024), 0, s, dn, 1, cap, dur, ddp, dsd, cap, dn + 2, dkeys);
    ORB_HIP_TRY(hipGetLastError());
    float* hur = (float*)h;
    float* hdp = hur + cap;
    ORB_HIP_TRY(hipMemcpyAsync(hur, dur, (size_t)n_l * 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipMemcpyAsync(hdp, ddp, (size_t)n_l * 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipMemcpyAsync(hn + 2, dn + 2, 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(uright, hur, (size_t)n_l * 4);
    std::memcpy(depth, hdp, (size_t)n_l * 4);
    return hn[2];
} ORB_ABI_CATCH

int orb_compute_stereo_matches_batch_device(orb_extractor* ex, const orb_keypoint* d_kps, const uint8_t* d_desc,
                                            const int32_t* d_counts, int cap, int n_pairs, float mbf, float mb,
                                            float* d_uright, float* d_depth, int32_t* d_nstereo, void* stream) try {
    if (!ex || !d_kps || !d_desc || !d_counts || cap <= 0 || n_pairs <= 0 || !d_uright || !d_depth || !d_nstereo)
        return ORB_EINVAL;
    if (ex->gw < 0 || ex->lastB < 2 * n_pairs) return ORB_EINVAL;   // frames 2p (left), 2p+1 (right)
    ORB_HIP_TRY(hipSetDevice(ex->device));
    const size_t bytes = (size_t)n_pairs * cap * (4 + 8) + 64;
    int st = stereo_scratch(ex, bytes);
    if (st) return st;
    int32_t* dsd = (int32_t*)ex->d_st;
    unsigned long long* dkeys = (unsigned long long*)(((uintptr_t)(dsd + (size_t)n_pairs * cap) + 7) & ~(uintptr_t)7);
    hipStream_t s = stream ? (hipStream_t)stream : ex->stream;
    const Geom& g = ex->g;
    const float maxD = mbf / mb;
    // frames 2p (left) and 2p + 1 (right) of the last batch: level 0 at twice the frame stride
    L0Src zL = ex->l0, zR = ex->l0;
    zL.frameStride = zR.frameStride = 2 * ex->l0.frameStride;
    zR.p = ex->l0.p + ex->l0.frameStride;
    hipLaunchKernelGGL(k_stereo_match, dim3((cap + 3) / 4, n_pairs), dim3(256), 0, s, g, stereo_tabs(ex), ex->d_pyr,
                       ex->d_pyr + g.frameBytes, (size_t)(2 * g.frameBytes), zL, zR, d_kps, d_desc, d_counts, d_kps + cap,
                       d_desc + (size_t)cap * 32, d_counts + 1, 2 * cap, 2, cap, mbf, maxD, d_uright, d_depth, dsd, cap);
    hipLaunchKernelGGL(k_stereo_median, dim3(n_pairs), dim3(1024), 0, s, d_counts, 2, cap, d_uright, d_depth, dsd, cap,
                       d_nstereo, dkeys);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

int orb_pack_rows_device(const void* d_src, int row_bytes, int cap, const int32_t* d_counts, int B, void* d_dst,
                         int32_t* d_offsets, void* stream) try {
    if (!d_src || !d_counts || !d_dst || !d_offsets || B <= 0 || cap < 0 || row_bytes <= 0 || (row_bytes & 3))
        return ORB_EINVAL;
    hipLaunchKernelGGL(k_pack_rows, dim3(B), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)d_src, row_bytes / 4,
                       cap, d_counts, B, (uint32_t*)d_dst, d_offsets);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

}  // extern "C"
