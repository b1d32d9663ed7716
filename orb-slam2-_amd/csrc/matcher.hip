// MI355X-native ORBmatcher cores (R/src/ORBmatcher.cpp; R/ = /root/reference/ORB-SLAM2注释版/).
//
// The reference's searches are sequential and greedy: a later query sees the
// matches (and stolen matches) of every earlier one.  They are
// restated as two gfx950 kernels per frame pair:
//   k_cand_*   — parallel: one wave per query enumerates the GetFeaturesInArea
//                candidates (R/src/Frame.cpp:387-440) and their Hamming distances
//                (wave64 XOR + v_bcnt over 8 dwords, R/src/ORBmatcher.cpp:1901-1917);
//   k_resolve_* — one wave per frame pair replays the queries in order, keeping the
//                greedy state (vMatchedDistance / vnMatches21 / occupied slots) in
//                LDS and reducing each query's candidates with wave reductions whose
//                tie-break is the reference's candidate order (cell-major, then index).
// The rotation-consistency histogram (HISTO_LENGTH=30, ComputeThreeMaxima) runs at
// the end of the resolve kernel.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <vector>

#include "common.h"

namespace orbamd {

constexpr int kGridCols = 64;    // FRAME_GRID_COLS (R/include/Frame.h:38)
constexpr int kGridRows = 48;    // FRAME_GRID_ROWS
constexpr int kHisto = 30;       // HISTO_LENGTH
constexpr int kThLow = 50;       // TH_LOW
constexpr int kThHigh = 100;     // TH_HIGH
constexpr size_t kMaxLds = 160 * 1024;   // LDS of one gfx950 workgroup
constexpr int kMaxCand = 1024;   // per-query candidate list capacity (overflow -> status)

struct GridParams {
    float min_x, min_y, max_x, max_y, winv, hinv;
};

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
    const uint4* pa = reinterpret_cast<const uint4*>(a);
    const uint4* pb = reinterpret_cast<const uint4*>(b);
    const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// PosInGrid (R/src/Frame.cpp:442-452); returns cell key ix*48+iy or -1.
__device__ __forceinline__ int grid_cell(const GridParams& g, float x, float y) {
    const int px = (int)roundf((x - g.min_x) * g.winv);
    const int py = (int)roundf((y - g.min_y) * g.hinv);
    if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return -1;
    return px * kGridRows + py;
}

struct AreaQuery {
    int cx0, cx1, cy0, cy1;   // inclusive cell ranges; cx0 > cx1 -> empty
    bool checkLevels;
    int minLevel, maxLevel;
    float x, y, r;
};

// GetFeaturesInArea bounds (R/src/Frame.cpp:392-408).
__device__ __forceinline__ AreaQuery make_area(const GridParams& g, float x, float y, float r, int minLevel,
                                               int maxLevel) {
    AreaQuery q;
    q.x = x; q.y = y; q.r = r;
    q.minLevel = minLevel; q.maxLevel = maxLevel;
    q.checkLevels = (minLevel > 0) || (maxLevel >= 0);
    q.cx0 = max(0, (int)floorf((x - g.min_x - r) * g.winv));
    q.cx1 = min(kGridCols - 1, (int)ceilf((x - g.min_x + r) * g.winv));
    q.cy0 = max(0, (int)floorf((y - g.min_y - r) * g.hinv));
    q.cy1 = min(kGridRows - 1, (int)ceilf((y - g.min_y + r) * g.hinv));
    if (q.cx0 >= kGridCols || q.cx1 < 0 || q.cy0 >= kGridRows || q.cy1 < 0) q.cx0 = 1, q.cx1 = 0;
    return q;
}

__device__ __forceinline__ bool in_area(const AreaQuery& q, int cell, int octave, float kx, float ky) {
    if (cell < 0) return false;
    const int ix = cell / kGridRows, iy = cell % kGridRows;
    if (ix < q.cx0 || ix > q.cx1 || iy < q.cy0 || iy > q.cy1) return false;
    if (q.checkLevels) {
        if (octave < q.minLevel) return false;
        if (q.maxLevel >= 0 && octave > q.maxLevel) return false;
    }
    const float dx = kx - q.x, dy = ky - q.y;
    return fabsf(dx) < q.r && fabsf(dy) < q.r;
}

__device__ __forceinline__ int rot_bin(float rot) {
    const float factor = kHisto / 360.0f;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == kHisto) bin = 0;
    return bin;
}

// ---------------------------------------------------------------- wave reductions

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return v;
}

// Best (dist, order) and the multiset-second-smallest distance of a candidate set: this
// is exactly what the reference's `if(dist<best){best2=best;...} else if(dist<best2)` loop
// returns for any visiting order, with ties resolved by the visiting order.
struct Best2 {
    int best, best2, idx;
};
__device__ __forceinline__ Best2 wave_best2(int d, unsigned order, int idx, bool valid) {
    const unsigned long long key = valid ? (((unsigned long long)(unsigned)d << 40) | ((unsigned long long)order << 20) |
                                            (unsigned long long)(unsigned)idx)
                                         : ~0ull;
    const unsigned long long m = wave_min_u64(key);
    Best2 r;
    if (m == ~0ull) { r.best = INT_MAX; r.best2 = INT_MAX; r.idx = -1; return r; }
    r.best = (int)(m >> 40);
    r.idx = (int)(m & 0xFFFFFull);
    // second: another candidate with the same distance, else the smallest larger distance
    const bool isArg = valid && key == m;
    const int d2 = (valid && !isArg) ? d : INT_MAX;
    r.best2 = wave_min_i32(d2);
    return r;
}

// ---------------------------------------------------------------- SearchForInitialization

constexpr int kTopK = 8;   // candidates kept per query, in the reference's preference order

#ifdef ORB_TIMING   // instrumented variant (tools/build_variant.py): per-phase clocks of one wave
#define TSTAMP(v) const long long v = clock64()
#define TACC(acc, a) acc += clock64() - (a)
#else
#define TSTAMP(v)
#define TACC(acc, a)
#endif

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// F2's octave-0 keypoints bucketed by grid cell, in the order Frame::AssignFeaturesToGrid
// fills mGrid (R/src/Frame.cpp:244-260): per pair, cellStart[0..3072] (prefix over cell key
// ix*48+iy) and the keypoint index / position of each bucket entry.  SearchForInitialization
// only asks for level-0 keypoints (minLevel = maxLevel = 0), so only those are bucketed.
constexpr int kCells = kGridCols * kGridRows;

__global__ __launch_bounds__(256) void k_grid_sfi(const orb_keypoint* __restrict__ kps2, const int32_t* __restrict__ n2s,
                                                  int cap, GridParams g, int* __restrict__ cellStart,
                                                  int* __restrict__ gj, float2* __restrict__ gxy) {
    __shared__ int cnt[kCells + 1];
    __shared__ int wsum[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n2 = min((int)n2s[b], cap);
    const orb_keypoint* K2 = kps2 + (size_t)b * cap;
    int* CS = cellStart + (size_t)b * (kCells + 1);
    int* GJ = gj + (size_t)b * cap;
    float2* GXY = gxy + (size_t)b * cap;
    for (int c = tid; c <= kCells; c += 256) cnt[c] = 0;
    __syncthreads();
    for (int j = tid; j < n2; j += 256) {
        const orb_keypoint k = K2[j];
        if (k.octave != 0) continue;
        const int c = grid_cell(g, k.x, k.y);
        if (c >= 0) atomicAdd(&cnt[c], 1);
    }
    __syncthreads();
    // exclusive scan of the 3072 counts: 12 per thread
    constexpr int kPer = kCells / 256;
    int loc[kPer], s = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) { loc[u] = cnt[tid * kPer + u]; s += loc[u]; }
    const int incl = wave_incl_scan_i32(s);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int run = incl - s;
    for (int w = 0; w < wid; w++) run += wsum[w];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        cnt[tid * kPer + u] = run;
        CS[tid * kPer + u] = run;
        run += loc[u];
    }
    if (tid == 0) CS[kCells] = total;
    __syncthreads();
    for (int j = tid; j < n2; j += 256) {
        const orb_keypoint k = K2[j];
        if (k.octave != 0) continue;
        const int c = grid_cell(g, k.x, k.y);
        if (c < 0) continue;
        const int pos = atomicAdd(&cnt[c], 1);
        GJ[pos] = j;
    }
    __syncthreads();
    // restore ascending keypoint order inside every cell (insertion sort; cells hold a few)
    for (int c = tid; c < kCells; c += 256) {
        const int s0 = CS[c], s1 = CS[c + 1];
        for (int a = s0 + 1; a < s1; a++) {
            const int v = GJ[a];
            int q = a - 1;
            while (q >= s0 && GJ[q] > v) { GJ[q + 1] = GJ[q]; q--; }
            GJ[q + 1] = v;
        }
    }
    __syncthreads();
    for (int p = tid; p < total; p += 256) {
        const orb_keypoint k = K2[GJ[p]];
        GXY[p] = make_float2(k.x, k.y);
    }
}

// Candidate lists for F1 level-0 keypoints, enumerated exactly as GetFeaturesInArea returns
// them (R/src/Frame.cpp:387-440: cell column ix outer, row iy inner, bucket order), so a
// candidate's list position is its visiting order in the reference's loop.
//   cand[b][i1][*] = (i2 | dist << 20) in visiting order, ncand[b][i1] = list length;
//   topk[b][i1][0..7] = the kTopK smallest (dist, position) entries, packed the same way
//   (0xFFFFFFFF past the end).  For the reference's loop (R/src/ORBmatcher.cpp:523-549)
//   the first entry of this order not skipped by vMatchedDistance is bestIdx2 and the next
//   one carries bestDist2, so the sequential replay reads only this prefix.
__device__ __forceinline__ void cand_query(const orb_keypoint& kp1, int i1, int b, int lane, const uint8_t* __restrict__ desc1,
                                           const uint8_t* __restrict__ desc2, const int* __restrict__ cellStart,
                                           const int* __restrict__ gj, const float2* __restrict__ gxy,
                                           const float* __restrict__ prev, int cap, const GridParams& g, float window,
                                           uint32_t* __restrict__ cand, int* __restrict__ ncand,
                                           uint32_t* __restrict__ topk, int* __restrict__ status, int* so, uint32_t* J) {
    int* nc = ncand + (size_t)b * cap + i1;
    float px, py;
    if (prev) { px = prev[((size_t)b * cap + i1) * 2]; py = prev[((size_t)b * cap + i1) * 2 + 1]; }
    else { px = kp1.x; py = kp1.y; }
    const AreaQuery q = make_area(g, px, py, window, 0, 0);
    uint32_t* out = cand + ((size_t)b * cap + i1) * kMaxCand;
    const int* CS = cellStart + (size_t)b * (kCells + 1);
    const int* GJ = gj + (size_t)b * cap;
    const float2* GXY = gxy + (size_t)b * cap;
    const uint4* dq4 = reinterpret_cast<const uint4*>(desc1 + ((size_t)b * cap + i1) * 32);
    const uint4 qa = dq4[0], qb = dq4[1];
    // one lane per grid column of the window: bucket range [cy0, cy1] of that column
    const int ncx = q.cx1 - q.cx0 + 1;   // <= 64
    int segS = 0, segL = 0;
    if (lane < ncx) {
        const int c0 = (q.cx0 + lane) * kGridRows + q.cy0;
        segS = CS[c0];
        segL = CS[c0 + (q.cy1 - q.cy0) + 1] - segS;
    }
    const int incl = wave_incl_scan_dpp(segL);   // (the whole wave runs a query)
    const int T = __builtin_amdgcn_readlane(incl, 63);
    if (lane < ncx) so[lane] = incl - segL;
    if (lane == 0) so[kGridCols] = T;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int n = 0;
    for (int t0 = 0; t0 < T; t0 += 64) {
        const int t = t0 + lane;
        bool ok = false;
        int d = 0, j = 0;
        int seg = 0;   // window column of entry t: last column whose offset <= t
        if (t < T) {
            int lo = 0, hi = ncx - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (so[mid] <= t) lo = mid; else hi = mid - 1;
            }
            seg = lo;
        }
        const int base = __shfl(segS, seg, 64);
        if (t < T) {
            const int p = base + (t - so[seg]);
            const float2 xy = GXY[p];
            ok = fabsf(xy.x - q.x) < q.r && fabsf(xy.y - q.y) < q.r;
            if (ok) {
                j = GJ[p];
                const uint4* d4 = reinterpret_cast<const uint4*>(desc2 + ((size_t)b * cap + j) * 32);
                const uint4 a0 = d4[0], a1 = d4[1];
                d = __popc(a0.x ^ qa.x) + __popc(a0.y ^ qa.y) + __popc(a0.z ^ qa.z) + __popc(a0.w ^ qa.w) +
                    __popc(a1.x ^ qb.x) + __popc(a1.y ^ qb.y) + __popc(a1.z ^ qb.z) + __popc(a1.w ^ qb.w);
            }
        }
        const uint64_t m = __ballot(ok);
        const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
        if (ok && pos < kMaxCand) {
            const uint32_t e = (uint32_t)j | ((uint32_t)d << 20);
            out[pos] = e;
            J[pos] = e;
        }
        n += __popcll(m);
    }
    if (n > kMaxCand) {
        if (lane == 0) atomicOr(status, 1);
        n = kMaxCand;
    }
    if (lane == 0) *nc = n;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // top-K by (dist, list position): 32-bit keys dist << 11 | position
    uint32_t run = ~0u;
    for (int c0 = 0; c0 < n; c0 += 64) {
        uint32_t v = (c0 + lane < n) ? ((J[c0 + lane] >> 20) << 11) | (uint32_t)(c0 + lane) : ~0u;
#pragma unroll
        for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
            for (int jj = k >> 1; jj > 0; jj >>= 1) {
                const uint32_t o = __shfl_xor(v, jj, 64);
                const bool takeMin = ((lane & jj) == 0) == ((lane & k) == 0);
                v = takeMin ? min(o, v) : max(o, v);
            }
        }
        if (c0 == 0) {
            run = v;
        } else {
            const uint32_t rev = __shfl(v, (kTopK - 1 - lane) & 63, 64);
            uint32_t t = lane < kTopK ? min(run, rev) : ~0u;
#pragma unroll
            for (int s2 = kTopK >> 1; s2 > 0; s2 >>= 1) {
                const uint32_t o = __shfl_xor(t, s2, 64);
                t = ((lane & s2) == 0) ? min(o, t) : max(o, t);
            }
            run = t;
        }
    }
    if (lane < kTopK) {
        uint32_t* tk = topk + ((size_t)b * cap + i1) * kTopK;
        tk[lane] = run == ~0u ? ~0u : J[run & 0x7FFu];
    }
}


// One wave per query would launch a wave for every keypoint slot of every frame although only
// the level-0 queries (about a fifth, and the first ones: keypoints are concatenated by level)
// do work.  Instead kCandWaves waves per frame: wave w owns queries w, w + kCandWaves, ...; it
// reads their octaves in one load per lane, zeroes the candidate count of the others in
// parallel, and runs cand_query on its level-0 ones.
constexpr int kCandWaves = 128;
__global__ __launch_bounds__(256) void k_cand_sfi(const orb_keypoint* __restrict__ kps1, const uint8_t* __restrict__ desc1,
                                                  const int32_t* __restrict__ n1s, const uint8_t* __restrict__ desc2,
                                                  const int* __restrict__ cellStart, const int* __restrict__ gj,
                                                  const float2* __restrict__ gxy, const float* __restrict__ prev,
                                                  int cap, GridParams g, float window, uint32_t* __restrict__ cand,
                                                  int* __restrict__ ncand, uint32_t* __restrict__ topk,
                                                  int* __restrict__ status) {
    __shared__ int segOff[4][kGridCols + 1];
    __shared__ uint32_t sj[4][kMaxCand];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int bx, b;
    xcd_block_2d(bx, b);
    const int w = bx * 4 + wid;
    const int n1 = min((int)n1s[b], cap);
    const orb_keypoint* K1 = kps1 + (size_t)b * cap;
    int* NC = ncand + (size_t)b * cap;
    for (int base = w; base < n1; base += kCandWaves * 64) {
        const int iq = base + kCandWaves * lane;
        const bool in = iq < n1;
        const int oct = K1[in ? iq : 0].octave;
        if (in && oct > 0) NC[iq] = 0;
        uint64_t act = __ballot(in && oct == 0);
        while (act) {
            const int k = __builtin_ctzll(act);
            act &= act - 1;
            const int i1 = base + kCandWaves * k;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();   // the wave's LDS scratch is reused query after query
            cand_query(K1[i1], i1, b, lane, desc1, desc2, cellStart, gj, gxy, prev, cap, g, window, cand, ncand, topk,
                       status, segOff[wid], sj[wid]);
        }
    }
}

// SearchForInitialization's sequential loop (R/src/ORBmatcher.cpp:512-566) for one frame pair per
// 256-thread workgroup, as the fixpoint of a parallel iteration.  A query's decision (bestIdx2,
// bestDist or none) depends on the state vMatchedDistance has when the loop reaches it, and that
// state is fixed by the decisions of the earlier queries alone: vMatchedDistance[i2] is the
// smallest bestDist among the earlier queries that matched i2 (a later match of i2 passed the
// `vMatchedDistance[i2] <= dist` skip test, so it is strictly smaller), INT_MAX if none did.
// Iteration t recomputes every query's decision from the decisions of iteration t-1 (Jacobi
// sweep; iteration 0 assumes no match).  Query k is exact from iteration k on, so the sweeps
// reach a fixpoint, and at a fixpoint every query sees the sequential state (induction over the
// query order): the fixpoint is the sequential result.  Conflicts between nearby queries are
// rare, so a pair takes a few sweeps.
//   sweep = (A) claim lists: every matched query links itself into the list of its keypoint
//           (LDS head stamped with the sweep number, so no reset); (B) per query: its top-K
//           candidates (distance, visiting order) probe the state through the lists, the first
//           survivor is bestIdx2 and the second carries bestDist2; a query with fewer than two
//           survivors among the top-K and a longer list is (F) rescanned over its whole list by
//           a wave.
// vnMatches12 follows: a query keeps its match iff it is the last query that matched the keypoint
// (a later one stole it), and every query that ever matched sits in the rotation histogram, as
// rotHist[bin].push_back(i1) does; then ComputeThreeMaxima (:1854-1895) filters.
constexpr int kRsT = 256;
__global__ __launch_bounds__(kRsT) void k_resolve_sfi(const orb_keypoint* __restrict__ kps1, const int32_t* __restrict__ n1s,
                                                      const orb_keypoint* __restrict__ kps2, const int32_t* __restrict__ n2s,
                                                      int cap, float nnratio, int checkOri,
                                                      const uint32_t* __restrict__ cand, const int* __restrict__ ncand,
                                                      const uint32_t* __restrict__ topk, float* __restrict__ prev,
                                                      int32_t* __restrict__ matches12, int32_t* __restrict__ nmatches_out,
                                                      int* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) int sm[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b = blockIdx.x;
    const int n1 = min((int)n1s[b], cap), n2 = min((int)n2s[b], cap);
    int* qidx = sm;                  // [cap] i1 of the active query of rank q (ascending i1)
    int* qnc = qidx + cap;           // [cap] its candidate count
    int* dec0 = qnc + cap;           // [cap] decision per rank, ping-pong: i2 | bestDist << 20, -1 = none
    int* dec1 = dec0 + cap;
    int* nxt = dec1 + cap;           // [cap] claim list link
    int* fbq = nxt + cap;            // [cap] queries rescanned this sweep; later i1 -> rank
    int* head = fbq + cap;           // [cap] per F2 keypoint: claim list head (sweep << 16 | rank); later last claimant
    int* qrank = head + cap;         // [cap] rank of query i1, -1 if inactive
    int* hcount = qrank + cap;       // [32]
    int* sc = hcount + 32;           // [16] uniform scalars
    const orb_keypoint* K1 = kps1 + (size_t)b * cap;
    const orb_keypoint* K2 = kps2 + (size_t)b * cap;
    const uint32_t* TK = topk + (size_t)b * cap * kTopK;
    const int* NC = ncand + (size_t)b * cap;
    const uint32_t* CAND = cand + (size_t)b * cap * kMaxCand;
    // ---- active queries (non-empty window) compacted in i1 order: contiguous chunk per thread
    const int chunk = (n1 + kRsT - 1) / kRsT;
    const int c0 = min(tid * chunk, n1), c1 = min(c0 + chunk, n1);
    int loc = 0;
    for (int i = c0; i < c1; i++) loc += NC[i] > 0 ? 1 : 0;
    {
        const int incl = wave_incl_scan_i32(loc);
        if (lane == 63) sc[8 + wid] = incl;
        for (int j = tid; j < n2; j += kRsT) head[j] = -1;
        if (tid < 32) hcount[tid] = 0;
        if (tid < 6) sc[tid] = 0;
        __syncthreads();
        int run = incl - loc;
        for (int w = 0; w < wid; w++) run += sc[8 + w];
        for (int i = c0; i < c1; i++) {
            const int nc = NC[i];
            qrank[i] = -1;
            if (nc > 0) { qidx[run] = i; qnc[run] = nc; dec0[run] = -1; qrank[i] = run; run++; }
        }
    }
    const int na = sc[8] + sc[9] + sc[10] + sc[11];
    __syncthreads();
    int* dcur = dec0;
    int* dnew = dec1;
    int it = 0;
    for (;; it++) {
        if (it > na + 1) { if (tid == 0) atomicOr(status, 2); break; }   // unreachable: converges by sweep na
        // (A) claim lists of the current decisions
        for (int q = tid; q < na; q += kRsT) {
            const int dq = dcur[q];
            if (dq < 0) continue;
            const int old = atomicExch(&head[dq & 0xFFFFF], (it << 16) | q);
            nxt[q] = (old >> 16) == it ? (old & 0xFFFF) : -1;
        }
        // convergence flags rotate through three slots: the slot cleared here (the next sweep's) is
        // neither this sweep's nor the previous one, which a slower wave may still be reading below
        if (tid == 0) { sc[(it + 1) % 3] = 0; sc[4 + ((it + 1) & 1)] = 0; }
        __syncthreads();
        // state seen by query q at keypoint j: smallest bestDist of an earlier query that matched j
        auto seen = [&](int j, int q) {
            int s = INT_MAX;
            const int h = head[j];
            int u = (h >> 16) == it ? (h & 0xFFFF) : -1;
            while (u >= 0) {
                if (u < q) s = min(s, dcur[u] >> 20);
                u = nxt[u];
            }
            return s;
        };
        // (B) decisions from the top-K lists
        for (int q = tid; q < na; q += kRsT) {
            const int nc = qnc[q];
            const uint4* t4 = reinterpret_cast<const uint4*>(TK + (size_t)qidx[q] * kTopK);
            const uint4 ta = t4[0], tb = t4[1];
            const uint32_t e[kTopK] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
            const int kn = min(nc, kTopK);
            int f = -1, f2 = -1;
#pragma unroll
            for (int k = 0; k < kTopK; k++) {
                if (k < kn && f2 < 0) {
                    const int j = (int)(e[k] & 0xFFFFFu), d = (int)(e[k] >> 20);
                    if (seen(j, q) > d) {
                        if (f < 0) f = k; else f2 = k;
                    }
                }
            }
            if (f2 < 0 && nc > kTopK) {      // fewer than two survivors among the top-K
                fbq[atomicAdd(&sc[4 + (it & 1)], 1)] = q;
                continue;
            }
            int nd = -1;
            if (f >= 0) {
                const int bd = (int)(e[f] >> 20);
                const int b2 = f2 >= 0 ? (int)(e[f2] >> 20) : INT_MAX;
                if (bd <= kThLow && (float)bd < (float)b2 * nnratio) nd = (int)e[f];
            }
            dnew[q] = nd;
            if (nd != dcur[q]) sc[it % 3] = 1;
        }
        __syncthreads();
        // (F) whole-list rescans, one wave per query: best = smallest (dist, visiting position) among
        //     the survivors, bestDist2 = the multiset second smallest (the reference's running pair)
        const int nfb = sc[4 + (it & 1)];
        for (int f = wid; f < nfb; f += kRsT / 64) {
            const int q = fbq[f];
            const int nc = min(qnc[q], kMaxCand);
            const uint32_t* L = CAND + (size_t)qidx[q] * kMaxCand;
            unsigned long long bestKey = ~0ull;   // dist << 32 | position << 20 | i2
            int best2 = INT_MAX;
            for (int cb = 0; cb < nc; cb += 64) {
                const int c = cb + lane;
                bool ok = false;
                int d = 0, j = 0;
                if (c < nc) {
                    const uint32_t ce = L[c];
                    j = (int)(ce & 0xFFFFFu);
                    d = (int)(ce >> 20);
                    ok = seen(j, q) > d;
                }
                const unsigned long long key = ok ? (((unsigned long long)d << 32) | ((unsigned long long)c << 20) | (unsigned)j) : ~0ull;
                const unsigned long long mk = wave_min_u64(key);
                // second: the chunk's other survivors and the previous running pair
                const int d2 = (ok && key != mk) ? d : INT_MAX;
                const int cb2 = wave_min_i32(d2);
                if (mk != ~0ull) {
                    const int mkd = (int)(mk >> 32);
                    if (mk < bestKey) {
                        best2 = min(bestKey == ~0ull ? INT_MAX : (int)(bestKey >> 32), min(best2, cb2));
                        bestKey = mk;
                    } else {
                        best2 = min(best2, min(mkd, cb2));
                    }
                }
            }
            if (lane == 0) {
                int nd = -1;
                if (bestKey != ~0ull) {
                    const int bd = (int)(bestKey >> 32);
                    if (bd <= kThLow && (float)bd < (float)best2 * nnratio) nd = (int)(bestKey & 0xFFFFFull) | (bd << 20);
                }
                dnew[q] = nd;
                if (nd != dcur[q]) sc[it % 3] = 1;
            }
        }
        __syncthreads();
        const bool again = sc[it % 3] != 0;
        int* t = dcur; dcur = dnew; dnew = t;
        if (!again) break;
    }
    __syncthreads();
    // ---- last claimant per keypoint (vnMatches21), rotation histogram of every match
    for (int j = tid; j < n2; j += kRsT) head[j] = -1;
    __syncthreads();
    for (int q = tid; q < na; q += kRsT) {
        const int dq = dcur[q];
        if (dq < 0) continue;
        const int j = dq & 0xFFFFF;
        atomicMax(&head[j], q);
        if (checkOri) atomicAdd(&hcount[rot_bin(K1[qidx[q]].angle - K2[j].angle)], 1);
    }
    __syncthreads();
    int ind1 = -1, ind2 = -1, ind3 = -1;
    if (checkOri) {
        // ComputeThreeMaxima (R/src/ORBmatcher.cpp:1854-1895)
        int max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < kHisto; i++) {
            const int s = hcount[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
    }
    int32_t* m12 = matches12 + (size_t)b * cap;
    int kept = 0;
    for (int i = tid; i < n1; i += kRsT) {
        const int q = qrank[i];
        int j = -1;
        if (q >= 0) {
            const int dq = dcur[q];
            if (dq >= 0 && head[dq & 0xFFFFF] == q) {
                j = dq & 0xFFFFF;
                if (checkOri) {
                    const int bin = rot_bin(K1[i].angle - K2[j].angle);
                    if (bin != ind1 && bin != ind2 && bin != ind3) j = -1;
                }
            }
        }
        m12[i] = j;
        if (j >= 0) {
            kept++;
            if (prev) {
                const orb_keypoint k2 = K2[j];
                prev[((size_t)b * cap + i) * 2] = k2.x;
                prev[((size_t)b * cap + i) * 2 + 1] = k2.y;
            }
        }
    }
    kept = wave_reduce_sum_i32(kept);
    if (lane == 0) sc[12 + wid] = kept;
    __syncthreads();
    if (tid == 0) nmatches_out[b] = sc[12] + sc[13] + sc[14] + sc[15];
}

static size_t resolve_sfi_lds(int cap) { return (8 * (size_t)cap + 32 + 16) * 4; }

// ---------------------------------------------------------------- SearchByProjection(Frame, Frame)

struct SbpCam {
    float fx, fy, cx, cy, mbf, mb;
};

// One wave per last-frame keypoint: projection + candidates (R/src/ORBmatcher.cpp:1590-1671).
__global__ __launch_bounds__(256) void k_cand_sbp(const orb_keypoint* __restrict__ kc, const uint8_t* __restrict__ dc,
                                                  const float* __restrict__ urc, int nc_, const orb_keypoint* __restrict__ kl,
                                                  int nl, const int32_t* __restrict__ hasMp, const uint8_t* __restrict__ outl,
                                                  const float* __restrict__ mpXYZ, const uint8_t* __restrict__ mpDesc,
                                                  const float* __restrict__ Tcw, const float* __restrict__ sf, SbpCam cam,
                                                  GridParams g, float th, int bForward, int bBackward,
                                                  uint32_t* __restrict__ cand, int* __restrict__ ncand, int* __restrict__ status) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wid;
    if (i >= nl) return;
    int* ncount = ncand + i;
    if (!hasMp[i] || outl[i]) { if (lane == 0) *ncount = 0; return; }
    float x3[3];
    const float* X = mpXYZ + 3 * (size_t)i;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double s = (double)Tcw[4 * r] * X[0] + (double)Tcw[4 * r + 1] * X[1] + (double)Tcw[4 * r + 2] * X[2];
        x3[r] = (float)(s + (double)Tcw[4 * r + 3]);
    }
    const float xc = x3[0], yc = x3[1];
    const float invzc = (float)(1.0 / (double)x3[2]);
    if (invzc < 0) { if (lane == 0) *ncount = 0; return; }
    const float u = cam.fx * xc * invzc + cam.cx;
    const float v = cam.fy * yc * invzc + cam.cy;
    if (u < g.min_x || u > g.max_x || v < g.min_y || v > g.max_y) { if (lane == 0) *ncount = 0; return; }
    const int nLastOctave = kl[i].octave;
    const float radius = th * sf[nLastOctave];
    AreaQuery q;
    if (bForward) q = make_area(g, u, v, radius, nLastOctave, -1);
    else if (bBackward) q = make_area(g, u, v, radius, 0, nLastOctave);
    else q = make_area(g, u, v, radius, nLastOctave - 1, nLastOctave + 1);
    const float ur = u - cam.mbf * invzc;
    uint32_t* out = cand + (size_t)i * kMaxCand;
    const uint8_t* dq = mpDesc + (size_t)i * 32;
    int n = 0;
    for (int j0 = 0; j0 < nc_; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        int d = 0;
        if (j < nc_ && q.cx0 <= q.cx1) {
            const orb_keypoint k2 = kc[j];
            ok = in_area(q, grid_cell(g, k2.x, k2.y), k2.octave, k2.x, k2.y);
            if (ok && urc && urc[j] > 0) {
                const float er = fabsf(ur - urc[j]);
                if (er > radius) ok = false;
            }
            if (ok) d = hamming32(dq, dc + (size_t)j * 32);
        }
        const uint64_t m = __ballot(ok);
        const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
        if (ok && pos < kMaxCand) out[pos] = (uint32_t)j | ((uint32_t)d << 20);
        n += __popcll(m);
    }
    if (lane == 0) {
        if (n > kMaxCand) { atomicOr(status, 1); n = kMaxCand; }
        *ncount = n;
    }
}

__global__ __launch_bounds__(64) void k_resolve_sbp(const orb_keypoint* __restrict__ kc, int ncur,
                                                    const orb_keypoint* __restrict__ kl, int nl, GridParams g,
                                                    int checkOri, const uint32_t* __restrict__ cand,
                                                    const int* __restrict__ ncand, int32_t* __restrict__ curMp,
                                                    int32_t* __restrict__ nmatches_out, int32_t* __restrict__ histIdx,
                                                    uint8_t* __restrict__ histBin, int thDist,
                                                    const int32_t* __restrict__ lastHas) {
    extern __shared__ __attribute__((aligned(16))) int sm[];
    const int lane = threadIdx.x;
    int* ckey = sm;              // [ncur]
    int* hcount = sm + ncur;     // [kHisto]
    for (int j = lane; j < ncur; j += 64) ckey[j] = grid_cell(g, kc[j].x, kc[j].y);
    if (lane < kHisto) hcount[lane] = 0;
    __syncthreads();
    int nmatches = 0, nh = 0;
    for (int i = 0; i < nl; i++) {
        const int nc = ncand[i];
        if (nc == 0) continue;
        const uint32_t* C = cand + (size_t)i * kMaxCand;
        unsigned long long accKey = ~0ull;
        for (int c0 = 0; c0 < nc; c0 += 64) {
            const int c = c0 + lane;
            unsigned long long key = ~0ull;
            if (c < nc) {
                const uint32_t e = C[c];
                const int j = (int)(e & 0xFFFFFu), d = (int)(e >> 20);
                // occupied slots are skipped (R :1649-1651), but only when the slot's map point has
                // observations: with lastHas (the Frame form) a slot holding a point without any
                // (-3 on entry, or one this call assigned from a last-frame point marked 2: the
                // temporal visual-odometry points of Tracking::UpdateLastFrame) stays a candidate
                const int cm = curMp[j];
                if (cm == -1 || (lastHas && (cm == -3 || (cm >= 0 && lastHas[cm] == 2))))
                    key = ((unsigned long long)(unsigned)d << 40) | ((unsigned long long)(unsigned)ckey[j] << 20) |
                          (unsigned long long)(unsigned)j;
            }
            const unsigned long long m = wave_min_u64(key);
            accKey = m < accKey ? m : accKey;
        }
        if (accKey == ~0ull) continue;
        const int bestDist = (int)(accKey >> 40), bestIdx2 = (int)(accKey & 0xFFFFFull);
        if (bestDist <= thDist) {   // TH_HIGH (:1671), ORBdist for the relocalisation form (:1789)
            if (lane == 0) {
                curMp[bestIdx2] = i;
                if (checkOri) {
                    const int bin = rot_bin(kl[i].angle - kc[bestIdx2].angle);
                    histIdx[nh] = bestIdx2;
                    histBin[nh] = (uint8_t)bin;
                    hcount[bin]++;
                }
            }
            nmatches++;
            if (checkOri) nh++;
            __syncthreads();
        }
    }
    __syncthreads();
    if (checkOri) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHisto; i++) {
            const int s = hcount[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        int removed = 0;
        for (int e = lane; e < nh; e += 64) {
            const int bin = histBin[e];
            if (bin == ind1 || bin == ind2 || bin == ind3) continue;
            curMp[histIdx[e]] = -1;
            removed++;
        }
        nmatches -= wave_reduce_sum_i32(removed);
    }
    if (lane == 0) *nmatches_out = nmatches;
}

// The replay above is one wave walking the points in order, three dependent global round trips each
// (~0.7 us per point: 550-700 us for 800 points).  Its fast form: k_best_sbp finds every point's best
// candidate against the slot occupancy at entry, all points in parallel (one wave each), and
// k_resolve_sbp_lds replays with the occupancy, the grid-cell keys and those bests in LDS.  A slot's
// eligibility only ever goes from true to false during the replay (an assignment makes it ineligible
// unless the assigned point is a visual-odometry one, lastHas == 2), so a point whose entry-time best
// slot is still eligible keeps it: the reference's scan over its candidates (R/src/ORBmatcher.cpp:
// 1640-1671) would pick the same minimum; only a point whose best slot was taken re-scans its list.
__global__ __launch_bounds__(256) void k_best_sbp(const orb_keypoint* __restrict__ kc, const orb_keypoint* __restrict__ kl,
                                                  int nl, GridParams g, int checkOri, const uint32_t* __restrict__ cand,
                                                  const int* __restrict__ ncand, const int32_t* __restrict__ curMp,
                                                  const int32_t* __restrict__ lastHas,
                                                  unsigned long long* __restrict__ best) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wid;
    if (i >= nl) return;
    const int nc = ncand[i];
    const uint32_t* C = cand + (size_t)i * kMaxCand;
    unsigned long long acc = ~0ull;
    for (int c0 = 0; c0 < nc; c0 += 64) {
        const int c = c0 + lane;
        unsigned long long key = ~0ull;
        if (c < nc) {
            const uint32_t e = C[c];
            const int j = (int)(e & 0xFFFFFu), d = (int)(e >> 20);
            const int cm = curMp[j];
            if (cm == -1 || (lastHas && (cm == -3 || (cm >= 0 && lastHas[cm] == 2)))) {
                const orb_keypoint k = kc[j];
                key = ((unsigned long long)(unsigned)d << 40) | ((unsigned long long)(unsigned)grid_cell(g, k.x, k.y) << 20) |
                      (unsigned long long)(unsigned)j;
            }
        }
        const unsigned long long m = wave_min_u64(key);
        acc = m < acc ? m : acc;
    }
    if (lane == 0) {
        if (acc != ~0ull && checkOri)   // the rotation bin of this pair rides in bits 56..60
            acc |= (unsigned long long)rot_bin(kl[i].angle - kc[(int)(acc & 0xFFFFFull)].angle) << 56;
        best[i] = acc;
    }
}

static size_t resolve_sbp_lds_bytes(int ncur, int nl) {
    return (size_t)nl * (8 + 4 + 1 + 1) + (size_t)ncur * 12 + (kHisto + 8) * 4 + 64;
}

// The replay, 64 points at a time.  A point whose entry-time best is within the threshold claims its
// slot; the lowest-indexed claimant of each slot is "clean": no earlier point takes that slot through
// its own entry-time best, so the clean point keeps it unless an earlier point re-scans onto it.
// Every other claimant is "dirty" and replays the reference's scan in order against the occupancy so
// far.  Per batch: the clean points before the next dirty one are applied together (one store each),
// the dirty one re-scans (wave-parallel over its list); if it lands on a slot whose clean claimant
// comes later, that claimant turns dirty.  Every point sees exactly the occupancy of the sequential
// replay (R/src/ORBmatcher.cpp:1640-1671 in point order).  Points whose entry-time best is over the
// threshold never assign (a re-scan could only find a worse one) and are skipped.
__global__ __launch_bounds__(64) void k_resolve_sbp_lds(const orb_keypoint* __restrict__ kc, int ncur,
                                                        const orb_keypoint* __restrict__ kl, int nl, GridParams g,
                                                        int checkOri, const uint32_t* __restrict__ cand,
                                                        const int* __restrict__ ncand,
                                                        const unsigned long long* __restrict__ best,
                                                        int32_t* __restrict__ curMp, int32_t* __restrict__ nmatches_out,
                                                        int thDist, const int32_t* __restrict__ lastHas) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smq[];
    unsigned long long* bestL = smq;                 // [nl]
    int* histIdx = (int*)(bestL + nl);               // [nl]
    int* ckey = histIdx + nl;                        // [ncur]
    int* cmL = ckey + ncur;                          // [ncur]
    int* firstL = cmL + ncur;                        // [ncur]
    int* hcount = firstL + ncur;                     // [kHisto]
    uint8_t* histBin = (uint8_t*)(hcount + kHisto + 8);   // [nl]
    uint8_t* dem = histBin + nl;                     // [nl]
    const int lane = threadIdx.x;
    for (int j = lane; j < ncur; j += 64) {
        const orb_keypoint k = kc[j];
        ckey[j] = grid_cell(g, k.x, k.y);
        cmL[j] = curMp[j];
        firstL[j] = 0x7fffffff;
    }
    for (int i = lane; i < nl; i += 64) {
        bestL[i] = best[i];
        dem[i] = 0;
    }
    if (lane < kHisto) hcount[lane] = 0;
    __syncthreads();
    auto claims = [&](unsigned long long key) { return key != ~0ull && (int)((key >> 40) & 0xFFFF) <= thDist; };
    for (int i = lane; i < nl; i += 64) {
        const unsigned long long key = bestL[i];
        if (claims(key)) atomicMin(&firstL[(int)(key & 0xFFFFFull)], i);
    }
    __syncthreads();
    auto elig = [&](int cm) { return cm == -1 || (lastHas && (cm == -3 || (cm >= 0 && lastHas[cm] == 2))); };
    int nmatches = 0, nh = 0;
    for (int base = 0; base < nl; base += 64) {
        const int i = base + lane;
        const unsigned long long key = i < nl ? bestL[i] : ~0ull;
        const bool cl = claims(key);
        const int j = (int)(key & 0xFFFFFull);
        const bool first = cl && firstL[j] == i;
        int pos = 0;
        for (;;) {
            const bool dirty = cl && (!first || dem[i] != 0);
            const uint64_t D = __ballot(dirty && lane >= pos);
            const int nd = D ? (int)__builtin_ctzll(D) : 64;
            // the clean claims in [pos, nd) in one step
            const bool apply = cl && !dirty && lane >= pos && lane < nd;
            const uint64_t A = __ballot(apply);
            if (apply) {
                cmL[j] = i;
                if (checkOri) {
                    const int at = nh + __popcll(A & ((1ull << lane) - 1ull));
                    histIdx[at] = j;
                    histBin[at] = (uint8_t)((key >> 56) & 31);
                }
            }
            nmatches += __popcll(A);
            if (checkOri) nh += __popcll(A);
            if (nd == 64) break;
            // the dirty point at lane nd: the reference's scan against the occupancy so far
            const int id = base + nd;
            const int nc = ncand[id];
            const uint32_t* C = cand + (size_t)id * kMaxCand;
            unsigned long long acc = ~0ull;
            for (int c0 = 0; c0 < nc; c0 += 64) {
                const int c = c0 + lane;
                unsigned long long k2 = ~0ull;
                if (c < nc) {
                    const uint32_t e = C[c];
                    const int jj = (int)(e & 0xFFFFFu), d = (int)(e >> 20);
                    if (elig(cmL[jj]))
                        k2 = ((unsigned long long)(unsigned)d << 40) | ((unsigned long long)(unsigned)ckey[jj] << 20) |
                             (unsigned long long)(unsigned)jj;
                }
                const unsigned long long m = wave_min_u64(k2);
                acc = m < acc ? m : acc;
            }
            if (acc != ~0ull && (int)(acc >> 40) <= thDist) {
                const int js = (int)(acc & 0xFFFFFull);
                const int fc = firstL[js];   // a later clean claimant of this slot loses it
                if (lane == 0) {
                    cmL[js] = id;
                    if (fc > id && fc < nl) dem[fc] = 1;
                    if (checkOri) {
                        histIdx[nh] = js;
                        histBin[nh] = (uint8_t)rot_bin(kl[id].angle - kc[js].angle);
                    }
                }
                nmatches++;
                if (checkOri) nh++;
            }
            pos = nd + 1;
        }
    }
    __syncthreads();
    if (checkOri) {
        for (int e = lane; e < nh; e += 64) atomicAdd(&hcount[histBin[e]], 1);
        __syncthreads();
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int b = 0; b < kHisto; b++) {
            const int c = hcount[b];
            if (c > max1) { max3 = max2; max2 = max1; max1 = c; ind3 = ind2; ind2 = ind1; ind1 = b; }
            else if (c > max2) { max3 = max2; max2 = c; ind3 = ind2; ind2 = b; }
            else if (c > max3) { max3 = c; ind3 = b; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        int removed = 0;
        for (int e = lane; e < nh; e += 64) {
            const int bin = histBin[e];
            if (bin == ind1 || bin == ind2 || bin == ind3) continue;
            cmL[histIdx[e]] = -1;
            removed++;
        }
        nmatches -= wave_reduce_sum_i32(removed);
        __syncthreads();
    }
    for (int j = lane; j < ncur; j += 64) curMp[j] = cmL[j];
    if (lane == 0) *nmatches_out = nmatches;
}

// ---------------------------------------------------------------- SearchByProjection(Frame, KeyFrame, set, th, ORBdist)

struct SbkParams {
    float Tcw[12];
    float Ow[3];
    float fx, fy, cx, cy;
    float logsf;
    int nlev;
    float sf[32];
    float th;
};

// One wave per keyframe map point (Tracking::Relocalization's projection search,
// R/src/ORBmatcher.cpp:1719-1800): Rcw x + tcw (double-accumulated rows rounded to float),
// invzc = 1.0 / z with no depth test, the frame-bounds test, cv::norm(PO) against 0.8 / 1.2 x the
// point's min / max distance, PredictScale on the frame, GetFeaturesInArea(level-1, level+1) and
// the Hamming distances; k_resolve_sbp then replays the keyframe order with the occupancy skip.
__global__ __launch_bounds__(256) void k_cand_sbk(const orb_keypoint* __restrict__ kc, const uint8_t* __restrict__ dc,
                                                  int nc_, int nmp, const uint8_t* __restrict__ valid,
                                                  const float* __restrict__ xyz, const float* __restrict__ mind,
                                                  const float* __restrict__ maxd, const uint8_t* __restrict__ mdesc,
                                                  SbkParams P, GridParams g, uint32_t* __restrict__ cand,
                                                  int* __restrict__ ncand, int* __restrict__ status) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wid;
    if (i >= nmp) return;
    int* ncount = ncand + i;
    if (!valid[i]) { if (lane == 0) *ncount = 0; return; }
    const float* X = xyz + 3 * (size_t)i;
    float x3[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double s = (double)P.Tcw[4 * r] * X[0] + (double)P.Tcw[4 * r + 1] * X[1] + (double)P.Tcw[4 * r + 2] * X[2];
        x3[r] = (float)(s + (double)P.Tcw[4 * r + 3]);
    }
    const float invzc = (float)(1.0 / (double)x3[2]);
    const float u = P.fx * x3[0] * invzc + P.cx;
    const float v = P.fy * x3[1] * invzc + P.cy;
    if (u < g.min_x || u > g.max_x || v < g.min_y || v > g.max_y) { if (lane == 0) *ncount = 0; return; }
    const float PO[3] = {X[0] - P.Ow[0], X[1] - P.Ow[1], X[2] - P.Ow[2]};
    const float ss = (PO[0] * PO[0] + PO[1] * PO[1]) + PO[2] * PO[2];
    const float dist3D = (float)sqrt((double)ss);
    const float maxDistance = 1.2f * maxd[i], minDistance = 0.8f * mind[i];
    if (dist3D < minDistance || dist3D > maxDistance) { if (lane == 0) *ncount = 0; return; }
    const float ratio = maxd[i] / dist3D;
    int lev = (int)ceil(log((double)ratio) / (double)P.logsf);
    if (lev < 0) lev = 0;
    else if (lev >= P.nlev) lev = P.nlev - 1;
    const float radius = P.th * P.sf[lev];
    const AreaQuery q = make_area(g, u, v, radius, lev - 1, lev + 1);
    uint32_t* out = cand + (size_t)i * kMaxCand;
    const uint8_t* dq = mdesc + (size_t)i * 32;
    int n = 0;
    for (int j0 = 0; j0 < nc_; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        int d = 0;
        if (j < nc_ && q.cx0 <= q.cx1) {
            const orb_keypoint k2 = kc[j];
            ok = in_area(q, grid_cell(g, k2.x, k2.y), k2.octave, k2.x, k2.y);
            if (ok) d = hamming32(dq, dc + (size_t)j * 32);
        }
        const uint64_t m = __ballot(ok);
        const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
        if (ok && pos < kMaxCand) out[pos] = (uint32_t)j | ((uint32_t)d << 20);
        n += __popcll(m);
    }
    if (lane == 0) {
        if (n > kMaxCand) { atomicOr(status, 1); n = kMaxCand; }
        *ncount = n;
    }
}

// ---------------------------------------------------------------- SearchByProjection(Frame, local map points)

// One wave per local map point: RadiusByViewingCos window, GetFeaturesInArea(level-1, level),
// the stereo reprojection gate and the Hamming distances (R/src/ORBmatcher.cpp:63-137).
__global__ __launch_bounds__(256) void k_cand_sbl(const orb_keypoint* __restrict__ kc, const uint8_t* __restrict__ dc,
                                                  const float* __restrict__ urc, int nc_, int nmp,
                                                  const uint8_t* __restrict__ inView, const float* __restrict__ proj,
                                                  const int32_t* __restrict__ lvl, const float* __restrict__ vcos,
                                                  const uint8_t* __restrict__ mpDesc, const float* __restrict__ sf,
                                                  GridParams g, float th, uint32_t* __restrict__ cand,
                                                  int* __restrict__ ncand, int* __restrict__ status) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wid;
    if (i >= nmp) return;
    int* ncount = ncand + i;
    if (!inView[i]) { if (lane == 0) *ncount = 0; return; }
    const int level = lvl[i];
    float r = vcos[i] > 0.998f ? 2.5f : 4.0f;   // RadiusByViewingCos (R :166-172)
    if (th != 1.0f) r *= th;
    const float rad = r * sf[level];
    const float px = proj[3 * (size_t)i], py = proj[3 * (size_t)i + 1], pxr = proj[3 * (size_t)i + 2];
    const AreaQuery q = make_area(g, px, py, rad, level - 1, level);
    uint32_t* out = cand + (size_t)i * kMaxCand;
    const uint8_t* dq = mpDesc + (size_t)i * 32;
    int n = 0;
    for (int j0 = 0; j0 < nc_; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        int d = 0;
        if (j < nc_ && q.cx0 <= q.cx1) {
            const orb_keypoint k2 = kc[j];
            ok = in_area(q, grid_cell(g, k2.x, k2.y), k2.octave, k2.x, k2.y);
            if (ok && urc && urc[j] > 0) {
                const float er = fabsf(pxr - urc[j]);
                if (er > rad) ok = false;
            }
            if (ok) d = hamming32(dq, dc + (size_t)j * 32);
        }
        const uint64_t m = __ballot(ok);
        const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
        if (ok && pos < kMaxCand) out[pos] = (uint32_t)j | ((uint32_t)d << 20);
        n += __popcll(m);
    }
    if (lane == 0) {
        if (n > kMaxCand) { atomicOr(status, 1); n = kMaxCand; }
        *ncount = n;
    }
}

// Sequential replay over the map points (R :66-160), one wave: a slot matched earlier in the
// call by a map point with observations is skipped by later ones.  Best / second candidate in
// the reference's visiting order (cell-major, then index) from two wave minima per chunk.
__global__ __launch_bounds__(64) void k_resolve_sbl(const orb_keypoint* __restrict__ kc, int ncur, int nmp, GridParams g,
                                                    float nnratio, const uint8_t* __restrict__ hasObs,
                                                    const uint32_t* __restrict__ cand, const int* __restrict__ ncand,
                                                    int32_t* __restrict__ curMpG, int32_t* __restrict__ nmatches_out) {
    extern __shared__ __attribute__((aligned(16))) int sm[];
    const int lane = threadIdx.x;
    int* ckey = sm;              // [ncur]
    int* curMp = sm + ncur;      // [ncur] slot state (see orb_search_by_projection_local)
    for (int j = lane; j < ncur; j += 64) {
        ckey[j] = grid_cell(g, kc[j].x, kc[j].y);
        curMp[j] = curMpG[j];
    }
    __syncthreads();
    int nmatches = 0;
    for (int i = 0; i < nmp; i++) {
        const int nc = ncand[i];
        if (nc == 0) continue;
        const uint32_t* C = cand + (size_t)i * kMaxCand;
        unsigned long long k1 = ~0ull, k2 = ~0ull;   // best and second (dist, visit order, index)
        for (int c0 = 0; c0 < nc; c0 += 64) {
            const int c = c0 + lane;
            unsigned long long key = ~0ull;
            if (c < nc) {
                const uint32_t e = C[c];
                const int j = (int)(e & 0xFFFFFu), d = (int)(e >> 20);
                const int st = curMp[j];
                if (!(st == -2 || (st >= 0 && hasObs[st])))   // `mvpMapPoints[idx]->Observations()>0`
                    key = ((unsigned long long)(unsigned)d << 40) | ((unsigned long long)(unsigned)ckey[j] << 20) |
                          (unsigned long long)(unsigned)j;
            }
            const unsigned long long m1 = wave_min_u64(key);
            const unsigned long long m2 = wave_min_u64(key == m1 ? ~0ull : key);
            if (m1 < k1) {
                k2 = k1 < m2 ? k1 : m2;
                k1 = m1;
            } else {
                k2 = k2 < m1 ? k2 : m1;
            }
        }
        if (k1 == ~0ull) continue;
        const int bestDist = (int)(k1 >> 40), bestIdx = (int)(k1 & 0xFFFFFull);
        if (bestDist > kThHigh) continue;
        const int bestLevel = kc[bestIdx].octave;
        int bestDist2 = 256, bestLevel2 = -1;
        if (k2 != ~0ull) {
            bestDist2 = (int)(k2 >> 40);
            bestLevel2 = kc[(int)(k2 & 0xFFFFFull)].octave;
        }
        // ratio test only if best and second share the scale level (R :151-153)
        if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
        if (lane == 0) curMp[bestIdx] = i;
        nmatches++;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (int j = lane; j < ncur; j += 64) curMpG[j] = curMp[j];
    if (lane == 0) *nmatches_out = nmatches;
}

// ---------------------------------------------------------------- brute-force 2-NN

// One wave per query row: lanes stride over train rows; ties -> lowest train index.
__global__ __launch_bounds__(256) void k_knn2(const uint8_t* __restrict__ q, const int32_t* __restrict__ nqs,
                                              const uint8_t* __restrict__ t, const int32_t* __restrict__ nts, int qStride,
                                              int tStride, int32_t* __restrict__ bi, int32_t* __restrict__ bd,
                                              int32_t* __restrict__ sd) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int bx, b;
    xcd_block_2d(bx, b);
    const int i = bx * 4 + wid;
    const int nq = nqs[b], nt = nts[b];
    if (i >= nq) return;
    const uint8_t* dq = q + ((size_t)b * qStride + i) * 32;
    const uint4 a0 = reinterpret_cast<const uint4*>(dq)[0], a1 = reinterpret_cast<const uint4*>(dq)[1];
    const uint8_t* T = t + (size_t)b * tStride * 32;
    unsigned long long best = ~0ull;
    int second = INT_MAX;
    for (int j = lane; j < nt; j += 64) {
        const uint4* pb = reinterpret_cast<const uint4*>(T + (size_t)j * 32);
        const uint4 b0 = pb[0], b1 = pb[1];
        const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                      __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
        const unsigned long long key = ((unsigned long long)d << 32) | (unsigned)j;
        if (key < best) {
            if (best != ~0ull) second = min(second, (int)(best >> 32));
            best = key;
        } else {
            second = min(second, d);
        }
    }
    const unsigned long long m = wave_min_u64(best);
    // lanes whose best lost contribute it as a second candidate
    const int mine = (best != ~0ull && best != m) ? (int)(best >> 32) : INT_MAX;
    const int s2 = wave_min_i32(min(second, mine));
    if (lane == 0) {
        const size_t o = (size_t)b * qStride + i;
        if (m == ~0ull) { bi[o] = -1; bd[o] = INT_MAX; sd[o] = INT_MAX; }
        else { bi[o] = (int)(m & 0xFFFFFFFFull); bd[o] = (int)(m >> 32); sd[o] = s2; }
    }
}

}  // namespace orbamd

using namespace orbamd;

// ---------------------------------------------------------------- host handle

struct orb_matcher {
    int device = 0;
    float nnratio = 0.6f;
    int checkOri = 1;
    hipStream_t stream = nullptr;
    // device scratch (grown on demand)
    size_t capPairs = 0, capPts = 0;
    orb_keypoint *d_k1 = nullptr, *d_k2 = nullptr;
    uint8_t *d_d1 = nullptr, *d_d2 = nullptr;
    float* d_prev = nullptr;
    float* d_ur = nullptr;
    int32_t *d_n = nullptr, *d_m12 = nullptr, *d_nm = nullptr, *d_hI = nullptr;
    uint8_t* d_hB = nullptr;
    uint32_t* d_cand = nullptr;
    uint32_t* d_topk = nullptr;
    unsigned long long* d_best = nullptr;   // SBP: each point's best candidate at entry
    int *d_cs = nullptr, *d_gj = nullptr;   // SFI grid buckets
    float2* d_gxy = nullptr;
    int *d_ncand = nullptr, *d_status = nullptr;
    hipStream_t batch_stream = nullptr;   // stream of the last orb_search_for_initialization_batch_device
    // SBP extras
    int32_t* d_hasMp = nullptr;
    uint8_t* d_outl = nullptr;
    float *d_xyz = nullptr, *d_T = nullptr, *d_sf = nullptr;
    uint8_t* d_mpd = nullptr;
    void* h_pin = nullptr;
    size_t h_pin_bytes = 0;
    // the per-call host entry points' staging: inputs cross PCIe in one copy, outputs in one (common.h)
    HostScratch hs;
};

static void mfree(orb_matcher* m) {
    void* ptrs[] = {m->d_k1, m->d_k2, m->d_d1, m->d_d2, m->d_prev, m->d_ur, m->d_n, m->d_m12, m->d_nm, m->d_hI,
                    m->d_hB, m->d_cand, m->d_topk, m->d_best, m->d_cs, m->d_gj, m->d_gxy, m->d_ncand, m->d_status, m->d_hasMp, m->d_outl, m->d_xyz, m->d_T,
                    m->d_sf, m->d_mpd};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    m->d_k1 = m->d_k2 = nullptr; m->d_d1 = m->d_d2 = nullptr; m->d_prev = m->d_ur = nullptr;
    m->d_n = m->d_m12 = m->d_nm = m->d_hI = nullptr; m->d_hB = nullptr; m->d_cand = nullptr; m->d_topk = nullptr; m->d_best = nullptr;
    m->d_cs = m->d_gj = nullptr; m->d_gxy = nullptr;
    m->d_ncand = m->d_status = nullptr; m->d_hasMp = nullptr; m->d_outl = nullptr;
    m->d_xyz = m->d_T = m->d_sf = nullptr; m->d_mpd = nullptr;
    m->capPairs = m->capPts = 0;
}

static int mensure(orb_matcher* m, size_t pairs, size_t pts) {
    if (pairs <= m->capPairs && pts <= m->capPts) return ORB_OK;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // hipMalloc / hipFree (common.h)
    ORB_HIP_TRY(hipStreamSynchronize(m->stream));
    pairs = std::max(pairs, m->capPairs);
    pts = std::max(pts, m->capPts);
    mfree(m);
    const size_t P = pairs * pts;
#define MALLOC(p, bytes) \
    if (hipMalloc((void**)&(p), (bytes)) != hipSuccess) { mfree(m); return ORB_ENOMEM; }
    MALLOC(m->d_k1, P * sizeof(orb_keypoint));
    MALLOC(m->d_k2, P * sizeof(orb_keypoint));
    MALLOC(m->d_d1, P * 32);
    MALLOC(m->d_d2, P * 32);
    MALLOC(m->d_prev, P * 8);
    MALLOC(m->d_ur, P * 4);
    MALLOC(m->d_n, pairs * 8 + 64);
    MALLOC(m->d_m12, P * 4);
    MALLOC(m->d_nm, pairs * 4 + 64);
    MALLOC(m->d_hI, P * 4);
    MALLOC(m->d_hB, P);
    MALLOC(m->d_cand, P * kMaxCand * 4);
    MALLOC(m->d_topk, P * kTopK * 4);
    MALLOC(m->d_best, P * 8);
    MALLOC(m->d_cs, pairs * (kCells + 1) * 4);
    MALLOC(m->d_gj, P * 4);
    MALLOC(m->d_gxy, P * 8);
    MALLOC(m->d_ncand, P * 4);
    MALLOC(m->d_status, 64);
    MALLOC(m->d_hasMp, P * 4);
    MALLOC(m->d_outl, P);
    MALLOC(m->d_xyz, P * 12);
    MALLOC(m->d_T, 64 * 4);
    MALLOC(m->d_sf, 64 * 4);
    MALLOC(m->d_mpd, P * 32);
#undef MALLOC
    // the batch path accumulates overflow bits until orb_matcher_batch_status reads them
    ORB_HIP_TRY(hipMemsetAsync(m->d_status, 0, 64, m->stream));
    ORB_HIP_TRY(hipStreamSynchronize(m->stream));
    m->capPairs = pairs;
    m->capPts = pts;
    return ORB_OK;
}

static int mpin(orb_matcher* m, size_t bytes) {
    if (m->h_pin_bytes >= bytes) return ORB_OK;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // (common.h)
    if (m->h_pin) (void)hipHostFree(m->h_pin);
    m->h_pin = nullptr;
    m->h_pin_bytes = 0;
    if (hipHostMalloc(&m->h_pin, bytes, hipHostMallocDefault) != hipSuccess) return ORB_ENOMEM;
    m->h_pin_bytes = bytes;
    return ORB_OK;
}

static int mstage(orb_matcher* m, size_t bytes) {
    m->hs.device = m->device;
    m->hs.stream = m->stream;
    return grow_scratch(&m->hs, bytes);
}

// Launches the candidate replay: the LDS form when its state fits, else k_resolve_sbp.
static void launch_resolve_sbp(orb_matcher* m, hipStream_t s, const orb_keypoint* kc, int ncur, const orb_keypoint* kl,
                               int nl, GridParams g, int checkOri, int32_t* curMp, int32_t* nm, int thDist,
                               const int32_t* lastHas) {
    const size_t lds = resolve_sbp_lds_bytes(ncur, nl);
    static const bool seqOnly = std::getenv("ORB_SBP_SEQ_RESOLVE") != nullptr;   // A/B of the two replays
    if (nl > 0 && lds <= 65536 && !seqOnly) {
        hipLaunchKernelGGL(k_best_sbp, dim3((nl + 3) / 4), dim3(256), 0, s, kc, kl, nl, g, checkOri, m->d_cand,
                           m->d_ncand, curMp, lastHas, m->d_best);
        hipLaunchKernelGGL(k_resolve_sbp_lds, dim3(1), dim3(64), lds, s, kc, ncur, kl, nl, g, checkOri, m->d_cand,
                           m->d_ncand, m->d_best, curMp, nm, thDist, lastHas);
        return;
    }
    hipLaunchKernelGGL(k_resolve_sbp, dim3(1), dim3(64), ((size_t)ncur + kHisto + 4) * 4, s, kc, ncur, kl, nl, g,
                       checkOri, m->d_cand, m->d_ncand, curMp, nm, m->d_hI, m->d_hB, thDist, lastHas);
}

static GridParams grid_of(const orb_frame_view* f) {
    GridParams g;
    g.min_x = f->min_x; g.min_y = f->min_y; g.max_x = f->max_x; g.max_y = f->max_y;
    g.winv = f->grid_w_inv; g.hinv = f->grid_h_inv;
    return g;
}

static void pack_view(const orb_frame_view* f, orb_keypoint* k) {
    for (int i = 0; i < f->n; i++) {
        k[i].x = f->x[i]; k[i].y = f->y[i]; k[i].size = 0.f; k[i].angle = f->angle[i];
        k[i].response = 0.f; k[i].octave = f->octave[i]; k[i].class_id = -1;
    }
}

// ------------------------------------------------------------------ Fuse
// ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th), matching step
// (R/src/ORBmatcher.cpp:995-1121): one wave per map point.  The projection, IsInImage, the scale
// invariance distances, the viewing-angle test and PredictScale are evaluated uniformly by the
// wave (OpenCV's float products restated as in oracle_fuse); the lanes then take the keyframe's
// keypoints j, j + 64, ..., keep those GetFeaturesInArea returns (grid cells of the search
// square, |dx| < r, |dy| < r), apply the level band [nPredictedLevel - 1, nPredictedLevel] and
// the chi2 gate (7.8 stereo / 5.99 mono), and the wave takes the least distance with the first
// candidate in GetFeaturesInArea order (cell ix-major, then keypoint index) winning ties — the
// reference's strict < over that order.  best_idx = -1 unless the distance is <= TH_LOW.
struct FuseKf {
    float Tcw[12], Ow[3];
    float fx, fy, cx, cy, bf, logsf;
    int nlev;
    float sf[32], isig2[32];
};

__global__ __launch_bounds__(256) void k_fuse(const orb_keypoint* __restrict__ kk, const uint8_t* __restrict__ kd,
                                              const float* __restrict__ kur, int nk, GridParams g, FuseKf K, int n_mp,
                                              const uint8_t* __restrict__ valid, const float* __restrict__ xyz,
                                              const float* __restrict__ nrm, const float* __restrict__ mind,
                                              const float* __restrict__ maxd, const uint8_t* __restrict__ mdesc,
                                              float th, int32_t* __restrict__ best_idx, int32_t* __restrict__ best_dist,
                                              int sim3) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_mp) return;
    int out = -1, outd = 256;
    bool go = valid[i] != 0;
    const float* X = xyz + 3 * (size_t)i;
    float u = 0, v = 0, ur = 0, radius = 0;
    int lev = 0;
    if (go) {
        float p3[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double s = (double)K.Tcw[4 * r] * X[0] + (double)K.Tcw[4 * r + 1] * X[1] + (double)K.Tcw[4 * r + 2] * X[2];
            p3[r] = (float)(s + (double)K.Tcw[4 * r + 3]);
        }
        go = !(p3[2] < 0.0f);
        // Fuse(pKF, vpMapPoints) divides in float (:1042), Fuse(pKF, Scw, ..) in double (:1194)
        const float invz = sim3 ? (float)(1.0 / (double)p3[2]) : 1 / p3[2];
        const float x = p3[0] * invz, y = p3[1] * invz;
        u = K.fx * x + K.cx;
        v = K.fy * y + K.cy;
        go = go && u >= g.min_x && u < g.max_x && v >= g.min_y && v < g.max_y;   // KeyFrame::IsInImage
        ur = u - K.bf * invz;
        const float maxDistance = 1.2f * maxd[i], minDistance = 0.8f * mind[i];
        const float PO[3] = {X[0] - K.Ow[0], X[1] - K.Ow[1], X[2] - K.Ow[2]};
        const float ss = (PO[0] * PO[0] + PO[1] * PO[1]) + PO[2] * PO[2];
        const float dist3D = (float)sqrt((double)ss);
        go = go && !(dist3D < minDistance || dist3D > maxDistance);
        const float* Pn = nrm + 3 * (size_t)i;
        const float dot = (PO[0] * Pn[0] + PO[1] * Pn[1]) + PO[2] * Pn[2];
        go = go && !((double)dot < 0.5 * dist3D);
        const float ratio = maxd[i] / dist3D;
        lev = (int)ceil(log((double)ratio) / (double)K.logsf);
        if (lev < 0) lev = 0;
        else if (lev >= K.nlev) lev = K.nlev - 1;
        radius = th * K.sf[lev];
    }
    if (go) {
        const AreaQuery q = make_area(g, u, v, radius, -1, -1);
        const uint8_t* dq = mdesc + (size_t)i * 32;
        int bd = 256, bk = 0x7fffffff;   // (distance, cell * 2^16 + index) lexicographic minimum
        for (int j = lane; j < nk && q.cx0 <= q.cx1; j += 64) {
            const orb_keypoint k2 = kk[j];
            const int cell = grid_cell(g, k2.x, k2.y);
            if (!in_area(q, cell, k2.octave, k2.x, k2.y)) continue;
            const int kl = k2.octave;
            if (kl < lev - 1 || kl > lev) continue;
            const float ex = u - k2.x, ey = v - k2.y;
            if (sim3) {
                // the Scw form has no reprojection-error gate (:1232-1249)
            } else if (kur && kur[j] >= 0) {
                const float er = ur - kur[j];
                const float e2 = ex * ex + ey * ey + er * er;
                if ((double)(e2 * K.isig2[kl]) > 7.8) continue;
            } else {
                const float e2 = ex * ex + ey * ey;
                if ((double)(e2 * K.isig2[kl]) > 5.99) continue;
            }
            const int d = hamming32(dq, kd + (size_t)j * 32);
            const int key = (cell << 16) | j;
            if (d < bd || (d == bd && key < bk)) { bd = d; bk = key; }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int od = __shfl_xor(bd, o, 64), ok = __shfl_xor(bk, o, 64);
            if (od < bd || (od == bd && ok < bk)) { bd = od; bk = ok; }
        }
        outd = bd;
        if (bd <= 50) out = bk & 0xffff;   // TH_LOW
    }
    if (lane == 0) {
        best_idx[i] = out;
        best_dist[i] = outd;
    }
}

// ------------------------------------------------------------------ SearchByProjection(KeyFrame, Scw, points, matched, th)
// LoopClosing's projection search (R/src/ORBmatcher.cpp:370-497): one wave per candidate map
// point with Fuse's gates minus the reprojection test — depth >= 0, KeyFrame::IsInImage, 0.8 / 1.2 x
// the min / max distance, the viewing-angle test, PredictScale on the keyframe, GetFeaturesInArea
// with octaves level-1 .. level — and every candidate's distance; k_resolve_sbp replays the point
// order with the vpMatched skip (first window entry on ties, bestDist <= TH_LOW, no rotation test).
__global__ __launch_bounds__(256) void k_cand_sbs(const orb_keypoint* __restrict__ kk, const uint8_t* __restrict__ kd,
                                                  int nk, GridParams g, FuseKf K, int n_mp,
                                                  const uint8_t* __restrict__ valid, const float* __restrict__ xyz,
                                                  const float* __restrict__ nrm, const float* __restrict__ mind,
                                                  const float* __restrict__ maxd, const uint8_t* __restrict__ mdesc,
                                                  float th, uint32_t* __restrict__ cand, int* __restrict__ ncand,
                                                  int* __restrict__ status) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_mp) return;
    bool go = valid[i] != 0;
    const float* X = xyz + 3 * (size_t)i;
    float u = 0, v = 0, radius = 0;
    int lev = 0;
    if (go) {
        float p3[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double s = (double)K.Tcw[4 * r] * X[0] + (double)K.Tcw[4 * r + 1] * X[1] + (double)K.Tcw[4 * r + 2] * X[2];
            p3[r] = (float)(s + (double)K.Tcw[4 * r + 3]);
        }
        go = !(p3[2] < 0.0f);
        const float invz = 1 / p3[2];
        const float x = p3[0] * invz, y = p3[1] * invz;
        u = K.fx * x + K.cx;
        v = K.fy * y + K.cy;
        go = go && u >= g.min_x && u < g.max_x && v >= g.min_y && v < g.max_y;   // KeyFrame::IsInImage
        const float maxDistance = 1.2f * maxd[i], minDistance = 0.8f * mind[i];
        const float PO[3] = {X[0] - K.Ow[0], X[1] - K.Ow[1], X[2] - K.Ow[2]};
        const float ss = (PO[0] * PO[0] + PO[1] * PO[1]) + PO[2] * PO[2];
        const float dist = (float)sqrt((double)ss);
        go = go && !(dist < minDistance || dist > maxDistance);
        const float* Pn = nrm + 3 * (size_t)i;
        const float dot = (PO[0] * Pn[0] + PO[1] * Pn[1]) + PO[2] * Pn[2];
        go = go && !((double)dot < 0.5 * dist);
        const float ratio = maxd[i] / dist;
        lev = (int)ceil(log((double)ratio) / (double)K.logsf);
        if (lev < 0) lev = 0;
        else if (lev >= K.nlev) lev = K.nlev - 1;
        radius = th * K.sf[lev];
    }
    int n = 0;
    if (go) {
        const AreaQuery q = make_area(g, u, v, radius, -1, -1);
        const uint8_t* dq = mdesc + (size_t)i * 32;
        uint32_t* out = cand + (size_t)i * kMaxCand;
        for (int j0 = 0; j0 < nk && q.cx0 <= q.cx1; j0 += 64) {
            const int j = j0 + lane;
            bool ok = false;
            int d = 0;
            if (j < nk) {
                const orb_keypoint k2 = kk[j];
                ok = in_area(q, grid_cell(g, k2.x, k2.y), k2.octave, k2.x, k2.y) && !(k2.octave < lev - 1 || k2.octave > lev);
                if (ok) d = hamming32(dq, kd + (size_t)j * 32);
            }
            const uint64_t m = __ballot(ok);
            const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
            if (ok && pos < kMaxCand) out[pos] = (uint32_t)j | ((uint32_t)d << 20);
            n += __popcll(m);
        }
    }
    if (lane == 0) {
        if (n > kMaxCand) { atomicOr(status, 1); n = kMaxCand; }
        ncand[i] = n;
    }
}

// ------------------------------------------------------------------ SearchBySim3
// ORBmatcher::SearchBySim3 (R/src/ORBmatcher.cpp:1305-1503): one direction per launch — each
// eligible map point of one keyframe goes through [R|t] (world -> its camera) and [sR|t] (its
// camera -> the other camera; double-accumulated rows rounded to float), is projected with
// pKF1's intrinsics, tested with the other keyframe's IsInImage and the 0.8 / 1.2 x distance
// range on |p3Dc| (the reference's cv::norm of the camera-frame point), PredictScale on the other
// keyframe, and takes the least-distance keypoint of the window at octaves level-1 .. level
// (first window entry on ties) if <= TH_HIGH.  The mutual check runs on the host.
struct Sim3Side {
    float T[12], S[12];
    float fx, fy, cx, cy;
    float logsf;
    int nlev;
    float sf[32];
    float th;
};

__global__ __launch_bounds__(256) void k_sim3_match(const orb_keypoint* __restrict__ kk, const uint8_t* __restrict__ kd,
                                                    int nk, GridParams g, Sim3Side P, int n_mp,
                                                    const uint8_t* __restrict__ valid, const float* __restrict__ xyz,
                                                    const float* __restrict__ mind, const float* __restrict__ maxd,
                                                    const uint8_t* __restrict__ mdesc, int32_t* __restrict__ match) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_mp) return;
    int out = -1;
    bool go = valid[i] != 0;
    float u = 0, v = 0, radius = 0;
    int lev = 0;
    if (go) {
        const float* X = xyz + 3 * (size_t)i;
        float c1[3], c2[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double s = (double)P.T[4 * r] * X[0] + (double)P.T[4 * r + 1] * X[1] + (double)P.T[4 * r + 2] * X[2];
            c1[r] = (float)(s + (double)P.T[4 * r + 3]);
        }
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double s = (double)P.S[4 * r] * c1[0] + (double)P.S[4 * r + 1] * c1[1] + (double)P.S[4 * r + 2] * c1[2];
            c2[r] = (float)(s + (double)P.S[4 * r + 3]);
        }
        go = !(c2[2] < 0.0f);
        const float invz = (float)(1.0 / (double)c2[2]);
        u = P.fx * (c2[0] * invz) + P.cx;
        v = P.fy * (c2[1] * invz) + P.cy;
        go = go && u >= g.min_x && u < g.max_x && v >= g.min_y && v < g.max_y;   // KeyFrame::IsInImage
        const float maxDistance = 1.2f * maxd[i], minDistance = 0.8f * mind[i];
        const float ss = (c2[0] * c2[0] + c2[1] * c2[1]) + c2[2] * c2[2];
        const float dist3D = (float)sqrt((double)ss);
        go = go && !(dist3D < minDistance || dist3D > maxDistance);
        const float ratio = maxd[i] / dist3D;
        lev = (int)ceil(log((double)ratio) / (double)P.logsf);
        if (lev < 0) lev = 0;
        else if (lev >= P.nlev) lev = P.nlev - 1;
        radius = P.th * P.sf[lev];
    }
    if (go) {
        const AreaQuery q = make_area(g, u, v, radius, -1, -1);
        const uint8_t* dq = mdesc + (size_t)i * 32;
        int bd = 0x7fffffff, bk = 0x7fffffff;
        for (int j = lane; j < nk && q.cx0 <= q.cx1; j += 64) {
            const orb_keypoint k2 = kk[j];
            const int cell = grid_cell(g, k2.x, k2.y);
            if (!in_area(q, cell, k2.octave, k2.x, k2.y)) continue;
            if (k2.octave < lev - 1 || k2.octave > lev) continue;
            const int d = hamming32(dq, kd + (size_t)j * 32);
            const int key = (cell << 16) | j;
            if (d < bd || (d == bd && key < bk)) { bd = d; bk = key; }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int od = __shfl_xor(bd, o, 64), ok = __shfl_xor(bk, o, 64);
            if (od < bd || (od == bd && ok < bk)) { bd = od; bk = ok; }
        }
        if (bd <= kThHigh) out = bk & 0xffff;
    }
    if (lane == 0) match[i] = out;
}

// ------------------------------------------------------------------ SearchForTriangulation
// ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
// (R/src/ORBmatcher.cpp:785-983).  Keypoints only meet inside a common vocabulary node, and a
// keyframe-2 keypoint lies in one node, so nodes are independent: one wave per common node runs
// the node's keyframe-1 features in order (the reference's greedy vbMatched2 sequence), the
// lanes taking the node's keyframe-2 features.  For each feature the wave keeps the candidate
// the reference's running `dist > bestDist -> continue` loop ends with — the least distance
// <= TH_LOW passing the epipole and CheckDistEpipolarLine (:175-203) tests, ties to the later
// candidate — and the owning lane marks it matched in a register bitmask.  A second one-
// workgroup kernel applies the rotation-consistency histogram (ComputeThreeMaxima).
constexpr int kSftMaxNode = 2048;   // keyframe-2 features of one node (32 bitmask slots per lane)
struct SftParams {
    float F[9];
    float ex, ey;
    float sf2[32], sig2[32];
    int onlyStereo;
};

__global__ __launch_bounds__(64) void k_sft(const orb_keypoint* __restrict__ k1, const uint8_t* __restrict__ d1,
                                            const float* __restrict__ ur1, const uint8_t* __restrict__ mp1,
                                            const orb_keypoint* __restrict__ k2, const uint8_t* __restrict__ d2,
                                            const float* __restrict__ ur2, const uint8_t* __restrict__ mp2,
                                            const int4* __restrict__ nodes, const int32_t* __restrict__ idx1,
                                            const int32_t* __restrict__ idx2, SftParams P,
                                            int32_t* __restrict__ matches12) {
    const int lane = threadIdx.x;
    const int4 nd = nodes[blockIdx.x];   // KF1 list [x, y), KF2 list [z, w)
    const int c2 = nd.w - nd.z;
    uint32_t taken = 0;                  // bit r: candidate lane + 64 r matched (vbMatched2)
    for (int p1 = nd.x; p1 < nd.y; p1++) {
        const int i1 = idx1[p1];
        if (mp1[i1]) continue;
        const bool st1 = ur1 && ur1[i1] >= 0;
        if (P.onlyStereo && !st1) continue;
        const orb_keypoint a = k1[i1];
        const uint4* da = reinterpret_cast<const uint4*>(d1 + (size_t)i1 * 32);
        const uint4 a0 = da[0], a1 = da[1];
        const float ea = a.x * P.F[0] + a.y * P.F[3] + P.F[6];   // CheckDistEpipolarLine's line
        const float eb = a.x * P.F[1] + a.y * P.F[4] + P.F[7];
        const float ec = a.x * P.F[2] + a.y * P.F[5] + P.F[8];
        int best = 0x7fffffff;   // (dist << 16) | (65535 - position): least dist, ties to the later
        for (int r = 0; r * 64 < c2; r++) {
            const int pos = r * 64 + lane;
            if (pos >= c2 || ((taken >> r) & 1u)) continue;
            const int i2 = idx2[nd.z + pos];
            if (mp2[i2]) continue;
            const bool st2 = ur2 && ur2[i2] >= 0;
            if (P.onlyStereo && !st2) continue;
            const uint4* db = reinterpret_cast<const uint4*>(d2 + (size_t)i2 * 32);
            const uint4 b0 = db[0], b1 = db[1];
            const int dist = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                             __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
            if (dist > 50) continue;   // TH_LOW
            const orb_keypoint b = k2[i2];
            if (!st1 && !st2) {
                const float dex = P.ex - b.x, dey = P.ey - b.y;
                if (dex * dex + dey * dey < 100 * P.sf2[b.octave]) continue;
            }
            const float num = ea * b.x + eb * b.y + ec;
            const float den = ea * ea + eb * eb;
            if (den == 0) continue;
            const float dsqr = num * num / den;
            if (!((double)dsqr < 3.84 * P.sig2[b.octave])) continue;
            const int key = (dist << 16) | (65535 - pos);
            best = min(best, key);
        }
        best = wave_min_i32(best);
        if (best != 0x7fffffff) {
            const int pos = 65535 - (best & 0xffff);
            if ((pos & 63) == lane) taken |= 1u << (pos >> 6);
            if (lane == 0) matches12[i1] = idx2[nd.z + pos];
        }
    }
}

// The rotation-consistency filter of SearchForTriangulation (:944-961) over all matches: bin
// counts in LDS, ComputeThreeMaxima, matches outside the three bins dropped; *nmatches.
__global__ __launch_bounds__(256) void k_sft_rot(const orb_keypoint* __restrict__ k1, const orb_keypoint* __restrict__ k2,
                                                 int n1, int checkOri, int32_t* __restrict__ matches12,
                                                 int32_t* __restrict__ nmatches, int32_t* __restrict__ outMatches) {
    __shared__ int hcount[kHisto];
    __shared__ int ind[3], total;
    const int tid = threadIdx.x;
    if (tid < kHisto) hcount[tid] = 0;
    if (tid == 0) total = 0;
    __syncthreads();
    for (int i = tid; i < n1; i += 256) {
        const int j = matches12[i];
        if (j < 0) continue;
        if (checkOri) atomicAdd(&hcount[rot_bin(k1[i].angle - k2[j].angle)], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        int max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < kHisto; i++) {
            const int s = hcount[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        ind[0] = ind1; ind[1] = ind2; ind[2] = ind3;
    }
    __syncthreads();
    int kept = 0;
    for (int i = tid; i < n1; i += 256) {   // (outMatches: the final matches, host-mapped, every entry)
        int j = matches12[i];
        if (j >= 0 && checkOri) {
            const int bin = rot_bin(k1[i].angle - k2[j].angle);
            if (bin != ind[0] && bin != ind[1] && bin != ind[2]) { matches12[i] = -1; j = -1; }
        }
        if (outMatches) outMatches[i] = j;
        kept += j >= 0 ? 1 : 0;
    }
    atomicAdd(&total, kept);
    __syncthreads();
    if (tid == 0) *nmatches = total;
}

// ------------------------------------------------------------------ SearchByBoW
// ORBmatcher::SearchByBoW(pKF, F, vpMapPointMatches) (R/src/ORBmatcher.cpp:220-372) and
// SearchByBoW(pKF1, pKF2, vpMatches12) (:632-760): over the vocabulary nodes both feature
// vectors hold, each side-1 feature of the node (in list order) takes its nearest unmatched
// side-2 feature of the node.  Side-2 features belong to one node only, so nodes are independent:
// one wave per common node, walking the node's side-1 features in order (the reference's greedy
// vpMapPointMatches / vbMatched2 sequence), the lanes taking its side-2 features.  The wave
// reduces the reference's running (bestDist1, bestIdx, bestDist2): the least distance, its first
// position (strict <), and the second least of the multiset; the match is kept when bestDist1
// passes TH_LOW (<= for the frame overload, < for the keyframe one) and the ratio test.
constexpr int kSbbMaxNode = 2048;
__global__ __launch_bounds__(64) void k_sbb(const uint8_t* __restrict__ d1, const uint8_t* __restrict__ ok1,
                                            const uint8_t* __restrict__ d2, const uint8_t* __restrict__ ok2,
                                            const int4* __restrict__ nodes, const int32_t* __restrict__ idx1,
                                            const int32_t* __restrict__ idx2, int thIncl, float ratio,
                                            int32_t* __restrict__ matches12) {
    const int lane = threadIdx.x;
    const int4 nd = nodes[blockIdx.x];   // side-1 list [x, y), side-2 list [z, w)
    const int c2 = nd.w - nd.z;
    uint32_t taken = 0;                  // bit r: candidate lane + 64 r matched
    for (int p1 = nd.x; p1 < nd.y; p1++) {
        const int i1 = idx1[p1];
        if (!ok1[i1]) continue;
        const uint4* da = reinterpret_cast<const uint4*>(d1 + (size_t)i1 * 32);
        const uint4 a0 = da[0], a1 = da[1];
        int key1 = 0x7fffffff, dd2 = 256;    // lane's (dist << 16 | pos) minimum, second least dist
        for (int r = 0; r * 64 < c2; r++) {
            const int pos = r * 64 + lane;
            if (pos >= c2 || ((taken >> r) & 1u)) continue;
            const int i2 = idx2[nd.z + pos];
            if (ok2 && !ok2[i2]) continue;
            const uint4* db = reinterpret_cast<const uint4*>(d2 + (size_t)i2 * 32);
            const uint4 b0 = db[0], b1 = db[1];
            const int dist = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                             __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
            const int key = (dist << 16) | pos;
            if (key < key1) { dd2 = min(dd2, key1 >> 16); key1 = key; }
            else dd2 = min(dd2, dist);
        }
        const int g1 = wave_min_i32(key1);
        if (g1 == 0x7fffffff) continue;
        const int best1 = g1 >> 16;
        const int best2 = wave_min_i32(key1 == g1 ? dd2 : min(dd2, key1 >> 16));
        if (best1 <= thIncl && (float)best1 < ratio * (float)min(best2, 256)) {
            const int pos = g1 & 0xffff;
            if ((pos & 63) == lane) taken |= 1u << (pos >> 6);
            if (lane == 0) matches12[i1] = idx2[nd.z + pos];
        }
    }
}

// ------------------------------------------------------------------ distinctive descriptors
// MapPoint::ComputeDistinctiveDescriptors (R/src/MapPoint.cpp:306-385) for a batch of map
// points: point m's observed descriptors are rows [start[m], start[m+1]) (observation order,
// bad keyframes already left out).  One 64-lane workgroup per point: the descriptors are staged
// in LDS (up to kDdLds rows, else read from HBM), lane i takes rows i, i + 64, ... and finds the
// row's median distance — vDists[0.5 * (N - 1)] of the sorted row, self distance 0 included —
// as the smallest v with #{j : d(i, j) <= v} > (N - 1) / 2, by binary search over 0..256; the
// least median wins, ties to the lower index (strict <).  best_idx[m] = -1 for an empty list.
constexpr int kDdLds = 1024;
__global__ __launch_bounds__(64) void k_distinctive(const uint8_t* __restrict__ desc, const int32_t* __restrict__ start,
                                                    int32_t* __restrict__ best_idx, uint8_t* __restrict__ best_desc) {
    __shared__ uint4 sd[kDdLds * 2];
    const int m = blockIdx.x, lane = threadIdx.x;
    const int s0 = start[m], N = start[m + 1] - s0;
    const uint4* g = reinterpret_cast<const uint4*>(desc + (size_t)s0 * 32);
    const bool lds = N <= kDdLds;
    if (lds)
        for (int t = lane; t < 2 * N; t += 64) sd[t] = g[t];
    __syncthreads();
    const uint4* D = lds ? sd : g;
    const int k = (int)(0.5 * (N - 1));   // size_t(0.5 * (N - 1)) in the reference's vDists index
    int best = INT_MAX, bi = 0x7fffffff;
    for (int i = lane; i < N; i += 64) {
        const uint4 a0 = D[2 * i], a1 = D[2 * i + 1];
        int lo = 0, hi = 256;   // smallest v with count(d <= v) >= k + 1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < N; j++) {
                const uint4 b0 = D[2 * j], b1 = D[2 * j + 1];
                const int dd = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                               __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
                cnt += dd <= mid;
            }
            if (cnt >= k + 1) hi = mid;
            else lo = mid + 1;
        }
        if (lo < best) { best = lo; bi = i; }
    }
    // lexicographic (median, index) minimum over the wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int ob = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) best_idx[m] = N > 0 ? bi : -1;
    if (best_desc && N > 0 && lane < 2)
        reinterpret_cast<uint4*>(best_desc + (size_t)m * 32)[lane] = g[2 * bi + lane];
}

extern "C" {

int orb_descriptor_distance(const uint8_t* a, const uint8_t* b) try {
    if (!a || !b) return ORB_EINVAL;
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        dist += __builtin_popcount(pa ^ pb);
    }
    return dist;
} ORB_ABI_CATCH

int orb_matcher_create(int device, float nnratio, int check_ori, orb_matcher** out) try {
    if (!out) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    ORB_HIP_TRY(hipSetDevice(device));
    orb_matcher* m = new orb_matcher();
    m->device = device;
    m->nnratio = nnratio;
    m->checkOri = check_ori ? 1 : 0;
    {
        std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // (common.h)
        if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) { delete m; return ORB_EGPU; }
    }
    *out = m;
    return ORB_OK;
} ORB_ABI_CATCH

void orb_matcher_destroy(orb_matcher* m) try {
    if (!m) return;
    std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // hipFree (common.h)
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    mfree(m);
    if (m->h_pin) (void)hipHostFree(m->h_pin);
    if (m->hs.base) (void)hipFree(m->hs.base);
    if (m->hs.pin) (void)hipHostFree(m->hs.pin);
    if (m->hs.pout) (void)hipHostFree(m->hs.pout);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
} ORB_ABI_CATCH_VOID

int orb_search_for_initialization(orb_matcher* m, const orb_frame_view* f1, const orb_frame_view* f2, float* prev_xy,
                                  int32_t* matches12, int window) try {
    if (!m || !f1 || !f2 || !prev_xy || !matches12 || f1->n < 0 || f2->n < 0) return ORB_EINVAL;
    if (f2->n >= (1 << 20)) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int cap = std::max(std::max(f1->n, f2->n), 1);
    int st = mensure(m, 1, cap);
    if (st) return st;
    const size_t n1 = (size_t)f1->n, n2 = (size_t)f2->n;
    st = mstage(m, Staging::bytes_for({n1 * sizeof(orb_keypoint), n2 * sizeof(orb_keypoint), n1 * 32, n2 * 32, 8, n1 * 8,
                                       8, n1 * 4, 4}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of the inputs, one D2H of prev / status / matches / count
    char* hp;
    auto* dK1 = (orb_keypoint*)sg.in_place(n1 * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(f1, (orb_keypoint*)hp);
    auto* dK2 = (orb_keypoint*)sg.in_place(n2 * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(f2, (orb_keypoint*)hp);
    auto* dD1 = (uint8_t*)sg.in(f1->desc, n1 * 32);
    auto* dD2 = (uint8_t*)sg.in(f2->desc, n2 * 32);
    const int32_t nn[2] = {f1->n, f2->n}, zero[2] = {0, 0};
    auto* dN = (int32_t*)sg.in(nn, 8);
    auto* dPrev = (float*)sg.in(prev_xy, n1 * 8);
    auto* dSt = (int32_t*)sg.in(zero, 8);
    auto* dM12 = (int32_t*)sg.out(n1 * 4);
    auto* dNm = (int32_t*)sg.out(4);
    if (int e_ = sg.upload_pull(s)) return e_;
    const GridParams g = grid_of(f2);
    hipLaunchKernelGGL(k_grid_sfi, dim3(1), dim3(256), 0, s, dK2, dN + 1, cap, g, m->d_cs, m->d_gj, m->d_gxy);
    hipLaunchKernelGGL(k_cand_sfi, dim3(kCandWaves / 4, 1), dim3(256), 0, s, dK1, dD1, dN, dD2, m->d_cs, m->d_gj,
                       m->d_gxy, dPrev, cap, g, (float)window, m->d_cand, m->d_ncand, m->d_topk, dSt);
    const size_t lds = resolve_sfi_lds(cap);
    if (lds > kMaxLds || cap > 32767) return ORB_E2BIG;
    hipLaunchKernelGGL(k_resolve_sfi, dim3(1), dim3(kRsT), lds, s, dK1, dN, dK2, dN + 1, cap, m->nnratio, m->checkOri,
                       m->d_cand, m->d_ncand, m->d_topk, dPrev, dM12, dNm, dSt);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dPrev)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    if (*sg.host(dSt)) return ORB_EOVERFLOW;
    std::memcpy(matches12, sg.host(dM12), n1 * 4);
    std::memcpy(prev_xy, sg.host(dPrev), n1 * 8);
    return *sg.host(dNm);
} ORB_ABI_CATCH

int orb_search_for_initialization_batch_device(orb_matcher* m, const orb_keypoint* d_kps1, const uint8_t* d_desc1,
                                               const int32_t* d_n1, const orb_keypoint* d_kps2, const uint8_t* d_desc2,
                                               const int32_t* d_n2, int nb, int cap, int width, int height, int window,
                                               int32_t* d_matches12, int32_t* d_nmatches, void* stream) try {
    if (!m || nb <= 0 || cap <= 0 || width <= 0 || height <= 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    int st = mensure(m, nb, cap);
    if (st) return st;
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    if (m->batch_stream && m->batch_stream != s) ORB_HIP_TRY(hipStreamSynchronize(m->batch_stream));
    m->batch_stream = s;
    GridParams g;
    g.min_x = 0.f; g.min_y = 0.f; g.max_x = (float)width; g.max_y = (float)height;
    g.winv = (float)kGridCols / (float)width;
    g.hinv = (float)kGridRows / (float)height;
    hipLaunchKernelGGL(k_grid_sfi, dim3(nb), dim3(256), 0, s, d_kps2, d_n2, cap, g, m->d_cs, m->d_gj, m->d_gxy);
    hipLaunchKernelGGL(k_cand_sfi, dim3(kCandWaves / 4, nb), dim3(256), 0, s, d_kps1, d_desc1, d_n1, d_desc2, m->d_cs,
                       m->d_gj, m->d_gxy, (const float*)nullptr, cap, g, (float)window, m->d_cand, m->d_ncand,
                       m->d_topk, m->d_status);
    const size_t lds = resolve_sfi_lds(cap);
    if (lds > kMaxLds || cap > 32767) return ORB_E2BIG;
    hipLaunchKernelGGL(k_resolve_sfi, dim3(nb), dim3(kRsT), lds, s, d_kps1, d_n1, d_kps2, d_n2, cap, m->nnratio,
                       m->checkOri, m->d_cand, m->d_ncand, m->d_topk, (float*)nullptr, d_matches12, d_nmatches,
                       m->d_status);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

int orb_matcher_batch_status(orb_matcher* m, int32_t* status) try {
    if (!m || !status) return ORB_EINVAL;
    *status = 0;
    if (!m->d_status) return ORB_OK;
    ORB_HIP_TRY(hipSetDevice(m->device));
    if (m->batch_stream) ORB_HIP_TRY(hipStreamSynchronize(m->batch_stream));
    int32_t v = 0;
    ORB_HIP_TRY(hipMemcpyAsync(&v, m->d_status, 4, hipMemcpyDeviceToHost, m->stream));
    ORB_HIP_TRY(hipMemsetAsync(m->d_status, 0, 4, m->stream));
    ORB_HIP_TRY(hipStreamSynchronize(m->stream));
    *status = v;
    return v ? ORB_EOVERFLOW : ORB_OK;
} ORB_ABI_CATCH

int orb_search_by_projection_frame(orb_matcher* m, const orb_frame_view* cur, const float* Tcw_cur,
                                   const orb_frame_view* last, const float* Tcw_last, const int32_t* last_has_mp,
                                   const uint8_t* last_outlier, const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                   const float* scale_factors, const float cam[6], float th, int mono, int32_t* cur_mp) try {
    if (!m || !cur || !last || !Tcw_cur || !Tcw_last || !last_has_mp || !last_outlier || !last_mp_xyz ||
        !last_mp_desc || !scale_factors || !cam || !cur_mp)
        return ORB_EINVAL;
    if (cur->n >= (1 << 20)) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int cap = std::max(std::max(cur->n, last->n), 1);
    int st = mensure(m, 1, cap);
    if (st) return st;
    // tlc = Rlw * twc + tlw with twc = -Rcw^T tcw (float Mat products, double accumulation)
    float twc[3], tlc[3];
    for (int c = 0; c < 3; c++) {
        double s = 0;
        for (int r = 0; r < 3; r++) s += (double)Tcw_cur[4 * r + c] * (double)Tcw_cur[4 * r + 3];
        twc[c] = (float)(-s);
    }
    for (int r = 0; r < 3; r++) {
        const double s = (double)Tcw_last[4 * r] * twc[0] + (double)Tcw_last[4 * r + 1] * twc[1] +
                         (double)Tcw_last[4 * r + 2] * twc[2];
        tlc[r] = (float)(s + (double)Tcw_last[4 * r + 3]);
    }
    SbpCam c;
    c.fx = cam[0]; c.fy = cam[1]; c.cx = cam[2]; c.cy = cam[3]; c.mbf = cam[4]; c.mb = cam[5];
    const int bForward = tlc[2] > c.mb && !mono;
    const int bBackward = -tlc[2] > c.mb && !mono;
    const size_t nc = (size_t)cur->n, nl = (size_t)last->n;
    st = mstage(m, Staging::bytes_for({nc * sizeof(orb_keypoint), nl * sizeof(orb_keypoint), nc * 32, nl * 32, nc * 4,
                                       nl * 12, nl * 4, nl, 48, 128, nc * 4, 8, 4}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of the inputs, one D2H of matches / status / count
    char* hp;
    auto* dKc = (orb_keypoint*)sg.in_place(nc * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(cur, (orb_keypoint*)hp);
    auto* dKl = (orb_keypoint*)sg.in_place(nl * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(last, (orb_keypoint*)hp);
    auto* dDc = (uint8_t*)sg.in(cur->desc, nc * 32);
    auto* dMd = (uint8_t*)sg.in(last_mp_desc, nl * 32);
    auto* dUr = (float*)sg.in_place(nc * 4, &hp);
    if (hp)
        for (size_t i = 0; i < nc; i++) ((float*)hp)[i] = cur->uright ? cur->uright[i] : -1.f;
    auto* dXyz = (float*)sg.in(last_mp_xyz, nl * 12);
    auto* dHas = (int32_t*)sg.in(last_has_mp, nl * 4);
    auto* dOut = (uint8_t*)sg.in(last_outlier, nl);
    auto* dT = (float*)sg.in(Tcw_cur, 48);
    int maxOct = 0;
    for (int i = 0; i < last->n; i++) maxOct = std::max(maxOct, (int)last->octave[i]);
    float sf[32] = {0.f};
    for (int i = 0; i <= maxOct && i < 32; i++) sf[i] = scale_factors[i];
    auto* dSf = (float*)sg.in(sf, 128);
    auto* dM12 = (int32_t*)sg.in(cur_mp, nc * 4);
    const int32_t zero[2] = {0, 0};
    auto* dSt = (int32_t*)sg.in(zero, 8);
    auto* dNm = (int32_t*)sg.out(4);
    if (int e_ = sg.upload_pull(s)) return e_;
    const GridParams g = grid_of(cur);
    if (last->n > 0) {
        hipLaunchKernelGGL(k_cand_sbp, dim3((last->n + 3) / 4), dim3(256), 0, s, dKc, dDc,
                           cur->uright ? (const float*)dUr : (const float*)nullptr, cur->n, dKl, last->n, dHas, dOut,
                           dXyz, dMd, dT, dSf, c, g, th, bForward, bBackward, m->d_cand, m->d_ncand, dSt);
    }
    launch_resolve_sbp(m, s, dKc, cur->n, dKl, last->n, g, m->checkOri, dM12, dNm, kThHigh, (const int32_t*)dHas);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dM12)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    if (*sg.host(dSt)) return ORB_EOVERFLOW;
    std::memcpy(cur_mp, sg.host(dM12), nc * 4);
    return *sg.host(dNm);
} ORB_ABI_CATCH

int orb_search_by_projection_kf(orb_matcher* m, const orb_frame_view* cur, const float* Tcw_cur, const float Ow[3],
                                const orb_frame_view* kf, const uint8_t* mp_valid, const float* mp_xyz,
                                const float* mp_min_dist, const float* mp_max_dist, const uint8_t* mp_desc,
                                const float cam[4], float log_scale_factor, int n_levels, const float* scale_factors,
                                float th, int orb_dist, int32_t* cur_mp) try {
    if (!m || !cur || !Tcw_cur || !Ow || !kf || !mp_valid || !mp_xyz || !mp_min_dist || !mp_max_dist || !mp_desc ||
        !cam || !scale_factors || !cur_mp || n_levels < 1 || n_levels > 32)
        return ORB_EINVAL;
    if (cur->n >= (1 << 20)) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int nmp = kf->n;
    const int cap = std::max(std::max(cur->n, nmp), 1);
    int st = mensure(m, 1, cap);
    if (st) return st;
    SbkParams P;
    std::memcpy(P.Tcw, Tcw_cur, sizeof(P.Tcw));
    std::memcpy(P.Ow, Ow, sizeof(P.Ow));
    P.fx = cam[0]; P.fy = cam[1]; P.cx = cam[2]; P.cy = cam[3];
    P.logsf = log_scale_factor;
    P.nlev = n_levels;
    for (int l = 0; l < 32; l++) P.sf[l] = l < n_levels ? scale_factors[l] : 0.f;
    P.th = th;
    const size_t nc = (size_t)cur->n, nk = (size_t)nmp;
    st = mstage(m, Staging::bytes_for({nc * sizeof(orb_keypoint), nk * sizeof(orb_keypoint), nc * 32, nk * 32, nk * 12,
                                       nk * 4, nk * 4, nk, nc * 4, 8, 4}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of the inputs, one D2H of matches / status / count
    char* hp;
    auto* dKc = (orb_keypoint*)sg.in_place(nc * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(cur, (orb_keypoint*)hp);
    auto* dKk = (orb_keypoint*)sg.in_place(nk * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(kf, (orb_keypoint*)hp);
    auto* dDc = (uint8_t*)sg.in(cur->desc, nc * 32);
    auto* dMd = (uint8_t*)sg.in(mp_desc, nk * 32);
    auto* dXyz = (float*)sg.in(mp_xyz, nk * 12);
    auto* dMin = (float*)sg.in(mp_min_dist, nk * 4);
    auto* dMax = (float*)sg.in(mp_max_dist, nk * 4);
    auto* dVal = (uint8_t*)sg.in(mp_valid, nk);
    auto* dM12 = (int32_t*)sg.in(cur_mp, nc * 4);
    const int32_t zero[2] = {0, 0};
    auto* dSt = (int32_t*)sg.in(zero, 8);
    auto* dNm = (int32_t*)sg.out(4);
    if (int e_ = sg.upload_pull(s)) return e_;
    const GridParams g = grid_of(cur);
    if (nmp > 0) {
        hipLaunchKernelGGL(k_cand_sbk, dim3((nmp + 3) / 4), dim3(256), 0, s, dKc, dDc, cur->n, nmp, dVal, dXyz,
                           (const float*)dMin, (const float*)dMax, dMd, P, g, m->d_cand, m->d_ncand, dSt);
    }
    launch_resolve_sbp(m, s, dKc, cur->n, dKk, nmp, g, m->checkOri, dM12, dNm, orb_dist, (const int32_t*)nullptr);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dM12)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    if (*sg.host(dSt)) return ORB_EOVERFLOW;
    std::memcpy(cur_mp, sg.host(dM12), nc * 4);
    return *sg.host(dNm);
} ORB_ABI_CATCH

int orb_search_by_projection_sim3(orb_matcher* m, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp,
                                  const uint8_t* mp_valid, const float* mp_xyz, const float* mp_normal,
                                  const float* mp_min_dist, const float* mp_max_dist, const uint8_t* mp_desc, float th,
                                  int32_t* matched) try {
    if (!m || !kf || !kp || !matched || n_mp < 0 || (n_mp > 0 && (!mp_valid || !mp_xyz || !mp_normal || !mp_min_dist ||
                                                                   !mp_max_dist || !mp_desc)))
        return ORB_EINVAL;
    if (kp->n_levels < 1 || kp->n_levels > 32 || !kp->scale_factors || kf->n >= (1 << 20)) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int cap = std::max(std::max(kf->n, n_mp), 1);
    int st = mensure(m, 1, cap);
    if (st) return st;
    FuseKf K;
    std::memcpy(K.Tcw, kp->Tcw, sizeof(K.Tcw));
    std::memcpy(K.Ow, kp->Ow, sizeof(K.Ow));
    K.fx = kp->fx; K.fy = kp->fy; K.cx = kp->cx; K.cy = kp->cy; K.bf = kp->bf; K.logsf = kp->log_scale_factor;
    K.nlev = kp->n_levels;
    for (int l = 0; l < 32; l++) {
        K.sf[l] = l < kp->n_levels ? kp->scale_factors[l] : 0.f;
        K.isig2[l] = 0.f;
    }
    const size_t nk = (size_t)kf->n, np = (size_t)n_mp;
    st = mstage(m, Staging::bytes_for({nk * sizeof(orb_keypoint), nk * 32, np * 32, np * 12, np * 12, np * 4, np * 4, np,
                                       nk * 4, 8, 4}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of the inputs, one D2H of matches / status / count
    char* hp;
    auto* dK = (orb_keypoint*)sg.in_place(nk * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(kf, (orb_keypoint*)hp);
    auto* dD = (uint8_t*)sg.in(kf->desc, nk * 32);
    auto* dMd = (uint8_t*)sg.in(mp_desc, np * 32);
    auto* dXyz = (float*)sg.in(mp_xyz, np * 12);
    auto* dNrm = (float*)sg.in(mp_normal, np * 12);
    auto* dMin = (float*)sg.in(mp_min_dist, np * 4);
    auto* dMax = (float*)sg.in(mp_max_dist, np * 4);
    auto* dVal = (uint8_t*)sg.in(mp_valid, np);
    auto* dM = (int32_t*)sg.in(matched, nk * 4);
    const int32_t zero[2] = {0, 0};
    auto* dSt = (int32_t*)sg.in(zero, 8);
    auto* dNm = (int32_t*)sg.out(4);
    if (int e_ = sg.upload_pull(s)) return e_;
    const GridParams g = grid_of(kf);
    if (n_mp > 0) {
        hipLaunchKernelGGL(k_cand_sbs, dim3((n_mp + 3) / 4), dim3(256), 0, s, dK, dD, kf->n, g, K, n_mp, dVal, dXyz,
                           (const float*)dNrm, (const float*)dMin, (const float*)dMax, dMd, th, m->d_cand, m->d_ncand,
                           dSt);
    }
    launch_resolve_sbp(m, s, dK, kf->n, dK, n_mp, g, 0, dM, dNm, kThLow, (const int32_t*)nullptr);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dM)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    if (*sg.host(dSt)) return ORB_EOVERFLOW;
    std::memcpy(matched, sg.host(dM), nk * 4);
    return *sg.host(dNm);
} ORB_ABI_CATCH

int orb_search_by_projection_local(orb_matcher* m, const orb_frame_view* f, int n_mp, const uint8_t* mp_in_view,
                                   const float* mp_proj, const int32_t* mp_level, const float* mp_view_cos,
                                   const uint8_t* mp_desc, const uint8_t* mp_has_obs, const float* scale_factors,
                                   float th, int32_t* cur_mp) try {
    if (!m || !f || n_mp < 0 || !cur_mp || !scale_factors || f->n < 0) return ORB_EINVAL;
    if (n_mp > 0 && (!mp_in_view || !mp_proj || !mp_level || !mp_view_cos || !mp_desc || !mp_has_obs)) return ORB_EINVAL;
    if (f->n >= (1 << 20)) return ORB_EINVAL;
    if (n_mp == 0 || f->n == 0) return 0;
    int maxLevel = 0;
    for (int i = 0; i < f->n; i++) maxLevel = std::max(maxLevel, (int)f->octave[i]);
    for (int i = 0; i < n_mp; i++) {
        if (!mp_in_view[i]) continue;
        if (mp_level[i] < 0 || mp_level[i] > 31) return ORB_EINVAL;
        maxLevel = std::max(maxLevel, (int)mp_level[i]);
    }
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int cap = std::max(std::max(f->n, n_mp), 1);
    int st = mensure(m, 1, cap);
    if (st) return st;
    const size_t lds = (size_t)2 * f->n * 4;
    if (lds > 65536) return ORB_E2BIG;
    const size_t nf = (size_t)f->n, np = (size_t)n_mp;
    st = mstage(m, Staging::bytes_for({nf * sizeof(orb_keypoint), nf * 32, nf * 4, np * 12, np * 4, np * 4, 128, np * 32,
                                       np, np, nf * 4, 8, 4}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of the inputs, one D2H of matches / status / count
    char* hp;
    auto* dK = (orb_keypoint*)sg.in_place(nf * sizeof(orb_keypoint), &hp);
    if (hp) pack_view(f, (orb_keypoint*)hp);
    auto* dD = (uint8_t*)sg.in(f->desc, nf * 32);
    auto* dUr = (float*)sg.in_place(nf * 4, &hp);
    if (hp)
        for (size_t i = 0; i < nf; i++) ((float*)hp)[i] = f->uright ? f->uright[i] : -1.f;
    auto* dProj = (float*)sg.in(mp_proj, np * 12);
    auto* dLvl = (int32_t*)sg.in(mp_level, np * 4);
    auto* dCos = (float*)sg.in(mp_view_cos, np * 4);
    float sf[32] = {0.f};
    for (int i = 0; i <= maxLevel && i < 32; i++) sf[i] = scale_factors[i];
    auto* dSf = (float*)sg.in(sf, 128);
    auto* dMd = (uint8_t*)sg.in(mp_desc, np * 32);
    auto* dIn = (uint8_t*)sg.in(mp_in_view, np);
    auto* dObs = (uint8_t*)sg.in(mp_has_obs, np);
    auto* dM12 = (int32_t*)sg.in(cur_mp, nf * 4);
    const int32_t zero[2] = {0, 0};
    auto* dSt = (int32_t*)sg.in(zero, 8);
    auto* dNm = (int32_t*)sg.out(4);
    if (int e_ = sg.upload_pull(s)) return e_;
    const GridParams g = grid_of(f);
    hipLaunchKernelGGL(k_cand_sbl, dim3((n_mp + 3) / 4), dim3(256), 0, s, dK, dD,
                       f->uright ? (const float*)dUr : (const float*)nullptr, f->n, n_mp, dIn, dProj, dLvl, dCos, dMd,
                       dSf, g, th, m->d_cand, m->d_ncand, dSt);
    hipLaunchKernelGGL(k_resolve_sbl, dim3(1), dim3(64), lds, s, dK, f->n, n_mp, g, m->nnratio, dObs, m->d_cand,
                       m->d_ncand, dM12, dNm);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dM12)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    if (*sg.host(dSt)) return ORB_EOVERFLOW;
    std::memcpy(cur_mp, sg.host(dM12), nf * 4);
    return *sg.host(dNm);
} ORB_ABI_CATCH

int orb_hamming_knn2(orb_matcher* m, const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* best_idx,
                     int32_t* best_d, int32_t* second_d) try {
    if (!m || nq < 0 || nt < 0 || (nq && (!q || !best_idx || !best_d || !second_d)) || (nt && !t)) return ORB_EINVAL;
    if (nq == 0) return ORB_OK;
    ORB_HIP_TRY(hipSetDevice(m->device));
    const int cap = std::max(std::max(nq, nt), 1);
    const size_t bq = (size_t)nq * 4;
    int st = mstage(m, Staging::bytes_for({(size_t)nq * 32, (size_t)nt * 32, 8, bq, bq, bq}));
    if (st) return st;
    hipStream_t s = m->stream;
    Staging sg(&m->hs);   // one H2D of both descriptor sets, one D2H of the three outputs
    auto* dQ = (uint8_t*)sg.in(q, (size_t)nq * 32);
    auto* dT = (uint8_t*)sg.in(t, (size_t)nt * 32);
    const int32_t nn[2] = {nq, nt};
    auto* dN = (int32_t*)sg.in(nn, 8);
    auto* dBi = (int32_t*)sg.out(bq);
    auto* dBd = (int32_t*)sg.out(bq);
    auto* dSd = (int32_t*)sg.out(bq);
    if (int e_ = sg.upload_pull(s)) return e_;
    hipLaunchKernelGGL(k_knn2, dim3((nq + 3) / 4, 1), dim3(256), 0, s, dQ, dN, dT, dN + 1, cap, cap, dBi, dBd, dSd);
    ORB_HIP_TRY(hipGetLastError());
    if (int e_ = sg.download(s, dBi)) return e_;
    ORB_HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(best_idx, sg.host(dBi), bq);
    std::memcpy(best_d, sg.host(dBd), bq);
    std::memcpy(second_d, sg.host(dSd), bq);
    return ORB_OK;
} ORB_ABI_CATCH

int orb_hamming_knn2_batch_device(orb_matcher* m, const uint8_t* d_q, const int32_t* d_nq, const uint8_t* d_t,
                                  const int32_t* d_nt, int nb, int q_stride_rows, int t_stride_rows, int32_t* d_best_idx,
                                  int32_t* d_best_d, int32_t* d_second_d, void* stream) try {
    if (!m || !d_q || !d_nq || !d_t || !d_nt || nb <= 0 || q_stride_rows <= 0 || t_stride_rows <= 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    hipLaunchKernelGGL(k_knn2, dim3((q_stride_rows + 3) / 4, nb), dim3(256), 0, s, d_q, d_nq, d_t, d_nt, q_stride_rows,
                       t_stride_rows, d_best_idx, d_best_d, d_second_d);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

// MapPoint::ComputeDistinctiveDescriptors over a batch (device-resident, asynchronous).
int orb_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_start, int n_points,
                                       int32_t* d_best_idx, uint8_t* d_best_desc, void* stream) try {
    if (n_points < 0 || (n_points > 0 && (!d_desc || !d_start || !d_best_idx))) return ORB_EINVAL;
    if (n_points == 0) return ORB_OK;
    hipLaunchKernelGGL(k_distinctive, dim3(n_points), dim3(64), 0, (hipStream_t)stream, d_desc, d_start, d_best_idx,
                       d_best_desc);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

int orb_distinctive_descriptors(int device, const uint8_t* desc, const int32_t* start, int n_points, int32_t* best_idx,
                                uint8_t* best_desc) try {
    if (n_points < 0 || (n_points > 0 && (!desc || !start || !best_idx))) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    if (n_points == 0) return ORB_OK;
    for (int m = 0; m < n_points; m++)
        if (start[m + 1] < start[m]) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(device));
    const size_t T = (size_t)start[n_points] - (size_t)start[0];
    const size_t bD = ((T * 32 + 255) & ~(size_t)255), bS = (((size_t)n_points + 1) * 4 + 255) & ~(size_t)255,
                 bI = ((size_t)n_points * 4 + 255) & ~(size_t)255;
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, bD + bS + bI + (size_t)n_points * 32 + 8 * 256, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D (descriptors + relative starts), one D2H (index + descriptor)
    uint8_t* dD = (uint8_t*)sg.in(T ? desc + (size_t)start[0] * 32 : nullptr, T * 32);
    int32_t* dS = (int32_t*)sg.in(nullptr, ((size_t)n_points + 1) * 4);
    int32_t* hrel = sg.host(dS);
    for (int m = 0; m <= n_points; m++) hrel[m] = start[m] - start[0];
    if (int e_ = sg.upload_pull(s)) return e_;
    int32_t* dI = (int32_t*)sg.out((size_t)n_points * 4);
    uint8_t* dB = (uint8_t*)sg.out((size_t)n_points * 32);
    int rc = orb_distinctive_descriptors_device(dD, dS, n_points, dI, best_desc ? dB : nullptr, s);
    if (rc == ORB_OK) {
        rc = sg.download(s, dI);
        if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
        if (rc == ORB_OK) {
            std::memcpy(best_idx, sg.host(dI), (size_t)n_points * 4);
            if (best_desc) std::memcpy(best_desc, sg.host(dB), (size_t)n_points * 32);
        }
    }
    return rc;
} ORB_ABI_CATCH

static int fuse_impl(int device, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp, const uint8_t* mp_valid,
                     const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                     const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist, int sim3) {
    if (!kf || !kp || n_mp < 0 || kf->n < 0 || kf->n >= (1 << 16)) return ORB_EINVAL;
    if (n_mp > 0 && (!mp_valid || !mp_xyz || !mp_normal || !mp_min_dist || !mp_max_dist || !mp_desc || !best_idx ||
                     !best_dist))
        return ORB_EINVAL;
    if (kp->n_levels < 1 || kp->n_levels > 32 || !kp->scale_factors || (!sim3 && !kp->inv_level_sigma2))
        return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    if (n_mp == 0) return ORB_OK;
    for (int i = 0; i < kf->n; i++)
        if (kf->octave[i] < 0 || kf->octave[i] >= kp->n_levels) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(device));
    FuseKf K;
    std::memcpy(K.Tcw, kp->Tcw, sizeof(K.Tcw));
    std::memcpy(K.Ow, kp->Ow, sizeof(K.Ow));
    K.fx = kp->fx; K.fy = kp->fy; K.cx = kp->cx; K.cy = kp->cy; K.bf = kp->bf; K.logsf = kp->log_scale_factor;
    K.nlev = kp->n_levels;
    for (int l = 0; l < 32; l++) {
        K.sf[l] = l < kp->n_levels ? kp->scale_factors[l] : 0.f;
        K.isig2[l] = (l < kp->n_levels && kp->inv_level_sigma2) ? kp->inv_level_sigma2[l] : 0.f;
    }
    const int nk = kf->n;
    std::vector<orb_keypoint> hk((size_t)std::max(nk, 1));
    pack_view(kf, hk.data());
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bK = al((size_t)nk * sizeof(orb_keypoint) + 1), bD = al((size_t)nk * 32 + 1), bU = al((size_t)nk * 4 + 1),
                 bV = al((size_t)n_mp), bX = al((size_t)n_mp * 12), bM = al((size_t)n_mp * 4), bMD = al((size_t)n_mp * 32),
                 bO = al((size_t)n_mp * 4);
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, bK + bD + bU + bV + 2 * bX + 2 * bM + bMD + 2 * bO + 12 * 256, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D of every input, one D2H of both outputs
    orb_keypoint* dK = (orb_keypoint*)sg.in(hk.data(), (size_t)nk * sizeof(orb_keypoint));
    uint8_t* dD = (uint8_t*)sg.in(kf->desc, (size_t)nk * 32);
    float* dU = (float*)sg.in(kf->uright, kf->uright ? (size_t)nk * 4 : 0);
    uint8_t* dV = (uint8_t*)sg.in(mp_valid, (size_t)n_mp);
    float* dX = (float*)sg.in(mp_xyz, (size_t)n_mp * 12);
    float* dN = (float*)sg.in(mp_normal, (size_t)n_mp * 12);
    float* dMin = (float*)sg.in(mp_min_dist, (size_t)n_mp * 4);
    float* dMax = (float*)sg.in(mp_max_dist, (size_t)n_mp * 4);
    uint8_t* dMD = (uint8_t*)sg.in(mp_desc, (size_t)n_mp * 32);
    if (int e_ = sg.upload_pull(s)) return e_;
    // the two results go straight into host-mapped memory: no copy back
    int32_t* dBI = (int32_t*)sg.out_host((size_t)n_mp * 4);
    int32_t* dBD = (int32_t*)sg.out_host((size_t)n_mp * 4);
    if (sg.over) return ORB_EINTERNAL;
    const GridParams g = grid_of(kf);
    hipLaunchKernelGGL(k_fuse, dim3((n_mp + 3) / 4), dim3(256), 0, s, dK, dD, kf->uright ? (const float*)dU : nullptr,
                       nk, g, K, n_mp, dV, dX, dN, dMin, dMax, dMD, th, dBI, dBD, sim3);
    int rc = hipGetLastError() == hipSuccess ? ORB_OK : ORB_EGPU;
    if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
    if (rc == ORB_OK) {
        std::memcpy(best_idx, sg.host_out(dBI), (size_t)n_mp * 4);
        std::memcpy(best_dist, sg.host_out(dBD), (size_t)n_mp * 4);
    }
    return rc;
}

int orb_fuse(int device, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp, const uint8_t* mp_valid,
             const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
             const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist) try {
    return fuse_impl(device, kf, kp, n_mp, mp_valid, mp_xyz, mp_normal, mp_min_dist, mp_max_dist, mp_desc, th, best_idx,
                     best_dist, 0);
} ORB_ABI_CATCH

int orb_fuse_sim3(int device, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp, const uint8_t* mp_valid,
                  const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                  const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist) try {
    return fuse_impl(device, kf, kp, n_mp, mp_valid, mp_xyz, mp_normal, mp_min_dist, mp_max_dist, mp_desc, th, best_idx,
                     best_dist, 1);
} ORB_ABI_CATCH

int orb_search_by_sim3(int device, const orb_frame_view* kf1, const orb_frame_view* kf2, const orb_sim3_points* p1,
                       const orb_sim3_points* p2, const float cam1[4], const orb_scale_params* sc1,
                       const orb_scale_params* sc2, float th, int32_t* matches12) try {
    if (!kf1 || !kf2 || !p1 || !p2 || !cam1 || !sc1 || !sc2 || !matches12) return ORB_EINVAL;
    if (kf1->n < 0 || kf2->n < 0 || kf1->n >= (1 << 16) || kf2->n >= (1 << 16) || p1->n != kf1->n || p2->n != kf2->n)
        return ORB_EINVAL;
    if (sc1->n_levels < 1 || sc1->n_levels > 32 || sc2->n_levels < 1 || sc2->n_levels > 32 || !sc1->scale_factors ||
        !sc2->scale_factors)
        return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    const int n1 = kf1->n, n2 = kf2->n;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    if (n1 == 0 || n2 == 0) return 0;
    ORB_HIP_TRY(hipSetDevice(device));
    auto side = [&](const orb_sim3_points* p, const orb_scale_params* sc) {
        Sim3Side S;
        std::memcpy(S.T, p->Tcw, sizeof(S.T));
        std::memcpy(S.S, p->S, sizeof(S.S));
        S.fx = cam1[0]; S.fy = cam1[1]; S.cx = cam1[2]; S.cy = cam1[3];
        S.logsf = sc->log_scale_factor;
        S.nlev = sc->n_levels;
        for (int l = 0; l < 32; l++) S.sf[l] = l < sc->n_levels ? sc->scale_factors[l] : 0.f;
        S.th = th;
        return S;
    };
    // points of keyframe 1 project into keyframe 2 (its scale table) and vice versa
    const Sim3Side S12 = side(p1, sc2), S21 = side(p2, sc1);
    std::vector<orb_keypoint> hk1((size_t)n1), hk2((size_t)n2);
    pack_view(kf1, hk1.data());
    pack_view(kf2, hk2.data());
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t per1 = al((size_t)n1 * sizeof(orb_keypoint)) + al((size_t)n1 * 32) + al(n1) + al((size_t)n1 * 12) +
                        2 * al((size_t)n1 * 4) + al((size_t)n1 * 32) + al((size_t)n1 * 4);
    const size_t per2 = al((size_t)n2 * sizeof(orb_keypoint)) + al((size_t)n2 * 32) + al(n2) + al((size_t)n2 * 12) +
                        2 * al((size_t)n2 * 4) + al((size_t)n2 * 32) + al((size_t)n2 * 4);
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, per1 + per2 + 16 * 256, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D of both sides' inputs, one D2H of both directions' matches
    auto* dK1 = (orb_keypoint*)sg.in(hk1.data(), (size_t)n1 * sizeof(orb_keypoint));
    auto* dD1 = (uint8_t*)sg.in(kf1->desc, (size_t)n1 * 32);
    auto* dV1 = (uint8_t*)sg.in(p1->valid, n1);
    auto* dX1 = (float*)sg.in(p1->xyz, (size_t)n1 * 12);
    auto* dMin1 = (float*)sg.in(p1->min_dist, (size_t)n1 * 4);
    auto* dMax1 = (float*)sg.in(p1->max_dist, (size_t)n1 * 4);
    auto* dMD1 = (uint8_t*)sg.in(p1->desc, (size_t)n1 * 32);
    auto* dK2 = (orb_keypoint*)sg.in(hk2.data(), (size_t)n2 * sizeof(orb_keypoint));
    auto* dD2 = (uint8_t*)sg.in(kf2->desc, (size_t)n2 * 32);
    auto* dV2 = (uint8_t*)sg.in(p2->valid, n2);
    auto* dX2 = (float*)sg.in(p2->xyz, (size_t)n2 * 12);
    auto* dMin2 = (float*)sg.in(p2->min_dist, (size_t)n2 * 4);
    auto* dMax2 = (float*)sg.in(p2->max_dist, (size_t)n2 * 4);
    auto* dMD2 = (uint8_t*)sg.in(p2->desc, (size_t)n2 * 32);
    if (int e_ = sg.upload_pull(s)) return e_;
    auto* dM1 = (int32_t*)sg.out((size_t)n1 * 4);
    auto* dM2 = (int32_t*)sg.out((size_t)n2 * 4);
    hipLaunchKernelGGL(k_sim3_match, dim3((n1 + 3) / 4), dim3(256), 0, s, dK2, dD2, n2, grid_of(kf2), S12, n1, dV1, dX1,
                       dMin1, dMax1, dMD1, dM1);
    hipLaunchKernelGGL(k_sim3_match, dim3((n2 + 3) / 4), dim3(256), 0, s, dK1, dD1, n1, grid_of(kf1), S21, n2, dV2, dX2,
                       dMin2, dMax2, dMD2, dM2);
    int rc = hipGetLastError() == hipSuccess ? ORB_OK : ORB_EGPU;
    if (rc == ORB_OK) {
        rc = sg.download(s, dM1);
        if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
    }
    const int32_t* m1 = sg.host(dM1);
    const int32_t* m2 = sg.host(dM2);
    if (rc) return rc;
    int nFound = 0;   // R :1490-1503: keep the pairs both directions agree on
    for (int i1 = 0; i1 < n1; i1++) {
        const int idx2 = m1[i1];
        if (idx2 >= 0 && m2[idx2] == i1) {
            matches12[i1] = idx2;
            nFound++;
        }
    }
    return nFound;
} ORB_ABI_CATCH

int orb_search_for_triangulation(int device, const orb_frame_view* kf1, const orb_frame_view* kf2,
                                 const uint8_t* has_mp1, const uint8_t* has_mp2, int n_nodes1, const uint32_t* nodes1,
                                 const int32_t* start1, const int32_t* fidx1, int n_nodes2, const uint32_t* nodes2,
                                 const int32_t* start2, const int32_t* fidx2, const float F12[9], float ex, float ey,
                                 const float* scale_factors2, const float* level_sigma2, int n_levels2, int only_stereo,
                                 int check_ori, int32_t* matches12) try {
    if (!kf1 || !kf2 || !has_mp1 || !has_mp2 || !F12 || !scale_factors2 || !level_sigma2 || !matches12) return ORB_EINVAL;
    if (n_nodes1 < 0 || n_nodes2 < 0 || kf1->n < 0 || kf2->n < 0 || n_levels2 < 1 || n_levels2 > 32) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    for (int i = 0; i < kf1->n; i++) matches12[i] = -1;
    // common nodes (the reference's lower_bound walk) and their list ranges
    std::vector<int4> common;
    for (int a = 0, b = 0; a < n_nodes1 && b < n_nodes2;) {
        if (nodes1[a] == nodes2[b]) {
            if (start2[b + 1] - start2[b] > kSftMaxNode) return ORB_E2BIG;
            if (start1[a + 1] > start1[a] && start2[b + 1] > start2[b])
                common.push_back(make_int4(start1[a], start1[a + 1], start2[b], start2[b + 1]));
            a++;
            b++;
        } else if (nodes1[a] < nodes2[b]) {
            a++;
        } else {
            b++;
        }
    }
    const int L1 = n_nodes1 ? start1[n_nodes1] : 0, L2 = n_nodes2 ? start2[n_nodes2] : 0;
    for (int t = 0; t < L1; t++)
        if (fidx1[t] < 0 || fidx1[t] >= kf1->n) return ORB_EINVAL;
    for (int t = 0; t < L2; t++)
        if (fidx2[t] < 0 || fidx2[t] >= kf2->n) return ORB_EINVAL;
    for (int i = 0; i < kf2->n; i++)
        if (kf2->octave[i] < 0 || kf2->octave[i] >= n_levels2) return ORB_EINVAL;
    if (common.empty() || kf1->n == 0) return 0;
    ORB_HIP_TRY(hipSetDevice(device));
    SftParams P;
    std::memcpy(P.F, F12, sizeof(P.F));
    P.ex = ex; P.ey = ey; P.onlyStereo = only_stereo ? 1 : 0;
    for (int l = 0; l < 32; l++) {
        P.sf2[l] = l < n_levels2 ? scale_factors2[l] : 0.f;
        P.sig2[l] = l < n_levels2 ? level_sigma2[l] : 0.f;
    }
    const int n1 = kf1->n, n2 = kf2->n;
    std::vector<orb_keypoint> hk1((size_t)n1), hk2((size_t)std::max(n2, 1));
    pack_view(kf1, hk1.data());
    pack_view(kf2, hk2.data());
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t tot = al((size_t)n1 * sizeof(orb_keypoint)) + al((size_t)n2 * sizeof(orb_keypoint) + 1) +
                       al((size_t)n1 * 32) + al((size_t)n2 * 32 + 1) + 2 * al((size_t)n1 * 4) + 2 * al((size_t)n2 * 4 + 1) +
                       al((size_t)n1) + al((size_t)n2 + 1) + al(common.size() * 16) + al((size_t)L1 * 4 + 1) +
                       al((size_t)L2 * 4 + 1) + al(4) + 4096;
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, tot, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D of every input, one D2H of the matches and their count
    auto* dK1 = (orb_keypoint*)sg.in(hk1.data(), (size_t)n1 * sizeof(orb_keypoint));
    auto* dK2 = (orb_keypoint*)sg.in(hk2.data(), (size_t)n2 * sizeof(orb_keypoint));
    auto* dD1 = (uint8_t*)sg.in(kf1->desc, (size_t)n1 * 32);
    auto* dD2 = (uint8_t*)sg.in(kf2->desc, (size_t)n2 * 32);
    auto* dU1 = (float*)sg.in(kf1->uright, kf1->uright ? (size_t)n1 * 4 : 0);
    auto* dU2 = (float*)sg.in(kf2->uright, kf2->uright ? (size_t)n2 * 4 : 0);
    auto* dM1 = (uint8_t*)sg.in(has_mp1, (size_t)n1);
    auto* dM2 = (uint8_t*)sg.in(has_mp2, (size_t)n2);
    auto* dN = (int4*)sg.in(common.data(), common.size() * 16);
    auto* dI1 = (int32_t*)sg.in(fidx1, (size_t)L1 * 4);
    auto* dI2 = (int32_t*)sg.in(fidx2, (size_t)L2 * 4);
    auto* dMt = (int32_t*)sg.in(matches12, (size_t)n1 * 4);
    // the final matches and their count go straight into host-mapped memory (no copy back)
    auto* hMt = (int32_t*)sg.out_host((size_t)n1 * 4);
    auto* hNm = (int32_t*)sg.out_host(4);
    if (sg.over) return ORB_EINTERNAL;
    if (int e_ = sg.upload_pull(s)) return e_;
    hipLaunchKernelGGL(k_sft, dim3((unsigned)common.size()), dim3(64), 0, s, dK1, dD1, kf1->uright ? dU1 : nullptr, dM1,
                       dK2, dD2, kf2->uright ? dU2 : nullptr, dM2, dN, dI1, dI2, P, dMt);
    hipLaunchKernelGGL(k_sft_rot, dim3(1), dim3(256), 0, s, dK1, dK2, n1, check_ori ? 1 : 0, dMt, hNm, hMt);
    int rc = hipGetLastError() == hipSuccess ? ORB_OK : ORB_EGPU;
    int nm = 0;
    if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
    if (rc == ORB_OK) {
        std::memcpy(matches12, sg.host_out(hMt), (size_t)n1 * 4);
        nm = *sg.host_out(hNm);
    }
    return rc == ORB_OK ? nm : rc;
} ORB_ABI_CATCH

}  // extern "C"

// Shared host body of both SearchByBoW overloads: side 1 / side 2 views, per-feature eligibility
// (ok2 may be NULL: every side-2 feature), the two mFeatVec CSR forms; matches12 by side-1 index.
static int search_by_bow(int device, const orb_frame_view* v1, const uint8_t* ok1, int n_nodes1, const uint32_t* nodes1,
                         const int32_t* start1, const int32_t* fidx1, const orb_frame_view* v2, const uint8_t* ok2,
                         int n_nodes2, const uint32_t* nodes2, const int32_t* start2, const int32_t* fidx2,
                         int thIncl, float ratio, int check_ori, int32_t* matches12) {
    if (!v1 || !v2 || !ok1 || !matches12 || n_nodes1 < 0 || n_nodes2 < 0 || v1->n < 0 || v2->n < 0) return ORB_EINVAL;
    if ((n_nodes1 && (!nodes1 || !start1 || !fidx1)) || (n_nodes2 && (!nodes2 || !start2 || !fidx2))) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    for (int i = 0; i < v1->n; i++) matches12[i] = -1;
    std::vector<int4> common;
    for (int a = 0, b = 0; a < n_nodes1 && b < n_nodes2;) {
        if (nodes1[a] == nodes2[b]) {
            if (start2[b + 1] - start2[b] > kSbbMaxNode) return ORB_E2BIG;
            if (start1[a + 1] > start1[a] && start2[b + 1] > start2[b])
                common.push_back(make_int4(start1[a], start1[a + 1], start2[b], start2[b + 1]));
            a++;
            b++;
        } else if (nodes1[a] < nodes2[b]) {
            a++;
        } else {
            b++;
        }
    }
    const int L1 = n_nodes1 ? start1[n_nodes1] : 0, L2 = n_nodes2 ? start2[n_nodes2] : 0;
    for (int t = 0; t < L1; t++)
        if (fidx1[t] < 0 || fidx1[t] >= v1->n) return ORB_EINVAL;
    for (int t = 0; t < L2; t++)
        if (fidx2[t] < 0 || fidx2[t] >= v2->n) return ORB_EINVAL;
    if (common.empty() || v1->n == 0) return 0;
    ORB_HIP_TRY(hipSetDevice(device));
    const int n1 = v1->n, n2 = v2->n;
    std::vector<orb_keypoint> hk1((size_t)n1), hk2((size_t)std::max(n2, 1));
    pack_view(v1, hk1.data());
    pack_view(v2, hk2.data());
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t tot = al((size_t)n1 * sizeof(orb_keypoint) + 1) + al((size_t)n2 * sizeof(orb_keypoint) + 1) +
                       al((size_t)n1 * 32 + 1) + al((size_t)n2 * 32 + 1) + al((size_t)n1 + 1) + al((size_t)n2 + 1) +
                       al(common.size() * 16 + 1) + al((size_t)L1 * 4 + 1) + al((size_t)L2 * 4 + 1) +
                       al((size_t)n1 * 4 + 1) + al(4 + 1) + 4096;
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, tot, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D of every input, one D2H of the matches and their count
    auto* dK1 = (orb_keypoint*)sg.in(hk1.data(), (size_t)n1 * sizeof(orb_keypoint));
    auto* dK2 = (orb_keypoint*)sg.in(hk2.data(), (size_t)n2 * sizeof(orb_keypoint));
    auto* dD1 = (uint8_t*)sg.in(v1->desc, (size_t)n1 * 32);
    auto* dD2 = (uint8_t*)sg.in(v2->desc, (size_t)n2 * 32);
    auto* dO1 = (uint8_t*)sg.in(ok1, (size_t)n1);
    auto* dO2 = (uint8_t*)sg.in(ok2, ok2 ? (size_t)n2 : 0);
    auto* dN = (int4*)sg.in(common.data(), common.size() * 16);
    auto* dI1 = (int32_t*)sg.in(fidx1, (size_t)L1 * 4);
    auto* dI2 = (int32_t*)sg.in(fidx2, (size_t)L2 * 4);
    auto* dMt = (int32_t*)sg.in(matches12, (size_t)n1 * 4);
    auto* hMt = (int32_t*)sg.out_host((size_t)n1 * 4);   // final matches + count: host-mapped, no copy back
    auto* hNm = (int32_t*)sg.out_host(4);
    if (sg.over) return ORB_EINTERNAL;
    if (int e_ = sg.upload_pull(s)) return e_;
    hipLaunchKernelGGL(k_sbb, dim3((unsigned)common.size()), dim3(64), 0, s, dD1, dO1, dD2, ok2 ? dO2 : nullptr, dN,
                       dI1, dI2, thIncl, ratio, dMt);
    hipLaunchKernelGGL(k_sft_rot, dim3(1), dim3(256), 0, s, dK1, dK2, n1, check_ori ? 1 : 0, dMt, hNm, hMt);
    int rc = hipGetLastError() == hipSuccess ? ORB_OK : ORB_EGPU;
    int nm = 0;
    if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
    if (rc == ORB_OK) {
        std::memcpy(matches12, sg.host_out(hMt), (size_t)n1 * 4);
        nm = *sg.host_out(hNm);
    }
    return rc == ORB_OK ? nm : rc;
}

extern "C" {

int orb_search_by_bow_frame(int device, const orb_frame_view* kf, const uint8_t* kf_ok, int n_nodes_kf,
                            const uint32_t* nodes_kf, const int32_t* start_kf, const int32_t* fidx_kf,
                            const orb_frame_view* f, int n_nodes_f, const uint32_t* nodes_f, const int32_t* start_f,
                            const int32_t* fidx_f, float nn_ratio, int check_ori, int32_t* matches_f) try {
    if (!kf || !f || !matches_f || f->n < 0) return ORB_EINVAL;
    std::vector<int32_t> m12((size_t)std::max(kf->n, 1));
    const int n = search_by_bow(device, kf, kf_ok, n_nodes_kf, nodes_kf, start_kf, fidx_kf, f, nullptr, n_nodes_f,
                                nodes_f, start_f, fidx_f, 50 /* bestDist1 <= TH_LOW */, nn_ratio, check_ori, m12.data());
    if (n < 0) return n;
    for (int j = 0; j < f->n; j++) matches_f[j] = -1;
    for (int i = 0; i < kf->n; i++)
        if (m12[i] >= 0) matches_f[m12[i]] = i;
    return n;
} ORB_ABI_CATCH

int orb_search_by_bow_kf(int device, const orb_frame_view* kf1, const uint8_t* ok1, int n_nodes1,
                         const uint32_t* nodes1, const int32_t* start1, const int32_t* fidx1,
                         const orb_frame_view* kf2, const uint8_t* ok2, int n_nodes2, const uint32_t* nodes2,
                         const int32_t* start2, const int32_t* fidx2, float nn_ratio, int check_ori,
                         int32_t* matches12) try {
    if (!ok2) return ORB_EINVAL;
    return search_by_bow(device, kf1, ok1, n_nodes1, nodes1, start1, fidx1, kf2, ok2, n_nodes2, nodes2, start2, fidx2,
                         49 /* bestDist1 < TH_LOW */, nn_ratio, check_ori, matches12);
} ORB_ABI_CATCH

}  // extern "C"
