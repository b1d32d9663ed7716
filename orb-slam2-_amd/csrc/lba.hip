// MI355X-native Optimizer::LocalBundleAdjustment (R/src/Optimizer.cpp:564-918) — the g2o
// Levenberg–Marquardt / BlockSolver<6,3> Schur pipeline it runs, rebuilt for gfx950 in f64.
// R/ = /root/reference/ORB-SLAM2注释版/, G/ = R/Thirdparty/g2o/g2o/.
//
// Per LM outer iteration (G/core/optimization_algorithm_levenberg.cpp:61-164):
//   k_edge_lin        computeActiveErrors + EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ Jacobians
//                     and Huber-weighted quadratic-form blocks per edge (base_binary_edge.hpp:54-120)
//   k_vertex_reduce   Hpp, b_p per free pose and Hll, b_l per landmark
//   (LM iteration start: chi2, lambda init — inside k_point_schur in a single process)
// Per LM trial (lambda):
//   k_point_schur     D^-1 = (Hll + lambda I)^-1 per landmark (and the LM iteration start, fused)
//   k_schur_pairs     reduced camera matrix S = Hpp + lambda I - sum W D^-1 W^T and b_s, one
//                     wave per 6x6 pose-pair block (G/core/block_solver.hpp:382-440)
//   k_ldlt_solve      dense LDL^T of S in one workgroup, trailing updates on the f64 MFMA units
//                     (LinearSolverEigen's SimplicialLDLT role)
//   k_backsub_update  x_l, push + oplus (SE3Quat::exp * T, X += x_l)
//   k_edge_errors     trial chi2 (the rho test, lambda update and pop on rejection are taken by
//                     the next slot's k_edge_lin, or by k_lm_decide_fused closing a group of slots)
// The LM control state lives on the device: a "slot" (linearisation + one trial) is enqueued
// without host round trips, its kernels run only in their phase, and in a single process the
// slot is a HIP graph replayed per trial.  Every reduction has a fixed order, so results are
// bitwise reproducible run to run.  With a communicator (lba_set_comm) the landmarks are
// sharded over ranks, the bookkeeping runs as separate kernels around the all-reduces of Hpp,
// b_p, S, b_s and the chi2 / scale scalars (RCCL via the caller's callback), and every rank
// solves the same reduced system.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <initializer_list>
#include <thread>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <functional>
#include <vector>

#include "common.h"
#include "lba_host.h"
#include "lm_common.h"
#include "se3.h"

#ifdef ORB_TIMING   // instrumented variant (tools/build_variant.py)
#define TSTAMP(v) const long long v = clock64()
#define TACC(acc, a) acc += clock64() - (a)
#define HSTAMP(i) hT[i] = std::chrono::steady_clock::now()
#else
#define TSTAMP(v)
#define TACC(acc, a)
#define HSTAMP(i)
#endif

namespace orbamd {

// ------------------------------------------------------------------ device state

// Levenberg-Marquardt control state of one optimize() call, kept on the device so the host
// can enqueue trials without waiting for each decision (G/core/optimization_algorithm_levenberg.cpp:61-189).
struct LmState {
    double lambda, ni, currentChi, iniChi, rho;
    int phase;      // 0: linearise next, 1: trial next, 2: done
    int it, qmax, nBad, itersDone, trials, pop;
    int traceBase;  // first trace row of this optimize() call
    // SparseOptimizer::terminate() (the mbAbortBA flag, G/core/sparse_optimizer.h:189): sampled
    // after every trial, where g2o tests it in the trial loop (optimization_algorithm_levenberg.cpp:149)
    // and right after in the iteration loop (sparse_optimizer.cpp:376)
    int stopAfter;  // test hook: stop once trialBase + trials reaches it (-1: off)
    int trialBase;  // trials of this solve before this optimize() call
    int stopped;    // 1 once the stop was observed
    int pending;    // single process, fused slots: a trial's decision is still to be taken
};

// Kernels of the LM loop run only in their phase (`want`): 0 linearisation, 1 trial,
// 3 linearisation of iteration 0 (lambda init), -1 always.
__device__ __forceinline__ bool lm_off(const LmState* st, int want) {
    if (!st || want < 0) return false;
    if (want == 3) return st->phase != 0 || st->it != 0;
    return st->phase != want;
}

struct LbaDev {
    // problem
    double *q, *t, *X;          // estimates
    double *bq, *bt, *bX;       // push() backup
    const uint8_t* fixed;
    const int32_t *ept, *eps;   // edge -> point, pose
    const uint8_t* est;         // stereo flag
    const double *obs, *info, *cam;
    uint8_t* robust;
    uint8_t* emask;             // [NE] 1 = the edge takes part (its level is the optimized one), 0 = outlier
    const uint8_t* bad;         // [NM] MapPoint::isBad() at the call (kept out of the outlier pass)
    double* err;                // [NE][3] last computed error
    // active structure (per optimize())
    const int32_t* act;         // active edges
    int nact;
    const int32_t* poseIdx;     // pose -> hessian index or -1
    const int32_t* ptGlob;      // local -> global point
    const int32_t *actPt, *actPi; // per act position: local point, pose hessian index (-1 fixed)
    int P, M;                   // free active poses, owned active points
    const int32_t *ptStart, *ptAct;         // CSR by local point (act positions, sorted by pose index)
    const int32_t *poStart, *poAct, *poPt;  // CSR by pose index (act positions sorted by landmark; landmarks)
    // linearisation (indexed by act position)
    double *Hll_e, *Hpp_e, *Hpl_e, *bl_e, *bp_e, *echi;
    // reduced per vertex
    double *Hll, *bl, *Dinv, *db, *Hpp, *bp;   // db = Dinv b_l
    double* Ae;                 // [pose-major position][18] Hpl_e D^-1 of the edge's landmark (per trial)
    const int32_t* poPos;       // per act position: its index in the pose-major lists (-1: fixed pose)
    const int32_t* pairs;       // pose-pair blocks of S with shared landmarks, (bi << 16 | bj), bi <= bj
    const int32_t* npairs;      // their count; [1] / [2]: k_schur_pairs' workgroup / wave pairs (pairUnits)
    const int32_t* pairUnits;   // indices into pairs: [0, npairs[1]) one workgroup each, then npairs[2] one wave each
    const int32_t* tripStart;   // per listed pair: first entry of its shared-landmark list, count at +1
    const int2* trips;          // (pose-major position of pose i's edge, act position of pose j's edge), landmark order
    double *S, *bs, *x;         // x: [6P + 3M]
    double* red;                // reduction scratch
    double *partChi, *partScale, *partMax;   // per-workgroup partials (single-process LM kernels)
    double* partLin;            // fused slots: k_edge_lin's chi2 partials (partChi holds the trial's)
    int* flags;                 // [0] LDLT failure
    LmState* lm;                // LM control state (device)
    LmState* lmMid;             // fused slots: the state between k_edge_lin and k_point_schur (never
                                // written by a kernel whose other workgroups read it)
    const uint32_t* stopWord;   // host-mapped mirror of the caller's stop flag (lba_wait copies it)
};

// terminate() as the device sees it after a trial: the test hook's trial count, else the stop word
// (single process: the host-mapped word itself; with a communicator: the ranks' all-reduced sample)
__device__ __forceinline__ bool lm_stop_now(const LmState* st, const uint32_t* word, double shared) {
    if (st->stopAfter >= 0 && st->trialBase + st->trials >= st->stopAfter) return true;
    if (word) return __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    return shared > 0.0;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// Lane `lane`'s share of a partial-sum vector, p[lane] + p[lane + 64] + ... in that order (then
// a wave_sum_d): eight loads in flight per round trip instead of one dependent load per step.
__device__ __forceinline__ double lane_sum(const double* __restrict__ p, int n, int lane) {
    double c = 0.0;
    for (int b = 0; b < n; b += 8 * 64) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = b + 64 * u + lane;
            v[u] = p[i < n ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (b + 64 * u + lane < n) c += v[u];
    }
    return c;
}
__device__ __forceinline__ double lane_max(const double* __restrict__ p, int n, int lane) {
    double m = 0.0;
    for (int b = 0; b < n; b += 8 * 64) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = b + 64 * u + lane;
            v[u] = p[i < n ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (b + 64 * u + lane < n) m = fmax(m, v[u]);
    }
    return m;
}

__device__ __forceinline__ void d_transform(const LbaDev& d, int pose, int pt, double Xc[3]) {
    double r[3];
    d_quat_rot(d.q + 4 * pose, d.X + 3 * pt, r);
    for (int i = 0; i < 3; i++) Xc[i] = r[i] + d.t[3 * pose + i];
}

__device__ __forceinline__ double d_edge_chi2(const LbaDev& d, int e) {
    const double* er = d.err + 3 * e;
    const double w = d.info[e];
    double s = er[0] * (w * er[0]) + er[1] * (w * er[1]);
    if (d.est[e]) s += er[2] * (w * er[2]);
    return s;
}

// computeError of active edge k; echi[k] = its robust chi2 (activeRobustChi2 term), returned.
// An edge the outlier pass moved to level 1 (emask 0) is not active in the second optimize():
// chi2 0, and its stored error is left as the first round last computed it (g2o's chi2() of a
// level-1 edge reads that stale error in the final check, R/src/Optimizer.cpp:850-880).
// (Xw: the edge's point, read from d.X unless the caller holds it)
__device__ __forceinline__ double edge_error(const LbaDev& d, int k, double hmono, double hstereo,
                                             const double* Xw = nullptr) {
    const int e = d.act[k];
    if (!d.emask[e]) {
        d.echi[k] = 0.0;
        return 0.0;
    }
    double Xc[3];
    {
        const int pose = d.eps[e];
        double r[3];
        d_quat_rot(d.q + 4 * pose, Xw ? Xw : d.X + 3 * d.ept[e], r);
        for (int i = 0; i < 3; i++) Xc[i] = r[i] + d.t[3 * pose + i];
    }
    const double* cam = d.cam + 5 * e;
    const double* obs = d.obs + 3 * e;
    double* er = d.err + 3 * e;
    if (!d.est[e]) {
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * cam[0] + cam[2]);
        er[1] = obs[1] - (v * cam[1] + cam[3]);
        er[2] = 0;
    } else {
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * cam[0] + cam[2];
        const double r1 = Xc[1] * invz * cam[1] + cam[3];
        const float bff = (float)cam[4];
        const double r2 = r0 - (double)(bff * invz);
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
    double chi = d_edge_chi2(d, e);
    if (d.robust[e]) {
        const double delta = d.est[e] ? hstereo : hmono, dsqr = delta * delta;
        if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
    }
    d.echi[k] = chi;
    return chi;
}

__device__ void lm_begin(LmState* st, double chi, double maxDiag);
__device__ void lm_decide(LmState* st, double chiSum, double scaleSum, int fail, int maxTrials, int iterations,
                          int fixedIterations, double* __restrict__ trace, const uint32_t* stopWord, double sharedStop);

// Fused LM bookkeeping (single process).  A trial's decision and an iteration's start are not
// separate launches: every workgroup of the next kernel that needs them recomputes them from
// the producers' partials — the same loads in the same order, so the same bits — and
// workgroup 0 alone writes the result (and the trace row).  A kernel never writes the state
// copy its own workgroups read: k_edge_lin reads `lm` and writes `lmMid`, k_vertex_reduce
// reads `lmMid`, k_point_schur reads `lmMid` and writes `lm`, the trial kernels read `lm`.
struct LmFuse {
    int nChi, nScale, maxTrials, iterations, fixedIterations;
    const int32_t* freePoses;
    double* trace;
};
// The pending trial decision (lm_decide on the trial's chi2 and scale partials and the stop
// sample k_edge_errors took), as k_lm_decide_fused takes it.  Returns the state after it.
// (The partial sums are loaded whether or not a decision is pending, with the state, so a
// caller pays one memory round trip.)
__device__ __forceinline__ LmState lm_decide_local(const LbaDev& d, const LmFuse& f, int lane, bool writer) {
    LmState ls = *d.lm;
    double c = lane_sum(d.partChi, f.nChi, lane), sc = lane_sum(d.partScale, f.nScale, lane);
    const int fail = d.flags[0];
    const double stop = d.red[4];
    c = wave_sum_d(c);
    sc = wave_sum_d(sc);
    ls.pop = 0;
    if (ls.pending) {
        lm_decide(&ls, c, sc, fail, f.maxTrials, f.iterations, f.fixedIterations, writer ? f.trace : nullptr, nullptr,
                  stop);
        ls.pending = 0;
    }
    return ls;
}
// pop() of the slice [g0, g0 + stride) ... of points and free poses after a rejected trial
__device__ __forceinline__ void lm_pop_slice(const LbaDev& d, const int32_t* freePoses, int g0, int stride) {
    for (int i = g0; i < d.M; i += stride) {
        const int g = d.ptGlob[i];
        for (int j = 0; j < 3; j++) d.X[3 * (size_t)g + j] = d.bX[3 * (size_t)g + j];
    }
    for (int i = g0; i < d.P; i += stride) {
        const int p = freePoses[i];
        for (int j = 0; j < 4; j++) d.q[4 * p + j] = d.bq[4 * p + j];
        for (int j = 0; j < 3; j++) d.t[3 * p + j] = d.bt[3 * p + j];
    }
}

// Trial errors (one wave per 64 edges); partChi[block] = the wave's robust chi2 sum.
// Fused slots (`fuse`): workgroup 0 marks the decision pending and samples terminate() (the
// host-mapped stop word) once into red[4], so every decider sees the same sample.
__global__ __launch_bounds__(64) void k_edge_errors(LbaDev d, double hmono, double hstereo, int want, int fuse) {
    if (lm_off(d.lm, want)) return;
    const int k = blockIdx.x * 64 + threadIdx.x;
    const double chi = k < d.nact ? edge_error(d, k, hmono, hstereo) : 0.0;
    const double sum = wave_sum_d(chi);
    if (threadIdx.x == 0) {
        d.partChi[blockIdx.x] = sum;
        if (fuse && blockIdx.x == 0) {
            d.lm->pending = 1;
            d.red[4] = lm_stop_now(d.lm, d.stopWord, 0.0) ? 1.0 : 0.0;
        }
    }
}

// The read-only inputs of active edge k (k_edge_lin loads them before it reads the LM state,
// so the two load chains overlap).
struct EdgeStatic {
    int e, pose, pt;
    bool on, st, rob;
    double info, obs[3], cam[5];
};
__device__ __forceinline__ EdgeStatic edge_static(const LbaDev& d, int k) {
    EdgeStatic s;
    const int e = d.act[k];
    s.e = e;
    s.on = d.emask[e] != 0;
    s.pose = d.eps[e];
    s.pt = d.ept[e];
    s.st = d.est[e] != 0;
    s.rob = d.robust[e] != 0;
    s.info = d.info[e];
#pragma unroll
    for (int i = 0; i < 3; i++) s.obs[i] = d.obs[3 * (size_t)e + i];
#pragma unroll
    for (int i = 0; i < 5; i++) s.cam[i] = d.cam[5 * (size_t)e + i];
    return s;
}

// edge_error of active edge k from its prefetched read-only inputs, at the point Xw
__device__ __forceinline__ double edge_error_s(const LbaDev& d, int k, const EdgeStatic& s, double hmono,
                                               double hstereo, const double* Xw) {
    if (!s.on) {
        d.echi[k] = 0.0;
        return 0.0;
    }
    const int e = s.e, pose = s.pose;
    double Xc[3];
    {
        double r[3];
        d_quat_rot(d.q + 4 * pose, Xw, r);
        for (int i = 0; i < 3; i++) Xc[i] = r[i] + d.t[3 * pose + i];
    }
    const double* cam = s.cam;
    const double* obs = s.obs;
    double er[3];
    if (!s.st) {
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * cam[0] + cam[2]);
        er[1] = obs[1] - (v * cam[1] + cam[3]);
        er[2] = 0;
    } else {
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * cam[0] + cam[2];
        const double r1 = Xc[1] * invz * cam[1] + cam[3];
        const float bff = (float)cam[4];
        const double r2 = r0 - (double)(bff * invz);
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
    for (int i = 0; i < 3; i++) d.err[3 * (size_t)e + i] = er[i];
    const double w = s.info;
    double chi = er[0] * (w * er[0]) + er[1] * (w * er[1]);   // d_edge_chi2
    if (s.st) chi += er[2] * (w * er[2]);
    if (s.rob) {
        const double delta = s.st ? hstereo : hmono, dsqr = delta * delta;
        if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
    }
    d.echi[k] = chi;
    return chi;
}

// computeError (edge_error's arithmetic) then the Jacobians and Huber-weighted quadratic-form
// blocks of active edge k from the error just computed (no reload).  Returns the robust chi2.
// Hll_e: 3x3 upper (00 01 02 11 12 22); Hpp_e: 6x6 upper row-major (21); Hpl_e: 6x3; bl_e: 3; bp_e: 6
// (formed in registers; edge_lin_body stores them coalesced through LDS)
struct EdgeBlocks {
    double hl[6], bl[3], hp[21], bp[6], hpl[18];
};
constexpr int kEdgeStageMin = 100000;   // k_edge_lin<true> (stores through LDS) from this many active edges
// kStage: the blocks go to `ob` (zeroed by the caller) for edge_lin_body's coalesced stores;
// otherwise each lane stores its own rows (free-pose edges only for the pose blocks)
template <bool kStage>
__device__ __forceinline__ double edge_error_lin(const LbaDev& d, int k, const EdgeStatic& s, double hmono,
                                                 double hstereo, const double* qp, const double* tp, const double* Xp,
                                                 EdgeBlocks& ob) {
    const int e = s.e, pose = s.pose;
    const bool freePose = d.poseIdx[pose] >= 0;
    if (!s.on) {   // level-1 edge: chi2 0, its stored error stays, its blocks are exact zeros
        d.echi[k] = 0.0;
        if (!kStage) {
            for (int i = 0; i < 6; i++) d.Hll_e[6 * (size_t)k + i] = 0.0;
            for (int i = 0; i < 3; i++) d.bl_e[3 * (size_t)k + i] = 0.0;
            if (freePose) {
                for (int i = 0; i < 21; i++) d.Hpp_e[21 * (size_t)k + i] = 0.0;
                for (int i = 0; i < 6; i++) d.bp_e[6 * (size_t)k + i] = 0.0;
                for (int i = 0; i < 18; i++) d.Hpl_e[18 * (size_t)k + i] = 0.0;
            }
        }
        return 0.0;
    }
    double Xc[3];
    {
        double r[3];
        d_quat_rot(qp, Xp, r);
        for (int i = 0; i < 3; i++) Xc[i] = r[i] + tp[i];
    }
    const double* cam = s.cam;
    const double* obs = s.obs;
    double er[3];
    if (!s.st) {
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * cam[0] + cam[2]);
        er[1] = obs[1] - (v * cam[1] + cam[3]);
        er[2] = 0;
    } else {
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * cam[0] + cam[2];
        const double r1 = Xc[1] * invz * cam[1] + cam[3];
        const float bff = (float)cam[4];
        const double r2 = r0 - (double)(bff * invz);
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
    for (int i = 0; i < 3; i++) d.err[3 * (size_t)e + i] = er[i];
    const double w = s.info;
    double chi2 = er[0] * (w * er[0]) + er[1] * (w * er[1]);   // d_edge_chi2
    if (s.st) chi2 += er[2] * (w * er[2]);
    double chi = chi2;
    if (s.rob) {
        const double delta = s.st ? hstereo : hmono, dsqr = delta * delta;
        if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
    }
    d.echi[k] = chi;
    // linearizeOplus + constructQuadraticForm at the same estimate (Xc as d_transform gives it)
    double R[9];
    d_quat_to_R(qp, R);
    const double x = Xc[0], y = Xc[1], z = Xc[2], z_2 = z * z;
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    const bool st = s.st;
    const int D = st ? 3 : 2;
    double A[9], B[18];
    if (!st) {
        const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 3; c++)
                A[r * 3 + c] = -1. / z * (tmp[r * 3] * R[c] + tmp[r * 3 + 1] * R[3 + c] + tmp[r * 3 + 2] * R[6 + c]);
        A[6] = A[7] = A[8] = 0;
    } else {
        for (int c = 0; c < 3; c++) {
            A[c] = -fx * R[c] / z + fx * x * R[6 + c] / z_2;
            A[3 + c] = -fy * R[3 + c] / z + fy * y * R[6 + c] / z_2;
            A[6 + c] = A[c] - bf * R[6 + c] / z_2;
        }
    }
    B[0] = x * y / z_2 * fx;       B[1] = -(1 + (x * x / z_2)) * fx; B[2] = y / z * fx;
    B[3] = -1. / z * fx;           B[4] = 0;                         B[5] = x / z_2 * fx;
    B[6] = (1 + y * y / z_2) * fy; B[7] = -x * y / z_2 * fy;         B[8] = -x / z * fy;
    B[9] = 0;                      B[10] = -1. / z * fy;             B[11] = y / z_2 * fy;
    if (st) {
        B[12] = B[0] - bf * y / z_2; B[13] = B[1] + bf * x / z_2; B[14] = B[2];
        B[15] = B[3];                B[16] = 0;                   B[17] = B[5] - bf / z_2;
    } else {
        for (int i = 12; i < 18; i++) B[i] = 0;
    }
    double rho1 = 1.0;
    if (s.rob) {
        const double delta = st ? hstereo : hmono;
        if (chi2 > delta * delta) rho1 = delta / sqrt(chi2);
    }
    const double W = rho1 * w;
    double om[3];
    for (int r = 0; r < 3; r++) om[r] = r < D ? -(w * er[r]) * rho1 : 0.0;
    // the products below run over all 3 rows: a mono edge's third Jacobian row and om[2] are
    // zero, so the extra terms add exact zeros (constant trip counts keep A, B in registers)
    double* hl = kStage ? ob.hl : d.Hll_e + 6 * (size_t)k;
    double* bl = kStage ? ob.bl : d.bl_e + 3 * (size_t)k;
    {
        int o = 0;
        for (int i = 0; i < 3; i++) {
            double sm = 0;
            for (int r = 0; r < 3; r++) sm += A[r * 3 + i] * om[r];
            bl[i] = sm;
            for (int j = i; j < 3; j++) {
                double h = 0;
                for (int r = 0; r < 3; r++) h += A[r * 3 + i] * W * A[r * 3 + j];
                hl[o++] = h;
            }
        }
    }
    if (kStage || freePose) {   // (staged, a fixed pose's edge fills its unused slots: nothing reads them)
        double* hp = kStage ? ob.hp : d.Hpp_e + 21 * (size_t)k;
        double* bp = kStage ? ob.bp : d.bp_e + 6 * (size_t)k;
        double* hpl = kStage ? ob.hpl : d.Hpl_e + 18 * (size_t)k;
        int o = 0;
        for (int i = 0; i < 6; i++) {
            double sm = 0;
            for (int r = 0; r < 3; r++) sm += B[r * 6 + i] * om[r];
            bp[i] = sm;
            for (int j = i; j < 6; j++) {
                double h = 0;
                for (int r = 0; r < 3; r++) h += B[r * 6 + i] * W * B[r * 6 + j];
                hp[o++] = h;
            }
            for (int j = 0; j < 3; j++) {
                double h = 0;
                for (int r = 0; r < 3; r++) h += B[r * 6 + i] * W * A[r * 3 + j];
                hpl[i * 3 + j] = h;
            }
        }
    }
    return chi;
}

// Phase-0 linearisation of active edge k (computeActiveErrors + linearizeOplus +
// constructQuadraticForm, G/core/sparse_optimizer.cpp:384-394, block_solver.hpp:502-561).
// One wave per 64 edges (a launch wide enough to reach every CU); partChi[block] as above.
struct EdgeVars {   // the edge's pose and point estimates, loaded with its static inputs
    double q[4], t[3], X[3];
};
__device__ __forceinline__ void edge_vars(const LbaDev& d, const EdgeStatic& es, EdgeVars& v) {
#pragma unroll
    for (int i = 0; i < 4; i++) v.q[i] = d.q[4 * es.pose + i];
#pragma unroll
    for (int i = 0; i < 3; i++) v.t[i] = d.t[3 * es.pose + i];
#pragma unroll
    for (int i = 0; i < 3; i++) v.X[i] = d.X[3 * (size_t)es.pt + i];
}
template <bool kStage>
__device__ __forceinline__ void edge_lin_body(const LbaDev& d, const EdgeStatic& es, const EdgeVars& ev, double hmono,
                                              double hstereo, int fuse);
// Fused slots: first takes the previous trial's pending decision (lm_decide_local; workgroup
// 0 writes it back) and, after a rejection, restores this workgroup's slice of the estimates.
template <bool kStage>
__global__ __launch_bounds__(64) void k_edge_lin(LbaDev d, double hmono, double hstereo, int fuse, LmFuse f) {
    const EdgeStatic es = edge_static(d, max(min((int)(blockIdx.x * 64 + threadIdx.x), d.nact - 1), 0));
    // the estimates as they stand: what the linearisation reads unless the decision below pops
    // (then the push() backups are read instead and these are dropped)
    EdgeVars ev;
    edge_vars(d, es, ev);
    if (fuse) {
        const LmState ls = lm_decide_local(d, f, threadIdx.x, blockIdx.x == 0 && threadIdx.x == 0);
        if (blockIdx.x == 0 && threadIdx.x == 0) *d.lmMid = ls;
        const int phase = ls.phase, pop = ls.pop;
        if (pop) lm_pop_slice(d, f.freePoses, blockIdx.x * 64 + threadIdx.x, (int)gridDim.x * 64);
        if (phase != 0) return;
        if (pop) {
            // a rejected trial that still ends the iteration (fixed-iteration mode, rho == 0 or a
            // failed solve) is followed by the next linearisation in this same launch, while other
            // workgroups are still restoring their slices: read the restored values from the push()
            // backups instead (bX for every active point, bq / bt for every pose — fixed poses'
            // backups are their never-changing estimates, copied at the solve's start)
            LbaDev db = d;
            db.X = d.bX;
            db.q = d.bq;
            db.t = d.bt;
            EdgeVars evb;
            edge_vars(db, es, evb);
            edge_lin_body<kStage>(db, es, evb, hmono, hstereo, fuse);
            return;
        }
    } else if (lm_off(d.lm, 0)) {
        return;
    }
    edge_lin_body<kStage>(d, es, ev, hmono, hstereo, fuse);
}
template <bool kStage>
__device__ __forceinline__ void edge_lin_body(const LbaDev& d, const EdgeStatic& es, const EdgeVars& ev, double hmono,
                                              double hstereo, int fuse) {
    const int k = blockIdx.x * 64 + threadIdx.x;
    double chi = 0.0;
    EdgeBlocks ob;
    if (kStage) {
#pragma unroll
        for (int i = 0; i < 6; i++) ob.hl[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; i++) ob.bl[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 21; i++) ob.hp[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 6; i++) ob.bp[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 18; i++) ob.hpl[i] = 0.0;
    }
    if (k < d.nact) chi = edge_error_lin<kStage>(d, k, es, hmono, hstereo, ev.q, ev.t, ev.X, ob);
    const double sum = wave_sum_d(chi);
    if (threadIdx.x == 0) (fuse ? d.partLin : d.partChi)[blockIdx.x] = sum;
    if (!kStage) return;
    // the wave's 64 edges' blocks, each array through LDS, then stored as one contiguous run (a
    // lane writing its own 168-byte row makes every store instruction touch 64 lines: 1.9x the
    // bytes below L2 at 200 KF, PMC).  Small problems take k_edge_lin<false> (latency-bound there:
    // the LDS round trips cost more than the lines).
    __shared__ double stg[64 * 21];
    const int base = blockIdx.x * 64, nk = min(d.nact - base, 64), lane = threadIdx.x;
    auto put = [&](double* dst, const double* v, int W) {
        for (int i = 0; i < W; i++) stg[lane * W + i] = v[i];
        __syncthreads();
        for (int t = lane; t < nk * W; t += 64) dst[(size_t)base * W + t] = stg[t];
        __syncthreads();
    };
    put(d.Hpp_e, ob.hp, 21);
    put(d.Hpl_e, ob.hpl, 18);
    put(d.bp_e, ob.bp, 6);
    put(d.Hll_e, ob.hl, 6);
    put(d.bl_e, ob.bl, 3);
}

// Vertex blocks (256 threads): workgroups [0, P) reduce Hpp, b_p of one free pose over its
// edges (thread partials meet in LDS in a fixed order); the rest reduce Hll, b_l of 64 owned
// landmarks each, four lanes per landmark (edges in pose-index order, lanes combined by xor).
// partMax[block] = the block's largest |diagonal| (computeLambdaInit).
constexpr int kLanesPerPt = 4;
// Pose block p (256 threads): Hpp_p, b_p over its edges; returns the block's max |diagonal|
// (valid in thread 0).
// Pose block p (256 threads): Hpp_p (21 upper entries) and b_p over its edges.  The 27 values
// of an edge are read by 27 lanes of a 32-lane group (one edge's Hpp_e and bp_e rows are
// contiguous: a few cache lines per load instruction, where a lane reading a whole 27-value row
// makes every instruction touch 64 lines); group g of the 8 takes edges g, g + 8, ... of the
// pose's list.  The list's first kPoseIdx act positions are fetched by the block in one round
// trip (pose_prefetch, which k_vertex_schur issues before it reads the LM state) and shared
// through LDS; the value loads go out kPoseBatch per lane at a time.  The 8 group partials meet
// in LDS in group order.  Returns the block's max |diagonal| (thread 0).
constexpr int kPoseIdx = 1024, kPoseBatch = 32;
struct PosePrefetch {
    int a0, a1;
    int k[kPoseIdx / 256];
};
__device__ __forceinline__ const double* pose_val_ptr(const LbaDev& d, int k, int v) {
    return v < 21 ? d.Hpp_e + 21 * (size_t)k + v : d.bp_e + 6 * (size_t)k + (v - 21);
}
__device__ __forceinline__ void pose_prefetch(const LbaDev& d, int p, PosePrefetch& f) {
    const int tid = threadIdx.x;
    f.a0 = d.poStart[p];
    f.a1 = d.poStart[p + 1];
    const int last = max(f.a1 - 1, 0);
#pragma unroll
    for (int u = 0; u < kPoseIdx / 256; u++) f.k[u] = d.poAct[min(f.a0 + tid + 256 * u, last)];
}
__device__ __forceinline__ double pose_block_reduce(const LbaDev& d, int p, double (*part)[257],
                                                    const PosePrefetch& f) {
    const int tid = threadIdx.x, g = tid >> 5, v = min(tid & 31, 26);
    int* idx = reinterpret_cast<int*>(&part[0][0]);   // (9 * 257 doubles hold kPoseIdx ints)
#pragma unroll
    for (int u = 0; u < kPoseIdx / 256; u++) idx[tid + 256 * u] = f.k[u];
    __syncthreads();
    const int n = f.a1 - f.a0;
    double acc = 0.0;
    // the list in chunks of kPoseIdx act positions: the first chunk came with pose_prefetch, the
    // next ones (poses with more edges, the scaled windows) are staged the same way, so every
    // value load of a chunk is issued without waiting on an index load
    for (int c0 = 0; c0 < n; c0 += kPoseIdx) {
        if (c0 > 0) {
            __syncthreads();   // the previous chunk's indices are consumed
            const int last = f.a1 - 1;
#pragma unroll
            for (int u = 0; u < kPoseIdx / 256; u++) idx[tid + 256 * u] = d.poAct[min(f.a0 + c0 + tid + 256 * u, last)];
            __syncthreads();
        }
        const int nl = min(n - c0, kPoseIdx);
        for (int jb = g; jb < nl; jb += 8 * kPoseBatch) {   // edges jb, jb + 8, ... of this group
            double x[kPoseBatch];
#pragma unroll
            for (int u = 0; u < kPoseBatch; u++) x[u] = *pose_val_ptr(d, idx[min(jb + 8 * u, nl - 1)], v);
#pragma unroll
            for (int u = 0; u < kPoseBatch; u++) acc = jb + 8 * u < nl ? acc + x[u] : acc;
        }
    }
    __syncthreads();   // idx aliases part
    if ((tid & 31) < 27) part[g][tid & 31] = acc;
    __syncthreads();
    if (tid < 27) {
        double val = 0.0;
#pragma unroll
        for (int q = 0; q < 8; q++) val += part[q][tid];
        if (tid < 21) {
            int i = 0, o = tid;
            while (o >= 6 - i) { o -= 6 - i; i++; }
            const int j = i + o;
            d.Hpp[36 * (size_t)p + i * 6 + j] = val;
            d.Hpp[36 * (size_t)p + j * 6 + i] = val;
        } else {
            d.bp[6 * (size_t)p + tid - 21] = val;
        }
        part[8][tid] = val;
    }
    __syncthreads();
    double m = 0;
    if (tid == 0) {   // diagonal entries sit at upper-row offsets 0, 6, 11, 15, 18, 20
        const int dia[6] = {0, 6, 11, 15, 18, 20};
        for (int i = 0; i < 6; i++) m = fmax(m, fabs(part[8][dia[i]]));
    }
    return m;
}

// Landmark l's Hll (6 upper entries) and b_l over its edges, kLanesPerPt lanes per landmark
// (edges in pose-index order, lanes combined by xor); every lane of the group returns the sums.
// The lane's first kPtBatch edges are fetched with all loads in flight (landmark_prefetch, which
// k_vertex_schur issues before it reads the LM state); further edges follow in order.
constexpr int kPtBatch = 2;
struct PtPrefetch {
    int a0, a1;
    double v[kPtBatch][9];
    int k[kPtBatch], pi[kPtBatch];   // the same edges' act positions, pose indices and Hpl blocks
    double w[kPtBatch][18];          // (k_vertex_schur's Hpl D^-1 products)
};
__device__ __forceinline__ void landmark_prefetch(const LbaDev& d, int l, int sub, PtPrefetch& f) {
    const int lc = min(l, d.M - 1);
    f.a0 = d.ptStart[lc] + sub;
    f.a1 = l < d.M ? d.ptStart[lc + 1] : f.a0;
    const int last = max(d.ptStart[lc + 1] - 1, 0);
    int* const k = f.k;
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) k[u] = d.ptAct[min(f.a0 + kLanesPerPt * u, last)];
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) {
#pragma unroll
        for (int i = 0; i < 6; i++) f.v[u][i] = d.Hll_e[6 * (size_t)k[u] + i];
#pragma unroll
        for (int i = 0; i < 3; i++) f.v[u][6 + i] = d.bl_e[3 * (size_t)k[u] + i];
        f.pi[u] = d.actPi[k[u]];
        const double2* B = reinterpret_cast<const double2*>(d.Hpl_e + 18 * (size_t)k[u]);
#pragma unroll
        for (int h = 0; h < 9; h++) {   // (a fixed pose's edge reads its unused Hpl slot)
            const double2 x = B[h];
            f.w[u][2 * h] = x.x;
            f.w[u][2 * h + 1] = x.y;
        }
    }
}
__device__ __forceinline__ void landmark_reduce(const LbaDev& d, int l, int sub, double h[6], double b[3],
                                                const PtPrefetch& f) {
    for (int i = 0; i < 6; i++) h[i] = 0.0;
    for (int i = 0; i < 3; i++) b[i] = 0.0;
    if (l < d.M) {
#pragma unroll
        for (int u = 0; u < kPtBatch; u++) {
            const bool in = f.a0 + kLanesPerPt * u < f.a1;
#pragma unroll
            for (int i = 0; i < 6; i++) h[i] = in ? h[i] + f.v[u][i] : h[i];
#pragma unroll
            for (int i = 0; i < 3; i++) b[i] = in ? b[i] + f.v[u][6 + i] : b[i];
        }
        for (int a = f.a0 + kLanesPerPt * kPtBatch; a < f.a1; a += kLanesPerPt) {
            const int k = d.ptAct[a];
#pragma unroll
            for (int i = 0; i < 6; i++) h[i] += d.Hll_e[6 * (size_t)k + i];
#pragma unroll
            for (int i = 0; i < 3; i++) b[i] += d.bl_e[3 * (size_t)k + i];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) { h[i] += __shfl_xor(h[i], 1, 64); h[i] += __shfl_xor(h[i], 2, 64); }
#pragma unroll
    for (int i = 0; i < 3; i++) { b[i] += __shfl_xor(b[i], 1, 64); b[i] += __shfl_xor(b[i], 2, 64); }
}
__device__ __forceinline__ void landmark_store(const LbaDev& d, int l, const double h[6], const double b[3]) {
    double* H = d.Hll + 9 * (size_t)l;
    H[0] = h[0]; H[1] = h[1]; H[2] = h[2];
    H[3] = h[1]; H[4] = h[3]; H[5] = h[4];
    H[6] = h[2]; H[7] = h[4]; H[8] = h[5];
    for (int i = 0; i < 3; i++) d.bl[3 * (size_t)l + i] = b[i];
}

__global__ __launch_bounds__(256) void k_vertex_reduce(LbaDev d) {
    if (lm_off(d.lm, 0)) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ double part[9][257];   // (the pose blocks' 8 group partials + the sums; kPoseIdx ints alias it)
    __shared__ double wmax[4];
    if ((int)blockIdx.x < d.P) {
        PosePrefetch pf;
        pose_prefetch(d, blockIdx.x, pf);
        const double m = pose_block_reduce(d, blockIdx.x, part, pf);
        if (tid == 0) d.partMax[blockIdx.x] = m;
        return;
    }
    const int l = ((int)blockIdx.x - d.P) * (256 / kLanesPerPt) + (tid / kLanesPerPt), sub = tid % kLanesPerPt;
    double h[6], b[3];
    PtPrefetch pf;
    landmark_prefetch(d, l, sub, pf);
    landmark_reduce(d, l, sub, h, b, pf);
    double m = 0.0;
    if (l < d.M && sub == 0) {
        landmark_store(d, l, h, b);
        m = fmax(fabs(h[0]), fmax(fabs(h[3]), fabs(h[5])));
    }
    m = wave_max_d(m);
    if (lane == 0) wmax[wave] = m;
    __syncthreads();
    if (tid == 0) d.partMax[blockIdx.x] = fmax(fmax(wmax[0], wmax[1]), fmax(wmax[2], wmax[3]));
}

// D^-1 = (Hll + lambda I)^-1 (Eigen's 3x3 cofactor inverse) of a landmark block m (row-major)
__device__ __forceinline__ void dinv_of(double m[9], double lambda, double Di[9]) {
    m[0] += lambda; m[4] += lambda; m[8] += lambda;
    double c[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            c[i * 3 + j] = m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
        }
    const double det = c[0] * m[0] + c[3] * m[3] + c[6] * m[6];
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Di[j * 3 + i] = c[i * 3 + j] * invdet;
}
// D^-1 and D^-1 b_l of landmark l
__device__ __forceinline__ void dinv_store(const LbaDev& d, int l, const double Di[9], const double blv[3]) {
    for (int i = 0; i < 9; i++) d.Dinv[9 * (size_t)l + i] = Di[i];
    for (int i = 0; i < 3; i++) d.db[3 * (size_t)l + i] = Di[i * 3] * blv[0] + Di[i * 3 + 1] * blv[1] + Di[i * 3 + 2] * blv[2];
}
// Hpl_e D^-1 (the product of G/core/block_solver.hpp:419) of every free-pose edge of landmark l,
// edges a0, a0 + stride, ... of its list: formed once per edge and trial here, where D^-1 is in
// registers, instead of once per pose pair in k_schur_pairs.  It goes to the edge's pose-major
// position, so k_schur_pairs reads each pose's blocks as one contiguous run (the Hpl_e it pairs
// them with are read in place: trips and poAct carry their act positions)
__device__ __forceinline__ void hpl_dinv_edges(const LbaDev& d, int l, const double Di[9], int sub, int stride) {
    const int a1 = d.ptStart[l + 1];
    for (int a = d.ptStart[l] + sub; a < a1; a += stride) {
        const int k = d.ptAct[a];
        if (d.actPi[k] < 0) continue;   // fixed pose: no Hpl block
        const double2* B = reinterpret_cast<const double2*>(d.Hpl_e + 18 * (size_t)k);
        double w[18];
#pragma unroll
        for (int h = 0; h < 9; h++) {
            const double2 x = B[h];
            w[2 * h] = x.x; w[2 * h + 1] = x.y;
        }
        double u[18];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int q = 0; q < 3; q++)
                u[r * 3 + q] = __builtin_fma(w[r * 3 + 2], Di[6 + q], __builtin_fma(w[r * 3 + 1], Di[3 + q], w[r * 3] * Di[q]));
        double2* U = reinterpret_cast<double2*>(d.Ae + 18 * (size_t)d.poPos[k]);
#pragma unroll
        for (int h = 0; h < 9; h++) U[h] = make_double2(u[2 * h], u[2 * h + 1]);
    }
}

// hpl_dinv_edges for lane `sub` of a landmark's kLanesPerPt group with its first kPtBatch edges'
// Hpl blocks already in registers (landmark_prefetch)
__device__ __forceinline__ void hpl_dinv_prefetched(const LbaDev& d, const double Di[9], const PtPrefetch& f) {
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) {
        if (f.a0 + kLanesPerPt * u >= f.a1 || f.pi[u] < 0) continue;
        double v[18];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int q = 0; q < 3; q++)
                v[r * 3 + q] = __builtin_fma(f.w[u][r * 3 + 2], Di[6 + q],
                                             __builtin_fma(f.w[u][r * 3 + 1], Di[3 + q], f.w[u][r * 3] * Di[q]));
        double2* U = reinterpret_cast<double2*>(d.Ae + 18 * (size_t)d.poPos[f.k[u]]);
#pragma unroll
        for (int h = 0; h < 9; h++) U[h] = make_double2(v[2 * h], v[2 * h + 1]);
    }
}

// Per landmark with lambda (G/core/block_solver.hpp:380-398): D^-1 = (Hll + lambda I)^-1
// (Eigen's 3x3 cofactor inverse) and D^-1 b_l.
// Fused slots: an iteration that was just linearised (phase 0) starts here — lm_begin from
// k_edge_lin's chi2 partials and k_vertex_reduce's maxima (workgroup 0 writes the state).
__global__ __launch_bounds__(64) void k_point_schur(LbaDev d, int fuse, int nChi, int nMax) {
    // every load of the workgroup is issued before the state is known (one memory round trip):
    // the landmark's Hll, b_l and, fused, the state and the partials
    const int l = blockIdx.x * 64 + threadIdx.x, lc = min(l, d.M - 1);
    double m[9], blv[3];
    for (int i = 0; i < 9; i++) m[i] = d.Hll[9 * (size_t)lc + i];
    for (int i = 0; i < 3; i++) blv[i] = d.bl[3 * (size_t)lc + i];
    double lambda;
    if (fuse) {
        LmState ls = *d.lmMid;
        const int lane = threadIdx.x;
        if (ls.phase == 0) {
            // lm_begin: only workgroup 0 (which writes the state) needs the chi2 sum; the others
            // need the maximum diagonal only at iteration 0, where it sets lambda
            if (blockIdx.x == 0 || ls.it == 0) {
                double c = blockIdx.x == 0 ? lane_sum(d.partLin, nChi, lane) : 0.0;
                double mx = ls.it == 0 ? lane_max(d.partMax, nMax, lane) : 0.0;
                c = wave_sum_d(c);
                mx = wave_max_d(mx);
                lm_begin(&ls, c, mx);
            } else {
                ls.phase = 1;   // (lm_begin at it > 0 leaves lambda as it is)
            }
        }
        if (blockIdx.x == 0 && lane == 0) *d.lm = ls;
        if (ls.phase != 1) return;
        lambda = ls.lambda;
    } else {
        if (lm_off(d.lm, 1)) return;
        lambda = d.lm->lambda;
    }
    if (l >= d.M) return;
    double Di[9];
    dinv_of(m, lambda, Di);
    dinv_store(d, l, Di, blv);
    hpl_dinv_edges(d, l, Di, 0, 1);
}

// Landmarks of the fused slots after an optimize()'s first (slots 2.., where the iteration
// start never initialises lambda): k_vertex_reduce's reduction and k_point_schur's D^-1 in one
// launch.  Workgroups [0, P) reduce the free poses' Hpp, b_p; the others reduce 64 landmarks'
// Hll, b_l (phase 0) or read them back (a retrial, phase 1) and form D^-1, D^-1 b_l with the
// trial's lambda.  Wave 0 of every workgroup reads the state from lmMid: a just-linearised
// iteration starts here (lm_begin at it > 0 leaves lambda alone, so only workgroup 0, which
// writes the state to lm, sums k_edge_lin's chi2 partials).
__global__ __launch_bounds__(256) void k_vertex_schur(LbaDev d, int nChi) {
    __shared__ double part[9][257];   // (the pose blocks' 8 group partials + the sums; kPoseIdx ints alias it)
    __shared__ double lamS;
    __shared__ int ph0S, phS;
    const int tid = threadIdx.x, lane = tid & 63;
    // a pose block's edge data is fetched before the state is known (wasted on a retrial, where
    // the reduction is not redone): the two load chains overlap
    PosePrefetch pf;
    PtPrefetch lf;
    const int l = ((int)blockIdx.x - d.P) * (256 / kLanesPerPt) + (tid / kLanesPerPt), sub = tid % kLanesPerPt;
    if ((int)blockIdx.x < d.P) pose_prefetch(d, blockIdx.x, pf);
    else landmark_prefetch(d, l, sub, lf);
    if (tid < 64) {
        LmState ls = *d.lmMid;
        const int ph0 = ls.phase;
        if (ph0 == 0) {
            if (blockIdx.x == 0) {
                double c = lane_sum(d.partLin, nChi, lane);
                c = wave_sum_d(c);
                lm_begin(&ls, c, 0.0);   // (it > 0 here: the max diagonal is not used)
            } else {
                ls.phase = 1;
            }
        }
        if (blockIdx.x == 0 && lane == 0) *d.lm = ls;
        if (lane == 0) {
            lamS = ls.lambda;
            ph0S = ph0;
            phS = ls.phase;
        }
    }
    __syncthreads();
    if (phS != 1) return;
    const int ph0 = ph0S;
    const double lambda = lamS;
    if ((int)blockIdx.x < d.P) {
        if (ph0 == 0) (void)pose_block_reduce(d, blockIdx.x, part, pf);
        return;
    }
    double h[6], b[3];
    if (ph0 == 0) landmark_reduce(d, l, sub, h, b, lf);
    if (l >= d.M) return;
    // every lane of the landmark's group forms D^-1 (the reduced sums are in all four), lane 0
    // stores it, and the four lanes split the landmark's Hpl D^-1 products
    double m[9], blv[3];
    if (ph0 == 0) {
        if (sub == 0) landmark_store(d, l, h, b);
        m[0] = h[0]; m[1] = h[1]; m[2] = h[2]; m[3] = h[1]; m[4] = h[3]; m[5] = h[4]; m[6] = h[2]; m[7] = h[4]; m[8] = h[5];
        blv[0] = b[0]; blv[1] = b[1]; blv[2] = b[2];
    } else {
        for (int i = 0; i < 9; i++) m[i] = d.Hll[9 * (size_t)l + i];
        for (int i = 0; i < 3; i++) blv[i] = d.bl[3 * (size_t)l + i];
    }
    double Di[9];
    dinv_of(m, lambda, Di);
    if (sub == 0) dinv_store(d, l, Di, blv);
    hpl_dinv_prefetched(d, Di, lf);   // the lane's first kPtBatch edges, their Hpl blocks prefetched
    hpl_dinv_edges(d, l, Di, sub + kLanesPerPt * kPtBatch, kLanesPerPt);
}

// Reduced camera system (G/core/block_solver.hpp:408-440): one workgroup per pose-pair block
// (i <= j, row-major triangular order; workgroups stride over the listed pairs), S_ij = [i == j]
// (Hpp_i + lambda I) - sum_l (Hpl_il D_l^-1) Hpl_jl^T over the landmarks l seen by both
// (k_pair_trip's list).  Thread t accumulates the whole 6 x 6 product of the pair's landmarks
// t, t + 256, ... in registers (A_e = Hpl_e D^-1 from the landmark kernel); each wave's 64
// partials of the 36 (42) values meet by recursive halving across the wave (reduce_halve, lane v
// then holds value v) and the four waves' sums in 2 KB of LDS, in a fixed order, so the result is
// reproducible run to run.  (The former form reduced 256 partials through 86 KB of LDS: one
// workgroup per CU.)  The diagonal blocks also form b_s,i = b_p,i - sum_e Hpl_e D_l^-1 b_l over
// pose i's edges (rank 0 carries Hpp + lambda I and b_p).
constexpr int kSpT = 256;
constexpr int kSpList = 4096;   // pose j's landmark list held in LDS up to this length
constexpr int kSpChunk = 1024;  // pose i's edges looked up per round (4 per thread)
constexpr int kSpW = kSpT / 64;   // k_schur_pairs: waves per workgroup
constexpr int kSpMaxWg = 4096;    // k_schur_pairs: workgroups at most (they stride over the pairs; a multiple of 8)

// cur[0 .. 2W) of every lane -> cur[0 .. W): lanes with bit W set keep the upper half, the others
// the lower, each adding its xor-W partner's copy of the half it keeps
template <int W>
__device__ __forceinline__ void reduce_halve(double* cur, int lane) {
    const bool up = (lane & W) != 0;
#pragma unroll
    for (int k = 0; k < W; k++) {
        const double keep = up ? cur[W + k] : cur[k];
        const double send = up ? cur[k] : cur[W + k];
        cur[k] = keep + __shfl_xor(send, W, 64);
    }
}

// the product of one shared landmark: A_e1 (pose-major position e1) against Hpl_k2 (act position
// k2) into acc[0 .. 36); diagonal blocks (the same edge) also b_s's Hpl_e1 D^-1 b_l into acc[36 .. 42)
__device__ __forceinline__ void sp_product(const LbaDev& d, double acc[64], int e1, int k2, int l, bool diag) {
    const double2* Ui = reinterpret_cast<const double2*>(d.Ae + 18 * (size_t)e1);
    const double2* Bj = reinterpret_cast<const double2*>(d.Hpl_e + 18 * (size_t)k2);
    double v[18], u[18];
#pragma unroll
    for (int h = 0; h < 9; h++) {
        const double2 x = Ui[h], y = Bj[h];
        u[2 * h] = x.x; u[2 * h + 1] = x.y;
        v[2 * h] = y.x; v[2 * h + 1] = y.y;
    }
    // three fused multiply-adds per entry (the terms accumulate straight into the partial)
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
        for (int q = 0; q < 6; q++)
            acc[r * 6 + q] = __builtin_fma(u[r * 3 + 2], v[q * 3 + 2],
                                           __builtin_fma(u[r * 3 + 1], v[q * 3 + 1],
                                                         __builtin_fma(u[r * 3], v[q * 3], acc[r * 6 + q])));
    if (diag) {
        const double* db = d.db + 3 * (size_t)l;
        const double g0 = db[0], g1 = db[1], g2 = db[2];
#pragma unroll
        for (int i = 0; i < 6; i++)
            acc[36 + i] = __builtin_fma(v[i * 3 + 2], g2, __builtin_fma(v[i * 3 + 1], g1, __builtin_fma(v[i * 3], g0, acc[36 + i])));
    }
}

// the wave's 64 partials of 64 values -> lane v holds value v (recursive halving, fixed order)
__device__ __forceinline__ void sp_wave_reduce(double acc[64], int lane) {
    reduce_halve<32>(acc, lane);
    reduce_halve<16>(acc, lane);
    reduce_halve<8>(acc, lane);
    reduce_halve<4>(acc, lane);
    reduce_halve<2>(acc, lane);
    reduce_halve<1>(acc, lane);
}

// Work units (k_pair_list, once per solve): the diagonal blocks and the off-diagonal pairs sharing
// more than kSpSmall landmarks take a workgroup each (its four waves' partials meet in LDS); the
// others a wave each, four per workgroup, with no LDS and no barrier — a 200 KF corridor window's
// ~8 k pairs share ~140 landmarks each, so a workgroup per pair spent most of its time in four
// waves' reductions and barriers at half its lanes.
__global__ __launch_bounds__(kSpT) void k_schur_pairs(LbaDev d, int addDiag) {
    const int np = d.npairs[0], nBig = d.npairs[1], nSmall = d.npairs[2];
    const int phase = d.lm->phase;
    if (phase != 1) return;     // lm_off(d.lm, 1)
    __shared__ double wsum[kSpW][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nUnits = nBig + (nSmall + kSpW - 1) / kSpW;
    // XCD-aware: workgroup b runs on XCD b % 8 (gridDim.x is a multiple of 8), and each XCD takes
    // one contiguous eighth of the unit list (pair order), so a pose's blocks are reused from that
    // XCD's L2
    const int chunk = (nUnits + 7) >> 3;
    const int n = 6 * d.P;
    for (int vb = blockIdx.x; (vb >> 3) < chunk; vb += gridDim.x) {
        const int un = (vb & 7) * chunk + (vb >> 3);
        if (un >= nUnits) continue;
        double acc[64];
#pragma unroll
        for (int i = 0; i < 64; i++) acc[i] = 0.0;
        if (un >= nBig) {   // one pair per wave
            const int sidx = (un - nBig) * kSpW + wave;
            if (sidx >= nSmall) continue;
            const int k = d.pairUnits[nBig + sidx];
            if (k >= np) continue;
            const int pr = __builtin_amdgcn_readfirstlane(d.pairs[k]);
            const int bi = pr >> 16, bj = pr & 0xFFFF;
            const int t0 = d.tripStart[2 * k], tn = d.tripStart[2 * k + 1];
            for (int m = lane; m < tn; m += 64) {
                const int2 tr = d.trips[t0 + m];
                sp_product(d, acc, tr.x, tr.y, 0, false);
            }
            sp_wave_reduce(acc, lane);   // lane v: value v
            if (lane < 36) {
                const int r = lane / 6, qq = lane % 6;
                const double val = 0.0 - acc[0];
                d.S[(size_t)(6 * bi + r) * n + 6 * bj + qq] = val;
                d.S[(size_t)(6 * bj + qq) * n + 6 * bi + r] = val;
            }
            continue;
        }
        const int k = d.pairUnits[un];
        if (k >= np) continue;
        const int pr = __builtin_amdgcn_readfirstlane(d.pairs[k]);
        const int bi = pr >> 16, bj = pr & 0xFFFF;
        const bool diag = bi == bj;
        if (diag) {   // every edge of pose i pairs with itself: already a dense list
            const int a0 = d.poStart[bi], a1 = d.poStart[bi + 1];
            for (int a = a0 + tid; a < a1; a += kSpT) sp_product(d, acc, a, d.poAct[a], d.poPt[a], true);
        } else {
            // off-diagonal: the pair's shared landmarks, listed once per solve by k_pair_trip
            const int t0 = d.tripStart[2 * k], tn = d.tripStart[2 * k + 1];
            for (int m = tid; m < tn; m += kSpT) {
                const int2 tr = d.trips[t0 + m];
                sp_product(d, acc, tr.x, tr.y, 0, false);
            }
        }
        sp_wave_reduce(acc, lane);
        wsum[wave][lane] = acc[0];   // value v = lane
        __syncthreads();
        const int v = lane, nv = diag ? 42 : 36;
        double sum = 0.0;
        if (wave == 0) {
#pragma unroll
            for (int w = 0; w < kSpW; w++) sum += wsum[w][v];
        }
        __syncthreads();   // wsum is rewritten by the next pair
        // a diagonal block's product (Hpl D^-1) Hpl^T is not bitwise symmetric: only its upper
        // triangle (r <= qq) is stored, mirrored, as g2o fills S from the upper blocks
        if (wave == 0 && v < nv && !(diag && v < 36 && v / 6 > v % 6)) {
            if (v < 36) {
                const int r = v / 6, qq = v % 6;
                double val = 0.0;
                if (diag && addDiag) {
                    val = d.Hpp[36 * (size_t)bi + v];
                    if (r == qq) val += d.lm->lambda;
                }
                val -= sum;
                d.S[(size_t)(6 * bi + r) * n + 6 * bj + qq] = val;
                d.S[(size_t)(6 * bj + qq) * n + 6 * bi + r] = val;
            } else {
                d.bs[6 * bi + v - 36] = (addDiag ? d.bp[6 * bi + v - 36] : 0.0) - sum;
            }
        }
    }
}

// The pose-pair blocks of S that receive a Schur term (G/core/block_solver.hpp:192-207 builds
// the same set as the sparsity pattern of the reduced matrix): per landmark, every pair of its
// free-pose edges marks block (i, j), i <= j, row-major upper-triangle index; all == 1 marks every
// block (with a communicator a block may get its terms on another rank only).
// (the per-pair landmark counts go through an LDS histogram when the pair table fits: a few
// hundred global counters hit by every landmark serialise on their atomics)
// (dynamic LDS of np2 counters up to kPairHist: 144 KB, 268 poses; 200 KF's 20,100 pairs through
// global atomics took 270 us per solve)
constexpr int kPairHist = 36864;
__global__ __launch_bounds__(256) void k_pair_mark(LbaDev d, int32_t* __restrict__ flag, int32_t* __restrict__ cnt,
                                                   int all) {
    extern __shared__ int32_t hist[];
    const int P = d.P, np2 = P * (P + 1) / 2;
    const bool lds = np2 <= kPairHist;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (lds) {
        for (int i = threadIdx.x; i < np2; i += 256) hist[i] = 0;
        __syncthreads();
    }
    if (all && t < np2) flag[t] = 1;
    if (t < P) flag[t * P - t * (t - 1) / 2] = 1;   // every diagonal block (Hpp + lambda I)
    if (t < d.M) {
        const int a0 = d.ptStart[t], a1 = d.ptStart[t + 1];
        for (int a = a0; a < a1; a++) {
            const int pa = d.actPi[d.ptAct[a]];
            if (pa < 0) continue;
            for (int b = a + 1; b < a1; b++) {
                const int pb = d.actPi[d.ptAct[b]];
                if (pb < 0 || pb == pa) continue;
                const int i = min(pa, pb), j = max(pa, pb), k = i * P - i * (i - 1) / 2 + (j - i);
                flag[k] = 1;
                if (lds) atomicAdd(&hist[k], 1);   // this landmark is one of the pair's shared ones
                else atomicAdd(&cnt[k], 1);
            }
        }
    }
    if (lds) {
        __syncthreads();
        for (int i = threadIdx.x; i < np2; i += 256)
            if (hist[i]) atomicAdd(&cnt[i], hist[i]);
    }
}
// the marked blocks compacted in index order (one workgroup): pairs[k] = bi << 16 | bj, *npairs
// ... and, per listed pair, where its shared-landmark list starts (tripStart[2k]) and its length
// ([2k + 1]) in the trips buffer k_pair_trip fills (offsets in list order); k_schur_pairs' work
// units: units[0 .. npairs[1]) the pairs a workgroup takes (diagonal, or more than `small` shared
// landmarks), then the npairs[2] pairs a wave takes, each in list order
__global__ __launch_bounds__(1024) void k_pair_list(const int32_t* __restrict__ flag, const int32_t* __restrict__ cnt,
                                                    int P, int32_t* __restrict__ pairs, int32_t* __restrict__ npairs,
                                                    int32_t* __restrict__ tripStart, int32_t* __restrict__ units,
                                                    int small) {
    __shared__ int wsum[16], tsum[16], bsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = P * (P + 1) / 2;
    const int chunk = (N + 1023) / 1024, c0 = min(tid * chunk, N), c1 = min(c0 + chunk, N);
    int bi0 = 0, bj0 = 0;
    if (c0 < c1) {   // index -> (bi, bj) of the first entry, then walk
        int rem = c0;
        while (rem >= P - bi0) { rem -= P - bi0; bi0++; }
        bj0 = bi0 + rem;
    }
    int loc = 0, tloc = 0, bloc = 0;
    {
        int bi = bi0, bj = bj0;
        for (int i = c0; i < c1; i++) {
            if (flag[i]) {
                loc++;
                tloc += cnt[i];
                bloc += (bi == bj || cnt[i] > small) ? 1 : 0;
            }
            if (++bj == P) { bi++; bj = bi; }
        }
    }
    const int incl = wave_incl_scan_i32(loc), tincl = wave_incl_scan_i32(tloc), bincl = wave_incl_scan_i32(bloc);
    if (lane == 63) { wsum[wave] = incl; tsum[wave] = tincl; bsum[wave] = bincl; }
    __syncthreads();
    int run = incl - loc, trun = tincl - tloc, brun = bincl - bloc, nBig = 0;
    for (int w = 0; w < 16; w++) {
        if (w < wave) { run += wsum[w]; trun += tsum[w]; brun += bsum[w]; }
        nBig += bsum[w];
    }
    int srun = nBig + (run - brun);   // the wave pairs follow the workgroup pairs
    if (c0 < c1) {
        int bi = bi0, bj = bj0;
        for (int i = c0; i < c1; i++) {
            if (flag[i]) {
                tripStart[2 * run] = trun;
                tripStart[2 * run + 1] = cnt[i];
                trun += cnt[i];
                if (bi == bj || cnt[i] > small) units[brun++] = run;
                else units[srun++] = run;
                pairs[run++] = (bi << 16) | bj;
            }
            if (++bj == P) { bi++; bj = bi; }
        }
    }
    if (tid == 1023) {
        npairs[0] = run;
        npairs[1] = nBig;
        npairs[2] = run - nBig;
    }
}

// the inverse of the pose-major lists: poPos[poAct[a]] = a
__global__ __launch_bounds__(256) void k_po_pos(LbaDev d, int32_t* __restrict__ poPos) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a < d.poStart[d.P]) poPos[d.poAct[a]] = a;
}

// Once per solve (the block structure is fixed for both optimize() rounds): every off-diagonal
// pair's shared landmarks as (pose i's edge's pose-major position, pose j's edge's act position) in pose i's
// landmark order.  Four edges of pose i per thread are looked up in pose j's sorted landmark list (LDS up
// to kSpList entries) and the matches compacted in thread order (a workgroup scan).
__global__ __launch_bounds__(kSpT) void k_pair_trip(LbaDev d, int2* __restrict__ trips) {
    if ((int)blockIdx.x >= *d.npairs) return;
    const int pr = d.pairs[blockIdx.x];
    const int bi = pr >> 16, bj = pr & 0xFFFF;
    if (bi == bj) return;
    __shared__ int32_t listJ[kSpList];
    __shared__ int wtot[kSpT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int a0 = d.poStart[bi], a1 = d.poStart[bi + 1], b0 = d.poStart[bj], nb = d.poStart[bj + 1] - b0;
    const bool inLds = nb <= kSpList;
    if (inLds)
        for (int t = tid; t < nb; t += kSpT) listJ[t] = d.poPt[b0 + t];
    __syncthreads();
    const int32_t* Lj = inLds ? listJ : d.poPt + b0;
    int2* out = trips + d.tripStart[2 * blockIdx.x];
    int written = 0;
    for (int base = a0; base < a1; base += kSpChunk) {
        int m1[kSpChunk / kSpT], m2[kSpChunk / kSpT], lm[kSpChunk / kSpT];
#pragma unroll
        for (int u = 0; u < kSpChunk / kSpT; u++) {
            const int a = min(base + tid + kSpT * u, a1 - 1);   // clamped: unconditional loads
            m1[u] = a;
            const int lv = d.poPt[a];
            lm[u] = base + tid + kSpT * u < a1 ? lv : -1;
        }
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < kSpChunk / kSpT; u++) {
            const int l = lm[u];
            int lo = 0, hi = nb;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (Lj[mid] < l) lo = mid + 1;
                else hi = mid;
            }
            const bool hit = l >= 0 && lo < nb && Lj[lo] == l;
            m2[u] = hit ? d.poAct[b0 + lo] : -1;   // (pose j's edge by act position: Hpl_e in place)
            cnt += hit ? 1 : 0;
        }
        const int incl = wave_incl_scan_i32(cnt);
        if (lane == 63) wtot[wave] = incl;
        __syncthreads();
        int off = written + incl - cnt, total = 0;
#pragma unroll
        for (int w = 0; w < kSpT / 64; w++) {
            off += w < wave ? wtot[w] : 0;
            total += wtot[w];
        }
#pragma unroll
        for (int u = 0; u < kSpChunk / kSpT; u++)
            if (m2[u] >= 0) out[off++] = make_int2(m1[u], m2[u]);
        written += total;
        __syncthreads();   // wtot is rewritten by the next chunk
    }
    if (tid == 0) const_cast<int32_t*>(d.tripStart)[2 * blockIdx.x + 1] = written;   // the listed length
}

// ---- The Schur complement as a dense f64 MFMA GEMM (A/B against k_schur_pairs; ORB_LBA_SCHUR_MFMA=1,
// reduced systems in the LDS image).  SURVEY 8d's densified form of G/core/block_solver.hpp:382-433:
// S = Hpp + lambda I - Y Y^T with Y = W L^-T, W the 6P x 3M matrix of the Hpl blocks and D_l = L L^T
// the landmark's Cholesky factor (W D^-1 W^T = (W L^-T)(W L^-T)^T).  Y^T is built k-major
// (k_schur_ymat), split over chunks of kYLm landmarks (48 k) each workgroup of k_schur_gemm multiplies
// its chunk into all upper 16 x 16 tiles of S with v_mfma_f64_16x16x4 (partials in HBM), and
// k_schur_msum adds the chunks in a fixed order (bitwise reproducible) with Hpp + lambda I and b_s.
// Y is dense: a landmark's 3 columns are non-zero only in its observers' 6-row blocks, so the MFMA
// units execute ~P / k_mean times the algorithmic flops (the measurement this mode exists for).
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kYLm = 16;   // landmarks per GEMM chunk
constexpr int kYLmB = 8;   // landmarks per k_schur_ymat workgroup

__global__ __launch_bounds__(256) void k_schur_ymat(LbaDev d, double* __restrict__ Yt, int np, double* __restrict__ ce) {
    if (d.lm->phase != 1) return;
    __shared__ double tile[3 * kYLmB][128];
    const int tid = threadIdx.x;
    for (int i = tid; i < 3 * kYLmB * 128; i += 256) (&tile[0][0])[i] = 0.0;
    __syncthreads();
    const int l = blockIdx.x * kYLmB + tid;
    if (tid < kYLmB && l < d.M) {
        const double lambda = d.lm->lambda;
        double D[9];
        for (int i = 0; i < 9; i++) D[i] = d.Hll[9 * (size_t)l + i];
        D[0] += lambda; D[4] += lambda; D[8] += lambda;
        // D = L L^T; Li = L^-1 (lower)
        const double l00 = sqrt(D[0]), l10 = D[3] / l00, l20 = D[6] / l00;
        const double l11 = sqrt(D[4] - l10 * l10), l21 = (D[7] - l20 * l10) / l11;
        const double l22 = sqrt(D[8] - l20 * l20 - l21 * l21);
        const double m00 = 1.0 / l00, m11 = 1.0 / l11, m22 = 1.0 / l22;
        const double m10 = -l10 * m00 * m11, m21 = -l21 * m11 * m22, m20 = -(l20 * m00 + l21 * m10) * m22;
        const double Li[9] = {m00, 0.0, 0.0, m10, m11, 0.0, m20, m21, m22};
        const double* db = d.db + 3 * (size_t)l;
        for (int a = d.ptStart[l]; a < d.ptStart[l + 1]; a++) {
            const int k = d.ptAct[a];
            const int pi = d.actPi[k];
            if (pi < 0) continue;
            const double* W = d.Hpl_e + 18 * (size_t)k;
            for (int r = 0; r < 6; r++) {
                for (int q = 0; q < 3; q++) {   // Y_e = W L^-T: (W L^-T)[r][q] = sum_m W[r][m] Li[q][m]
                    double y = 0.0;
                    for (int m = 0; m <= q; m++) y += W[r * 3 + m] * Li[q * 3 + m];
                    tile[3 * tid + q][6 * pi + r] = y;
                }
                ce[6 * (size_t)k + r] = W[r * 3] * db[0] + W[r * 3 + 1] * db[1] + W[r * 3 + 2] * db[2];
            }
        }
    }
    __syncthreads();
    const int nl = min(kYLmB, d.M - (int)blockIdx.x * kYLmB);
    for (int i = tid; i < 3 * nl * np; i += 256) {
        const int c = i / np, r = i % np;
        Yt[((size_t)blockIdx.x * 3 * kYLmB + c) * np + r] = tile[c][r];
    }
}

// workgroup w: chunks w * kYLmG .. w * kYLmG + kYLmG - 1 (kYLm landmarks = 48 rows of Y^T each) into
// every upper tile (I <= K) of Y Y^T, 12 MFMAs per tile and chunk; wave v keeps the accumulators
// of tiles v, v + 4, ... (up to kGemmTiles per wave) in registers across the chunks, so the
// partial sums k_schur_msum adds are one set per workgroup
constexpr int kYLmG = 1;         // chunks per k_schur_gemm workgroup (4: 47 workgroups, 49 us; 1: 188)
constexpr int kGemmTiles = 9;    // upper tiles per wave: T (T + 1) / 2 <= 36 at np <= 128
__global__ __launch_bounds__(256) void k_schur_gemm(LbaDev d, const double* __restrict__ Yt, int np,
                                                    double* __restrict__ part) {
    if (d.lm->phase != 1) return;
    __shared__ double ys[3 * kYLm][128];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = np / 16, nt = T * (T + 1) / 2;
    const int li = lane & 15, lk = lane >> 4;
    int tI[kGemmTiles], tK[kGemmTiles];
#pragma unroll
    for (int j = 0; j < kGemmTiles; j++) {
        int ti = 0, rem = min(wave + 4 * j, nt - 1);   // row-major upper triangle: (ti, tk), ti <= tk
        while (rem >= T - ti) { rem -= T - ti; ti++; }
        tI[j] = ti;
        tK[j] = ti + rem;
    }
    dbl4 acc[kGemmTiles];
#pragma unroll
    for (int j = 0; j < kGemmTiles; j++) acc[j] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int g = 0; g < kYLmG; g++) {
        const int ch = blockIdx.x * kYLmG + g;
        const int kr = min(3 * kYLm, 3 * d.M - ch * 3 * kYLm);   // rows of Y^T in this chunk
        if (kr <= 0) break;
        __syncthreads();
        for (int i = tid; i < 3 * kYLm * np; i += 256) {
            const int r = i / np, c = i % np;
            ys[r][c] = r < kr ? Yt[((size_t)ch * 3 * kYLm + r) * np + c] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kGemmTiles; j++) {
            if (wave + 4 * j >= nt) break;
#pragma unroll
            for (int s = 0; s < 3 * kYLm / 4; s++) {
                const double a = ys[4 * s + lk][16 * tI[j] + li], b = ys[4 * s + lk][16 * tK[j] + li];
                acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kGemmTiles; j++) {
        const int t = wave + 4 * j;
        if (t >= nt) break;
        double* o = part + ((size_t)blockIdx.x * nt + t) * 256;
#pragma unroll
        for (int q = 0; q < 4; q++) o[(lk + 4 * q) * 16 + li] = acc[j][q];
    }
}

// S (upper, mirrored) = [root] Hpp + lambda I - sum over chunks (chunk order), b_s = [root] b_p - the
// edges' Hpl D^-1 b_l (pose's edges in list order)
__global__ __launch_bounds__(256) void k_schur_msum(LbaDev d, const double* __restrict__ part, int nchunks, int np,
                                                    const double* __restrict__ ce, int addDiag) {
    if (d.lm->phase != 1) return;
    const int T = np / 16, nt = T * (T + 1) / 2, n = 6 * d.P;
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g < nt * 256) {
        const int t = g >> 8, e = g & 255;
        int ti = 0, rem = t;
        while (rem >= T - ti) { rem -= T - ti; ti++; }
        const int tk = ti + rem;
        const int R = 16 * ti + (e >> 4), Cc = 16 * tk + (e & 15);
        if (R < n && Cc < n && R <= Cc) {
            double v = 0.0;
#pragma unroll 8
            for (int c = 0; c < nchunks; c++) v += part[((size_t)c * nt + t) * 256 + e];
            double val = 0.0;
            if (addDiag && R / 6 == Cc / 6) {
                val = d.Hpp[36 * (size_t)(R / 6) + (R % 6) * 6 + Cc % 6];
                if (R == Cc) val += d.lm->lambda;
            }
            val -= v;
            d.S[(size_t)R * n + Cc] = val;
            d.S[(size_t)Cc * n + R] = val;
        }
    } else {
        // b_s: one wave per pose (the tile part fills whole workgroups), lanes strided over the
        // pose's edges, then a fixed-order wave reduction
        const int p = (g - nt * 256) >> 6, lane = threadIdx.x & 63;
        if (p >= d.P) return;
        double v[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int a = d.poStart[p] + lane; a < d.poStart[p + 1]; a += 64) {
            const double* c = ce + 6 * (size_t)d.poAct[a];
#pragma unroll
            for (int r = 0; r < 6; r++) v[r] += c[r];
        }
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const double t = wave_sum_d(v[r]);
            if (lane == r) d.bs[6 * p + r] = (addDiag ? d.bp[6 * p + r] : 0.0) - t;
        }
    }
}

// Broadcast of lane `src` (a compile-time constant at every call site) through two
// v_readlane_b32 into SGPRs: a few cycles, against a ds_bpermute round trip for __shfl.
__device__ __forceinline__ double shfl_d(double v, int src) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the same with a wave-uniform lane index held in an SGPR
__device__ __forceinline__ double shfl_d_dyn(double v, int src) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ------------------------------------------------------------------ reduced camera solve
// Dense LDL^T of S (no pivoting; fails only on a zero or non-finite pivot, like
// SimplicialLDLT, G/solvers/linear_solver_eigen.h:94-120) + both triangular solves, one
// workgroup of kLdlT threads.  Blocked right-looking in 16-column panels (one f64 MFMA tile
// edge).  The matrix is padded to np = 16 * ceil(n / 16) with the identity and held in LDS
// when it fits (np <= 128, i.e. up to 21 free keyframes), otherwise in a global scratch
// (L2-resident).  W(i,j) = A(i,j) before the scaling by 1/d_j is kept in the upper triangle
// at (j, i), L(i,j) = W(i,j) / d_j in the lower.  Per panel [jb, jb+16):
//  1. wave 0 factors the panel with its rows (up to 192, three per lane) in registers: pivots
//     and L entries broadcast with v_readlane, 1/d_j by v_rcp_f64 + two Newton steps, the
//     forward substitution folded in; rows beyond 192 (large systems) follow one per thread;
//  2. trailing lower triangle: A(I, K) -= W(I, panel) L(K, panel)^T per 16 x 16 tile with four
//     v_mfma_f64_16x16x4_f64 (tiles dealt round-robin to the 8 waves).
// Then y /= d and the backward substitution with L^T on one wave in 16-row blocks.  The
// oracle (oracle/lba_oracle.c) runs the unblocked column recurrence with IEEE divisions; the
// two agree to rounding (tests compare the LM traces to 1e-9 relative).
constexpr int kNB = 16;
constexpr int kLdlT = 512;
constexpr int kLdlLdsMaxN = 128;   // padded order held in LDS: (128 * 129 + 3 * 128 + 256 + 16 * 129 + 64) * 8 B = 151 KB

__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}

// Panel [jb, jb+16) on wave 0 for rows jb + lane + 64u, u < NS (rows >= np are skipped):
// column j = jb + c: d_j = A(j, j) (lane c, slot 0), W(i, j) = A(i, j) goes to the upper
// triangle at (j, i), L(i, j) = W(i, j) / d_j to the lower, the panel's later columns take
// A(i, k) = fma(-L(i, j), W(k, j), A(i, k)), and the forward substitution advances with the
// factorisation (y_i = fma(-L(i, j), y_j, y_i) once y_j is final).  W(jb+k, j) reaches the
// other lanes by v_readlane for k = c+1 (the next pivot's column) and as a broadcast LDS read
// of the row just stored for k > c+1.  Branch-free: a zero or non-finite pivot only clears
// the returned flag; stores a lane must not make go to its `dummy` slot.
template <int NS>
__device__ __forceinline__ bool ldlt_panel(double* __restrict__ A, int ld, int np, int jb, double* __restrict__ dg,
                                           double* __restrict__ rdg, double* __restrict__ y, double* dummy,
                                           int lane) {
    double P[NS][kNB], Y[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) {   // rows past np read row np-1 (never stored): no exec-masked loads
        const int r = min(jb + lane + 64 * u, np - 1);
        Y[u] = y[r];
#pragma unroll
        for (int c = 0; c < kNB; c++) P[u][c] = A[(size_t)r * ld + jb + c];
    }
    // Software-pipelined by one column: column c's updates of columns k > c+1 are issued
    // between the steps of the next pivot's reciprocal (the dependent chain
    // readlane -> v_rcp_f64 -> Newton -> scale -> column c+1 update -> readlane), so the
    // in-order wave has independent work while the chain's results are in flight.
    double dj = shfl_d(P[0][0], 0);
    bool ok = dj != 0.0 && isfinite(dj);
    double rd = rcp_nr(dj);
#pragma unroll
    for (int c = 0; c < kNB; c++) {
        const int j = jb + c;
        const double yj = shfl_d(Y[0], c);   // final: every k < j has been applied
        double w[NS], l[NS];
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int r = jb + lane + 64 * u;
            w[u] = P[u][c];
            l[u] = w[u] * rd;
            P[u][c] = l[u];
            const bool st = r < np && lane + 64 * u > c;
            *(st ? A + (size_t)j * ld + r : dummy + lane) = w[u];   // W(r, j)
            *(st ? A + (size_t)r * ld + j : dummy + lane) = l[u];   // L(r, j)
        }
        // (lane 0 stores d_j, 1/d_j; the others write their sink: no branch in the column loop,
        // which keeps it one basic block for the scheduler)
        *(lane == 0 ? dg + j : dummy + lane) = dj;
        *(lane == 0 ? rdg + j : dummy + lane) = rd;
        double wk[kNB];
        const double* Wrow = A + (size_t)j * ld + jb;
#pragma unroll
        for (int k = c + 2; k < kNB; k++) wk[k] = Wrow[k];   // W(jb+k, j): broadcast LDS reads
        double djn = 1.0, r0 = 1.0, e0 = 0.0, r1 = 1.0, e1 = 0.0;
        if (c + 1 < kNB) {   // next pivot: column c+1 first
            const double w1 = shfl_d(w[0], c + 1);   // W(j+1, j)
#pragma unroll
            for (int u = 0; u < NS; u++) P[u][c + 1] = __builtin_fma(-l[u], w1, P[u][c + 1]);
            djn = shfl_d(P[0][c + 1], c + 1);
            r0 = __builtin_amdgcn_rcp(djn);
        }
        // sched_barrier: without it the scheduler sinks every update to just before its column
        // becomes the pivot, turning the right-looking step into a dependent fma chain there
        __builtin_amdgcn_sched_barrier(0);
        // the deferred updates, in three groups between the reciprocal's steps
        const int nk = kNB - 2 - c > 0 ? kNB - 2 - c : 0;   // folded: the loop is unrolled
        const int g1 = c + 2 + (nk + 2) / 3, g2 = c + 2 + 2 * (nk + 2) / 3;
#pragma unroll
        for (int k = c + 2; k < kNB && k < g1; k++)
#pragma unroll
            for (int u = 0; u < NS; u++) P[u][k] = __builtin_fma(-l[u], wk[k], P[u][k]);
        if (c + 1 < kNB) { e0 = __builtin_fma(-djn, r0, 1.0); r1 = __builtin_fma(r0, e0, r0); }
#pragma unroll
        for (int u = 0; u < NS; u++)
            if (lane + 64 * u > c) Y[u] = __builtin_fma(-l[u], yj, Y[u]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = g1; k < kNB && k < g2; k++)
#pragma unroll
            for (int u = 0; u < NS; u++) P[u][k] = __builtin_fma(-l[u], wk[k], P[u][k]);
        if (c + 1 < kNB) { e1 = __builtin_fma(-djn, r1, 1.0); r1 = __builtin_fma(r1, e1, r1); }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = g2; k < kNB; k++)
#pragma unroll
            for (int u = 0; u < NS; u++) P[u][k] = __builtin_fma(-l[u], wk[k], P[u][k]);
        __builtin_amdgcn_sched_barrier(0);
        if (c + 1 < kNB) {
            ok = ok && djn != 0.0 && isfinite(djn);
            dj = djn;
            rd = r1;
        }
    }
#pragma unroll
    for (int u = 0; u < NS; u++) {
        const int r = jb + lane + 64 * u;
        if (r < np) y[r] = Y[u];
    }
    return ok;
}

// The LDS-image panel split over waves: group g (wave g) holds the panel's 16 diagonal rows in
// lanes 0..15 and rows jb + 16 + 48 g + (lane - 16) in lanes 16..63, so every group computes
// the pivots, 1/d_j and W(jb+k, j) itself and no wave waits on another inside the column loop.
// The diagonal rows are computed identically by every group (same operations in the same
// order); group 0 alone stores them and 1/d.  Groups only write rows they own, after every
// group has read its inputs (arrival counter `arrive`, group 0 waits for `target`).
// Column j = jb + c: W(r, j) = A(r, j) goes to the upper triangle at (j, r), L(r, j) = W(r, j) / d_j
// to the lower, and the later columns take A(r, k) = fma(-L(r, j), W(jb+k, j), A(r, k)), k > c,
// in column order.  W(jb+k, j) reaches the lanes by v_readlane for k = c+1, c+2 (applied at
// once: the next two pivots depend on them) and through the group's 16-double LDS row `wsc` for
// k > c+2, read at column c and applied at the start of column c+1, so the LDS round trip
// overlaps a column of work.  The pivot chain is one multiply-add per column: the next pivot
//   d_{j+1} = A(j+1, j+1) - W(j+1, j)^2 / d_j = fma(-W(j+1, j)^2, 1/d_j, A(j+1, j+1))
// takes A(j+1, j+1) and W(j+1, j) by v_readlane (final before column j), then v_rcp_f64 and two
// Newton steps.  (Lane j+1's own A(j+1, j+1) rounds differently; it is never used: 1/d is the
// broadcast value.)  Stores are unconditional at loop-invariant bases: the rows below the
// diagonal block write their W and L in place, the diagonal lanes and rows past np write into
// the `shadow` sink (kNB * ld + 64 doubles); group 0's diagonal lanes store their L row and 1/d
// after the loop (the diagonal block's W, its upper triangle, is never read again).  A zero or
// non-finite pivot only clears the returned flag.
template <bool kTail>
__device__ __forceinline__ bool ldlt_panel_grp(double* __restrict__ A, int ld, int np, int nr, int jb,
                                               double* __restrict__ rdg, double* __restrict__ y,
                                               double* __restrict__ shadow, double* __restrict__ wsc, int lane,
                                               int g, int* arrive, int target) {
    const int r = lane < kNB ? jb + lane : jb + kNB + 48 * g + (lane - kNB);
    const bool live = r < np, inplace = live && lane >= kNB;
    const int rc = min(r, np - 1);
    double P[kNB];
    double Y = y[rc];
#pragma unroll
    for (int c = 0; c < kNB; c++) P[c] = A[(size_t)rc * ld + jb + c];
    // inputs read (this wave's LDS operations complete in order): arrive; group 0 then waits
    // for every group before its first store
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (g == 0)
        while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double* const Lrow = inplace ? A + (size_t)r * ld + jb : shadow + (size_t)(lane & (kNB - 1)) * ld;
    double* const Wcol = inplace ? A + (size_t)jb * ld + r : shadow + lane;
    double* const wst = lane < kNB ? wsc + lane : shadow + lane;
    double dj = shfl_d(P[0], 0);
    bool ok = dj != 0.0 && isfinite(dj);
    double rd = rcp_nr(dj);
    double myrd = 1.0;             // lane c keeps 1/d_{jb+c} (padding: 1)
    double Wd[kNB], lprev = 0.0;   // column c-1's deferred W(jb+k, j-1), k > c+1, and L(r, j-1)
#pragma unroll
    for (int c = 0; c < kNB; c++) {
        const int j = jb + c;
        // the identity padding's columns (j >= nr, last panel only: kTail) stay as staged: their W
        // and L entries are zero, 1/d = 1 (set with the staging), so the chain stops at the
        // order.  (A full panel has no exit: a loop exit is a block boundary where the deferred
        // LDS reads would be waited for.)
        if (kTail && j >= nr) break;
        const double w = P[c];   // final: column c-1 applied its update of column c at once
        double djn = 1.0, rn = 1.0, w1 = 0.0, w2 = 0.0;
        if (c + 1 < kNB) {   // the chain: W(j+1, j) and A(j+1, j+1) are final
            w1 = shfl_d(w, c + 1);
            const double a1 = shfl_d(P[c + 1], c + 1);
            djn = __builtin_fma(-(w1 * w1), rd, a1);
            rn = __builtin_amdgcn_rcp(djn);
        }
        if (c + 2 < kNB) w2 = shfl_d(w, c + 2);
        const double yj = shfl_d(Y, c);   // final: every k < j has been applied
        __builtin_amdgcn_sched_barrier(0);
        // column c-1's deferred updates (its LDS reads were issued a column ago)
        if (c >= 1) {
#pragma unroll
            for (int k = c + 2; k < kNB; k++) P[k] = __builtin_fma(-lprev, Wd[k], P[k]);
        }
        const double l = w * rd;
        P[c] = l;
        Wcol[(size_t)c * ld] = w;   // W(r, j)
        Lrow[c] = l;                // L(r, j)
        myrd = lane == c ? rd : myrd;
        *wst = w;                   // the diagonal block's W(jb+k, j)
#pragma unroll
        for (int k = c + 3; k < kNB; k++) Wd[k] = wsc[k];     // consumed at column c+1
        if (c + 1 < kNB) P[c + 1] = __builtin_fma(-l, w1, P[c + 1]);
        if (c + 2 < kNB) P[c + 2] = __builtin_fma(-l, w2, P[c + 2]);
        if (r > j) Y = __builtin_fma(-l, yj, Y);
        lprev = l;
        if (c + 1 < kNB) {
            const double e0 = __builtin_fma(-djn, rn, 1.0);
            const double r1 = __builtin_fma(rn, e0, rn);
            ok = ok && djn != 0.0 && isfinite(djn);
            dj = djn;
            // (one Newton step instead of two measured the same: 1.40 vs 1.41 ms per solve)
            const double e1 = __builtin_fma(-djn, r1, 1.0);
            rd = __builtin_fma(r1, e1, r1);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g == 0 && lane < kNB) {   // the diagonal block's L row (entries past the diagonal: unread)
        double* const Ld = A + (size_t)r * ld + jb;
#pragma unroll
        for (int c = 0; c < kNB; c++) Ld[c] = P[c];
        rdg[r] = myrd;
    }
    if (live && (g == 0 || lane >= kNB)) y[r] = Y;
    return ok;
}
// groups for the panel at jb: the 16 diagonal rows plus 48 rows below per group
__host__ __device__ __forceinline__ int panel_groups(int np, int jb) {
    const int g = (np - jb - kNB + 47) / 48;
    return g > 1 ? g : 1;
}

// rows of a panel factored in registers: all of them with the LDS image (ldlt_panel_grp), 192
// (three per lane of wave 0) with the global image, the rest one per thread (step 1b)
constexpr int kPanelRowsLds = 128, kPanelRowsGlobal = 192;

// The free poses' update after the reduced solve (the pose block of the back-substitution,
// G/core/block_solver.hpp:462-484, sparse_optimizer.cpp:422-435): push() of T and
// T <- exp(x_p) T, and the poses' share of x^T (lambda x + b) into *scaleOut.  Fused slots run it
// on wave 0 of k_ldlt_solve, so the landmark blocks of k_backsub_errors see the new poses.
struct PoseTail {
    double *q, *t, *bq, *bt, *scaleOut;
    const double* bp;
    const int32_t *freePoses, *poseIdx;
    int P;
};
__device__ __forceinline__ void pose_tail(const PoseTail& pt, const double* xs, double lambda, int lane) {
    double sc = 0.0;
    for (int i = lane; i < pt.P; i += 64) {
        const int p = pt.freePoses[i];
        const int k = pt.poseIdx[p];
        double q[4], t[3], u[6];
        for (int j = 0; j < 4; j++) { q[j] = pt.q[4 * p + j]; pt.bq[4 * p + j] = q[j]; }
        for (int j = 0; j < 3; j++) { t[j] = pt.t[3 * p + j]; pt.bt[3 * p + j] = t[j]; }
        for (int j = 0; j < 6; j++) {
            u[j] = xs[6 * k + j];
            sc += u[j] * (lambda * u[j] + pt.bp[6 * k + j]);
        }
        d_se3_exp_left(u, q, t);
        for (int j = 0; j < 4; j++) pt.q[4 * p + j] = q[j];
        for (int j = 0; j < 3; j++) pt.t[3 * p + j] = t[j];
    }
    sc = wave_sum_d(sc);
    if (lane == 0) *pt.scaleOut = sc;
}

// pose_tail for at most 64 free poses in two halves: the inputs that do not depend on x (pose,
// b_p, indices) loaded before the backward substitution, so their latency hides under it
struct PoseTailPre {
    double q[4], t[3], bp[6];
    int k;
};
__device__ __forceinline__ void pose_tail_prefetch(const PoseTail& pt, int lane, PoseTailPre& f) {
    const int i = min(lane, max(pt.P - 1, 0));
    const int p = pt.freePoses[i];
    f.k = pt.poseIdx[p];
    for (int j = 0; j < 4; j++) f.q[j] = pt.q[4 * p + j];
    for (int j = 0; j < 3; j++) f.t[j] = pt.t[3 * p + j];
    for (int j = 0; j < 6; j++) f.bp[j] = pt.bp[6 * f.k + j];
}
__device__ __forceinline__ void pose_tail_finish(const PoseTail& pt, const double* xs, double lambda, int lane,
                                                 PoseTailPre& f) {
    double sc = 0.0;
    if (lane < pt.P) {
        const int p = pt.freePoses[lane];
        for (int j = 0; j < 4; j++) pt.bq[4 * p + j] = f.q[j];
        for (int j = 0; j < 3; j++) pt.bt[3 * p + j] = f.t[j];
        double u[6];
        for (int j = 0; j < 6; j++) {
            u[j] = xs[6 * f.k + j];
            sc += u[j] * (lambda * u[j] + f.bp[j]);
        }
        d_se3_exp_left(u, f.q, f.t);
        for (int j = 0; j < 4; j++) pt.q[4 * p + j] = f.q[j];
        for (int j = 0; j < 3; j++) pt.t[3 * p + j] = f.t[j];
    }
    sc = wave_sum_d(sc);
    if (lane == 0) *pt.scaleOut = sc;
}

template <bool kLds>
__global__ __launch_bounds__(kLdlT) void k_ldlt_solve(const double* __restrict__ Sg, const double* __restrict__ b,
                                                      int n, double* __restrict__ work, double* __restrict__ x,
                                                      int* __restrict__ flags, const LmState* st, PoseTail ptail) {
    if (lm_off(st, 1)) return;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    TSTAMP(t_l0);
    long long tDiag = 0, tRows = 0, tTrail = 0;
    (void)tDiag; (void)tRows; (void)tTrail;
#ifdef ORB_TIMING
    long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tpb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    const int np = (n + kNB - 1) & ~(kNB - 1);
    const int ld = np + 1;   // odd: column-strided lanes spread over the LDS banks
    constexpr int kPanelRows = kLds ? kPanelRowsLds : kPanelRowsGlobal;
    double* A = kLds ? sh : work;
    double* dg = sh + (kLds ? (size_t)np * ld : 0);
    double* rdg = dg + np;
    double* y = rdg + np;
    // 64 per-lane sinks for masked-off panel stores; with the LDS image the grouped panels' W-row
    // scratch follows (16 doubles per group at dummy + 64), then their store sink
    double* dummy = y + np;
    double* shadow = dummy + 256;   // LDS image: the grouped panels' store sink (kNB * ld + 64)
    __shared__ int failS, arriveS;
    int arriveTarget = 0;     // the grouped panels' cumulative arrivals (uniform over the workgroup)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- stage S (n x n, row-major, n = 6P even) into the padded np x np image (identity
    //      padding).  In LDS: wave w copies rows w, w + 8, ... with lane c moving the column pair
    //      (2c, 2c+1) by one 16-byte load — every load of the wave in flight at once (one round
    //      trip; out-of-range rows read 0 through the buffer resource).  Global image: 8-byte loads.
    {
        constexpr int kW = kLdlT / 64;
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(Sg, (uint32_t)n * n * 8);
        if (kLds && (n & 1) == 0 && np <= 128) {
            // phase 1 (here, every wave): column block 0 of every row, the padding included —
            // panel 0's input.  The rest of the lower triangle (phase 2) is staged by the waves
            // that do not factor panel 0, while it is factored (below).  Nothing reads S's upper
            // triangle: the diagonal lanes of a panel load theirs but never consume it, the
            // trailing tiles of the diagonal carry it along unread, and the W stores fill the rest
            // before a trailing tile reads it.
            const int col = tid & 15;
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = (tid >> 4) + 32 * u;
                v[u] = buf_ld_f64(rs, i < n && col < n ? (i * n + col) * 8 : kBufOob);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = (tid >> 4) + 32 * u;
                if (i < np) A[(size_t)i * ld + col] = v[u] + ((i >= n || col >= n) && i == col ? 1.0 : 0.0);
            }
        } else {
            for (int j0 = 0; j0 < np; j0 += 64) {
                const int j = j0 + lane;
                for (int i0 = wave; i0 < np; i0 += kW * 16) {
                    double v[16];
#pragma unroll
                    for (int u = 0; u < 16; u++) {   // padding: offset out of range -> 0, plus identity
                        const int i = i0 + kW * u;
                        const bool in = i < n && j < n;
                        v[u] = buf_ld_f64(rs, in ? (i * n + j) * 8 : kBufOob) + ((!in && i == j) ? 1.0 : 0.0);
                    }
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        const int i = i0 + kW * u;
                        if (i < np && j < np) A[(size_t)i * ld + j] = v[u];
                    }
                }
            }
        }
        for (int t = tid; t < np; t += kLdlT) y[t] = t < n ? b[t] : 0.0;
        for (int t = n + tid; t < np; t += kLdlT) dg[t] = rdg[t] = 1.0;   // padding pivots (not factored)
    }
    TSTAMP(t_sa);
    if (tid == 0) { failS = 0; arriveS = 0; }
    __syncthreads();
    TSTAMP(t_f0);
    const int T = np / kNB;
    // One 16 x 16 tile of the trailing update: A(I, K) -= W(I, panel) L(K, panel)^T, four
    // v_mfma_f64_16x16x4_f64 per tile
    auto trail_tile = [&](int jb, int I0, int K0) {
        const int li = lane & 15, lk = lane >> 4;
        double a[kNB / 4], bb[kNB / 4];
        dbl4 acc;
#pragma unroll
        for (int s = 0; s < kNB / 4; s++) {
            const int p = jb + 4 * s + lk;
            a[s] = -A[(size_t)p * ld + I0 + li];   // -W(I0 + li, p): this kernel's panels store +W
            bb[s] = A[(size_t)(K0 + li) * ld + p];      //  L(K0 + li, p)
        }
#pragma unroll
        for (int q = 0; q < 4; q++) acc[q] = A[(size_t)(I0 + lk + 4 * q) * ld + K0 + li];
#pragma unroll
        for (int s = 0; s < kNB / 4; s++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], bb[s], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) A[(size_t)(I0 + lk + 4 * q) * ld + K0 + li] = acc[q];
    };
    auto tri = [](int t, int& ti, int& tk) {   // t -> (ti, tk), tk <= ti, row-major lower triangle
        ti = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
        while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
        while (ti * (ti + 1) / 2 > t) ti--;
        tk = t - ti * (ti + 1) / 2;
    };
    bool factored = false;   // panel kb already factored during the previous step (look-ahead)
    for (int kb = 0; kb < T; kb++) {
        const int jb = kb * kNB;
        TSTAMP(t_d0);
        // ---- 1. panel: rows [jb, jb + 192) in wave 0's registers
        if (kLds && !factored) {
            const int ng = panel_groups(np, jb);
            arriveTarget += ng;
            if (wave < ng) {
                const bool okp = jb + kNB > n ? ldlt_panel_grp<true>(A, ld, np, n, jb, rdg, y, shadow, dummy + 64 + 16 * wave, lane, wave, &arriveS,
                                                arriveTarget)
                                                 : ldlt_panel_grp<false>(A, ld, np, n, jb, rdg, y, shadow, dummy + 64 + 16 * wave, lane, wave, &arriveS,
                                                arriveTarget);
                if (!okp && wave == 0 && lane == 0) failS = 1;
            } else if (kb == 0 && kLds && (n & 1) == 0 && np <= 128) {
                // staging phase 2: rows 16.., column pairs (2c, 2c+1) from column 16 up to the
                // diagonal (identity padding beyond n).  Rows are folded (16 + f with np - 1 - f:
                // together at most 58 pairs, one per lane), so one round of 16-byte loads covers
                // the triangle: every load of a wave in flight at once
                const __amdgpu_buffer_rsrc_t rs = buf_rsrc(Sg, (uint32_t)n * n * 8);
                const int nw = kLdlT / 64 - ng, nf = (np - kNB + 1) >> 1;
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                constexpr int kFold = 12;   // ceil(56 folded row pairs / 5 staging waves) at np = 128
                u32x4 v[kFold];
                int ri[kFold], ci[kFold];
#pragma unroll
                for (int u = 0; u < kFold; u++) {
                    const int f = (wave - ng) + nw * u;
                    const int rA = kNB + f, rB = np - 1 - f, cntA = (rA >> 1) - 7;
                    const bool onA = lane < cntA;
                    int i = onA ? rA : rB;
                    const int c = 8 + (onA ? lane : lane - cntA);
                    if (f >= nf || 2 * c > i || (!onA && rB <= rA)) i = -1;   // no pair for this lane
                    ri[u] = i;
                    ci[u] = c;
                    const bool in = i >= 0 && i < n;
                    v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? (i * n + 2 * c) * 8 : kBufOob, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < kFold; u++) {
                    const int i = ri[u], c = ci[u];
                    if (i >= 0) {
                        double* const dst = A + (size_t)i * ld + 2 * c;
                        dst[0] = __longlong_as_double((long long)(((unsigned long long)v[u].y << 32) | v[u].x)) +
                                 (i >= n && i == 2 * c ? 1.0 : 0.0);
                        dst[1] = __longlong_as_double((long long)(((unsigned long long)v[u].w << 32) | v[u].z)) +
                                 (i >= n && i == 2 * c + 1 ? 1.0 : 0.0);
                    }
                }
            }
        } else if (wave == 0 && !factored) {
            const int ns = min(np - jb, kPanelRows);
            bool okp;
            if (ns <= 64) okp = ldlt_panel<1>(A, ld, jb + ns, jb, dg, rdg, y, dummy, lane);
            else if (kLds || ns <= 128) okp = ldlt_panel<2>(A, ld, jb + ns, jb, dg, rdg, y, dummy, lane);   // LDS: np <= 128
            else okp = ldlt_panel<3>(A, ld, jb + ns, jb, dg, rdg, y, dummy, lane);
            if (!okp && lane == 0) failS = 1;
        }
#ifdef ORB_TIMING
        const long long t_d1 = clock64();
#endif
        __syncthreads();
        TACC(tDiag, t_d0);
#ifdef ORB_TIMING
        if (kb < 8) { tp[kb] = t_d1 - t_d0; tpb[kb] = clock64() - t_d1; }
#endif
        if (failS) break;
        TSTAMP(t_r0);
        // ---- 1b. rows beyond the register panel (large systems only), one thread per row:
        //          W(i, jb+c) = A(i, jb+c) - sum_{k<c} W(i, jb+k) L(jb+c, jb+k)
        if (np - jb > kPanelRows) {
            for (int i = jb + kPanelRows + tid; i < np; i += kLdlT) {
                double w[kNB];
                double Y = y[i];
#pragma unroll
                for (int c = 0; c < kNB; c++) {
                    double v = A[(size_t)i * ld + jb + c];
                    const double* Lc = A + (size_t)(jb + c) * ld + jb;
#pragma unroll
                    for (int k = 0; k < c; k++) v = __builtin_fma(-w[k], Lc[k], v);
                    w[c] = v;
                }
#pragma unroll
                for (int c = 0; c < kNB; c++) {
                    const double l = w[c] * rdg[jb + c];
                    A[(size_t)i * ld + jb + c] = l;
                    A[(size_t)(jb + c) * ld + i] = w[c];
                    Y = __builtin_fma(-l, y[jb + c], Y);
                }
                y[i] = Y;
            }
            __syncthreads();
        }
        TACC(tRows, t_r0);
        TSTAMP(t_t0);
        // ---- 2. trailing lower triangle, 16 x 16 tiles (I >= K > kb) on the MFMA units.
        //         LDS image (np <= 128): look-ahead — the tiles of column block kb+1 first (all
        //         waves), then wave 0 factors panel kb+1 while waves 1..7 update the other tiles
        //         (disjoint addresses; every tile still sees its panel updates in panel order, so
        //         the result is bitwise that of the plain order)
        const int m = T - kb - 1;
        if (kLds && m > 0) {
            for (int ti = wave; ti < m; ti += kLdlT / 64) trail_tile(jb, (kb + 1 + ti) * kNB, (kb + 1) * kNB);
            __syncthreads();
            // (tried: these tiles on the panel waves only, each its own rows, the diagonal one
            // flagged by group 0 — no barrier, but the panel waves' 3-4 tile updates then sit on
            // the pivot chain's critical path: 46.5 k -> 59 k cycles for the look-ahead steps)
            const int jn = jb + kNB, ng = panel_groups(np, jn);
            arriveTarget += ng;
            if (wave < ng) {
                const bool okp = jn + kNB > n ? ldlt_panel_grp<true>(A, ld, np, n, jn, rdg, y, shadow, dummy + 64 + 16 * wave, lane, wave, &arriveS,
                                                arriveTarget)
                                                 : ldlt_panel_grp<false>(A, ld, np, n, jn, rdg, y, shadow, dummy + 64 + 16 * wave, lane, wave, &arriveS,
                                                arriveTarget);
                if (!okp && wave == 0 && lane == 0) failS = 1;
            } else {
                const int nt = m * (m - 1) / 2;   // tiles with K > kb + 1
                for (int t = wave - ng; t < nt; t += kLdlT / 64 - ng) {
                    int ti, tk;
                    tri(t, ti, tk);
                    trail_tile(jb, (kb + 2 + ti) * kNB, (kb + 2 + tk) * kNB);
                }
            }
            factored = true;
        } else {
            const int nt = m * (m + 1) / 2;
            for (int t = wave; t < nt; t += kLdlT / 64) {
                int ti, tk;
                tri(t, ti, tk);
                trail_tile(jb, (kb + 1 + ti) * kNB, (kb + 1 + tk) * kNB);
            }
            factored = false;
        }
        __syncthreads();
        TACC(tTrail, t_t0);
        if (failS) break;
    }
    TSTAMP(t_s0);
    if (failS) {
        if (tid == 0) flags[0] = 1;
        // the update still runs (with the previous x), as the separate pose block did: the
        // failed trial is then rejected and popped
        if (ptail.scaleOut && wave == 0) pose_tail(ptail, x, st->lambda, lane);
        return;
    }
    if (kLds) {
        // ---- y /= d and the backward substitution with L^T on wave 0 alone, in registers (rows
        //      lane and 64 + lane, np <= 128): for j descending, x_j is final (v_readlane) and every
        //      row i < j takes x_i = fma(-L(j, i), x_j, x_i), L(j, i) read along row j of the lower
        //      triangle (conflict-free, immediate offsets).  Each row subtracts its terms in
        //      descending j, as the blocked form below does.  The diagonal and upper part of the
        //      two 64-row diagonal blocks (W, unread after the factorisation) are zeroed first, so
        //      the loads need no mask (a zero term adds -0 * x_j: x_i is unchanged but for the sign
        //      of an exact zero).  The identity padding (j >= n) has x_j = 0 and is skipped.
        {   // four threads per row j < 128: columns j + q, j + q + 4, ... up to the block's end
            const int j = tid >> 2, q = tid & 3, end = min((j | 63) + 1, np);
            if (j < np)
                for (int i = j + q; i < end; i += 4) A[(size_t)j * ld + i] = 0.0;
        }
        __syncthreads();
        if (wave != 0) return;
        const int i1 = 64 + lane;
        double X0 = lane < np ? y[lane] * rdg[lane] : 0.0;
        double X1 = i1 < np ? y[i1] * rdg[i1] : 0.0;
        TSTAMP(t_b0);
        const int kTop = (n - 1) & ~(kNB - 1);
        for (int kb = kTop; kb >= 0; kb -= kNB) {
            const double* Lk = A + (size_t)kb * ld;
            double La[kNB], Lb[kNB];
            if (kb >= 64) {
#pragma unroll
                for (int t = 0; t < kNB; t++) { La[t] = Lk[(size_t)t * ld + lane]; Lb[t] = Lk[(size_t)t * ld + i1]; }
                if (kb + kNB > n) {   // the top block: its padding rows skipped
                    for (int j = n - 1; j >= kb; j--) {
                        const double xj = shfl_d_dyn(X1, j - 64);
                        X0 = __builtin_fma(-A[(size_t)j * ld + lane], xj, X0);
                        X1 = __builtin_fma(-A[(size_t)j * ld + i1], xj, X1);
                    }
                    continue;
                }
#pragma unroll
                for (int t = kNB - 1; t >= 0; t--) {
                    const double xj = shfl_d_dyn(X1, kb + t - 64);
                    X0 = __builtin_fma(-La[t], xj, X0);
                    X1 = __builtin_fma(-Lb[t], xj, X1);
                }
            } else {
#pragma unroll
                for (int t = 0; t < kNB; t++) La[t] = Lk[(size_t)t * ld + lane];
                if (kb + kNB > n) {
                    for (int j = n - 1; j >= kb; j--) X0 = __builtin_fma(-A[(size_t)j * ld + lane], shfl_d_dyn(X0, j), X0);
                    continue;
                }
#pragma unroll
                for (int t = kNB - 1; t >= 0; t--) X0 = __builtin_fma(-La[t], shfl_d_dyn(X0, kb + t), X0);
            }
        }
#ifdef ORB_TIMING
        if (lane == 0) printf("ldlt backsolve: zero+init %lld chain %lld\n", t_b0 - t_s0, clock64() - t_b0);
#endif
        if (lane < n) x[lane] = X0;
        if (i1 < n) x[i1] = X1;
        if (lane == 0) flags[0] = 0;
        if (ptail.scaleOut) {   // x through LDS to the pose lanes (this wave's LDS operations are in order)
            y[lane] = X0;
            if (i1 < np) y[i1] = X1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            pose_tail(ptail, y, st->lambda, lane);
        }
#ifdef ORB_TIMING
        if (lane == 0) printf("ldlt n %d: stage %lld (own %lld) panel %lld rows %lld trailing %lld solve %lld | panels %lld %lld %lld %lld %lld %lld %lld %lld | bar %lld %lld\n", n, t_f0 - t_l0, t_sa - t_l0, tDiag, tRows, tTrail, clock64() - t_s0, tp[0], tp[1], tp[2], tp[3], tp[4], tp[5], tp[6], tp[7], tpb[0], tpb[1]);
#endif
        return;
    }
    for (int i = tid; i < np; i += kLdlT) y[i] = y[i] * rdg[i];
    __syncthreads();
    // ---- backward substitution with L^T: x_i = y_i - sum_{k > i} L(k, i) x_k, k descending,
    //      in 16-row blocks from the bottom: wave 0 solves the block's 16 x 16 triangle
    //      (v_readlane chain), then every thread takes one row above the block (the block's x
    //      read back from LDS as broadcasts, its column of L conflict-free)
    for (int kb = np - kNB; kb >= 0; kb -= kNB) {
        if (wave == 0) {
            const int r = lane & 15;
            double Ab[kNB];
#pragma unroll
            for (int c = 0; c < kNB; c++) Ab[c] = A[(size_t)(kb + c) * ld + kb + r];   // L(kb+c, kb+r), used for r < c
            double xb = y[kb + r];
#pragma unroll
            for (int c = kNB - 1; c > 0; c--) {
                const double xc = shfl_d(xb, c);
                xb = r < c ? __builtin_fma(-Ab[c], xc, xb) : xb;
            }
            if (lane < kNB) y[kb + r] = xb;
        }
        __syncthreads();
        if (kb == 0) break;
        for (int i = tid; i < kb; i += kLdlT) {
            double v = y[i];
#pragma unroll
            for (int c = kNB - 1; c >= 0; c--) v = __builtin_fma(-A[(size_t)(kb + c) * ld + i], y[kb + c], v);
            y[i] = v;
        }
        __syncthreads();
    }
    if (wave != 0) return;
    for (int i = lane; i < n; i += 64) x[i] = y[i];
    if (lane == 0) flags[0] = 0;
#ifdef ORB_TIMING
    if (lane == 0) printf("ldlt n %d: stage %lld (own %lld) panel %lld rows %lld trailing %lld solve %lld | panels %lld %lld %lld %lld %lld %lld %lld %lld | bar %lld %lld\n", n, t_f0 - t_l0, t_sa - t_l0, tDiag, tRows, tTrail, clock64() - t_s0, tp[0], tp[1], tp[2], tp[3], tp[4], tp[5], tp[6], tp[7], tpb[0], tpb[1]);
#endif
}


// ------------------------------------------------------------------ reduced camera solve, dataflow form
// k_ldlt_df: the same blocked right-looking LDL^T with the forward substitution folded in, and the same
// backward substitution, as k_ldlt_solve<true> (S in LDS, even n, np <= 128), organised so the 16-column
// pivot chain is the only sequential work and no workgroup barrier sits between panels:
//  * wave 0 (PivotCols) factors every panel's 16 x 16 diagonal block E (the current Schur complement,
//    both triangles) with lane (k, q) = k + 16 q holding column k, rows q, q+4, q+8, q+12.  Column c:
//    u(k) = E(c, k) / d_c for k > c (0 otherwise) is L(k, c) and every lane takes X -= E(row, c) u(k),
//    E(., c) broadcast within its 16-lane row by v_mov_b64_dpp row_newbcast (no v_readlane: ~24 cycles
//    of issue each, profiles/r03_lat_micro.txt).  The next pivot comes one column ahead,
//    d_{c+1} = E(c+1, c+1) - E(c+1, c)^2 / d_c from row c+1 before column c's update, so 1/d_{c+1}
//    (v_rcp_f64 + Newton) overlaps the update; row c+1 replicated over the four lane rows comes from an
//    LDS round trip issued a column earlier and corrected by the missing column (no cross-row
//    permutation on the chain).  Per column the wave publishes u (16 doubles), 1/d_c and y_c/d_c, then a
//    sequence counter, into per-panel LDS buffers (a late reader never sees them overwritten);
//  * wave I (1..T-1) owns row block I (FollowCols): for each panel kb < I it follows the pivot's columns
//    over its 16 rows (the same update with the published u; its y rides along), stores their W
//    (upper triangle, the tiles' left operand) and L, then applies panel kb's trailing update to its own
//    tiles (I, K), K = kb+1..I, with f64 MFMA (the diagonal tile last);
//  * LDS flags (monotonic; one wave's LDS operations complete in order): rowDone[I] = kb+1 once row block
//    I's panel-kb L is stored (the owners of lower blocks wait for it before a tile (., I)), diagReady =
//    I once tile (I, I) holds every earlier panel's update and y of block I is stored (the pivot's input
//    for panel I).  Waves 1 and 4 swap blocks so the pivot's SIMD partner (wave 4) owns the lightest one.
// The elimination is the unblocked recurrence's, reassociated per panel (agreement to rounding with
// oracle/lba_oracle.c: tests compare LM traces to 1e-9 and decisions exactly).
template <int L>
__device__ __forceinline__ double rbc16(double v) {   // lane L of each 16-lane row to the whole row
    return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), 0x150 + L, 0xf, 0xf, true));
}
template <int R>
__device__ __forceinline__ unsigned xrow32(unsigned v) {   // lane row R to all four rows (permlane swaps)
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const unsigned t = (R & 1) ? a[1] : a[0];
    const auto b = __builtin_amdgcn_permlane32_swap(t, t, false, false);
    return (R & 2) ? b[1] : b[0];
}
template <int R>
__device__ __forceinline__ double xrow(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return __longlong_as_double((long long)(((unsigned long long)xrow32<R>((unsigned)(u >> 32)) << 32) |
                                            xrow32<R>((unsigned)u)));
}
template <int C, int N>
struct ColUnroll {
    template <class F>
    __device__ __forceinline__ static void run(F& f) {
        f.template col<C>();
        ColUnroll<C + 1, N>::run(f);
    }
};
template <int N>
struct ColUnroll<N, N> {
    template <class F>
    __device__ __forceinline__ static void run(F&) {}
};
template <int C, int N>
struct ColUnrollTo {   // the last panel: columns past the order are identity padding, one uniform exit test each
    template <class F>
    __device__ __forceinline__ static void run(F& f, int nc) {
        if (C >= nc) return;
        f.template col<C>();
        ColUnrollTo<C + 1, N>::run(f, nc);
    }
};
template <int N>
struct ColUnrollTo<N, N> {
    template <class F>
    __device__ __forceinline__ static void run(F&, int) {}
};
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) int lds_i32;

struct DfPivot {
    // entering column C: X = E^(C-1), R = row C of E^(C-1) (replicated), rd = 1/d_C, Q = row C+1 of
    // E^(C-2) (replicated), up = u_(C-1)
    // stores go through per-lane bases fixed for the panel (the publishing lanes' records, the other
    // lanes' private sinks), so a column's stores carry only immediate offsets
    double X[4], Y, rd, R, Q, up;
    int k, seq;
    volatile lds_f64 *pU, *pRG, *rowW, *rowR;
    volatile lds_i32* pC;
#ifdef ORB_TIMING
    long long* tp = nullptr;   // per column: the publish time
#endif
    template <int C>
    __device__ __forceinline__ void col() {
        double P1 = 0.0, w = 0.0, rdn = 1.0;
        if constexpr (C + 1 < kNB) {   // row C+1 of E^(C-1), then the next pivot's reciprocal
            P1 = C == 0 ? Q : __builtin_fma(-rbc16<(C > 0 ? C - 1 : 0)>(Q), up, Q);
            const double a = rbc16<C + 1>(P1);
            w = rbc16<C>(P1);
            rdn = rcp_nr(__builtin_fma(-(w * w), rd, a));
        }
        double Qn = 0.0;   // row C+2 of E^(C-1) through LDS, consumed at the next column's start
        if constexpr (C + 2 < kNB) {   // every lane writes its own slot, all read lane row (C+2) % 4's
            *rowW = X[(C + 2) >> 2];
            Qn = rowR[((C + 2) & 3) * kNB];
        }
        const double u = R * (k > C ? rd : 0.0);
#pragma unroll
        for (int s = 0; s < 4; s++) X[s] = __builtin_fma(-rbc16<C>(X[s]), u, X[s]);
        const double yc = rbc16<C>(Y);
        Y = __builtin_fma(-u, yc, Y);
        pU[C * kNB] = u;
        pRG[2 * C] = rd;
        pRG[2 * C + 1] = rd * yc;
        *pC = seq + C + 1;
#ifdef ORB_TIMING
        if (tp) tp[C] = clock64();
#endif
        if constexpr (C + 1 < kNB) {
            R = __builtin_fma(-w, u, P1);
            rd = rdn;
            up = u;
            Q = Qn;
        }
    }
};

// Follower modes.  kPlain: follow the panel, store W / L afterwards.  kDiag: this row block is the next
// panel's diagonal block: its W / L go to LDS four columns at a time (column k is frozen from column
// k on), each group published on the chunk counter, and its diagonal tile T takes the panel's update
// one f64 MFMA per group (applied a group later, behind the next group's LDS round trip); the
// previous panel's update of T, deferred from then, is applied while the follower first waits for
// the pivot.  kNext: the block after the next diagonal block: it stores its W / L per group the same
// way and, as the diagonal block's chunks appear, applies this panel's update of its tile
// (I, I - 1) — the tile it will follow next panel — to T in registers, so when the pivot starts
// that panel this wave follows at once, its X being T (the MFMA output layout is the follow layout).
enum { kPlain = 0, kDiag = 1, kNext = 2 };
template <int kMode>
struct DfFollow {
    double X[4], Y[4];
    double uq[4], gq[4];     // the current group of four published columns
    double rdk;              // 1 / d of this lane's column k (loaded with k's group)
    bool pf;                 // uq / gq already hold the group starting at the current column
    dbl4 T;                  // kDiag: the diagonal tile; kNext: tile (I, I - 1); MFMA output layout
    double pa, pb;           // the last group's MFMA operands, applied one group later
    int k, seq, seen, jb, rb, ld, rbK;   // rbK (kNext): the diagonal block's first row
    bool defer;              // kDiag: the previous panel's update of T is still to apply
    const volatile lds_f64 *pubU, *pubRG;
    const volatile lds_i32* cnt;
    volatile lds_i32* chunk;
    lds_f64 *A, *sinkD;
#ifdef ORB_TIMING
    long long* tg = nullptr;   // per group: arrival, poll satisfied, group end; [12..15]: counter seen on arrival
#endif
    template <int C>
    __device__ __forceinline__ void col() {
        const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#ifdef ORB_TIMING
        if constexpr ((C & 3) == 0) if (tg) { tg[3 * (C / 4)] = clock64(); tg[12 + C / 4] = __builtin_amdgcn_readfirstlane(*cnt) - seq; }
#endif
        if constexpr (kMode == kDiag && C == 0) {
            if (defer) {   // (the pivot has only just started: this overlaps the wait for its columns)
                const int jp = jb - kNB;
#pragma unroll
                for (int s = 0; s < kNB / 4; s++) {
                    const int pp = jp + 4 * s + lk;
                    T = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(size_t)pp * ld + rb + li], A[(size_t)(rb + li) * ld + pp], T, 0,
                                                             0, 0);
                }
            }
        }
        // the follower trails the pivot, so it takes the pivot's columns four at a time: one poll of the
        // sequence counter (wave-uniform) and one LDS round trip for the group's u and y_c / d_c instead
        // of one per column
        if constexpr ((C & 3) == 0) {
            if (!(C > 0 && pf)) {   // (pf: loaded at the previous group's end)
                if (__builtin_amdgcn_readfirstlane(seen) < seq + C + 4) {
                    int v;
                    while ((v = __builtin_amdgcn_readfirstlane(*cnt)) < seq + C + 4) __builtin_amdgcn_s_sleep(1);
                    seen = v;
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    uq[j] = pubU[(C + j) * kNB + k];
                    gq[j] = pubRG[2 * (C + j) + 1];
                }
                if constexpr (kMode != kPlain) rdk = pubRG[2 * k];   // (used by the lanes of this group)
            }
            // the previous group's MFMA, its operands' LDS round trip hidden behind this group's
            if constexpr (kMode != kPlain && C > 0) T = __builtin_amdgcn_mfma_f64_16x16x4f64(pa, pb, T, 0, 0, 0);
#ifdef ORB_TIMING
            if (tg) tg[3 * (C / 4) + 1] = clock64();
#endif
        }
        const double u = uq[C & 3];
        const double g = gq[C & 3];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const double wi = rbc16<C>(X[s]);
            X[s] = __builtin_fma(-wi, u, X[s]);
            Y[s] = __builtin_fma(-wi, g, Y[s]);
        }
        if constexpr (kMode != kPlain && (C & 3) == 3) {
            // columns C-3..C are final: their -W (upper triangle) and L (lower) out, the MFMA operands
            // read back (the MFMA itself waits for the next group, or the caller)
            const double rdkThis = rdk;
            if constexpr (kMode == kDiag && C + 1 < kNB) {
                // the diagonal block's follower gates the pivot: when the pivot has already published the
                // next group, its loads go out now and overlap this group's stores and operand reads
                if (__builtin_amdgcn_readfirstlane(seen) < seq + C + 5) seen = __builtin_amdgcn_readfirstlane(*cnt);
                pf = __builtin_amdgcn_readfirstlane(seen) >= seq + C + 5;
                if (pf) {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        uq[j] = pubU[(C + 1 + j) * kNB + k];
                        gq[j] = pubRG[2 * (C + 1 + j) + 1];
                    }
                    rdk = pubRG[2 * k];
                }
            }
            if ((k >> 2) == (C >> 2)) {
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int r = rb + lk + 4 * s;
                    A[(size_t)(jb + k) * ld + r] = -X[s];
                    A[(size_t)r * ld + jb + k] = X[s] * rdkThis;
                }
            }
#ifdef ORB_TIMING
            if (tg) tg[3 * (C / 4) + 2] = clock64();
#endif
            const int pc = jb + (C - 3) + lk;
            const int grp = (seq + C + 1) >> 2;   // 4 kb + this group + 1
            if constexpr (kMode == kDiag) {
                if (lane == 0) *chunk = grp;       // (after this wave's stores: LDS is in order per wave)
                pa = A[(size_t)pc * ld + rb + li];
                pb = A[(size_t)(rb + li) * ld + pc];
            } else {
                while (__builtin_amdgcn_readfirstlane(*chunk) < grp) __builtin_amdgcn_s_sleep(1);
                pa = A[(size_t)pc * ld + rb + li];
                pb = A[(size_t)(rbK + li) * ld + pc];
            }
        }
    }
};

__host__ __device__ inline size_t ldlt_df_lds_bytes(int n) {
    const int np = (n + kNB - 1) & ~(kNB - 1);
    return 8 * ((size_t)np * (np + 1) + 2 * (size_t)np + (size_t)(np / kNB) * (kNB * kNB + 2 * kNB) + 64 + kNB * kNB + 4 * kNB + 64 + 32);
}

__global__ __launch_bounds__(kLdlT) void k_ldlt_df(const double* __restrict__ Sg, const double* __restrict__ b, int n,
                                                  double* __restrict__ x, int* __restrict__ flags, const LmState* st,
                                                  PoseTail ptail) {
#ifdef ORB_TIMING
    const long long tEntry = clock64();
#endif
    if (lm_off(st, 1)) return;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int np = (n + kNB - 1) & ~(kNB - 1), ld = np + 1, T = np / kNB;
    const int k = lane & 15, q = lane >> 4;
#ifdef ORB_TIMING
    long long tdf[40] = {0};
    tdf[0] = clock64();
    __shared__ long long waveT[16];
#endif
    double* A = sh;
    double* rdg = A + (size_t)np * ld;
    double* y = rdg + np;
    double* pubU = y + np;                           // [T][16][16]
    double* pubRG = pubU + (size_t)T * kNB * kNB;     // [T][16][2]
    double* sinkD = pubRG + (size_t)T * 2 * kNB;      // per-lane sinks: lane + up to 15 columns x 16
    double* rowbuf = sinkD + 64 + kNB * kNB;          // [4][16]: the pivot's next-row exchange
    int* cnt = (int*)(rowbuf + 4 * kNB);
    int* sinkI = cnt + 2;                             // 64
    volatile lds_i32* rowDone = (volatile lds_i32*)(sinkI + 64);   // [8]
    volatile lds_i32* diagReady = rowDone + 8;
    volatile lds_i32* chunk = rowDone + 9;   // the current diagonal follower's published column groups
    __shared__ int failS;
#ifdef ORB_TIMING
    __shared__ long long dbgT[32];
    __shared__ long long tgS[16], tpS[16];
#endif
    if (tid == 0) { failS = 0; *cnt = 0; }
    if (tid < 10) rowDone[tid] = 0;
#ifdef ORB_TIMING
    if (lane == 0) { waveT[wave] = tEntry; waveT[8 + wave] = tdf[0]; }
#endif
    __syncthreads();
#ifdef ORB_TIMING
    tdf[35] = clock64();
    if (tid == 0) {
        long long e0 = waveT[0], e1 = waveT[0], m1 = waveT[8];
        for (int w = 1; w < 8; w++) { e0 = min(e0, waveT[w]); e1 = max(e1, waveT[w]); m1 = max(m1, waveT[8 + w]); }
        printf("ldlt_df entry: wave0 %lld (rel first), last wave entry +%lld, last lm_off done +%lld, wave0 lm_off %lld, barrier exit +%lld\n",
               waveT[0] - e0, e1 - e0, m1 - e0, waveT[8] - waveT[0], tdf[35] - e0);
    }
#endif
    // ---- staging, per owner, no barrier: the wave of row block I loads its rows' columns
    //      [0, 16(I+1)) (its lower tiles and the whole diagonal tile) and their b, one 16-byte load per
    //      (row, column pair), all in flight; identity padding past n (n even: no pair straddles it)
    const __amdgpu_buffer_rsrc_t rsS = buf_rsrc(Sg, (uint32_t)n * n * 8);
    auto stage_rows = [&](int I) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const int rbs = kNB * I, ncp = 8 * (I + 1);
        u32x4 v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int idx = lane + 64 * u, i = rbs + (idx & 15), c2 = 2 * (idx >> 4);
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsS, (idx >> 4) < ncp && i < n && c2 < n ? (i * n + c2) * 8 : kBufOob,
                                                         0, 0);
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int idx = lane + 64 * u, i = rbs + (idx & 15), c2 = 2 * (idx >> 4);
            if ((idx >> 4) < ncp) {
                double* dst = A + (size_t)i * ld + c2;
                dst[0] = __longlong_as_double((long long)(((unsigned long long)v[u].y << 32) | v[u].x)) +
                         (i >= n && i == c2 ? 1.0 : 0.0);
                dst[1] = __longlong_as_double((long long)(((unsigned long long)v[u].w << 32) | v[u].z)) +
                         (i >= n && i == c2 + 1 ? 1.0 : 0.0);
            }
        }
        if (lane < kNB) y[rbs + lane] = rbs + lane < n ? b[rbs + lane] : 0.0;
    };
    auto wait_ge = [&](volatile lds_i32* f, int v) {
        while (__builtin_amdgcn_readfirstlane(*f) < v) __builtin_amdgcn_s_sleep(1);
    };
    auto tile = [&](int jb, int I0, int K0) {   // A(I, K) -= W(I, panel) L(K, panel)^T, four f64 MFMA
        const int li = lane & 15, lk = lane >> 4;
        double a[kNB / 4], bb[kNB / 4];
        dbl4 acc;
#pragma unroll
        for (int s = 0; s < kNB / 4; s++) {
            const int p = jb + 4 * s + lk;
            a[s] = A[(size_t)p * ld + I0 + li];   // -W
            bb[s] = A[(size_t)(K0 + li) * ld + p];
        }
#pragma unroll
        for (int s = 0; s < 4; s++) acc[s] = A[(size_t)(I0 + lk + 4 * s) * ld + K0 + li];
#pragma unroll
        for (int s = 0; s < kNB / 4; s++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], bb[s], acc, 0, 0, 0);
#pragma unroll
        for (int s = 0; s < 4; s++) A[(size_t)(I0 + lk + 4 * s) * ld + K0 + li] = acc[s];
    };
    if (wave == 0) {
        stage_rows(0);
#ifdef ORB_TIMING
        tdf[36] = clock64();
#endif
        for (int kb = 0; kb < T; kb++) {
            const int jb = kb * kNB;
#ifdef ORB_TIMING
            if (kb < 8) tdf[1 + 4 * kb] = clock64();
#endif
            if (kb > 0) wait_ge(diagReady, kb);
#ifdef ORB_TIMING
            if (kb < 8) tdf[2 + 4 * kb] = clock64();
#endif
            DfPivot P;
            P.k = k;
            P.seq = kNB * kb;
            P.pU = (volatile lds_f64*)(q == 0 ? pubU + (size_t)kb * kNB * kNB + k : sinkD + lane);
            P.pRG = (volatile lds_f64*)(lane == 0 ? pubRG + (size_t)kb * 2 * kNB : sinkD + lane);
            P.pC = (volatile lds_i32*)(lane == 0 ? cnt : sinkI + lane);
            P.rowW = (volatile lds_f64*)(rowbuf + lane);
            P.rowR = (volatile lds_f64*)(rowbuf + k);
#pragma unroll
            for (int s = 0; s < 4; s++) P.X[s] = A[(size_t)(jb + q + 4 * s) * ld + jb + k];
            P.Y = y[jb + k];
            P.R = xrow<0>(P.X[0]);
            P.Q = xrow<1>(P.X[0]);
            P.up = 0.0;
            P.rd = rcp_nr(rbc16<0>(P.R));
            const int nc = n - jb;
#ifdef ORB_TIMING
            if (kb < 8) tdf[3 + 4 * kb] = clock64();
#endif
#ifdef ORB_TIMING
            long long tpl[16];
            P.tp = kb == 3 ? tpl : nullptr;
#endif
            if (nc >= kNB) ColUnroll<0, kNB>::run(P);
            else ColUnrollTo<0, kNB>::run(P, nc);
#ifdef ORB_TIMING
            if (kb == 3 && lane == 0)
                for (int i = 0; i < 16; i++) tpS[i] = tpl[i];
#endif
#ifdef ORB_TIMING
            if (kb < 8) tdf[4 + 4 * kb] = clock64();
#endif
            // the diagonal block's L (strict lower), 1/d and its finished y; a zero or non-finite pivot
            // (1/d zero or non-finite) flags the solve
            const double rdk = jb + k < n ? pubRG[(size_t)kb * 2 * kNB + 2 * k] : 1.0;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int i = q + 4 * s;
                *(i > k ? A + (size_t)(jb + i) * ld + jb + k : sinkD + lane) = P.X[s] * rdk;
            }
            if (q == 0) { rdg[jb + k] = rdk; y[jb + k] = P.Y; }
            const bool bad = !(rdk != 0.0 && isfinite(rdk));
            if (__builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) failS = 1;
        }
    } else if (wave < T) {
        const int I = wave == 4 ? 1 : (wave == 1 && T > 4) ? 4 : wave, rb = kNB * I;
        stage_rows(I);
        double Yr[4];
#pragma unroll
        for (int s = 0; s < 4; s++) Yr[s] = y[rb + q + 4 * s];
        int seen = 0;
        dbl4 Tn;   // tile (I, I - 1) carried from the kNext panel into the diagonal panel
        const int li = lane & 15, lk = lane >> 4;
        for (int kb = 0; kb < I; kb++) {
            const int jb = kb * kNB;
            auto follow = [&](auto& F, bool xFromT) {
                F.k = k;
                F.seq = kNB * kb;
                F.seen = seen;
                F.jb = jb;
                F.rb = rb;
                F.ld = ld;
                F.pubU = (const volatile lds_f64*)(pubU + (size_t)kb * kNB * kNB);
                F.pubRG = (const volatile lds_f64*)(pubRG + (size_t)kb * 2 * kNB);
                F.cnt = (const volatile lds_i32*)cnt;
                F.chunk = chunk;
                F.A = (lds_f64*)A;
                F.sinkD = (lds_f64*)(sinkD + lane);
                F.pf = false;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    F.X[s] = xFromT ? Tn[s] : A[(size_t)(rb + q + 4 * s) * ld + jb + k];
                    F.Y[s] = Yr[s];
                }
                ColUnroll<0, kNB>::run(F);
                seen = F.seen;
#pragma unroll
                for (int s = 0; s < 4; s++) Yr[s] = F.Y[s];
            };
            if (kb == I - 1) {   // this block is the next diagonal block
                DfFollow<kDiag> F;
#pragma unroll
                for (int s = 0; s < 4; s++) F.T[s] = A[(size_t)(rb + lk + 4 * s) * ld + rb + li];
                F.defer = kb >= 1;
#ifdef ORB_TIMING
                const long long tfs = clock64();
#endif
                // the diagonal block's follower gates the next panel: it takes issue priority over
                // the plain follower sharing its SIMD (solve stage 0.484 -> 0.470 ms per config-4
                // solve in a same-box A/B; the same for the kNext follower gained nothing more)
                __builtin_amdgcn_s_setprio(3);
#ifdef ORB_TIMING
                long long tgl[16];
                F.tg = kb == 3 ? tgl : nullptr;
#endif
                follow(F, I >= 2);
#ifdef ORB_TIMING
                if (kb == 3 && lane == 0)
                    for (int i = 0; i < 16; i++) tgS[i] = tgl[i];
#endif
#ifdef ORB_TIMING
                if (lane == 0 && kb < 8) { dbgT[2 * kb] = tfs; dbgT[2 * kb + 1] = clock64(); }
#endif
                F.T = __builtin_amdgcn_mfma_f64_16x16x4f64(F.pa, F.pb, F.T, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < 4; s++) A[(size_t)(rb + lk + 4 * s) * ld + rb + li] = F.T[s];
#pragma unroll
                for (int s = 0; s < 4; s++)
                    if (k == 0) y[rb + q + 4 * s] = Yr[s];
                // tile (I, I) complete: the pivot's panel I may start
#ifdef ORB_TIMING
                if (lane == 0 && kb < 8) dbgT[16 + kb] = clock64();
#endif
                *(lane == 0 ? diagReady : (volatile lds_i32*)(sinkI + lane)) = I;
                *(lane == 0 ? rowDone + I : (volatile lds_i32*)(sinkI + lane)) = kb + 1;
                __builtin_amdgcn_s_setprio(0);
            } else if (kb == I - 2) {   // the diagonal block is I - 1: tile (I, I - 1) in registers
                DfFollow<kNext> F;
                F.rbK = rb - kNB;
#pragma unroll
                for (int s = 0; s < 4; s++) F.T[s] = A[(size_t)(rb + lk + 4 * s) * ld + rb - kNB + li];
                follow(F, false);
                Tn = __builtin_amdgcn_mfma_f64_16x16x4f64(F.pa, F.pb, F.T, 0, 0, 0);
                *(lane == 0 ? rowDone + I : (volatile lds_i32*)(sinkI + lane)) = kb + 1;
                // (tile (I, I): deferred to the diagonal panel; tile (I, I - 1): Tn)
            } else {
                DfFollow<kPlain> F;
                follow(F, false);
                const double rdk = pubRG[(size_t)kb * 2 * kNB + 2 * k];
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int r = rb + q + 4 * s;
                    A[(size_t)(jb + k) * ld + r] = -F.X[s];         // -W(r, jb + k): the tiles' left operand
                    A[(size_t)r * ld + jb + k] = F.X[s] * rdk;      // L(r, jb + k)
                }
                *(lane == 0 ? rowDone + I : (volatile lds_i32*)(sinkI + lane)) = kb + 1;
                // panel kb's trailing update of this row block's tiles (I, K), K = kb + 1 .. I
                for (int K = kb + 1; K <= I; K++) {
                    if (K != I) wait_ge(rowDone + K, kb + 1);
                    tile(jb, rb, kNB * K);
                }
            }
        }
    }
    __syncthreads();
#ifdef ORB_TIMING
    tdf[33] = clock64();
#endif
    if (failS) {
        if (tid == 0) flags[0] = 1;
        // the update still runs (with the previous x), as in k_ldlt_solve: the trial is then rejected
        if (ptail.scaleOut && wave == 0) pose_tail(ptail, x, st->lambda, lane);
        return;
    }
    // ---- y /= d and the backward substitution with L^T on wave 0 (k_ldlt_solve<true>'s register form)
    {
        const int j = tid >> 2, qq = tid & 3, end = min((j | 63) + 1, np);
        if (j < np)
            for (int i = j + qq; i < end; i += 4) A[(size_t)j * ld + i] = 0.0;
    }
    __syncthreads();
    if (wave != 0) return;
    PoseTailPre ptf;   // (P <= 21 here: np <= 128)
    if (ptail.scaleOut) pose_tail_prefetch(ptail, lane, ptf);
    const int i1 = 64 + lane;
    double X0 = lane < np ? y[lane] * rdg[lane] : 0.0;
    double X1 = i1 < np ? y[i1] * rdg[i1] : 0.0;
    const int kTop = (n - 1) & ~(kNB - 1);
    for (int kb = kTop; kb >= 0; kb -= kNB) {
        const double* Lk = A + (size_t)kb * ld;
        double La[kNB], Lb[kNB];
        if (kb >= 64) {
#pragma unroll
            for (int t = 0; t < kNB; t++) { La[t] = Lk[(size_t)t * ld + lane]; Lb[t] = Lk[(size_t)t * ld + i1]; }
            if (kb + kNB > n) {
                for (int jj = n - 1; jj >= kb; jj--) {
                    const double xj = shfl_d_dyn(X1, jj - 64);
                    X0 = __builtin_fma(-A[(size_t)jj * ld + lane], xj, X0);
                    X1 = __builtin_fma(-A[(size_t)jj * ld + i1], xj, X1);
                }
                continue;
            }
#pragma unroll
            for (int t = kNB - 1; t >= 0; t--) {
                const double xj = shfl_d_dyn(X1, kb + t - 64);
                X0 = __builtin_fma(-La[t], xj, X0);
                X1 = __builtin_fma(-Lb[t], xj, X1);
            }
        } else {
#pragma unroll
            for (int t = 0; t < kNB; t++) La[t] = Lk[(size_t)t * ld + lane];
            if (kb + kNB > n) {
                for (int jj = n - 1; jj >= kb; jj--) X0 = __builtin_fma(-A[(size_t)jj * ld + lane], shfl_d_dyn(X0, jj), X0);
                continue;
            }
#pragma unroll
            for (int t = kNB - 1; t >= 0; t--) X0 = __builtin_fma(-La[t], shfl_d_dyn(X0, kb + t), X0);
        }
    }
    if (lane < n) x[lane] = X0;
    if (i1 < n) x[i1] = X1;
    if (lane == 0) flags[0] = 0;
#ifdef ORB_TIMING
    tdf[34] = clock64();
#endif
    if (ptail.scaleOut) {   // x through LDS to the pose lanes (this wave's LDS operations are in order)
        y[lane] = X0;
        if (i1 < np) y[i1] = X1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pose_tail_finish(ptail, y, st->lambda, lane, ptf);
    }
#ifdef ORB_TIMING
    if (lane == 0) {
        printf("ldlt_df n %d: to-factor-end %lld bsolve %lld tail %lld | per panel wait/prologue/loop/epilogue:", n,
               tdf[33] - tdf[0], tdf[34] - tdf[33], clock64() - tdf[34]);
        for (int kb = 0; kb < T && kb < 8; kb++)
            printf(" %lld/%lld/%lld/%lld", tdf[2 + 4 * kb] - tdf[1 + 4 * kb], tdf[3 + 4 * kb] - tdf[2 + 4 * kb],
                   tdf[4 + 4 * kb] - tdf[3 + 4 * kb], (kb + 1 < T && kb < 7 ? tdf[5 + 4 * kb] : tdf[33]) - tdf[4 + 4 * kb]);
        printf(" | stage0 %lld (barrier %lld, stage_rows %lld) | diag follower start/loop-end/flag vs pivot loop start/end:", tdf[1] - tdf[0], tdf[35] - tdf[0], tdf[36] - tdf[35]);
        for (int kb = 0; kb + 1 < T && kb < 7; kb++)
            printf(" %lld/%lld/%lld", dbgT[2 * kb] - tdf[3 + 4 * kb], dbgT[2 * kb + 1] - tdf[4 + 4 * kb], dbgT[16 + kb] - tdf[4 + 4 * kb]);
        printf("\n");
        if (T > 4) {   // panel 3: the pivot's column publish times and the diagonal follower's groups (vs the pivot loop start)
            const long long t0 = tdf[3 + 4 * 3];
            printf("ldlt_df panel 3 pivot publish:");
            for (int i = 0; i < 16; i++) printf(" %lld", tpS[i] - t0);
            printf(" | diag follower group arrive/polled/end (counter seen on arrival):");
            for (int g = 0; g < 4; g++) printf(" %lld/%lld/%lld(%lld)", tgS[3 * g] - t0, tgS[3 * g + 1] - t0, tgS[3 * g + 2] - t0, tgS[12 + g]);
            printf("\n");
        }
    }
#endif
}
// the dataflow solve applies to even orders that fit the LDS image (every local-BA system: n = 6P);
// ORB_LBA_LDLT_OLD=1 keeps k_ldlt_solve<true> (A/B runs)
static bool use_ldlt_df(int n) {
    const char* e = std::getenv("ORB_LBA_LDLT_OLD");   // read per solve, so a test can switch it
    const bool old = e && e[0] == '1';
    const int np = (n + kNB - 1) & ~(kNB - 1);
    return !old && (n & 1) == 0 && np <= kLdlLdsMaxN;
}

// ------------------------------------------------------------------ multi-workgroup reduced solve
// Reduced systems beyond the LDS image (np > 128, more than 21 free keyframes: LocalMapping's
// window is every covisible keyframe, unbounded, R/src/Optimizer.cpp:569-625).  The same blocked
// right-looking LDL^T in 16-column panels as k_ldlt_solve, spread over the chip, two launches
// per panel (a dependent kernel boundary, ~1.5 us, is the cheapest cross-XCD synchronisation):
//   k_ldlt_mw_panel  the panel's rows split over waves, 48 below the diagonal block per wave; every
//                    wave also holds the 16 diagonal rows and computes the pivots, 1/d and the
//                    diagonal block's W itself (ldlt_panel_grp's scheme), so no wave waits on another
//   k_ldlt_mw_trail  the trailing lower triangle, one 16 x 16 tile per wave, four v_mfma_f64_16x16x4
// then the backward substitution in 128-row super-blocks (k_ldlt_mw_bsolve / k_ldlt_mw_bupd, below;
// in fused slots it ends with the free poses' update, as k_ldlt_solve's tail).  The work image is np x np (ld = np): W in
// the upper triangle, L in the lower; a diagonal block's L rows go to Ldg[np][16] and its rows'
// finished forward substitution to yfin (the diagonal rows are read by every wave of the panel
// while it runs, so nothing writes them in place).
struct MwLdl {
    double *A, *rdg, *y, *yfin, *Ldg, *sink, *yb;   // yb: the backward substitution's working vector
    int* fail;
    // the envelope (k_mw_envelope, once per solve; null: dense): per 16-row tile of the image, the
    // first column any of its rows holds a non-zero in.  LDL^T keeps a row's leading zeros (L(r, p)
    // = 0 for p < first(r): no fill-in outside the envelope), so a trailing tile, a panel's row
    // group or a back-substitution row block whose operands all lie left of the envelope adds
    // exact zeros and is skipped — a banded window (a corridor of keyframes) updates only its band
    const int32_t* tfirst;
    int n, np;
};

// The envelope of the reduced matrix from the listed pose-pair blocks (the block pattern of
// G/core/block_solver.hpp:192-207; block (i, j), i <= j): pose j's rows start at column
// 6 min{i : (i, j) listed} (the diagonal is always listed), a padding row r at r.  One workgroup,
// the per-pose minima in LDS (4 P bytes).
__global__ __launch_bounds__(1024) void k_mw_envelope(const int32_t* __restrict__ pairs, const int32_t* __restrict__ npairs,
                                                      int P, int np, int32_t* __restrict__ tfirst) {
    extern __shared__ int32_t fpose[];
    const int tid = threadIdx.x;
    for (int j = tid; j < P; j += 1024) fpose[j] = j;
    __syncthreads();
    const int G = *npairs;
    for (int k = tid; k < G; k += 1024) {
        const int pr = pairs[k];
        atomicMin(&fpose[pr & 0xFFFF], pr >> 16);
    }
    __syncthreads();
    for (int T = tid; T < np / 16; T += 1024) {
        int f = 16 * T;
        for (int r = 16 * T; r < 16 * T + 16; r++) f = min(f, r < 6 * P ? 6 * fpose[r / 6] : r);
        tfirst[T] = f;
    }
}
constexpr int kMwWaves = 4;   // waves per workgroup of the panel / trailing kernels

__device__ __forceinline__ void tri_index(int t, int& ti, int& tk) {   // t -> (ti, tk), tk <= ti, row-major
    ti = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
    while (ti * (ti + 1) / 2 > t) ti--;
    tk = t - ti * (ti + 1) / 2;
}

// S (n x n) -> the padded image (identity padding), y = b, the padding pivots' 1/d = 1
__global__ __launch_bounds__(256) void k_ldlt_mw_stage(MwLdl m, const double* __restrict__ S, const double* __restrict__ b,
                                                      const LmState* st) {
    if (lm_off(st, 1)) return;
    const int np = m.np, n = m.n;
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t == 0) *m.fail = 0;
    if (t < (size_t)np * np) {
        const int i = (int)(t / np), j = (int)(t % np);
        m.A[t] = (i < n && j < n) ? S[(size_t)i * n + j] : (i == j ? 1.0 : 0.0);
    }
    if (t < (size_t)np) {
        m.y[t] = (int)t < n ? b[t] : 0.0;
        if ((int)t >= n) m.rdg[t] = 1.0;
    }
}

// With the envelope: row i of the lower triangle from its tile's first column (one workgroup per
// row).  Nothing reads the image left of the envelope or its upper triangle before the panels
// write W there, and the image is zeroed once per solve (build_pairs), so only this part changes
// from trial to trial.
__global__ __launch_bounds__(256) void k_ldlt_mw_stage_env(MwLdl m, const double* __restrict__ S, const double* __restrict__ b,
                                                          const LmState* st) {
    if (lm_off(st, 1)) return;
    const int np = m.np, n = m.n, i = blockIdx.x;
    if (i == 0 && threadIdx.x == 0) *m.fail = 0;
    for (int j = m.tfirst[i >> 4] + (int)threadIdx.x; j <= i; j += 256)
        m.A[(size_t)i * np + j] = (i < n && j < n) ? S[(size_t)i * n + j] : (i == j ? 1.0 : 0.0);
    if (threadIdx.x == 0) {
        m.y[i] = i < n ? b[i] : 0.0;
        if (i >= n) m.rdg[i] = 1.0;
    }
}

// Panel jb of the multi-workgroup factorisation, kMwNB columns wide (twice k_ldlt_solve's: half
// the launches and half the passes of the trailing update over the matrix).  Lanes 0..kMwNB-1 of
// every wave hold the panel's diagonal rows, lanes kMwNB..63 its own rows below (group g: rows
// jb + kMwNB + (64 - kMwNB) g + ...); the column recurrence is ldlt_panel_grp's.
constexpr int kMwNB = 32;
__host__ __device__ __forceinline__ int mw_groups(int np, int jb) {
    const int g = (np - jb - kMwNB + (64 - kMwNB) - 1) / (64 - kMwNB);
    return g > 1 ? g : 1;
}
// row group g of panel jb runs (group 0 always: it holds the diagonal block's results)
__device__ __forceinline__ bool mw_group_live(const MwLdl& m, int jb, int g) {
    constexpr int NB = kMwNB, RB = 64 - kMwNB;
    if (g > 0 && jb + NB + RB * g >= m.np) return false;   // no rows below for this group
    if (g > 0 && m.tfirst) {   // the group's 32 rows have no non-zero in the panel's columns
        const int T0 = (jb + NB + RB * g) >> 4;
        if (min(m.tfirst[T0], m.tfirst[T0 + 1]) > jb + NB - 1) return false;
    }
    return true;
}
// the panel's column recurrence for the wave's rows (lane < NB: diagonal row jb + lane; else row
// jb + NB + RB g + lane - NB), P = the rows' panel columns after every earlier update, Y = y(row),
// wsc = 64 doubles of LDS
template <bool kTail>
__device__ __forceinline__ void mw_panel_core(const MwLdl& m, int jb, int g, int lane, double (&P)[kMwNB], double Y,
                                              double* const wsc) {
    constexpr int NB = kMwNB, RB = 64 - kMwNB;   // diagonal lanes, rows below per wave
    const int np = m.np, ld = np, nr = m.n;
    double* const A = m.A;
    const int r = lane < NB ? jb + lane : jb + NB + RB * g + (lane - NB);
    const bool live = r < np, inplace = live && lane >= NB;
    double* const Lrow = inplace ? A + (size_t)r * ld + jb : m.sink + (size_t)(lane & (NB - 1)) * ld;
    double* const Wcol = inplace ? A + (size_t)jb * ld + r : m.sink + lane;
    double* const wst = wsc + lane;   // (wsc holds 64: the rows below write unread slots, no flat store)
    double dj = shfl_d(P[0], 0);
    bool ok = dj != 0.0 && isfinite(dj);
    double rd = rcp_nr(dj);
    double myrd = 1.0;
    double Wd[NB], lprev = 0.0;
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int j = jb + c;
        if (kTail && j >= nr) break;
        const double w = P[c];
        double djn = 1.0, rn = 1.0, w1 = 0.0, w2 = 0.0;
        if (c + 1 < NB) {
            w1 = shfl_d(w, c + 1);
            const double a1 = shfl_d(P[c + 1], c + 1);
            djn = __builtin_fma(-(w1 * w1), rd, a1);
            rn = __builtin_amdgcn_rcp(djn);
        }
        if (c + 2 < NB) w2 = shfl_d(w, c + 2);
        const double yj = shfl_d(Y, c);
        __builtin_amdgcn_sched_barrier(0);
        if (c >= 1) {
#pragma unroll
            for (int k = c + 2; k < NB; k++) P[k] = __builtin_fma(-lprev, Wd[k], P[k]);
        }
        const double l = w * rd;
        P[c] = l;
        Wcol[(size_t)c * ld] = w;
        Lrow[c] = l;
        myrd = lane == c ? rd : myrd;
        *wst = w;
#pragma unroll
        for (int k = c + 3; k < NB; k++) Wd[k] = wsc[k];
        if (c + 1 < NB) P[c + 1] = __builtin_fma(-l, w1, P[c + 1]);
        if (c + 2 < NB) P[c + 2] = __builtin_fma(-l, w2, P[c + 2]);
        if (r > j) Y = __builtin_fma(-l, yj, Y);
        lprev = l;
        if (c + 1 < NB) {
            const double e0 = __builtin_fma(-djn, rn, 1.0);
            const double r1 = __builtin_fma(rn, e0, rn);
            const double e1 = __builtin_fma(-djn, r1, 1.0);
            ok = ok && djn != 0.0 && isfinite(djn);
            dj = djn;
            rd = __builtin_fma(r1, e1, r1);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g == 0 && lane < NB) {   // the diagonal block: L rows, 1/d, finished y
#pragma unroll
        for (int c = 0; c < NB; c++) m.Ldg[(size_t)r * NB + c] = P[c];
        m.rdg[r] = myrd;
        m.yfin[r] = Y;
        if (lane == 0 && !ok) *m.fail = 1;
    }
    if (inplace) m.y[r] = Y;
}
template <bool kTail>
__global__ __launch_bounds__(64 * kMwWaves) void k_ldlt_mw_panel(MwLdl m, int jb, const LmState* st) {
    constexpr int NB = kMwNB, RB = 64 - kMwNB;
    if (lm_off(st, 1)) return;
    if (__builtin_amdgcn_readfirstlane(*m.fail)) return;
    __shared__ double wscS[kMwWaves][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g = __builtin_amdgcn_readfirstlane((int)blockIdx.x * kMwWaves + wv);
    if (!mw_group_live(m, jb, g)) return;
    const int np = m.np, ld = np;
    const int r = lane < NB ? jb + lane : jb + NB + RB * g + (lane - NB);
    const int rc = min(r, np - 1);
    double P[NB];
    const double Y = m.y[rc];
#pragma unroll
    for (int c = 0; c < NB; c++) P[c] = m.A[(size_t)rc * ld + jb + c];
    mw_panel_core<kTail>(m, jb, g, lane, P, Y, wscS[wv]);
}

// one 16 x 16 tile (I0, K0) of the trailing update after the panel at column jb:
// A(I0.., K0..) - W(I0.., panel) L(K0.., panel)^T, kMwNB / 4 v_mfma_f64_16x16x4; lane (li, lk)
// returns rows I0 + lk + 4 q of column K0 + li
struct MwTileOps {
    double a[kMwNB / 4], bb[kMwNB / 4];
    dbl4 acc;
};
__device__ __forceinline__ void mw_tile_load(const MwLdl& m, int jb, int I0, int K0, int lane, MwTileOps& o) {
    const int ld = m.np, li = lane & 15, lk = lane >> 4;
    const double* __restrict__ A = m.A;
#pragma unroll
    for (int s = 0; s < kMwNB / 4; s++) {
        const int p = jb + 4 * s + lk;
        o.a[s] = -A[(size_t)p * ld + I0 + li];        // -W(I0 + li, p)
        o.bb[s] = A[(size_t)(K0 + li) * ld + p];      //  L(K0 + li, p)
    }
#pragma unroll
    for (int q = 0; q < 4; q++) o.acc[q] = A[(size_t)(I0 + lk + 4 * q) * ld + K0 + li];
}
__device__ __forceinline__ dbl4 mw_tile_mma(const MwTileOps& o) {
    dbl4 acc = o.acc;
#pragma unroll
    for (int s = 0; s < kMwNB / 4; s++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[s], o.bb[s], acc, 0, 0, 0);
    return acc;
}
__device__ __forceinline__ dbl4 mw_tile(const MwLdl& m, int jb, int I0, int K0, int lane) {
    MwTileOps o;
    mw_tile_load(m, jb, I0, K0, lane, o);
    return mw_tile_mma(o);
}
// outside the envelope W(I, panel) or L(K, panel) is all zeros: the tile's update adds nothing
__device__ __forceinline__ bool mw_tile_live(const MwLdl& m, int jb, int I, int K) {
    return !m.tfirst || max(m.tfirst[I], m.tfirst[K]) <= jb + kMwNB - 1;
}

// trailing update after the panel at column block kb (kMwNB wide): 16 x 16 tiles (I, K) of the
// lower triangle beyond it, one per wave (tile rows / columns from tBase: k_ldlt_mw_step's
// trailing part starts two tile columns later)
__device__ __forceinline__ void mw_trail_tile(const MwLdl& m, int jb, int tBase, int t, int lane) {
    const int T = m.np / 16, mm = T - tBase;
    if (mm <= 0 || t >= mm * (mm + 1) / 2) return;
    int ti, tk;
    tri_index(t, ti, tk);
    if (!mw_tile_live(m, jb, tBase + ti, tBase + tk)) return;
    const int I0 = (tBase + ti) * 16, K0 = (tBase + tk) * 16, ld = m.np;
    const int li = lane & 15, lk = lane >> 4;
    const dbl4 acc = mw_tile(m, jb, I0, K0, lane);
#pragma unroll
    for (int q = 0; q < 4; q++) m.A[(size_t)(I0 + lk + 4 * q) * ld + K0 + li] = acc[q];
}
__global__ __launch_bounds__(64 * kMwWaves) void k_ldlt_mw_trail(MwLdl m, int kb, const LmState* st) {
    if (lm_off(st, 1)) return;
    if (__builtin_amdgcn_readfirstlane(*m.fail)) return;
    const int jb = kb * kMwNB;
    const int t = __builtin_amdgcn_readfirstlane((int)blockIdx.x * kMwWaves + (int)(threadIdx.x >> 6));
    mw_trail_tile(m, jb, (jb + kMwNB) / 16, t, threadIdx.x & 63);
}

// LDS-only workgroup barrier: orders the workgroup's LDS accesses and leaves its global loads in
// flight (a plain __syncthreads waits for every outstanding load, prefetches included)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Panel kb's trailing update and panel kb + 1's factorisation in one launch (one kernel boundary
// per panel instead of two).  Workgroup g < nPanelWg takes panel kb + 1's row group g: its four
// waves form the two tile columns of the next panel for the group's 64 rows (the diagonal block's
// three lower tiles and the group's own four, two per wave, all loads of a wave in flight at once)
// with the same v_mfma sequence as the trailing tiles, into a 64 x 33 LDS image, and wave 0 runs
// the column recurrence on them; the other workgroups update the tiles right of those two columns
// in place.  Neither part reads what the other writes (the next panel's tile columns are read only
// by the workgroups that factor them; its L and W land left of and above the trailing tiles), and
// the panel's values are bitwise those the separate trailing launch would have stored.
template <bool kTail>
__global__ __launch_bounds__(64 * kMwWaves) void k_ldlt_mw_step(MwLdl m, int kb, int nPanelWg, const LmState* st) {
    constexpr int NB = kMwNB, RB = 64 - kMwNB;
    __shared__ double wscS[64];
    __shared__ double tileS[64][NB + 1];   // rows: the diagonal block's 32, then the group's 32
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int jb = kb * NB, jn = jb + NB, t0 = jn / 16;
    if ((int)blockIdx.x >= nPanelWg) {
        if (lm_off(st, 1)) return;
        if (__builtin_amdgcn_readfirstlane(*m.fail)) return;
        const int t = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - nPanelWg) * kMwWaves + wv);
        mw_trail_tile(m, jb, t0 + 2, t, lane);
        return;
    }
    const int g = blockIdx.x;
    const int np = m.np, ld = np;
    const bool below = jn + NB + RB * g < np;   // (group 0 of the last panel has no rows below)
    if (g > 0 && !below) return;
    TSTAMP(ts0);
    const int Ig = (jn + NB + RB * g) >> 4;
    // tile s of 7: 0..2 the diagonal block's (t0, t0), (t0 + 1, t0), (t0 + 1, t0 + 1); 3..6 the
    // group's (Ig + u, t0 + v).  Formed whether or not the envelope reaches them: outside it the
    // update adds exact zeros (L left of a row's envelope is never written: zero from the
    // once-per-solve clear), so the values equal the skipping trailing launch's, and no load
    // waits on the envelope table
    auto tile_of = [&](int s, int& I, int& K, int& row0) {
        if (s < 3) { I = t0 + (s > 0 ? 1 : 0); K = t0 + (s == 2 ? 1 : 0); row0 = 16 * (I - t0); }
        else { I = Ig + ((s - 3) >> 1); K = t0 + ((s - 3) & 1); row0 = 32 + 16 * ((s - 3) >> 1); }
    };
    auto tile_on = [&](int s) { return s < 3 || (s < 7 && below); };
    const int li = lane & 15, lk = lane >> 4;
    // every load of the workgroup before any test of the state: the recurrence wave's raw rows
    // and both tiles' operands of each wave in flight at once (one memory round trip: they were
    // just written on other XCDs), then the LM phase, the failure flag and the envelope
    double P[NB];
    double Y = 0.0;
    if (wv == 0) {
        const int r = lane < NB ? jn + lane : jn + NB + RB * g + (lane - NB);
        const int rc = min(r, np - 1);
        Y = m.y[rc];
#pragma unroll
        for (int c = 0; c < NB; c++) P[c] = m.A[(size_t)rc * ld + jn + c];   // (the diagonal block's upper tile: as stored)
    }
    MwTileOps to[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int s = wv + kMwWaves * k;
        int I, K, row0;
        tile_of(min(s, 6), I, K, row0);
        if (tile_on(s)) mw_tile_load(m, jb, 16 * I, 16 * K, lane, to[k]);
    }
    if (lm_off(st, 1)) return;
    if (__builtin_amdgcn_readfirstlane(*m.fail)) return;
    if (!mw_group_live(m, jn, g)) return;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int s = wv + kMwWaves * k;
        if (!tile_on(s)) continue;
        int I, K, row0;
        tile_of(s, I, K, row0);
        const dbl4 acc = mw_tile_mma(to[k]);
#pragma unroll
        for (int q = 0; q < 4; q++) tileS[row0 + lk + 4 * q][16 * (K - t0) + li] = acc[q];
    }
    lds_barrier();
    if (wv != 0) return;
    TSTAMP(ts1);
    {
        const int u = lane >> 4;   // this lane's tile row: 0, 1 the diagonal block, 2, 3 the group's
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const int s = u == 0 ? (v == 0 ? 0 : 7) : u == 1 ? 1 + v : 3 + 2 * (u - 2) + v;   // (0, 1): upper, as stored
            if (s == 7 || !tile_on(s)) continue;
#pragma unroll
            for (int c = 0; c < 16; c++) P[16 * v + c] = tileS[lane][16 * v + c];
        }
    }
    mw_panel_core<kTail>(m, jn, g, lane, P, Y, wscS);
#ifdef ORB_TIMING
    if (lane == 0 && g == 0 && kb == 5) printf("mw step kb 5 g 0: tiles %lld recurrence %lld\n", ts1 - ts0, clock64() - ts1);
#endif
}

// The backward substitution x = L^-T (y / d) in super-blocks of kSB rows from the bottom, two
// launches each: k_ldlt_mw_bsolve (one workgroup) stages the super-block's lower triangle of L in
// LDS and solves its 16-row blocks bottom-up there (the chain of 16-row triangles runs out of LDS,
// not out of L2); k_ldlt_mw_bupd (every row above, one per thread, over the chip) subtracts the
// super-block's contribution L(K0 + c, i) x_{K0 + c}.  The bottom super-block first forms y / d
// for every row; the top one ends with the fused slots' pose update.
constexpr int kSB = 128;   // (64 measured no faster at np = 1224: 24.1 vs 23.7-23.9 ms per solve)
__global__ __launch_bounds__(512) void k_ldlt_mw_bsolve(MwLdl m, int K0, double* __restrict__ x, int* __restrict__ flags,
                                                        const LmState* st, PoseTail ptail, int first, int last) {
    if (lm_off(st, 1)) return;
    TSTAMP(t_b0);
    extern __shared__ __attribute__((aligned(16))) double bsm[];
    double* Ls = bsm;                        // [kSB][kSB + 1]: L(K0 + r, K0 + c), c < r
    double* ysb = Ls + kSB * (kSB + 1);      // [kSB]  (LDS independent of the order: any window size)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int np = m.np, n = m.n, ld = np, nsb = min(kSB, np - K0);
    if (__builtin_amdgcn_readfirstlane(*m.fail)) {
        if (last) {   // as k_ldlt_solve: the update still runs (with the previous x), the trial is rejected
            if (tid == 0) flags[0] = 1;
            if (ptail.scaleOut && wave == 0) pose_tail(ptail, x, st->lambda, lane);
        }
        return;
    }
    if (first)
        for (int i = tid; i < np; i += 512) {
            const double v = m.yfin[i] * m.rdg[i];
            m.yb[i] = v;
            if (i >= K0) ysb[i - K0] = v;
        }
    else
        for (int r = tid; r < nsb; r += 512) ysb[r] = m.yb[K0 + r];
    {   // the strict lower triangle only (the chain and the updates read nothing else), row-major
        // triangle order (coalesced rows); every load unconditional at a clamped index, all of a
        // thread's in flight at once (the rows were just written by trailing updates on other XCDs)
        constexpr int kPer = (kSB * (kSB - 1) / 2 + 511) / 512;
        const int ntri = nsb * (nsb - 1) / 2;
        double v[kPer];
        int at[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            int r, c;
            tri_index(min(tid + 512 * k, max(ntri - 1, 0)), r, c);   // (r, c), c <= r
            r += 1;                                                   // strict: c < r
            const bool sameBlk = (K0 + r) / kMwNB == (K0 + c) / kMwNB;   // a panel's diagonal block: from Ldg
            v[k] = sameBlk ? m.Ldg[(size_t)(K0 + r) * kMwNB + (K0 + c) % kMwNB] : m.A[(size_t)(K0 + r) * ld + K0 + c];
            at[k] = r * (kSB + 1) + c;
        }
#pragma unroll
        for (int k = 0; k < kPer; k++)
            if (tid + 512 * k < ntri) Ls[at[k]] = v[k];
    }
    __syncthreads();
    TSTAMP(t_b1);
    // kBB-row blocks bottom-up: wave 0 solves the block's triangle (its L entries read from LDS
    // first, then the v_readlane chain), then every thread takes one row above the block
    constexpr int kBB = 32;
    for (int jb = nsb - kBB; jb >= 0; jb -= kBB) {
        if (wave == 0) {
            const int r = lane & (kBB - 1);
            double Lb[kBB];
#pragma unroll
            for (int c = 1; c < kBB; c++) Lb[c] = Ls[(jb + c) * (kSB + 1) + jb + min(r, c - 1)];
            double xb = ysb[jb + r];
#pragma unroll
            for (int c = kBB - 1; c > 0; c--) {
                const double xc = shfl_d(xb, c);
                xb = r < c ? __builtin_fma(-Lb[c], xc, xb) : xb;
            }
            if (lane < kBB) ysb[jb + r] = xb;
        }
        __syncthreads();
        for (int i = tid; i < jb; i += 512) {   // four partial sums: a quarter of the dependent chain
            double v[4] = {ysb[i], 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = kBB - 1; c >= 0; c--)
                v[c & 3] = __builtin_fma(-Ls[(jb + c) * (kSB + 1) + i], ysb[jb + c], v[c & 3]);
            ysb[i] = (v[0] + v[1]) + (v[2] + v[3]);
        }
        __syncthreads();
    }
    for (int r = tid; r < nsb; r += 512)
        if (K0 + r < n) x[K0 + r] = ysb[r];
#ifdef ORB_TIMING
    if (tid == 0) printf("mw bsolve K0 %d: stage %lld chain %lld\n", K0, t_b1 - t_b0, clock64() - t_b1);
#endif
    if (!last) return;
    if (tid == 0) flags[0] = 0;
    if (ptail.scaleOut) {   // x as stored: this super-block's rows just now (visible to the workgroup
                            // after the barrier), the rest by the earlier launches
        __syncthreads();
        if (wave == 0) pose_tail(ptail, x, st->lambda, lane);
    }
}
// 64 rows per workgroup; wave w takes the super-block's columns [kSB/4 w, kSB/4 (w + 1)) with all
// its loads in flight, the four partial sums are added in wave order (deterministic)
__global__ __launch_bounds__(256) void k_ldlt_mw_bupd(MwLdl m, int K0, const double* __restrict__ x, const LmState* st) {
    if (lm_off(st, 1)) return;
    if (__builtin_amdgcn_readfirstlane(*m.fail)) return;
    constexpr int kC = kSB / 4;   // columns per wave
    __shared__ double xs[kSB];
    __shared__ double part[4][64];
    const int np = m.np, n = m.n, ld = np, nsb = min(kSB, np - K0);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (m.tfirst) {   // rows left of every super-block row's envelope: L(K0 + c, i) = 0
        int f = K0;
        for (int T = K0 >> 4; T < (K0 + nsb) >> 4; T++) f = min(f, m.tfirst[T]);
        if ((int)blockIdx.x * 64 + 63 < f) return;
    }
    for (int c = threadIdx.x; c < kSB; c += 256) xs[c] = c < nsb && K0 + c < n ? x[K0 + c] : 0.0;
    __syncthreads();
    const int i = blockIdx.x * 64 + lane;
    if (i < K0) {
        double a[kC];
#pragma unroll
        for (int k = 0; k < kC; k++) {
            const int c = kC * w + k;
            a[k] = c < nsb ? m.A[(size_t)(K0 + c) * ld + i] : 0.0;
        }
        double v = 0.0;
#pragma unroll
        for (int k = kC - 1; k >= 0; k--) v = __builtin_fma(-a[k], xs[kC * w + k], v);
        part[w][lane] = v;
    }
    __syncthreads();
    if (w == 0 && i < K0) m.yb[i] = m.yb[i] + ((part[3][lane] + part[2][lane]) + (part[1][lane] + part[0][lane]));
}

// The whole backward substitution in one launch (one workgroup, np <= kMwBackMaxN): the working
// vector y / d lives in LDS and the super-blocks go bottom-up as k_ldlt_mw_bsolve /
// k_ldlt_mw_bupd take them, with the same arithmetic (the 32-row chains, and each row update's
// four column-quarter partials added in the same order), so x is bitwise theirs; the next
// super-block's L triangle is loaded into registers while this one's chain runs, and rows left of
// a super-block's envelope take no update (their terms are exact zeros).  2 (np / kSB) - 1
// dependent launches become one.
constexpr int kMwBackMaxN = 2048;   // LDS: the 128 x 129 triangle + 64 + np doubles (148 KB at 2048)
__global__ __launch_bounds__(512) void k_ldlt_mw_back(MwLdl m, double* __restrict__ x, int* __restrict__ flags,
                                                      const LmState* st, PoseTail ptail) {
    if (lm_off(st, 1)) return;
    extern __shared__ __attribute__((aligned(16))) double bsm[];
    double* const Ls = bsm;                       // [kSB][kSB + 1]: L(K0 + r, K0 + c), c < r (+ 64 spare)
    double* const yb = Ls + kSB * (kSB + 1) + 64; // [np]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int np = m.np, n = m.n, ld = np;
    if (__builtin_amdgcn_readfirstlane(*m.fail)) {   // as k_ldlt_mw_bsolve: the trial is rejected
        if (tid == 0) flags[0] = 1;
        if (ptail.scaleOut && wave == 0) pose_tail(ptail, x, st->lambda, lane);
        return;
    }
    for (int i = tid; i < np; i += 512) yb[i] = m.yfin[i] * m.rdg[i];
    // each super-block's envelope start: the least tile start of its rows (kSB / 16 tiles)
    __shared__ int sLo[kMwBackMaxN / kSB];
    if (tid < (np + kSB - 1) / kSB) {
        const int K0 = tid * kSB, nsb = min(kSB, np - K0);
        int lo = 0;
        if (m.tfirst) {
            lo = K0;
            for (int T = K0 >> 4; T < (K0 + nsb) >> 4; T++) lo = min(lo, m.tfirst[T]);
        }
        sLo[tid] = lo;
    }
    TSTAMP(tb0);
    long long tStage = 0, tChain = 0, tUpd = 0, tComb = 0;
    (void)tStage; (void)tChain; (void)tUpd; (void)tComb;
    constexpr int kPer = (kSB * (kSB - 1) / 2 + 511) / 512, kTri = kSB * (kSB - 1) / 2;
    // this thread's entries (r, c) of a full super-block's strict lower triangle, row-major (a
    // partial one, nsb rows, takes the entries with r < nsb: the first nsb (nsb - 1) / 2, as
    // k_ldlt_mw_bsolve stages it); found once, not per super-block
    int rcP[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        int r, c;
        tri_index(min(tid + 512 * k, kTri - 1), r, c);
        rcP[k] = tid + 512 * k < kTri ? ((r + 1) << 8) | c : -1;
    }
    double v[kPer];
    int at[kPer];
    auto load_tri = [&](int K0) {   // the super-block's strict lower triangle of L, branch-free
        const int nsb = min(kSB, np - K0);
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int r = rcP[k] >> 8, c = rcP[k] & 0xFF;
            const bool ok = rcP[k] >= 0 && r < nsb;
            const int rr = ok ? r : 1, cc = ok ? c : 0;
            const double* pL = m.Ldg + (size_t)(K0 + rr) * kMwNB + (cc & (kMwNB - 1));   // (K0: a multiple of kMwNB)
            const double* pA = m.A + (size_t)(K0 + rr) * ld + K0 + cc;
            v[k] = *((rr >> 5) == (cc >> 5) ? pL : pA);   // a panel's diagonal block: from Ldg
            at[k] = ok ? rr * (kSB + 1) + cc : kSB * (kSB + 1) + lane;
        }
    };
    const int nsbk = (np + kSB - 1) / kSB;
    load_tri((nsbk - 1) * kSB);
    for (int q = nsbk - 1; q >= 0; q--) {
        const int K0 = q * kSB, nsb = min(kSB, np - K0);
        TSTAMP(tq0);
        lds_barrier();   // the previous super-block is done with Ls (and the partials aliasing it)
#pragma unroll
        for (int k = 0; k < kPer; k++) Ls[at[k]] = v[k];
        if (q > 0) load_tri(K0 - kSB);   // in flight during this super-block's chain
        lds_barrier();
        TACC(tStage, tq0);
        TSTAMP(tq1);
        double* const ysb = yb + K0;
        constexpr int kBB = 32;
        for (int jb = nsb - kBB; jb >= 0; jb -= kBB) {
            if (wave == 0) {
                const int r = lane & (kBB - 1);
                double Lb[kBB];
#pragma unroll
                for (int c = 1; c < kBB; c++) Lb[c] = Ls[(jb + c) * (kSB + 1) + jb + min(r, c - 1)];
                double xb = ysb[jb + r];
#pragma unroll
                for (int c = kBB - 1; c > 0; c--) {
                    const double xc = shfl_d(xb, c);
                    xb = r < c ? __builtin_fma(-Lb[c], xc, xb) : xb;
                }
                if (lane < kBB) ysb[jb + r] = xb;
            }
            lds_barrier();
            for (int i = tid; i < jb; i += 512) {
                double w4[4] = {ysb[i], 0.0, 0.0, 0.0};
#pragma unroll
                for (int c = kBB - 1; c >= 0; c--)
                    w4[c & 3] = __builtin_fma(-Ls[(jb + c) * (kSB + 1) + i], ysb[jb + c], w4[c & 3]);
                ysb[i] = (w4[0] + w4[1]) + (w4[2] + w4[3]);
            }
            lds_barrier();
        }
        for (int r = tid; r < nsb; r += 512)
            if (K0 + r < n) x[K0 + r] = ysb[r];
        TACC(tChain, tq1);
        if (q == 0) break;
        TSTAMP(tq2);
        // the rows above: k_ldlt_mw_bupd's four column quarters (x of the padding rows as 0), each
        // (quarter, row) a task with its 32 loads in flight, the partials through LDS (aliasing the
        // triangle, whose chain is done) and added in bupd's order
        const int lo = sLo[q];
        constexpr int kC = kSB / 4;
        const int R = (K0 - lo + 63) & ~63;
        double* const part = Ls;   // [4][R]
        for (int t = tid; t < 4 * R; t += 512) {
            const int w = t / R, i = lo + t % R;
            if (i >= K0) continue;
            double a[kC];
#pragma unroll
            for (int k = 0; k < kC; k++) {   // (loads at clamped rows, unconditional)
                const int c = kC * w + k;
                const double t2 = m.A[(size_t)(K0 + min(c, nsb - 1)) * ld + i];
                a[k] = c < nsb ? t2 : 0.0;
            }
            double acc = 0.0;
#pragma unroll
            for (int k = kC - 1; k >= 0; k--) {
                const int c = kC * w + k;
                acc = __builtin_fma(-a[k], c < nsb && K0 + c < n ? ysb[c] : 0.0, acc);
            }
            part[w * R + (i - lo)] = acc;
        }
        lds_barrier();
        TACC(tUpd, tq2);
        TSTAMP(tq3);
        for (int i = lo + tid; i < K0; i += 512) {
            const int o = i - lo;
            yb[i] = yb[i] + ((part[3 * R + o] + part[2 * R + o]) + (part[R + o] + part[o]));
        }
        TACC(tComb, tq3);
    }
#ifdef ORB_TIMING
    if (tid == 0)
        printf("mw back np %d: total %lld stage %lld chain %lld update %lld combine %lld\n", np, clock64() - tb0, tStage, tChain,
               tUpd, tComb);
#endif
    if (tid == 0) flags[0] = 0;
    if (ptail.scaleOut) {   // x as stored by this workgroup (visible after the barrier)
        __syncthreads();
        if (wave == 0) pose_tail(ptail, x, st->lambda, lane);
    }
}

// enqueue the multi-workgroup solve of S x = b (n = order of S) on s
static void enqueue_ldlt_mw(hipStream_t s, const MwLdl& m, const double* S, const double* b, double* x, int* flags,
                            const LmState* st, const PoseTail& pt) {
    const int np = m.np, T = np / kMwNB;
    const size_t tot = (size_t)np * np;
    if (m.tfirst) hipLaunchKernelGGL(k_ldlt_mw_stage_env, dim3((unsigned)np), dim3(256), 0, s, m, S, b, st);
    else hipLaunchKernelGGL(k_ldlt_mw_stage, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, m, S, b, st);
    // ORB_LBA_MW_SPLIT=1: a panel launch and a trailing launch per panel (A/B runs)
    const bool split = std::getenv("ORB_LBA_MW_SPLIT") != nullptr;
    auto wgs = [](int n) { return (n + kMwWaves - 1) / kMwWaves; };
    for (int kb = 0; kb < T; kb++) {
        const int jb = kb * kMwNB;
        if (kb == 0 || split) {
            const dim3 gp((unsigned)wgs(mw_groups(np, jb)));
            if (jb + kMwNB > m.n) hipLaunchKernelGGL(k_ldlt_mw_panel<true>, gp, dim3(64 * kMwWaves), 0, s, m, jb, st);
            else hipLaunchKernelGGL(k_ldlt_mw_panel<false>, gp, dim3(64 * kMwWaves), 0, s, m, jb, st);
        }
        const int mm = np / 16 - (jb + kMwNB) / 16, tiles = mm * (mm + 1) / 2;
        if (tiles <= 0) continue;
        if (split) {
            hipLaunchKernelGGL(k_ldlt_mw_trail, dim3((unsigned)wgs(tiles)), dim3(64 * kMwWaves), 0, s, m, kb, st);
            continue;
        }
        // this panel's trailing update with the next panel's factorisation
        const int jn = jb + kMwNB, pw = mw_groups(np, jn), mr = mm - 2, rest = mr > 0 ? mr * (mr + 1) / 2 : 0;
        const dim3 gs((unsigned)(pw + wgs(rest)));
        if (jn + kMwNB > m.n) hipLaunchKernelGGL(k_ldlt_mw_step<true>, gs, dim3(64 * kMwWaves), 0, s, m, kb, pw, st);
        else hipLaunchKernelGGL(k_ldlt_mw_step<false>, gs, dim3(64 * kMwWaves), 0, s, m, kb, pw, st);
    }
    if (np <= kMwBackMaxN && !split) {
        hipLaunchKernelGGL(k_ldlt_mw_back, dim3(1), dim3(512), ((size_t)kSB * (kSB + 1) + 64 + np) * 8, s, m, x, flags, st, pt);
        return;
    }
    const int nsbk = (np + kSB - 1) / kSB;
    for (int q = nsbk - 1; q >= 0; q--) {
        const int K0 = q * kSB;
        hipLaunchKernelGGL(k_ldlt_mw_bsolve, dim3(1), dim3(512), ((size_t)kSB * (kSB + 1) + kSB) * 8, s, m, K0, x,
                           flags, st, q == 0 ? pt : PoseTail{}, q == nsbk - 1 ? 1 : 0, q == 0 ? 1 : 0);
        if (q > 0) hipLaunchKernelGGL(k_ldlt_mw_bupd, dim3((K0 + 63) / 64), dim3(256), 0, s, m, K0, x, st);
    }
}


// Back-substitution and update (G/core/block_solver.hpp:462-484, sparse_optimizer.cpp:422-435),
// 64 landmarks per 256-thread block, four lanes per landmark: x_l = D^-1 (b_l - sum_e
// Hpl_e^T x_p(pose_e)), push() of X_l and X_l += x_l.  The block after the landmark blocks
// pushes and applies T <- exp(x_p) T to the free poses.  partScale[block] = the block's share
// of x^T (lambda x + b) (OptimizationAlgorithmLevenberg::computeScale).
__global__ __launch_bounds__(256) void k_backsub_update(LbaDev d, const int32_t* __restrict__ freePoses) {
    if (lm_off(d.lm, 1)) return;
    const double lambda = d.lm->lambda;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ double wsum[4];
    const int nPtBlocks = (d.M + 63) / 64;
    double sc = 0.0;
    if ((int)blockIdx.x < nPtBlocks) {
        const int l = blockIdx.x * 64 + tid / kLanesPerPt, sub = tid % kLanesPerPt;
        double cl[3] = {0.0, 0.0, 0.0};
        if (l < d.M) {
            for (int a = d.ptStart[l] + sub; a < d.ptStart[l + 1]; a += kLanesPerPt) {
                const int k = d.ptAct[a];
                const int pi = d.actPi[k];
                if (pi < 0) break;   // fixed poses are last
                const double* Bi = d.Hpl_e + 18 * (size_t)k;
                const double* xp = d.x + 6 * pi;
#pragma unroll
                for (int q = 0; q < 3; q++)
#pragma unroll
                    for (int r = 0; r < 6; r++) cl[q] += Bi[r * 3 + q] * (-xp[r]);
            }
        }
#pragma unroll
        for (int q = 0; q < 3; q++) { cl[q] += __shfl_xor(cl[q], 1, 64); cl[q] += __shfl_xor(cl[q], 2, 64); }
        if (l < d.M && sub == 0) {
            const double* bl = d.bl + 3 * (size_t)l;
            const double c0 = bl[0] + cl[0], c1 = bl[1] + cl[1], c2 = bl[2] + cl[2];
            const double* Di = d.Dinv + 9 * (size_t)l;
            double* xl = d.x + 6 * (size_t)d.P + 3 * (size_t)l;
            const int g = d.ptGlob[l];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const double v = Di[q * 3] * c0 + Di[q * 3 + 1] * c1 + Di[q * 3 + 2] * c2;
                xl[q] = v;
                const double X = d.X[3 * (size_t)g + q];
                d.bX[3 * (size_t)g + q] = X;
                d.X[3 * (size_t)g + q] = X + v;
                sc += v * (lambda * v + bl[q]);
            }
        }
    } else {
        for (int i = tid; i < d.P; i += 256) {
            const int p = freePoses[i];
            const int k = d.poseIdx[p];
            double q[4], t[3], u[6];
            for (int j = 0; j < 4; j++) { q[j] = d.q[4 * p + j]; d.bq[4 * p + j] = q[j]; }
            for (int j = 0; j < 3; j++) { t[j] = d.t[3 * p + j]; d.bt[3 * p + j] = t[j]; }
            for (int j = 0; j < 6; j++) {
                u[j] = d.x[6 * k + j];
                sc += u[j] * (lambda * u[j] + d.bp[6 * k + j]);
            }
            d_se3_exp_left(u, q, t);
            for (int j = 0; j < 4; j++) d.q[4 * p + j] = q[j];
            for (int j = 0; j < 3; j++) d.t[3 * p + j] = t[j];
        }
    }
    sc = wave_sum_d(sc);
    if (lane == 0) wsum[wave] = sc;
    __syncthreads();
    if (tid == 0) d.partScale[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

// Fused slots: the landmark blocks of k_backsub_update followed by the trial errors of each
// landmark's edges (k_edge_errors' work, one launch fewer per slot).  k_ldlt_solve's tail has
// already pushed and updated the free poses and written their share of the scale; here lane
// sub of a landmark's four evaluates its edges sub, sub + 4, ... at the new X_l (broadcast from
// lane 0 of the four), so partChi[block] holds the robust chi2 of the block's 64 landmarks'
// edges.  Workgroup 0 marks the decision pending and samples terminate() as k_edge_errors did.
__global__ __launch_bounds__(256) void k_backsub_errors(LbaDev d, double hmono, double hstereo) {
    // Every load that does not depend on another is issued before the phase guard and the
    // first use (clamped indices, unconditional): the state, the landmark's CSR range, its
    // first kPtBatch edges (act position, pose index, Hpl block, the pose's x) and its bl,
    // D^-1, X, so the chain is ptStart -> ptAct -> (actPi, Hpl) -> x instead of one round
    // trip per dependent load per edge.  The summation order is the original's.
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ double wsum[4], csum[4];
    const int l = blockIdx.x * 64 + tid / kLanesPerPt, sub = tid % kLanesPerPt;
    const int lc = min(l, d.M - 1);
    const int phase = d.lm->phase;
    const double lambda = d.lm->lambda;
    const int a0 = d.ptStart[lc] + sub, a1 = l < d.M ? d.ptStart[lc + 1] : a0;
    const int g = d.ptGlob[lc];
    double blv[3], Di[9], Xo[3];
#pragma unroll
    for (int q = 0; q < 3; q++) blv[q] = d.bl[3 * (size_t)lc + q];
#pragma unroll
    for (int q = 0; q < 9; q++) Di[q] = d.Dinv[9 * (size_t)lc + q];
#pragma unroll
    for (int q = 0; q < 3; q++) Xo[q] = d.X[3 * (size_t)g + q];
    const int last = max(d.ptStart[lc + 1] - 1, 0);
    int kk[kPtBatch], pi[kPtBatch];
    double B[kPtBatch][18], xp[kPtBatch][6];
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) kk[u] = d.ptAct[min(a0 + kLanesPerPt * u, last)];
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) {
        pi[u] = d.actPi[kk[u]];
#pragma unroll
        for (int i = 0; i < 18; i++) B[u][i] = d.Hpl_e[18 * (size_t)kk[u] + i];
    }
#pragma unroll
    for (int u = 0; u < kPtBatch; u++)
#pragma unroll
        for (int r = 0; r < 6; r++) xp[u][r] = d.x[6 * max(pi[u], 0) + r];
    EdgeStatic es[kPtBatch];   // the same edges' inputs for the trial errors below
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) es[u] = edge_static(d, kk[u]);
    if (phase != 1) return;   // lm_off(d.lm, 1)
    double cl[3] = {0.0, 0.0, 0.0};
    bool open = true;   // fixed poses are last: the first one ends the landmark's sum
#pragma unroll
    for (int u = 0; u < kPtBatch; u++) {
        open = open && a0 + kLanesPerPt * u < a1 && pi[u] >= 0;
        if (open) {
#pragma unroll
            for (int q = 0; q < 3; q++)
#pragma unroll
                for (int r = 0; r < 6; r++) cl[q] += B[u][r * 3 + q] * (-xp[u][r]);
        }
    }
    if (open) {
        for (int a = a0 + kLanesPerPt * kPtBatch; a < a1; a += kLanesPerPt) {
            const int k = d.ptAct[a];
            const int pik = d.actPi[k];
            if (pik < 0) break;
            const double* Bi = d.Hpl_e + 18 * (size_t)k;
            const double* xq = d.x + 6 * pik;
#pragma unroll
            for (int q = 0; q < 3; q++)
#pragma unroll
                for (int r = 0; r < 6; r++) cl[q] += Bi[r * 3 + q] * (-xq[r]);
        }
    }
#pragma unroll
    for (int q = 0; q < 3; q++) { cl[q] += __shfl_xor(cl[q], 1, 64); cl[q] += __shfl_xor(cl[q], 2, 64); }
    double sc = 0.0, Xn[3] = {0.0, 0.0, 0.0};
    if (l < d.M && sub == 0) {
        const double c0 = blv[0] + cl[0], c1 = blv[1] + cl[1], c2 = blv[2] + cl[2];
        double* xl = d.x + 6 * (size_t)d.P + 3 * (size_t)l;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const double v = Di[q * 3] * c0 + Di[q * 3 + 1] * c1 + Di[q * 3 + 2] * c2;
            xl[q] = v;
            const double X = Xo[q];
            d.bX[3 * (size_t)g + q] = X;
            Xn[q] = X + v;
            d.X[3 * (size_t)g + q] = Xn[q];
            sc += v * (lambda * v + blv[q]);
        }
    }
    // the new X_l from lane 0 of the four (ds_swizzle-free: a 4-lane broadcast by shuffles)
#pragma unroll
    for (int q = 0; q < 3; q++) Xn[q] = __shfl(Xn[q], lane & ~(kLanesPerPt - 1), 64);
    double chi = 0.0;
    if (l < d.M) {
#pragma unroll
        for (int u = 0; u < kPtBatch; u++)
            if (a0 + kLanesPerPt * u < a1) chi += edge_error_s(d, kk[u], es[u], hmono, hstereo, Xn);
        for (int a = a0 + kLanesPerPt * kPtBatch; a < a1; a += kLanesPerPt) chi += edge_error(d, d.ptAct[a], hmono, hstereo, Xn);
    }
    sc = wave_sum_d(sc);
    chi = wave_sum_d(chi);
    if (lane == 0) { wsum[wave] = sc; csum[wave] = chi; }
    __syncthreads();
    if (tid == 0) {
        d.partScale[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
        d.partChi[blockIdx.x] = (csum[0] + csum[1]) + (csum[2] + csum[3]);
        if (blockIdx.x == 0) {
            d.lm->pending = 1;
            d.red[4] = lm_stop_now(d.lm, d.stopWord, 0.0) ? 1.0 : 0.0;
        }
    }
}

// pop() after a rejected trial (communicator path; k_lm_decide_fused does it in one process)
__global__ __launch_bounds__(256) void k_pop(LbaDev d, int nposes, const int32_t* freePoses) {
    if (d.lm && !d.lm->pop) return;   // only after a rejected trial
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < d.M) {
        const int g = d.ptGlob[i];
        for (int j = 0; j < 3; j++) d.X[3 * (size_t)g + j] = d.bX[3 * (size_t)g + j];
    }
    if (i < nposes) {
        const int p = freePoses[i];
        for (int j = 0; j < 4; j++) d.q[4 * p + j] = d.bq[4 * p + j];
        for (int j = 0; j < 3; j++) d.t[3 * p + j] = d.bt[3 * p + j];
    }
}

// Deterministic single-workgroup sum of n doubles (fixed stride assignment + fixed tree).
__global__ __launch_bounds__(1024) void k_sum(const double* __restrict__ v, int n, double* __restrict__ out,
                                               const LmState* st, int want) {
    if (lm_off(st, want)) return;
    __shared__ double sh[1024];
    const int tid = threadIdx.x;
    double s = 0;
    for (int i = tid; i < n; i += 1024) s += v[i];
    sh[tid] = s;
    __syncthreads();
    for (int w = 512; w >= 1; w >>= 1) {
        if (tid < w) sh[tid] += sh[tid + w];
        __syncthreads();
    }
    if (tid == 0) *out = sh[0];
}

// scale terms: x_j (lambda x_j + b_j) for poses (when includePoses) and owned points
__global__ __launch_bounds__(256) void k_scale_terms(LbaDev d, int includePoses, double* __restrict__ out) {
    if (lm_off(d.lm, 1)) return;
    const double lambda = d.lm->lambda;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int np = 6 * d.P, n = np + 3 * d.M;
    if (i >= n) return;
    const double xi = d.x[i];
    double b;
    if (i < np) b = includePoses ? d.bp[i] : 0.0;   // only rank 0 contributes the replicated pose part
    else b = d.bl[i - np];
    out[i] = (i < np && !includePoses) ? 0.0 : xi * (lambda * xi + b);
}

// max |diag| of Hpp (global) and Hll (owned): computeLambdaInit's maxDiagonal
__global__ __launch_bounds__(1024) void k_maxdiag(const double* __restrict__ Hpp, int P, const double* __restrict__ Hll,
                                                   int M, double* __restrict__ out, const LmState* st) {
    if (lm_off(st, 3)) return;
    __shared__ double sh[1024];
    const int tid = threadIdx.x;
    double m = 0;
    for (int i = tid; i < 6 * P; i += 1024) m = fmax(m, fabs(Hpp[36 * (i / 6) + 7 * (i % 6)]));
    for (int i = tid; i < 3 * M; i += 1024) m = fmax(m, fabs(Hll[9 * (i / 3) + 4 * (i % 3)]));
    sh[tid] = m;
    __syncthreads();
    for (int w = 512; w >= 1; w >>= 1) {
        if (tid < w) sh[tid] = fmax(sh[tid], sh[tid + w]);
        __syncthreads();
    }
    if (tid == 0) *out = sh[0];
}

// Collective staging for a guarded all-reduce: the phase's buffer, or zeros when the phase is
// skipped (every rank skips alike, so the sum stays zero and is not copied back).
__global__ __launch_bounds__(256) void k_pack(double* __restrict__ ws, const double* __restrict__ buf, size_t n,
                                              const LmState* st, int want) {
    const bool off = lm_off(st, want);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) ws[i] = off ? 0.0 : buf[i];
}
__global__ __launch_bounds__(256) void k_unpack(double* __restrict__ buf, const double* __restrict__ ws, size_t n,
                                                const LmState* st, int want) {
    if (lm_off(st, want)) return;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) buf[i] = ws[i];
}

// The reduced system's exchange with a communicator (the upper triangle only): the
// pose-pair blocks of the global pair list (every pair some landmark couples, the diagonal
// blocks, identical on every rank) and b_s, packed back to back — G 6x6 blocks + 6P doubles in
// place of the dense 36 P^2 + 6P.  Unpacking writes each block and its mirror, as k_schur_pairs
// stores them.  Guarded like k_pack: a skipped phase packs zeros and leaves S alone.
template <bool kSys>
__global__ __launch_bounds__(256) void k_pack_pairs(double* __restrict__ ws, const double* __restrict__ S,
                                                    const double* __restrict__ bs, const int32_t* __restrict__ pairs,
                                                    int G, int P, const LmState* st, int want) {
    const bool off = lm_off(st, want);
    const size_t n = 6 * (size_t)P, tot = 36 * (size_t)G + n;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (size_t)gridDim.x * 256) {
        double v;
        if (i < 36 * (size_t)G) {
            const int pr = pairs[i / 36], e = (int)(i % 36);
            const int bi = pr >> 16, bj = pr & 0xFFFF;
            v = S[(size_t)(6 * bi + e / 6) * n + 6 * bj + e % 6];
        } else {
            v = bs[i - 36 * (size_t)G];
        }
        v = off ? 0.0 : v;
        if (kSys) __hip_atomic_store(ws + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else ws[i] = v;
    }
}
__global__ __launch_bounds__(256) void k_unpack_pairs(double* __restrict__ S, double* __restrict__ bs,
                                                      const double* __restrict__ ws, const int32_t* __restrict__ pairs,
                                                      int G, int P, const LmState* st, int want) {
    if (lm_off(st, want)) return;
    const size_t n = 6 * (size_t)P, tot = 36 * (size_t)G + n;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (size_t)gridDim.x * 256) {
        const double v = ws[i];
        if (i < 36 * (size_t)G) {
            const int pr = pairs[i / 36], e = (int)(i % 36);
            const int bi = pr >> 16, bj = pr & 0xFFFF, r = e / 6, q = e % 6;
            S[(size_t)(6 * bi + r) * n + 6 * bj + q] = v;
            S[(size_t)(6 * bj + q) * n + 6 * bi + r] = v;   // (a diagonal block: the same value twice)
        } else {
            bs[i - 36 * (size_t)G] = v;
        }
    }
}

// ---- device-side exchange of a device group (lba_group): no host in the loop, so the slots of a
// sharded solve are captured into HIP graphs like the single-process ones.  Every rank's
// workspace and flag words live in fine-grained memory on its own device; a collective is
//   k_pack_sys (system-scope stores of the rank's contribution)
//   k_grp_sync(0): epoch e = ++epoch; ready[rank] = e (release, system scope); wait ready[p] >= e
//   k_grp_reduce: every rank sums all ranks' slices in rank order (system-scope loads over xGMI)
//   k_grp_sync(1): read[rank] = e; wait read[p] >= e (nobody packs into a workspace still read)
// Every rank runs the same sequence of collectives (identical LM decisions), so epochs agree.
// A wait longer than GrpDev::waitTicks of the constant-rate wall clock (2 s; a peer's first launch,
// loading its code objects, takes ~0.3 s) sets the rank's error word and gives up: the solve then
// fails with ORB_EGPU instead of hanging the device, and the rank's later waits are skipped.
constexpr int kMaxGroupDev = 16;
struct GrpDev {
    uint32_t* flags[kMaxGroupDev];   // rank p's flag words: [0] ready epoch, [32] read epoch
    const double* ws[kMaxGroupDev];  // rank p's workspace
    uint32_t* epoch;                 // this rank's collective counter
    int* err;                        // this rank's error word
    int rank, n;
    uint64_t waitTicks;              // wait bound in wall_clock64() ticks (hipDeviceAttributeWallClockRate)
};
__global__ void k_grp_sync(GrpDev g, int which) {
    if (threadIdx.x != 0) return;
    const bool failed = __hip_atomic_load(g.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    uint32_t e = *g.epoch;
    if (which == 0) {
        e += 1;
        *g.epoch = e;
    }
    const int w = which ? 32 : 0;
    __hip_atomic_store(g.flags[g.rank] + w, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (failed) return;   // after one timed-out wait the rest of the solve does not wait (it fails anyway)
    // bounded by the constant-rate wall clock (not by an iteration count, whose duration depends on
    // the load latency over xGMI)
    const uint64_t t0 = wall_clock64();
    for (int q = 0; q < g.n; q++) {
        if (q == g.rank) continue;
        while (__hip_atomic_load(g.flags[q] + w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
            if (wall_clock64() - t0 > g.waitTicks) {
                __hip_atomic_store(g.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
}
__global__ __launch_bounds__(256) void k_pack_sys(double* __restrict__ ws, const double* __restrict__ buf, size_t n,
                                                  const LmState* st, int want) {
    const bool off = lm_off(st, want);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __hip_atomic_store(ws + i, off ? 0.0 : buf[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(256) void k_grp_reduce(GrpDev g, size_t n, int op, double* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        double v = __hip_atomic_load(g.ws[0] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int r = 1; r < g.n; r++) {
            const double w = __hip_atomic_load(g.ws[r] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v = op ? fmax(v, w) : v + w;
        }
        out[i] = v;
    }
}


// Start of an LM iteration (G/core/optimization_algorithm_levenberg.cpp:61-90): currentChi
// from the linearisation's robust chi2 (red[0]), lambda from computeLambdaInit (red[1]) at it 0.
__device__ void lm_begin(LmState* st, double chi, double maxDiag) {
    st->pop = 0;
    st->currentChi = chi;
    st->iniChi = chi;
    if (st->it == 0) {
        st->lambda = 1e-5 * maxDiag;   // tau = 1e-5
        st->ni = 2;
        st->nBad = 0;
    }
    st->qmax = 0;
    st->phase = 1;
}
__global__ void k_lm_begin(LmState* st, const double* __restrict__ red) {
    if (threadIdx.x != 0 || st->phase != 0) return;
    lm_begin(st, red[0], red[1]);
}

// Decision after a trial (:120-160) and the end-of-iteration bookkeeping of
// SparseOptimizer::optimize / OptimizationAlgorithmLevenberg (termination on qmax == max
// trials, rho == 0 or three iterations without 1e-3 relative progress).
__device__ void lm_decide(LmState* st, double chiSum, double scaleSum, int fail, int maxTrials, int iterations,
                          int fixedIterations, double* __restrict__ trace, const uint32_t* stopWord,
                          double sharedStop) {
    const double tempChi = fail ? DBL_MAX : chiSum;
    double rho = st->currentChi - tempChi;
    const double scale = scaleSum + 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - cube_rn(2 * rho - 1);
        alpha = fmin(alpha, 2. / 3.);
        const double sf = fmax(1. / 3., alpha);
        st->lambda *= sf;
        st->ni = 2;
        st->currentChi = tempChi;
    } else {
        st->lambda *= st->ni;
        st->ni *= 2;
        st->pop = 1;
    }
    st->rho = rho;
    st->qmax++;
    st->trials++;
    const bool stopNow = lm_stop_now(st, stopWord, sharedStop);
    if (rho < 0 && st->qmax < maxTrials && !stopNow) return;   // next trial of this iteration
    const int row = st->traceBase + st->itersDone;
    if (trace && row < 64) {
        trace[4 * row] = st->iniChi;
        trace[4 * row + 1] = st->currentChi;
        trace[4 * row + 2] = st->lambda;
        trace[4 * row + 3] = st->qmax;
    }
    st->itersDone++;
    st->it++;
    bool go = true;
    if (!fixedIterations) {
        if (st->qmax == maxTrials || rho == 0) {
            go = false;
        } else {
            if ((st->iniChi - st->currentChi) * 1e3 < st->iniChi) st->nBad++;
            else st->nBad = 0;
            if (st->nBad >= 3) go = false;
        }
    }
    if (stopNow) st->stopped = 1;   // the iteration loop ends as well (sparse_optimizer.cpp:376)
    st->phase = (go && st->it < iterations && !stopNow) ? 0 : 2;
}
__global__ void k_lm_decide(LmState* st, const double* __restrict__ red, const int* __restrict__ flags, int maxTrials,
                            int iterations, int fixedIterations, double* __restrict__ trace) {
    if (threadIdx.x != 0) return;
    st->pop = 0;
    if (st->phase != 1) return;
    lm_decide(st, red[4], red[2], flags[0], maxTrials, iterations, fixedIterations, trace, nullptr, red[3]);
}

// Communicator path: this rank's stop sample into red[3], summed over the ranks with the scale
// term (red[2..3]) so every rank takes the same terminate() decision.
__global__ void k_stop_sample(const LmState* st, const uint32_t* __restrict__ word, double* __restrict__ red) {
    if (threadIdx.x != 0 || st->phase != 1) return;
    red[3] = (word && __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) ? 1.0 : 0.0;
}

// Single process: the start of an LM iteration in one wave — the linearisation's robust chi2
// (sum of k_edge_lin's per-wave partials), computeLambdaInit's max diagonal at iteration 0
// (k_vertex_reduce's per-block maxima) and lm_begin.
__global__ __launch_bounds__(64) void k_lm_begin_fused(LbaDev d, int nChi, int nMax) {
    LmState* st = d.lm;
    if (st->phase != 0) return;
    const int lane = threadIdx.x;
    double c = lane_sum(d.partChi, nChi, lane), m = lane_max(d.partMax, nMax, lane);
    c = wave_sum_d(c);
    m = wave_max_d(m);
    if (lane == 0) lm_begin(st, c, m);
}

// Single process: the end of an LM trial in one workgroup — the trial's robust chi2 and the
// scale x^T (lambda x + b) from the producers' partials, the rho decision (lm_decide) and,
// after a rejected trial, pop() of every free pose and owned point.
// With fused slots (`fuse`) it closes a group of slots: the last trial's pending decision.
__global__ __launch_bounds__(1024) void k_lm_decide_fused(LbaDev d, const int32_t* __restrict__ freePoses,
                                                          int maxTrials, int iterations, int fixedIterations,
                                                          double* __restrict__ trace, int nChi, int nScale, int fuse) {
    __shared__ int go, pop;
    LmState* st = d.lm;
    const int tid = threadIdx.x;
    if (fuse) {
        if (tid < 64 && st->pending) {
            const LmFuse f{nChi, nScale, maxTrials, iterations, fixedIterations, freePoses, trace};
            const LmState ls = lm_decide_local(d, f, tid, tid == 0);
            if (tid == 0) {
                *st = ls;
                pop = ls.pop;
            }
        } else if (tid == 0) {
            pop = 0;
        }
        __syncthreads();
        if (pop) lm_pop_slice(d, freePoses, tid, 1024);
        return;
    }
    if (tid == 0) {
        st->pop = 0;
        go = st->phase == 1;
        pop = 0;
    }
    __syncthreads();
    if (!go) return;
    if (tid < 64) {
        double c = lane_sum(d.partChi, nChi, tid), sc = lane_sum(d.partScale, nScale, tid);
        c = wave_sum_d(c);
        sc = wave_sum_d(sc);
        if (tid == 0) {
            lm_decide(st, c, sc, d.flags[0], maxTrials, iterations, fixedIterations, trace, d.stopWord, 0.0);
            pop = st->pop;
        }
    }
    __syncthreads();
    if (!pop) return;
    for (int i = tid; i < d.M; i += 1024) {
        const int g = d.ptGlob[i];
        for (int j = 0; j < 3; j++) d.X[3 * (size_t)g + j] = d.bX[3 * (size_t)g + j];
    }
    for (int i = tid; i < d.P; i += 1024) {
        const int p = freePoses[i];
        for (int j = 0; j < 4; j++) d.q[4 * p + j] = d.bq[4 * p + j];
        for (int j = 0; j < 3; j++) d.t[3 * p + j] = d.bt[3 * p + j];
    }
}

// Measurement hook (ORB_LBA_EXTRA_BOUNDARY=1): one empty 256-workgroup launch after each kernel of
// an LM slot, so the slot graph carries 5 more dependent kernel boundaries; the difference in solve
// time / (5 x slots) is what one boundary costs inside this graph.
__global__ __launch_bounds__(64) void k_nop() {}

__global__ __launch_bounds__(256) void k_lba_init(double* __restrict__ err, uint8_t* __restrict__ emask, int ne,
                                                  double* __restrict__ bq, const double* __restrict__ q,
                                                  double* __restrict__ bt, const double* __restrict__ t, int np,
                                                  int32_t* __restrict__ cnt, int ncnt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 3 * ne) err[i] = 0.0;
    if (i < ne) emask[i] = 1;
    if (i < 4 * np) bq[i] = q[i];
    if (i < 3 * np) bt[i] = t[i];
    if (i < ncnt) cnt[i] = 0;
}

constexpr int kStructHistMax = 4096;   // k_struct_count's LDS key histogram (ints)
constexpr int kSortReg = 16;           // k_struct_ptsort: landmark buckets ranked in registers
constexpr int kPoRun = 16;             // k_struct_po: consecutive entries per thread

// ---- The block structure of the first optimize() on the device (single process: every edge
//      is active at level 0, so act is the identity), the arrays build_csr (lba_host.h) makes on
//      the host from the vertex maps build_maps made: per edge its local landmark and pose index,
//      the CSR by landmark (entries ordered by (pose key, edge); key P = fixed pose) and the CSR
//      by free pose (entries in the landmark-major order of the first CSR).  Counts by atomics
//      (order-free), exclusive scans on one workgroup, the landmark buckets filled by atomics and
//      then sorted (a bucket holds one edge per observing keyframe), the pose buckets by one
//      workgroup per pose ranking its entries along the landmark-major list: the same arrays,
//      bit for bit, as the host build (checked by ORB_LBA_CHECK_STRUCT, tests/test_lba_gpu.py).
__global__ __launch_bounds__(256) void k_struct_count(const int32_t* __restrict__ ept, const int32_t* __restrict__ eps,
                                                      int ne, const int32_t* __restrict__ ptLocal,
                                                      const int32_t* __restrict__ poseIdx, int P,
                                                      int32_t* __restrict__ act, int32_t* __restrict__ actPt,
                                                      int32_t* __restrict__ actPi, int32_t* __restrict__ ptCnt,
                                                      int32_t* __restrict__ keyCnt, uint8_t* __restrict__ robust,
                                                      int robustFlag) {
    extern __shared__ int32_t hist[];   // P + 1 key counts when they fit (else global atomics)
    const int tid = threadIdx.x, k = blockIdx.x * 256 + tid;
    const bool lds = P + 1 <= kStructHistMax;
    if (lds) {
        for (int i = tid; i <= P; i += 256) hist[i] = 0;
        __syncthreads();
    }
    if (k < ne) {
        const int pt = ptLocal[ept[k]], pi = poseIdx[eps[k]];
        act[k] = k;
        actPt[k] = pt;
        actPi[k] = pi;
        robust[k] = (uint8_t)robustFlag;
        atomicAdd(ptCnt + pt, 1);
        if (lds) atomicAdd(hist + (pi < 0 ? P : pi), 1);
        else atomicAdd(keyCnt + (pi < 0 ? P : pi), 1);
    }
    if (lds) {
        __syncthreads();
        for (int i = tid; i <= P; i += 256)
            if (hist[i]) atomicAdd(keyCnt + i, hist[i]);
    }
}

// exclusive scan of v over a 1024-thread workgroup; *total = the sum (uniform)
__device__ __forceinline__ int blk_excl_scan(int v, int* wsum, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan_i32(v);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = 0, all = 0;
    for (int w = 0; w < 16; w++) {
        const int t = wsum[w];
        before += w < wave ? t : 0;
        all += t;
    }
    __syncthreads();
    total = all;
    return before + incl - v;
}

// ptStart[0..M] and poStart[0..P] (kStart of the host build) by exclusive scans
__global__ __launch_bounds__(1024) void k_struct_scan(const int32_t* __restrict__ ptCnt, int M,
                                                      const int32_t* __restrict__ keyCnt, int P,
                                                      int32_t* __restrict__ ptStart, int32_t* __restrict__ poStart) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x;
    int carry = 0;
    for (int i0 = 0; i0 <= M; i0 += 1024) {
        const int i = i0 + tid, v = i < M ? ptCnt[i] : 0;
        int tot;
        const int ex = blk_excl_scan(v, wsum, tot);
        if (i <= M) ptStart[i] = carry + ex;
        carry += tot;
    }
    carry = 0;
    for (int i0 = 0; i0 <= P; i0 += 1024) {
        const int i = i0 + tid, v = i < P ? keyCnt[i] : 0;
        int tot;
        const int ex = blk_excl_scan(v, wsum, tot);
        if (i <= P) poStart[i] = carry + ex;
        carry += tot;
    }
}

// the landmark buckets: entries in arrival order, then each bucket sorted by (pose key, edge)
__global__ __launch_bounds__(256) void k_struct_pt(int ne, const int32_t* __restrict__ actPt,
                                                   const int32_t* __restrict__ ptStart, int32_t* __restrict__ ptFill,
                                                   int32_t* __restrict__ ptAct) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= ne) return;
    const int pt = actPt[k];
    ptAct[ptStart[pt] + atomicAdd(ptFill + pt, 1)] = k;
}
// ... and each landmark-major entry's pose key and landmark (piT, ptT) for k_struct_po
__global__ __launch_bounds__(256) void k_struct_ptsort(int M, int P, const int32_t* __restrict__ ptStart,
                                                       const int32_t* __restrict__ actPi, int32_t* __restrict__ ptAct,
                                                       int32_t* __restrict__ piT, int32_t* __restrict__ ptT) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= M) return;
    const int b = ptStart[m], e = ptStart[m + 1], n = e - b;
    if (n <= 0) return;
    auto key = [&](int k) { const int pi = actPi[k]; return ((long long)(pi < 0 ? P : pi) << 32) | (unsigned)k; };
    if (n <= kSortReg) {   // ranks in registers: every load in flight at once, keys are distinct
        int kv[kSortReg];
        long long kk[kSortReg];
#pragma unroll
        for (int i = 0; i < kSortReg; i++) kv[i] = ptAct[b + min(i, n - 1)];
#pragma unroll
        for (int i = 0; i < kSortReg; i++) kk[i] = key(kv[i]);   // unconditional (clamped index): no
#pragma unroll                                                       // exec-masked load chain
        for (int i = 0; i < kSortReg; i++) kk[i] = i < n ? kk[i] : LLONG_MAX;
#pragma unroll
        for (int i = 0; i < kSortReg; i++) {
            int r = 0;
#pragma unroll
            for (int j = 0; j < kSortReg; j++) r += kk[j] < kk[i] ? 1 : 0;
            if (i < n) {
                ptAct[b + r] = kv[i];
                piT[b + r] = (int)(kk[i] >> 32);
                ptT[b + r] = m;
            }
        }
        return;
    }
    for (int i = b + 1; i < e; i++) {   // a landmark seen by more keyframes: insertion sort
        const int k = ptAct[i];
        const long long kk = key(k);
        int j = i - 1;
        while (j >= b && key(ptAct[j]) > kk) {
            ptAct[j + 1] = ptAct[j];
            j--;
        }
        ptAct[j + 1] = k;
    }
    for (int i = b; i < e; i++) {
        piT[i] = (int)(key(ptAct[i]) >> 32);
        ptT[i] = m;
    }
}
// the pose buckets: workgroup i ranks the entries of pose i along the landmark-major list, each
// thread a run of kPoRun consecutive entries (their pose keys and landmarks from
// k_struct_ptsort: contiguous 16-byte loads, no gathers), one scan per pass
__global__ __launch_bounds__(1024) void k_struct_po(int na, const int32_t* __restrict__ ptAct,
                                                    const int32_t* __restrict__ piT, const int32_t* __restrict__ ptT,
                                                    const int32_t* __restrict__ poStart, int32_t* __restrict__ poAct,
                                                    int32_t* __restrict__ poPt) {
    __shared__ int wsum[16];
    const int i = blockIdx.x, tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rk = buf_rsrc(ptAct, (uint32_t)na * 4), rp = buf_rsrc(piT, (uint32_t)na * 4),
                                 rl = buf_rsrc(ptT, (uint32_t)na * 4);
    int at = poStart[i];
    for (int t0 = 0; t0 < na; t0 += 1024 * kPoRun) {
        const int tb = t0 + tid * kPoRun;
        int kv[kPoRun], pi[kPoRun], pt[kPoRun];
        typedef int i32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int u = 0; u < kPoRun; u += 4) {   // past the end: the buffer resource reads 0
            const i32x4 a = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, (tb + u) * 4, 0, 0));
            const i32x4 b = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (tb + u) * 4, 0, 0));
            const i32x4 c = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, (tb + u) * 4, 0, 0));
#pragma unroll
            for (int q = 0; q < 4; q++) { kv[u + q] = a[q]; pi[u + q] = b[q]; pt[u + q] = c[q]; }
        }
        unsigned mine = 0;
#pragma unroll
        for (int u = 0; u < kPoRun; u++) mine |= (tb + u < na && pi[u] == i) ? 1u << u : 0u;
        int tot;
        int pos = at + blk_excl_scan(__popc(mine), wsum, tot);
#pragma unroll
        for (int u = 0; u < kPoRun; u++)
            if ((mine >> u) & 1u) {
                poAct[pos] = kv[u];
                poPt[pos] = pt[u];
                pos++;
            }
        at += tot;
    }
}

// The outlier pass between the two optimize() rounds (R/src/Optimizer.cpp:805-836) on the
// device: every active edge of a good point whose chi2 (k_readback) exceeds the threshold or
// whose depth is not positive leaves the optimisation (level 1 -> emask 0), and every edge of a
// good point loses its robust kernel.  The block structure is kept: a level-1 edge contributes
// exact zeros, so a vertex left without active edges keeps a decoupled lambda-only block and
// a zero step, as g2o leaves an inactive vertex untouched.
__global__ __launch_bounds__(256) void k_outlier_mask(LbaDev d, const double* __restrict__ chi2,
                                                      const uint8_t* __restrict__ depthPos, double thMono,
                                                      double thStereo) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= d.nact) return;
    const int e = d.act[k];
    if (d.bad && d.bad[d.ept[e]]) return;
    const double thr = d.est[e] ? thStereo : thMono;
    if (chi2[e] > thr || !depthPos[e]) d.emask[e] = 0;
    d.robust[e] = 0;
}

// chi2 / depth of every edge (final check and outlier pass): chi2() uses the stored error

// What the host reads after an optimize() (the final check, R/src/Optimizer.cpp:850-880, and the
// write-back): per edge the chi2 and the depth test (kept on the device too, for
// k_outlier_mask), the estimates q | t | X and the LM state, stored by the kernel straight into
// host-coherent pinned memory: no copy commands.  Queued speculatively behind every group of LM
// slots (the host reads it once the state says the loop is over).
__global__ __launch_bounds__(256) void k_readback(LbaDev d, int ne, double* __restrict__ chi2,
                                                  uint8_t* __restrict__ depthPos, char* __restrict__ h, size_t estOff,
                                                  size_t offT, size_t offX, int np, int nm, size_t lmOff,
                                                  const double* __restrict__ trace, size_t traceOff) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 4 * 64) reinterpret_cast<double*>(h + traceOff)[i] = trace[i];
    if (i < ne) {
        const double c2 = d_edge_chi2(d, i);
        double Xc[3];
        d_transform(d, d.eps[i], d.ept[i], Xc);
        const uint8_t dp = Xc[2] > 0.0 ? 1 : 0;
        chi2[i] = c2;
        depthPos[i] = dp;
        reinterpret_cast<double*>(h)[i] = c2;
        reinterpret_cast<uint8_t*>(h + 8 * (size_t)ne)[i] = dp;
    }
    if (i < 4 * np) reinterpret_cast<double*>(h + estOff)[i] = d.q[i];
    if (i < 3 * np) reinterpret_cast<double*>(h + estOff + offT)[i] = d.t[i];
    if (i < 3 * nm) reinterpret_cast<double*>(h + estOff + offX)[i] = d.X[i];
    if (i < (int)(sizeof(LmState) / 4)) reinterpret_cast<int*>(h + lmOff)[i] = reinterpret_cast<const int*>(d.lm)[i];
}

}  // namespace orbamd

using namespace orbamd;

// ------------------------------------------------------------------ host side

// Keep in sync with lba_problem / lba_options / lba_result in include/orbslam2_amd.h.
struct lba_context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool ownStream = true;
    // communicator
    int rank = 0, world = 1;
    double* ws = nullptr;          // caller-owned device workspace (doubles)
    double* wsOut = nullptr;       // where a collective leaves its result (NULL: in place in ws)
    size_t wsDoubles = 0;
    lba_allreduce_fn allreduce = nullptr;
    void* commUser = nullptr;
    const orbamd::GrpDev* grp = nullptr;   // device-side exchange (lba_group): replaces the callback
    bool grpGraphs = false;                // ... and its slots may be graph-captured (every rank on its own device)
    std::vector<int32_t> gflagStage;       // the global pair flags of the last solve (packed exchange)
    // device buffers: a grow-only arena reused across solves (hipMalloc / hipFree per buffer
    // and per call cost more than a small LBA's whole LM loop; hipFree also synchronises)
    std::vector<std::pair<char*, size_t>> chunks;   // (base, size); the last one is bumped
    size_t used = 0, usedTotal = 0, peak = 0;
    // stats
    double ms_linearize = 0, ms_schur = 0, ms_solve = 0, ms_update = 0;
    int n_iters = 0, n_trials = 0;
    bool profile = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // stage timing
    hipEvent_t evSync = nullptr;                               // LM decision hand-off
    double* h_scal = nullptr;                                  // pinned LM scalars / state (4 KB)
    // terminate(): the caller's stop flag (mbAbortBA) mirrored into a host-mapped word the LM
    // decision kernels read after every trial; lba_wait copies it while the host waits
    uint32_t* h_stop = nullptr;
    uint32_t* d_stop = nullptr;
    const volatile uint8_t* stopSrc = nullptr;
    int stopAfter = -1;                                        // test hook (lba_debug_stop_after_trials)
    orbamd::LbaDev last{};                                     // device buffers of the last solve (lba_debug_buffer)
    std::vector<hipEvent_t> slotEv;                            // per-slot stage timing
    // grow-only pinned staging: [0] problem upload, [1] per-optimize() structure, [2] downloads
    char* stage[3] = {nullptr, nullptr, nullptr};
    char* stageDev[3] = {nullptr, nullptr, nullptr};   // device address of a mapped (coherent) slot
    size_t stageCap[3] = {0, 0, 0};
    // instantiated LM-slot graphs keyed by every captured launch parameter: a solve of the same
    // shape reuses them (the arena hands out the same addresses in the same order)
    struct SlotGraph {
        std::vector<char> key;
        hipGraphExec_t exec = nullptr;
    };
    std::vector<SlotGraph> graphs;
};

// Resets the arena for a new solve; if the last solve spilled into several chunks, they are
// replaced by one chunk of the peak size (the device is idle between solves).
static void lba_free_all(lba_context* c) {
    if (c->chunks.size() > 1) {
        for (auto& ch : c->chunks) (void)hipFree(ch.first);
        c->chunks.clear();
        char* p = nullptr;
        if (hipMalloc((void**)&p, c->peak) == hipSuccess) c->chunks.push_back({p, c->peak});
    }
    c->used = 0;
    c->usedTotal = 0;
}

static void lba_release(lba_context* c) {
    for (auto& ch : c->chunks) (void)hipFree(ch.first);
    c->chunks.clear();
    c->used = c->usedTotal = c->peak = 0;
}

template <typename T>
static int dalloc(lba_context* c, T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    const size_t bytes = (n * sizeof(T) + 255) & ~(size_t)255;
    if (c->chunks.empty() || c->used + bytes > c->chunks.back().second) {
        const size_t prev = c->chunks.empty() ? 0 : c->chunks.back().second;
        const size_t sz = std::max(bytes, std::max((size_t)4 << 20, 2 * prev));
        char* base = nullptr;
        if (hipMalloc((void**)&base, sz) != hipSuccess) return ORB_ENOMEM;
        c->chunks.push_back({base, sz});
        c->used = 0;
    }
    *p = reinterpret_cast<T*>(c->chunks.back().first + c->used);
    c->used += bytes;
    c->usedTotal += bytes;
    c->peak = std::max(c->peak, c->usedTotal);
    return ORB_OK;
}

#define TRY(x)                 \
    do {                       \
        int s_ = (x);          \
        if (s_) return s_;     \
    } while (0)

// buffers of the multi-workgroup reduced solve for orders up to nMax (k_ldlt_mw_*); the order
// itself is set per solve.  Used above the LDS image unless ORB_LBA_LDLT_SINGLE selects the
// one-workgroup global-memory k_ldlt_solve<false> (kept for A/B runs).
static bool use_mw(int np) { return np > kLdlLdsMaxN && !std::getenv("ORB_LBA_LDLT_SINGLE"); }
static int mw_alloc(lba_context* c, int nMax, MwLdl* m) {
    std::memset(m, 0, sizeof(*m));
    const size_t np = ((size_t)nMax + kMwNB - 1) & ~(size_t)(kMwNB - 1);
    TRY(dalloc(c, &m->A, np * np)); TRY(dalloc(c, &m->rdg, np)); TRY(dalloc(c, &m->y, np));
    TRY(dalloc(c, &m->yfin, np)); TRY(dalloc(c, &m->Ldg, np * kMwNB)); TRY(dalloc(c, &m->sink, kMwNB * np + 64));
    TRY(dalloc(c, &m->yb, np));
    TRY(dalloc(c, &m->fail, 1));
    return ORB_OK;
}
static MwLdl mw_order(MwLdl m, int n) {
    m.n = n;
    m.np = (n + kMwNB - 1) & ~(kMwNB - 1);
    return m;
}

// Pinned staging slot; `mapped`: host-coherent memory the kernels store into directly (slot 2,
// the post-optimize read-back)
static int stage_reserve(lba_context* c, int slot, size_t bytes, bool mapped = false) {
    if (c->stageCap[slot] >= bytes) return ORB_OK;
    if (c->stage[slot]) (void)hipHostFree(c->stage[slot]);
    c->stage[slot] = c->stageDev[slot] = nullptr;
    c->stageCap[slot] = 0;
    const size_t cap = std::max(bytes + bytes / 2, (size_t)1 << 16);
    const unsigned flags = mapped ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault;
    if (hipHostMalloc((void**)&c->stage[slot], cap, flags) != hipSuccess) return ORB_ENOMEM;
    if (mapped && hipHostGetDevicePointer((void**)&c->stageDev[slot], c->stage[slot], 0) != hipSuccess) {
        (void)hipHostFree(c->stage[slot]);
        c->stage[slot] = nullptr;
        return ORB_ENOMEM;
    }
    c->stageCap[slot] = cap;
    return ORB_OK;
}

// Host-to-device batch: the arrays are packed at 256-byte offsets into pinned staging slot
// `slot` and sent with one copy into one arena block (a pageable copy costs ~10 us each).  A
// slot is reused only after the stream has passed its previous copy (every caller waits on
// the stream between two uses of the same slot).
struct UpItem {
    void** dst;
    const void* src;
    size_t bytes;
};
static int upload_batch(lba_context* c, int slot, const std::vector<UpItem>& items) {
    size_t total = 0;
    for (const auto& it : items) total += (it.bytes + 255) & ~(size_t)255;
    char* dbase = nullptr;
    TRY(dalloc(c, &dbase, std::max<size_t>(total, 1)));
    TRY(stage_reserve(c, slot, total));
    size_t off = 0;
    for (const auto& it : items) {
        if (it.bytes) std::memcpy(c->stage[slot] + off, it.src, it.bytes);
        *it.dst = dbase + off;
        off += (it.bytes + 255) & ~(size_t)255;
    }
    // (one copy: sending it in pieces as the staging fills measured no faster, 128-384 KB pieces)
    if (total) ORB_HIP_TRY(hipMemcpyAsync(dbase, c->stage[slot], total, hipMemcpyHostToDevice, c->stream));
    return ORB_OK;
}
template <typename T>
static UpItem up(T** dst, const std::vector<T>& v) {
    return UpItem{reinterpret_cast<void**>(dst), v.data(), v.size() * sizeof(T)};
}
template <typename T>
static UpItem up(T** dst, const T* src, size_t n) {
    return UpItem{reinterpret_cast<void**>(dst), src, n * sizeof(T)};
}

// Waits for the stream by spinning on an event (a blocking hipStreamSynchronize sleeps and
// adds tens of microseconds per LM trial).
static inline void mirror_stop(lba_context* c) {
    if (c->stopSrc && *c->stopSrc && c->h_stop && !__atomic_load_n(c->h_stop, __ATOMIC_RELAXED))
        __atomic_store_n(c->h_stop, 1u, __ATOMIC_RELEASE);
}
static int lba_wait(lba_context* c) {
    if (hipEventRecord(c->evSync, c->stream) != hipSuccess) return ORB_EGPU;
    hipError_t e;
    while ((e = hipEventQuery(c->evSync)) == hipErrorNotReady) mirror_stop(c);
    return e == hipSuccess ? ORB_OK : ORB_EGPU;
}


namespace {



template <typename T>
int upload(lba_context* c, T** dst, const std::vector<T>& v) {
    TRY(dalloc(c, dst, v.size()));
    if (!v.empty()) ORB_HIP_TRY(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return ORB_OK;
}

}  // namespace

// All-reduce of an LM-loop buffer: staged through the workspace by guarded kernels, so a
// slot whose phase is skipped reduces zeros and leaves the buffer alone.
// the device-side collective of a group over the first n doubles of the ranks' workspaces
static int grp_exchange(lba_context* c, size_t n, int op) {
    const orbamd::GrpDev& g = *c->grp;
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(1024, (n + 255) / 256));
    hipLaunchKernelGGL(k_grp_sync, dim3(1), dim3(64), 0, c->stream, g, 0);
    hipLaunchKernelGGL(k_grp_reduce, dim3(blocks), dim3(256), 0, c->stream, g, n, op, c->wsOut);
    hipLaunchKernelGGL(k_grp_sync, dim3(1), dim3(64), 0, c->stream, g, 1);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

// Several buffers with the same op ride in one collective (packed back to back in the workspace):
// a collective costs far more than the pack / unpack launches around it.
struct CommSeg {
    double* p;
    size_t n;
};
static int comm_allreduce_segs(lba_context* c, std::initializer_list<CommSeg> segs, int op, const LmState* st, int want) {
    if (c->world <= 1) return ORB_OK;
    size_t tot = 0;
    for (const CommSeg& sg : segs) tot += sg.n;
    if ((!c->allreduce && !c->grp) || !c->ws || tot > c->wsDoubles) return ORB_EINVAL;
    size_t off = 0;
    for (const CommSeg& sg : segs) {
        const unsigned g = (unsigned)std::min<size_t>(1024, (sg.n + 255) / 256);
        if (c->grp) hipLaunchKernelGGL(k_pack_sys, dim3(g), dim3(256), 0, c->stream, c->ws + off, sg.p, sg.n, st, want);
        else hipLaunchKernelGGL(k_pack, dim3(g), dim3(256), 0, c->stream, c->ws + off, sg.p, sg.n, st, want);
        off += sg.n;
    }
    if (c->grp) {
        TRY(grp_exchange(c, tot, op));
    } else if (c->allreduce(c->commUser, 0, tot, op) != 0) {
        return ORB_EGPU;
    }
    const double* res = c->wsOut ? c->wsOut : c->ws;
    off = 0;
    for (const CommSeg& sg : segs) {
        const unsigned g = (unsigned)std::min<size_t>(1024, (sg.n + 255) / 256);
        hipLaunchKernelGGL(k_unpack, dim3(g), dim3(256), 0, c->stream, sg.p, res + off, sg.n, st, want);
        off += sg.n;
    }
    return ORB_OK;
}
static int comm_allreduce_g(lba_context* c, double* dbuf, size_t n, int op, const LmState* st, int want) {
    return comm_allreduce_segs(c, {CommSeg{dbuf, n}}, op, st, want);
}
// S + b_s over the communicator as the G listed pair blocks + b_s (k_pack_pairs)
static int comm_allreduce_schur(lba_context* c, double* S, double* bs, const int32_t* pairs, int G, int P,
                                const LmState* st, int want) {
    if (c->world <= 1) return ORB_OK;
    const size_t tot = 36 * (size_t)G + 6 * (size_t)P;
    if ((!c->allreduce && !c->grp) || !c->ws || tot > c->wsDoubles) return ORB_EINVAL;
    const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>(1024, (tot + 255) / 256));
    if (c->grp) hipLaunchKernelGGL(k_pack_pairs<true>, dim3(g), dim3(256), 0, c->stream, c->ws, S, bs, pairs, G, P, st, want);
    else hipLaunchKernelGGL(k_pack_pairs<false>, dim3(g), dim3(256), 0, c->stream, c->ws, S, bs, pairs, G, P, st, want);
    if (c->grp) {
        TRY(grp_exchange(c, tot, 0));
    } else if (c->allreduce(c->commUser, 0, tot, 0) != 0) {
        return ORB_EGPU;
    }
    const double* res = c->wsOut ? c->wsOut : c->ws;
    hipLaunchKernelGGL(k_unpack_pairs, dim3(g), dim3(256), 0, c->stream, S, bs, res, pairs, G, P, st, want);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

extern "C" {

int lba_create(int device, lba_context** out) try {
    if (!out) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    ORB_HIP_TRY(hipSetDevice(device));
    lba_context* c = new lba_context();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return ORB_EGPU; }
    bool ok = hipEventCreateWithFlags(&c->evSync, hipEventDisableTiming) == hipSuccess &&
              hipHostMalloc((void**)&c->h_scal, 4096, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void**)&c->h_stop, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
              hipHostGetDevicePointer((void**)&c->d_stop, c->h_stop, 0) == hipSuccess;
    if (c->h_stop) *c->h_stop = 0;
    for (auto& e : c->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) { lba_destroy(c); return ORB_EGPU; }
    *out = c;
    return ORB_OK;
} ORB_ABI_CATCH

void lba_destroy(lba_context* c) try {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    lba_release(c);
    for (auto e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->evSync) (void)hipEventDestroy(c->evSync);
    for (auto e : c->slotEv) (void)hipEventDestroy(e);
    if (c->h_scal) (void)hipHostFree(c->h_scal);
    if (c->h_stop) (void)hipHostFree(c->h_stop);
    for (auto p : c->stage)
        if (p) (void)hipHostFree(p);
    for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    if (c->stream && c->ownStream) (void)hipStreamDestroy(c->stream);
    delete c;
} ORB_ABI_CATCH_VOID

int lba_set_stream(lba_context* c, void* stream, int use_given) try {
    if (!c) return ORB_EINVAL;
    if (c->stream && c->ownStream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    c->stream = nullptr;
    if (use_given) {   // NULL = the device's legacy default stream
        c->stream = (hipStream_t)stream;
        c->ownStream = false;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return ORB_EGPU;
        c->ownStream = true;
    }
    return ORB_OK;
} ORB_ABI_CATCH

int lba_set_comm(lba_context* c, int rank, int world, double* d_workspace, size_t ws_doubles, lba_allreduce_fn fn,
                 void* user) try {
    if (!c || world < 1 || rank < 0 || rank >= world) return ORB_EINVAL;
    if (world > 1 && (!d_workspace || !fn)) return ORB_EINVAL;
    c->rank = rank;
    c->world = world;
    c->ws = d_workspace;
    c->wsDoubles = ws_doubles;
    c->allreduce = fn;
    c->commUser = user;
    c->grp = nullptr;   // (lba_group installs its device-side exchange after this call)
    c->grpGraphs = false;
    return ORB_OK;
} ORB_ABI_CATCH

int lba_stats(lba_context* c, double* ms4, int* iters, int* trials) try {
    if (!c) return ORB_EINVAL;
    if (ms4) { ms4[0] = c->ms_linearize; ms4[1] = c->ms_schur; ms4[2] = c->ms_solve; ms4[3] = c->ms_update; }
    if (iters) *iters = c->n_iters;
    if (trials) *trials = c->n_trials;
    return ORB_OK;
} ORB_ABI_CATCH

int lba_dense_solve(lba_context* c, const double* S, const double* b, int n, double* x) try {
    if (!c || !S || !b || !x || n <= 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(c->device));
    lba_free_all(c);
    hipStream_t s = c->stream;
    const int np = (n + kNB - 1) & ~(kNB - 1);
    double *dS, *db, *dx, *dw = nullptr;
    int* df;
    TRY(dalloc(c, &dS, (size_t)n * n)); TRY(dalloc(c, &db, n)); TRY(dalloc(c, &dx, n)); TRY(dalloc(c, &df, 1));
    MwLdl mw{};
    if (use_mw(np)) TRY(mw_alloc(c, n, &mw));
    else if (np > kLdlLdsMaxN) TRY(dalloc(c, &dw, (size_t)np * (np + 1)));
    ORB_HIP_TRY(hipMemcpyAsync(dS, S, 8 * (size_t)n * n, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(db, b, 8 * (size_t)n, hipMemcpyHostToDevice, s));
    if (use_mw(np))
        enqueue_ldlt_mw(s, mw_order(mw, n), dS, db, dx, df, nullptr, PoseTail{});
    else if (use_ldlt_df(n))
        hipLaunchKernelGGL(k_ldlt_df, dim3(1), dim3(kLdlT), ldlt_df_lds_bytes(n), s, dS, db, n, dx, df, nullptr, PoseTail{});
    else if (np <= kLdlLdsMaxN)
        hipLaunchKernelGGL(k_ldlt_solve<true>, dim3(1), dim3(kLdlT), ((size_t)np * (np + 1) + 3 * (size_t)np + 256 + (size_t)kNB * (np + 1) + 64) * 8, s,
                           dS, db, n, nullptr, dx, df, nullptr, PoseTail{});
    else
        hipLaunchKernelGGL(k_ldlt_solve<false>, dim3(1), dim3(kLdlT), (3 * (size_t)np + 64) * 8, s, dS, db, n, dw, dx, df,
                           nullptr, PoseTail{});
    ORB_HIP_TRY(hipGetLastError());
    int fail = 0;
    ORB_HIP_TRY(hipMemcpyAsync(x, dx, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipMemcpyAsync(&fail, df, 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipStreamSynchronize(s));
    return fail ? ORB_EINVAL : ORB_OK;
} ORB_ABI_CATCH

int lba_debug_stop_after_trials(lba_context* c, int n_trials) try {
    if (!c) return ORB_EINVAL;
    c->stopAfter = n_trials < 0 ? -1 : n_trials;
    return ORB_OK;
} ORB_ABI_CATCH

int lba_debug_buffer(lba_context* c, int which, double* out, size_t n) try {
    if (!c || !out) return ORB_EINVAL;
    const LbaDev& d = c->last;
    const double* src = nullptr;
    size_t avail = 0;
    const size_t P = (size_t)d.P, M = (size_t)d.M;
    switch (which) {
        case 0: src = d.S; avail = 36 * P * P; break;
        case 1: src = d.bs; avail = 6 * P; break;
        case 2: src = d.x; avail = 6 * P + 3 * M; break;
        case 3: src = d.Hpp; avail = 36 * P; break;
        case 4: src = d.bp; avail = 6 * P; break;
        case 5: src = d.Hll; avail = 9 * M; break;
        case 6: src = d.bl; avail = 3 * M; break;
        case 7: src = d.Dinv; avail = 9 * M; break;
        default: return ORB_EINVAL;
    }
    if (!src || n > avail) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(c->device));
    ORB_HIP_TRY(hipMemcpyAsync(out, src, 8 * n, hipMemcpyDeviceToHost, c->stream));   // own stream (§8b threading)
    ORB_HIP_TRY(hipStreamSynchronize(c->stream));
    return (int)avail;
} ORB_ABI_CATCH

int lba_profile(lba_context* c, int enable) try {
    if (!c) return ORB_EINVAL;
    c->profile = enable != 0;
    c->ms_linearize = c->ms_schur = c->ms_solve = c->ms_update = 0;
    c->n_iters = c->n_trials = 0;
    return ORB_OK;
} ORB_ABI_CATCH

void lba_pose_from_Tcw(const float Tcw[16], double q[4], double t[3]) try {
    // Converter::toSE3Quat (R/src/Converter.cpp:47-57): float Mat -> Matrix3d -> SE3Quat
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)Tcw[i * 4 + j];
    hd_quat_from_matrix(R, q);
    for (int i = 0; i < 3; i++) t[i] = (double)Tcw[i * 4 + 3];
} ORB_ABI_CATCH_VOID

void lba_poses_from_Tcw(const float* Tcw, int n, double* q, double* t) try {
    for (int i = 0; i < n; i++) lba_pose_from_Tcw(Tcw + 16 * (size_t)i, q + 4 * (size_t)i, t + 3 * (size_t)i);
} ORB_ABI_CATCH_VOID

void lba_pose_to_Tcw(const double q[4], const double t[3], float Tcw[16]) try {
    // Converter::toCvMat(SE3Quat): to_homogeneous_matrix() cast to float
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                         txz - twy, tyz + twx, 1 - (txx + tyy)};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Tcw[i * 4 + j] = (float)R[i * 3 + j];
        Tcw[i * 4 + 3] = (float)t[i];
    }
    Tcw[12] = Tcw[13] = Tcw[14] = 0.f;
    Tcw[15] = 1.f;
} ORB_ABI_CATCH_VOID

// slots per captured LM graph (see optimize())
constexpr int kGraphSlots = 16;

static int lba_run(lba_context* c, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop,
                   lba_result* r, bool global, bool robustKernels);

int lba_solve(lba_context* c, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop, lba_result* r) try {
    return lba_run(c, p, o, stop, r, false, true);
} ORB_ABI_CATCH

int lba_solve_global(lba_context* c, const lba_problem* p, const lba_options* o, int robust,
                     const volatile uint8_t* stop, lba_result* r) try {
    return lba_run(c, p, o, stop, r, true, robust != 0);
} ORB_ABI_CATCH

static int lba_run(lba_context* c, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop,
                   lba_result* r, bool global, bool robustKernels) {
#ifdef ORB_TIMING
    const auto hEntry = std::chrono::steady_clock::now();
#endif
    if (!c || !p || !o || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0) return ORB_EINVAL;
    const int NP = p->n_poses, NM = p->n_points, NE = p->n_edges;
    if ((NP > 0 && (!p->pose_q || !p->pose_t || !p->pose_fixed || !p->pose_id)) ||
        (NM > 0 && (!p->point_xyz || !p->point_id)) ||
        (NE > 0 && (!p->edge_point || !p->edge_pose || !p->edge_stereo || !p->edge_obs || !p->edge_info ||
                    !p->edge_cam)))
        return ORB_EINVAL;
    for (int e = 0; e < NE; e++)   // every index the structure build and the kernels dereference
        if (p->edge_point[e] < 0 || p->edge_point[e] >= NM || p->edge_pose[e] < 0 || p->edge_pose[e] >= NP)
            return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    r->iterations[0] = r->iterations[1] = 0;
    r->trials = 0;
    r->n_trace = 0;
    r->aborted = 0;
    struct StopScope {   // the stop mirror is live for this call only
        lba_context* c;
        ~StopScope() { c->stopSrc = nullptr; }
    } stopScope{c};
    c->stopSrc = stop;
    __atomic_store_n(c->h_stop, (stop && *stop) ? 1u : 0u, __ATOMIC_RELEASE);
    auto stopped = [&]() { return (stop && *stop) || (c->stopAfter >= 0 && r->trials >= c->stopAfter); };
    // with a communicator every rank must take the same stop decision: a rank's flag is summed
    // over the ranks (the decision points are rare: entry, after each optimize())
    auto agreed = [&](bool mine, bool* out) -> int {
        *out = mine;
        if (c->world <= 1) return ORB_OK;
        if ((!c->allreduce && !c->grp) || !c->ws || c->wsDoubles < 1) return ORB_EINVAL;
        double* h = c->h_scal + 256;
        h[0] = mine ? 1.0 : 0.0;
        ORB_HIP_TRY(hipMemcpyAsync(c->ws, h, 8, hipMemcpyHostToDevice, s));
        TRY(lba_wait(c));
        if (c->grp) TRY(grp_exchange(c, 1, 0));
        else if (c->allreduce(c->commUser, 0, 1, 0) != 0) return ORB_EGPU;
        ORB_HIP_TRY(hipMemcpyAsync(h, c->wsOut ? c->wsOut : c->ws, 8, hipMemcpyDeviceToHost, s));
        TRY(lba_wait(c));
        *out = h[0] > 0.5;
        return ORB_OK;
    };
    bool stopEntry = false;
    TRY(agreed(!global && stop && *stop, &stopEntry));
    if (stopEntry) {   // R/src/Optimizer.cpp:784-786: return before optimizing, no write-back
        r->aborted = 1;
        return ORB_OK;
    }
    lba_free_all(c);
    std::memset(&c->last, 0, sizeof(c->last));   // lba_debug_buffer: no pointers into a freed arena
    // single process: the edge-level part of the block structure is built on the device
    // (k_struct_*); with a communicator (owned landmark ranges) on the host
    const bool devStruct = c->world == 1 && NE > 0 && !std::getenv("ORB_LBA_HOST_STRUCT");
    std::vector<uint8_t> level(NE, 0);
    HostStructure hs;
    int gPairs = 0;   // with a communicator: the global pair list's length (the packed exchange)
    int32_t* d_freePoses = nullptr;
    int32_t *d_poseIdx0 = nullptr, *d_ptLocal0 = nullptr, *d_ptGlob0 = nullptr;
    LbaDev d;
    std::memset(&d, 0, sizeof(d));
    double *q, *t, *X, *obs, *info, *cam;
    uint8_t *fixed, *est, *robust = nullptr;
    int32_t *ept, *eps;
    TRY(dalloc(c, &d.bq, 4 * (size_t)NP)); TRY(dalloc(c, &d.bt, 3 * (size_t)NP)); TRY(dalloc(c, &d.bX, 3 * (size_t)NM));
    TRY(dalloc(c, &d.err, 3 * (size_t)NE));
    uint8_t* bad = nullptr;
    {   // one pinned batch (q, t, X first and contiguous: the estimates come back the same way)
        std::vector<UpItem> items{up(&q, p->pose_q, 4 * (size_t)NP), up(&t, p->pose_t, 3 * (size_t)NP),
                                  up(&X, p->point_xyz, 3 * (size_t)NM), up(&fixed, p->pose_fixed, NP),
                                  up(&ept, p->edge_point, NE), up(&eps, p->edge_pose, NE),
                                  up(&est, p->edge_stereo, NE), up(&obs, p->edge_obs, 3 * (size_t)NE),
                                  up(&info, p->edge_info, NE), up(&cam, p->edge_cam, 5 * (size_t)NE)};
        if (p->point_bad && NM > 0) items.push_back(up(&bad, p->point_bad, NM));
        if (devStruct) {   // the vertex maps of the first optimize() (host, O(NE) flags + the id order)
            build_maps(p, level, 0, 0, 1, hs, false);
            items.push_back(up(&d_poseIdx0, hs.poseIdx));
            items.push_back(up(&d_ptLocal0, hs.ptLocal));
            items.push_back(up(&d_ptGlob0, hs.ptGlob));
            items.push_back(up(&d_freePoses, hs.freePoses));
        }
        TRY(upload_batch(c, 0, items));
    }
    // one launch: the errors zeroed, every edge at level 0 for the first optimize(), the push()
    // backups start as the estimates (a fixed pose's backup then always equals its never updated
    // estimate, which the fused linearisation after a pop reads, k_edge_lin), and the device
    // structure build's counters zeroed
    TRY(dalloc(c, &d.emask, std::max(NE, 1)));
    int32_t* d_structCnt = nullptr;   // k_struct_*: ptCnt [M], ptFill [M], keyCnt [P + 1]
    const int nCnt = devStruct ? 2 * hs.M + hs.P + 1 : 0;
    if (devStruct) TRY(dalloc(c, &d_structCnt, nCnt));
    hipLaunchKernelGGL(k_lba_init, dim3(std::max(1, (std::max({3 * NE, 4 * NP, nCnt}) + 255) / 256)), dim3(256), 0, s,
                       d.err, d.emask, NE, d.bq, q, d.bt, t, NP, d_structCnt, nCnt);
    ORB_HIP_TRY(hipGetLastError());
    d.q = q; d.t = t; d.X = X; d.fixed = fixed; d.ept = ept; d.eps = eps; d.est = est; d.obs = obs; d.info = info;
    d.cam = cam; d.robust = robust;
    d.bad = bad;
    d.stopWord = c->d_stop;
    // per-edge / per-vertex scratch sized for the full problem
    TRY(dalloc(c, &d.Hll_e, 6 * (size_t)NE)); TRY(dalloc(c, &d.Hpp_e, 21 * (size_t)NE));
    TRY(dalloc(c, &d.Hpl_e, 18 * (size_t)NE)); TRY(dalloc(c, &d.bl_e, 3 * (size_t)NE));
    TRY(dalloc(c, &d.bp_e, 6 * (size_t)NE));
    TRY(dalloc(c, &d.echi, (size_t)NE + 6 * (size_t)NP + 3 * (size_t)NM));
    TRY(dalloc(c, &d.Ae, 18 * (size_t)NE));
    TRY(dalloc(c, &d.Hll, 9 * (size_t)NM)); TRY(dalloc(c, &d.bl, 3 * (size_t)NM)); TRY(dalloc(c, &d.Dinv, 9 * (size_t)NM));
    TRY(dalloc(c, &d.db, 3 * (size_t)NM));
    TRY(dalloc(c, &d.Hpp, 36 * (size_t)NP)); TRY(dalloc(c, &d.bp, 6 * (size_t)NP));
    const size_t nS = (size_t)6 * NP;
    TRY(dalloc(c, &d.S, nS * nS + nS));   // S followed by b_s (contiguous for one all-reduce)
    d.bs = d.S + nS * nS;
    TRY(dalloc(c, &d.x, 6 * (size_t)NP + 3 * (size_t)NM));
    TRY(dalloc(c, &d.red, 16));
    TRY(dalloc(c, &d.partChi, (size_t)NE / 64 + 2));
    TRY(dalloc(c, &d.partLin, (size_t)NE / 64 + 2));
    TRY(dalloc(c, &d.partScale, (size_t)NM / 64 + 3));
    TRY(dalloc(c, &d.partMax, (size_t)NP + (size_t)NM / 64 + 2));
    TRY(dalloc(c, &d.flags, 4));
    TRY(dalloc(c, &d.lm, 1));
    TRY(dalloc(c, &d.lmMid, 1));
    double* d_trace = nullptr;
    TRY(dalloc(c, &d_trace, 4 * 64));
    double* d_ldlw = nullptr;   // global image of the padded reduced matrix when it exceeds LDS
    MwLdl mwBase{};             // or the multi-workgroup solve's buffers
    // the dense MFMA Schur (A/B): Y^T, per-chunk partial tiles, per-edge Hpl D^-1 b_l
    int nFree = 0;   // the reduced system's order is 6 x the free poses
    for (int i = 0; i < NP; i++) nFree += p->pose_fixed[i] ? 0 : 1;
    const bool schurMfma = std::getenv("ORB_LBA_SCHUR_MFMA") != nullptr && c->world == 1 &&
                           (((size_t)6 * nFree + kNB - 1) & ~(size_t)(kNB - 1)) <= (size_t)kLdlLdsMaxN;
    double *d_Yt = nullptr, *d_ypart = nullptr, *d_ce = nullptr;
    if (schurMfma) {
        const size_t npm = ((size_t)6 * NP + 15) & ~(size_t)15, T = npm / 16;
        const size_t nch = ((size_t)NM + kYLm - 1) / kYLm;
        TRY(dalloc(c, &d_Yt, ((size_t)NM + kYLmB) * 3 * npm));
        TRY(dalloc(c, &d_ypart, nch * (T * (T + 1) / 2) * 256));
        TRY(dalloc(c, &d_ce, 6 * (size_t)NE));
    }
    {
        const size_t npMax = ((size_t)6 * NP + kNB - 1) & ~(size_t)(kNB - 1);
        if (use_mw((int)npMax)) TRY(mw_alloc(c, 6 * NP, &mwBase));
        else if (npMax > (size_t)kLdlLdsMaxN) TRY(dalloc(c, &d_ldlw, npMax * (npMax + 1)));
    }
    double* d_chi2 = nullptr;
    uint8_t* d_depth = nullptr;
    TRY(dalloc(c, &d_chi2, NE));
    TRY(dalloc(c, &d_depth, NE));

    std::vector<uint8_t> robustH;
    const double hm = o->huber_mono, hsv = o->huber_stereo;
    const int maxTrials = o->max_trials > 0 ? o->max_trials : 10;
    bool devStopped = false;   // the LM kernels observed terminate()

    auto elapsed = [&](hipEvent_t a, hipEvent_t b) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        return (double)ms;
    };

    const bool root = c->rank == 0;

    // global sum of the owned-point partials (and replicated pose part) of a scalar vector

    auto grid = [](int n) { return dim3((unsigned)std::max(1, (n + 255) / 256)); };
    auto init_opt_device = [&]() -> int {
        const int P = hs.P, M = hs.M;
        int32_t *act, *actPt, *actPi, *ptStart, *ptAct, *poStart, *poAct, *poPt, *cnt;
        TRY(dalloc(c, &act, NE)); TRY(dalloc(c, &actPt, NE)); TRY(dalloc(c, &actPi, NE));
        TRY(dalloc(c, &ptStart, (size_t)M + 1)); TRY(dalloc(c, &ptAct, NE));
        TRY(dalloc(c, &poStart, (size_t)P + 1)); TRY(dalloc(c, &poAct, NE)); TRY(dalloc(c, &poPt, NE));
        TRY(dalloc(c, &robust, NE));
        int32_t *piT, *ptT;   // per landmark-major entry: pose key, landmark
        TRY(dalloc(c, &piT, NE)); TRY(dalloc(c, &ptT, NE));
        cnt = d_structCnt;   // zeroed by k_lba_init
        int32_t *ptCnt = cnt, *ptFill = cnt + M, *keyCnt = cnt + 2 * M;
        const size_t hist = 4 * (size_t)(P + 1 <= kStructHistMax ? P + 1 : 0);
        hipLaunchKernelGGL(k_struct_count, grid(NE), dim3(256), hist, s, d.ept, d.eps, NE, d_ptLocal0, d_poseIdx0, P,
                           act, actPt, actPi, ptCnt, keyCnt, robust, robustKernels ? 1 : 0);
        hipLaunchKernelGGL(k_struct_scan, dim3(1), dim3(1024), 0, s, ptCnt, M, keyCnt, P, ptStart, poStart);
        hipLaunchKernelGGL(k_struct_pt, grid(NE), dim3(256), 0, s, NE, actPt, ptStart, ptFill, ptAct);
        hipLaunchKernelGGL(k_struct_ptsort, grid(M), dim3(256), 0, s, M, P, ptStart, actPi, ptAct, piT, ptT);
        if (P > 0)
            hipLaunchKernelGGL(k_struct_po, dim3(P), dim3(1024), 0, s, NE, ptAct, piT, ptT, poStart, poAct, poPt);
        ORB_HIP_TRY(hipGetLastError());
        d.robust = robust;
        d.act = act; d.nact = NE; d.poseIdx = d_poseIdx0; d.ptGlob = d_ptGlob0;
        d.P = P; d.M = M; d.ptStart = ptStart; d.ptAct = ptAct; d.poStart = poStart; d.poAct = poAct; d.poPt = poPt;
        d.actPt = actPt; d.actPi = actPi;
        d.bs = d.S + (size_t)36 * d.P * d.P;
        if (std::getenv("ORB_LBA_CHECK_STRUCT")) {   // test hook: the device arrays against the host build
            HostStructure h;
            build_structure(p, level, 0, 0, 1, h);
            const int nPo = h.poStart.empty() ? 0 : h.poStart.back();
            const std::pair<const int32_t*, const std::vector<int32_t>*> cmp[] = {
                {act, &h.act}, {actPt, &h.actPt}, {actPi, &h.actPi}, {ptStart, &h.ptStart}, {ptAct, &h.ptAct},
                {poStart, &h.poStart}, {poAct, &h.poAct}, {poPt, &h.poPt}};
            if (h.P != P || h.M != M || (int)h.act.size() != NE || nPo > NE) return ORB_EGPU;
            std::vector<int32_t> got;
            for (const auto& pr : cmp) {
                got.assign(pr.second->size(), 0);
                if (!got.empty())
                    ORB_HIP_TRY(hipMemcpyAsync(got.data(), pr.first, 4 * got.size(), hipMemcpyDeviceToHost, s));
                TRY(lba_wait(c));
                if (got != *pr.second) {
                    std::fprintf(stderr, "lba: device structure differs from the host build (array %d)\n",
                                 (int)(&pr - cmp));
                    return ORB_EGPU;
                }
            }
        }
        return ORB_OK;
    };
    auto init_opt = [&](int lvl) -> int {
        if (devStruct && lvl == 0) return init_opt_device();
        build_structure(p, level, lvl, c->rank, c->world, hs);
        robustH.assign(NE, robustKernels ? 1 : 0);
        int32_t *act, *poseIdx, *ptGlob, *actPt, *actPi, *ptStart, *ptAct, *poStart, *poAct, *poPt;
        TRY(upload_batch(c, 1, {up(&act, hs.act), up(&poseIdx, hs.poseIdx), up(&ptGlob, hs.ptGlob), up(&actPt, hs.actPt),
                                up(&actPi, hs.actPi), up(&ptStart, hs.ptStart), up(&ptAct, hs.ptAct),
                                up(&poStart, hs.poStart), up(&poAct, hs.poAct), up(&poPt, hs.poPt),
                                up(&d_freePoses, hs.freePoses), up(&robust, robustH)}));
        d.robust = robust;
        d.act = act; d.nact = (int)hs.act.size(); d.poseIdx = poseIdx; d.ptGlob = ptGlob;
        d.P = hs.P; d.M = hs.M; d.ptStart = ptStart; d.ptAct = ptAct; d.poStart = poStart; d.poAct = poAct; d.poPt = poPt;
        d.actPt = actPt; d.actPi = actPi;
        d.bs = d.S + (size_t)36 * d.P * d.P;   // b_s right after the 6P x 6P matrix: one all-reduce
        return ORB_OK;
    };



#ifdef ORB_NO_FUSE
    auto fuse_slots = [&]() { return false; };
#else
    auto fuse_slots = [&]() { return c->world == 1 && d.nact > 0 && d.M > 0; };
#endif
    // fused slots whose reduced system fits the LDS image: the pose update rides in
    // k_ldlt_solve's tail and the trial errors in k_backsub_errors (no k_edge_errors launch)
    auto merge_errors = [&]() {
        const int np = (6 * d.P + kNB - 1) & ~(kNB - 1);
        return fuse_slots() && d.P > 0 && (np <= kLdlLdsMaxN || use_mw(np));
    };
    // fused slots: the decision of a group's last trial (k_edge_lin takes the others)
    auto enqueue_close = [&](int iterations) {
        if (!fuse_slots()) return;
        const int nbE = (d.nact + 63) / 64, nbB = (d.M + 63) / 64 + 1;
        hipLaunchKernelGGL(k_lm_decide_fused, dim3(1), dim3(1024), 0, s, d, d_freePoses, maxTrials, iterations,
                           o->fixed_iterations ? 1 : 0, d_trace, merge_errors() ? nbB - 1 : nbE, nbB, 1);
    };

    // One LM "slot": the linearisation of an iteration (runs only when the device state says a
    // new iteration starts) followed by one trial (runs only while the iteration's trial loop
    // is open) and its decision.  Slots are enqueued back to back without host round trips.
    // `first`: the first slot of an optimize() call (its iteration start initialises lambda from
    // the maximum diagonal, so the fused slots keep k_vertex_reduce + k_point_schur there; the
    // others merge them into k_vertex_schur)
    auto enqueue_slot = [&](int iterations, hipEvent_t* ev, bool first) -> int {
        const bool prof = ev != nullptr;
        const bool single = c->world == 1;   // no collectives: the LM bookkeeping fuses into single kernels
        if (prof) (void)hipEventRecord(ev[0], s);
        // ---- linearisation (G/core/sparse_optimizer.cpp:384-394, block_solver.hpp:502-561)
        const int nbE = (d.nact + 63) / 64, nbV = d.P + (d.M + 63) / 64, nbB = (d.M + 63) / 64 + 1;
        // single process with edges and points: the decision and the iteration start ride in
        // k_edge_lin and k_point_schur (LmFuse), the group of slots ends with one decision kernel
        const bool fuse = fuse_slots();
        const bool merge = merge_errors();
        const LmFuse f{merge ? nbB - 1 : nbE, nbB, maxTrials, iterations, o->fixed_iterations ? 1 : 0, d_freePoses,
                       d_trace};
        const bool extraB = std::getenv("ORB_LBA_EXTRA_BOUNDARY") != nullptr;
        auto boundary = [&]() { if (extraB) hipLaunchKernelGGL(k_nop, dim3(256), dim3(64), 0, s); };
        if (d.nact >= kEdgeStageMin)
            hipLaunchKernelGGL(k_edge_lin<true>, dim3(nbE), dim3(64), 0, s, d, hm, hsv, fuse ? 1 : 0, f);
        else if (d.nact > 0)
            hipLaunchKernelGGL(k_edge_lin<false>, dim3(nbE), dim3(64), 0, s, d, hm, hsv, fuse ? 1 : 0, f);
        boundary();
        LbaDev dv = d;
        if (fuse) dv.lm = d.lmMid;
        const bool merged = fuse && !first && nbV > 0;
        if (merged) { hipLaunchKernelGGL(k_vertex_schur, dim3(nbV), dim3(256), 0, s, d, nbE); boundary(); }
        else if (nbV > 0) hipLaunchKernelGGL(k_vertex_reduce, dim3(nbV), dim3(256), 0, s, dv);
        if (single) {
            if (!fuse) hipLaunchKernelGGL(k_lm_begin_fused, dim3(1), dim3(64), 0, s, d, nbE, nbV);
        } else {
            hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, d.echi, d.nact, d.red, d.lm, 0);
            // the iteration's chi2 with the pose blocks: one collective
            if (d.P > 0)
                TRY(comm_allreduce_segs(c, {CommSeg{d.red, 1}, CommSeg{d.Hpp, 36 * (size_t)d.P}, CommSeg{d.bp, 6 * (size_t)d.P}}, 0,
                                        d.lm, 0));
            else
                TRY(comm_allreduce_g(c, d.red, 1, 0, d.lm, 0));
            hipLaunchKernelGGL(k_maxdiag, dim3(1), dim3(1024), 0, s, d.Hpp, d.P, d.Hll, d.M, d.red + 1, d.lm);
            TRY(comm_allreduce_g(c, d.red + 1, 1, 1, d.lm, 3));
            hipLaunchKernelGGL(k_lm_begin, dim3(1), dim3(64), 0, s, d.lm, d.red);
        }
        if (prof) (void)hipEventRecord(ev[1], s);
        // ---- trial: Schur complement, reduced solve, back-substitution + update, new chi2
        if (d.M > 0 && !merged)
            hipLaunchKernelGGL(k_point_schur, dim3((d.M + 63) / 64), dim3(64), 0, s, d, fuse ? 1 : 0, nbE, nbV);
        const int npairs = d.P * (d.P + 1) / 2;
        if (schurMfma && d.P > 0 && d.M > 0) {
            const int npm = (6 * d.P + 15) & ~15, T = npm / 16, nt = T * (T + 1) / 2;
            const int nch = ((d.M + kYLm - 1) / kYLm + kYLmG - 1) / kYLmG;   // gemm workgroups = partial sets
            hipLaunchKernelGGL(k_schur_ymat, dim3((d.M + kYLmB - 1) / kYLmB), dim3(256), 0, s, d, d_Yt, npm, d_ce);
            hipLaunchKernelGGL(k_schur_gemm, dim3(nch), dim3(256), 0, s, d, d_Yt, npm, d_ypart);
            hipLaunchKernelGGL(k_schur_msum, dim3(nt + (d.P + 3) / 4), dim3(256), 0, s, d, d_ypart, nch, npm,
                               d_ce, root ? 1 : 0);
        } else if (npairs > 0) {
            hipLaunchKernelGGL(k_schur_pairs, dim3(std::min((npairs + 7) & ~7, kSpMaxWg)), dim3(kSpT), 0, s, d,
                               root ? 1 : 0);
            boundary();
        }
        if (d.P > 0) TRY(comm_allreduce_schur(c, d.S, d.bs, d.pairs, gPairs, d.P, d.lm, 1));
        if (prof) (void)hipEventRecord(ev[2], s);
        if (d.P > 0) {
            const int n = 6 * d.P, np = (n + kNB - 1) & ~(kNB - 1);
            PoseTail pt{};
            if (merge)
                pt = PoseTail{d.q, d.t, d.bq, d.bt, d.partScale + (nbB - 1), d.bp, d_freePoses, d.poseIdx, d.P};
            if (use_ldlt_df(n)) {
                hipLaunchKernelGGL(k_ldlt_df, dim3(1), dim3(kLdlT), ldlt_df_lds_bytes(n), s, d.S, d.bs, n, d.x, d.flags,
                                   d.lm, pt);
                boundary();
            } else if (np <= kLdlLdsMaxN) {
                hipLaunchKernelGGL(k_ldlt_solve<true>, dim3(1), dim3(kLdlT), ((size_t)np * (np + 1) + 3 * (size_t)np + 256 + (size_t)kNB * (np + 1) + 64) * 8,
                                   s, d.S, d.bs, n, nullptr, d.x, d.flags, d.lm, pt);
                boundary();
            } else if (use_mw(np))
                enqueue_ldlt_mw(s, mw_order(mwBase, n), d.S, d.bs, d.x, d.flags, d.lm, pt);
            else
                hipLaunchKernelGGL(k_ldlt_solve<false>, dim3(1), dim3(kLdlT), (3 * (size_t)np + 64) * 8, s, d.S, d.bs, n,
                                   d_ldlw, d.x, d.flags, d.lm, PoseTail{});
        } else {
            ORB_HIP_TRY(hipMemsetAsync(d.flags, 0, 4, s));
        }
        if (prof) (void)hipEventRecord(ev[3], s);
        if (merge) {
            hipLaunchKernelGGL(k_backsub_errors, dim3(nbB - 1), dim3(256), 0, s, d, hm, hsv);
            boundary();
        } else {
            hipLaunchKernelGGL(k_backsub_update, dim3(nbB), dim3(256), 0, s, d, d_freePoses);
            if (d.nact > 0) hipLaunchKernelGGL(k_edge_errors, dim3(nbE), dim3(64), 0, s, d, hm, hsv, 1, fuse ? 1 : 0);
        }
        if (single) {
            if (!fuse)
                hipLaunchKernelGGL(k_lm_decide_fused, dim3(1), dim3(1024), 0, s, d, d_freePoses, maxTrials, iterations,
                                   o->fixed_iterations ? 1 : 0, d_trace, nbE, nbB, 0);
        } else {
            // the trial's chi2 (red[4]), the scale term (red[2]) and the stop sample (red[3]): one collective
            hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, d.echi, d.nact, d.red + 4, d.lm, 1);
            const int nx = 6 * d.P + 3 * d.M;
            hipLaunchKernelGGL(k_scale_terms, grid(nx), dim3(256), 0, s, d, root ? 1 : 0, d.echi);
            hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, d.echi, nx, d.red + 2, d.lm, 1);
            hipLaunchKernelGGL(k_stop_sample, dim3(1), dim3(64), 0, s, d.lm, d.stopWord, d.red);
            TRY(comm_allreduce_g(c, d.red + 2, 3, 0, d.lm, 1));
            hipLaunchKernelGGL(k_lm_decide, dim3(1), dim3(64), 0, s, d.lm, d.red, d.flags, maxTrials, iterations,
                               o->fixed_iterations ? 1 : 0, d_trace);
            hipLaunchKernelGGL(k_pop, grid(std::max(d.M, d.P)), dim3(256), 0, s, d, d.P, d_freePoses);
        }
        if (prof) (void)hipEventRecord(ev[4], s);
        return ORB_OK;
    };

    // pinned staging of everything the host reads after an optimize(): chi2 (8 NE), depth flag
    // (NE), then q, t, X (contiguous in the problem batch); reserved before any copy is queued
    const size_t estOff = (9 * (size_t)NE + 255) & ~(size_t)255;
    const size_t bq = ((32 * (size_t)NP + 255) & ~(size_t)255), bt = ((24 * (size_t)NP + 255) & ~(size_t)255);
    const size_t estBytes = bq + bt + 24 * (size_t)NM;
    const size_t lmOff = (estOff + estBytes + 255) & ~(size_t)255;   // then the LM state
    const size_t traceOff = (lmOff + sizeof(LmState) + 255) & ~(size_t)255;   // and the trace rows
    TRY(stage_reserve(c, 2, traceOff + 32 * 64, true));
    char* const hStage = c->stage[2];
    // one optimize() call (G/core/sparse_optimizer.cpp:354-419).  The host enqueues as many
    // slots as iterations remain (one trial each), then reads the device state once: more
    // slots only when trials were rejected.  The stop flag is polled between those groups.
    auto optimize = [&](int iterations, int& itersDone, const std::function<int()>& tail, bool& tailRan) -> int {
        itersDone = 0;
        tailRan = false;
        if (d.P + d.M == 0 && c->world == 1) return ORB_OK;
        bool stopNow = false;
        TRY(agreed(stopped(), &stopNow));
        if (iterations <= 0 || stopNow) return ORB_OK;   // sparse_optimizer.cpp:376 before iteration 0
        LmState* hst = reinterpret_cast<LmState*>(reinterpret_cast<char*>(c->h_scal) + 512);
        std::memset(hst, 0, sizeof(LmState));
        hst->ni = 2;
        hst->traceBase = r->trace ? r->n_trace : 64;
        hst->stopAfter = c->stopAfter;
        hst->trialBase = r->trials;
        ORB_HIP_TRY(hipMemcpyAsync(d.lm, hst, sizeof(LmState), hipMemcpyHostToDevice, s));
        // Single process, no stage events: the slots are captured into HIP graphs and
        // replayed, so the LM loop pays one graph launch per group of slots instead of a host
        // dispatch per kernel.  (With a communicator the all-reduce is a host callback and the
        // slot is enqueued kernel by kernel.)
        // graphs of `iterations` slots (the first group) and of one slot (the slots after
        // rejected trials), looked up by every captured launch parameter
        auto slot_graph = [&](int nslots, hipGraphExec_t* out, bool firstGroup, bool close) -> int {
            *out = nullptr;
            if ((c->world != 1 && !(c->grp && c->grpGraphs)) || c->profile || s == nullptr || std::getenv("ORB_LBA_NO_GRAPH"))
                return ORB_OK;
            struct {
                LbaDev d;
                const void* ptrs[5];
                double h[2];
                int v[8];
                orbamd::GrpDev grp;   // a group's exchange pointers (zero without one)
            } k;
            std::memset(&k, 0, sizeof(k));
            k.d = d;
            if (c->grp) k.grp = *c->grp;
            k.ptrs[0] = d_freePoses; k.ptrs[1] = d_trace; k.ptrs[2] = d_ldlw ? (const void*)d_ldlw : (const void*)mwBase.A; k.ptrs[3] = s;
            k.ptrs[4] = mwBase.tfirst;
            k.h[0] = hm; k.h[1] = hsv;
            k.v[0] = iterations; k.v[1] = maxTrials; k.v[2] = o->fixed_iterations; k.v[3] = root; k.v[4] = nslots;
            k.v[5] = firstGroup ? 1 : 0;
            k.v[6] = close ? 1 : 0;
            k.v[7] = (schurMfma ? 1 : 0) | (std::getenv("ORB_LBA_EXTRA_BOUNDARY") ? 2 : 0) |
                     (std::getenv("ORB_LBA_MW_SPLIT") ? 4 : 0);
            std::vector<char> key(reinterpret_cast<const char*>(&k), reinterpret_cast<const char*>(&k) + sizeof(k));
            for (size_t i = 0; i < c->graphs.size(); i++)
                if (c->graphs[i].key == key) {   // most recently used last: eviction takes the front
                    *out = c->graphs[i].exec;
                    std::rotate(c->graphs.begin() + i, c->graphs.begin() + i + 1, c->graphs.end());
                    return ORB_OK;
                }
            hipGraph_t g = nullptr;
            int st = ORB_OK;
            hipError_t ce;
            {   // no other thread's legacy-stream setup call inside the capture (common.h)
                std::lock_guard<std::mutex> lk(legacy_capture_mutex());
                ORB_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                for (int i = 0; i < nslots && !st; i++) st = enqueue_slot(iterations, nullptr, firstGroup && i == 0);
                if (!st && close) enqueue_close(iterations);
                ce = hipStreamEndCapture(s, &g);
            }
            if (st) { if (g) (void)hipGraphDestroy(g); return st; }
            if (ce != hipSuccess) return ORB_EGPU;
            const hipError_t ie = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ie != hipSuccess) return ORB_EGPU;
            if (c->graphs.size() >= 16) {
                (void)hipGraphExecDestroy(c->graphs.front().exec);
                c->graphs.erase(c->graphs.begin());
            }
            c->graphs.push_back({std::move(key), *out});
            return ORB_OK;
        };
        // the first group as graphs of at most kGraphSlots slots each (the decision kernel closes
        // the last; a graph boundary costs ~8 us).  Under rocprofv3 a 10-slot graph shows a
        // 300-390 us hole after its 30th node (the profiler slows the dispatch of the nodes);
        // without it one graph and chunks of 5 time the same (ORB_LBA_GRAPH_SLOTS sweep)
        int chunk = kGraphSlots;
        if (const char* e = std::getenv("ORB_LBA_GRAPH_SLOTS")) chunk = std::max(1, std::atoi(e));
        chunk = std::max(chunk, (iterations + 7) / 8);   // at most 8 graphs: the cache (16) keeps them all
        std::vector<hipGraphExec_t> gFirst;
        for (int i0 = 0; i0 < iterations; i0 += chunk) {
            hipGraphExec_t ge = nullptr;
            const int ns = std::min(chunk, iterations - i0);
            TRY(slot_graph(ns, &ge, i0 == 0, i0 + ns >= iterations));
            if (!ge) { gFirst.clear(); break; }
            gFirst.push_back(ge);
        }
        hipGraphExec_t gOne = nullptr;
        const bool gAll = !gFirst.empty();
        int known = 0;
        for (;;) {
            const int G = std::max(1, iterations - known);
            if (c->profile && c->slotEv.size() < 5 * (size_t)G) {
                while (c->slotEv.size() < 5 * (size_t)G) {
                    hipEvent_t e;
                    if (hipEventCreate(&e) != hipSuccess) return ORB_EGPU;
                    c->slotEv.push_back(e);
                }
            }
            if (gAll && G == iterations) {
                for (hipGraphExec_t ge : gFirst) ORB_HIP_TRY(hipGraphLaunch(ge, s));
            } else {
                if (gAll && !gOne) TRY(slot_graph(1, &gOne, false, true));
                for (int g = 0; g < G; g++) {
                    if (gOne) ORB_HIP_TRY(hipGraphLaunch(gOne, s));
                    else TRY(enqueue_slot(iterations, c->profile ? &c->slotEv[5 * (size_t)g] : nullptr,
                                          known == 0 && g == 0));
                }
                if (!gOne) enqueue_close(iterations);
            }
            // speculative: what the host reads after optimize() (edge chi2 / depth, estimates)
            // rides behind every group, so the last group's copy is already there when the LM
            // state says the loop is over
            TRY(tail());
            tailRan = true;
            TRY(lba_wait(c));
            std::memcpy(hst, c->stage[2] + lmOff, sizeof(LmState));   // stored by k_readback
            if (c->profile) {
                for (int g = 0; g < G; g++) {
                    hipEvent_t* ev = &c->slotEv[5 * (size_t)g];
                    c->ms_linearize += elapsed(ev[0], ev[1]);
                    c->ms_schur += elapsed(ev[1], ev[2]);
                    c->ms_solve += elapsed(ev[2], ev[3]);
                    c->ms_update += elapsed(ev[3], ev[4]);
                }
            }
            known = hst->itersDone;
            if (hst->phase == 2) break;
            // single process: a stop seen by the host between iterations ends the loop where
            // g2o's iteration loop would test terminate(); mid-iteration the device decides
            if (c->world == 1 && hst->phase == 0 && stopped()) { devStopped = true; break; }
        }
        if (hst->stopped) devStopped = true;
        itersDone = hst->itersDone;
        r->trials += hst->trials;
        c->n_trials += hst->trials;
        c->n_iters += itersDone;
        if (r->trace && r->n_trace < 64) {
            const int rows = std::min(64 - r->n_trace, itersDone);
            if (rows > 0) {
                // the last group's k_readback stored the rows (the loop above waited for it)
                std::memcpy(r->trace + 4 * r->n_trace,
                            reinterpret_cast<const double*>(c->stage[2] + traceOff) + 4 * r->n_trace, 32 * (size_t)rows);
                r->n_trace += rows;
            }
        }
        return ORB_OK;
    };

#ifdef ORB_TIMING
    std::chrono::steady_clock::time_point hT[10];
#endif
    const std::function<int()> tail = [&]() -> int {
        const int n = std::max({NE, 4 * NP, 3 * NM, (int)(sizeof(LmState) / 4), 4 * 64});
        hipLaunchKernelGGL(k_readback, grid(n), dim3(256), 0, s, d, NE, d_chi2, d_depth, c->stageDev[2], estOff, bq,
                           bq + bt, NP, NM, lmOff, d_trace, traceOff);
        ORB_HIP_TRY(hipGetLastError());
        return ORB_OK;
    };
    auto ensure_tail = [&](bool ran) -> int {   // an optimize() that ran no group queued no tail
        if (ran) return ORB_OK;
        TRY(tail());
        return lba_wait(c);
    };
    const double* chi = reinterpret_cast<const double*>(hStage);
    const uint8_t* dep = reinterpret_cast<const uint8_t*>(hStage + 8 * (size_t)NE);
    HSTAMP(0);
    // the pose-pair blocks of S with shared landmarks (k_schur_pairs runs only those; the
    // others are zeroed here once and stay zero: the outlier pass keeps the block structure)
    auto build_pairs = [&]() -> int {
        const int P = d.P, np2 = P * (P + 1) / 2;
        // the shared-landmark lists' total: sum over landmarks of C(k, 2), k = its free-pose edges
        // (an upper bound with a communicator, where each rank lists its own landmarks only)
        std::vector<int32_t> kf((size_t)NM, 0);
        for (int e = 0; e < NE; e++) kf[(size_t)p->edge_point[e]] += p->pose_fixed[p->edge_pose[e]] ? 0 : 1;
        size_t ntrip = 0;
        for (int l = 0; l < NM; l++) ntrip += (size_t)kf[(size_t)l] * (kf[(size_t)l] - 1) / 2;
        int32_t *flag, *cnt, *pairs, *npairs, *tripStart, *poPos, *units;
        int2* trips;
        TRY(dalloc(c, &poPos, std::max(NE, 1)));
        ORB_HIP_TRY(hipMemsetAsync(poPos, 0xFF, 4 * (size_t)std::max(NE, 1), s));   // -1: fixed-pose edges
        if (P > 0) hipLaunchKernelGGL(k_po_pos, grid(NE), dim3(256), 0, s, d, poPos);
        d.poPos = poPos;
        TRY(dalloc(c, &flag, 2 * (size_t)np2)); TRY(dalloc(c, &pairs, np2)); TRY(dalloc(c, &npairs, 3));
        TRY(dalloc(c, &units, std::max(np2, 1)));
        TRY(dalloc(c, &tripStart, 2 * (size_t)np2)); TRY(dalloc(c, &trips, std::max<size_t>(ntrip, 1)));
        cnt = flag + np2;
        ORB_HIP_TRY(hipMemsetAsync(npairs, 0, 12, s));
        if (P > 0) {
            ORB_HIP_TRY(hipMemsetAsync(flag, 0, 8 * (size_t)np2, s));
            ORB_HIP_TRY(hipMemsetAsync(d.S, 0, 8 * (size_t)36 * P * P, s));
            if (c->world > 1) {
                // with a communicator every rank lists the GLOBAL pair set (every pair some landmark of
                // any rank couples, and the diagonal): the same list on every rank, so the exchange can
                // pack exactly those blocks (k_pack_pairs); each rank's own landmarks still set the
                // trip counts below.  Built on the host from the problem arrays every rank holds.
                std::vector<int32_t> gflag((size_t)np2, 0);
                std::vector<std::vector<int>> lp((size_t)NM);
                for (int e = 0; e < NE; e++) {   // every edge, every rank's landmarks: a superset is harmless
                    const int pi = hs.poseIdx[(size_t)p->edge_pose[e]];
                    if (pi >= 0) lp[(size_t)p->edge_point[e]].push_back(pi);
                }
                for (int i = 0; i < P; i++) gflag[(size_t)(i * P - i * (i - 1) / 2)] = 1;
                for (const auto& v : lp)
                    for (size_t a = 0; a < v.size(); a++)
                        for (size_t b = a + 1; b < v.size(); b++) {
                            if (v[a] == v[b]) continue;
                            const int i = std::min(v[a], v[b]), j = std::max(v[a], v[b]);
                            gflag[(size_t)(i * P - i * (i - 1) / 2 + (j - i))] = 1;
                        }
                gPairs = 0;
                for (int32_t f : gflag) gPairs += f;
                c->gflagStage = gflag;   // (kept: the copy is asynchronous)
                ORB_HIP_TRY(hipMemcpyAsync(flag, c->gflagStage.data(), 4 * (size_t)np2, hipMemcpyHostToDevice, s));
            }
            hipLaunchKernelGGL(k_pair_mark, grid(std::max(d.M, P)), dim3(256), np2 <= kPairHist ? 4 * (size_t)np2 : 0, s, d,
                               flag, cnt, 0);
            // off-diagonal pairs sharing at most this many landmarks take one wave in k_schur_pairs
            // (read per solve: tests and A/B runs switch it within one process)
            const char* spEnv = std::getenv("ORB_LBA_SMALL_PAIR");
            const int smallPair = spEnv ? std::atoi(spEnv) : 512;
            hipLaunchKernelGGL(k_pair_list, dim3(1), dim3(1024), 0, s, flag, cnt, P, pairs, npairs, tripStart, units,
                               smallPair);
            d.pairs = pairs;
            d.npairs = npairs;
            d.tripStart = tripStart;
            hipLaunchKernelGGL(k_pair_trip, dim3(np2), dim3(kSpT), 0, s, d, trips);
            // the multi-workgroup solve's envelope (ORB_LBA_MW_DENSE=1: the dense passes, A/B runs)
            mwBase.tfirst = nullptr;
            if (mwBase.A && P <= 16384 && !std::getenv("ORB_LBA_MW_DENSE")) {
                const int npm = (6 * P + kMwNB - 1) & ~(kMwNB - 1);
                int32_t* tf = nullptr;
                TRY(dalloc(c, &tf, npm / 16));
                hipLaunchKernelGGL(k_mw_envelope, dim3(1), dim3(1024), 4 * (size_t)P, s, pairs, npairs, P, npm, tf);
                ORB_HIP_TRY(hipMemsetAsync(mwBase.A, 0, 8 * (size_t)npm * npm, s));   // (k_ldlt_mw_stage_env)
                mwBase.tfirst = tf;
            }
            ORB_HIP_TRY(hipGetLastError());
            if (c->world > 1) {
                // the packed exchange carries the first gPairs blocks of d.pairs: the device's list
                // (gflag plus k_pair_mark's own marks) must be exactly the host's global set, or the
                // all-reduced S would silently miss blocks.  Once per solve.
                int32_t devPairs = -1;
                ORB_HIP_TRY(hipMemcpyAsync(&devPairs, npairs, 4, hipMemcpyDeviceToHost, s));
                ORB_HIP_TRY(hipStreamSynchronize(s));
                if (devPairs != gPairs) {
                    std::fprintf(stderr, "[orbslam2_amd] lba: rank %d lists %d pose pairs, the global set has %d\n",
                                 c->rank, devPairs, gPairs);
                    return ORB_EINTERNAL;
                }
            }
        }
        d.pairs = pairs;
        d.npairs = npairs;
        d.pairUnits = units;
        d.tripStart = tripStart;
        d.trips = trips;
        return ORB_OK;
    };
    // ---- R/src/Optimizer.cpp:789-841
    TRY(init_opt(0));
    TRY(build_pairs());
    HSTAMP(1);
    bool tailRan = false;
    TRY(optimize(o->iters1, r->iterations[0], tail, tailRan));
    HSTAMP(2);
    bool stopAfter1 = false;
    TRY(agreed(stopped() || devStopped, &stopAfter1));
    const bool bDoMore = !global && !stopAfter1;   // global BA: one optimize(nIterations), R :230-231
    const int own0 = (int)((long long)NM * c->rank / c->world), own1 = (int)((long long)NM * (c->rank + 1) / c->world);
    if (bDoMore) {
        // the outlier pass on the device (k_outlier_mask), behind the edge check the last group's
        // tail queued: no host round trip and no second structure build between the rounds
        if (!tailRan) TRY(tail());
        if (d.nact > 0)
            hipLaunchKernelGGL(k_outlier_mask, grid(d.nact), dim3(256), 0, s, d, d_chi2, d_depth,
                               o->chi2_mono, o->chi2_stereo);
        HSTAMP(3);
        HSTAMP(4);
        TRY(optimize(o->iters2, r->iterations[1], tail, tailRan));
    }
    HSTAMP(5);
    // ---- final check (R/src/Optimizer.cpp:850-880) and write-back data
    TRY(ensure_tail(tailRan));
    for (int e = 0; e < NE; e++) {
        const int pt = p->edge_point[e];
        const bool mine = pt >= own0 && pt < own1;
        if (r->edge_chi2) r->edge_chi2[e] = mine ? chi[e] : 0.0;
        uint8_t er = 0;
        if (!global && mine && !(p->point_bad && p->point_bad[pt])) {
            const double thr = p->edge_stereo[e] ? o->chi2_stereo : o->chi2_mono;
            er = (chi[e] > thr || !dep[e]) ? 1 : 0;
        }
        if (r->edge_erase) r->edge_erase[e] = er;
    }
    {   // estimates (q, t, X)
        const char* h = hStage + estOff;
        if (r->pose_q) std::memcpy(r->pose_q, h, 32 * (size_t)NP);
        if (r->pose_t) std::memcpy(r->pose_t, h + bq, 24 * (size_t)NP);
        if (r->point_xyz) std::memcpy(r->point_xyz, h + bq + bt, 24 * (size_t)NM);
    }
    c->last = d;
#ifdef ORB_TIMING
    HSTAMP(6);
    auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(hT[b] - hT[a]).count(); };
    std::printf("lba host: init1 %.0f opt1 %.0f check %.0f init2 %.0f opt2 %.0f final %.0f us (entry->init %.0f)\n",
                us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(5, 6),
                std::chrono::duration<double, std::micro>(hT[0] - hEntry).count());
#endif
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}


// ------------------------------------------------------------------ device group (one process, N GPUs)
// LocalBundleAdjustment sharded over the GPUs of one process, the drop-in's model (LocalMapping
// runs the local BA on one thread, R/src/LocalMapping.cpp:94-95).  Rank r (context on devices[r])
// owns the landmark range [r M / n, (r+1) M / n), as lba_set_comm; the collectives are the library's
// own: a one-shot peer-to-peer all-reduce kernel (k_peer_allreduce) in which every rank reads every
// rank's workspace slice through peer access over xGMI and sums it in rank order, so all ranks hold
// bitwise the same reduced system and take the same LM decisions.  Each collective is ordered by
// events between the ranks' streams: rank r records "ready", waits for its peers' ready events,
// reduces into its own result buffer, records "read", and waits for its peers' read events before
// anything may overwrite its workspace; a host spin barrier between the records makes sure every
// event a stream waits on has been recorded.  One host thread per rank runs lba_solve.
constexpr int kMaxGroup = 16;
struct PeerPtrs {
    const double* p[kMaxGroup];
};
__global__ __launch_bounds__(256) void k_peer_allreduce(PeerPtrs in, int nr, size_t n, int op, double* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        double v = in.p[0][i];
        for (int r = 1; r < nr; r++) {
            const double w = in.p[r][i];
            v = op ? fmax(v, w) : v + w;
        }
        out[i] = v;
    }
}

struct lba_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<lba_context*> ctx;
    std::vector<double*> ws, res;
    size_t wsDoubles = 0;
    std::vector<hipEvent_t> evReady, evRead;
    // device-side exchange (default; ORB_LBA_GROUP_HOST=1 keeps the host-ordered callback above):
    // per rank 256 B of fine-grained flag memory (ready / read epochs, epoch counter, error word)
    bool hostPath = false;
    size_t warmNP = 0, warmNM = 0, warmNE = 0;   // the largest problem the ranks' buffers were grown for
    std::vector<uint32_t*> sync;
    orbamd::GrpDev gdev[kMaxGroup];
    std::atomic<int> arrive{0};
    std::atomic<unsigned> bgen{0};
    std::atomic<bool> abort{false};
    struct Rank {
        lba_group* g;
        int r;
    } ranks[kMaxGroup];
    // exchange timing on rank 0's stream: (before ready, after the peers' read) per collective
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    size_t ntev = 0;
    double exchangeMs = 0.0;
    long exchanges = 0;
};

static bool group_barrier(lba_group* g) {
    const unsigned gen = g->bgen.load(std::memory_order_acquire);
    if (g->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == g->n) {
        g->arrive.store(0, std::memory_order_relaxed);
        g->bgen.fetch_add(1, std::memory_order_acq_rel);
        return !g->abort.load();
    }
    for (int spins = 0; g->bgen.load(std::memory_order_acquire) == gen; spins++) {
        if (g->abort.load()) return false;
        if (spins > 256) std::this_thread::yield();
    }
    return !g->abort.load();
}

static int group_allreduce(void* user, size_t off, size_t cnt, int op) {
    auto* rk = static_cast<lba_group::Rank*>(user);
    lba_group* g = rk->g;
    const int r = rk->r, n = g->n;
    lba_context* c = g->ctx[r];
    hipStream_t s = c->stream;
    if (hipSetDevice(c->device) != hipSuccess) return 1;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    if (r == 0) {
        if (g->ntev == g->tev.size()) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
            g->tev.push_back({a, b});
        }
        t0 = g->tev[g->ntev].first;
        t1 = g->tev[g->ntev].second;
        g->ntev++;
        if (hipEventRecord(t0, s) != hipSuccess) return 1;
    }
    if (hipEventRecord(g->evReady[r], s) != hipSuccess) return 1;
    if (!group_barrier(g)) return 1;
    for (int p = 0; p < n; p++)
        if (p != r && hipStreamWaitEvent(s, g->evReady[p], 0) != hipSuccess) return 1;
    PeerPtrs pp{};
    for (int p = 0; p < n; p++) pp.p[p] = g->ws[p] + off;
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(1024, (cnt + 255) / 256));
    hipLaunchKernelGGL(k_peer_allreduce, dim3(blocks), dim3(256), 0, s, pp, n, cnt, op, g->res[r] + off);
    if (hipGetLastError() != hipSuccess) return 1;
    if (hipEventRecord(g->evRead[r], s) != hipSuccess) return 1;
    if (!group_barrier(g)) return 1;
    for (int p = 0; p < n; p++)
        if (p != r && hipStreamWaitEvent(s, g->evRead[p], 0) != hipSuccess) return 1;
    if (r == 0 && hipEventRecord(t1, s) != hipSuccess) return 1;
    return 0;
}

static int group_alloc_fine(int dev, size_t bytes, void** p) {
    *p = nullptr;
    if (hipSetDevice(dev) != hipSuccess) return ORB_EGPU;
    return hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained) == hipSuccess ? ORB_OK : ORB_ENOMEM;
}

static void group_free_ws(lba_group* g) {
    for (int r = 0; r < g->n; r++) {
        (void)hipSetDevice(g->dev[r]);
        if (g->ws[r]) (void)hipFree(g->ws[r]);
        if (g->res[r]) (void)hipFree(g->res[r]);
        g->ws[r] = g->res[r] = nullptr;
    }
    g->wsDoubles = 0;
}

void lba_group_destroy(lba_group* g) try {
    if (!g) return;
    for (int r = 0; r < g->n; r++)
        if (g->ctx[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipStreamSynchronize(g->ctx[r]->stream);
        }
    group_free_ws(g);
    for (int r = 0; r < g->n; r++) {
        (void)hipSetDevice(g->dev[r]);
        if (r < (int)g->sync.size() && g->sync[r]) (void)hipFree(g->sync[r]);
        if (g->evReady[r]) (void)hipEventDestroy(g->evReady[r]);
        if (g->evRead[r]) (void)hipEventDestroy(g->evRead[r]);
        if (g->ctx[r]) lba_destroy(g->ctx[r]);
    }
    if (!g->dev.empty()) (void)hipSetDevice(g->dev[0]);
    for (auto& e : g->tev) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    delete g;
} ORB_ABI_CATCH_VOID

int lba_group_create(const int* devices, int n, lba_group** out) try {
    if (!devices || !out || n < 1 || n > kMaxGroup) return ORB_EINVAL;
    *out = nullptr;
    lba_group* g = new lba_group();
    g->n = n;
    g->dev.assign(devices, devices + n);
    g->ctx.assign(n, nullptr);
    g->ws.assign(n, nullptr);
    g->res.assign(n, nullptr);
    g->evReady.assign(n, nullptr);
    g->evRead.assign(n, nullptr);
    g->sync.assign(n, nullptr);
    // The device-side exchange needs every rank on a device of its own: ranks sharing a device
    // may find their streams on one hardware queue, where a rank's waiting k_grp_sync blocks the
    // peer it waits for (seen as timeouts in a long-lived process with many streams).  Ranks on one
    // device therefore use the host-ordered exchange, unless ORB_LBA_GROUP_DEVICE=1 (the test hook
    // that rehearses the device-side protocol of an N-GPU node on one device: every rank after the
    // first on a CU-masked stream of its own, which the runtime gives a dedicated hardware queue)
    bool distinct = true;
    for (int a = 0; a < n; a++)
        for (int b2 = a + 1; b2 < n; b2++) distinct = distinct && devices[a] != devices[b2];
    const bool forceDev = std::getenv("ORB_LBA_GROUP_DEVICE") != nullptr;
    g->hostPath = std::getenv("ORB_LBA_GROUP_HOST") != nullptr || (!distinct && !forceDev);
    for (int r = 0; r < n; r++) {
        g->ranks[r] = {g, r};
        int st = lba_create(devices[r], &g->ctx[r]);
        if (st) { lba_group_destroy(g); return st; }
        if (hipEventCreateWithFlags(&g->evReady[r], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->evRead[r], hipEventDisableTiming) != hipSuccess) {
            lba_group_destroy(g);
            return ORB_EGPU;
        }
    }
    // peer access between every pair of distinct devices (xGMI)
    for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) {
            if (devices[a] == devices[b]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[a], devices[b]) != hipSuccess || !can) {
                lba_group_destroy(g);
                return ORB_ENODEV;
            }
            (void)hipSetDevice(devices[a]);
            const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                lba_group_destroy(g);
                return ORB_EGPU;
            }
            (void)hipGetLastError();
        }
    if (!g->hostPath)
        for (int r = 0; r < n; r++) {
            int st = group_alloc_fine(devices[r], 256, reinterpret_cast<void**>(&g->sync[r]));
            if (st) { lba_group_destroy(g); return st; }
        }
    if (!g->hostPath && !distinct) {   // (the test hook) ranks 1.. each on a hardware queue of its own
        for (int r = 1; r < n; r++) {
            (void)hipSetDevice(devices[r]);
            lba_context* cr = g->ctx[r];
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, devices[r]) != hipSuccess || cus <= 0) {
                lba_group_destroy(g);
                return ORB_EGPU;
            }
            std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xFFFFFFFFu);   // every CU
            hipStream_t hs = nullptr;
            if (hipExtStreamCreateWithCUMask(&hs, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
                lba_group_destroy(g);
                return ORB_EGPU;
            }
            if (cr->stream && cr->ownStream) (void)hipStreamDestroy(cr->stream);
            cr->stream = hs;
            cr->ownStream = true;
        }
    }
    *out = g;
    return ORB_OK;
} ORB_ABI_CATCH

int lba_group_solve(lba_group* g, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop,
                    lba_result* r) try {
    if (!g || !p || !o || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0) return ORB_EINVAL;
    const int n = g->n;
    if (n == 1) return lba_solve(g->ctx[0], p, o, stop, r);
    const size_t NP = (size_t)p->n_poses, NM = (size_t)p->n_points, NE = (size_t)p->n_edges;
    const size_t need = std::max(36 * NP * NP + 6 * NP, NE) + 64;
    if (need > g->wsDoubles) {
        group_free_ws(g);
        for (int q = 0; q < n; q++) {
            ORB_HIP_TRY(hipSetDevice(g->dev[q]));
            const bool wsOk = g->hostPath ? hipMalloc((void**)&g->ws[q], need * 8) == hipSuccess
                                          : group_alloc_fine(g->dev[q], need * 8, reinterpret_cast<void**>(&g->ws[q])) == ORB_OK;
            if (!wsOk || hipSetDevice(g->dev[q]) != hipSuccess || hipMalloc((void**)&g->res[q], need * 8) != hipSuccess) {
                group_free_ws(g);
                return ORB_ENOMEM;
            }
        }
        g->wsDoubles = need;
    }
    for (int q = 0; q < n; q++) {
        TRY(lba_set_comm(g->ctx[q], q, n, g->ws[q], g->wsDoubles, group_allreduce, &g->ranks[q]));
        g->ctx[q]->wsOut = g->res[q];
    }
    if (!g->hostPath) {   // fresh epochs: every rank's flags, counter and error word zeroed
        for (int q = 0; q < n; q++) {   // (ordered before every rank's work: the streams are non-blocking)
            ORB_HIP_TRY(hipSetDevice(g->dev[q]));
            ORB_HIP_TRY(hipMemsetAsync(g->sync[q], 0, 256, g->ctx[q]->stream));
        }
        for (int q = 0; q < n; q++) {
            ORB_HIP_TRY(hipSetDevice(g->dev[q]));
            ORB_HIP_TRY(hipStreamSynchronize(g->ctx[q]->stream));
        }
        for (int q = 0; q < n; q++) {
            orbamd::GrpDev& gd = g->gdev[q];
            std::memset(&gd, 0, sizeof(gd));
            for (int p2 = 0; p2 < n; p2++) {
                gd.flags[p2] = g->sync[p2];
                gd.ws[p2] = g->ws[p2];
            }
            gd.epoch = g->sync[q] + 48;
            gd.err = reinterpret_cast<int*>(g->sync[q] + 56);
            gd.rank = q;
            gd.n = n;
            int khz = 0;   // wall-clock rate (100 MHz on gfx9); a 2 s bound
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, g->dev[q]) != hipSuccess || khz <= 0)
                khz = 100000;
            gd.waitTicks = (uint64_t)khz * 1000ull * 2ull;
            g->ctx[q]->grp = &gd;
        }
        // Graph-captured slots only when every rank has a device of its own: two ranks on one
        // device may see their graph launches share a hardware queue, where a rank's waiting
        // k_grp_sync would block the peer it waits for (measured: a ~1 s stall, then the timeout)
        bool distinct = true;
        for (int a = 0; a < n; a++)
            for (int b2 = a + 1; b2 < n; b2++) distinct = distinct && g->dev[a] != g->dev[b2];
        for (int q = 0; q < n; q++) g->ctx[q]->grpGraphs = distinct;
    }
    g->abort.store(false);
    g->arrive.store(0);
    g->ntev = 0;
    // every rank writes its own copy of the outputs; the owners' slices are merged below
    struct Out {
        std::vector<double> q, t, X, chi, trace;
        std::vector<uint8_t> er;
        lba_result res{};
    };
    std::vector<Out> outs(n);
    for (int q = 0; q < n; q++) {
        Out& u = outs[q];
        u.q.assign(4 * NP + 1, 0.0); u.t.assign(3 * NP + 1, 0.0); u.X.assign(3 * NM + 1, 0.0);
        u.chi.assign(NE + 1, 0.0); u.er.assign(NE + 1, 0); u.trace.assign(4 * 64, 0.0);
        u.res = lba_result{u.q.data(), u.t.data(), u.X.data(), u.er.data(), u.chi.data(), {0, 0}, 0,
                           q == 0 && r->trace ? u.trace.data() : nullptr, 0, 0};
    }
    // No rank may block in a device-synchronising host call (hipFree, and the first-use growth of
    // the arena / pinned staging) while a peer's exchange kernel waits for it.  A problem larger
    // than any this group has solved is first solved once per rank alone (world 1, one rank at a
    // time), which grows every arena and staging buffer to what the sharded solve needs; then the
    // arenas are consolidated, so inside the sharded solves nothing is allocated or freed.
    if (!g->hostPath && (NP > g->warmNP || NM > g->warmNM || NE > g->warmNE)) {
        for (int q = 0; q < n; q++) {
            lba_context* c = g->ctx[q];
            const orbamd::GrpDev* gp = c->grp;
            const bool gg = c->grpGraphs;
            TRY(lba_set_comm(c, 0, 1, nullptr, 0, nullptr, nullptr));
            lba_result dry = outs[q].res;
            dry.trace = nullptr;
            const int st0 = lba_solve(c, p, o, nullptr, &dry);
            TRY(lba_set_comm(c, q, n, g->ws[q], g->wsDoubles, group_allreduce, &g->ranks[q]));
            c->wsOut = g->res[q];
            c->grp = gp;
            c->grpGraphs = gg;
            if (st0 != ORB_OK) return st0;
        }
        g->warmNP = std::max(g->warmNP, NP);
        g->warmNM = std::max(g->warmNM, NM);
        g->warmNE = std::max(g->warmNE, NE);
    }
    for (int q = 0; q < n; q++) {
        ORB_HIP_TRY(hipSetDevice(g->dev[q]));
        ORB_HIP_TRY(hipStreamSynchronize(g->ctx[q]->stream));
        lba_free_all(g->ctx[q]);
    }
    std::vector<int> st(n, ORB_OK);
    auto run = [&](int q) {
        st[q] = lba_solve(g->ctx[q], p, o, stop, &outs[q].res);
        if (st[q] != ORB_OK) g->abort.store(true);
    };
    std::vector<std::thread> th;
    for (int q = 1; q < n; q++) th.emplace_back(run, q);
    run(0);
    for (auto& t : th) t.join();
    if (std::getenv("ORB_LBA_GROUP_DEBUG"))
        for (int q = 0; q < n; q++) {
            uint32_t w[64] = {0};
            if (!g->hostPath) {
                (void)hipSetDevice(g->dev[q]);
                (void)hipMemcpy(w, g->sync[q], 256, hipMemcpyDeviceToHost);
            }
            fprintf(stderr, "lba_group rank %d: status %d ready %u read %u epoch %u err %u\n", q, st[q], w[0], w[32], w[48],
                    w[56]);
        }
    for (int q = 0; q < n; q++)
        if (st[q] != ORB_OK) return st[q];
    if (!g->hostPath) {   // a timed-out wait on any rank fails the solve; collectives counted from the epoch
        for (int q = 0; q < n; q++) {
            uint32_t w[64];
            ORB_HIP_TRY(hipSetDevice(g->dev[q]));
            ORB_HIP_TRY(hipMemcpy(w, g->sync[q], 256, hipMemcpyDeviceToHost));
            if (w[56] != 0) return ORB_EGPU;
            if (q == 0) g->exchanges += (long)w[48];
        }
    }
    // rank 0's exchange timing (its stream is idle: lba_solve waited for its last group)
    if (g->ntev) {
        ORB_HIP_TRY(hipSetDevice(g->dev[0]));
        for (size_t i = 0; i < g->ntev; i++) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, g->tev[i].first, g->tev[i].second) == hipSuccess) g->exchangeMs += ms;
        }
        g->exchanges += (long)g->ntev;
    }
    const lba_result& r0 = outs[0].res;
    if (r->pose_q) std::memcpy(r->pose_q, outs[0].q.data(), 32 * NP);
    if (r->pose_t) std::memcpy(r->pose_t, outs[0].t.data(), 24 * NP);
    for (int q = 0; q < n; q++) {   // landmark shards: [q M / n, (q+1) M / n) from rank q
        const size_t a = (size_t)((long long)NM * q / n), b = (size_t)((long long)NM * (q + 1) / n);
        if (r->point_xyz && b > a) std::memcpy(r->point_xyz + 3 * a, outs[q].X.data() + 3 * a, 24 * (b - a));
    }
    for (size_t e = 0; e < NE; e++) {   // each edge's chi2 / erase flag from its landmark's owner (others 0)
        double c2 = 0.0;
        uint8_t er = 0;
        for (int q = 0; q < n; q++) { c2 += outs[q].chi[e]; er |= outs[q].er[e]; }
        if (r->edge_chi2) r->edge_chi2[e] = c2;
        if (r->edge_erase) r->edge_erase[e] = er;
    }
    r->iterations[0] = r0.iterations[0];
    r->iterations[1] = r0.iterations[1];
    r->trials = r0.trials;
    r->aborted = r0.aborted;
    r->n_trace = 0;
    if (r->trace && r0.n_trace > 0) {
        std::memcpy(r->trace, outs[0].trace.data(), 32 * (size_t)r0.n_trace);
        r->n_trace = r0.n_trace;
    }
    return ORB_OK;
} ORB_ABI_CATCH

int lba_group_stats(lba_group* g, double* exchange_ms, long* n_exchanges) try {
    if (!g) return ORB_EINVAL;
    if (exchange_ms) *exchange_ms = g->exchangeMs;
    if (n_exchanges) *n_exchanges = g->exchanges;
    return ORB_OK;
} ORB_ABI_CATCH

}  // extern "C"
