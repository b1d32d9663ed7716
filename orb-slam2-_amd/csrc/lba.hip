// MI355X-native Optimizer::LocalBundleAdjustment (R/src/Optimizer.cpp:564-918) — the g2o
// Levenberg–Marquardt / BlockSolver<6,3> Schur pipeline it runs, rebuilt for gfx950 in f64.
// R/ = /root/reference/ORB-SLAM2注释版/, G/ = R/Thirdparty/g2o/g2o/.
//
// Per LM outer iteration (G/core/optimization_algorithm_levenberg.cpp:61-164):
//   k_edge_errors     computeActiveErrors + robust chi2 per edge (one thread per edge)
//   k_edge_linearize  EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ Jacobians + Huber-weighted
//                     quadratic-form blocks per edge (G/core/base_binary_edge.hpp:54-120)
//   k_point_reduce    Hll, b_l per landmark; k_pose_reduce: Hpp, b_p per pose (one wave per pose)
// Per LM trial (lambda):
//   k_point_schur     D^-1 = (Hll + lambda I)^-1, per-edge Hpl D^-1 and Hpl D^-1 b_l
//   k_schur_pairs     reduced camera matrix S = Hpp + lambda I - sum W D^-1 W^T, one wave per
//                     6x6 pose-pair block, deterministic contribution order (G/core/block_solver.hpp:382-433)
//   k_ldlt_solve      dense LDL^T of S in one workgroup (LinearSolverEigen's SimplicialLDLT role)
//   k_backsub / k_update / k_edge_errors / reductions: x_l, oplus (SE3Quat::exp * T), chi2, scale.
// The LM control flow (rho test, lambda schedule, Raul's stop rule, push/pop, the two
// optimize() rounds and the chi2 outlier passes) runs on the host exactly as g2o/ORB-SLAM2 do,
// reading back two scalars per trial.  Every reduction has a fixed order, so results are
// bitwise reproducible run to run.  With a communicator (lba_set_comm) the landmarks are
// sharded over ranks and S, b_s and the chi2 / scale scalars are all-reduced (RCCL via the
// caller's callback); every rank then solves the same reduced system.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "common.h"
#include "se3.h"

#ifdef ORB_TIMING   // instrumented variant (tools/build_variant.py)
#define TSTAMP(v) const long long v = clock64()
#define TACC(acc, a) acc += clock64() - (a)
#else
#define TSTAMP(v)
#define TACC(acc, a)
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
    double* err;                // [NE][3] last computed error
    // active structure (per optimize())
    const int32_t* act;         // active edges
    int nact;
    const int32_t* poseIdx;     // pose -> hessian index or -1
    const int32_t* ptLocal;     // global point -> local index or -1 (owned points only)
    const int32_t* ptGlob;      // local -> global point
    const int32_t* actPos;      // edge -> position in act (or -1)
    const int32_t *actPt, *actPi; // per act position: local point, pose hessian index (-1 fixed)
    int P, M;                   // free active poses, owned active points
    const int32_t *ptStart, *ptEdges;     // CSR by local point (edge ids, sorted by pose index)
    const int32_t *poStart, *poEdges;     // CSR by pose index (edge ids)
    const int32_t *prStart, *prE1, *prE2; // CSR by pose-pair block (i<=j), contributions (act positions)
    // linearisation (indexed by act position)
    double *Hll_e, *Hpp_e, *Hpl_e, *bl_e, *bp_e, *BD, *coef, *echi;
    // reduced per vertex
    double *Hll, *bl, *Dinv, *db, *Hpp, *bp;   // db = Dinv b_l
    double *S, *bs, *x;         // x: [6P + 3M]
    double* red;                // reduction scratch
    int* flags;                 // [0] LDLT failure
    LmState* lm;                // LM control state (device)
};

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

// computeError for the active edges; echi[k] = robust chi2 (activeRobustChi2 term)
__global__ __launch_bounds__(256) void k_edge_errors(LbaDev d, double hmono, double hstereo, int want) {
    if (lm_off(d.lm, want)) return;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= d.nact) return;
    const int e = d.act[k];
    double Xc[3];
    d_transform(d, d.eps[e], d.ept[e], Xc);
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
}

// Jacobians + Huber-weighted quadratic-form blocks per active edge.
// Hll_e: 3x3 upper (00 01 02 11 12 22); Hpp_e: 6x6 upper row-major (21); Hpl_e: 6x3; bl_e: 3; bp_e: 6
__global__ __launch_bounds__(256) void k_edge_linearize(LbaDev d, double hmono, double hstereo) {
    if (lm_off(d.lm, 0)) return;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= d.nact) return;
    const int e = d.act[k];
    const int pose = d.eps[e];
    double R[9], Xc[3];
    d_quat_to_R(d.q + 4 * pose, R);
    d_transform(d, pose, d.ept[e], Xc);
    const double x = Xc[0], y = Xc[1], z = Xc[2], z_2 = z * z;
    const double* cam = d.cam + 5 * e;
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    const bool st = d.est[e] != 0;
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
    const double w = d.info[e];
    const double* er = d.err + 3 * e;
    double rho1 = 1.0;
    if (d.robust[e]) {
        const double chi = d_edge_chi2(d, e);
        const double delta = st ? hstereo : hmono;
        if (chi > delta * delta) rho1 = delta / sqrt(chi);
    }
    const double W = rho1 * w;
    double om[3];
    for (int r = 0; r < 3; r++) om[r] = r < D ? -(w * er[r]) * rho1 : 0.0;
    double* hl = d.Hll_e + 6 * (size_t)k;
    double* bl = d.bl_e + 3 * (size_t)k;
    {
        int o = 0;
        for (int i = 0; i < 3; i++) {
            double s = 0;
            for (int r = 0; r < D; r++) s += A[r * 3 + i] * om[r];
            bl[i] = s;
            for (int j = i; j < 3; j++) {
                double h = 0;
                for (int r = 0; r < D; r++) h += A[r * 3 + i] * W * A[r * 3 + j];
                hl[o++] = h;
            }
        }
    }
    if (d.poseIdx[pose] >= 0) {
        double* hp = d.Hpp_e + 21 * (size_t)k;
        double* bp = d.bp_e + 6 * (size_t)k;
        double* hpl = d.Hpl_e + 18 * (size_t)k;
        int o = 0;
        for (int i = 0; i < 6; i++) {
            double s = 0;
            for (int r = 0; r < D; r++) s += B[r * 6 + i] * om[r];
            bp[i] = s;
            for (int j = i; j < 6; j++) {
                double h = 0;
                for (int r = 0; r < D; r++) h += B[r * 6 + i] * W * B[r * 6 + j];
                hp[o++] = h;
            }
            for (int j = 0; j < 3; j++) {
                double h = 0;
                for (int r = 0; r < D; r++) h += B[r * 6 + i] * W * A[r * 3 + j];
                hpl[i * 3 + j] = h;
            }
        }
    }
}

// Hll, b_l per owned landmark (edges in pose-index order)
__global__ __launch_bounds__(256) void k_point_reduce(LbaDev d) {
    if (lm_off(d.lm, 0)) return;
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l >= d.M) return;
    double h[6] = {0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
    for (int a = d.ptStart[l]; a < d.ptStart[l + 1]; a++) {
        const int k = d.actPos[d.ptEdges[a]];
        for (int i = 0; i < 6; i++) h[i] += d.Hll_e[6 * (size_t)k + i];
        for (int i = 0; i < 3; i++) b[i] += d.bl_e[3 * (size_t)k + i];
    }
    double* H = d.Hll + 9 * (size_t)l;
    H[0] = h[0]; H[1] = h[1]; H[2] = h[2];
    H[3] = h[1]; H[4] = h[3]; H[5] = h[4];
    H[6] = h[2]; H[7] = h[4]; H[8] = h[5];
    for (int i = 0; i < 3; i++) d.bl[3 * (size_t)l + i] = b[i];
}

// Hpp, b_p per pose: one wave per pose, lanes stride over the pose's edges, fixed tree.
__global__ __launch_bounds__(64) void k_pose_reduce(LbaDev d) {
    if (lm_off(d.lm, 0)) return;
    const int p = blockIdx.x, lane = threadIdx.x;
    double acc[27];
    for (int i = 0; i < 27; i++) acc[i] = 0;
    for (int a = d.poStart[p] + lane; a < d.poStart[p + 1]; a += 64) {
        const int k = d.actPos[d.poEdges[a]];
        for (int i = 0; i < 21; i++) acc[i] += d.Hpp_e[21 * (size_t)k + i];
        for (int i = 0; i < 6; i++) acc[21 + i] += d.bp_e[6 * (size_t)k + i];
    }
    for (int i = 0; i < 27; i++) {
        double v = acc[i];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[i] = v;
    }
    if (lane == 0) {
        double* H = d.Hpp + 36 * (size_t)p;
        int o = 0;
        for (int i = 0; i < 6; i++)
            for (int j = i; j < 6; j++) {
                H[i * 6 + j] = acc[o];
                H[j * 6 + i] = acc[o];
                o++;
            }
        for (int i = 0; i < 6; i++) d.bp[6 * (size_t)p + i] = acc[21 + i];
    }
}

// Per landmark with lambda: Dinv (Eigen 3x3 cofactor inverse) and db = Dinv b_l
// (G/core/block_solver.hpp:380-398).
__global__ __launch_bounds__(256) void k_point_schur(LbaDev d) {
    if (lm_off(d.lm, 1)) return;
    const double lambda = d.lm->lambda;
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l >= d.M) return;
    double m[9];
    for (int i = 0; i < 9; i++) m[i] = d.Hll[9 * (size_t)l + i];
    m[0] += lambda; m[4] += lambda; m[8] += lambda;
    double c[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            c[i * 3 + j] = m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
        }
    const double det = c[0] * m[0] + c[3] * m[3] + c[6] * m[6];
    const double invdet = 1.0 / det;
    double Di[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Di[j * 3 + i] = c[i * 3 + j] * invdet;
    for (int i = 0; i < 9; i++) d.Dinv[9 * (size_t)l + i] = Di[i];
    const double* b = d.bl + 3 * (size_t)l;
    for (int i = 0; i < 3; i++) d.db[3 * (size_t)l + i] = Di[i * 3] * b[0] + Di[i * 3 + 1] * b[1] + Di[i * 3 + 2] * b[2];
}

// Per active edge with a free pose: BD_e = Hpl_e Dinv, coef_e = Hpl_e Dinv b_l.
__global__ __launch_bounds__(256) void k_edge_schur(LbaDev d) {
    if (lm_off(d.lm, 1)) return;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= d.nact || d.actPi[k] < 0) return;
    const int l = d.actPt[k];
    double Di[9], db[3];
    for (int i = 0; i < 9; i++) Di[i] = d.Dinv[9 * (size_t)l + i];
    for (int i = 0; i < 3; i++) db[i] = d.db[3 * (size_t)l + i];
    const double* Bi = d.Hpl_e + 18 * (size_t)k;
    double* BD = d.BD + 18 * (size_t)k;
    double* cf = d.coef + 6 * (size_t)k;
    for (int r = 0; r < 6; r++) {
        for (int q = 0; q < 3; q++)
            BD[r * 3 + q] = Bi[r * 3] * Di[q] + Bi[r * 3 + 1] * Di[3 + q] + Bi[r * 3 + 2] * Di[6 + q];
        cf[r] = Bi[r * 3] * db[0] + Bi[r * 3 + 1] * db[1] + Bi[r * 3 + 2] * db[2];
    }
}

// S_ij block of the reduced camera system, one workgroup per pose pair (i <= j):
// S_ij = [i == j](Hpp_i + lambda I) - sum_c BD_c Hpl_c'^T over the landmarks c seen by both
// (G/core/block_solver.hpp:408-440).  Thread t owns output element t % 36 of contribution
// group t / 36 (7 groups); the group partial sums meet in LDS.
constexpr int kSpGroups = 7;
__global__ __launch_bounds__(256) void k_schur_pairs(LbaDev d, int addDiag, const int32_t* pairI,
                                                     const int32_t* pairJ) {
    if (lm_off(d.lm, 1)) return;
    const double lambda = d.lm->lambda;
    __shared__ double part[kSpGroups][36];
    const int pr = blockIdx.x, tid = threadIdx.x;
    const int bi = pairI[pr], bj = pairJ[pr];
    const int o = tid % 36, grp = tid / 36;
    const int r = o / 6, q = o % 6;
    if (grp < kSpGroups) {
        double acc = 0.0;
        const int c0 = d.prStart[pr], c1 = d.prStart[pr + 1];
        for (int c = c0 + grp; c < c1; c += kSpGroups) {
            const double* BD = d.BD + 18 * (size_t)d.prE1[c] + r * 3;
            const double* Bj = d.Hpl_e + 18 * (size_t)d.prE2[c] + q * 3;
            acc += BD[0] * Bj[0] + BD[1] * Bj[1] + BD[2] * Bj[2];
        }
        part[grp][o] = acc;
    }
    __syncthreads();
    if (tid < 36) {
        double sacc = 0.0;
        for (int g2 = 0; g2 < kSpGroups; g2++) sacc += part[g2][tid];
        double v = 0.0;
        if (bi == bj && addDiag) {     // rank 0 carries the (already all-reduced) Hpp + lambda I
            v = d.Hpp[36 * (size_t)bi + tid];
            if (r == q) v += lambda;
        }
        v -= sacc;
        const int n = 6 * d.P;
        d.S[(size_t)(6 * bi + r) * n + 6 * bj + q] = v;
        d.S[(size_t)(6 * bj + q) * n + 6 * bi + r] = v;
    }
}

// b_s = b_p - sum_e coef_e, one wave per pose
__global__ __launch_bounds__(64) void k_bschur(LbaDev d, int addBp) {
    if (lm_off(d.lm, 1)) return;
    const int p = blockIdx.x, lane = threadIdx.x;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int a = d.poStart[p] + lane; a < d.poStart[p + 1]; a += 64) {
        const double* cf = d.coef + 6 * (size_t)d.actPos[d.poEdges[a]];
        for (int i = 0; i < 6; i++) acc[i] += cf[i];
    }
    for (int i = 0; i < 6; i++) {
        double v = acc[i];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[i] = v;
    }
    if (lane < 6) {
        double s = 0;
        for (int i = 0; i < 6; i++) s = (i == lane) ? acc[i] : s;
        d.bs[6 * p + lane] = (addBp ? d.bp[6 * p + lane] : 0.0) - s;
    }
}

constexpr int kLdltW = 8;     // panel width (columns per pair of workgroup barriers)
constexpr int kLdltT = 512;   // 8 waves: 2 per SIMD for the trailing update
constexpr int kLdltMaxN = 192; // panel rows held in registers: 3 per lane

// Broadcast of lane `src` (a compile-time constant at every call site) through two
// v_readlane_b32 into SGPRs: a few cycles, against a ds_bpermute round trip for __shfl.
__device__ __forceinline__ double shfl_d(double v, int src) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Dense LDL^T (no pivoting; fails only on a zero pivot, like SimplicialLDLT) + solve, one
// workgroup of kLdltT threads; the n x n matrix is staged in LDS when it fits (n <= 136, i.e.
// up to 22 free keyframes), otherwise factored in place in global memory (L2-resident).
// Element recurrence (oracle/lba_oracle.c states it column by column): with W(i,k) the value
// of A(i,k) before the division by d_k and L(i,k) = W(i,k)/d_k,
//     A(i,j) = fma(-W(i,k), L(j,k), A(i,j))   for k = 0 .. j-1 in order,
// one fused multiply-add per update (against (L_ik L_jk) d_k, three rounded operations).
// W is kept in the upper triangle, L in the lower.  Right-looking in panels of kLdltW columns:
//  * wave 0 factors the panel in registers (3 panel rows per lane, pivots and L entries
//    broadcast with v_readlane);
//  * all threads apply the panel's updates to the trailing lower triangle in 4 x 4 register
//    tiles, each element taking them in column order;
// so every element sees the recurrence's exact operation sequence, with two workgroup barriers
// per panel.  The triangular solves (y_i = fma(-L_ik, y_k, y_i), k in order) are blocked the
// same way on one wave.
// Panel [jb, je) of the factorisation on one wave, rows jb + lane + 64u for u < NS (NS = slots
// that hold rows: the matrix has n - jb rows left).  Column j: d_j = A(j,j); W(i,j) = A(i,j)
// before the division goes to the upper triangle at (j, i), L(i,j) = W(i,j)/d_j to the lower;
// the panel's later columns take A(i,k) = fma(-W(i,j), L(k,j), A(i,k)), and the forward
// substitution advances with the factorisation: y_i = fma(-L(i,j), y_j, y_i) for i > j once
// y_j is final.  Values computed on or above the diagonal are not stored.  Returns false on a
// zero or non-finite pivot.
template <int NS>
__device__ __forceinline__ bool ldlt_panel(double* __restrict__ A, int ld, int n, int jb, int je, double* __restrict__ dg,
                                           double* __restrict__ y, int lane) {
    double P[NS][kLdltW], Wp[NS][kLdltW], Y[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) {
        const int r = jb + lane + 64 * u;
        Y[u] = r < n ? y[r] : 0.0;
#pragma unroll
        for (int c = 0; c < kLdltW; c++) {
            P[u][c] = (r < n && jb + c < je) ? A[(size_t)r * ld + jb + c] : 0.0;
            Wp[u][c] = 0.0;
        }
    }
    bool bad = false;
#pragma unroll
    for (int c = 0; c < kLdltW; c++) {
        const int j = jb + c;
        if (j < je && !bad) {
            const double dj = shfl_d(P[0][c], c);   // A(j, j): row j is lane c, slot 0
            if (dj == 0.0 || !isfinite(dj)) {
                bad = true;
            } else {
#pragma unroll
                for (int u = 0; u < NS; u++) {
                    Wp[u][c] = P[u][c];
                    P[u][c] = P[u][c] / dj;
                }
                if (lane == 0) dg[j] = dj;
                const double yj = shfl_d(Y[0], c);   // final: every k < j has been applied
#pragma unroll
                for (int u = 0; u < NS; u++)
                    if (jb + lane + 64 * u > j) Y[u] = __builtin_fma(-P[u][c], yj, Y[u]);
                double lkv[kLdltW];
#pragma unroll
                for (int k = c + 1; k < kLdltW; k++) lkv[k] = shfl_d(P[0][c], k);   // L(jb+k, j)
#pragma unroll
                for (int k = c + 1; k < kLdltW; k++)
#pragma unroll
                    for (int u = 0; u < NS; u++) P[u][k] = __builtin_fma(-Wp[u][c], lkv[k], P[u][k]);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < NS; u++) {
        const int r = jb + lane + 64 * u;
        if (r < n) y[r] = Y[u];
#pragma unroll
        for (int c = 0; c < kLdltW; c++)
            if (r < n && r > jb + c && jb + c < je) {
                A[(size_t)r * ld + jb + c] = P[u][c];      // L(r, jb+c), strict lower
                A[(size_t)(jb + c) * ld + r] = Wp[u][c];   // W(r, jb+c) at (jb+c, r)
            }
    }
    return !bad;
}

template <bool kLds>
__global__ __launch_bounds__(kLdltT) void k_ldlt_solve(double* __restrict__ Ag, const double* __restrict__ b, int n,
                                                       double* __restrict__ x, int* __restrict__ flags,
                                                       const LmState* st) {
    if (lm_off(st, 1)) return;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    TSTAMP(t_l0);
    long long tPanel = 0, tTrail = 0, tPLoad = 0, tPCol = 0, tFLoad = 0, tFChain = 0, tFRows = 0;
    (void)tPanel; (void)tTrail; (void)tPLoad; (void)tPCol; (void)tFLoad; (void)tFChain; (void)tFRows;
    // (forward substitution runs inside the panels; tPLoad/tPCol/tF* stay 0 in this layout)
    // LDS rows padded to an odd number of doubles: the panel's column accesses (lanes one row
    // apart) then spread over the banks instead of hitting a few of them
    const int ld = kLds ? (n | 1) : n;
    double* A = kLds ? sh : Ag;
    double* dg = sh + (kLds ? (size_t)n * ld : 0);
    double* y = dg + n;
    __shared__ int failS;
    const int tid = threadIdx.x, lane = tid & 63;
    if (kLds) {
        for (int t0 = 0; t0 < n * n; t0 += kLdltT * 8) {   // 8 loads in flight per thread
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = t0 + u * kLdltT + tid < n * n ? Ag[t0 + u * kLdltT + tid] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int t = t0 + u * kLdltT + tid;
                if (t < n * n) A[(size_t)(t / n) * ld + t % n] = v[u];
            }
        }
    }
    for (int t = tid; t < n; t += kLdltT) y[t] = b[t];
    if (tid == 0) failS = 0;
    __syncthreads();
#ifdef ORB_TIMING
    const long long t_p_first = clock64() - t_l0;
#endif
    for (int jb = 0; jb < n; jb += kLdltW) {
        const int je = min(jb + kLdltW, n);
        TSTAMP(t_p0);
        if (tid < 64) {
            const int ns = (n - jb + 63) >> 6;
            const bool okp = ns == 1   ? ldlt_panel<1>(A, ld, n, jb, je, dg, y, lane)
                             : ns == 2 ? ldlt_panel<2>(A, ld, n, jb, je, dg, y, lane)
                                       : ldlt_panel<3>(A, ld, n, jb, je, dg, y, lane);
            if (!okp && lane == 0) failS = 1;
        }
        __syncthreads();
        TACC(tPanel, t_p0);
        TSTAMP(t_t0);
        if (failS) break;
        // ---- trailing lower triangle (rows, columns >= je) in 4 x 4 tiles, one tile per thread
        //      (triangular numbering t -> (ti, tk), tk <= ti); element (i, k) takes
        //      A(i,k) = fma(-W(i,p), L(k,p), A(i,k)) for the panel's columns p in order
        {
            const int m = n - je, T = (m + 3) >> 2, nt = T * (T + 1) / 2;
            for (int t = tid; t < nt; t += kLdltT) {
                int ti = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
                while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
                while (ti * (ti + 1) / 2 > t) ti--;
                const int tk = t - ti * (ti + 1) / 2;
                double wi[4][kLdltW], lk[4][kLdltW], v[4][4];
#pragma unroll
                for (int p = 0; p < kLdltW; p++)
#pragma unroll
                    for (int a2 = 0; a2 < 4; a2++) {
                        const int i = je + 4 * ti + a2, k = je + 4 * tk + a2;
                        wi[a2][p] = (i < n && jb + p < je) ? A[(size_t)(jb + p) * ld + i] : 0.0;   // W(i, jb+p)
                        lk[a2][p] = (k < n && jb + p < je) ? A[(size_t)k * ld + jb + p] : 0.0;     // L(k, jb+p)
                    }
#pragma unroll
                for (int a2 = 0; a2 < 4; a2++)
#pragma unroll
                    for (int b2 = 0; b2 < 4; b2++) {
                        const int i = je + 4 * ti + a2, k = je + 4 * tk + b2;
                        v[a2][b2] = (i < n && k <= i) ? A[(size_t)i * ld + k] : 0.0;
                    }
#pragma unroll
                for (int p = 0; p < kLdltW; p++)
#pragma unroll
                    for (int a2 = 0; a2 < 4; a2++)
#pragma unroll
                        for (int b2 = 0; b2 < 4; b2++) v[a2][b2] = __builtin_fma(-wi[a2][p], lk[b2][p], v[a2][b2]);
#pragma unroll
                for (int a2 = 0; a2 < 4; a2++)
#pragma unroll
                    for (int b2 = 0; b2 < 4; b2++) {
                        const int i = je + 4 * ti + a2, k = je + 4 * tk + b2;
                        if (i < n && k <= i) A[(size_t)i * ld + k] = v[a2][b2];
                    }
            }
        }
        __syncthreads();
        TACC(tTrail, t_t0);
    }
    TSTAMP(t_l1);
    if (failS) {
        if (tid == 0) flags[0] = 1;
        return;
    }
    if (tid >= 64) return;
    for (int i = lane; i < n; i += 64) y[i] = y[i] / dg[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- backward substitution with L^T (per element: y_i -= L_ki x_k, k descending)
    for (int ke = n; ke > 0; ke -= kLdltW) {
        const int kb = max(ke - kLdltW, 0), w = ke - kb;
        double Ab[kLdltW], Ar[3][kLdltW], yr[3];
#pragma unroll
        for (int c = 0; c < kLdltW; c++) Ab[c] = (lane < c && c < w) ? A[(size_t)(kb + c) * ld + kb + lane] : 0.0;
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = lane + 64 * u;
            yr[u] = i < kb ? y[i] : 0.0;
#pragma unroll
            for (int c = 0; c < kLdltW; c++) Ar[u][c] = (i < kb && c < w) ? A[(size_t)(kb + c) * ld + i] : 0.0;
        }
        double xb = lane < w ? y[kb + lane] : 0.0;
#pragma unroll
        for (int c = kLdltW - 1; c >= 0; c--) {
            if (c >= w) continue;
            const double xc = shfl_d(xb, c);
            if (lane < c) xb = __builtin_fma(-Ab[c], xc, xb);
        }
        double xs[kLdltW];
#pragma unroll
        for (int c = 0; c < kLdltW; c++) xs[c] = shfl_d(xb, c);
        if (lane < w) y[kb + lane] = xb;
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = lane + 64 * u;
            double v = yr[u];
#pragma unroll
            for (int c = kLdltW - 1; c >= 0; c--)
                if (c < w) v = __builtin_fma(-Ar[u][c], xs[c], v);
            if (i < kb) y[i] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    for (int i = lane; i < n; i += 64) x[i] = y[i];
    if (tid == 0) flags[0] = 0;
#ifdef ORB_TIMING
    if (tid == 0) printf("ldlt n %d: stage %lld panel %lld (load %lld cols %lld) trailing %lld solves %lld (fwd load %lld chain %lld rows %lld)\n", n, t_p_first, tPanel, tPLoad, tPCol, tTrail, clock64() - t_l1, tFLoad, tFChain, tFRows);
#endif
}

// x_l = Dinv (b_l - sum_e Hpl_e^T x_p(pose_e))
__global__ __launch_bounds__(256) void k_backsub(LbaDev d) {
    if (lm_off(d.lm, 1)) return;
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l >= d.M) return;
    double cl[3] = {d.bl[3 * (size_t)l], d.bl[3 * (size_t)l + 1], d.bl[3 * (size_t)l + 2]};
    for (int a = d.ptStart[l]; a < d.ptStart[l + 1]; a++) {
        const int e = d.ptEdges[a];
        const int pi = d.poseIdx[d.eps[e]];
        if (pi < 0) continue;
        const double* Bi = d.Hpl_e + 18 * (size_t)d.actPos[e];
        for (int q = 0; q < 3; q++)
            for (int r = 0; r < 6; r++) cl[q] += Bi[r * 3 + q] * (-d.x[6 * pi + r]);
    }
    const double* Di = d.Dinv + 9 * (size_t)l;
    double* xl = d.x + 6 * (size_t)d.P + 3 * (size_t)l;
    for (int q = 0; q < 3; q++) xl[q] = Di[q * 3] * cl[0] + Di[q * 3 + 1] * cl[1] + Di[q * 3 + 2] * cl[2];
}

// push (backup) + oplus for all free poses and owned points
__global__ __launch_bounds__(256) void k_update(LbaDev d, int nposes, const int32_t* freePoses, int applyPoses) {
    if (lm_off(d.lm, 1)) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < d.M) {
        const int g = d.ptGlob[i];
        for (int j = 0; j < 3; j++) {
            d.bX[3 * (size_t)g + j] = d.X[3 * (size_t)g + j];
            d.X[3 * (size_t)g + j] += d.x[6 * (size_t)d.P + 3 * (size_t)i + j];
        }
    }
    if (i < nposes && applyPoses) {
        const int p = freePoses[i];
        const int k = d.poseIdx[p];
        double q[4], t[3], u[6];
        for (int j = 0; j < 4; j++) { q[j] = d.q[4 * p + j]; d.bq[4 * p + j] = q[j]; }
        for (int j = 0; j < 3; j++) { t[j] = d.t[3 * p + j]; d.bt[3 * p + j] = t[j]; }
        for (int j = 0; j < 6; j++) u[j] = d.x[6 * k + j];
        d_se3_exp_left(u, q, t);
        for (int j = 0; j < 4; j++) d.q[4 * p + j] = q[j];
        for (int j = 0; j < 3; j++) d.t[3 * p + j] = t[j];
    }
}

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

// t^3 rounded once (double-double product): the host path used std::pow(t, 3), which glibc
// rounds correctly except in vanishingly rare cases.
__device__ __forceinline__ double cube_rn(double t) {
    const double p = t * t, ep = __builtin_fma(t, t, -p);
    const double q = p * t, eq = __builtin_fma(p, t, -q);
    return q + __builtin_fma(ep, t, eq);
}

// Start of an LM iteration (G/core/optimization_algorithm_levenberg.cpp:61-90): currentChi
// from the linearisation's robust chi2 (red[0]), lambda from computeLambdaInit (red[1]) at it 0.
__global__ void k_lm_begin(LmState* st, const double* __restrict__ red) {
    if (threadIdx.x != 0 || st->phase != 0) return;
    st->pop = 0;
    st->currentChi = red[0];
    st->iniChi = red[0];
    if (st->it == 0) {
        st->lambda = 1e-5 * red[1];   // tau = 1e-5
        st->ni = 2;
        st->nBad = 0;
    }
    st->qmax = 0;
    st->phase = 1;
}

// Decision after a trial (:120-160) and the end-of-iteration bookkeeping of
// SparseOptimizer::optimize / OptimizationAlgorithmLevenberg (termination on qmax == max
// trials, rho == 0 or three iterations without 1e-3 relative progress).
__global__ void k_lm_decide(LmState* st, const double* __restrict__ red, const int* __restrict__ flags, int maxTrials,
                            int iterations, int fixedIterations, double* __restrict__ trace) {
    if (threadIdx.x != 0) return;
    st->pop = 0;
    if (st->phase != 1) return;
    const double tempChi = flags[0] ? DBL_MAX : red[0];
    double rho = st->currentChi - tempChi;
    const double scale = red[2] + 1e-3;
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
    if (rho < 0 && st->qmax < maxTrials) return;   // next trial of this iteration
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
    st->phase = (go && st->it < iterations) ? 0 : 2;
}

// chi2 / depth of every edge (final check and outlier pass): chi2() uses the stored error
__global__ __launch_bounds__(256) void k_edge_check(LbaDev d, int ne, double* __restrict__ chi2,
                                                    uint8_t* __restrict__ depthPos) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= ne) return;
    chi2[e] = d_edge_chi2(d, e);
    double Xc[3];
    d_transform(d, d.eps[e], d.ept[e], Xc);
    depthPos[e] = Xc[2] > 0.0 ? 1 : 0;
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
    size_t wsDoubles = 0;
    lba_allreduce_fn allreduce = nullptr;
    void* commUser = nullptr;
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
    std::vector<hipEvent_t> slotEv;                            // per-slot stage timing
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

// Waits for the stream by spinning on an event (a blocking hipStreamSynchronize sleeps and
// adds tens of microseconds per LM trial).
static int lba_wait(lba_context* c) {
    if (hipEventRecord(c->evSync, c->stream) != hipSuccess) return ORB_EGPU;
    hipError_t e;
    while ((e = hipEventQuery(c->evSync)) == hipErrorNotReady) {
    }
    return e == hipSuccess ? ORB_OK : ORB_EGPU;
}

#define TRY(x)                 \
    do {                       \
        int s_ = (x);          \
        if (s_) return s_;     \
    } while (0)

namespace {

struct HostStructure {
    std::vector<int32_t> act, poseIdx, ptLocal, ptGlob, actPos, ptStart, ptEdges, poStart, poEdges, prStart, prE1,
        prE2, pairI, pairJ, freePoses, actPt, actPi;
    int P = 0, M = 0;
};

// initializeOptimization(level) (G/core/sparse_optimizer.cpp:199-267) restricted to the
// landmarks owned by this rank (contiguous range of point indices).
void build_structure(const lba_problem* p, const std::vector<uint8_t>& level, int lvl, int rank, int world,
                     HostStructure& s) {
    const int NP = p->n_poses, NM = p->n_points, NE = p->n_edges;
    const int own0 = (int)((long long)NM * rank / world), own1 = (int)((long long)NM * (rank + 1) / world);
    std::vector<uint8_t> poseAct(NP, 0), ptAct(NM, 0);
    // every rank must see the same pose index mapping: poses active on any rank count
    for (int e = 0; e < NE; e++) {
        if (level[e] != lvl) continue;
        poseAct[p->edge_pose[e]] = 1;
        ptAct[p->edge_point[e]] = 1;
    }
    s.act.clear();
    for (int e = 0; e < NE; e++) {
        if (level[e] != lvl) continue;
        const int pt = p->edge_point[e];
        if (pt < own0 || pt >= own1) continue;
        s.act.push_back(e);
    }
    std::vector<int> order;
    for (int i = 0; i < NP; i++)
        if (poseAct[i] && !p->pose_fixed[i]) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return p->pose_id[a] < p->pose_id[b]; });
    s.poseIdx.assign(NP, -1);
    for (size_t k = 0; k < order.size(); k++) s.poseIdx[order[k]] = (int)k;
    s.freePoses = order;
    s.P = (int)order.size();
    order.clear();
    for (int i = own0; i < own1; i++)
        if (ptAct[i]) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return p->point_id[a] < p->point_id[b]; });
    s.ptLocal.assign(NM, -1);
    for (size_t k = 0; k < order.size(); k++) s.ptLocal[order[k]] = (int)k;
    s.ptGlob = order;
    s.M = (int)order.size();
    s.actPos.assign(NE, -1);
    for (size_t k = 0; k < s.act.size(); k++) s.actPos[s.act[k]] = (int)k;
    s.actPt.resize(s.act.size());
    s.actPi.resize(s.act.size());
    for (size_t k = 0; k < s.act.size(); k++) {
        s.actPt[k] = s.ptLocal[p->edge_point[s.act[k]]];
        s.actPi[k] = s.poseIdx[p->edge_pose[s.act[k]]];
    }
    // CSR by local point, edges sorted by pose index (fixed poses last)
    s.ptStart.assign(s.M + 1, 0);
    for (int e : s.act) s.ptStart[s.ptLocal[p->edge_point[e]] + 1]++;
    for (int i = 0; i < s.M; i++) s.ptStart[i + 1] += s.ptStart[i];
    s.ptEdges.assign(s.act.size(), 0);
    {
        std::vector<int> fill(s.ptStart.begin(), s.ptStart.end() - 1);
        for (int e : s.act) s.ptEdges[fill[s.ptLocal[p->edge_point[e]]]++] = e;
        for (int l = 0; l < s.M; l++) {
            auto key = [&](int e) { const int k = s.poseIdx[p->edge_pose[e]]; return k < 0 ? (1 << 30) : k; };
            std::stable_sort(s.ptEdges.begin() + s.ptStart[l], s.ptEdges.begin() + s.ptStart[l + 1],
                             [&](int a, int b) { return key(a) < key(b); });
        }
    }
    // CSR by pose (edges with a free pose, edge order)
    s.poStart.assign(s.P + 1, 0);
    for (int e : s.act) {
        const int k = s.poseIdx[p->edge_pose[e]];
        if (k >= 0) s.poStart[k + 1]++;
    }
    for (int i = 0; i < s.P; i++) s.poStart[i + 1] += s.poStart[i];
    s.poEdges.assign(s.poStart[s.P], 0);
    {
        std::vector<int> fill(s.poStart.begin(), s.poStart.end() - 1);
        for (int e : s.act) {
            const int k = s.poseIdx[p->edge_pose[e]];
            if (k >= 0) s.poEdges[fill[k]++] = e;
        }
    }
    // pose-pair blocks (i <= j) with their contributions (landmark order, then edge order)
    const int P = s.P;
    const int npairs = P * (P + 1) / 2;
    s.pairI.resize(npairs);
    s.pairJ.resize(npairs);
    std::vector<int> pairOf((size_t)P * P, -1);
    {
        int k = 0;
        for (int i = 0; i < P; i++)
            for (int j = i; j < P; j++) {
                s.pairI[k] = i;
                s.pairJ[k] = j;
                pairOf[(size_t)i * P + j] = k++;
            }
    }
    std::vector<int> cnt(npairs + 1, 0);
    for (int l = 0; l < s.M; l++)
        for (int a = s.ptStart[l]; a < s.ptStart[l + 1]; a++) {
            const int i1 = s.poseIdx[p->edge_pose[s.ptEdges[a]]];
            if (i1 < 0) continue;
            for (int b = a; b < s.ptStart[l + 1]; b++) {
                const int i2 = s.poseIdx[p->edge_pose[s.ptEdges[b]]];
                if (i2 < 0) continue;
                cnt[pairOf[(size_t)i1 * P + i2] + 1]++;
            }
        }
    for (int i = 0; i < npairs; i++) cnt[i + 1] += cnt[i];
    s.prStart = cnt;
    s.prE1.assign(cnt[npairs], 0);
    s.prE2.assign(cnt[npairs], 0);
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int l = 0; l < s.M; l++)
        for (int a = s.ptStart[l]; a < s.ptStart[l + 1]; a++) {
            const int i1 = s.poseIdx[p->edge_pose[s.ptEdges[a]]];
            if (i1 < 0) continue;
            for (int b = a; b < s.ptStart[l + 1]; b++) {
                const int i2 = s.poseIdx[p->edge_pose[s.ptEdges[b]]];
                if (i2 < 0) continue;
                const int pr = pairOf[(size_t)i1 * P + i2];
                s.prE1[fill[pr]] = s.actPos[s.ptEdges[a]];   // act positions (BD / Hpl_e rows)
                s.prE2[fill[pr]] = s.actPos[s.ptEdges[b]];
                fill[pr]++;
            }
        }
}

template <typename T>
int upload(lba_context* c, T** dst, const std::vector<T>& v) {
    TRY(dalloc(c, dst, v.size()));
    if (!v.empty()) ORB_HIP_TRY(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return ORB_OK;
}

}  // namespace

// All-reduce of an LM-loop buffer: staged through the workspace by guarded kernels, so a
// slot whose phase is skipped reduces zeros and leaves the buffer alone.
static int comm_allreduce_g(lba_context* c, double* dbuf, size_t n, int op, const LmState* st, int want) {
    if (c->world <= 1) return ORB_OK;
    if (!c->allreduce || !c->ws || n > c->wsDoubles) return ORB_EINVAL;
    const unsigned g = (unsigned)std::min<size_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_pack, dim3(g), dim3(256), 0, c->stream, c->ws, dbuf, n, st, want);
    if (c->allreduce(c->commUser, 0, n, op) != 0) return ORB_EGPU;
    hipLaunchKernelGGL(k_unpack, dim3(g), dim3(256), 0, c->stream, dbuf, c->ws, n, st, want);
    return ORB_OK;
}

extern "C" {

int lba_create(int device, lba_context** out) {
    if (!out) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    ORB_HIP_TRY(hipSetDevice(device));
    lba_context* c = new lba_context();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return ORB_EGPU; }
    bool ok = hipEventCreateWithFlags(&c->evSync, hipEventDisableTiming) == hipSuccess &&
              hipHostMalloc((void**)&c->h_scal, 4096, hipHostMallocDefault) == hipSuccess;
    for (auto& e : c->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) { lba_destroy(c); return ORB_EGPU; }
    *out = c;
    return ORB_OK;
}

void lba_destroy(lba_context* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    lba_release(c);
    for (auto e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->evSync) (void)hipEventDestroy(c->evSync);
    for (auto e : c->slotEv) (void)hipEventDestroy(e);
    if (c->h_scal) (void)hipHostFree(c->h_scal);
    if (c->stream && c->ownStream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int lba_set_stream(lba_context* c, void* stream, int use_given) {
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
}

int lba_set_comm(lba_context* c, int rank, int world, double* d_workspace, size_t ws_doubles, lba_allreduce_fn fn,
                 void* user) {
    if (!c || world < 1 || rank < 0 || rank >= world) return ORB_EINVAL;
    if (world > 1 && (!d_workspace || !fn)) return ORB_EINVAL;
    c->rank = rank;
    c->world = world;
    c->ws = d_workspace;
    c->wsDoubles = ws_doubles;
    c->allreduce = fn;
    c->commUser = user;
    return ORB_OK;
}

int lba_stats(lba_context* c, double* ms4, int* iters, int* trials) {
    if (!c) return ORB_EINVAL;
    if (ms4) { ms4[0] = c->ms_linearize; ms4[1] = c->ms_schur; ms4[2] = c->ms_solve; ms4[3] = c->ms_update; }
    if (iters) *iters = c->n_iters;
    if (trials) *trials = c->n_trials;
    return ORB_OK;
}

int lba_profile(lba_context* c, int enable) {
    if (!c) return ORB_EINVAL;
    c->profile = enable != 0;
    c->ms_linearize = c->ms_schur = c->ms_solve = c->ms_update = 0;
    c->n_iters = c->n_trials = 0;
    return ORB_OK;
}

void lba_pose_from_Tcw(const float Tcw[16], double q[4], double t[3]) {
    // Converter::toSE3Quat (R/src/Converter.cpp:47-57): float Mat -> Matrix3d -> SE3Quat
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)Tcw[i * 4 + j];
    hd_quat_from_matrix(R, q);
    for (int i = 0; i < 3; i++) t[i] = (double)Tcw[i * 4 + 3];
}

void lba_pose_to_Tcw(const double q[4], const double t[3], float Tcw[16]) {
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
}

int lba_solve(lba_context* c, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop, lba_result* r) {
    if (!c || !p || !o || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0) return ORB_EINVAL;
    ORB_HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int NP = p->n_poses, NM = p->n_points, NE = p->n_edges;
    r->iterations[0] = r->iterations[1] = 0;
    r->trials = 0;
    r->n_trace = 0;
    r->aborted = 0;
    if (stop && *stop) {      // R/src/Optimizer.cpp:784-786: return before optimizing, no write-back
        r->aborted = 1;
        return ORB_OK;
    }
    lba_free_all(c);
    LbaDev d;
    std::memset(&d, 0, sizeof(d));
    double *q, *t, *X, *obs, *info, *cam;
    uint8_t *fixed, *est, *robust;
    int32_t *ept, *eps;
    TRY(dalloc(c, &q, 4 * (size_t)NP)); TRY(dalloc(c, &t, 3 * (size_t)NP)); TRY(dalloc(c, &X, 3 * (size_t)NM));
    TRY(dalloc(c, &d.bq, 4 * (size_t)NP)); TRY(dalloc(c, &d.bt, 3 * (size_t)NP)); TRY(dalloc(c, &d.bX, 3 * (size_t)NM));
    TRY(dalloc(c, &fixed, NP)); TRY(dalloc(c, &ept, NE)); TRY(dalloc(c, &eps, NE)); TRY(dalloc(c, &est, NE));
    TRY(dalloc(c, &obs, 3 * (size_t)NE)); TRY(dalloc(c, &info, NE)); TRY(dalloc(c, &cam, 5 * (size_t)NE));
    TRY(dalloc(c, &robust, NE)); TRY(dalloc(c, &d.err, 3 * (size_t)NE));
    ORB_HIP_TRY(hipMemcpyAsync(q, p->pose_q, 32 * (size_t)NP, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(t, p->pose_t, 24 * (size_t)NP, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(X, p->point_xyz, 24 * (size_t)NM, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(fixed, p->pose_fixed, NP, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(ept, p->edge_point, 4 * (size_t)NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(eps, p->edge_pose, 4 * (size_t)NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(est, p->edge_stereo, NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(obs, p->edge_obs, 24 * (size_t)NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(info, p->edge_info, 8 * (size_t)NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemcpyAsync(cam, p->edge_cam, 40 * (size_t)NE, hipMemcpyHostToDevice, s));
    ORB_HIP_TRY(hipMemsetAsync(robust, 1, NE, s));
    ORB_HIP_TRY(hipMemsetAsync(d.err, 0, 24 * (size_t)NE, s));
    d.q = q; d.t = t; d.X = X; d.fixed = fixed; d.ept = ept; d.eps = eps; d.est = est; d.obs = obs; d.info = info;
    d.cam = cam; d.robust = robust;
    // per-edge / per-vertex scratch sized for the full problem
    TRY(dalloc(c, &d.Hll_e, 6 * (size_t)NE)); TRY(dalloc(c, &d.Hpp_e, 21 * (size_t)NE));
    TRY(dalloc(c, &d.Hpl_e, 18 * (size_t)NE)); TRY(dalloc(c, &d.bl_e, 3 * (size_t)NE));
    TRY(dalloc(c, &d.bp_e, 6 * (size_t)NE)); TRY(dalloc(c, &d.BD, 18 * (size_t)NE));
    TRY(dalloc(c, &d.coef, 6 * (size_t)NE)); TRY(dalloc(c, &d.echi, (size_t)NE + 6 * (size_t)NP + 3 * (size_t)NM));
    TRY(dalloc(c, &d.Hll, 9 * (size_t)NM)); TRY(dalloc(c, &d.bl, 3 * (size_t)NM)); TRY(dalloc(c, &d.Dinv, 9 * (size_t)NM));
    TRY(dalloc(c, &d.db, 3 * (size_t)NM));
    TRY(dalloc(c, &d.Hpp, 36 * (size_t)NP)); TRY(dalloc(c, &d.bp, 6 * (size_t)NP));
    const size_t nS = (size_t)6 * NP;
    TRY(dalloc(c, &d.S, nS * nS + nS));   // S followed by b_s (contiguous for one all-reduce)
    d.bs = d.S + nS * nS;
    TRY(dalloc(c, &d.x, 6 * (size_t)NP + 3 * (size_t)NM));
    TRY(dalloc(c, &d.red, 16));
    TRY(dalloc(c, &d.flags, 4));
    TRY(dalloc(c, &d.lm, 1));
    double* d_trace = nullptr;
    TRY(dalloc(c, &d_trace, 4 * 64));
    double* d_chi2 = nullptr;
    uint8_t* d_depth = nullptr;
    TRY(dalloc(c, &d_chi2, NE));
    TRY(dalloc(c, &d_depth, NE));

    std::vector<uint8_t> level(NE, 0), robustH(NE, 1);
    const double hm = o->huber_mono, hsv = o->huber_stereo;
    const int maxTrials = o->max_trials > 0 ? o->max_trials : 10;
    auto stopped = [&]() { return stop && *stop; };

    auto elapsed = [&](hipEvent_t a, hipEvent_t b) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        return (double)ms;
    };

    HostStructure hs;
    int32_t* d_freePoses = nullptr;
    int32_t *d_pairI = nullptr, *d_pairJ = nullptr;
    const bool root = c->rank == 0;

    // global sum of the owned-point partials (and replicated pose part) of a scalar vector

    auto init_opt = [&](int lvl) -> int {
        build_structure(p, level, lvl, c->rank, c->world, hs);
        int32_t *act, *poseIdx, *ptLocal, *ptGlob, *actPos, *ptStart, *ptEdges, *poStart, *poEdges, *prStart, *prE1, *prE2;
        int32_t *actPt, *actPi;
        TRY(upload(c, &actPt, hs.actPt)); TRY(upload(c, &actPi, hs.actPi));
        TRY(upload(c, &act, hs.act)); TRY(upload(c, &poseIdx, hs.poseIdx)); TRY(upload(c, &ptLocal, hs.ptLocal));
        TRY(upload(c, &ptGlob, hs.ptGlob)); TRY(upload(c, &actPos, hs.actPos)); TRY(upload(c, &ptStart, hs.ptStart));
        TRY(upload(c, &ptEdges, hs.ptEdges)); TRY(upload(c, &poStart, hs.poStart)); TRY(upload(c, &poEdges, hs.poEdges));
        TRY(upload(c, &prStart, hs.prStart)); TRY(upload(c, &prE1, hs.prE1)); TRY(upload(c, &prE2, hs.prE2));
        TRY(upload(c, &d_freePoses, hs.freePoses)); TRY(upload(c, &d_pairI, hs.pairI)); TRY(upload(c, &d_pairJ, hs.pairJ));
        ORB_HIP_TRY(hipMemcpyAsync(robust, robustH.data(), NE, hipMemcpyHostToDevice, s));
        d.act = act; d.nact = (int)hs.act.size(); d.poseIdx = poseIdx; d.ptLocal = ptLocal; d.ptGlob = ptGlob;
        d.actPos = actPos; d.P = hs.P; d.M = hs.M; d.ptStart = ptStart; d.ptEdges = ptEdges; d.poStart = poStart;
        d.poEdges = poEdges; d.prStart = prStart; d.prE1 = prE1; d.prE2 = prE2;
        d.actPt = actPt; d.actPi = actPi;
        d.bs = d.S + (size_t)36 * d.P * d.P;   // b_s right after the 6P x 6P matrix: one all-reduce
        return ORB_OK;
    };

    auto grid = [](int n) { return dim3((unsigned)std::max(1, (n + 255) / 256)); };

    // computeActiveErrors + activeRobustChi2 (global over ranks) -> red[0], in phase `want`
    auto errors_chi2 = [&](int want) -> int {
        if (d.nact > 0) hipLaunchKernelGGL(k_edge_errors, grid(d.nact), dim3(256), 0, s, d, hm, hsv, want);
        hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, d.echi, d.nact, d.red, d.lm, want);
        TRY(comm_allreduce_g(c, d.red, 1, 0, d.lm, want));
        return ORB_OK;
    };

    // One LM "slot": the linearisation of an iteration (runs only when the device state says a
    // new iteration starts) followed by one trial (runs only while the iteration's trial loop
    // is open) and its decision.  Slots are enqueued back to back without host round trips.
    auto enqueue_slot = [&](int iterations, hipEvent_t* ev) -> int {
        const bool prof = ev != nullptr;
        if (prof) (void)hipEventRecord(ev[0], s);
        // ---- linearisation (G/core/sparse_optimizer.cpp:384-394, block_solver.hpp:502-561)
        TRY(errors_chi2(0));
        if (d.nact > 0) hipLaunchKernelGGL(k_edge_linearize, grid(d.nact), dim3(256), 0, s, d, hm, hsv);
        if (d.M > 0) hipLaunchKernelGGL(k_point_reduce, grid(d.M), dim3(256), 0, s, d);
        if (d.P > 0) hipLaunchKernelGGL(k_pose_reduce, dim3(d.P), dim3(64), 0, s, d);
        if (d.P > 0) {
            TRY(comm_allreduce_g(c, d.Hpp, 36 * (size_t)d.P, 0, d.lm, 0));
            TRY(comm_allreduce_g(c, d.bp, 6 * (size_t)d.P, 0, d.lm, 0));
        }
        hipLaunchKernelGGL(k_maxdiag, dim3(1), dim3(1024), 0, s, d.Hpp, d.P, d.Hll, d.M, d.red + 1, d.lm);
        TRY(comm_allreduce_g(c, d.red + 1, 1, 1, d.lm, 3));
        hipLaunchKernelGGL(k_lm_begin, dim3(1), dim3(64), 0, s, d.lm, d.red);
        if (prof) (void)hipEventRecord(ev[1], s);
        // ---- trial: Schur complement, reduced solve, back-substitution, update, new chi2
        if (d.M > 0) hipLaunchKernelGGL(k_point_schur, grid(d.M), dim3(256), 0, s, d);
        if (d.nact > 0) hipLaunchKernelGGL(k_edge_schur, grid(d.nact), dim3(256), 0, s, d);
        const int npairs = d.P * (d.P + 1) / 2;
        if (npairs > 0) {
            hipLaunchKernelGGL(k_schur_pairs, dim3(npairs), dim3(256), 0, s, d, root ? 1 : 0, d_pairI, d_pairJ);
            hipLaunchKernelGGL(k_bschur, dim3(d.P), dim3(64), 0, s, d, root ? 1 : 0);
        }
        if (d.P > 0) TRY(comm_allreduce_g(c, d.S, (size_t)36 * d.P * d.P + 6 * (size_t)d.P, 0, d.lm, 1));
        if (prof) (void)hipEventRecord(ev[2], s);
        if (d.P > 0) {
            const int n = 6 * d.P;
            if ((size_t)n * (n | 1) * 8 + 3 * (size_t)n * 8 <= 160 * 1024)
                hipLaunchKernelGGL(k_ldlt_solve<true>, dim3(1), dim3(kLdltT), ((size_t)n * (n | 1) + 2 * (size_t)n) * 8, s,
                                   d.S, d.bs, n, d.x, d.flags, d.lm);
            else
                hipLaunchKernelGGL(k_ldlt_solve<false>, dim3(1), dim3(kLdltT), 2 * (size_t)n * 8, s, d.S, d.bs, n,
                                   d.x, d.flags, d.lm);
        } else {
            ORB_HIP_TRY(hipMemsetAsync(d.flags, 0, 4, s));
        }
        if (prof) (void)hipEventRecord(ev[3], s);
        if (d.M > 0) hipLaunchKernelGGL(k_backsub, grid(d.M), dim3(256), 0, s, d);
        hipLaunchKernelGGL(k_update, grid(std::max(d.M, d.P)), dim3(256), 0, s, d, d.P, d_freePoses, 1);
        TRY(errors_chi2(1));
        const int nx = 6 * d.P + 3 * d.M;
        hipLaunchKernelGGL(k_scale_terms, grid(nx), dim3(256), 0, s, d, root ? 1 : 0, d.echi);
        hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, d.echi, nx, d.red + 2, d.lm, 1);
        TRY(comm_allreduce_g(c, d.red + 2, 1, 0, d.lm, 1));
        hipLaunchKernelGGL(k_lm_decide, dim3(1), dim3(64), 0, s, d.lm, d.red, d.flags, maxTrials, iterations,
                           o->fixed_iterations ? 1 : 0, d_trace);
        hipLaunchKernelGGL(k_pop, grid(std::max(d.M, d.P)), dim3(256), 0, s, d, d.P, d_freePoses);
        if (prof) (void)hipEventRecord(ev[4], s);
        return ORB_OK;
    };

    // one optimize() call (G/core/sparse_optimizer.cpp:354-419).  The host enqueues as many
    // slots as iterations remain (one trial each), then reads the device state once: more
    // slots only when trials were rejected.  The stop flag is polled between those groups.
    auto optimize = [&](int iterations, int& itersDone) -> int {
        itersDone = 0;
        if (hs.P + hs.M == 0 && c->world == 1) return ORB_OK;
        if (iterations <= 0 || stopped()) return ORB_OK;
        if (6 * d.P > kLdltMaxN) return ORB_E2BIG;   // panel rows are held in registers
        LmState* hst = reinterpret_cast<LmState*>(reinterpret_cast<char*>(c->h_scal) + 512);
        std::memset(hst, 0, sizeof(LmState));
        hst->ni = 2;
        hst->traceBase = r->trace ? r->n_trace : 64;
        ORB_HIP_TRY(hipMemcpyAsync(d.lm, hst, sizeof(LmState), hipMemcpyHostToDevice, s));
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
            for (int g = 0; g < G; g++) TRY(enqueue_slot(iterations, c->profile ? &c->slotEv[5 * (size_t)g] : nullptr));
            ORB_HIP_TRY(hipMemcpyAsync(hst, d.lm, sizeof(LmState), hipMemcpyDeviceToHost, s));
            TRY(lba_wait(c));
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
            if (hst->phase == 2 || stopped()) break;
        }
        itersDone = hst->itersDone;
        r->trials += hst->trials;
        c->n_trials += hst->trials;
        c->n_iters += itersDone;
        if (r->trace && r->n_trace < 64) {
            const int rows = std::min(64 - r->n_trace, itersDone);
            if (rows > 0) {
                ORB_HIP_TRY(hipMemcpyAsync(r->trace + 4 * r->n_trace, d_trace + 4 * r->n_trace, 32 * (size_t)rows,
                                           hipMemcpyDeviceToHost, s));
                TRY(lba_wait(c));
                r->n_trace += rows;
            }
        }
        return ORB_OK;
    };

    // ---- R/src/Optimizer.cpp:789-841
    TRY(init_opt(0));
    TRY(optimize(o->iters1, r->iterations[0]));
    const bool bDoMore = !stopped();
    auto edge_check = [&](std::vector<double>& chi, std::vector<uint8_t>& dep) -> int {
        if (NE > 0) hipLaunchKernelGGL(k_edge_check, grid(NE), dim3(256), 0, s, d, NE, d_chi2, d_depth);
        chi.resize(NE);
        dep.resize(NE);
        if (NE > 0) {
            ORB_HIP_TRY(hipMemcpyAsync(chi.data(), d_chi2, 8 * (size_t)NE, hipMemcpyDeviceToHost, s));
            ORB_HIP_TRY(hipMemcpyAsync(dep.data(), d_depth, NE, hipMemcpyDeviceToHost, s));
        }
        TRY(lba_wait(c));
        return ORB_OK;
    };
    std::vector<double> chi;
    std::vector<uint8_t> dep;
    const int own0 = (int)((long long)NM * c->rank / c->world), own1 = (int)((long long)NM * (c->rank + 1) / c->world);
    if (bDoMore) {
        TRY(edge_check(chi, dep));
        for (int e = 0; e < NE; e++) {
            if (p->point_bad && p->point_bad[p->edge_point[e]]) continue;
            const double thr = p->edge_stereo[e] ? o->chi2_stereo : o->chi2_mono;
            if (chi[e] > thr || !dep[e]) level[e] = 1;
            robustH[e] = 0;
        }
        // every rank only knows the errors of its own edges: share the level decisions
        if (c->world > 1) {
            std::vector<double> lv(NE);
            for (int e = 0; e < NE; e++) {
                const int pt = p->edge_point[e];
                lv[e] = (pt >= own0 && pt < own1) ? (double)level[e] : 0.0;
            }
            if (NE > (int)c->wsDoubles) return ORB_EINVAL;
            ORB_HIP_TRY(hipMemcpyAsync(c->ws, lv.data(), 8 * (size_t)NE, hipMemcpyHostToDevice, s));
            TRY(lba_wait(c));
            if (c->allreduce(c->commUser, 0, NE, 0) != 0) return ORB_EGPU;
            ORB_HIP_TRY(hipMemcpyAsync(lv.data(), c->ws, 8 * (size_t)NE, hipMemcpyDeviceToHost, s));
            TRY(lba_wait(c));
            for (int e = 0; e < NE; e++) level[e] = lv[e] > 0.5 ? 1 : 0;
        }
        TRY(init_opt(0));
        TRY(optimize(o->iters2, r->iterations[1]));
    }
    // ---- final check (R/src/Optimizer.cpp:850-880) and write-back data
    TRY(edge_check(chi, dep));
    for (int e = 0; e < NE; e++) {
        const int pt = p->edge_point[e];
        const bool mine = pt >= own0 && pt < own1;
        if (r->edge_chi2) r->edge_chi2[e] = mine ? chi[e] : 0.0;
        uint8_t er = 0;
        if (mine && !(p->point_bad && p->point_bad[pt])) {
            const double thr = p->edge_stereo[e] ? o->chi2_stereo : o->chi2_mono;
            er = (chi[e] > thr || !dep[e]) ? 1 : 0;
        }
        if (r->edge_erase) r->edge_erase[e] = er;
    }
    if (r->pose_q) ORB_HIP_TRY(hipMemcpyAsync(r->pose_q, q, 32 * (size_t)NP, hipMemcpyDeviceToHost, s));
    if (r->pose_t) ORB_HIP_TRY(hipMemcpyAsync(r->pose_t, t, 24 * (size_t)NP, hipMemcpyDeviceToHost, s));
    if (r->point_xyz) ORB_HIP_TRY(hipMemcpyAsync(r->point_xyz, X, 24 * (size_t)NM, hipMemcpyDeviceToHost, s));
    TRY(lba_wait(c));
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

}  // extern "C"
