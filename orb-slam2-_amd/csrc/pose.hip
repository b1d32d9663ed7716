// MI355X-native Optimizer::PoseOptimization(Frame*) (R/src/Optimizer.cpp:306-535): motion-only
// bundle adjustment of a frame's pose against its matched map points — one VertexSE3Expmap,
// unary EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges
// (G/types/types_six_dof_expmap.h:210-320, .cpp:285-390) with Huber kernels, g2o's
// Levenberg-Marquardt (G/core/optimization_algorithm_levenberg.cpp:61-189) over BlockSolver_6_3
// + LinearSolverDense (G/solvers/linear_solver_dense.h), four optimize(10) rounds from the
// frame's initial pose with the chi2 inlier/outlier reclassification between rounds and the
// robust kernel dropped after round 2.
//
// One 256-thread workgroup per frame runs the whole thing: the edges are strided over the
// threads, each pass over them (errors + robust chi2, Jacobians + 6x6 normal equations) ends
// in a fixed-order workgroup reduction, and every thread then takes the same LM decision on
// the broadcast sums (the 6x6 LDL^T is solved redundantly per thread).  A batch of frames is
// one launch (frames of several cameras or sequences); nothing returns to the host between LM
// trials.  Per-edge state (inputs, last error, level, robust flag) stays in registers for frames of
// up to 1,024 edges (PoEdgesReg: the LM passes touch no memory) and in the caller-sized device
// arena beyond; either way the stale-error semantics of g2o's e->chi2() after a rejected trial
// carry over.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"
#include "lm_common.h"
#include "se3.h"

namespace orbamd {

constexpr int kPoT = 256;   // threads per frame

struct PoseDev {
    const double *q0, *t0, *cam;           // [B][4], [B][3], [B][5]
    const int32_t* start;                  // [B + 1]
    const double *obs, *xw, *info;         // [E][3], [E][3], [E]
    double *err;                           // [E][3] last computed error
    uint8_t *level, *robust;               // [E]
    double *qo, *to;                       // [B][4], [B][3]
    uint8_t* outlier;                      // [E]
    int32_t* ninl;                         // [B]
    int32_t* iters;                        // [B][5]: LM iterations per round, trials
};

struct FrameCam {
    double fx, fy, cx, cy, bf;
};

__device__ __forceinline__ void po_transform(const double q[4], const double t[3], const double* X, double Xc[3]) {
    double r[3];
    d_quat_rot(q, X, r);
    for (int i = 0; i < 3; i++) Xc[i] = r[i] + t[i];
}

// computeError (types_six_dof_expmap.h:223-227 / 282-286): obs - cam_project(T.map(Xw)); the
// stereo form takes float invz and the double member bf.
__device__ __forceinline__ void po_error(const PoseDev& d, const FrameCam& k, int e, const double q[4],
                                         const double t[3]) {
    double Xc[3];
    po_transform(q, t, d.xw + 3 * (size_t)e, Xc);
    const double* obs = d.obs + 3 * (size_t)e;
    double* er = d.err + 3 * (size_t)e;
    if (obs[2] < 0) {
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * k.fx + k.cx);
        er[1] = obs[1] - (v * k.fy + k.cy);
        er[2] = 0;
    } else {
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * k.fx + k.cx;
        const double r1 = Xc[1] * invz * k.fy + k.cy;
        const double r2 = r0 - k.bf * invz;
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
}

__device__ __forceinline__ double po_chi2(const PoseDev& d, int e) {
    const double* er = d.err + 3 * (size_t)e;
    const double w = d.info[e];
    double s = er[0] * (w * er[0]) + er[1] * (w * er[1]);
    if (d.obs[3 * (size_t)e + 2] >= 0) s += er[2] * (w * er[2]);
    return s;
}

__device__ __forceinline__ double po_delta(const PoseDev& d, int e) {
    // deltaStereo / deltaMono = (float)sqrt(7.815), (float)sqrt(5.991) (R/src/Optimizer.cpp:356-357)
    return d.obs[3 * (size_t)e + 2] >= 0 ? 2.7955322265625 : 2.4476518630981445;
}

// Fixed-order workgroup sum of one value per thread (wave xor butterfly, then the four waves
// in order); every thread gets the result.
__device__ __forceinline__ double po_block_sum(double v, double* sh) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    const int tid = threadIdx.x;
    __syncthreads();
    if ((tid & 63) == 0) sh[tid >> 6] = v;
    __syncthreads();
    return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// The 27 per-thread sums (21 upper H entries, 6 of b) reduced over the workgroup through LDS in a
// fixed order; every thread gets H (full) and b.
__device__ __forceinline__ void po_reduce27(const double acc[27], double (*part)[kPoT + 1], double* res, double H[36],
                                            double b[6]) {
    const int tid = threadIdx.x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 27; i++) part[i][tid] = acc[i];
    __syncthreads();
    const int v = tid >> 3, e8 = tid & 7;   // 27 values x 8 eighths of 32 partials
    double sum = 0.0;
    if (v < 27) {
#pragma unroll 8
        for (int i = 0; i < 32; i++) sum += part[v][32 * e8 + i];
    }
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    if (v < 27 && e8 == 0) res[v] = sum;
    __syncthreads();
    int o = 0;
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) {
            H[i * 6 + j] = res[o];
            H[j * 6 + i] = res[o];
            o++;
        }
    for (int i = 0; i < 6; i++) b[i] = res[21 + i];
}

// One active edge's linearizeOplus + constructQuadraticForm added to acc (Xc = the point in the
// camera, er = its last computed error).
__device__ __forceinline__ void po_accum_edge(const FrameCam& k, const double Xc[3], bool st, double w, bool robust,
                                              double chi2, double delta, const double er[3], double acc[27]) {
    const double x = Xc[0], y = Xc[1], invz = 1.0 / Xc[2], invz_2 = invz * invz;
    double J[18];
    J[0] = x * y * invz_2 * k.fx;       J[1] = -(1 + (x * x * invz_2)) * k.fx; J[2] = y * invz * k.fx;
    J[3] = -invz * k.fx;                J[4] = 0;                              J[5] = x * invz_2 * k.fx;
    J[6] = (1 + y * y * invz_2) * k.fy; J[7] = -x * y * invz_2 * k.fy;         J[8] = -x * invz * k.fy;
    J[9] = 0;                           J[10] = -invz * k.fy;                  J[11] = y * invz_2 * k.fy;
    if (st) {
        J[12] = J[0] - k.bf * y * invz_2; J[13] = J[1] + k.bf * x * invz_2; J[14] = J[2];
        J[15] = J[3];                     J[16] = 0;                        J[17] = J[5] - k.bf * invz_2;
    } else {
#pragma unroll
        for (int i = 12; i < 18; i++) J[i] = 0.0;
    }
    double rho1 = 1.0;
    if (robust && chi2 > delta * delta) rho1 = delta / sqrt(chi2);
    const double W = rho1 * w;
    double om[3];
#pragma unroll
    for (int r = 0; r < 3; r++) om[r] = (r < 2 || st) ? -(w * er[r]) * rho1 : 0.0;
    // all 3 rows: a monocular edge's third row and om[2] are zero (exact zeros added)
    int o = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < 3; r++) s += J[r * 6 + i] * om[r];
        acc[21 + i] += s;
#pragma unroll
        for (int j = i; j < 6; j++) {
            double h = 0;
#pragma unroll
            for (int r = 0; r < 3; r++) h += J[r * 6 + i] * W * J[r * 6 + j];
            acc[o++] += h;
        }
    }
}

// (H + lambda I) x = b by LDL^T without pivoting (the oracle's recurrence); false when a pivot
// is not positive (Eigen::LDLT::isPositive in LinearSolverDense::solve)
__device__ bool po_solve(const double H[36], const double b[6], double lambda, double x[6]) {
    double A[36], dd[6], y[6];
    for (int i = 0; i < 36; i++) A[i] = H[i];
    for (int i = 0; i < 6; i++) A[i * 7] += lambda;
    for (int j = 0; j < 6; j++) {
        double dj = A[j * 6 + j];
        for (int k = 0; k < j; k++) dj -= A[j * 6 + k] * A[j * 6 + k] * dd[k];
        if (!(dj > 0.0) || !isfinite(dj)) return false;
        dd[j] = dj;
        for (int i = j + 1; i < 6; i++) {
            double v = A[i * 6 + j];
            for (int k = 0; k < j; k++) v -= A[i * 6 + k] * A[j * 6 + k] * dd[k];
            A[i * 6 + j] = v / dj;
        }
    }
    for (int i = 0; i < 6; i++) {
        double v = b[i];
        for (int k = 0; k < i; k++) v -= A[i * 6 + k] * y[k];
        y[i] = v;
    }
    for (int i = 5; i >= 0; i--) {
        double v = y[i] / dd[i];
        for (int k = i + 1; k < 6; k++) v -= A[k * 6 + i] * x[k];
        x[i] = v;
    }
    return true;
}

// Per-edge state in the device arena (any edge count): the frame's edges strided over the threads.
struct PoEdgesGlobal {
    const PoseDev& d;
    FrameCam k;
    int e0, e1;
    __device__ void init() {
        for (int e = e0 + (int)threadIdx.x; e < e1; e += kPoT) {
            d.level[e] = 0;
            d.robust[e] = 1;
            d.outlier[e] = 0;
        }
    }
    __device__ double active_count() const {
        double cnt = 0.0;
        for (int e = e0 + (int)threadIdx.x; e < e1; e += kPoT) cnt += d.level[e] ? 0.0 : 1.0;
        return cnt;
    }
    __device__ double chi2(const double q[4], const double t[3]) const {
        double s = 0.0;
        for (int e = e0 + (int)threadIdx.x; e < e1; e += kPoT) {
            if (d.level[e]) continue;
            po_error(d, k, e, q, t);
            double chi = po_chi2(d, e);
            if (d.robust[e]) {
                const double delta = po_delta(d, e), dsqr = delta * delta;
                if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
            }
            s += chi;
        }
        return s;
    }
    __device__ void accum(const double q[4], const double t[3], double acc[27]) const {
        for (int e = e0 + (int)threadIdx.x; e < e1; e += kPoT) {
            if (d.level[e]) continue;
            double Xc[3];
            po_transform(q, t, d.xw + 3 * (size_t)e, Xc);
            const bool st = d.obs[3 * (size_t)e + 2] >= 0;
            const double* er = d.err + 3 * (size_t)e;
            const double ev[3] = {er[0], er[1], er[2]};
            po_accum_edge(k, Xc, st, d.info[e], d.robust[e] != 0, d.robust[e] ? po_chi2(d, e) : 0.0, po_delta(d, e), ev,
                          acc);
        }
    }
    // classification (R/src/Optimizer.cpp:461-520): inactive edges get their error at the final
    // estimate, active ones keep the last computed one (e->chi2())
    __device__ double classify(int it, const double q[4], const double t[3]) {
        double bad = 0.0;
        for (int e = e0 + (int)threadIdx.x; e < e1; e += kPoT) {
            if (d.level[e]) po_error(d, k, e, q, t);
            const float chi2 = (float)po_chi2(d, e);
            const float thr = d.obs[3 * (size_t)e + 2] >= 0 ? 7.815f : 5.991f;
            const uint8_t o = chi2 > thr ? 1 : 0;
            d.outlier[e] = o;
            d.level[e] = o;
            bad += o;
            if (it == 2) d.robust[e] = 0;
        }
        return bad;
    }
};

// The same state in registers for frames of at most kPoT * EPT edges: edge tid + kPoT s in slot s
// (the strided order above), loaded once; the LM passes touch no memory but the reductions' LDS.
// Arithmetic and summation order are PoEdgesGlobal's, so results are bit-identical.
template <int EPT>
struct PoEdgesReg {
    FrameCam k;
    double obs[EPT][3], xw[EPT][3], info[EPT], er[EPT][3];
    bool valid[EPT], st[EPT], level[EPT], robust[EPT];
    uint8_t* outlier;
    int e0;
    __device__ void load(const PoseDev& d, int e0_, int e1) {
        e0 = e0_;
        outlier = d.outlier;
        if (e1 <= e0) {   // a frame without edges touches no memory (e0 may be one past the arrays)
#pragma unroll
            for (int s = 0; s < EPT; s++) {
                valid[s] = st[s] = false;
                info[s] = 0.0;
#pragma unroll
                for (int c = 0; c < 3; c++) obs[s][c] = xw[s][c] = er[s][c] = 0.0;
            }
            return;
        }
#pragma unroll
        for (int s = 0; s < EPT; s++) {
            const int e = e0 + (int)threadIdx.x + kPoT * s;
            valid[s] = e < e1;
            const int ec = valid[s] ? e : e1 - 1;   // clamped to the frame's last edge
#pragma unroll
            for (int c = 0; c < 3; c++) {
                obs[s][c] = d.obs[3 * (size_t)ec + c];
                xw[s][c] = d.xw[3 * (size_t)ec + c];
                er[s][c] = 0.0;
            }
            info[s] = d.info[ec];
            st[s] = obs[s][2] >= 0;
        }
    }
    __device__ void init() {
#pragma unroll
        for (int s = 0; s < EPT; s++) {
            level[s] = false;
            robust[s] = true;
            if (valid[s]) outlier[e0 + (int)threadIdx.x + kPoT * s] = 0;
        }
    }
    __device__ double active_count() const {
        double cnt = 0.0;
#pragma unroll
        for (int s = 0; s < EPT; s++)
            if (valid[s]) cnt += level[s] ? 0.0 : 1.0;
        return cnt;
    }
    __device__ void error(int s, const double q[4], const double t[3]) {   // po_error in registers
        double Xc[3];
        po_transform(q, t, xw[s], Xc);
        if (!st[s]) {
            const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
            er[s][0] = obs[s][0] - (u * k.fx + k.cx);
            er[s][1] = obs[s][1] - (v * k.fy + k.cy);
            er[s][2] = 0;
        } else {
            const float invz = (float)(1.0f / Xc[2]);
            const double r0 = Xc[0] * invz * k.fx + k.cx;
            const double r1 = Xc[1] * invz * k.fy + k.cy;
            const double r2 = r0 - k.bf * invz;
            er[s][0] = obs[s][0] - r0;
            er[s][1] = obs[s][1] - r1;
            er[s][2] = obs[s][2] - r2;
        }
    }
    __device__ double chi2_of(int s) const {   // po_chi2
        const double w = info[s];
        double c = er[s][0] * (w * er[s][0]) + er[s][1] * (w * er[s][1]);
        if (st[s]) c += er[s][2] * (w * er[s][2]);
        return c;
    }
    __device__ double delta_of(int s) const { return st[s] ? 2.7955322265625 : 2.4476518630981445; }
    __device__ double chi2(const double q[4], const double t[3]) {
        double sum = 0.0;
#pragma unroll
        for (int s = 0; s < EPT; s++) {
            if (!valid[s] || level[s]) continue;
            error(s, q, t);
            double chi = chi2_of(s);
            if (robust[s]) {
                const double delta = delta_of(s), dsqr = delta * delta;
                if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
            }
            sum += chi;
        }
        return sum;
    }
    __device__ void accum(const double q[4], const double t[3], double acc[27]) const {
#pragma unroll
        for (int s = 0; s < EPT; s++) {
            if (!valid[s] || level[s]) continue;
            double Xc[3];
            po_transform(q, t, xw[s], Xc);
            po_accum_edge(k, Xc, st[s], info[s], robust[s], robust[s] ? chi2_of(s) : 0.0, delta_of(s), er[s], acc);
        }
    }
    __device__ double classify(int it, const double q[4], const double t[3]) {
        double bad = 0.0;
#pragma unroll
        for (int s = 0; s < EPT; s++) {
            if (!valid[s]) continue;
            if (level[s]) error(s, q, t);
            const float chi2 = (float)chi2_of(s);
            const float thr = st[s] ? 7.815f : 5.991f;
            const bool o = chi2 > thr;
            outlier[e0 + (int)threadIdx.x + kPoT * s] = o ? 1 : 0;
            level[s] = o;
            bad += o ? 1.0 : 0.0;
            if (it == 2) robust[s] = false;
        }
        return bad;
    }
};

// The four optimize(10) rounds over one frame's edges (any edge store above).
template <class ES>
__device__ void pose_rounds(ES& es, const PoseDev& d, const FrameCam& k, int f, int n, double (*part)[kPoT + 1],
                            double* res, double* sh) {
    const int tid = threadIdx.x;
    double q0[4], t0[3];
    for (int i = 0; i < 4; i++) q0[i] = d.q0[4 * f + i];
    for (int i = 0; i < 3; i++) t0[i] = d.t0[3 * f + i];
    es.init();
    int its[4] = {0, 0, 0, 0}, trials = 0;
    double q[4], t[3];
    for (int i = 0; i < 4; i++) q[i] = q0[i];
    for (int i = 0; i < 3; i++) t[i] = t0[i];
    int nBad = 0;
#ifdef ORB_TIMING
    long long tChi = 0, tBuild = 0, tSolve = 0, tClass = 0, tK0 = clock64(), tc;
#define PO_T0() tc = clock64()
#define PO_T(acc) acc += clock64() - tc
#else
#define PO_T0()
#define PO_T(acc)
#endif
    if (n >= 3) {   // nInitialCorrespondences < 3: return 0, pose untouched
        __syncthreads();
        for (int it = 0; it < 4; it++) {
            for (int i = 0; i < 4; i++) q[i] = q0[i];   // vSE3->setEstimate(toSE3Quat(pFrame->mTcw))
            for (int i = 0; i < 3; i++) t[i] = t0[i];
            const int nact = (int)po_block_sum(es.active_count(), sh);
            if (nact > 0) {
                double lambda = 0.0, ni = 2.0;
                int nBadLM = 0;
                for (int iter = 0; iter < 10; iter++) {
                    PO_T0();
                    double currentChi = po_block_sum(es.chi2(q, t), sh);   // computeActiveErrors + activeRobustChi2
                    PO_T(tChi);
                    const double iniChi = currentChi;
                    double H[36], b[6];
                    PO_T0();
                    {
                        double acc[27];
#pragma unroll
                        for (int i = 0; i < 27; i++) acc[i] = 0.0;
                        es.accum(q, t, acc);
                        po_reduce27(acc, part, res, H, b);
                    }
                    PO_T(tBuild);
                    if (iter == 0) {
                        double m = 0;
                        for (int j = 0; j < 6; j++) m = fmax(fabs(H[j * 7]), m);
                        lambda = 1e-5 * m;
                        ni = 2;
                        nBadLM = 0;
                    }
                    double rho = 0.0;
                    int qmax = 0;
                    do {
                        double bq[4], bt[3], x[6] = {0, 0, 0, 0, 0, 0};
                        for (int i = 0; i < 4; i++) bq[i] = q[i];
                        for (int i = 0; i < 3; i++) bt[i] = t[i];
                        const double lam = lambda;
                        PO_T0();
                        const bool ok2 = po_solve(H, b, lam, x);
                        if (!ok2)
                            for (int i = 0; i < 6; i++) x[i] = 0.0;
                        d_se3_exp_left(x, q, t);
                        PO_T(tSolve);
                        PO_T0();
                        double tempChi = po_block_sum(es.chi2(q, t), sh);
                        PO_T(tChi);
                        if (!ok2) tempChi = DBL_MAX;
                        rho = currentChi - tempChi;
                        double scale = 0.0;
                        for (int j = 0; j < 6; j++) scale += x[j] * (lam * x[j] + b[j]);
                        scale += 1e-3;
                        rho /= scale;
                        if (rho > 0 && isfinite(tempChi)) {
                            double alpha = 1. - cube_rn(2 * rho - 1);
                            alpha = fmin(alpha, 2. / 3.);
                            lambda *= fmax(1. / 3., alpha);
                            ni = 2;
                            currentChi = tempChi;
                        } else {
                            lambda *= ni;
                            ni *= 2;
                            for (int i = 0; i < 4; i++) q[i] = bq[i];
                            for (int i = 0; i < 3; i++) t[i] = bt[i];
                        }
                        qmax++;
                        trials++;
                    } while (rho < 0 && qmax < 10);
                    its[it]++;
                    if (qmax == 10 || rho == 0) break;
                    if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                    else nBadLM = 0;
                    if (nBadLM >= 3) break;
                }
            }
            PO_T0();
            nBad = (int)po_block_sum(es.classify(it, q, t), sh);
            PO_T(tClass);
            if (n < 10) break;   // optimizer.edges().size(): every edge of the graph
        }
    }
#ifdef ORB_TIMING
    if (tid == 0 && f == 0)
        printf("pose_opt f0 n %d: total %lld cycles | chi2 passes %lld build %lld solve+exp %lld classify %lld | trials %d iters %d %d %d %d\n",
               n, clock64() - tK0, tChi, tBuild, tSolve, tClass, trials, its[0], its[1], its[2], its[3]);
#endif
#undef PO_T0
#undef PO_T
    if (tid == 0) {
        for (int i = 0; i < 4; i++) d.qo[4 * f + i] = q[i];
        for (int i = 0; i < 3; i++) d.to[3 * f + i] = t[i];
        d.ninl[f] = n >= 3 ? n - nBad : 0;
        if (d.iters) {
            for (int i = 0; i < 4; i++) d.iters[5 * f + i] = its[i];
            d.iters[5 * f + 4] = trials;
        }
    }
}

constexpr int kPoEPT = 4;   // frames of up to 1024 edges keep their edges in registers

__global__ __launch_bounds__(kPoT) void k_pose_opt(PoseDev d) {
    __shared__ double part[27][kPoT + 1];
    __shared__ double res[32];
    __shared__ double sh[8];
    const int f = blockIdx.x;
    const int e0 = d.start[f], e1 = d.start[f + 1], n = e1 - e0;
    const FrameCam k{d.cam[5 * f], d.cam[5 * f + 1], d.cam[5 * f + 2], d.cam[5 * f + 3], d.cam[5 * f + 4]};
    if (n <= kPoT * kPoEPT) {
        PoEdgesReg<kPoEPT> es;
        es.k = k;
        es.load(d, e0, e1);
        pose_rounds(es, d, k, f, n, part, res, sh);
    } else {
        PoEdgesGlobal es{d, k, e0, e1};
        pose_rounds(es, d, k, f, n, part, res, sh);
    }
}

}  // namespace orbamd

using namespace orbamd;

extern "C" {

int pose_optimize_batch_device(const pose_batch* p, const pose_batch_result* r, double* d_work, uint8_t* d_flags,
                               int32_t* d_iters, void* stream) try {
    if (!p || !r || p->n_frames < 0 || !d_work || !d_flags) return ORB_EINVAL;
    if (p->n_frames == 0) return ORB_OK;
    PoseDev d;
    d.q0 = p->pose_q; d.t0 = p->pose_t; d.cam = p->cam; d.start = p->edge_start;
    d.obs = p->edge_obs; d.xw = p->edge_xw; d.info = p->edge_info;
    d.err = d_work;
    d.level = d_flags;
    d.robust = d_flags + p->n_edges;
    d.qo = r->pose_q; d.to = r->pose_t; d.outlier = r->outlier; d.ninl = r->n_inliers; d.iters = d_iters;
    hipLaunchKernelGGL(k_pose_opt, dim3(p->n_frames), dim3(kPoT), 0, (hipStream_t)stream, d);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

int pose_optimize_batch(int device, const pose_batch* p, pose_batch_result* r, int32_t* iters) try {
    if (!p || !r || p->n_frames < 0 || p->n_edges < 0) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    ORB_HIP_TRY(hipSetDevice(device));
    const int B = p->n_frames, E = p->n_edges;
    if (B == 0) return ORB_OK;
    for (int b = 0; b < B; b++)
        if (p->edge_start[b + 1] < p->edge_start[b]) return ORB_EINVAL;
    if (p->edge_start[0] != 0 || p->edge_start[B] != E) return ORB_EINVAL;
    // one device block: inputs, outputs and per-edge working state
    const size_t szIn = (size_t)B * (4 + 3 + 5) * 8 + (size_t)(B + 1) * 4 + (size_t)E * 7 * 8;
    const size_t szOut = (size_t)B * 7 * 8 + (size_t)B * 4 + (size_t)B * 5 * 4 + (size_t)E;
    const size_t szWork = (size_t)E * 3 * 8 + 2 * (size_t)E;
    HostScratch* hsc = nullptr;
    if (int e_ = host_scratch(device, szIn + szOut + szWork + 16 * 256, &hsc)) return e_;
    hipStream_t s = hsc->stream;
    Staging sg(hsc);   // one H2D of the batch, one D2H of the results
    pose_batch dp = *p;
    dp.pose_q = (const double*)sg.in(p->pose_q, (size_t)B * 32);
    dp.pose_t = (const double*)sg.in(p->pose_t, (size_t)B * 24);
    dp.cam = (const double*)sg.in(p->cam, (size_t)B * 40);
    dp.edge_start = (const int32_t*)sg.in(p->edge_start, (size_t)(B + 1) * 4);
    dp.edge_obs = (const double*)sg.in(p->edge_obs, (size_t)E * 24);
    dp.edge_xw = (const double*)sg.in(p->edge_xw, (size_t)E * 24);
    dp.edge_info = (const double*)sg.in(p->edge_info, (size_t)E * 8);
    if (int e_ = sg.upload_pull(s)) return e_;
    double* dWork = (double*)sg.out((size_t)E * 24 + 8);
    uint8_t* dFlags = (uint8_t*)sg.out(2 * (size_t)E + 2);
    pose_batch_result dr;
    dr.pose_q = (double*)sg.out((size_t)B * 32);
    dr.pose_t = (double*)sg.out((size_t)B * 24);
    dr.n_inliers = (int32_t*)sg.out((size_t)B * 4);
    dr.outlier = (uint8_t*)sg.out((size_t)E + 1);
    int32_t* dIters = (int32_t*)sg.out((size_t)B * 20);
    int rc = pose_optimize_batch_device(&dp, &dr, dWork, dFlags, dIters, s);
    if (rc == ORB_OK) {
        rc = sg.download(s, dr.pose_q);
        if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_EGPU;
        if (rc == ORB_OK) {
            std::memcpy(r->pose_q, sg.host(dr.pose_q), (size_t)B * 32);
            std::memcpy(r->pose_t, sg.host(dr.pose_t), (size_t)B * 24);
            std::memcpy(r->n_inliers, sg.host(dr.n_inliers), (size_t)B * 4);
            if (E) std::memcpy(r->outlier, sg.host(dr.outlier), (size_t)E);
            if (iters) std::memcpy(iters, sg.host(dIters), (size_t)B * 20);
        }
    }
    return rc;
} ORB_ABI_CATCH

}  // extern "C"
