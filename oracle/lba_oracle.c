/*
 * ORACLE / TEST INFRASTRUCTURE ONLY — restatement of the reference's local bundle
 * adjustment (see lba_oracle.h for anchors and parity status).
 */
#include "lba_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ SE3Quat (G/types/se3quat.h) */

static void quat_to_R(const double q[4], double R[9])
{   /* Eigen QuaternionBase::toRotationMatrix */
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

static void cross3(const double a[3], const double b[3], double o[3])
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

static void quat_rot(const double q[4], const double v[3], double o[3])
{   /* Eigen _transformVector: uv = 2 q.vec x v; v + w uv + q.vec x uv */
    double uv[3], c[3];
    cross3(q, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    cross3(q, uv, c);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q[3] * uv[i] + c[i];
}

static void quat_mul(const double a[4], const double b[4], double o[4])
{
    double r[4];
    r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    memcpy(o, r, sizeof(r));
}

static void normalize_rotation(double q[4])
{   /* SE3Quat::normalizeRotation */
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

void oracle_quat_from_matrix(const double m[9], double q[4])
{   /* Eigen quaternionbase_assign_impl<Matrix3>, then normalizeRotation */
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        double s = sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (m[7] - m[5]) * s;
        q[1] = (m[2] - m[6]) * s;
        q[2] = (m[3] - m[1]) * s;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 3 + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(m[i * 3 + i] - m[j * 3 + j] - m[k * 3 + k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
        q[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
        q[k] = (m[k * 3 + i] + m[i * 3 + k]) * s;
    }
    normalize_rotation(q);
}

static void mat3_mul(const double A[9], const double B[9], double C[9])
{
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

void oracle_se3_exp_left(const double upd[6], const double q[4], const double t[3], double qo[4], double to[3])
{   /* SE3Quat::exp(update) * T  (VertexSE3Expmap::oplusImpl) */
    const double* w = upd;
    const double* u = upd + 3;
    const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double O2[9], R[9], V[9];
    mat3_mul(O, O, O2);
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        memcpy(V, R, sizeof(R));
    } else {
        const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        const double c = (theta - sin(theta)) / pow(theta, 3);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    double qe[4], te[3];
    oracle_quat_from_matrix(R, qe);
    for (int i = 0; i < 3; i++) te[i] = V[i * 3] * u[0] + V[i * 3 + 1] * u[1] + V[i * 3 + 2] * u[2];
    double rt[3];
    quat_rot(qe, t, rt);
    for (int i = 0; i < 3; i++) to[i] = te[i] + rt[i];
    quat_mul(qe, q, qo);
    normalize_rotation(qo);
}

/* ------------------------------------------------------------ edges */

typedef struct {
    const lba_problem_t* p;
    const lba_options_t* o;
    double *pq, *pt, *X;            /* current estimates */
    double *bq, *bt, *bX;           /* push() backup */
    double* err;                    /* [n_edges][3] last computed error (stale after pop, like g2o) */
    uint8_t *level, *robust;
    /* active structure */
    int* act_edges; int n_act;
    int* pose_idx; int P;           /* pose -> hessian index or -1 */
    int* point_idx; int M;
    /* system */
    double* Hpp;    /* [P][6][6] diagonal blocks + dense S assembly */
    double* S;      /* [6P][6P] */
    double* bp;     /* [6P] */
    double* Hll;    /* [M][9] */
    double* bl;     /* [M][3] */
    double* Hpl;    /* [n_edges][18] (6x3 per active edge with a free pose) */
    double* x;      /* [6P + 3M] */
    double* Dinv;   /* [M][9] */
    int* pt_edge_start; int* pt_edges;   /* active edges grouped by point index (ascending pose index) */
    double lambda, ni;
    int nBad;
    /* landmark sharding (oracle_lba_solve_dist): this rank owns points [own0, own1) */
    int rank, world, own0, own1;
    oracle_allreduce_fn ar;
    void* ar_user;
    int stop_after;   /* terminate() once this many trials ran (-1: off) */
    /* OpenMP variant (oracle_lba_solve_omp): threads > 1 parallelises the loops g2o's
     * G2O_OPENMP build parallelises (G/core/sparse_optimizer.cpp:70-71 computeActiveErrors,
     * G/core/block_solver.hpp:528 buildSystem's edge loop, :379-380 the Schur landmark loop) plus
     * the landmark back-substitution and point updates.  Unlike g2o (vertex locks: arrival-order sums) every sum keeps the
     * serial order, so the variant is bitwise identical to the single-thread oracle. */
    int threads;
    double* eprod;    /* [n_edges][54] per-edge pose terms of the parallel buildSystem */
    double* BD;       /* [n_edges][18] Hpl_e Dinv of the parallel Schur */
    double* dbl;      /* [M][3] Dinv b_l of the parallel Schur */
    int *pose_a_start, *pose_a;   /* per free pose index: its pt_edges positions, landmark-ascending */
    int *pt_k_start, *pt_k;       /* per point index / free pose index: its act positions k, ascending */
    int *po_k_start, *po_k;       /* (the parallel merge of buildSystem keeps the serial edge order) */
} lba_ctx;

#define OMP_IF(c) if ((c)->threads > 1) num_threads((c)->threads)

static void allreduce(lba_ctx* c, double* v, int n, int op)
{
    if (c->world > 1 && n > 0) c->ar(c->ar_user, v, n, op);
}

static void transform(const lba_ctx* c, int pose, int pt, double Xc[3])
{
    double r[3];
    quat_rot(c->pq + 4 * pose, c->X + 3 * pt, r);
    for (int i = 0; i < 3; i++) Xc[i] = r[i] + c->pt[3 * pose + i];
}

static void compute_error(lba_ctx* c, int e)
{
    const lba_problem_t* p = c->p;
    double Xc[3];
    transform(c, p->edge_pose[e], p->edge_point[e], Xc);
    const double* cam = p->edge_cam + 5 * e;
    const double* obs = p->edge_obs + 3 * e;
    double* er = c->err + 3 * e;
    if (!p->edge_stereo[e]) {
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * cam[0] + cam[2]);
        er[1] = obs[1] - (v * cam[1] + cam[3]);
        er[2] = 0;
    } else {   /* EdgeStereoSE3ProjectXYZ::cam_project: float invz, float bf */
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * cam[0] + cam[2];
        const double r1 = Xc[1] * invz * cam[1] + cam[3];
        const float bff = (float)cam[4];
        const double r2 = r0 - (double)(bff * invz);
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
}

static double edge_chi2(const lba_ctx* c, int e)
{
    const double* er = c->err + 3 * e;
    const double w = c->p->edge_info[e];
    double s = er[0] * (w * er[0]) + er[1] * (w * er[1]);
    if (c->p->edge_stereo[e]) s += er[2] * (w * er[2]);
    return s;
}

static double huber_delta(const lba_ctx* c, int e)
{
    return c->p->edge_stereo[e] ? c->o->huber_stereo : c->o->huber_mono;
}

static double robust_chi2(const lba_ctx* c, int e)
{
    const double chi = edge_chi2(c, e);
    if (!c->robust[e]) return chi;
    const double d = huber_delta(c, e), dsqr = d * d;
    if (chi <= dsqr) return chi;
    return 2 * sqrt(chi) * d - dsqr;
}

static int depth_positive(const lba_ctx* c, int e)
{
    double Xc[3];
    transform(c, c->p->edge_pose[e], c->p->edge_point[e], Xc);
    return Xc[2] > 0.0;
}

/* Jacobians (G/types/types_six_dof_expmap.cpp:112-245): A = d e / d X (rows x 3), B = d e / d xi (rows x 6) */
static int linearize(const lba_ctx* c, int e, double A[9], double B[18])
{
    const lba_problem_t* p = c->p;
    const int pose = p->edge_pose[e];
    double R[9], Xc[3];
    quat_to_R(c->pq + 4 * pose, R);
    transform(c, pose, p->edge_point[e], Xc);
    const double x = Xc[0], y = Xc[1], z = Xc[2], z_2 = z * z;
    const double* cam = p->edge_cam + 5 * e;
    const double fx = cam[0], fy = cam[1], bf = cam[4];
    if (!p->edge_stereo[e]) {
        const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
        for (int r = 0; r < 2; r++)
            for (int k = 0; k < 3; k++)
                A[r * 3 + k] = -1. / z * (tmp[r * 3] * R[k] + tmp[r * 3 + 1] * R[3 + k] + tmp[r * 3 + 2] * R[6 + k]);
    } else {
        for (int k = 0; k < 3; k++) {
            A[0 * 3 + k] = -fx * R[0 * 3 + k] / z + fx * x * R[2 * 3 + k] / z_2;
            A[1 * 3 + k] = -fy * R[1 * 3 + k] / z + fy * y * R[2 * 3 + k] / z_2;
            A[2 * 3 + k] = A[0 * 3 + k] - bf * R[2 * 3 + k] / z_2;
        }
    }
    B[0] = x * y / z_2 * fx;      B[1] = -(1 + (x * x / z_2)) * fx; B[2] = y / z * fx;
    B[3] = -1. / z * fx;          B[4] = 0;                         B[5] = x / z_2 * fx;
    B[6] = (1 + y * y / z_2) * fy; B[7] = -x * y / z_2 * fy;        B[8] = -x / z * fy;
    B[9] = 0;                     B[10] = -1. / z * fy;             B[11] = y / z_2 * fy;
    if (p->edge_stereo[e]) {
        B[12] = B[0] - bf * y / z_2; B[13] = B[1] + bf * x / z_2; B[14] = B[2];
        B[15] = B[3];                B[16] = 0;                   B[17] = B[5] - bf / z_2;
        return 3;
    }
    return 2;
}

/* ------------------------------------------------------------ structure (initializeOptimization) */

static int cmp_i64_idx_base;
static const int64_t* g_ids;
static int cmp_by_id(const void* a, const void* b)
{
    const int64_t x = g_ids[*(const int*)a], y = g_ids[*(const int*)b];
    return x < y ? -1 : (x > y ? 1 : 0);
}

static void init_optimization(lba_ctx* c, int level)
{
    const lba_problem_t* p = c->p;
    c->n_act = 0;
    uint8_t* pose_act = (uint8_t*)calloc(p->n_poses + 1, 1);
    uint8_t* pt_act = (uint8_t*)calloc(p->n_points + 1, 1);
    for (int e = 0; e < p->n_edges; e++) {
        if (c->level[e] != level) continue;
        /* allVerticesFixed() is false: points are never fixed */
        pose_act[p->edge_pose[e]] = 1;         /* pose mapping is global across ranks */
        const int pt = p->edge_point[e];
        if (pt < c->own0 || pt >= c->own1) continue;
        c->act_edges[c->n_act++] = e;
        pt_act[pt] = 1;
    }
    /* index mapping: free active poses by id, then active points by id (G/core/sparse_optimizer.cpp:166-190) */
    int* order = (int*)malloc(sizeof(int) * (p->n_poses + p->n_points + 1));
    int n = 0;
    for (int i = 0; i < p->n_poses; i++) if (pose_act[i] && !p->pose_fixed[i]) order[n++] = i;
    g_ids = p->pose_id;
    qsort(order, n, sizeof(int), cmp_by_id);
    for (int i = 0; i < p->n_poses; i++) c->pose_idx[i] = -1;
    for (int k = 0; k < n; k++) c->pose_idx[order[k]] = k;
    c->P = n;
    n = 0;
    for (int i = 0; i < p->n_points; i++) if (pt_act[i]) order[n++] = i;
    g_ids = p->point_id;
    qsort(order, n, sizeof(int), cmp_by_id);
    for (int i = 0; i < p->n_points; i++) c->point_idx[i] = -1;
    for (int k = 0; k < n; k++) c->point_idx[order[k]] = k;
    c->M = n;
    /* edges per point index, sorted by pose index */
    memset(c->pt_edge_start, 0, sizeof(int) * (c->M + 1));
    for (int k = 0; k < c->n_act; k++) c->pt_edge_start[c->point_idx[p->edge_point[c->act_edges[k]]] + 1]++;
    for (int i = 0; i < c->M; i++) c->pt_edge_start[i + 1] += c->pt_edge_start[i];
    int* fill = (int*)malloc(sizeof(int) * (c->M + c->P + 2));
    memcpy(fill, c->pt_edge_start, sizeof(int) * (c->M + 1));
    for (int k = 0; k < c->n_act; k++) {
        const int e = c->act_edges[k];
        c->pt_edges[fill[c->point_idx[p->edge_point[e]]]++] = e;
    }
    for (int m = 0; m < c->M; m++) {   /* insertion sort by pose hessian index (fixed poses last) */
        int* a = c->pt_edges + c->pt_edge_start[m];
        const int len = c->pt_edge_start[m + 1] - c->pt_edge_start[m];
        for (int i = 1; i < len; i++) {
            const int v = a[i];
            const int kv = c->pose_idx[p->edge_pose[v]] < 0 ? 1 << 30 : c->pose_idx[p->edge_pose[v]];
            int j = i - 1;
            while (j >= 0) {
                const int kj = c->pose_idx[p->edge_pose[a[j]]] < 0 ? 1 << 30 : c->pose_idx[p->edge_pose[a[j]]];
                if (kj <= kv) break;
                a[j + 1] = a[j];
                j--;
            }
            a[j + 1] = v;
        }
    }
    if (c->threads > 1) {   /* per pose row: its edge positions in landmark order (parallel Schur) */
        memset(c->pose_a_start, 0, sizeof(int) * (c->P + 1));
        for (int a = 0; a < c->n_act; a++) {
            const int i1 = c->pose_idx[p->edge_pose[c->pt_edges[a]]];
            if (i1 >= 0) c->pose_a_start[i1 + 1]++;
        }
        for (int i = 0; i < c->P; i++) c->pose_a_start[i + 1] += c->pose_a_start[i];
        memcpy(fill, c->pose_a_start, sizeof(int) * (c->P + 1));
        for (int a = 0; a < c->n_act; a++) {
            const int i1 = c->pose_idx[p->edge_pose[c->pt_edges[a]]];
            if (i1 >= 0) c->pose_a[fill[i1]++] = a;
        }
    }
    if (c->threads > 1) {   /* per point / per free pose: act positions in ascending order */
        memset(c->pt_k_start, 0, sizeof(int) * (c->M + 1));
        memset(c->po_k_start, 0, sizeof(int) * (c->P + 1));
        for (int k = 0; k < c->n_act; k++) {
            const int e = c->act_edges[k];
            c->pt_k_start[c->point_idx[p->edge_point[e]] + 1]++;
            const int pi = c->pose_idx[p->edge_pose[e]];
            if (pi >= 0) c->po_k_start[pi + 1]++;
        }
        for (int i = 0; i < c->M; i++) c->pt_k_start[i + 1] += c->pt_k_start[i];
        for (int i = 0; i < c->P; i++) c->po_k_start[i + 1] += c->po_k_start[i];
        int* f2 = (int*)malloc(sizeof(int) * (c->M + c->P + 2));
        memcpy(f2, c->pt_k_start, sizeof(int) * (c->M + 1));
        memcpy(f2 + c->M + 1, c->po_k_start, sizeof(int) * (c->P + 1));
        for (int k = 0; k < c->n_act; k++) {
            const int e = c->act_edges[k];
            c->pt_k[f2[c->point_idx[p->edge_point[e]]]++] = k;
            const int pi = c->pose_idx[p->edge_pose[e]];
            if (pi >= 0) c->po_k[f2[c->M + 1 + pi]++] = k;
        }
        free(f2);
    }
    free(fill);
    free(order);
    free(pose_act);
    free(pt_act);
}

/* ------------------------------------------------------------ buildSystem */

#ifdef LBA_ORACLE_TIMING
#include <time.h>
static double g_tp[8];
static double now_s(void) { struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec + 1e-9 * ts.tv_nsec; }
#define TP(i, stmt) do { const double t0_ = now_s(); stmt; g_tp[i] += now_s() - t0_; } while (0)
void oracle_lba_phase_times(double* out)   /* errors, chi2, build, push, schur_solve, update (s); resets */
{
    for (int i = 0; i < 8; i++) { out[i] = g_tp[i]; g_tp[i] = 0; }
}
#else
#define TP(i, stmt) stmt
#endif
/* OpenMP buildSystem (G/core/block_solver.hpp:528), bitwise the serial loop: every accumulator
 * receives the serial loop's additions in the serial (act) order.
 *  A. in parallel over landmarks: each landmark's edges in act order are linearised, the landmark
 *     blocks Hll / b_l accumulated in place, Hpl written per edge, and the edge's pose terms
 *     (Hpp_e 36 | b_p,e 6 per residual row) stored per act edge;
 *  B. in parallel over (pose, row of the 6x6 block): the pose's edges in act order add their
 *     stored terms — 6 P work items, so a window with fewer poses than threads still spreads. */
static void build_system_omp(lba_ctx* c)
{
    const lba_problem_t* p = c->p;
#ifdef LBA_ORACLE_TIMING
    const double tA = now_s();
#endif
#pragma omp parallel for schedule(dynamic, 16) OMP_IF(c)
    for (int li = 0; li < c->M; li++) {
        double hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};   /* stored once, below */
        for (int a = c->pt_k_start[li]; a < c->pt_k_start[li + 1]; a++) {
            const int k = c->pt_k[a];
            const int e = c->act_edges[k];
            double A[9], B[18];
            const int D = linearize(c, e, A, B);
            const double w = p->edge_info[e];
            const double* er = c->err + 3 * e;
            double rho1 = 1.0;
            if (c->robust[e]) {
                const double chi = edge_chi2(c, e), d = huber_delta(c, e);
                if (chi > d * d) rho1 = d / sqrt(chi);
            }
            const double W = rho1 * w;
            double om_r[3] = {0, 0, 0};
            for (int r = 0; r < D; r++) om_r[r] = -(w * er[r]) * rho1;
            for (int i = 0; i < 3; i++) {
                for (int r = 0; r < D; r++) bl[i] += A[r * 3 + i] * om_r[r];
                for (int j = 0; j < 3; j++) {
                    double s = 0;
                    for (int r = 0; r < D; r++) s += A[r * 3 + i] * W * A[r * 3 + j];
                    hl[i * 3 + j] += s;
                }
            }
            if (c->pose_idx[p->edge_pose[e]] >= 0) {
                double* hpl = c->Hpl + 18 * e;
                double* t = c->eprod + 54 * (size_t)k;   /* per block row i: hp 6 | bp terms 3 */
                for (int i = 0; i < 6; i++) {
                    for (int r = 0; r < 3; r++) t[9 * i + 6 + r] = r < D ? B[r * 6 + i] * om_r[r] : 0.0;
                    for (int j = 0; j < 6; j++) {
                        double s = 0;
                        for (int r = 0; r < D; r++) s += B[r * 6 + i] * W * B[r * 6 + j];
                        t[9 * i + j] = s;
                    }
                    for (int j = 0; j < 3; j++) {
                        double s = 0;
                        for (int r = 0; r < D; r++) s += B[r * 6 + i] * W * A[r * 3 + j];
                        hpl[i * 3 + j] = s;
                    }
                }
            }
        }
        memcpy(c->Hll + 9 * li, hl, sizeof(hl));
        memcpy(c->bl + 3 * li, bl, sizeof(bl));
    }
#ifdef LBA_ORACLE_TIMING
    const double tB = now_s();
    g_tp[6] += tB - tA;
#endif
#pragma omp parallel for schedule(dynamic, 1) OMP_IF(c)
    for (int item = 0; item < 6 * c->P; item++) {
        const int pi = item / 6, i = item % 6;
        /* local accumulators (neighbouring items' rows share cache lines), stored once */
        double hp[6] = {0, 0, 0, 0, 0, 0}, bp = 0.0;
        for (int a = c->po_k_start[pi]; a < c->po_k_start[pi + 1]; a++) {
            const int k = c->po_k[a];
            const int D = p->edge_stereo[c->act_edges[k]] ? 3 : 2;
            const double* t = c->eprod + 54 * (size_t)k + 9 * i;
            for (int r = 0; r < D; r++) bp += t[6 + r];
            for (int j = 0; j < 6; j++) hp[j] += t[j];
        }
        for (int j = 0; j < 6; j++) c->Hpp[36 * pi + 6 * i + j] = hp[j];
        c->bp[6 * pi + i] = bp;
    }
}

static void build_system(lba_ctx* c)
{
    const lba_problem_t* p = c->p;
    const int np = 6 * c->P;
    memset(c->Hpp, 0, sizeof(double) * 36 * c->P);
    memset(c->bp, 0, sizeof(double) * np);
    memset(c->Hll, 0, sizeof(double) * 9 * c->M);
    memset(c->bl, 0, sizeof(double) * 3 * c->M);
    memset(c->S, 0, sizeof(double) * np * np);     /* off-diagonal pose blocks stay zero in Hpp */
    if (c->threads > 1) {
        build_system_omp(c);
        return;
    }
    for (int k = 0; k < c->n_act; k++) {
        const int e = c->act_edges[k];
        double A[9], B[18];
        const int D = linearize(c, e, A, B);
        const double w = p->edge_info[e];
        const double* er = c->err + 3 * e;
        double rho1 = 1.0;
        if (c->robust[e]) {
            const double chi = edge_chi2(c, e), d = huber_delta(c, e);
            if (chi > d * d) rho1 = d / sqrt(chi);
        }
        const double W = rho1 * w;          /* weightedOmega = rho' * Omega (diagonal) */
        double om_r[3];
        for (int r = 0; r < D; r++) om_r[r] = -(w * er[r]) * rho1;
        const int li = c->point_idx[p->edge_point[e]];
        const int pi = c->pose_idx[p->edge_pose[e]];
        double* hl = c->Hll + 9 * li;
        double* bl = c->bl + 3 * li;
        for (int i = 0; i < 3; i++) {
            for (int r = 0; r < D; r++) bl[i] += A[r * 3 + i] * om_r[r];
            for (int j = 0; j < 3; j++) {
                double s = 0;
                for (int r = 0; r < D; r++) s += A[r * 3 + i] * W * A[r * 3 + j];
                hl[i * 3 + j] += s;
            }
        }
        if (pi >= 0) {
            double* hp = c->Hpp + 36 * pi;
            double* bp = c->bp + 6 * pi;
            double* hpl = c->Hpl + 18 * e;
            for (int i = 0; i < 6; i++) {
                for (int r = 0; r < D; r++) bp[i] += B[r * 6 + i] * om_r[r];
                for (int j = 0; j < 6; j++) {
                    double s = 0;
                    for (int r = 0; r < D; r++) s += B[r * 6 + i] * W * B[r * 6 + j];
                    hp[i * 6 + j] += s;
                }
                for (int j = 0; j < 3; j++) {
                    double s = 0;
                    for (int r = 0; r < D; r++) s += B[r * 6 + i] * W * A[r * 3 + j];
                    hpl[i * 3 + j] = s;
                }
            }
        }
    }
}

static void share_pose_system(lba_ctx* c)
{
    allreduce(c, c->Hpp, 36 * c->P, 0);
    allreduce(c, c->bp, 6 * c->P, 0);
}

static double lambda_init(lba_ctx* c)
{
    double m = 0.;
    for (int i = 0; i < c->P; i++)
        for (int j = 0; j < 6; j++) m = fmax(fabs(c->Hpp[36 * i + j * 7]), m);
    for (int i = 0; i < c->M; i++)
        for (int j = 0; j < 3; j++) m = fmax(fabs(c->Hll[9 * i + j * 4]), m);
    allreduce(c, &m, 1, 1);
    return 1e-5 * m;
}

static void inv3(const double m[9], double o[9])
{   /* Eigen compute_inverse_size3_helper */
    double c[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            c[i * 3 + j] = m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
        }
    const double det = c[0] * m[0] + c[3] * m[3] + c[6] * m[6];
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) o[j * 3 + i] = c[i * 3 + j] * invdet;
}

/* BlockSolver::solve with lambda on the diagonal; returns 0 if the LDL^T fails */
static int schur_solve(lba_ctx* c, double lambda)
{
    const lba_problem_t* p = c->p;
    const int np = 6 * c->P;
    double* S = c->S;
    memset(S, 0, sizeof(double) * np * np);
    const int root = c->rank == 0;
    for (int i = 0; i < c->P && root; i++)
        for (int r = 0; r < 6; r++)
            for (int q = 0; q < 6; q++) S[(6 * i + r) * np + 6 * i + q] = c->Hpp[36 * i + r * 6 + q] + (r == q ? lambda : 0.);
    double* coef = (double*)calloc(np + 1, sizeof(double));
    if (c->threads > 1) {
        /* Dinv and Dinv b_l per landmark in parallel (G/core/block_solver.hpp:379-380), then the
         * S blocks and coef by pose row i1 in parallel: each row walks the landmarks in ascending
         * order, so every block receives its products in the serial loop's order. */
#pragma omp parallel for schedule(static) OMP_IF(c)
        for (int l = 0; l < c->M; l++) {
            double D[9];
            memcpy(D, c->Hll + 9 * l, sizeof(D));
            D[0] += lambda; D[4] += lambda; D[8] += lambda;
            double* Di = c->Dinv + 9 * l;
            inv3(D, Di);
            const double* b = c->bl + 3 * l;
            for (int i = 0; i < 3; i++) c->dbl[3 * l + i] = Di[i * 3] * b[0] + Di[i * 3 + 1] * b[1] + Di[i * 3 + 2] * b[2];
            for (int a = c->pt_edge_start[l]; a < c->pt_edge_start[l + 1]; a++) {   /* Hpl_e Dinv, once per edge */
                const int e = c->pt_edges[a];
                if (c->pose_idx[p->edge_pose[e]] < 0) continue;
                const double* Bi = c->Hpl + 18 * e;
                double* BD = c->BD + 18 * (size_t)e;
                for (int r = 0; r < 6; r++)
                    for (int q = 0; q < 3; q++)
                        BD[r * 3 + q] = Bi[r * 3] * Di[q] + Bi[r * 3 + 1] * Di[3 + q] + Bi[r * 3 + 2] * Di[6 + q];
            }
        }
        /* work items = pose row x a range of block columns (the row's landmarks are walked by
         * every item of the row, each forming the products of its own columns only), so a
         * window with fewer rows than threads still spreads; coef by the first item of a row */
        const int nq = c->P >= 4 * c->threads ? 1 : (4 * c->threads + c->P - 1) / (c->P > 0 ? c->P : 1);
#pragma omp parallel for schedule(dynamic, 1) OMP_IF(c)
        for (int item = 0; item < c->P * nq; item++) {
            const int row = item / nq, qc = item % nq;
            const int col0 = row + (int)((long long)(c->P - row) * qc / nq);
            const int col1 = row + (int)((long long)(c->P - row) * (qc + 1) / nq);
            if (col0 >= col1 && qc > 0) continue;
            /* the item's 6 x 6 (col1 - col0) blocks and the row's coef accumulate in locals (items
             * of neighbouring rows / column ranges share cache lines), from S's current values,
             * in the serial order; stored once */
            const int nc = 6 * (col1 - col0);
            double acc[6 * (nc > 0 ? nc : 1)];
            double cf[6] = {0, 0, 0, 0, 0, 0};
            for (int r = 0; r < 6; r++)
                for (int q = 0; q < nc; q++) acc[r * nc + q] = S[(6 * row + r) * np + 6 * col0 + q];
            if (qc == 0)
                for (int r = 0; r < 6; r++) cf[r] = coef[6 * row + r];
            for (int ka = c->pose_a_start[row]; ka < c->pose_a_start[row + 1]; ka++) {
                const int a = c->pose_a[ka];
                const int l = c->point_idx[p->edge_point[c->pt_edges[a]]];
                const double* db = c->dbl + 3 * l;
                const int s1 = c->pt_edge_start[l + 1];
                const int e1 = c->pt_edges[a];
                const double* Bi = c->Hpl + 18 * e1;
                const double* BD = c->BD + 18 * (size_t)e1;
                if (qc == 0)
                    for (int r = 0; r < 6; r++) cf[r] += Bi[r * 3] * db[0] + Bi[r * 3 + 1] * db[1] + Bi[r * 3 + 2] * db[2];
                for (int bb = a; bb < s1; bb++) {
                    const int e2 = c->pt_edges[bb];
                    const int i2 = c->pose_idx[p->edge_pose[e2]];
                    if (i2 < col0 || i2 >= col1) continue;   /* (fixed poses: -1) */
                    const double* Bj = c->Hpl + 18 * e2;
                    double* blk = acc + 6 * (i2 - col0);
                    for (int r = 0; r < 6; r++)
                        for (int q = 0; q < 6; q++) {
                            const double v = BD[r * 3] * Bj[q * 3] + BD[r * 3 + 1] * Bj[q * 3 + 1] + BD[r * 3 + 2] * Bj[q * 3 + 2];
                            blk[r * nc + q] -= v;
                        }
                }
            }
            for (int r = 0; r < 6; r++)
                for (int q = 0; q < nc; q++) S[(6 * row + r) * np + 6 * col0 + q] = acc[r * nc + q];
            if (qc == 0)
                for (int r = 0; r < 6; r++) coef[6 * row + r] = cf[r];
        }
    }
    for (int l = 0; l < c->M && c->threads <= 1; l++) {
        double D[9];
        memcpy(D, c->Hll + 9 * l, sizeof(D));
        D[0] += lambda; D[4] += lambda; D[8] += lambda;
        double* Di = c->Dinv + 9 * l;
        inv3(D, Di);
        const double* b = c->bl + 3 * l;
        double db[3];
        for (int i = 0; i < 3; i++) db[i] = Di[i * 3] * b[0] + Di[i * 3 + 1] * b[1] + Di[i * 3 + 2] * b[2];
        const int s0 = c->pt_edge_start[l], s1 = c->pt_edge_start[l + 1];
        for (int a = s0; a < s1; a++) {
            const int e1 = c->pt_edges[a];
            const int i1 = c->pose_idx[p->edge_pose[e1]];
            if (i1 < 0) continue;
            const double* Bi = c->Hpl + 18 * e1;
            double BD[18];
            for (int r = 0; r < 6; r++)
                for (int q = 0; q < 3; q++)
                    BD[r * 3 + q] = Bi[r * 3] * Di[q] + Bi[r * 3 + 1] * Di[3 + q] + Bi[r * 3 + 2] * Di[6 + q];
            for (int r = 0; r < 6; r++) coef[6 * i1 + r] += Bi[r * 3] * db[0] + Bi[r * 3 + 1] * db[1] + Bi[r * 3 + 2] * db[2];
            for (int bb = a; bb < s1; bb++) {
                const int e2 = c->pt_edges[bb];
                const int i2 = c->pose_idx[p->edge_pose[e2]];
                if (i2 < 0) continue;
                const double* Bj = c->Hpl + 18 * e2;
                for (int r = 0; r < 6; r++)
                    for (int q = 0; q < 6; q++) {
                        const double v = BD[r * 3] * Bj[q * 3] + BD[r * 3 + 1] * Bj[q * 3 + 1] + BD[r * 3 + 2] * Bj[q * 3 + 2];
                        S[(6 * i1 + r) * np + 6 * i2 + q] -= v;
                    }
            }
        }
    }
    /* symmetric fill of the lower triangle from the upper blocks */
    for (int r = 0; r < np; r++)
        for (int q = 0; q < r; q++) S[r * np + q] = S[q * np + r];
    double* bs = (double*)malloc(sizeof(double) * (np + 1));
    for (int i = 0; i < np; i++) bs[i] = (root ? c->bp[i] : 0.0) - coef[i];
    allreduce(c, S, np * np, 0);
    allreduce(c, bs, np, 0);
    /* dense LDL^T (no pivoting); fails only on an exactly zero pivot, like SimplicialLDLT.
     * Crout order, one fused multiply-add per update: with W(i,k) = A(i,k) before the
     * division by d_k (kept in the upper triangle at (k, i)) and L(i,k) = W(i,k) / d_k (lower),
     * A(i,j) = fma(-W(i,k), L(j,k), A(i,j)) for k = 0 .. j-1.  SimplicialLDLT's own order
     * (AMD-permuted, sparse) is not reproducible without Eigen; this recurrence is the one the
     * GPU factorisation (k_ldlt_solve) follows element for element. */
    int ok = 1;
#ifdef LBA_ORACLE_TIMING
    const double tL = now_s();
#endif
    double* d = (double*)malloc(sizeof(double) * (np + 1));
    /* (OpenMP variant, large systems: the rows i > j of column j in parallel — each element is
     * the same operation sequence, so the factor is bitwise the serial one) */
#pragma omp parallel if (c->threads > 1 && np >= 256) num_threads(c->threads > 1 ? c->threads : 1)
    for (int j = 0; j < np; j++) {
#pragma omp single
        {
            double dj = S[j * np + j];
            for (int k = 0; k < j; k++) dj = fma(-S[k * np + j], S[j * np + k], dj);
            if (ok && (dj == 0.0 || !isfinite(dj))) ok = 0;
            d[j] = dj;
        }
        if (!ok) continue;   /* (every thread reads ok after the single's barrier) */
        const double dj = d[j];
#pragma omp for schedule(static)
        for (int i = j + 1; i < np; i++) {
            double v = S[i * np + j];
            for (int k = 0; k < j; k++) v = fma(-S[k * np + i], S[j * np + k], v);
            S[j * np + i] = v;        /* W(i, j) */
            S[i * np + j] = v / dj;   /* L(i, j) */
        }
    }
#ifdef LBA_ORACLE_TIMING
    g_tp[7] += now_s() - tL;
#endif
    double* xp = c->x;
    if (ok) {
        for (int i = 0; i < np; i++) {
            double v = bs[i];
            for (int k = 0; k < i; k++) v = fma(-S[i * np + k], xp[k], v);
            xp[i] = v;
        }
        for (int i = 0; i < np; i++) xp[i] /= d[i];
        /* back substitution with L^T, column-oriented: x_k is final once every k' > k has
         * been applied, then x_i = fma(-L(k,i), x_k, x_i) for i < k (k descending per element) */
        for (int k = np - 1; k >= 0; k--)
            for (int i = 0; i < k; i++) xp[i] = fma(-S[k * np + i], xp[k], xp[i]);
        /* landmarks: x_l = Dinv (b_l - Hpl^T x_p) */
#pragma omp parallel for schedule(static) OMP_IF(c)
        for (int l = 0; l < c->M; l++) {
            double cl[3] = {c->bl[3 * l], c->bl[3 * l + 1], c->bl[3 * l + 2]};
            for (int a = c->pt_edge_start[l]; a < c->pt_edge_start[l + 1]; a++) {
                const int e = c->pt_edges[a];
                const int i1 = c->pose_idx[p->edge_pose[e]];
                if (i1 < 0) continue;
                const double* Bi = c->Hpl + 18 * e;
                for (int q = 0; q < 3; q++)
                    for (int r = 0; r < 6; r++) cl[q] += Bi[r * 3 + q] * (-xp[6 * i1 + r]);
            }
            const double* Di = c->Dinv + 9 * l;
            double* xl = c->x + np + 3 * l;
            for (int q = 0; q < 3; q++) xl[q] = Di[q * 3] * cl[0] + Di[q * 3 + 1] * cl[1] + Di[q * 3 + 2] * cl[2];
        }
    }
    free(d);
    free(bs);
    free(coef);
    return ok;
}

static void push_state(lba_ctx* c)
{
    memcpy(c->bq, c->pq, sizeof(double) * 4 * c->p->n_poses);
    memcpy(c->bt, c->pt, sizeof(double) * 3 * c->p->n_poses);
    memcpy(c->bX, c->X, sizeof(double) * 3 * c->p->n_points);
}
static void pop_state(lba_ctx* c)
{
    memcpy(c->pq, c->bq, sizeof(double) * 4 * c->p->n_poses);
    memcpy(c->pt, c->bt, sizeof(double) * 3 * c->p->n_poses);
    memcpy(c->X, c->bX, sizeof(double) * 3 * c->p->n_points);
}

static void update(lba_ctx* c)
{
    const lba_problem_t* p = c->p;
    for (int i = 0; i < p->n_poses; i++) {
        const int k = c->pose_idx[i];
        if (k < 0) continue;
        double q[4], t[3];
        oracle_se3_exp_left(c->x + 6 * k, c->pq + 4 * i, c->pt + 3 * i, q, t);
        memcpy(c->pq + 4 * i, q, sizeof(q));
        memcpy(c->pt + 3 * i, t, sizeof(t));
    }
#pragma omp parallel for schedule(static) OMP_IF(c)
    for (int i = 0; i < p->n_points; i++) {
        const int k = c->point_idx[i];
        if (k < 0) continue;
        for (int j = 0; j < 3; j++) c->X[3 * i + j] += c->x[6 * c->P + 3 * k + j];
    }
}

static double active_robust_chi2(lba_ctx* c)
{
    double s = 0;
    for (int k = 0; k < c->n_act; k++) s += robust_chi2(c, c->act_edges[k]);
    allreduce(c, &s, 1, 0);
    return s;
}
static void compute_active_errors(lba_ctx* c)
{
#pragma omp parallel for schedule(static) OMP_IF(c)
    for (int k = 0; k < c->n_act; k++) compute_error(c, c->act_edges[k]);
}

enum { LM_OK = 0, LM_TERMINATE = 1 };

/* OptimizationAlgorithmLevenberg::solve (G/core/optimization_algorithm_levenberg.cpp:61-164) */
/* SparseOptimizer::terminate(): the caller's flag, or the test hook's trial count */
static int terminated(const lba_ctx* c, const volatile uint8_t* stop, const lba_result_t* r)
{
    return (stop && *stop) || (c->stop_after >= 0 && r->trials >= c->stop_after);
}

static int lm_iteration(lba_ctx* c, int iteration, const volatile uint8_t* stop, lba_result_t* r)
{
    TP(0, compute_active_errors(c));
    double currentChi;
    TP(1, currentChi = active_robust_chi2(c));
    double tempChi = currentChi;
    const double iniChi = currentChi;
    TP(2, build_system(c));
    share_pose_system(c);
    if (iteration == 0) {
        c->lambda = lambda_init(c);
        c->ni = 2;
        c->nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    const int nx = 6 * c->P + 3 * c->M;
    do {
        TP(3, push_state(c));
        const double lam = c->lambda;
        int ok2;
        TP(4, ok2 = schur_solve(c, lam));
        if (!ok2) memset(c->x, 0, sizeof(double) * nx);   /* _x is left unchanged on failure; update is harmless */
        TP(5, update(c));
        TP(0, compute_active_errors(c));
        TP(1, tempChi = active_robust_chi2(c));
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = 0.;
        if (c->rank == 0)
            for (int j = 0; j < 6 * c->P; j++) scale += c->x[j] * (lam * c->x[j] + c->bp[j]);
        for (int j = 0; j < 3 * c->M; j++) scale += c->x[6 * c->P + j] * (lam * c->x[6 * c->P + j] + c->bl[j]);
        allreduce(c, &scale, 1, 0);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            const double sf = fmax(1. / 3., alpha);
            c->lambda *= sf;
            c->ni = 2;
            currentChi = tempChi;
        } else {
            c->lambda *= c->ni;
            c->ni *= 2;
            pop_state(c);
        }
        qmax++;
        r->trials++;
    } while (rho < 0 && qmax < c->o->max_trials && !terminated(c, stop, r));
    if (r->trace && r->n_trace < 64) {
        double* t = r->trace + 4 * r->n_trace++;
        t[0] = iniChi; t[1] = currentChi; t[2] = c->lambda; t[3] = qmax;
    }
    if (c->o->fixed_iterations) return LM_OK;
    if (qmax == c->o->max_trials || rho == 0) return LM_TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) c->nBad++;
    else c->nBad = 0;
    if (c->nBad >= 3) return LM_TERMINATE;
    return LM_OK;
}

static int optimize(lba_ctx* c, int iterations, const volatile uint8_t* stop, lba_result_t* r)
{
    if (c->P + c->M == 0 && c->world == 1) return 0;
    int it = 0, ok = 1;
    for (int i = 0; i < iterations && !terminated(c, stop, r) && ok; i++) {
        ok = lm_iteration(c, i, stop, r) == LM_OK;
        it++;
    }
    return it;
}

static int lba_run(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop, lba_result_t* r,
                   int rank, int world, oracle_allreduce_fn ar, void* user, int global, int robust, int stop_after,
                   int threads);

int oracle_lba_solve(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop, lba_result_t* r)
{
    return lba_run(p, o, stop, r, 0, 1, NULL, NULL, 0, 1, -1, 1);
}

/* The OpenMP CPU path of SURVEY 8d(b): the same solve with the g2o G2O_OPENMP loops run on
 * `threads` host threads; bitwise identical results to oracle_lba_solve. */
int oracle_lba_solve_omp(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop,
                         lba_result_t* r, int threads)
{
    return lba_run(p, o, stop, r, 0, 1, NULL, NULL, 0, 1, -1, threads < 1 ? 1 : threads);
}

int oracle_lba_solve_stop_after(const lba_problem_t* p, const lba_options_t* o, int stop_after_trials,
                                lba_result_t* r)
{
    return lba_run(p, o, NULL, r, 0, 1, NULL, NULL, 0, 1, stop_after_trials < 0 ? -1 : stop_after_trials, 1);
}

int oracle_lba_solve_dist(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop,
                          lba_result_t* r, int rank, int world, oracle_allreduce_fn ar, void* user)
{
    return lba_run(p, o, stop, r, rank, world, ar, user, 0, 1, -1, 1);
}

/* Optimizer::BundleAdjustment (R/src/Optimizer.cpp:78-277): one optimize(nIterations) = iters1
 * over every edge, Huber kernels (deltas (float)sqrt(5.99) / (float)sqrt(7.815)) only when
 * bRobust, no outlier pass; the force-stop flag only ends the iterations (no early return). */
int oracle_global_ba(const lba_problem_t* p, const lba_options_t* o, int robust, const volatile uint8_t* stop,
                     lba_result_t* r)
{
    return lba_run(p, o, stop, r, 0, 1, NULL, NULL, 1, robust, -1, 1);
}

static int lba_run(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop, lba_result_t* r,
                   int rank, int world, oracle_allreduce_fn ar, void* user, int global, int robust, int stop_after,
                   int threads)
{
    lba_ctx c;
    memset(&c, 0, sizeof(c));
    c.p = p;
    c.o = o;
    c.rank = rank;
    c.world = world;
    c.ar = ar;
    c.ar_user = user;
    c.stop_after = stop_after;
    c.threads = threads;
    c.own0 = (int)((long long)p->n_points * rank / world);
    c.own1 = (int)((long long)p->n_points * (rank + 1) / world);
    const int NP = p->n_poses, NM = p->n_points, NE = p->n_edges;
    c.pq = (double*)malloc(sizeof(double) * 4 * (NP + 1));
    c.pt = (double*)malloc(sizeof(double) * 3 * (NP + 1));
    c.X = (double*)malloc(sizeof(double) * 3 * (NM + 1));
    c.bq = (double*)malloc(sizeof(double) * 4 * (NP + 1));
    c.bt = (double*)malloc(sizeof(double) * 3 * (NP + 1));
    c.bX = (double*)malloc(sizeof(double) * 3 * (NM + 1));
    c.err = (double*)calloc(3 * (NE + 1), sizeof(double));
    c.level = (uint8_t*)calloc(NE + 1, 1);
    c.robust = (uint8_t*)malloc(NE + 1);
    memset(c.robust, robust ? 1 : 0, NE + 1);
    c.act_edges = (int*)malloc(sizeof(int) * (NE + 1));
    c.pose_idx = (int*)malloc(sizeof(int) * (NP + 1));
    c.point_idx = (int*)malloc(sizeof(int) * (NM + 1));
    c.Hpp = (double*)malloc(sizeof(double) * 36 * (NP + 1));
    c.S = (double*)malloc(sizeof(double) * 36 * (NP + 1) * (NP + 1));
    c.bp = (double*)malloc(sizeof(double) * 6 * (NP + 1));
    c.Hll = (double*)malloc(sizeof(double) * 9 * (NM + 1));
    c.bl = (double*)malloc(sizeof(double) * 3 * (NM + 1));
    c.Hpl = (double*)malloc(sizeof(double) * 18 * (NE + 1));
    c.x = (double*)malloc(sizeof(double) * (6 * NP + 3 * NM + 1));
    c.Dinv = (double*)malloc(sizeof(double) * 9 * (NM + 1));
    c.pt_edge_start = (int*)malloc(sizeof(int) * (NM + 2));
    c.pt_edges = (int*)malloc(sizeof(int) * (NE + 1));
    if (threads > 1) {
        c.eprod = (double*)malloc(sizeof(double) * 54 * (NE + 1));
        c.BD = (double*)malloc(sizeof(double) * 18 * (NE + 1));
        c.dbl = (double*)malloc(sizeof(double) * 3 * (NM + 1));
        c.pose_a_start = (int*)malloc(sizeof(int) * (NP + 2));
        c.pose_a = (int*)malloc(sizeof(int) * (NE + 1));
        c.pt_k_start = (int*)malloc(sizeof(int) * (NM + 2));
        c.pt_k = (int*)malloc(sizeof(int) * (NE + 1));
        c.po_k_start = (int*)malloc(sizeof(int) * (NP + 2));
        c.po_k = (int*)malloc(sizeof(int) * (NE + 1));
    }
    memcpy(c.pq, p->pose_q, sizeof(double) * 4 * NP);
    memcpy(c.pt, p->pose_t, sizeof(double) * 3 * NP);
    memcpy(c.X, p->point_xyz, sizeof(double) * 3 * NM);
    r->iterations[0] = r->iterations[1] = 0;
    r->trials = 0;
    r->n_trace = 0;
    int status = 0;
    if (!global && stop && *stop) {
        status = 1;
        goto done;
    }
    /* optimize(5) on every edge with Huber kernels (R/src/Optimizer.cpp:789-790); global BA:
     * optimize(nIterations), R/src/Optimizer.cpp:230-231 */
    init_optimization(&c, 0);
    r->iterations[0] = optimize(&c, o->iters1, stop, r);
    int bDoMore = !global && !terminated(&c, stop, r);
    if (bDoMore) {
        /* outlier pass (R/src/Optimizer.cpp:805-836) */
        for (int e = 0; e < NE; e++) {
            if (p->point_bad && p->point_bad[p->edge_point[e]]) continue;
            const double thr = p->edge_stereo[e] ? o->chi2_stereo : o->chi2_mono;
            if (edge_chi2(&c, e) > thr || !depth_positive(&c, e)) c.level[e] = 1;
            c.robust[e] = 0;
        }
        if (world > 1) {   /* each rank decided only its own edges: share the level vector */
            double* lv = (double*)calloc(NE + 1, sizeof(double));
            for (int e = 0; e < NE; e++) {
                const int pt = p->edge_point[e];
                lv[e] = (pt >= c.own0 && pt < c.own1) ? (double)c.level[e] : 0.0;
            }
            allreduce(&c, lv, NE, 0);
            for (int e = 0; e < NE; e++) c.level[e] = lv[e] > 0.5 ? 1 : 0;
            free(lv);
        }
        init_optimization(&c, 0);
        r->iterations[1] = optimize(&c, o->iters2, stop, r);
    }
    /* final check (R/src/Optimizer.cpp:850-880): e->chi2() uses each edge's last computed error */
    for (int e = 0; e < NE; e++) {
        const int mine = p->edge_point[e] >= c.own0 && p->edge_point[e] < c.own1;
        const double chi = mine ? edge_chi2(&c, e) : 0.0;
        if (r->edge_chi2) r->edge_chi2[e] = chi;
        uint8_t er = 0;
        if (!global && mine && !(p->point_bad && p->point_bad[p->edge_point[e]])) {
            const double thr = p->edge_stereo[e] ? o->chi2_stereo : o->chi2_mono;
            er = (chi > thr || !depth_positive(&c, e)) ? 1 : 0;
        }
        if (r->edge_erase) r->edge_erase[e] = er;
    }
    if (r->pose_q) memcpy(r->pose_q, c.pq, sizeof(double) * 4 * NP);
    if (r->pose_t) memcpy(r->pose_t, c.pt, sizeof(double) * 3 * NP);
    if (r->point_xyz) memcpy(r->point_xyz, c.X, sizeof(double) * 3 * NM);
done:
    free(c.pq); free(c.pt); free(c.X); free(c.bq); free(c.bt); free(c.bX); free(c.err);
    free(c.level); free(c.robust); free(c.act_edges); free(c.pose_idx); free(c.point_idx);
    free(c.Hpp); free(c.S); free(c.bp); free(c.Hll); free(c.bl); free(c.Hpl); free(c.x); free(c.Dinv);
    free(c.pt_edge_start); free(c.pt_edges); free(c.eprod); free(c.BD); free(c.dbl);
    free(c.pose_a_start); free(c.pose_a);
    free(c.pt_k_start); free(c.pt_k); free(c.po_k_start); free(c.po_k);
    (void)cmp_i64_idx_base;
    return status;
}

/* ======================================================================== PoseOptimization
 * Optimizer::PoseOptimization (R/src/Optimizer.cpp:306-535): one VertexSE3Expmap, unary
 * EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges
 * (G/types/types_six_dof_expmap.h:210-320, .cpp:285-390), Huber (float)sqrt(5.991) /
 * (float)sqrt(7.815), LM (optimization_algorithm_levenberg.cpp:61-189) with
 * BlockSolver_6_3 + LinearSolverDense (an LDL^T of the 6x6 H + lambda I; Eigen's pivoted LDLT is
 * restated without pivoting: same solution to rounding), four rounds of optimize(10) from the
 * frame's initial pose with the chi2 inlier/outlier reclassification between rounds and the
 * robust kernel dropped after round 2. */

typedef struct {
    const pose_problem_t* p;
    double q[4], t[3];     /* current estimate */
    double bq[4], bt[3];   /* push() */
    uint8_t* level;        /* 0 active, 1 outlier */
    uint8_t* robust;
    double* err;           /* [n][3] last computed error */
    double H[36], b[6], x[6];
    double lambda, ni;
    int nBad;
    int g2o_order;         /* 1: every sum in edge order, as g2o accumulates (no GPU reduction shape) */
} pose_ctx;

static void pose_compute_error(pose_ctx* c, int e)
{   /* computeError(): obs - cam_project(v1->estimate().map(Xw)) */
    const pose_problem_t* p = c->p;
    const double* X = p->xw + 3 * e;
    const double* obs = p->obs + 3 * e;
    double Xc[3];
    quat_rot(c->q, X, Xc);
    for (int i = 0; i < 3; i++) Xc[i] += c->t[i];
    double* er = c->err + 3 * e;
    if (obs[2] < 0) {   /* EdgeSE3ProjectXYZOnlyPose: project2d then *f + c (all double) */
        const double u = Xc[0] / Xc[2], v = Xc[1] / Xc[2];
        er[0] = obs[0] - (u * p->fx + p->cx);
        er[1] = obs[1] - (v * p->fy + p->cy);
        er[2] = 0;
    } else {            /* EdgeStereoSE3ProjectXYZOnlyPose: float invz, double member bf */
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * p->fx + p->cx;
        const double r1 = Xc[1] * invz * p->fy + p->cy;
        const double r2 = r0 - p->bf * invz;
        er[0] = obs[0] - r0;
        er[1] = obs[1] - r1;
        er[2] = obs[2] - r2;
    }
}

static double pose_chi2(const pose_ctx* c, int e)
{
    const double* er = c->err + 3 * e;
    const double w = c->p->info[e];
    double s = er[0] * (w * er[0]) + er[1] * (w * er[1]);
    if (c->p->obs[3 * e + 2] >= 0) s += er[2] * (w * er[2]);
    return s;
}

static double pose_robust_chi2(const pose_ctx* c, int e)
{
    double chi = pose_chi2(c, e);
    if (c->robust[e]) {
        const double delta = c->p->obs[3 * e + 2] >= 0 ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991);
        const double dsqr = delta * delta;
        if (chi > dsqr) chi = 2 * sqrt(chi) * delta - dsqr;
    }
    return chi;
}

/* The GPU kernel's fixed reduction order (csrc/pose.hip), restated so that the LM decisions
 * (rho signs near convergence) agree exactly: thread t of 256 adds the terms of edges t, t + 256,
 * ... in order; each wave of 64 combines its lanes by an xor butterfly (offsets 32 .. 1) and
 * keeps lane 0's value; the four waves add as (w0 + w1) + (w2 + w3).  g2o adds the edges in
 * order — the same sum to rounding. */
enum { POSE_T = 256 };

static double pose_wave_lane0(double* v)
{   /* xor butterfly over 64 lanes, lane 0's result */
    for (int o = 32; o >= 1; o >>= 1) {
        double nv[64];
        for (int i = 0; i < 64; i++) nv[i] = v[i] + v[i ^ o];
        memcpy(v, nv, sizeof(nv));
    }
    return v[0];
}

static double pose_block_sum(double* th /* [256] per-thread partials */)
{
    double w[4];
    for (int k = 0; k < 4; k++) w[k] = pose_wave_lane0(th + 64 * k);
    return (w[0] + w[1]) + (w[2] + w[3]);
}

static double pose_active_errors(pose_ctx* c)
{   /* computeActiveErrors + activeRobustChi2 */
    if (c->g2o_order) {   /* G/core/sparse_optimizer.cpp activeRobustChi2: edges in order */
        double s = 0;
        for (int e = 0; e < c->p->n; e++) {
            if (c->level[e]) continue;
            pose_compute_error(c, e);
            s += pose_robust_chi2(c, e);
        }
        return s;
    }
    double th[POSE_T] = {0};
    for (int e = 0; e < c->p->n; e++) {
        if (c->level[e]) continue;
        pose_compute_error(c, e);
        th[e % POSE_T] += pose_robust_chi2(c, e);
    }
    return pose_block_sum(th);
}

/* linearizeOplus (types_six_dof_expmap.cpp:285-308, 355-388) + BaseUnaryEdge::constructQuadraticForm;
 * per-thread partials of the 21 upper H entries and b (GPU order), then per value eight groups of
 * 32 consecutive threads added in order and combined by an xor butterfly (offsets 1, 2, 4). */
static void pose_build_system(pose_ctx* c)
{
    const pose_problem_t* p = c->p;
    double part[27][POSE_T];   /* 55 KB on the stack: the oracle runs one frame per thread in bench.py */
    memset(part, 0, sizeof(part));
    double seqsum[27] = {0};   /* g2o order: each edge's 6x6 / 6 terms added to the vertex in edge order */
    for (int e = 0; e < p->n; e++) {
        if (c->level[e]) continue;
        double* acc = NULL;
        const int th = e % POSE_T;
        double* col[27];
        for (int v = 0; v < 27; v++) col[v] = c->g2o_order ? &seqsum[v] : &part[v][th];
        const double* X = p->xw + 3 * e;
        double Xc[3];
        quat_rot(c->q, X, Xc);
        for (int i = 0; i < 3; i++) Xc[i] += c->t[i];
        const double x = Xc[0], y = Xc[1], invz = 1.0 / Xc[2], invz_2 = invz * invz;
        const int st = p->obs[3 * e + 2] >= 0;
        double J[18] = {0};
        J[0] = x * y * invz_2 * p->fx;       J[1] = -(1 + (x * x * invz_2)) * p->fx; J[2] = y * invz * p->fx;
        J[3] = -invz * p->fx;                J[4] = 0;                               J[5] = x * invz_2 * p->fx;
        J[6] = (1 + y * y * invz_2) * p->fy; J[7] = -x * y * invz_2 * p->fy;         J[8] = -x * invz * p->fy;
        J[9] = 0;                            J[10] = -invz * p->fy;                  J[11] = y * invz_2 * p->fy;
        if (st) {
            J[12] = J[0] - p->bf * y * invz_2; J[13] = J[1] + p->bf * x * invz_2; J[14] = J[2];
            J[15] = J[3];                      J[16] = 0;                         J[17] = J[5] - p->bf * invz_2;
        }
        const double w = p->info[e];
        const double* er = c->err + 3 * e;
        double rho1 = 1.0;
        if (c->robust[e]) {
            const double chi = pose_chi2(c, e);
            const double delta = st ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991);
            if (chi > delta * delta) rho1 = delta / sqrt(chi);
        }
        const double W = rho1 * w;
        double om[3];
        for (int r = 0; r < 3; r++) om[r] = (r < 2 || st) ? -(w * er[r]) * rho1 : 0.0;
        (void)acc;
        int o = 0;
        for (int i = 0; i < 6; i++) {   /* all three rows: a mono edge's third row adds exact zeros */
            double sb = 0;
            for (int r = 0; r < 3; r++) sb += J[r * 6 + i] * om[r];
            *col[21 + i] += sb;
            for (int j = i; j < 6; j++) {
                double h = 0;
                for (int r = 0; r < 3; r++) h += J[r * 6 + i] * W * J[r * 6 + j];
                *col[o++] += h;
            }
        }
    }
    double res[27];
    for (int v = 0; v < 27 && c->g2o_order; v++) res[v] = seqsum[v];
    for (int v = 0; v < 27 && !c->g2o_order; v++) {
        double g[8];
        for (int k = 0; k < 8; k++) {
            double sg = 0.0;
            for (int i = 0; i < 32; i++) sg += part[v][32 * k + i];
            g[k] = sg;
        }
        for (int o = 1; o <= 4; o <<= 1) {
            double ng[8];
            for (int k = 0; k < 8; k++) ng[k] = g[k] + g[k ^ o];
            memcpy(g, ng, sizeof(g));
        }
        res[v] = g[0];
    }
    int o = 0;
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) {
            c->H[i * 6 + j] = res[o];
            c->H[j * 6 + i] = res[o];
            o++;
        }
    for (int i = 0; i < 6; i++) c->b[i] = res[21 + i];
}

/* H + lambda I = L D L^T (no pivoting), x = (H + lambda I)^-1 b; 0 when a pivot is not positive
 * (Eigen::LDLT::isPositive) */
static int pose_solve(pose_ctx* c, double lambda)
{
    double A[36], d[6], y[6];
    memcpy(A, c->H, sizeof(A));
    for (int i = 0; i < 6; i++) A[i * 7] += lambda;
    for (int j = 0; j < 6; j++) {
        double dj = A[j * 6 + j];
        for (int k = 0; k < j; k++) dj -= A[j * 6 + k] * A[j * 6 + k] * d[k];
        if (!(dj > 0.0) || !isfinite(dj)) return 0;
        d[j] = dj;
        for (int i = j + 1; i < 6; i++) {
            double v = A[i * 6 + j];
            for (int k = 0; k < j; k++) v -= A[i * 6 + k] * A[j * 6 + k] * d[k];
            A[i * 6 + j] = v / dj;
        }
    }
    for (int i = 0; i < 6; i++) {
        double v = c->b[i];
        for (int k = 0; k < i; k++) v -= A[i * 6 + k] * y[k];
        y[i] = v;
    }
    for (int i = 5; i >= 0; i--) {
        double v = y[i] / d[i];
        for (int k = i + 1; k < 6; k++) v -= A[k * 6 + i] * c->x[k];
        c->x[i] = v;
    }
    return 1;
}

static int pose_lm_iteration(pose_ctx* c, int iteration, pose_result_t* r)
{
    double currentChi = pose_active_errors(c);
    double tempChi = currentChi;
    const double iniChi = currentChi;
    pose_build_system(c);
    if (iteration == 0) {
        double m = 0;
        for (int j = 0; j < 6; j++) m = fmax(fabs(c->H[j * 7]), m);
        c->lambda = 1e-5 * m;
        c->ni = 2;
        c->nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
        memcpy(c->bq, c->q, sizeof(c->q));
        memcpy(c->bt, c->t, sizeof(c->t));
        const double lam = c->lambda;
        const int ok2 = pose_solve(c, lam);
        if (!ok2) memset(c->x, 0, sizeof(c->x));
        double qn[4], tn[3];
        oracle_se3_exp_left(c->x, c->q, c->t, qn, tn);
        memcpy(c->q, qn, sizeof(qn));
        memcpy(c->t, tn, sizeof(tn));
        tempChi = pose_active_errors(c);
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = 0.;
        for (int j = 0; j < 6; j++) scale += c->x[j] * (lam * c->x[j] + c->b[j]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            c->lambda *= fmax(1. / 3., alpha);
            c->ni = 2;
            currentChi = tempChi;
        } else {
            c->lambda *= c->ni;
            c->ni *= 2;
            memcpy(c->q, c->bq, sizeof(c->q));
            memcpy(c->t, c->bt, sizeof(c->t));
        }
        qmax++;
        r->trials++;
    } while (rho < 0 && qmax < 10);
    if (qmax == 10 || rho == 0) return LM_TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) c->nBad++;
    else c->nBad = 0;
    if (c->nBad >= 3) return LM_TERMINATE;
    return LM_OK;
}

static int pose_optimization(const pose_problem_t* p, pose_result_t* r, int g2o_order);

int oracle_pose_optimization(const pose_problem_t* p, pose_result_t* r) { return pose_optimization(p, r, 0); }

/* The same with g2o's summation order (edges accumulated in order, G/core/sparse_optimizer.cpp
 * activeRobustChi2 and BlockSolver::buildSystem over the unary edges): the reference's own order,
 * against which the GPU's (reduction-shaped) decisions are compared in tests/test_pose_gpu.py. */
int oracle_pose_optimization_g2o_order(const pose_problem_t* p, pose_result_t* r) { return pose_optimization(p, r, 1); }

static int pose_optimization(const pose_problem_t* p, pose_result_t* r, int g2o_order)
{
    const int n = p->n;
    memcpy(r->pose_q, p->pose_q, sizeof(r->pose_q));
    memcpy(r->pose_t, p->pose_t, sizeof(r->pose_t));
    r->trials = 0;
    for (int i = 0; i < 4; i++) r->iterations[i] = 0;
    for (int e = 0; e < n; e++) r->outlier[e] = 0;
    r->n_inliers = 0;
    if (n < 3) return 0;   /* nInitialCorrespondences < 3: return 0, pose untouched */
    pose_ctx c;
    memset(&c, 0, sizeof(c));
    c.p = p;
    c.g2o_order = g2o_order;
    c.level = (uint8_t*)calloc(n, 1);
    c.robust = (uint8_t*)malloc(n);
    c.err = (double*)calloc(3 * (size_t)n, sizeof(double));
    memset(c.robust, 1, n);
    const double chi2Mono = 5.991, chi2Stereo = 7.815;
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        memcpy(c.q, p->pose_q, sizeof(c.q));   /* vSE3->setEstimate(toSE3Quat(pFrame->mTcw)) */
        memcpy(c.t, p->pose_t, sizeof(c.t));
        int nact = 0;
        for (int e = 0; e < n; e++) nact += c.level[e] == 0;
        if (nact > 0) {   /* an empty level-0 graph has no vertex to optimise (optimize returns -1) */
            int ok = 1;
            for (int i = 0; i < 10 && ok; i++) {
                ok = pose_lm_iteration(&c, i, r) == LM_OK;
                r->iterations[it]++;
            }
        }
        nBad = 0;
        for (int e = 0; e < n; e++) {
            if (c.level[e]) pose_compute_error(&c, e);
            const double chi2 = pose_chi2(&c, e);
            const double thr = p->obs[3 * e + 2] >= 0 ? chi2Stereo : chi2Mono;
            if ((float)chi2 > (float)thr) {   /* const float chi2 = e->chi2(); chi2 > chi2Mono[it] */
                r->outlier[e] = 1;
                c.level[e] = 1;
                nBad++;
            } else {
                r->outlier[e] = 0;
                c.level[e] = 0;
            }
            if (it == 2) c.robust[e] = 0;
        }
        if (n < 10) break;   /* optimizer.edges().size() counts every edge of the graph */
    }
    memcpy(r->pose_q, c.q, sizeof(c.q));
    memcpy(r->pose_t, c.t, sizeof(c.t));
    r->n_inliers = n - nBad;
    free(c.level);
    free(c.robust);
    free(c.err);
    return 0;
}
