/*
 * ORACLE / TEST INFRASTRUCTURE ONLY — CPU restatement of
 * Optimizer::LocalBundleAdjustment (R/src/Optimizer.cpp:564-918) with the g2o
 * pieces it runs: OptimizationAlgorithmLevenberg::solve
 * (G/core/optimization_algorithm_levenberg.cpp:61-164), BlockSolver<6,3> Schur
 * solve (G/core/block_solver.hpp:354-605), EdgeSE3ProjectXYZ /
 * EdgeStereoSE3ProjectXYZ (G/types/types_six_dof_expmap.{h,cpp}), SE3Quat exp /
 * map / product (G/types/se3quat.h), RobustKernelHuber (G/core/robust_kernel_impl.cpp:78-91).
 * R/ = /root/reference/ORB-SLAM2注释版/, G/ = R/Thirdparty/g2o/g2o/.
 *
 * Parity status: g2o/Eigen cannot be compiled here (Eigen absent); the linear
 * solve is a dense LDL^T without fill-reducing permutation in place of
 * SimplicialLDLT+AMD, so results agree with the reference up to floating-point
 * reordering — compared at 1e-5 (poses/points) as north_star states.
 * Parity unpinned against a real g2o run (none is possible offline).
 */
#ifndef LBA_ORACLE_H
#define LBA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n_poses;
    const double* pose_q;        /* [n_poses][4] Eigen coeffs (x, y, z, w) */
    const double* pose_t;        /* [n_poses][3] */
    const uint8_t* pose_fixed;   /* setFixed */
    const int64_t* pose_id;      /* g2o vertex id (KeyFrame::mnId) */
    int n_points;
    const double* point_xyz;     /* [n_points][3] */
    const int64_t* point_id;     /* mnId + maxKFid + 1 */
    const uint8_t* point_bad;    /* MapPoint::isBad() as seen by the outlier passes (may be NULL) */
    int n_edges;
    const int32_t* edge_point;   /* vertex 0 */
    const int32_t* edge_pose;    /* vertex 1 */
    const uint8_t* edge_stereo;  /* 0: EdgeSE3ProjectXYZ (u,v); 1: EdgeStereoSE3ProjectXYZ (u,v,ur) */
    const double* edge_obs;      /* [n_edges][3] */
    const double* edge_info;     /* Information = I * invSigma2 (float value) */
    const double* edge_cam;      /* [n_edges][5] fx fy cx cy bf */
} lba_problem_t;

typedef struct {
    int iters1, iters2;            /* 5, 10 */
    double chi2_mono, chi2_stereo; /* 5.991, 7.815 */
    double huber_mono, huber_stereo;   /* (float)sqrt(5.991), (float)sqrt(7.815) */
    int max_trials;                /* maxTrialsAfterFailure = 10 */
    int fixed_iterations;          /* 1: no early termination (kernel-parity mode) */
} lba_options_t;

typedef struct {
    double* pose_q;      /* out [n_poses][4] */
    double* pose_t;      /* out [n_poses][3] */
    double* point_xyz;   /* out [n_points][3] */
    uint8_t* edge_erase; /* out: vToErase membership */
    double* edge_chi2;   /* out: e->chi2() at the final check */
    int iterations[2];   /* outer iterations executed per optimize() call */
    int trials;          /* total LM trials */
    double* trace;       /* optional [max 64][4]: per outer iteration (iniChi, currentChi, lambda, qmax) */
    int n_trace;
} lba_result_t;

/* Returns 0, or 1 when *stop was already set before the first optimize() (the
 * reference returns without writing back, R/src/Optimizer.cpp:784-786). */
int oracle_lba_solve(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop,
                     lba_result_t* r);
/* OpenMP CPU path: g2o's G2O_OPENMP loops on `threads` host threads, serial sum
 * order kept, so the result is bitwise identical to oracle_lba_solve. */
int oracle_lba_solve_omp(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop,
                         lba_result_t* r, int threads);

/* Same, with the stop flag treated as set once the solve's LM trial count reaches stop_after_trials
 * (the test hook lba_debug_stop_after_trials of the library): terminate() is sampled after every
 * trial (G/core/optimization_algorithm_levenberg.cpp:149), before every iteration
 * (G/core/sparse_optimizer.cpp:376) and before the second optimize() (R/src/Optimizer.cpp:792-796). */
int oracle_lba_solve_stop_after(const lba_problem_t* p, const lba_options_t* o, int stop_after_trials,
                                lba_result_t* r);

/* Landmark-sharded variant (the multi-GPU algorithm of liborbslam2_amd): rank
 * `rank` of `world` owns points [rank*M/world, (rank+1)*M/world); `ar` all-reduces
 * n doubles in place across ranks (op 0 sum, 1 max). */
typedef void (*oracle_allreduce_fn)(void* user, double* v, int n, int op);
int oracle_lba_solve_dist(const lba_problem_t* p, const lba_options_t* o, const volatile uint8_t* stop,
                          lba_result_t* r, int rank, int world, oracle_allreduce_fn ar, void* user);

/* Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust)
 * (R/src/Optimizer.cpp:78-277): optimize(o->iters1) over every edge, Huber kernels with deltas
 * o->huber_mono / o->huber_stereo ((float)sqrt(5.99) / (float)sqrt(7.815)) when robust; no outlier
 * pass, edge_erase all 0; *stop ends the iterations but the estimates are still written. */
int oracle_global_ba(const lba_problem_t* p, const lba_options_t* o, int robust, const volatile uint8_t* stop,
                     lba_result_t* r);

/* Optimizer::PoseOptimization(Frame*) (R/src/Optimizer.cpp:306-535) on one frame: the edges are
 * the frame's keypoints with a map point, obs = (u, v, ur) with ur < 0 for a monocular
 * observation (Frame::mvuRight), xw the map point (float values), info = invSigma2 of the
 * keypoint octave. */
typedef struct {
    double pose_q[4], pose_t[3];   /* Converter::toSE3Quat(pFrame->mTcw) */
    int n;
    const double* obs;             /* [n][3] */
    const double* xw;              /* [n][3] */
    const double* info;            /* [n] */
    double fx, fy, cx, cy, bf;
} pose_problem_t;

typedef struct {
    double pose_q[4], pose_t[3];   /* optimised pose (input pose when n < 3) */
    uint8_t* outlier;              /* [n] Frame::mvbOutlier */
    int n_inliers;                 /* return value: nInitialCorrespondences - nBad */
    int iterations[4];             /* LM iterations per round */
    int trials;
} pose_result_t;

int oracle_pose_optimization(const pose_problem_t* p, pose_result_t* r);
/* g2o's summation order (edges in order) instead of the GPU kernel's reduction shape. */
int oracle_pose_optimization_g2o_order(const pose_problem_t* p, pose_result_t* r);

/* Helpers shared with tests: Converter::toSE3Quat / SE3Quat::exp semantics. */
void oracle_quat_from_matrix(const double R[9], double q[4]);
void oracle_se3_exp_left(const double upd[6], const double q[4], const double t[3], double qo[4], double to[3]);

#ifdef __cplusplus
}
#endif
#endif
