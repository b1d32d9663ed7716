// SE3Quat device/host math shared by the local-BA and pose-only optimisers (G/types/se3quat.h:
// map :217, exp :223, normalizeRotation :280; Eigen Quaterniond(Matrix3d) and toRotationMatrix).
#pragma once
#include <hip/hip_runtime.h>

namespace orbamd {

__device__ __forceinline__ void d_cross(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ void d_quat_rot(const double q[4], const double v[3], double o[3]) {
    double uv[3], c[3];
    d_cross(q, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    d_cross(q, uv, c);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q[3] * uv[i] + c[i];
}
__device__ __forceinline__ void d_quat_to_R(const double q[4], double R[9]) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
__host__ __device__ inline void hd_normalize_rotation(double q[4]) {
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}
// Eigen's branch for a non-positive trace with the largest diagonal entry at I
template <int I>
__host__ __device__ inline void quat_from_matrix_major(const double m[9], double q[4]) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double s = sqrt(m[I * 3 + I] - m[J * 3 + J] - m[K * 3 + K] + 1.0);
    q[I] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (m[K * 3 + J] - m[J * 3 + K]) * s;
    q[J] = (m[J * 3 + I] + m[I * 3 + J]) * s;
    q[K] = (m[K * 3 + I] + m[I * 3 + K]) * s;
}
// Eigen Quaterniond(const Matrix3d&) + SE3Quat::normalizeRotation
__host__ __device__ inline void hd_quat_from_matrix(const double m[9], double q[4]) {
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
        if (m[8] > (i ? m[4] : m[0])) i = 2;
        // the three cases spelled out so every index is a constant (no scratch-indexed arrays)
        if (i == 0) quat_from_matrix_major<0>(m, q);
        else if (i == 1) quat_from_matrix_major<1>(m, q);
        else quat_from_matrix_major<2>(m, q);
    }
    hd_normalize_rotation(q);
}
// T <- exp(upd) * T  (VertexSE3Expmap::oplusImpl, SE3Quat::exp, SE3Quat::operator*)
__device__ inline void d_se3_exp_left(const double upd[6], double q[4], double t[3]) {
    const double w0 = upd[0], w1 = upd[1], w2 = upd[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9], R[9], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            O2[i * 3 + j] = O[i * 3] * O[j] + O[i * 3 + 1] * O[3 + j] + O[i * 3 + 2] * O[6 + j];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) { R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i]; V[i] = R[i]; }
    } else {
        // (g2o's pow(theta, 3) as two products: the same value to an ulp, where theta - sin(theta)
        // already carries the cancellation error; ocml's f64 pow was the longest link of the pose
        // update that ends every reduced solve)
        double sn, cs;
        sincos(theta, &sn, &cs);
        const double t2 = theta * theta;
        const double a = sn / theta, b = (1 - cs) / t2;
        const double c = (theta - sn) / (t2 * theta);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    double qe[4], te[3], rt[3];
    hd_quat_from_matrix(R, qe);
    for (int i = 0; i < 3; i++) te[i] = V[i * 3] * upd[3] + V[i * 3 + 1] * upd[4] + V[i * 3 + 2] * upd[5];
    d_quat_rot(qe, t, rt);
    for (int i = 0; i < 3; i++) t[i] = te[i] + rt[i];
    double r[4];
    r[3] = qe[3] * q[3] - qe[0] * q[0] - qe[1] * q[1] - qe[2] * q[2];
    r[0] = qe[3] * q[0] + qe[0] * q[3] + qe[1] * q[2] - qe[2] * q[1];
    r[1] = qe[3] * q[1] + qe[1] * q[3] + qe[2] * q[0] - qe[0] * q[2];
    r[2] = qe[3] * q[2] + qe[2] * q[3] + qe[0] * q[1] - qe[1] * q[0];
    hd_normalize_rotation(r);
    for (int i = 0; i < 4; i++) q[i] = r[i];
}

}  // namespace orbamd
