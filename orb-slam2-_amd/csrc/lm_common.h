// Levenberg-Marquardt helpers shared by the local-BA and pose-only optimisers
// (G/core/optimization_algorithm_levenberg.cpp).
#pragma once
#include <hip/hip_runtime.h>

namespace orbamd {

// t^3 rounded once (double-double product): the host path used std::pow(t, 3), which glibc
// rounds correctly except in vanishingly rare cases.
__device__ __forceinline__ double cube_rn(double t) {
    const double p = t * t, ep = __builtin_fma(t, t, -p);
    const double q = p * t, eq = __builtin_fma(p, t, -q);
    return q + __builtin_fma(ep, t, eq);
}

}  // namespace orbamd
