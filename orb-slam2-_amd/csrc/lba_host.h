// Host side of lba_solve: SparseOptimizer::initializeOptimization(level) + the block
// structure of BlockSolver<6,3> (G/core/sparse_optimizer.cpp:199-267,
// G/core/block_solver.hpp:143-296) as flat index arrays for the kernels.  Plain C++ (no HIP),
// so the CPU micro-benchmark tools/micro/build_structure_bench.cpp can include it.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/orbslam2_amd.h"

namespace orbamd {

// act: active edges (edge order); poseIdx: pose -> Hessian index or -1; ptGlob: owned landmark
// local -> global index; actPt / actPi: per active edge its local landmark and pose Hessian
// index (-1 fixed).  CSR by landmark (ptStart, ptAct: act positions sorted by pose index,
// fixed poses last) and CSR by free pose (poStart, poAct: act positions sorted by landmark;
// poPt: their landmarks) — the Schur kernel intersects two poses' landmark lists instead of
// reading a precomputed pair list.
struct HostStructure {
    std::vector<int32_t> act, poseIdx, ptLocal, ptGlob, actPt, actPi, ptStart, ptAct, poStart, poAct, poPt, freePoses;
    int P = 0, M = 0;
};

// initializeOptimization(level) (G/core/sparse_optimizer.cpp:199-267) restricted to the
// landmarks owned by this rank (contiguous range of point indices), first half: the active
// edges (unless `withAct` is false: the caller knows they are all of them) and the vertex
// index maps (poseIdx / freePoses, ptLocal / ptGlob).  build_csr makes the rest; the single-
// process solver builds that part on the device instead (k_struct_*, lba.hip).
inline void build_maps(const lba_problem* p, const std::vector<uint8_t>& level, int lvl, int rank, int world,
                       HostStructure& s, bool withAct = true) {
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
    if (withAct) s.act.reserve(NE);
    for (int e = 0; withAct && e < NE; e++) {
        if (level[e] != lvl) continue;
        const int pt = p->edge_point[e];
        if (pt < own0 || pt >= own1) continue;
        s.act.push_back(e);
    }
    // g2o orders the Hessian blocks by vertex id; callers usually pass ids ascending already
    auto by_id = [](std::vector<int>& o, const int64_t* id) {
        if (std::is_sorted(o.begin(), o.end(), [&](int a, int b) { return id[a] < id[b]; })) return;
        std::stable_sort(o.begin(), o.end(), [&](int a, int b) { return id[a] < id[b]; });
    };
    std::vector<int> order;
    order.reserve(std::max(NP, NM));
    for (int i = 0; i < NP; i++)
        if (poseAct[i] && !p->pose_fixed[i]) order.push_back(i);
    by_id(order, p->pose_id);
    s.poseIdx.assign(NP, -1);
    for (size_t k = 0; k < order.size(); k++) s.poseIdx[order[k]] = (int)k;
    s.freePoses = order;
    s.P = (int)order.size();
    order.clear();
    for (int i = own0; i < own1; i++)
        if (ptAct[i]) order.push_back(i);
    by_id(order, p->point_id);
    s.ptLocal.assign(NM, -1);
    for (size_t k = 0; k < order.size(); k++) s.ptLocal[order[k]] = (int)k;
    s.ptGlob = order;
    s.M = (int)order.size();
}

// Second half: per active edge its local landmark and pose index, the CSR by landmark and the
// CSR by free pose.
inline void build_csr(const lba_problem* p, HostStructure& s) {
    const int NA = (int)s.act.size();
    s.actPt.resize(NA);
    s.actPi.resize(NA);
    for (int k = 0; k < NA; k++) {
        s.actPt[k] = s.ptLocal[p->edge_point[s.act[k]]];
        s.actPi[k] = s.poseIdx[p->edge_pose[s.act[k]]];
    }
    // CSR by landmark sorted by pose key (Hessian index, fixed poses last as key P): a stable
    // counting sort by key, scattered in key order into the landmark buckets
    const int P = s.P;
    std::vector<int32_t> byKey(NA), kStart(P + 2, 0);
    for (int k = 0; k < NA; k++) kStart[(s.actPi[k] < 0 ? P : s.actPi[k]) + 1]++;
    for (int i = 0; i <= P; i++) kStart[i + 1] += kStart[i];
    {
        std::vector<int32_t> fill(kStart.begin(), kStart.end() - 1);
        for (int k = 0; k < NA; k++) byKey[fill[s.actPi[k] < 0 ? P : s.actPi[k]]++] = k;
    }
    s.ptStart.assign(s.M + 1, 0);
    for (int k = 0; k < NA; k++) s.ptStart[s.actPt[k] + 1]++;
    for (int i = 0; i < s.M; i++) s.ptStart[i + 1] += s.ptStart[i];
    s.ptAct.resize(NA);
    {
        std::vector<int32_t> fill(s.ptStart.begin(), s.ptStart.end() - 1);
        for (int t = 0; t < NA; t++) {
            const int k = byKey[t];
            s.ptAct[fill[s.actPt[k]]++] = k;
        }
    }
    // CSR by free pose sorted by landmark: the landmark-major list scattered into pose buckets
    s.poStart.assign(kStart.begin(), kStart.begin() + P + 1);
    s.poAct.resize(kStart[P]);
    s.poPt.resize(kStart[P]);
    {
        std::vector<int32_t> fill(kStart.begin(), kStart.begin() + P);
        for (int t = 0; t < NA; t++) {
            const int k = s.ptAct[t], i = s.actPi[k];
            if (i < 0) continue;
            const int at = fill[i]++;
            s.poAct[at] = k;
            s.poPt[at] = s.actPt[k];
        }
    }
}

inline void build_structure(const lba_problem* p, const std::vector<uint8_t>& level, int lvl, int rank, int world,
                            HostStructure& s) {
    build_maps(p, level, lvl, rank, world, s);
    build_csr(p, s);
}

}  // namespace orbamd
