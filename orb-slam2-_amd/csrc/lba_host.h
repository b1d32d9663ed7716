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

struct HostStructure {
    std::vector<int32_t> act, poseIdx, ptLocal, ptGlob, actPos, ptStart, ptEdges, poStart, poEdges, prStart, prE1,
        prE2, pairI, pairJ, freePoses, actPt, actPi;
    int P = 0, M = 0;
};

// initializeOptimization(level) (G/core/sparse_optimizer.cpp:199-267) restricted to the
// landmarks owned by this rank (contiguous range of point indices).
inline void build_structure(const lba_problem* p, const std::vector<uint8_t>& level, int lvl, int rank, int world,
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
    // Edges bucketed by pose key (Hessian index, fixed poses last as key P) with a stable
    // counting sort; scattering the buckets in key order into per-landmark lists gives the CSR
    // by landmark with each list sorted by pose index (fixed last, edge order among them), and
    // the free-pose buckets are the CSR by pose (edge order) as they stand.
    const int P = s.P, NA = (int)s.act.size();
    std::vector<int32_t> key(NA), byKey(NA), kStart(P + 2, 0);
    for (int k = 0; k < NA; k++) {
        const int pi = s.actPi[k];
        key[k] = pi < 0 ? P : pi;
        kStart[key[k] + 1]++;
    }
    for (int i = 0; i <= P; i++) kStart[i + 1] += kStart[i];
    {
        std::vector<int32_t> fill(kStart.begin(), kStart.end() - 1);
        for (int k = 0; k < NA; k++) byKey[fill[key[k]]++] = k;   // act positions
    }
    s.ptStart.assign(s.M + 1, 0);
    for (int k = 0; k < NA; k++) s.ptStart[s.actPt[k] + 1]++;
    for (int i = 0; i < s.M; i++) s.ptStart[i + 1] += s.ptStart[i];
    s.ptEdges.resize(NA);
    std::vector<int32_t> ptPos(NA);   // act positions, landmark-major (parallel to ptEdges)
    {
        std::vector<int32_t> fill(s.ptStart.begin(), s.ptStart.end() - 1);
        for (int t = 0; t < NA; t++) {
            const int k = byKey[t], at = fill[s.actPt[k]]++;
            ptPos[at] = k;
            s.ptEdges[at] = s.act[k];
        }
    }
    s.poStart.assign(kStart.begin(), kStart.begin() + P + 1);
    s.poEdges.resize(kStart[P]);
    for (int t = 0; t < kStart[P]; t++) s.poEdges[t] = s.act[byKey[t]];
    // pose-pair blocks (i <= j) with their contributions (landmark order, then edge order)
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
    for (int l = 0; l < s.M; l++) {
        const int a0 = s.ptStart[l], a1 = s.ptStart[l + 1];
        for (int a = a0; a < a1; a++) {
            const int i1 = key[ptPos[a]];
            if (i1 == P) break;   // fixed poses are last
            const int* row = pairOf.data() + (size_t)i1 * P;
            for (int b = a; b < a1; b++) {
                const int i2 = key[ptPos[b]];
                if (i2 == P) break;
                cnt[row[i2] + 1]++;
            }
        }
    }
    for (int i = 0; i < npairs; i++) cnt[i + 1] += cnt[i];
    s.prStart = cnt;
    s.prE1.resize(cnt[npairs]);
    s.prE2.resize(cnt[npairs]);
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int l = 0; l < s.M; l++) {
        const int a0 = s.ptStart[l], a1 = s.ptStart[l + 1];
        for (int a = a0; a < a1; a++) {
            const int i1 = key[ptPos[a]];
            if (i1 == P) break;
            const int* row = pairOf.data() + (size_t)i1 * P;
            for (int b = a; b < a1; b++) {
                const int i2 = key[ptPos[b]];
                if (i2 == P) break;
                const int at = fill[row[i2]]++;
                s.prE1[at] = ptPos[a];   // act positions (Hpl_e rows)
                s.prE2[at] = ptPos[b];
            }
        }
    }
}

}  // namespace orbamd
