// CPU timing of the local-BA host structure build (csrc/lba_host.h) on a config-4-sized graph:
// 24 keyframes (4 fixed), 3000 points, each seen by 2..8 keyframes.
// g++ -O2 -std=c++17 -I/opt/rocm/include tools/micro/build_structure_bench.cpp -o /tmp/bsb && /tmp/bsb
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>

#include "../../orb-slam2-_amd/csrc/lba_host.h"

int main() {
    const int NP = 24, NM = 3000;
    std::mt19937 rng(42);
    std::vector<uint8_t> fixed(NP, 0);
    std::vector<int64_t> pid(NP), mid(NM);
    for (int i = 0; i < NP; i++) { pid[i] = i; fixed[i] = (i == 0 || i >= 20); }
    for (int i = 0; i < NM; i++) mid[i] = 100 + i;
    std::vector<int32_t> ep, epo;
    for (int m = 0; m < NM; m++) {
        const int k = 2 + rng() % 7;
        std::vector<int> kf(NP);
        for (int i = 0; i < NP; i++) kf[i] = i;
        std::shuffle(kf.begin(), kf.end(), rng);
        for (int j = 0; j < k; j++) { ep.push_back(m); epo.push_back(kf[j]); }
    }
    lba_problem p{};
    p.n_poses = NP; p.pose_fixed = fixed.data(); p.pose_id = pid.data();
    p.n_points = NM; p.point_id = mid.data();
    p.n_edges = (int)ep.size(); p.edge_point = ep.data(); p.edge_pose = epo.data();
    std::vector<uint8_t> level(p.n_edges, 0);
    orbamd::HostStructure hs;
    double best = 1e30;
    for (int rep = 0; rep < 200; rep++) {
        const auto t0 = std::chrono::steady_clock::now();
        orbamd::build_structure(&p, level, 0, 0, 1, hs);
        const auto t1 = std::chrono::steady_clock::now();
        best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("edges %d active %zu: best of 200 %.1f us\n", p.n_edges, hs.act.size(), best);
    return 0;
}
