// ORACLE / TEST INFRASTRUCTURE ONLY (N1 measurement): DistributeOctTree
// (R/src/ORBextractor.cpp:571-817, ExtractorNode::DivideNode :513-569) restated on a real
// std::list of heap-allocated nodes, with the final phase's sort over (size, node pointer) as the
// reference does it (:736), so equal-size nodes are ordered by their glibc heap addresses.  The
// node type mirrors ExtractorNode's members (a vector of 28-byte keypoints, four int corners, a
// list iterator, a flag) and the same allocation sequence (children built as locals reserving the
// parent's size, copied into the list, locals freed), so the heap sees the same request sizes.
// It pins nothing (the addresses depend on everything the process allocated before); it measures
// how often the build's creation-order tie-break (oracle_distribute_octree, csrc k_octree) and a
// real allocator disagree.
#include <algorithm>
#include <cmath>
#include <list>
#include <utility>
#include <vector>

namespace {
struct Kp {   // cv::KeyPoint layout: pt, size, angle, response, octave, class_id (28 bytes)
    float x, y, size, angle, response;
    int octave, class_id;
};
struct P2 {
    int x, y;
};
struct Node {
    std::vector<Kp> keys;
    P2 ul, ur, bl, br;
    std::list<Node>::iterator self;
    bool noMore = false;
    long seq = 0;   // creation sequence (mode 1 only)
    void divide(Node& a, Node& b, Node& c, Node& d) const {
        const int hx = (int)std::ceil((float)(ur.x - ul.x) / 2), hy = (int)std::ceil((float)(br.y - ul.y) / 2);
        a.ul = ul; a.ur = {ul.x + hx, ul.y}; a.bl = {ul.x, ul.y + hy}; a.br = {ul.x + hx, ul.y + hy};
        b.ul = a.ur; b.ur = ur; b.bl = a.br; b.br = {ur.x, ul.y + hy};
        c.ul = a.bl; c.ur = a.br; c.bl = bl; c.br = {a.br.x, bl.y};
        d.ul = c.ur; d.ur = b.br; d.bl = c.br; d.br = br;
        for (Node* n : {&a, &b, &c, &d}) n->keys.reserve(keys.size());
        for (const Kp& k : keys) {
            if (k.x < a.ur.x) (k.y < a.br.y ? a : c).keys.push_back(k);
            else (k.y < a.br.y ? b : d).keys.push_back(k);
        }
        for (Node* n : {&a, &b, &c, &d}) if (n->keys.size() == 1) n->noMore = true;
    }
};
}  // namespace

// mode 0: ties by heap address (the reference); mode 1: ties by creation sequence (the build's
// rule; must reproduce oracle_distribute_octree exactly, which validates this restatement)
extern "C" int n1_list_octree(const float* kx, const float* ky, const float* kr, int n, int minX, int maxX, int minY,
                              int maxY, int N, int mode, int* out_idx) {
    long created = 0;
    // the keypoint's class_id carries its input index, so the caller can compare selections
    const int nIni = (int)std::round((float)(maxX - minX) / (float)(maxY - minY));
    const float hX = (float)(maxX - minX) / (float)nIni;
    std::list<Node> nodes;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; i++) {
        Node s;
        s.ul = {(int)(hX * (float)i), 0};
        s.ur = {(int)(hX * (float)(i + 1)), 0};
        s.bl = {s.ul.x, maxY - minY};
        s.br = {s.ur.x, maxY - minY};
        s.keys.reserve(n);
        nodes.push_back(s);
        ini[i] = &nodes.back();
    }
    for (int i = 0; i < n; i++) ini[(int)(kx[i] / hX)]->keys.push_back(Kp{kx[i], ky[i], 7.f, -1.f, kr[i], 0, i});
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->noMore = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }
    bool finish = false;
    std::vector<std::pair<int, Node*>> cand;
    cand.reserve(nodes.size() * 4);
    auto pushChildren = [&](Node& a, Node& b, Node& c, Node& d, std::vector<std::pair<int, Node*>>& out, int* nExp) {
        for (Node* ch : {&a, &b, &c, &d}) {
            if (ch->keys.empty()) continue;
            nodes.push_front(*ch);
            nodes.front().seq = created++;
            if (ch->keys.size() > 1) {
                if (nExp) (*nExp)++;
                out.push_back({(int)ch->keys.size(), &nodes.front()});
                nodes.front().self = nodes.begin();
            }
        }
    };
    while (!finish) {
        const int prev = (int)nodes.size();
        int nToExpand = 0;
        cand.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->noMore) { ++it; continue; }
            Node a, b, c, d;
            it->divide(a, b, c, d);
            pushChildren(a, b, c, d, cand, &nToExpand);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prev) {
            finish = true;
        } else if ((int)nodes.size() + nToExpand * 3 > N) {
            while (!finish) {
                const int prev2 = (int)nodes.size();
                std::vector<std::pair<int, Node*>> prevCand = cand;
                cand.clear();
                if (mode == 0)
                    std::sort(prevCand.begin(), prevCand.end());   // (size, heap address)
                else
                    std::sort(prevCand.begin(), prevCand.end(), [](const std::pair<int, Node*>& a, const std::pair<int, Node*>& b) {
                        return a.first != b.first ? a.first < b.first : a.second->seq < b.second->seq;
                    });
                for (int j = (int)prevCand.size() - 1; j >= 0; j--) {
                    Node a, b, c, d;
                    prevCand[j].second->divide(a, b, c, d);
                    pushChildren(a, b, c, d, cand, nullptr);
                    nodes.erase(prevCand[j].second->self);
                    if ((int)nodes.size() >= N) break;
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == prev2) finish = true;
            }
        }
    }
    int m = 0;
    for (const Node& nd : nodes) {
        const Kp* best = &nd.keys[0];
        for (size_t k = 1; k < nd.keys.size(); k++)
            if (nd.keys[k].response > best->response) best = &nd.keys[k];
        out_idx[m++] = best->class_id;
    }
    return m;
}
