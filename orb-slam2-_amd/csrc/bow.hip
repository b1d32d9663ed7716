// MI355X-native DBoW2 vocabulary descent: TemplatedVocabulary<FORB::TDescriptor, FORB>::transform
// (D/DBoW2/TemplatedVocabulary.h:1151-1283) as ORB-SLAM2 runs it for every frame and keyframe
// (Frame::ComputeBoW, R/src/Frame.cpp; KeyFrame::ComputeBoW): each 256-bit descriptor walks the
// k-ary tree from the root, taking at every level the child with the least Hamming distance
// (FORB::distance, D/DBoW2/FORB.cpp:82-103; strict <, so the first child wins ties) until a
// leaf; the leaf gives the word id and its weight, the node passed at level L - levelsup is the
// FeatureVector node.  One thread per descriptor; the vocabulary (node descriptors, child lists,
// word ids, weights — ~35 MB for the 10^6-word ORBvoc) is uploaded once and stays in HBM.
// BowVector / FeatureVector assembly (map insertion in feature order, L1 normalisation) is
// O(#features) host bookkeeping left to the caller.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "common.h"

namespace orbamd {

// Device layout: the tree renumbered breadth first, so the children of every node are one
// contiguous run of node records (their 32-byte descriptors adjacent in HBM, one 2-int record
// (first child, count) per node); orig maps back to the caller's node ids for the FeatureVector.
struct VocDev {
    const uint4* desc;         // [n][2], breadth-first order
    const int2* fc;            // [n] (first child, child count)
    const int32_t* word;       // [n]
    const double* weight;      // [n]
    const int32_t* orig;       // [n] caller's node id
    int L;
};

constexpr int kBowChunk = 10;   // children compared per batch of independent loads (k = 10 in ORBvoc)

__device__ __forceinline__ int hamming256(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(256) void k_bow_transform(VocDev v, const uint4* __restrict__ feats, int n, int levelsup,
                                                       int32_t* __restrict__ word_id, double* __restrict__ weight,
                                                       int32_t* __restrict__ node_id) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 a0 = feats[2 * i], a1 = feats[2 * i + 1];
    const int nid_level = v.L - levelsup;
    int nid = -1, node = 0, level = 0;
    for (;;) {
        const int2 fc = v.fc[node];
        if (fc.y == 0) break;   // isLeaf
        ++level;
        int best = fc.x, bestD = 0x7fffffff;
        for (int base = 0; base < fc.y; base += kBowChunk) {
            // a chunk's loads are issued together; indices past the last child repeat it, which
            // cannot win under the strict < (the reference's first-child-wins tie rule)
            uint4 b[2 * kBowChunk];
#pragma unroll
            for (int j = 0; j < kBowChunk; j++) {
                const int id = fc.x + min(base + j, fc.y - 1);
                b[2 * j] = v.desc[2 * id];
                b[2 * j + 1] = v.desc[2 * id + 1];
            }
#pragma unroll
            for (int j = 0; j < kBowChunk; j++) {
                const int d = hamming256(a0, a1, b[2 * j], b[2 * j + 1]);
                if (d < bestD) { bestD = d; best = fc.x + min(base + j, fc.y - 1); }
            }
        }
        node = best;
        if (level == nid_level) nid = node;
    }
    word_id[i] = v.word[node];
    weight[i] = v.weight[node];
    node_id[i] = nid < 0 ? 0 : v.orig[nid];
}

}  // namespace orbamd

using namespace orbamd;

struct orb_vocab {
    int device = 0;
    int n_nodes = 0, L = 0;
    char* base = nullptr;
    VocDev v{};
    hipStream_t stream = nullptr;
    char* scratch = nullptr;
    size_t scratchCap = 0;
};

extern "C" {

int orb_vocabulary_create(int device, const orb_vocabulary* voc, orb_vocab** out) try {
    if (!voc || !out || voc->n_nodes < 1 || !voc->desc || !voc->child_start || !voc->word_id || !voc->weight ||
        voc->L < 1)
        return ORB_EINVAL;
    const int n = voc->n_nodes;
    const int nc = voc->child_start[n];
    if (voc->child_start[0] != 0 || nc < 0 || (nc > 0 && !voc->child_idx)) return ORB_EINVAL;
    for (int i = 0; i < n; i++)
        if (voc->child_start[i + 1] < voc->child_start[i]) return ORB_EINVAL;
    for (int c = 0; c < nc; c++)
        if (voc->child_idx[c] <= 0 || voc->child_idx[c] >= n) return ORB_EINVAL;
    int st = check_device(device);
    if (st) return st;
    // breadth-first renumbering: children of each node become consecutive ids in their order
    std::vector<int32_t> orig(n), renum(n, -1);
    std::vector<int2> fc(n);
    orig[0] = 0;
    renum[0] = 0;
    int next = 1;
    for (int q = 0; q < next; q++) {
        const int o = orig[q];
        const int c0 = voc->child_start[o], c1 = voc->child_start[o + 1];
        fc[q] = make_int2(next, c1 - c0);
        for (int c = c0; c < c1; c++) {
            const int ch = voc->child_idx[c];
            if (renum[ch] >= 0 || next >= n) return ORB_EINVAL;   // not a tree
            renum[ch] = next;
            orig[next++] = ch;
        }
    }
    std::vector<uint8_t> desc((size_t)next * 32);
    std::vector<int32_t> word(next);
    std::vector<double> weight(next);
    for (int q = 0; q < next; q++) {
        memcpy(&desc[(size_t)q * 32], voc->desc + (size_t)orig[q] * 32, 32);
        word[q] = voc->word_id[orig[q]];
        weight[q] = voc->weight[orig[q]];
    }
    ORB_HIP_TRY(hipSetDevice(device));
    orb_vocab* h = new orb_vocab();
    h->device = device;
    h->n_nodes = next;
    h->L = voc->L;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bD = al((size_t)next * 32), bF = al((size_t)next * 8), bW = al((size_t)next * 4),
                 bG = al((size_t)next * 8), bO = al((size_t)next * 4);
    if (hipMalloc(&h->base, bD + bF + bW + bG + bO) != hipSuccess) { delete h; return ORB_ENOMEM; }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(h->base);
        delete h;
        return ORB_EGPU;
    }
    char* c = h->base;
    auto put = [&](const void* src, size_t bytes, size_t cap) {
        char* r = c;
        c += cap;
        (void)hipMemcpyAsync(r, src, bytes, hipMemcpyHostToDevice, h->stream);
        return r;
    };
    h->v.desc = (const uint4*)put(desc.data(), (size_t)next * 32, bD);
    h->v.fc = (const int2*)put(fc.data(), (size_t)next * 8, bF);
    h->v.word = (const int32_t*)put(word.data(), (size_t)next * 4, bW);
    h->v.weight = (const double*)put(weight.data(), (size_t)next * 8, bG);
    h->v.orig = (const int32_t*)put(orig.data(), (size_t)next * 4, bO);
    h->v.L = voc->L;
    if (hipStreamSynchronize(h->stream) != hipSuccess) { orb_vocabulary_destroy(h); return ORB_EGPU; }
    *out = h;
    return ORB_OK;
} ORB_ABI_CATCH

void orb_vocabulary_destroy(orb_vocab* h) try {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->base) (void)hipFree(h->base);
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
} ORB_ABI_CATCH_VOID

int orb_vocabulary_transform_device(orb_vocab* h, const uint8_t* d_desc, int n, int levelsup, int32_t* d_word_id,
                                    double* d_weight, int32_t* d_node_id, void* stream) try {
    if (!h || n < 0 || (n > 0 && (!d_desc || !d_word_id || !d_weight || !d_node_id))) return ORB_EINVAL;
    if (n == 0) return ORB_OK;
    ORB_HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(k_bow_transform, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       h->v, reinterpret_cast<const uint4*>(d_desc), n, levelsup, d_word_id, d_weight, d_node_id);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
} ORB_ABI_CATCH

int orb_vocabulary_transform(orb_vocab* h, const uint8_t* desc, int n, int levelsup, int32_t* word_id, double* weight,
                             int32_t* node_id) try {
    if (!h || n < 0 || (n > 0 && (!desc || !word_id || !weight || !node_id))) return ORB_EINVAL;
    if (n == 0) return ORB_OK;
    ORB_HIP_TRY(hipSetDevice(h->device));
    const size_t need = (size_t)n * (32 + 4 + 8 + 4) + 1024;
    if (h->scratchCap < need) {
        std::lock_guard<std::mutex> lk(legacy_capture_mutex());   // hipFree / hipMalloc (common.h)
        if (h->scratch) (void)hipFree(h->scratch);
        h->scratch = nullptr;
        h->scratchCap = 0;
        if (hipMalloc(&h->scratch, need) != hipSuccess) return ORB_ENOMEM;
        h->scratchCap = need;
    }
    uint8_t* dD = (uint8_t*)h->scratch;
    double* dG = (double*)(h->scratch + (((size_t)n * 32 + 255) & ~(size_t)255));
    int32_t* dW = (int32_t*)((char*)dG + (((size_t)n * 8 + 255) & ~(size_t)255));
    int32_t* dN = dW + (((size_t)n + 63) & ~(size_t)63);
    hipStream_t s = h->stream;
    ORB_HIP_TRY(hipMemcpyAsync(dD, desc, (size_t)n * 32, hipMemcpyHostToDevice, s));
    int rc = orb_vocabulary_transform_device(h, dD, n, levelsup, dW, dG, dN, s);
    if (rc) return rc;
    ORB_HIP_TRY(hipMemcpyAsync(word_id, dW, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipMemcpyAsync(weight, dG, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipMemcpyAsync(node_id, dN, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_TRY(hipStreamSynchronize(s));
    return ORB_OK;
} ORB_ABI_CATCH

}  // extern "C"
