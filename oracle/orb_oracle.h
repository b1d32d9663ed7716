/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the ORB-SLAM2 hot path (reference: YHY138/ORB-SLAM2-,
 * mounted at /root/reference/ORB-SLAM2注释版, abbreviated R/ below).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline.  The product
 * (orb-slam2-_amd/) never links or calls it.
 *
 * Parity status:
 *  - The reference cannot be compiled here (OpenCV / Eigen absent)
 *    and ships no tests or golden vectors.
 *  - OpenCV primitives (resize INTER_LINEAR 8U, GaussianBlur 7x7 8U, FAST-9,
 *    fastAtan2, cvRound) are restated from their published scalar algorithms
 *    (OpenCV 2.4/3.x non-IPP, non-SIMD path): PARITY UNPINNED against a real
 *    OpenCV build (none exists offline); pinned by the committed fixtures in
 *    tests/golden/ that this restatement generated.
 *  - glibc sinf/cosf: restated and pinned bit-exactly (exhaustive over
 *    [0, 2*pi]) against the host libm (tests/test_sincosf.py).
 *  - DistributeOctTree's equal-size tie break (pointer order, R/src/ORBextractor.cpp:736)
 *    is allocator dependent; pinned here to node creation order.
 *  - FP contraction pinned OFF; build with -ffp-contract=off.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {            /* == cv::KeyPoint memory layout (28 bytes) */
    float x, y, size, angle, response;
    int32_t octave, class_id;
} oracle_keypoint;

typedef struct {
    int nfeatures;
    float scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
} oracle_orb_params;

/* Extractor constant tables (R/src/ORBextractor.cpp:418-502). Arrays sized nlevels; umax sized 16. */
void oracle_orb_tables(const oracle_orb_params* p, float* scale, float* inv_scale,
                       float* sigma2, float* inv_sigma2, int* features_per_level, int* umax);

/* Level geometry: cvRound(W*invScale) x cvRound(H*invScale) (R/src/ORBextractor.cpp:1203). */
void oracle_level_sizes(const oracle_orb_params* p, int w, int h, int* lw, int* lh);

/* cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for 8UC1, scalar fixed-point path. */
void oracle_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstride,
                             uint8_t* dst, int dw, int dh, size_t dstride);

/* cv::GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) for 8UC1. */
void oracle_gaussian_blur7_u8(const uint8_t* src, int w, int h, size_t stride,
                              uint8_t* dst, size_t dstride);

/* cv::FAST(roi, kps, threshold, nonmax=true), TYPE_9_16, on the ROI [x0,x0+w) x [y0,y0+h)
 * of img.  Writes ROI-relative (x, y, score) triples; returns the count (<= cap). */
int oracle_fast_roi(const uint8_t* img, size_t stride, int x0, int y0, int w, int h,
                    int threshold, int* out_xys, int cap);

/* OpenCV fastAtan2 (degrees, [0,360)). */
float oracle_fast_atan2(float y, float x);

/* glibc-exact sinf/cosf (see sincosf_glibc.h); returns 0 on success. */
long oracle_sincosf_check(unsigned stride, long* n_checked);
int oracle_sincosf(float x, float* s, float* c);

/* Full ORBextractor::operator() (R/src/ORBextractor.cpp:1120-1188).
 * Returns number of keypoints N (possibly > capacity: then only the status is
 * -7 (E2BIG) and *n_out = N).  Empty image (w==0||h==0) -> returns 0 and leaves
 * outputs untouched, *n_out untouched (N13).
 * Optional outputs (may be NULL):
 *   level_counts[nlevels] : keypoints per level after DistributeOctTree
 *   pre_counts[nlevels]   : FAST keypoints per level before distribution
 *   pyramid               : concatenation of all levels (row-major, stride=width)
 *   blurred               : concatenation of all blurred levels
 */
int oracle_orb_extract(const oracle_orb_params* p, const uint8_t* img, int w, int h, size_t stride,
                       oracle_keypoint* kps, uint8_t* desc, int capacity, int* n_out,
                       int* level_counts, int* pre_counts, uint8_t* pyramid, uint8_t* blurred);

/* One level's FAST keys before DistributeOctTree (the cell loop of R/src/ORBextractor.cpp:819-896),
 * in vToDistributeKeys order, border-relative; returns the count (only the first cap written). */
int oracle_level_keys(const oracle_orb_params* p, const uint8_t* img, int cols, int rows, float* kx, float* ky,
                      float* kr, int cap);

/* DistributeOctTree on explicit inputs (for unit tests): keys are (x,y,response)
 * triples in level-interior coordinates; writes the indices of the retained keys
 * (into the input array) in output order; returns count. */
int oracle_distribute_octree(const float* kx, const float* ky, const float* kresp, int nkeys,
                             int minX, int maxX, int minY, int maxY, int N, int* out_idx);

/* ORBmatcher::DescriptorDistance (R/src/ORBmatcher.cpp:1901-1917). */
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Frame grid geometry + undistorted keypoint view used by the matcher. */
typedef struct {
    int n;                       /* number of keypoints */
    const float* x;              /* mvKeysUn[i].pt.x */
    const float* y;
    const float* angle;
    const int32_t* octave;
    const uint8_t* desc;         /* n x 32 */
    const float* uright;         /* mvuRight (may be NULL: all -1) */
    float min_x, min_y, max_x, max_y;          /* mnMinX.. */
    float grid_w_inv, grid_h_inv;              /* mfGridElementWidthInv.. */
} oracle_frame;

/* Frame::GetFeaturesInArea (R/src/Frame.cpp:387-440) with grid built by
 * AssignFeaturesToGrid/PosInGrid (R/src/Frame.cpp:244-260,442-452). Returns count. */
int oracle_features_in_area(const oracle_frame* f, float x, float y, float r,
                            int minLevel, int maxLevel, int* out, int cap);

/* ORBmatcher::SearchForInitialization (R/src/ORBmatcher.cpp:499-617).
 * prev_xy: 2*N1 floats (in/out, vbPrevMatched); matches12: N1 ints (out). Returns nmatches. */
int oracle_search_for_initialization(const oracle_frame* f1, const oracle_frame* f2,
                                     float nnratio, int check_ori, float* prev_xy,
                                     int* matches12, int window);

/* ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th, bMono)
 * (R/src/ORBmatcher.cpp:1564-1718).  Last-frame map points are given per last
 * keypoint (last_has_mp, world xyz, 32-B descriptor); Tcw poses are row-major
 * 3x4 float.  cur_mp (in/out, cur->n ints): -1 = empty slot, -2 = pre-occupied
 * by a map point with observations, >=0 = index of the last-frame keypoint whose
 * map point this call assigned.  Returns nmatches. */
typedef struct {
    float fx, fy, cx, cy, mbf, mb;
} oracle_camera;
int oracle_search_by_projection_ff(const oracle_frame* cur, const float* Tcw_cur,
                                   const oracle_frame* last, const float* Tcw_last,
                                   const int32_t* last_has_mp, const uint8_t* last_outlier,
                                   const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                   const float* scale_factors, const oracle_camera* cam,
                                   float th, int bMono, int check_ori, int32_t* cur_mp);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, th)
 * (R/src/ORBmatcher.cpp:63-163) with RadiusByViewingCos (:166-172).  Map points are given
 * in vector order: in_view = mbTrackInView && !isBad(); proj = (mTrackProjX, mTrackProjY,
 * mTrackProjXR); level = mnTrackScaleLevel; view_cos = mTrackViewCos; desc = GetDescriptor();
 * has_obs = Observations() > 0.  cur_mp (in/out, F.N ints) holds the slots mvpMapPoints:
 * -1 empty, -2 occupied by a map point with observations (skipped), -3 occupied by one
 * without (not skipped, may be overwritten); on return a slot matched by this call holds the
 * map point's index.  Returns nmatches. */
int oracle_search_by_projection_local(const oracle_frame* f, int n_mp, const uint8_t* in_view,
                                      const float* proj, const int32_t* level, const float* view_cos,
                                      const uint8_t* mp_desc, const uint8_t* has_obs,
                                      const float* scale_factors, float nnratio, float th, int32_t* cur_mp);

/* Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770): row-band candidates, best Hamming
 * distance below (TH_HIGH+TH_LOW)/2, 11x11 SAD over +-5 px on the keypoint's pyramid level,
 * parabola sub-pixel fit, disparity gate and the 2.1 x median SAD cut.  pyr_l / pyr_r:
 * nlevels level images (row stride = level width) of the left / right extractors'
 * mvImagePyramid; lw / lh: level sizes.  scale / inv_scale: mvScaleFactors /
 * mvInvScaleFactors.  mb is the baseline as seen by the call — 0 in the reference, whose
 * constructor sets mb only afterwards, giving maxD = mbf/0 = +inf.  Writes
 * uright / depth (N_left floats, -1 = none); returns the number of stereo matches kept. */
int oracle_compute_stereo_matches(const uint8_t* const* pyr_l, const uint8_t* const* pyr_r, const int* lw,
                                  const int* lh, const float* scale, const float* inv_scale,
                                  const oracle_keypoint* kl, const uint8_t* dl, int nl,
                                  const oracle_keypoint* kr, const uint8_t* dr, int nr,
                                  float mbf, float mb, float* uright, float* depth);

/* Brute-force Hamming k=2 (best, second) with lowest-index tie break. */
void oracle_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt,
                         int32_t* best_idx, int32_t* best_d, int32_t* second_d);

/* MapPoint::ComputeDistinctiveDescriptors on one point's N observed descriptors: the index of
 * the descriptor with the least median distance (-1 for N = 0). */
int oracle_distinctive_descriptor(const uint8_t* desc, int N);

/* Keyframe geometry Fuse reads: rows 0..2 of GetPose(), GetCameraCenter(), intrinsics, mbf,
 * mfLogScaleFactor, mnScaleLevels, mvScaleFactors, mvInvLevelSigma2. */
typedef struct {
    float Tcw[12];
    float Ow[3];
    float fx, fy, cx, cy, bf;
    float log_scale_factor;
    int n_levels;
    const float* scale_factors;
    const float* inv_level_sigma2;
} oracle_kf_params;

/* ORBmatcher::Fuse(pKF, vpMapPoints, th) matching step per map point: best_idx[i] = the keyframe
 * keypoint it fuses into (-1: none within TH_LOW), best_dist[i] = its distance (256: none). */
void oracle_fuse(const oracle_frame* kf, const oracle_kf_params* kp, int n_mp, const uint8_t* mp_valid,
                 const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                 const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist);

/* ORBmatcher::SearchForTriangulation (R/src/ORBmatcher.cpp:785-983): FeatureVectors as ascending
 * node ids + CSR feature lists; F12 row-major; (ex, ey) the epipole; returns nmatches. */
int oracle_search_for_triangulation(const oracle_frame* k1, const oracle_frame* k2, const uint8_t* has_mp1,
                                    const uint8_t* has_mp2, int n1, const uint32_t* nodes1, const int32_t* start1,
                                    const int32_t* idx1, int n2, const uint32_t* nodes2, const int32_t* start2,
                                    const int32_t* idx2, const float* F12, float ex, float ey,
                                    const float* scale_factors2, const float* level_sigma2, int only_stereo,
                                    int check_ori, int32_t* matches12);

/* DBoW2 vocabulary (TemplatedVocabulary<FORB::TDescriptor, FORB>) flattened: node 0 = root;
 * children of node i = child_idx[child_start[i] .. child_start[i+1]) in m_nodes[i].children
 * order; word_id / weight per node (leaves). */
typedef struct {
    int n_nodes;
    int L;
    const uint8_t* desc;
    const int32_t* child_start;
    const int32_t* child_idx;
    const int32_t* word_id;
    const double* weight;
} oracle_vocabulary;

/* TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup)
 * (D/DBoW2/TemplatedVocabulary.h:1242-1283) for n descriptors. */
void oracle_vocab_transform(const oracle_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* word_id,
                            double* weight, int32_t* node_id);

/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup) for the TF_IDF /
 * L1 configuration ORB-SLAM2 loads (ORBvoc.txt header "10 6 0 0"; :1151-1190, BowVector.cpp
 * addWeight / normalize(L1), FeatureVector.cpp addFeature).  Outputs in std::map order:
 * bow_words / bow_values (n_words), fv_nodes (n_fv) with fv_start[n_fv + 1] into fv_idx.
 * Each output array holds at most n entries.  Returns n_words; *n_fv receives the node count. */
int oracle_bow_transform(const oracle_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_words,
                         double* bow_values, int32_t* fv_nodes, int32_t* fv_start, int32_t* fv_idx, int* n_fv);

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (R/src/ORBmatcher.cpp:220-372):
 * kf_ok[i] = the keyframe's map point i is set and not bad; matches_f[j] = keyframe feature
 * matched to frame feature j or -1.  Returns nmatches. */
int oracle_search_by_bow_frame(const oracle_frame* kf, const uint8_t* kf_ok, int n1, const uint32_t* nodes1,
                               const int32_t* start1, const int32_t* idx1, const oracle_frame* f, int n2,
                               const uint32_t* nodes2, const int32_t* start2, const int32_t* idx2, float nnratio,
                               int check_ori, int32_t* matches_f);

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (R/src/ORBmatcher.cpp:632-760):
 * matches12[i] = keyframe-2 feature matched to keyframe-1 feature i or -1.  Returns nmatches. */
int oracle_search_by_bow_kf(const oracle_frame* k1, const uint8_t* ok1, int n1, const uint32_t* nodes1,
                            const int32_t* start1, const int32_t* idx1, const oracle_frame* k2, const uint8_t* ok2,
                            int n2, const uint32_t* nodes2, const int32_t* start2, const int32_t* idx2, float nnratio,
                            int check_ori, int32_t* matches12);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, float th, int ORBdist) (R/src/ORBmatcher.cpp:1719-1800, Tracking::Relocalization):
 * per keyframe map point i (mp_valid = set, not bad, not already found): projection with
 * Tcw (3x4), Ow = the frame's camera centre, mp_min/max_dist = mfMinDistance / mfMaxDistance,
 * PredictScale on the frame (log_scale_factor, n_levels), window levels level-1 .. level+1.
 * cur_mp as for oracle_search_by_projection_ff (new matches hold i).  Returns nmatches. */
int oracle_search_by_projection_kf(const oracle_frame* cur, const float* Tcw, const float* Ow, const oracle_frame* kf,
                                   const uint8_t* mp_valid, const float* mp_xyz, const float* mp_min_dist,
                                   const float* mp_max_dist, const uint8_t* mp_desc, const float* cam4,
                                   float log_scale_factor, int n_levels, const float* scale_factors, float th,
                                   int orb_dist, int check_ori, int32_t* cur_mp);

/* ORBmatcher::SearchByProjection(KeyFrame*, cv::Mat Scw, vpPoints, vpMatched, th)
 * (R/src/ORBmatcher.cpp:370-497): kp as for oracle_fuse (Tcw with the scale removed, Ow);
 * matched (in/out): -1 empty, other negatives pre-set, >= 0 the point index assigned.  Returns
 * nmatches. */
int oracle_search_by_projection_sim3(const oracle_frame* kf, const oracle_kf_params* kp, int n_mp,
                                     const uint8_t* mp_valid, const float* mp_xyz, const float* mp_normal,
                                     const float* mp_min_dist, const float* mp_max_dist, const uint8_t* mp_desc,
                                     float th, int32_t* matched);

/* ORBmatcher::Fuse(KeyFrame*, cv::Mat Scw, vpPoints, th, vpReplacePoint) matching step
 * (R/src/ORBmatcher.cpp:1164-1261): as oracle_fuse without the reprojection-error gate. */
void oracle_fuse_sim3(const oracle_frame* kf, const oracle_kf_params* kp, int n_mp, const uint8_t* mp_valid,
                      const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                      const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist);

/* One keyframe's side of ORBmatcher::SearchBySim3 (see orb_sim3_points in the C-ABI). */
typedef struct {
    float Tcw[12];
    float S[12];
    int n;
    const uint8_t* valid;
    const float* xyz;
    const float* min_dist;
    const float* max_dist;
    const uint8_t* desc;
} oracle_sim3_points;

/* ORBmatcher::SearchBySim3 (R/src/ORBmatcher.cpp:1305-1503) for the map points of this call
 * (valid = set, not bad, not already matched): matches12[i1] = idx2 of the mutual pairs or -1.
 * cam1 = pKF1's fx, fy, cx, cy; lsf / nlev / sf per keyframe.  Returns nFound. */
int oracle_search_by_sim3(const oracle_frame* kf1, const oracle_frame* kf2, const oracle_sim3_points* p1,
                          const oracle_sim3_points* p2, const float* cam1, float lsf1, int nlev1, const float* sf1,
                          float lsf2, int nlev2, const float* sf2, float th, int32_t* matches12);

#ifdef __cplusplus
}
#endif
#endif
