/*
 * orbslam2_amd.h — C-ABI of the MI355X-native ORB-SLAM2 hot path.
 *
 * Drop-in boundary for the reference's ORBextractor / ORBmatcher /
 * Optimizer::LocalBundleAdjustment class surfaces (reference:
 * YHY138/ORB-SLAM2-, abbreviated R/ = ORB-SLAM2注释版/).  Plain pointers and
 * sizes only; no C++ exceptions cross this boundary.  Every entry point
 * returns 0 (or a non-negative count) on success and a negative ORB_E* code on
 * failure.  The library is hand-written HIP for gfx950 (liborbslam2_amd.so);
 * there is no CPU fallback: without a usable GPU every compute entry point
 * returns ORB_ENODEV.
 *
 * Threading: a handle is not re-entrant; each handle owns one HIP stream, so two
 * handles may be driven concurrently from two host threads (the stereo L/R
 * extraction of R/src/Frame.cpp:86-89).  Matcher and BA calls take an explicit
 * context handle for the same reason.
 */
#ifndef ORBSLAM2_AMD_H
#define ORBSLAM2_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ----------------------------------------------------------------- errors */
#define ORB_OK 0
#define ORB_EINVAL (-22)   /* bad argument */
#define ORB_E2BIG (-7)     /* output capacity too small; *n_out holds the required count */
#define ORB_ENOMEM (-12)   /* device or pinned allocation failed */
#define ORB_ENODEV (-19)   /* no usable gfx950 device */
#define ORB_EGPU (-5)      /* a HIP call or kernel failed */
#define ORB_EOVERFLOW (-75) /* an internal fixed-capacity table overflowed */
#define ORB_EINTERNAL (-131) /* an internal consistency check failed (a library bug; the call did nothing useful) */
/* No C++ exception crosses this ABI: every entry point is a function-try-block, std::bad_alloc
 * returns ORB_ENOMEM and any other exception ORB_EINTERNAL (the void destroy / conversion
 * functions swallow them). */

/* cv::KeyPoint memory layout (pt.x, pt.y, size, angle, response, octave, class_id). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orb_keypoint;

/* ------------------------------------------------------------- extractor */

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST)  —  R/include/ORBextractor.h:51-52, R/src/ORBextractor.cpp:418. */
typedef struct {
    int nfeatures;
    float scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
} orb_extractor_params;

typedef struct orb_extractor orb_extractor;

/* Creates a handle on HIP device `device` able to process up to max_batch
 * frames of at most max_w x max_h pixels per call. */
int orb_extractor_create(const orb_extractor_params* params, int device, int max_w, int max_h,
                         int max_batch, orb_extractor** out);
void orb_extractor_destroy(orb_extractor* ex);

/* Inline getters of R/include/ORBextractor.h:66-86 (arrays of nlevels floats). */
int orb_extractor_levels(const orb_extractor* ex);
int orb_extractor_scale_tables(const orb_extractor* ex, float* scale, float* inv_scale,
                               float* sigma2, float* inv_sigma2);
int orb_extractor_features_per_level(const orb_extractor* ex, int* per_level);

/* ORBextractor::operator()(image, mask(ignored), keypoints, descriptors) —
 * R/src/ORBextractor.cpp:1120-1188.  Host 8-bit grey image in, host keypoints
 * (level-0 coordinates, levels concatenated 0..nlevels-1) and N x 32-byte
 * descriptors out.  Synchronous.  Empty image (w==0 || h==0 || img==NULL):
 * returns 0 and leaves every output, including *n_out, untouched (R :1123-1124).
 * If N > capacity: returns ORB_E2BIG, *n_out = N, outputs unspecified. */
int orb_extract(orb_extractor* ex, const uint8_t* img, int w, int h, size_t stride,
                orb_keypoint* kps, uint8_t* desc, int capacity, int* n_out);

/* Batched, device-resident form (the throughput path): d_imgs holds B frames of
 * w x h bytes (frame b at d_imgs + b*img_stride_frame, row stride w) in device
 * memory.  Results stay on the device: frame b's keypoints at d_kps + b*cap,
 * descriptors at d_desc + b*cap*32, count at d_counts[b] (may exceed cap; then
 * only the first cap are written).  Asynchronous on `stream` (hipStream_t; NULL =
 * the handle's own stream).  Returns 0 when the work was enqueued.
 *
 * LEVEL-0 LIFETIME.  As R/src/ORBextractor.cpp:1223 rebinds mvImagePyramid[0] to the input
 * image instead of copying it, level 0 of this call IS d_imgs whenever its rows are
 * dword-aligned (w, img_stride_frame and d_imgs multiples of 4): the extraction reads it in
 * place, and so do the later readers of this handle's last extraction — orb_pyramid_level
 * (level 0), orb_pyramid_level_device (raw level 0 is returned as a pointer into d_imgs, and
 * the on-demand blurred pyramid is computed from it) and orb_compute_stereo_matches(_batch_device).
 * d_imgs must therefore stay allocated and unchanged until the last of those reads has
 * completed on its stream (or the next extraction of the handle is enqueued).  A caller that
 * refills or frees d_imgs earlier (e.g. uploads the next batch into the same buffer) calls
 * orb_extractor_set_level0_copy(ex, 1) first: level 0 is then copied into the handle's own
 * pyramid slab and d_imgs is free once this call's work has run.  Unaligned frames are
 * always copied. */
int orb_extract_batch_device(orb_extractor* ex, const uint8_t* d_imgs, size_t img_stride_frame,
                             int B, int w, int h, orb_keypoint* d_kps, uint8_t* d_desc, int cap,
                             int32_t* d_counts, void* stream);

/* Compacts per-frame device rows stored at a capacity stride into one contiguous run, so a
 * host consumer downloads exactly the rows the batch produced (Tracking builds each Frame's
 * mvKeys / mDescriptors / the initializer's vnMatches12 from them, R/src/Frame.cpp:262-268,
 * R/src/Tracking.cpp:780): frame b's min(d_counts[b], cap) rows of row_bytes (a multiple of 4)
 * at d_src + b*cap*row_bytes go to d_dst + d_offsets[b]*row_bytes; d_offsets[0..B] receives the
 * exclusive prefix and the total.  Keypoints (28 B), descriptors (32 B) and matches12 (4 B rows,
 * d_counts = the first frames' counts) alike.  Asynchronous on `stream`. */
int orb_pack_rows_device(const void* d_src, int row_bytes, int cap, const int32_t* d_counts, int B, void* d_dst,
                         int32_t* d_offsets, void* stream);

/* copy = 1: every later extraction of `ex` copies level 0 into the handle's pyramid slab, so
 * no later call reads the caller's frames (see LEVEL-0 LIFETIME above; one extra read + write
 * of the frame per extraction).  copy = 0 (default): level 0 is read in place when aligned. */
int orb_extractor_set_level0_copy(orb_extractor* ex, int copy);

/* Status of the handle's last extraction (orb_extract or orb_extract_batch_device), after waiting
 * for the stream it ran on: *status = 0 when every internal table held, else a bit set —
 * 1 a FAST cell window wider than the kernel's limit, 2 a cell's keypoint list truncated,
 * 4 the octree iteration bound hit, 8 an octree node table full during a split phase,
 * 16 a level's node list truncated.  Returns ORB_EOVERFLOW when *status != 0 (then some
 * frame's keypoints of that batch may be incomplete), 0 otherwise. */
int orb_extractor_batch_status(orb_extractor* ex, int32_t* status);

/* Public `std::vector<cv::Mat> mvImagePyramid` (R/include/ORBextractor.h:88),
 * read by Frame::ComputeStereoMatches (R/src/Frame.cpp:558,675,689,695): returns a
 * host pointer to level `level` of frame `frame` of the last extraction
 * (downloaded lazily, valid until the next extraction).  After orb_extract_batch_device,
 * level 0 is downloaded from the caller's d_imgs unless level-0 copy is on (LEVEL-0 LIFETIME). */
int orb_pyramid_level(orb_extractor* ex, int frame, int level, const uint8_t** host, int* w,
                      int* h, size_t* stride);

/* Device pointer of the blurred or raw level (for on-device consumers).  The
 * blurred pyramid is computed on the first such request after an extraction
 * (the extraction itself evaluates the Gaussian only where descriptors sample).
 * Raw level 0 after orb_extract_batch_device points into the caller's d_imgs, and the
 * blurred pyramid's level 0 is computed from it, unless level-0 copy is on (LEVEL-0 LIFETIME). */
int orb_pyramid_level_device(orb_extractor* ex, int frame, int level, int blurred,
                             const uint8_t** dptr, int* w, int* h, size_t* pitch);

/* Stage profiling: while enabled, every extraction records HIP events on its
 * launch stream around the six kernel stages (0 resize, 1 FAST detection per
 * cell incl. NMS and the minThFAST retry, 2 reserved (always 0), 3 octree,
 * 4 reserved (always 0), 5 orientation + Gaussian + descriptor).  orb_extractor_stage_times
 * waits for them, writes the summed milliseconds per stage to ms[0..n_stages)
 * and the number of profiled calls to *n_calls, then resets; returns the number
 * of stages.  enable = 2 records only the two events bracketing stage 1
 * (k_fast_cell), so a timed run pays two event records per call; the other
 * stages then read 0.  enable = 3 records the four kernels' boundaries only (five events per
 * call: k_pyramid, k_fast_cell, k_octree, k_orient_desc in stages 0, 1, 3, 5). */
int orb_extractor_profile(orb_extractor* ex, int enable);
int orb_extractor_stage_times(orb_extractor* ex, double* ms, int n_stages, int* n_calls);

/* Level geometry for a w x h input (level sizes, FAST cells per level) and the
 * per-frame keypoint capacity the device batch path needs (cap >= this value
 * never truncates). */
int orb_extractor_geometry(orb_extractor* ex, int w, int h, int* level_w, int* level_h,
                           int* cells_per_level, int* max_keypoints_per_frame);

/* Per-level FAST keypoint counts before DistributeOctTree and retained counts
 * after it, for frame `frame` of the last extraction (diagnostics / roofline). */
int orb_extractor_last_counts(orb_extractor* ex, int frame, int* pre_counts, int* level_counts);

/* Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770) on the device, reading the two
 * extractors' pyramids in place (no mvImagePyramid download).  `left` / `right` hold the
 * extraction of the left / right image (frame 0 of their last call, same geometry); the
 * keypoints / descriptors are those extractions' outputs (mvKeys / mvKeysRight, host).
 * mbf = baseline x fx; mb = the baseline as the call sees it — the reference passes 0
 * (its constructor sets mb afterwards), so maxD = mbf/mb = +inf.  Writes
 * mvuRight / mvDepth (n_l floats, -1 = none); returns the number of stereo matches. */
int orb_compute_stereo_matches(orb_extractor* left, orb_extractor* right, const orb_keypoint* kps_l,
                               const uint8_t* desc_l, int n_l, const orb_keypoint* kps_r, const uint8_t* desc_r,
                               int n_r, float mbf, float mb, float* uright, float* depth);

/* Batched device form for stereo streams: the last orb_extract_batch_device call of `ex`
 * held frames 2p (left) and 2p+1 (right) of n_pairs stereo pairs, with outputs d_kps /
 * d_desc / d_counts as that call wrote them (cap keypoints per frame).  Writes
 * d_uright / d_depth ([n_pairs][cap]) and d_nstereo[p].  Asynchronous on `stream`.
 * The SAD search reads level 0 of both images: the extraction's d_imgs must still hold
 * those frames when this runs, unless level-0 copy is on (LEVEL-0 LIFETIME). */
int orb_compute_stereo_matches_batch_device(orb_extractor* ex, const orb_keypoint* d_kps, const uint8_t* d_desc,
                                            const int32_t* d_counts, int cap, int n_pairs, float mbf, float mb,
                                            float* d_uright, float* d_depth, int32_t* d_nstereo, void* stream);

/* --------------------------------------------------------------- matcher */

typedef struct orb_matcher orb_matcher;

/* ORBmatcher(float nnratio=0.6, bool checkOri=true) — R/src/ORBmatcher.cpp:46. */
int orb_matcher_create(int device, float nnratio, int check_ori, orb_matcher** out);
void orb_matcher_destroy(orb_matcher* m);

/* Host view of a Frame as the matcher reads it: mvKeysUn (x, y, angle,
 * octave), mDescriptors (n x 32), mvuRight (NULL = monocular, all -1) and the
 * static grid bounds mnMinX/mnMinY/mnMaxX/mnMaxY, mfGridElementWidthInv /
 * HeightInv (R/include/Frame.h:175-206). */
typedef struct {
    int n;
    const float* x;
    const float* y;
    const float* angle;
    const int32_t* octave;
    const uint8_t* desc;
    const float* uright;
    float min_x, min_y, max_x, max_y;
    float grid_w_inv, grid_h_inv;
} orb_frame_view;

/* ORBmatcher::DescriptorDistance — R/src/ORBmatcher.cpp:1901-1917 (host inline helper). */
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Keyframe geometry read by ORBmatcher::Fuse: rows 0..2 of GetPose(), GetCameraCenter(), fx, fy,
 * cx, cy, mbf, mfLogScaleFactor, mnScaleLevels, mvScaleFactors, mvInvLevelSigma2. */
typedef struct {
    float Tcw[12];
    float Ow[3];
    float fx, fy, cx, cy, bf;
    float log_scale_factor;
    int n_levels;
    const float* scale_factors;
    const float* inv_level_sigma2;
} orb_kf_params;

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th) — the matching
 * step of R/src/ORBmatcher.cpp:995-1121 for every map point of the vector:
 *   kf = the keyframe as a frame view (mvKeysUn, mDescriptors, mvuRight, grid bounds);
 *   mp_valid[i] = pMP && !pMP->isBad() && !pMP->IsInKeyFrame(pKF); mp_xyz / mp_normal =
 *   GetWorldPos / GetNormal; mp_min_dist / mp_max_dist = mfMinDistance / mfMaxDistance;
 *   mp_desc = GetDescriptor().
 * best_idx[i] = the keyframe keypoint the point fuses into (-1: none within TH_LOW) and
 * best_dist[i] its distance (256: no candidate).  The replace / add resolution (:1123-1150)
 * mutates the map and stays with the caller, in vector order.  Host buffers. */
int orb_fuse(int device, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp, const uint8_t* mp_valid,
             const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
             const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist);

/* ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, float th,
 * vector<MapPoint*>& vpReplacePoint) — the matching step of R/src/ORBmatcher.cpp:1164-1290
 * (LoopClosing::SearchAndFuse): kp->Tcw / Ow = [Rcw | tcw] with the Sim3 scale removed and
 * -Rcw^T tcw as the reference derives them from Scw (bf, inv_level_sigma2 unused); mp_valid[i] =
 * !isBad() && the point is not among pKF->GetMapPoints().  No reprojection-error gate.  best_idx /
 * best_dist as for orb_fuse; the replace / add step (:1263-1283) stays with the caller, in vector
 * order.  Host buffers. */
int orb_fuse_sim3(int device, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp, const uint8_t* mp_valid,
                  const float* mp_xyz, const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                  const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist);

/* One keyframe's side of ORBmatcher::SearchBySim3: Tcw = [R|t] world -> this camera
 * (GetRotation / GetTranslation); S = [sR|t] this camera -> the other camera (keyframe 1: sR21 =
 * (1/s12) R12^T, t21 = -sR21 t12; keyframe 2: sR12 = s12 R12, t12 — as the reference computes them);
 * per keypoint i (n = the keyframe's N): valid[i] != 0 when GetMapPointMatches()[i] is set, not bad
 * and not already matched (vbAlreadyMatched1 / 2); xyz, min_dist / max_dist (mfMinDistance /
 * mfMaxDistance) and desc of that map point. */
typedef struct {
    float Tcw[12];
    float S[12];
    int n;
    const uint8_t* valid;
    const float* xyz;
    const float* min_dist;
    const float* max_dist;
    const uint8_t* desc;
} orb_sim3_points;
/* mfLogScaleFactor, mnScaleLevels, mvScaleFactors of a keyframe. */
typedef struct {
    float log_scale_factor;
    int n_levels;
    const float* scale_factors;
} orb_scale_params;

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) — R/src/ORBmatcher.cpp:
 * 1305-1503 (LoopClosing::ComputeSim3): both projection directions on the GPU (pKF1's fx, fy, cx,
 * cy = cam1 for both, as the reference), the mutual check on the host.  matches12 (kf1->n ints)
 * receives the keyframe-2 index whose map point becomes vpMatches12[i1] (pairs found by this call
 * only), or -1.  Returns nFound.  Host buffers. */
int orb_search_by_sim3(int device, const orb_frame_view* kf1, const orb_frame_view* kf2, const orb_sim3_points* p1,
                       const orb_sim3_points* p2, const float cam1[4], const orb_scale_params* sc1,
                       const orb_scale_params* sc2, float th, int32_t* matches12);

/* ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) —
 * R/src/ORBmatcher.cpp:785-983 (LocalMapping::CreateNewMapPoints, R/src/LocalMapping.cpp:374).
 *   kf1 / kf2: the keyframes as frame views (mvKeysUn incl. angle and octave, mDescriptors,
 *   mvuRight); has_mp1/2[i] != 0 when GetMapPoint(i) is set;
 *   mFeatVec of each keyframe: n_nodes ascending node ids, CSR start[n_nodes + 1] into the
 *   feature-index lists (DBoW2 insertion order);
 *   F12 = LocalMapping::ComputeF12 (row-major 3x3 float); (ex, ey) = KF1's camera centre
 *   projected into KF2 (:799-803); scale_factors2 / level_sigma2 = pKF2->mvScaleFactors /
 *   mvLevelSigma2 (n_levels2 entries); check_ori = mbCheckOrientation.
 * matches12 (kf1->n ints) receives the KF2 keypoint or -1; vMatchedPairs are its (i, j) pairs in
 * i order.  Returns nmatches; ORB_E2BIG when a node holds more than 2048 KF2 features. */
int orb_search_for_triangulation(int device, const orb_frame_view* kf1, const orb_frame_view* kf2,
                                 const uint8_t* has_mp1, const uint8_t* has_mp2, int n_nodes1, const uint32_t* nodes1,
                                 const int32_t* start1, const int32_t* fidx1, int n_nodes2, const uint32_t* nodes2,
                                 const int32_t* start2, const int32_t* fidx2, const float F12[9], float ex, float ey,
                                 const float* scale_factors2, const float* level_sigma2, int n_levels2, int only_stereo,
                                 int check_ori, int32_t* matches12);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) —
 * R/src/ORBmatcher.cpp:220-372 (Tracking::TrackReferenceKeyFrame, Relocalization).
 *   kf / f: the keyframe (mvKeysUn, mDescriptors) and the frame (mvKeys angles, mDescriptors)
 *   as frame views; kf_ok[i] != 0 when GetMapPointMatches()[i] is set and not bad;
 *   mFeatVec of each: n_nodes ascending node ids, CSR start[n_nodes + 1] into feature indices;
 *   nn_ratio = mfNNratio, check_ori = mbCheckOrientation.
 * matches_f (f->n ints) receives, per frame feature, the keyframe feature whose map point it
 * matched (vpMapPointMatches[j] = vpMapPointsKF[matches_f[j]]) or -1.  Returns nmatches;
 * ORB_E2BIG when a node holds more than 2048 frame features.  Host buffers. */
int orb_search_by_bow_frame(int device, const orb_frame_view* kf, const uint8_t* kf_ok, int n_nodes_kf,
                            const uint32_t* nodes_kf, const int32_t* start_kf, const int32_t* fidx_kf,
                            const orb_frame_view* f, int n_nodes_f, const uint32_t* nodes_f, const int32_t* start_f,
                            const int32_t* fidx_f, float nn_ratio, int check_ori, int32_t* matches_f);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12) —
 * R/src/ORBmatcher.cpp:632-760 (LoopClosing::ComputeSim3).  okN[i] != 0 when keyframe N's map
 * point i is set and not bad.  matches12 (kf1->n ints) receives the keyframe-2 feature whose map
 * point becomes vpMatches12[i], or -1.  Returns nmatches.  Host buffers. */
int orb_search_by_bow_kf(int device, const orb_frame_view* kf1, const uint8_t* ok1, int n_nodes1,
                         const uint32_t* nodes1, const int32_t* start1, const int32_t* fidx1,
                         const orb_frame_view* kf2, const uint8_t* ok2, int n_nodes2, const uint32_t* nodes2,
                         const int32_t* start2, const int32_t* fidx2, float nn_ratio, int check_ori,
                         int32_t* matches12);

/* MapPoint::ComputeDistinctiveDescriptors (R/src/MapPoint.cpp:306-385) for n_points map points:
 * point m's descriptors (one per observation by a non-bad keyframe, in mObservations order) are
 * rows [start[m], start[m+1]) of desc (32 B each).  best_idx[m] = index within the point's list
 * of the descriptor with the least median distance to the others (the new mDescriptor), -1 for
 * an empty list; best_desc (optional, [n_points][32]) receives that row.  Host buffers. */
int orb_distinctive_descriptors(int device, const uint8_t* desc, const int32_t* start, int n_points, int32_t* best_idx,
                                uint8_t* best_desc);
/* Device-resident form (asynchronous on `stream`); start is relative to d_desc. */
int orb_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_start, int n_points,
                                       int32_t* d_best_idx, uint8_t* d_best_desc, void* stream);

/* DBoW2 ORB vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>,
 * R/include/ORBVocabulary.h; D/DBoW2/TemplatedVocabulary.h m_nodes / m_L) flattened:
 *   node 0 is the root; desc[i] = m_nodes[i].descriptor (32 B, root's unused);
 *   children of node i = child_idx[child_start[i] .. child_start[i+1]) in m_nodes[i].children
 *   order (empty list: leaf); word_id[i] / weight[i] = m_nodes[i].word_id / weight (leaves). */
typedef struct {
    int n_nodes;
    int L;
    const uint8_t* desc;
    const int32_t* child_start;
    const int32_t* child_idx;
    const int32_t* word_id;
    const double* weight;
} orb_vocabulary;
typedef struct orb_vocab orb_vocab;

/* Uploads the vocabulary once (device-resident handle; the loader / TemplatedVocabulary
 * constructor stays on the host). */
int orb_vocabulary_create(int device, const orb_vocabulary* voc, orb_vocab** out);
void orb_vocabulary_destroy(orb_vocab* h);
/* TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup) —
 * D/DBoW2/TemplatedVocabulary.h:1242-1283 — for n descriptors ([n][32] B): the per-feature part
 * of transform(features, BowVector&, FeatureVector&, levelsup) (:1151-1190; ORB-SLAM2 calls it
 * with levelsup 4 from Frame::ComputeBoW / KeyFrame::ComputeBoW).  node_id = the node passed at
 * level L - levelsup (0 when that level is <= 0).  The BowVector (weights > 0 summed per word in
 * feature order, then L1-normalised) and FeatureVector (feature indices per node in feature
 * order) assembly stays with the caller.  Host buffers. */
int orb_vocabulary_transform(orb_vocab* h, const uint8_t* desc, int n, int levelsup, int32_t* word_id, double* weight,
                             int32_t* node_id);
/* Device-resident form (asynchronous on `stream`; NULL is the null stream). */
int orb_vocabulary_transform_device(orb_vocab* h, const uint8_t* d_desc, int n, int levelsup, int32_t* d_word_id,
                                    double* d_weight, int32_t* d_node_id, void* stream);

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12,
 * windowSize) — R/src/ORBmatcher.cpp:499-617.  prev_xy (2*F1.n floats) is
 * updated in place; matches12 (F1.n ints) receives the F2 index or -1.
 * Returns nmatches (>= 0) or an error. */
int orb_search_for_initialization(orb_matcher* m, const orb_frame_view* f1, const orb_frame_view* f2,
                                  float* prev_xy, int32_t* matches12, int window);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
 * float th, bool bMono) — R/src/ORBmatcher.cpp:1564-1718.
 *   Tcw_cur / Tcw_last: row-major 3x4 float poses (mTcw rows 0..2).
 *   last_has_mp[i]: 0 when LastFrame.mvpMapPoints[i] is NULL, 1 when it is set to a map point
 *   with observations, 2 when set to one with Observations() == 0 (the temporal points
 *   Tracking::UpdateLastFrame creates for stereo / RGB-D, R/src/Tracking.cpp:1132-1137, with
 *   nObs(0), R/src/MapPoint.cpp:65: a current slot given such a point stays open to later
 *   last-frame points, R :1649-1651);
 *   last_outlier[i] = mvbOutlier[i]; last_mp_xyz (3 floats) / last_mp_desc (32 B) per last
 *   keypoint (GetWorldPos / GetDescriptor).  scale_factors = CurrentFrame.mvScaleFactors.
 *   cam = {fx, fy, cx, cy, mbf, mb}.
 *   cur_mp (in/out, cur.n ints) is CurrentFrame.mvpMapPoints: -1 empty slot, -2 occupied by a
 *   map point with observations (skipped), -3 occupied by one without (a candidate; returned as
 *   -3 when untouched); on return >= 0 = the last-frame keypoint index whose map point this call
 *   assigned, -1 = empty (including a slot the rotation check cleared).
 * Returns nmatches. */
int orb_search_by_projection_frame(orb_matcher* m, const orb_frame_view* cur, const float* Tcw_cur,
                                   const orb_frame_view* last, const float* Tcw_last,
                                   const int32_t* last_has_mp, const uint8_t* last_outlier,
                                   const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                   const float* scale_factors, const float cam[6], float th,
                                   int mono, int32_t* cur_mp);

/* ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
 * vector<MapPoint*>& vpMatched, int th) — R/src/ORBmatcher.cpp:370-497 (LoopClosing::ComputeSim3).
 *   kf: the keyframe as a frame view (mvKeysUn, mDescriptors, bounds, grid); kp: Tcw = rows of
 *   [Rcw | tcw] with the scale removed and Ow = -Rcw^T tcw as the reference computes them from Scw,
 *   fx .. cy, mfLogScaleFactor, mnScaleLevels, mvScaleFactors (bf, inv_level_sigma2 unused);
 *   mp_valid[i] != 0 when vpPoints[i] is not bad and not already in vpMatched; mp_* as for orb_fuse.
 * matched (in/out, kf->n ints): -1 = vpMatched[idx] empty, any other negative value = set before the
 * call, >= 0 on return = the vpPoints index assigned.  Returns nmatches. */
int orb_search_by_projection_sim3(orb_matcher* m, const orb_frame_view* kf, const orb_kf_params* kp, int n_mp,
                                  const uint8_t* mp_valid, const float* mp_xyz, const float* mp_normal,
                                  const float* mp_min_dist, const float* mp_max_dist, const uint8_t* mp_desc, float th,
                                  int32_t* matched);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, float th, int ORBdist) — R/src/ORBmatcher.cpp:1719-1800 (Tracking::Relocalization).
 *   cur: the frame (mvKeysUn, mDescriptors, bounds, grid); Tcw_cur: rows 0..2 of mTcw; Ow: its
 *   camera centre -Rcw^T tcw as the reference computes it; cam = fx, fy, cx, cy;
 *   kf: the keyframe as a frame view (mvKeysUn angles; kf->n = its N);
 *   mp_valid[i] != 0 when GetMapPointMatches()[i] is set, not bad and not in sAlreadyFound;
 *   mp_xyz / mp_min_dist / mp_max_dist / mp_desc = GetWorldPos, mfMinDistance, mfMaxDistance,
 *   GetDescriptor; log_scale_factor / n_levels / scale_factors = the frame's mfLogScaleFactor,
 *   mnScaleLevels, mvScaleFactors.
 * cur_mp (in/out, cur->n ints): -1 = mvpMapPoints[i2] empty, any other negative value = set
 * before the call, >= 0 on return = the keyframe map point index this call assigned.
 * Returns nmatches (after the rotation filter when the matcher checks orientation).
 * Deviation: with orb_dist >= 256 a map point whose window candidates are all occupied passes
 * the reference's `bestDist <= ORBdist` with bestIdx2 = -1 and the reference then writes
 * CurrentFrame.mvpMapPoints[-1] and counts a match (R/src/ORBmatcher.cpp:1806-1808, out of
 * bounds).  Here such a point is skipped: nothing is written and it is not counted.  The
 * reference's call sites pass 100 and 64 (R/src/Tracking.cpp:1921, 1936), where this cannot
 * happen. */
int orb_search_by_projection_kf(orb_matcher* m, const orb_frame_view* cur, const float* Tcw_cur, const float Ow[3],
                                const orb_frame_view* kf, const uint8_t* mp_valid, const float* mp_xyz,
                                const float* mp_min_dist, const float* mp_max_dist, const uint8_t* mp_desc,
                                const float cam[4], float log_scale_factor, int n_levels, const float* scale_factors,
                                float th, int orb_dist, int32_t* cur_mp);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, float th)
 * — R/src/ORBmatcher.cpp:63-163 (Tracking::SearchLocalPoints, R/src/Tracking.cpp:1413-1460).
 * Map points in vector order (n_mp):
 *   mp_in_view[i]  = mbTrackInView && !isBad();
 *   mp_proj[3i..]  = mTrackProjX, mTrackProjY, mTrackProjXR (from Frame::isInFrustum);
 *   mp_level[i]    = mnTrackScaleLevel; mp_view_cos[i] = mTrackViewCos;
 *   mp_desc        = GetDescriptor() (32 B each); mp_has_obs[i] = Observations() > 0.
 * scale_factors = F.mvScaleFactors.  cur_mp (in/out, f->n ints) is F.mvpMapPoints:
 *   -1 empty, -2 holds a map point with observations (skipped), -3 holds one without
 *   (not skipped, may be overwritten); a slot matched by this call receives the map point's
 *   index i.  The matcher's nnratio applies (ratio test only within one scale level).
 * Returns nmatches. */
int orb_search_by_projection_local(orb_matcher* m, const orb_frame_view* f, int n_mp, const uint8_t* mp_in_view,
                                   const float* mp_proj, const int32_t* mp_level, const float* mp_view_cos,
                                   const uint8_t* mp_desc, const uint8_t* mp_has_obs, const float* scale_factors,
                                   float th, int32_t* cur_mp);

/* Brute-force 2-NN Hamming matching (all pairs; ties -> lowest train index):
 * for every query i, best_idx[i], best_d[i], second_d[i] (INT32_MAX when absent).
 * Host arrays in and out. */
int orb_hamming_knn2(orb_matcher* m, const uint8_t* q, int nq, const uint8_t* t, int nt,
                     int32_t* best_idx, int32_t* best_d, int32_t* second_d);

/* Device-resident batched 2-NN: nb independent (query, train) pairs
 * d_q + b*q_stride_rows*32, counts d_nq[b] / d_nt[b]; outputs at + b*q_stride_rows. */
int orb_hamming_knn2_batch_device(orb_matcher* m, const uint8_t* d_q, const int32_t* d_nq,
                                  const uint8_t* d_t, const int32_t* d_nt, int nb, int q_stride_rows,
                                  int t_stride_rows, int32_t* d_best_idx, int32_t* d_best_d,
                                  int32_t* d_second_d, void* stream);

/* Device-resident SearchForInitialization over nb frame pairs (frame pairs
 * (f1[b], f2[b]) laid out as keypoint/descriptor arrays of the device batch
 * extractor output, i.e. orb_keypoint rows).  prev_xy is initialised from f1's
 * own keypoints (the Tracking.cpp:779 first call) and the result matches12 is
 * written per pair.  Used by the throughput benchmark. */
int orb_search_for_initialization_batch_device(orb_matcher* m, const orb_keypoint* d_kps1,
                                               const uint8_t* d_desc1, const int32_t* d_n1,
                                               const orb_keypoint* d_kps2, const uint8_t* d_desc2,
                                               const int32_t* d_n2, int nb, int cap, int width,
                                               int height, int window, int32_t* d_matches12,
                                               int32_t* d_nmatches, void* stream);

/* Overflow bits of the batched SearchForInitialization calls since the last query (waits for the
 * stream of the last batch call, then clears them): 1 a query's candidate list (the
 * GetFeaturesInArea result, R/src/ORBmatcher.cpp:523) was longer than the kernel's 1024-entry
 * capacity and was truncated, 2 the resolution sweeps did not converge.  Returns ORB_EOVERFLOW
 * when *status != 0 (then some pair's matches12 may differ from the reference's), 0 otherwise. */
int orb_matcher_batch_status(orb_matcher* m, int32_t* status);

/* ------------------------------------------------------------ local BA */

/* The g2o graph Optimizer::LocalBundleAdjustment builds (R/src/Optimizer.cpp:629-782),
 * as plain arrays.  Poses are VertexSE3Expmap estimates (Eigen quaternion coeffs
 * x,y,z,w and translation, f64; lba_pose_from_Tcw converts a float Tcw the way
 * Converter::toSE3Quat does); pose_fixed is setFixed (mnId==0 or a fixed camera);
 * ids are the g2o vertex ids (KeyFrame::mnId, MapPoint::mnId+maxKFid+1), used only
 * for g2o's index ordering.  Edges: vertex 0 = point, vertex 1 = pose; stereo
 * edges carry (u, v, ur); information = I * invSigma2[octave] (float value);
 * cam = fx, fy, cx, cy, bf of the observing keyframe.  point_bad is the
 * MapPoint::isBad() snapshot the outlier passes test (NULL = none bad). */
typedef struct {
    int n_poses;
    const double* pose_q;
    const double* pose_t;
    const uint8_t* pose_fixed;
    const int64_t* pose_id;
    int n_points;
    const double* point_xyz;
    const int64_t* point_id;
    const uint8_t* point_bad;
    int n_edges;
    const int32_t* edge_point;
    const int32_t* edge_pose;
    const uint8_t* edge_stereo;
    const double* edge_obs;
    const double* edge_info;
    const double* edge_cam;
} lba_problem;

typedef struct {
    int iters1, iters2;              /* optimize(5), optimize(10) */
    double chi2_mono, chi2_stereo;   /* 5.991, 7.815 */
    double huber_mono, huber_stereo; /* (float)sqrt(5.991), (float)sqrt(7.815) */
    int max_trials;                  /* maxTrialsAfterFailure (10) */
    int fixed_iterations;            /* 1: ignore g2o's early termination (parity mode) */
} lba_options;

typedef struct {
    double* pose_q;       /* out [n_poses][4] */
    double* pose_t;       /* out [n_poses][3] */
    double* point_xyz;    /* out [n_points][3] */
    uint8_t* edge_erase;  /* out: the (KF, MapPoint) pairs of vToErase (R :850-880) */
    double* edge_chi2;    /* out: e->chi2() at the final check */
    int iterations[2];    /* outer iterations of each optimize() call */
    int trials;           /* LM trials in total */
    double* trace;        /* optional [64][4]: per outer iteration iniChi, chi2, lambda, trials */
    int n_trace;
    int aborted;          /* 1: *stop was set on entry, nothing optimised or written (R :784-786) */
} lba_result;

typedef struct lba_context lba_context;

/* All-reduce callback for multi-GPU local BA: reduces `count` doubles at
 * `offset_doubles` of the workspace registered with lba_set_comm across all
 * ranks (op 0 = sum, 1 = max), ordered after the work already enqueued on the
 * context's stream (lba_set_stream).  Return 0 on success. */
typedef int (*lba_allreduce_fn)(void* user, size_t offset_doubles, size_t count, int op);

int lba_create(int device, lba_context** out);
void lba_destroy(lba_context* c);
/* use_given = 1: run on `stream` (a hipStream_t; NULL = the legacy default stream), e.g.
 * the caller's torch stream so its all-reduces are ordered with the solver's work;
 * use_given = 0: a private non-blocking stream (the default). */
int lba_set_stream(lba_context* c, void* stream, int use_given);
/* Shards the landmarks over `world` ranks (rank r owns the contiguous index range
 * [r*M/world, (r+1)*M/world)); every rank passes the same full problem. */
int lba_set_comm(lba_context* c, int rank, int world, double* d_workspace, size_t ws_doubles,
                 lba_allreduce_fn fn, void* user);

/* Optimizer::LocalBundleAdjustment's optimisation (R/src/Optimizer.cpp:784-880):
 * optimize(5) with Huber kernels, chi2/depth outlier pass, optimize(10) on the
 * inliers without kernels, final chi2/depth check.  *stop (mbAbortBA) is read like
 * SparseOptimizer::terminate(): on entry, after every LM trial (the device's decision
 * kernel reads a host-mapped mirror of it, refreshed while the host waits) and between
 * the two optimize() calls; with a communicator the ranks' flags are summed so every rank
 * stops at the same point.  Every edge index must lie in [0, n_points) / [0, n_poses) and
 * every array of a non-empty set must be non-NULL (ORB_EINVAL otherwise).  The caller
 * applies the results under Map::mMutexMapUpdate exactly as R :883-917 do. */
int lba_solve(lba_context* c, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop,
              lba_result* r);

/* Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust) —
 * R/src/Optimizer.cpp:78-277 (global BA: Tracking initialisation with 20 iterations, LoopClosing's
 * RunGlobalBundleAdjustment with 10): one optimize(o->iters1) over every edge of the problem, Huber
 * kernels with deltas o->huber_mono / o->huber_stereo ((float)sqrt(5.99), (float)sqrt(7.815)) only
 * when robust; no outlier pass (edge_erase all 0).  Poses with pose_id 0 are the fixed ones the
 * caller marks; points without edges are left out (vbNotIncludedMP) and returned unchanged.  *stop
 * (setForceStopFlag) ends the iterations; the estimates are written back either way. */
int lba_solve_global(lba_context* c, const lba_problem* p, const lba_options* o, int robust,
                     const volatile uint8_t* stop, lba_result* r);

/* Stage timing of the LM loop (HIP events): ms4 = linearise, Schur, solve, update. */
/* The reduced camera system solver on its own (LinearSolverEigen::solve's role,
 * G/solvers/linear_solver_eigen.h:94-120): x = S^-1 b for a symmetric positive-definite
 * row-major n x n S by the blocked MFMA LDL^T lba_solve runs per LM trial (no pivoting).
 * Host buffers; synchronous on the context's stream.  Returns ORB_EINVAL when a pivot is
 * zero or non-finite (the factorisation failure g2o turns into chi2 = inf). */
int lba_dense_solve(lba_context* c, const double* S, const double* b, int n, double* x);
int lba_profile(lba_context* c, int enable);
/* Test hook for the stop semantics: the LM loop behaves as if *stop became set the moment the
 * solve's trial count reached n_trials (sampled where g2o calls terminate(): after every trial,
 * G/core/optimization_algorithm_levenberg.cpp:149, and before every iteration,
 * G/core/sparse_optimizer.cpp:376), so a stop point is reproducible; n_trials < 0 turns it off. */
int lba_debug_stop_after_trials(lba_context* c, int n_trials);
/* Diagnostics: copies n doubles of a device buffer of the last solve's final LM state (0 the reduced
 * matrix S, 1 b_s, 2 x, 3 Hpp blocks, 4 b_p, 5 Hll blocks, 6 b_l, 7 D^-1 blocks) to out; returns
 * the buffer's length in doubles. */
int lba_debug_buffer(lba_context* c, int which, double* out, size_t n);
int lba_stats(lba_context* c, double* ms4, int* iters, int* trials);

/* Multi-GPU Optimizer::LocalBundleAdjustment from ONE process — the drop-in's model: LocalMapping
 * calls it on its own thread (R/src/LocalMapping.cpp:94-95, R/src/System.cpp:104-105).  A group
 * holds one context per entry of devices[0..n) (n <= 16; a device may repeat: two contexts on one
 * device rehearse the exchange on a one-GPU machine).  lba_group_solve shards the landmarks as
 * lba_set_comm does (rank r owns [r M / n, (r+1) M / n)) and all-reduces the pose blocks, the
 * reduced camera system S + b_s and the LM scalars with the library's own exchange over xGMI
 * (every rank reads every rank's slice through peer access and sums in rank order: all ranks take
 * bitwise the same LM decisions); no caller callback.  With every rank on its own device the
 * exchange is device-side (flag words in fine-grained memory, no host in the loop, the LM slots
 * replayed from HIP graphs); ranks sharing a device are ordered from the host (cross-stream
 * events).  Same arguments and results as lba_solve (points, edge chi2 and erase flags merged from
 * their owners).  Returns ORB_ENODEV when two listed devices cannot access each other, ORB_EGPU
 * when a device-side wait timed out (a rank that never arrived). */
typedef struct lba_group lba_group;
int lba_group_create(const int* devices, int n, lba_group** out);
void lba_group_destroy(lba_group* g);
int lba_group_solve(lba_group* g, const lba_problem* p, const lba_options* o, const volatile uint8_t* stop,
                    lba_result* r);
/* The number of collectives since creation and, for the host-ordered exchange only, their
 * cumulative time on rank 0's stream (from its partial being ready to every rank having read it;
 * 0 with the device-side exchange, whose cost is in a kernel trace as k_grp_sync / k_grp_reduce). */
int lba_group_stats(lba_group* g, double* exchange_ms, long* n_exchanges);

/* Converter::toSE3Quat(const cv::Mat& Tcw) / Converter::toCvMat(const SE3Quat&)
 * (R/src/Converter.cpp:47-57, 59-63): row-major 4x4 float <-> quaternion + t. */
void lba_pose_from_Tcw(const float Tcw[16], double q[4], double t[3]);
/* ---------------------------------------------------------------- PoseOptimization
 * Optimizer::PoseOptimization(Frame*) (R/src/Optimizer.cpp:306-535, declared
 * R/include/Optimizer.h:44) over a batch of frames.  Frame b's edges are
 * [edge_start[b], edge_start[b+1]): one per keypoint with a map point, obs = (u, v, ur) with
 * ur < 0 for a monocular observation (Frame::mvuRight), xw = MapPoint::GetWorldPos (float
 * values), info = mvInvLevelSigma2[octave] (float value); cam = fx, fy, cx, cy, mbf; pose =
 * Converter::toSE3Quat(pFrame->mTcw).  Results: the optimised pose (pFrame->SetPose), the
 * per-edge outlier flags (Frame::mvbOutlier) and the return value nInitialCorrespondences -
 * nBad (0 and the pose untouched below 3 edges). */
typedef struct {
    int n_frames;
    int n_edges;
    const double* pose_q;       /* [B][4] x, y, z, w */
    const double* pose_t;       /* [B][3] */
    const double* cam;          /* [B][5] */
    const int32_t* edge_start;  /* [B + 1] */
    const double* edge_obs;     /* [E][3] */
    const double* edge_xw;      /* [E][3] */
    const double* edge_info;    /* [E] */
} pose_batch;

typedef struct {
    double* pose_q;      /* [B][4] */
    double* pose_t;      /* [B][3] */
    uint8_t* outlier;    /* [E] */
    int32_t* n_inliers;  /* [B] */
} pose_batch_result;

/* Host buffers, synchronous.  iters (optional, [B][5]): LM iterations of rounds 0-3, trials. */
int pose_optimize_batch(int device, const pose_batch* p, pose_batch_result* r, int32_t* iters);
/* Device-resident form, asynchronous on `stream`: every pointer of p and r in device memory;
 * d_work holds 3 * n_edges doubles and d_flags 2 * n_edges bytes of per-edge state; d_iters
 * ([B][5]) may be NULL. */
int pose_optimize_batch_device(const pose_batch* p, const pose_batch_result* r, double* d_work, uint8_t* d_flags,
                               int32_t* d_iters, void* stream);

/* lba_pose_from_Tcw over n row-major 4x4 float poses (q: n x 4, t: n x 3). */
void lba_poses_from_Tcw(const float* Tcw, int n, double* q, double* t);
void lba_pose_to_Tcw(const double q[4], const double t[3], float Tcw[16]);

#ifdef __cplusplus
}
#endif
#endif /* ORBSLAM2_AMD_H */
