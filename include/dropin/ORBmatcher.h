// Drop-in replacement for R/include/ORBmatcher.h: the same class declaration.  Defined here over
// liborbslam2_amd through include/orbslam2_amd_shim.hpp: the constructor (R/src/ORBmatcher.cpp:46-48),
// DescriptorDistance (:1901-1917), SearchForInitialization (:499-617), the two tracking forms of
// SearchByProjection (:63-163, :1564-1718), both SearchByBoW overloads (:220-372, :632-760),
// SearchForTriangulation (:785-983), both Fuse overloads (:995-1154, :1164-1290), the
// relocalisation and Sim3 forms of SearchByProjection (:1719-1800, :370-497) and SearchBySim3
// (:1305-1503) — every matcher the reference defines; R/src/ORBmatcher.cpp then keeps only
// TH_LOW / TH_HIGH / HISTO_LENGTH and the protected helpers.  The matchers read a point's raw
// mfMinDistance / mfMaxDistance through MapPoint::GetDistances (one accessor added
// to R/include/MapPoint.h).  Compiles inside the reference tree only (OpenCV, Frame.h); the shim
// is compiled and tested here with mock types (tests/test_cpp_shim*.py).
#ifndef ORBMATCHER_H
#define ORBMATCHER_H

#include <set>
#include <vector>
#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "orbslam2_amd_shim.hpp"

namespace ORB_SLAM2 {

class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri), mDev(nnratio, checkOri) {}

    // 256-bit Hamming distance of two 32-byte rows (R :1901-1917)
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
        return orbslam2_amd::Matcher::DescriptorDistance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
    }

    // tracking matchers on the GPU: the local map (R :63-163) and the motion model (R :1564-1718)
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3) {
        return mDev.SearchByProjection(F, vpMapPoints, th);
    }
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
        return mDev.SearchByProjection(CurrentFrame, LastFrame, th, bMono);
    }
    // relocalisation (R :1719-1800) and loop closing's Sim3 projection (R :370-497) on the GPU
    int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                           const float th, const int ORBdist) {
        return mDev.SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist);
    }
    int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                           std::vector<MapPoint*>& vpMatched, int th) {
        return mDev.SearchByProjection(pKF, Scw, vpPoints, vpMatched, th);
    }
    // BoW matchers on the GPU: tracking's reference keyframe / relocalisation (R :220-372) and
    // loop closing (R :632-760)
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
        return mDev.SearchByBoW(pKF, F, vpMapPointMatches);
    }
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
        return mDev.SearchByBoW(pKF1, pKF2, vpMatches12);
    }

    // monocular initialisation matching on the GPU (R :499-617): same outputs, same order
    int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) {
        return mDev.SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize);
    }

    // LocalMapping's matchers on the GPU: new map points (R :785-983) and fusion (R :995-1154)
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                               std::vector<std::pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo) {
        return mDev.SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo);
    }
    // loop closing: both Sim3 projection directions plus the mutual check (R :1305-1503)
    int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                     const cv::Mat& R12, const cv::Mat& t12, const float th) {
        return mDev.SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th);
    }
    int Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th = 3.0) {
        return mDev.Fuse(pKF, vpMapPoints, th);
    }
    int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
             vector<MapPoint*>& vpReplacePoint) {
        return mDev.Fuse(pKF, Scw, vpPoints, th, vpReplacePoint);
    }

public:
    static const int TH_LOW;
    static const int TH_HIGH;
    static const int HISTO_LENGTH;

protected:
    bool CheckDistEpipolarLine(const cv::KeyPoint& kp1, const cv::KeyPoint& kp2, const cv::Mat& F12,
                               const KeyFrame* pKF);
    float RadiusByViewingCos(const float& viewCos);
    void ComputeThreeMaxima(std::vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3);

    float mfNNratio;
    bool mbCheckOrientation;

private:
    orbslam2_amd::Matcher mDev;
};

}  // namespace ORB_SLAM2

#endif  // ORBMATCHER_H
