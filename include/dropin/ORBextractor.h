// Drop-in replacement for R/include/ORBextractor.h (R = the reference's ORB-SLAM2 tree): the same
// class surface (ctor, operator(), the inline getters, the public mvImagePyramid — filled on request,
// see operator()) implemented by
// liborbslam2_amd through include/orbslam2_amd_shim.hpp.  Compiles inside the reference tree only
// (OpenCV); the shim it wraps is compiled and tested here with mock types (tests/test_cpp_shim.py).
// R/src/ORBextractor.cpp drops out of the build.
#ifndef ORBEXTRACTOR_H
#define ORBEXTRACTOR_H

#include <list>
#include <vector>
#include <opencv/cv.h>

#include "orbslam2_amd_shim.hpp"

namespace ORB_SLAM2 {

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : mDev(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) {}
    ~ORBextractor() {}

    // R/src/ORBextractor.cpp:1120-1188; the mask is ignored, as there
    void operator()(cv::InputArray image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint>& keypoints,
                    cv::OutputArray descriptors) {
        if (image.empty()) return;   // :1123-1124: outputs untouched
        cv::Mat im = image.getMat();
        assert(im.type() == CV_8UC1);
        cv::Mat d;
        mDev.extract(im, keypoints, d);
        if (d.empty()) descriptors.release();
        else d.copyTo(descriptors);
        // mvImagePyramid (:88): its only reader in the reference is Frame::ComputeStereoMatches
        // (R/src/Frame.cpp:558, 675), which the drop-in runs on the device pyramids
        // (include/dropin/Frame_ComputeStereoMatches.cc), so a call downloads nothing beyond the
        // keypoints and descriptors.  A caller that reads the levels on the host opts in once with
        // SetHostPyramid(true); each call then refreshes the host views (one download per call).
        mvImagePyramid.clear();
        if (mbHostPyramid)
            for (const auto& L : mDev.pyramid())
                mvImagePyramid.push_back(cv::Mat(L.rows, L.cols, CV_8U, const_cast<uint8_t*>(L.data), L.step));
    }

    void SetHostPyramid(bool on) { mbHostPyramid = on; }

    int inline GetLevels() { return mDev.GetLevels(); }
    float inline GetScaleFactor() { return mDev.GetScaleFactor(); }
    std::vector<float> inline GetScaleFactors() { return mDev.GetScaleFactors(); }
    std::vector<float> inline GetInverseScaleFactors() { return mDev.GetInverseScaleFactors(); }
    std::vector<float> inline GetScaleSigmaSquares() { return mDev.GetScaleSigmaSquares(); }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mDev.GetInverseScaleSigmaSquares(); }

    std::vector<cv::Mat> mvImagePyramid;
    orb_extractor* dev() const { return mDev.handle(); }   // for Frame::ComputeStereoMatches

private:
    orbslam2_amd::Extractor mDev;
    bool mbHostPyramid = false;
};

}  // namespace ORB_SLAM2

#endif  // ORBEXTRACTOR_H
