// Drop-in definition of Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770): replace the
// reference's definition in R/src/Frame.cpp with this one (or delete it there and add this file to
// the library's sources).  The stereo Frame constructor (R/src/Frame.cpp:68-129) runs the two
// extractions on two threads and then calls this: the matching runs on the GPU against the two
// extractors' device pyramids (orb_compute_stereo_matches), so no pyramid level is downloaded and
// mvImagePyramid stays empty (include/dropin/ORBextractor.h).  mb is still 0 at this point of the
// constructor, and the library keeps the reference's resulting maxD = +inf.
#include "Frame.h"
#include "ORBextractor.h"
#include "orbslam2_amd_shim.hpp"

namespace ORB_SLAM2 {

void Frame::ComputeStereoMatches() {
    orbslam2_amd::ComputeStereoMatches(*this, mpORBextractorLeft->dev(), mpORBextractorRight->dev());
}

}  // namespace ORB_SLAM2
