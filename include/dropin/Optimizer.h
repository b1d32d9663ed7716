// Drop-in replacement for R/include/Optimizer.h: the same static interface.  LocalBundleAdjustment
// (R/src/Optimizer.cpp:564-918) and PoseOptimization (:306-535) run on liborbslam2_amd through
// include/orbslam2_amd_shim.hpp (graph gathering and write-back as the reference does them, the
// solve on the GPU); delete those two definitions from R/src/Optimizer.cpp.  The other methods keep
// their reference definitions; BundleAdjustment over the same library (lba_solve_global) is wired
// as INTEGRATION.md shows.  Compiles inside the reference tree only (OpenCV, g2o headers).
#ifndef OPTIMIZER_H
#define OPTIMIZER_H

#include "Frame.h"
#include "KeyFrame.h"
#include "LoopClosing.h"
#include "Map.h"
#include "MapPoint.h"
#include "Thirdparty/g2o/g2o/types/types_seven_dof_expmap.h"
#include "orbslam2_amd_shim.hpp"

namespace ORB_SLAM2 {

class LoopClosing;

class Optimizer {
public:
    void static BundleAdjustment(const std::vector<KeyFrame*>& vpKF, const std::vector<MapPoint*>& vpMP,
                                 int nIterations = 5, bool* pbStopFlag = NULL, const unsigned long nLoopKF = 0,
                                 const bool bRobust = true);
    void static GlobalBundleAdjustemnt(Map* pMap, int nIterations = 5, bool* pbStopFlag = NULL,
                                       const unsigned long nLoopKF = 0, const bool bRobust = true);
    void static LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap) {
        orbslam2_amd::LocalBundleAdjustment(pKF, pbStopFlag, pMap);
    }
    int static PoseOptimization(Frame* pFrame) { return orbslam2_amd::PoseOptimization(pFrame); }
    void static OptimizeEssentialGraph(Map* pMap, KeyFrame* pLoopKF, KeyFrame* pCurKF,
                                       const LoopClosing::KeyFrameAndPose& NonCorrectedSim3,
                                       const LoopClosing::KeyFrameAndPose& CorrectedSim3,
                                       const map<KeyFrame*, set<KeyFrame*> >& LoopConnections, const bool& bFixScale);
    static int OptimizeSim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches1, g2o::Sim3& g2oS12,
                            const float th2, const bool bFixScale);
};

}  // namespace ORB_SLAM2

#endif  // OPTIMIZER_H
