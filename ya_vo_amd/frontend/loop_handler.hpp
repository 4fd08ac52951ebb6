// loop_handler.hpp -- the reference's LoopHandler (include/LoopHandler.hpp, src/LoopHandler.cc) restated in C++
// over the C ABI: the same state machine (INIT -> buildInitMap -> TRACKING; track = trackLastFrame (LK) +
// optimizePoseOnly, reinitialize when fewer than 2 points track or fewer than 100 survive the pose LM), the same
// Frame / Feature / MapPoint / Map bookkeeping and the same config keys (basePath / sequence / cameraType).  Every
// per-frame primitive runs on the GPU through libyavo.so:
//
//   getFastFeatures / computeBrief      yv_detect / yv_describe            (frontend.hpp FastDetector / Brief)
//   matchFeatures / removeOutliers      yv_match_features / yv_filter_matches
//   getFRANSAC                          yv_f_ransac
//   cv::findEssentialMat / recoverPose  yv_find_essential / yv_recover_pose
//   triangulation + pixel2camera        yv_triangulate
//   Frame::world2Camera                 yv_world2camera
//   cv::calcOpticalFlowPyrLK            yv_calc_optical_flow_pyr_lk
//   optimizePoseOnly (g2o LM)           yv_pose_lm
//   cv::imread / getFilesInFolder /     yv_imread_gray / yv_seq_open / yv_seq_calib
//   getCalibParams
//
// Pose algebra (Sophus) runs on the host in se3_host.hpp.  Out of scope, as in DESIGN.md section 9: the Pangolin
// viewer, drawMatches / imwrite debugging, the ORB path (insertFrameFeaturesOPENCV) and the stdout chatter (the
// per-frame events are kept in `events()` instead).
#pragma once

#include <cstdint>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/yavo/yavo.h"
#include "../../include/yavo/yavo_io.h"
#include "frontend.hpp"
#include "se3_host.hpp"

namespace yavo_fe {

class SideLane;

enum voStatus { INIT, TRACKING, ERROR, RESET };  // include/LoopHandler.hpp:26

struct MapPoint {  // include/MapPoint.hpp: ptID from a process-wide counter (src/MapPoint.cc:6-11, first id 1)
    using ptr = std::shared_ptr<MapPoint>;
    unsigned long ptID = 0;
    double position[3] = {0, 0, 0};
    int observations = 0;  // addObservation count (the observation list itself only feeds the viewer)
    static ptr createMapPoint();
};

struct Feature {  // include/Feature.hpp: kp (x = row, y = column), a weak link to its map point, the outlier flag
    Point kp;
    std::weak_ptr<MapPoint> mapPoint;
    bool isOutlier = false;
};

struct Frame : Image {  // include/Frame.hpp: the raw image + computeBrief's keypoints (Image), pose T_cw, features
    using ptr = std::shared_ptr<Frame>;
    unsigned long frameID = 0;
    SE3 pose;
    std::vector<Feature> features;
    static unsigned long createFrameID();  // src/Frame.cc:43-47: first id 1
};

class Map {  // src/Map.cc:9-40: frames by frameID, landmarks by ptID
public:
    using ptr = std::shared_ptr<Map>;
    void insertKeyFrame(const Frame::ptr& f) { keyframes_[f->frameID] = f; }
    void insertMapPoint(const MapPoint::ptr& mp) { landmarks_[mp->ptID] = mp; }
    const std::map<unsigned long, Frame::ptr>& getFrames() const { return keyframes_; }
    const std::map<unsigned long, MapPoint::ptr>& getMps() const { return landmarks_; }

private:
    std::map<unsigned long, Frame::ptr> keyframes_;
    std::map<unsigned long, MapPoint::ptr> landmarks_;
};

// What addFrame did with one frame (the reference prints these to stdout).
struct FrameEvent {
    enum Kind { FIRST = 0, INIT_MAP = 1, TRACKED = 2, REINIT = 3 };
    int frame = 0;           // index in the path train
    int kind = FIRST;
    int keypoints = 0;       // computeBrief output
    int matches_kept = 0;    // removeOutliers (init / reinit)
    int essential_found = 0;
    int tracked = 0;         // trackLastFrame's good features (tracking)
    int inliers = -1;        // optimizePoseOnly (tracking), -1 when not reached
    int new_landmarks = 0;   // triangulate2View
    int f_inliers = 0;       // getFRANSAC's best count (F itself is unused, as in the reference)
};

class LoopHandler {
public:
    // The reference's constructor (src/LoopHandler.cc:7-33).  `dev` may be null or without a GPU: config parsing,
    // the path train and frame reading still work (the accessors below), the VO steps fail.
    LoopHandler(const std::string& config, Device* dev);
    ~LoopHandler();
    bool ok() const { return ok_; }
    const std::string& error() const { return error_; }

    std::string getSeqNo() const { return seqNo_; }
    bool stereoStatus() const { return isStereo_; }
    std::string getLeftImagesPath() const { return leftImagesPath_; }
    int getLeftTrainLength() const { return (int)leftPathTrain.size(); }

    Frame::ptr getNextFrame();          // cv::imread(path, 0) of the next left image, or nullptr at the end
    bool takeVOStep();                  // getNextFrame + insertFrameFeatures + addFrame; false at the end
    void insertFrameFeatures(const Frame::ptr& frame);
    void addFrame(const Frame::ptr& frame);
    bool buildInitMap();
    bool track();
    int trackLastFrame();
    int optimizePoseOnly(bool lk_ahead = false);  // lk_ahead: hand the next frame's LK to the side lane first
    bool reinitialize();
    int triangulate2View(const Frame::ptr& last, const Frame::ptr& curr, const std::vector<Matches>& filtMatches,
                         bool firstView);
    void runVO(int max_frames = -1);

    // Pipelined loop (the reference runs takeVOStep strictly in series, src/LoopHandler.cc:453-530): frame k + 1's
    // getNextFrame + insertFrameFeatures (PNG decode, detect, describe) do not depend on frame k's addFrame, so a
    // worker thread with its own GPU context (its own stream) computes them while this thread tracks frame k.  The
    // queue between the two holds at most `depth` frames.  Every result is the serial loop's: same frames, same
    // ids, same kernels, only earlier.  BRIEF's offsets must be given here (they are per context).  `readers` frames
    // are read and PNG-decoded ahead on threads of their own.
    // gpu_batch > 0: the worker decodes the look-ahead frames on the GPU instead (yv_pngdec: the files are read by
    // `readers` host threads, inflated and unfiltered by kernels), gpu_batch frames per decode, and detects / describes
    // them in one yv_batch run on the decoded device images (the same kernels as yv_detect / yv_describe); the next
    // batch is decoded while this one's frames are handed over.
    void setPipeline(int depth, int device, const std::vector<int8_t>& briefOffsets, int readers = 4,
                     int gpu_batch = 0);
    // One call of every primitive on this context with synthetic data of the sequence's size, before the loop: the
    // first call of a primitive loads its kernels and sizes its workspaces (setPipeline does the same for the worker
    // context and the side lane).  Results are unchanged; t_warmup has the time.
    bool warmup();
    double t_warmup = 0;
    static Frame::ptr readFrame(const std::string& path);  // cv::imread(path, IMREAD_GRAYSCALE)

    // every added frame's pose (T_cw, SE3d::data()) in order, and what happened to it
    const std::vector<SE3>& trajectory() const { return trajectory_; }
    const std::vector<FrameEvent>& events() const { return events_; }
    voStatus status() const { return status_; }
    const double* K() const { return K_; }
    int gpuStatus() const { return gpu_status_; }

    std::vector<std::string> leftPathTrain, rightPathTrain;
    Map::ptr map;
    SE3 relativeMotion;
    double t_features = 0, t_init = 0, t_track = 0, t_reinit = 0;  // seconds, summed
    double t_read = 0;  // getNextFrame (file read + PNG decode), summed; pipelined: waiting for the decode pool
    double t_wait = 0;  // pipelined: the tracking thread waiting for the worker's next frame
    struct PrimitiveTimes {  // seconds per host-pointer primitive of the tracking thread, summed
        double world2camera = 0, lk = 0, pose_lm = 0, match = 0, f_ransac = 0, find_essential = 0, recover_pose = 0;
    };
    const PrimitiveTimes& primitiveTimes() const { return prim_; }

private:
    std::string seqNo_, leftImagesPath_, rightImagesPath_, basePath_;
    bool isStereo_ = true;
    bool ok_ = false;
    std::string error_;
    double K_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 1};
    int H_ = 0, W_ = 0;  // the sequence's image size (yv_seq_size)
    Device* dev_ = nullptr;
    std::unique_ptr<FastDetector> fd_;
    std::unique_ptr<Brief> brief_;
    size_t train_it_ = 0;
    int currentFrameId_ = -1;
    voStatus status_ = INIT;
    Frame::ptr currentFrame_, lastFrame_;
    std::vector<SE3> trajectory_;
    std::vector<FrameEvent> events_;
    FrameEvent ev_;
    std::mt19937 ransac_rng_{0};  // getFRANSAC's sample draws (the reference seeds from std::random_device)
    int gpu_status_ = YV_OK;
    PrimitiveTimes prim_;

    int pipeline_depth_ = 0, pipeline_device_ = 0, pipeline_readers_ = 4, pipeline_gpu_batch_ = 0;
    std::vector<int8_t> pipeline_offsets_;
    // pipelined loop: getFRANSAC runs on a helper thread with its own GPU context (nothing downstream reads its
    // result: the reference discards F and the count, src/LoopHandler.cc:225, 567); each pending call's count is
    // written into its frame's event when the loop ends
    struct FResult {
        int status = YV_OK, inliers = 0;
        double seconds = 0;
    };
    SideLane* side_ = nullptr;
    // the pipelined loop's worker context and side lane, made by setPipeline (like the tracking thread's context,
    // before the loop: a context costs a few ms of allocations and stream set-up)
    std::unique_ptr<Device> worker_dev_;
    std::unique_ptr<SideLane> side_lane_;
    std::vector<std::pair<size_t, std::future<FResult>>> pending_f_;
    void resolvePendingF(bool wait);
    // pipelined loop: frame k + 1's pyramidal LK runs on the side lane during frame k's pose LM, over every frame-k
    // feature holding a map point at that moment (a superset of what trackLastFrame(k + 1) tracks: the LM only drops
    // map points, world2Camera only drops points).  LK tracks each point on its own, so the rows trackLastFrame(k + 1)
    // takes are the values its own call would return.  Dropped when frame k reinitialises.
    struct LKAhead {
        Frame::ptr last, next;
        std::vector<int> row_of;  // row per feature index of `last`, -1 without a map point
        std::vector<float> pts, nxt, err;
        std::vector<uint8_t> status;
        std::future<int> done;
        double seconds = 0;
    };
    std::function<Frame::ptr()> peek_next_;  // the pipelined loop's next queued frame, or nullptr
    std::shared_ptr<LKAhead> lk_ahead_;      // launched during the current frame's LM, for the next frame
    std::shared_ptr<LKAhead> lk_cur_;        // launched during the last frame's LM, for the current frame
    void launchLKAhead(const std::vector<int>& fi);
    void dropLKAhead(std::shared_ptr<LKAhead>& a);

public:
    int lk_ahead_frames = 0;  // tracked frames whose LK came from the side lane
    double lk_ahead_seconds = 0;  // side-lane LK time, summed (beside the tracking thread)

private:

    bool gpu(int st, const char* what);
    void runVOPipelined(int max_frames);
    int getFRANSAC(const std::vector<Matches>& m, double F[9]);
    bool essentialPose(const std::vector<Matches>& filt, SE3& currPose);
};

}  // namespace yavo_fe
