// loop_handler.cpp -- LoopHandler over the C ABI (see loop_handler.hpp).  Line references are to
// /root/reference/src/LoopHandler.cc unless noted.
#include "loop_handler.hpp"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <fstream>
#include <functional>
#include <future>
#include <iostream>
#include <iterator>
#include <mutex>
#include <thread>

#include "../../include/yavo/yavo_geom.h"
#include "json_config.hpp"

namespace yavo_fe {

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// int(v) for the reference's cv::Point2i(double, double) / Point2i(float, float): truncation toward zero; a value
// outside int (or NaN) gives INT_MIN, what x86-64's cvttsd2si returns (the reference's conversion is UB there)
int trunc_int(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return (int)v;
}

// One call of every host-pointer primitive a context serves in the loop, on synthetic data of the sequence's size
// (an H x W noise image and a copy shifted by (1, 3) pixels; its 2000 keypoints, matches, points and edges).  The
// first call of each primitive on a context loads its kernels and sizes its workspaces and pinned staging (the
// essential-matrix workspace, the LK image slots and pyramids, the call arenas); done here, at construction, that
// one-time cost stays out of the per-frame loop.  No state that a later call reads survives it (the BRIEF offsets
// are the caller's; the LK image slots are overwritten by the first real call, which finds no match).
struct WarmParts {
    bool features = false, matching = false, geometry = false, ransac = false, lk = false;
};

int warm_context(yv_ctx* ctx, int H, int W, const double K[9], const WarmParts& w) {
    if (!ctx || H < 32 || W < 32) return YV_OK;
    std::vector<uint8_t> a((size_t)H * W), b((size_t)H * W);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& v : a) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        v = (uint8_t)(x >> 56);
    }
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) b[(size_t)r * W + c] = a[(size_t)std::min(r + 1, H - 1) * W + std::min(c + 3, W - 1)];
    const int max_kp = 2000;
    std::vector<int32_t> rc(2 * max_kp);
    std::vector<float> resp(max_kp);
    int n = 0, nc = 0, st = YV_OK;
    if ((st = yv_detect(ctx, a.data(), H, W, W, max_kp, rc.data(), resp.data(), &n, &nc)) != YV_OK) return st;
    std::vector<yv_keypoint> kp(std::max(n, 1));
    int nk = 0;
    if ((w.features || w.matching) &&
        (st = yv_describe(ctx, a.data(), H, W, W, rc.data(), n, kp.data(), &nk)) != YV_OK)
        return st;
    std::vector<yv_match> m(std::max(nk, 1)), f(std::max(nk, 1));
    int nf = 0;
    if (w.matching && ((st = yv_match_features(ctx, kp.data(), nk, kp.data(), nk, m.data())) != YV_OK ||
                       (st = yv_filter_matches(ctx, m.data(), nk, 20, f.data(), &nf)) != YV_OK))
        return st;
    for (int i = 0; i < nk; ++i) {  // the second view: the keypoint moved by (1, 3)
        m[i].pt1 = kp[i];
        m[i].pt2 = kp[i];
        m[i].pt2.x = kp[i].x + 1;
        m[i].pt2.y = kp[i].y + 3;
        m[i].distance = 0;
    }
    if (w.ransac && nk >= 8) {
        std::vector<int32_t> samples(8 * 400);
        for (size_t i = 0; i < samples.size(); ++i) samples[i] = (int32_t)((i * 7919u) % (unsigned)nk);
        double F[9];
        int inl = 0, found = 0;
        if ((st = yv_f_ransac(ctx, m.data(), nk, samples.data(), 400, 0.1, F, &inl, &found)) != YV_OK) return st;
    }
    if (w.geometry && nk >= 5) {
        std::vector<float> p1(2 * (size_t)nk), p2(2 * (size_t)nk);
        for (int i = 0; i < nk; ++i) {
            p1[2 * i] = (float)m[i].pt1.x, p1[2 * i + 1] = (float)m[i].pt1.y;
            p2[2 * i] = (float)m[i].pt2.x, p2[2 * i + 1] = (float)m[i].pt2.y;
        }
        double E[9], R[9], t[3];
        std::vector<uint8_t> mask(nk);
        int found = 0, good = 0;
        if ((st = yv_find_essential(ctx, p2.data(), p1.data(), nk, K[0], K[2], K[5], 0.999, 1.0, E, mask.data(),
                                    &found)) != YV_OK ||
            (st = yv_recover_pose(ctx, E, p2.data(), p1.data(), nk, K, R, t, &good)) != YV_OK)
            return st;
        const double Ta[7] = {0, 0, 0, 1, 0, 0, 0}, Tb[7] = {0, 0, 0, 1, -0.5, 0, 0};
        std::vector<double> X(3 * (size_t)nk), proj(3 * (size_t)nk), uv(2 * (size_t)nk);
        std::vector<uint8_t> ok(nk), outl(nk);
        int n_ok = 0, inl = 0;
        if ((st = yv_triangulate(ctx, Ta, Tb, K, m.data(), nk, X.data(), ok.data(), &n_ok)) != YV_OK) return st;
        for (int i = 0; i < nk; ++i) {  // points in front of the camera, measured where they project
            X[3 * i] = (m[i].pt1.y - K[2]) / K[0] * 10.0;
            X[3 * i + 1] = (m[i].pt1.x - K[5]) / K[4] * 10.0;
            X[3 * i + 2] = 10.0;
            uv[2 * i] = m[i].pt1.x;
            uv[2 * i + 1] = m[i].pt1.y;
        }
        double pose[7] = {0, 0, 0, 1, 0.01, 0, 0};
        if ((st = yv_world2camera(ctx, X.data(), nk, pose, K, proj.data())) != YV_OK ||
            (st = yv_pose_lm(ctx, X.data(), uv.data(), nk, K, pose, outl.data(), &inl)) != YV_OK)
            return st;
    }
    if (w.lk && nk > 0) {
        std::vector<float> pts(2 * (size_t)nk), nxt(2 * (size_t)nk), err(nk);
        std::vector<uint8_t> status(nk);
        for (int i = 0; i < nk; ++i) pts[2 * i] = (float)kp[i].y, pts[2 * i + 1] = (float)kp[i].x;
        if ((st = yv_calc_optical_flow_pyr_lk(ctx, a.data(), b.data(), H, W, W, pts.data(), nk, 11, 3, 30, 0.01,
                                              0.001, nxt.data(), status.data(), err.data())) != YV_OK)
            return st;
    }
    return yv_sync(ctx);
}

}  // namespace

MapPoint::ptr MapPoint::createMapPoint() {
    static unsigned long _ptID = 0;
    auto mp = std::make_shared<MapPoint>();
    mp->ptID = ++_ptID;
    return mp;
}

unsigned long Frame::createFrameID() {
    static unsigned long frameID_ = 0;
    frameID_++;
    return frameID_;
}

// :7-33.  cameraType "mono" -> image_0 only; anything else -> stereo with image_1.  Calibration from
// basePath + sequence + "/calib.txt" (handler3D.setCalibParams -> Camera::K of P0).
LoopHandler::LoopHandler(const std::string& config, Device* dev) : dev_(dev) {
    JsonConfig value;
    if (!value.parse_file(config)) {
        error_ = "cannot parse config " + config;
        return;
    }
    basePath_ = value.asString("basePath");
    seqNo_ = value.asString("sequence");
    const std::string camType = value.asString("cameraType");
    if (camType == "mono") {
        isStereo_ = false;
        leftImagesPath_ = basePath_ + seqNo_ + "/image_0/";
        rightImagesPath_ = "";
    } else {
        isStereo_ = true;
        leftImagesPath_ = basePath_ + seqNo_ + "/image_0/";
        rightImagesPath_ = basePath_ + seqNo_ + "/image_1/";
    }
    // generatePathTrain (:37-57): the sorted listings of getFilesInFolder
    yv_seq* seq = nullptr;
    int st = yv_seq_open((basePath_ + seqNo_).c_str(), isStereo_ ? 1 : 0, &seq);
    if (st != YV_OK) {
        error_ = "no image_0 listing under " + basePath_ + seqNo_;
        return;
    }
    const int n = yv_seq_frames(seq);
    char buf[4096];
    for (int i = 0; i < n; ++i) {
        if (yv_seq_path(seq, i, 0, buf, sizeof buf) > 0) leftPathTrain.emplace_back(buf);
        if (isStereo_ && yv_seq_path(seq, i, 1, buf, sizeof buf) > 0) rightPathTrain.emplace_back(buf);
    }
    double P0[16], P1[16], K1[9];
    if (yv_seq_size(seq, &H_, &W_) != YV_OK) H_ = W_ = 0;  // the first image's size (warmup)
    st = yv_seq_calib(seq, P0, P1, K_, K1);
    yv_seq_close(seq);
    if (st != YV_OK) {
        error_ = "no calib.txt under " + basePath_ + seqNo_;
        return;
    }
    map = std::make_shared<Map>();
    if (dev_ && dev_->ok()) {
        fd_ = std::make_unique<FastDetector>(*dev_, 12, 50);  // fd(12, 50), brief(256) (:7)
        brief_ = std::make_unique<Brief>(*dev_, 256);
    }
    ok_ = true;
}

bool LoopHandler::gpu(int st, const char* what) {
    if (st == YV_OK) return true;
    gpu_status_ = st;
    std::cerr << "yavo: " << what << " failed: " << yv_status_string(st) << std::endl;
    return false;
}

// cv::imread(path, IMREAD_GRAYSCALE) (:919) = the PNG file decoded to 8-bit grey; nullptr (with a message) when
// the file cannot be read.  Thread-safe: the pipelined loop decodes several frames at once.
Frame::ptr LoopHandler::readFrame(const std::string& path) {
    std::ifstream fin(path, std::ios::binary);
    std::vector<uint8_t> file((std::istreambuf_iterator<char>(fin)), std::istreambuf_iterator<char>());
    int H = 0, W = 0;
    if (file.empty() || yv_png_info(file.data(), file.size(), &H, &W) != YV_OK) {
        std::cerr << "yavo: cannot read " << path << std::endl;
        return nullptr;
    }
    auto frame = std::make_shared<Frame>();
    frame->rows = H;
    frame->cols = W;
    frame->data.resize((size_t)H * W);
    const int st = yv_png_decode_gray(file.data(), file.size(), frame->data.data(), W, H, W);
    if (st != YV_OK) {
        std::cerr << "yavo: cannot decode " << path << " (" << yv_status_string(st) << ")" << std::endl;
        return nullptr;
    }
    return frame;
}

// :918-930
Frame::ptr LoopHandler::getNextFrame() {
    if (train_it_ >= leftPathTrain.size()) return nullptr;
    const double t0 = now_s();
    Frame::ptr frame = readFrame(leftPathTrain[train_it_]);
    if (!frame) return nullptr;
    currentFrameId_ = (int)train_it_;
    train_it_++;
    frame->frameID = Frame::createFrameID();
    t_read += now_s() - t0;
    return frame;
}

// :457-466
bool LoopHandler::takeVOStep() {
    Frame::ptr frame = getNextFrame();
    if (!frame) return false;
    insertFrameFeatures(frame);
    addFrame(frame);
    return gpu_status_ == YV_OK;
}

// :468-485: getFastFeatures + computeBrief (the keypoints go to the frame's Image)
void LoopHandler::insertFrameFeatures(const Frame::ptr& frame) {
    const double t0 = now_s();
    if (!fd_ || !brief_) {
        gpu(YV_ERR_NODEVICE, "insertFrameFeatures");
        return;
    }
    auto features = fd_->getFastFeatures(*frame);
    if (!gpu(fd_->status(), "getFastFeatures")) return;
    brief_->computeBrief(features, *frame);
    gpu(brief_->status(), "computeBrief");
    t_features += now_s() - t0;
}

// :80-124
void LoopHandler::addFrame(const Frame::ptr& frame) {
    currentFrame_ = frame;
    lk_cur_ = std::move(lk_ahead_);
    ev_ = FrameEvent();
    ev_.frame = currentFrameId_;
    ev_.keypoints = (int)frame->keypoints.size();
    if (status_ == INIT) {
        if (lastFrame_) {
            const double t0 = now_s();
            if (buildInitMap()) status_ = TRACKING;
            ev_.kind = FrameEvent::INIT_MAP;
            t_init += now_s() - t0;
        }
    } else if (status_ == TRACKING) {
        const double t0 = now_s();
        const bool trackSuccess = track();
        t_track += now_s() - t0;
        ev_.kind = FrameEvent::TRACKED;
        if (!trackSuccess) {
            dropLKAhead(lk_ahead_);  // its rows index the features reinitialize() replaces
            const double t1 = now_s();
            reinitialize();
            map->insertKeyFrame(currentFrame_);
            ev_.kind = FrameEvent::REINIT;
            t_reinit += now_s() - t1;
        }
    } else if (status_ == RESET) {
        if (reinitialize()) status_ = TRACKING;
        ev_.kind = FrameEvent::REINIT;
    }
    dropLKAhead(lk_cur_);  // reads lastFrame_'s pixels
    // the previous frame's pixels and descriptors are not read again (the map keeps the frame for its pose)
    if (lastFrame_) {
        lastFrame_->data.clear();
        lastFrame_->data.shrink_to_fit();
        lastFrame_->keypoints.clear();
        lastFrame_->keypoints.shrink_to_fit();
    }
    lastFrame_ = currentFrame_;
    trajectory_.push_back(currentFrame_->pose);
    events_.push_back(ev_);
}

// A helper thread with a GPU context of its own, running the calls it is handed in order (SideLane::submit); the
// destructor runs what is queued and joins.
class SideLane {
public:
    explicit SideLane(int device) : th_([this, device]() { run(device); }) {}
    ~SideLane() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    SideLane(const SideLane&) = delete;
    SideLane& operator=(const SideLane&) = delete;
    void submit(std::function<void(Device&)> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    void run(int device) {
        Device dev(device);
        while (true) {
            std::function<void(Device&)> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&]() { return stop_ || !q_.empty(); });
                if (q_.empty()) return;  // stop_ and nothing left
                f = std::move(q_.front());
                q_.pop_front();
            }
            f(dev);
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void(Device&)>> q_;
    bool stop_ = false;
    std::thread th_;  // last: starts after the members it uses exist
};

// _3DHandler::getFRANSAC(filterMatches, F, 400, 0.1) (src/3DHandler.cc:145-195): 400 hypotheses of 8 indices drawn
// uniformly from [0, n) with replacement.  The reference's F is never used after the call (:222, :562), and neither is
// the count: with a side lane (the pipelined loop) the call is handed to it with its samples (drawn here, in loop
// order) and its count lands in the frame's event later (resolvePendingF: finished calls are folded in at the next
// getFRANSAC, the rest at the end of the run); F stays zero.
int LoopHandler::getFRANSAC(const std::vector<Matches>& m, double F[9]) {
    const int n = (int)m.size();
    for (int i = 0; i < 9; ++i) F[i] = 0;
    if (n < 8) return 0;
    const int iters = 400;
    std::vector<int32_t> samples(8 * iters);
    std::uniform_int_distribution<int> dist(0, n - 1);
    for (auto& s : samples) s = dist(ransac_rng_);
    if (side_) {
        resolvePendingF(false);
        if (gpu_status_ != YV_OK) return 0;
        auto task = std::make_shared<std::packaged_task<FResult(Device&)>>(
            [m, samples = std::move(samples), n, iters](Device& d) {
                FResult r;
                const double t0 = now_s();
                double Fs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                int max_inl = 0, found = 0;
                r.status = d.ok() ? yv_f_ransac(d.ctx(), m.data(), n, samples.data(), iters, 0.1, Fs, &max_inl, &found)
                                  : d.status();
                r.inliers = r.status == YV_OK && found ? max_inl : 0;
                r.seconds = now_s() - t0;
                return r;
            });
        pending_f_.emplace_back(events_.size(), task->get_future());  // this frame's event is pushed at that index
        side_->submit([task](Device& d) { (*task)(d); });
        return 0;
    }
    int max_inl = 0, found = 0;
    const double t0 = now_s();
    struct Acc {
        double& v;
        double t;
        ~Acc() { v += now_s() - t; }
    } acc{prim_.f_ransac, t0};
    if (!gpu(yv_f_ransac(dev_->ctx(), m.data(), n, samples.data(), iters, 0.1, F, &max_inl, &found), "getFRANSAC"))
        return 0;
    return found ? max_inl : 0;
}

// :575-648 / :228-290: E = findEssentialMat(curr, prev, 718.8560, (607.1928, 185.2157), RANSAC, 0.999, 1.0);
// recoverPose(E, curr, last, K, R, t); currPose = SE3(R, t)
bool LoopHandler::essentialPose(const std::vector<Matches>& filt, SE3& currPose) {
    const int n = (int)filt.size();
    std::vector<float> curr(2 * n), prev(2 * n);
    for (int i = 0; i < n; ++i) {
        prev[2 * i] = (float)filt[i].pt1.x;
        prev[2 * i + 1] = (float)filt[i].pt1.y;
        curr[2 * i] = (float)filt[i].pt2.x;
        curr[2 * i + 1] = (float)filt[i].pt2.y;
    }
    double E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<uint8_t> mask(n > 0 ? n : 1);
    int found = 0;
    const double t0 = now_s();
    if (!gpu(yv_find_essential(dev_->ctx(), curr.data(), prev.data(), n, 718.8560, 607.1928, 185.2157, 0.999, 1.0,
                               E, mask.data(), &found),
             "findEssentialMat"))
        return false;
    ev_.essential_found = found;
    const double t1 = now_s();
    prim_.find_essential += t1 - t0;
    double R[9], t[3];
    int good = 0;
    if (!gpu(yv_recover_pose(dev_->ctx(), E, curr.data(), prev.data(), n, K_, R, t, &good), "recoverPose"))
        return false;
    prim_.recover_pose += now_s() - t1;
    currPose = se3::from_Rt(R, t);
    return true;
}

// :532-652
bool LoopHandler::buildInitMap() {
    std::vector<Matches> matches = brief_->matchFeatures(*lastFrame_, *currentFrame_);
    std::vector<Matches> filterMatches;
    brief_->removeOutliers(matches, filterMatches, 20);
    if (!gpu(brief_->status(), "matchFeatures / removeOutliers")) return false;
    ev_.matches_kept = (int)filterMatches.size();
    // only the matched-and-kept points become features (:555-561)
    for (const auto& m : filterMatches) {
        Feature f1, f2;
        f1.kp = Point{m.pt1.x, m.pt1.y};
        f2.kp = Point{m.pt2.x, m.pt2.y};
        lastFrame_->features.push_back(f1);
        currentFrame_->features.push_back(f2);
    }
    double F[9];
    ev_.f_inliers = getFRANSAC(filterMatches, F);
    SE3 currPose;
    if (!essentialPose(filterMatches, currPose)) return false;
    currentFrame_->pose = se3::inverse(currPose);  // :621-622
    map->insertKeyFrame(lastFrame_);
    map->insertKeyFrame(currentFrame_);
    ev_.new_landmarks = triangulate2View(lastFrame_, currentFrame_, filterMatches, true);
    relativeMotion = se3::mul(currentFrame_->pose, se3::inverse(lastFrame_->pose));  // :649
    return true;
}

// :658-726: each kept match triangulated from the two poses (pixel2camera of pt1 / pt2, DLT + SVD); accepted
// points (triangulation ok and Z > 0) become map points.  firstView: linked to the existing features i of both
// frames; otherwise a new current-frame feature at pt2 carries the point.
int LoopHandler::triangulate2View(const Frame::ptr& last, const Frame::ptr& curr,
                                  const std::vector<Matches>& filtMatches, bool firstView) {
    const int n = (int)filtMatches.size();
    if (n == 0) return 0;
    std::vector<double> X(3 * (size_t)n);
    std::vector<uint8_t> ok(n);
    int n_ok = 0;
    if (!gpu(yv_triangulate(dev_->ctx(), last->pose.d, curr->pose.d, K_, filtMatches.data(), n, X.data(), ok.data(),
                            &n_ok),
             "triangulation"))
        return 0;
    int landMarks = 0;
    for (int i = 0; i < n; ++i) {
        if (!ok[i]) continue;
        auto mp = MapPoint::createMapPoint();
        mp->position[0] = X[3 * i];
        mp->position[1] = X[3 * i + 1];
        mp->position[2] = X[3 * i + 2];
        if (firstView) {
            mp->observations += 2;
            currentFrame_->features[i].mapPoint = mp;
            last->features[i].mapPoint = mp;
        } else {
            Feature f;
            f.kp = Point{filtMatches[i].pt2.x, filtMatches[i].pt2.y};
            f.mapPoint = mp;
            currentFrame_->features.push_back(f);
            mp->observations += 1;
        }
        map->insertMapPoint(mp);
        landMarks++;
    }
    return landMarks;
}

// :132-165
bool LoopHandler::track() {
    if (lastFrame_) currentFrame_->pose = se3::mul(relativeMotion, lastFrame_->pose);
    const int goodInliers = trackLastFrame();
    ev_.tracked = goodInliers;
    if (goodInliers < 2) return false;
    const int optimizedInliers = optimizePoseOnly(side_ && peek_next_);
    ev_.inliers = optimizedInliers;
    if (optimizedInliers < 100) return false;
    relativeMotion = se3::mul(currentFrame_->pose, se3::inverse(lastFrame_->pose));
    return true;
}

// :306-449: the last frame's features with a map point, projected with the current pose guess (world2Camera;
// kept when neither truncated coordinate is negative), tracked by pyramidal LK (11x11, 3 levels, 30 its / 0.01,
// flags 0: the projection is not an initial guess), status-1 points become current features at
// Point2i(next.y, next.x) carrying the same map point.
int LoopHandler::trackLastFrame() {
    std::vector<int> idx;
    std::vector<double> Xs;
    std::vector<MapPoint::ptr> mps;
    for (int i = 0; i < (int)lastFrame_->features.size(); ++i) {
        if (auto mp = lastFrame_->features[i].mapPoint.lock()) {
            idx.push_back(i);
            mps.push_back(mp);
            Xs.insert(Xs.end(), mp->position, mp->position + 3);
        }
    }
    const int nc = (int)idx.size();
    std::vector<double> proj(3 * (size_t)std::max(nc, 1));
    const double tw = now_s();
    if (nc > 0 &&
        !gpu(yv_world2camera(dev_->ctx(), Xs.data(), nc, currentFrame_->pose.d, K_, proj.data()), "world2Camera"))
        return 0;
    prim_.world2camera += now_s() - tw;
    std::vector<float> lastKpt, currKpt;
    std::vector<int> lastIndex;
    std::vector<MapPoint::ptr> lastMps;
    for (int k = 0; k < nc; ++k) {
        const int nx = trunc_int(proj[3 * k + 1] / proj[3 * k + 2]);  // Point2i(coeff(1)/coeff(2), coeff(0)/coeff(2))
        const int ny = trunc_int(proj[3 * k] / proj[3 * k + 2]);
        if (!(nx < 0 || ny < 0)) {
            currKpt.push_back((float)nx);
            currKpt.push_back((float)ny);
            const Point kp = lastFrame_->features[idx[k]].kp;
            lastKpt.push_back((float)kp.y);  // Point2i(kp.y, kp.x)
            lastKpt.push_back((float)kp.x);
            lastIndex.push_back(idx[k]);
            lastMps.push_back(mps[k]);
        }
    }
    const int n = (int)lastIndex.size();
    if (n == 0) return 0;  // an empty point set: calcOpticalFlowPyrLK returns empty status
    std::vector<float> next(2 * (size_t)n), err(n);
    std::vector<uint8_t> flowStatus(n);
    const double tl = now_s();
    bool have = false;
    if (lk_cur_ && lk_cur_->last == lastFrame_ && lk_cur_->next == currentFrame_) {
        LKAhead& a = *lk_cur_;
        have = a.done.get() == YV_OK;
        if (have) {
            lk_ahead_seconds += a.seconds;
            for (int i = 0; i < n && have; ++i) {
                const int r = lastIndex[i] < (int)a.row_of.size() ? a.row_of[lastIndex[i]] : -1;
                if (r < 0 || a.pts[2 * r] != lastKpt[2 * i] || a.pts[2 * r + 1] != lastKpt[2 * i + 1]) {
                    have = false;  // not in the superset: the call below tracks the list itself
                    break;
                }
                next[2 * i] = a.nxt[2 * r];
                next[2 * i + 1] = a.nxt[2 * r + 1];
                flowStatus[i] = a.status[r];
                err[i] = a.err[r];
            }
        }
        lk_cur_.reset();
        if (have) ++lk_ahead_frames;
    }
    if (!have && !gpu(yv_calc_optical_flow_pyr_lk(dev_->ctx(), lastFrame_->data.data(), currentFrame_->data.data(),
                                                  currentFrame_->rows, currentFrame_->cols, currentFrame_->cols,
                                                  lastKpt.data(), n, 11, 3, 30, 0.01, 0.001, next.data(),
                                                  flowStatus.data(), err.data()),
                      "calcOpticalFlowPyrLK"))
        return 0;
    prim_.lk += now_s() - tl;
    int goodFeatures = 0;
    for (int i = 0; i < n; ++i) {
        if (flowStatus[i] != 1) continue;
        if (const MapPoint::ptr& mp = lastMps[i]) {  // locked above; nothing has released it since
            Feature f;
            f.kp = Point{trunc_int(next[2 * i + 1]), trunc_int(next[2 * i])};  // Point2i(currFrameKpt.y, .x)
            f.mapPoint = mp;
            currentFrame_->features.push_back(f);
            goodFeatures++;
        }
    }
    return goodFeatures;
}

void LoopHandler::launchLKAhead(const std::vector<int>& fi) {
    const Frame::ptr nf = peek_next_();
    if (!nf || nf->rows != currentFrame_->rows || nf->cols != currentFrame_->cols || nf->data.empty()) return;
    const int n = (int)fi.size();
    if (n == 0) return;
    auto a = std::make_shared<LKAhead>();
    a->last = currentFrame_;
    a->next = nf;
    a->row_of.assign(currentFrame_->features.size(), -1);
    a->pts.resize(2 * (size_t)n);
    for (int r = 0; r < n; ++r) {
        const Feature& f = currentFrame_->features[fi[r]];
        a->row_of[fi[r]] = r;
        a->pts[2 * r] = (float)f.kp.y;  // trackLastFrame's Point2i(kp.y, kp.x)
        a->pts[2 * r + 1] = (float)f.kp.x;
    }
    a->nxt.resize(2 * (size_t)n);
    a->err.resize((size_t)n);
    a->status.resize((size_t)n);
    auto task = std::make_shared<std::packaged_task<int(Device&)>>([a, n](Device& d) {
        const double t0 = now_s();
        const int st = d.ok() ? yv_calc_optical_flow_pyr_lk(d.ctx(), a->last->data.data(), a->next->data.data(),
                                                           a->last->rows, a->last->cols, a->last->cols, a->pts.data(),
                                                           n, 11, 3, 30, 0.01, 0.001, a->nxt.data(), a->status.data(),
                                                           a->err.data())
                              : d.status();
        a->seconds = now_s() - t0;
        return st;
    });
    a->done = task->get_future();
    side_->submit([task](Device& d) { (*task)(d); });
    lk_ahead_ = std::move(a);
}

// a look-ahead no one will read: its call may still be reading the frames' pixels, so wait for it
void LoopHandler::dropLKAhead(std::shared_ptr<LKAhead>& a) {
    if (!a) return;
    if (a->done.valid()) a->done.wait();
    a.reset();
}

// :730-861: one pose vertex at the current pose, one projection edge per feature with a map point (measurement
// (kp.x, kp.y), Huber), 4 rounds of optimize(10) with chi2 > 5.991 outliers; outliers lose their map point
int LoopHandler::optimizePoseOnly(bool lk_ahead) {
    std::vector<int> fi;
    std::vector<double> X, uv;
    for (int i = 0; i < (int)currentFrame_->features.size(); ++i) {
        const Feature& f = currentFrame_->features[i];
        if (auto mp = f.mapPoint.lock()) {
            fi.push_back(i);
            X.insert(X.end(), mp->position, mp->position + 3);
            uv.push_back((double)f.kp.x);
            uv.push_back((double)f.kp.y);
        }
    }
    const int n = (int)fi.size();
    if (lk_ahead) launchLKAhead(fi);  // fi: the features holding a map point now
    std::vector<uint8_t> outlier(n > 0 ? n : 1);
    int inliers = 0;
    SE3 pose = currentFrame_->pose;
    const double t0 = now_s();
    if (!gpu(yv_pose_lm(dev_->ctx(), X.data(), uv.data(), n, K_, pose.d, outlier.data(), &inliers),
             "optimizePoseOnly"))
        return 0;
    prim_.pose_lm += now_s() - t0;
    currentFrame_->pose = pose;
    for (int k = 0; k < n; ++k) {
        Feature& f = currentFrame_->features[fi[k]];
        if (outlier[k]) f.mapPoint.reset();
        f.isOutlier = false;
    }
    return inliers;
}

// :168-296
bool LoopHandler::reinitialize() {
    currentFrame_->features.clear();
    const double t0 = now_s();
    std::vector<Matches> matches = brief_->matchFeatures(*lastFrame_, *currentFrame_);
    std::vector<Matches> filterMatches;
    brief_->removeOutliers(matches, filterMatches, 20);
    prim_.match += now_s() - t0;
    if (!gpu(brief_->status(), "matchFeatures / removeOutliers")) return false;
    ev_.matches_kept = (int)filterMatches.size();
    double F[9];
    ev_.f_inliers = getFRANSAC(filterMatches, F);
    SE3 currPose;
    if (!essentialPose(filterMatches, currPose)) return false;
    currPose = se3::inverse(currPose);
    currentFrame_->pose = se3::mul(currPose, lastFrame_->pose);  // :283-285
    ev_.new_landmarks = triangulate2View(lastFrame_, currentFrame_, filterMatches, false);
    relativeMotion = se3::mul(currentFrame_->pose, se3::inverse(lastFrame_->pose));
    return true;
}

// :501-512
void LoopHandler::runVO(int max_frames) {
    if (pipeline_depth_ > 0) {
        runVOPipelined(max_frames);
        return;
    }
    int k = 0;
    while (max_frames < 0 || k < max_frames) {
        if (!takeVOStep()) break;
        ++k;
    }
}

// the tracking thread's context: every primitive addFrame calls (and detect / describe of the serial loop)
bool LoopHandler::warmup() {
    if (!dev_ || !dev_->ok()) return false;
    const double t0 = now_s();
    WarmParts w;
    w.features = w.matching = w.geometry = w.ransac = w.lk = true;
    const bool ok = gpu(warm_context(dev_->ctx(), H_, W_, K_, w), "warmup");
    t_warmup += now_s() - t0;
    return ok;
}

void LoopHandler::setPipeline(int depth, int device, const std::vector<int8_t>& briefOffsets, int readers,
                              int gpu_batch) {
    pipeline_readers_ = readers;
    pipeline_gpu_batch_ = gpu_batch > 0 ? gpu_batch : 0;
    pipeline_depth_ = depth > 0 ? depth : 0;
    pipeline_device_ = device;
    pipeline_offsets_ = briefOffsets;
    if (pipeline_depth_ > 0) {
        const double t0 = now_s();
        worker_dev_ = std::make_unique<Device>(device);
        side_lane_ = std::make_unique<SideLane>(device);  // its thread makes its own context meanwhile
        // warm both: the worker's detect / describe (its offsets are set again by the worker thread) and the side
        // lane's getFRANSAC / LK, on the side lane's own thread
        std::promise<int> side_done;
        auto side_st = side_done.get_future();
        const int H = H_, W = W_;
        const double* K = K_;
        side_lane_->submit([&side_done, H, W, K](Device& d) {
            WarmParts w;
            w.ransac = w.lk = true;
            side_done.set_value(d.ok() ? warm_context(d.ctx(), H, W, K, w) : d.status());
        });
        if (worker_dev_->ok() && yv_set_brief_offsets(worker_dev_->ctx(), pipeline_offsets_.data()) == YV_OK) {
            WarmParts w;
            w.features = true;
            gpu(warm_context(worker_dev_->ctx(), H_, W_, K_, w), "warmup (pipeline worker)");
        }
        gpu(side_st.get(), "warmup (side lane)");
        t_warmup += now_s() - t0;
    }
}

LoopHandler::~LoopHandler() = default;

namespace {

// The pipelined worker's GPU look-ahead: frames [first, first + n) of the left train read by host threads, inflated +
// unfiltered on the GPU (yv_seq_upload_gpu, the device half of cv::imread), detected and described by one yv_batch run
// over the decoded device images (no match pairs), then the images and keypoint records copied back for the frames.
class GpuLookahead {
public:
    GpuLookahead(yv_ctx* ctx, const std::string& seq_dir, int batch) : ctx_(ctx), B_(batch) {
        st_ = yv_seq_open(seq_dir.c_str(), 0, &seq_);
        if (st_ == YV_OK) st_ = yv_seq_size(seq_, &H_, &W_);
        const size_t img = (size_t)H_ * W_;
        if (st_ == YV_OK) st_ = yv_pngdec_create(ctx_, B_, H_, W_, &dec_);
        if (st_ == YV_OK) st_ = yv_batch_create(ctx_, B_, H_, W_, kMaxKp, 1, &batch_);
        if (st_ == YV_OK) st_ = yv_batch_view_get(batch_, &view_);
        if (st_ == YV_OK) st_ = yv_device_alloc(ctx_, B_ * img, &d_img_);
        if (st_ == YV_OK) st_ = yv_host_alloc(ctx_, B_ * img, reinterpret_cast<void**>(&h_img_));
        if (st_ == YV_OK) st_ = yv_host_alloc(ctx_, (size_t)B_ * kMaxKp * sizeof(KeyPoint), reinterpret_cast<void**>(&h_kp_));
        if (st_ == YV_OK) st_ = yv_host_alloc(ctx_, sizeof(int32_t) * (B_ + 1), reinterpret_cast<void**>(&h_cnt_));
        if (st_ == YV_OK) st_ = yv_host_alloc(ctx_, sizeof(uint32_t) * (B_ + 1), reinterpret_cast<void**>(&h_cand_));
    }
    ~GpuLookahead() {
        if (dec_) yv_pngdec_destroy(dec_);
        if (batch_) yv_batch_destroy(batch_);
        if (seq_) yv_seq_close(seq_);
        yv_device_free(ctx_, d_img_);
        yv_host_free(ctx_, h_img_);
        yv_host_free(ctx_, h_kp_);
        yv_host_free(ctx_, h_cnt_);
        yv_host_free(ctx_, h_cand_);
    }
    int status() const { return st_; }
    int H() const { return H_; }
    int W() const { return W_; }

    // enqueue frames [first, first + n): the file reads on `readers` threads now, decode + detect + describe on the
    // context stream (returns before the kernels finish)
    int launch(int first, int n, int readers) {
        first_ = first;
        n_ = n;
        if (n <= 0) return YV_OK;
        int st = yv_seq_upload_gpu(seq_, dec_, first, n, static_cast<uint8_t*>(d_img_), (int64_t)H_ * W_, readers,
                                   nullptr);
        if (st == YV_OK)
            st = yv_batch_run(batch_, static_cast<const uint8_t*>(d_img_), n, W_, (int64_t)H_ * W_, 20, -1, nullptr);
        return st;
    }
    // waits for the launched frames; frames[i] = frame first + i, or nullptr when its PNG failed a check (the reference's
    // cv::imread returns an empty Mat: the loop ends there)
    int collect(std::vector<Frame::ptr>& frames) {
        frames.assign((size_t)n_, nullptr);
        const int n = n_;
        n_ = 0;  // collected once: a further collect without a launch returns no frames (the end of the train)
        if (n <= 0) return YV_OK;
        std::vector<int32_t> codes((size_t)B_);
        int bad = 0;
        int st = yv_pngdec_status(dec_, codes.data(), &bad);
        const size_t img = (size_t)H_ * W_;
        if (st == YV_OK) st = yv_download(ctx_, h_cnt_, view_.kp_count, sizeof(int32_t) * n);
        if (st == YV_OK) st = yv_download(ctx_, h_cand_, view_.cand_count, sizeof(uint32_t) * n);
        if (st == YV_OK) st = yv_download(ctx_, h_kp_, view_.keypoints, sizeof(KeyPoint) * (size_t)n * kMaxKp);
        if (st == YV_OK) st = yv_download(ctx_, h_img_, d_img_, img * n);
        if (st != YV_OK) return st;
        for (int i = 0; i < n; ++i) {
            if (codes[(size_t)i] != 0) break;
            auto f = std::make_shared<Frame>();
            f->rows = H_;
            f->cols = W_;
            f->data.assign(h_img_ + img * i, h_img_ + img * (i + 1));
            const int nk = h_cnt_[i];
            // the FAST candidate count, as getFastFeatures prints it (src/FastDetector.cc:364-366, frontend.cpp)
            if (h_cand_[i] == 0) std::cout << "No corners found" << std::endl;
            f->keypoints.assign(h_kp_ + (size_t)i * kMaxKp, h_kp_ + (size_t)i * kMaxKp + nk);
            frames[(size_t)i] = f;
        }
        return YV_OK;
    }

private:
    static constexpr int kMaxKp = 2000;  // FastDetector's top-2000 (include/FastDetector.hpp:36)
    yv_ctx* ctx_;
    int B_, H_ = 0, W_ = 0, st_ = YV_OK, first_ = 0, n_ = 0;
    yv_seq* seq_ = nullptr;
    yv_pngdec* dec_ = nullptr;
    yv_batch* batch_ = nullptr;
    yv_batch_view view_{};
    void* d_img_ = nullptr;
    uint8_t* h_img_ = nullptr;
    KeyPoint* h_kp_ = nullptr;
    int32_t* h_cnt_ = nullptr;
    uint32_t* h_cand_ = nullptr;
};

}  // namespace

// takeVOStep split over two threads: the worker runs getNextFrame + insertFrameFeatures on its own context for
// frame k + 1 while this thread runs addFrame(frame k).  Frames leave the worker in path-train order, so ids,
// keypoints and every later result are the serial loop's.
// the tracking thread's bound on waiting for the pipeline worker's next frame
constexpr int kPipelineStallSeconds = 60;

void LoopHandler::runVOPipelined(int max_frames) {
    struct Item {
        Frame::ptr frame;  // nullptr: the end of the train (or a failure, with status != YV_OK)
        int index = -1;
        int status = YV_OK;
    };
    std::mutex mu;
    std::condition_variable cv_put, cv_get;
    std::deque<Item> q;
    bool stop = false;
    double worker_features = 0, worker_read = 0;
    const size_t depth = (size_t)pipeline_depth_;
    // PNG decoding (the reference's cv::imread) is the longest per-frame step on the host: the worker keeps the next
    // `readers` frames decoding on their own threads and consumes them in path-train order, so ids stay sequential
    const int readers = std::max(1, pipeline_readers_);
    if (!worker_dev_) worker_dev_ = std::make_unique<Device>(pipeline_device_);  // a second run: made again here
    if (!side_lane_) side_lane_ = std::make_unique<SideLane>(pipeline_device_);
    side_ = side_lane_.get();
    peek_next_ = [&]() -> Frame::ptr {
        std::lock_guard<std::mutex> lk(mu);
        return q.empty() ? nullptr : q.front().frame;
    };
    std::thread worker([&]() {
        Device& wdev = *worker_dev_;
        int st = wdev.ok() ? YV_OK : wdev.status();
        std::unique_ptr<FastDetector> wfd;
        std::unique_ptr<Brief> wbrief;
        if (st == YV_OK) {
            wfd = std::make_unique<FastDetector>(wdev, 12, 50);
            wbrief = std::make_unique<Brief>(wdev, 256);
            if (!wbrief->setOffsets(pipeline_offsets_)) st = wbrief->status() != YV_OK ? wbrief->status() : YV_ERR_INVALID;
            if (st == YV_OK) st = wfd->status();
        }
        int produced = 0;
        const size_t n_train = leftPathTrain.size();
        const size_t limit = max_frames < 0 ? n_train : std::min(n_train, train_it_ + (size_t)max_frames);
        auto push = [&](Item&& it) -> bool {  // false: the tracking thread stopped the pipeline
            std::unique_lock<std::mutex> lk(mu);
            cv_put.wait(lk, [&]() { return stop || q.size() < depth; });
            if (stop) return false;
            q.push_back(std::move(it));
            lk.unlock();
            cv_get.notify_one();
            return true;
        };
        if (pipeline_gpu_batch_ > 0) {
            // GPU look-ahead: batch j + 1 is read and enqueued on the GPU before batch j's frames are handed over
            std::unique_ptr<GpuLookahead> la;
            if (st == YV_OK) {
                la = std::make_unique<GpuLookahead>(wdev.ctx(), basePath_ + seqNo_, pipeline_gpu_batch_);
                st = la->status();  // (the worker context's BRIEF offsets were set above)
            }
            size_t next = train_it_;
            auto launch_next = [&]() -> int {
                const int n = (int)std::min((size_t)pipeline_gpu_batch_, limit - next);
                const double t0 = now_s();
                const int s = la->launch((int)next, n, readers);
                worker_read += now_s() - t0;
                next += (size_t)n;
                return s;
            };
            if (st == YV_OK) st = launch_next();
            bool done = false;
            while (!done) {
                std::vector<Frame::ptr> frames;
                if (st == YV_OK) {
                    const double t0 = now_s();
                    st = la->collect(frames);
                    worker_features += now_s() - t0;
                }
                if (st == YV_OK && next < limit) st = launch_next();
                bool ended = st != YV_OK || frames.empty();
                for (auto& f : frames) {
                    Item it;
                    it.status = st;
                    if (f && train_it_ >= limit) {
                        // never more frames than the train holds: a look-ahead that hands a batch over twice (the
                        // round-4 r04c6 hang: collect() returned the last batch again once nothing was launched, and
                        // the loop never ended) fails the run instead
                        std::cerr << "yavo: GPU look-ahead handed over frame " << train_it_ << " of a " << limit
                                  << "-frame train" << std::endl;
                        it.status = YV_ERR_INVALID;
                        f = nullptr;
                    }
                    if (f) {
                        it.index = (int)train_it_;
                        train_it_++;
                        f->frameID = Frame::createFrameID();
                        it.frame = f;
                    }
                    const bool last = !it.frame;
                    if (!push(std::move(it))) {
                        done = true;
                        break;
                    }
                    if (last) {
                        done = true;
                        break;
                    }
                }
                if (!done && ended) {
                    Item it;
                    it.status = st;
                    push(std::move(it));
                    done = true;
                }
            }
            return;
        }
        std::deque<std::future<Frame::ptr>> ahead;  // decodes of frames next_read - ahead.size() .. next_read - 1
        size_t next_read = train_it_;
        auto refill = [&]() {
            while (ahead.size() < (size_t)readers && next_read < limit) {
                const std::string path = leftPathTrain[next_read++];
                ahead.push_back(std::async(std::launch::async, [path]() { return readFrame(path); }));
            }
        };
        while (true) {
            Item it;
            it.status = st;
            if (st == YV_OK && (max_frames < 0 || produced < max_frames)) {
                // getNextFrame, its decode done ahead (only this thread advances the path train)
                refill();
                if (!ahead.empty()) {
                    const double t0 = now_s();
                    it.frame = ahead.front().get();
                    ahead.pop_front();
                    refill();
                    worker_read += now_s() - t0;
                    // the index travels with the item: only the tracking thread sets currentFrameId_, and
                    // train_it_ is advanced by this thread alone while the pipeline runs
                    if (it.frame) {
                        it.index = (int)train_it_;
                        train_it_++;
                        it.frame->frameID = Frame::createFrameID();
                    }
                }
                if (it.frame) {
                    const double t0 = now_s();
                    auto features = wfd->getFastFeatures(*it.frame);
                    it.status = wfd->status();
                    if (it.status == YV_OK) {
                        wbrief->computeBrief(features, *it.frame);
                        it.status = wbrief->status();
                    }
                    worker_features += now_s() - t0;
                    if (it.status != YV_OK) it.frame = nullptr;
                }
            }
            const bool last = !it.frame;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_put.wait(lk, [&]() { return stop || q.size() < depth; });
                if (stop) break;
                q.push_back(std::move(it));
            }
            cv_get.notify_one();
            if (last) break;
            ++produced;
        }
        for (auto& f : ahead) f.wait();  // no decode outlives the loop
    });
    bool stalled = false;
    while (true) {
        Item it;
        {
            const double t0 = now_s();
            std::unique_lock<std::mutex> lk(mu);
            // a bounded wait: no frame's read + detect + describe takes this long, so a worker that delivers nothing
            // is reported and the run ends non-zero instead of blocking
            if (!cv_get.wait_for(lk, std::chrono::seconds(kPipelineStallSeconds), [&]() { return !q.empty(); })) {
                stalled = true;
                break;
            }
            it = std::move(q.front());
            q.pop_front();
            t_wait += now_s() - t0;
        }
        cv_put.notify_one();
        if (!it.frame) {
            if (it.status != YV_OK) gpu(it.status, "insertFrameFeatures (pipeline worker)");
            break;
        }
        currentFrameId_ = it.index;
        addFrame(it.frame);
        if (gpu_status_ != YV_OK) break;
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
    }
    cv_put.notify_all();
    if (stalled) {
        std::cerr << "yavo: the pipeline worker delivered no frame for " << kPipelineStallSeconds << " s" << std::endl;
        gpu_status_ = YV_ERR_HIP;
        std::cout.flush();
        std::cerr.flush();
        std::_Exit(3);  // the worker may be inside a call that never returns: do not wait for it
    }
    worker.join();
    peek_next_ = nullptr;
    dropLKAhead(lk_ahead_);
    dropLKAhead(lk_cur_);
    side_ = nullptr;
    side_lane_.reset();  // runs what is still queued
    resolvePendingF(true);
    t_features += worker_features;
    t_read += worker_read;  // in the pipelined loop: the worker waiting for the next decoded frame
}

// wait = false: only the side-lane calls that have finished (polled at every getFRANSAC, so a failing side lane stops
// tracking at the next reinit frame as a failure on the tracking context does); wait = true: all of them (end of run)
void LoopHandler::resolvePendingF(bool wait) {
    size_t keep = 0;
    for (size_t i = 0; i < pending_f_.size(); ++i) {
        auto& p = pending_f_[i];
        if (!wait && p.second.wait_for(std::chrono::seconds(0)) != std::future_status::ready) {
            if (keep != i) pending_f_[keep] = std::move(p);
            ++keep;
            continue;
        }
        const FResult r = p.second.get();
        prim_.f_ransac += r.seconds;  // on the side lane, beside the tracking thread
        if (!gpu(r.status, "getFRANSAC (side lane)")) continue;
        if (p.first < events_.size()) events_[p.first].f_inliers = r.inliers;
    }
    pending_f_.resize(keep);
}

}  // namespace yavo_fe
