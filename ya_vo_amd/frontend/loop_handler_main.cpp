// loop_handler_main.cpp -- the reference's app entry (src/main.cc: LoopHandler(config) + runVO) over libyavo.so,
// without the viewer thread.
//
// usage: yavo_loop_handler CONFIG.json [--frames N] [--poses KITTI.txt] [--poses-bin POSES.bin]
//                                      [--events EVENTS.bin] [--offsets-seed S] [--device D] [--check-config]
//                                      [--pipeline DEPTH] [--readers N] [--gpu-decode B]
//   --check-config   no GPU: print the parsed configuration, the path train and the first frames as JSON (the
//                    reference's LoopHandlerTest cases: stereoStatus, getSeqNo, getLeftImagesPath,
//                    getLeftTrainLength, getNextFrame dimensions, frame ids)
//   --poses-bin      n x 7 doubles (SE3d::data() of T_cw per frame), exact
//   --events         n x 9 int32 (FrameEvent fields)
//   --offsets-seed   BRIEF's preComputeOffsets seed (the reference uses std::random_device; default 42)
//   --pipeline       DEPTH > 0: frame k + 1's read + detect + describe on a worker thread (own GPU context) while
//                    frame k is tracked (LoopHandler::setPipeline); the results are the serial loop's
//   --readers        pipelined: frames read + PNG-decoded ahead on their own threads (default 4)
//   --no-warmup      skip LoopHandler::warmup (every context's primitives called once before runVO)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>

#include "loop_handler.hpp"

using namespace yavo_fe;

static std::string json_escape(const std::string& s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') o.push_back('\\');
        o.push_back(c);
    }
    return o;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::cerr << "usage: " << argv[0] << " CONFIG.json [--frames N] [--poses KITTI.txt] [--poses-bin F] "
                  << "[--events F] [--offsets-seed S] [--device D] [--check-config]" << std::endl;
        return 2;
    }
    const std::string config = argv[1];
    int frames = -1, device = 0, pipeline = 0, readers = 4, gpu_decode = 0, warm = 1;
    uint32_t seed = 42;
    bool check = false;
    std::string poses_txt, poses_bin, events_bin;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : std::string(); };
        if (a == "--frames") frames = std::atoi(next().c_str());
        else if (a == "--poses") poses_txt = next();
        else if (a == "--poses-bin") poses_bin = next();
        else if (a == "--events") events_bin = next();
        else if (a == "--offsets-seed") seed = (uint32_t)std::strtoul(next().c_str(), nullptr, 10);
        else if (a == "--device") device = std::atoi(next().c_str());
        else if (a == "--pipeline") pipeline = std::atoi(next().c_str());
        else if (a == "--readers") readers = std::atoi(next().c_str());
        else if (a == "--gpu-decode") gpu_decode = std::atoi(next().c_str());
        else if (a == "--check-config") check = true;
        else if (a == "--no-warmup") warm = 0;
        else {
            std::cerr << "unknown option " << a << std::endl;
            return 2;
        }
    }

    if (check) {
        LoopHandler lh(config, nullptr);
        if (!lh.ok()) {
            std::cout << "{\"ok\": false, \"error\": \"" << json_escape(lh.error()) << "\"}" << std::endl;
            return 1;
        }
        std::cout << "{\"ok\": true, \"sequence\": \"" << json_escape(lh.getSeqNo()) << "\", \"stereo\": "
                  << (lh.stereoStatus() ? "true" : "false") << ", \"left_images_path\": \""
                  << json_escape(lh.getLeftImagesPath()) << "\", \"left_train_length\": " << lh.getLeftTrainLength()
                  << ", \"right_train_length\": " << lh.rightPathTrain.size() << ", \"K\": [";
        std::cout.precision(17);
        for (int i = 0; i < 9; ++i) std::cout << (i ? ", " : "") << lh.K()[i];
        std::cout << "], \"frames\": [";
        for (int k = 0; k < 3; ++k) {
            auto f = lh.getNextFrame();
            if (!f) break;
            std::cout << (k ? ", " : "") << "{\"id\": " << f->frameID << ", \"H\": " << f->getH()
                      << ", \"W\": " << f->getW() << "}";
        }
        std::cout << "]}" << std::endl;
        return 0;
    }

    Device dev(device);
    if (!dev.ok()) return 3;
    LoopHandler lh(config, &dev);
    if (!lh.ok()) {
        std::cerr << lh.error() << std::endl;
        return 1;
    }
    Brief offsets_setter(dev, 256);
    const std::vector<int8_t> offsets = Brief::preComputeOffsets(seed);
    if (!offsets_setter.setOffsets(offsets)) return 3;
    // every context is warmed before the loop (LoopHandler::warmup): kernels loaded, workspaces sized
    if (warm && !lh.warmup()) return 3;
    if (pipeline > 0) lh.setPipeline(pipeline, device, offsets, readers, gpu_decode);
    if (lh.gpuStatus() != YV_OK) return 3;

    const auto t0 = std::chrono::steady_clock::now();
    lh.runVO(frames);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (lh.gpuStatus() != YV_OK) return 4;

    const auto& traj = lh.trajectory();
    const int n = (int)traj.size();
    if (!poses_txt.empty()) {
        std::vector<double> flat(7 * (size_t)n);
        for (int k = 0; k < n; ++k) std::memcpy(&flat[7 * (size_t)k], traj[k].d, 7 * sizeof(double));
        if (yv_write_kitti_poses(poses_txt.c_str(), flat.data(), n) != YV_OK) return 5;
    }
    if (!poses_bin.empty()) {
        std::ofstream f(poses_bin, std::ios::binary);
        for (const auto& p : traj) f.write(reinterpret_cast<const char*>(p.d), 7 * sizeof(double));
    }
    if (!events_bin.empty()) {
        std::ofstream f(events_bin, std::ios::binary);
        for (const auto& e : lh.events()) {
            const int32_t v[9] = {e.frame, e.kind, e.keypoints, e.matches_kept, e.essential_found, e.tracked,
                                  e.inliers, e.new_landmarks, e.f_inliers};
            f.write(reinterpret_cast<const char*>(v), sizeof v);
        }
    }
    int n_init = 0, n_track = 0, n_reinit = 0;
    for (const auto& e : lh.events()) {
        n_init += e.kind == FrameEvent::INIT_MAP;
        n_track += e.kind == FrameEvent::TRACKED;
        n_reinit += e.kind == FrameEvent::REINIT;
    }
    std::cout << "{\"frames\": " << n << ", \"seconds\": " << dt << ", \"frames_per_s\": " << (dt > 0 ? n / dt : 0)
              << ", \"init\": " << n_init << ", \"tracked\": " << n_track << ", \"reinit\": " << n_reinit
              << ", \"keyframes\": " << lh.map->getFrames().size() << ", \"map_points\": " << lh.map->getMps().size()
              << ", \"seconds_features\": " << lh.t_features << ", \"seconds_init\": " << lh.t_init
              << ", \"seconds_track\": " << lh.t_track << ", \"seconds_reinit\": " << lh.t_reinit
              << ", \"seconds_read\": " << lh.t_read << ", \"seconds_wait\": " << lh.t_wait
              << ", \"seconds_warmup\": " << lh.t_warmup
              << ", \"pipeline\": " << pipeline << ", \"readers\": " << (pipeline > 0 ? readers : 0)
              << ", \"gpu_decode_batch\": " << (pipeline > 0 ? gpu_decode : 0) << ", \"primitives_s\": {"
              << "\"world2camera\": " << lh.primitiveTimes().world2camera << ", \"lk\": " << lh.primitiveTimes().lk
              << ", \"pose_lm\": " << lh.primitiveTimes().pose_lm << ", \"match_reinit\": " << lh.primitiveTimes().match
              << ", \"f_ransac\": " << lh.primitiveTimes().f_ransac
              << ", \"find_essential\": " << lh.primitiveTimes().find_essential
              << ", \"recover_pose\": " << lh.primitiveTimes().recover_pose << "}"
              << ", \"lk_ahead_frames\": " << lh.lk_ahead_frames << ", \"lk_ahead_s\": " << lh.lk_ahead_seconds << "}"
              << std::endl;
    return 0;
}
