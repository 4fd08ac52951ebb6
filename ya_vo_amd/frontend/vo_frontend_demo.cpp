// vo_frontend_demo.cpp -- the caller side of the hot path, shaped like LoopHandler:
//   takeVOStep -> insertFrameFeatures (getFastFeatures + computeBrief, src/LoopHandler.cc:468-485)
//   -> with a previous frame: matchFeatures(last, curr) + removeOutliers(20) (src/LoopHandler.cc:534-537)
// over a raw frame file, timing each call with steady_clock like the reference's own timers.
//
// usage: yavo_frontend_demo FRAMES.raw OFFSETS.bin OUT.bin
//   FRAMES.raw : int32 n, int32 H, int32 W, then n*H*W bytes
//   OUT.bin    : per frame int32 n_kp + KeyPoint[n_kp]; per consecutive pair int32 n + Matches[n]
//                + int32 n_f + Matches[n_f]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>

#include "frontend.hpp"

using namespace yavo_fe;

int main(int argc, char** argv) {
    if (argc != 4) {
        std::cerr << "usage: " << argv[0] << " FRAMES.raw OFFSETS.bin OUT.bin" << std::endl;
        return 2;
    }
    std::ifstream fin(argv[1], std::ios::binary);
    int32_t hdr[3];
    if (!fin.read(reinterpret_cast<char*>(hdr), sizeof hdr)) return 2;
    const int n = hdr[0], H = hdr[1], W = hdr[2];
    std::vector<int8_t> offsets(1024);
    std::ifstream foff(argv[2], std::ios::binary);
    if (!foff.read(reinterpret_cast<char*>(offsets.data()), 1024)) return 2;

    Device dev(0);
    if (!dev.ok()) return 3;
    FastDetector fd(dev, 12, 50);  // src/LoopHandler.cc:7
    Brief brief(dev, 256);
    if (!brief.setOffsets(offsets)) return 3;

    std::ofstream fout(argv[3], std::ios::binary);
    Image last;
    bool have_last = false;
    double t_feat = 0, t_desc = 0, t_match = 0;
    for (int k = 0; k < n; ++k) {
        Image cur;
        cur.rows = H;
        cur.cols = W;
        cur.data.resize((size_t)H * W);
        if (!fin.read(reinterpret_cast<char*>(cur.data.data()), (std::streamsize)cur.data.size())) return 2;
        auto t1 = std::chrono::steady_clock::now();
        auto features = fd.getFastFeatures(cur);
        auto t2 = std::chrono::steady_clock::now();
        brief.computeBrief(features, cur);
        auto t3 = std::chrono::steady_clock::now();
        t_feat += std::chrono::duration<double>(t2 - t1).count();
        t_desc += std::chrono::duration<double>(t3 - t2).count();
        if (fd.status() != YV_OK || brief.status() != YV_OK) return 4;
        int32_t nk = (int32_t)cur.keypoints.size();
        fout.write(reinterpret_cast<const char*>(&nk), 4);
        fout.write(reinterpret_cast<const char*>(cur.keypoints.data()), (std::streamsize)(nk * sizeof(KeyPoint)));
        if (have_last) {
            auto t4 = std::chrono::steady_clock::now();
            std::vector<Matches> matches = brief.matchFeatures(last, cur);
            std::vector<Matches> filterMatches;
            brief.removeOutliers(matches, filterMatches, 20);
            t_match += std::chrono::duration<double>(std::chrono::steady_clock::now() - t4).count();
            if (brief.status() != YV_OK) return 4;
            int32_t nm = (int32_t)matches.size(), nf = (int32_t)filterMatches.size();
            fout.write(reinterpret_cast<const char*>(&nm), 4);
            fout.write(reinterpret_cast<const char*>(matches.data()), (std::streamsize)(nm * sizeof(Matches)));
            fout.write(reinterpret_cast<const char*>(&nf), 4);
            fout.write(reinterpret_cast<const char*>(filterMatches.data()), (std::streamsize)(nf * sizeof(Matches)));
            std::cout << "frame " << k << ": " << features.size() << " corners, " << nk << " keypoints, "
                      << nf << "/" << nm << " matches kept" << std::endl;
        }
        last = std::move(cur);
        have_last = true;
    }
    std::cout << "Feat extraction cost time: " << t_feat / n << " seconds/frame." << std::endl;
    std::cout << "Descriptor generation cost time: " << t_desc / n << " seconds/frame." << std::endl;
    std::cout << "Matching cost time: " << (n > 1 ? t_match / (n - 1) : 0.0) << " seconds/pair." << std::endl;
    return 0;
}
