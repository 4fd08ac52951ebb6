// frontend.cpp -- the reference's operator classes over the C ABI (see frontend.hpp).
#include "frontend.hpp"

#include <iostream>
#include <random>

namespace yavo_fe {

Device::Device(int device) {
    status_ = yv_create(device, &ctx_);
    if (status_ != YV_OK) {
        std::cerr << "yavo: no GPU context (" << yv_status_string(status_) << ")" << std::endl;
        ctx_ = nullptr;
    }
}

Device::~Device() {
    if (ctx_) yv_destroy(ctx_);
}

FastDetector::FastDetector(Device& dev, int minDetectionThreshold, uint8_t intensityThreshold)
    : dev_(dev), minDetectionThreshold_(minDetectionThreshold), intensityThreshold_(intensityThreshold) {
    // include/FastDetector.hpp:32-38: bresRadius 3, intensityThreshold forced to 40, 2000 corners
    if (dev_.ok()) status_ = yv_set_fast_params(dev_.ctx(), 40, 2000);
}

std::vector<Point> FastDetector::getFastFeatures(const Image& img) {
    std::vector<Point> out;
    resp_.clear();
    ncand_ = 0;
    if (!dev_.ok()) {
        status_ = YV_ERR_NODEVICE;
        return out;
    }
    const int max_kp = 2000;
    std::vector<int32_t> rc(2 * max_kp);
    resp_.resize(max_kp);
    int n = 0;
    status_ = yv_detect(dev_.ctx(), img.data.data(), img.rows, img.cols, img.cols, max_kp, rc.data(),
                        resp_.data(), &n, &ncand_);
    if (status_ != YV_OK) {
        std::cerr << "yavo: getFastFeatures failed: " << yv_status_string(status_) << std::endl;
        resp_.clear();
        return out;
    }
    if (ncand_ == 0) std::cout << "No corners found" << std::endl;  // src/FastDetector.cc:364-366
    resp_.resize(n);
    out.resize(n);
    for (int i = 0; i < n; ++i) out[i] = Point{rc[2 * i], rc[2 * i + 1]};
    return out;
}

Brief::Brief(Device& dev, int numTests) : dev_(dev), patchSize_(numTests) {}

std::vector<int8_t> Brief::preComputeOffsets(uint32_t seed) {
    // src/BriefDescriptor.cc:4-20 with the random_device seed made explicit
    std::mt19937 generator(seed);
    std::uniform_int_distribution<int> dist(-8, 8);
    std::vector<int8_t> v(256 * 4);
    for (auto& o : v) o = (int8_t)dist(generator);
    return v;
}

bool Brief::setOffsets(const std::vector<int8_t>& offsets) {
    if (!dev_.ok() || offsets.size() != 256 * 4) return false;
    status_ = yv_set_brief_offsets(dev_.ctx(), offsets.data());
    return status_ == YV_OK;
}

void Brief::computeBrief(const std::vector<Point>& pts, Image& img) {
    if (!dev_.ok()) {
        status_ = YV_ERR_NODEVICE;
        return;
    }
    std::vector<int32_t> rc(2 * pts.size());
    for (size_t i = 0; i < pts.size(); ++i) {
        rc[2 * i] = pts[i].x;
        rc[2 * i + 1] = pts[i].y;
    }
    std::vector<KeyPoint> out(pts.size());
    int m = 0;
    status_ = yv_describe(dev_.ctx(), img.data.data(), img.rows, img.cols, img.cols, rc.data(), (int)pts.size(),
                          out.data(), &m);
    if (status_ != YV_OK) {
        std::cerr << "yavo: computeBrief failed: " << yv_status_string(status_) << std::endl;
        return;
    }
    out.resize(m);
    img.keypoints.insert(img.keypoints.end(), out.begin(), out.end());  // appends, as the reference
}

std::vector<Matches> Brief::matchFeatures(Image& img1, Image& img2) {
    std::vector<Matches> out(img1.keypoints.size());
    if (!dev_.ok()) {
        status_ = YV_ERR_NODEVICE;
        return {};
    }
    status_ = yv_match_features(dev_.ctx(), img1.keypoints.data(), (int)img1.keypoints.size(),
                                img2.keypoints.data(), (int)img2.keypoints.size(), out.data());
    if (status_ != YV_OK) {
        std::cerr << "yavo: matchFeatures failed: " << yv_status_string(status_) << std::endl;
        return {};
    }
    return out;
}

void Brief::removeOutliers(std::vector<Matches>& matches, std::vector<Matches>& newMatches, int threshold) {
    if (!dev_.ok()) {
        status_ = YV_ERR_NODEVICE;
        return;
    }
    std::vector<Matches> out(matches.size());
    int n = 0;
    status_ = yv_filter_matches(dev_.ctx(), matches.data(), (int)matches.size(), threshold, out.data(), &n);
    if (status_ != YV_OK) {
        std::cerr << "yavo: removeOutliers failed: " << yv_status_string(status_) << std::endl;
        return;
    }
    out.resize(n);
    newMatches.insert(newMatches.end(), out.begin(), out.end());
}

}  // namespace yavo_fe
