// frontend.hpp -- C++ host side above the C ABI: the reference's operator classes, same names and
// argument meaning, backed by libyavo.so (gfx950).  This is what LoopHandler
// (/root/reference/src/LoopHandler.cc:468-485, 532-567) calls; INTEGRATION.md shows the same calls
// patched into the reference's own classes.
//
// Types: cv::Mat / cv::Point are replaced by the PODs below (the reference's Image keeps a CV_8UC1
// Mat and a std::vector<KeyPoint>; src/Image.cc, include/BriefDescriptor.hpp:11-39).  KeyPoint and
// Matches are byte-identical to the reference (yv_keypoint / yv_match).
// Errors: the reference reports failure by empty results and stdout; these classes do
// the same (empty vectors, message on std::cerr) and keep the last yavo status in status().
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/yavo/yavo.h"

namespace yavo_fe {

using KeyPoint = yv_keypoint;
using Matches = yv_match;

struct Point {  // cv::Point as the reference uses it: x = row, y = column
    int x = 0, y = 0;
};

struct Image {  // Image / Frame: an 8-bit grey image plus the keypoints computeBrief appends
    int rows = 0, cols = 0;
    std::vector<uint8_t> data;  // rows * cols, continuous (getPixelVal(i, j) = data[i*cols + j])
    std::vector<KeyPoint> keypoints;
    int getH() const { return rows; }
    int getW() const { return cols; }
    uint8_t getPixelVal(int i, int j) const { return data[(size_t)i * cols + j]; }
};

// One GPU context shared by the operator objects of a thread (the reference is single-threaded).
class Device {
public:
    explicit Device(int device = 0);
    ~Device();
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    yv_ctx* ctx() const { return ctx_; }
    bool ok() const { return ctx_ != nullptr; }
    int status() const { return status_; }

private:
    yv_ctx* ctx_ = nullptr;
    int status_ = YV_OK;
};

// FastDetector (include/FastDetector.hpp:17-55): FAST-12 on the 16-pixel ring, threshold 40, Harris
// ranking, top-2000.  The (12, 50) constructor arguments are accepted and, as in the reference,
// ignored except for being stored.
class FastDetector {
public:
    FastDetector(Device& dev, int minDetectionThreshold = 12, uint8_t intensityThreshold = 50);
    std::vector<Point> getFastFeatures(const Image& img);
    const std::vector<float>& lastResponses() const { return resp_; }
    int lastCandidates() const { return ncand_; }
    int status() const { return status_; }

private:
    Device& dev_;
    int minDetectionThreshold_;
    uint8_t intensityThreshold_;  // the reference overrides it with 40 (include/FastDetector.hpp:35)
    std::vector<float> resp_;
    int ncand_ = 0;
    int status_ = YV_OK;
};

// Brief (include/BriefDescriptor.hpp:41-68): 256 tests; offsets come from the caller (the reference
// draws them from std::random_device, src/BriefDescriptor.cc:4-20; precomputeOffsets(seed) reproduces
// that algorithm with a fixed seed).
class Brief {
public:
    Brief(Device& dev, int numTests = 256);
    static std::vector<int8_t> preComputeOffsets(uint32_t seed);
    bool setOffsets(const std::vector<int8_t>& offsets);  // 256 x 4
    void computeBrief(const std::vector<Point>& detectedCornerPoints, Image& img);
    std::vector<Matches> matchFeatures(Image& img1, Image& img2);
    void removeOutliers(std::vector<Matches>& matches, std::vector<Matches>& newMatches, int threshold);
    int status() const { return status_; }

private:
    Device& dev_;
    int patchSize_;
    int status_ = YV_OK;
};

}  // namespace yavo_fe
