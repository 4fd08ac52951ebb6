// Test infrastructure (the oracle): libstdc++ std::sort of the reference's corner list, for the "sort ties"
// diagnostic of SURVEY.md section 7 hard part 2.  FastDetector::getFastFeatures (src/FastDetector.cc:343-368) sorts
// its scan-ordered corners with std::sort(begin, end, [](a, b) { return a.cornerResponse > b.cornerResponse; }) and
// keeps the first fastCornerNumThreshold.  std::sort is unstable, so corners with equal responses may come out in
// any order; the product (and the oracle's or_fast_detect) use the canonical order instead: response descending,
// then row-major index ascending (= a stable sort of the scan order).  This entry point runs the reference's
// actual call on the same list so the tools can count where the two orders (and the 2000-corner cuts) differ.
#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <vector>

namespace {
struct FastFeature {  // include/FastDetector.hpp: the point (row, col) and its Harris score
    int x, y;
    float cornerResponse;
};
}  // namespace

// idx[n]: row-major pixel indices in scan order, resp[n] their responses; writes the first min(n, K) indices of the
// std::sort result to out_idx and returns that count.
extern "C" int or_std_sort_cut(const int32_t* idx, const float* resp, int n, int W, int K, int32_t* out_idx) {
    std::vector<FastFeature> v((size_t)n);
    for (int i = 0; i < n; ++i) v[(size_t)i] = FastFeature{idx[i] / W, idx[i] % W, resp[i]};
    std::sort(v.begin(), v.end(),
              [](const FastFeature& a, const FastFeature& b) { return a.cornerResponse > b.cornerResponse; });
    const int m = n < K ? n : K;
    for (int i = 0; i < m; ++i) out_idx[i] = v[(size_t)i].x * W + v[(size_t)i].y;
    return m;
}

// The literal mode's ring (CPU baseline only): FastDetector::getBresenhamCirclePoints (src/FastDetector.cc:50-112)
// with the reference's containers, so the per-pixel cost includes what the reference pays for them: a returned
// std::vector of points (no reserve, push_back growth), a fresh std::vector from getAllSymPoints on every loop
// iteration (src/FastDetector.cc:114-116), and two std::set whose comparators order by .second only
// (src/FastDetector.cc:19-45: pairs with equal .second are equivalent, so their second insert is dropped).  The output
// is the same ring as or_bresenham_ring's (tests/test_oracle_fast.py checks it).
#include <set>
#include <utility>
namespace {
struct RingPoint {
    int x, y;
};
bool ring_comp_first(std::pair<int, int> a, std::pair<int, int> b) { return a.second < b.second; }
bool ring_comp_sec(std::pair<int, int> a, std::pair<int, int> b) { return a.second > b.second; }
std::vector<RingPoint> ring_sym_points(int x, int y) {
    return {{x, y}, {y, x}, {y, -x}, {x, -y}, {-x, -y}, {-y, -x}, {-y, x}, {-x, y}};
}
}  // namespace

extern "C" void or_bresenham_ring_stl(int xc, int yc, int out[16][2]) {
    const int bresRadius = 3;  // include/FastDetector.hpp:34
    int xLoop = 0, yLoop = bresRadius, d = 3 - 2 * bresRadius;
    std::vector<RingPoint> circlePoints;
    std::set<std::pair<int, int>, decltype(&ring_comp_first)> ordFirstHalf(&ring_comp_first);
    std::set<std::pair<int, int>, decltype(&ring_comp_sec)> ordSecHalf(&ring_comp_sec);
    while (yLoop >= xLoop) {
        xLoop++;
        if (d <= 0) {
            d = d + 4 * xLoop + 6;
        } else {
            yLoop--;
            d = d + 4 * (xLoop - yLoop) + 10;
        }
        const std::vector<RingPoint> sym = ring_sym_points(xLoop, yLoop);
        for (size_t i = 0; i < sym.size(); i++) {
            const int xAct = sym[i].x >= 0 ? xc + std::abs(sym[i].x) : xc - std::abs(sym[i].x);
            const int yAct = sym[i].y >= 0 ? yc - std::abs(sym[i].y) : yc + std::abs(sym[i].y);
            if (sym[i].x >= 0) ordFirstHalf.insert(std::make_pair(xAct, yAct));
            else ordSecHalf.insert(std::make_pair(xAct, yAct));
        }
    }
    ordFirstHalf.insert(std::make_pair(xc + bresRadius, yc));
    ordSecHalf.insert(std::make_pair(xc - bresRadius, yc));
    circlePoints.push_back({xc, yc - bresRadius});
    for (const auto& v : ordFirstHalf) circlePoints.push_back({v.first, v.second});
    circlePoints.push_back({xc, yc + bresRadius});
    for (const auto& v : ordSecHalf) circlePoints.push_back({v.first, v.second});
    for (size_t k = 0; k < 16 && k < circlePoints.size(); ++k) {
        out[k][0] = circlePoints[k].x;
        out[k][1] = circlePoints[k].y;
    }
}
