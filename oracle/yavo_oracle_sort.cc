// Test infrastructure (the oracle): libstdc++ std::sort of the reference's corner list, for the "sort ties"
// diagnostic of SURVEY.md section 7 hard part 2.  FastDetector::getFastFeatures (src/FastDetector.cc:343-368) sorts
// its scan-ordered corners with std::sort(begin, end, [](a, b) { return a.cornerResponse > b.cornerResponse; }) and
// keeps the first fastCornerNumThreshold.  std::sort is unstable, so corners with equal responses may come out in
// any order; the product (and the oracle's or_fast_detect) use the canonical order instead: response descending,
// then row-major index ascending (= a stable sort of the scan order).  This entry point runs the reference's
// actual call on the same list so the tools can count where the two orders (and the 2000-corner cuts) differ.
#include <algorithm>
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
