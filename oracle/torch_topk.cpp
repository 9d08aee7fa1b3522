// Oracle (test infrastructure only): torch.topk's CPU row selection, restated.
//
// The reference ranks every score row with torch.topk on the CPU
// (main.py:335,365,375: `torch.topk(scores[i], k)` for k = 1, 5, 10). With
// ColPali's bf16-quantised MaxSim sums exact ties are the rule, not the
// exception, so Recall@k depends on WHICH tied columns torch keeps and in what
// order. torch's CPU kernel (aten/src/ATen/native/cpu/SortingKernel.cpp,
// topk_impl_loop; not vendored in /root/reference -- torch is a third-party
// dependency of the reference, requirements.txt) fills a vector of
// (value, column) pairs (the value widened to the accumulate type, double for
// float) and, with comp(x, y) = x.value > y.value (NaN first):
//   * k * 64 <= n : std::partial_sort(q, q + k, q + n, comp)
//                   (libstdc++: heap select over the first k, then sort_heap);
//   * otherwise   : std::nth_element(q, q + k - 1, q + n, comp), then
//                   std::sort(q, q + k - 1, comp) when sorted
// and returns the first k pairs. This file calls the very same libstdc++
// algorithms with that element type and comparator. It is pinned by
// tests/golden/torch_topk.npz (torch.topk's own outputs on tie-heavy rows,
// written by tests/golden/make_goldens.py) and by the reference's own
// torch.topk results in tests/golden/colpali_full.npz.
//
// Build: oracle/Makefile -> oracle/libtorch_topk.so (C ABI, ctypes).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace {
using elem_t = std::pair<double, int64_t>;

inline bool greater_nan_first(const elem_t& x, const elem_t& y) {
    return (std::isnan(x.first) && !std::isnan(y.first)) || (x.first > y.first);
}

void topk_row(const float* s, int64_t n, int64_t k, int sort_k_minus_1, std::vector<elem_t>& q, int64_t* idx,
              float* val) {
    for (int64_t j = 0; j < n; ++j) q[j] = elem_t((double)s[j], j);
    if (k * 64 <= n) {
        std::partial_sort(q.begin(), q.begin() + k, q.begin() + n, greater_nan_first);
    } else {
        std::nth_element(q.begin(), q.begin() + (k - 1), q.begin() + n, greater_nan_first);
        std::sort(q.begin(), q.begin() + (sort_k_minus_1 ? k - 1 : k), greater_nan_first);
    }
    for (int64_t j = 0; j < k; ++j) {
        idx[j] = q[j].second;
        if (val) val[j] = (float)q[j].first;
    }
}
}  // namespace

extern "C" {
// scores [rows][ld] fp32 (the first n columns of each row), k <= n;
// idx [rows][k] int64 (+ val [rows][k] fp32, may be null) in torch.topk's order.
// sort_k_minus_1: 1 = sort the first k - 1 after nth_element (torch), 0 = the first k.
int oracle_torch_topk(const float* s, int64_t rows, int64_t n, int64_t ld, int64_t k, int sort_k_minus_1,
                      int64_t* idx, float* val) {
    if (k < 1 || k > n || ld < n) return 1;
    std::vector<elem_t> q((size_t)n);
    for (int64_t r = 0; r < rows; ++r)
        topk_row(s + r * ld, n, k, sort_k_minus_1, q, idx + r * k, val ? val + r * k : nullptr);
    return 0;
}
}
