// topk.cpp -- A2 keypoint selection: the last k elements of libstdc++ std::sort(SegRatio,
// comparator) (src/lidar_odometry.cpp:49-50,131-153) WITHOUT sorting everything.
//
// std::sort is introsort: median-of-3 quicksort partitions down to 16-element blocks (heapsort past
// 2*lg(n) levels), then one insertion-sort pass. Partitions never move an element across a cut and
// every element left of a cut is <= every element right of it, so the final insertion pass acts
// block-locally. Hence the contents of positions [n-k, n) depend only on the partition steps of
// ranges that intersect [n-k, n) and on the insertion sort of the blocks covering it. We replay
// exactly those steps (same pivot rule, same unguarded partition, same swaps) and skip every range
// that ends before n-k: O(n) expected instead of O(n log n), identical output including the order
// of equal ratios (the keypoint ORDER feeds descriptor indices, matching and RANSAC sampling).
// Validated against std::sort in tests/test_topk.py on tie-heavy inputs.
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

#include "../../include/bshot_abi.h"

namespace {

typedef std::pair<int, float> Elem;
struct Comp {
    bool operator()(const Elem& l, const Elem& r) const { return l.second < r.second; }
};

inline int lg(long n) { return (int)(sizeof(long) * 8 - 1 - __builtin_clzl((unsigned long)n)); }

inline void move_median_to_first(Elem* result, Elem* a, Elem* b, Elem* c) {
    Comp comp;
    if (comp(*a, *b)) {
        if (comp(*b, *c)) std::iter_swap(result, b);
        else if (comp(*a, *c)) std::iter_swap(result, c);
        else std::iter_swap(result, a);
    } else if (comp(*a, *c)) {
        std::iter_swap(result, a);
    } else if (comp(*b, *c)) {
        std::iter_swap(result, c);
    } else {
        std::iter_swap(result, b);
    }
}

inline Elem* unguarded_partition(Elem* first, Elem* last, Elem* pivot) {
    Comp comp;
    while (true) {
        while (comp(*first, *pivot)) ++first;
        --last;
        while (comp(*pivot, *last)) --last;
        if (!(first < last)) return first;
        std::iter_swap(first, last);
        ++first;
    }
}

// introsort loop restricted to ranges that reach into [top, end); records the leftmost
// leaf/heap-sorted block start that intersects the top region.
void introsort_top(Elem* first, Elem* last, int depth, Elem* top, Elem** block_lo) {
    while (last - first > 16) {
        if (last <= top) return;
        if (depth == 0) {
            std::partial_sort(first, last, last, Comp());
            if (first < *block_lo) *block_lo = first;
            return;
        }
        --depth;
        Elem* mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1);
        Elem* cut = unguarded_partition(first + 1, last, first);
        introsort_top(cut, last, depth, top, block_lo);
        last = cut;
    }
    if (last > top && first < *block_lo) *block_lo = first;
}

inline void unguarded_linear_insert(Elem* last) {
    Comp comp;
    Elem val = *last;
    Elem* next = last - 1;
    while (comp(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

}  // namespace

extern "C" int bshot_select_topk(const int32_t* idx, const float* ratio, int n, int k, int32_t* kp_idx,
                                 float* kp_ratio, int* k_out) {
    if (n < 0 || k < 0 || !k_out) return BSHOT_EINVAL;
    std::vector<Elem> v(n);
    for (int i = 0; i < n; ++i) v[i] = Elem(idx[i], ratio[i]);
    const int start = n >= k ? n - k : 0;
    if (n > 0) {
        Elem* first = v.data();
        Elem* last = first + n;
        Elem* top = first + start;
        Elem* block_lo = last;
        introsort_top(first, last, lg(n) * 2, top, &block_lo);
        if (block_lo - first < 16) {
            // small arrays: the guarded head of the final insertion pass is involved -> replay all
            std::vector<Elem> w(idx ? n : 0);
            for (int i = 0; i < n; ++i) w[i] = Elem(idx[i], ratio[i]);
            std::sort(w.begin(), w.end(), Comp());
            v.swap(w);
        } else {
            for (Elem* i = block_lo; i < last; ++i) unguarded_linear_insert(i);
        }
    }
    int m = 0;
    for (int i = start; i < n; ++i, ++m) {
        kp_idx[m] = v[i].first;
        kp_ratio[m] = v[i].second;
    }
    *k_out = m;
    return BSHOT_OK;
}
