// topk.cpp -- A2 keypoint selection: the last k elements of libstdc++ std::sort(SegRatio,
// comparator) (src/lidar_odometry.cpp:49-50,131-153) WITHOUT sorting everything.
//
// std::sort is introsort: median-of-3 quicksort partitions down to 16-element blocks (heapsort past
// 2*lg(n) levels), then one insertion-sort pass. Partitions never move an element across a cut and
// every element left of a cut is <= every element right of it, so the final insertion pass acts
// block-locally. Hence the contents of positions [n-k, n) depend only on the partition steps of
// ranges that intersect [n-k, n) and on the insertion sort of the blocks covering it. We replay
// exactly those steps (same pivot rule, same partition outcome, same swaps) and skip every range
// that ends before n-k: O(n) expected instead of O(n log n), identical output including the order
// of equal ratios (the keypoint ORDER feeds descriptor indices, matching and RANSAC sampling).
//
// The partition itself runs branch-free in blocks. libstdc++'s __unguarded_partition(first, last,
// pivot) swaps the i-th element from the left with !(v < p) (a "left stopper") with the i-th
// element from the right with !(p < v) (a "right stopper"; the pivot at first - 1 ends that scan)
// for i = 1, 2, ... as long as the left one lies before the right one, and returns
// min(L_m, R_(m-1)) for the first m where L_m >= R_m (R_0 = last): a swapped element is a stopper
// for the other scan, so the scans meet there. Blocks of stopper offsets (a flag per position, no
// data-dependent branch) find the same pairs in the same order; a block read after some swaps sees
// swapped values only past the meeting point, where they change neither the meeting test nor the
// returned cut (the cut takes the min with the last right position swapped). The scalar replay's
// per-element branches mispredicted on about half the elements of a sweep's 130k ratios (0.6 ms
// on the odometry's critical path).
// Validated against std::sort in tests/test_host.py on tie-heavy and adversarial inputs.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
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

constexpr int kBlock = 128;

// __unguarded_partition(first, last, first - 1) with the outcome of libstdc++'s loop (see above)
inline Elem* unguarded_partition_block(Elem* first, Elem* last) {
    const float p = (first - 1)->second;
    uint8_t lofs[kBlock], rofs[kBlock];
    Elem* lnext = first;  // next position the left blocks examine (upward)
    Elem* rnext = last;   // the right blocks examine rnext - 1, rnext - 2, ... down to first - 1
    Elem* lbase = first;
    Elem* rbase = last - 1;
    int nl = 0, il = 0, nr = 0, ir = 0;
    bool lend = false;  // the left scan ran past the range (no further left stopper inside it)
    Elem* last_b = last;
    while (true) {
        if (il == nl && !lend) {
            const long cnt = std::min<long>(kBlock, last - lnext);
            if (cnt <= 0) {
                lend = true;
            } else {
                lbase = lnext;
                nl = 0;
                for (long k = 0; k < cnt; ++k) {
                    lofs[nl] = (uint8_t)k;
                    nl += !(lbase[k].second < p);
                }
                il = 0;
                lnext += cnt;
            }
            continue;
        }
        if (ir == nr) {
            // the pivot at first - 1 is a right stopper: the right scan always finds one
            const long cnt = std::min<long>(kBlock, rnext - (first - 1));
            rbase = rnext - 1;
            nr = 0;
            for (long k = 0; k < cnt; ++k) {
                rofs[nr] = (uint8_t)k;
                nr += !(p < rbase[-k].second);
            }
            ir = 0;
            rnext -= cnt;
            continue;
        }
        Elem* b = rbase - rofs[ir];
        if (lend) return last_b;  // no left stopper left in the range: the scans meet at the last swap
        Elem* a = lbase + lofs[il];
        if (!(a < b)) return std::min(a, last_b);
        std::iter_swap(a, b);
        last_b = b;
        ++il;
        ++ir;
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
        Elem* cut = unguarded_partition_block(first + 1, last);
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

// the std::sort tail of v (n elements) -> out (its last min(n, k) elements, in order)
int topk_of(std::vector<Elem>& v, int k, int32_t* kp_idx, float* kp_ratio) {
    const int n = (int)v.size();
    const int start = n >= k ? n - k : 0;
    if (n > 0) {
        Elem* first = v.data();
        Elem* last = first + n;
        Elem* top = first + start;
        Elem* block_lo = last;
        introsort_top(first, last, lg(n) * 2, top, &block_lo);
        // the final insertion pass restricted to [block_lo, last): every element left of block_lo is
        // <= every element from it on, and insertion stops at equal keys, so no element crosses
        // block_lo and the pass there is a plain (guarded) insertion sort -- what libstdc++'s guarded
        // head [first, first + 16) and unguarded rest do to these positions
        Comp comp;
        for (Elem* i = block_lo + 1; i < last; ++i) {
            if (comp(*i, *block_lo)) {
                const Elem val = *i;
                std::move_backward(block_lo, i, i + 1);
                *block_lo = val;
            } else {
                unguarded_linear_insert(i);
            }
        }
    }
    int m = 0;
    for (int i = start; i < n; ++i, ++m) {
        kp_idx[m] = v[i].first;
        kp_ratio[m] = v[i].second;
    }
    return m;
}

}  // namespace

extern "C" int bshot_select_topk(const int32_t* idx, const float* ratio, int n, int k, int32_t* kp_idx,
                                 float* kp_ratio, int* k_out) {
    if (n < 0 || k < 0 || !k_out) return BSHOT_EINVAL;
    std::vector<Elem> v(n);
    for (int i = 0; i < n; ++i) v[i] = Elem(idx[i], ratio[i]);
    *k_out = topk_of(v, k, kp_idx, kp_ratio);
    return BSHOT_OK;
}

namespace bsh {

// the odometry's A2 straight from a sweep's ratio array (NaN = skipped, src/lidar_odometry.cpp:
// 121-122): the valid (index, ratio) pairs in index order, then their std::sort tail
int topk_from_ratios(const float* ratio, int n, int k, int32_t* kp_idx, float* kp_ratio, int* k_out, int* nv_out) {
    if (n < 0 || k < 0 || !k_out || !nv_out) return BSHOT_EINVAL;
    std::vector<Elem> v((size_t)(n > 0 ? n : 1));
    int nv = 0;
    for (int i = 0; i < n; ++i) {
        const float r = ratio[i];
        v[nv] = Elem(i, r);
        nv += r == r;  // branch-free compaction
    }
    v.resize(nv);
    *nv_out = nv;
    *k_out = topk_of(v, k, kp_idx, kp_ratio);
    return BSHOT_OK;
}

}  // namespace bsh
