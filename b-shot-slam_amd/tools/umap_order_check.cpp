// umap_order_check.cpp -- checks csrc/umap_order.h against this image's libstdc++ std::unordered_map:
// the reference's block type (unordered_map<Vector3f, ., MapHasher>, include/mymap.h:11-25) filled
// with random 10 mm-grid keys (with repeats), iteration orders compared after every insert.
// Built and run by tests/test_host.py (no GPU). Exit 0 = identical orders.
#include <cmath>
#include <cstdio>
#include <random>
#include <unordered_map>
#include <vector>

#include "../csrc/umap_order.h"
#include "../../include/bshot/types.h"

struct Hasher {  // include/mymap.h MapHasher over the shim's Vector3f (Eigen redux order)
    unsigned long operator()(const myslam::Vector3f& p) const { return (unsigned long)std::fabs(std::round(p.sum())); }
};

template <typename I, typename C>
static int run(int trials, unsigned seed) {
    std::mt19937 rng(seed);
    for (int t = 0; t < trials; ++t) {
        const int target = 1 + (int)(rng() % (t < 20 ? 6000u : 700u));
        const float span = (float)(100 + rng() % 10000);
        std::unordered_map<myslam::Vector3f, int, Hasher> ref;
        std::vector<myslam::Vector3f> keys;
        std::vector<I> ord, pos, bk, nxt;
        std::vector<C> code;
        um::State s = um::initial();
        std::uniform_real_distribution<float> U(-span, span);
        for (int i = 0; i < target; ++i) {
            myslam::Vector3f p((float)((int)std::trunc(U(rng) / 10.f) * 10), (float)((int)std::trunc(U(rng) / 10.f) * 10),
                               (float)((int)std::trunc(U(rng) / 100.f) * 10));
            if (i > 0 && rng() % 7 == 0) p = keys[rng() % keys.size()];  // an existing key: value replaced only
            const bool is_new = ref.find(p) == ref.end();
            ref[p] = i;
            if (!is_new) continue;
            const int x = (int)keys.size();
            keys.push_back(p);
            code.push_back((C)Hasher()(p));
            ord.resize(keys.size());
            pos.resize(keys.size());
            nxt.resize(keys.size());
            int nb;
            um::State probe = s;
            const int need = um::need_rehash(probe, &nb) ? nb : s.bkt;
            if ((int)bk.size() < need) bk.resize(need);
            um::insert(s, x, ord.data(), pos.data(), code.data(), bk.data(), nxt.data());
            if ((size_t)s.bkt != ref.bucket_count()) {
                std::printf("trial %d insert %d: bucket count %d vs %zu\n", t, x, s.bkt, ref.bucket_count());
                return 1;
            }
            int k = 0;
            for (auto& e : ref) {
                const myslam::Vector3f& q = keys[ord[k]];
                if (!(q == e.first)) {
                    std::printf("trial %d after %d keys: order differs at %d\n", t, x + 1, k);
                    return 1;
                }
                ++k;
            }
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 200;
    // int / uint64 (the restatement as written) and ushort / uint32 (the GPU map's LDS image)
    if (run<int, uint64_t>(trials, 7) || run<unsigned short, uint32_t>(trials, 11)) return 1;
    std::printf("umap order: %d trials x 2 index types identical\n", trials);
    return 0;
}
