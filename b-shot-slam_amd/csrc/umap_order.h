// umap_order.h -- the iteration order of a libstdc++ std::unordered_map with unique keys, restated
// over flat arrays so that it runs inside a GPU kernel (and, compiled by g++, in the CPU test that
// checks it against the real container). The reference's map blocks are
// std::unordered_map<Vector3f, Keypoint::Ptr, MapHasher> (include/mymap.h:11-25); Map::getKeypoints
// concatenates a block's entries in that order (src/mymap.cpp:28-74), and the order decides the
// first-index ties of the Hamming match.
//
// What is restated (libstdc++ bits/hashtable.h, _Prime_rehash_policy with max_load_factor 1):
//  * a node is inserted at the BEGINNING of its bucket: after the bucket's "before" node when the
//    bucket is non-empty, else at the front of the singly linked list, the old front's bucket then
//    pointing at the new node (_M_insert_bucket_begin);
//  * before inserting element n+1 the table rehashes when n + 1 > next_resize (_M_need_rehash); the
//    bucket counts follow the chain measured on this image's libstdc++ (1 -> 13 -> 29 -> 59 -> ...,
//    tests/test_host.py checks the restatement against the container itself);
//  * a rehash walks the list in order and re-links each node at the front of the list when its new
//    bucket is empty, else after its bucket's before node (_M_rehash_aux, unique keys);
//  * bucket index = hash code % bucket count.
// State per map: n (elements), bkt (bucket count), next_resize; arrays ord[n] (member ids in
// iteration order), pos[member] (its index in ord), code[member] (hash code), buckets[bkt] (member id
// of the bucket's before node, UM_BB for the list head, UM_EMPTY for none). Members are numbered in
// insertion order (0, 1, ...). Replacing the value of an existing key changes nothing here.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define UM_HD __host__ __device__
#else
#define UM_HD
#endif

namespace um {

constexpr int UM_EMPTY = -1;
constexpr int UM_BB = -2;

struct State {
    int n;
    int bkt;
    int next_resize;
};

// bucket counts taken when element `at` is inserted (measured: tools/umap_chain, test_host.py)
UM_HD inline int next_bucket_count(int bkt) {
    const int chain[] = {1, 13, 29, 59, 127, 257, 541, 1109, 2357, 5087, 10273, 20753, 42043, 85229, 172933,
                         351061, 712697, 1447153, 2938679, 5967347, 12117689, 24607243, 49969847};
    for (int i = 0; i + 1 < (int)(sizeof(chain) / sizeof(chain[0])); ++i)
        if (chain[i] == bkt) return chain[i + 1];
    return -1;  // beyond the table (not reached: blocks stay far smaller)
}

UM_HD inline State initial() { return State{0, 1, 0}; }

// true when inserting one more element rehashes; *nb = the new bucket count
UM_HD inline bool need_rehash(State& s, int* nb) {
    if (s.n + 1 <= s.next_resize) return false;
    // min_bkts = max(n + 1, next_resize ? 0 : 11) >= bkt always holds here (next_resize == bkt)
    *nb = next_bucket_count(s.bkt);
    return true;
}

// Rehash to nb buckets. nxt: scratch of >= n ints (a singly linked list over member ids).
UM_HD inline void rehash(State& s, int nb, int* ord, int* pos, const uint64_t* code, int* buckets, int* nxt) {
    for (int b = 0; b < nb; ++b) buckets[b] = UM_EMPTY;
    int head = UM_EMPTY, bbegin = 0;
    for (int i = 0; i < s.n; ++i) {
        const int p = ord[i];
        const int b = (int)(code[p] % (uint64_t)nb);
        if (buckets[b] == UM_EMPTY) {
            nxt[p] = head;
            head = p;
            buckets[b] = UM_BB;
            if (nxt[p] != UM_EMPTY) buckets[bbegin] = p;
            bbegin = b;
        } else if (buckets[b] == UM_BB) {
            // the bucket's first node is the list head: p goes in front of it
            nxt[p] = head;
            head = p;
        } else {
            const int before = buckets[b];
            nxt[p] = nxt[before];
            nxt[before] = p;
        }
    }
    int i = 0;
    for (int p = head; p != UM_EMPTY; p = nxt[p]) { ord[i] = p; pos[p] = i; ++i; }
    s.bkt = nb;
    s.next_resize = nb;
}

// list position the new member x takes (and the bucket bookkeeping), before the shift of ord
UM_HD inline int insert_position(State& s, int x, const int* ord, const int* pos, const uint64_t* code, int* buckets) {
    const int b = (int)(code[x] % (uint64_t)s.bkt);
    if (buckets[b] != UM_EMPTY) {
        const int before = buckets[b];
        return before == UM_BB ? 0 : pos[before] + 1;
    }
    if (s.n > 0) buckets[(int)(code[ord[0]] % (uint64_t)s.bkt)] = x;
    buckets[b] = UM_BB;
    return 0;
}

// the whole insert of a new member x (one thread): rehash if due, then link at its bucket's begin
UM_HD inline void insert(State& s, int x, int* ord, int* pos, const uint64_t* code, int* buckets, int* nxt) {
    int nb;
    if (need_rehash(s, &nb)) rehash(s, nb, ord, pos, code, buckets, nxt);
    const int at = insert_position(s, x, ord, pos, code, buckets);
    for (int i = s.n; i > at; --i) { ord[i] = ord[i - 1]; pos[ord[i]] = i; }
    ord[at] = x;
    pos[x] = at;
    s.n += 1;
}

}  // namespace um
