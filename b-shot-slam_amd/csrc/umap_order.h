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
// The GPU map instantiates the index type as unsigned short and the code type as uint32_t (hash
// codes of 10 mm-grid keys fit); the CPU check runs both that and the int / uint64 form.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define UM_HD __host__ __device__
#else
#define UM_HD
#endif

namespace um {

// index arrays (ord, pos, buckets, scratch) may be int or a narrower unsigned type (the GPU map keeps
// them as ushort in LDS); the two sentinels are the type's all-ones and all-ones-minus-one
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

// Rehash to nb buckets. nxt: scratch of >= n entries (a singly linked list over member ids).
template <typename I, typename C>
UM_HD inline void rehash(State& s, int nb, I* ord, I* pos, const C* code, I* buckets, I* nxt) {
    const I E = (I)UM_EMPTY, BB = (I)UM_BB;
    for (int b = 0; b < nb; ++b) buckets[b] = E;
    I head = E;
    int bbegin = 0;
    for (int i = 0; i < s.n; ++i) {
        const I p = ord[i];
        const int b = (int)(code[p] % (C)nb);
        if (buckets[b] == E) {
            nxt[p] = head;
            head = p;
            buckets[b] = BB;
            if (nxt[p] != E) buckets[bbegin] = p;
            bbegin = b;
        } else if (buckets[b] == BB) {
            // the bucket's first node is the list head: p goes in front of it
            nxt[p] = head;
            head = p;
        } else {
            const I before = buckets[b];
            nxt[p] = nxt[before];
            nxt[before] = p;
        }
    }
    int i = 0;
    for (I p = head; p != E; p = nxt[p]) { ord[i] = p; pos[p] = (I)i; ++i; }
    s.bkt = nb;
    s.next_resize = nb;
}

// list position the new member x takes (and the bucket bookkeeping), before the shift of ord
template <typename I, typename C>
UM_HD inline int insert_position(State& s, int x, const I* ord, const I* pos, const C* code, I* buckets) {
    const I E = (I)UM_EMPTY, BB = (I)UM_BB;
    const int b = (int)(code[x] % (C)s.bkt);
    if (buckets[b] != E) {
        const I before = buckets[b];
        return before == BB ? 0 : (int)pos[before] + 1;
    }
    if (s.n > 0) buckets[(int)(code[ord[0]] % (C)s.bkt)] = (I)x;
    buckets[b] = BB;
    return 0;
}

// the whole insert of a new member x (one thread): rehash if due, then link at its bucket's begin
template <typename I, typename C>
UM_HD inline void insert(State& s, int x, I* ord, I* pos, const C* code, I* buckets, I* nxt) {
    int nb;
    if (need_rehash(s, &nb)) rehash(s, nb, ord, pos, code, buckets, nxt);
    const int at = insert_position(s, x, ord, pos, code, buckets);
    for (int i = s.n; i > at; --i) { ord[i] = ord[i - 1]; pos[ord[i]] = (I)i; }
    ord[at] = (I)x;
    pos[x] = (I)at;
    s.n += 1;
}

}  // namespace um
