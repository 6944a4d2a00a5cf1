// bshot_bits.h -- the public pieces of the reference's include/bshot_bits.h that the API exposes:
// minVect (first-index minimum, :6-20) and bshot_descriptor (std::bitset<352>, :23-27). The
// descriptor computation itself (class bshot, :30-281) runs on the GPU behind bshot_describe().
#pragma once
#include <bitset>
#include <cassert>
#include <cstdint>
#include <cstring>

template <typename T>
T minVect(const T* v, int n, int* ind = nullptr) {
    assert(n > 0);
    T mn = v[0];
    if (ind != nullptr) *ind = 0;
    for (int i = 1; i < n; i++)
        if (v[i] < mn) {
            mn = v[i];
            if (ind != nullptr) *ind = i;
        }
    return mn;
}

class bshot_descriptor {
  public:
    std::bitset<352> bits;
};

namespace myslam {
// bit j of the bitset <-> bit (j % 32) of word j / 32 (11 words); the same layout the C ABI uses.
// libstdc++ stores std::bitset<352> as unsigned long[6] with bit j at word j/64, bit j%64, so on
// little-endian x86-64 its first 44 bytes ARE the 11 words (checked in tests/test_host.py).
static_assert(sizeof(std::bitset<352>) == 48, "unexpected std::bitset<352> layout");
inline void bits_to_words(const std::bitset<352>& b, uint32_t w[11]) { std::memcpy(w, &b, 44); }
inline std::bitset<352> words_to_bits(const uint32_t w[11]) {
    std::bitset<352> b;
    std::memcpy(&b, w, 44);
    return b;
}
}  // namespace myslam
