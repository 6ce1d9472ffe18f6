// Test harness: the product's deflate-length header (taxi2_amd/csrc/deflate_len.hpp) compiled
// for the host, so its zlib-1.2.11 exactness is checked on CPU against Python's zlib
// (tests/test_ncd.py).  Not part of the product library.
#include <vector>

#include "../../taxi2_amd/csrc/deflate_len.hpp"

using namespace taxi2::zl;

extern "C" int zlen_host(const uint8_t* a, int na, const uint8_t* b, int nb, int latin1) {
    static std::vector<uint8_t> win(WIN_BYTES + 16);
    static std::vector<uint16_t> prev(WSIZE), head(HASH_SIZE, 0);
    static Trees t;
    Scratch z{win.data(), prev.data(), head.data()};
    return compressed_len(a, na, b, nb, z, t, latin1 != 0);
}
