// Out-of-line members of seastar::net::checksummer and ip_checksum() — the
// per-packet API kept from src/net/ip_checksum.cc:31-74 (same results, same
// accumulator domain: big-endian 16-bit words as host integers, so the inline
// sum(uint8/16/32) members of the header compose with sum(const char*, size_t)).
//
// checksummer::sum(const packet&) lives in checksummer_packet.cc, which needs
// Seastar's real packet type and is compiled only inside the Seastar tree
// (INTEGRATION.md).
#include <seastar/net/ip_checksum.hh>

#include <cstring>

namespace seastar {

namespace net {

namespace {

inline uint64_t load_be64(const char* p) {
    uint64_t w;
    std::memcpy(&w, p, sizeof(w));
    return __builtin_bswap64(w);
}

inline uint32_t load_be16(const char* p) {
    return (uint32_t(uint8_t(p[0])) << 8) | uint8_t(p[1]);
}

}  // namespace

void checksummer::sum(const char* data, size_t len) {
    if (len == 0) {
        return;
    }
    const bool flip = len & 1;
    if (odd) {
        // completes the word whose high byte was consumed earlier
        csum += uint8_t(*data);
        ++data;
        --len;
    }
    // Four independent 64-bit lanes of big-endian words, carried in 128 bits.
    unsigned __int128 a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (; len >= 32; data += 32, len -= 32) {
        a0 += load_be64(data);
        a1 += load_be64(data + 8);
        a2 += load_be64(data + 16);
        a3 += load_be64(data + 24);
    }
    for (; len >= 8; data += 8, len -= 8) {
        a0 += load_be64(data);
    }
    for (; len >= 2; data += 2, len -= 2) {
        a1 += load_be16(data);
    }
    if (len) {
        a2 += uint32_t(uint8_t(*data)) << 8;
    }
    csum += __int128(a0 + a1 + a2 + a3);
    odd ^= flip;
}

uint16_t checksummer::get() const {
    // 128 -> 64 with end-around carry, twice; then 64 -> 16.
    const unsigned __int128 x = static_cast<unsigned __int128>(csum);
    const unsigned __int128 lo64 = ~uint64_t(0);
    unsigned __int128 y = (x & lo64) + (x >> 64);
    uint64_t s = uint64_t((y & lo64) + (y >> 64));
    s = (s >> 48) + ((s >> 32) & 0xffff) + ((s >> 16) & 0xffff) + (s & 0xffff);
    while (s >> 16) {
        s = (s & 0xffff) + (s >> 16);
    }
    return htons(uint16_t(~s));
}

uint16_t ip_checksum(const void* data, size_t len) {
    checksummer c;
    c.sum(static_cast<const char*>(data), len);
    return c.get();
}

}  // namespace net

}  // namespace seastar
