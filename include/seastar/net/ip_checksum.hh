// seastar/net/ip_checksum.hh — drop-in replacement for the reference header
// of the same path (include/seastar/net/ip_checksum.hh:33-71 in
// scylladb/seastar).  Same names, same signatures, same object layout
// (__int128 csum; bool odd; sizeof 32, align 16) and the same semantics for
// the inline members, so src/net/{ip,udp,tcp}.cc, include/seastar/net/tcp.hh
// and demos/{udp_server,tcp_demo,echo_demo}.cc compile and link unchanged.
//
// This header is the synchronous per-packet API (one packet on the calling
// reactor thread, CPU by design: a GPU launch per packet is latency-absurd).
// Batches of packets go to the MI355X through <seastar/net/ip_checksum_batch.hh>
// (C++) / <sccsum.h> (C-ABI); that path never falls back to this one.
#pragma once

#include <arpa/inet.h>

#include <cstddef>
#include <cstdint>

// Inside the Seastar tree the real packet type comes with this header, as in
// the reference; standalone, only the forward declaration below is needed.
#if __has_include(<seastar/net/packet.hh>)
#include <seastar/net/packet.hh>
#endif

namespace seastar {

namespace net {

class packet;

// One-shot checksum of a contiguous span; result bytes are in network order.
uint16_t ip_checksum(const void* data, size_t len);

struct checksummer {
    // Running sum of big-endian 16-bit words (host integers), and whether an
    // odd number of bytes has been consumed so far.
    __int128 csum = 0;
    bool odd = false;

    void sum(const char* data, size_t len);
    void sum(const packet& p);

    // A single byte is the high half of a word at an even position and the
    // low half at an odd one.
    void sum(uint8_t data) {
        csum += odd ? __int128(data) : __int128(uint32_t(data) << 8);
        odd = !odd;
    }
    // Host-order 16-bit value: one word when aligned, else split into bytes.
    void sum(uint16_t data) {
        if (!odd) {
            csum += data;
            return;
        }
        sum(uint8_t(data >> 8));
        sum(uint8_t(data & 0xff));
    }
    // Host-order 32-bit value: added whole when aligned; when odd, the low
    // 16 bits go first, then the high 16 bits.
    void sum(uint32_t data) {
        if (!odd) {
            csum += data;
            return;
        }
        sum(uint16_t(data & 0xffff));
        sum(uint16_t(data >> 16));
    }
    void sum_many() {}
    template <typename First, typename... Rest>
    void sum_many(First first, Rest... rest) {
        sum(first);
        sum_many(rest...);
    }
    // Folded, complemented checksum with its bytes in network order.
    uint16_t get() const;
};

}  // namespace net

}  // namespace seastar
