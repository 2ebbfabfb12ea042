// Per-packet C++ API (include/seastar/net/ip_checksum.hh + checksummer.cc)
// against the oracle (C restatement, test-only), plus the call shapes the
// reference's callers use (src/net/ip.cc, src/net/udp.cc, tcp.hh,
// demos/echo_demo.cc).  Exit status 0 = all equal.
#include <seastar/net/ip_checksum.hh>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
#include "sccsum_oracle.h"
}

using seastar::net::checksummer;
using seastar::net::ip_checksum;

static_assert(sizeof(checksummer) == 32, "checksummer layout (ip_checksum.hh:35-37)");
static_assert(alignof(checksummer) == 16, "checksummer alignment");

static int failures = 0;
#define EXPECT_EQ(a, b, ctx)                                                                            \
    do {                                                                                                \
        auto _a = (a);                                                                                  \
        auto _b = (b);                                                                                  \
        if (_a != _b) {                                                                                 \
            if (failures++ < 10) std::printf("MISMATCH %s: %x != %x (%s)\n", #a, unsigned(_a), unsigned(_b), ctx); \
        }                                                                                               \
    } while (0)

int main() {
    std::mt19937_64 rng(1234);
    std::vector<uint8_t> buf(70000);
    for (auto& b : buf) b = uint8_t(rng());

    // one-shot ip_checksum over every length 0..2100 at 4 alignments, and long spans
    for (size_t a = 0; a < 4; ++a) {
        for (size_t n = 0; n <= 2100; ++n) {
            EXPECT_EQ(ip_checksum(buf.data() + a, n), oracle_ip_checksum(buf.data() + a, n), "one-shot");
        }
    }
    for (size_t n : {9000u, 65535u, 65536u, 69999u}) {
        EXPECT_EQ(ip_checksum(buf.data() + 1, n), oracle_ip_checksum(buf.data() + 1, n), "long");
    }

    // fragment chains (odd carries across fragments, packet_test.cc sizes)
    const std::vector<std::vector<size_t>> chains = {{7, 1, 333, 1160}, {5, 31, 65, 4096, 4096}, {1, 1, 1, 2, 3, 5, 8}};
    for (const auto& ch : chains) {
        checksummer c;
        oracle_checksummer o;
        oracle_init(&o);
        size_t pos = 3;
        for (size_t s : ch) {
            c.sum(reinterpret_cast<const char*>(buf.data() + pos), s);
            oracle_sum_bytes(&o, buf.data() + pos, s);
            pos += s;
        }
        EXPECT_EQ(c.get(), oracle_get(&o), "fragments");
        EXPECT_EQ(c.odd, bool(o.odd), "fragments odd");
    }

    // inline members mixed with spans, both parities (ip_checksum.hh:40-69)
    for (int t = 0; t < 5000; ++t) {
        checksummer c;
        oracle_checksummer o;
        oracle_init(&o);
        int ops = 1 + int(rng() % 10);
        for (int i = 0; i < ops; ++i) {
            switch (rng() % 4) {
                case 0: {
                    uint8_t v = uint8_t(rng());
                    c.sum(v);
                    oracle_sum_u8(&o, v);
                    break;
                }
                case 1: {
                    uint16_t v = uint16_t(rng());
                    c.sum(v);
                    oracle_sum_u16(&o, v);
                    break;
                }
                case 2: {
                    uint32_t v = uint32_t(rng());
                    c.sum(v);
                    oracle_sum_u32(&o, v);
                    break;
                }
                default: {
                    size_t off = rng() % 1000, n = 1 + rng() % 97;
                    c.sum(reinterpret_cast<const char*>(buf.data() + off), n);
                    oracle_sum_bytes(&o, buf.data() + off, n);
                }
            }
        }
        EXPECT_EQ(c.get(), oracle_get(&o), "mixed");
    }

    // caller shapes: pseudo-header via sum_many (ip.hh:70-75), UDP generate
    // (udp.cc:184-193), TCP verify (tcp.hh:876-883), IPv4 header (ip.cc:121-127),
    // ICMP / echo_demo one-shot (echo_demo.cc:76-78)
    for (int t = 0; t < 2000; ++t) {
        uint32_t src = uint32_t(rng()), dst = uint32_t(rng());
        uint16_t len = uint16_t(8 + rng() % 1472);
        checksummer c;
        c.sum_many(src, dst, uint8_t(0), uint8_t(17), len);
        c.sum(reinterpret_cast<const char*>(buf.data() + 10), len);
        oracle_checksummer o;
        oracle_init(&o);
        oracle_pseudo_header(&o, src, dst, 17, len);
        oracle_sum_bytes(&o, buf.data() + 10, len);
        EXPECT_EQ(c.get(), oracle_get(&o), "udp generate");
    }
    {
        uint8_t iph[20] = {0x45, 0, 0, 0x73, 0, 0, 0x40, 0, 0x40, 0x11, 0, 0, 0xc0, 0xa8, 0, 1, 0xc0, 0xa8, 0, 0xc7};
        checksummer csum;
        csum.sum(reinterpret_cast<char*>(iph), sizeof(iph));
        uint16_t v = csum.get();
        std::memcpy(iph + 10, &v, 2);
        EXPECT_EQ(iph[10], 0xb8, "ipv4 generate byte 0");
        EXPECT_EQ(iph[11], 0x61, "ipv4 generate byte 1");
        checksummer verify;
        verify.sum(reinterpret_cast<char*>(iph), sizeof(iph));
        EXPECT_EQ(verify.get(), 0, "ipv4 verify");
        EXPECT_EQ(ip_checksum(iph, 20), 0, "echo_demo one-shot");
    }
    {
        // TCP pseudo-header length wraps at 65536 (uint16_t parameter)
        checksummer a, b;
        a.sum_many(0x0a000001u, 0x0a000002u, uint8_t(0), uint8_t(6), uint16_t(65536u));
        b.sum_many(0x0a000001u, 0x0a000002u, uint8_t(0), uint8_t(6), uint16_t(0));
        EXPECT_EQ(a.get(), b.get(), "tcp len wrap");
    }
    if (failures) {
        std::printf("FAILED: %d mismatches\n", failures);
        return 1;
    }
    std::printf("api_parity: OK\n");
    return 0;
}
