// checksummer::sum(const packet&) (seastar_amd/csrc/checksummer_packet.cc, the
// replacement of src/net/ip_checksum.cc:64-68) built against the REFERENCE's
// own seastar::net::packet (include/seastar/net/packet.hh, used where it lies)
// and checked against the oracle.  Compiled by tests/test_packet_ref.py with
// the repo's include/ first and /root/reference/include after it, so
// <seastar/net/ip_checksum.hh> is the replacement header (its
// __has_include(<seastar/net/packet.hh>) branch) and packet.hh the real one.
//
// Packets are built the way the reference's own tests build them:
// tests/unit/packet_test.cc:32-84 (temporary_buffer fragments of 5/31/65/
// 4096/4096 bytes, trim_front by 1/6/29/1024, append of a 9+7-byte packet),
// plus random chains through packet(std::vector<fragment>, deleter)
// (packet.hh:400-409) and packet(packet&&, fragment) (packet.hh:425-434) at odd
// addresses, and the TCP verify call shape (tcp.hh:876-883).
// Exit status 0 = all equal.
#include <seastar/net/ip_checksum.hh>
#include <seastar/net/packet.hh>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

extern "C" {
#include "sccsum_oracle.h"
}

// Test-only definition of the reference library's assertion sink
// (src/util/log.cc:120 — that TU needs fmt, absent here).  packet.hh's inline
// members reach it only when an assertion fails.
namespace seastar::internal {
[[noreturn]] void assert_fail(const char* msg, const char* file, int line, const char* func) {
    std::fprintf(stderr, "assertion failed: %s at %s:%d (%s)\n", msg, file, line, func);
    std::abort();
}
}  // namespace seastar::internal

using namespace seastar;
using seastar::net::checksummer;

static int failures = 0;
static int checks = 0;

static void check(const net::packet& p, const std::vector<char>& expect, const char* ctx) {
    ++checks;
    checksummer c;
    c.sum(p);  // the function under test
    oracle_checksummer o;
    oracle_init(&o);
    size_t total = 0;
    for (auto&& f : p.fragments()) {
        oracle_sum_bytes(&o, reinterpret_cast<const uint8_t*>(f.base), f.size);
        total += f.size;
    }
    const uint16_t flat = oracle_ip_checksum(reinterpret_cast<const uint8_t*>(expect.data()), expect.size());
    if (c.get() != oracle_get(&o) || c.get() != flat || c.odd != bool(o.odd) || total != expect.size() ||
        p.len() != expect.size()) {
        if (failures++ < 10) {
            std::printf("MISMATCH %s: got %04x oracle %04x flat %04x odd %d/%d len %zu/%zu frags %u\n", ctx, c.get(),
                        oracle_get(&o), flat, int(c.odd), o.odd, size_t(p.len()), expect.size(),
                        unsigned(p.nr_frags()));
        }
    }
}

static void packet_test_chain() {
    std::vector<char> expected;
    auto append = [&expected](net::packet p, char c, size_t n) {
        auto tmp = temporary_buffer<char>(n);
        std::fill_n(tmp.get_write(), n, c);
        std::fill_n(std::back_inserter(expected), n, c);
        return net::packet(std::move(p), std::move(tmp));
    };
    net::packet p;
    p = append(std::move(p), 'a', 5);
    p = append(std::move(p), 'b', 31);
    p = append(std::move(p), 'c', 65);
    p = append(std::move(p), 'c', 4096);
    p = append(std::move(p), 'd', 4096);
    check(p, expected, "packet_test initial");
    for (size_t n : {1u, 6u, 29u, 1024u}) {
        p.trim_front(n);
        expected.erase(expected.begin(), expected.begin() + n);
        check(p, expected, "packet_test trim_front");
    }
    net::packet p2;
    p2 = append(std::move(p2), 'z', 9);
    p2 = append(std::move(p2), 'x', 7);
    p.append(std::move(p2));
    check(p, expected, "packet_test append");
}

static void random_chains() {
    std::mt19937_64 rng(77);
    std::vector<char> pool(1 << 20);
    for (auto& b : pool) b = char(rng());
    for (int t = 0; t < 3000; ++t) {
        const int nf = 1 + int(rng() % 9);
        std::vector<net::fragment> frags;
        std::vector<char> expect;
        for (int i = 0; i < nf; ++i) {
            // sizes like DPDK mbuf segments, virtio buffers and packet_test's odd pieces
            static const size_t kSizes[] = {1, 2, 3, 5, 7, 20, 31, 65, 1460, 2048, 4096};
            const size_t sz = (rng() & 1) ? kSizes[rng() % 11] : 1 + rng() % 3000;
            const size_t at = rng() % (pool.size() - sz);  // any alignment
            frags.push_back(net::fragment{pool.data() + at, sz});
            expect.insert(expect.end(), pool.data() + at, pool.data() + at + sz);
        }
        if (t % 2) {
            net::packet p(std::move(frags), make_deleter([] {}));
            check(p, expect, "vector<fragment>");
        } else {
            net::packet p(frags[0], make_deleter([] {}));
            for (size_t i = 1; i < frags.size(); ++i) p = net::packet(std::move(p), frags[i]);
            check(p, expect, "packet(packet&&, fragment)");
            if (p.len() > 3) {  // trimmed front: the chain then starts at an odd packet offset of its buffer
                const size_t k = 1 + rng() % (p.len() - 1);
                p.trim_front(k);
                expect.erase(expect.begin(), expect.begin() + k);
                check(p, expect, "trimmed");
            }
        }
    }
}

static void tcp_verify_shape() {
    // tcp.hh:876-883: pseudo-header of p.len() as uint16_t, then sum(p) over
    // header + payload fragments; a segment carrying its own checksum verifies
    std::mt19937_64 rng(5);
    for (int t = 0; t < 500; ++t) {
        std::vector<char> seg(20 + rng() % 3000);
        for (auto& b : seg) b = char(rng());
        seg[16] = seg[17] = 0;
        const uint32_t src = uint32_t(rng()), dst = uint32_t(rng());
        checksummer gen;
        gen.sum_many(src, dst, uint8_t(0), uint8_t(6), uint16_t(seg.size()));
        gen.sum(seg.data(), seg.size());
        const uint16_t v = gen.get();
        std::memcpy(seg.data() + 16, &v, 2);
        const size_t cut = 1 + rng() % (seg.size() - 1);
        std::vector<net::fragment> fr{{seg.data(), cut}, {seg.data() + cut, seg.size() - cut}};
        net::packet p(std::move(fr), make_deleter([] {}));
        checksummer ver;
        ver.sum_many(src, dst, uint8_t(0), uint8_t(6), uint16_t(p.len()));
        ver.sum(p);
        ++checks;
        if (ver.get() != 0 && failures++ < 10) std::printf("MISMATCH tcp verify: %04x\n", ver.get());
    }
}

int main() {
    static_assert(sizeof(checksummer) == 32 && alignof(checksummer) == 16, "checksummer layout");
    packet_test_chain();
    random_chains();
    tcp_verify_shape();
    if (failures) {
        std::printf("FAILED: %d of %d checks\n", failures, checks);
        return 1;
    }
    std::printf("packet_ref: OK (%d checks)\n", checks);
    return 0;
}
