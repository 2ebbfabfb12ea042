// Native host program over the burst queue (seastar::net::burst_queue over
// <sccsum.h> sccsum_burst_*): IPv4/UDP frames sit in mbuf-shaped host slots
// (2304 B, data at +256, dpdk.cc:139-156) and are handed over one at a time,
// as the DPDK rx loop delivers them (bursts of 32, dpdk.cc:2190-2204, after
// which the reactor polls); every 7th frame arrives as two fragments split at
// an odd offset (the `odd` carry of checksummer::sum(const packet&),
// ip_checksum.cc:64-68).  Every result is checked against the per-packet API;
// the hook's throughput is printed.  Usage: burst_gpu [frames] [depth]
// [max_delay_ns] [copy|copy_pageable|mapped] [poll_every] [fused] [pool_slots]:
// copy_pageable = copied from an ordinary malloc'd pool; mapped = the pool is pinned (as a
// DPDK mempool registered with the device) and frames go in by zero-copy
// submit_mapped; poll_every = frames handed over between reactor polls
// (default 32, one rx burst); fused = how zero-copy batches run
// (sccsum_set_burst_fused: 2 one launch on pinned metadata, the default; 1
// with metadata / result copies; 0 gather, then sum).  The time spent inside poll() is
// reported apart.
#include <seastar/net/ip_checksum.hh>
#include <seastar/net/ip_checksum_batch.hh>
#include <sccsum_diag.h>

#include <arpa/inet.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace seastar::net;

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 50000;
    const int depth = argc > 2 ? std::atoi(argv[2]) : 4;
    const uint64_t delay_ns = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 100000;
    constexpr uint32_t kSlot = 2304, kData = 256;
    uint64_t pool_cap = argc > 7 ? std::strtoull(argv[7], nullptr, 0) : 65536;  // slots, reused round robin
    pool_cap = pool_cap ? pool_cap : 1;
    const uint32_t pool_n = static_cast<uint32_t>(n < pool_cap ? n : pool_cap);
    std::mt19937 rng(11);
    const bool mapped = argc > 4 && std::strcmp(argv[4], "mapped") == 0;
    const bool pageable = argc > 4 && std::strcmp(argv[4], "copy_pageable") == 0;
    const uint64_t poll_every = argc > 5 ? std::strtoull(argv[5], nullptr, 0) : 32;
    const int fused = argc > 6 ? std::atoi(argv[6]) : 2;
    if (sccsum_set_burst_fused(fused) != SCCSUM_OK) {
        std::printf("FAILED: fused must be 0, 1 or 2\n");
        return 2;
    }
    uint8_t* pool = nullptr;
    if (pageable) {
        pool = static_cast<uint8_t*>(std::aligned_alloc(4096, uint64_t(pool_n) * kSlot));
    } else if (sccsum_host_alloc(reinterpret_cast<void**>(&pool), uint64_t(pool_n) * kSlot) != SCCSUM_OK) {
        std::printf("FAILED: sccsum_host_alloc\n");
        return 2;
    }
    std::vector<uint32_t> len(pool_n);
    std::vector<uint16_t> want(2 * size_t(pool_n));
    for (uint32_t i = 0; i < pool_n; ++i) {
        const uint32_t L = 28 + rng() % 1473;  // 20 B IPv4 + 8 B UDP + payload, up to 1500
        uint8_t* f = pool + size_t(i) * kSlot + kData;
        for (uint32_t k = 0; k < L; ++k) f[k] = uint8_t(rng());
        const uint32_t src = rng(), dst = rng();
        f[0] = 0x45;
        f[1] = 0;
        uint16_t be = htons(uint16_t(L));
        std::memcpy(f + 2, &be, 2);
        std::memset(f + 4, 0, 4);
        f[8] = 64;
        f[9] = 17;
        f[10] = f[11] = 0;
        const uint32_t s = htonl(src), d = htonl(dst);
        std::memcpy(f + 12, &s, 4);
        std::memcpy(f + 16, &d, 4);
        be = htons(uint16_t(L - 20));
        std::memcpy(f + 24, &be, 2);
        f[26] = f[27] = 0;
        len[i] = L;
        checksummer ipc;
        ipc.sum(reinterpret_cast<const char*>(f), 20);
        checksummer l4;
        l4.sum_many(src, dst, uint8_t(0), uint8_t(17), uint16_t(L - 20));
        l4.sum(reinterpret_cast<const char*>(f + 20), L - 20);
        want[2 * i] = ipc.get();
        want[2 * i + 1] = l4.get();
    }

    std::vector<uint16_t> got(2 * n, 0xdead);
    uint64_t batches = 0, delivered = 0;
    auto done = [&](uint64_t first, uint32_t count, const uint16_t* r, const uint8_t*) {
        std::memcpy(got.data() + 2 * first, r, 4 * size_t(count));
        ++batches;
        delivered += count;
    };
    int bad = 0;
    uint64_t busy = 0, bytes = 0, polls = 0;
    double secs = 0, poll_secs = 0;
    try {
        burst_queue<decltype(done)> q(0, SCCSUM_PIPE_IPV4, 16u << 20, 16384, delay_ns, depth, done);
        const auto t0 = std::chrono::steady_clock::now();
        auto timed_poll = [&] {
            const auto a = std::chrono::steady_clock::now();
            q.poll();
            poll_secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
            ++polls;
        };
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t k = static_cast<uint32_t>(i % pool_n);
            const uint8_t* f = pool + size_t(k) * kSlot + kData;
            sccsum_fragment fr[2] = {{f, len[k]}, {nullptr, 0}};
            uint32_t nf = 1;
            if (i % 7 == 3 && len[k] > 333) {  // a chained mbuf with an odd-length first segment
                fr[0].size = 333;
                fr[1] = {f + 333, len[k] - 333u};
                nf = 2;
            }
            uint64_t t = 0;
            while (!(mapped ? q.submit_mapped(fr, nf, 0, &t) : q.submit(fr, nf, 0, &t))) {
                ++busy;
                timed_poll();
            }
            if (t != i && bad++ < 5) std::printf("ticket %llu for packet %llu\n", (unsigned long long)t, (unsigned long long)i);
            bytes += len[k];
            if ((i + 1) % poll_every == 0) timed_poll();  // a burst handed over: the reactor runs its pollers
        }
        q.drain();
        secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } catch (const std::exception& e) {
        std::printf("FAILED: %s\n", e.what());
        return 2;
    }
    if (delivered != n) {
        std::printf("delivered %llu of %llu\n", (unsigned long long)delivered, (unsigned long long)n);
        ++bad;
    }
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t k = static_cast<uint32_t>(i % pool_n);
        if ((got[2 * i] != want[2 * k] || got[2 * i + 1] != want[2 * k + 1]) && bad++ < 10) {
            std::printf("frame %llu: gpu %04x/%04x cpu %04x/%04x\n", (unsigned long long)i, got[2 * i], got[2 * i + 1],
                        want[2 * k], want[2 * k + 1]);
        }
    }
    std::printf("burst_gpu: %llu frames, %.1f MB, %llu batches, depth %d, delay %llu ns, %s, %.3f s: %.2f Mpkt/s, %.2f GiB/s of packet "
                "bytes, %llu busy polls, %llu polls %.3f s in poll, %s, pool %u slots\n",
                (unsigned long long)n, bytes / 1e6, (unsigned long long)batches, depth, (unsigned long long)delay_ns, mapped ? "mapped" : "copy", secs, n / secs / 1e6,
                bytes / secs / (1u << 30), (unsigned long long)busy, (unsigned long long)polls, poll_secs, mapped ? (fused == 2 ? "zero-copy launch" : fused ? "fused+copies" : "gather+sum") : pageable ? "staged from pageable" : "staged from pinned", pool_n);
    if (pageable) {
        std::free(pool);
    } else {
        sccsum_host_free(pool);
    }
    if (bad) {
        std::printf("FAILED: %d mismatches\n", bad);
        return 1;
    }
    std::printf("burst_gpu: OK\n");
    return 0;
}
