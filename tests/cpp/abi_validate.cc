// Argument validation of every C-ABI entry point (include/sccsum.h,
// include/sccsum_diag.h) without a device: each bad call must return its
// error code and touch nothing.  Built by tests/test_sanitize.py with host
// AddressSanitizer + UndefinedBehaviorSanitizer (the reference's `sanitize`
// build mode, cmake/FindSanitizers.cmake:37-43) over the library sources, and
// with ThreadSanitizer, the checks run from several threads at once (Seastar
// calls from one reactor thread per shard: src/core/reactor.cc:3437-3438).
// Usage: abi_validate [threads].  Exit status 0 = every check held.
#include "sccsum.h"
#include "sccsum_diag.h"

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static std::atomic<int> failures{0};
#define EXPECT(cond)                                                       \
    do {                                                                   \
        if (!(cond)) {                                                     \
            ++failures;                                                    \
            std::printf("FAILED %s (line %d)\n", #cond, __LINE__);         \
        }                                                                  \
    } while (0)

static void noop(void*, uint64_t, uint32_t, const uint16_t*, const uint8_t*) {}

static void checks() {
    void* const d16 = reinterpret_cast<void*>(uintptr_t(0x10000));  // aligned non-null stand-ins, never dereferenced
    void* const odd = reinterpret_cast<void*>(uintptr_t(0x10002));
    // n == 0 is a no-op whatever the pointers
    EXPECT(sccsum_spans(nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr) == SCCSUM_OK);
    EXPECT(sccsum_ipv4_frames(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr) == SCCSUM_OK);
    EXPECT(sccsum_fragments(nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr,
                            nullptr) == SCCSUM_OK);
    EXPECT(sccsum_gather(nullptr, 0, nullptr, nullptr) == SCCSUM_OK);
    // null / misaligned pointers
    EXPECT(sccsum_spans(nullptr, 64, nullptr, nullptr, nullptr, nullptr, nullptr, 3, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_spans(odd, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), nullptr,
                        static_cast<uint16_t*>(d16), nullptr, 3, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_frames(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16),
                              static_cast<uint16_t*>(odd), nullptr, 3, 0, nullptr) == SCCSUM_EINVAL);
    // frames: neither d_out2 nor d_status (a verify-only launch needs the status array)
    EXPECT(sccsum_ipv4_frames(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), nullptr,
                              nullptr, 3, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_fragments(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), 4,
                            static_cast<const uint32_t*>(d16), nullptr, static_cast<uint16_t*>(d16), nullptr, 2, 0,
                            nullptr, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_fragments_workspace(1000) >= 3000);
    EXPECT(sccsum_gather(static_cast<const sccsum_gather_desc*>(odd), 1, d16, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_read_probe(nullptr, 16, nullptr, nullptr) == SCCSUM_EINVAL);
    // fragment lists: nothing to do, then null / misaligned arrays
    EXPECT(sccsum_ipv4_frames_desc(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr) ==
           SCCSUM_OK);
    EXPECT(sccsum_ipv4_frames_desc(nullptr, nullptr, static_cast<const uint64_t*>(d16),
                                   static_cast<const uint32_t*>(d16), nullptr, static_cast<uint16_t*>(d16), nullptr, 2,
                                   64, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_frames_desc(nullptr, static_cast<const uint32_t*>(d16), static_cast<const uint64_t*>(d16),
                                   static_cast<const uint32_t*>(d16), nullptr, static_cast<uint16_t*>(odd), nullptr, 2,
                                   64, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_spans_desc(static_cast<const sccsum_gather_desc*>(odd), static_cast<const uint32_t*>(d16),
                             static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), nullptr, nullptr,
                             static_cast<uint16_t*>(d16), nullptr, 2, 64, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_spans_desc(static_cast<const sccsum_gather_desc*>(d16), static_cast<const uint32_t*>(d16),
                             static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), nullptr, nullptr,
                             nullptr, nullptr, 2, 64, nullptr) == SCCSUM_EINVAL);
    // fill modes
    EXPECT(sccsum_ipv4_fill(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_fill(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0,
                            SCCSUM_FILL_L4 | SCCSUM_FILL_L4_PSEUDO, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_fill(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, SCCSUM_FILL_TSO, nullptr) ==
           SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_fill(nullptr, 64, nullptr, nullptr, nullptr, nullptr, 3, 0, SCCSUM_FILL_IP, nullptr) ==
           SCCSUM_EINVAL);
    // FILL_L4 / FILL_ICMP_ECHO: d_out2 is optional, the batch is checked like a frames batch
    EXPECT(sccsum_ipv4_fill(static_cast<uint8_t*>(d16) + 1, 64, static_cast<const uint64_t*>(d16),
                            static_cast<const uint32_t*>(d16), nullptr, nullptr, 3, 0,
                            SCCSUM_FILL_IP | SCCSUM_FILL_L4, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_fill(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16),
                            reinterpret_cast<uint16_t*>(static_cast<uint8_t*>(d16) + 2), nullptr, 3, 0,
                            SCCSUM_FILL_ICMP_ECHO, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_fill(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0,
                            SCCSUM_FILL_ICMP_ECHO | SCCSUM_FILL_L4_PSEUDO, nullptr) == SCCSUM_EINVAL);
    // RSS
    const uint8_t key3[3] = {1, 2, 3};
    EXPECT(sccsum_ipv4_rss(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), key3, 3, 0,
                           static_cast<uint32_t*>(d16), nullptr, 1, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_ipv4_frames_rss(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16),
                                  static_cast<uint16_t*>(d16), nullptr, 1, 0, key3, 40, 7,
                                  static_cast<uint32_t*>(d16), nullptr) == SCCSUM_EINVAL);
    // burst queue: arguments are checked before any device call
    sccsum_burst* b = reinterpret_cast<sccsum_burst*>(1);
    EXPECT(sccsum_burst_create(0, 7, 1 << 20, 64, 0, 2, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 1 << 20, 64, 0, 0, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 1 << 20, 64, 0, 65, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 1 << 20, 0, 0, 2, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 32, 64, 0, 2, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, uint64_t(1) << 32, 64, 0, 2, noop, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 1 << 20, 64, 0, 2, nullptr, nullptr, &b) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_create(0, 0, 1 << 20, 64, 0, 2, noop, nullptr, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_submit(nullptr, nullptr, 0, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_submit_mapped(nullptr, nullptr, 0, 0, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_poll(nullptr, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_drain(nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_burst_destroy(nullptr) == SCCSUM_OK);
    // resident engine: arguments are checked before any runtime call
    sccsum_engine* eng = nullptr;
    EXPECT(sccsum_engine_create(0, 7, 16, 2, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_IPV4, 0, 2, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_IPV4, 65537, 2, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_SPANS, 16, 0, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_SPANS, 16, 257, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_IPV4, 16, 2, nullptr) == SCCSUM_EINVAL);
    // fill steps: frames only, and at least 2 steps in flight (a fill is two)
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_SPANS | SCCSUM_ENGINE_FILL, 16, 2, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_IPV4 | SCCSUM_ENGINE_FILL, 16, 1, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create(0, SCCSUM_PIPE_IPV4 | 0x200, 16, 2, &eng) == SCCSUM_EINVAL);
    EXPECT(eng == nullptr);
    EXPECT(sccsum_engine_start(nullptr, nullptr) == SCCSUM_EINVAL);
    uint64_t step = 0;
    EXPECT(sccsum_engine_submit(nullptr, nullptr, 1, 0, 0, &step) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_submit_fill(nullptr, nullptr, 1, 0, SCCSUM_FILL_IP | SCCSUM_FILL_L4, 0, &step) ==
           SCCSUM_EINVAL);
    EXPECT(sccsum_engine_wait(nullptr, 0, 0) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_stop(nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_destroy(nullptr) == SCCSUM_OK);
    EXPECT(sccsum_set_engine_write_through(0) == SCCSUM_OK && sccsum_set_engine_write_through(1) == SCCSUM_OK);
    EXPECT(sccsum_set_engine_idle_ms(-1) == SCCSUM_EINVAL && sccsum_set_engine_idle_ms(3600001) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_engine_idle_ms(250) == SCCSUM_OK && sccsum_set_engine_idle_ms(0) == SCCSUM_OK);
    // create with every limit (ABI 4): ranges are checked before any runtime call
    const sccsum_engine_opts big_ring = {65537, 8, 0, 0}, many = {1024, 257, 0, 0}, idle = {1024, 8, 3600001, 0},
                             dep = {1024, 8, 0, 3600001}, fill1 = {1024, 1, 0, 0},
                             producer = {1024, 8, 0, 0, 9}, producer_default_mif = {1024, 0, 0, 0, 9};
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4, nullptr, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4, &big_ring, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4, &many, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_SPANS, &idle, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_SPANS, &dep, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4 | SCCSUM_ENGINE_FILL, &fill1, &eng) == SCCSUM_EINVAL);
    // a producer's own limit above the shared one (given, or the default 8)
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4, &producer, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_SPANS, &producer_default_mif, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_SPANS | SCCSUM_ENGINE_FILL, &many, &eng) == SCCSUM_EINVAL);
    EXPECT(sccsum_engine_create_opts(0, SCCSUM_PIPE_IPV4, &big_ring, nullptr) == SCCSUM_EINVAL);
    EXPECT(eng == nullptr);
    EXPECT(sccsum_set_engine_sync_every(-2) == SCCSUM_EINVAL && sccsum_set_engine_sync_every(65537) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_engine_sync_every(20) == SCCSUM_OK && sccsum_set_engine_sync_every(0) == SCCSUM_OK);
    EXPECT(sccsum_set_engine_sync_every(-1) == SCCSUM_OK);
    // host pipeline
    sccsum_pipeline* p = nullptr;
    EXPECT(sccsum_pipeline_create(0, 1 << 20, 1024, 0, &p) == SCCSUM_EINVAL);
    EXPECT(sccsum_pipeline_create(0, 1 << 20, 1024, 17, &p) == SCCSUM_EINVAL);
    EXPECT(sccsum_pipeline_create(0, 32, 1024, 2, &p) == SCCSUM_EINVAL);
    EXPECT(sccsum_pipeline_create(0, 1 << 20, 0, 2, &p) == SCCSUM_EINVAL);
    EXPECT(sccsum_pipeline_create(0, 1 << 20, 1024, 2, nullptr) == SCCSUM_EINVAL);
    EXPECT(sccsum_host_alloc(nullptr, 64) == SCCSUM_EINVAL);
    // diagnostics: thread-local knobs validate their ranges
    EXPECT(sccsum_set_kernel_variant(3) == SCCSUM_EINVAL && sccsum_set_kernel_variant(5) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_kernel_variant(20) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_kernel_variant(10) == SCCSUM_EINVAL && sccsum_set_kernel_variant(17) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_kernel_variant(16) == SCCSUM_OK && sccsum_set_kernel_variant(0) == SCCSUM_OK);
    EXPECT(sccsum_set_blocks_per_cu(0) == SCCSUM_EINVAL && sccsum_set_blocks_per_cu(33) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_group_units(3) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_tile_packets(65) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_tile_bytes(-1) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_dynamic_tiles(2) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_tail_split(3, 4) == SCCSUM_EINVAL && sccsum_set_tail_split(16, 4) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_tail_split(4, -1) == SCCSUM_EINVAL && sccsum_set_tail_split(4, 65) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_tail_split(4, 4) == SCCSUM_OK && sccsum_set_tail_split(1, 4) == SCCSUM_OK);
    EXPECT(sccsum_set_out_policy(-1) == SCCSUM_EINVAL && sccsum_set_out_policy(5) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_out_policy(3) == SCCSUM_OK && sccsum_set_out_policy(0) == SCCSUM_OK);
    EXPECT(sccsum_set_short_chunks(2) == SCCSUM_EINVAL && sccsum_set_short_chunks(-1) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_short_chunks(0) == SCCSUM_OK && sccsum_set_short_chunks(1) == SCCSUM_OK);
    EXPECT(sccsum_set_run_align(0) == SCCSUM_EINVAL && sccsum_set_run_align(2) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_run_align(16) == SCCSUM_EINVAL && sccsum_set_run_align(8) == SCCSUM_OK);
    EXPECT(sccsum_set_run_align(4) == SCCSUM_OK && sccsum_set_run_align(1) == SCCSUM_OK);
    EXPECT(sccsum_set_burst_fused(3) == SCCSUM_EINVAL && sccsum_set_burst_fused(-1) == SCCSUM_EINVAL);
    EXPECT(sccsum_set_burst_fused(2) == SCCSUM_OK);
    EXPECT(sccsum_pipeline_run(nullptr, SCCSUM_PIPE_IPV4, SCCSUM_GATHER_ZERO_COPY, nullptr, 0, nullptr, nullptr,
                               nullptr, 0, 0, nullptr, nullptr) == SCCSUM_EINVAL);
    // well-formed arguments without a device: the launch device is resolved
    // (hipGetDevice, then the stream's device) before anything is launched, so
    // the call returns that HIP error and touches nothing.  (Only where no
    // device is visible: on a GPU these stand-in pointers would be launched.)
    EXPECT(sccsum_device_numa_node(0, nullptr) == SCCSUM_EINVAL);
    int ndev = 0;
    if (sccsum_device_count(&ndev) != SCCSUM_OK || ndev == 0) {
        EXPECT(sccsum_spans(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16), nullptr,
                            static_cast<uint16_t*>(d16), nullptr, 3, 0, nullptr) > 0);
        EXPECT(sccsum_ipv4_fill(d16, 64, static_cast<const uint64_t*>(d16), static_cast<const uint32_t*>(d16),
                                static_cast<uint16_t*>(d16), nullptr, 3, 0, SCCSUM_FILL_IP | SCCSUM_FILL_L4,
                                nullptr) > 0);
        EXPECT(sccsum_read_probe(d16, 64, static_cast<uint64_t*>(d16), nullptr) > 0);
        // a NULL descriptor array is accepted (no packet has fragments: an empty rx burst), so the
        // call gets as far as the launch device
        EXPECT(sccsum_ipv4_frames_desc(nullptr, static_cast<const uint32_t*>(d16), static_cast<const uint64_t*>(d16),
                                       static_cast<const uint32_t*>(d16), nullptr, static_cast<uint16_t*>(d16),
                                       nullptr, 2, 64, nullptr) > 0);
        EXPECT(sccsum_spans_desc(nullptr, static_cast<const uint32_t*>(d16), static_cast<const uint64_t*>(d16),
                                 static_cast<const uint32_t*>(d16), nullptr, nullptr, static_cast<uint16_t*>(d16),
                                 nullptr, 2, 0, nullptr) > 0);
    }
    // host arithmetic and strings
    EXPECT(sccsum_pseudo_seed(1, 2, 17, 8) == 28u);
    EXPECT(sccsum_pseudo_seed(0xffffffffu, 0xffffffffu, 255, 0xffff) <= 0xffffu);
    EXPECT(std::strcmp(sccsum_strerror(SCCSUM_EBUSY),
                       "busy: every batch slot or engine step is in flight, or the device's engine is running") == 0);
    EXPECT(std::strcmp(sccsum_strerror(-99), "unknown sccsum error") == 0);
    EXPECT(std::strcmp(sccsum_strerror(SCCSUM_EFAULT), "the engine's grid stopped on an internal fault") == 0);
    EXPECT(sccsum_abi_version() == SCCSUM_ABI_VERSION);
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 1;
    checks();
    if (threads > 1) {
        std::vector<std::thread> ts;
        for (int t = 0; t < threads; ++t) {
            ts.emplace_back([] {
                for (int rep = 0; rep < 20; ++rep) checks();
            });
        }
        for (auto& t : ts) t.join();
    }
    if (failures.load()) {
        std::printf("abi_validate: %d FAILED\n", failures.load());
        return 1;
    }
    std::printf("abi_validate: OK (%d thread%s)\n", threads, threads > 1 ? "s" : "");
    return 0;
}
