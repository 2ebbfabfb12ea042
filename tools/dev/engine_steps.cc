// Small steps through the resident engine against one launch per step, native
// host side (no Python between steps): the reactor model of SURVEY §8(f)3,
// where a shard hands its GPU bursts of 32 packets (DPDK rx, dpdk.cc:2190-2204)
// or tx refills of up to 128 (qp::poll_tx, net.cc:81-105) as they come.
// For each step size B, k steps over distinct slices of a batch of 1500 B
// IPv4/UDP frames (verify-only: status bytes), timed on the host clock from
// the first submit to the last step's completion:
//   launch  sccsum_ipv4_frames per step on one stream, then one sync
//   engine  one resident grid per run, sccsum_engine_submit per step
//           (64 steps in flight), then a wait on the last step
// With the argument `fill`, every step is an in-place fill of its slice
// (SCCSUM_FILL_IP | SCCSUM_FILL_L4: the tx half, ip.cc:266-278, udp.cc:184-195):
//   launch  sccsum_ipv4_fill per step (a generate and a store kernel)
//   engine  a fill engine, sccsum_engine_submit_fill per step (two engine steps)
// With the argument `producers` (and optionally a thread count, default 8),
// the engine's steps come from that many host threads at once — the shards of
// one GPU feeding its one engine (include/sccsum.h "Producers") — each
// submitting its share of the k steps; the clock runs from a common start to
// the last thread's last step done.  ENGINE_STEPS_RING sets the engine's ring
// slots (default 1 024, the library's default), ENGINE_STEPS_IN_FLIGHT its
// in-flight limit (default 64).
// Prints one JSON line per size.  Build (tools/gpu_session.sh bin: step):
//   hipcc -O2 -std=c++17 -I include tools/dev/engine_steps.cc -L seastar_amd/lib -lsccsum \
//         -Wl,-rpath,$PWD/seastar_amd/lib -o tools/dev/engine_steps
#include <hip/hip_runtime.h>
#include <sccsum.h>
#include <sccsum_diag.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstdio>
#include <cstring>
#include <vector>

#define HIP_OK(x)                                                                                \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
            return 2;                                                                            \
        }                                                                                        \
    } while (0)
#define SC_OK(x)                                                                                 \
    do {                                                                                         \
        int r_ = (x);                                                                            \
        if (r_ != SCCSUM_OK) {                                                                   \
            std::printf("sccsum error %s at %s:%d\n", sccsum_strerror(r_), __FILE__, __LINE__);   \
            return 3;                                                                            \
        }                                                                                        \
    } while (0)

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// k steps of B frames from `threads` producer threads into one running engine
// e: µs per step (aggregate), or a negative value on an error.
static double producers_run(sccsum_engine* e, void* s, int threads, uint64_t k, uint32_t B, uint64_t slices,
                            void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                            uint8_t* d_st) {
    if (sccsum_engine_start(e, s) != SCCSUM_OK) return -1;
    std::atomic<int> ready{0}, bad{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
        ts.emplace_back([&, t] {
            ++ready;
            while (!go.load()) {
            }
            uint64_t step = 0;
            bool any = false;
            for (uint64_t j = t; j < k; j += threads) {
                const uint64_t q = j % slices;
                sccsum_batch b{};
                b.d_bytes = d_bytes;
                b.bytes_len = bytes_len;
                b.d_off = d_off + q * B;
                b.d_len = d_len + q * B;
                b.d_status = d_st + q * B;
                b.n = B;
                if (sccsum_engine_submit(e, &b, 1, 1500, 10'000'000'000ull, &step) != SCCSUM_OK) {
                    ++bad;
                    return;
                }
                any = true;
            }
            if (any && sccsum_engine_wait(e, step, 10'000'000'000ull) != SCCSUM_OK) ++bad;
        });
    }
    while (ready.load() < threads) {
    }
    const double t0 = now_s();
    go = true;
    for (auto& th : ts) th.join();
    const double dt = now_s() - t0;
    if (sccsum_engine_stop(e) != SCCSUM_OK) ++bad;
    if (hipStreamSynchronize(static_cast<hipStream_t>(s)) != hipSuccess) ++bad;
    return bad.load() ? -1.0 : dt / k * 1e6;
}

int main(int argc, char** argv) {
    const bool fill = argc > 1 && std::strcmp(argv[1], "fill") == 0;
    const bool producers = argc > 1 && std::strcmp(argv[1], "producers") == 0;
    const int nprod = producers && argc > 2 ? std::atoi(argv[2]) : 8;
    const uint32_t ring = std::getenv("ENGINE_STEPS_RING") ? std::atoi(std::getenv("ENGINE_STEPS_RING")) : 1024;
    // steps in flight (ENGINE_STEPS_IN_FLIGHT, default 64: the engine's most)
    const uint32_t mif = std::getenv("ENGINE_STEPS_IN_FLIGHT") ? std::atoi(std::getenv("ENGINE_STEPS_IN_FLIGHT")) : 64;
    const uint32_t mode = SCCSUM_FILL_IP | SCCSUM_FILL_L4;
    const uint64_t n_all = 1 << 18;  // 262 144 frames, 393 MB
    const uint32_t L = 1500;
    std::vector<uint8_t> host(n_all * L);
    uint64_t x = 0x5EA57A2C;
    for (auto& b : host) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        b = uint8_t(x >> 56);
    }
    for (uint64_t i = 0; i < n_all; ++i) {  // IPv4 / UDP headers, fields as sent
        uint8_t* f = host.data() + i * L;
        f[0] = 0x45; f[1] = 0; f[2] = L >> 8; f[3] = L & 0xff;
        f[6] = f[7] = 0; f[8] = 64; f[9] = 17;
    }
    std::vector<uint64_t> off(n_all);
    std::vector<uint32_t> len(n_all, L);
    for (uint64_t i = 0; i < n_all; ++i) off[i] = i * L;
    SC_OK(sccsum_init(0));
    if (const char* tb = std::getenv("ENGINE_STEPS_TILE_BYTES")) SC_OK(sccsum_set_tile_bytes(std::atoi(tb)));  // A/B
    void* d_bytes;
    uint64_t* d_off;
    uint32_t* d_len;
    uint8_t* d_st;
    uint16_t* d_out2;
    HIP_OK(hipMalloc(&d_bytes, host.size() + 16));
    HIP_OK(hipMalloc(&d_out2, n_all * 4));
    HIP_OK(hipMalloc(&d_off, n_all * 8));
    HIP_OK(hipMalloc(&d_len, n_all * 4));
    HIP_OK(hipMalloc(&d_st, n_all));
    HIP_OK(hipMemcpy(d_bytes, host.data(), host.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off.data(), n_all * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len.data(), n_all * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    HIP_OK(hipStreamCreate(&s));
    if (const char* fs = std::getenv("ENGINE_STEPS_FILL_SINGLE_MAX")) SC_OK(sccsum_set_fill_single_max(std::atoi(fs)));
    if (const char* dy = std::getenv("ENGINE_STEPS_DYNAMIC")) SC_OK(sccsum_set_dynamic_tiles(std::atoi(dy)));  // A/B
    if (const char* va = std::getenv("ENGINE_STEPS_VARIANT")) SC_OK(sccsum_set_kernel_variant(std::atoi(va)));  // A/B
    const uint32_t sizes[] = {32, 128, 1024, 16384, 65536, 262144};
    if (producers) {
        for (uint32_t B : sizes) {
            if (B > 1024) continue;
            const uint64_t slices = n_all / B;
            const uint64_t k = B <= 128 ? 40000 : 10000;
            sccsum_engine* e = nullptr;
            SC_OK(sccsum_engine_create(0, SCCSUM_PIPE_IPV4, ring, mif, &e));
            (void)producers_run(e, s, 1, 256, B, slices, d_bytes, host.size(), d_off, d_len, d_st);  // warm
            const double one = producers_run(e, s, 1, k, B, slices, d_bytes, host.size(), d_off, d_len, d_st);
            const double many = producers_run(e, s, nprod, k, B, slices, d_bytes, host.size(), d_off, d_len, d_st);
            SC_OK(sccsum_engine_destroy(e));
            if (one < 0 || many < 0) {
                std::printf("producers: an engine call failed\n");
                return 4;
            }
            std::printf("{\"form\": \"producers\", \"packets_per_step\": %u, \"steps\": %llu, \"ring\": %u, "
                        "\"one_thread_us_per_step\": %.2f, \"threads\": %d, \"threads_us_per_step\": %.2f, "
                        "\"threads_GiBps\": %.1f}\n",
                        B, (unsigned long long)k, ring, one, nprod, many, double(B) * L / (many * 1e-6) / (1u << 30));
            std::fflush(stdout);
        }
        return 0;
    }
    for (uint32_t B : sizes) {
        if (!fill && B > 16384) continue;
        const uint64_t slices = n_all / B;
        const uint64_t k = B <= 128 ? 20000 : (B <= 1024 ? 5000 : (B <= 16384 ? 400 : 100));
        // a slice: B frames; its offsets are absolute in the one buffer (each step
        // reads its own B frames: distinct slices, rotating)
        auto slice = [&](uint64_t j) {
            sccsum_batch b{};
            const uint64_t q = j % slices;
            b.d_bytes = d_bytes;
            b.bytes_len = host.size();
            b.d_off = d_off + q * B;
            b.d_len = d_len + q * B;
            b.d_status = d_st + q * B;
            b.d_out = fill ? d_out2 + 2 * q * B : nullptr;
            b.n = B;
            return b;
        };
        auto launch = [&](const sccsum_batch& b) {
            return fill ? sccsum_ipv4_fill(const_cast<void*>(b.d_bytes), b.bytes_len, b.d_off, b.d_len, static_cast<uint16_t*>(b.d_out),
                                           b.d_status, B, L, mode, s)
                        : sccsum_ipv4_frames(b.d_bytes, b.bytes_len, b.d_off, b.d_len, nullptr, b.d_status, B, L, s);
        };
        // launches
        for (uint64_t j = 0; j < 64; ++j) SC_OK(launch(slice(j)));
        HIP_OK(hipStreamSynchronize(s));
        double t0 = now_s();
        for (uint64_t j = 0; j < k; ++j) SC_OK(launch(slice(j)));
        HIP_OK(hipStreamSynchronize(s));
        const double launch_s = now_s() - t0;
        // engine
        sccsum_engine* e = nullptr;
        SC_OK(sccsum_engine_create(0, SCCSUM_PIPE_IPV4 | (fill ? SCCSUM_ENGINE_FILL : 0), ring, mif, &e));
        double engine_s = 0;
        for (int run = 0; run < 2; ++run) {  // the first run warms up
            const uint64_t kk = run ? k : 64;
            SC_OK(sccsum_engine_start(e, s));
            uint64_t step = 0;
            t0 = now_s();
            for (uint64_t j = 0; j < kk; ++j) {
                const sccsum_batch b = slice(j);
                if (fill) {
                    SC_OK(sccsum_engine_submit_fill(e, &b, 1, L, mode, 10'000'000'000ull, &step));
                } else {
                    SC_OK(sccsum_engine_submit(e, &b, 1, L, 10'000'000'000ull, &step));
                }
            }
            SC_OK(sccsum_engine_wait(e, step, 10'000'000'000ull));
            if (run) engine_s = now_s() - t0;
            SC_OK(sccsum_engine_stop(e));
            HIP_OK(hipStreamSynchronize(s));
        }
        SC_OK(sccsum_engine_destroy(e));
        // (a timing probe: the checksum fields are random, so most frames fail their checks; the
        // engine's results are checked against the oracle by tests/test_gpu_engine.py)
        const double bytes = double(k) * B * L;
        std::printf("{\"form\": \"%s\", \"packets_per_step\": %u, \"steps\": %llu, \"launch_us_per_step\": %.2f, "
                    "\"launch_GiBps\": %.1f, \"engine_us_per_step\": %.2f, \"engine_GiBps\": %.1f, "
                    "\"engine_over_launch\": %.2f, \"ring\": %u}\n",
                    fill ? "fill" : "verify", B, (unsigned long long)k, launch_s / k * 1e6, bytes / launch_s / (1u << 30), engine_s / k * 1e6,
                    bytes / engine_s / (1u << 30), launch_s / engine_s, ring);
        std::fflush(stdout);
    }
    return 0;
}
