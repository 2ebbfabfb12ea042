// Seastar's threading model: one reactor thread per shard
// (src/core/reactor.cc:3437-3438), shard i on device i % (visible devices),
// so every visible device's counter pool and launch sizing are used; with
// several devices each shard also checks that a launch on another device's
// stream is refused (SCCSUM_EINVAL).  Each shard binds itself with sccsum_init,
// owning its streams, its batches and a burst queue, and launching at the
// same time as every other shard: frames (verify), seeded spans, a multi
// launch, the in-place fill, a burst queue fed one frame at a time, and a
// loop that creates a stream, launches on it and destroys it without waiting
// (a new stream may get the old one's address while that launch still runs).
// Every result is checked against the oracle (test infrastructure, linked
// into this test program only).  Usage: shards_gpu [threads] [rounds].
//
// shards_gpu engine [threads] [steps]: the shards of ONE GPU feeding its one
// resident engine (include/sccsum.h, "Producers"; Seastar's per-core
// reactors, src/core/reactor.cc:3437-3441, forwarding to the GPU's owner,
// src/net/net.cc:309-322): a frames + fill engine with a 64-slot ring, then a
// spans engine, each taking random steps from every thread at once (some after
// runs of steps without tiles) — frames
// (generate, verify-only, both), in-place fills, seeded spans — every step's
// results against the oracle.
#include <hip/hip_runtime.h>

#include "sccsum.h"
#include "sccsum_diag.h"
#include "sccsum_oracle.h"

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

namespace {

std::atomic<int> g_bad{0};
std::mutex g_print;
unsigned long long g_devices_used = 0;  // under g_print
std::atomic<int> g_cross_checked{0};    // launches refused on another device's stream
long g_engine_steps = 0;                // under g_print: steps the engine producers checked
std::vector<sccsum_burst*> g_queues;    // under g_print: the shards' drained burst queues, destroyed by main

void fail(int shard, const char* what, long i) {
    if (g_bad.fetch_add(1) < 20) {
        std::lock_guard<std::mutex> l(g_print);
        std::printf("shard %d: %s mismatch at %ld\n", shard, what, i);
    }
}

bool hip_ok(hipError_t e, int shard, const char* what) {
    if (e == hipSuccess) return true;
    std::lock_guard<std::mutex> l(g_print);
    std::printf("shard %d: %s: %s\n", shard, what, hipGetErrorString(e));
    g_bad.fetch_add(1);
    return false;
}

bool ok(int rc, int shard, const char* what) {
    if (rc == SCCSUM_OK) return true;
    std::lock_guard<std::mutex> l(g_print);
    std::printf("shard %d: %s: %s\n", shard, what, sccsum_strerror(rc));
    g_bad.fetch_add(1);
    return false;
}

// IPv4 frames as the native stack sees them: UDP / TCP / ICMP (echo requests
// among them), IP fragments, options, padding, runts, odd offsets.
struct Frames {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
};

Frames make_frames(std::mt19937_64& rng, uint32_t n) {
    Frames F;
    F.off.resize(n);
    F.len.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t L = 20 + static_cast<uint32_t>(rng() % 3000);
        if (rng() % 64 == 0) L = static_cast<uint32_t>(rng() % 20);
        F.off[i] = F.bytes.size() + rng() % 4;
        F.len[i] = L;
        F.bytes.resize(F.off[i] + L);
        uint8_t* f = F.bytes.data() + F.off[i];
        for (uint32_t k = 0; k < L; ++k) f[k] = static_cast<uint8_t>(rng());
        if (L < 20) continue;
        const uint32_t ihl = rng() % 8 == 0 ? 6 + rng() % 4 : 5;
        const uint32_t ip_len = rng() % 10 == 0 ? L - static_cast<uint32_t>(rng() % 8) : L;
        f[0] = static_cast<uint8_t>(0x40 | ihl);
        f[2] = static_cast<uint8_t>(ip_len >> 8);
        f[3] = static_cast<uint8_t>(ip_len);
        const uint32_t r = rng() % 10;
        const uint32_t fragw = r == 0 ? 0x2000 : (r == 1 ? 0x2000 | (rng() % 0x100) : (r == 2 ? rng() % 0x100 : 0));
        f[6] = static_cast<uint8_t>(fragw >> 8);
        f[7] = static_cast<uint8_t>(fragw);
        const uint8_t protos[3] = {17, 6, 1};
        f[9] = protos[rng() % 3];
        if (f[9] == 1 && ip_len > 4 * ihl && rng() % 4 != 0) f[4 * ihl] = 8;  // echo request
    }
    F.bytes.resize(F.bytes.size() + 16);
    return F;
}

struct DevBatch {
    uint8_t* bytes = nullptr;
    uint64_t* off = nullptr;
    uint32_t* len = nullptr;
    uint64_t n = 0, bytes_len = 0;
};

bool upload(const Frames& F, DevBatch& D, int shard) {
    D.n = F.off.size();
    D.bytes_len = F.bytes.size();
    return hip_ok(hipMalloc(&D.bytes, (D.bytes_len + 15) & ~uint64_t(15)), shard, "malloc") &&
           hip_ok(hipMalloc(&D.off, D.n * 8), shard, "malloc") && hip_ok(hipMalloc(&D.len, D.n * 4), shard, "malloc") &&
           hip_ok(hipMemcpy(D.bytes, F.bytes.data(), D.bytes_len, hipMemcpyHostToDevice), shard, "copy") &&
           hip_ok(hipMemcpy(D.off, F.off.data(), D.n * 8, hipMemcpyHostToDevice), shard, "copy") &&
           hip_ok(hipMemcpy(D.len, F.len.data(), D.n * 4, hipMemcpyHostToDevice), shard, "copy");
}

void release(DevBatch& D) {
    (void)hipFree(D.bytes);
    (void)hipFree(D.off);
    (void)hipFree(D.len);
}

template <typename T>
std::vector<T> fetch(const T* d, size_t count, int shard) {
    std::vector<T> h(count);
    hip_ok(hipMemcpy(h.data(), d, count * sizeof(T), hipMemcpyDeviceToHost), shard, "fetch");
    return h;
}

struct BurstSink {
    std::vector<uint16_t> out;
    std::vector<uint8_t> st;
};

void burst_done(void* user, uint64_t first, uint32_t count, const uint16_t* results, const uint8_t* status) {
    auto* S = static_cast<BurstSink*>(user);
    for (uint32_t k = 0; k < count; ++k) {
        S->out[2 * (first + k)] = results[2 * k];
        S->out[2 * (first + k) + 1] = results[2 * k + 1];
        S->st[first + k] = status[k];
    }
}

void shard_main(int shard, int rounds) {
    // shard i on device i % ndev (this_shard_id() % ngpus), so
    // every visible device's counter pool and CU count are exercised
    int ndev = 0;
    if (!ok(sccsum_device_count(&ndev), shard, "device count") || ndev < 1) return;
    const int dev = shard % ndev;
    if (!ok(sccsum_init(dev), shard, "sccsum_init")) return;
    {
        std::lock_guard<std::mutex> l(g_print);
        g_devices_used |= 1ull << dev;
    }
    // per-thread knobs: each shard runs another kernel form; none leaks into another shard
    const int forms[6] = {0, 16, 15, 14, 1, 2};
    if (!ok(sccsum_set_kernel_variant(forms[shard % 6]), shard, "variant")) return;
    std::mt19937_64 rng(0x5EA57A2Cull + 7919ull * shard);
    const uint32_t n = 6000 + 1000 * (shard % 3);
    Frames A = make_frames(rng, n), B = make_frames(rng, n / 2);
    // oracle results
    std::vector<uint16_t> wantA(2 * A.off.size()), wantB(2 * B.off.size());
    std::vector<uint8_t> wstA(A.off.size()), wstB(B.off.size());
    oracle_batch_ipv4(A.bytes.data(), A.off.data(), A.len.data(), wantA.data(), wstA.data(), A.off.size(), 1);
    oracle_batch_ipv4(B.bytes.data(), B.off.data(), B.len.data(), wantB.data(), wstB.data(), B.off.size(), 1);
    std::vector<uint32_t> seeds(n);
    for (auto& s : seeds) s = static_cast<uint32_t>(rng() & 0xffff);
    std::vector<uint16_t> want_sp(n);
    oracle_batch_spans(A.bytes.data(), A.off.data(), A.len.data(), seeds.data(), want_sp.data(), n, 1);
    const uint32_t fmode = SCCSUM_FILL_IP | SCCSUM_FILL_L4 | SCCSUM_FILL_ICMP_ECHO;
    std::vector<uint8_t> want_fill = A.bytes;
    std::vector<uint16_t> want_fout(2 * n);
    std::vector<uint8_t> want_fst(n);
    oracle_batch_ipv4_fill(want_fill.data(), A.off.data(), A.len.data(), want_fout.data(), want_fst.data(), n, fmode);

    DevBatch dA, dB;
    if (!upload(A, dA, shard) || !upload(B, dB, shard)) return;
    uint8_t* fill_bytes = nullptr;
    uint16_t *o1 = nullptr, *o2 = nullptr, *o3 = nullptr, *osp = nullptr, *ofill = nullptr;
    uint8_t *s1 = nullptr, *s2 = nullptr, *ssp = nullptr, *sfill = nullptr;
    uint32_t* d_seed = nullptr;
    const int kTemp = 8;  // launches on streams destroyed without a sync, per round
    uint16_t* otemp = nullptr;
    if (!hip_ok(hipMalloc(&fill_bytes, (dA.bytes_len + 15) & ~uint64_t(15)), shard, "malloc") ||
        !hip_ok(hipMalloc(&o1, 4 * n), shard, "malloc") || !hip_ok(hipMalloc(&o2, 4 * n), shard, "malloc") ||
        !hip_ok(hipMalloc(&o3, 4 * n), shard, "malloc") || !hip_ok(hipMalloc(&osp, 2 * n), shard, "malloc") ||
        !hip_ok(hipMalloc(&ofill, 4 * n), shard, "malloc") || !hip_ok(hipMalloc(&s1, n), shard, "malloc") ||
        !hip_ok(hipMalloc(&s2, n), shard, "malloc") || !hip_ok(hipMalloc(&ssp, n), shard, "malloc") ||
        !hip_ok(hipMalloc(&sfill, n), shard, "malloc") || !hip_ok(hipMalloc(&d_seed, 4 * n), shard, "malloc") ||
        !hip_ok(hipMalloc(&otemp, size_t(4) * n * kTemp), shard, "malloc") ||
        !hip_ok(hipMemcpy(d_seed, seeds.data(), 4 * n, hipMemcpyHostToDevice), shard, "copy")) {
        return;
    }
    hipStream_t s0, sx;
    if (!hip_ok(hipStreamCreate(&s0), shard, "stream") || !hip_ok(hipStreamCreate(&sx), shard, "stream")) return;
    if (ndev > 1) {
        // a stream of another device is refused (sccsum.h: launches run on the
        // stream's device, which must be the calling thread's current one)
        hipStream_t other;
        const int od = (dev + 1) % ndev;
        if (hip_ok(hipSetDevice(od), shard, "set other device") && hip_ok(hipStreamCreate(&other), shard, "stream")) {
            hip_ok(hipSetDevice(dev), shard, "set device back");
            const int rc = sccsum_ipv4_frames(dA.bytes, dA.bytes_len, dA.off, dA.len, o1, s1, n, 3100, other);
            if (rc != SCCSUM_EINVAL) fail(shard, "stream of another device accepted", rc);
            g_cross_checked.fetch_add(1);
            hip_ok(hipSetDevice(od), shard, "set other device");
            (void)hipStreamDestroy(other);
        }
        hip_ok(hipSetDevice(dev), shard, "set device back");
    }
    auto check2 = [&](const std::vector<uint16_t>& got, const std::vector<uint16_t>& want, const char* what) {
        for (size_t i = 0; i < want.size(); ++i) {
            if (got[i] != want[i]) {
                fail(shard, what, static_cast<long>(i));
                return;
            }
        }
    };
    for (int round = 0; round < rounds; ++round) {
        // frames + status on s0; seeded spans on sx; a multi launch over A and B on s0
        ok(sccsum_ipv4_frames(dA.bytes, dA.bytes_len, dA.off, dA.len, o1, s1, n, 3100, s0), shard, "frames");
        ok(sccsum_spans(dA.bytes, dA.bytes_len, dA.off, dA.len, d_seed, osp, ssp, n, 3100, sx), shard, "spans");
        sccsum_batch mb[2] = {{dA.bytes, dA.bytes_len, dA.off, dA.len, nullptr, o2, nullptr, n},
                              {dB.bytes, dB.bytes_len, dB.off, dB.len, nullptr, o3, s2, dB.n}};
        ok(sccsum_ipv4_frames_multi(mb, 2, 3100, s0), shard, "multi");
        // in place, on a fresh copy of A
        hip_ok(hipMemcpyAsync(fill_bytes, dA.bytes, dA.bytes_len, hipMemcpyDeviceToDevice, sx), shard, "copy");
        ok(sccsum_ipv4_fill(fill_bytes, dA.bytes_len, dA.off, dA.len, ofill, sfill, n, 3100, fmode, sx), shard, "fill");
        // streams created, launched on and destroyed without waiting
        hipEvent_t ev[kTemp];
        for (int k = 0; k < kTemp; ++k) {
            hipStream_t t;
            hip_ok(hipStreamCreateWithFlags(&t, hipStreamNonBlocking), shard, "stream");
            ok(sccsum_ipv4_frames(dA.bytes, dA.bytes_len, dA.off, dA.len, otemp + size_t(2) * n * k, nullptr, n, 3100,
                                  t),
               shard, "frames (temp stream)");
            hip_ok(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), shard, "event");
            hip_ok(hipEventRecord(ev[k], t), shard, "event");
            hip_ok(hipStreamDestroy(t), shard, "stream destroy");
        }
        hip_ok(hipStreamSynchronize(s0), shard, "sync");
        hip_ok(hipStreamSynchronize(sx), shard, "sync");
        for (int k = 0; k < kTemp; ++k) {
            hip_ok(hipEventSynchronize(ev[k]), shard, "event sync");
            (void)hipEventDestroy(ev[k]);
        }
        check2(fetch(o1, 2 * n, shard), wantA, "frames");
        if (fetch(s1, n, shard) != wstA) fail(shard, "frames status", round);
        check2(fetch(osp, n, shard), want_sp, "spans");
        check2(fetch(o2, 2 * n, shard), wantA, "multi batch 0");
        check2(fetch(o3, 2 * dB.n, shard), wantB, "multi batch 1");
        if (fetch(s2, dB.n, shard) != wstB) fail(shard, "multi status", round);
        check2(fetch(ofill, 2 * n, shard), want_fout, "fill values");
        if (fetch(sfill, n, shard) != want_fst) fail(shard, "fill status", round);
        const std::vector<uint8_t> fb = fetch(fill_bytes, dA.bytes_len, shard);
        if (std::memcmp(fb.data(), want_fill.data(), dA.bytes_len) != 0) fail(shard, "fill bytes", round);
        const std::vector<uint16_t> ot = fetch(otemp, size_t(2) * n * kTemp, shard);
        for (int k = 0; k < kTemp; ++k) {
            if (std::memcmp(ot.data() + size_t(2) * n * k, wantA.data(), 4 * size_t(n)) != 0) {
                fail(shard, "frames on a destroyed stream", k);
            }
        }
    }
    // the shard's burst queue: frames handed over one at a time (host memory)
    BurstSink sink;
    sink.out.assign(2 * n, 0xEEEE);
    sink.st.assign(n, 0xEE);
    sccsum_burst* q = nullptr;
    if (ok(sccsum_burst_create(dev, SCCSUM_PIPE_IPV4, 1u << 20, 256, 20000, 4, burst_done, &sink, &q), shard,
           "burst create")) {
        for (uint32_t i = 0; i < n; ++i) {
            sccsum_fragment fr{A.bytes.data() + A.off[i], A.len[i]};
            int rc;
            while ((rc = sccsum_burst_submit(q, &fr, 1, 0, nullptr)) == SCCSUM_EBUSY) ok(sccsum_burst_poll(q, nullptr), shard, "poll");
            ok(rc, shard, "burst submit");
            if (i % 32 == 31) ok(sccsum_burst_poll(q, nullptr), shard, "poll");
        }
        ok(sccsum_burst_drain(q), shard, "drain");
        // destroyed by main once every shard has joined: a queue's pinned
        // staging freed now could be handed to another shard's queue while it
        // runs, a reuse ThreadSanitizer cannot see through the ROCm allocator
        {
            std::lock_guard<std::mutex> l(g_print);
            g_queues.push_back(q);
        }
        check2(sink.out, wantA, "burst");
        if (sink.st != wstA) fail(shard, "burst status", 0);
    }
    (void)hipStreamDestroy(s0);
    (void)hipStreamDestroy(sx);
    for (void* p : {static_cast<void*>(fill_bytes), static_cast<void*>(o1), static_cast<void*>(o2),
                    static_cast<void*>(o3), static_cast<void*>(osp), static_cast<void*>(ofill), static_cast<void*>(s1),
                    static_cast<void*>(s2), static_cast<void*>(ssp), static_cast<void*>(sfill),
                    static_cast<void*>(d_seed), static_cast<void*>(otemp)}) {
        (void)hipFree(p);
    }
    release(dA);
    release(dB);
}

// ---- the shards of one GPU feeding its one resident engine ---------------------

// A start line every producer waits at (C++17: no std::barrier).
struct Gate {
    std::mutex mu;
    std::condition_variable cv;
    int waiting = 0, generation = 0;
    void arrive(int parties) {
        std::unique_lock<std::mutex> l(mu);
        const int gen = generation;
        if (++waiting == parties) {
            waiting = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return generation != gen; });
        }
    }
};

struct ProducerStep {
    int kind;          // 0 frames (A generate + B verify-only), 1 A verify-only, 2 fill of copy r, 3 spans
    int round;
    uint64_t step;
};

// One shard: its own frames and buffers (uploaded before the run: while the
// grid runs, a device-to-device copy would queue behind it), `steps` random
// steps submitted into the shared engine (sometimes waiting on one), and after
// the owner's stop every result against the oracle.  gate: 0 = buffers ready,
// 1 = submits done, 2 = the run has stopped.
void producer_main(int shard, sccsum_engine* e, bool spans, int steps, Gate* gate, int parties) {
    std::mt19937_64 rng(0xE61E5ull + 104729ull * shard + (spans ? 7 : 0));
    if (!ok(sccsum_init(0), shard, "sccsum_init")) {
        for (int k = 0; k < 4; ++k) gate->arrive(parties);
        return;
    }
    const uint32_t n = 200 + static_cast<uint32_t>(rng() % 600);
    Frames A = make_frames(rng, n), B = make_frames(rng, n / 3 + 1);
    std::vector<uint16_t> wantA(2 * n), wantB(2 * B.off.size()), want_sp(n), want_fout(2 * n);
    std::vector<uint8_t> wstA(n), wstB(B.off.size()), want_fst(n), want_fill = A.bytes;
    std::vector<uint32_t> seeds(n);
    for (auto& s : seeds) s = static_cast<uint32_t>(rng() & 0xffff);
    const uint32_t fmode = SCCSUM_FILL_IP | SCCSUM_FILL_L4 | SCCSUM_FILL_ICMP_ECHO;
    oracle_batch_ipv4(A.bytes.data(), A.off.data(), A.len.data(), wantA.data(), wstA.data(), n, 1);
    oracle_batch_ipv4(B.bytes.data(), B.off.data(), B.len.data(), wantB.data(), wstB.data(), B.off.size(), 1);
    oracle_batch_spans(A.bytes.data(), A.off.data(), A.len.data(), seeds.data(), want_sp.data(), n, 1);
    oracle_batch_ipv4_fill(want_fill.data(), A.off.data(), A.len.data(), want_fout.data(), want_fst.data(), n, fmode);
    DevBatch dA, dB;
    const size_t cap = (A.bytes.size() + 15) & ~size_t(15);
    uint8_t *fills = nullptr, *st = nullptr;
    uint16_t* outs = nullptr;
    uint32_t* d_seed = nullptr;
    // per step: 2n + 2|B| values, n + 1 status bytes; a fill copy of A per step
    const size_t per_out = 2 * (size_t(n) + B.off.size()), per_st = n;
    bool good = upload(A, dA, shard) && upload(B, dB, shard) &&
                hip_ok(hipMalloc(&fills, cap * steps), shard, "malloc") &&
                hip_ok(hipMalloc(&outs, 2 * per_out * steps), shard, "malloc") &&
                hip_ok(hipMalloc(&st, per_st * steps), shard, "malloc") &&
                hip_ok(hipMalloc(&d_seed, 4 * n), shard, "malloc") &&
                hip_ok(hipMemcpy(d_seed, seeds.data(), 4 * n, hipMemcpyHostToDevice), shard, "copy") &&
                hip_ok(hipMemset(outs, 0xEE, 2 * per_out * steps), shard, "memset") &&
                hip_ok(hipMemset(st, 0xEE, per_st * steps), shard, "memset");
    for (int r = 0; good && r < steps; ++r) {
        good = hip_ok(hipMemcpy(fills + cap * r, A.bytes.data(), A.bytes.size(), hipMemcpyHostToDevice), shard,
                      "copy");
    }
    good = good && hip_ok(hipDeviceSynchronize(), shard, "sync");
    std::vector<ProducerStep> done;
    gate->arrive(parties);  // 0: every shard's buffers are in place; the owner starts the run
    gate->arrive(parties);  // (the run is started)
    for (int r = 0; good && r < steps; ++r) {
        uint16_t* o = outs + per_out * r;
        uint8_t* s = st + per_st * r;
        ProducerStep ps{spans ? 3 : static_cast<int>(rng() % 3), r, 0};
        int rc = SCCSUM_OK;
        if (rng() % 4 == 0) {  // a run of steps without tiles first (each done once the grid has copied it)
            const sccsum_batch z = {dA.bytes, 0, dA.off, dA.len, nullptr, o, s, 0};
            uint64_t zs = 0;
            for (int k = 1 + static_cast<int>(rng() % 20); k > 0 && rc == SCCSUM_OK; --k) {
                rc = sccsum_engine_submit(e, &z, 1, 3100, 10'000'000'000ull, &zs);
            }
            if (!ok(rc, shard, "engine submit (no tiles)")) break;
            if (rng() % 2 == 0 && !ok(sccsum_engine_wait(e, zs, 10'000'000'000ull), shard, "engine wait (no tiles)")) {
                break;
            }
        }
        if (ps.kind == 3) {
            const sccsum_batch b = {dA.bytes, dA.bytes_len, dA.off, dA.len, d_seed, o, s, n};
            rc = sccsum_engine_submit(e, &b, 1, 3100, 10'000'000'000ull, &ps.step);
        } else if (ps.kind == 0) {
            const sccsum_batch b[2] = {{dA.bytes, dA.bytes_len, dA.off, dA.len, nullptr, o, nullptr, n},
                                       {dB.bytes, dB.bytes_len, dB.off, dB.len, nullptr, o + 2 * n, s, dB.n}};
            rc = sccsum_engine_submit(e, b, 2, 3100, 10'000'000'000ull, &ps.step);
        } else if (ps.kind == 1) {
            const sccsum_batch b = {dA.bytes, dA.bytes_len, dA.off, dA.len, nullptr, nullptr, s, n};
            rc = sccsum_engine_submit(e, &b, 1, 3100, 10'000'000'000ull, &ps.step);
        } else {
            const sccsum_batch b = {fills + cap * r, dA.bytes_len, dA.off, dA.len, nullptr, o, s, n};
            rc = sccsum_engine_submit_fill(e, &b, 1, 3100, fmode, 10'000'000'000ull, &ps.step);
        }
        if (!ok(rc, shard, "engine submit")) break;
        done.push_back(ps);
        if (rng() % 8 == 0) ok(sccsum_engine_wait(e, ps.step, 10'000'000'000ull), shard, "engine wait");
    }
    for (const ProducerStep& ps : done) ok(sccsum_engine_wait(e, ps.step, 10'000'000'000ull), shard, "engine wait");
    gate->arrive(parties);  // 1: submits done
    gate->arrive(parties);  // 2: the owner stopped the run (device copies run again)
    if (good) {
        const std::vector<uint16_t> ho = fetch(outs, per_out * steps, shard);
        const std::vector<uint8_t> hs = fetch(st, per_st * steps, shard);
        const std::vector<uint8_t> hf = fetch(fills, cap * steps, shard);
        for (const ProducerStep& ps : done) {
            const uint16_t* o = ho.data() + per_out * ps.round;
            const uint8_t* s = hs.data() + per_st * ps.round;
            bool same = true;
            if (ps.kind == 3) {
                same = std::memcmp(o, want_sp.data(), 2 * size_t(n)) == 0;
                for (uint32_t i = 0; same && i < n; ++i) same = s[i] == (want_sp[i] == 0 ? 1 : 0);
            } else if (ps.kind == 0) {
                same = std::memcmp(o, wantA.data(), 4 * size_t(n)) == 0 &&
                       std::memcmp(o + 2 * n, wantB.data(), 4 * B.off.size()) == 0 &&
                       std::memcmp(s, wstB.data(), B.off.size()) == 0;
            } else if (ps.kind == 1) {
                same = std::memcmp(s, wstA.data(), n) == 0;
            } else {
                same = std::memcmp(o, want_fout.data(), 4 * size_t(n)) == 0 &&
                       std::memcmp(s, want_fst.data(), n) == 0 &&
                       std::memcmp(hf.data() + cap * ps.round, want_fill.data(), A.bytes.size()) == 0;
            }
            if (!same) fail(shard, ps.kind == 3 ? "engine spans step" : (ps.kind == 2 ? "engine fill step"
                                                                        : "engine frames step"), ps.round);
        }
    }
    for (void* q : {static_cast<void*>(fills), static_cast<void*>(outs), static_cast<void*>(st),
                    static_cast<void*>(d_seed)}) {
        (void)hipFree(q);
    }
    release(dA);
    release(dB);
    std::lock_guard<std::mutex> l(g_print);
    g_engine_steps += static_cast<long>(done.size());
}

// One engine run fed by `threads` producers: frames + fills, or spans.
int engine_run(int threads, int steps, bool spans) {
    if (sccsum_init(0) != SCCSUM_OK) return 1;
    sccsum_engine* e = nullptr;
    const sccsum_engine_opts o = {64, 16, 0, 0};  // a 64-slot ring: every slot reused many times
    if (!ok(sccsum_engine_create_opts(0, spans ? SCCSUM_PIPE_SPANS : (SCCSUM_PIPE_IPV4 | SCCSUM_ENGINE_FILL), &o, &e),
            -1, "engine create")) {
        return 1;
    }
    hipStream_t s;
    if (!hip_ok(hipStreamCreate(&s), -1, "stream")) return 1;
    Gate gate;
    const int parties = threads + 1;
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(producer_main, t, e, spans, steps, &gate, parties);
    gate.arrive(parties);  // 0: buffers in place
    const bool started = ok(sccsum_engine_start(e, s), -1, "engine start");
    gate.arrive(parties);  // the run is started (a producer's submit on a stopped engine is SCCSUM_EINVAL)
    gate.arrive(parties);  // 1: every producer's steps are done
    if (started) {
        ok(sccsum_engine_stop(e), -1, "engine stop");
        hip_ok(hipStreamSynchronize(s), -1, "sync");
    }
    gate.arrive(parties);  // 2
    for (auto& t : ts) t.join();
    ok(sccsum_engine_destroy(e), -1, "engine destroy");
    (void)hipStreamDestroy(s);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "engine") == 0) {
        const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
        const int steps = argc > 3 ? std::atoi(argv[3]) : 40;
        engine_run(threads, steps, false);
        const long frame_steps = g_engine_steps;
        engine_run(threads, steps, true);
        if (g_bad.load()) {
            std::printf("shards_gpu engine: FAILED (%d)\n", g_bad.load());
            return 1;
        }
        std::printf("shards_gpu engine: OK (%d producer threads into one engine per run: %ld frame / fill steps, "
                    "then %ld span steps, every result against the oracle)\n",
                    threads, frame_steps, g_engine_steps - frame_steps);
        return 0;
    }
    const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(shard_main, t, rounds);
    for (auto& t : ts) t.join();
    for (sccsum_burst* q : g_queues) ok(sccsum_burst_destroy(q), -1, "burst destroy");
    if (g_bad.load()) {
        std::printf("shards_gpu: FAILED (%d)\n", g_bad.load());
        return 1;
    }
    int ndev = 0;
    (void)sccsum_device_count(&ndev);
    std::printf("shards_gpu: OK (%d shards x %d rounds on %d device%s, mask 0x%llx: frames, spans, multi, fill, %d "
                "launches on destroyed streams per round, burst queue; %d launches on another device's stream "
                "refused)\n",
                threads, rounds, ndev, ndev == 1 ? "" : "s", g_devices_used, 8, g_cross_checked.load());
    return 0;
}
