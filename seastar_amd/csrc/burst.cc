// burst.cc — the burst-batching hook at the qp boundary.
//
// The native stack checksums packet by packet on the shard's reactor thread:
// qp::poll_tx refills up to 128 packets per poll (src/net/net.cc:81-105), DPDK
// rx hands over bursts of 32 (src/net/dpdk.cc:2190-2204).  A burst queue
// accumulates those packets into GPU batches and completes them
// asynchronously.  It is shaped like a reactor poller (pollfn::poll,
// include/seastar/core/internal/poll.hh:26-29, registered as net.cc:109 does):
// every call but drain is non-blocking and sccsum_burst_poll reports whether
// it did work.
//
//   submit:  copy the packet's fragments (sccsum_fragment = the layout of
//            seastar::net::fragment, packet.hh:43-46) back to back into the
//            open slot's pinned staging, starting 16-byte aligned (full-rate
//            loads); landing contiguously keeps checksummer::sum(const
//            packet&)'s odd carry (ip_checksum.cc:64-68) with no device work.
//            SCCSUM_EBUSY when every slot is in flight (poll, then retry)
//   poll:    launch the open slot when full (bytes / packets) or older than
//            max_delay_ns — on the slot's own stream: H2D of the staged bytes
//            + metadata, the kernel, D2H of the results, an event, so one
//            batch's copies overlap the previous batch's kernel; then deliver
//            every finished slot, oldest first, through the completion
//            callback (results in submit order, tickets consecutive)
//   drain:   launch what is staged, wait for everything, deliver
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "sccsum.h"

struct sccsum_burst {
    enum class state { free, open, inflight };
    struct Slot {
        state st = state::free;
        hipStream_t stream = nullptr;
        uint8_t* h_bytes = nullptr;  // pinned staging: packets back to back
        uint64_t* h_off = nullptr;
        uint32_t* h_len = nullptr;
        uint32_t* h_seed = nullptr;
        uint16_t* h_out = nullptr;
        uint8_t* h_status = nullptr;
        uint8_t* d_bytes = nullptr;
        uint64_t* d_off = nullptr;
        uint32_t* d_len = nullptr;
        uint32_t* d_seed = nullptr;
        uint16_t* d_out = nullptr;
        uint8_t* d_status = nullptr;
        hipEvent_t done = nullptr;
        uint64_t used = 0;  // staged bytes
        uint32_t npk = 0;
        uint32_t max_len = 0;
        uint64_t first_ticket = 0;
        std::chrono::steady_clock::time_point opened{};
    };
    int device = 0;
    int mode = SCCSUM_PIPE_SPANS;
    uint64_t batch_bytes = 0;
    uint32_t batch_packets = 0;
    uint64_t max_delay_ns = 0;
    sccsum_burst_done_fn fn = nullptr;
    void* user = nullptr;
    std::vector<Slot> slots;
    size_t open = SIZE_MAX;  // index of the open slot, if any
    size_t next_launch = 0;  // slots open, launch and deliver in ring order
    size_t next_deliver = 0;
    uint64_t next_ticket = 0;
    uint64_t inflight = 0;
};

namespace {

int hip_rc(hipError_t e) { return e == hipSuccess ? SCCSUM_OK : static_cast<int>(e); }

#define SCCSUM_TRY(x)                     \
    do {                                  \
        const int rc_ = hip_rc(x);        \
        if (rc_ != SCCSUM_OK) return rc_; \
    } while (0)

void free_slot(sccsum_burst::Slot& s) {
    (void)hipHostFree(s.h_bytes);
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_seed);
    (void)hipHostFree(s.h_out);
    (void)hipHostFree(s.h_status);
    (void)hipFree(s.d_bytes);
    (void)hipFree(s.d_off);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_seed);
    (void)hipFree(s.d_out);
    (void)hipFree(s.d_status);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
}

int width(const sccsum_burst* b) { return b->mode == SCCSUM_PIPE_IPV4 ? 2 : 1; }

int launch_slot(sccsum_burst* b, sccsum_burst::Slot& s) {
    const hipStream_t st = s.stream;
    const uint64_t n = s.npk;
    SCCSUM_TRY(hipMemcpyAsync(s.d_bytes, s.h_bytes, (s.used + 15) & ~uint64_t(15), hipMemcpyHostToDevice, st));
    SCCSUM_TRY(hipMemcpyAsync(s.d_off, s.h_off, n * 8, hipMemcpyHostToDevice, st));
    SCCSUM_TRY(hipMemcpyAsync(s.d_len, s.h_len, n * 4, hipMemcpyHostToDevice, st));
    int rk;
    if (b->mode == SCCSUM_PIPE_IPV4) {
        rk = sccsum_ipv4_frames(s.d_bytes, s.used, s.d_off, s.d_len, s.d_out, s.d_status, n, s.max_len, st);
    } else {
        SCCSUM_TRY(hipMemcpyAsync(s.d_seed, s.h_seed, n * 4, hipMemcpyHostToDevice, st));
        rk = sccsum_spans(s.d_bytes, s.used, s.d_off, s.d_len, s.d_seed, s.d_out, s.d_status, n, s.max_len, st);
    }
    if (rk != SCCSUM_OK) return rk;
    SCCSUM_TRY(hipMemcpyAsync(s.h_out, s.d_out, n * width(b) * 2, hipMemcpyDeviceToHost, st));
    SCCSUM_TRY(hipMemcpyAsync(s.h_status, s.d_status, n, hipMemcpyDeviceToHost, st));
    SCCSUM_TRY(hipEventRecord(s.done, st));
    s.st = sccsum_burst::state::inflight;
    ++b->inflight;
    b->next_launch = (b->next_launch + 1) % b->slots.size();
    if (b->open != SIZE_MAX && &b->slots[b->open] == &s) b->open = SIZE_MAX;
    return SCCSUM_OK;
}

// Deliver finished slots in ring order; `wait` blocks on the oldest.
int deliver(sccsum_burst* b, bool wait, bool* did) {
    while (b->inflight) {
        auto& s = b->slots[b->next_deliver];
        if (s.st != sccsum_burst::state::inflight) break;
        if (wait) {
            SCCSUM_TRY(hipEventSynchronize(s.done));
        } else {
            const hipError_t q = hipEventQuery(s.done);
            if (q == hipErrorNotReady) break;
            SCCSUM_TRY(q);
        }
        b->fn(b->user, s.first_ticket, s.npk, s.h_out, s.h_status);
        s.st = sccsum_burst::state::free;
        s.used = 0;
        s.npk = 0;
        s.max_len = 0;
        --b->inflight;
        b->next_deliver = (b->next_deliver + 1) % b->slots.size();
        *did = true;
    }
    return SCCSUM_OK;
}

}  // namespace

extern "C" {

int sccsum_burst_create(int device, int mode, uint64_t batch_bytes, uint32_t batch_packets, uint64_t max_delay_ns,
                        int depth, sccsum_burst_done_fn fn, void* user, sccsum_burst** out) {
    if (!out || !fn || (mode != SCCSUM_PIPE_SPANS && mode != SCCSUM_PIPE_IPV4) || batch_bytes < 64 ||
        batch_packets < 1 || depth < 1 || depth > 64) {
        return SCCSUM_EINVAL;
    }
    *out = nullptr;
    const int rc0 = sccsum_init(device);
    if (rc0 != SCCSUM_OK) return rc0;
    auto* b = new (std::nothrow) sccsum_burst();
    if (!b) return SCCSUM_EINVAL;
    b->device = device;
    b->mode = mode;
    b->batch_bytes = (batch_bytes + 15) & ~uint64_t(15);
    b->batch_packets = batch_packets;
    b->max_delay_ns = max_delay_ns;
    b->fn = fn;
    b->user = user;
    b->slots.resize(depth);
    const uint64_t np = batch_packets, w = mode == SCCSUM_PIPE_IPV4 ? 2 : 1;
    int rc = SCCSUM_OK;
    for (auto& s : b->slots) {
        rc = hip_rc(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_bytes, b->batch_bytes, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_off, np * 8, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_len, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_seed, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_out, np * w * 2, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_status, np, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_bytes, b->batch_bytes));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_off, np * 8));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_len, np * 4));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_seed, np * 4));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_out, np * w * 2));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_status, np));
        if (rc == SCCSUM_OK) rc = hip_rc(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        if (rc != SCCSUM_OK) break;
    }
    if (rc != SCCSUM_OK) {
        sccsum_burst_destroy(b);
        return rc;
    }
    *out = b;
    return SCCSUM_OK;
}

int sccsum_burst_submit(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed,
                        uint64_t* ticket) {
    if (!b || (nfrag && !frags)) return SCCSUM_EINVAL;
    uint64_t L = 0;
    for (uint32_t j = 0; j < nfrag; ++j) {
        if ((!frags[j].base && frags[j].size) || frags[j].size > b->batch_bytes) return SCCSUM_EINVAL;
        L += frags[j].size;
    }
    if (L > b->batch_bytes || L > UINT32_MAX) return SCCSUM_EINVAL;  // never fits a batch
    SCCSUM_TRY(hipSetDevice(b->device));
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (b->open == SIZE_MAX) {
            auto& s = b->slots[b->next_launch];
            if (s.st != sccsum_burst::state::free) return SCCSUM_EBUSY;  // every slot in flight: poll, retry
            s.st = sccsum_burst::state::open;
            s.first_ticket = b->next_ticket;
            s.opened = std::chrono::steady_clock::now();
            b->open = b->next_launch;
        }
        auto& s = b->slots[b->open];
        const uint64_t at = (s.used + 15) & ~uint64_t(15);  // 16-byte aligned starts: full-rate loads
        if (s.npk == b->batch_packets || at + L > b->batch_bytes) {
            const int rc = launch_slot(b, s);  // full: send it, open the next slot
            if (rc != SCCSUM_OK) return rc;
            continue;
        }
        uint64_t pos = at;
        for (uint32_t j = 0; j < nfrag; ++j) {
            if (frags[j].size) std::memcpy(s.h_bytes + pos, frags[j].base, frags[j].size);
            pos += frags[j].size;
        }
        s.h_off[s.npk] = at;
        s.h_len[s.npk] = static_cast<uint32_t>(L);
        s.h_seed[s.npk] = seed;
        s.max_len = static_cast<uint32_t>(L) > s.max_len ? static_cast<uint32_t>(L) : s.max_len;
        s.used = pos;
        ++s.npk;
        if (ticket) *ticket = b->next_ticket;
        ++b->next_ticket;
        return SCCSUM_OK;
    }
    return SCCSUM_EBUSY;
}

int sccsum_burst_poll(sccsum_burst* b, int* did_work) {
    if (!b) return SCCSUM_EINVAL;
    SCCSUM_TRY(hipSetDevice(b->device));
    bool did = false;
    if (b->open != SIZE_MAX) {
        auto& s = b->slots[b->open];
        const auto age =
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - s.opened).count();
        const bool full = s.npk == b->batch_packets || s.used + 64 > b->batch_bytes;
        if (s.npk && (full || static_cast<uint64_t>(age) >= b->max_delay_ns)) {
            const int rc = launch_slot(b, s);
            if (rc != SCCSUM_OK) return rc;
            did = true;
        }
    }
    const int rc = deliver(b, false, &did);
    if (did_work) *did_work = did ? 1 : 0;
    return rc;
}

int sccsum_burst_drain(sccsum_burst* b) {
    if (!b) return SCCSUM_EINVAL;
    SCCSUM_TRY(hipSetDevice(b->device));
    if (b->open != SIZE_MAX) {
        auto& s = b->slots[b->open];
        if (s.npk) {
            const int rc = launch_slot(b, s);
            if (rc != SCCSUM_OK) return rc;
        } else {
            s.st = sccsum_burst::state::free;
            b->open = SIZE_MAX;
        }
    }
    bool did = false;
    return deliver(b, true, &did);
}

int sccsum_burst_destroy(sccsum_burst* b) {
    if (!b) return SCCSUM_OK;
    (void)hipSetDevice(b->device);
    for (auto& s : b->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    }
    for (auto& s : b->slots) free_slot(s);
    delete b;
    return SCCSUM_OK;
}

}  // extern "C"
