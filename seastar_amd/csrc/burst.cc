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
//   submit_mapped: zero-copy — the fragments lie in memory the device reads
//            (pinned / registered host memory, e.g. a DPDK mempool): only a
//            {src, dst, len} descriptor is recorded; at launch the
//            fragment-list kernel (sccsum_*_desc) reads the bytes over PCIe
//            straight into the sum, so no host thread touches packet bytes and
//            they cross PCIe once with no gathered copy in HBM (a copied
//            packet of the same batch is one descriptor into the staged
//            bytes)
//   poll:    launch the open slot when full (bytes / packets) or older than
//            max_delay_ns — on the slot's own stream: ONE H2D of the staged
//            bytes with the metadata packed behind them, the kernel, ONE D2H
//            of results + status, an event (4 stream operations: launch cost
//            is per batch, not per array), so one batch's copies overlap the
//            previous batch's kernel; then deliver
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
#include "sccsum_diag.h"

struct sccsum_burst {
    enum class state { free, open, inflight, delivering };
    struct Slot {
        state st = state::free;
        hipStream_t stream = nullptr;
        // pinned staging: packets back to back, then (at launch) the metadata
        // arrays packed right behind them, so one H2D carries the whole batch
        uint8_t* h_stage = nullptr;
        uint64_t* h_off = nullptr;  // metadata as submitted
        uint32_t* h_len = nullptr;
        uint32_t* h_seed = nullptr;
        uint32_t* h_first = nullptr;           // packet p's descriptors: h_desc[h_first[p] .. h_first[p+1])
        sccsum_gather_desc* h_desc = nullptr;  // every packet's fragments (src NULL: staged by copy)
        uint8_t* h_res = nullptr;  // results then status, one D2H
        uint8_t* d_stage = nullptr;
        uint8_t* d_res = nullptr;
        hipEvent_t done = nullptr;
        uint64_t used = 0;  // staged bytes
        uint32_t npk = 0;
        uint32_t ndesc = 0;   // descriptors recorded
        bool copied = false;  // some packet was memcpy'd into h_stage
        bool mapped = false;  // some packet is zero-copy (the batch runs the fragment-list kernel)
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
    bool in_callback = false;  // a completion callback is running (poll / drain / destroy refuse)
};

namespace {

int hip_rc(hipError_t e) { return e == hipSuccess ? SCCSUM_OK : static_cast<int>(e); }

#define SCCSUM_TRY(x)                     \
    do {                                  \
        const int rc_ = hip_rc(x);        \
        if (rc_ != SCCSUM_OK) return rc_; \
    } while (0)

void free_slot(sccsum_burst::Slot& s) {
    (void)hipHostFree(s.h_stage);
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_seed);
    (void)hipHostFree(s.h_first);
    (void)hipHostFree(s.h_desc);
    (void)hipHostFree(s.h_res);
    (void)hipFree(s.d_stage);
    (void)hipFree(s.d_res);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
}

int width(const sccsum_burst* b) { return b->mode == SCCSUM_PIPE_IPV4 ? 2 : 1; }

// fragment descriptors per slot (a packet of more fragments launches its slot early)
uint64_t desc_cap(const sccsum_burst* b) { return 4ull * b->batch_packets; }

// staging bytes per slot: the data room plus room for the packed metadata
// (offsets, lengths, seeds, descriptor starts) and descriptors
uint64_t stage_bytes(const sccsum_burst* b) {
    return b->batch_bytes + 20ull * b->batch_packets + sizeof(sccsum_gather_desc) * desc_cap(b) + 48;
}

// Diagnostic (sccsum_diag.h), how a batch holding zero-copy packets runs:
// 2 = the fragment-list kernel reads the metadata and descriptors where the
// host wrote them and writes the results straight into the pinned result
// block (one launch, no copies); 1 = metadata H2D, fragment-list kernel,
// results D2H; 0 = metadata H2D, gather into the batch, sum, results D2H.
thread_local int t_fused = 2;

// A batch of copied packets: one H2D (packets + metadata packed behind them),
// the kernel, one D2H (results + status), an event — 4 stream operations.  A
// batch holding zero-copy packets: the fragment-list launch and an event (see
// one_launch), or, in the A/B forms, the same 4 operations.  On failure
// the slot is left exactly as before the call (still open, its packets
// staged) once whatever part of the batch reached the stream has finished,
// so a later poll / drain retries the launch.
int launch_slot_ops(sccsum_burst* b, sccsum_burst::Slot& s);

// A zero-copy one-launch batch (t_fused 2) is a single kernel with no copies
// to overlap, so every such batch goes to ONE stream: the kernels run in
// submit order, the oldest batch — the one delivery waits for — finishes
// first, and the host refills its slot while the GPU runs the next ones
// (on separate streams they share PCIe and finish together, leaving the GPU
// idle while the host refills).  Batches with copies keep their slot's stream
// so one batch's copies overlap another's kernel.
bool one_launch(const sccsum_burst::Slot& s) { return s.mapped && t_fused == 2; }

hipStream_t stream_of(const sccsum_burst* b, const sccsum_burst::Slot& s) {
    return one_launch(s) ? b->slots[0].stream : s.stream;
}

int launch_slot(sccsum_burst* b, sccsum_burst::Slot& s) {
    const hipStream_t st = stream_of(b, s);
    const int rc = launch_slot_ops(b, s);
    if (rc != SCCSUM_OK) (void)hipStreamSynchronize(st);
    return rc;
}

int launch_slot_ops(sccsum_burst* b, sccsum_burst::Slot& s) {
    SCCSUM_TRY(hipSetDevice(b->device));
    const hipStream_t st = stream_of(b, s);
    const uint64_t n = s.npk;
    const bool spans = b->mode != SCCSUM_PIPE_IPV4;
    if (one_launch(s)) {
        // zero-copy batch: the kernel reads the pinned metadata, descriptors
        // and (for copied packets) staged bytes over PCIe and writes the
        // results into the pinned result block the callback reads
        s.h_first[n] = s.ndesc;
        auto* h_out = reinterpret_cast<uint16_t*>(s.h_res);
        uint8_t* h_status = s.h_res + 2 * width(b) * n;
        const int rk = spans ? sccsum_spans_desc(s.h_desc, s.h_first, s.h_off, s.h_len, s.h_seed, s.h_stage, h_out,
                                                 h_status, n, s.max_len, st)
                             : sccsum_ipv4_frames_desc(s.h_desc, s.h_first, s.h_off, s.h_len, s.h_stage, h_out,
                                                       h_status, n, s.max_len, st);
        if (rk != SCCSUM_OK) return rk;
        SCCSUM_TRY(hipEventRecord(s.done, st));
        s.st = sccsum_burst::state::inflight;
        ++b->inflight;
        b->next_launch = (b->next_launch + 1) % b->slots.size();
        if (b->open != SIZE_MAX && &b->slots[b->open] == &s) b->open = SIZE_MAX;
        return SCCSUM_OK;
    }
    const uint64_t a_off = (s.used + 15) & ~uint64_t(15), a_len = a_off + 8 * n, a_seed = a_len + 4 * n;
    const uint64_t a_first = spans ? a_seed + 4 * n : a_seed;
    const bool fused = s.mapped && t_fused;
    const uint64_t a_desc = ((fused ? a_first + 4 * (n + 1) : a_first) + 7) & ~uint64_t(7);
    const uint64_t total = a_desc + (s.mapped ? sizeof(sccsum_gather_desc) * s.ndesc : 0);
    std::memcpy(s.h_stage + a_off, s.h_off, 8 * n);
    std::memcpy(s.h_stage + a_len, s.h_len, 4 * n);
    if (spans) std::memcpy(s.h_stage + a_seed, s.h_seed, 4 * n);
    if (fused) {
        s.h_first[n] = s.ndesc;
        std::memcpy(s.h_stage + a_first, s.h_first, 4 * (n + 1));
    }
    if (s.mapped) std::memcpy(s.h_stage + a_desc, s.h_desc, sizeof(sccsum_gather_desc) * s.ndesc);
    // only mapped packets: their bytes come over PCIe as the kernel reads them,
    // the H2D carries the metadata alone
    const uint64_t from = s.copied ? 0 : a_off;
    SCCSUM_TRY(hipMemcpyAsync(s.d_stage + from, s.h_stage + from, total - from, hipMemcpyHostToDevice, st));
    const auto* d_off = reinterpret_cast<const uint64_t*>(s.d_stage + a_off);
    const auto* d_len = reinterpret_cast<const uint32_t*>(s.d_stage + a_len);
    const auto* d_seed = reinterpret_cast<const uint32_t*>(s.d_stage + a_seed);
    const auto* d_desc = reinterpret_cast<const sccsum_gather_desc*>(s.d_stage + a_desc);
    auto* d_out = reinterpret_cast<uint16_t*>(s.d_res);
    uint8_t* d_status = s.d_res + 2 * width(b) * n;
    int rk = SCCSUM_OK;
    if (fused) {
        const auto* d_first = reinterpret_cast<const uint32_t*>(s.d_stage + a_first);
        rk = spans ? sccsum_spans_desc(d_desc, d_first, d_off, d_len, d_seed, s.d_stage, d_out, d_status, n,
                                       s.max_len, st)
                   : sccsum_ipv4_frames_desc(d_desc, d_first, d_off, d_len, s.d_stage, d_out, d_status, n, s.max_len,
                                             st);
    } else {
        if (s.mapped) {  // gather the zero-copy fragments into the batch, then sum it (diagnostic form)
            const int rg = sccsum_gather(d_desc, s.ndesc, s.d_stage, st);
            if (rg != SCCSUM_OK) return rg;
        }
        rk = spans ? sccsum_spans(s.d_stage, s.used, d_off, d_len, d_seed, d_out, d_status, n, s.max_len, st)
                   : sccsum_ipv4_frames(s.d_stage, s.used, d_off, d_len, d_out, d_status, n, s.max_len, st);
    }
    if (rk != SCCSUM_OK) return rk;
    SCCSUM_TRY(hipMemcpyAsync(s.h_res, s.d_res, (2 * width(b) + 1) * n, hipMemcpyDeviceToHost, st));
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
        // bookkeeping first, so the queue is consistent whatever the callback
        // does; the slot stays out of use (its results are what the callback
        // reads) until the callback returns
        const uint64_t first = s.first_ticket;
        const uint32_t npk = s.npk;
        s.st = sccsum_burst::state::delivering;
        --b->inflight;
        b->next_deliver = (b->next_deliver + 1) % b->slots.size();
        b->in_callback = true;
        b->fn(b->user, first, npk, reinterpret_cast<const uint16_t*>(s.h_res), s.h_res + 2 * width(b) * npk);
        b->in_callback = false;
        s.used = 0;
        s.npk = 0;
        s.ndesc = 0;
        s.copied = false;
        s.mapped = false;
        s.max_len = 0;
        s.st = sccsum_burst::state::free;
        *did = true;
    }
    return SCCSUM_OK;
}

}  // namespace

extern "C" {

int sccsum_burst_create(int device, int mode, uint64_t batch_bytes, uint32_t batch_packets, uint64_t max_delay_ns,
                        int depth, sccsum_burst_done_fn fn, void* user, sccsum_burst** out) {
    // batch offsets travel as 32-bit gather destinations (sccsum_gather_desc)
    if (!out || !fn || (mode != SCCSUM_PIPE_SPANS && mode != SCCSUM_PIPE_IPV4) || batch_bytes < 64 ||
        batch_bytes > (UINT32_MAX & ~uint64_t(15)) || batch_packets < 1 || depth < 1 || depth > 64) {
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
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_stage, stage_bytes(b), hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_off, np * 8, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_len, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_seed, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_first, (np + 1) * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) {
            rc = hip_rc(hipHostMalloc(&s.h_desc, desc_cap(b) * sizeof(sccsum_gather_desc), hipHostMallocDefault));
        }
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_res, np * (2 * w + 1), hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_stage, stage_bytes(b)));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_res, np * (2 * w + 1)));
        if (rc == SCCSUM_OK) rc = hip_rc(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        // first use of a stream creates its hardware queue (milliseconds):
        // pay that here, not on the first batches
        if (rc == SCCSUM_OK) rc = hip_rc(hipMemsetAsync(s.d_res, 0, 1, s.stream));
        if (rc == SCCSUM_OK) rc = hip_rc(hipStreamSynchronize(s.stream));
        if (rc != SCCSUM_OK) break;
    }
    if (rc != SCCSUM_OK) {
        sccsum_burst_destroy(b);
        return rc;
    }
    *out = b;
    return SCCSUM_OK;
}

// Both submits: validate, find room in the open slot (launching it when the
// packet does not fit), then place the packet by copy or by descriptor.
static int submit(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed, uint64_t* ticket,
                  bool mapped) {
    if (!b || (nfrag && !frags)) return SCCSUM_EINVAL;
    uint64_t L = 0;
    uint32_t nd = 0;
    for (uint32_t j = 0; j < nfrag; ++j) {
        if ((!frags[j].base && frags[j].size) || frags[j].size > b->batch_bytes) return SCCSUM_EINVAL;
        L += frags[j].size;
        nd += frags[j].size != 0;
    }
    if (L > b->batch_bytes || L > UINT32_MAX) return SCCSUM_EINVAL;  // never fits a batch
    if (!mapped) nd = L != 0;  // a copied packet: one descriptor into the staged bytes
    if (nd > desc_cap(b)) return SCCSUM_EINVAL;
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
        if (s.npk == b->batch_packets || at + L > b->batch_bytes || s.ndesc + nd > desc_cap(b)) {
            const int rc = launch_slot(b, s);  // full: send it, open the next slot
            if (rc != SCCSUM_OK) return rc;
            continue;
        }
        s.h_first[s.npk] = s.ndesc;
        uint64_t pos = at;
        for (uint32_t j = 0; j < nfrag; ++j) {
            if (frags[j].size) {
                if (mapped) {
                    s.h_desc[s.ndesc++] = {frags[j].base, static_cast<uint32_t>(pos),
                                           static_cast<uint32_t>(frags[j].size)};
                } else {
                    std::memcpy(s.h_stage + pos, frags[j].base, frags[j].size);
                }
            }
            pos += frags[j].size;
        }
        if (!mapped && L) s.h_desc[s.ndesc++] = {nullptr, static_cast<uint32_t>(at), static_cast<uint32_t>(L)};
        s.copied |= !mapped && L;
        s.mapped |= mapped && L;
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

int sccsum_burst_submit(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed,
                        uint64_t* ticket) {
    return submit(b, frags, nfrag, seed, ticket, false);
}

int sccsum_burst_submit_mapped(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed,
                               uint64_t* ticket) {
    return submit(b, frags, nfrag, seed, ticket, true);
}

int sccsum_burst_poll(sccsum_burst* b, int* did_work) {
    if (!b || b->in_callback) return SCCSUM_EINVAL;
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
    if (!b || b->in_callback) return SCCSUM_EINVAL;
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

int sccsum_set_burst_fused(int on) {
    if (on < 0 || on > 2) return SCCSUM_EINVAL;
    t_fused = on;
    return SCCSUM_OK;
}

int sccsum_burst_destroy(sccsum_burst* b) {
    if (!b) return SCCSUM_OK;
    if (b->in_callback) return SCCSUM_EINVAL;
    (void)hipSetDevice(b->device);
    for (auto& s : b->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    }
    for (auto& s : b->slots) free_slot(s);
    delete b;
    return SCCSUM_OK;
}

}  // extern "C"
