// pipeline.cc — host-memory batches through the GPU: the end-to-end path of
// BASELINE cfg 5 (DPDK-mbuf-shaped pinned host buffers, hipMemcpyAsync in and
// out, overlapped with the kernel on side streams).
//
// The native stack's packets start and end in host memory (DPDK mbufs,
// dpdk.cc:139-156: 128 B rte_mbuf + 128 B headroom + 2048 B data room per
// slot; virtio rx buffers).  A pipeline cuts a host batch into chunks; chunk
// c uses stage c % depth:
//   copy stream:    [gather into pinned staging (host memcpy) |] H2D bytes (as they lie, or one 2D
//                   DMA of each slot's packet bytes) + offsets/lengths/seeds
//   compute stream: wait(copied[c]) -> sccsum kernel -> D2H results -> record(done[c])
// so the H2D of chunk c+1 overlaps the kernel of chunk c and the D2H of c-1.
// Zero copy (gather 3): no copies at all — one fragment-list launch per chunk
// reads each packet where it lies in the pinned pool (over PCIe, packet bytes
// only) and the chunk's metadata from pinned staging, and writes the results
// into pinned staging (sccsum_*_desc).
// Results land in pinned staging and are copied to the caller's arrays when
// the stage is recycled or at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "sccsum.h"

struct sccsum_pipeline {
    struct Stage {
        uint8_t* d_bytes = nullptr;
        uint64_t* d_off = nullptr;
        uint32_t* d_len = nullptr;
        uint32_t* d_seed = nullptr;
        uint16_t* d_out = nullptr;
        uint8_t* d_status = nullptr;
        uint8_t* h_bytes = nullptr;  // pinned gather staging
        uint64_t* h_off = nullptr;   // pinned rebased offsets
        uint32_t* h_len = nullptr;
        uint32_t* h_seed = nullptr;
        uint16_t* h_out = nullptr;   // pinned results
        uint8_t* h_status = nullptr;
        sccsum_gather_desc* h_desc = nullptr;  // zero copy: one descriptor per packet
        uint32_t* h_first = nullptr;
        hipEvent_t copied = nullptr, done = nullptr;
        // pending result copy-out (caller arrays)
        uint16_t* dst_out = nullptr;
        uint8_t* dst_status = nullptr;
        uint64_t npk = 0;
        int width = 1;
        bool busy = false;
    };
    int device = 0;
    uint64_t chunk_bytes = 0;
    uint32_t chunk_packets = 0;
    hipStream_t copy = nullptr, compute = nullptr;
    std::vector<Stage> stages;
};

namespace {

int hip_rc(hipError_t e) { return e == hipSuccess ? SCCSUM_OK : static_cast<int>(e); }

#define SCCSUM_TRY(x)                  \
    do {                               \
        const int rc_ = hip_rc(x);     \
        if (rc_ != SCCSUM_OK) return rc_; \
    } while (0)

int finish_stage(sccsum_pipeline::Stage& s) {
    if (!s.busy) return SCCSUM_OK;
    SCCSUM_TRY(hipEventSynchronize(s.done));
    std::memcpy(s.dst_out, s.h_out, s.npk * s.width * sizeof(uint16_t));
    if (s.dst_status) std::memcpy(s.dst_status, s.h_status, s.npk);
    s.busy = false;
    return SCCSUM_OK;
}

void free_stage(sccsum_pipeline::Stage& s) {
    (void)hipFree(s.d_bytes);
    (void)hipFree(s.d_off);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_seed);
    (void)hipFree(s.d_out);
    (void)hipFree(s.d_status);
    (void)hipHostFree(s.h_bytes);
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_seed);
    (void)hipHostFree(s.h_out);
    (void)hipHostFree(s.h_status);
    (void)hipHostFree(s.h_desc);
    (void)hipHostFree(s.h_first);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.done) (void)hipEventDestroy(s.done);
}

}  // namespace

extern "C" {

int sccsum_pipeline_create(int device, uint64_t chunk_bytes, uint32_t chunk_packets, int depth,
                           sccsum_pipeline** out) {
    if (!out || depth < 1 || depth > 16 || chunk_bytes < 64 || chunk_packets < 1) return SCCSUM_EINVAL;
    *out = nullptr;
    const int rc0 = sccsum_init(device);
    if (rc0 != SCCSUM_OK) return rc0;
    auto* p = new (std::nothrow) sccsum_pipeline();
    if (!p) return SCCSUM_EINVAL;
    p->device = device;
    p->chunk_bytes = (chunk_bytes + 15) & ~uint64_t(15);
    p->chunk_packets = chunk_packets;
    int rc = hip_rc(hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking));
    if (rc == SCCSUM_OK) rc = hip_rc(hipStreamCreateWithFlags(&p->compute, hipStreamNonBlocking));
    p->stages.resize(depth);
    for (auto& s : p->stages) {
        if (rc != SCCSUM_OK) break;
        const uint64_t np = chunk_packets;
        rc = hip_rc(hipMalloc(&s.d_bytes, p->chunk_bytes));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_off, np * 8));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_len, np * 4));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_seed, np * 4));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_out, np * 4));
        if (rc == SCCSUM_OK) rc = hip_rc(hipMalloc(&s.d_status, np));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_bytes, p->chunk_bytes, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_off, np * 8, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_len, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_seed, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_out, np * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_status, np, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_desc, np * sizeof(sccsum_gather_desc), hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipHostMalloc(&s.h_first, (np + 1) * 4, hipHostMallocDefault));
        if (rc == SCCSUM_OK) rc = hip_rc(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
        if (rc == SCCSUM_OK) rc = hip_rc(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }
    if (rc != SCCSUM_OK) {
        sccsum_pipeline_destroy(p);
        return rc;
    }
    *out = p;
    return SCCSUM_OK;
}

int sccsum_pipeline_destroy(sccsum_pipeline* p) {
    if (!p) return SCCSUM_OK;
    (void)hipSetDevice(p->device);
    if (p->copy) (void)hipStreamSynchronize(p->copy);
    if (p->compute) (void)hipStreamSynchronize(p->compute);
    for (auto& s : p->stages) free_stage(s);
    if (p->copy) (void)hipStreamDestroy(p->copy);
    if (p->compute) (void)hipStreamDestroy(p->compute);
    delete p;
    return SCCSUM_OK;
}

}  // extern "C"

namespace {

// The device may read [p, p + len) in place: both ends lie in pinned or
// registered host memory (or device memory).  Pageable memory would fault the
// GPU, so a zero-copy run refuses it up front.
bool device_readable(const void* p, uint64_t len) {
    if (len == 0) return true;
    const auto* b = static_cast<const uint8_t*>(p);
    // one allocation must hold the whole range: two pinned blocks with pageable
    // memory between them pass an ends-only check, and the zero-copy kernel
    // would then read the pageable hole over PCIe
    void* start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                               reinterpret_cast<hipDeviceptr_t>(const_cast<uint8_t*>(b))) == hipSuccess &&
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                               reinterpret_cast<hipDeviceptr_t>(const_cast<uint8_t*>(b))) == hipSuccess &&
        start != nullptr && size != 0) {
        const auto* s0 = static_cast<const uint8_t*>(start);
        if (b < s0 || len > size || static_cast<uint64_t>(b - s0) > size - len) return false;
    } else {
        (void)hipGetLastError();  // the range query is not answered for this memory: the two-end check below
    }
    for (const uint8_t* q : {b, b + len - 1}) {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();  // clear the sticky "not registered" error
            return false;
        }
        if (a.type != hipMemoryTypeHost && a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged) {
            return false;
        }
    }
    return true;
}

int run_chunks(sccsum_pipeline* p, int mode, int gather, const void* host_bytes, uint64_t host_len,
               const uint64_t* host_off, const uint32_t* host_lens, const uint32_t* host_seed, uint64_t n,
               uint32_t max_len, uint16_t* host_out, uint8_t* host_status) {
    if (!p || (mode != SCCSUM_PIPE_SPANS && mode != SCCSUM_PIPE_IPV4) || !host_off || !host_lens || !host_out ||
        (n && !host_bytes) || gather < 0 || gather > SCCSUM_GATHER_ZERO_COPY) {
        return SCCSUM_EINVAL;
    }
    SCCSUM_TRY(hipSetDevice(p->device));
    const bool zc = gather == SCCSUM_GATHER_ZERO_COPY;
    if (zc && n && !device_readable(host_bytes, host_len)) return SCCSUM_EINVAL;
    const auto* src = static_cast<const uint8_t*>(host_bytes);
    const int width = mode == SCCSUM_PIPE_IPV4 ? 2 : 1;
    uint64_t i = 0;
    uint64_t chunk = 0;
    while (i < n) {
        auto& s = p->stages[chunk % p->stages.size()];
        const int rcf = finish_stage(s);  // recycle: its previous results go to the caller
        if (rcf != SCCSUM_OK) return rcf;
        // take packets while they fit the chunk (by count and by bytes)
        uint64_t j = i, lo = UINT64_MAX, hi = 0, packed = 0;
        // strided (gather == 2): packets at one pitch P (an mbuf pool's slots);
        // each row's first W bytes (the longest packet so far) cross PCIe as
        // one 2D DMA into rows of Wd = round16(W) bytes on the device
        bool rows = gather == SCCSUM_GATHER_STRIDED && n - i >= 2;
        const uint64_t P = rows ? host_off[i + 1] - host_off[i] : 0;
        rows = rows && host_off[i + 1] > host_off[i];
        uint64_t W = 0;
        for (; j < n && j - i < p->chunk_packets; ++j) {
            const uint64_t o = host_off[j], L = host_lens[j];
            if (o > host_len || L > host_len - o) return SCCSUM_EINVAL;  // outside the caller's buffer
            if (rows) {
                const bool on_pitch = j == i || o == host_off[j - 1] + P;
                const uint64_t nW = std::max(W, L);
                // every row is read W bytes wide: earlier rows stay inside their slot (W <= P),
                // the last row must stay inside the caller's buffer
                if (j > i && (!on_pitch || L > P || o + nW > host_len ||
                              (j - i + 1) * ((nW + 15) & ~uint64_t(15)) > p->chunk_bytes)) {
                    break;
                }
                if (j == i && L > P) rows = false;  // not slot-shaped after all: copy as it lies
                W = nW;
            }
            if (gather == 1 || zc) {
                // zero copy: descriptor positions are 32-bit
                const uint64_t cap = zc ? std::min<uint64_t>(p->chunk_bytes, UINT32_MAX) : p->chunk_bytes;
                if (j > i && packed + L > cap) break;
                packed += L;
            } else if (!rows) {
                const uint64_t nlo = std::min(lo, o), nhi = std::max(hi, o + L);
                if (j > i && nhi - nlo > p->chunk_bytes) break;
                lo = nlo;
                hi = nhi;
            }
        }
        const uint64_t npk = j - i;
        if (rows && npk < 2) rows = false;
        if (!rows && gather == SCCSUM_GATHER_STRIDED) {  // irregular chunk: recompute its covering range
            lo = UINT64_MAX;
            hi = 0;
            for (uint64_t k = i; k < j; ++k) {
                lo = std::min(lo, host_off[k]);
                hi = std::max(hi, host_off[k] + host_lens[k]);
            }
        }
        const uint64_t Wd = (W + 15) & ~uint64_t(15);
        if ((gather == 1 || zc) ? packed > p->chunk_bytes
                                : (rows ? npk * Wd > p->chunk_bytes : hi - lo > p->chunk_bytes)) {
            return SCCSUM_EINVAL;  // one oversized packet
        }
        if (zc) {
            // one descriptor per (non-empty) packet, read in place; the layout
            // offsets are the packets' positions packed back to back
            uint64_t pos = 0;
            uint32_t nd = 0;
            for (uint64_t k = 0; k < npk; ++k) {
                const uint32_t L = host_lens[i + k];
                s.h_first[k] = nd;
                s.h_off[k] = pos;
                if (L) s.h_desc[nd++] = {src + host_off[i + k], static_cast<uint32_t>(pos), L};
                pos += L;
            }
            s.h_first[npk] = nd;
            std::memcpy(s.h_len, host_lens + i, npk * 4);
            if (host_seed) std::memcpy(s.h_seed, host_seed + i, npk * 4);
            const int rk = mode == SCCSUM_PIPE_IPV4
                               ? sccsum_ipv4_frames_desc(s.h_desc, s.h_first, s.h_off, s.h_len, nullptr, s.h_out,
                                                         host_status ? s.h_status : nullptr, npk, max_len, p->compute)
                               : sccsum_spans_desc(s.h_desc, s.h_first, s.h_off, s.h_len,
                                                   host_seed ? s.h_seed : nullptr, nullptr, s.h_out,
                                                   host_status ? s.h_status : nullptr, npk, max_len, p->compute);
            if (rk != SCCSUM_OK) return rk;
            SCCSUM_TRY(hipEventRecord(s.done, p->compute));
            s.dst_out = host_out + i * width;
            s.dst_status = host_status ? host_status + i : nullptr;
            s.npk = npk;
            s.width = width;
            s.busy = true;
            i = j;
            ++chunk;
            continue;
        }
        uint64_t nbytes;
        if (gather == 1) {
            uint64_t pos = 0;
            for (uint64_t k = 0; k < npk; ++k) {
                std::memcpy(s.h_bytes + pos, src + host_off[i + k], host_lens[i + k]);
                s.h_off[k] = pos;
                pos += host_lens[i + k];
            }
            nbytes = pos;
        } else if (rows) {
            for (uint64_t k = 0; k < npk; ++k) s.h_off[k] = k * Wd;
            nbytes = npk * Wd;
        } else {
            for (uint64_t k = 0; k < npk; ++k) s.h_off[k] = host_off[i + k] - lo;
            nbytes = hi - lo;
        }
        std::memcpy(s.h_len, host_lens + i, npk * 4);
        if (host_seed) std::memcpy(s.h_seed, host_seed + i, npk * 4);
        if (rows) {
            SCCSUM_TRY(hipMemcpy2DAsync(s.d_bytes, Wd, src + host_off[i], P, W, npk, hipMemcpyHostToDevice, p->copy));
        } else {
            SCCSUM_TRY(hipMemcpyAsync(s.d_bytes, gather == 1 ? s.h_bytes : src + lo, nbytes, hipMemcpyHostToDevice,
                                      p->copy));
        }
        SCCSUM_TRY(hipMemcpyAsync(s.d_off, s.h_off, npk * 8, hipMemcpyHostToDevice, p->copy));
        SCCSUM_TRY(hipMemcpyAsync(s.d_len, s.h_len, npk * 4, hipMemcpyHostToDevice, p->copy));
        if (host_seed) SCCSUM_TRY(hipMemcpyAsync(s.d_seed, s.h_seed, npk * 4, hipMemcpyHostToDevice, p->copy));
        SCCSUM_TRY(hipEventRecord(s.copied, p->copy));
        SCCSUM_TRY(hipStreamWaitEvent(p->compute, s.copied, 0));
        const int rk = mode == SCCSUM_PIPE_IPV4
                           ? sccsum_ipv4_frames(s.d_bytes, nbytes, s.d_off, s.d_len, s.d_out,
                                                host_status ? s.d_status : nullptr, npk, max_len, p->compute)
                           : sccsum_spans(s.d_bytes, nbytes, s.d_off, s.d_len, host_seed ? s.d_seed : nullptr,
                                          s.d_out, host_status ? s.d_status : nullptr, npk, max_len, p->compute);
        if (rk != SCCSUM_OK) return rk;
        SCCSUM_TRY(hipMemcpyAsync(s.h_out, s.d_out, npk * width * 2, hipMemcpyDeviceToHost, p->compute));
        if (host_status) SCCSUM_TRY(hipMemcpyAsync(s.h_status, s.d_status, npk, hipMemcpyDeviceToHost, p->compute));
        SCCSUM_TRY(hipEventRecord(s.done, p->compute));
        s.dst_out = host_out + i * width;
        s.dst_status = host_status ? host_status + i : nullptr;
        s.npk = npk;
        s.width = width;
        s.busy = true;
        i = j;
        ++chunk;
    }
    for (auto& s : p->stages) {
        const int rc = finish_stage(s);
        if (rc != SCCSUM_OK) return rc;
    }
    return SCCSUM_OK;
}

}  // namespace

extern "C" {

int sccsum_pipeline_run(sccsum_pipeline* p, int mode, int gather, const void* host_bytes, uint64_t host_len,
                        const uint64_t* host_off, const uint32_t* host_lens, const uint32_t* host_seed, uint64_t n,
                        uint32_t max_len, uint16_t* host_out, uint8_t* host_status) {
    const int rc = run_chunks(p, mode, gather, host_bytes, host_len, host_off, host_lens, host_seed, n, max_len,
                              host_out, host_status);
    if (rc != SCCSUM_OK && p) {
        // leave no stage pointing at the caller's arrays after a failed run
        (void)hipStreamSynchronize(p->copy);
        (void)hipStreamSynchronize(p->compute);
        for (auto& s : p->stages) s.busy = false;
    }
    return rc;
}

int sccsum_host_alloc(void** p, uint64_t bytes) { return p ? hip_rc(hipHostMalloc(p, bytes, hipHostMallocDefault)) : SCCSUM_EINVAL; }

int sccsum_host_free(void* p) { return hip_rc(hipHostFree(p)); }

}  // extern "C"
