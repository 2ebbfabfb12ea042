// seastar/net/ip_checksum_batch.hh — C++ batch interface to the MI355X
// checksum engine (libsccsum, C-ABI in <sccsum.h>), in Seastar's vocabulary.
//
// The per-packet API (<seastar/net/ip_checksum.hh>) stays synchronous and on
// the reactor thread.  This header is what a shard uses to hand a burst of
// packets to its GPU: one launch checksums every packet of the burst.
//
//   per-packet reference call                          batch equivalent
//   ------------------------------------------------   --------------------------------
//   ip_checksum(data, len)           ip_checksum.cc:70-74     sum_spans(batch, nullptr, ...)
//   checksummer + *_pseudo_header_checksum + sum + get        sum_spans(batch, seeds, ...)
//       udp.cc:184-195, tcp.hh:1656-1694, tcp.hh:1004-1016
//   ip.cc:121-127 (IPv4 verify) + tcp.hh:876-883 (TCP verify) ipv4_frames(batch, ...)
//   ip.cc:271-277 (IPv4 generate) + udp/tcp generate          ipv4_frames(batch, ...) on zeroed fields
//   the same, stored into the frames (wire-ready tx)          ipv4_fill(batch, SCCSUM_FILL_IP | SCCSUM_FILL_L4, ...)
//   checksummer::sum(const packet&)  ip_checksum.cc:64-68     spans_desc / ipv4_frames_desc (fragments
//                                                             anywhere the device reads); C-ABI sccsum_fragments
//   toeplitz_hash(rss_key(), forward_hash)  net.cc:330-341    ipv4_rss(batch, key, ...) / ipv4_frames_rss(...)
//   per packet as qp::poll_tx / DPDK rx hand them over         burst_queue (host packets, async completion)
//       net.cc:81-105, dpdk.cc:2190-2204
//   a shard's steady stream of bursts, polled like its queues  resident_engine (one grid, steps streamed in;
//       reactor.cc:3543-3550                                   fills too: submit_fill)
//
// Results are network-order uint16 values, exactly what checksummer::get()
// returns; a verify passes when the value is 0.  Errors throw
// std::runtime_error (the C-ABI underneath never throws).
#pragma once

#include <sccsum.h>

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>

#if __cplusplus >= 202002L
#include <span>
#endif

namespace seastar {

namespace net {

// Packets resident in device memory: one byte buffer plus offset/length
// arrays (see <sccsum.h> "Memory contract").
struct device_packet_batch {
    const void* bytes = nullptr;   // 16-byte aligned device pointer
    uint64_t bytes_len = 0;        // valid bytes at `bytes`
    const uint64_t* off = nullptr; // device, n entries
    const uint32_t* len = nullptr; // device, n entries
    uint64_t n = 0;
    uint32_t max_len = 0;          // upper bound of len[] (0 = unknown); tunes the launch only
};

enum class checksum_status : uint8_t {
    ok = SCCSUM_ST_OK,               // spans: result 0; frames: IPv4 header verifies
    l4_ok = SCCSUM_ST_L4_OK,         // frames: TCP/UDP checksum verifies
    malformed = SCCSUM_ST_MALFORMED, // frames: shorter than 20 B / than the IP length, bad ihl
    out_of_range = SCCSUM_ST_RANGE,  // span outside the byte buffer (not read)
    ip_fragment = SCCSUM_ST_IPFRAG,  // frames: MF or offset set — L4 is checked after reassembly (ip.cc:164-220)
};

class batch_checksummer {
    int _device;

    static void check(int rc, const char* what) {
        if (rc != SCCSUM_OK) {
            throw std::runtime_error(std::string(what) + ": " + sccsum_strerror(rc));
        }
    }

public:
    // Binds the calling thread (the shard's reactor thread) to `device`.
    explicit batch_checksummer(int device) : _device(device) { check(sccsum_init(device), "sccsum_init"); }

    int device() const noexcept { return _device; }

    // The pseudo-header partial sum ipv4_traits::{tcp,udp}_pseudo_header_checksum
    // leaves in a fresh checksummer (ip.hh:70-75); host-order addresses, len
    // truncated to 16 bits exactly like the reference's uint16_t parameter.
    static uint32_t pseudo_header_seed(uint32_t src_host, uint32_t dst_host, uint8_t proto, uint16_t len) noexcept {
        return sccsum_pseudo_seed(src_host, dst_host, proto, len);
    }

    // out[i] = checksum of span i, seeded with seeds[i] when seeds != nullptr.
    void sum_spans(const device_packet_batch& b, const uint32_t* d_seeds, uint16_t* d_out, uint8_t* d_status,
                   void* stream) const {
        check(sccsum_spans(b.bytes, b.bytes_len, b.off, b.len, d_seeds, d_out, d_status, b.n, b.max_len, stream),
              "sccsum_spans");
    }

    // out2[2i] = IPv4 header checksum, out2[2i+1] = TCP/UDP checksum of frame i.
    // d_out2 may be null when d_status is given: verify only, 1 status byte
    // written per frame (what the reference keeps of the sum, ip.cc:121-127).
    void ipv4_frames(const device_packet_batch& b, uint16_t* d_out2, uint8_t* d_status, void* stream) const {
        check(sccsum_ipv4_frames(b.bytes, b.bytes_len, b.off, b.len, d_out2, d_status, b.n, b.max_len, stream),
              "sccsum_ipv4_frames");
    }

    // Generate IPv4 header and/or TCP/UDP checksums (ICMP echo replies with
    // SCCSUM_FILL_ICMP_ECHO) and store them into the frames (mode:
    // SCCSUM_FILL_*; d_status and d_out2 may be null: without d_out2 the
    // two passes of SCCSUM_FILL_L4 / SCCSUM_FILL_ICMP_ECHO hand the values over
    // in stream-ordered scratch).  IP fragments get their IPv4 header checksum only.
    void ipv4_fill(const device_packet_batch& b, uint32_t mode, uint16_t* d_out2, uint8_t* d_status,
                   void* stream) const {
        check(sccsum_ipv4_fill(const_cast<void*>(b.bytes), b.bytes_len, b.off, b.len, d_out2, d_status, b.n,
                               b.max_len, mode, stream),
              "sccsum_ipv4_fill");
    }

    // RSS: d_hash[i] = toeplitz_hash(key, forward_hash of frame i) (toeplitz.hh:78-98, net.cc:330-341);
    // mode SCCSUM_RSS_DISPATCH or SCCSUM_RSS_REASSEMBLED.  key is host memory
    // (the reference's rss_key_type: 40 or 52 bytes, at least 4).
    void ipv4_rss(const device_packet_batch& b, const uint8_t* key, size_t key_len, int mode, uint32_t* d_hash,
                  uint8_t* d_status, void* stream) const {
        check(sccsum_ipv4_rss(b.bytes, b.bytes_len, b.off, b.len, key, static_cast<uint32_t>(key_len), mode, d_hash,
                              d_status, b.n, stream),
              "sccsum_ipv4_rss");
    }

    // ipv4_frames and ipv4_rss in one pass over the bytes.
    void ipv4_frames_rss(const device_packet_batch& b, const uint8_t* key, size_t key_len, int mode,
                         uint16_t* d_out2, uint8_t* d_status, uint32_t* d_hash, void* stream) const {
        check(sccsum_ipv4_frames_rss(b.bytes, b.bytes_len, b.off, b.len, d_out2, d_status, b.n, b.max_len, key,
                                     static_cast<uint32_t>(key_len), mode, d_hash, stream),
              "sccsum_ipv4_frames_rss");
    }

#if __cplusplus >= 202002L
    // The same with the reference's key type (rss_key_type = std::span<const uint8_t>, toeplitz.hh:49).
    void ipv4_rss(const device_packet_batch& b, std::span<const uint8_t> key, int mode, uint32_t* d_hash,
                  uint8_t* d_status, void* stream) const {
        ipv4_rss(b, key.data(), key.size(), mode, d_hash, d_status, stream);
    }
#endif

    // Packets as fragment lists summed where the fragments lie (HBM, pinned /
    // registered host memory over PCIe, or d_stage for src == nullptr):
    // checksummer::sum(const packet&) (ip_checksum.cc:64-68) without a gather.
    // Packet i is d_desc[d_first[i] .. d_first[i+1]), tiling its bytes from
    // dst_off = d_off[i]; d_len / max_len as in device_packet_batch.
    void spans_desc(const sccsum_gather_desc* d_desc, const uint32_t* d_first, const uint64_t* d_off,
                    const uint32_t* d_len, uint64_t n, uint32_t max_len, const void* d_stage, const uint32_t* d_seeds,
                    uint16_t* d_out, uint8_t* d_status, void* stream) const {
        check(sccsum_spans_desc(d_desc, d_first, d_off, d_len, d_seeds, d_stage, d_out, d_status, n, max_len, stream),
              "sccsum_spans_desc");
    }

    void ipv4_frames_desc(const sccsum_gather_desc* d_desc, const uint32_t* d_first, const uint64_t* d_off,
                          const uint32_t* d_len, uint64_t n, uint32_t max_len, const void* d_stage, uint16_t* d_out2,
                          uint8_t* d_status, void* stream) const {
        check(sccsum_ipv4_frames_desc(d_desc, d_first, d_off, d_len, d_stage, d_out2, d_status, n, max_len, stream),
              "sccsum_ipv4_frames_desc");
    }

    void sync(void* stream) const { check(sccsum_sync(stream), "sccsum_sync"); }
};

// Burst queue (<sccsum.h> sccsum_burst_*): packets from HOST memory, handed
// over one at a time as qp::poll_tx and the DPDK rx loop do, batched for the
// GPU and completed through `done(first_ticket, count, results, status)` on
// the polling thread, in submit order.  poll() has pollfn::poll's contract
// (core/internal/poll.hh:26-29: true = did work), so it registers as a poller
// the way qp registers poll_tx (net.cc:109):
//   burst_queue q(gpu, SCCSUM_PIPE_IPV4, 16 << 20, 8192, 50'000, 4, on_done);
//   auto p = reactor::poller::simple([&] { return q.poll(); });
//   q.submit(reinterpret_cast<const sccsum_fragment*>(pkt.fragment_array()), pkt.nr_frags());
// The queue hands `this` to the C-ABI, so it neither copies nor moves.
template <typename Done>
class burst_queue {
    sccsum_burst* _q = nullptr;
    Done _done;

    static void complete(void* self, uint64_t first, uint32_t count, const uint16_t* results, const uint8_t* status) {
        static_cast<burst_queue*>(self)->_done(first, count, results, status);
    }
    static void check(int rc, const char* what) {
        if (rc != SCCSUM_OK) {
            throw std::runtime_error(std::string(what) + ": " + sccsum_strerror(rc));
        }
    }

public:
    burst_queue(int device, int mode, uint64_t batch_bytes, uint32_t batch_packets, uint64_t max_delay_ns, int depth,
                Done done)
        : _done(std::move(done)) {
        check(sccsum_burst_create(device, mode, batch_bytes, batch_packets, max_delay_ns, depth, &complete, this, &_q),
              "sccsum_burst_create");
    }
    burst_queue(const burst_queue&) = delete;
    burst_queue& operator=(const burst_queue&) = delete;
    ~burst_queue() { sccsum_burst_destroy(_q); }

    // false: every batch slot is in flight (poll, then submit again)
    bool submit(const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed = 0, uint64_t* ticket = nullptr) {
        const int rc = sccsum_burst_submit(_q, frags, nfrag, seed, ticket);
        if (rc == SCCSUM_EBUSY) return false;
        check(rc, "sccsum_burst_submit");
        return true;
    }
    // zero-copy: fragments in device-readable pinned / registered host memory,
    // untouched until their completion (sccsum_burst_submit_mapped)
    bool submit_mapped(const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed = 0, uint64_t* ticket = nullptr) {
        const int rc = sccsum_burst_submit_mapped(_q, frags, nfrag, seed, ticket);
        if (rc == SCCSUM_EBUSY) return false;
        check(rc, "sccsum_burst_submit_mapped");
        return true;
    }
    bool poll() {
        int did = 0;
        check(sccsum_burst_poll(_q, &did), "sccsum_burst_poll");
        return did != 0;
    }
    void drain() { check(sccsum_burst_drain(_q), "sccsum_burst_drain"); }
};

// Resident engine (<sccsum.h> sccsum_engine_*): one grid kept on the GPU
// while the shards stream steps into it, as the reactor keeps polling its
// queues (reactor.cc:3543-3550); each step is up to 4 batches, computed
// exactly as the one-launch calls compute them.  A run takes any number of
// steps (their descriptors cycle through a ring of ring_slots slots), and
// any number of threads may submit into it and wait — the shards that share
// the GPU; start / stop / the destructor are the owner's.  Frames engines may
// take in-place fills (fill = true).  One engine runs per device at a time:
// try_start() is false while another engine of the process runs there.
//   resident_engine eng(gpu, SCCSUM_PIPE_IPV4, /*ring_slots=*/1024, /*in flight=*/8, /*fill=*/true);
//   eng.start(stream);
//   sccsum_batch tx = {...}, rx = {...};
//   uint64_t a = eng.submit_fill(&tx, 1, SCCSUM_FILL_IP | SCCSUM_FILL_L4);   // from any shard
//   uint64_t b = eng.submit(&rx, 1);
//   eng.wait(b); eng.wait(a); eng.stop();
class resident_engine {
    sccsum_engine* _e = nullptr;

    static void check(int rc, const char* what) {
        if (rc != SCCSUM_OK) {
            throw std::runtime_error(std::string(what) + ": " + sccsum_strerror(rc));
        }
    }

public:
    resident_engine(int device, int mode, uint32_t ring_slots, uint32_t max_in_flight, bool fill = false) {
        check(sccsum_engine_create(device, mode | (fill ? SCCSUM_ENGINE_FILL : 0), ring_slots, max_in_flight, &_e),
              "sccsum_engine_create");
    }
    // every limit (ring, in flight, idle and dependency limits; 0 fields = defaults)
    resident_engine(int device, int mode, const sccsum_engine_opts& opts, bool fill = false) {
        check(sccsum_engine_create_opts(device, mode | (fill ? SCCSUM_ENGINE_FILL : 0), &opts, &_e),
              "sccsum_engine_create_opts");
    }
    resident_engine(const resident_engine&) = delete;
    resident_engine& operator=(const resident_engine&) = delete;
    ~resident_engine() { sccsum_engine_destroy(_e); }
    // destroy now, reporting a run that left a published step undone (the destructor cannot)
    void close() {
        sccsum_engine* e = _e;
        _e = nullptr;
        check(sccsum_engine_destroy(e), "sccsum_engine_destroy");
    }

    // launch the grid on `stream` (the calling thread's current device, the engine's)
    void start(void* stream) { check(sccsum_engine_start(_e, stream), "sccsum_engine_start"); }
    // false: another engine of this process runs on the device (SCCSUM_EBUSY)
    bool try_start(void* stream) {
        const int rc = sccsum_engine_start(_e, stream);
        if (rc == SCCSUM_EBUSY) return false;
        check(rc, "sccsum_engine_start");
        return true;
    }
    // max_len: the longest packet, if known (sizes the step's tiles; 0 = from bytes_len / n)
    uint64_t submit(const sccsum_batch* batches, uint32_t nbatch, uint64_t timeout_ns = 1'000'000'000,
                    uint32_t max_len = 0) {
        uint64_t step = 0;
        check(sccsum_engine_submit(_e, batches, nbatch, max_len, timeout_ns, &step), "sccsum_engine_submit");
        return step;
    }
    // in-place fill of every batch (d_out: the values, required); the step returned is done once
    // the frames hold their checksums
    uint64_t submit_fill(const sccsum_batch* batches, uint32_t nbatch, uint32_t mode,
                         uint64_t timeout_ns = 1'000'000'000, uint32_t max_len = 0) {
        uint64_t step = 0;
        check(sccsum_engine_submit_fill(_e, batches, nbatch, max_len, mode, timeout_ns, &step),
              "sccsum_engine_submit_fill");
        return step;
    }
    void wait(uint64_t step, uint64_t timeout_ns = 1'000'000'000) {
        check(sccsum_engine_wait(_e, step, timeout_ns), "sccsum_engine_wait");
    }
    void stop() { check(sccsum_engine_stop(_e), "sccsum_engine_stop"); }
};

}  // namespace net

}  // namespace seastar
