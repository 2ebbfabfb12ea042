/*
 * sccsum.h — C-ABI boundary of the MI355X (gfx950) batch Internet-checksum
 * engine.  Plain pointers and sizes only; every entry point returns 0 on
 * success, a positive hipError_t value for a HIP runtime failure, or a
 * negative SCCSUM_E* code; nothing throws.
 *
 * What each entry replaces in scylladb/seastar (paths relative to the
 * reference tree):
 *
 *   sccsum_spans        N x { checksummer c; [pseudo-header seed];
 *                             c.sum(data, len); c.get(); }
 *                       = ip_checksum(const void*, size_t)  src/net/ip_checksum.cc:70-74
 *                         checksummer::sum(const char*, size_t)  src/net/ip_checksum.cc:31-53
 *                         checksummer::get() const  src/net/ip_checksum.cc:55-62
 *                       as used by UDP generate  src/net/udp.cc:184-195,
 *                       TCP generate  include/seastar/net/tcp.hh:1656-1694, 1004-1016,
 *                       ICMP echo  src/net/ip.cc:471-474, demos/echo_demo.cc:76-78
 *   sccsum_ipv4_frames  N x { IPv4 header verify/generate over sizeof(ip_hdr)=20 B
 *                             src/net/ip.cc:121-127, 271-277;
 *                             length checks / trim / strip 4*ihl  src/net/ip.cc:128-140, 220-225;
 *                             L4 pseudo-header + segment  include/seastar/net/tcp.hh:876-883 }
 *   sccsum_fragments    N x checksummer::sum(const packet&)  src/net/ip_checksum.cc:64-68
 *                       (fragment lists with the odd-byte carry) + get()
 *   sccsum_*_multi      the above for up to 16 batches (rx queues) in one launch
 *   sccsum_pseudo_seed  ipv4_traits::{tcp,udp}_pseudo_header_checksum
 *                       include/seastar/net/ip.hh:70-75 (host arithmetic, O(1))
 *
 * Result convention (same as the reference): each 16-bit checksum is returned
 * with its bytes already in network order, i.e. storing the uint16_t to the
 * packet's checksum field writes the wire bytes (ip_checksum.cc:61,
 * tcp.hh:283-285).  A verify passes when the recomputed value is 0.
 *
 * Memory contract:
 *   - d_bytes, d_off, d_len, d_seed, d_out*, d_status are DEVICE pointers
 *     (hipMalloc / torch CUDA tensors) on the calling thread's current device.
 *   - bytes_len is the number of valid bytes at d_bytes.  The kernels read in
 *     aligned 16-byte units, so the allocation must be readable up to
 *     roundup(bytes_len, 16) (hipMalloc allocations always are).
 *   - A packet whose [off, off+len) is not inside [0, bytes_len) is not read:
 *     its outputs are 0 and its status has SCCSUM_ST_RANGE.
 *   - d_bytes must be 16-byte aligned, d_off 8-byte aligned, d_len/d_seed/d_out2 4-byte aligned,
 *     d_out 2-byte aligned.
 *   - `stream` must belong to the calling thread's current device (the one
 *     the data lives on; NULL = that device's null stream).  HIP runs a kernel
 *     on its stream's device, so each launch takes the device from the stream
 *     (hipStreamGetDevice) and sizes its grid and takes its tile-counter slot
 *     on that device; a stream of another device returns SCCSUM_EINVAL and
 *     launches nothing.  A shard thread bound to device d (sccsum_init(d))
 *     launches on streams it created while d was current.
 *   - Errors: an entry returns its own launch's error (hipLaunchKernel's);
 *     a pending HIP error from an earlier, unrelated call on the thread is
 *     left pending, neither cleared nor reported as this call's.
 *   - Launches are asynchronous on `stream` (a hipStream_t; NULL = the
 *     device's null stream), one kernel each (two for in-place fill and
 *     fragment lists).  No allocation, no memset and no host synchronisation
 *     on the launch path — sccsum_init allocates the device's pool of tile
 *     counters once; the one exception is sccsum_ipv4_fill with a NULL
 *     d_out2, whose scratch is a stream-ordered hipMallocAsync / hipFreeAsync
 *     pair on `stream` — so the calls are safe inside hipStreamBeginCapture
 *     (global or relaxed mode) and never stall another stream.  Any number
 *     of launches may be in flight, on any streams: a launch takes a counter
 *     slot no unfinished launch holds, and the kernel itself reports when it
 *     is done with it (streams may be created and destroyed freely; a
 *     destroyed stream's address reused by a new stream shares nothing).
 *     Captured launches, and launches that find no free slot, use a static
 *     tile order instead (same results, without the dynamic balance).
 *
 * Threading: Seastar's model — one reactor thread per shard, all of them
 * on one device or each on its own — is supported: any number of host
 * threads may call concurrently, each on its own streams (the counter pool
 * is shared under a per-device lock held for a few ring probes per launch).
 * Diagnostic knobs (sccsum_diag.h) are per thread.  A burst queue or a
 * pipeline object belongs to one thread; a resident engine takes steps from
 * any number of threads (its "Producers" paragraph below).
 */
#ifndef SCCSUM_H
#define SCCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 3): frames leave IP fragments' L4 alone (SCCSUM_ST_IPFRAG), L4
 * values of protocols other than TCP / UDP carry no pseudo-header, fill gained
 * SCCSUM_FILL_ICMP_ECHO ("Migration from ABI 1").
 * 3 (round 5): a launch on a stream of another device is SCCSUM_EINVAL and a
 * pending HIP error is left pending (round 4, unversioned then); the engine
 * gained SCCSUM_EIDLE, fill steps (SCCSUM_ENGINE_FILL,
 * sccsum_engine_submit_fill), one running engine per device
 * (sccsum_engine_start: SCCSUM_EBUSY), and sccsum_engine_create no longer
 * changes the caller's current device.
 * 4 (round 6): engine runs are unbounded (max_steps sizes a descriptor ring),
 * any number of threads may submit into one engine, sccsum_engine_create_opts
 * (idle and dependency limits), SCCSUM_EFAULT; the desc calls accept a NULL
 * descriptor array when no packet has fragments; sccsum_engine_stop / _destroy
 * report SCCSUM_EIDLE only when a published step was left undone. */
#define SCCSUM_ABI_VERSION 4

#define SCCSUM_OK 0
#define SCCSUM_EINVAL (-1)   /* bad argument (null pointer, misalignment) */
#define SCCSUM_ENODEV (-2)   /* no HIP device / device index out of range */
#define SCCSUM_EBUSY  (-3)   /* burst queue: every batch slot is in flight; poll and retry.  engine: the
                                run's steps are used up, a wait timed out, or another engine runs on the device */
#define SCCSUM_EIDLE  (-4)   /* engine: its grid gave up waiting for steps (idle limit); start a new run */
#define SCCSUM_EFAULT (-5)   /* engine: its grid stopped on an internal fault (a wait on a dependency past its
                                limit, a step it could not find); the run is over.  Never expected */

/* per-packet status bits (d_status) */
#define SCCSUM_ST_OK        0x01u /* spans: result == 0; frames: IPv4 header verifies */
#define SCCSUM_ST_L4_OK     0x02u /* frames: L4 (pseudo-header + segment) verifies */
#define SCCSUM_ST_MALFORMED 0x04u /* frames: len < 20, len < ip total length, 4*ihl > ip length, or
                                     fragment offset + ip length > 65535 (ip.cc:115-144: dropped) */
#define SCCSUM_ST_RANGE     0x08u /* [off, off+len) outside the byte buffer: not read */
#define SCCSUM_ST_IPFRAG    0x10u /* frames: an IP fragment (MF set or fragment offset != 0, ip.hh:400-402):
                                     its L4 value is not computed (0, never SCCSUM_ST_L4_OK) — the
                                     reference sums L4 over the reassembled datagram only (ip.cc:164-220) */

/* ABI version of the loaded library (== SCCSUM_ABI_VERSION it was built with). */
int sccsum_abi_version(void);

/* Static text for an error code returned by any entry point. */
const char* sccsum_strerror(int err);

/* Number of visible HIP devices. */
int sccsum_device_count(int* count);

/* The NUMA node a device's PCI function sits on (sysfs numa_node of its
 * hipDeviceGetPCIBusId address), -1 when the platform reports none.  Seastar
 * pins each shard's thread to a core and binds its memory to that core's
 * node (src/core/reactor.cc:4163, src/core/memory.cc:1898-1951); a shard
 * should drive a GPU on its own node, so its batches and pinned pools do not
 * cross the socket link ("Which GPU a shard drives"). */
int sccsum_device_numa_node(int device, int* node);

/* Bind the calling host thread to `device` (hipSetDevice), cache its
 * compute-unit count for launch sizing and, on the device's first call,
 * allocate its pool of tile counters (2048 slots, 34 MB of HBM, plus 8 KiB
 * of pinned memory the kernels report completion to; zeroed, synchronously).
 * Call it on every thread that launches; launches on a device nobody
 * initialised use the static tile order (same results). */
int sccsum_init(int device);

/* Pseudo-header partial sum exactly as ipv4_traits::*_pseudo_header_checksum
 * leaves it in a fresh checksummer (ip.hh:70-75), folded to 16 bits with
 * end-around carry.  src_host/dst_host are host-order addresses
 * (ipv4_address.ip); len is uint16_t so 65536 wraps to 0 like the reference. */
uint32_t sccsum_pseudo_seed(uint32_t src_host, uint32_t dst_host, uint8_t proto, uint16_t len);

/* Checksum n independent byte spans.
 *   d_out[i]    = checksum of d_bytes[d_off[i] .. d_off[i]+d_len[i]) started
 *                 from seed d_seed[i] (d_seed may be NULL: no seed).
 *   d_status[i] = SCCSUM_ST_OK if d_out[i] == 0 (verify); may be NULL.
 *   max_len     = upper bound of d_len[] used to pick the kernel variant
 *                 (0 = unknown; any value is correct, it only tunes speed). */
int sccsum_spans(const void* d_bytes, uint64_t bytes_len,
                 const uint64_t* d_off, const uint32_t* d_len, const uint32_t* d_seed,
                 uint16_t* d_out, uint8_t* d_status, uint64_t n, uint32_t max_len,
                 void* stream);

/* Checksum n IPv4 frames (IPv4 header first, no Ethernet header), as the rx
 * path ipv4::handle_received_packet (ip.cc:114-229) takes them.
 *   d_out2[2i]   = IPv4 header checksum over 20 bytes (ip.cc:121-127; checked
 *                  on every frame, fragments included)
 *   d_out2[2i+1] = L4 checksum over [4*ihl, min(ip_len, len)): for TCP (6) and
 *                  UDP (17) seeded with the pseudo-header (src, dst, proto from
 *                  the header; length = that L4 span's length as uint16_t:
 *                  tcp.hh:876-883, udp.cc:184-195); for ICMP and every other
 *                  protocol the plain sum, no pseudo-header (ip.cc:471-474);
 *                  0 for an IP fragment (SCCSUM_ST_IPFRAG): the reference
 *                  checks L4 only on the reassembled datagram — sum that with
 *                  sccsum_spans_desc over the fragments' payloads and the
 *                  pseudo-header seed ("Fragments")
 *   For generate, pass frames whose checksum fields are zero and store the
 *   outputs; for verify, pass received frames and test the status bits.
 *   d_status may be NULL.  max_len as for sccsum_spans.
 *   Verify only: d_out2 may be NULL when d_status is given — the launch then
 *   writes 1 status byte per frame instead of 4 + 1 (the reference's verify
 *   keeps only get() != 0: ip.cc:121-127, tcp.hh:876-883).  The same holds
 *   per batch in sccsum_ipv4_frames_multi.  Neither given: SCCSUM_EINVAL. */
int sccsum_ipv4_frames(const void* d_bytes, uint64_t bytes_len,
                       const uint64_t* d_off, const uint32_t* d_len,
                       uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len,
                       void* stream);

/* ---- Several batches in one launch ------------------------------------------
 * Up to SCCSUM_MAX_BATCHES independent batches (e.g. the rx queues of a shard,
 * or a step's tx and rx halves) checksummed by ONE kernel launch: each batch
 * is exactly what sccsum_spans / sccsum_ipv4_frames would compute for it (its
 * own bytes, offsets, lengths, seeds and outputs; same memory contract), but
 * the launch's ramp and drain (~6-7 us on MI355X) are paid once.  batches is
 * a HOST array (read before the call returns); empty batches are skipped.
 * Frames take no seeds (d_seed must be NULL).  SCCSUM_EINVAL for nbatch >
 * SCCSUM_MAX_BATCHES or a bad batch. */
#define SCCSUM_MAX_BATCHES 16

typedef struct sccsum_batch {
    const void* d_bytes;
    uint64_t bytes_len;
    const uint64_t* d_off;
    const uint32_t* d_len;
    const uint32_t* d_seed; /* spans: optional per-packet seed; frames: NULL */
    void* d_out;            /* spans: uint16_t[n]; frames: uint16_t[2n] */
    uint8_t* d_status;      /* optional */
    uint64_t n;
} sccsum_batch;

int sccsum_spans_multi(const sccsum_batch* batches, uint32_t nbatch, uint32_t max_len, void* stream);
int sccsum_ipv4_frames_multi(const sccsum_batch* batches, uint32_t nbatch, uint32_t max_len, void* stream);

/* ---- Resident engine: steps streamed into a running grid -------------------
 * A launch pays a fixed cost — the grid's ramp, the drain of its last tiles
 * and the kernel boundary, ~18-21 us on MI355X — on every call.
 * An engine launches ONE grid that stays resident and takes STEPS from the
 * host while it runs, the way Seastar's reactor keeps polling its queues
 * (src/core/reactor.cc:3543-3550): each step is up to SCCSUM_ENGINE_MAX_BATCHES
 * batches (a step's tx and rx halves, a shard's rx queues), computed exactly
 * as sccsum_*_multi would compute them, and its tiles flow into the same
 * grid without a boundary.  Per step the engine reports completion; its
 * results are written through to device memory, so a DEVICE-TO-HOST copy
 * (hipMemcpy / hipMemcpyAsync to host memory, which a copy engine runs) may
 * read them as soon as sccsum_engine_wait returns for the step.  Anything
 * that runs as a kernel on the device — another library launch, a torch op,
 * a device-to-device copy that HIP runs as a blit kernel — waits for the run
 * to stop (see "Sharing the device" below).
 *
 *   sccsum_engine_create(device, mode, max_steps, max_in_flight, &e)
 *       mode SCCSUM_PIPE_IPV4 (frames) or SCCSUM_PIPE_SPANS, frames may add
 *       SCCSUM_ENGINE_FILL (the run also takes fill steps; max_in_flight >= 2);
 *       max_steps (1..65536, rounded up to a power of two, at least 2) = the
 *       slots of the engine's descriptor RING (512 B of pinned memory and as
 *       much device memory each): a run takes any number of steps, a slot
 *       being reused once its step is done; at most min(max_in_flight (1..256),
 *       max_steps) steps submitted and not yet done.  Allocates on `device`;
 *       the calling thread's current device is left as it was.
 *   sccsum_engine_create_opts(device, mode, &opts, &e)   the same with every
 *       limit given (sccsum_engine_opts; a 0 field takes its default)
 *   sccsum_engine_start(e, stream)      launch the grid on `stream` (a run);
 *       `stream` belongs to the engine's device, which must be the calling
 *       thread's current device (sccsum_init(device)).  SCCSUM_EBUSY when
 *       another engine of this process runs on the device.
 *   sccsum_engine_submit(e, batches, nbatch, max_len, timeout_ns, &step)
 *       publish one step; waits (spinning, up to timeout_ns) while the
 *       in-flight limit's steps are pending.  SCCSUM_EBUSY: the wait timed
 *       out; SCCSUM_EINVAL: the engine is not running (never started, or
 *       stopped); SCCSUM_EIDLE / SCCSUM_EFAULT: the run is over.
 *       max_len (0 = unknown) caps the mean packet length the step's tiles
 *       are sized by (bytes_len / n otherwise, too big for a batch that is a
 *       slice of a larger buffer).  The engine always runs the flat kernel, so
 *       sparse layouts give exact results but belong on the launches, whose
 *       row kernel reads them faster.  Frames take no seeds.  A step whose
 *       batches are all empty is done once the grid has taken it in.
 *   sccsum_engine_submit_fill(e, batches, nbatch, max_len, mode, timeout_ns, &step)
 *       an in-place fill (sccsum_ipv4_fill's SCCSUM_FILL_L4 and/or
 *       SCCSUM_FILL_ICMP_ECHO, optionally | SCCSUM_FILL_IP) of every batch
 *       (d_bytes is written; each batch's d_out, required here, gets the
 *       values stored and d_status the status bits).  A fill of at most
 *       524 288 frames (sccsum_set_fill_single_max) is ONE step whose tiles
 *       store the fields themselves; a larger one is two consecutive steps: a
 *       generate step into d_out and a store step whose tiles wait for it and
 *       write the values into the frames' fields (both or neither are
 *       published).  *step = the fill's last step: once it is done the frames
 *       are wire-ready in device memory and d_out holds the values stored.  No
 *       other step may write a fill's d_out (nor its frames) before the fill is
 *       done.  max_len as for submit.
 *   sccsum_engine_wait(e, step, timeout_ns)   0 once the step is done;
 *       SCCSUM_EBUSY on time out, SCCSUM_EIDLE / SCCSUM_EFAULT if the grid
 *       gave up before the step was done
 *   sccsum_engine_stop(e)               no more steps: the grid leaves once the
 *       published steps are done (synchronise `stream` to wait for it).
 *       SCCSUM_EIDLE (SCCSUM_EFAULT) when the grid had already given up with a
 *       published step not done: after the stream sync,
 *       sccsum_engine_wait(e, step, 0) still answers for every step of the
 *       run's last max_steps (0 done, the give-up's code otherwise)
 *   sccsum_engine_destroy(e)            stops and synchronises a running engine;
 *       SCCSUM_EIDLE (SCCSUM_EFAULT) if its last run left a published step
 *       undone (a give-up after every step was done loses nothing: 0)
 *
 * Producers.  Any number of host threads may submit into one running engine
 * and wait on its steps — the shards that share a GPU, each with its own
 * batches: a step's number, first tile and descriptor are taken and published
 * under the engine's lock (a few hundred ns, no device call), so steps are
 * published in the order their submits took the lock, and a submit that waits
 * for room waits outside it.  The in-flight limit is the engine's, shared by
 * every producer; opts.producer_in_flight adds one per producer thread, so
 * that no shard holds the whole shared limit: a thread's submit past it first
 * waits (within its timeout) for that thread's oldest step not yet done.  (A
 * fill counts once: by its last step.)  Start, stop and destroy belong to the engine's owner (a
 * submit after stop returns SCCSUM_EINVAL; destroy only after every producer's
 * last call has returned).
 *
 * Sharing the device.  The grid holds the device's compute units while it
 * runs (every CU, all of their LDS): kernels that other threads or streams
 * launch on the device — this library's launches included — queue until the
 * run stops, and then complete.  So one engine runs per device at a time
 * (per process: a second start returns SCCSUM_EBUSY until the first run's
 * stop), and the shards of a GPU submit into its one engine (Producers) or
 * use launches while no engine runs there.  A grid given no new step (and no
 * stop) for its idle limit (default 1 s) leaves on its own, and every later
 * call on that run returns SCCSUM_EIDLE: the limit counts from the last step
 * the grid received, so steady light traffic never trips it. */
#define SCCSUM_ENGINE_MAX_BATCHES 4
#define SCCSUM_ENGINE_FILL 0x100 /* sccsum_engine_create mode flag: the run takes fill steps too */
typedef struct sccsum_engine sccsum_engine;
typedef struct sccsum_engine_opts {
    uint32_t ring_slots;    /* descriptor ring slots, 1..65536 (a power of two, at least 2, above); 0 = 1024 */
    uint32_t max_in_flight; /* steps submitted and not yet done, 1..256 (fill engines: >= 2); 0 = 8 */
    uint32_t idle_ms;       /* the grid leaves after this long without a new step (SCCSUM_EIDLE),
                               1..3 600 000; 0 = 1000 */
    uint32_t dep_ms;        /* limit of a step's wait on the step it depends on (a fill's store step on its
                               generate step, a barrier; SCCSUM_EFAULT past it), 1..3 600 000; 0 = 2000 */
    uint32_t producer_in_flight; /* one producer thread's own steps submitted and not yet done,
                                    1..max_in_flight; 0 = no limit of its own (Producers) */
} sccsum_engine_opts;
int sccsum_engine_create(int device, int mode, uint32_t max_steps, uint32_t max_in_flight, sccsum_engine** out);
int sccsum_engine_create_opts(int device, int mode, const sccsum_engine_opts* opts, sccsum_engine** out);
int sccsum_engine_start(sccsum_engine* e, void* stream);
int sccsum_engine_submit(sccsum_engine* e, const sccsum_batch* batches, uint32_t nbatch, uint32_t max_len,
                         uint64_t timeout_ns, uint64_t* step);
int sccsum_engine_submit_fill(sccsum_engine* e, const sccsum_batch* batches, uint32_t nbatch, uint32_t max_len,
                              uint32_t mode, uint64_t timeout_ns, uint64_t* step);
int sccsum_engine_wait(sccsum_engine* e, uint64_t step, uint64_t timeout_ns);
int sccsum_engine_stop(sccsum_engine* e);
int sccsum_engine_destroy(sccsum_engine* e);

/* Checksum n packets that are FRAGMENT LISTS, like checksummer::sum(const
 * packet&) (src/net/ip_checksum.cc:64-68): packet i is the concatenation of
 * fragments d_pkt_first[i] .. d_pkt_first[i+1]-1, fragment j being
 * d_bytes[d_frag_off[j] .. +d_frag_len[j]) (any order, any alignment; DPDK
 * multi-segment mbufs, virtio mergeable buffers).  A fragment that starts at
 * an odd offset of its packet contributes byte-swapped, exactly the
 * reference's `odd` carry.  d_pkt_first has n+1 nondecreasing entries ending
 * at nfrag; d_seed / d_status optional as for sccsum_spans.  d_workspace:
 * device scratch of sccsum_fragments_workspace(nfrag) bytes, 16-byte aligned.
 * A packet with a fragment outside the buffer (or a bad d_pkt_first range)
 * gets 0 and SCCSUM_ST_RANGE. */
int sccsum_fragments(const void* d_bytes, uint64_t bytes_len,
                     const uint64_t* d_frag_off, const uint32_t* d_frag_len, uint64_t nfrag,
                     const uint32_t* d_pkt_first, const uint32_t* d_seed,
                     uint16_t* d_out, uint8_t* d_status, uint64_t n, uint32_t max_frag_len,
                     void* d_workspace, void* stream);
uint64_t sccsum_fragments_workspace(uint64_t nfrag);

/* sccsum_ipv4_fill modes */
/* ---- RSS: the Toeplitz hash the rx path steers flows by --------------------
 * include/seastar/net/toeplitz.hh:78-98 over the forward_hash the stack
 * builds for a frame (net.hh:53-75):
 *   SCCSUM_RSS_DISPATCH (net.cc:330-341 -> ip.cc:77-92): src + dst IP, then
 *     for an atomic TCP / UDP datagram (MF clear, fragment offset 0) the 4
 *     port bytes at frame offset 20 (sizeof(ip_hdr): options not skipped),
 *     if the frame holds the TCP (20 B) / UDP (8 B) header there
 *     (tcp.hh:852-862, udp.cc:153-161);
 *   SCCSUM_RSS_REASSEMBLED (ip.cc:186-197): src + dst IP, then the ports at
 *     4*ihl when the L4 part (up to min(ip total length, len)) holds the
 *     TCP / UDP header.
 * key: HOST pointer, key_len >= 4 bytes (the reference's defaults are 40 and
 * 52 bytes, toeplitz.hh:52-71; only the first 16 can reach a 12-byte input).
 * d_hash[i] = the 32-bit hash; 0 for a malformed frame (shorter than 20 B, or
 * REASSEMBLED with 4*ihl past the datagram: status SCCSUM_ST_MALFORMED) or an
 * out-of-range one (SCCSUM_ST_RANGE). */
#define SCCSUM_RSS_DISPATCH    0
#define SCCSUM_RSS_REASSEMBLED 1

/* RSS hashes alone (one thread per frame, reads ~28 header bytes each). */
int sccsum_ipv4_rss(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                    const uint8_t* key, uint32_t key_len, int mode, uint32_t* d_hash, uint8_t* d_status, uint64_t n,
                    void* stream);

/* sccsum_ipv4_frames plus the RSS hash of every frame in the same pass (the
 * flat kernel computes it from the header bytes it already holds; no extra
 * HBM traffic beyond the 4-byte hash). */
int sccsum_ipv4_frames_rss(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                           uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len, const uint8_t* key,
                           uint32_t key_len, int rss_mode, uint32_t* d_hash, void* stream);

#define SCCSUM_FILL_IP        0x01u /* IPv4 header checksum, field at +10 (ip.cc:266-278) */
#define SCCSUM_FILL_L4        0x02u /* full TCP/UDP checksum: pseudo-header + segment (udp.cc:190-192,
                                       tcp.hh:1691-1692 without tx offload) */
#define SCCSUM_FILL_L4_PSEUDO 0x04u /* tx-offload partial: the folded pseudo-header alone, i.e. the
                                       reference's `~csum.get()` (udp.cc:188-189, tcp.hh:1688-1689) */
#define SCCSUM_FILL_TSO       0x08u /* with L4_PSEUDO: TCP pseudo-header length 0 (tcp.hh:1674-1676) */
#define SCCSUM_FILL_ICMP_ECHO 0x10u /* ICMP echo request -> echo reply in place: type 0, code 0, checksum
                                       over the ICMP message, no pseudo-header (icmp::received,
                                       ip.cc:464-474); other ICMP types are left alone */

/* GENERATE checksums for n IPv4 frames and STORE them in the frames, in
 * place: wire-ready frames, the tx half of the native stack.  Each checksum
 * is computed as if its own field were zero, as the reference does (fresh
 * headers are value-initialised, packet.hh:586-589; ip.cc:270), so the
 * fields' current contents do not matter.  The L4 field is UDP +6 / TCP +16
 * (ICMP +2 with SCCSUM_FILL_ICMP_ECHO) after 4*ihl; other protocols' L4 is
 * left alone, as is any frame that is malformed (as in sccsum_ipv4_frames),
 * too short to hold the field, or whose ihl is below 5 (its L4 header would
 * overlap the 20-byte IP header; ipv4::send always writes ihl 5, ip.cc:249).  An IP fragment gets the IP header checksum
 * only (ipv4::send checksums each fragment's header, ip.cc:256-278, after the
 * L4 writer summed the whole datagram, ip.cc:283-294): its L4 bytes — the
 * first fragment's L4 header, a later fragment's payload — are never written.
 *   mode: SCCSUM_FILL_IP and/or one of SCCSUM_FILL_L4 / SCCSUM_FILL_L4_PSEUDO
 *         (| SCCSUM_FILL_TSO), and/or SCCSUM_FILL_ICMP_ECHO (not with
 *         L4_PSEUDO).  FILL_L4 and FILL_ICMP_ECHO read every byte (the flat
 *         kernel generates into d_out2, then a second pass stores the
 *         fields); the others read only the 20-byte header.
 *   d_out2[2i] / [2i+1] = the IP / L4 values stored (0 where nothing was
 *         stored); may be NULL: FILL_L4 / FILL_ICMP_ECHO then hand the values
 *         between the passes in a stream-ordered allocation (hipMallocAsync /
 *         hipFreeAsync on `stream`; ABI 2 as first released in round 3
 *         refused NULL here).
 *   d_status[i] = SCCSUM_ST_OK if the IP field was written, SCCSUM_ST_L4_OK
 *         if the L4 field was written, plus MALFORMED / RANGE / IPFRAG; may
 *         be NULL.
 * Frames must not overlap each other. */
int sccsum_ipv4_fill(void* d_bytes, uint64_t bytes_len,
                     const uint64_t* d_off, const uint32_t* d_len,
                     uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len,
                     uint32_t mode, void* stream);

/* Wait for all work queued on `stream`. */
int sccsum_sync(void* stream);

/* ---------------------------------------------------------------------------
 * Host pipeline: batches that live in HOST memory (DPDK mbuf pools, socket
 * buffers).  The batch is cut into chunks of at most chunk_packets packets /
 * chunk_bytes bytes; each chunk is copied to HBM on a copy stream
 * (hipMemcpyAsync, pinned staging), checksummed on a compute stream and its
 * results copied back, with `depth` chunks in flight so the copies overlap
 * the kernels.  The device work is the same sccsum_spans / sccsum_ipv4_frames.
 * ------------------------------------------------------------------------- */
typedef struct sccsum_pipeline sccsum_pipeline;

#define SCCSUM_PIPE_SPANS 0
#define SCCSUM_PIPE_IPV4  1

#define SCCSUM_GATHER_NONE    0 /* copy each chunk's covering byte range as it lies */
#define SCCSUM_GATHER_HOST    1 /* pack packets into pinned staging on the host first */
#define SCCSUM_GATHER_STRIDED 2 /* packets at one pitch (mbuf slots): one 2D DMA of each slot's packet bytes */
#define SCCSUM_GATHER_ZERO_COPY 3 /* no copies: the kernel reads each packet in place (host_bytes pinned / registered) */

/* Allocate device buffers and pinned staging for `depth` chunks on `device`. */
int sccsum_pipeline_create(int device, uint64_t chunk_bytes, uint32_t chunk_packets, int depth,
                           sccsum_pipeline** out);

/* Checksum n packets at host_bytes[host_off[i] .. +host_len[i]) (all HOST
 * pointers; host_bytes should be pinned — sccsum_host_alloc — unless gather
 * is 1).  gather = 0: each chunk's covering byte range is copied as it lies
 * (e.g. whole mbuf slots, headers and headroom included); gather = 1: the
 * packets are first packed into pinned staging on the host (only packet bytes
 * cross PCIe); gather = 2: where a chunk's packets sit at one pitch P (the
 * slots of an mbuf pool, dpdk.cc:139-156) and none is longer than P, one 2D
 * DMA (hipMemcpy2DAsync) copies the first W bytes of each slot, W = the
 * chunk's longest packet — only packet bytes cross PCIe, with no host copy;
 * other chunks are copied as they lie; gather = 3: nothing is copied — one
 * fragment-list launch per chunk reads every packet in place over PCIe
 * (packet bytes only) and writes its results to pinned staging; host_bytes
 * must be pinned or registered (SCCSUM_EINVAL otherwise, checked with
 * hipPointerGetAttributes on both ends).  mode = SCCSUM_PIPE_SPANS (host_seed optional, host_out[n]) or
 * SCCSUM_PIPE_IPV4 (host_out[2n]); host_status optional.  Returns when all
 * results are in host_out.  host_len is the size of the host_bytes area. */
int sccsum_pipeline_run(sccsum_pipeline* p, int mode, int gather, const void* host_bytes, uint64_t host_len,
                        const uint64_t* host_off, const uint32_t* host_lens, const uint32_t* host_seed,
                        uint64_t n, uint32_t max_len, uint16_t* host_out, uint8_t* host_status);

int sccsum_pipeline_destroy(sccsum_pipeline* p);

/* ---- Burst queue: the batching hook at the qp boundary ----------------------
 * The native stack checksums packet by packet on the shard's reactor thread;
 * qp::poll_tx refills up to 128 packets per poll (src/net/net.cc:81-105) and
 * DPDK rx hands over bursts of 32 (src/net/dpdk.cc:2190-2204).  A burst queue
 * accumulates such packets from HOST memory into GPU batches and completes
 * them asynchronously.  It is shaped like a reactor::poller (net.cc:109):
 * every call is non-blocking except sccsum_burst_drain, and sccsum_burst_poll
 * reports whether it did work.  One queue per shard / thread; not thread-safe.
 *
 * mode: SCCSUM_PIPE_SPANS (each packet's sum seeded with its seed, results
 * [count]) or SCCSUM_PIPE_IPV4 (frames: IPv4 header + L4 checksums, results
 * [2*count]).  A batch launches when it holds batch_packets packets or no room
 * for the next one, or on the first poll after max_delay_ns.  depth = batch
 * slots (staging + device buffers each). */
typedef struct sccsum_burst sccsum_burst;

/* Completion, called from sccsum_burst_poll / _drain on the caller's thread:
 * the packets with tickets first_ticket .. first_ticket + count - 1, in submit
 * order; results / status point into the queue's pinned memory, valid until
 * the callback returns.  The callback may submit (a queue never reuses the
 * batch being delivered before the callback returns); poll, drain and
 * destroy called from inside it return SCCSUM_EINVAL and do nothing. */
typedef void (*sccsum_burst_done_fn)(void* user, uint64_t first_ticket, uint32_t count, const uint16_t* results,
                                     const uint8_t* status);

/* batch_bytes: 64 .. 4 GiB - 16 (a batch's byte offsets are 32-bit);
 * depth: 1 .. 64 slots.  SCCSUM_EINVAL otherwise. */
int sccsum_burst_create(int device, int mode, uint64_t batch_bytes, uint32_t batch_packets, uint64_t max_delay_ns,
                        int depth, sccsum_burst_done_fn fn, void* user, sccsum_burst** out);

/* One piece of a packet, in the layout of seastar::net::fragment {char* base;
 * size_t size;} (include/seastar/net/packet.hh:43-46): a packet's
 * fragment_array() / nr_frags() (packet.hh:245-247) pass as they are. */
typedef struct sccsum_fragment {
    const void* base;
    size_t size;
} sccsum_fragment;

/* Stage one packet given as its fragments (checksummer::sum(const packet&)
 * over the fragments in order, ip_checksum.cc:64-68): they are copied into
 * pinned staging now, so the caller may reuse them on return.  *ticket (may be
 * NULL) identifies the packet in the completion.  seed: SCCSUM_PIPE_SPANS only.
 * SCCSUM_EBUSY: every slot is in flight (poll, then retry); SCCSUM_EINVAL: a
 * packet longer than a batch. */
int sccsum_burst_submit(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed,
                        uint64_t* ticket);

/* Zero-copy submit: as sccsum_burst_submit, but the fragments lie in memory
 * the device can read at the same address (see sccsum_gather: pinned or
 * hipHostRegister'd host memory, or device memory) and must stay untouched
 * until the packet's completion.  Only a descriptor is recorded; the batch's
 * launch gathers the bytes on the device (over PCIe for host memory), so no
 * host thread copies packet bytes.  Both submits may be mixed in one queue.
 * SCCSUM_EINVAL also when a packet has more than 4 * batch_packets fragments. */
int sccsum_burst_submit_mapped(sccsum_burst* b, const sccsum_fragment* frags, uint32_t nfrag, uint32_t seed,
                               uint64_t* ticket);

/* Reactor poller: launch the open batch if full or aged; deliver every
 * finished batch.  *did_work (may be NULL) = 1 when it launched or delivered.
 * If a launch fails (an error code from any call that launches: submit, poll,
 * drain), its batch stays staged, nothing of it still runs on the device, and
 * the next poll / drain launches it again. */
int sccsum_burst_poll(sccsum_burst* b, int* did_work);

/* Launch what is staged, wait for every batch in flight, deliver them all. */
int sccsum_burst_drain(sccsum_burst* b);

int sccsum_burst_destroy(sccsum_burst* b);

/* Gather: copy n fragments into one device buffer, d_dst[dst_off ..
 * +len) = src[0 .. len), for every descriptor (one kernel).  src may be device
 * memory or pinned host memory the device can read at the same address
 * (sccsum_host_alloc / hipHostMalloc; hipHostRegister'd memory such as a DPDK
 * mempool, registered once) — then the bytes cross PCIe without a host thread
 * touching them.  Any alignment; destinations must not overlap.  d_desc is a
 * DEVICE array (8-byte aligned).  A descriptor with src == NULL is skipped
 * (its bytes are already in place). */
typedef struct sccsum_gather_desc {
    const void* src;
    uint32_t dst_off;
    uint32_t len;
} sccsum_gather_desc;

int sccsum_gather(const sccsum_gather_desc* d_desc, uint64_t n, void* d_dst, void* stream);

/* Packets as fragment lists, summed where the fragments lie (one kernel, each
 * byte read once — over PCIe for pinned / registered host memory — with no
 * gather into a batch first): checksummer::sum(const packet&)
 * (ip_checksum.cc:64-68) for packets whose fragments may be anywhere the
 * device can read.  Packet p (p < n) has the fragments d_desc[d_first[p] ..
 * d_first[p+1]) (d_first has n + 1 entries), which must tile its bytes in
 * order: fragment j holds packet bytes [dst_off_j - d_off[p], + len_j), so
 * the first starts at dst_off = d_off[p] and the lengths add up to d_len[p].
 * A fragment with src == NULL lies at d_stage + dst_off (bytes already in a
 * device batch; d_stage may be NULL when no fragment uses it).  A packet whose
 * fragments do not tile it gets result 0 and status SCCSUM_ST_RANGE; the
 * d_first entries themselves must index inside d_desc (not checked: the
 * descriptor count is not an argument).  d_desc may be NULL when no packet has
 * a fragment (every packet empty): each packet then has zero fragments, so an
 * empty one gets the empty sum and a non-empty one 0 + SCCSUM_ST_RANGE.
 * Results and status as sccsum_spans / sccsum_ipv4_frames (frames: IPv4
 * header + L4, the header may be split across fragments).  d_desc, d_first,
 * d_off, d_len, d_seed, d_out, d_status: device arrays (aligned to their
 * element size, d_desc to 8).  max_len: the longest packet (sizes the loop). */
int sccsum_spans_desc(const sccsum_gather_desc* d_desc, const uint32_t* d_first, const uint64_t* d_off,
                      const uint32_t* d_len, const uint32_t* d_seed, const void* d_stage, uint16_t* d_out,
                      uint8_t* d_status, uint64_t n, uint32_t max_len, void* stream);
int sccsum_ipv4_frames_desc(const sccsum_gather_desc* d_desc, const uint32_t* d_first, const uint64_t* d_off,
                            const uint32_t* d_len, const void* d_stage, uint16_t* d_out2, uint8_t* d_status,
                            uint64_t n, uint32_t max_len, void* stream);

/* Pinned (page-locked) host memory for packet pools. */
int sccsum_host_alloc(void** p, uint64_t bytes);
int sccsum_host_free(void* p);

#ifdef __cplusplus
}
#endif

#endif /* SCCSUM_H */
