/*
 * sccsum ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of Seastar's software Internet checksum and of the
 * native-stack call sites that feed it.  It exists to CHECK the product (the
 * HIP batch kernels behind include/sccsum.h) and to provide bench.py's
 * cpu_baseline leg.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it; the product library never links or calls it.
 *
 * Parity pinning: the reference's own build of src/net/ip_checksum.cc is not
 * possible in this image (its TU includes seastar/net/net.hh, which needs the
 * absent fmt library; making it compile would need a stand-in header).  The
 * restatement is pinned instead by the known answers recorded in SURVEY.md
 * §8(c) (outputs of the reference compiled during the survey session) and by
 * the published RFC 1071 / RFC 791 example vectors: tests/golden/kat.json.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to scylladb/seastar).
 */
#ifndef SCCSUM_ORACLE_H
#define SCCSUM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* struct checksummer { __int128 csum = 0; bool odd = false; }
 * include/seastar/net/ip_checksum.hh:35-37 */
typedef struct oracle_checksummer {
    __int128 csum;
    int odd;
} oracle_checksummer;

void oracle_init(oracle_checksummer* c);
/* checksummer::sum(const char*, size_t)   src/net/ip_checksum.cc:31-53 */
void oracle_sum_bytes(oracle_checksummer* c, const uint8_t* data, size_t len);
/* checksummer::sum(uint8_t/uint16_t/uint32_t)   ip_checksum.hh:40-63 */
void oracle_sum_u8(oracle_checksummer* c, uint8_t v);
void oracle_sum_u16(oracle_checksummer* c, uint16_t v);
void oracle_sum_u32(oracle_checksummer* c, uint32_t v);
/* checksummer::get() const   src/net/ip_checksum.cc:55-62 (network-order bytes in a uint16_t) */
uint16_t oracle_get(const oracle_checksummer* c);
/* checksummer::sum(const packet&)   src/net/ip_checksum.cc:64-68 (walks fragments) */
void oracle_sum_fragments(oracle_checksummer* c, const uint8_t* const* bases,
                          const size_t* sizes, size_t nfrag);
/* ip_checksum(const void*, size_t)   src/net/ip_checksum.cc:70-74 */
uint16_t oracle_ip_checksum(const uint8_t* data, size_t len);
/* ipv4_traits::{tcp,udp}_pseudo_header_checksum   include/seastar/net/ip.hh:70-75
 * src/dst are HOST-order addresses (ipv4_address.ip, ipv4_address.hh:42);
 * len is uint16_t, so 65536 wraps to 0 exactly as the reference signature does. */
void oracle_pseudo_header(oracle_checksummer* c, uint32_t src_host, uint32_t dst_host,
                          uint8_t proto, uint16_t len);

/* ---- batch drivers (the reference has none; these apply the per-packet
 *      reference calls to an offset/length array, used as checker + CPU
 *      baseline; nthreads <= 1 runs inline) ---- */

/* out[i] = checksum of bytes[off[i], off[i]+len[i]) after seeding the
 * checksummer with csum = seed[i] (seed may be NULL = 0).  A seed is what a
 * checksummer holds after the pseudo-header, folded (oracle_fold_seed). */
void oracle_batch_spans(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                        const uint32_t* seed, uint16_t* out, uint64_t n, int nthreads);

/* IPv4 frames starting at bytes+off[i] with len[i] bytes, as the rx path
 * src/net/ip.cc:114-229 takes them:
 *   out[2i]   = IPv4 header checksum over exactly 20 B (ip.cc:121-127, 271-277)
 *   out[2i+1] = L4 checksum of [4*ihl, min(ip_len, len)): TCP / UDP seeded with
 *               the pseudo-header (tcp.hh:876-883 verify / udp.cc:184-195
 *               generate), any other protocol without (ICMP, ip.cc:471-474);
 *               0 for an IP fragment (reassembly first, ip.cc:164-220)
 *   status[i] bit0 = IP sum verifies (== 0), bit1 = L4 sum verifies (never for
 *             a fragment), bit2 = malformed (len < 20, len < ip_len, 4*ihl >
 *             ip_len, fragment offset + ip_len > 65535: ip.cc:115-144),
 *             bit4 = IP fragment (MF set or offset != 0, ip.cc:165-166).
 *   status may be NULL. */
void oracle_batch_ipv4(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                       uint16_t* out2, uint8_t* status, uint64_t n, int nthreads);
/* the same, thread t pinned to CPU cpus[t] (the CPU baseline's one thread per
 * physical core, smp::pin at src/core/reactor.cc:4163) */
void oracle_batch_ipv4_cpus(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                            uint16_t* out2, uint8_t* status, uint64_t n, const int* cpus, int nthreads);

/* Fragment lists: packet i = fragments pkt_first[i] .. pkt_first[i+1]-1, each
 * bytes[frag_off[j] .. +frag_len[j]); seeded like oracle_batch_spans, then
 * checksummer::sum(const packet&) (ip_checksum.cc:64-68) + get(). */
void oracle_batch_fragments(const uint8_t* bytes, const uint64_t* frag_off, const uint32_t* frag_len,
                            const uint32_t* pkt_first, const uint32_t* seed, uint16_t* out, uint64_t n);

/* Tx generate, in place, for IPv4 frames (the writers the reference runs on
 * fresh, zero-checksum headers):
 *   mode & 1:  iph->csum = 0; csum.sum(iph, 20); iph->csum = get()      ip.cc:270-276
 *              (every frame, fragments included: ip.cc:256-278 runs per fragment)
 *   mode & 2:  L4 field = 0; pseudo-header + csum.sum(segment); get()    udp.cc:186,192-193 / tcp.hh:1683,1691-1694
 *   mode & 4:  L4 field = ~get() of the pseudo-header alone (tx offload) udp.cc:188-189 / tcp.hh:1688-1689
 *   mode & 8:  with 4, TCP pseudo-header length 0 (TSO)                  tcp.hh:1674-1676
 *   mode & 16: ICMP echo request -> echo reply: type 0, code 0, checksum
 *              over the message, no pseudo-header                        ip.cc:464-474
 * L4 field: UDP +6, TCP +16, ICMP +2 after 4*ihl; written only for proto
 * 17/6 (modes 2, 4) or an ICMP echo request of >= 8 B (mode 16), never into
 * an IP fragment (the reference sums the datagram before ipv4::send cuts it,
 * ip.cc:283-294), only when the frame is not malformed (as oracle_batch_ipv4)
 * and the segment holds the field.  out2 (may be NULL) gets the values stored
 * (0 = none); status bit0 = IP stored, bit1 = L4 stored, bit2 malformed,
 * bit4 fragment, bit3 never (no range checks). */
void oracle_batch_ipv4_fill(uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                            uint16_t* out2, uint8_t* status, uint64_t n, uint32_t mode);

/* Fold a checksummer csum to a seed value (end-around carry, zero stays zero). */
uint32_t oracle_fold_seed(const oracle_checksummer* c);

/* toeplitz_hash(key, data), include/seastar/net/toeplitz.hh:78-98: for each
 * data bit, MSB first, XOR in the 32-bit key window that starts at that bit;
 * key bits shift into the window while i + 4 < key_len. */
uint32_t oracle_toeplitz(const uint8_t* key, size_t key_len, const uint8_t* data, size_t len);

/* RSS hash of one IPv4 frame (no Ethernet header) as the native stack builds
 * its forward_hash (net.hh:53-75: bytes in wire order):
 *   mode 0 (dispatch, net.cc:330-341 -> ip.cc:77-92): src + dst IP, then for
 *     an atomic datagram (MF clear, offset 0) of TCP (tcp.hh:852-862, needs
 *     20 B) or UDP (udp.cc:153-161, needs 8 B) the 4 port bytes at frame
 *     offset 20 (sizeof(ip_hdr), IP options not skipped);
 *   mode 1 (reassembled datagram, ip.cc:186-197): src + dst IP, then for TCP /
 *     UDP the 4 port bytes at 4*ihl when the L4 part (up to min(ip_len, len))
 *     holds 20 / 8 bytes.
 * status: 0 ok, 4 malformed (shorter than 20 B, or 4*ihl past the end: hash 0). */
uint32_t oracle_ipv4_rss(const uint8_t* frame, size_t len, const uint8_t* key, size_t key_len, int mode,
                         uint8_t* status);
void oracle_batch_ipv4_rss(const uint8_t* bytes, const uint64_t* off, const uint32_t* len, uint64_t n,
                           const uint8_t* key, size_t key_len, int mode, uint32_t* hash, uint8_t* status);

#ifdef __cplusplus
}
#endif

#endif
