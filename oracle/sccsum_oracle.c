/*
 * sccsum ORACLE — TEST INFRASTRUCTURE ONLY (see sccsum_oracle.h).
 *
 * Restates scylladb/seastar's software Internet checksum in C, keeping the
 * reference's arithmetic shape (big-endian 64-bit words into a 128-bit
 * accumulator, 128->16 fold, htons(~x)) so that its timing is representative
 * when bench.py reports it as the CPU baseline.  Compiled -O2 like Seastar's
 * release mode (configure.py:265).
 */
#define _GNU_SOURCE /* pthread_attr_setaffinity_np (the pinned CPU baseline) */
#include "sccsum_oracle.h"

#include <arpa/inet.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

void oracle_init(oracle_checksummer* c) {
    c->csum = 0;
    c->odd = 0;
}

/* src/net/ip_checksum.cc:31-53.  A pending odd byte (odd==1) is the LOW half
 * of the current 16-bit word (:33-36); then 8-byte big-endian words (:37-41,
 * ntohq = bswap64 on little-endian, byteorder.hh:32-40); then 2-byte words
 * (:42-46); then a trailing byte as the HIGH half (:47-51); odd flips on odd
 * lengths (:52). */
void oracle_sum_bytes(oracle_checksummer* c, const uint8_t* data, size_t len) {
    size_t n = len;
    if (c->odd && n) {
        c->csum += *data++;
        --n;
    } else if (c->odd) {
        /* the reference dereferences data even for len==0 when odd; it then
         * decrements a size_t 0 -> huge.  No caller passes len==0 with odd
         * set (fragments are non-empty, packet.hh:43-46), so stop here. */
        return;
    }
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, data, 8);
        c->csum += __builtin_bswap64(w);
        data += 8;
        n -= 8;
    }
    while (n >= 2) {
        uint16_t h;
        memcpy(&h, data, 2);
        c->csum += ntohs(h);
        data += 2;
        n -= 2;
    }
    if (n) {
        c->csum += (uint32_t)(*data) << 8;
    }
    c->odd ^= (int)(len & 1);
}

/* include/seastar/net/ip_checksum.hh:40-47 */
void oracle_sum_u8(oracle_checksummer* c, uint8_t v) {
    if (!c->odd) {
        c->csum += (uint32_t)v << 8;
    } else {
        c->csum += v;
    }
    c->odd = !c->odd;
}

/* include/seastar/net/ip_checksum.hh:48-55 */
void oracle_sum_u16(oracle_checksummer* c, uint16_t v) {
    if (c->odd) {
        oracle_sum_u8(c, (uint8_t)(v >> 8));
        oracle_sum_u8(c, (uint8_t)v);
    } else {
        c->csum += v;
    }
}

/* include/seastar/net/ip_checksum.hh:56-63 (odd case adds the LOW half first) */
void oracle_sum_u32(oracle_checksummer* c, uint32_t v) {
    if (c->odd) {
        oracle_sum_u16(c, (uint16_t)v);
        oracle_sum_u16(c, (uint16_t)(v >> 16));
    } else {
        c->csum += v;
    }
}

/* src/net/ip_checksum.cc:55-62: 128->64 (twice, end-around), 64->16 by four
 * 16-bit lanes, two more end-around folds, complement, htons. */
uint16_t oracle_get(const oracle_checksummer* c) {
    const unsigned __int128 m64 = (unsigned __int128)0xffffffffffffffffULL;
    unsigned __int128 x = (unsigned __int128)c->csum;
    unsigned __int128 y = (x & m64) + (x >> 64);
    uint64_t s = (uint64_t)((y & m64) + (y >> 64));
    s = (s & 0xffff) + ((s >> 16) & 0xffff) + ((s >> 32) & 0xffff) + (s >> 48);
    s = (s & 0xffff) + (s >> 16);
    s = (s & 0xffff) + (s >> 16);
    return htons((uint16_t)~s);
}

/* src/net/ip_checksum.cc:64-68 */
void oracle_sum_fragments(oracle_checksummer* c, const uint8_t* const* bases,
                          const size_t* sizes, size_t nfrag) {
    for (size_t i = 0; i < nfrag; ++i) {
        oracle_sum_bytes(c, bases[i], sizes[i]);
    }
}

/* src/net/ip_checksum.cc:70-74 */
uint16_t oracle_ip_checksum(const uint8_t* data, size_t len) {
    oracle_checksummer c;
    oracle_init(&c);
    oracle_sum_bytes(&c, data, len);
    return oracle_get(&c);
}

/* include/seastar/net/ip.hh:70-75: sum_many(src.ip.raw, dst.ip.raw,
 * uint8_t(0), uint8_t(proto), uint16_t len) */
void oracle_pseudo_header(oracle_checksummer* c, uint32_t src_host, uint32_t dst_host,
                          uint8_t proto, uint16_t len) {
    oracle_sum_u32(c, src_host);
    oracle_sum_u32(c, dst_host);
    oracle_sum_u8(c, 0);
    oracle_sum_u8(c, proto);
    oracle_sum_u16(c, len);
}

uint32_t oracle_fold_seed(const oracle_checksummer* c) {
    unsigned __int128 x = (unsigned __int128)c->csum;
    while (x >> 16) {
        x = (x & 0xffff) + (x >> 16);
    }
    return (uint32_t)x;
}

/* ---------------- batch drivers ---------------- */

static uint32_t rd_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void one_span(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                     const uint32_t* seed, uint16_t* out, uint64_t i) {
    oracle_checksummer c;
    oracle_init(&c);
    if (seed) {
        c.csum = seed[i];
    }
    oracle_sum_bytes(&c, bytes + off[i], len[i]);
    out[i] = oracle_get(&c);
}

/* IPv4 header fields the rx path decodes (ip_hdr, include/seastar/net/ip.hh:381-403). */
typedef struct {
    uint32_t ihl, ip_len, proto, l4_off, l4_len;
    int frag;      /* MF set or fragment offset != 0 (ip.hh:400-402, ip.cc:165-166) */
    uint8_t st;    /* MALFORMED / IPFRAG bits */
} frame_info;

/* The length / fragment checks of ipv4::handle_received_packet
 * (src/net/ip.cc:129-144, 165-166) for a frame of n >= 20 bytes. */
static frame_info decode_frame(const uint8_t* p, uint32_t n) {
    frame_info f;
    f.st = 0;
    f.ihl = p[0] & 0xf;
    f.ip_len = ((uint32_t)p[2] << 8) | p[3];
    f.proto = p[9];
    f.l4_off = 4 * f.ihl;
    const uint32_t fragw = ((uint32_t)p[6] << 8) | p[7];
    const uint32_t offset = (fragw & 0x1fff) * 8; /* ip_hdr::offset(): frag << 3, 16 bits (ip.hh:402) */
    f.frag = (fragw & 0x3fff) != 0;               /* mf() (0x2000) or offset != 0 */
    const uint32_t l4_end = f.ip_len < n ? f.ip_len : n;
    if (n < f.ip_len) f.st |= 4; /* :137-139 drop when shorter than the IP length (:134-136 trim when longer) */
    if (offset + l4_end > 65535) f.st |= 4; /* :141-144 (net::ip_packet_len_max, const.hh:42) */
    f.l4_len = 0;
    if (f.l4_off > l4_end) {
        f.st |= 4; /* the 4*ihl strip (:225) would run past the datagram */
    } else {
        f.l4_len = l4_end - f.l4_off;
    }
    if (f.frag) f.st |= 16;
    return f;
}

/* One received IPv4 frame, following ipv4::handle_received_packet
 * (src/net/ip.cc:114-229) and the L4 receivers it hands the datagram to:
 *   :115-118   get_header<ip_hdr>(0): a frame shorter than 20 B     -> MALFORMED
 *   :121-127   header checksum over sizeof(ip_hdr) = 20 B           -> out2[2i], bit0
 *   :129-144   length checks (decode_frame)                          -> MALFORMED
 *   :164-220   MF set or offset != 0: the fragment goes to reassembly and no
 *              L4 checksum is computed on it — only on the reassembled
 *              datagram, whose IP header is not checked again (:120-121,
 *              :456-460)                                             -> IPFRAG, out2[2i+1] = 0
 *   :222-227   otherwise [4*ihl, ip_len) goes to the L4 receiver:
 *              TCP verifies pseudo-header + segment (tcp.hh:876-883);
 *              UDP's value is the same sum (what udp.cc:184-195 generates;
 *              its rx does not verify, udp.cc:164-173); ICMP and any other
 *              protocol: the plain sum, no pseudo-header (ip.cc:471-474)
 *                                                                    -> out2[2i+1], bit1 */
static void one_ipv4(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                     uint16_t* out2, uint8_t* status, uint64_t i) {
    const uint8_t* p = bytes + off[i];
    uint32_t n = len[i];
    if (n < 20) {
        out2[2 * i] = 0;
        out2[2 * i + 1] = 0;
        if (status) status[i] = 4;
        return;
    }
    uint16_t ipc = oracle_ip_checksum(p, 20);
    const frame_info f = decode_frame(p, n);
    uint8_t st = f.st;
    uint16_t l4c = 0;
    if (!f.frag) {
        oracle_checksummer c;
        oracle_init(&c);
        if (f.proto == 6 || f.proto == 17) {
            oracle_pseudo_header(&c, rd_be32(p + 12), rd_be32(p + 16), (uint8_t)f.proto, (uint16_t)f.l4_len);
        }
        oracle_sum_bytes(&c, p + f.l4_off, f.l4_len);
        l4c = oracle_get(&c);
        if (l4c == 0) st |= 2;
    }
    out2[2 * i] = ipc;
    out2[2 * i + 1] = l4c;
    if (ipc == 0) st |= 1;
    if (status) status[i] = st;
}

typedef struct {
    int kind;
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* seed;
    uint16_t* out;
    uint8_t* status;
    uint64_t lo, hi;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        if (j->kind == 0) {
            one_span(j->bytes, j->off, j->len, j->seed, j->out, i);
        } else {
            one_ipv4(j->bytes, j->off, j->len, j->out, j->status, i);
        }
    }
    return 0;
}

/* Shard-per-core like Seastar's smp: contiguous index ranges per thread.
 * With `cpus`, thread t runs pinned to CPU cpus[t] (smp::pin,
 * src/core/reactor.cc:4163 — one shard per core). */
#define ORACLE_MAX_THREADS 1024
/* Never fails: an empty or missing cpus list, a CPU id outside cpu_set_t, a
 * failed allocation or thread creation all fall back to running the work (or
 * that thread's share of it) on the calling thread, unpinned. */
static void run_batch(job_t base, uint64_t n, int nthreads, const int* cpus) {
    if (nthreads < 1 || n < 2 || (nthreads == 1 && !cpus)) {
        base.lo = 0;
        base.hi = n;
        run_job(&base);
        return;
    }
    if (nthreads > ORACLE_MAX_THREADS) nthreads = ORACLE_MAX_THREADS;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    job_t* jobs = (job_t*)malloc(sizeof(job_t) * (size_t)nthreads);
    char* started = (char*)calloc((size_t)nthreads, 1);
    if (!th || !jobs || !started) {
        free(th);
        free(jobs);
        free(started);
        base.lo = 0;
        base.hi = n;
        run_job(&base);
        return;
    }
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = base;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
        pthread_attr_t attr;
        if (pthread_attr_init(&attr) != 0) continue; /* run inline below */
        if (cpus && cpus[t] >= 0 && cpus[t] < CPU_SETSIZE) {
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(cpus[t], &set);
            pthread_attr_setaffinity_np(&attr, sizeof(set), &set);
        }
        started[t] = pthread_create(&th[t], &attr, run_job, &jobs[t]) == 0;
        pthread_attr_destroy(&attr);
    }
    for (int t = 0; t < nthreads; ++t) {
        if (started[t]) {
            pthread_join(th[t], 0);
        } else {
            run_job(&jobs[t]);
        }
    }
    free(th);
    free(jobs);
    free(started);
}

void oracle_batch_spans(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                        const uint32_t* seed, uint16_t* out, uint64_t n, int nthreads) {
    job_t b = {0, bytes, off, len, seed, out, 0, 0, 0};
    run_batch(b, n, nthreads, 0);
}

void oracle_batch_ipv4(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                       uint16_t* out2, uint8_t* status, uint64_t n, int nthreads) {
    job_t b = {1, bytes, off, len, 0, out2, status, 0, 0};
    run_batch(b, n, nthreads, 0);
}

void oracle_batch_ipv4_cpus(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                            uint16_t* out2, uint8_t* status, uint64_t n, const int* cpus, int nthreads) {
    job_t b = {1, bytes, off, len, 0, out2, status, 0, 0};
    run_batch(b, n, nthreads, cpus);
}

/* src/net/ip_checksum.cc:64-68 applied per packet of a fragment-list batch */
void oracle_batch_fragments(const uint8_t* bytes, const uint64_t* frag_off, const uint32_t* frag_len,
                            const uint32_t* pkt_first, const uint32_t* seed, uint16_t* out, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        oracle_checksummer c;
        oracle_init(&c);
        if (seed) {
            c.csum = seed[i];
        }
        for (uint32_t j = pkt_first[i]; j < pkt_first[i + 1]; ++j) {
            oracle_sum_bytes(&c, bytes + frag_off[j], frag_len[j]);
        }
        out[i] = oracle_get(&c);
    }
}

/* Tx generate in place (see the header for the reference lines). */
void oracle_batch_ipv4_fill(uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                            uint16_t* out2, uint8_t* status, uint64_t n, uint32_t mode) {
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t* p = bytes + off[i];
        uint32_t L = len[i];
        uint16_t ipw = 0, l4w = 0;
        uint8_t st = 0;
        if (L < 20) {
            st = 4;
        } else {
            const frame_info f = decode_frame(p, L);
            st = f.st;
            const uint8_t proto = (uint8_t)f.proto;
            if (mode & 1) { /* every frame, fragments included: ipv4::send's send_pkt per fragment, ip.cc:256-278 */
                p[10] = p[11] = 0;
                ipw = oracle_ip_checksum(p, 20);
                memcpy(p + 10, &ipw, 2);
                st |= 1;
            }
            /* L4 writers never touch a fragment: the reference sums the whole
             * datagram before ipv4::send cuts it (udp.cc:184-195 / tcp.hh:1656-1694
             * run first, ip.cc:283-294 fragments after).  Nor a frame whose ihl is
             * below 5: its L4 header would overlap the 20-byte IP header, which
             * no reference writer builds (ipv4::send writes ihl 5, ip.cc:249) */
            const int atomic = !f.frag && !(st & 4) && f.ihl >= 5;
            uint32_t fo = proto == 17 ? 6 : (proto == 6 ? 16 : 0);
            if ((mode & 6) && fo && atomic && f.l4_len >= fo + 2) {
                uint8_t* field = p + f.l4_off + fo;
                oracle_checksummer c;
                oracle_init(&c);
                if (mode & 2) {
                    field[0] = field[1] = 0;
                    oracle_pseudo_header(&c, rd_be32(p + 12), rd_be32(p + 16), proto, (uint16_t)f.l4_len);
                    oracle_sum_bytes(&c, p + f.l4_off, f.l4_len);
                    l4w = oracle_get(&c);
                } else {
                    uint32_t plen = ((mode & 8) && proto == 6) ? 0 : f.l4_len;
                    oracle_pseudo_header(&c, rd_be32(p + 12), rd_be32(p + 16), proto, (uint16_t)plen);
                    l4w = (uint16_t)~oracle_get(&c);
                }
                memcpy(field, &l4w, 2);
                st |= 2;
            }
            /* icmp::received (ip.cc:464-474): get_header<icmp_hdr>(0) needs the
             * 8-byte header (ip.hh:143-156); an echo request becomes the reply
             * in place: type echo_reply, code 0, csum 0, sum over p.len() (the
             * message after the 4*ihl strip), csum = get() */
            uint8_t* ih = p + f.l4_off;
            if ((mode & 16) && proto == 1 && atomic && f.l4_len >= 8 && ih[0] == 8) {
                ih[0] = 0;
                ih[1] = 0;
                ih[2] = ih[3] = 0;
                l4w = oracle_ip_checksum(ih, f.l4_len);
                memcpy(ih + 2, &l4w, 2);
                st |= 2;
            }
        }
        if (out2) {
            out2[2 * i] = ipw;
            out2[2 * i + 1] = l4w;
        }
        if (status) status[i] = st;
    }
}

/* ---- RSS (Toeplitz) -------------------------------------------------------- */

/* include/seastar/net/toeplitz.hh:78-98, bit for bit. */
uint32_t oracle_toeplitz(const uint8_t* key, size_t key_len, const uint8_t* data, size_t len) {
    uint32_t hash = 0;
    uint32_t v = ((uint32_t)key[0] << 24) + ((uint32_t)key[1] << 16) + ((uint32_t)key[2] << 8) + key[3];
    for (size_t i = 0; i < len; i++) {
        for (unsigned b = 0; b < 8; b++) {
            if (data[i] & (1u << (7 - b))) hash ^= v;
            v <<= 1;
            if ((i + 4) < key_len && (key[i + 4] & (1u << (7 - b)))) v |= 1;
        }
    }
    return hash;
}

uint32_t oracle_ipv4_rss(const uint8_t* p, size_t len, const uint8_t* key, size_t key_len, int mode,
                         uint8_t* status) {
    uint8_t data[12];
    size_t n = 0;
    *status = 0;
    if (len < 20) {
        *status = 4;
        return 0;
    }
    memcpy(data, p + 12, 8); /* ip.cc:81-82: src_ip, dst_ip as stored (network order) */
    n = 8;
    const uint8_t proto = p[9];
    const uint32_t need = proto == 6 ? 20 : (proto == 17 ? 8 : 0); /* tcp_hdr::len / sizeof(udp_hdr) */
    if (mode == 0) {
        const uint32_t frag = ((uint32_t)p[6] << 8) | p[7];
        const int mf = (frag & 0x2000) != 0, offset = (frag & 0x1fff) != 0; /* ip.hh:390-391 */
        if (need && !mf && !offset && len >= 20 + need) {                 /* ip.cc:87-89 */
            memcpy(data + 8, p + 20, 4);
            n = 12;
        }
    } else {
        const uint32_t ihl = p[0] & 0xf, ip_len = ((uint32_t)p[2] << 8) | p[3];
        const uint32_t l4_off = 4 * ihl, l4_end = ip_len < len ? ip_len : (uint32_t)len;
        if (l4_off > l4_end) {
            *status = 4;
            return 0;
        }
        if (need && l4_end - l4_off >= need) {
            memcpy(data + 8, p + l4_off, 4);
            n = 12;
        }
    }
    return oracle_toeplitz(key, key_len, data, n);
}

void oracle_batch_ipv4_rss(const uint8_t* bytes, const uint64_t* off, const uint32_t* len, uint64_t n,
                           const uint8_t* key, size_t key_len, int mode, uint32_t* hash, uint8_t* status) {
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t st = 0;
        hash[i] = oracle_ipv4_rss(bytes + off[i], len[i], key, key_len, mode, &st);
        if (status) status[i] = st;
    }
}
