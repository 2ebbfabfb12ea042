// Native host program over the C++ batch interface: a shard builds a burst of
// IPv4/UDP frames the way ipv4::send / ipv4_udp::send do (ip.cc:249-269,
// udp.cc:178-182), copies it to its GPU, gets every frame's IPv4 and UDP
// checksum from one launch, and checks each against the per-packet API.
#include <hip/hip_runtime.h>
#include <seastar/net/ip_checksum.hh>
#include <seastar/net/ip_checksum_batch.hh>

#include <arpa/inet.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

using namespace seastar::net;

#define HIP_OK(x)                                                             \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 2;                                                         \
        }                                                                     \
    } while (0)

int main() {
    const uint32_t n = 4096;
    std::mt19937 rng(7);
    std::vector<uint8_t> host;
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    std::vector<uint32_t> src(n), dst(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = 28 + rng() % 1473;  // 20 B IPv4 + 8 B UDP + payload
        off[i] = host.size() + (rng() % 3);   // unaligned, sometimes odd
        host.resize(off[i] + L);
        uint8_t* f = host.data() + off[i];
        for (uint32_t k = 0; k < L; ++k) f[k] = uint8_t(rng());
        src[i] = rng();
        dst[i] = rng();
        f[0] = 0x45; f[1] = 0;
        uint16_t be = htons(uint16_t(L)); std::memcpy(f + 2, &be, 2);
        std::memset(f + 4, 0, 4);
        f[8] = 64; f[9] = 17; f[10] = f[11] = 0;
        uint32_t s = htonl(src[i]), d = htonl(dst[i]);
        std::memcpy(f + 12, &s, 4); std::memcpy(f + 16, &d, 4);
        be = htons(uint16_t(L - 20)); std::memcpy(f + 24, &be, 2);
        f[26] = f[27] = 0;
        len[i] = L;
    }
    const size_t cap = (host.size() + 15) & ~size_t(15);
    void* d_bytes; uint64_t* d_off; uint32_t* d_len; uint16_t* d_out; uint8_t* d_st;
    HIP_OK(hipMalloc(&d_bytes, cap));
    HIP_OK(hipMalloc(&d_off, n * 8));
    HIP_OK(hipMalloc(&d_len, n * 4));
    HIP_OK(hipMalloc(&d_out, n * 4));
    HIP_OK(hipMalloc(&d_st, n));
    HIP_OK(hipMemcpy(d_bytes, host.data(), host.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));

    batch_checksummer engine(0);
    device_packet_batch b{d_bytes, host.size(), d_off, d_len, n, 1500};
    hipStream_t stream;
    HIP_OK(hipStreamCreate(&stream));
    engine.ipv4_frames(b, d_out, d_st, stream);
    engine.sync(stream);
    std::vector<uint16_t> out(2 * n);
    std::vector<uint8_t> st(n);
    HIP_OK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(st.data(), d_st, n, hipMemcpyDeviceToHost));

    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = host.data() + off[i];
        checksummer ipc;
        ipc.sum(reinterpret_cast<const char*>(f), 20);
        checksummer l4;
        l4.sum_many(src[i], dst[i], uint8_t(0), uint8_t(17), uint16_t(len[i] - 20));
        l4.sum(reinterpret_cast<const char*>(f + 20), len[i] - 20);
        if (out[2 * i] != ipc.get() || out[2 * i + 1] != l4.get() || (st[i] & SCCSUM_ST_MALFORMED)) {
            if (bad++ < 5) std::printf("frame %u: gpu %04x/%04x cpu %04x/%04x\n", i, out[2 * i], out[2 * i + 1], ipc.get(), l4.get());
        }
    }
    // spans with pseudo-header seeds == the UDP generate calls
    std::vector<uint64_t> off2(n);
    std::vector<uint32_t> len2(n), seed(n);
    for (uint32_t i = 0; i < n; ++i) {
        off2[i] = off[i] + 20;
        len2[i] = len[i] - 20;
        seed[i] = batch_checksummer::pseudo_header_seed(src[i], dst[i], 17, uint16_t(len2[i]));
    }
    uint32_t* d_seed;
    HIP_OK(hipMalloc(&d_seed, n * 4));
    HIP_OK(hipMemcpy(d_off, off2.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len2.data(), n * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed.data(), n * 4, hipMemcpyHostToDevice));
    engine.sum_spans(b, d_seed, d_out, nullptr, stream);
    engine.sync(stream);
    HIP_OK(hipMemcpy(out.data(), d_out, n * 2, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        checksummer l4;
        l4.sum_many(src[i], dst[i], uint8_t(0), uint8_t(17), uint16_t(len2[i]));
        l4.sum(reinterpret_cast<const char*>(host.data() + off2[i]), len2[i]);
        if (out[i] != l4.get() && bad++ < 10) std::printf("span %u: gpu %04x cpu %04x\n", i, out[i], l4.get());
    }
    // the same frames as fragment lists read where they lie: a pinned host copy
    // (zero-copy, over PCIe), each frame cut once at a random point (inside the
    // IPv4 header too) — checksummer::sum(const packet&) without a gather
    uint8_t* pinned = nullptr;
    if (sccsum_host_alloc(reinterpret_cast<void**>(&pinned), host.size()) != SCCSUM_OK) {
        std::printf("FAILED: sccsum_host_alloc\n");
        return 2;
    }
    std::memcpy(pinned, host.data(), host.size());
    std::vector<sccsum_gather_desc> desc;
    std::vector<uint32_t> first(n + 1);
    for (uint32_t i = 0; i < n; ++i) {
        first[i] = static_cast<uint32_t>(desc.size());
        const uint32_t cut = rng() % len[i];  // 0: one fragment
        if (cut) desc.push_back({pinned + off[i], static_cast<uint32_t>(off[i]), cut});
        desc.push_back({pinned + off[i] + cut, static_cast<uint32_t>(off[i] + cut), len[i] - cut});
    }
    first[n] = static_cast<uint32_t>(desc.size());
    sccsum_gather_desc* d_desc;
    uint32_t* d_first;
    HIP_OK(hipMalloc(&d_desc, desc.size() * sizeof(sccsum_gather_desc)));
    HIP_OK(hipMalloc(&d_first, (n + 1) * 4));
    HIP_OK(hipMemcpy(d_desc, desc.data(), desc.size() * sizeof(sccsum_gather_desc), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_first, first.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));
    engine.ipv4_frames_desc(d_desc, d_first, d_off, d_len, n, 1500, nullptr, d_out, d_st, stream);
    engine.sync(stream);
    HIP_OK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = host.data() + off[i];
        checksummer ipc;
        ipc.sum(reinterpret_cast<const char*>(f), 20);
        checksummer l4;
        l4.sum_many(src[i], dst[i], uint8_t(0), uint8_t(17), uint16_t(len[i] - 20));
        l4.sum(reinterpret_cast<const char*>(f + 20), len[i] - 20);
        if ((out[2 * i] != ipc.get() || out[2 * i + 1] != l4.get()) && bad++ < 15) {
            std::printf("fragmented frame %u: gpu %04x/%04x cpu %04x/%04x\n", i, out[2 * i], out[2 * i + 1], ipc.get(),
                        l4.get());
        }
    }
    sccsum_host_free(pinned);
    // in-place generate through the C++ API with no d_out2 (the values cross
    // between the two passes in the library's stream-ordered scratch): each
    // frame's stored fields == the reference writers' checksums
    engine.ipv4_fill(b, SCCSUM_FILL_IP | SCCSUM_FILL_L4, nullptr, nullptr, stream);
    engine.sync(stream);
    std::vector<uint8_t> filled(host.size());
    HIP_OK(hipMemcpy(filled.data(), d_bytes, host.size(), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = host.data() + off[i];  // fields zero: what the writers sum over
        checksummer ipc;
        ipc.sum(reinterpret_cast<const char*>(f), 20);
        checksummer l4;
        l4.sum_many(src[i], dst[i], uint8_t(0), uint8_t(17), uint16_t(len[i] - 20));
        l4.sum(reinterpret_cast<const char*>(f + 20), len[i] - 20);
        uint16_t ip_f, udp_f;
        std::memcpy(&ip_f, filled.data() + off[i] + 10, 2);
        std::memcpy(&udp_f, filled.data() + off[i] + 26, 2);
        if ((ip_f != ipc.get() || udp_f != l4.get()) && bad++ < 20) {
            std::printf("filled frame %u: gpu %04x/%04x cpu %04x/%04x\n", i, ip_f, udp_f, ipc.get(), l4.get());
        }
    }
    if (bad) {
        std::printf("FAILED: %d mismatches\n", bad);
        return 1;
    }
    std::printf("batch_gpu: OK (%u frames + %u seeded spans + %u fragmented frames from pinned memory + %u filled)\n",
                n, n, n, n);
    return 0;
}
