// Native host program over the C++ resident engine (seastar::net::resident_engine,
// <sccsum.h> sccsum_engine_*): a shard keeps one grid on its GPU and streams
// steps into it.  Tx frames built the way ipv4::send / ipv4_udp::send build
// them (ip.cc:249-269, udp.cc:178-182) are filled in place as a fill step
// (generate step + store step), then verified by a step of the same run
// (it reads the bytes the store step just wrote); a copy of the frames is
// generated into out2 by a plain step.  Every value is checked against the
// per-packet API (checksummer).  A second engine on the device is refused
// while the first runs (try_start false) and runs after its stop.
#include <hip/hip_runtime.h>
#include <seastar/net/ip_checksum.hh>
#include <seastar/net/ip_checksum_batch.hh>

#include <arpa/inet.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

using namespace seastar::net;

#define HIP_OK(x)                                                                                \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
            return 2;                                                                            \
        }                                                                                        \
    } while (0)

int main() {
    const uint32_t n = 8192;
    std::mt19937 rng(11);
    std::vector<uint8_t> host;
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n), src(n), dst(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = 28 + rng() % 1473;
        off[i] = host.size() + (rng() % 3);
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
    // the reference writers' values over the zero-field frames
    std::vector<uint16_t> want_ip(n), want_udp(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = host.data() + off[i];
        checksummer ipc;
        ipc.sum(reinterpret_cast<const char*>(f), 20);
        checksummer l4;
        l4.sum_many(src[i], dst[i], uint8_t(0), uint8_t(17), uint16_t(len[i] - 20));
        l4.sum(reinterpret_cast<const char*>(f + 20), len[i] - 20);
        want_ip[i] = ipc.get();
        want_udp[i] = l4.get();
    }
    const size_t cap = (host.size() + 15) & ~size_t(15);
    void *d_tx, *d_copy;
    uint64_t* d_off;
    uint32_t* d_len;
    uint16_t *d_vals, *d_out;
    uint8_t *d_st, *d_st2;
    HIP_OK(hipMalloc(&d_tx, cap));
    HIP_OK(hipMalloc(&d_copy, cap));
    HIP_OK(hipMalloc(&d_off, n * 8));
    HIP_OK(hipMalloc(&d_len, n * 4));
    HIP_OK(hipMalloc(&d_vals, n * 4));
    HIP_OK(hipMalloc(&d_out, n * 4));
    HIP_OK(hipMalloc(&d_st, n));
    HIP_OK(hipMalloc(&d_st2, n));
    HIP_OK(hipMemcpy(d_tx, host.data(), host.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_copy, host.data(), host.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));

    batch_checksummer shard(0);  // binds this thread to device 0 (sccsum_init)
    hipStream_t stream, other;
    HIP_OK(hipStreamCreate(&stream));
    HIP_OK(hipStreamCreate(&other));
    int bad = 0;
    bool refused = false;
    {
        resident_engine eng(0, SCCSUM_PIPE_IPV4, 64, 8, /*fill=*/true);
        resident_engine second(0, SCCSUM_PIPE_IPV4, 8, 2);
        eng.start(stream);
        refused = !second.try_start(other);  // the device is held by eng's run
        sccsum_batch tx = {d_tx, host.size(), d_off, d_len, nullptr, d_vals, nullptr, n};
        const uint64_t filled = eng.submit_fill(&tx, 1, SCCSUM_FILL_IP | SCCSUM_FILL_L4);
        eng.wait(filled);
        // verify the filled frames in the same run: status bits only (ip.cc:121-127, udp rx keeps none,
        // but a frame that carries its checksums must pass both checks)
        sccsum_batch rx = {d_tx, host.size(), d_off, d_len, nullptr, nullptr, d_st, n};
        sccsum_batch gen = {d_copy, host.size(), d_off, d_len, nullptr, d_out, d_st2, n};
        sccsum_batch step[2] = {rx, gen};
        eng.wait(eng.submit(step, 2));
        eng.stop();
        HIP_OK(hipStreamSynchronize(stream));
        if (!second.try_start(other)) {
            std::printf("second engine still refused after the first run's stop\n");
            ++bad;
        } else {
            sccsum_batch again = {d_copy, host.size(), d_off, d_len, nullptr, d_out, d_st2, n};
            second.wait(second.submit(&again, 1));
            second.stop();
            HIP_OK(hipStreamSynchronize(other));
        }
    }
    if (!refused) {
        std::printf("a second engine started while the first ran\n");
        ++bad;
    }
    std::vector<uint8_t> filled(host.size()), st(n), st2(n);
    std::vector<uint16_t> vals(2 * n), out(2 * n);
    HIP_OK(hipMemcpy(filled.data(), d_tx, host.size(), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(vals.data(), d_vals, n * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(st.data(), d_st, n, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(st2.data(), d_st2, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        uint16_t ip_f, udp_f;
        std::memcpy(&ip_f, filled.data() + off[i] + 10, 2);
        std::memcpy(&udp_f, filled.data() + off[i] + 26, 2);
        if ((ip_f != want_ip[i] || udp_f != want_udp[i] || vals[2 * i] != want_ip[i] ||
             vals[2 * i + 1] != want_udp[i]) && bad++ < 5) {
            std::printf("filled frame %u: fields %04x/%04x values %04x/%04x cpu %04x/%04x\n", i, ip_f, udp_f,
                        vals[2 * i], vals[2 * i + 1], want_ip[i], want_udp[i]);
        }
        if (st[i] != (SCCSUM_ST_OK | SCCSUM_ST_L4_OK) && bad++ < 10) {
            std::printf("filled frame %u does not verify in the same run: status %02x\n", i, st[i]);
        }
        if ((out[2 * i] != want_ip[i] || out[2 * i + 1] != want_udp[i]) && bad++ < 15) {
            std::printf("generated frame %u: %04x/%04x cpu %04x/%04x\n", i, out[2 * i], out[2 * i + 1], want_ip[i],
                        want_udp[i]);
        }
    }
    if (bad) {
        std::printf("FAILED: %d mismatches\n", bad);
        return 1;
    }
    std::printf("engine_gpu: OK (%u frames filled in place and verified in one run, %u generated; "
                "second engine refused while the first ran, then ran)\n", n, n);
    return 0;
}
