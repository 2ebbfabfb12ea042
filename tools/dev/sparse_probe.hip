// sparse_probe — read ceilings of the mbuf-slot layout (development probe, not
// part of libsccsum).
//
// 1,048,576 packets of 1500 B, one per 2304-byte slot at +256 (the DPDK mbuf
// geometry, src/net/dpdk.cc:139-156), in each of R = 4 rotated buffers.  Every
// variant reads the packet bytes (and the slot gaps only in `slab`), sums them
// and writes one status byte per packet, so the compiler keeps the loads.
//   slab     plain nt stream of the whole slot array (gaps included)
//   rows     one packet per 16-lane row, 6 units per lane (the row kernel's loads)
//   rows_pf  rows, with the next step's packets loaded before this step's reduce
//   wave     one packet per wave, 2 units per lane
//   half     one packet per 32-lane half wave, 3 units per lane
//   wrows<K> a wave takes K packets per round trip, two 64-lane rows each
//   rows_m<M>[h] rows with the offsets and lengths loaded from arrays (per step, or 4 steps at once) and
//            with the header dword loads
//   virt<U>  a wave streams a tile of T packets as ONE virtual extent of units
//            (packet k's 94 units follow packet k-1's): U units per lane per
//            round trip, each lane's address from its virtual unit
// usage: sparse_probe [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t kN = 1 << 20;
constexpr uint64_t kSlot = 2304, kData = 256, kLen = 1500;
constexpr uint32_t kUnits = (kLen + 15) / 16;  // 94: the packet is 16-byte aligned
constexpr uint64_t kBytes = kN * kSlot;

__device__ __forceinline__ uint32_t s4(const u32x4& a) { return a.x + a.y + a.z + a.w; }

__global__ __launch_bounds__(256) void k_slab(const u32x4* __restrict__ src, uint64_t units, uint8_t* st) {
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < units; i += stride) {
        acc += s4(__builtin_nontemporal_load(src + i));
    }
    if (acc == 0x12345u) st[0] = 1;
}

// 16 lanes per packet, V units per lane; a block takes 64 consecutive packets (4 steps of 16 rows)
template <int V, bool PF>
__global__ __launch_bounds__(256) void k_rows(const uint8_t* __restrict__ buf, uint64_t n, uint8_t* __restrict__ st) {
    const uint32_t r = threadIdx.x & 15, row = threadIdx.x >> 4;
    const uint64_t nch = (n + 63) / 64;
    auto ld = [&](uint64_t p, u32x4 (&v)[V]) {
        const u32x4* a = reinterpret_cast<const u32x4*>(buf + p * kSlot + kData);
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const uint32_t c = u * 16 + r;
            v[u] = c < kUnits ? __builtin_nontemporal_load(a + c) : u32x4{0, 0, 0, 0};
        }
    };
    for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
        u32x4 cur[V], nxt[V];
        uint64_t p = ch * 64 + row;
        if (p < n) ld(p, cur);
        for (int step = 0; step < 4; ++step) {
            const uint64_t q = p + 16;
            if (PF && step < 3 && q < n) ld(q, nxt);
            if (p < n) {
                uint32_t s = 0;
#pragma unroll
                for (int u = 0; u < V; ++u) s += s4(cur[u]);
                s += __shfl_xor(s, 1, 16) + __shfl_xor(s, 2, 16) + __shfl_xor(s, 4, 16) + __shfl_xor(s, 8, 16);
                if (r == 0) st[p] = static_cast<uint8_t>(s);
            }
            if (!PF && step < 3 && q < n) ld(q, cur);
            if (PF) {
#pragma unroll
                for (int u = 0; u < V; ++u) cur[u] = nxt[u];
            }
            p = q;
        }
    }
}

// rows with the product's metadata: each step's packet offset and length
// loaded from arrays (M = 1: per step, a dependent round trip before the
// data; M = 4: the chunk's four steps loaded at the chunk's start); HDR: the
// row's lanes 0..5 also load the packet's first 24 bytes as dwords (the row
// kernel's IPv4 header loads)
template <int V, int M, bool HDR>
__global__ __launch_bounds__(256) void k_rows_meta(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                   const uint32_t* __restrict__ len, uint64_t n,
                                                   uint8_t* __restrict__ st) {
    const uint32_t r = threadIdx.x & 15, row = threadIdx.x >> 4;
    const uint64_t nch = (n + 63) / 64;
    for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
        uint64_t mo[4];
        uint32_t ml[4];
        if (M == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t p = ch * 64 + k * 16 + row;
                mo[k] = p < n ? off[p] : 0;
                ml[k] = p < n ? len[p] : 0;
            }
        }
#pragma unroll 1
        for (int step = 0; step < 4; ++step) {
            const uint64_t p = ch * 64 + step * 16 + row;
            if (p >= n) break;
            uint64_t o;
            uint32_t L;
            if (M == 4) {
                o = step == 0 ? mo[0] : step == 1 ? mo[1] : step == 2 ? mo[2] : mo[3];
                L = step == 0 ? ml[0] : step == 1 ? ml[1] : step == 2 ? ml[2] : ml[3];
            } else {
                o = off[p];
                L = len[p];
            }
            const uint32_t nu = (L + 15) / 16;
            const u32x4* a = reinterpret_cast<const u32x4*>(buf + o);
            uint32_t hv = 0;
            if (HDR && r < 6) hv = reinterpret_cast<const uint32_t*>(buf + o)[r];
            u32x4 v[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const uint32_t c = u * 16 + r;
                v[u] = c < nu ? __builtin_nontemporal_load(a + c) : u32x4{0, 0, 0, 0};
            }
            uint32_t s = hv;
#pragma unroll
            for (int u = 0; u < V; ++u) s += s4(v[u]);
            s += __shfl_xor(s, 1, 16) + __shfl_xor(s, 2, 16) + __shfl_xor(s, 4, 16) + __shfl_xor(s, 8, 16);
            if (r == 0) st[p] = static_cast<uint8_t>(s);
        }
    }
}

// G lanes per packet (64 = a wave, 32 = a half wave), V units per lane
template <int G, int V>
__global__ __launch_bounds__(256) void k_group(const uint8_t* __restrict__ buf, uint64_t n, uint8_t* __restrict__ st) {
    const uint32_t l = threadIdx.x % G;
    const uint64_t gid = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / G;
    const uint64_t ng = uint64_t(gridDim.x) * 256 / G;
    for (uint64_t p = gid; p < n; p += ng) {
        const u32x4* a = reinterpret_cast<const u32x4*>(buf + p * kSlot + kData);
        u32x4 v[V];
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const uint32_t c = u * G + l;
            v[u] = c < kUnits ? __builtin_nontemporal_load(a + c) : u32x4{0, 0, 0, 0};
        }
        uint32_t s = 0;
#pragma unroll
        for (int u = 0; u < V; ++u) s += s4(v[u]);
        if (l == 0) st[p] = static_cast<uint8_t>(s);
    }
}

// a wave takes K packets per round trip, 2 rows of 64 lanes each (1 KiB + 476 B):
// every row belongs to one packet, so a row's address is wave-uniform
template <int K>
__global__ __launch_bounds__(256) void k_wrows(const uint8_t* __restrict__ buf, uint64_t n, uint8_t* __restrict__ st) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wid = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    for (uint64_t p0 = wid * K; p0 < n; p0 += nw * K) {
        u32x4 v[2 * K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u32x4* a = reinterpret_cast<const u32x4*>(buf + (p0 + k) * kSlot + kData);
            const bool in = p0 + k < n;
            v[2 * k] = in ? __builtin_nontemporal_load(a + lane) : u32x4{0, 0, 0, 0};
            v[2 * k + 1] = in && 64 + lane < kUnits ? __builtin_nontemporal_load(a + 64 + lane) : u32x4{0, 0, 0, 0};
        }
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t s = s4(v[2 * k]) + s4(v[2 * k + 1]);
            s += __shfl_xor(s, 32);
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 8);
            if (lane == static_cast<uint32_t>(k)) mine = s;
        }
        if (lane < K && p0 + lane < n) st[p0 + lane] = static_cast<uint8_t>(mine);
    }
}

// virtual extent: wave w takes tiles of T packets; chunk g holds virtual units [g, g + 64 U)
template <int U, int T>
__global__ __launch_bounds__(256) void k_virt(const uint8_t* __restrict__ buf, uint64_t n, uint8_t* __restrict__ st) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wid = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t ntiles = (n + T - 1) / T;
    for (uint64_t t = wid; t < ntiles; t += nw) {
        const uint64_t p0 = t * T;
        const uint32_t cnt = static_cast<uint32_t>(n - p0 < T ? n - p0 : T);
        const uint32_t ext = cnt * kUnits;
        uint32_t acc = 0;
        for (uint32_t g = 0; g < ext; g += 64 * U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t vu = g + 64 * u + lane;
                const uint32_t k = vu / kUnits, c = vu - k * kUnits;
                v[u] = vu < ext ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                                      buf + (p0 + k) * kSlot + kData) + c)
                                : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += s4(v[u]);
        }
        if (lane < cnt) st[p0 + lane] = static_cast<uint8_t>(acc);
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int R = 4;
    std::vector<uint8_t*> bufs(R);
    for (auto& b : bufs) {
        CK(hipMalloc(&b, kBytes + 64));
        CK(hipMemset(b, 0x5a, kBytes + 64));
    }
    uint8_t* st;
    CK(hipMalloc(&st, kN));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < R; ++w) launch(bufs[w]);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < reps * R; ++k) launch(bufs[k % R]);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / (reps * R);
        const double alg = double(kN) * (kLen + 12 + 1);  // the bench's algorithmic bytes for --config slots
        std::printf("%-10s %8.1f us  packet bytes %6.0f GB/s  alg frac %.4f\n", name, us, kN * kLen / us / 1e3,
                    alg / us / 1e3 / 8000.0);
    };
    const unsigned g8 = static_cast<unsigned>(cus * 8);
    run("slab", [&](uint8_t* b) { k_slab<<<g8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, st); });
    run("rows", [&](uint8_t* b) { k_rows<6, false><<<g8, 256>>>(b, kN, st); });
    run("rows_pf", [&](uint8_t* b) { k_rows<6, true><<<g8, 256>>>(b, kN, st); });
    uint64_t* d_off;
    uint32_t* d_len;
    {
        std::vector<uint64_t> ho(kN);
        std::vector<uint32_t> hl(kN, kLen);
        for (uint64_t i = 0; i < kN; ++i) ho[i] = i * kSlot + kData;
        CK(hipMalloc(&d_off, kN * 8));
        CK(hipMalloc(&d_len, kN * 4));
        CK(hipMemcpy(d_off, ho.data(), kN * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_len, hl.data(), kN * 4, hipMemcpyHostToDevice));
    }
    run("rows_m1", [&](uint8_t* b) { k_rows_meta<6, 1, false><<<g8, 256>>>(b, d_off, d_len, kN, st); });
    run("rows_m4", [&](uint8_t* b) { k_rows_meta<6, 4, false><<<g8, 256>>>(b, d_off, d_len, kN, st); });
    run("rows_m1h", [&](uint8_t* b) { k_rows_meta<6, 1, true><<<g8, 256>>>(b, d_off, d_len, kN, st); });
    run("rows_m4h", [&](uint8_t* b) { k_rows_meta<6, 4, true><<<g8, 256>>>(b, d_off, d_len, kN, st); });
    run("rows", [&](uint8_t* b) { k_rows<6, false><<<g8, 256>>>(b, kN, st); });
    run("wave", [&](uint8_t* b) { k_group<64, 2><<<g8, 256>>>(b, kN, st); });
    run("half", [&](uint8_t* b) { k_group<32, 3><<<g8, 256>>>(b, kN, st); });
    run("wrows4", [&](uint8_t* b) { k_wrows<4><<<g8, 256>>>(b, kN, st); });
    run("wrows8", [&](uint8_t* b) { k_wrows<8><<<static_cast<unsigned>(cus * 4), 256>>>(b, kN, st); });
    run("virt8", [&](uint8_t* b) { k_virt<8, 32><<<g8, 256>>>(b, kN, st); });
    run("virt16", [&](uint8_t* b) { k_virt<16, 32><<<static_cast<unsigned>(cus * 4), 256>>>(b, kN, st); });
    run("virt16t64", [&](uint8_t* b) { k_virt<16, 64><<<static_cast<unsigned>(cus * 4), 256>>>(b, kN, st); });
    run("slab", [&](uint8_t* b) { k_slab<<<g8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, st); });
    std::printf("sparse_probe: %d reps x %d buffers of %llu slots\n", reps, R, static_cast<unsigned long long>(kN));
    return 0;
}
