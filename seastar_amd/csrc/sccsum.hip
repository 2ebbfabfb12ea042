// sccsum.hip — CDNA4 (gfx950) batch Internet checksum kernels and the C-ABI
// launchers declared in include/sccsum.h.
//
// Arithmetic (see DESIGN.md "Arithmetic domain"): the reference adds
// big-endian 16-bit words into an __int128 and returns htons(~fold(S))
// (src/net/ip_checksum.cc:31-62).  Because 2^16 == 1 (mod 65535) and
// byte-swapping a 16-bit word multiplies it by 256 (mod 65535), the same
// uint16_t comes out of: sum the bytes as LITTLE-endian 32-bit words, fold
// with end-around carry (zero stays zero, nonzero stays nonzero), byte-swap if
// the span starts at an odd address, complement.  So the kernel may group,
// reorder and widen freely — it loads aligned 16-byte units.
//
// Layout: packets live anywhere inside one byte buffer behind an
// offset (u64) / length (u32) array.  One wavefront owns one packet at a time:
// lane i loads 16-byte units i, i+64, ... of the aligned span covering the
// packet, masks the bytes outside it, accumulates 64-bit lane sums, and the
// wave folds them with DPP row operations + 4 readlanes.  No LDS, no MFMA: a
// byte reduction at the HBM read roofline.

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

#include "sccsum.h"

namespace sccsum {
namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kBlocksPerCU = 8;  // 32 waves/CU: needs <= 64 VGPRs
constexpr int kMaxDevices = 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- device helpers

// End-around-carry fold of a 64-bit sum to [0, 0xffff]; 0 iff s == 0.
__device__ __forceinline__ uint32_t fold16(uint64_t s) {
    s = (s & 0xffffffffull) + (s >> 32);
    s = (s & 0xffffull) + (s >> 16);
    s = (s & 0xffffull) + (s >> 16);
    s = (s & 0xffffull) + (s >> 16);
    return static_cast<uint32_t>(s);
}

__device__ __forceinline__ uint32_t swap16(uint32_t x) {
    return ((x & 0xffu) << 8) | (x >> 8);
}

// Keep the bytes of dword `d` (bytes 4d..4d+3 of a 16-byte unit) that fall in
// [lo, hi) (unit-relative, may be out of [0,16]).
__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int lo, int hi, int d) {
    const int a = min(max(lo - 4 * d, 0), 4);
    const int b = min(max(hi - 4 * d, 0), 4);
    const uint64_t m = ((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull);
    return w & static_cast<uint32_t>(m);
}

__device__ __forceinline__ uint64_t unit_sum(const u32x4& v, int lo, int hi) {
    uint64_t s = keep_bytes(v.x, lo, hi, 0);
    s += keep_bytes(v.y, lo, hi, 1);
    s += keep_bytes(v.z, lo, hi, 2);
    s += keep_bytes(v.w, lo, hi, 3);
    return s;
}

// Sum of a 32-bit value over the 64 lanes of the wave.  All lanes must be
// active.  quad_perm xor1/xor2 and row_ror 4/8 give every lane its 16-lane
// row total; four readlanes add the rows.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));
    v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));
    v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x124, 0xF, 0xF, false));
    v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x128, 0xF, 0xF, false));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 0)) +
           static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 16)) +
           static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 32)) +
           static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 48));
}

__device__ __forceinline__ u32x4 load_unit(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// Logical block id with XCD affinity: blocks b, b+8, b+16 ... are dealt to one
// XCD, so give them consecutive logical ids; neighbouring packets (which share
// their boundary 16-byte unit / cache line) then land on one XCD's L2.
__device__ __forceinline__ uint32_t xcd_block_id() {
    const uint32_t g = gridDim.x;  // host keeps it a multiple of 8
    const uint32_t b = blockIdx.x;
    return (b & 7u) * (g >> 3) + (b >> 3);
}

// ---------------------------------------------------------------- kernels

// U = 16-byte units in flight per lane per group (packet bytes covered by one
// group = U * 1 KiB).  IPV4 = frame mode (IPv4 header + L4 with pseudo-header).
template <int U, bool IPV4>
__global__ __launch_bounds__(kBlock) void csum_kernel(
    const uint8_t* __restrict__ bytes, uint64_t bytes_len,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
    const uint32_t* __restrict__ seed, uint16_t* __restrict__ out,
    uint8_t* __restrict__ status, uint64_t n) {
    const int lane = static_cast<int>(threadIdx.x & (kWave - 1));
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;

    for (uint64_t p = static_cast<uint64_t>(xcd_block_id()) * kWavesPerBlock + wv; p < n; p += stride) {
        const uint64_t o = off[p];
        const uint32_t L = len[p];
        if (o > bytes_len || L > bytes_len - o || (IPV4 && L < 20)) {
            if (lane == 0) {
                if (IPV4) {
                    reinterpret_cast<uint32_t*>(out)[p] = 0;
                } else {
                    out[p] = 0;
                }
                if (status) {
                    status[p] = (o > bytes_len || L > bytes_len - o) ? SCCSUM_ST_RANGE : SCCSUM_ST_MALFORMED;
                }
            }
            continue;
        }
        const uint8_t* ptr = bytes + o;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(ptr);
        const int head = static_cast<int>(addr & 15u);
        const uint8_t* a0 = ptr - head;
        const uint32_t nunits = L ? (static_cast<uint32_t>(head) + L + 15u) >> 4 : 0u;

        // Frame mode: the 20-byte IPv4 header as 5 dwords re-aligned to the
        // packet start (lanes 0..5 load the covering dwords; lane 5 only when
        // the packet is not 4-byte aligned, so every dword read holds a
        // header byte and stays inside the 16-byte unit bound).
        uint32_t hv = 0;
        const int s = static_cast<int>(addr & 3u);
        if (IPV4) {
            if (lane < 5 || (lane == 5 && s != 0)) {
                hv = *reinterpret_cast<const uint32_t*>(ptr - s + 4 * lane);
            }
        }

        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = static_cast<uint32_t>(u * kWave + lane);
            v[u] = c < nunits ? load_unit(a0 + 16u * c) : u32x4{0, 0, 0, 0};
        }

        int rs = head;                        // summed range, relative to a0
        int re = head + static_cast<int>(L);
        uint32_t ipc = 0, pseudo = 0;
        uint8_t st = 0;
        if (IPV4) {
            const uint32_t nxt = static_cast<uint32_t>(
                __builtin_amdgcn_update_dpp(0, static_cast<int>(hv), 0x101, 0xF, 0xF, false));  // row_shl:1
            const uint32_t al = __builtin_amdgcn_alignbyte(nxt, hv, static_cast<uint32_t>(s));
            const uint32_t h0 = __builtin_amdgcn_readlane(al, 0);
            const uint32_t h1 = __builtin_amdgcn_readlane(al, 1);
            const uint32_t h2 = __builtin_amdgcn_readlane(al, 2);
            const uint32_t h3 = __builtin_amdgcn_readlane(al, 3);
            const uint32_t h4 = __builtin_amdgcn_readlane(al, 4);
            ipc = ~fold16(static_cast<uint64_t>(h0) + h1 + h2 + h3 + h4) & 0xffffu;
            const uint32_t ihl = h0 & 0xfu;
            const uint32_t ip_len = swap16(h0 >> 16);
            const uint32_t proto = (h2 >> 8) & 0xffu;
            const uint32_t l4_off = 4u * ihl;
            const uint32_t l4_end = ip_len < L ? ip_len : L;
            uint32_t l4_len = 0;
            if (L < ip_len) st |= SCCSUM_ST_MALFORMED;
            if (l4_off > l4_end) {
                st |= SCCSUM_ST_MALFORMED;
            } else {
                l4_len = l4_end - l4_off;
            }
            rs = head + static_cast<int>(l4_off);
            re = rs + static_cast<int>(l4_len);
            // pseudo-header in the little-endian domain: the address words are
            // header dwords 3 and 4; (0, proto) and the big-endian length swap.
            pseudo = fold16(static_cast<uint64_t>(h3 & 0xffffu) + (h3 >> 16) + (h4 & 0xffffu) + (h4 >> 16) +
                            (proto << 8) + swap16(l4_len & 0xffffu));
        }

        uint64_t acc = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c16 = 16 * (u * kWave + lane);
            acc += unit_sum(v[u], rs - c16, re - c16);
        }
        for (uint32_t g = U * kWave; g < nunits; g += U * kWave) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = g + static_cast<uint32_t>(u * kWave + lane);
                v[u] = c < nunits ? load_unit(a0 + 16u * c) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c16 = 16 * static_cast<int>(g + u * kWave + lane);
                acc += unit_sum(v[u], rs - c16, re - c16);
            }
        }

        uint32_t S = fold16(wave_sum(fold16(acc)));
        if (addr & 1u) S = swap16(S);  // span starts at an odd address (4*ihl is even)
        if (IPV4) {
            S = fold16(static_cast<uint64_t>(S) + pseudo);
        } else if (seed) {
            S = fold16(static_cast<uint64_t>(S) + swap16(fold16(seed[p])));
        }
        const uint32_t r = ~S & 0xffffu;
        if (lane == 0) {
            if (IPV4) {
                reinterpret_cast<uint32_t*>(out)[p] = ipc | (r << 16);
                if (status) {
                    status[p] = st | (ipc == 0 ? SCCSUM_ST_OK : 0u) | (r == 0 ? SCCSUM_ST_L4_OK : 0u);
                }
            } else {
                out[p] = static_cast<uint16_t>(r);
                if (status) status[p] = r == 0 ? SCCSUM_ST_OK : 0u;
            }
        }
    }
}

// Plain stream-read of the same load shape (16 B per lane, nontemporal).
__global__ __launch_bounds__(kBlock) void read_probe_kernel(const u32x4* __restrict__ src, uint64_t units,
                                                             uint64_t* __restrict__ sink) {
    uint64_t acc = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock;
    uint64_t i = static_cast<uint64_t>(xcd_block_id()) * kBlock + threadIdx.x;
    for (; i + 3 * stride < units; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(src + i);
        const u32x4 b = __builtin_nontemporal_load(src + i + stride);
        const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
        const u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
        acc += static_cast<uint64_t>(a.x) + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
        acc += static_cast<uint64_t>(c.x) + c.y + c.z + c.w + d.x + d.y + d.z + d.w;
    }
    for (; i < units; i += stride) {
        const u32x4 a = __builtin_nontemporal_load(src + i);
        acc += static_cast<uint64_t>(a.x) + a.y + a.z + a.w;
    }
    const uint32_t f = wave_sum(fold16(acc));
    if ((threadIdx.x & (kWave - 1)) == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(sink + blockIdx.x), static_cast<unsigned long long>(f));
    }
}

// ---------------------------------------------------------------- host side

std::atomic<int> g_cu_count[kMaxDevices];

int cu_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
    int c = g_cu_count[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    g_cu_count[dev].store(c, std::memory_order_relaxed);
    return c;
}

unsigned grid_for(uint64_t n) {
    const uint64_t cap = static_cast<uint64_t>(cu_count()) * kBlocksPerCU;
    uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    if (want > cap) want = cap;
    want = (want + 7) & ~uint64_t(7);  // multiple of 8 for the XCD mapping
    return static_cast<unsigned>(want);
}

int units_class(uint32_t max_len) {
    if (max_len == 0) return 4;
    const uint64_t units = (static_cast<uint64_t>(max_len) + 30) / 16;  // worst-case head of 15
    if (units <= 64) return 1;
    if (units <= 128) return 2;
    if (units <= 256) return 4;
    return 8;
}

template <bool IPV4>
int launch(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
           const uint32_t* d_seed, uint16_t* d_out, uint8_t* d_status, uint64_t n, uint32_t max_len,
           void* stream) {
    if (n == 0) return SCCSUM_OK;
    if (!d_bytes || !d_off || !d_len || !d_out) return SCCSUM_EINVAL;
    if ((reinterpret_cast<uintptr_t>(d_off) & 7u) || (reinterpret_cast<uintptr_t>(d_len) & 3u) ||
        (reinterpret_cast<uintptr_t>(d_seed) & 3u) ||
        (reinterpret_cast<uintptr_t>(d_out) & (IPV4 ? 3u : 1u))) {
        return SCCSUM_EINVAL;
    }
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(grid_for(n)), block(kBlock);
    const uint8_t* b = static_cast<const uint8_t*>(d_bytes);
    switch (units_class(max_len)) {
        case 1:
            csum_kernel<1, IPV4><<<grid, block, 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n);
            break;
        case 2:
            csum_kernel<2, IPV4><<<grid, block, 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n);
            break;
        case 4:
            csum_kernel<4, IPV4><<<grid, block, 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n);
            break;
        default:
            csum_kernel<8, IPV4><<<grid, block, 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n);
            break;
    }
    return static_cast<int>(hipGetLastError());
}

}  // namespace
}  // namespace sccsum

extern "C" {

int sccsum_abi_version(void) { return SCCSUM_ABI_VERSION; }

const char* sccsum_strerror(int err) {
    if (err == SCCSUM_OK) return "success";
    if (err == SCCSUM_EINVAL) return "invalid argument";
    if (err == SCCSUM_ENODEV) return "no such HIP device";
    if (err > 0) return hipGetErrorString(static_cast<hipError_t>(err));
    return "unknown sccsum error";
}

int sccsum_device_count(int* count) {
    if (!count) return SCCSUM_EINVAL;
    return static_cast<int>(hipGetDeviceCount(count));
}

int sccsum_init(int device) {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return static_cast<int>(e);
    if (device < 0 || device >= n) return SCCSUM_ENODEV;
    const hipError_t e2 = hipSetDevice(device);
    if (e2 != hipSuccess) return static_cast<int>(e2);
    (void)sccsum::cu_count();
    return SCCSUM_OK;
}

// ip.hh:70-75 via checksummer::sum_many(uint32 src, uint32 dst, uint8 0,
// uint8 proto, uint16 len) from a fresh (even) checksummer: the uint8 pair
// forms the big-endian word (0, proto); everything is added as host integers.
uint32_t sccsum_pseudo_seed(uint32_t src_host, uint32_t dst_host, uint8_t proto, uint16_t len) {
    uint64_t s = static_cast<uint64_t>(src_host) + dst_host + proto + len;
    while (s >> 16) s = (s & 0xffffu) + (s >> 16);
    return static_cast<uint32_t>(s);
}

int sccsum_spans(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                 const uint32_t* d_seed, uint16_t* d_out, uint8_t* d_status, uint64_t n, uint32_t max_len,
                 void* stream) {
    return sccsum::launch<false>(d_bytes, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, max_len, stream);
}

int sccsum_ipv4_frames(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                       uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len, void* stream) {
    return sccsum::launch<true>(d_bytes, bytes_len, d_off, d_len, nullptr, d_out2, d_status, n, max_len, stream);
}

int sccsum_sync(void* stream) { return static_cast<int>(hipStreamSynchronize(static_cast<hipStream_t>(stream))); }

int sccsum_read_probe_blocks(void) { return sccsum::cu_count() * sccsum::kBlocksPerCU; }

int sccsum_read_probe(const void* d_src, uint64_t bytes, uint64_t* d_sink, void* stream) {
    if (!d_src || !d_sink || (bytes & 15u) || (reinterpret_cast<uintptr_t>(d_src) & 15u)) return SCCSUM_EINVAL;
    const unsigned grid = static_cast<unsigned>(sccsum_read_probe_blocks()) & ~7u;
    sccsum::read_probe_kernel<<<dim3(grid), dim3(sccsum::kBlock), 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const sccsum::u32x4*>(d_src), bytes / 16, d_sink);
    return static_cast<int>(hipGetLastError());
}

}  // extern "C"
