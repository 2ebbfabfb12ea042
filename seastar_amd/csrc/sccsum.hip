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
// offset (u64) / length (u32) array.  Default kernel (csum_batch_kernel): a
// wavefront takes a tile of up to 64 packets, plans them one per lane, then
// streams them one packet at a time — every lane loads 16-byte units of the
// packet through a raw buffer descriptor sized to the packet's unit span
// (lanes past it read zeros, no per-lane masking), sums them with v_sad_u16,
// folds the 64 lanes with DPP row ops + 4 readlanes — and finally each lane
// finishes one packet (edge-byte correction from units stashed in LDS, IPv4
// header decode, pseudo-header, complement) with one coalesced store per
// tile.  No MFMA: a byte reduction at the HBM read roofline.
// csum_kernel is a deliberately plain second implementation (one packet per
// wave, per-lane byte masks) kept for cross-checking.

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <type_traits>

#include "sccsum.h"

namespace sccsum {
namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kBlocksPerCU = 8;  // 32 waves/CU: needs <= 64 VGPRs
constexpr int kMaxDevices = 64;
constexpr uint32_t kFlagRaw = 1;     // spans: output the folded span-relative sum (no seed, no complement)
constexpr uint32_t kFlagFillL4 = 2;  // frames: generate the TCP/UDP checksum and store it in the frame
constexpr uint32_t kFlagFillIp = 4;  // frames (with kFlagFillL4): also generate + store the IPv4 header checksum

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
    uint8_t* __restrict__ status, uint64_t n, uint32_t flags) {
    const bool raw = !IPV4 && (flags & kFlagRaw);
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
        } else if (seed && !raw) {
            S = fold16(static_cast<uint64_t>(S) + swap16(fold16(seed[p])));
        }
        const uint32_t r = raw ? S : ~S & 0xffffu;
        if (lane == 0) {
            if (IPV4) {
                reinterpret_cast<uint32_t*>(out)[p] = ipc | (r << 16);
                if (status) {
                    status[p] = st | (ipc == 0 ? SCCSUM_ST_OK : 0u) | (r == 0 ? SCCSUM_ST_L4_OK : 0u);
                }
            } else {
                out[p] = static_cast<uint16_t>(r);
                if (status) status[p] = (!raw && r == 0) ? SCCSUM_ST_OK : 0u;
            }
        }
    }
}

// ---------------------------------------------------------------- batch-kernel helpers

// Keep bytes [lo, hi) of a 64-bit half unit (half-relative byte indices).
__device__ __forceinline__ uint64_t keep_half(uint64_t q, int lo, int hi) {
    const int a = min(max(lo, 0), 8);
    const int b = min(max(hi, 0), 8);
    const int w = b - a;
    const int sh = w > 0 ? 64 - 8 * w : 0;
    const uint64_t m = (~0ull >> sh) << (8 * (w > 0 ? a : 0));
    return w > 0 ? (q & m) : 0ull;
}

// Sum the four dwords of a unit as 16-bit halves into a 32-bit accumulator
// (v_sad_u16 with a zero operand: lo16 + hi16 + acc, one instruction per dword).
__device__ __forceinline__ uint32_t sad4(const u32x4& v, uint32_t acc) {
    acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
    return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

// Masked unit (bytes [lo, hi) kept, unit-relative) summed like sad4.
__device__ __forceinline__ uint32_t sad4_masked(const u32x4& v, int lo, int hi, uint32_t acc) {
    const uint64_t k0 = keep_half(static_cast<uint64_t>(v.x) | (static_cast<uint64_t>(v.y) << 32), lo, hi);
    const uint64_t k1 = keep_half(static_cast<uint64_t>(v.z) | (static_cast<uint64_t>(v.w) << 32), lo - 8, hi - 8);
    acc = __builtin_amdgcn_sad_u16(static_cast<uint32_t>(k0), 0u, acc);
    acc = __builtin_amdgcn_sad_u16(static_cast<uint32_t>(k0 >> 32), 0u, acc);
    acc = __builtin_amdgcn_sad_u16(static_cast<uint32_t>(k1), 0u, acc);
    return __builtin_amdgcn_sad_u16(static_cast<uint32_t>(k1 >> 32), 0u, acc);
}

constexpr int kRsrcFlags = 0x00020000;  // raw buffer, 32-bit data format (gfx950)
constexpr int kNT = 2;                  // nontemporal: streamed once

// Descriptor inputs pass through readfirstlane so the compiler can prove the
// descriptor wave-uniform (otherwise it wraps every buffer op in a waterfall
// loop: guide T20).  Callers only pass wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b >> 32));
    const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
    void* p = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), static_cast<int>(nb), kRsrcFlags);
}

// ---------------------------------------------------------------- batch kernel (default)

// Put a wave-uniform value into lane `k` of `v` (compare + select; gfx9's
// v_writelane cannot read both a value and a lane select from SGPRs).
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t value, uint32_t k, uint32_t lane) {
    return lane == k ? value : v;
}

// Sum of the bytes [lo, hi) of a 16-byte unit as little-endian 16-bit words
// at their unit-relative positions (sad4 of the masked unit).
__device__ __forceinline__ uint32_t unit_part(const u32x4& v, int lo, int hi) {
    return sad4_masked(v, lo, hi, 0u);
}

constexpr uint32_t kStashHead = 4;      // frames: units 0..3 (IPv4 header + the TCP/UDP checksum field)
constexpr uint32_t kStashLast = 64;     // byte offset of the packet's last unit in its row
constexpr uint32_t kStashUnits = 5;     // head units + the last unit
constexpr uint32_t kStashStride = 80;   // bytes per packet row (5 x 16 B: conflict-free ds_read_b128)
constexpr uint32_t kExactMax = 131072;  // fast path keeps exact 32-bit sums up to this length
// tile-head counters: each on its own 256-byte line (atomics to one line
// serialise at the memory side: ~12 ns each chip-wide)
constexpr uint32_t kHeadStride = 64;                      // uint32 words between counters
constexpr uint32_t kGroups = 64;                            // tile-dequeue counters per launch
constexpr uint32_t kHeadSlotWords = kGroups * kHeadStride;  // one launch's counters
#ifndef SCCSUM_LONG_GROUPS
#define SCCSUM_LONG_GROUPS 3
#endif
constexpr int kLongGroups = SCCSUM_LONG_GROUPS;  // groups in flight per step of a long packet
#ifndef SCCSUM_BATCH_MIN_WAVES
#define SCCSUM_BATCH_MIN_WAVES 1  // __launch_bounds__ waves per SIMD floor (8 = cap VGPRs at 64)
#endif
#ifndef SCCSUM_FILL_MIN_WAVES
#define SCCSUM_FILL_MIN_WAVES SCCSUM_BATCH_MIN_WAVES
#endif
static_assert(kStashStride >= 16 * kStashUnits && kStashStride % 16 == 0, "stash row layout");

// Exact folded sum (little-endian domain relative to a0) of [rs, re), one
// wave, any length: the slow path for packets the batch pass cannot take.
__device__ uint32_t exact_range_sum(const uint8_t* a0, uint64_t rs, uint64_t re, uint32_t lane) {
    uint64_t acc = 0;
    if (re > rs) {
        const uint64_t c0 = rs >> 4, c1 = (re - 1) >> 4;
        for (uint64_t c = c0; c <= c1; c += kWave) {
            const uint64_t cu = c + lane;
            u32x4 w = u32x4{0, 0, 0, 0};
            if (cu <= c1) w = load_unit(a0 + 16 * cu);
            const int64_t lo = static_cast<int64_t>(rs) - static_cast<int64_t>(16 * cu);
            const int64_t hi = static_cast<int64_t>(re) - static_cast<int64_t>(16 * cu);
            const int l = static_cast<int>(lo < -16 ? -16 : (lo > 32 ? 32 : lo));
            const int h = static_cast<int>(hi < -16 ? -16 : (hi > 32 ? 32 : hi));
            acc += sad4_masked(w, l, h, 0u);
        }
    }
    return fold16(wave_sum(fold16(acc)));
}

// Batch kernel.  Wave w owns tiles t = w, w + W, ... of B consecutive packets.
//  A: lane i takes packet i of the tile: offset, length, seed, unit span.
//  B: per packet (wave-uniform loop): 3 readlanes, one raw buffer descriptor
//     sized to the packet's 16-byte unit span (lanes past it read zeros),
//     unmasked v_sad_u16 sums, DPP row sums + 4 readlanes -> exact 32-bit
//     sum written into lane k; units 0..2 and the last unit are stashed in LDS.
//  C: lane i finishes packet i: subtracts the stashed bytes outside the
//     summed range, decodes the IPv4 header (frames), folds, adds the seed or
//     pseudo-header, complements; one coalesced store for the tile.
//  D: packets the fast path cannot take (frames with options or a trimmed
//     IP length, spans longer than 128 KiB) are redone exactly, one wave each.
template <int U, bool IPV4, bool PIPE, int AUX, bool HYB, bool MULTI, bool FILL = false>
__global__ __launch_bounds__(kBlock, FILL ? SCCSUM_FILL_MIN_WAVES : SCCSUM_BATCH_MIN_WAVES) void csum_batch_kernel(
    const uint8_t* __restrict__ bytes, uint64_t bytes_len,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
    const uint32_t* __restrict__ seed, uint16_t* __restrict__ out,
    uint8_t* __restrict__ status, uint64_t n, uint32_t B, uint32_t* __restrict__ heads, uint32_t flags) {
    const bool raw = !IPV4 && (flags & kFlagRaw);
    static_assert(!FILL || IPV4, "in-place generate is a frames mode");
    constexpr bool fill = FILL;                          // generate L4 checksums and store them in place
    const bool fill_ip = FILL && (flags & kFlagFillIp);  // ... and the IPv4 header checksum
    __shared__ __attribute__((aligned(16))) uint8_t stash_all[kWavesPerBlock][kWave * kStashStride];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint8_t* stash = stash_all[wv];
    const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
    const uint64_t ntiles = (n + B - 1) / B;
    const bool has_seed = !IPV4 && seed != nullptr;
    const uint32_t vo = 16u * lane;  // this lane's byte offset inside a 1 KiB slice

    // Tile order.  Wave w first takes tile w (static: no start-up contention).
    // With `heads`, the remaining tiles [W, ntiles) are split over kGroups
    // counters (each on its own line) and dequeued: wave w pulls
    // tile W + g + kGroups * atomicAdd(heads[g], 1) with g = w % kGroups, so
    // waves that drew short tiles take more (Zipf batches).  Each group's
    // dequeue count is known — one per remaining tile of the group plus one
    // failing dequeue per wave of the group — so the wave that draws the last
    // number zeroes the counter for the next launch on this slot (no memset,
    // graph-replay safe).  Without `heads`: static round robin.
    const uint64_t wglob = static_cast<uint64_t>(xcd_block_id()) * kWavesPerBlock + wv;
    const uint32_t grp = static_cast<uint32_t>(wglob % kGroups);
    const uint64_t rest = ntiles > nwaves ? ntiles - nwaves : 0;
    const uint32_t tiles_g = rest > grp ? static_cast<uint32_t>((rest - grp + kGroups - 1) / kGroups) : 0u;
    const uint32_t waves_g = static_cast<uint32_t>(nwaves / kGroups);  // host keeps nwaves % kGroups == 0
    auto next_tile = [&](uint64_t prev) -> uint64_t {
        if (heads == nullptr) return prev + nwaves;
        uint32_t d = 0;
        if (lane == 0) {
            uint32_t* h = heads + grp * kHeadStride;
            d = __hip_atomic_fetch_add(h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == tiles_g + waves_g - 1) __hip_atomic_store(h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        d = __builtin_amdgcn_readfirstlane(d);
        return d < tiles_g ? nwaves + grp + static_cast<uint64_t>(kGroups) * d : ntiles;
    };
    // the next tile is dequeued when a tile starts, so the atomic's round trip
    // hides under the tile's loads; a wave stops after its one failing dequeue
    uint64_t t = wglob;
    if (t >= ntiles && heads != nullptr) t = next_tile(t);
    while (t < ntiles) {
        const uint64_t t_next = next_tile(t);
        // ---- A: per-lane packet plan
        const uint64_t base = t * B;
        const uint64_t left = n - base;
        const uint32_t cnt = left < B ? static_cast<uint32_t>(left) : B;
        const bool mine = lane < cnt;
        const uint64_t q = base + (mine ? lane : 0);
        const uint64_t o = off[q];
        const uint32_t L = mine ? len[q] : 0u;
        const uint32_t sd = has_seed ? seed[q] : 0u;
        const bool range_bad = o > bytes_len || L > bytes_len - o;
        const bool short_frame = IPV4 && L < 20;
        const bool huge = L > kExactMax;
        const uint8_t* ptr = bytes + (range_bad ? 0 : o);
        const uint32_t head = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ptr) & 15u);
        const uint64_t a0 = reinterpret_cast<uint64_t>(ptr - head);
        const bool fast = mine && !range_bad && !short_frame && !huge;
        const uint32_t nunits = (fast && L) ? (head + L + 15u) >> 4 : 0u;

        // ---- B: one packet at a time
        // HYB: the units of the packet's last 128-byte line (shared with the
        // next packet when packets are packed back to back) are loaded with
        // the default cache policy so the next packet's first line hits in
        // L2; all other units stream nontemporally.
        uint32_t res = 0;
        struct PktLoad {
            __amdgpu_buffer_rsrc_t r;  // units [0, s)
            uint32_t nu, s;
            u32x4 v[U];
            u32x4 w;  // HYB: lane i <- unit s + i of the last line (i < 8)
        };
        auto issue = [&](uint32_t k, bool valid, PktLoad& P) {
            P.nu = valid ? __builtin_amdgcn_readlane(nunits, k) : 0u;
            const uint32_t alo = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0), k);
            const uint32_t ahi = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0 >> 32), k);
            const uint8_t* pa = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(ahi) << 32) | alo);
            if (HYB) {
                const uint32_t f = (alo >> 4) & 7u;  // first unit's slot in its 128-byte line
                const uint32_t ls = P.nu ? ((f + P.nu - 1) & ~7u) : 0u;
                P.s = ls > f ? ls - f : 0u;
                const auto rw = rsrc(pa + 16u * P.s, 16u * (P.nu - P.s));
                P.w = __builtin_amdgcn_raw_buffer_load_b128(rw, static_cast<int>(vo), 0, 0);
            } else {
                P.s = P.nu;
                P.w = u32x4{0, 0, 0, 0};
            }
            P.r = rsrc(pa, 16u * P.s);
#pragma unroll
            for (int u = 0; u < U; ++u)
                P.v[u] = __builtin_amdgcn_raw_buffer_load_b128(P.r, static_cast<int>(vo + 1024u * u), 0, AUX);
        };
        auto body = [&](uint32_t k, PktLoad& P) {
            uint32_t acc = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) acc = sad4(P.v[u], acc);
            if (HYB) acc = sad4(P.w, acc);
            uint8_t* row = stash + k * kStashStride;
            constexpr uint32_t kHead = FILL ? kStashHead : (IPV4 ? 3u : 1u);
            if (lane < kHead && lane < P.s) *reinterpret_cast<u32x4*>(row + 16u * lane) = P.v[0];
            if (HYB && lane + P.s < kHead) *reinterpret_cast<u32x4*>(row + 16u * (lane + P.s)) = P.w;
            const uint32_t gu = static_cast<uint32_t>(U) * kWave;
            uint32_t g = gu;
            // long packets: kLongGroups groups of loads in flight per step;
            // the final group always goes through the single-group loop below
            // so P.v ends up holding it (tail stash)
            constexpr int kLG = (PIPE || MULTI) ? 2 : kLongGroups;  // leave registers for the second load set / shared passes
            for (; g + kLG * gu < P.s; g += kLG * gu) {
                u32x4 w[kLG][U];
#pragma unroll
                for (int q = 0; q < kLG; ++q)
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        w[q][u] = __builtin_amdgcn_raw_buffer_load_b128(
                            P.r, static_cast<int>(16u * (g + q * gu) + vo + 1024u * u), 0, AUX);
#pragma unroll
                for (int q = 0; q < kLG; ++q)
#pragma unroll
                    for (int u = 0; u < U; ++u) acc = sad4(w[q][u], acc);
            }
            for (; g < P.s; g += gu) {
                u32x4 w[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    w[u] = __builtin_amdgcn_raw_buffer_load_b128(P.r, static_cast<int>(16u * g + vo + 1024u * u), 0,
                                                                 AUX);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    acc = sad4(w[u], acc);
                    P.v[u] = w[u];
                }
            }
            // last unit of the span -> the row's last slot
            if (P.nu) {
                const uint32_t last = P.nu - 1;
                if (HYB) {
                    if (lane + P.s == last) *reinterpret_cast<u32x4*>(row + kStashLast) = P.w;
                } else {
                    const uint32_t slot = (last >> 6) % U;
                    u32x4 lu = P.v[0];
#pragma unroll
                    for (int u = 1; u < U; ++u) lu = slot == static_cast<uint32_t>(u) ? P.v[u] : lu;
                    if (lane == (last & 63u)) *reinterpret_cast<u32x4*>(row + kStashLast) = lu;
                }
            }
            const uint32_t S = wave_sum(acc);
            res = writelane(res, S, k, lane);
        };

        // MULTI: several short packets share one pass — NP packets x (64/NP)
        // lanes x U units; per-lane packet addresses come from the plan lanes by
        // ds_bpermute and 16-lane DPP row sums give one total per packet, so
        // the per-pass issue work is divided by NP.
        auto multi = [&](auto npc, uint32_t k) {
            constexpr uint32_t NP = decltype(npc)::value;
            constexpr uint32_t SL = kWave / NP;  // lanes per packet (32 or 16)
            constexpr uint32_t kHead = FILL ? kStashHead : (IPV4 ? 3u : 1u);
            const uint32_t seg = lane / SL, j = lane % SL;
            const int src = static_cast<int>(k + seg);
            const uint32_t qlo = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(a0)), src));
            const uint32_t qhi = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(a0 >> 32)), src));
            const uint32_t qnu = static_cast<uint32_t>(__shfl(static_cast<int>(nunits), src));
            const uint8_t* qa = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(qhi) << 32) | qlo);
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = j + SL * u;
                v[u] = u32x4{0, 0, 0, 0};
                if (c < qnu) v[u] = load_unit(qa + 16u * c);
            }
            uint32_t acc = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) acc = sad4(v[u], acc);
            uint8_t* row = stash + static_cast<uint32_t>(src) * kStashStride;
            if (j < kHead) *reinterpret_cast<u32x4*>(row + 16u * j) = v[0];
            if (qnu) {
                const uint32_t last = qnu - 1;
                u32x4 lu = v[0];
#pragma unroll
                for (int u = 1; u < U; ++u) lu = last / SL == static_cast<uint32_t>(u) ? v[u] : lu;
                if (j == last % SL) *reinterpret_cast<u32x4*>(row + kStashLast) = lu;
            }
            // 16-lane row sums
            acc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(acc), 0xB1, 0xF, 0xF, false));
            acc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(acc), 0x4E, 0xF, 0xF, false));
            acc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(acc), 0x124, 0xF, 0xF, false));
            acc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(acc), 0x128, 0xF, 0xF, false));
            const uint32_t r0 = __builtin_amdgcn_readlane(acc, 0), r1 = __builtin_amdgcn_readlane(acc, 16);
            const uint32_t r2 = __builtin_amdgcn_readlane(acc, 32), r3 = __builtin_amdgcn_readlane(acc, 48);
            if (NP == 4) {
                res = writelane(res, r0, k, lane);
                res = writelane(res, r1, k + 1, lane);
                res = writelane(res, r2, k + 2, lane);
                res = writelane(res, r3, k + 3, lane);
            } else {
                res = writelane(res, r0 + r1, k, lane);
                res = writelane(res, r2 + r3, k + 1, lane);
            }
        };

        if (MULTI) {
            const uint64_t quad_ok = __ballot(nunits <= 16u * U);
            const uint64_t pair_ok = __ballot(nunits <= 32u * U);
            uint32_t k = 0;
            while (k < cnt) {
                if (k + 4 <= cnt && ((quad_ok >> k) & 0xFull) == 0xFull) {
                    multi(std::integral_constant<uint32_t, 4>{}, k);
                    k += 4;
                } else if (k + 2 <= cnt && ((pair_ok >> k) & 0x3ull) == 0x3ull) {
                    multi(std::integral_constant<uint32_t, 2>{}, k);
                    k += 2;
                } else {
                    PktLoad P;
                    issue(k, true, P);
                    body(k, P);
                    k += 1;
                }
            }
        } else if (!PIPE) {
            for (uint32_t k = 0; k < cnt; ++k) {
                PktLoad P;
                issue(k, true, P);
                body(k, P);
            }
        } else {
            // ping-pong: packet k+1's loads are in flight while packet k is
            // summed; two named load sets, no register copies (copying an
            // in-flight load's destination would force a full vmcnt(0) wait)
            PktLoad PA, PB;
            issue(0, true, PA);
            for (uint32_t k = 0; k < cnt; k += 2) {
                const bool m1 = k + 1 < cnt;
                issue(m1 ? k + 1 : k, m1, PB);
                body(k, PA);
                const bool m2 = k + 2 < cnt;
                issue(m2 ? k + 2 : k, m2, PA);
                if (m1) body(k + 1, PB);
            }
        }
        if (IPV4 && huge && mine && !range_bad) {  // not streamed (phase D redoes its sum): head units from the frame
            constexpr uint32_t kHeadH = FILL ? kStashHead : 3u;
            uint8_t* hrow = stash + lane * kStashStride;
            const auto* hu = reinterpret_cast<const u32x4*>(a0);
#pragma unroll
            for (uint32_t j = 0; j < kHeadH; ++j) *reinterpret_cast<u32x4*>(hrow + 16u * j) = hu[j];
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): stash writes visible to this wave's reads
        __builtin_amdgcn_wave_barrier();

        // ---- C: lane i finishes packet i
        const int rs0 = static_cast<int>(head) + (IPV4 ? 20 : 0);
        const int re0 = static_cast<int>(head + L);
        const uint8_t* row = stash + lane * kStashStride;
        const u32x4 s0 = *reinterpret_cast<const u32x4*>(row);
        const u32x4 s1 = *reinterpret_cast<const u32x4*>(row + 16);
        const u32x4 s2 = *reinterpret_cast<const u32x4*>(row + 32);
        const u32x4 s3 = *reinterpret_cast<const u32x4*>(row + kStashLast);
        const int lastu16 = 16 * (static_cast<int>(nunits) - 1);
        uint32_t excl = unit_part(s0, 0, rs0);
        if (IPV4) {
            excl += unit_part(s1, 0, rs0 - 16) + unit_part(s2, 0, rs0 - 32);
        }
        excl += unit_part(s3, re0 - lastu16, 16);
        // a unit that is both a head unit and the last one is excluded twice,
        // but on disjoint byte ranges ([0, rs) and [re, 16)).
        const uint32_t kept = nunits ? res - excl : 0u;
        uint32_t S = fold16(kept);
        if (head & 1u) S = swap16(S);
        uint32_t word = 0, st = 0;
        bool slow = huge && mine && !range_bad;
        uint32_t ipc = 0, pseudo = 0;
        uint32_t fpos = 0;  // fill: the L4 checksum field's byte offset from a0 (0 = no field to store)
        int srs = 0, sre = 0;
        if (IPV4) {
            // header dwords at byte `head` of the stash row
            const uint32_t* hw = reinterpret_cast<const uint32_t*>(row + (head & ~3u));
            const uint32_t sh = head & 3u;
            const uint32_t d0 = hw[0], d1 = hw[1], d2 = hw[2], d3 = hw[3], d4 = hw[4], d5 = hw[5];
            const uint32_t h0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t h1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            const uint32_t h2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
            const uint32_t h3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
            const uint32_t h4 = __builtin_amdgcn_alignbyte(d5, d4, sh);
            // generate (fill) treats the header checksum field (bytes 10-11) as zero (ip.cc:270-276)
            ipc = ~fold16(static_cast<uint64_t>(h0) + h1 + (fill ? h2 & 0xffffu : h2) + h3 + h4) & 0xffffu;
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
            pseudo = fold16(static_cast<uint64_t>(h3 & 0xffffu) + (h3 >> 16) + (h4 & 0xffffu) + (h4 >> 16) +
                            (proto << 8) + swap16(l4_len & 0xffffu));
            slow = slow || (fast && (ihl != 5u || ip_len != L));
            srs = static_cast<int>(head + l4_off);
            sre = srs + static_cast<int>(l4_len);
            if (fill) {
                // the L4 checksum field (UDP +6, udp.cc:184-195; TCP +16, tcp.hh:283-285) counts as
                // zero: subtract its current value (ones' complement: add ~field).  The pseudo-header
                // is never zero, so the fold lands in [1, 0xffff] exactly like the reference's.
                const uint32_t fo = proto == 17u ? 6u : (proto == 6u ? 16u : 0u);
                const bool has_field = fo != 0u && l4_len >= fo + 2u && (st & SCCSUM_ST_MALFORMED) == 0u;
                fpos = has_field ? static_cast<uint32_t>(srs) + fo : 0u;
                uint32_t fv = 0;
                if (has_field && !slow) {  // ihl == 5 here: the field is inside head units 0..3
                    fv = static_cast<uint32_t>(row[fpos]) | (static_cast<uint32_t>(row[fpos + 1]) << 8);
                }
                const uint32_t r = ~fold16(static_cast<uint64_t>(S) + pseudo + (~fv & 0xffffu)) & 0xffffu;
                word = (fill_ip ? ipc : 0u) | (has_field ? r << 16 : 0u);
                st |= (fill_ip ? SCCSUM_ST_OK : 0u) | (has_field ? SCCSUM_ST_L4_OK : 0u);
            } else {
                const uint32_t r = ~fold16(static_cast<uint64_t>(S) + pseudo) & 0xffffu;
                word = ipc | (r << 16);
                st |= (ipc == 0 ? SCCSUM_ST_OK : 0u) | (r == 0 ? SCCSUM_ST_L4_OK : 0u);
            }
        } else {
            const uint32_t r = raw ? S : ~fold16(static_cast<uint64_t>(S) + swap16(fold16(sd))) & 0xffffu;
            word = r;
            st = (!raw && r == 0) ? SCCSUM_ST_OK : 0u;
        }
        if (range_bad) {
            word = 0;
            st = SCCSUM_ST_RANGE;
        } else if (short_frame) {
            word = 0;
            st = SCCSUM_ST_MALFORMED;
        }

        // ---- D: exact redo of the packets the fast path could not take
        uint64_t todo = __ballot(slow);
        while (todo) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint32_t jlo = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0), j);
            const uint32_t jhi = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0 >> 32), j);
            const uint8_t* ja0 = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(jhi) << 32) | jlo);
            const uint32_t jhead = __builtin_amdgcn_readlane(head, j);
            uint64_t rs, re;
            if (IPV4) {
                rs = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(srs), j));
                re = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(sre), j));
            } else {
                rs = jhead;
                re = static_cast<uint64_t>(jhead) + static_cast<uint32_t>(__builtin_amdgcn_readlane(L, j));
            }
            uint32_t SJ = exact_range_sum(ja0, rs, re, lane);
            if (jhead & 1u) SJ = swap16(SJ);
            if (lane == j) {
                if (IPV4 && fill) {
                    if (fpos) {
                        const uint8_t* fp = reinterpret_cast<const uint8_t*>(a0) + fpos;
                        const uint32_t fv = static_cast<uint32_t>(fp[0]) | (static_cast<uint32_t>(fp[1]) << 8);
                        const uint32_t r = ~fold16(static_cast<uint64_t>(SJ) + pseudo + (~fv & 0xffffu)) & 0xffffu;
                        word = (word & 0xffffu) | (r << 16);
                    }
                } else if (IPV4) {
                    const uint32_t r = ~fold16(static_cast<uint64_t>(SJ) + pseudo) & 0xffffu;
                    word = ipc | (r << 16);
                    st = (st & ~SCCSUM_ST_L4_OK) | (r == 0 ? SCCSUM_ST_L4_OK : 0u);
                } else {
                    const uint32_t r = raw ? SJ : ~fold16(static_cast<uint64_t>(SJ) + swap16(fold16(sd))) & 0xffffu;
                    word = r;
                    st = (!raw && r == 0) ? SCCSUM_ST_OK : 0u;
                }
            }
        }

        if (fill && mine && !range_bad && !short_frame) {
            // in-place write-back: wire-ready frames (network-order bytes = the LE store of the sum).
            // ~1 M scattered 2-byte stores per 1.5 GB batch cost ~75 us on top of the read stream
            // whatever their form (byte, nontemporal, full 64-byte blocks, a separate pass): HBM
            // read/write turnarounds, DESIGN.md §5.5.
            uint8_t* wp = reinterpret_cast<uint8_t*>(a0);
            if (fill_ip) {
                wp[head + 10] = static_cast<uint8_t>(word);
                wp[head + 11] = static_cast<uint8_t>(word >> 8);
            }
            if (fpos) {
                wp[fpos] = static_cast<uint8_t>(word >> 16);
                wp[fpos + 1] = static_cast<uint8_t>(word >> 24);
            }
        }
        if (mine) {
            if (IPV4) {
                if (out) reinterpret_cast<uint32_t*>(out)[base + lane] = word;
            } else {
                out[base + lane] = static_cast<uint16_t>(word);
            }
            if (status) status[base + lane] = static_cast<uint8_t>(st);
        }
        __builtin_amdgcn_wave_barrier();  // stash rows are rewritten by the next tile
        t = t_next;
    }
}

// ---------------------------------------------------------------- RSS (Toeplitz)

// toeplitz_hash (include/seastar/net/toeplitz.hh:78-98) XORs, for every set
// data bit j (MSB first), the 32-bit key window that starts at key bit j; key
// bits past key_len read as 0.  The host precomputes the 96 windows a 12-byte
// IPv4 forward_hash can touch, so a lane's hash is 96 select-XORs, and a
// datagram without ports hashes its 8 IP bytes by zeroing the port word.
struct RssParams {
    uint32_t* hash;  // per-frame output (nullptr: no RSS)
    uint32_t mode;   // SCCSUM_RSS_DISPATCH / SCCSUM_RSS_REASSEMBLED
    uint32_t w[96];  // key window at data bit j
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t toeplitz96(const RssParams& P, uint32_t d0, uint32_t d1, uint32_t d2) {
    uint32_t h = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        h ^= (d0 & (0x80000000u >> j)) ? P.w[j] : 0u;
        h ^= (d1 & (0x80000000u >> j)) ? P.w[32 + j] : 0u;
        h ^= (d2 & (0x80000000u >> j)) ? P.w[64 + j] : 0u;
    }
    return h;
}

// The forward_hash of one IPv4 frame (net.hh:53-75, bytes in wire order):
// h0..h4 = the header's dwords as loaded (little-endian), ports20 = the dword
// at frame byte 20, ports_l4 = the dword at 4*ihl (REASSEMBLED only).
//  DISPATCH (net.cc:330-341 -> ip.cc:77-92): src, dst; then for an atomic
//    datagram (MF clear, offset 0, ip.cc:87) of TCP (tcp.hh:852-862, 20 B
//    header) or UDP (udp.cc:153-161, 8 B) the port bytes at +20
//    (sizeof(ip_hdr): options are not skipped), if the frame holds them.
//  REASSEMBLED (ip.cc:186-197): src, dst; then the ports at 4*ihl when the
//    L4 part, up to min(ip_len, len), holds the TCP / UDP header.
// Returns false (hash 0) for a malformed frame: shorter than 20 B, or (mode 1)
// 4*ihl past the end of the datagram.
__device__ __forceinline__ bool rss_ipv4(const RssParams& P, uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                         uint32_t h4, uint32_t ports20, uint32_t ports_l4, uint32_t L,
                                         uint32_t& hash) {
    const uint32_t proto = (h2 >> 8) & 0xffu;
    const uint32_t need = proto == 6u ? 20u : (proto == 17u ? 8u : 0u);
    uint32_t ports = 0;
    if (P.mode == SCCSUM_RSS_DISPATCH) {
        const uint32_t frag = swap16(h1 >> 16);  // flags + fragment offset (ip.hh:390-391)
        if (need && (frag & 0x3fffu) == 0u && L >= 20u + need) ports = ports20;
    } else {
        const uint32_t l4_off = 4u * (h0 & 0xfu);
        const uint32_t ip_len = swap16(h0 >> 16);
        const uint32_t l4_end = ip_len < L ? ip_len : L;
        if (l4_off > l4_end) {
            hash = 0;
            return false;
        }
        if (need && l4_end - l4_off >= need) ports = ports_l4;
    }
    hash = toeplitz96(P, bswap32(h3), bswap32(h4), bswap32(ports));
    return true;
}

// Standalone RSS over a frame batch: one thread per frame, header dwords
// loaded aligned and re-aligned with v_alignbyte (frames at any offset; the
// buffer is readable to round16(bytes_len)).
__global__ __launch_bounds__(kBlock) void rss_kernel(const uint8_t* __restrict__ bytes, uint64_t bytes_len,
                                                     const uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ len, uint8_t* __restrict__ status,
                                                     uint64_t n, const RssParams P) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint32_t L = len[i];
    uint32_t hash = 0, st = 0;
    if (o > bytes_len || L > bytes_len - o) {
        st = SCCSUM_ST_RANGE;
    } else if (L < 20u) {
        st = SCCSUM_ST_MALFORMED;
    } else {
        const uint8_t* p = bytes + o;
        const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3u);
        const uint64_t padded = (bytes_len + 15u) & ~uint64_t(15);  // readable extent of the buffer
        auto dword_at = [&](uint64_t byte_off) -> uint32_t {          // aligned dword at bytes + byte_off
            return byte_off + 4u <= padded ? *reinterpret_cast<const uint32_t*>(bytes + byte_off) : 0u;
        };
        uint32_t d[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = dword_at(o - sh + 4u * k);  // bytes [-sh, 28 - sh) of the frame
        const uint32_t h0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh), h1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
        const uint32_t h2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh), h3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
        const uint32_t h4 = __builtin_amdgcn_alignbyte(d[5], d[4], sh), h5 = __builtin_amdgcn_alignbyte(d[6], d[5], sh);
        uint32_t pl = h5;
        const uint32_t l4_off = 4u * (h0 & 0xfu);
        if (P.mode != SCCSUM_RSS_DISPATCH && l4_off != 20u && l4_off + 4u <= L) {
            const uint64_t q = o + l4_off - sh;
            pl = __builtin_amdgcn_alignbyte(dword_at(q + 4u), dword_at(q), sh);
        }
        if (!rss_ipv4(P, h0, h1, h2, h3, h4, h5, pl, L, hash)) st = SCCSUM_ST_MALFORMED;
    }
    P.hash[i] = hash;
    if (status) status[i] = static_cast<uint8_t>(st);
}

// ---------------------------------------------------------------- flat kernel

// Inclusive prefix sums over the 64 lanes: Hillis-Steele row scans by
// row_shr 1/2/4/8 (zero fill at the row edge), then row_bcast 15/31 carry the
// row totals into rows 1-3 (gfx9 DPP; six v_add_u32_dpp per value).
// tools/dev/scan_check.hip checks the sequence lane by lane on the device.
// U independent scans, step-interleaved so that no DPP op
// reads the result of the instruction just before it (no hazard nops).
template <int U>
__device__ __forceinline__ void wave_scan_n(uint32_t (&x)[U]) {
#define SCCSUM_SCAN_STEP(ctrl, rm, bm)                                                                          \
    _Pragma("unroll") for (int u = 0; u < U; ++u) x[u] +=                                                       \
        static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x[u]), ctrl, rm, bm, true));
    SCCSUM_SCAN_STEP(0x111, 0xF, 0xF)
    SCCSUM_SCAN_STEP(0x112, 0xF, 0xF)
    SCCSUM_SCAN_STEP(0x114, 0xF, 0xF)
    SCCSUM_SCAN_STEP(0x118, 0xF, 0xF)
    SCCSUM_SCAN_STEP(0x142, 0xA, 0xF)
    SCCSUM_SCAN_STEP(0x143, 0xC, 0xF)
#undef SCCSUM_SCAN_STEP
}

// Dword i of the 64 bytes held in four units.
__device__ __forceinline__ uint32_t unit_dword(const u32x4 (&h)[4], int i) {
    const u32x4& u = h[i >> 2];
    return (i & 3) == 0 ? u.x : (i & 3) == 1 ? u.y : (i & 3) == 2 ? u.z : u.w;
}

// The dword at byte `head + 4 i` of the four units (head < 16): a 4-way
// select on head / 4 and a byte funnel shift.
__device__ __forceinline__ uint32_t header_dword(const u32x4 (&h)[4], uint32_t head, int i) {
    const uint32_t q = head >> 2;
    auto pick = [&](int j) {
        const uint32_t a = unit_dword(h, j), b = unit_dword(h, j + 1), c = unit_dword(h, j + 2),
                       d = unit_dword(h, j + 3);
        return q == 0 ? a : q == 1 ? b : q == 2 ? c : d;
    };
    return __builtin_amdgcn_alignbyte(pick(i + 1), pick(i), head & 3u);
}

constexpr int kGapUnits = 4;  // flat runs tolerate gaps of up to 4 units (64 B) between packets

// Flat kernel.  Same tiles, tile order and outputs as csum_batch_kernel, but
// the bytes are streamed per RUN instead of per packet: a run is a maximal
// sequence of tile packets whose 16-byte unit spans go forward with gaps of
// at most kGapUnits (packed batches: the whole tile).  The wave reads the
// run's unit extent densely — U units per lane per chunk, no empty lane
// loads whatever the packet sizes — sums each unit (v_sad_u16), takes a
// wave-wide inclusive prefix scan of the unit sums (DPP) and parks the chunk's
// prefix values and units in LDS; every packet lane then picks up the prefix
// just before its first unit and at its last unit, plus the units the
// finishing step needs (the first 1/3/4 units, the last), when they pass.  A
// packet's sum of units is the difference of its two prefix values (exact
// mod 2^32; sums stay below 2^32 up to kExactMax bytes), after which the
// finishing step is the batch kernel's (edge bytes, IPv4 header,
// pseudo-header, exact redo of the packets the fast path cannot take).
// Layouts that do not run forward (shuffled offsets) degrade to one run per
// packet — the per-packet cost of the batch kernel.
template <int U, bool IPV4, bool FILL, bool PIPE>
__global__ __launch_bounds__(kBlock) void csum_flat_kernel(
    const uint8_t* __restrict__ bytes, uint64_t bytes_len,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
    const uint32_t* __restrict__ seed, uint16_t* __restrict__ out,
    uint8_t* __restrict__ status, uint64_t n, uint32_t B, uint32_t B2, uint64_t T1, uint32_t* __restrict__ heads,
    uint32_t flags, const RssParams rss) {
    static_assert(!FILL || IPV4, "in-place generate is a frames mode");
    constexpr uint32_t C = kWave * U;  // units per chunk
    constexpr int kHead = FILL ? 4 : (IPV4 ? 3 : 1);
    const bool raw = !IPV4 && (flags & kFlagRaw);
    const bool fill_ip = FILL && (flags & kFlagFillIp);
    __shared__ u32x4 ubuf_all[kWavesPerBlock][C];
    __shared__ uint32_t pbuf_all[kWavesPerBlock][C];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    u32x4* ubuf = ubuf_all[wv];
    uint32_t* pbuf = pbuf_all[wv];
    const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
    // guided tiles: T1 tiles of B packets, then tiles of B2 (< B) packets, so
    // the dequeue's last draws are short and the launch ends evenly
    const uint64_t big = T1 * B;
    const uint64_t ntiles = T1 + (n - big + B2 - 1) / B2;
    const bool has_seed = !IPV4 && seed != nullptr;
    const uint32_t vo = 16u * lane;

    // tile order: as csum_batch_kernel (static first tile, then dequeued)
    const uint64_t wglob = static_cast<uint64_t>(xcd_block_id()) * kWavesPerBlock + wv;
    const uint32_t grp = static_cast<uint32_t>(wglob % kGroups);
    const uint64_t rest = ntiles > nwaves ? ntiles - nwaves : 0;
    const uint32_t tiles_g = rest > grp ? static_cast<uint32_t>((rest - grp + kGroups - 1) / kGroups) : 0u;
    const uint32_t waves_g = static_cast<uint32_t>(nwaves / kGroups);
    auto next_tile = [&](uint64_t prev) -> uint64_t {
        if (heads == nullptr) return prev + nwaves;
        uint32_t d = 0;
        if (lane == 0) {
            uint32_t* h = heads + grp * kHeadStride;
            d = __hip_atomic_fetch_add(h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == tiles_g + waves_g - 1) __hip_atomic_store(h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        d = __builtin_amdgcn_readfirstlane(d);
        return d < tiles_g ? nwaves + grp + static_cast<uint64_t>(kGroups) * d : ntiles;
    };
    auto tile_base = [&](uint64_t tt) { return tt < T1 ? tt * B : big + (tt - T1) * B2; };
    // Two-deep tile pipeline: while tile t streams, the plan (offset, length,
    // seed) of the next tile is already loading and the tile after it is being
    // dequeued, so no tile starts on an exposed metadata or atomic round trip.
    // Every wave still makes exactly one failing dequeue (the counter reset
    // relies on it).
    uint64_t t = wglob;
    if (t >= ntiles && heads != nullptr) t = next_tile(t);
    uint64_t t1 = t < ntiles ? next_tile(t) : ntiles;
    auto plan_load = [&](uint64_t tt, uint64_t& o_, uint32_t& L_, uint32_t& sd_) {
        const uint64_t b_ = tile_base(tt < ntiles ? tt : 0);
        const uint32_t bb = tt < T1 ? B : B2;
        const uint32_t c_ = tt < ntiles ? static_cast<uint32_t>(n - b_ < bb ? n - b_ : bb) : 0u;
        const uint64_t q_ = b_ + (lane < c_ ? lane : 0);
        o_ = off[q_];
        L_ = lane < c_ ? len[q_] : 0u;
        sd_ = has_seed ? seed[q_] : 0u;
    };
    // ---- A: a tile's per-lane packet plan and its runs: lane j starts a new
    // run unless packet j-1 and j both take part and j's span starts at most
    // kGapUnits past j-1's end and ends no earlier (so a run's extent is
    // [fu of its first, lu of its last])
    struct Tile {
        uint64_t base, o, a0, fu, lu, starts, streamed;
        uint32_t cnt, L, sd, head, nunits;
        bool mine, range_bad, short_frame, huge, fast, part;
    };
    auto derive = [&](uint64_t tt, uint64_t o_, uint32_t L_, uint32_t sd_) {
        Tile c;
        c.base = tile_base(tt);
        const uint32_t bt = tt < T1 ? B : B2;
        const uint64_t left = n - c.base;
        c.cnt = left < bt ? static_cast<uint32_t>(left) : bt;
        c.mine = lane < c.cnt;
        c.o = o_;
        c.L = L_;
        c.sd = sd_;
        c.range_bad = c.o > bytes_len || c.L > bytes_len - c.o;
        c.short_frame = IPV4 && c.L < 20;
        c.huge = c.L > kExactMax;
        const uint8_t* ptr = bytes + (c.range_bad ? 0 : c.o);
        c.head = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ptr) & 15u);
        c.a0 = reinterpret_cast<uint64_t>(ptr - c.head);
        c.fast = c.mine && !c.range_bad && !c.short_frame && !c.huge;
        c.nunits = (c.fast && c.L) ? (c.head + c.L + 15u) >> 4 : 0u;
        c.part = c.nunits != 0;
        c.fu = c.a0 >> 4;
        c.lu = c.fu + c.nunits - 1;
        const int pl = static_cast<int>(lane == 0 ? 0 : lane - 1);
        const uint64_t pfu =
            (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(c.fu >> 32), pl))) << 32) |
            static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(c.fu)), pl));
        const uint64_t plu =
            (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(c.lu >> 32), pl))) << 32) |
            static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(c.lu)), pl));
        const bool ppart = __shfl(static_cast<int>(c.part), pl) != 0;
        const bool joins = lane != 0 && c.part && ppart && c.fu >= pfu && c.lu >= plu && c.fu <= plu + kGapUnits;
        c.starts = __ballot(c.mine && !joins) | (c.cnt < 64 ? (1ull << c.cnt) : 0ull);
        c.streamed = c.starts & __ballot(c.part);  // runs that stream bytes start at a lane that takes part
        return c;
    };
    // Run [k, k2) of tile c: its extent's first unit F and unit count.
    struct Run {
        uint32_t k, k2, ext;
        uint64_t F;
    };
    auto run_of = [&](const Tile& c, uint32_t k) {
        Run rn;
        rn.k = k;
        const uint64_t after = c.starts & ~((2ull << k) - 1ull);  // k < 64; bit cnt is the sentinel
        rn.k2 = after ? static_cast<uint32_t>(__builtin_ctzll(after)) : c.cnt;
        // (readlane returns int: widen through uint32_t, never sign-extend an address half)
        const uint32_t Fhi = __builtin_amdgcn_readlane(static_cast<uint32_t>(c.fu >> 32), k);
        const uint32_t Flo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c.fu), k);
        rn.F = (static_cast<uint64_t>(Fhi) << 32) | Flo;
        const uint32_t Llo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c.lu), rn.k2 - 1);
        rn.ext = Llo - static_cast<uint32_t>(rn.F) + 1u;  // units in the run's extent
        return rn;
    };
    auto run_rsrc = [&](const Run& rn) { return rsrc(reinterpret_cast<const uint8_t*>(rn.F << 4), 16u * rn.ext); };
    auto load = [&](const __amdgpu_buffer_rsrc_t& r, uint32_t g, u32x4 (&v)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(16u * g + vo + 1024u * u), 0, kNT);
    };

    uint64_t o_n = 0;
    uint32_t L_n = 0, sd_n = 0;
    plan_load(t, o_n, L_n, sd_n);
    Tile cur{};
    while (t < ntiles) {
        const uint64_t t2 = t1 < ntiles ? next_tile(t1) : ntiles;
        cur = derive(t, o_n, L_n, sd_n);
        if (t1 < ntiles) plan_load(t1, o_n, L_n, sd_n);
        const uint64_t base = cur.base;
        const bool mine = cur.mine;
        const uint32_t L = cur.L, sd = cur.sd, head = cur.head, nunits = cur.nunits;
        const uint64_t a0 = cur.a0;
        const bool range_bad = cur.range_bad, short_frame = cur.short_frame, huge = cur.huge, fast = cur.fast;

        // ---- B: stream each run's extent
        u32x4 hs[4] = {u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}};
        u32x4 hl = u32x4{0, 0, 0, 0};
        uint32_t pst = 0, pend = 0;
        uint64_t rem = cur.streamed;
        while (rem != 0) {
            const Run rn = run_of(cur, static_cast<uint32_t>(__builtin_ctzll(rem)));
            rem &= rem - 1;
            const uint32_t k = rn.k, k2 = rn.k2, ext = rn.ext;
            const uint64_t F = rn.F;
            const auto r = run_rsrc(rn);
            const bool cap = lane >= k && lane < k2;
            const int rf = cap ? static_cast<int>(static_cast<uint32_t>(cur.fu - F)) : -0x40000000;
            const int rl = cap ? static_cast<int>(static_cast<uint32_t>(cur.lu - F)) : -0x40000000;
            uint32_t carry = 0;
            // one chunk = U rows of 64 units: unit sums, scanned, parked in
            // LDS with the units; packet lanes pick up what falls in it
            auto chunk = [&](uint32_t g, const u32x4 (&v)[U]) {
                uint32_t x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = sad4(v[u], 0u);
                wave_scan_n<U>(x);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    pbuf[kWave * u + lane] = carry + x[u];
                    ubuf[kWave * u + lane] = v[u];
                    carry += __builtin_amdgcn_readlane(x[u], 63);
                }
                __builtin_amdgcn_wave_barrier();
                const int a = rf - static_cast<int>(g);
                if (static_cast<uint32_t>(a) < C) {
                    const u32x4 w = ubuf[a];
                    pst = pbuf[a] - sad4(w, 0u);  // prefix just before the first unit
                    hs[0] = w;
                }
#pragma unroll
                for (int j = 1; j < kHead; ++j) {
                    if (static_cast<uint32_t>(a + j) < C) hs[j] = ubuf[a + j];
                }
                const int b = rl - static_cast<int>(g);
                if (static_cast<uint32_t>(b) < C) {
                    pend = pbuf[b];
                    hl = ubuf[b];
                }
                __builtin_amdgcn_wave_barrier();  // this chunk's LDS reads precede the next chunk's writes
            };
            if (PIPE) {
                u32x4 va[U], vb[U];
                load(r, 0, va);
                for (uint32_t g = 0; g < ext; g += 2 * C) {
                    load(r, g + C, vb);
                    chunk(g, va);
                    load(r, g + 2 * C, va);
                    chunk(g + C, vb);
                }
            } else {
                for (uint32_t g = 0; g < ext; g += C) {
                    u32x4 v[U];
                    load(r, g, v);
                    chunk(g, v);
                }
            }
        }
        const uint32_t res = pend - pst;  // sum of the packet's units, mod 2^32
        if (IPV4 && huge && mine && !range_bad) {  // not streamed (phase D redoes its sum): head units from the frame
            const auto* hu = reinterpret_cast<const u32x4*>(a0);
#pragma unroll
            for (int j = 0; j < kHead; ++j) hs[j] = hu[j];
        }

        // ---- C: lane i finishes packet i (as csum_batch_kernel, stash in registers)
        const int rs0 = static_cast<int>(head) + (IPV4 ? 20 : 0);
        const int re0 = static_cast<int>(head + L);
        const int lastu16 = 16 * (static_cast<int>(nunits) - 1);
        uint32_t excl = unit_part(hs[0], 0, rs0);
        if (IPV4) excl += unit_part(hs[1], 0, rs0 - 16) + unit_part(hs[2], 0, rs0 - 32);
        excl += unit_part(hl, re0 - lastu16, 16);
        const uint32_t kept = nunits ? res - excl : 0u;
        uint32_t S = fold16(kept);
        if (head & 1u) S = swap16(S);
        uint32_t word = 0, st = 0;
        bool slow = huge && mine && !range_bad;
        uint32_t ipc = 0, pseudo = 0, fpos = 0;
        int srs = 0, sre = 0;
        if (IPV4) {
            const uint32_t h0 = header_dword(hs, head, 0), h1 = header_dword(hs, head, 1);
            const uint32_t h2 = header_dword(hs, head, 2), h3 = header_dword(hs, head, 3);
            const uint32_t h4 = header_dword(hs, head, 4);
            ipc = ~fold16(static_cast<uint64_t>(h0) + h1 + (FILL ? h2 & 0xffffu : h2) + h3 + h4) & 0xffffu;
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
            pseudo = fold16(static_cast<uint64_t>(h3 & 0xffffu) + (h3 >> 16) + (h4 & 0xffffu) + (h4 >> 16) +
                            (proto << 8) + swap16(l4_len & 0xffffu));
            slow = slow || (fast && (ihl != 5u || ip_len != L));
            srs = static_cast<int>(head + l4_off);
            sre = srs + static_cast<int>(l4_len);
            if (rss.hash != nullptr) {  // fused RSS: the 4-tuple is already in registers
                const uint32_t h5 = header_dword(hs, head, 5);
                uint32_t pl = h5;
                if (rss.mode != SCCSUM_RSS_DISPATCH && ihl != 5u && l4_off + 4u <= L && mine && !range_bad) {
                    const uint8_t* q = reinterpret_cast<const uint8_t*>(a0) + head + l4_off;  // options: rare
                    pl = static_cast<uint32_t>(q[0]) | (static_cast<uint32_t>(q[1]) << 8) |
                         (static_cast<uint32_t>(q[2]) << 16) | (static_cast<uint32_t>(q[3]) << 24);
                }
                uint32_t hv = 0;
                rss_ipv4(rss, h0, h1, h2, h3, h4, h5, pl, L, hv);
                if (mine) rss.hash[base + lane] = (range_bad || short_frame) ? 0u : hv;
            }
            if (FILL) {
                const uint32_t fo = proto == 17u ? 6u : (proto == 6u ? 16u : 0u);
                const bool has_field = fo != 0u && l4_len >= fo + 2u && (st & SCCSUM_ST_MALFORMED) == 0u;
                fpos = has_field ? static_cast<uint32_t>(srs) + fo : 0u;
                uint32_t fv = 0;
                if (has_field && !slow) {  // ihl == 5: frame bytes 26-27 (UDP) / 36-37 (TCP)
                    fv = fo == 6u ? header_dword(hs, head, 6) >> 16 : header_dword(hs, head, 9) & 0xffffu;
                }
                const uint32_t rr = ~fold16(static_cast<uint64_t>(S) + pseudo + (~fv & 0xffffu)) & 0xffffu;
                word = (fill_ip ? ipc : 0u) | (has_field ? rr << 16 : 0u);
                st |= (fill_ip ? SCCSUM_ST_OK : 0u) | (has_field ? SCCSUM_ST_L4_OK : 0u);
            } else {
                const uint32_t rr = ~fold16(static_cast<uint64_t>(S) + pseudo) & 0xffffu;
                word = ipc | (rr << 16);
                st |= (ipc == 0 ? SCCSUM_ST_OK : 0u) | (rr == 0 ? SCCSUM_ST_L4_OK : 0u);
            }
        } else {
            const uint32_t rr = raw ? S : ~fold16(static_cast<uint64_t>(S) + swap16(fold16(sd))) & 0xffffu;
            word = rr;
            st = (!raw && rr == 0) ? SCCSUM_ST_OK : 0u;
        }
        if (range_bad) {
            word = 0;
            st = SCCSUM_ST_RANGE;
        } else if (short_frame) {
            word = 0;
            st = SCCSUM_ST_MALFORMED;
        }

        // ---- D: exact redo of the packets the fast path could not take
        uint64_t todo = __ballot(slow);
        while (todo) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint32_t jlo = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0), j);
            const uint32_t jhi = __builtin_amdgcn_readlane(static_cast<uint32_t>(a0 >> 32), j);
            const uint8_t* ja0 = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(jhi) << 32) | jlo);
            const uint32_t jhead = __builtin_amdgcn_readlane(head, j);
            uint64_t rs, re;
            if (IPV4) {
                rs = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(srs), j));
                re = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(sre), j));
            } else {
                rs = jhead;
                re = static_cast<uint64_t>(jhead) + static_cast<uint32_t>(__builtin_amdgcn_readlane(L, j));
            }
            uint32_t SJ = exact_range_sum(ja0, rs, re, lane);
            if (jhead & 1u) SJ = swap16(SJ);
            if (lane == j) {
                if (IPV4 && FILL) {
                    if (fpos) {
                        const uint8_t* fp = reinterpret_cast<const uint8_t*>(a0) + fpos;
                        const uint32_t fv = static_cast<uint32_t>(fp[0]) | (static_cast<uint32_t>(fp[1]) << 8);
                        const uint32_t rr = ~fold16(static_cast<uint64_t>(SJ) + pseudo + (~fv & 0xffffu)) & 0xffffu;
                        word = (word & 0xffffu) | (rr << 16);
                    }
                } else if (IPV4) {
                    const uint32_t rr = ~fold16(static_cast<uint64_t>(SJ) + pseudo) & 0xffffu;
                    word = ipc | (rr << 16);
                    st = (st & ~SCCSUM_ST_L4_OK) | (rr == 0 ? SCCSUM_ST_L4_OK : 0u);
                } else {
                    const uint32_t rr = raw ? SJ : ~fold16(static_cast<uint64_t>(SJ) + swap16(fold16(sd))) & 0xffffu;
                    word = rr;
                    st = (!raw && rr == 0) ? SCCSUM_ST_OK : 0u;
                }
            }
        }

        if (FILL && mine && !range_bad && !short_frame) {
            uint8_t* wp = reinterpret_cast<uint8_t*>(a0);
            if (fill_ip) {
                wp[head + 10] = static_cast<uint8_t>(word);
                wp[head + 11] = static_cast<uint8_t>(word >> 8);
            }
            if (fpos) {
                wp[fpos] = static_cast<uint8_t>(word >> 16);
                wp[fpos + 1] = static_cast<uint8_t>(word >> 24);
            }
        }
        if (mine) {
            if (IPV4) {
                if (out) reinterpret_cast<uint32_t*>(out)[base + lane] = word;
            } else {
                out[base + lane] = static_cast<uint16_t>(word);
            }
            if (status) status[base + lane] = static_cast<uint8_t>(st);
        }
        t = t1;
        t1 = t2;
    }
}

// Fragment lists (checksummer::sum(const packet&), src/net/ip_checksum.cc:64-68):
// stage 1 = the span kernel in raw mode gives every fragment's folded sum
// relative to the fragment's own start; here one thread per packet walks its
// fragments in order and byte-swaps each sum whose fragment starts at an odd
// packet-relative offset — the reference's `odd` carry (ip_checksum.cc:33-36,
// 52) — then adds the seed and complements.
__global__ __launch_bounds__(kBlock) void frag_combine_kernel(const uint32_t* __restrict__ frag_len, uint64_t nfrag,
                                                               const uint32_t* __restrict__ pkt_first,
                                                               const uint16_t* __restrict__ raw,
                                                               const uint8_t* __restrict__ raw_status,
                                                               const uint32_t* __restrict__ seed,
                                                               uint16_t* __restrict__ out,
                                                               uint8_t* __restrict__ status, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t f0 = pkt_first[i], f1 = pkt_first[i + 1];
    bool bad = f1 < f0 || f1 > nfrag;
    uint64_t S = 0;
    uint32_t par = 0;
    for (uint64_t j = f0; !bad && j < f1; ++j) {
        const uint32_t t = raw[j];
        bad = (raw_status[j] & SCCSUM_ST_RANGE) != 0;
        S += par ? swap16(t) : t;
        par ^= frag_len[j] & 1u;
    }
    const uint32_t r = ~fold16(fold16(S) + static_cast<uint64_t>(swap16(fold16(seed ? seed[i] : 0u)))) & 0xffffu;
    out[i] = bad ? uint16_t(0) : static_cast<uint16_t>(r);
    if (status) status[i] = bad ? SCCSUM_ST_RANGE : (r == 0 ? SCCSUM_ST_OK : 0u);
}

// Header-only generate (no payload bytes read): the IPv4 header checksum
// (ip.cc:266-278) and/or the tx-offload partial that a NIC completes — the
// folded pseudo-header stored in the L4 field (udp.cc:188-189, tcp.hh:1688-1689,
// `~csum.get()` of the pseudo-header alone; TSO: length 0 for TCP).
// One thread per frame.
__global__ __launch_bounds__(kBlock) void fill_header_kernel(uint8_t* __restrict__ bytes, uint64_t bytes_len,
                                                             const uint64_t* __restrict__ off,
                                                             const uint32_t* __restrict__ len,
                                                             uint32_t* __restrict__ out2,
                                                             uint8_t* __restrict__ status, uint64_t n, uint32_t mode) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint32_t L = len[i];
    uint32_t word = 0, st = 0;
    if (o > bytes_len || L > bytes_len - o) {
        st = SCCSUM_ST_RANGE;
    } else if (L < 20u) {
        st = SCCSUM_ST_MALFORMED;
    } else {
        uint8_t* p = bytes + o;
        uint32_t h[10];  // little-endian 16-bit words of the 20-byte header
#pragma unroll
        for (int k = 0; k < 10; ++k) h[k] = static_cast<uint32_t>(p[2 * k]) | (static_cast<uint32_t>(p[2 * k + 1]) << 8);
        const uint32_t ihl = p[0] & 0xfu;
        const uint32_t ip_len = (static_cast<uint32_t>(p[2]) << 8) | p[3];
        const uint32_t proto = p[9];
        const uint32_t l4_off = 4u * ihl;
        const uint32_t l4_end = ip_len < L ? ip_len : L;
        uint32_t l4_len = 0;
        if (L < ip_len) st |= SCCSUM_ST_MALFORMED;
        if (l4_off > l4_end) {
            st |= SCCSUM_ST_MALFORMED;
        } else {
            l4_len = l4_end - l4_off;
        }
        if (mode & SCCSUM_FILL_IP) {
            const uint32_t ipc =
                ~fold16(static_cast<uint64_t>(h[0]) + h[1] + h[2] + h[3] + h[4] + h[6] + h[7] + h[8] + h[9]) & 0xffffu;
            p[10] = static_cast<uint8_t>(ipc);
            p[11] = static_cast<uint8_t>(ipc >> 8);
            word |= ipc;
            st |= SCCSUM_ST_OK;
        }
        if (mode & SCCSUM_FILL_L4_PSEUDO) {
            const uint32_t fo = proto == 17u ? 6u : (proto == 6u ? 16u : 0u);
            if (fo != 0u && l4_len >= fo + 2u && (st & SCCSUM_ST_MALFORMED) == 0u) {
                const uint32_t plen = ((mode & SCCSUM_FILL_TSO) && proto == 6u) ? 0u : l4_len;
                const uint32_t ps = fold16(static_cast<uint64_t>(h[6]) + h[7] + h[8] + h[9] + (proto << 8) +
                                           swap16(plen & 0xffffu));
                p[l4_off + fo] = static_cast<uint8_t>(ps);
                p[l4_off + fo + 1] = static_cast<uint8_t>(ps >> 8);
                word |= ps << 16;
                st |= SCCSUM_ST_L4_OK;
            }
        }
    }
    if (out2) out2[i] = word;
    if (status) status[i] = static_cast<uint8_t>(st);
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

std::atomic<int> g_blocks_per_cu{kBlocksPerCU};

unsigned grid_for(uint64_t n) {
    const uint64_t cap = static_cast<uint64_t>(cu_count()) * g_blocks_per_cu.load(std::memory_order_relaxed);
    uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    if (want > cap) want = cap;
    want = (want + 7) & ~uint64_t(7);  // multiple of 8 for the XCD mapping
    return static_cast<unsigned>(want);
}

std::atomic<int> g_group_units{0};  // diagnostic override of U (0 = by max_len)
std::atomic<int> g_tile_packets{kWave};  // max packets per batch-kernel tile
std::atomic<int> g_dynamic{1};           // batch kernel: dequeue tiles (1) or static round robin (0)

// Per-device ring of tile-head slots (kGroups heads, each on its own line),
// allocated and zeroed once in sccsum_init; each launch takes the next slot
// and leaves it zeroed again (the last dequeue of each group resets it), so
// launches need no memset and launches on different streams do not share
// counters (up to kHeadSlots launches in flight per device).
constexpr int kHeadSlots = 256;
uint32_t* g_heads[kMaxDevices];
std::atomic<uint32_t> g_head_next[kMaxDevices];

int ensure_heads(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return SCCSUM_ENODEV;
    if (g_heads[dev] != nullptr) return SCCSUM_OK;
    void* p = nullptr;
    const size_t bytes = size_t(kHeadSlots) * kHeadSlotWords * sizeof(uint32_t);
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return static_cast<int>(e);
    e = hipMemset(p, 0, bytes);  // once: from here on every launch leaves its slot zeroed
    if (e != hipSuccess) return static_cast<int>(e);
    g_heads[dev] = static_cast<uint32_t*>(p);
    return SCCSUM_OK;
}

uint32_t* next_heads() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices || g_heads[dev] == nullptr) return nullptr;
    const uint32_t slot = g_head_next[dev].fetch_add(1, std::memory_order_relaxed) % kHeadSlots;
    return g_heads[dev] + kHeadSlotWords * slot;
}

int units_class(uint32_t max_len) {
    const int forced = g_group_units.load(std::memory_order_relaxed);
    if (forced) return forced;
    if (max_len == 0) return 4;
    const uint64_t units = (static_cast<uint64_t>(max_len) + 30) / 16;  // worst-case head of 15
    if (units <= 64) return 1;
    if (units <= 128) return 2;
    if (units <= 256) return 4;
    return 8;
}

// Kernel variant: 0 = default (the flat kernel: 16 for batches of >= 512 Ki
// packets and >= 256 MiB, else 15), 10-16 = the flat kernel's forms (launch_u),
// 1 = simple one-packet-per-wave loop (independent second implementation),
// 2 = batch kernel, 3 = batch kernel with the next packet in flight (both
// with nontemporal loads), 4 / 5 = 2 / 3 with default-policy loads,
// 6 / 7 = 2 / 3 with each packet's last 128-byte line loaded default-policy,
// 8 / 9 = 2 / 6 with short packets sharing passes (4 x 16 or 2 x 32 lanes).
std::atomic<int> g_variant{0};

std::atomic<int> g_tile_bytes{0};  // flat kernel: target bytes per tile (0 = packets cap only)

// Flat-kernel launch: the grid is what the chip holds at once (the kernel's
// occupancy, from its VGPR and LDS use, capped by the blocks-per-CU knob), so
// every wave's static first tile starts at launch; tiles hold about
// g_tile_bytes of packets (mean length from bytes_len / n), capped at 64.
using FlatKernel = void (*)(const uint8_t*, uint64_t, const uint64_t*, const uint32_t*, const uint32_t*, uint16_t*,
                            uint8_t*, uint64_t, uint32_t, uint32_t, uint64_t, uint32_t*, uint32_t, const RssParams);
std::atomic<int> g_tail_div{1};    // flat kernel: tail tiles hold B / g_tail_div packets (1 = no guided tail)
std::atomic<int> g_tail_tiles{4};  // ... and cover about this many tail tiles per wave slot

int flat_occupancy(FlatKernel k) {
    constexpr int kSlots = 16;
    static std::atomic<FlatKernel> keys[kSlots];
    static std::atomic<int> vals[kSlots];
    for (int i = 0; i < kSlots; ++i) {
        if (keys[i].load(std::memory_order_acquire) == k) return vals[i].load(std::memory_order_relaxed);
    }
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k), kBlock, 0) != hipSuccess ||
        nb <= 0) {
        nb = 1;
    }
    for (int i = 0; i < kSlots; ++i) {
        FlatKernel expect = nullptr;
        if (keys[i].load(std::memory_order_relaxed) == nullptr) {
            vals[i].store(nb, std::memory_order_relaxed);
            if (keys[i].compare_exchange_strong(expect, k, std::memory_order_release)) break;
        }
    }
    return nb;
}

void launch_flat(FlatKernel kern, hipStream_t s, const uint8_t* b, uint64_t bytes_len, const uint64_t* d_off,
                 const uint32_t* d_len, const uint32_t* d_seed, uint16_t* d_out, uint8_t* d_status, uint64_t n,
                 uint32_t flags, const RssParams& rss) {
    const int occ = flat_occupancy(kern);
    const int knob = g_blocks_per_cu.load(std::memory_order_relaxed);
    const uint64_t bpc = static_cast<uint64_t>(occ < knob ? occ : knob);
    const uint64_t cap = static_cast<uint64_t>(cu_count()) * bpc;
    const uint64_t slots = cap * kWavesPerBlock;
    uint64_t bmax = static_cast<uint64_t>(g_tile_packets.load(std::memory_order_relaxed));
    const uint64_t tb = static_cast<uint64_t>(g_tile_bytes.load(std::memory_order_relaxed));
    if (tb) {
        const uint64_t mean = bytes_len / n ? bytes_len / n : 1;
        const uint64_t bb = tb / mean ? tb / mean : 1;
        bmax = bb < bmax ? bb : bmax;
    }
    uint64_t B = (n + slots - 1) / slots;
    B = B < 1 ? 1 : (B > bmax ? bmax : B);
    // guided tail: the last ~g_tail_tiles small tiles per wave slot hold B / g_tail_div packets each
    const int div = g_tail_div.load(std::memory_order_relaxed);
    const uint64_t B2 = div > 1 && B / div ? B / div : B;
    const uint64_t tail = B2 < B ? slots * B2 * static_cast<uint64_t>(g_tail_tiles.load(std::memory_order_relaxed)) : 0;
    const uint64_t T1 = tail < n ? (n - tail) / B : 0;
    const uint64_t tiles = T1 + (n - T1 * B + B2 - 1) / B2;
    uint64_t blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    blocks = blocks < cap ? blocks : cap;
    blocks = (blocks + 15) & ~uint64_t(15);  // multiple of 16: XCD mapping, waves divide into kGroups
    uint32_t* heads = g_dynamic.load(std::memory_order_relaxed) ? next_heads() : nullptr;
    kern<<<dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, s>>>(
        b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, static_cast<uint32_t>(B), static_cast<uint32_t>(B2), T1,
        heads, flags, rss);
}

template <int U, bool IPV4>
void launch_u(int variant, hipStream_t s, const uint8_t* b, uint64_t bytes_len, const uint64_t* d_off,
              const uint32_t* d_len, const uint32_t* d_seed, uint16_t* d_out, uint8_t* d_status, uint64_t n,
              uint32_t flags, const RssParams& rss) {
    if (variant == 1) {
        csum_kernel<U, IPV4>
            <<<dim3(grid_for(n)), dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags);
        return;
    }
    if (variant >= 10) {  // flat kernel: 10 / 11 = U 2, 12 / 13 = U 4, 14 / 15 = U 8 (odd: next chunk in flight), 16 = U 16
        auto go = [&](auto kern) {
            launch_flat(kern, s, b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags, rss);
        };
        constexpr bool F = IPV4;  // frames may fill in place; spans never do
        const bool fill = IPV4 && (flags & kFlagFillL4);
        switch (variant) {
            case 10: fill ? go(csum_flat_kernel<2, IPV4, F, false>) : go(csum_flat_kernel<2, IPV4, false, false>); break;
            case 11: fill ? go(csum_flat_kernel<2, IPV4, F, true>) : go(csum_flat_kernel<2, IPV4, false, true>); break;
            case 12: fill ? go(csum_flat_kernel<4, IPV4, F, false>) : go(csum_flat_kernel<4, IPV4, false, false>); break;
            case 13: fill ? go(csum_flat_kernel<4, IPV4, F, true>) : go(csum_flat_kernel<4, IPV4, false, true>); break;
            case 14: fill ? go(csum_flat_kernel<8, IPV4, F, false>) : go(csum_flat_kernel<8, IPV4, false, false>); break;
            case 15: fill ? go(csum_flat_kernel<8, IPV4, F, true>) : go(csum_flat_kernel<8, IPV4, false, true>); break;
            default: fill ? go(csum_flat_kernel<16, IPV4, F, false>) : go(csum_flat_kernel<16, IPV4, false, false>); break;
        }
        return;
    }
    // batch kernel: tiles of B <= 64 packets, enough tiles to fill every wave slot
    const uint64_t slots = static_cast<uint64_t>(cu_count()) * g_blocks_per_cu.load() * kWavesPerBlock;
    const uint64_t bmax = static_cast<uint64_t>(g_tile_packets.load(std::memory_order_relaxed));
    uint64_t B = (n + slots - 1) / slots;
    B = B < 1 ? 1 : (B > bmax ? bmax : B);
    // grid: multiple of 16 workgroups so the wave count divides into kGroups
    const dim3 grid((grid_for((n + B - 1) / B) + 15u) & ~15u);
    const uint32_t b32 = static_cast<uint32_t>(B);
    uint32_t* heads = nullptr;
    if (g_dynamic.load(std::memory_order_relaxed)) heads = next_heads();
    if constexpr (IPV4) {
        if (flags & kFlagFillL4) {
            if (variant == 8 || variant == 9) {
                csum_batch_kernel<U, true, false, kNT, false, true, true><<<grid, dim3(kBlock), 0, s>>>(
                    b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            } else {
                csum_batch_kernel<U, true, false, kNT, true, false, true><<<grid, dim3(kBlock), 0, s>>>(
                    b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            }
            return;
        }
    }
    switch (variant) {
        case 8:
            csum_batch_kernel<U, IPV4, false, kNT, false, true>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 9:
            csum_batch_kernel<U, IPV4, false, kNT, true, true>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 6:
            csum_batch_kernel<U, IPV4, false, kNT, true, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 7:
            csum_batch_kernel<U, IPV4, true, kNT, true, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 2:
            csum_batch_kernel<U, IPV4, false, kNT, false, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 4:
            csum_batch_kernel<U, IPV4, false, 0, false, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        case 5:
            csum_batch_kernel<U, IPV4, true, 0, false, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
        default:
            csum_batch_kernel<U, IPV4, true, kNT, false, false>
                <<<grid, dim3(kBlock), 0, s>>>(b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, b32, heads, flags);
            break;
    }
}

// Host-side Toeplitz windows: w[j] = the 32 key bits starting at bit j (MSB
// first), bits past key_len zero — what toeplitz.hh:84-94 holds in `v` when it
// reaches data bit j.
RssParams make_rss(const uint8_t* key, uint32_t key_len, uint32_t mode, uint32_t* d_hash) {
    RssParams P{};
    P.hash = d_hash;
    P.mode = mode;
    auto bit = [&](uint32_t k) -> uint32_t { return k < 8u * key_len ? (key[k >> 3] >> (7u - (k & 7u))) & 1u : 0u; };
    for (uint32_t j = 0; j < 96; ++j) {
        uint32_t w = 0;
        for (uint32_t t = 0; t < 32; ++t) w |= bit(j + t) << (31u - t);
        P.w[j] = w;
    }
    return P;
}

const RssParams kNoRss{};

template <bool IPV4>
int launch(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
           const uint32_t* d_seed, uint16_t* d_out, uint8_t* d_status, uint64_t n, uint32_t max_len,
           void* stream, uint32_t flags = 0, const RssParams& rss = kNoRss) {
    if (n == 0) return SCCSUM_OK;
    if (!d_bytes || !d_off || !d_len || (!d_out && !(flags & kFlagFillL4))) return SCCSUM_EINVAL;
    if ((reinterpret_cast<uintptr_t>(d_bytes) & 15u) || (reinterpret_cast<uintptr_t>(d_off) & 7u) ||
        (reinterpret_cast<uintptr_t>(d_len) & 3u) || (reinterpret_cast<uintptr_t>(d_seed) & 3u) ||
        (reinterpret_cast<uintptr_t>(d_out) & (IPV4 ? 3u : 1u))) {
        return SCCSUM_EINVAL;
    }
    int variant = g_variant.load(std::memory_order_relaxed);
    // default: the flat kernel, all loads nontemporal — 16 units per lane per
    // chunk for big batches (>= 512 Ki packets and 256 MiB), else 8 units with
    // the next chunk in flight: the 16-unit form runs 2 waves per SIMD, too
    // few tiles per wave on smaller batches (DESIGN.md §5.1 has the A/B)
    if (variant == 0) variant = (n >= (512u << 10) && bytes_len >= (256ull << 20)) ? 16 : 15;
    if (variant == 1 && (flags & kFlagFillL4)) variant = 6;  // in-place write-back lives in the batch kernel
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t* b = static_cast<const uint8_t*>(d_bytes);
    // batch kernel: U = 2 for every size (long packets keep 4 groups in flight
    // in their loop); the simple kernel sizes U by max_len.
    const int forced = g_group_units.load(std::memory_order_relaxed);
    const int uc = variant == 1 ? units_class(max_len) : (forced ? forced : 2);
    switch (uc) {
        case 1:
            launch_u<1, IPV4>(variant, s, b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags, rss);
            break;
        case 2:
            launch_u<2, IPV4>(variant, s, b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags, rss);
            break;
        case 4:
            launch_u<4, IPV4>(variant, s, b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags, rss);
            break;
        default:
            launch_u<8, IPV4>(variant, s, b, bytes_len, d_off, d_len, d_seed, d_out, d_status, n, flags, rss);
            break;
    }
    if (IPV4 && rss.hash != nullptr && variant < 10) {  // RSS is fused only in the flat kernel
        rss_kernel<<<dim3(static_cast<unsigned>((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s>>>(
            b, bytes_len, d_off, d_len, nullptr, n, rss);
    }
    return static_cast<int>(hipGetLastError());
}

// ---- gather: fragments from device-readable memory (HBM, or pinned host
// memory read over PCIe) into one device buffer.  The burst queue's zero-copy
// submit (burst.cc) uses it so that no host thread touches packet bytes.
// One wave per fragment, grid-stride; interior 16-byte blocks of the
// destination move as one (possibly unaligned) 16-byte load + one aligned
// store, the two edge blocks byte by byte (neighbouring fragments are written
// by other waves at the same time).
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__global__ __launch_bounds__(kBlock) void gather_kernel(const sccsum_gather_desc* __restrict__ desc, uint64_t n,
                                                        uint8_t* __restrict__ dst) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
    for (uint64_t w = (static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x) >> 6; w < n; w += nw) {
        const sccsum_gather_desc d = desc[w];
        const uint8_t* src = static_cast<const uint8_t*>(d.src);
        uint8_t* o = dst + d.dst_off;
        const uintptr_t a = reinterpret_cast<uintptr_t>(o), e = a + d.len;
        for (uintptr_t blk = (a & ~uintptr_t(15)) + 16u * lane; blk < e; blk += 1024u) {
            if (blk >= a && blk + 16u <= e) {
                *reinterpret_cast<u32x4*>(blk) = *reinterpret_cast<const u32x4u*>(src + (blk - a));
            } else {
                for (uint32_t k = 0; k < 16u; ++k) {
                    const uintptr_t p = blk + k;
                    if (p >= a && p < e) *reinterpret_cast<uint8_t*>(p) = src[p - a];
                }
            }
        }
    }
}

}  // namespace
}  // namespace sccsum

extern "C" {

int sccsum_abi_version(void) { return SCCSUM_ABI_VERSION; }

const char* sccsum_strerror(int err) {
    if (err == SCCSUM_OK) return "success";
    if (err == SCCSUM_EINVAL) return "invalid argument";
    if (err == SCCSUM_ENODEV) return "no such HIP device";
    if (err == SCCSUM_EBUSY) return "every batch slot is in flight";
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
    return sccsum::ensure_heads(device);
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

static int rss_args_ok(const uint8_t* key, uint32_t key_len, int mode, const uint32_t* d_hash) {
    return key && key_len >= 4 && (mode == SCCSUM_RSS_DISPATCH || mode == SCCSUM_RSS_REASSEMBLED) && d_hash &&
           !(reinterpret_cast<uintptr_t>(d_hash) & 3u);
}

int sccsum_ipv4_rss(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                    const uint8_t* key, uint32_t key_len, int mode, uint32_t* d_hash, uint8_t* d_status, uint64_t n,
                    void* stream) {
    if (n == 0) return SCCSUM_OK;
    if (!rss_args_ok(key, key_len, mode, d_hash) || !d_bytes || !d_off || !d_len ||
        (reinterpret_cast<uintptr_t>(d_bytes) & 15u) || (reinterpret_cast<uintptr_t>(d_off) & 7u) ||
        (reinterpret_cast<uintptr_t>(d_len) & 3u)) {
        return SCCSUM_EINVAL;
    }
    const sccsum::RssParams P = sccsum::make_rss(key, key_len, static_cast<uint32_t>(mode), d_hash);
    sccsum::rss_kernel<<<dim3(static_cast<unsigned>((n + sccsum::kBlock - 1) / sccsum::kBlock)), dim3(sccsum::kBlock),
                         0, static_cast<hipStream_t>(stream)>>>(static_cast<const uint8_t*>(d_bytes), bytes_len, d_off,
                                                                d_len, d_status, n, P);
    return static_cast<int>(hipGetLastError());
}

int sccsum_ipv4_frames_rss(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                           uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len, const uint8_t* key,
                           uint32_t key_len, int rss_mode, uint32_t* d_hash, void* stream) {
    if (n == 0) return SCCSUM_OK;
    if (!rss_args_ok(key, key_len, rss_mode, d_hash)) return SCCSUM_EINVAL;
    const sccsum::RssParams P = sccsum::make_rss(key, key_len, static_cast<uint32_t>(rss_mode), d_hash);
    return sccsum::launch<true>(d_bytes, bytes_len, d_off, d_len, nullptr, d_out2, d_status, n, max_len, stream, 0u,
                                P);
}

int sccsum_gather(const sccsum_gather_desc* d_desc, uint64_t n, void* d_dst, void* stream) {
    if (n == 0) return SCCSUM_OK;
    if (!d_desc || !d_dst || (reinterpret_cast<uintptr_t>(d_desc) & 7u)) return SCCSUM_EINVAL;
    const uint64_t blocks = std::min<uint64_t>((n + 3) / 4, 65536);
    sccsum::gather_kernel<<<dim3(static_cast<unsigned>(blocks)), dim3(sccsum::kBlock), 0,
                            static_cast<hipStream_t>(stream)>>>(d_desc, n, static_cast<uint8_t*>(d_dst));
    return static_cast<int>(hipGetLastError());
}

uint64_t sccsum_fragments_workspace(uint64_t nfrag) { return ((2 * nfrag + 15) & ~uint64_t(15)) + nfrag + 16; }

int sccsum_fragments(const void* d_bytes, uint64_t bytes_len, const uint64_t* d_frag_off, const uint32_t* d_frag_len,
                     uint64_t nfrag, const uint32_t* d_pkt_first, const uint32_t* d_seed, uint16_t* d_out,
                     uint8_t* d_status, uint64_t n, uint32_t max_frag_len, void* d_workspace, void* stream) {
    if (n == 0) return SCCSUM_OK;
    if (!d_pkt_first || !d_out || (nfrag && (!d_workspace || !d_frag_off || !d_frag_len)) ||
        (reinterpret_cast<uintptr_t>(d_workspace) & 15u) || (reinterpret_cast<uintptr_t>(d_pkt_first) & 3u) ||
        (reinterpret_cast<uintptr_t>(d_seed) & 3u) || (reinterpret_cast<uintptr_t>(d_out) & 1u)) {
        return SCCSUM_EINVAL;
    }
    auto* raw = static_cast<uint16_t*>(d_workspace);
    auto* raw_st = static_cast<uint8_t*>(d_workspace) + ((2 * nfrag + 15) & ~uint64_t(15));
    if (nfrag) {
        const int rc = sccsum::launch<false>(d_bytes, bytes_len, d_frag_off, d_frag_len, nullptr, raw, raw_st, nfrag,
                                             max_frag_len, stream, sccsum::kFlagRaw);
        if (rc != SCCSUM_OK) return rc;
    }
    const unsigned grid = static_cast<unsigned>((n + sccsum::kBlock - 1) / sccsum::kBlock);
    sccsum::frag_combine_kernel<<<dim3(grid), dim3(sccsum::kBlock), 0, static_cast<hipStream_t>(stream)>>>(
        d_frag_len, nfrag, d_pkt_first, raw, raw_st, d_seed, d_out, d_status, n);
    return static_cast<int>(hipGetLastError());
}

int sccsum_ipv4_fill(void* d_bytes, uint64_t bytes_len, const uint64_t* d_off, const uint32_t* d_len,
                     uint16_t* d_out2, uint8_t* d_status, uint64_t n, uint32_t max_len, uint32_t mode,
                     void* stream) {
    constexpr uint32_t kAll = SCCSUM_FILL_IP | SCCSUM_FILL_L4 | SCCSUM_FILL_L4_PSEUDO | SCCSUM_FILL_TSO;
    if (mode == 0 || (mode & ~kAll) || ((mode & SCCSUM_FILL_L4) && (mode & SCCSUM_FILL_L4_PSEUDO)) ||
        ((mode & SCCSUM_FILL_TSO) && !(mode & SCCSUM_FILL_L4_PSEUDO))) {
        return SCCSUM_EINVAL;
    }
    if (n == 0) return SCCSUM_OK;
    if (mode & SCCSUM_FILL_L4) {
        const uint32_t flags = sccsum::kFlagFillL4 | ((mode & SCCSUM_FILL_IP) ? sccsum::kFlagFillIp : 0u);
        return sccsum::launch<true>(d_bytes, bytes_len, d_off, d_len, nullptr, d_out2, d_status, n, max_len, stream,
                                    flags);
    }
    if (!d_bytes || !d_off || !d_len || (reinterpret_cast<uintptr_t>(d_off) & 7u) ||
        (reinterpret_cast<uintptr_t>(d_len) & 3u) || (reinterpret_cast<uintptr_t>(d_out2) & 3u)) {
        return SCCSUM_EINVAL;
    }
    const unsigned grid = static_cast<unsigned>((n + sccsum::kBlock - 1) / sccsum::kBlock);
    sccsum::fill_header_kernel<<<dim3(grid), dim3(sccsum::kBlock), 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<uint8_t*>(d_bytes), bytes_len, d_off, d_len, reinterpret_cast<uint32_t*>(d_out2), d_status, n,
        mode);
    return static_cast<int>(hipGetLastError());
}

int sccsum_set_kernel_variant(int variant) {
    if (variant < 0 || variant > 16) return SCCSUM_EINVAL;
    sccsum::g_variant.store(variant, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_blocks_per_cu(int blocks) {
    if (blocks < 1 || blocks > 32) return SCCSUM_EINVAL;
    sccsum::g_blocks_per_cu.store(blocks, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_group_units(int units) {
    if (units != 0 && units != 1 && units != 2 && units != 4 && units != 8) return SCCSUM_EINVAL;
    sccsum::g_group_units.store(units, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_tile_packets(int packets) {
    if (packets < 1 || packets > sccsum::kWave) return SCCSUM_EINVAL;
    sccsum::g_tile_packets.store(packets, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_tile_bytes(int bytes) {
    if (bytes < 0) return SCCSUM_EINVAL;
    sccsum::g_tile_bytes.store(bytes, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_tail_tiles(int divisor, int per_slot) {
    if (divisor < 1 || divisor > 64 || per_slot < 0 || per_slot > 64) return SCCSUM_EINVAL;
    sccsum::g_tail_div.store(divisor, std::memory_order_relaxed);
    sccsum::g_tail_tiles.store(per_slot, std::memory_order_relaxed);
    return SCCSUM_OK;
}

int sccsum_set_dynamic_tiles(int on) {
    if (on != 0 && on != 1) return SCCSUM_EINVAL;
    sccsum::g_dynamic.store(on, std::memory_order_relaxed);
    return SCCSUM_OK;
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
