// store_probe — what do the in-place fill's scattered field stores cost?
// (development probe, not part of libsccsum)
//
// 1,048,576 "frames" of 1500 B back to back in each of R = 4 rotated 1.5 GB
// buffers.  Variants (one launch per buffer, R launches timed with events):
//   read      nt 16-B stream of the whole buffer (the verify kernel's floor)
//   st2       store-only: one 2-byte store at frame+10 and one at frame+26
//   st16      store-only: the aligned 16-B unit(s) holding those fields, rewritten whole
//   st64      store-only: the aligned 64-B line holding frame+10, written whole by 4 lanes
//   st128     store-only: the aligned 128-B line, written whole by 8 lanes
//   rd+st2    each wave streams a tile of 64 frames (nt), then lane i stores frame i's two fields
//   rd+st16   ... and rewrites the 16-B units holding them from the loaded bytes
//   rd+st64   ... rewrites the aligned 64-B line holding frame+10 (bytes as read)
//   rd+st2d   as rd+st2, but the tile's first line of each frame is loaded default-policy
//   rd+side   the read pass stashes each frame's head line in a dense side array
//   side2line a second pass writes the stashed lines back whole (no partial-line RMW)
//   rdH16/64  the read pass with the units over each frame's first 16 / 64 bytes loaded default-policy
//             (the rest nt), so the heads may still be cached when a store pass follows; rdD: every unit
//             default-policy
//   rdbar+... register stash + grid barrier + whole-line drain (set 3, round 5; see k_rdbar)
// usage: store_probe [reps] [set: 1 = the side-buffer set only, 2 = the fill-floor set,
//                           3 = the register-stash / grid-barrier set (round 5)]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
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
constexpr uint64_t kFrames = 1 << 20;
constexpr uint64_t kFrame = 1500;
constexpr uint64_t kBytes = kFrames * kFrame;

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ src, uint64_t units, uint64_t* sink) {
    uint64_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < units; i += stride) {
        const u32x4 a = __builtin_nontemporal_load(src + i);
        acc += uint64_t(a.x) + a.y + a.z + a.w;
    }
    if (acc == 0x123456789ull) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_st2(uint8_t* buf, uint64_t n, uint16_t v) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t* f = buf + i * kFrame;
    *reinterpret_cast<uint16_t*>(f + 10) = v;
    *reinterpret_cast<uint16_t*>(f + 26) = v;
}

__global__ __launch_bounds__(256) void k_st16(uint8_t* buf, uint64_t n, uint32_t v) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = reinterpret_cast<uint64_t>(buf) + i * kFrame;
    u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
    u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
    *u0 = u32x4{v, v, v, v};
    if (u1 != u0) *u1 = u32x4{v, v, v, v};
}

template <int LINE>
__global__ __launch_bounds__(256) void k_stline(uint8_t* buf, uint64_t n, uint32_t v) {
    constexpr int P = LINE / 16;  // lanes per frame
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t i = t / P;
    if (i >= n) return;
    const uint64_t a = (reinterpret_cast<uint64_t>(buf) + i * kFrame + 10) & ~uint64_t(LINE - 1);
    reinterpret_cast<u32x4*>(a)[t % P] = u32x4{v, v, v, v};
}

// second pass: 4 lanes per frame read-modify-write the aligned 64-B line holding frame+10
__global__ __launch_bounds__(256) void k_st64rw(uint8_t* buf, uint64_t n, uint32_t v) {
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t i = t / 4;
    if (i >= n) return;
    const uint64_t a = (reinterpret_cast<uint64_t>(buf) + i * kFrame + 10) & ~uint64_t(63);
    u32x4* L = reinterpret_cast<u32x4*>(a);
    u32x4 x = L[t % 4];
    x.z ^= v;
    L[t % 4] = x;
}

// second pass, one lane per frame: read-modify-write the aligned 64-B line (4 loads, 4 stores)
__global__ __launch_bounds__(256) void k_st64rw1(uint8_t* buf, uint64_t n, uint32_t v) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = (reinterpret_cast<uint64_t>(buf) + i * kFrame + 10) & ~uint64_t(63);
    u32x4* L = reinterpret_cast<u32x4*>(a);
    u32x4 x0 = L[0], x1 = L[1], x2 = L[2], x3 = L[3];
    x0.z ^= v;
    x2.x ^= v;
    L[0] = x0;
    L[1] = x1;
    L[2] = x2;
    L[3] = x3;
}

// second pass, one lane per frame: read-modify-write the two 16-B units holding the fields
__global__ __launch_bounds__(256) void k_st16rw1(uint8_t* buf, uint64_t n, uint32_t v) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = reinterpret_cast<uint64_t>(buf) + i * kFrame;
    u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
    u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
    u32x4 x = *u0, y = *u1;
    x.x ^= v;
    y.y ^= v;
    *u0 = x;
    *u1 = y;
}

// MODE 0 = 2-byte field stores, 1 = whole 16-B units re-read first, 2 = whole 64-B line re-read first,
// 4 = 2-byte stores after a re-read of their units, 5 = whole 16-B units from registers (no re-read);
// DFL = frame's first line default policy
template <int MODE, bool DFL>
__global__ __launch_bounds__(256) void k_rdst(uint8_t* buf, uint64_t n, uint64_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t tiles = n / 64;
    uint32_t acc = 0;
    for (uint64_t t = wave; t < tiles; t += nw) {
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + t * 64 * kFrame);
        constexpr uint32_t units = 64 * kFrame / 16;  // 6000
        for (uint32_t u = lane; u < units; u += 64 * 8) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t uu = u + 64 * k;
                if (uu < units) {
                    const bool head = DFL && ((uu * 16u) % kFrame) < 16u;
                    v[k] = head ? base[uu] : __builtin_nontemporal_load(base + uu);
                } else {
                    v[k] = u32x4{0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        uint8_t* f = buf + (t * 64 + lane) * kFrame;
        const uint16_t w = uint16_t(acc);
        if (MODE == 0) {
            *reinterpret_cast<uint16_t*>(f + 10) = w;
            *reinterpret_cast<uint16_t*>(f + 26) = w;
        } else if (MODE == 1) {
            const uint64_t a = reinterpret_cast<uint64_t>(f);
            u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
            u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
            u32x4 x = *u0;
            x.x ^= acc | 1u;  // re-read and rewrite whole (modified: the store cannot be elided)
            *u0 = x;
            if (u1 != u0) {
                u32x4 y = *u1;
                y.y ^= acc | 1u;
                *u1 = y;
            }
        } else if (MODE == 4) {
            const uint64_t a = reinterpret_cast<uint64_t>(f);
            const u32x4 x0 = *reinterpret_cast<const u32x4*>((a + 10) & ~15ull);
            const u32x4 x1 = *reinterpret_cast<const u32x4*>((a + 26) & ~15ull);
            const uint16_t w2 = uint16_t(w + (x0.x == 0x5a5a5a5au) + (x1.y == 0x5a5a5a5au));  // stores wait for the loads
            *reinterpret_cast<uint16_t*>(f + 10) = w2;
            *reinterpret_cast<uint16_t*>(f + 26) = w2;
        } else if (MODE == 5) {
            const uint64_t a = reinterpret_cast<uint64_t>(f);
            u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
            u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
            *u0 = u32x4{acc, acc, acc, acc};
            if (u1 != u0) *u1 = u32x4{acc, w, acc, w};
        } else if (MODE == 9) {  // nontemporal 2-byte stores
            __builtin_nontemporal_store(w, reinterpret_cast<uint16_t*>(f + 10));
            __builtin_nontemporal_store(w, reinterpret_cast<uint16_t*>(f + 26));
        } else if (MODE == 6 || MODE == 7 || MODE == 8) {
            // whole aligned 32 / 64 / 128-byte block(s) holding both fields, from registers (no re-read)
            constexpr uint64_t B = MODE == 6 ? 32 : (MODE == 7 ? 64 : 128);
            const uint64_t a = reinterpret_cast<uint64_t>(f);
            const uint64_t lo = (a + 10) & ~(B - 1), hi = (a + 27) & ~(B - 1);
            for (uint64_t blk = lo; blk <= hi; blk += B) {
#pragma unroll
                for (uint64_t k = 0; k < B / 16; ++k) reinterpret_cast<u32x4*>(blk)[k] = u32x4{acc, w, acc, w};
            }
        } else if (MODE == 2) {
            const uint64_t a = (reinterpret_cast<uint64_t>(f) + 10) & ~63ull;
            u32x4* L = reinterpret_cast<u32x4*>(a);
            u32x4 x0 = L[0], x1 = L[1], x2 = L[2], x3 = L[3];
            x0.x ^= acc | 1u;
            L[0] = x0;
            L[1] = x1;
            L[2] = x2;
            L[3] = x3;
        }
    }
    if (MODE == 10 || MODE == 12) {  // deferred: this wave's stores after its whole stream
        for (uint64_t t = wave; t < tiles; t += nw) {
            uint8_t* f = buf + (t * 64 + lane) * kFrame;
            if (MODE == 12) {
                *reinterpret_cast<uint16_t*>(f + 10) = uint16_t(acc);
                *reinterpret_cast<uint16_t*>(f + 26) = uint16_t(acc);
            } else {
                const uint64_t a = reinterpret_cast<uint64_t>(f);
                u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
                u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
                *u0 = u32x4{acc, acc, acc, acc};
                if (u1 != u0) *u1 = u32x4{acc, 1u, acc, 1u};
            }
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

// Reverse streaming: each wave walks its tile's chunks from the END to the
// START, so a frame's head (where the fields are) is read last; the fields go
// out right after the chunk holding the head, while its DRAM rows are fresh.
// MODE 0 = 2-byte stores, 1 = 16-B unit RMW, 2 = no stores (read only, reversed)
template <int MODE>
__global__ __launch_bounds__(256) void k_rdrev(uint8_t* buf, uint64_t n, uint64_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t tiles = n / 64;
    uint32_t acc = 0;
    constexpr uint32_t units = 64 * kFrame / 16;  // 6000
    constexpr uint32_t CH = 64 * 8;               // units per chunk
    for (uint64_t t = wave; t < tiles; t += nw) {
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + t * 64 * kFrame);
        const uint32_t head_unit = uint32_t((uint64_t(lane) * kFrame) / 16);
        for (int32_t c = int32_t((units + CH - 1) / CH) - 1; c >= 0; --c) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t uu = uint32_t(c) * CH + 64 * k + lane;
                v[k] = uu < units ? __builtin_nontemporal_load(base + uu) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
            if (MODE != 2 && head_unit >= uint32_t(c) * CH && head_unit < uint32_t(c + 1) * CH) {
                uint8_t* f = buf + (t * 64 + lane) * kFrame;
                if (MODE == 0) {
                    *reinterpret_cast<uint16_t*>(f + 10) = uint16_t(acc);
                    *reinterpret_cast<uint16_t*>(f + 26) = uint16_t(acc);
                } else {
                    const uint64_t a = reinterpret_cast<uint64_t>(f);
                    u32x4* u0 = reinterpret_cast<u32x4*>((a + 10) & ~15ull);
                    u32x4* u1 = reinterpret_cast<u32x4*>((a + 26) & ~15ull);
                    u32x4 x = *u0, y = *u1;
                    x.x ^= acc | 1u;
                    y.y ^= acc | 1u;
                    *u0 = x;
                    *u1 = y;
                }
            }
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

// Side-buffer variants: the read pass stashes each frame's head line (the
// aligned 64 B holding frame+10) in a dense side array — coalesced full-line
// writes, 4 KB per wave per tile — and a second pass writes those lines back
// whole (full-line writes, no partial-line read-modify-write in HBM).
// RELOAD: the stash is the line's real content (4 loads after the tile);
// otherwise a register value (pure write cost).
template <bool RELOAD>
__global__ __launch_bounds__(256) void k_rdside(uint8_t* buf, uint64_t n, u32x4* side, uint64_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t tiles = n / 64;
    uint32_t acc = 0;
    for (uint64_t t = wave; t < tiles; t += nw) {
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + t * 64 * kFrame);
        constexpr uint32_t units = 64 * kFrame / 16;
        for (uint32_t u = lane; u < units; u += 64 * 8) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t uu = u + 64 * k;
                v[k] = uu < units ? __builtin_nontemporal_load(base + uu) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        const uint64_t f = reinterpret_cast<uint64_t>(buf) + (t * 64 + lane) * kFrame;
        const u32x4* L = reinterpret_cast<const u32x4*>((f + 10) & ~63ull);
        u32x4* out = side + (t * 64 + lane) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32x4 x = RELOAD ? L[k] : u32x4{acc, acc, acc, acc};
            x.x ^= acc | 1u;
            __builtin_nontemporal_store(x, out + k);
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

// Second pass: 4 lanes per frame copy its stashed 64 B back over the head line.
__global__ __launch_bounds__(256) void k_side2line(uint8_t* buf, uint64_t n, const u32x4* side) {
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t i = t / 4;
    if (i >= n) return;
    u32x4* L = reinterpret_cast<u32x4*>((reinterpret_cast<uint64_t>(buf) + i * kFrame + 10) & ~63ull);
    L[t % 4] = __builtin_nontemporal_load(side + i * 4 + t % 4);
}

// Read pass whose units overlapping the first HB bytes of each frame are
// loaded with the default policy (the rest nt), so the frame heads — where
// the fields are — may stay in L2 / MALL for a store pass right after it.
template <uint32_t HB>
__global__ __launch_bounds__(256) void k_rdhead(const uint8_t* buf, uint64_t n, uint64_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t tiles = n / 64;
    uint32_t acc = 0;
    for (uint64_t t = wave; t < tiles; t += nw) {
        const uint64_t tb = reinterpret_cast<uint64_t>(buf) + t * 64 * kFrame;
        const u32x4* base = reinterpret_cast<const u32x4*>(tb);
        constexpr uint32_t units = 64 * kFrame / 16;
        for (uint32_t u = lane; u < units; u += 64 * 8) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t uu = u + 64 * k;
                if (uu < units) {
                    // frame holding this unit's first byte, and the unit's offset from that frame's start
                    const uint64_t a = tb + uint64_t(uu) * 16;
                    const uint64_t fo = (a - reinterpret_cast<uint64_t>(buf)) % kFrame;
                    const bool head = fo < HB || fo + 16 > kFrame;  // overlaps [frame, frame + HB)
                    v[k] = head ? base[uu] : __builtin_nontemporal_load(base + uu);
                } else {
                    v[k] = u32x4{0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

// Round 5: register stash + grid barrier + whole-line drain.  Every wave streams
// its TPW tiles of 64 frames (nt), keeps each frame's aligned 64-B head line
// (holding frame+10) in registers, then all waves meet at a grid barrier
// (one counter, system-scope polls, 400 us limit) and only then write the
// head lines back WHOLE: full-line writes need no read-modify-write in HBM and
// none of them lands inside the read stream.
// MODE 0 = barrier only (no stores), 1 = barrier then 2-byte field stores,
// 2 = barrier then whole lines (stash reloaded default-policy after each tile),
// 3 = barrier then whole lines from register values (no reload: pure write
// cost), 4 = no barrier, whole reloaded lines after the wave's own stream,
// 5 = as 2 but the stash is cut out of the streamed registers' lanes through
// LDS instead of reloaded (the product's form: no extra read).
constexpr int kTpw = 4;
#ifndef POLL_SLEEP
#define POLL_SLEEP 127
#endif
__device__ __forceinline__ uint64_t probe_clock() { return static_cast<uint64_t>(wall_clock64()); }
__device__ uint64_t g_trace[4096 * 3];  // per wave: start, arrival, leave (100 MHz), last launch
template <int MODE>
__global__ __launch_bounds__(256) void k_rdbar(uint8_t* buf, uint64_t n, uint64_t* bar, uint64_t target,
                                               uint64_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t t_start = probe_clock();
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    const uint64_t tiles = n / 64;
    __shared__ u32x4 lds[4][64 * 4];
    u32x4* my = lds[threadIdx.x >> 6];
    uint32_t acc = 0;
    u32x4 stash[kTpw][4];
#pragma unroll
    for (int j = 0; j < kTpw; ++j) {
        const uint64_t t = wave + uint64_t(j) * nw;
        if (t >= tiles) break;
        const uint64_t tb = reinterpret_cast<uint64_t>(buf) + t * 64 * kFrame;
        const u32x4* base = reinterpret_cast<const u32x4*>(tb);
        constexpr uint32_t units = 64 * kFrame / 16;  // 6000
        for (uint32_t u = lane; u < units; u += 64 * 8) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t uu = u + 64 * k;
                v[k] = uu < units ? __builtin_nontemporal_load(base + uu) : u32x4{0, 0, 0, 0};
            }
            if (MODE == 5) {
                // units inside some frame's head line go to that frame's LDS slot
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t uu = u + 64 * k;
                    if (uu < units) {
                        const uint64_t a = tb + uint64_t(uu) * 16;
                        const uint64_t rel = a - tb;
                        const uint32_t fr = uint32_t(rel / kFrame);
                        const uint64_t hl = (tb + uint64_t(fr) * kFrame + 10) & ~63ull;
                        if (a >= hl && a < hl + 64) my[fr * 4 + uint32_t((a - hl) >> 4)] = v[k];
                        if (fr + 1 < 64) {  // a unit may also sit in the next frame's head line
                            const uint64_t hn = (tb + uint64_t(fr + 1) * kFrame + 10) & ~63ull;
                            if (a >= hn && a < hn + 64) my[(fr + 1) * 4 + uint32_t((a - hn) >> 4)] = v[k];
                        }
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        const uint64_t f = tb + uint64_t(lane) * kFrame;
        const u32x4* L = reinterpret_cast<const u32x4*>((f + 10) & ~63ull);
        if (MODE == 2 || MODE == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) stash[j][k] = L[k];
        } else if (MODE == 5) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 4; ++k) stash[j][k] = my[lane * 4 + k];
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) stash[j][k] = u32x4{acc, acc + k, acc, acc};
        }
        stash[j][0].z ^= acc | 1u;
    }
    if (MODE != 4) {
        // block barrier in hardware, then one poller per block (every ~3.4 us)
        __syncthreads();
        if (threadIdx.x == 0) {
            // the block that completes the count publishes the generation to 64 flag lines
            // (4 352 B apart: different channels); each block polls its own line
            const uint64_t got = __hip_atomic_fetch_add(bar, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint64_t gen = target / (uint64_t(gridDim.x) * 4);
            uint64_t* flags = bar + 8;
            if (got + 4 == target) {
                for (int i = 0; i < 64; ++i)
                    __hip_atomic_store(flags + i * 544, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            const uint64_t t0 = probe_clock();
            uint64_t seen = 0;
            uint64_t* mine = flags + (blockIdx.x & 63) * 544;
            while ((seen = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) < gen) {
                if (probe_clock() - t0 > 40000) {  // 400 us: the grid was not co-resident
                    __hip_atomic_fetch_add(sink + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (blockIdx.x == 0) { sink[2] = got; sink[3] = seen; sink[4] = target; }
                    break;
                }
                __builtin_amdgcn_s_sleep(POLL_SLEEP);
            }
            const uint64_t wv = blockIdx.x;
            if (wv < 4096) {
                g_trace[wv * 3] = t_start;
                g_trace[wv * 3 + 1] = t0;
                g_trace[wv * 3 + 2] = probe_clock();
            }
        }
        __syncthreads();
    }
    if (MODE != 0) {
#pragma unroll
        for (int j = 0; j < kTpw; ++j) {
            const uint64_t t = wave + uint64_t(j) * nw;
            if (t >= tiles) break;
            uint8_t* f = buf + (t * 64 + lane) * kFrame;
            if (MODE == 1) {
                *reinterpret_cast<uint16_t*>(f + 10) = uint16_t(stash[j][0].z);
                *reinterpret_cast<uint16_t*>(f + 26) = uint16_t(stash[j][0].z);
            } else {
                u32x4* L = reinterpret_cast<u32x4*>((reinterpret_cast<uint64_t>(f) + 10) & ~63ull);
#pragma unroll
                for (int k = 0; k < 4; ++k) L[k] = stash[j][k];
            }
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    constexpr int R = 4;
    uint8_t* bufs[R];
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&bufs[r], kBytes + 4096));
        CK(hipMemset(bufs[r], r + 1, kBytes + 4096));
    }
    uint64_t* sink;
    CK(hipMalloc(&sink, 64));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned g_frames = unsigned((kFrames + 255) / 256);
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < R; ++r) launch(bufs[r]);  // warm
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int k = 0; k < reps; ++k) {
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < R; ++r) launch(bufs[r]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        CK(hipGetLastError());
        const double us = best * 1e3 / R;
        std::printf("%-10s %9.1f us/launch  %7.0f GB/s of frame bytes\n", name, us, kBytes / us / 1e3);
        std::fflush(stdout);
    };
    u32x4* side;
    CK(hipMalloc(&side, kFrames * 64));
    if (argc > 2 && std::atoi(argv[2]) == 3) {  // register stash + grid barrier + whole-line drain (round 5)
        uint64_t* bar;
        CK(hipMalloc(&bar, 64 + 64 * 4352));
        CK(hipMemset(bar, 0, 64 + 64 * 4352));
        CK(hipMemset(sink, 0, 64));
        const unsigned blocks = unsigned(kFrames / 64 / kTpw / 4);  // 4 waves per block, kTpw tiles per wave
        const uint64_t nwaves = uint64_t(blocks) * 4;
        uint64_t gen = 0;
        auto bar_launch = [&](auto kern, uint8_t* b) {
            ++gen;
            kern<<<blocks, 256>>>(b, kFrames, bar, gen * nwaves, sink);
        };
        std::printf("blocks %u (%.1f per CU), waves %llu\n", blocks, double(blocks) / cus,
                    (unsigned long long)nwaves);
        run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("rdbar only", [&](uint8_t* b) { bar_launch(k_rdbar<0>, b); });
        run("rdbar+st2", [&](uint8_t* b) { bar_launch(k_rdbar<1>, b); });
        run("rdbar+lineR", [&](uint8_t* b) { bar_launch(k_rdbar<2>, b); });
        run("rdbar+lineV", [&](uint8_t* b) { bar_launch(k_rdbar<3>, b); });
        run("rd+lineR", [&](uint8_t* b) { k_rdbar<4><<<blocks, 256>>>(b, kFrames, bar, 0, sink); });
        run("rdbar+lineL", [&](uint8_t* b) { bar_launch(k_rdbar<5>, b); });
        run("rd;st2", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rd;st64rw", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st64rw<<<g_frames * 4, 256>>>(b, kFrames, 0x1234);
        });
        run("rdbar+lineR", [&](uint8_t* b) { bar_launch(k_rdbar<2>, b); });
        run("rdbar+lineL", [&](uint8_t* b) { bar_launch(k_rdbar<5>, b); });
        run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
        {
            int nb0 = 0, nb5 = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb0, k_rdbar<0>, 256, 0));
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb5, k_rdbar<5>, 256, 0));
            std::printf("occupancy blocks/CU: mode0 %d mode5 %d\n", nb0, nb5);
            std::vector<uint64_t> tr(4096 * 3);
            CK(hipMemset(sink, 0, 64));
            bar_launch(k_rdbar<0>, bufs[0]);
            CK(hipDeviceSynchronize());
            CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_trace), tr.size() * 8));
            uint64_t s0 = ~0ull, s1 = 0, a0 = ~0ull, a1 = 0, l0 = ~0ull, l1 = 0;
            for (uint64_t w = 0; w < blocks; ++w) {
                s0 = std::min(s0, tr[w * 3]); s1 = std::max(s1, tr[w * 3]);
                a0 = std::min(a0, tr[w * 3 + 1]); a1 = std::max(a1, tr[w * 3 + 1]);
                l0 = std::min(l0, tr[w * 3 + 2]); l1 = std::max(l1, tr[w * 3 + 2]);
            }
            std::printf("mode0 one launch (us from first start): start %.1f..%.1f arrive %.1f..%.1f leave %.1f..%.1f\n",
                        0.0, (s1 - s0) / 100.0, (a0 - s0) / 100.0, (a1 - s0) / 100.0, (l0 - s0) / 100.0, (l1 - s0) / 100.0);
            for (uint64_t w = 0; w < blocks; w += 128)
                std::printf("  block %4llu start %.1f arrive %.1f leave %.1f\n", (unsigned long long)w,
                            (tr[w * 3] - s0) / 100.0, (tr[w * 3 + 1] - s0) / 100.0, (tr[w * 3 + 2] - s0) / 100.0);
        }
        uint64_t h[5];
        CK(hipMemcpy(h, sink, 40, hipMemcpyDeviceToHost));
        std::printf("block 0: fetch_add got %llu, last seen %llu, target %llu\n", (unsigned long long)h[2],
                    (unsigned long long)h[3], (unsigned long long)h[4]);
        std::printf("barrier time-outs (waves): %llu\n", (unsigned long long)h[1]);
        return 0;
    }
    if (argc > 2 && std::atoi(argv[2]) == 2) {  // the fill's floor: does a cached frame head make the store pass cheap?
        const unsigned g4 = g_frames * 4;
        run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("rdH16 only", [&](uint8_t* b) { k_rdhead<16><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("rdH64 only", [&](uint8_t* b) { k_rdhead<64><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("st2", [&](uint8_t* b) { k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234); });
        run("st64rw", [&](uint8_t* b) { k_st64rw<<<g4, 256>>>(b, kFrames, 0x1234); });
        run("st64rw1", [&](uint8_t* b) { k_st64rw1<<<g_frames, 256>>>(b, kFrames, 0x1234); });
        run("st16rw1", [&](uint8_t* b) { k_st16rw1<<<g_frames, 256>>>(b, kFrames, 0x1234); });
        run("rd;st2", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rd;st64rw", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st64rw<<<g4, 256>>>(b, kFrames, 0x1234);
        });
        run("rd;st16rw1", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st16rw1<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdH16;st2", [&](uint8_t* b) {
            k_rdhead<16><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdH64;st2", [&](uint8_t* b) {
            k_rdhead<64><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdH64;st64rw", [&](uint8_t* b) {
            k_rdhead<64><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st64rw<<<g4, 256>>>(b, kFrames, 0x1234);
        });
        run("rdH64;st64rw1", [&](uint8_t* b) {
            k_rdhead<64><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st64rw1<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdH64;st16rw1", [&](uint8_t* b) {
            k_rdhead<64><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st16rw1<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdD only", [&](uint8_t* b) { k_rdhead<1500><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("rdD;st2", [&](uint8_t* b) {
            k_rdhead<1500><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rdD;st64rw", [&](uint8_t* b) {
            k_rdhead<1500><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st64rw<<<g4, 256>>>(b, kFrames, 0x1234);
        });
        run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
        return 0;
    }
    if (argc > 2 && std::atoi(argv[2]) == 1) {  // side-buffer set only
        run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
        run("rd;st2", [&](uint8_t* b) {
            k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink);
            k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
        });
        run("rd+sideR", [&](uint8_t* b) { k_rdside<false><<<cus * 4, 256>>>(b, kFrames, side, sink); });
        run("rd+side", [&](uint8_t* b) { k_rdside<true><<<cus * 4, 256>>>(b, kFrames, side, sink); });
        run("side2line", [&](uint8_t* b) { k_side2line<<<g_frames * 4, 256>>>(b, kFrames, side); });
        run("rd+side;2line", [&](uint8_t* b) {
            k_rdside<true><<<cus * 4, 256>>>(b, kFrames, side, sink);
            k_side2line<<<g_frames * 4, 256>>>(b, kFrames, side);
        });
        run("st64", [&](uint8_t* b) { k_stline<64><<<g_frames * 4, 256>>>(b, kFrames, 0x1234); });
        run("st2", [&](uint8_t* b) { k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234); });
        return 0;
    }
    run("read", [&](uint8_t* b) { k_read<<<cus * 8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, sink); });
    run("st2", [&](uint8_t* b) { k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234); });
    run("st16", [&](uint8_t* b) { k_st16<<<g_frames, 256>>>(b, kFrames, 0x1234); });
    run("st64", [&](uint8_t* b) { k_stline<64><<<g_frames * 4, 256>>>(b, kFrames, 0x1234); });
    run("st128", [&](uint8_t* b) { k_stline<128><<<g_frames * 8, 256>>>(b, kFrames, 0x1234); });
    run("rd+st2", [&](uint8_t* b) { k_rdst<0, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st16", [&](uint8_t* b) { k_rdst<1, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st64", [&](uint8_t* b) { k_rdst<2, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st2d", [&](uint8_t* b) { k_rdst<0, true><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st16d", [&](uint8_t* b) { k_rdst<1, true><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st64d", [&](uint8_t* b) { k_rdst<2, true><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st2r", [&](uint8_t* b) { k_rdst<4, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st16n", [&](uint8_t* b) { k_rdst<5, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st32n", [&](uint8_t* b) { k_rdst<6, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st64n", [&](uint8_t* b) { k_rdst<7, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+st128n", [&](uint8_t* b) { k_rdst<8, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd8w only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 2, 256>>>(b, kFrames, sink); });
    run("rd8w+st16", [&](uint8_t* b) { k_rdst<1, false><<<cus * 2, 256>>>(b, kFrames, sink); });
    run("rd8w+st64n", [&](uint8_t* b) { k_rdst<7, false><<<cus * 2, 256>>>(b, kFrames, sink); });
    run("rd+st2nt", [&](uint8_t* b) { k_rdst<9, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd;st2", [&](uint8_t* b) {
        k_read<<<cus * 8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, sink);
        k_st2<<<g_frames, 256>>>(b, kFrames, 0x1234);
    });
    run("rd;st64rw", [&](uint8_t* b) {
        k_read<<<cus * 8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, sink);
        k_st64rw<<<g_frames * 4, 256>>>(b, kFrames, 0x1234);
    });
    run("st64rw", [&](uint8_t* b) { k_st64rw<<<g_frames * 4, 256>>>(b, kFrames, 0x1234); });
    run("st64rw1", [&](uint8_t* b) { k_st64rw1<<<g_frames, 256>>>(b, kFrames, 0x1234); });
    run("st16rw1", [&](uint8_t* b) { k_st16rw1<<<g_frames, 256>>>(b, kFrames, 0x1234); });
    run("rd;st64rw1", [&](uint8_t* b) {
        k_read<<<cus * 8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, sink);
        k_st64rw1<<<g_frames, 256>>>(b, kFrames, 0x1234);
    });
    run("rd;st16rw1", [&](uint8_t* b) {
        k_read<<<cus * 8, 256>>>(reinterpret_cast<const u32x4*>(b), kBytes / 16, sink);
        k_st16rw1<<<g_frames, 256>>>(b, kFrames, 0x1234);
    });
    run("rd+dfr16", [&](uint8_t* b) { k_rdst<10, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd+dfr2", [&](uint8_t* b) { k_rdst<12, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rd8w+dfr16", [&](uint8_t* b) { k_rdst<10, false><<<cus * 2, 256>>>(b, kFrames, sink); });
    run("rev only", [&](uint8_t* b) { k_rdrev<2><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rev+st2", [&](uint8_t* b) { k_rdrev<0><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rev+st16rw", [&](uint8_t* b) { k_rdrev<1><<<cus * 4, 256>>>(b, kFrames, sink); });
    run("rev8w+st2", [&](uint8_t* b) { k_rdrev<0><<<cus * 2, 256>>>(b, kFrames, sink); });
    run("rd only", [&](uint8_t* b) { k_rdst<3, false><<<cus * 4, 256>>>(b, kFrames, sink); });
    return 0;
}
