// The resident engine's step seal: one 8-byte word of a
// step's descriptor that says which step a ring slot holds and where that step
// ends, so that a wave can decide "slot t holds step t, and tile v lies at or
// past its end" from one read -- atomic, where several words of a slot read
// by one load are not, while the grid's poller may be rewriting the slot.
//
// The seal is the step's index mod 2^28 over its end (first tile + tiles) mod
// 2^36.  It misjudges only if 2^28 steps were published between two tiles of
// one wave, or if 2^35 tiles lay between v and a probed step's end (2^35 tiles
// of >= 1 packet carry >= 400 GB of offsets and lengths: more than HBM); the
// walk then fails its last check, which reads the step's whole index
// (SCCSUM_EFAULT), and never uses a wrong step.
//
// Host and device code (sccsum.hip); a plain C++ compiler sees the same
// functions (tests/cpp/seal_check.cc).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define SCCSUM_SEAL_HD __host__ __device__
#else
#define SCCSUM_SEAL_HD
#endif

namespace sccsum {

constexpr uint32_t kSealLastBits = 36;
constexpr uint64_t kSealLastMask = (1ull << kSealLastBits) - 1;
constexpr uint64_t kSealTagMask = (1ull << (64 - kSealLastBits)) - 1;

// step's seal, for a step that ends at tile `end` (its first tile + tiles)
SCCSUM_SEAL_HD inline uint64_t engine_seal(uint64_t step, uint64_t end) {
    return (step << kSealLastBits) | (end & kSealLastMask);
}

// Step t's slot holds seal p: true when t ends at or before tile v, or when
// the slot holds another step (then t is done, and v's step, unprocessed,
// lies after it); false when t holds v or lies after it.
SCCSUM_SEAL_HD inline bool seal_before(uint64_t p, uint64_t t, uint64_t v) {
    if ((p >> kSealLastBits) != (t & kSealTagMask)) return true;
    return ((v - p) & kSealLastMask) < (1ull << (kSealLastBits - 1));
}

}  // namespace sccsum
