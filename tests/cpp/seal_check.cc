// The engine's step seal (seastar_amd/csrc/engine_seal.h) checked on the host:
// for steps and tile positions around every wrap of its two fields, a probe of
// step t's own seal answers "v at or past t's end" exactly when v >= end, and
// a slot holding any other step a ring may put there (t + k * ring, k >= 1,
// under 2^28 steps on) always reads as "before".  Prints OK.
#include "engine_seal.h"

#include <cstdint>
#include <cstdio>
#include <random>

namespace {

int g_bad = 0;

void expect(bool got, bool want, const char* what, uint64_t t, uint64_t end, uint64_t v) {
    if (got != want && g_bad++ < 20) {
        std::printf("%s: step %llu end %llu v %llu: got %d want %d\n", what, static_cast<unsigned long long>(t),
                    static_cast<unsigned long long>(end), static_cast<unsigned long long>(v), got, want);
    }
}

}  // namespace

int main() {
    using sccsum::engine_seal;
    using sccsum::seal_before;
    std::mt19937_64 rng(0x5EA1);
    const uint64_t lastwrap = 1ull << sccsum::kSealLastBits, tagwrap = 1ull << (64 - sccsum::kSealLastBits);
    // ends near 0, near every 2^36 wrap up to 2^40, and far out (an unbounded run's tile count)
    const uint64_t ends[] = {0, 1, 63, lastwrap - 1, lastwrap, lastwrap + 1, 3 * lastwrap - 2, 16 * lastwrap + 5,
                             (1ull << 62) + 12345, ~0ull - 70000};
    // steps near 0 and around every 2^28 wrap
    const uint64_t steps[] = {0, 1, tagwrap - 1, tagwrap, tagwrap + 1, 5 * tagwrap - 1, (1ull << 50) + 7};
    long n = 0;
    for (uint64_t t : steps) {
        for (uint64_t end : ends) {
            const uint64_t p = engine_seal(t, end);
            // v within 2^35 tiles of the end, either side (wrapping as uint64_t does)
            const uint64_t deltas[] = {0, 1, 2, 31, 4096, (1ull << 35) - 1};
            for (uint64_t d : deltas) {
                expect(seal_before(p, t, end + d), true, "own seal, v at/after end", t, end, end + d);
                if (d) expect(seal_before(p, t, end - d), false, "own seal, v before end", t, end, end - d);
                n += 2;
            }
            for (int i = 0; i < 200; ++i) {
                const uint64_t d = rng() & ((1ull << 35) - 1);
                expect(seal_before(p, t, end + d), true, "own seal, random v at/after end", t, end, end + d);
                if (d) expect(seal_before(p, t, end - d), false, "own seal, random v before end", t, end, end - d);
                n += 2;
            }
            // another step in the slot: t + k * ring for rings 2 .. 2^16, any tile position
            for (uint64_t ring = 2; ring <= (1u << 16); ring <<= 1) {
                for (uint64_t k : {uint64_t(1), uint64_t(2), uint64_t(977), (tagwrap / ring) - 1}) {
                    const uint64_t other = t + k * ring;
                    const uint64_t q = engine_seal(other, end + 64 * k);
                    for (uint64_t v : {end, end - 1, end + 64 * k - 1, uint64_t(0)}) {
                        expect(seal_before(q, t, v), true, "another step's seal", t, end, v);
                        ++n;
                    }
                }
            }
        }
    }
    if (g_bad) {
        std::printf("seal_check: FAILED (%d of %ld)\n", g_bad, n);
        return 1;
    }
    std::printf("seal_check: OK (%ld cases)\n", n);
    return 0;
}
