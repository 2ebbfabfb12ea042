// Driver for the REFERENCE's own toeplitz_hash (include/seastar/net/toeplitz.hh,
// compiled where it lies under /root/reference by oracle/Makefile's `ref`
// target; output only into oracle/_ref/).  Test infrastructure: it generates
// the golden vectors in tests/golden/rss.json (tests/golden/make_rss_vectors.py).
//
// stdin: one case per line, "<key hex> <data hex>" (data may be "-" for empty);
// stdout: the 32-bit hash per line as 8 hex digits.
#include <seastar/net/toeplitz.hh>

#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

static std::vector<uint8_t> unhex(const std::string& h) {
    std::vector<uint8_t> out;
    if (h == "-") return out;
    for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back(static_cast<uint8_t>(std::stoi(h.substr(i, 2), nullptr, 16)));
    return out;
}

int main() {
    std::string k, d;
    while (std::cin >> k >> d) {
        const auto key = unhex(k);
        const auto data = unhex(d);
        const seastar::rss_key_type ks{key.data(), key.size()};
        std::printf("%08x\n", seastar::toeplitz_hash(ks, data));
    }
    return 0;
}
