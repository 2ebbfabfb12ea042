// checksummer::sum(const packet&) — src/net/ip_checksum.cc:64-68: walk the
// packet's fragment list; `odd` carries across odd-sized fragments.
// Needs Seastar's real packet type, so it is compiled only inside the Seastar
// tree; the standalone library omits it.
#include <seastar/net/ip_checksum.hh>
#include <seastar/net/packet.hh>

namespace seastar {

namespace net {

void checksummer::sum(const packet& p) {
    for (const auto& frag : p.fragments()) {
        sum(frag.base, frag.size);
    }
}

}  // namespace net

}  // namespace seastar
