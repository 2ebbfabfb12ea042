"""The kept per-packet C++ API (include/seastar/net/ip_checksum.hh +
seastar_amd/csrc/checksummer.cc), compiled with g++ -O2 like Seastar's
release mode, against the oracle; and the batch C++ header compiles."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path, name, sources, extra=()):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "oracle"), *sources, "-o", exe, *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_per_packet_api_matches_oracle(tmp_path):
    obj = str(tmp_path / "oracle.o")
    subprocess.run(["gcc", "-O2", "-c", os.path.join(REPO, "oracle", "sccsum_oracle.c"), "-o", obj], check=True)
    exe = _build(tmp_path, "api_parity",
                 [os.path.join(REPO, "tests", "cpp", "api_parity.cc"),
                  os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"), obj], ["-lpthread"])
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_engine_seal_arithmetic(tmp_path):
    """The resident engine's step seal (seastar_amd/csrc/engine_seal.h,
    DESIGN.md §5.11) on the host: its own step's seal orders every tile within
    2^35 of the step's end correctly across both fields' wraps, and any other
    step a ring can put in the slot reads as "before"."""
    exe = _build(tmp_path, "seal_check", [os.path.join(REPO, "tests", "cpp", "seal_check.cc")],
                 ["-I", os.path.join(REPO, "seastar_amd", "csrc")])
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "seal_check: OK" in r.stdout


def test_batch_header_compiles(tmp_path):
    src = tmp_path / "b.cc"
    src.write_text('#include <seastar/net/ip_checksum_batch.hh>\n'
                   'int main() { return int(seastar::net::batch_checksummer::pseudo_header_seed(1, 2, 17, 8) == 0); }\n')
    exe = _build(tmp_path, "b", [str(src)], ["-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
                                             "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib")])
    assert os.path.exists(exe)


def test_batch_header_compiles_cxx20_rss_span(tmp_path):
    """The rss_key_type (std::span) overload, as the reference's callers hold the key."""
    src = tmp_path / "r.cc"
    src.write_text('#include <seastar/net/ip_checksum_batch.hh>\n'
                   'static const uint8_t key[40] = {0xd1, 0x81};\n'
                   'void f(const seastar::net::batch_checksummer& e, const seastar::net::device_packet_batch& b,\n'
                   '       uint32_t* h) { e.ipv4_rss(b, std::span<const uint8_t>(key), SCCSUM_RSS_DISPATCH, h, nullptr,\n'
                   '                                nullptr); }\n'
                   'int main() { return 0; }\n')
    exe = str(tmp_path / "r")
    cmd = ["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"), str(src), "-o", exe,
           "-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
           "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_batch_cpp_program_on_gpu(tmp_path):
    """Native host program: hipMalloc'd batch -> batch_checksummer ->
    compared frame by frame with the per-packet C++ API."""
    exe = str(tmp_path / "batch_gpu")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           os.path.join(REPO, "tests", "cpp", "batch_gpu.cc"), os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"),
           "-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
           "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def _engine_prog(tmp_path) -> str:
    exe = str(tmp_path / "engine_gpu")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           os.path.join(REPO, "tests", "cpp", "engine_gpu.cc"), os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"),
           "-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
           "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_engine_cpp_program_builds(tmp_path):
    """seastar::net::resident_engine over sccsum_engine_* compiles and links."""
    _engine_prog(tmp_path)


@pytest.mark.gpu
def test_engine_cpp_program_on_gpu(tmp_path):
    """Native host program: a shard's resident engine fills frames in place
    (generate + store steps), verifies them in the same run and generates a
    copy, all against the per-packet API; a second engine on the device is
    refused while the first runs and runs after its stop."""
    exe = _engine_prog(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_burst_queue_header_compiles(tmp_path):
    """seastar::net::burst_queue over sccsum_burst_*, fed a packet's fragment
    array in the reference's own layout (packet.hh:43-46)."""
    src = tmp_path / "q.cc"
    src.write_text(
        '#include <seastar/net/ip_checksum_batch.hh>\n'
        'struct fragment { char* base; size_t size; };  // seastar::net::fragment, packet.hh:43-46\n'
        'static_assert(sizeof(fragment) == sizeof(sccsum_fragment) && alignof(fragment) == alignof(sccsum_fragment));\n'
        'int main() {\n'
        '    auto done = [](uint64_t, uint32_t, const uint16_t*, const uint8_t*) {};\n'
        '    try {\n'
        '        seastar::net::burst_queue<decltype(done)> q(0, SCCSUM_PIPE_IPV4, 1 << 20, 256, 20000, 2, done);\n'
        '        char b[64] = {};\n'
        '        fragment f[1] = {{b, 64}};\n'
        '        (void)q.submit(reinterpret_cast<const sccsum_fragment*>(f), 1);\n'
        '        q.poll();\n'
        '        q.drain();\n'
        '    } catch (const std::exception&) {\n'
        '    }\n'
        '    return 0;\n'
        '}\n')
    _build(tmp_path, "q", [str(src)], ["-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
                                       "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib")])


@pytest.mark.gpu
def test_burst_cpp_program_on_gpu(tmp_path):
    """Native host program: frames handed to burst_queue one at a time from
    mbuf-shaped host slots (some as two fragments), compared frame by frame
    with the per-packet C++ API."""
    exe = _build(tmp_path, "burst_gpu",
                 [os.path.join(REPO, "tests", "cpp", "burst_gpu.cc"),
                  os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc")],
                 ["-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum",
                  "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib")])
    r = subprocess.run([exe, "200000", "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    print(r.stdout)
    # zero-copy submits (pinned pool), each batch form: one fragment-list launch (2), with copies (1), gather (0)
    for form in ("2", "1", "0"):
        r = subprocess.run([exe, "200000", "3", "100000", "mapped", "32", form, "4096"], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "OK" in r.stdout
        print(r.stdout)


def _shards_exe(tmp_path):
    obj = str(tmp_path / "oracle.o")
    subprocess.run(["gcc", "-O2", "-fPIC", "-c", os.path.join(REPO, "oracle", "sccsum_oracle.c"), "-o", obj],
                   check=True)
    exe = str(tmp_path / "shards_gpu")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "cpp", "shards_gpu.cc"), "-x", "none", obj,
           "-L", os.path.join(REPO, "seastar_amd", "lib"), "-lsccsum", "-lpthread",
           "-Wl,-rpath," + os.path.join(REPO, "seastar_amd", "lib"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_shards_cpp_program_builds(tmp_path):
    assert os.path.exists(_shards_exe(tmp_path))


@pytest.mark.gpu
def test_shards_cpp_program_on_gpu(tmp_path):
    """Seastar's threading model (one reactor thread per shard,
    reactor.cc:3437): 8 host threads on one device, each with its own
    sccsum_init, streams, batches, kernel form and burst queue, launching
    frames / spans / multi / fill concurrently, plus launches on streams
    destroyed without a sync; every result against the oracle."""
    exe = _shards_exe(tmp_path)
    r = subprocess.run([exe, "8", "4"], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    print(r.stdout)


@pytest.mark.gpu
def test_shards_feed_one_engine_on_gpu(tmp_path):
    """The shards of one GPU feeding its ONE resident engine (VERDICT r05 #2;
    include/sccsum.h "Producers"): 8 host threads submit random frame,
    verify-only, fill and (second run) seeded span steps into one engine with
    a 64-slot ring at once, each waiting on its own steps; every step's
    results against the oracle."""
    exe = _shards_exe(tmp_path)
    r = subprocess.run([exe, "engine", "8", "40"], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    print(r.stdout)
