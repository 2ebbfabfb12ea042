"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer — the
reference's `sanitize` build mode (cmake/FindSanitizers.cmake:37-43,
CMakeLists.txt:140-145), applied to the host side of this path:

1. the kept per-packet C++ API (checksummer.cc) against the oracle
   (tests/cpp/api_parity.cc), g++;
2. checksummer::sum(const packet&) over the reference's packet type
   (tests/cpp/packet_ref.cc; needs /root/reference), g++;
3. argument validation of every C-ABI entry point, the library's own sources
   (sccsum.hip host side, burst.cc, pipeline.cc, checksummer.cc) built with
   hipcc and the sanitizers on the host compilation only
   (`-Xarch_host -fsanitize=...`; device code is not instrumented), run
   without a device (tests/cpp/abi_validate.cc);
4. the same program under ThreadSanitizer, its checks run from 8 threads at
   once (one reactor thread per shard calls the library, reactor.cc:3437).
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
REF_INCLUDE = "/root/reference/include"


def _run(cmd, cwd):
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=cwd)
    assert r.returncode == 0, r.stderr[-4000:]


def _oracle_obj(tmp_path):
    obj = str(tmp_path / "oracle.o")
    _run(["gcc", "-O1", "-g", *SAN, "-c", os.path.join(REPO, "oracle", "sccsum_oracle.c"), "-o", obj], tmp_path)
    return obj


def _exec(exe, tmp_path, args=()):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=ENV, cwd=tmp_path)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "OK" in r.stdout and "runtime error" not in r.stderr
    return r


def test_api_parity_sanitized(tmp_path):
    exe = str(tmp_path / "api_parity_san")
    _run(["g++", "-std=c++17", "-O1", "-g", *SAN, "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "oracle"),
          os.path.join(REPO, "tests", "cpp", "api_parity.cc"), os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"),
          _oracle_obj(tmp_path), "-o", exe, "-lpthread"], tmp_path)
    _exec(exe, tmp_path)


@pytest.mark.skipif(not os.path.isdir(REF_INCLUDE), reason="needs /root/reference (build container only)")
def test_packet_ref_sanitized(tmp_path):
    exe = str(tmp_path / "packet_ref_san")
    _run(["g++", "-std=c++20", "-O1", "-g", *SAN, "-I", os.path.join(REPO, "include"), "-I", REF_INCLUDE,
          "-I", os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "cpp", "packet_ref.cc"),
          os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"),
          os.path.join(REPO, "seastar_amd", "csrc", "checksummer_packet.cc"), _oracle_obj(tmp_path), "-o", exe,
          "-lpthread"], tmp_path)
    _exec(exe, tmp_path)


def test_abi_validation_sanitized(tmp_path):
    exe = str(tmp_path / "abi_validate_san")
    host_san = []
    for f in SAN:  # each host-only flag right after -Xarch_host
        host_san += ["-Xarch_host", f]
    csrc = os.path.join(REPO, "seastar_amd", "csrc")
    _run(["/opt/rocm/bin/hipcc", "-O1", "-g", "--offload-arch=gfx950", "-std=c++17", *host_san,
          "-I", os.path.join(REPO, "include"), os.path.join(csrc, "sccsum.hip"), os.path.join(csrc, "checksummer.cc"),
          os.path.join(csrc, "pipeline.cc"), os.path.join(csrc, "burst.cc"),
          os.path.join(REPO, "tests", "cpp", "abi_validate.cc"), "-o", exe], tmp_path)
    _exec(exe, tmp_path)


def test_abi_validation_threads_tsan(tmp_path):
    """The C-ABI's host side (thread-local knobs, argument checks, the
    burst / pipeline constructors' failure paths) driven from 8 threads under
    ThreadSanitizer, host code only: no data race may be reported."""
    exe = str(tmp_path / "abi_validate_tsan")
    host_san = []
    for f in ("-fsanitize=thread", "-fno-omit-frame-pointer"):
        host_san += ["-Xarch_host", f]
    csrc = os.path.join(REPO, "seastar_amd", "csrc")
    _run(["/opt/rocm/bin/hipcc", "-O1", "-g", "--offload-arch=gfx950", "-std=c++17", *host_san,
          "-I", os.path.join(REPO, "include"), os.path.join(csrc, "sccsum.hip"), os.path.join(csrc, "checksummer.cc"),
          os.path.join(csrc, "pipeline.cc"), os.path.join(csrc, "burst.cc"),
          os.path.join(REPO, "tests", "cpp", "abi_validate.cc"), "-o", exe], tmp_path)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, "8"], capture_output=True, text=True, timeout=300, env=env, cwd=tmp_path)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "OK (8 threads)" in r.stdout and "ThreadSanitizer" not in r.stderr
