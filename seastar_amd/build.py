"""Build libsccsum.so in-tree with hipcc for gfx950."""
from __future__ import annotations

import os
import subprocess

from .native import LIB_PATH, PKG_DIR, REPO_DIR

SOURCES = [
    os.path.join(PKG_DIR, "csrc", "sccsum.hip"),
    os.path.join(PKG_DIR, "csrc", "checksummer.cc"),
    os.path.join(PKG_DIR, "csrc", "pipeline.cc"),
    os.path.join(PKG_DIR, "csrc", "burst.cc"),
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# The AMDGPU atomic optimizer rewrites the kernels' lane-0 atomics into
# wave-wide ones whose result it reads back where they are issued; the flat
# kernel's LATE form reads its tile claim back a tile later (sccsum.hip,
# flat_body).  No kernel has an atomic it would help: each is one lane's.
DEVICE_FLAGS = ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]


def hipcc_cmd(out: str = LIB_PATH) -> list[str]:
    return [
        HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared",
        "-Wall", "-Wno-unused-command-line-argument", *DEVICE_FLAGS,
        "-I", os.path.join(REPO_DIR, "include"),
        *SOURCES, "-o", out,
    ]


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    headers = [os.path.join(REPO_DIR, "include", h) for h in ("sccsum.h", "sccsum_diag.h")]
    newest = max(os.path.getmtime(p) for p in SOURCES + headers)
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= newest:
        return LIB_PATH
    cmd = hipcc_cmd()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return LIB_PATH
