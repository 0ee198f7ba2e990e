"""Build the HIP engine library in-tree for gfx950 (explicit hipcc, no JIT cache).

    python -m kwok_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = [os.path.join(PKG, "csrc", "engine.hip")]
HDR = [os.path.join(ROOT, "include", "kwok_engine.h")]
OUT = os.path.join(PKG, "lib", "libkwok_engine.so")
ARCH = "gfx950"  # MI355X only


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRC + HDR)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-unused-value", "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
