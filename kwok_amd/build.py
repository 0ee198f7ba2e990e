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
ENC_SRC = [os.path.join(PKG, "csrc", "encoder.cpp")]
ENC_HDR = [os.path.join(ROOT, "include", "kwok_encoder.h"), os.path.join(ROOT, "include", "kwok_engine.h")]
ENC_OUT = os.path.join(PKG, "lib", "libkwok_encoder.so")
ARCH = "gfx950"  # MI355X only


def _stale(out, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in srcs)


def build_encoder(force: bool = False, verbose: bool = False) -> str:
    """The native ingestion encoder: host C++ (no device code)."""
    if not force and not _stale(ENC_OUT, ENC_SRC + ENC_HDR):
        return ENC_OUT
    os.makedirs(os.path.dirname(ENC_OUT), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-I", os.path.join(ROOT, "include"),
           "-o", ENC_OUT + ".tmp"] + ENC_SRC
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(ENC_OUT + ".tmp", ENC_OUT)
    return ENC_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_encoder(force, verbose)
    if not force and not _stale(OUT, SRC + HDR):
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
