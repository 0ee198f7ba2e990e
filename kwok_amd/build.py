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
DOM_HDR = os.path.join(PKG, "csrc", "json_dom.hpp")
ENC_SRC = [os.path.join(PKG, "csrc", "encoder.cpp")]
ENC_HDR = [os.path.join(ROOT, "include", "kwok_encoder.h"), os.path.join(ROOT, "include", "kwok_engine.h"), DOM_HDR,
           os.path.join(PKG, "csrc", "host_common.hpp"), os.path.join(PKG, "csrc", "nextstate.hpp"),
           os.path.join(PKG, "csrc", "gotpl.hpp"), os.path.join(PKG, "csrc", "labelsel.hpp")]
ENC_OUT = os.path.join(PKG, "lib", "libkwok_encoder.so")
PATCH_SRC = [os.path.join(PKG, "csrc", "patch.cpp")]
PATCH_HDR = [os.path.join(ROOT, "include", "kwok_patch.h"), os.path.join(ROOT, "include", "kwok_engine.h"), DOM_HDR,
             os.path.join(PKG, "csrc", "timefmt.hpp")]
PATCH_OUT = os.path.join(PKG, "lib", "libkwok_patch.so")
COMPILER_SRC = [os.path.join(PKG, "csrc", "compiler.cpp"), os.path.join(PKG, "csrc", "metrics_compiler.cpp")]
COMPILER_HDR = [os.path.join(ROOT, "include", "kwok_compiler.h"), os.path.join(ROOT, "include", "kwok_metrics.h"),
                os.path.join(ROOT, "include", "kwok_engine.h"), DOM_HDR] + \
    [os.path.join(PKG, "csrc", h) for h in ("host_common.hpp", "gotpl.hpp", "patchtpl.hpp", "nextstate.hpp", "labelsel.hpp",
                                            "celc.hpp")]
COMPILER_OUT = os.path.join(PKG, "lib", "libkwok_compiler.so")
COMM_SRC = [os.path.join(PKG, "csrc", "comm.cpp")]
COMM_HDR = [os.path.join(ROOT, "include", "kwok_comm.h"), os.path.join(ROOT, "include", "kwok_engine.h")]
COMM_OUT = os.path.join(PKG, "lib", "libkwok_comm.so")
EMIT_SRC = [os.path.join(PKG, "csrc", "emit.hip")]
EMIT_HDR = [os.path.join(ROOT, "include", "kwok_emit.h"), os.path.join(ROOT, "include", "kwok_engine.h"),
            os.path.join(PKG, "csrc", "timefmt.hpp")]
EMIT_OUT = os.path.join(PKG, "lib", "libkwok_emit.so")
ARCH = "gfx950"  # MI355X only


def _stale(out, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in srcs)


def _host_lib(out, srcs, hdrs, force, verbose) -> str:
    """A host-only C++ library (no device code)."""
    if not force and not _stale(out, srcs + hdrs):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-I", os.path.join(ROOT, "include"),
           "-o", out + ".tmp"] + srcs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_encoder(force: bool = False, verbose: bool = False) -> str:
    """The native ingestion encoder."""
    return _host_lib(ENC_OUT, ENC_SRC, ENC_HDR, force, verbose)


def build_compiler(force: bool = False, verbose: bool = False) -> str:
    """The native Stage compiler (lifecycle.NewLifecycle behind the C ABI) and Metric CR compiler
    (kwok_metrics.h)."""
    return _host_lib(COMPILER_OUT, COMPILER_SRC, COMPILER_HDR, force, verbose)


def build_patch(force: bool = False, verbose: bool = False) -> str:
    """The native patch renderer (precompiled merge-patch byte templates)."""
    return _host_lib(PATCH_OUT, PATCH_SRC, PATCH_HDR, force, verbose)


def build_comm(force: bool = False, verbose: bool = False) -> str:
    """The RCCL cluster-aggregate collective (host code over librccl + the engine's streams)."""
    if not force and not _stale(COMM_OUT, COMM_SRC + COMM_HDR + [OUT]):
        return COMM_OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result",
           "-Wno-unused-value", "-I", os.path.join(ROOT, "include"),
           "-o", COMM_OUT + ".tmp"] + \
        COMM_SRC + ["-L", os.path.dirname(OUT), "-lkwok_engine", "-lrccl", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(COMM_OUT + ".tmp", COMM_OUT)
    return COMM_OUT


def build_emit(force: bool = False, verbose: bool = False) -> str:
    """The device patch emitter (HIP kernels over the engine's fired lists, linked to the engine)."""
    if not force and not _stale(EMIT_OUT, EMIT_SRC + EMIT_HDR + [OUT]):
        return EMIT_OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result",
           "-Wno-unused-value", "-I", os.path.join(ROOT, "include"), "-o", EMIT_OUT + ".tmp"] + \
        EMIT_SRC + ["-L", os.path.dirname(OUT), "-lkwok_engine", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(EMIT_OUT + ".tmp", EMIT_OUT)
    return EMIT_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_encoder(force, verbose)
    build_compiler(force, verbose)
    if os.path.exists(PATCH_SRC[0]):
        build_patch(force, verbose)
    _build_engine(force, verbose)
    build_comm(force, verbose)
    build_emit(force, verbose)
    return OUT


def _build_engine(force: bool = False, verbose: bool = False) -> str:
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
