"""Build the native libraries in-tree (they travel to the GPU box with the snapshot).

  libemqx_tm.so     the product: host engine (engine.cpp) + gfx950 kernels
                    (match_kernels.hip), C-ABI in include/emqx_tm.h
  libemqx_synth.so  seeded workload generator (tests / bench only)
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(out, srcs):
    return os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(s) for s in srcs)


TM_SRCS = ("emqx_amd/csrc/engine.cpp", "emqx_amd/csrc/batcher.cpp", "emqx_amd/csrc/match_kernels.hip",
           "emqx_amd/csrc/result_kernels.hip", "emqx_amd/csrc/filter_kernels.hip", "emqx_amd/csrc/layout.h",
           "emqx_amd/csrc/device_api.h", "emqx_amd/csrc/copy_api.h", "emqx_amd/csrc/image_api.h", "emqx_amd/csrc/filter_api.h", "emqx_amd/csrc/wave.h", "include/emqx_tm.h",
           "include/emqx_tm_batcher.h")


def src_sha() -> str:
    """sha256 over the product library's sources (path + content of each): embedded in the
    library at build time (tm_build_info), compared by build(), smoke() and bench.py."""
    import hashlib
    root = os.path.dirname(HERE)
    h = hashlib.sha256()
    for f in TM_SRCS:
        h.update(f.encode() + b"\0")
        h.update(open(os.path.join(root, f), "rb").read())
    return h.hexdigest()


def built_sha(lib_path: str):
    """The source hash a built libemqx_tm.so carries (None if it has none or cannot load).
    Read in a child process: loading the HIP library here would pin it in this process."""
    import subprocess
    if not os.path.exists(lib_path):
        return None
    code = ("import ctypes,sys; l=ctypes.CDLL(sys.argv[1]); l.tm_build_info.restype=ctypes.c_char_p; "
            "print(l.tm_build_info().decode())")
    try:
        out = subprocess.run([sys.executable, "-c", code, lib_path], capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.SubprocessError):
        return None
    for tok in out.stdout.split():
        if tok.startswith("src_sha="):
            return tok[len("src_sha="):]
    return None


def build(force: bool = False, verbose: bool = True):
    tm = os.path.join(HERE, "libemqx_tm.so")
    sha = src_sha()  # over TM_SRCS, the one list of the library's sources
    # rebuilt whenever the library's embedded source hash differs from the sources' (not mtimes:
    # the tree travels to the GPU box with its built library)
    if force or built_sha(tm) != sha:
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
               f'-DTM_SRC_SHA="{sha}"',
               "-Wno-unused-function", os.path.join(CSRC, "engine.cpp"), os.path.join(CSRC, "batcher.cpp"),
               os.path.join(CSRC, "match_kernels.hip"),
               os.path.join(CSRC, "result_kernels.hip"), os.path.join(CSRC, "filter_kernels.hip"), "-o", tm]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    # the bounds-checked debug build of the same sources (TM_BOUNDS=1): tests that
    # load it set EMQX_TM_LIB to it; never the product path
    tmb = os.path.join(HERE, "libemqx_tm_bounds.so")
    if force or built_sha(tmb) != sha:
        cmd = [HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-DTM_BOUNDS=1",
               f'-DTM_SRC_SHA="{sha}"',
               "-Wno-unused-function", os.path.join(CSRC, "engine.cpp"), os.path.join(CSRC, "batcher.cpp"),
               os.path.join(CSRC, "match_kernels.hip"),
               os.path.join(CSRC, "result_kernels.hip"), os.path.join(CSRC, "filter_kernels.hip"), "-o", tmb]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    syn = os.path.join(HERE, "libemqx_synth.so")
    ssrc = [os.path.join(CSRC, "synth.cpp")]
    if force or not _newer(syn, ssrc):
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", ssrc[0], "-o", syn]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    # bench tooling (not product code): closed-loop publisher load for the batching aggregator
    lg = os.path.join(os.path.dirname(HERE), "tools", "libtm_loadgen.so")
    lsrc = [os.path.join(os.path.dirname(HERE), "tools", "loadgen.cpp"),
            os.path.join(os.path.dirname(HERE), "include", "emqx_tm_batcher.h")]
    if force or not _newer(lg, lsrc):
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", lsrc[0], "-o", lg, tm, "-Wl,-rpath,$ORIGIN/../emqx_amd"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    return tm, syn


if __name__ == "__main__":
    build(force="--force" in sys.argv)
