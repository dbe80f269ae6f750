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


def build(force: bool = False, verbose: bool = True):
    tm = os.path.join(HERE, "libemqx_tm.so")
    srcs = [os.path.join(CSRC, f) for f in ("engine.cpp", "batcher.cpp", "match_kernels.hip",
                                            "result_kernels.hip", "filter_kernels.hip", "layout.h", "device_api.h", "filter_api.h",
                                            "wave.h")]
    srcs += [os.path.join(os.path.dirname(HERE), "include", h) for h in ("emqx_tm.h", "emqx_tm_batcher.h")]
    if force or not _newer(tm, srcs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
               "-Wno-unused-function", os.path.join(CSRC, "engine.cpp"), os.path.join(CSRC, "batcher.cpp"),
               os.path.join(CSRC, "match_kernels.hip"),
               os.path.join(CSRC, "result_kernels.hip"), os.path.join(CSRC, "filter_kernels.hip"), "-o", tm]
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
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", lsrc[0], "-o", lg, tm, "-Wl,-rpath,$ORIGIN/../emqx_amd"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    return tm, syn


if __name__ == "__main__":
    build(force="--force" in sys.argv)
