"""CPU: the C-ABI library loads, exports every symbol include/emqx_tm.h declares, and
fails loudly (TM_EDEVICE) when no gfx950 device is present — no silent CPU fallback.
No compute calls here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from emqx_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "emqx_tm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tm_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_surface():
    decl = _declared()
    assert set(decl) == set(N.EXPORTS), (decl, N.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = N.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH]).decode()
    exported = set(re.findall(r" T (tm_\w+)", out))
    for name in _declared():
        assert name in exported, name
        assert getattr(lib, name) is not None
    assert lib.tm_abi_version() == 10
    assert C.sizeof(N.tm_stats_t) == 21 * 8  # mirrors tm_stats_t in include/emqx_tm.h
    assert C.sizeof(N.tm_config) == 11 * 4
    assert C.sizeof(N.tm_runs_result) == 9 * 8 and C.sizeof(N.tm_span) == 16


def test_kernels_are_gfx950_code_objects():
    out = subprocess.check_output(["strings", N.LIB_PATH]).decode(errors="replace")
    assert "amdgcn-amd-amdhsa--gfx950" in out
    assert "k_match_fast" in out and "k_match_slow" in out


def test_create_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    cfg = N.tm_config()
    h = C.c_void_p()
    rc = N.load().tm_create(C.byref(cfg), C.byref(h))
    assert rc == N.TM_EDEVICE and not h.value
    # the calling thread's reason for the failed create (tm_create_last_error, round 6)
    assert N.load().tm_create_last_error() == b"tm_create: no such HIP device"
    with pytest.raises(N.TMError) as e:
        N.Engine(0)
    assert "no such HIP device" in str(e.value)


def test_null_and_bad_args_are_rejected_without_device():
    lib = N.load()
    assert lib.tm_apply(None, None, 0) == N.TM_EINVAL
    assert lib.tm_commit_epoch(None, None) == N.TM_EINVAL
    assert lib.tm_stats(None, None) == N.TM_EINVAL
    assert lib.tm_match_batch(None, None, None, 0, 0, None) == N.TM_EINVAL
    assert lib.tm_last_error(None) == b"null engine"


def test_pack_topics_layout():
    buf, off = N.pack_topics([b"a/b", "", b"$SYS/x"])
    assert off.tolist() == [0, 3, 3, 9]
    assert bytes(buf[:9]) == b"a/b$SYS/x"
