import os
import sys

import pytest

# torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's): whichever is loaded
# first serves the whole process.  Load torch's before libemqx_tm.so so that GPU tests
# that mix torch device tensors with the engine run on one HIP runtime (bench.py and
# __graft_entry__ already import in that order or do not use torch at all).
# Several host-form callers at once (tests/test_gpu_concurrency.py) each use their own streams;
# HIP's default of 4 hardware queues per process would put streams of different threads on one
# in-order queue.  bench.py asks for 8 as well.  Set before HIP starts.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402,F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; parity tests through the C-ABI")


GOLDEN = os.path.join(ROOT, "tests", "golden")


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


# Under the bounds-checked debug build (EMQX_TM_LIB=.../libemqx_tm_bounds.so)
# every GPU test also fails if it made the library record an out-of-bounds device index, a
# written canary tail or a host copy past a buffer's end.
_BOUNDS_SEEN = [0]


@pytest.fixture(autouse=True)
def _bounds_guard():
    yield
    if "bounds" not in os.path.basename(os.environ.get("EMQX_TM_LIB", "")):
        return
    from emqx_amd import _native as N
    if N._lib is None:
        return
    r = N.debug_bounds()
    if r is not None and r[0] > _BOUNDS_SEEN[0]:
        _BOUNDS_SEEN[0] = r[0]
        pytest.fail(f"bounds build: {r[0]} findings: {r[1]}")


_MEM_LOG = os.environ.get("EMQX_TM_TEST_MEMLOG", "")


@pytest.fixture(autouse=True)
def _device_memory_release(request):
    """After every GPU test: collect the engines a test left unreferenced (their __del__ closes
    them) and hand torch's cached blocks back, so one test's HBM is free for the next (the
    full-size config-D tests need tens of GiB).  EMQX_TM_TEST_MEMLOG=<file> records the free HBM
    after each test, to find a test that keeps device memory."""
    yield
    if request.node.get_closest_marker("gpu") is None or not torch.cuda.is_initialized():
        return
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if _MEM_LOG:
        free, total = torch.cuda.mem_get_info(0)
        with open(_MEM_LOG, "a") as f:
            f.write(f"{free / 2**30:9.2f} GiB free of {total / 2**30:.1f}  {request.node.nodeid}\n")


def pytest_terminal_summary(terminalreporter):
    """Under EMQX_TM_LIB: which library the run mapped, and (bounds build) its findings."""
    if not os.environ.get("EMQX_TM_LIB"):
        return
    from emqx_amd import _native as N
    if N._lib is None:
        return
    r = N.debug_bounds()
    terminalreporter.write_line(f"library {N.LIB_PATH}: bounds checks {'active' if r is not None else 'absent'}"
                                + (f", {r[0]} findings{': ' + r[1] if r[0] else ''}" if r is not None else ""))
