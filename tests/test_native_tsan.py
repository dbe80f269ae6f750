"""The engine's host code under ThreadSanitizer (tests/native/tsan_engine: the ASan driver's
churn, big epochs that run every parallel commit phase on the engine's helper threads, and the
aggregator with publishers racing a commit).  The HIP / HSA runtime is not instrumented, so
TSan reports races inside it that its own synchronisation rules out; the test fails on any
report whose racing access (frame #0 of either access) is in this repository's code."""
import glob
import os
import re
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "native", "tsan_engine")


@pytest.mark.gpu
def test_host_code_under_tsan():
    if not os.path.exists(DRIVER):
        pytest.fail("tests/native/tsan_engine not built (run __graft_entry__.build())")
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ)
        env["TSAN_OPTIONS"] = f"halt_on_error=0 report_signal_unsafe=0 log_path={d}/tsan"
        p = subprocess.run([DRIVER], capture_output=True, text=True, timeout=300, env=env)
        assert "asan driver ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
        ours = []
        for f in glob.glob(os.path.join(d, "tsan*")):
            for rep in open(f).read().split("==================")[1:]:
                # the two accesses of a data race: their innermost frames
                tops = re.findall(r"(?:Read|Write|Previous read|Previous write|Atomic \w+)[^\n]*\n\s+#0 ([^\n]*)", rep)
                if any("emqx_amd/csrc" in t or "include/emqx" in t for t in tops):
                    ours.append(rep[:1500])
        assert not ours, "\n\n".join(ours[:3])
