"""Reads of device memory nothing wrote (round 6).  With EMQX_TM_POISON=1 every device buffer
the engine allocates starts as 0xA7 bytes instead of the zeros a fresh page holds, so a kernel
that reads a counter block, an output slot or a key record before anything wrote it returns
garbage instead of a lucky zero.  tools/poison_probe.py runs config A (ids past 32 bits, then
small ids; the device walk as the engine's first launch, and after a host-form batch) in a
child process (the knob is read once per process) and reports, per check, the topics whose
route ids differ from the oracle's."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_poisoned_allocations_change_no_result():
    env = dict(os.environ, EMQX_TM_POISON="1")
    out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "poison_probe.py")], env=env, cwd=ROOT,
                         capture_output=True, text=True, timeout=220)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    checks = [r for r in recs if "check" in r]
    assert recs[0] == {"poison": "1"}
    assert len(checks) == 7, recs  # per run the key form and the id forms: u64 (big ids, twice), u32 + u64
    for r in checks:
        assert r["bad_topics"] == 0, r
        assert r.get("flags", 0) == 0, r
    assert all(r["image_check"] == [] for r in recs if "image_check" in r)
