"""Host placement (emqx_amd/placement.py): which cores a quota-sized pin takes."""
from emqx_amd import placement as P


def fake_core(c):  # 8 cores, CPU c and c + 8 are SMT siblings
    return ("0", str(c % 8))


def test_pick_cores_one_per_core_first():
    assert P.pick_cores(list(range(16)), 4, {}, 0, fake_core) == [0, 1, 2, 3]
    # siblings only once every core has one CPU taken
    assert P.pick_cores(list(range(16)), 10, {}, 0, fake_core) == list(range(10))


def test_pick_cores_skips_busy_cores():
    busy = {0: 1.0, 1: 0.9, 9: 0.8, 2: 0.5}  # cores 0, 1 (CPUs 1 and 9) and 2 are in use
    assert P.pick_cores(list(range(16)), 4, busy, 0, fake_core) == [3, 4, 5, 6]
    # a core whose sibling is busy counts as busy
    assert 1 not in P.pick_cores(list(range(16)), 7, {9: 1.0}, 0, fake_core)


def test_pick_cores_per_gpu_offset():
    a = P.pick_cores(list(range(16)), 4, {}, 0, fake_core)
    b = P.pick_cores(list(range(16)), 4, {}, 4, fake_core)
    assert not set(a) & set(b)


def test_cpu_busy_reads_proc_stat():
    b = P.cpu_busy([0], interval=0.05)
    assert set(b) <= {0} and all(0.0 <= v <= 1.0 for v in b.values())
