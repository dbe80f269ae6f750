"""GPU parity of emqx_topic:intersection/2 (tm_intersect_batch, filter_kernels.hip
k_intersect) against the oracle's restatement (oracle/emqx_topic.py), which
test_oracle_golden.py pins to the reference's KATs (emqx_topic_SUITE t_intersect).  Byte
results, exact."""
import random

import pytest

from emqx_amd import _native as N
from oracle import emqx_topic as et

pytestmark = pytest.mark.gpu


def _oracle(a, b):
    try:
        return et.intersection(a, b)
    except et.TopicError:
        return "badhash"


def _gpu(eng, pairs):
    return ["badhash" if isinstance(r, N.TopicInvalidHash) else r for r in eng.intersect(pairs)]


def test_intersection_kats(golden):
    eng = N.Engine(0)
    kats = golden("kat_topic.json")["intersection"]
    pairs = [(a.encode(), b.encode()) for a, b, _ in kats]
    pairs += [(b, a) for a, b in pairs]  # commutative
    exp = [(e.encode() if e else False) for _, _, e in kats] * 2
    assert _gpu(eng, pairs) == exp


@pytest.mark.parametrize("seed", range(4))
def test_intersection_random_vs_oracle(seed):
    rng = random.Random(0x1A7E + seed)
    vocab = [b"a", b"b", b"", b"$SYS", b"$x", b"+", b"#", b"long-level-word"]

    def topic():
        return b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 5)))

    pairs = [(topic(), topic()) for _ in range(4000)]
    pairs += [(b"", b""), (b"#", b""), (b"+", b""), (b"a/#", b"#/b"), (b"#/a", b"#/a")]
    eng = N.Engine(0)
    got = _gpu(eng, pairs)
    for (a, b), g in zip(pairs, got):
        assert g == _oracle(a, b), (a, b, g)


def test_intersection_empty_batch():
    assert N.Engine(0).intersect([]) == []
