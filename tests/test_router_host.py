"""CPU: the host-side mirrors of emqx_router_syncer (stash and batches) and
emqx_broker:aggre/1 — pure host logic, no GPU (the router they feed is a recorder here)."""
from emqx_amd.router import RouterSyncer, aggre


class _Recorder:
    def __init__(self):
        self.batches = []

    def do_batch(self, batch):
        self.batches.append(dict(batch))
        return {}


def test_syncer_last_op_wins_per_route():
    """merge_route_op/2 (emqx_router_syncer.erl:391-401): a later op on the same
    {Topic, Dest} cancels the former; the same action twice is one op."""
    r = _Recorder()
    s = RouterSyncer(r)
    s.push("add", "a/+", "n1")
    s.push("delete", "a/+", "n1")  # cancels the add
    s.push("add", "b/#", "n1")
    s.push("add", "b/#", "n1")     # merged
    s.push("add", "b/#", ("g", "n1"))  # a different route (share dest)
    assert s.run_batch() == 3
    (b,) = r.batches
    assert b[(b"a/+", "n1")] == ("delete",)
    assert b[(b"b/#", "n1")] == ("add",)
    assert b[(b"b/#", ("g", "n1"))] == ("add",)
    assert s.run_batch() == 0


def test_syncer_batches_by_priority_and_size():
    """mk_batch/2 (:297-328): at most max_batch ops per batch, taken hi (reply) > lo (add)
    > bg (delete)."""
    r = _Recorder()
    s = RouterSyncer(r, max_batch=3)
    s.push("delete", "d1", "n")
    s.push("delete", "d2", "n")
    s.push("add", "a1", "n")
    s.push("add", "a2", "n")
    s.push("add", "h1", "n", reply=True)
    assert s.run_batch() == 3
    first = set(r.batches[0])
    assert (b"h1", "n") in first and (b"a1", "n") in first and (b"a2", "n") in first
    s.flush()
    assert set(r.batches[1]) == {(b"d1", "n"), (b"d2", "n")}


def test_aggre_matches_reference():
    """emqx_broker:aggre/1 (emqx_broker.erl:361-377)."""
    assert aggre([]) == []
    assert aggre([(b"t/#", "n1")]) == [(b"t/#", "n1")]
    assert aggre([(b"t/#", ("g1", "n1"))]) == [(b"t/#", "g1")]
    # no share dest: no dedupe, accumulated in reverse
    assert aggre([(b"a", "n1"), (b"b", "n2")]) == [(b"b", "n2"), (b"a", "n1")]
    # a share dest anywhere: usort of {Topic, Node | Group} (two nodes of one group collapse)
    out = aggre([(b"t/+", ("g", "n1")), (b"t/+", ("g", "n2")), (b"t/#", "n1")])
    assert sorted(out) == sorted({(b"t/+", "g"), (b"t/#", "n1")})
    assert len(out) == 2
