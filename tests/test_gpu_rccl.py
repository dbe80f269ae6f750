"""The RCCL backend (torch.distributed "nccl" on ROCm) on the real device, at world size 1:
the GPU box has one MI355X and RCCL refuses two ranks on one GPU, so this is the most of the
multi-GPU path one box can run.  What it pins:
  - the process group comes up over RCCL and its collectives run on the engine's tensors
    (all-gather, all-to-all with explicit split sizes, broadcast, all-reduce MAX: the calls
    emqx_amd/shard.py and emqx_amd/replica.py make);
  - mode 2's a2a exchange (ShardedIndex._exchange_a2a: two all-gathers / all-to-alls and the
    device merge) over RCCL gives the oracle's route-id sets;
  - mode 1's image shipped through an RCCL broadcast loads as a replica that matches like
    the master.
The exchanges between different ranks are covered by the gloo world-2 tests
(tests/test_shard.py, tests/test_replica.py)."""
import socket

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import shard as S
from emqx_amd import workloads

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl():
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_on_device_tensors(rccl):
    import torch
    import torch.distributed as dist
    assert dist.get_backend() == "nccl"
    x = torch.arange(1000, dtype=torch.int32, device=rccl)
    g = torch.empty_like(x)
    dist.all_gather_into_tensor(g, x)
    assert torch.equal(g, x)
    y = torch.empty(700, dtype=torch.int64, device=rccl)
    src = torch.arange(900, dtype=torch.int64, device=rccl)
    dist.all_to_all_single(y, src[100:800].contiguous(), [700], [700])
    assert torch.equal(y, src[100:800])
    m = torch.tensor([3, 9, 4], dtype=torch.int64, device=rccl)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    assert m.tolist() == [3, 9, 4]
    torch.cuda.synchronize()


def test_a2a_exchange_over_rccl_matches_oracle(rccl):
    import torch
    w = workloads.generate("B", scale=0.05, n_topics=20000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    n = w.n_topics
    d_bytes = torch.from_numpy(w.t_bytes).to(rccl)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(rccl)
    tb = int(w.t_off[-1])
    six = S.ShardedIndex(S.EngineShard(eng), 0, 1, exchange="a2a")
    six.prepare_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb)
    s = torch.cuda.Stream(rccl)
    with torch.cuda.stream(s):
        hdr, ids = six.local_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, s.cuda_stream)
        H, Ids, bases = six._exchange_a2a(hdr, ids, n)  # the RCCL all-gather + all-to-alls
        off, out, flags = six.merge_device(eng, H, Ids, bases, n, s.cuda_stream)
    torch.cuda.synchronize()
    assert int(flags.max().item()) == 0
    o = off.cpu().numpy().view(np.uint32)
    got = out[:int(o[-1])].cpu().numpy().view(np.uint64)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eoff, eids, _ = ix.match(w.t_bytes, w.t_off, threads=8)
    assert np.array_equal(np.diff(o.astype(np.int64)), np.diff(eoff.astype(np.int64)))
    for t in range(n):
        assert np.array_equal(np.sort(got[o[t]:o[t + 1]]), eids[eoff[t]:eoff[t + 1]]), t
    # the step itself (world 1: no collective) agrees with the exchange path
    off2, out2, _ = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange="padded")
    torch.cuda.synchronize()
    o2 = off2.cpu().numpy().view(np.uint32)
    assert np.array_equal(o2, o)
    assert np.array_equal(out2[:int(o2[-1])].cpu().numpy().view(np.uint64), got)
    eng.close()


def test_replica_image_through_rccl_broadcast(rccl):
    import torch
    import torch.distributed as dist
    w = workloads.generate("E", scale=0.02, n_topics=5000)
    master = N.Engine(0, record_patch=True)
    master.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    master.commit()
    size = master.image_size()
    img = torch.empty(size, dtype=torch.uint8, device=rccl)
    torch.cuda.synchronize()
    master.image_export(img.data_ptr(), size)
    recv = img.clone()
    dist.broadcast(recv, src=0)  # what ReplicatedIndex._bcast sends to every replica
    torch.cuda.synchronize()
    assert torch.equal(recv, img)
    rep = N.Engine.replica_from_image(0, recv.data_ptr(), recv.numel())
    from test_replica import _sets  # statuses and id lists through the device path (replicas too)
    ms, mids = _sets(master, w)
    rs, rids = _sets(rep, w)
    assert np.array_equal(ms, rs) and mids == rids
    assert sum(len(x) for x in mids) > 0
    rep.close()
    master.close()
