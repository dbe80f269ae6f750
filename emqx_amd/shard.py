"""Filter-hash-sharded mode (BASELINE config D; DESIGN.md §6, SURVEY.md §8(e) mode 2).

In the reference every node holds the full route table (mria replication,
apps/emqx/src/emqx_router.erl:133-162) and matching never crosses a node boundary.  When
the filter set outgrows one GPU's budget, this mode splits the route keys instead:

  * key (filter, id) lives on rank shard_of(id) = splitmix64(id) % G, for adds and deletes
    alike, so a delete always reaches the shard that holds its key;
  * every rank matches the WHOLE topic batch against its shard;
  * one exchange step merges the per-shard results: an all-gather of per-topic counts,
    then an all-gather of each rank's topic-major route ids (padded to the largest
    rank's total), then a per-topic concatenation (tm_merge_shards[_device]).  Shards
    are disjoint, so nothing is deduplicated, exactly like one unsharded walk.

On GPUs the exchange runs over RCCL (backend "nccl") on device tensors and the merge is
the HIP kernel behind tm_merge_shards_device.  On CPU (gloo) the host path runs: local
host results, all-gather over gloo, host merge (tm_merge_shards).  The per-shard matcher
is any object with apply_packed / commit / match_ids; the product one is EngineShard.
"""
from __future__ import annotations

import numpy as np

from . import _native as N

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def shard_of(ids, G: int) -> np.ndarray:
    """Rank that owns each route key: splitmix64 finaliser of the id, mod G (the same
    placement csrc/synth.cpp uses when it generates one shard of config D)."""
    x = np.asarray(ids, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return (x % np.uint64(G)).astype(np.int64)


def select_keys(buf, off, ids, mask, flags=None):
    """The packed route keys where mask is true, repacked (bytes, u64 off, u64 ids, flags)."""
    buf = np.asarray(buf, dtype=np.uint8)
    off = np.asarray(off, dtype=np.uint64)
    ids = np.asarray(ids, dtype=np.uint64)
    mask = np.asarray(mask, dtype=bool)
    lens = (off[1:] - off[:-1])[mask]
    starts = off[:-1][mask]
    noff = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(lens, out=noff[1:])
    total = int(noff[-1])
    if total:
        idx = np.repeat(starts - noff[:-1], lens.astype(np.int64)) + np.arange(total, dtype=np.uint64)
        nbuf = buf[idx.astype(np.int64)]
    else:
        nbuf = np.zeros(0, dtype=np.uint8)
    nbuf = np.concatenate([nbuf, np.zeros(16, np.uint8)])
    nfl = None if flags is None else np.asarray(flags, dtype=np.uint32)[mask]
    return nbuf, noff, ids[mask], nfl


class EngineShard:
    """The product per-shard matcher: one HIP engine (one GPU) holding this rank's keys."""

    def __init__(self, engine: "N.Engine"):
        self.eng = engine

    def apply_packed(self, op, buf, off, ids, flags=None):
        self.eng.apply_packed(op, buf, off, ids, flags)

    def commit(self):
        return self.eng.commit()

    def match_ids(self, t_bytes, t_off):
        """Host path: (cnt u32 [n], ids u64 topic-major, status i32 [n])."""
        off, cnt, keys, st = self.eng.match_packed(t_bytes, t_off)
        n = len(cnt)
        total = int(cnt.sum(dtype=np.uint64))
        if total == 0:
            return cnt.astype(np.uint32), np.zeros(0, np.uint64), st
        # topic-major gather of the engine's (wave-ordered) key ranges
        starts = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(cnt, out=starts[1:])
        idx = np.repeat(off.astype(np.int64) - starts[:-1], cnt.astype(np.int64)) + np.arange(total)
        return cnt.astype(np.uint32), self.eng.key_ids(keys[idx]), st


class ShardedIndex:
    """One rank's view of a filter-sharded index over `world` ranks."""

    def __init__(self, shard, rank: int, world: int, group=None):
        self.shard, self.rank, self.world, self.group = shard, rank, world, group

    # ---- writes: every rank sees the same op stream and keeps its own keys
    def apply_packed(self, op, buf, off, ids, flags=None):
        mask = shard_of(ids, self.world) == self.rank
        b, o, i, f = select_keys(buf, off, ids, mask, flags)
        self.shard.apply_packed(op, b, o, i, f)

    def commit(self):
        return self.shard.commit()

    # ---- host path (gloo or nccl)
    def match(self, t_bytes, t_off):
        """Match the whole batch on every rank; returns the merged (off[n+1] u32, ids u64,
        status i32[n]) on every rank."""
        import torch
        import torch.distributed as dist
        cnt, ids, st = self.shard.match_ids(t_bytes, t_off)
        n = len(cnt)
        if self.world == 1:
            return N.merge_shards(cnt.reshape(1, n), ids.reshape(1, -1)) + (st,)
        dev = torch.device("cpu")
        if dist.get_backend(self.group) != "gloo":
            dev = torch.device("cuda", torch.cuda.current_device())
        c = torch.from_numpy(cnt.view(np.int32).copy()).to(dev)
        C = torch.empty(self.world * n, dtype=torch.int32, device=dev)  # flat: gloo and RCCL alike
        dist.all_gather_into_tensor(C, c, group=self.group)
        C = C.view(self.world, n)
        totals = C.to(torch.int64).sum(1)
        maxT = max(int(totals.max().item()), 1)
        mine = torch.zeros(maxT, dtype=torch.int64, device=dev)
        if len(ids):
            mine[:len(ids)] = torch.from_numpy(ids.view(np.int64)).to(dev)
        Ids = torch.empty(self.world * maxT, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(Ids, mine, group=self.group)
        Ids = Ids.view(self.world, maxT)
        off, merged = N.merge_shards(C.cpu().numpy().view(np.uint32), Ids.cpu().numpy().view(np.uint64))
        return off, merged, st

    # ---- device path (RCCL over xGMI)
    def match_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int):
        """GPU path: local walk, ids compacted on device, RCCL all-gathers, device merge.
        The engine calls and the torch ops between them all run on ONE torch stream (the
        engine's own stream is non-blocking, so torch's legacy default stream would not
        order after it); the caller's current stream waits for it before this returns.
        Returns device tensors (off[n+1] i32, ids i64 holding u64 route ids)."""
        import torch
        import torch.distributed as dist
        dev = torch.device("cuda", torch.cuda.current_device())
        caller = torch.cuda.current_stream()
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream(dev)
        s = self._stream
        s.wait_stream(caller)  # the topic batch was written on the caller's stream
        sp = s.cuda_stream
        with torch.cuda.stream(s):
            r = eng.match_device(d_bytes, d_off, n, total_bytes, sp)
            eng.device_sync()
            total = _read_u64(r.d_total)
            if total > r.keys_cap:
                eng.reserve_matches(int(total * 1.1) + 1024)
                r = eng.match_device(d_bytes, d_off, n, total_bytes, sp)
                eng.device_sync()
                total = _read_u64(r.d_total)
            loc_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
            maxT = torch.tensor([total], dtype=torch.int64, device=dev)
            if self.world > 1:
                dist.all_reduce(maxT, op=dist.ReduceOp.MAX, group=self.group)
            stride = max(int(maxT.item()), 1)
            mine = torch.zeros(stride, dtype=torch.int64, device=dev)
            eng.result_ids_device(mine.data_ptr(), stride, loc_off.data_ptr(), sp)
            cnt = (loc_off[1:] - loc_off[:-1]).contiguous()
            if self.world > 1:
                C = torch.empty(self.world * n, dtype=torch.int32, device=dev)
                dist.all_gather_into_tensor(C, cnt, group=self.group)
                Ids = torch.empty(self.world * stride, dtype=torch.int64, device=dev)
                dist.all_gather_into_tensor(Ids, mine, group=self.group)
            else:  # one shard: the exchange is the identity
                C, Ids = cnt, mine
            out_total = int(C.to(torch.int64).sum().item())
            out_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
            out_ids = torch.empty(max(out_total, 1), dtype=torch.int64, device=dev)
            eng.merge_shards_device(self.world, n, C.data_ptr(), Ids.data_ptr(), stride, out_off.data_ptr(),
                                    out_ids.data_ptr(), out_total, sp)
        caller.wait_stream(s)
        return out_off, out_ids[:out_total]


def _read_u64(ptr: int) -> int:
    """One u64 from device memory (a batch's requested-keys counter)."""
    import ctypes as C

    import torch
    h = torch.empty(1, dtype=torch.int64)
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    rc = lib.hipMemcpy(C.c_void_p(h.data_ptr()), C.c_void_p(ptr), 8, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError(f"hipMemcpy D2H failed: {rc}")
    return int(h.item())
