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
    def prepare_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int,
                       headroom: float = 1.25):
        """Size this rank's output arena and the exchange stride from one synchronous run of
        the batch (collective when world > 1).  Not part of the step: the step itself never
        waits on the host; a later batch that outgrows these sizes is flagged on the device
        (match_device's third result) and re-run by the caller after prepare_device."""
        import torch
        import torch.distributed as dist
        dev = torch.device("cuda", torch.cuda.current_device())
        torch.cuda.current_stream().synchronize()
        r = eng.match_device(d_bytes, d_off, n, total_bytes, 0)
        eng.device_sync()  # also sizes the chunk pools to this batch's demand
        total = _read_u64(r.d_total)
        eng.reserve_matches(int(total * headroom) + 1024)
        t = torch.tensor([total], dtype=torch.int64, device=dev)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.stride = int(int(t.item()) * headroom) + 1024
        return total

    def local_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int, sp: int):
        """This rank's half of the step, queued on stream `sp` with no host sync: the walk,
        then the route ids compacted topic-major (tm_result_ids_device_ex).  Returns
        (cnt_ext i32[n+1]: per-topic counts + the TM_RES_* overflow flags, ids i64[stride])."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        eng.match_device(d_bytes, d_off, n, total_bytes, sp)
        lo = torch.empty(n + 1, dtype=torch.int32, device=dev)
        ids = torch.empty(self.stride, dtype=torch.int64, device=dev)
        cnt_ext = torch.empty(n + 1, dtype=torch.int32, device=dev)
        eng.result_ids_device_ex(ids.data_ptr(), self.stride, lo.data_ptr(), cnt_ext[n:].data_ptr(), sp)
        torch.sub(lo[1:], lo[:-1], out=cnt_ext[:n])
        return cnt_ext, ids

    def merge_device(self, eng: "N.Engine", C_ext, Ids, G: int, n: int, sp: int):
        """Concatenate G shards' slices per topic on the device.  C_ext: (G, n+1) i32 (counts
        + flags rows), Ids: (G * stride) i64.  Returns (off i32[n+1], ids i64 buffer whose first
        off[n] entries are the result, flags i32[1]: nonzero if any shard overflowed)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        C = C_ext[:, :n].contiguous()
        flags = C_ext[:, n].max().reshape(1)
        out_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
        cap = G * self.stride
        out_ids = torch.empty(cap, dtype=torch.int64, device=dev)
        eng.merge_shards_device(G, n, C.data_ptr(), Ids.data_ptr(), self.stride, out_off.data_ptr(),
                                out_ids.data_ptr(), cap, sp)
        return out_off, out_ids, flags

    def match_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int):
        """GPU step: local walk, ids compacted on device, RCCL all-gathers of the counts and of
        the ids (padded to the stride prepare_device fixed), device merge.  Nothing in it
        waits on the host.  The engine calls and the torch ops between them run on ONE torch
        stream (the engine's own stream is non-blocking, so torch's legacy default stream
        would not order after it); the caller's current stream waits for it before this
        returns.  Returns device tensors (off i32[n+1], ids i64 buffer holding off[n] u64
        route ids, flags i32[1]); flags != 0 means a shard outgrew its sizes: call
        prepare_device again and re-run the batch."""
        import torch
        import torch.distributed as dist
        if getattr(self, "stride", None) is None:
            self.prepare_device(eng, d_bytes, d_off, n, total_bytes)
        dev = torch.device("cuda", torch.cuda.current_device())
        caller = torch.cuda.current_stream()
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream(dev)
        s = self._stream
        s.wait_stream(caller)  # the topic batch was written on the caller's stream
        sp = s.cuda_stream
        with torch.cuda.stream(s):
            cnt_ext, ids = self.local_device(eng, d_bytes, d_off, n, total_bytes, sp)
            if self.world > 1:
                C = torch.empty(self.world * (n + 1), dtype=torch.int32, device=dev)
                dist.all_gather_into_tensor(C, cnt_ext, group=self.group)
                Ids = torch.empty(self.world * self.stride, dtype=torch.int64, device=dev)
                dist.all_gather_into_tensor(Ids, ids, group=self.group)
            else:  # one shard: the exchange is the identity
                C, Ids = cnt_ext, ids
            out = self.merge_device(eng, C.view(self.world, n + 1), Ids, self.world, n, sp)
        caller.wait_stream(s)
        for t in out:
            t.record_stream(caller)  # consumed on the caller's stream from here on
        return out


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
