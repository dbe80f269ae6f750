"""Filter-hash-sharded mode (BASELINE config D; DESIGN.md §6, SURVEY.md §8(e) mode 2).

In the reference every node holds the full route table (mria replication,
apps/emqx/src/emqx_router.erl:133-162) and matching never crosses a node boundary.  When
the filter set outgrows one GPU's budget, this mode splits the route keys instead:

  * key (filter, id) lives on rank shard_of(id) = splitmix64(id) % G, for adds and deletes
    alike, so a delete always reaches the shard that holds its key;
  * every rank matches the WHOLE topic batch against its shard; the walk writes route ids
    (u32 while they fit) compacted topic-major (tm_match_ids_device);
  * one exchange step (ShardedIndex docstring: padded / exact / local) and a per-topic
    concatenation (tm_merge_shard_ids_device).  Shards are disjoint, so nothing is
    deduplicated, exactly like one unsharded walk.

On GPUs the exchange runs over RCCL (backend "nccl") on device tensors and the merge is
the HIP kernel behind tm_merge_shard_ids_device.  On CPU (gloo) the host path runs: local
host results, the same exchange over gloo, the host form of the merge
(merge_shard_ids_host).  The per-shard matcher is any object with apply_packed / commit /
match_ids; the product one is EngineShard.
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


EXCHANGES = ("padded", "exact", "local", "a2a")


def merge_shard_ids_host(H, ids, bases, n: int):
    """Host form of the device merge (tm_merge_shard_ids_device, result_kernels.hip
    k_merge_flat): H (G, n+2) u32 rows [topic-major offsets (n+1) | flags], rank r's ids at
    ids[bases[r]:].  Returns (off u32[n+1], merged u64 ids): topic t's ids are the
    concatenation of its slices from rank 0..G-1."""
    H = np.asarray(H).view(np.uint32).reshape(len(bases), -1)
    ids = np.asarray(ids)
    G = len(bases)
    roff = H[:, :n + 1].astype(np.int64)
    cnt = np.diff(roff, axis=1)
    off = roff.sum(0)
    out = np.zeros(int(off[-1]), dtype=np.uint64)
    before = np.zeros(n, dtype=np.int64)  # ids of ranks < r in each topic
    for r in range(G):
        c = cnt[r]
        tot = int(c.sum())
        if tot:
            t_of = np.repeat(np.arange(n), c)
            k = np.arange(tot) - np.repeat(roff[r, :-1] - roff[r, 0], c)
            src = int(bases[r]) + roff[r, :-1][t_of] + k
            out[off[:-1][t_of] + before[t_of] + k] = ids[src].astype(np.uint64)
        before += c
    return off.astype(np.uint32), out


class EngineShard:
    """The product per-shard matcher: one HIP engine (one GPU) holding this rank's keys."""

    def __init__(self, engine: "N.Engine"):
        self.eng = engine

    def apply_packed(self, op, buf, off, ids, flags=None):
        self.eng.apply_packed(op, buf, off, ids, flags)

    def commit(self):
        return self.eng.commit()

    def match_ids(self, t_bytes, t_off):
        """Host path: (topic-major offsets u32 [n+1], ids u64, status i32 [n])."""
        off, cnt, keys, st = self.eng.match_packed(t_bytes, t_off)
        n = len(cnt)
        starts = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(cnt, out=starts[1:])
        total = int(starts[-1])
        if total == 0:
            return starts.astype(np.uint32), np.zeros(0, np.uint64), st
        # topic-major gather of the engine's (wave-ordered) key ranges
        idx = np.repeat(off.astype(np.int64) - starts[:-1], cnt.astype(np.int64)) + np.arange(total)
        return starts.astype(np.uint32), self.eng.key_ids(keys[idx]), st


class ShardedIndex:
    """One rank's view of a filter-sharded index over `world` ranks.

    The exchange of a step (`exchange`, SURVEY.md §8(e) mode 2):
      padded  all-gather of every rank's header (topic-major offsets + flags) and of its ids
              padded to a common stride fixed by prepare_device: no host sync in the step;
      exact   all-gather of the headers, then every rank's ids at their exact size by grouped
              send/recv (the sizes come from the gathered headers: one host read per step);
      local   no collective: each rank copies its own shard's lists to the host, and the
              consumer reads the G shard lists of a topic side by side;
      a2a     by topic range: rank r keeps the merged results of topics [r*n/G, (r+1)*n/G)
              (the publishes it answers); every rank sends each other rank just that range
              of its ids (all_to_all at exact sizes, from an all-gather of G+1 offsets per
              rank: one host read per step), so a rank receives (G-1)/G of ONE shard's ids
              instead of G-1 shards' worth, and merges 1/G of the batch.
    Ids cross the wire as u32 while every id of every shard fits 32 bits (u64 otherwise)."""

    def __init__(self, shard, rank: int, world: int, group=None, exchange: str = "padded"):
        if exchange not in EXCHANGES:
            raise ValueError(f"exchange must be one of {EXCHANGES}")
        self.shard, self.rank, self.world, self.group = shard, rank, world, group
        self.exchange = exchange
        self.id_bytes = 8
        self.stride = None
        self.wire_bytes = 0  # bytes this rank received in the last step's exchange

    # ---- writes: every rank sees the same op stream and keeps its own keys
    def apply_packed(self, op, buf, off, ids, flags=None):
        mask = shard_of(ids, self.world) == self.rank
        b, o, i, f = select_keys(buf, off, ids, mask, flags)
        self.shard.apply_packed(op, b, o, i, f)

    def commit(self):
        return self.shard.commit()

    # ---- the collective part, shared by the host (gloo) and device (RCCL) paths
    def _staged(self, hdr):
        """A device step over a gloo group (rehearsing several ranks on one GPU): gloo moves
        host tensors, so the exchange runs on host copies and its results go back to the device.
        Over RCCL the device tensors go on the wire as they are."""
        import torch.distributed as dist
        return self.world > 1 and hdr.is_cuda and dist.get_backend(self.group) == "gloo"

    def _exchange(self, hdr, ids, n: int, exchange: str):
        """hdr: this rank's (n+2) i32 [offsets | flags]; ids: its ids buffer (>= its total, the
        padded stride long for `padded`).  Returns (H (G, n+2) i32, Ids flat, bases); Ids and
        bases are None when a rank overflowed and the ids were not exchanged (exact)."""
        import torch
        import torch.distributed as dist
        G = self.world
        if G == 1:
            self.wire_bytes = 0
            return hdr.view(1, n + 2), ids, [0]
        if self._staged(hdr):
            H, Ids, bases = self._exchange(hdr.cpu(), ids.cpu(), n, exchange)
            return H.to(hdr.device), (None if Ids is None else Ids.to(hdr.device)), bases
        H = torch.empty(G * (n + 2), dtype=hdr.dtype, device=hdr.device)
        dist.all_gather_into_tensor(H, hdr, group=self.group)
        H = H.view(G, n + 2)
        eb = ids.element_size()
        if exchange == "padded":
            stride = ids.numel()
            Ids = torch.empty(G * stride, dtype=ids.dtype, device=ids.device)
            dist.all_gather_into_tensor(Ids, ids, group=self.group)
            self.wire_bytes = (G - 1) * (stride * eb + (n + 2) * 4)
            return H, Ids, [r * stride for r in range(G)]
        # exact: the sizes are the headers' offsets[n] (one small D2H on a device path), read
        # together with every rank's flags: a rank that outgrew its id buffer holds fewer ids
        # than its offsets say, so on overflow EVERY rank skips the id exchange (a transfer sized
        # from those offsets would never complete) and the caller sees the flag
        hn = (H[:, n:n + 2].to(torch.int64) & 0xFFFFFFFF).cpu().tolist()
        tot = [r[0] for r in hn]
        if any(r[1] for r in hn):
            self.wire_bytes = (G - 1) * (n + 2) * 4
            return H, None, None
        bases = [0] * G
        for r in range(1, G):
            bases[r] = bases[r - 1] + tot[r - 1]
        Ids = torch.empty(max(1, bases[-1] + tot[-1]), dtype=ids.dtype, device=ids.device)
        me = self.rank
        if tot[me]:
            Ids[bases[me]:bases[me] + tot[me]].copy_(ids[:tot[me]])
        ops = []
        for q in range(G):
            if q == me:
                continue
            peer = dist.get_global_rank(self.group, q) if self.group is not None else q
            if tot[me]:
                ops.append(dist.P2POp(dist.isend, ids[:tot[me]], peer, self.group))
            if tot[q]:
                ops.append(dist.P2POp(dist.irecv, Ids[bases[q]:bases[q] + tot[q]], peer, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        self.wire_bytes = sum(tot[q] for q in range(G) if q != me) * eb + (G - 1) * (n + 2) * 4
        return H, Ids, bases

    def topic_range(self, n: int, rank: int | None = None):
        """a2a: the topics [lo, hi) whose merged results this rank keeps."""
        r = self.rank if rank is None else rank
        return r * n // self.world, (r + 1) * n // self.world

    def _exchange_a2a(self, hdr, ids, n: int):
        """a2a exchange: returns (H (G, m+2) i32 rows of this rank's topic range [offsets
        rebased to 0 | flags], Ids, bases) for m = the range's topic count."""
        import torch
        import torch.distributed as dist
        if self._staged(hdr):
            H, Ids, bases = self._exchange_a2a(hdr.cpu(), ids.cpu(), n)
            return H.to(hdr.device), (None if Ids is None else Ids.to(hdr.device)), bases
        G, me = self.world, self.rank
        T = [q * n // G for q in range(G + 1)]
        dev = hdr.device
        Tt = torch.tensor(T, dtype=torch.int64, device=dev)
        mine = torch.cat([hdr[:n + 1][Tt], hdr[n + 1:n + 2]])  # my offsets at the range bounds + flags
        B = torch.empty(G * (G + 2), dtype=hdr.dtype, device=dev)
        dist.all_gather_into_tensor(B, mine.contiguous(), group=self.group)
        Bh = (B.view(G, G + 2).to(torch.int64) & 0xFFFFFFFF).cpu().tolist()  # sizes + flags: one host read
        flags = B.view(G, G + 2)[:, G + 1]
        m = T[me + 1] - T[me]
        if any(row[G + 1] for row in Bh):  # some rank overflowed: nobody exchanges (see _exchange)
            self.wire_bytes = (G - 1) * (G + 2) * 4
            H = torch.zeros(G, m + 2, dtype=hdr.dtype, device=dev)
            H[:, m + 1] = flags
            return H, None, None
        send = [Bh[me][q + 1] - Bh[me][q] for q in range(G)]
        recv = [Bh[q][me + 1] - Bh[q][me] for q in range(G)]
        lo = Bh[me][0]
        Ids = torch.empty(max(1, sum(recv)), dtype=ids.dtype, device=ids.device)
        dist.all_to_all_single(Ids[:sum(recv)], ids[lo:lo + sum(send)].contiguous(), recv, send, group=self.group)
        # every rank's offsets over my topic range, rebased to its slice's start
        offs = torch.cat([hdr[T[q]:T[q + 1] + 1] - hdr[T[q]] for q in range(G)])
        O = torch.empty(G * (m + 1), dtype=hdr.dtype, device=dev)
        dist.all_to_all_single(O, offs, [m + 1] * G, [T[q + 1] - T[q] + 1 for q in range(G)], group=self.group)
        H = torch.cat([O.view(G, m + 1), flags.view(G, 1)], dim=1).contiguous()
        bases = [0] * G
        for q in range(1, G):
            bases[q] = bases[q - 1] + recv[q - 1]
        eb = ids.element_size()
        self.wire_bytes = sum(recv[q] for q in range(G) if q != me) * eb + (G - 1) * ((m + 1) * 4 + (G + 2) * 4)
        return H, Ids, bases

    # ---- host path (gloo or nccl)
    def match(self, t_bytes, t_off, exchange: str | None = None):
        """Match the whole batch on every rank.  padded / exact: the merged (off[n+1] u32,
        ids u64, status i32[n]) on every rank; local: this rank's own shard lists in the same
        form (the union over ranks is the result); a2a: the merged results of this rank's
        topic range (topic_range), as (off[m+1], ids, status[m])."""
        import torch
        import torch.distributed as dist
        exchange = exchange or self.exchange
        roff, ids, st = self.shard.match_ids(t_bytes, t_off)
        n = len(roff) - 1
        if exchange == "local":
            self.wire_bytes = 0
            return roff, ids, st
        dev = torch.device("cpu")
        if self.world > 1 and dist.get_backend(self.group) != "gloo":
            dev = torch.device("cuda", torch.cuda.current_device())
        hdr = torch.from_numpy(np.concatenate([roff, np.zeros(1, np.uint32)]).view(np.int32)).to(dev)
        total = int(roff[-1])
        if exchange == "a2a":
            buf = np.zeros(max(1, total), np.uint64)
            buf[:total] = ids
            if self.world == 1:
                return roff, ids, st
            H, Ids, bases = self._exchange_a2a(hdr, torch.from_numpy(buf.view(np.int64)).to(dev), n)
            lo, hi = self.topic_range(n)
            off, merged = merge_shard_ids_host(H.cpu().numpy(), Ids.cpu().numpy().view(np.uint64), bases, hi - lo)
            return off, merged, st[lo:hi]
        if exchange == "padded":
            # without prepare_device the host path pads to the largest rank's total
            t = torch.tensor([total], dtype=torch.int64, device=dev)
            if self.world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            buf = np.zeros(max(1, int(t.item())), np.uint64)
        else:
            buf = np.zeros(max(1, total), np.uint64)
        buf[:total] = ids
        H, Ids, bases = self._exchange(hdr, torch.from_numpy(buf.view(np.int64)).to(dev), n, exchange)
        off, merged = merge_shard_ids_host(H.cpu().numpy(), Ids.cpu().numpy().view(np.uint64), bases, n)
        return off, merged, st

    # ---- device path (RCCL over xGMI)
    def prepare_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int,
                       headroom: float = 1.25):
        """Size this rank's buffers and the exchange stride from one synchronous run of the
        batch (collective when world > 1), and pick the id width every rank can use.  Not part
        of the step: the step itself never waits on the host (padded); a later batch that
        outgrows these sizes is flagged on the device (match_device's flags) and re-run by
        the caller after prepare_device."""
        import torch
        import torch.distributed as dist
        dev = torch.device("cuda", torch.cuda.current_device())
        torch.cuda.current_stream().synchronize()
        r = eng.match_device(d_bytes, d_off, n, total_bytes, 0)
        eng.device_sync()  # also sizes the chunk pools to this batch's demand
        total = _read_u64(r.d_total)
        idb = 4
        probe = torch.empty(n + 1, dtype=torch.int32, device=dev)
        try:  # u32 ids unless this shard holds an id past 32 bits
            eng.match_ids_device(d_bytes, d_off, n, total_bytes, 4, 0, 0, probe.data_ptr(), 0, 0)
        except N.TMError as e:
            if e.rc != N.TM_ESTATE:
                raise
            idb = 8
        torch.cuda.synchronize()
        gloo = self.world > 1 and dist.get_backend(self.group) == "gloo"
        t = torch.tensor([total, idb], dtype=torch.int64, device="cpu" if gloo else dev)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.id_bytes = int(t[1].item())
        eng.reserve_matches((int(total * headroom) + 1024) * (self.id_bytes // 4))
        self.stride = int(int(t[0].item()) * headroom) + 1024
        return total

    def id_dtype(self):
        import torch
        return torch.int32 if self.id_bytes == 4 else torch.int64

    def local_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int, sp: int):
        """This rank's half of the step, queued on stream `sp` with no host sync: the walk with
        the route ids written by its copy-out and compacted topic-major (tm_match_ids_device).
        Returns (hdr i32[n+2]: topic-major offsets + the TM_RES_* flags, ids[stride])."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        hdr = torch.empty(n + 2, dtype=torch.int32, device=dev)
        ids = torch.empty(self.stride, dtype=self.id_dtype(), device=dev)
        eng.match_ids_device(d_bytes, d_off, n, total_bytes, self.id_bytes, ids.data_ptr(), self.stride,
                             hdr.data_ptr(), hdr[n + 1:].data_ptr(), sp)
        return hdr, ids

    def merge_device(self, eng: "N.Engine", H, Ids, bases, n: int, sp: int):
        """Concatenate the G shards' slices per topic on the device.  H: (G, n+2) i32 headers,
        rank r's ids at Ids[bases[r]:].  Returns (off i32[n+1], ids i64 buffer whose first
        off[n] entries are the result, flags i32[1]: nonzero if any shard overflowed)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        G = H.shape[0]
        flags = H[:, n + 1].max().reshape(1)
        if Ids is None:  # the exchange was skipped: a rank overflowed (flags != 0), nothing to merge
            return torch.zeros(n + 1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int64, device=dev), flags
        out_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
        cap = G * self.stride
        out_ids = torch.empty(cap, dtype=torch.int64, device=dev)
        eng.merge_shard_ids_device(G, n, H.data_ptr(), n + 2, Ids.data_ptr(), self.id_bytes, bases, self.stride,
                                   out_off.data_ptr(), out_ids.data_ptr(), cap, sp)
        return out_off, out_ids, flags

    def match_device(self, eng: "N.Engine", d_bytes: int, d_off: int, n: int, total_bytes: int,
                     exchange: str | None = None):
        """GPU step: the walk writes route ids, compacted topic-major; the exchange; the device
        merge.  The engine calls and the torch ops between them run on ONE torch stream (the
        engine's own stream is non-blocking, so torch's legacy default stream would not order
        after it); the caller's current stream waits for it before this returns.
        padded / exact: device tensors (off i32[n+1], ids i64 buffer holding off[n] u64 route
        ids, flags i32[1]); flags != 0 means a shard outgrew its sizes: call prepare_device
        again and re-run the batch.  local: this rank's own lists on the host (pinned):
        (offsets i32[n+1], ids, flags)."""
        import torch
        exchange = exchange or self.exchange
        if self.stride is None:
            self.prepare_device(eng, d_bytes, d_off, n, total_bytes)
        dev = torch.device("cuda", torch.cuda.current_device())
        caller = torch.cuda.current_stream()
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream(dev)
        s = self._stream
        s.wait_stream(caller)  # the topic batch was written on the caller's stream
        sp = s.cuda_stream
        with torch.cuda.stream(s):
            hdr, ids = self.local_device(eng, d_bytes, d_off, n, total_bytes, sp)
            if exchange == "local":
                if getattr(self, "_h_hdr", None) is None or self._h_hdr.numel() < n + 2:
                    self._h_hdr = torch.empty(n + 2, dtype=torch.int32, pin_memory=True)
                if getattr(self, "_h_ids", None) is None or self._h_ids.numel() < self.stride \
                        or self._h_ids.dtype != ids.dtype:
                    self._h_ids = torch.empty(self.stride, dtype=ids.dtype, pin_memory=True)
                h_hdr = self._h_hdr[:n + 2]
                h_hdr.copy_(hdr, non_blocking=True)
                s.synchronize()  # the shard's size, for an exact copy of its ids
                total = min(int(h_hdr[n].item()), self.stride)
                self._h_ids[:total].copy_(ids[:total], non_blocking=True)
                s.synchronize()
                self.wire_bytes = 0
                return h_hdr[:n + 1], self._h_ids[:total], h_hdr[n + 1:]
            if exchange == "a2a" and self.world > 1:
                H, Ids, bases = self._exchange_a2a(hdr, ids, n)
                lo, hi = self.topic_range(n)
                out = self.merge_device(eng, H, Ids, bases, hi - lo, sp)
            else:
                H, Ids, bases = self._exchange(hdr, ids, n, exchange)
                out = self.merge_device(eng, H, Ids, bases, n, sp)
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
