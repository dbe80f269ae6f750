"""Replicated mode (DESIGN.md §6 mode 1): one route table per node, every
GPU a reader.

The reference keeps ONE full route table per node (mria/ETS, apps/emqx/src/emqx_router.erl:
133-162), written by one syncer process per node (apps/emqx/src/emqx_router_syncer.erl:
244-280) and read by every publisher.  The MI355X counterpart:

  * rank 0 of the node group is the MASTER: it holds the host master copy (the engine built
    with TM_CFG_RECORD_PATCH), applies route ops and commits delta epochs;
  * every other rank is a READ REPLICA (tm_replica_create): the master's frozen device index,
    received as one device image over the process group (RCCL broadcast over xGMI), with no
    host copy of its own — host memory is one copy per node, not one per GPU;
  * each commit's device changes (tm_patch_export: the scatter/append records the master's
    own upload made) are broadcast and replayed on every replica; a commit that re-uploaded
    the whole index (full rebuild) ships the image again.

Publishes are then data-parallel: each rank matches its own batches against its copy, with
no collective on the match path.

The transport is torch.distributed (`nccl` = RCCL on device tensors; `gloo` on CPU tensors).
The engine side is an adapter with export_image() / load_image() / patch() / apply_patch();
EngineReplicaAdapter is the product one (libemqx_tm.so); tests on CPU plug a double.
"""
from __future__ import annotations

import numpy as np

from . import _native as N


class EngineReplicaAdapter:
    """Product adapter: image and patches of a HIP engine, as torch tensors on its GPU."""

    def __init__(self, device: int, engine: "N.Engine | None" = None):
        self.device = device
        self.eng = engine

    def tensor_device(self):
        import torch
        return torch.device("cuda", self.device)

    # master side
    def export_image(self):
        import torch
        n = self.eng.image_size()
        t = torch.empty(n, dtype=torch.uint8, device=self.tensor_device())
        torch.cuda.current_stream(self.device).synchronize()  # the buffer exists before the engine's copy
        self.eng.image_export(t.data_ptr(), n)
        return t

    def patch(self):
        buf, full = self.eng.patch_export()
        return buf, full

    def epoch(self) -> int:
        return int(self.eng.stats()["epoch"])

    @staticmethod
    def patch_epoch_from(buf) -> int:
        """The epoch a patch applies on (PatchHdr.epoch_from, engine.cpp)."""
        return int(np.frombuffer(bytes(buf[8:16]), dtype=np.uint64)[0]) if len(buf) >= 16 else -1

    # replica side
    def load_image(self, t):
        import torch
        torch.cuda.current_stream(self.device).synchronize()  # the broadcast landed
        if self.eng is None:
            self.eng = N.Engine.replica_from_image(self.device, t.data_ptr(), t.numel())
        else:
            self.eng.replica_load(t.data_ptr(), t.numel())

    def apply_patch(self, buf: np.ndarray):
        self.eng.apply_patch(buf)


class ReplicatedIndex:
    """One rank's view of a replicated index over the ranks of `group` (rank 0 = master)."""

    def __init__(self, adapter, rank: int, world: int, group=None):
        self.ad, self.rank, self.world, self.group = adapter, rank, world, group
        self.bytes_sent = 0  # image + patch bytes broadcast by the master (diagnostics)
        self.shipped = None  # master: the epoch every replica holds (the last one shipped)

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    def _dev(self):
        import torch
        import torch.distributed as dist
        if self.world > 1 and dist.get_backend(self.group) == "gloo":
            return torch.device("cpu")
        return self.ad.tensor_device()

    CHUNK = 1 << 30  # bytes per broadcast call: a 20 GiB image goes as 1 GiB pieces

    def _bcast(self, t):
        import torch.distributed as dist
        if self.world > 1:
            flat = t.view(-1)
            if flat.numel() * flat.element_size() <= self.CHUNK:
                dist.broadcast(t, src=0, group=self.group)
            else:  # keep every collective's element count well inside 32 bits
                step = self.CHUNK // flat.element_size()
                for i in range(0, flat.numel(), step):
                    dist.broadcast(flat[i:i + step], src=0, group=self.group)
        return t

    def _send_image(self):
        import torch
        dev = self._dev()
        if self.is_master:
            img = self.ad.export_image()
            if img.device != dev:
                img = img.to(dev)
            n = torch.tensor([img.numel()], dtype=torch.int64, device=dev)
        else:
            n = torch.zeros(1, dtype=torch.int64, device=dev)
        self._bcast(n)
        if not self.is_master:
            img = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
        self._bcast(img)
        if self.is_master:
            self.bytes_sent += img.numel() * (self.world - 1)
        else:
            self.ad.load_image(img if img.device == self.ad.tensor_device() else img.to(self.ad.tensor_device()))

    def start(self):
        """Collective: every replica receives the master's current image."""
        if self.is_master:
            self.shipped = self.ad.epoch()
        self._send_image()

    SYNC_PATCH, SYNC_IMAGE, SYNC_NONE = 0, 1, 2

    def sync(self):
        """Collective: bring every replica to the master's committed epoch.  One commit since
        the last sync ships that commit's patch; a full rebuild, or more than one commit
        (a patch only applies on the epoch it was made from), ships the whole image; no
        commit ships nothing.  Returns the SYNC_* kind that was shipped."""
        import torch
        dev = self._dev()
        if self.is_master:
            cur = self.ad.epoch()
            buf, kind = None, self.SYNC_NONE
            if cur != self.shipped:
                buf, full = self.ad.patch()
                kind = (self.SYNC_IMAGE if full or self.ad.patch_epoch_from(buf) != self.shipped
                        else self.SYNC_PATCH)
            hdr = torch.tensor([len(buf) if kind == self.SYNC_PATCH else 0, kind], dtype=torch.int64, device=dev)
            self.shipped = cur
        else:
            hdr = torch.zeros(2, dtype=torch.int64, device=dev)
        self._bcast(hdr)
        n, kind = int(hdr[0].item()), int(hdr[1].item())
        if kind == self.SYNC_NONE:
            return kind
        if kind == self.SYNC_IMAGE:
            self._send_image()
            return kind
        if self.is_master:
            t = torch.from_numpy(buf).to(dev)
        else:
            t = torch.empty(n, dtype=torch.uint8, device=dev)
        self._bcast(t)
        if self.is_master:
            self.bytes_sent += n * (self.world - 1)
        else:
            self.ad.apply_patch(t.cpu().numpy())
        return kind
