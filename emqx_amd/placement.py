"""Host placement of a process that drives one GPU (bench / test tooling and an example for
the embedding application).

An MI355X node has two CPU sockets; each GPU hangs off one of them.  The engine's pinned
staging buffers, its host id arena (what every runs-form reply reads) and the aggregator's
delivery threads all live in host memory, so a process pinned to the GPU's own socket keeps
that traffic off the inter-socket link: DMA to and from local memory, and callbacks that read
local memory.  This reads the GPU's PCI address from the HIP runtime and the CPUs local to
it from sysfs; it changes nothing when the information is missing."""
from __future__ import annotations

import os


def gpu_local_cpus(device: int = 0):
    """The CPUs on the GPU's own NUMA node (sysfs local_cpulist), or None."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        addr = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        txt = open(f"/sys/bus/pci/devices/{addr}/local_cpulist").read().strip()
    except Exception:
        return None
    cpus = set()
    for part in txt.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return sorted(cpus) or None


def pin_to_gpu(device: int = 0) -> dict:
    """Restrict this process (and the threads it creates later) to the GPU-local CPUs that
    it may use.  Returns what was done, for the bench line."""
    local = gpu_local_cpus(device)
    before = sorted(os.sched_getaffinity(0))
    if not local:
        return {"pinned": False, "reason": "no local_cpulist for the GPU"}
    use = sorted(set(local) & set(before))
    if not use:
        return {"pinned": False, "reason": "no GPU-local CPU in this process's affinity"}
    os.sched_setaffinity(0, use)
    return {"pinned": True, "cpus": len(use), "of": len(before)}
