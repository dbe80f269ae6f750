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


def cgroup_quota_cpus():
    """The cgroup v2 CPU quota (cpu.max) in whole CPUs, or None when unlimited / unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(q) // int(per))
    except (OSError, ValueError):
        return None


def one_per_core(cpus, k):
    """k of `cpus`, one per physical core first (SMT siblings only when the cores run out)."""
    seen, first, rest = set(), [], []
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            core = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            core = ("?", str(c))
        (rest if core in seen else first).append(c)
        seen.add(core)
    return sorted((first + rest)[:k])


def pin_to_gpu(device: int = 0, quota_cut: bool = True) -> dict:
    """Restrict this process (and the threads it creates later) to the GPU-local CPUs that
    it may use.  Returns what was done, for the bench line.

    Under a cgroup CPU quota (the GPU boxes here: cpu.max 16 CPUs per 100 ms period, while the
    process may run on every CPU of the machine) the set is cut to as many CPUs as the quota
    grants, one per physical core: with more runnable threads than that on more CPUs, the job
    spends its quota before the period ends and EVERY thread stops for the rest of it (tens of
    milliseconds: round 4's aggregator tail).  On exactly `quota` CPUs it can
    never run ahead of its quota; extra threads time-slice instead."""
    local = gpu_local_cpus(device)
    before = sorted(os.sched_getaffinity(0))
    if not local:
        return {"pinned": False, "reason": "no local_cpulist for the GPU"}
    use = sorted(set(local) & set(before))
    if not use:
        return {"pinned": False, "reason": "no GPU-local CPU in this process's affinity"}
    quota = cgroup_quota_cpus()
    if quota_cut and quota and quota < len(use):
        use = one_per_core(use, quota)
    os.sched_setaffinity(0, use)
    return {"pinned": True, "cpus": len(use), "of": len(before), "quota_cpus": quota,
            "gpu_local_cpus": len(local)}
