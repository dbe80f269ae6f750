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


def core_of(c):
    """(package, core) of logical CPU c, from sysfs."""
    try:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        return (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
    except OSError:
        return ("?", str(c))


def cpu_busy(cpus, interval=0.25):
    """Busy fraction of each CPU in `cpus` over `interval` seconds, whoever ran there (the
    machine's /proc/stat: every job on the host, not just this one).  {} when unreadable."""
    import time

    def snap():
        out = {}
        try:
            with open("/proc/stat") as f:
                for line in f:
                    if line.startswith("cpu") and line[3:4].isdigit():
                        v = line.split()
                        n = [int(x) for x in v[1:9]]  # user nice system idle iowait irq softirq steal
                        out[int(v[0][3:])] = (sum(n), n[3] + n[4])
        except (OSError, ValueError):
            return {}
        return out

    a = snap()
    time.sleep(interval)
    b = snap()
    res = {}
    for c in cpus:
        if c in a and c in b:
            tot, idle = b[c][0] - a[c][0], b[c][1] - a[c][1]
            res[c] = max(0.0, (tot - idle) / tot) if tot > 0 else 0.0
    return res


def pick_cores(cpus, k, busy=None, start=0, core=core_of):
    """k of `cpus`: one per physical core first (SMT siblings only when the cores run out),
    the least busy cores first.  Cores are taken in CPU order rotated to begin at core `start`
    (one slot per GPU, so processes driving different GPUs of one socket begin on different
    cores), then stably ordered by their busy fraction (both siblings, in steps of 0.1) --
    a job already running on a core pushes it to the back."""
    busy = busy or {}
    groups, order = {}, []
    for c in cpus:
        key = core(c)
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(c)
    if not order:
        return []
    s = start % len(order)
    order = order[s:] + order[:s]
    score = {key: round(sum(busy.get(c, 0.0) for c in groups[key]) * 10) for key in order}
    order.sort(key=lambda key: score[key])
    for key in order:
        groups[key].sort(key=lambda c: busy.get(c, 0.0))
    first = [groups[key][0] for key in order]
    rest = [c for key in order for c in groups[key][1:]]
    return sorted((first + rest)[:k])


def one_per_core(cpus, k):
    """k of `cpus`, one per physical core first (SMT siblings only when the cores run out)."""
    return pick_cores(cpus, k)


_first_affinity = None
KEEP_BUSY = 0.10  # a re-pick keeps its cores while at most this busy


def pin_to_gpu(device: int = 0, quota_cut: bool = True) -> dict:
    """Restrict this process (and the threads it creates later) to the GPU-local CPUs that
    it may use.  Returns what was done, for the bench line.

    Under a cgroup CPU quota (the GPU boxes here: cpu.max 16 CPUs per 100 ms period, while the
    process may run on every CPU of the machine) the set is cut to as many CPUs as the quota
    grants, one per physical core: with more runnable threads than that on more CPUs, the job
    spends its quota before the period ends and EVERY thread stops for the rest of it (tens of
    milliseconds: round 4's aggregator tail).  On exactly `quota` CPUs it can
    never run ahead of its quota; extra threads time-slice instead.

    Which cores: the least busy ones over a quarter second (other jobs on the machine run
    there too; round 5's final check saw a run pinned to the socket's first 16 cores get 3.4
    CPUs of use out of 16, with its aggregator at a fifth of its rate), beginning at a
    per-GPU offset."""
    global _first_affinity
    local = gpu_local_cpus(device)
    if _first_affinity is None:  # a later call picks again from the set the process started with
        _first_affinity = sorted(os.sched_getaffinity(0))
    before = _first_affinity
    if not local:
        return {"pinned": False, "reason": "no local_cpulist for the GPU"}
    use = sorted(set(local) & set(before))
    if not use:
        return {"pinned": False, "reason": "no GPU-local CPU in this process's affinity"}
    quota = cgroup_quota_cpus()
    info = {}
    if quota_cut and quota and quota < len(use):
        busy = cpu_busy(use)
        use_all = use
        cur = sorted(os.sched_getaffinity(0))
        if (_first_affinity != cur and len(cur) == quota and set(cur) <= set(use_all)
                and busy and sum(busy.get(c, 0.0) for c in cur) / len(cur) <= KEEP_BUSY):
            # a later call keeps the cores picked before while they stay free: the threads
            # started earlier (the HIP runtime's among them) stay on them
            return {"pinned": True, "kept": True, "cpus": len(cur), "of": len(before), "quota_cpus": quota,
                    "gpu_local_cpus": len(local),
                    "busy_kept": round(sum(busy.get(c, 0.0) for c in cur) / len(cur), 3)}
        use = pick_cores(use_all, quota, busy, start=device * quota)
        if busy:
            info = {"busy_chosen": round(sum(busy.get(c, 0.0) for c in use) / len(use), 3),
                    "busy_gpu_local": round(sum(busy.values()) / len(busy), 3),
                    "busy_first_cores": round(sum(busy.get(c, 0.0) for c in pick_cores(use_all, quota)) / quota, 3)}
    os.sched_setaffinity(0, use)
    return {"pinned": True, "cpus": len(use), "of": len(before), "quota_cpus": quota,
            "gpu_local_cpus": len(local), **info}
