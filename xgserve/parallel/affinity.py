"""Pin a GPU process's CPU affinity to its GPU's NUMA node -- before any HIP call.

One process per GPU (bench ranks, serving replicas): the host side of every step
(scheduler, launches, H2D / D2H staging through pinned buffers) runs on CPU cores;
on a two-socket MI355X node half of them sit across the socket interconnect from
a given GPU. The GPU's PCI function lists its local CPUs in sysfs; the KFD topology
maps HIP device indices (GPU nodes in order) to PCI functions. Reading sysfs does
not initialise the GPU, so this runs before torch touches it. Best effort: any
missing file, or a cpuset that excludes the node's CPUs, leaves the affinity alone.
"""
from __future__ import annotations

import glob
import logging
import os
from typing import List, Optional, Set

log = logging.getLogger("xgserve.affinity")

_KFD = "/sys/class/kfd/kfd/topology/nodes"


def _parse_cpulist(s: str) -> Set[int]:
    cpus: Set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def _gpu_pci_functions() -> List[str]:
    """PCI addresses of the GPUs in KFD node order (= HIP device order)."""
    nodes = []
    for d in glob.glob(os.path.join(_KFD, "*")):
        try:
            props = dict(line.split() for line in open(os.path.join(d, "properties")) if len(line.split()) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        loc = int(props.get("location_id", "0"))
        dom = int(props.get("domain", "0"))
        nodes.append((int(os.path.basename(d)), f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"))
    return [bdf for _, bdf in sorted(nodes)]


def gpu_local_cpus(gpu_index: int) -> Optional[Set[int]]:
    """CPUs local to HIP device `gpu_index` (honouring HIP/ROCR_VISIBLE_DEVICES), or None."""
    pcis = _gpu_pci_functions()
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        try:
            order = [int(v) for v in vis.split(",") if v.strip() != ""]
            pcis = [pcis[i] for i in order if i < len(pcis)]
        except ValueError:
            return None
    if not 0 <= gpu_index < len(pcis):
        return None
    try:
        with open(f"/sys/bus/pci/devices/{pcis[gpu_index]}/local_cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return None


def bind_to_gpu_numa(gpu_index: int) -> Optional[Set[int]]:
    """Restrict this process to the CPUs local to its GPU that it may use. Returns
    the new CPU set, or None when nothing was changed."""
    if os.environ.get("XGS_NUMA_BIND", "1") == "0":
        return None
    local = gpu_local_cpus(gpu_index)
    if not local:
        return None
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        return None
    want = allowed & local
    # a cpuset that already confines the process (e.g. a scheduler's CPU share) and only
    # grazes the GPU's node: keep it rather than squeeze the host threads onto a few cores
    if not want or want == allowed or len(want) < max(4, len(allowed) // 4):
        return None
    try:
        os.sched_setaffinity(0, want)
    except OSError:
        return None
    log.info("GPU %d: bound to its NUMA-local CPUs (%d of %d)", gpu_index, len(want), len(allowed))
    return want
