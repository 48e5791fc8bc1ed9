"""Core binding of a GPU worker (reference: BoxPSTrainer's
``enable_binding_train_cpu`` -- worker threads pinned to cores,
``boxps_trainer.cc:165-193``).

MI355X-first: one process per GPU, so the process (and the native threads it
starts afterwards: loader, batch assembler, key agent) is bound to the CPU
cores of the GPU's own NUMA node (sysfs ``local_cpulist`` of its PCI
function), split evenly between the local ranks that share that node, and
always within the cores this process is allowed to use (cgroup / taskset)."""
from __future__ import annotations

import os
from typing import List, Optional, Set

import torch

from ..utils.log import logger

log = logger()


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_local_cpus(device: torch.device) -> Optional[List[int]]:
    """CPU ids of the NUMA node the GPU's PCI function hangs off (None when
    sysfs does not say)."""
    try:
        p = torch.cuda.get_device_properties(device)
        dom = getattr(p, "pci_domain_id", 0)
        bus, dev = p.pci_bus_id, p.pci_device_id
    except Exception:
        return None
    path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.0/local_cpulist"
    try:
        with open(path) as f:
            return _parse_cpulist(f.read())
    except OSError:
        return None


def bind_worker(device: torch.device, local_rank: int = 0, ranks_on_node: int = 1) -> Optional[Set[int]]:
    """Pin this process to its share of the GPU-local cores; returns the new
    CPU set, or None when nothing was changed."""
    if device.type != "cuda" or not hasattr(os, "sched_setaffinity"):
        return None
    allowed = set(os.sched_getaffinity(0))
    local = gpu_local_cpus(device)
    cand = sorted(allowed & set(local)) if local else sorted(allowed)
    if not cand:
        cand = sorted(allowed)
    # ranks whose GPUs share this NUMA node split its cores
    share = max(1, ranks_on_node)
    per = max(1, len(cand) // share)
    i = local_rank % share
    mine = set(cand[i * per:(i + 1) * per]) or set(cand)
    if mine == allowed:
        return None
    os.sched_setaffinity(0, mine)
    log.info("worker bound to %d cores of the GPU-local node (%s..%s)", len(mine), min(mine), max(mine))
    return mine
