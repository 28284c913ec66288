"""NUMA placement of a rank's host threads and page-locked buffers next to its
GPU (block replay, configs[4]: each rank streams an ~8 GiB pinned shard over
its GPU's PCIe link; app/extend_block.go:14-22 per block).

The GPU's PCI address comes from the KFD topology (/sys/class/kfd/kfd/topology:
GPU nodes are those with simd_count > 0, in the order ROCr enumerates them,
location_id = bus << 8 | device << 3 | function), filtered by
ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES; its NUMA node from
/sys/bus/pci/devices/<addr>/numa_node; the node's CPUs from
/sys/devices/system/node/node<N>/cpulist.  bind() must run before the process
first touches the GPU (HIP's own threads keep the mask they start with) and
before the pinned buffers are allocated (their pages land on the node of the
allocating thread).  Host-side placement only; no GPU call.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_pci_addresses(sysfs: str = "/sys") -> List[str]:
    """PCI addresses of the GPU agents in KFD topology order ('dddd:bb:dd.f')."""
    base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        props = _read(os.path.join(base, str(n), "properties"))
        if not props:
            continue
        kv: Dict[str, int] = {}
        for line in props.splitlines():
            f = line.split()
            if len(f) == 2 and f[1].lstrip("-").isdigit():
                kv[f[0]] = int(f[1])
        if kv.get("simd_count", 0) <= 0:
            continue
        loc, dom = kv.get("location_id", 0), kv.get("domain", 0)
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}")
    return out


def _visible(addrs: List[str], env) -> Optional[List[str]]:
    # ROCr filters first; HIP then honours ONE of HIP_VISIBLE_DEVICES /
    # CUDA_VISIBLE_DEVICES (HIP_ wins when both are set, as launchers often
    # set both to the same list), indexing the devices ROCr left.
    hip_var = "HIP_VISIBLE_DEVICES" if env.get("HIP_VISIBLE_DEVICES") else "CUDA_VISIBLE_DEVICES"
    for var in ("ROCR_VISIBLE_DEVICES", hip_var):
        v = env.get(var)
        if v is None or v == "":
            continue
        try:
            idx = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            return None  # UUID lists: not mapped here
        if any(i < 0 or i >= len(addrs) for i in idx):
            return None
        addrs = [addrs[i] for i in idx]
    return addrs


_LINK_TYPES = {2: "pcie", 11: "xgmi"}  # KFD CRAT io-link types


def _props(path: str) -> Dict[str, int]:
    kv: Dict[str, int] = {}
    for line in (_read(path) or "").splitlines():
        f = line.split()
        if len(f) == 2 and f[1].lstrip("-").isdigit():
            kv[f[0]] = int(f[1])
    return kv


def gpu_links(sysfs: str = "/sys") -> Dict[str, Dict]:
    """Direct links between GPU agents from the KFD topology (io_links of each
    GPU node): {pci: {"xgmi": [peer pci...], "pcie_to_cpu": n, ...}}.  The
    transport RCCL can use between two ranks' GPUs (xGMI point to point, or
    PCIe through the host)."""
    base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return {}
    gpu_pci: Dict[int, str] = {}
    for n in nodes:
        kv = _props(os.path.join(base, str(n), "properties"))
        if kv.get("simd_count", 0) > 0:
            loc, dom = kv.get("location_id", 0), kv.get("domain", 0)
            gpu_pci[n] = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}"
    out: Dict[str, Dict] = {}
    for n, pci in gpu_pci.items():
        d: Dict = {"xgmi": [], "pcie_peers": [], "pcie_to_cpu": 0}
        ldir = os.path.join(base, str(n), "io_links")
        try:
            links = sorted(os.listdir(ldir))
        except OSError:
            links = []
        for li in links:
            kv = _props(os.path.join(ldir, li, "properties"))
            to, kind = kv.get("node_to", -1), _LINK_TYPES.get(kv.get("type", -1), "other")
            if to in gpu_pci:
                (d["xgmi"] if kind == "xgmi" else d["pcie_peers"]).append(gpu_pci[to])
            elif kind == "pcie":
                d["pcie_to_cpu"] += 1
        out[pci] = d
    return out


def gpu_numa(gpu_index: int, sysfs: str = "/sys", env=None) -> Dict:
    """{'pci', 'numa_node', 'node_cpus'} of HIP device `gpu_index` (numa_node
    -1 / node_cpus [] when the topology does not say)."""
    env = os.environ if env is None else env
    addrs = _visible(gpu_pci_addresses(sysfs), env)
    if not addrs or gpu_index >= len(addrs):
        return {"pci": None, "numa_node": -1, "node_cpus": []}
    pci = addrs[gpu_index]
    node = _read(os.path.join(sysfs, "bus/pci/devices", pci, "numa_node"))
    node_i = int(node) if node is not None and node.lstrip("-").isdigit() else -1
    cpus = parse_cpulist(_read(os.path.join(sysfs, f"devices/system/node/node{node_i}/cpulist")) or "") \
        if node_i >= 0 else []
    return {"pci": pci, "numa_node": node_i, "node_cpus": cpus}


def _fmt(cpus) -> str:
    cpus = sorted(cpus)
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(runs)


def bind(gpu_index: int, sysfs: str = "/sys", env=None) -> Dict:
    """Restrict this process to the CPUs of its GPU's NUMA node (intersected
    with the current affinity mask; unchanged when that would be empty or the
    node is unknown).  Returns a report for the bench line."""
    info = gpu_numa(gpu_index, sysfs, env)
    before = set(os.sched_getaffinity(0))
    want = before & set(info["node_cpus"])
    if want and want != before:
        os.sched_setaffinity(0, want)
    return {"gpu_index": gpu_index, "pci": info["pci"], "numa_node": info["numa_node"],
            "affinity": _fmt(os.sched_getaffinity(0)), "bound": bool(want),
            "note": None if info["numa_node"] >= 0 else "GPU NUMA node unknown: affinity unchanged"}
