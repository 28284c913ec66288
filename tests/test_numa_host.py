"""NUMA placement helper (celestia_da/numa.py) on a fake sysfs tree: KFD
topology order, PCI address from location_id/domain, visible-device
filtering, node cpulist parsing, and bind() keeping the mask when the node is
unknown."""
import os

from celestia_da import numa


def _node(root, n, props):
    d = root / "class/kfd/kfd/topology/nodes" / str(n)
    d.mkdir(parents=True)
    (d / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))


def _fake(tmp_path):
    _node(tmp_path, 0, {"cpu_cores_count": 64, "simd_count": 0})
    # GPU 0 at 0000:05:00.0, GPU 1 at 0001:85:00.0
    _node(tmp_path, 1, {"simd_count": 1024, "location_id": 0x05 << 8, "domain": 0})
    _node(tmp_path, 2, {"simd_count": 1024, "location_id": 0x85 << 8, "domain": 1})
    for pci, node in (("0000:05:00.0", 0), ("0001:85:00.0", 1)):
        d = tmp_path / "bus/pci/devices" / pci
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cpus in ((0, "0-3,8"), (1, "4-7,9-10")):
        d = tmp_path / f"devices/system/node/node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    return str(tmp_path)


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.parse_cpulist("") == []


def test_topology_order_and_nodes(tmp_path):
    root = _fake(tmp_path)
    assert numa.gpu_pci_addresses(root) == ["0000:05:00.0", "0001:85:00.0"]
    g1 = numa.gpu_numa(1, root, env={})
    assert g1 == {"pci": "0001:85:00.0", "numa_node": 1, "node_cpus": [4, 5, 6, 7, 9, 10]}
    # visible-device filtering renumbers the devices
    g0 = numa.gpu_numa(0, root, env={"ROCR_VISIBLE_DEVICES": "1"})
    assert g0["pci"] == "0001:85:00.0" and g0["numa_node"] == 1
    assert numa.gpu_numa(5, root, env={})["numa_node"] == -1


def test_bind_restricts_or_keeps_mask(tmp_path):
    root = _fake(tmp_path)
    before = os.sched_getaffinity(0)
    try:
        r = numa.bind(0, root, env={})
        want = before & {0, 1, 2, 3, 8}
        assert r["numa_node"] == 0 and r["bound"] == bool(want)
        if want:
            assert os.sched_getaffinity(0) == want
        os.sched_setaffinity(0, before)
        r = numa.bind(0, str(tmp_path / "nowhere"), env={})
        assert r["numa_node"] == -1 and not r["bound"] and os.sched_getaffinity(0) == before
    finally:
        os.sched_setaffinity(0, before)


def test_hip_and_cuda_visible_both_set(tmp_path):
    # HIP honours HIP_VISIBLE_DEVICES over CUDA_VISIBLE_DEVICES (one of them,
    # not both in sequence): launchers often set both to the same list
    root = _fake(tmp_path)
    env = {"HIP_VISIBLE_DEVICES": "1", "CUDA_VISIBLE_DEVICES": "1"}
    assert numa.gpu_numa(0, root, env=env)["pci"] == "0001:85:00.0"
    # CUDA_VISIBLE_DEVICES alone still applies; ROCR filters first
    assert numa.gpu_numa(0, root, env={"CUDA_VISIBLE_DEVICES": "1"})["pci"] == "0001:85:00.0"
    env = {"ROCR_VISIBLE_DEVICES": "1,0", "HIP_VISIBLE_DEVICES": "1", "CUDA_VISIBLE_DEVICES": "0"}
    assert numa.gpu_numa(0, root, env=env)["pci"] == "0000:05:00.0"


def test_gpu_links_xgmi_and_pcie(tmp_path):
    root = _fake(tmp_path)
    base = tmp_path / "class/kfd/kfd/topology/nodes"

    def link(n, i, props):
        d = base / str(n) / "io_links" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))

    link(1, 0, {"type": 2, "node_from": 1, "node_to": 0, "weight": 20})   # GPU 0 -> CPU over PCIe
    link(1, 1, {"type": 11, "node_from": 1, "node_to": 2, "weight": 15})  # GPU 0 <-> GPU 1 over xGMI
    link(2, 0, {"type": 11, "node_from": 2, "node_to": 1, "weight": 15})
    got = numa.gpu_links(root)
    assert got["0000:05:00.0"] == {"xgmi": ["0001:85:00.0"], "pcie_peers": [], "pcie_to_cpu": 1}
    assert got["0001:85:00.0"]["xgmi"] == ["0000:05:00.0"]
    assert numa.gpu_links(str(tmp_path / "nowhere")) == {}
