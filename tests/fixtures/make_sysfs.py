#!/usr/bin/env python3
"""Generate the fake sysfs/devfs trees under tests/fixtures/sysfs/.

Each tree is a ROOT for libmxnode (``--root``): it holds the KFD topology
(``sys/class/kfd/kfd/topology/nodes/*``), the PCI attributes libmxnode reads
(``sys/bus/pci/devices/<bdf>/{numa_node,drm/card*}``) and placeholder device
nodes (``dev/kfd``, ``dev/dri/renderD*``).

Property values follow what an MI355X node reports (gfx_target_version 90500,
device_id 0x75a3, 1024 SIMDs = 256 CUs, 288 GB HBM3E, 7 xGMI links at
weight 15 / 76000 Mb/s, PCIe at weight 20) — the single-GPU tree mirrors the
view from inside a 1-GPU container captured on the gpurun box
(scripts/capture_node.sh), where KFD hides the GPUs the container cannot open.

    python tests/fixtures/make_sysfs.py      # regenerates all trees
"""
from __future__ import annotations

import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "sysfs")
TOPO = "sys/class/kfd/kfd/topology/nodes"

MI355X_BDFS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
               "0000:85:00.0", "0000:95:00.0", "0000:e5:00.0", "0000:f5:00.0"]
HIVE = 0xA20DCAFE9B2F58BC
VRAM = 309220868096


def _w(root: str, rel: str, text: str) -> None:
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(text)


def _props(d: dict) -> str:
    return "".join(f"{k} {v}\n" for k, v in d.items())


def _loc(bdf: str) -> tuple[int, int]:
    dom, bus, devfn = bdf.split(":")
    dev, fn = devfn.split(".")
    return int(dom, 16), (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)


def cpu_node(root: str, node: int, numa_links: list[tuple[int, int]]) -> None:
    p = {"cpu_cores_count": 128, "simd_count": 0, "mem_banks_count": 1, "caches_count": 0,
         "io_links_count": len(numa_links), "p2p_links_count": 0, "cpu_core_id_base": 128 * node,
         "simd_id_base": 0, "max_waves_per_simd": 0, "lds_size_in_kb": 0, "gds_size_in_kb": 0,
         "num_gws": 0, "wave_front_size": 0, "array_count": 0, "simd_arrays_per_engine": 0,
         "cu_per_simd_array": 0, "simd_per_cu": 0, "max_slots_scratch_cu": 0,
         "gfx_target_version": 0, "vendor_id": 0, "device_id": 0, "location_id": 0,
         "domain": 0, "drm_render_minor": 0, "hive_id": 0, "num_sdma_engines": 0,
         "num_sdma_xgmi_engines": 0, "num_sdma_queues_per_engine": 0, "num_cp_queues": 0,
         "max_engine_clk_ccompute": 5008}
    base = f"{TOPO}/{node}"
    _w(root, f"{base}/properties", _props(p))
    _w(root, f"{base}/gpu_id", "0\n")
    _w(root, f"{base}/name", "\n")
    _w(root, f"{base}/mem_banks/0/properties",
       _props({"heap_type": 0, "size_in_bytes": 1623497555968, "flags": 0, "width": 64,
               "mem_clk_max": 6400}))
    for k, (to, typ) in enumerate(numa_links):
        _w(root, f"{base}/io_links/{k}/properties", _link(node, to, typ, 20, 0))


def _link(frm: int, to: int, typ: int, weight: int, bw: int) -> str:
    return _props({"type": typ, "version_major": 0, "version_minor": 0, "node_from": frm,
                   "node_to": to, "weight": weight, "min_latency": 0, "max_latency": 0,
                   "min_bandwidth": bw, "max_bandwidth": bw, "recommended_transfer_size": 0,
                   "recommended_sdma_engine_id_mask": 0, "flags": 1})


def gpu_node(root: str, node: int, idx: int, bdf: str, numa: int, cpu_node_id: int,
             peers: list[int], vendor: int = 4098, device: int = 0x75A3,
             gfx: int = 90500, render: bool = True) -> None:
    dom, loc = _loc(bdf)
    p = {"cpu_cores_count": 0, "simd_count": 1024, "mem_banks_count": 1, "caches_count": 0,
         "io_links_count": 1 + len(peers), "p2p_links_count": 0, "cpu_core_id_base": 0,
         "simd_id_base": 2147487744 + 1024 * idx, "max_waves_per_simd": 8,
         "lds_size_in_kb": 160, "gds_size_in_kb": 0, "num_gws": 64, "wave_front_size": 64,
         "array_count": 32, "simd_arrays_per_engine": 1, "cu_per_simd_array": 8,
         "simd_per_cu": 4, "max_slots_scratch_cu": 32, "gfx_target_version": gfx,
         "vendor_id": vendor, "device_id": device, "location_id": loc, "domain": dom,
         "drm_render_minor": 128 + idx, "hive_id": HIVE if peers else 0,
         "num_sdma_engines": 2, "num_sdma_xgmi_engines": 14, "num_sdma_queues_per_engine": 8,
         "num_cp_queues": 24, "max_engine_clk_fcompute": 2400, "local_mem_size": 0,
         "fw_version": 177, "capability": 1017308800, "debug_prop": 1495,
         "sdma_fw_version": 24, "unique_id": 0xF4071D07E8AC5500 + idx, "num_xcc": 8,
         "max_engine_clk_ccompute": 5008}
    base = f"{TOPO}/{node}"
    _w(root, f"{base}/properties", _props(p))
    _w(root, f"{base}/gpu_id", f"{16000 + 137 * idx}\n")
    _w(root, f"{base}/name", "gfx950\n")
    _w(root, f"{base}/mem_banks/0/properties",
       _props({"heap_type": 1, "size_in_bytes": VRAM, "flags": 0, "width": 8192,
               "mem_clk_max": 2000}))
    _w(root, f"{base}/io_links/0/properties", _link(node, cpu_node_id, 2, 20, 64000))
    for k, peer in enumerate(peers):
        _w(root, f"{base}/io_links/{k + 1}/properties", _link(node, peer, 11, 15, 76000))
    pci = f"sys/bus/pci/devices/{bdf}"
    _w(root, f"{pci}/numa_node", f"{numa}\n")
    _w(root, f"{pci}/vendor", f"0x{vendor:04x}\n")
    _w(root, f"{pci}/device", f"0x{device:04x}\n")
    # a uevent file in each drm child keeps the directory alive in git
    # (git drops empty directories, and discovery keys off their names)
    _w(root, f"{pci}/drm/card{idx + 1}/uevent", f"MAJOR=226\nMINOR={idx + 1}\n")
    _w(root, f"{pci}/drm/renderD{128 + idx}/uevent", f"MAJOR=226\nMINOR={128 + idx}\n")
    if render:
        _w(root, f"dev/dri/renderD{128 + idx}", "")
    _w(root, f"dev/dri/card{idx + 1}", "")


def tree_8gpu(root: str, missing_render: int | None = None, ngpu: int = 8) -> None:
    gpu_nodes = list(range(2, 2 + ngpu))
    cpu_node(root, 0, [(n, 2) for i, n in enumerate(gpu_nodes) if i < 4])
    cpu_node(root, 1, [(n, 2) for i, n in enumerate(gpu_nodes) if i >= 4])
    for i, n in enumerate(gpu_nodes):
        numa = 0 if i < 4 else 1
        peers = [m for m in gpu_nodes if m != n]
        gpu_node(root, n, i, MI355X_BDFS[i], numa, numa, peers,
                 render=(i != missing_render))
    _w(root, "dev/kfd", "")


PARTS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
NPS = {"NPS1": 1, "NPS2": 2, "NPS4": 4}


def write_partition_files(root: str, bdf: str, compute: str, memory: str) -> None:
    pci = f"sys/bus/pci/devices/{bdf}"
    _w(root, f"{pci}/current_compute_partition", compute + "\n")
    _w(root, f"{pci}/available_compute_partition", "SPX, DPX, QPX, CPX\n")
    _w(root, f"{pci}/current_memory_partition", memory + "\n")
    _w(root, f"{pci}/available_memory_partition", "NPS1, NPS2\n")


def tree_partitioned(root: str, compute: str = "CPX", memory: str = "NPS2", ngpu: int = 8) -> None:
    """An MI355X node in a DPX/QPX/CPX compute mode: every PCI device shows up
    as `parts` KFD nodes (num_xcc 8/parts, simd_count 1024/parts, the same BDF),
    each with its own render node and card; local memory split by the NPS mode.
    The partition sysfs files reflect the modes (tests use this as the state a
    driver would reach after a partition change)."""
    parts = PARTS[compute]
    nodes = list(range(2, 2 + ngpu * parts))
    cpu_node(root, 0, [(n, 2) for i, n in enumerate(nodes) if i // parts < 4])
    cpu_node(root, 1, [(n, 2) for i, n in enumerate(nodes) if i // parts >= 4])
    for gi in range(ngpu):
        numa = 0 if gi < 4 else 1
        bdf = MI355X_BDFS[gi]
        peers = [nodes[pg * parts] for pg in range(ngpu) if pg != gi]
        for k in range(parts):
            idx = gi * parts + k
            n = nodes[idx]
            gpu_node(root, n, idx, bdf, numa, numa, peers if k == 0 else [])
            props_path = os.path.join(root, TOPO, str(n), "properties")
            text = open(props_path).read()
            text = text.replace("simd_count 1024\n", f"simd_count {1024 // parts}\n")
            text = text.replace("num_xcc 8\n", f"num_xcc {8 // parts}\n")
            text = text.replace("array_count 32\n", f"array_count {32 // parts}\n")
            text = text.replace("hive_id 0\n", f"hive_id {HIVE}\n")   # one hive, every partition
            open(props_path, "w").write(text)
            _w(root, f"{TOPO}/{n}/mem_banks/0/properties",
               _props({"heap_type": 1, "size_in_bytes": VRAM // NPS[memory], "flags": 0,
                       "width": 8192, "mem_clk_max": 2000}))
        write_partition_files(root, bdf, compute, memory)
    _w(root, "dev/kfd", "")


def tree_1gpu(root: str) -> None:
    # the 1-GPU container view: one CPU node + the visible GPU at KFD node 8
    cpu_node(root, 1, [(8, 2)])
    gpu_node(root, 8, 0, "0000:d9:00.0", 1, 1, [])
    _w(root, "dev/kfd", "")


def tree_mixed(root: str) -> None:
    cpu_node(root, 0, [(1, 2), (2, 2)])
    gpu_node(root, 1, 0, "0000:05:00.0", 0, 0, [])
    # a non-AMD accelerator node (vendor 0x10de) must be ignored
    gpu_node(root, 2, 1, "0000:15:00.0", 0, 0, [], vendor=0x10DE, device=0x2330, gfx=0)
    _w(root, "dev/kfd", "")


def main() -> None:
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    tree_8gpu(os.path.join(OUT, "mi355x_8gpu"))
    tree_1gpu(os.path.join(OUT, "mi355x_1gpu"))
    tree_mixed(os.path.join(OUT, "mixed_nonamd"))
    tree_8gpu(os.path.join(OUT, "missing_render"), missing_render=3)
    os.makedirs(os.path.join(OUT, "no_driver", "sys"), exist_ok=True)
    _w(os.path.join(OUT, "no_driver"), "sys/README", "no KFD topology: amdgpu not loaded\n")
    print(f"fixtures written to {OUT}")


if __name__ == "__main__":
    main()
