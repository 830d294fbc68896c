"""MI355X node discovery: which GPUs an agent has, what they are, and how they are wired.

The reference's only GPU surface is the Mesos scalar resource ``gpus`` (``offer/Constants.java:62``),
the ``GPU_RESOURCES`` framework capability (``framework/FrameworkRunner.java:191-194``) and its
capability gate (``config/validate/PodSpecsCannotUseUnsupportedFeatures.java:30-47``). An agent there
advertises a GPU *count*; which devices a task gets is the containerizer's business. On an MI355X
node that choice matters: the eight GPUs of a node are joined point to point by xGMI (7 links per
GPU) inside one *hive*, and a node can also be split into several hives (partitioned systems) or
mix GPU models. This module turns what the node reports into

* agent resources: ``gpus`` = the number of visible GPUs;
* agent attributes: ``gpu_vendor`` (``amd``), ``gpu_model`` (``MI355X``), ``gpu_arch``
  (``gfx950``) and ``xgmi_hive`` (the hive id, ``none`` for a GPU without xGMI peers), so the
  Marathon-style placement language already works on them (``[["xgmi_hive","GROUP_BY"]]``,
  ``[["xgmi_hive","CLUSTER","<id>"]]``, ``[["gpu_model","LIKE","MI35.*"]]``);
* a device topology the agent uses to pick *which* devices a ``gpus: N`` task gets
  (:func:`select_devices`: all N inside one hive when any hive has N free, best fit first).

Three sources, tried in this order by :func:`discover`, each parsed from its recorded text so tests
run from fixtures (``tests/fixtures/gpu/``; there is no driver in the build container):

1. the KFD topology in sysfs (``/sys/class/kfd/kfd/topology/nodes/*/properties`` and
   ``io_links/*/properties``): device order, ``gfx_target_version``, ``hive_id``, ``unique_id``,
   CU count (``simd_count / simd_per_cu``), and xGMI links (io-link ``type 11``). No subprocess;
2. ``amd-smi static --json``: the marketing name (``asic.market_name``), ``device_id``, BDF, VRAM;
3. ``rocminfo``: agent blocks (``Marketing Name``, ``Name: gfx950``, ``Compute Unit``).

The KFD view is the authority for order and wiring; amd-smi / rocminfo only refine the model name.
``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` (the process's own, or given) restrict the result
the way the HIP runtime does. ``SDK_GPU_DISCOVERY_FIXTURE=<dir>`` points every source at a
recorded directory (``kfd/``, ``amd_smi_static.json``, ``rocminfo.txt``) instead of the live node.
"""
from __future__ import annotations

import json
import logging
import os
import re
import socket
import subprocess
from dataclasses import dataclass, field, replace
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, Tuple, Union

LOGGER = logging.getLogger(__name__)

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology"
IOLINK_TYPE_XGMI = 11  # kfd_ioctl.h / kfd_crat.h: CRAT_IOLINK_TYPE_XGMI
AMD_VENDOR_ID = 0x1002
NO_HIVE = "none"

# PCI device id -> model, for when no amd-smi/rocminfo marketing name is at hand (KFD only)
_DEVICE_MODELS = {
    0x75A3: "MI355X",
    0x75A0: "MI350X",
    0x74A5: "MI325X",
    0x74A1: "MI300X",
    0x74A9: "MI300X",
    0x74A2: "MI308X",
    0x74A0: "MI300A",
    0x740C: "MI250X",
    0x740F: "MI210",
}
# gfx target -> model family when nothing better is known
_ARCH_FAMILIES = {"gfx950": "MI350", "gfx942": "MI300", "gfx90a": "MI200", "gfx908": "MI100"}


@dataclass(frozen=True)
class GpuDevice:
    index: int                      # HIP device index on the node (order of the KFD GPU nodes)
    arch: str = ""                  # gfx target, e.g. "gfx950"
    model: str = ""                 # "MI355X"
    vendor: str = "amd"
    compute_units: int = 0
    vram_mib: int = 0
    hive: str = NO_HIVE             # xGMI hive id (hex), NO_HIVE without xGMI peers
    xgmi_peers: Tuple[int, ...] = ()  # HIP indices reachable over a direct xGMI link
    xgmi_links: int = 0             # direct xGMI links to any GPU of the node, visible or not
    kfd_node: Optional[int] = None
    unique_id: str = ""
    device_id: int = 0
    bdf: str = ""


@dataclass
class GpuInventory:
    devices: List[GpuDevice] = field(default_factory=list)
    source: str = "none"

    @property
    def count(self) -> int:
        return len(self.devices)

    def device(self, index: int) -> GpuDevice:
        for d in self.devices:
            if d.index == index:
                return d
        raise KeyError(index)

    def hives(self) -> Dict[str, List[int]]:
        out: Dict[str, List[int]] = {}
        for d in self.devices:
            out.setdefault(d.hive, []).append(d.index)
        return out

    def subset(self, indices: Iterable[int]) -> "GpuInventory":
        keep = set(indices)
        return GpuInventory([d for d in self.devices if d.index in keep], self.source)

    def attributes(self) -> Dict[str, str]:
        """Mesos agent attributes for these devices (text). Mixed values are joined with ``+``
        in device order, so a placement rule can still match them (``LIKE``/``UNLIKE``)."""
        if not self.devices:
            return {}

        def joined(values: Sequence[str]) -> str:
            seen: List[str] = []
            for v in values:
                if v and v not in seen:
                    seen.append(v)
            return "+".join(seen)

        attrs = {"gpu_vendor": joined([d.vendor for d in self.devices]) or "amd",
                 "gpu_model": joined([d.model for d in self.devices]),
                 "gpu_arch": joined([d.arch for d in self.devices]),
                 "xgmi_hive": joined([d.hive for d in self.devices]) or NO_HIVE}
        return {k: v for k, v in attrs.items() if v}

    def hive_map(self) -> Dict[int, str]:
        return {d.index: d.hive for d in self.devices}

    def to_dict(self) -> dict:
        return {"source": self.source, "devices": [
            {"index": d.index, "arch": d.arch, "model": d.model, "vendor": d.vendor, "compute_units": d.compute_units,
             "vram_mib": d.vram_mib, "hive": d.hive, "xgmi_peers": list(d.xgmi_peers), "xgmi_links": d.xgmi_links,
             "kfd_node": d.kfd_node,
             "unique_id": d.unique_id, "device_id": d.device_id, "bdf": d.bdf} for d in self.devices]}

    @staticmethod
    def from_dict(d: Mapping) -> "GpuInventory":
        return GpuInventory([GpuDevice(index=int(x["index"]), arch=x.get("arch", ""), model=x.get("model", ""),
                                       vendor=x.get("vendor", "amd"), compute_units=int(x.get("compute_units", 0)),
                                       vram_mib=int(x.get("vram_mib", 0)), hive=x.get("hive", NO_HIVE),
                                       xgmi_peers=tuple(int(p) for p in x.get("xgmi_peers", ())),
                                       xgmi_links=int(x.get("xgmi_links", 0)),
                                       kfd_node=x.get("kfd_node"), unique_id=x.get("unique_id", ""),
                                       device_id=int(x.get("device_id", 0)), bdf=x.get("bdf", ""))
                             for x in d.get("devices", ())], d.get("source", "dict"))


# -- KFD topology ----------------------------------------------------------------------------
def _read(path: str) -> Optional[str]:
    try:
        with open(path, "r", encoding="utf-8", errors="replace") as f:
            return f.read()
    except OSError:
        return None


def parse_kfd_properties(text: str) -> Dict[str, int]:
    """``key value`` lines of a KFD ``properties`` file (values are decimal integers)."""
    out: Dict[str, int] = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                continue
    return out


def arch_from_gfx_target_version(v: int) -> str:
    """KFD ``gfx_target_version`` (major*10000 + minor*100 + stepping, e.g. 90500) -> ``gfx950``."""
    if v <= 0:
        return ""
    major, minor, step = v // 10000, (v // 100) % 100, v % 100
    return f"gfx{major}{minor:x}{step:x}"


def _model_for(device_id: int, arch: str) -> str:
    if device_id in _DEVICE_MODELS:
        return _DEVICE_MODELS[device_id]
    return _ARCH_FAMILIES.get(arch, arch)


def parse_kfd_topology(root: str) -> GpuInventory:
    """GPU nodes (``simd_count > 0``) of a KFD topology tree, in node order = HIP device order."""
    nodes_dir = os.path.join(root, "nodes")
    try:
        names = sorted((n for n in os.listdir(nodes_dir) if n.isdigit()), key=int)
    except OSError:
        return GpuInventory([], "kfd")
    gpu_nodes: List[Tuple[int, Dict[str, int]]] = []
    restricted = 0
    for n in names:
        text = _read(os.path.join(nodes_dir, n, "properties"))
        if not text:
            # a GPU this process was not granted: the kernel hands out an empty properties file
            restricted += 1
            continue
        props = parse_kfd_properties(text)
        if props.get("simd_count", 0) > 0 and props.get("vendor_id", AMD_VENDOR_ID) in (AMD_VENDOR_ID, 0):
            gpu_nodes.append((int(n), props))
    index_of_node = {node: i for i, (node, _) in enumerate(gpu_nodes)}
    devices = []
    for i, (node, props) in enumerate(gpu_nodes):
        peers = set()
        xgmi_to = set()
        for links in ("io_links", "p2p_links"):
            ldir = os.path.join(nodes_dir, str(node), links)
            try:
                entries = sorted(os.listdir(ldir))
            except OSError:
                continue
            for e in entries:
                lp = _read(os.path.join(ldir, e, "properties"))
                if lp is None:
                    continue
                link = parse_kfd_properties(lp)
                to = link.get("node_to")
                if link.get("type") == IOLINK_TYPE_XGMI and to != node:
                    xgmi_to.add(to)
                    if to in index_of_node:
                        peers.add(index_of_node[to])
        arch = arch_from_gfx_target_version(props.get("gfx_target_version", 0))
        simd_per_cu = props.get("simd_per_cu", 4) or 4
        hive_id = props.get("hive_id", 0)
        devices.append(GpuDevice(
            index=i, arch=arch, model=_model_for(props.get("device_id", 0), arch),
            compute_units=props.get("simd_count", 0) // simd_per_cu,
            vram_mib=props.get("local_mem_size", 0) // (1 << 20),
            hive=f"{hive_id:x}" if hive_id else NO_HIVE, xgmi_peers=tuple(sorted(peers)), xgmi_links=len(xgmi_to),
            kfd_node=node,
            unique_id=f"{props['unique_id']:x}" if props.get("unique_id") else "",
            device_id=props.get("device_id", 0),
            bdf=_bdf_from_location(props.get("domain", 0), props.get("location_id", 0))))
    inv = GpuInventory(devices, "kfd")
    inv.restricted_nodes = restricted
    return inv


def _bdf_from_location(domain: int, location_id: int) -> str:
    """KFD ``location_id`` is ``(bus << 8) | (device << 3) | function``."""
    if not location_id:
        return ""
    return f"{domain:04x}:{(location_id >> 8) & 0xFF:02x}:{(location_id >> 3) & 0x1F:02x}.{location_id & 0x7}"


def parse_kfd_xgmi_links(root: str) -> Dict[int, set]:
    """KFD node -> the nodes it has a direct xGMI io/p2p link to. Link files stay readable where a
    node's own ``properties`` are not (a container granted one GPU of the node: the kernel's device
    cgroup check empties the other GPUs' properties, and its own)."""
    nodes_dir = os.path.join(root, "nodes")
    out: Dict[int, set] = {}
    try:
        names = [n for n in os.listdir(nodes_dir) if n.isdigit()]
    except OSError:
        return out
    for n in names:
        for links in ("io_links", "p2p_links"):
            ldir = os.path.join(nodes_dir, n, links)
            try:
                entries = os.listdir(ldir)
            except OSError:
                continue
            for e in entries:
                lp = _read(os.path.join(ldir, e, "properties"))
                link = parse_kfd_properties(lp or "")
                if link.get("type") == IOLINK_TYPE_XGMI and "node_to" in link and link["node_to"] != int(n):
                    out.setdefault(int(n), set()).add(link["node_to"])
                    out.setdefault(link["node_to"], set()).add(int(n))
    return out


def xgmi_hives(links: Mapping[int, Iterable[int]], label: str) -> Dict[int, str]:
    """KFD node -> hive label: the connected components of the xGMI link graph. Without readable
    ``hive_id``s the label is ``<label>:<lowest node of the component>`` (``label`` = the host: a
    hive never spans hosts, so host plus component is unique across the cluster)."""
    out: Dict[int, str] = {}
    for start in sorted(links):
        if start in out:
            continue
        comp, stack = set(), [start]
        while stack:
            x = stack.pop()
            if x in comp:
                continue
            comp.add(x)
            stack.extend(links.get(x, ()))
        name = f"{label}:{min(comp)}"
        for x in comp:
            out[x] = name
    return out


def parse_amd_smi_list(text: str) -> Dict[int, int]:
    """``amd-smi list --json``: visible GPU index -> its KFD topology node (``node_id``)."""
    data = json.loads(text)
    if isinstance(data, dict):
        data = data.get("gpu_data", [data])
    out = {}
    for g in data or []:
        if isinstance(g, dict) and "gpu" in g and isinstance(g.get("node_id"), int):
            out[_int(g["gpu"])] = g["node_id"]
    return out


def attach_kfd_wiring(inv: GpuInventory, node_of: Mapping[int, int], links: Mapping[int, Iterable[int]],
                      label: str) -> GpuInventory:
    """Hive and xGMI peers of tool-enumerated devices from the KFD link graph, through the
    device -> KFD node map of ``amd-smi list``."""
    if not node_of or not links:
        return inv
    hive_of_node = xgmi_hives(links, label)
    idx_of_node = {node_of[d.index]: d.index for d in inv.devices if d.index in node_of}
    devices = []
    for d in inv.devices:
        node = node_of.get(d.index)
        if node is None:
            devices.append(d)
            continue
        peers = tuple(sorted(idx_of_node[p] for p in links.get(node, ()) if p in idx_of_node))
        devices.append(replace(d, kfd_node=node, hive=hive_of_node.get(node, NO_HIVE), xgmi_peers=peers,
                               xgmi_links=len(set(links.get(node, ())))))
    return GpuInventory(devices, inv.source + "+kfd-links")


# -- amd-smi ------------------------------------------------------------------------------------
def _int(v) -> int:
    if isinstance(v, int):
        return v
    if isinstance(v, str):
        try:
            return int(v, 0)
        except ValueError:
            return 0
    return 0


def model_from_market_name(name: str) -> str:
    """``AMD Instinct MI355X`` -> ``MI355X`` (the token naming the accelerator)."""
    m = re.search(r"\b(MI\d{3}[A-Z]*)\b", name or "", re.IGNORECASE)
    if m:
        return m.group(1).upper()
    return (name or "").replace("AMD Instinct", "").strip()


def _best_model(market: str, device_id: int, arch: str) -> str:
    """The marketing name's model, unless the PCI device id names the same part more precisely
    (the MI355X box reports ``AMD Instinct MI355 OAM`` for device 0x75a3)."""
    known = _DEVICE_MODELS.get(device_id, "")
    if known and (not market or known.startswith(market)):
        return known
    return market or _model_for(device_id, arch)


def parse_amd_smi_static(text: str) -> GpuInventory:
    """``amd-smi static --json``: a list of per-GPU objects (or ``{"gpu_data": [...]}``) with
    ``gpu``, ``asic{market_name, device_id, num_compute_units, target_graphics_version}``,
    ``bus{bdf}``, ``vram{size{value, unit}}``."""
    data = json.loads(text)
    if isinstance(data, dict):
        data = data.get("gpu_data", data.get("gpus", [data]))
    devices = []
    for i, g in enumerate(data or []):
        if not isinstance(g, dict):
            continue
        asic = g.get("asic") if isinstance(g.get("asic"), dict) else {}
        bus = g.get("bus") if isinstance(g.get("bus"), dict) else {}
        vram = g.get("vram") if isinstance(g.get("vram"), dict) else {}
        size = vram.get("size")
        mib = 0
        if isinstance(size, dict):
            mib = _int(size.get("value"))
            if str(size.get("unit", "MB")).upper() in ("GB", "GIB"):
                mib *= 1024
        arch = asic.get("target_graphics_version") or ""
        arch = arch if isinstance(arch, str) and arch.startswith("gfx") else ""
        devices.append(GpuDevice(
            index=_int(g.get("gpu", i)), arch=arch,
            model=_best_model(model_from_market_name(str(asic.get("market_name", ""))), _int(asic.get("device_id")), arch),
            compute_units=_int(asic.get("num_compute_units")), vram_mib=mib,
            device_id=_int(asic.get("device_id")), bdf=str(bus.get("bdf", "")) if bus.get("bdf") != "N/A" else ""))
    return GpuInventory(devices, "amd-smi")


# -- rocminfo -----------------------------------------------------------------------------------
def parse_rocminfo(text: str) -> GpuInventory:
    """GPU agent blocks of ``rocminfo`` (``Device Type: GPU``), in agent order."""
    devices = []
    for block in re.split(r"\n\*+\s*\nAgent \d+\s*\n\*+\s*\n", "\n" + text):
        fields: Dict[str, str] = {}
        for line in block.splitlines():
            m = re.match(r"^  ([A-Za-z][A-Za-z0-9 ()#/_-]*?):\s+(.*?)\s*$", line)
            if m and m.group(1) not in fields:
                fields[m.group(1)] = m.group(2)
        if fields.get("Device Type") != "GPU":
            continue
        chip = re.search(r"\((0x[0-9a-fA-F]+)\)", fields.get("Chip ID", ""))
        node = fields.get("Node")
        arch = fields.get("Name", "") if fields.get("Name", "").startswith("gfx") else ""
        device_id = int(chip.group(1), 16) if chip else 0
        # rocminfo's "Node" numbers the runtime's agents, not KFD topology nodes
        devices.append(GpuDevice(
            index=len(devices), arch=arch,
            model=_best_model(model_from_market_name(fields.get("Marketing Name", "")), device_id, arch),
            compute_units=_int(fields.get("Compute Unit", "0")), device_id=device_id))
    return GpuInventory(devices, "rocminfo")


# -- merge / visibility / discover --------------------------------------------------------------
def merge(base: GpuInventory, *refinements: GpuInventory) -> GpuInventory:
    """``base`` (order, wiring) with model / arch / CUs / VRAM / BDF filled in from the
    refinements, matched by device index (same enumeration order for all three tools)."""
    devices = list(base.devices)
    for ref in refinements:
        by_index = {d.index: d for d in ref.devices}
        for i, d in enumerate(devices):
            r = by_index.get(d.index)
            if r is None:
                continue
            devices[i] = replace(d, model=r.model or d.model, arch=d.arch or r.arch,
                                 compute_units=d.compute_units or r.compute_units, vram_mib=d.vram_mib or r.vram_mib,
                                 bdf=d.bdf or r.bdf, device_id=d.device_id or r.device_id)
    return GpuInventory(devices, "+".join([base.source] + [r.source for r in refinements if r.devices]))


def parse_visible_devices(value: Optional[str]) -> Optional[List[Union[int, str]]]:
    """``HIP_VISIBLE_DEVICES``-style list (``0,2,3``, or ROCm's ``GPU-<unique id>`` UUIDs, which
    come back as strings); None when unset or empty (the ROCm runtime only filters on a non-empty
    value; containers often export the variable empty)."""
    if value is None:
        return None
    value = value.strip()
    if not value:
        return None
    out: List[Union[int, str]] = []
    for tok in value.split(","):
        tok = tok.strip()
        if tok.isdigit():
            out.append(int(tok))
        elif tok:
            out.append(tok)
    return out


def _uuid_key(tok: str) -> str:
    t = tok.lower()
    if t.startswith("gpu-"):
        t = t[4:]
    return t.lstrip("0") or "0"


def _resolve_selection(sel: List[Union[int, str]], devices: List["GpuDevice"]) -> Optional[List[int]]:
    """Positions in ``devices`` that ``sel`` names: an index, or a UUID matched against the
    device's KFD ``unique_id``. None when a token names nothing this inventory can identify (the
    caller then does not filter, rather than silently advertising zero GPUs: ADVICE r5)."""
    by_uuid = {_uuid_key(d.unique_id): n for n, d in enumerate(devices) if d.unique_id}
    out = []
    for tok in sel:
        if isinstance(tok, int):
            out.append(tok)
        elif _uuid_key(tok) in by_uuid:
            out.append(by_uuid[_uuid_key(tok)])
        else:
            return None
    return out


def apply_visibility(inv: GpuInventory, env: Mapping[str, str], already_filtered: bool = False) -> GpuInventory:
    """Restrict and renumber as the ROCm runtime does: ``ROCR_VISIBLE_DEVICES`` selects among the
    node's devices, then ``HIP_VISIBLE_DEVICES`` among those; the survivors are numbered 0..n-1
    (xGMI peers are kept only among the survivors). UUID entries (``GPU-<unique id>``) select the
    device with that unique id; a selection with an entry that matches no device is ignored with
    a warning."""
    devices = list(inv.devices)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        raw = parse_visible_devices(env.get(var))
        if raw is None:
            continue
        sel = _resolve_selection(raw, devices)
        if sel is None:
            LOGGER.warning("%s=%r names a device this node's inventory cannot identify; not filtering on it",
                           var, env.get(var))
            continue
        if already_filtered and any(i >= len(devices) for i in sel):
            # the tools only saw the devices this container was granted: the selection named
            # physical devices and has been applied already
            continue
        devices = [devices[i] for i in sel if 0 <= i < len(devices)]
        renumber = {d.index: n for n, d in enumerate(devices)}
        devices = [replace(d, index=n, xgmi_peers=tuple(sorted(renumber[p] for p in d.xgmi_peers if p in renumber)))
                   for n, d in enumerate(devices)]
    return GpuInventory(devices, inv.source)


def _run(cmd: List[str], timeout_s: float = 20.0) -> Optional[str]:
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, check=False)
    except (OSError, subprocess.SubprocessError):
        return None
    return p.stdout if p.returncode == 0 and p.stdout.strip() else None


_LIVE_CACHE: Dict[tuple, GpuInventory] = {}


def discover(env: Optional[Mapping[str, str]] = None, fixture_dir: Optional[str] = None,
             kfd_root: str = KFD_TOPOLOGY, use_tools: bool = True) -> GpuInventory:
    """The node's GPUs as this process would see them (see the module docstring). The live
    node's answer is cached per process (its topology does not change under a running agent)."""
    env = os.environ if env is None else env
    fixture_dir = fixture_dir or env.get("SDK_GPU_DISCOVERY_FIXTURE") or None
    if fixture_dir:
        return _discover(env, fixture_dir, os.path.join(fixture_dir, "kfd"), False)
    key = (kfd_root, use_tools, env.get("ROCR_VISIBLE_DEVICES"), env.get("HIP_VISIBLE_DEVICES"))
    inv = _LIVE_CACHE.get(key)
    if inv is None:
        # the tools need the driver (/dev/kfd); without it they only fail, slowly
        inv = _LIVE_CACHE[key] = _discover(env, None, kfd_root, use_tools and os.path.exists("/dev/kfd"))
    return GpuInventory(list(inv.devices), inv.source)


def _discover(env: Mapping[str, str], fixture_dir: Optional[str], kfd_root: str, use_tools: bool) -> GpuInventory:
    base = parse_kfd_topology(kfd_root)
    refinements: List[GpuInventory] = []
    smi_text = list_text = rocminfo_text = None
    if fixture_dir:
        smi_text = _read(os.path.join(fixture_dir, "amd_smi_static.json"))
        list_text = _read(os.path.join(fixture_dir, "amd_smi_list.json"))
        rocminfo_text = _read(os.path.join(fixture_dir, "rocminfo.txt"))
    elif use_tools:
        smi_text = _run(["amd-smi", "static", "--asic", "--bus", "--vram", "--json"])
        if smi_text is not None and not base.devices:
            list_text = _run(["amd-smi", "list", "--json"])
        if smi_text is None:
            rocminfo_text = _run(["rocminfo"])
    if smi_text:
        try:
            refinements.append(parse_amd_smi_static(smi_text))
        except (ValueError, TypeError):
            pass
    if rocminfo_text:
        refinements.append(parse_rocminfo(rocminfo_text))
    if base.devices:
        # with GPUs hidden from this container, the readable ones are already the granted subset
        return apply_visibility(merge(base, *refinements), env,
                                already_filtered=getattr(base, "restricted_nodes", 0) > 0)
    # no readable KFD GPU nodes (no driver, or a container granted only some GPUs): the tools
    # enumerate what this process may use; the KFD link graph (still readable) gives the wiring
    base = next((r for r in refinements if r.devices), GpuInventory([], "none"))
    refinements = [r for r in refinements if r is not base]
    inv = merge(base, *refinements)
    if list_text:
        try:
            node_of = parse_amd_smi_list(list_text)
        except (ValueError, TypeError):
            node_of = {}
        if fixture_dir:
            label = env.get("SDK_GPU_HOST_LABEL") or (_read(os.path.join(fixture_dir, "hostname")) or "").strip()
        else:
            label = env.get("SDK_GPU_HOST_LABEL") or socket.gethostname()
        inv = attach_kfd_wiring(inv, node_of, parse_kfd_xgmi_links(kfd_root), label or "host")
    return apply_visibility(inv, env, already_filtered=True)


# -- device selection -----------------------------------------------------------------------------
def select_devices(free: Sequence[int], count: int, hive_of: Optional[Mapping[int, str]] = None,
                   peers_of: Optional[Mapping[int, Sequence[int]]] = None) -> List[int]:
    """Which ``count`` of the ``free`` device indices a task gets.

    Topology-aware: if some hive has ``count`` free devices, all of them come from one hive --
    the one with the fewest free devices that still fits (best fit keeps whole hives free for
    bigger tasks); within it, a set whose members are pairwise xGMI peers when the link table
    allows, else the lowest indices. Without a hive that fits, devices are taken hive by hive,
    largest free group first, so the task spans as few hives as possible. Without topology the
    lowest free indices are used (the previous behaviour)."""
    free = list(free)
    if count <= 0:
        return []
    if count > len(free):
        raise ValueError(f"{count} devices requested, {len(free)} free")
    if not hive_of:
        return sorted(free)[:count]
    groups: Dict[str, List[int]] = {}
    for d in sorted(free):
        groups.setdefault(hive_of.get(d, NO_HIVE), []).append(d)
    fitting = [(len(v), k) for k, v in groups.items() if k != NO_HIVE and len(v) >= count]
    if fitting:
        _, hive = min(fitting)
        members = groups[hive]
        if peers_of and count > 1:
            clique = _xgmi_clique(members, count, peers_of)
            if clique:
                return clique
        return members[:count]
    out: List[int] = []
    for _, hive in sorted(((-len(v), k) for k, v in groups.items()), key=lambda x: (x[1] == NO_HIVE, x[0], x[1])):
        for d in groups[hive]:
            if len(out) < count:
                out.append(d)
    return sorted(out)


def _xgmi_clique(members: Sequence[int], count: int, peers_of: Mapping[int, Sequence[int]]) -> List[int]:
    """Greedy: the lowest-index set of ``count`` members that are pairwise direct xGMI peers."""
    for start in members:
        chosen = [start]
        for d in members:
            if d in chosen:
                continue
            if all(d in peers_of.get(c, ()) for c in chosen):
                chosen.append(d)
                if len(chosen) == count:
                    return sorted(chosen)
    return []


def synthetic_inventory(count: int, hives: Optional[Sequence[str]] = None, model: str = "MI355X",
                        arch: str = "gfx950") -> GpuInventory:
    """``count`` MI355X devices for nodes without a driver (build container, CPU tests): one
    fully xGMI-connected hive ``0`` unless ``hives`` gives each device's hive. ``source`` says
    ``synthetic`` so nobody mistakes it for a discovered node."""
    hives = list(hives) if hives is not None else ["0"] * count
    devices = []
    for i in range(count):
        peers = tuple(j for j in range(count) if j != i and hives[j] == hives[i] and hives[i] != NO_HIVE)
        devices.append(GpuDevice(index=i, arch=arch, model=model, compute_units=256, vram_mib=288 * 1024,
                                 hive=hives[i], xgmi_peers=peers, device_id=0x75A3))
    return GpuInventory(devices, "synthetic")


def node_inventory(min_devices: int = 0, env: Optional[Mapping[str, str]] = None) -> GpuInventory:
    """What an agent on this node advertises: the discovered GPUs, or -- when discovery finds
    fewer than ``min_devices`` (no driver, a CPU container) -- a synthetic inventory of that many
    so simulated GPU agents still carry the same resources and attributes."""
    inv = discover(env)
    if inv.count >= min_devices:
        return inv
    return synthetic_inventory(min_devices)


def synthetic_kfd_tree(root: str, hives: Sequence[int], device_id: int = 0x75A3, gfx_target_version: int = 90500,
                       cus: int = 256, vram_gib: int = 288, cpu_nodes: int = 2) -> None:
    """Writes a KFD topology tree in the sysfs layout: ``cpu_nodes`` CPU nodes, then one GPU per
    entry of ``hives`` (its xGMI hive id; GPUs of one hive are fully xGMI-connected, 0 = none).
    Used by tests and rehearsals to stand in for multi-GPU / multi-hive nodes."""
    nodes = os.path.join(root, "nodes")
    for n in range(cpu_nodes):
        d = os.path.join(nodes, str(n))
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(f"cpu_cores_count 64\nsimd_count 0\nmem_banks_count 1\nvendor_id 0\ndevice_id 0\nhive_id 0\n")
    gpu_nodes = list(range(cpu_nodes, cpu_nodes + len(hives)))
    for i, (node, hive) in enumerate(zip(gpu_nodes, hives)):
        d = os.path.join(nodes, str(node))
        os.makedirs(d, exist_ok=True)
        location = ((0x05 + 0x10 * i) << 8)
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(f"cpu_cores_count 0\nsimd_count {cus * 4}\nmem_banks_count 1\nio_links_count {len(hives)}\n"
                    f"simd_per_cu 4\nwave_front_size 64\nlds_size_in_kb 160\ngfx_target_version {gfx_target_version}\n"
                    f"vendor_id {AMD_VENDOR_ID}\ndevice_id {device_id}\nlocation_id {location}\ndomain 0\n"
                    f"hive_id {hive}\nunique_id {0xABC000 + i}\nnum_xcc 8\nlocal_mem_size {vram_gib << 30}\n")
        links = 0
        # PCIe link to the CPU node, xGMI links to every other GPU of the same hive
        for to, typ in [(0, 2)] + [(gpu_nodes[j], IOLINK_TYPE_XGMI) for j, h in enumerate(hives)
                                   if h and h == hive and j != i]:
            ld = os.path.join(d, "io_links", str(links))
            os.makedirs(ld, exist_ok=True)
            with open(os.path.join(ld, "properties"), "w") as f:
                f.write(f"type {typ}\nversion_major 0\nversion_minor 0\nnode_from {node}\nnode_to {to}\n"
                        f"weight {15 if typ == IOLINK_TYPE_XGMI else 20}\nmin_bandwidth 0\nmax_bandwidth 0\n")
            links += 1
