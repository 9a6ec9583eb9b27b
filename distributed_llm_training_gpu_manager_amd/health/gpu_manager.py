"""GPU fleet telemetry & health for MI355X via amdsmi (in-process) with an ``amd-smi --json`` fallback.

Replaces the reference's nvidia-smi parser (``ai_engine/gpu_manager.py:80-431``)
while keeping its wire contract: ``GPUDevice`` / ``GPUFleetStatus`` / ``GPUProcess``
field names and defaults, the health thresholds (``:93-98``), the escalation
order temp -> memory -> utilisation -> power and alert strings (``:348-379``),
fleet aggregation and alerts (``:275-321``), ``select_best_gpu`` (``:323-346``)
and a mock fleet for development (``:400-431``, here MI355X devices).

MI355X additions (new fields only, nothing renamed): junction (hotspot) and HBM
temperatures, HBM3E activity, xGMI link status / bandwidth per peer, ECC counts,
gfx arch. ``temperature_celsius`` carries the junction temperature because MI355X
reports no edge sensor; ``cuda_version`` carries the ROCm version.

Collection paths, in order (mirroring the reference's XML -> CSV -> empty-fleet
fallback): the amdsmi C library through its Python binding (no fork/exec per
poll) -> ``amd-smi static/metric/process/xgmi --json`` -> an empty fleet with an
alert. :meth:`GPUManager.start_polling` keeps a cached snapshot on a background
thread so REST handlers never block on the driver (fix A27).

The nvidia-smi XML/CSV parsers are kept (``parse_xml`` / ``parse_csv``) for mixed
fleets, with the ``[Not Supported]`` crash (A6) fixed.
"""
from __future__ import annotations

import json
import re
import subprocess
import threading
import time
import xml.etree.ElementTree as ET
from enum import Enum
from typing import Any, Dict, List, Optional, Tuple

from pydantic import BaseModel, Field

from ..launcher.config import utcnow


class GPUHealthStatus(str, Enum):
    HEALTHY = "healthy"
    WARNING = "warning"
    CRITICAL = "critical"
    UNREACHABLE = "unreachable"


class GPUProcess(BaseModel):
    pid: int
    name: str = ""
    used_memory_mib: int = 0
    gpu_instance_id: Optional[str] = None


class XGMILink(BaseModel):
    peer_bdf: str = ""
    status: str = "unknown"  # up | down | self | disabled | unknown
    bit_rate_gbps: float = 0.0
    max_bandwidth_gbps: float = 0.0
    read_kb: int = 0
    write_kb: int = 0


class GPUDevice(BaseModel):
    index: int
    name: str = Field(default="Unknown GPU")
    uuid: str = ""
    temperature_celsius: int = 0
    gpu_utilization_pct: float = 0.0
    memory_used_mib: int = 0
    memory_total_mib: int = 0
    memory_free_mib: int = 0
    memory_utilization_pct: float = 0.0
    power_draw_watts: float = 0.0
    power_limit_watts: float = 0.0
    fan_speed_pct: int = 0
    driver_version: str = ""
    cuda_version: str = ""
    compute_mode: str = "Default"
    pci_bus_id: str = ""
    processes: List[GPUProcess] = Field(default_factory=list)
    health: GPUHealthStatus = GPUHealthStatus.HEALTHY
    alerts: List[str] = Field(default_factory=list)
    # MI355X additions
    vendor: str = ""
    gfx_arch: str = ""
    hotspot_temperature_celsius: Optional[int] = None
    hbm_temperature_celsius: Optional[int] = None
    edge_temperature_celsius: Optional[int] = None
    memory_activity_pct: Optional[float] = None
    ecc_correctable: int = 0
    ecc_uncorrectable: int = 0
    xgmi_links: List[XGMILink] = Field(default_factory=list)
    numa_node: Optional[int] = None

    @property
    def is_available(self) -> bool:
        """Same rule as the reference: memory < 80 %, utilisation < 90 %, not critical."""
        return (self.memory_utilization_pct < 80 and self.gpu_utilization_pct < 90 and
                self.health != GPUHealthStatus.CRITICAL)


class GPUFleetStatus(BaseModel):
    timestamp: str = Field(default_factory=lambda: utcnow().isoformat())
    total_gpus: int = 0
    healthy_gpus: int = 0
    available_gpus: int = 0
    total_memory_mib: int = 0
    used_memory_mib: int = 0
    avg_utilization_pct: float = 0.0
    avg_temperature_celsius: float = 0.0
    total_power_watts: float = 0.0
    devices: List[GPUDevice] = Field(default_factory=list)
    alerts: List[str] = Field(default_factory=list)
    source: str = "none"  # amdsmi | amd-smi-cli | nvidia-smi | mock | none


# PCI device ids of the CDNA4 parts (amdsmi asic_info.device_id): used when the marketing name is generic
_DEVICE_NAMES = {"0x75a3": "AMD Instinct MI355X", "0x75a2": "AMD Instinct MI350X"}
_GENERIC = ("", "n/a", "amd radeon graphics", "amd instinct gpu", "unknown gpu")


def market_name(asic: Dict[str, Any], board: Optional[Dict[str, Any]] = None) -> str:
    """The product name of a GPU from amdsmi ASIC / board info. ``asic.market_name`` comes from libdrm's
    amdgpu.ids table; where that file is missing it reads "AMD Radeon Graphics" for every part (seen on the
    MI355X boxes), so fall back to the board FRU product name, then to the PCI device id, then to the gfx
    target (gfx950 = CDNA4 / MI350 series)."""
    asic, board = asic or {}, board or {}
    name = str(asic.get("market_name", "") or "").strip()
    if name.lower() not in _GENERIC:
        return name
    prod = str(board.get("product_name", "") or "").strip()
    if prod.lower() not in _GENERIC:
        return prod
    dev = str(asic.get("device_id", "") or "").lower()
    if dev in _DEVICE_NAMES:
        return _DEVICE_NAMES[dev]
    if str(asic.get("target_graphics_version", "")) == "gfx950":
        return "AMD Instinct MI350-series (gfx950)"
    return name or "AMD Instinct GPU"


def _num(v: Any, default: float = 0.0) -> float:
    """amd-smi JSON values are numbers, {"value": x, "unit": u} dicts or "N/A" strings."""
    if isinstance(v, dict):
        v = v.get("value", default)
    if isinstance(v, bool):
        return float(v)
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):
        m = re.search(r"-?\d+(\.\d+)?", v)
        return float(m.group(0)) if m else default
    return default


def _opt(v: Any) -> Optional[float]:
    if v is None or (isinstance(v, str) and not re.search(r"\d", v)):
        return None
    if isinstance(v, dict) and ("value" not in v or isinstance(v.get("value"), str) and not re.search(r"\d", v["value"])):
        return None
    return _num(v)


_LINK_STATUS = {"U": "up", "D": "down", "X": "self", "SELF": "self", "ENABLED": "up", "DISABLED": "disabled"}


class GPUManager:
    """Monitors and manages the MI355X fleet (reference-compatible API)."""

    TEMP_WARNING = 80      # junction, Celsius (reference thresholds)
    TEMP_CRITICAL = 90
    MEM_WARNING = 85       # percent of HBM used
    MEM_CRITICAL = 95
    UTIL_WARNING = 95
    POWER_WARNING = 0.9    # fraction of the socket power limit
    HBM_TEMP_WARNING = 85  # MI355X additions
    HBM_TEMP_CRITICAL = 95

    def __init__(self, amd_smi_path: str = "amd-smi", backend: str = "auto", nvidia_smi_path: str = "nvidia-smi",
                 timeout_s: float = 30.0):
        self.amd_smi_path = amd_smi_path
        self.nvidia_smi_path = nvidia_smi_path
        self.backend = backend
        self.timeout_s = timeout_s
        self._lib = None
        self._lib_lock = threading.Lock()
        self._snapshot: Optional[GPUFleetStatus] = None
        self._poller: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # ------------------------------------------------------------------ amdsmi (in-process)
    def _amdsmi(self):
        if self._lib is None:
            import amdsmi  # raises ImportError without the ROCm python binding

            amdsmi.amdsmi_init()
            self._lib = amdsmi
        return self._lib

    def query_amdsmi(self) -> List[GPUDevice]:
        with self._lib_lock:
            lib = self._amdsmi()
            handles = lib.amdsmi_get_processor_handles()
            if not handles:
                raise RuntimeError("amdsmi: no GPUs")
            try:
                rocm = lib.amdsmi_get_rocm_version()
                rocm = rocm[1] if isinstance(rocm, tuple) else str(rocm)
            except Exception:
                rocm = ""
            T = lib.AmdSmiTemperatureType
            M = lib.AmdSmiTemperatureMetric
            devs = []
            for idx, h in enumerate(handles):
                def safe(fn, *a, default=None):
                    try:
                        return fn(h, *a)
                    except Exception:
                        return default
                asic = safe(lib.amdsmi_get_gpu_asic_info, default={}) or {}
                board = safe(lib.amdsmi_get_gpu_board_info, default={}) or {}
                enum = safe(lib.amdsmi_get_gpu_enumeration_info, default={}) or {}
                act = safe(lib.amdsmi_get_gpu_activity, default={}) or {}
                vram = safe(lib.amdsmi_get_gpu_vram_usage, default={}) or {}
                pw = safe(lib.amdsmi_get_power_info, default={}) or {}
                drv = safe(lib.amdsmi_get_gpu_driver_info, default={}) or {}
                ecc = safe(lib.amdsmi_get_gpu_total_ecc_count, default={}) or {}
                xs = safe(lib.amdsmi_get_gpu_xgmi_link_status, default={}) or {}
                lm = safe(lib.amdsmi_get_link_metrics, default={}) or {}
                hot = safe(lib.amdsmi_get_temp_metric, T.HOTSPOT, M.CURRENT)
                mem_t = safe(lib.amdsmi_get_temp_metric, T.VRAM, M.CURRENT)
                edge = safe(lib.amdsmi_get_temp_metric, T.EDGE, M.CURRENT)
                procs = []
                for pr in safe(lib.amdsmi_get_gpu_process_list, default=[]) or []:
                    mu = pr.get("memory_usage", {}) if isinstance(pr, dict) else {}
                    procs.append(GPUProcess(pid=int(pr.get("pid", 0)), name=str(pr.get("name", "")),
                                            used_memory_mib=int(_num(mu.get("vram_mem", 0)) // (1 << 20))))
                links = []
                stat = xs.get("status", []) if isinstance(xs, dict) else []
                for i, ln in enumerate(lm.get("links", []) if isinstance(lm, dict) else []):
                    st = _LINK_STATUS.get(str(stat[i + 1]) if i + 1 < len(stat) else "", "unknown")
                    links.append(XGMILink(peer_bdf=str(ln.get("bdf", "")), status=st,
                                          bit_rate_gbps=_num(ln.get("bit_rate")),
                                          max_bandwidth_gbps=_num(ln.get("max_bandwidth")),
                                          read_kb=int(_num(ln.get("read"))), write_kb=int(_num(ln.get("write")))))
                total = int(_num(vram.get("vram_total")))
                used = int(_num(vram.get("vram_used")))
                limit_uw = _num(pw.get("power_limit"))
                devs.append(self._make_device(
                    index=int(enum.get("hip_id", idx)) if isinstance(enum.get("hip_id", idx), int) else idx,
                    name=market_name(asic, board),
                    uuid=str(safe(lib.amdsmi_get_gpu_device_uuid, default="") or ""),
                    pci=str(safe(lib.amdsmi_get_gpu_device_bdf, default="") or ""),
                    util=_num(act.get("gfx_activity")), mem_act=_opt(act.get("umc_activity")),
                    total=total, used=used, power=_num(pw.get("socket_power", pw.get("current_socket_power"))),
                    limit=limit_uw / 1e6 if limit_uw > 1e5 else limit_uw,
                    hot=int(hot) if isinstance(hot, (int, float)) else None,
                    hbm=int(mem_t) if isinstance(mem_t, (int, float)) else None,
                    edge=int(edge) if isinstance(edge, (int, float)) else None,
                    driver=str(drv.get("driver_version", "")), rocm=rocm, procs=procs,
                    ecc_c=int(_num(ecc.get("correctable_count"))), ecc_u=int(_num(ecc.get("uncorrectable_count"))),
                    links=links, vendor=str(asic.get("vendor_name", "AMD")),
                    arch=str(asic.get("target_graphics_version", "")) or
                    ("gfx950" if "MI35" in market_name(asic, board) else "")))
            return devs

    # ------------------------------------------------------------------ amd-smi CLI JSON
    def _run(self, argv: List[str]) -> str:
        try:
            r = subprocess.run(argv, capture_output=True, text=True, timeout=self.timeout_s)
        except FileNotFoundError:
            raise RuntimeError(f"'{argv[0]}' not found. Ensure ROCm (amd-smi) is installed.")
        except subprocess.TimeoutExpired:
            raise RuntimeError(f"'{' '.join(argv)}' timed out")
        if r.returncode != 0:
            raise RuntimeError(f"{argv[0]} failed: {r.stderr.strip()[:500]}")
        return r.stdout

    def parse_amdsmi_json(self, static_json: Optional[str] = None, metric_json: Optional[str] = None,
                          process_json: Optional[str] = None, xgmi_json: Optional[str] = None) -> List[GPUDevice]:
        """Parse ``amd-smi static/metric/process/xgmi --json`` (live when the strings are None)."""
        if metric_json is None:
            metric_json = self._run([self.amd_smi_path, "metric", "--json"])
        if static_json is None:
            static_json = self._run([self.amd_smi_path, "static", "--json"])
        if process_json is None:
            try:
                process_json = self._run([self.amd_smi_path, "process", "--json"])
            except RuntimeError:
                process_json = "[]"
        if xgmi_json is None:
            try:
                xgmi_json = self._run([self.amd_smi_path, "xgmi", "--json"])
            except RuntimeError:
                xgmi_json = "{}"

        def gpu_list(doc: Any) -> List[Dict]:
            if isinstance(doc, dict):
                doc = doc.get("gpu_data", doc.get("gpus", []))
            return doc if isinstance(doc, list) else []

        metrics = {int(g.get("gpu", i)): g for i, g in enumerate(gpu_list(json.loads(metric_json)))}
        statics = {int(g.get("gpu", i)): g for i, g in enumerate(gpu_list(json.loads(static_json)))}
        procs_by: Dict[int, List[GPUProcess]] = {}
        for ent in gpu_list(json.loads(process_json or "[]")):
            plist = ent.get("process_list", [])
            out = []
            for p in plist if isinstance(plist, list) else []:
                info = p.get("process_info", p) if isinstance(p, dict) else {}
                if not isinstance(info, dict):
                    continue
                mu = info.get("memory_usage", {}) or {}
                vb = _num(mu.get("vram_mem"))
                unit = mu.get("vram_mem", {}).get("unit", "B") if isinstance(mu.get("vram_mem"), dict) else "B"
                mib = vb / (1 << 20) if unit == "B" else vb / 1024 if unit == "KB" else vb
                out.append(GPUProcess(pid=int(_num(info.get("pid"))), name=str(info.get("name", "")),
                                      used_memory_mib=int(mib)))
            procs_by[int(ent.get("gpu", 0))] = out
        links_by: Dict[int, List[XGMILink]] = {}
        xdoc = json.loads(xgmi_json or "{}")
        status_by = {}
        if isinstance(xdoc, dict):
            for ent in xdoc.get("link_port_status", []):
                status_by[int(ent.get("gpu", 0))] = ent.get("link_status", [])
            for grp in xdoc.get("xgmi_metric", []):
                for ent in grp if isinstance(grp, list) else [grp]:
                    g = int(ent.get("gpu", 0))
                    lm = ent.get("link_metrics", {})
                    st = status_by.get(g, [])
                    peers = [ln for ln in lm.get("links", []) if ln.get("gpu") != g]
                    links = []
                    for i, s in enumerate(st):
                        if str(s) in ("X", "SELF"):
                            continue
                        peer = peers[i - 1] if 0 <= i - 1 < len(peers) else {}
                        links.append(XGMILink(peer_bdf=str(peer.get("bdf", "")), status=_LINK_STATUS.get(str(s), "unknown"),
                                              bit_rate_gbps=_num(lm.get("bit_rate")),
                                              max_bandwidth_gbps=_num(lm.get("max_bandwidth")),
                                              read_kb=int(_num(peer.get("read"))), write_kb=int(_num(peer.get("write")))))
                    links_by[g] = links
        devs = []
        for g in sorted(metrics):
            m, s = metrics[g], statics.get(g, {})
            usage, temp, mem = m.get("usage", {}), m.get("temperature", {}), m.get("mem_usage", {})
            power, ecc = m.get("power", {}), m.get("ecc", {})
            lim = s.get("limit", {})
            ppt = lim.get("ppt0", lim) if isinstance(lim, dict) else {}
            limit = _num(ppt.get("socket_power_limit", ppt.get("max_power_limit")))
            asic, drv, bus = s.get("asic", {}), s.get("driver", {}), s.get("bus", {})
            total = int(_num(mem.get("total_vram")))
            used = int(_num(mem.get("used_vram")))
            numa = s.get("numa", {})
            devs.append(self._make_device(
                index=g, name=market_name(asic, s.get("board", {})), uuid=str(asic.get("asic_serial", "")),
                pci=str(bus.get("bdf", "")), util=_num(usage.get("gfx_activity")), mem_act=_opt(usage.get("umc_activity")),
                total=total, used=used, power=_num(power.get("socket_power")), limit=limit,
                hot=_int_or_none(temp.get("hotspot")), hbm=_int_or_none(temp.get("mem")), edge=_int_or_none(temp.get("edge")),
                driver=str(drv.get("version", "")), rocm="", procs=procs_by.get(g, []),
                ecc_c=int(_num(ecc.get("total_correctable_count"))), ecc_u=int(_num(ecc.get("total_uncorrectable_count"))),
                links=links_by.get(g, []), vendor=str(asic.get("vendor_name", "AMD")),
                arch=str(asic.get("target_graphics_version", "")) or
                ("gfx950" if "MI35" in market_name(asic, s.get("board", {})) else ""),
                numa=int(_num(numa.get("node"))) if isinstance(numa, dict) and "node" in numa else None))
        return devs

    # ------------------------------------------------------------------ common
    def _make_device(self, *, index, name, uuid, pci, util, mem_act, total, used, power, limit, hot, hbm, edge,
                     driver, rocm, procs, ecc_c, ecc_u, links, vendor, arch, numa=None) -> GPUDevice:
        junction = hot if hot is not None else (edge if edge is not None else 0)
        mem_pct = (used / total * 100) if total > 0 else 0.0
        health, alerts = self._assess_health(junction, util, mem_pct, power, limit)
        health, alerts = self._assess_mi355x(health, alerts, hbm, ecc_u, links)
        return GPUDevice(
            index=index, name=name, uuid=uuid, temperature_celsius=int(junction), gpu_utilization_pct=float(util),
            memory_used_mib=used, memory_total_mib=total, memory_free_mib=max(total - used, 0),
            memory_utilization_pct=round(mem_pct, 1), power_draw_watts=float(power), power_limit_watts=float(limit),
            fan_speed_pct=0, driver_version=driver, cuda_version=rocm, compute_mode="Default", pci_bus_id=pci,
            processes=procs, health=health, alerts=alerts, vendor=vendor, gfx_arch=arch,
            hotspot_temperature_celsius=hot, hbm_temperature_celsius=hbm, edge_temperature_celsius=edge,
            memory_activity_pct=mem_act, ecc_correctable=ecc_c, ecc_uncorrectable=ecc_u, xgmi_links=links,
            numa_node=numa)

    def _assess_health(self, temp: float, util: float, mem_pct: float, power: float,
                       power_limit: float) -> Tuple[GPUHealthStatus, List[str]]:
        """Reference classification: temp -> memory -> utilisation -> power; critical is sticky."""
        alerts: List[str] = []
        health = GPUHealthStatus.HEALTHY
        if temp >= self.TEMP_CRITICAL:
            alerts.append(f"CRITICAL: Temperature {temp}°C exceeds {self.TEMP_CRITICAL}°C")
            health = GPUHealthStatus.CRITICAL
        elif temp >= self.TEMP_WARNING:
            alerts.append(f"WARNING: Temperature {temp}°C exceeds {self.TEMP_WARNING}°C")
            health = GPUHealthStatus.WARNING
        if mem_pct >= self.MEM_CRITICAL:
            alerts.append(f"CRITICAL: Memory {mem_pct:.0f}% exceeds {self.MEM_CRITICAL}%")
            health = GPUHealthStatus.CRITICAL
        elif mem_pct >= self.MEM_WARNING:
            alerts.append(f"WARNING: Memory {mem_pct:.0f}% exceeds {self.MEM_WARNING}%")
            if health != GPUHealthStatus.CRITICAL:
                health = GPUHealthStatus.WARNING
        if util >= self.UTIL_WARNING:
            alerts.append(f"WARNING: Utilization {util:.0f}% at max capacity")
            if health == GPUHealthStatus.HEALTHY:
                health = GPUHealthStatus.WARNING
        if power_limit > 0 and power / power_limit >= self.POWER_WARNING:
            alerts.append(f"WARNING: Power {power:.0f}W near limit {power_limit:.0f}W")
            if health == GPUHealthStatus.HEALTHY:
                health = GPUHealthStatus.WARNING
        return health, alerts

    def _assess_mi355x(self, health: GPUHealthStatus, alerts: List[str], hbm: Optional[int], ecc_u: int,
                       links: List[XGMILink]) -> Tuple[GPUHealthStatus, List[str]]:
        if hbm is not None:
            if hbm >= self.HBM_TEMP_CRITICAL:
                alerts.append(f"CRITICAL: HBM temperature {hbm}°C exceeds {self.HBM_TEMP_CRITICAL}°C")
                health = GPUHealthStatus.CRITICAL
            elif hbm >= self.HBM_TEMP_WARNING:
                alerts.append(f"WARNING: HBM temperature {hbm}°C exceeds {self.HBM_TEMP_WARNING}°C")
                if health == GPUHealthStatus.HEALTHY:
                    health = GPUHealthStatus.WARNING
        if ecc_u > 0:
            alerts.append(f"CRITICAL: {ecc_u} uncorrectable ECC errors")
            health = GPUHealthStatus.CRITICAL
        down = [l for l in links if l.status == "down"]
        if down:
            alerts.append(f"WARNING: {len(down)} xGMI link(s) down")
            if health == GPUHealthStatus.HEALTHY:
                health = GPUHealthStatus.WARNING
        return health, alerts

    def query_devices(self) -> Tuple[List[GPUDevice], str]:
        errors = []
        if self.backend in ("auto", "amdsmi"):
            try:
                return self.query_amdsmi(), "amdsmi"
            except Exception as e:  # noqa: BLE001
                errors.append(f"amdsmi: {e}")
        if self.backend in ("auto", "cli"):
            try:
                return self.parse_amdsmi_json(), "amd-smi-cli"
            except Exception as e:  # noqa: BLE001
                errors.append(f"amd-smi: {e}")
        if self.backend in ("nvidia",):
            return self.parse_xml(), "nvidia-smi"
        raise RuntimeError("; ".join(errors) or "no telemetry backend")

    def aggregate(self, devices: List[GPUDevice], source: str) -> GPUFleetStatus:
        total = len(devices)
        fleet_alerts = [f"GPU {d.index} ({d.name}): {a}" for d in devices for a in d.alerts]
        available = sum(1 for d in devices if d.is_available)
        if available == 0 and total > 0:
            fleet_alerts.insert(0, "CRITICAL: No GPUs available for scheduling")
        return GPUFleetStatus(
            total_gpus=total, healthy_gpus=sum(1 for d in devices if d.health == GPUHealthStatus.HEALTHY),
            available_gpus=available, total_memory_mib=sum(d.memory_total_mib for d in devices),
            used_memory_mib=sum(d.memory_used_mib for d in devices),
            avg_utilization_pct=round(sum(d.gpu_utilization_pct for d in devices) / max(total, 1), 1),
            avg_temperature_celsius=round(sum(d.temperature_celsius for d in devices) / max(total, 1), 1),
            total_power_watts=round(sum(d.power_draw_watts for d in devices), 1), devices=devices,
            alerts=fleet_alerts, source=source)

    def get_fleet_status(self, static_json: Optional[str] = None, metric_json: Optional[str] = None,
                         use_cache: bool = True) -> GPUFleetStatus:
        """Never raises: no GPU / no driver -> empty fleet with an alert (reference semantics)."""
        if metric_json is not None:
            return self.aggregate(self.parse_amdsmi_json(static_json or "[]", metric_json, "[]", "{}"), "amd-smi-cli")
        if use_cache and self._snapshot is not None:
            return self._snapshot
        try:
            devs, src = self.query_devices()
        except Exception:  # noqa: BLE001
            return GPUFleetStatus(alerts=["Unable to query amd-smi. No GPUs detected."])
        return self.aggregate(devs, src)

    def select_best_gpu(self, required_memory_mib: int = 0,
                        fleet: Optional[GPUFleetStatus] = None) -> Optional[GPUDevice]:
        """Most free HBM among available devices meeting the requirement, then lowest utilisation."""
        devices = (fleet or self.get_fleet_status()).devices
        cands = [d for d in devices if d.is_available and d.memory_free_mib >= required_memory_mib]
        if not cands:
            return None
        cands.sort(key=lambda d: (-d.memory_free_mib, d.gpu_utilization_pct))
        return cands[0]

    def topology(self) -> Dict[str, Any]:
        """xGMI topology matrix (replaces the unmounted, hard-coded NVLink stub)."""
        nodes: Dict[str, Dict[str, str]] = {}
        bottlenecks = []
        try:
            with self._lib_lock:
                lib = self._amdsmi()
                hs = lib.amdsmi_get_processor_handles()
                for i, a in enumerate(hs):
                    row = {}
                    for j, b in enumerate(hs):
                        if i == j:
                            row[f"GPU_{j}"] = "X"
                            continue
                        try:
                            lt = lib.amdsmi_topo_get_link_type(a, b)
                            hops = lt.get("hops", 0) if isinstance(lt, dict) else 0
                            typ = lt.get("type", "") if isinstance(lt, dict) else lt
                            row[f"GPU_{j}"] = f"{getattr(typ, 'name', str(typ)).replace('AMDSMI_LINK_TYPE_', '')}{hops}"
                        except Exception:
                            row[f"GPU_{j}"] = "N/A"
                    nodes[f"GPU_{i}"] = row
            src = "amdsmi"
        except Exception:  # noqa: BLE001
            src = "none"
        fleet = self.get_fleet_status()
        for d in fleet.devices:
            for l in d.xgmi_links:
                if l.status == "down":
                    bottlenecks.append({"type": "xGMI", "location": f"GPU_{d.index} -> {l.peer_bdf}", "severity": "high"})
        return {"status": "success" if nodes else "unavailable", "node_type": "AMD Instinct MI355X",
                "interconnect": "xGMI (7 links/GPU, point-to-point)", "bottlenecks": bottlenecks,
                "topology_matrix": nodes, "source": src}

    # ------------------------------------------------------------------ background polling (A27)
    def start_polling(self, interval_s: float = 5.0) -> None:
        if self._poller is not None:
            return

        def loop():
            while not self._stop.is_set():
                try:
                    devs, src = self.query_devices()
                    self._snapshot = self.aggregate(devs, src)
                except Exception:  # noqa: BLE001
                    self._snapshot = GPUFleetStatus(alerts=["Unable to query amd-smi. No GPUs detected."])
                self._stop.wait(interval_s)

        self._poller = threading.Thread(target=loop, daemon=True, name="gpu-telemetry")
        self._poller.start()

    def stop_polling(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ mock fleet
    def get_mock_fleet(self) -> GPUFleetStatus:
        """Two mock MI355X devices (healthy + warning) for development without GPUs."""
        total = 294896
        d0 = GPUDevice(index=0, name="AMD Instinct MI355X", uuid="GPU-mock-0001", temperature_celsius=45,
                       gpu_utilization_pct=23.0, memory_used_mib=44600, memory_total_mib=total,
                       memory_free_mib=total - 44600, memory_utilization_pct=15.1, power_draw_watts=310.0,
                       power_limit_watts=1400.0, driver_version="6.18", cuda_version="7.2.0",
                       pci_bus_id="0000:05:00.0", processes=[GPUProcess(pid=12345, name="python", used_memory_mib=44600)],
                       vendor="AMD", gfx_arch="gfx950", hotspot_temperature_celsius=45, hbm_temperature_celsius=38,
                       memory_activity_pct=12.0,
                       xgmi_links=[XGMILink(peer_bdf=f"0000:{p:02x}:00.0", status="up", bit_rate_gbps=38,
                                            max_bandwidth_gbps=608) for p in range(7)])
        used1 = 255600
        d1 = GPUDevice(index=1, name="AMD Instinct MI355X", uuid="GPU-mock-0002", temperature_celsius=72,
                       gpu_utilization_pct=89.0, memory_used_mib=used1, memory_total_mib=total,
                       memory_free_mib=total - used1, memory_utilization_pct=86.7, power_draw_watts=1050.0,
                       power_limit_watts=1400.0, driver_version="6.18", cuda_version="7.2.0",
                       pci_bus_id="0000:15:00.0",
                       processes=[GPUProcess(pid=23456, name="python", used_memory_mib=127800),
                                  GPUProcess(pid=23457, name="python", used_memory_mib=127800)],
                       health=GPUHealthStatus.WARNING, alerts=["WARNING: Memory 86.7% exceeds 85%"], vendor="AMD",
                       gfx_arch="gfx950", hotspot_temperature_celsius=72, hbm_temperature_celsius=61,
                       memory_activity_pct=71.0,
                       xgmi_links=[XGMILink(peer_bdf=f"0000:{p:02x}:00.0", status="up", bit_rate_gbps=38,
                                            max_bandwidth_gbps=608) for p in range(7)])
        devs = [d0, d1]
        return GPUFleetStatus(total_gpus=2, healthy_gpus=1, available_gpus=1, total_memory_mib=2 * total,
                              used_memory_mib=44600 + used1, avg_utilization_pct=56.0, avg_temperature_celsius=58.5,
                              total_power_watts=1360.0, devices=devs, alerts=list(d1.alerts), source="mock")

    # ------------------------------------------------------------------ nvidia-smi (mixed fleets)
    def parse_xml(self, xml_str: Optional[str] = None) -> List[GPUDevice]:
        """nvidia-smi ``-q -x`` parser (same fields as the reference's)."""
        if xml_str is None:
            xml_str = self._run([self.nvidia_smi_path, "-q", "-x"])
        root = ET.fromstring(xml_str)
        drv, cuda = _xt(root, "driver_version"), _xt(root, "cuda_version")
        out = []
        for idx, g in enumerate(root.findall("gpu")):
            mem = g.find("fb_memory_usage")
            pw = g.find("gpu_power_readings")
            if pw is None:
                pw = g.find("power_readings")
            total, used = _xi(mem, "total"), _xi(mem, "used")
            procs = []
            pnode = g.find("processes")
            for p in (pnode.findall("process_info") if pnode is not None else []):
                procs.append(GPUProcess(pid=_xi(p, "pid"), name=_xt(p, "process_name"), used_memory_mib=_xi(p, "used_memory")))
            temp, util = _xi(g.find("temperature"), "gpu_temp"), _xf(g.find("utilization"), "gpu_util")
            power, limit = _xf(pw, "power_draw"), _xf(pw, "power_limit")
            mem_pct = used / total * 100 if total else 0.0
            health, alerts = self._assess_health(temp, util, mem_pct, power, limit)
            pci = g.find("pci")
            out.append(GPUDevice(index=idx, name=_xt(g, "product_name", f"GPU {idx}"), uuid=_xt(g, "uuid"),
                                 temperature_celsius=temp, gpu_utilization_pct=util, memory_used_mib=used,
                                 memory_total_mib=total, memory_free_mib=_xi(mem, "free"),
                                 memory_utilization_pct=round(mem_pct, 1), power_draw_watts=power,
                                 power_limit_watts=limit, fan_speed_pct=_xi(g, "fan_speed"), driver_version=drv,
                                 cuda_version=cuda, compute_mode=_xt(g, "compute_mode", "Default"),
                                 pci_bus_id=_xt(pci, "pci_bus_id") if pci is not None else "", processes=procs,
                                 health=health, alerts=alerts, vendor="NVIDIA"))
        return out

    def parse_csv(self, csv_str: Optional[str] = None) -> List[GPUDevice]:
        """nvidia-smi ``--query-gpu`` CSV parser; non-numeric cells ([N/A], [Not Supported]) read as 0."""
        if csv_str is None:
            csv_str = self._run([self.nvidia_smi_path,
                                 "--query-gpu=index,name,uuid,temperature.gpu,utilization.gpu,utilization.memory,"
                                 "memory.used,memory.total,memory.free,power.draw,power.limit,fan.speed",
                                 "--format=csv,noheader,nounits"])
        out = []
        for line in csv_str.strip().splitlines():
            cells = [c.strip() for c in line.split(",")]
            if len(cells) < 12:
                continue
            f = [_num(c) for c in cells]
            total, used = int(f[7]), int(f[6])
            mem_pct = used / total * 100 if total else 0.0
            health, alerts = self._assess_health(int(f[3]), f[4], mem_pct, f[9], f[10])
            out.append(GPUDevice(index=int(f[0]), name=cells[1], uuid=cells[2], temperature_celsius=int(f[3]),
                                 gpu_utilization_pct=f[4], memory_used_mib=used, memory_total_mib=total,
                                 memory_free_mib=int(f[8]), memory_utilization_pct=round(mem_pct, 1),
                                 power_draw_watts=f[9], power_limit_watts=f[10], fan_speed_pct=int(f[11]),
                                 health=health, alerts=alerts, vendor="NVIDIA"))
        return out


def _int_or_none(v: Any) -> Optional[int]:
    x = _opt(v)
    return int(x) if x is not None else None


def _xt(node, tag: str, default: str = "") -> str:
    if node is None:
        return default
    el = node.find(tag)
    return el.text.strip() if el is not None and el.text else default


def _xi(node, tag: str) -> int:
    return int(_num(_xt(node, tag, "0")))


def _xf(node, tag: str) -> float:
    return _num(_xt(node, tag, "0"))
