"""In-job GPU telemetry: the amdsmi GPU manager polled from inside a training / bench process.

BASELINE config 2 runs "Llama-3 8B ZeRO-3 bf16 on 1xMI355X with amdsmi gpu_manager polling thermals/HBM";
the reference polls only from its API process (``ai_engine/gpu_manager.py:275-321`` behind
``GET /api/v1/gpu/fleet``). :class:`TelemetrySampler` runs :meth:`GPUManager.query_devices` (in-process
amdsmi, amd-smi CLI fallback) on a background thread every ``interval_s`` seconds for THIS rank's GPU
(matched by PCI bus id) and keeps running aggregates: junction (hotspot) and HBM temperature, HBM used,
socket power, GFX activity, xGMI link states, ECC counts and the health verdict with its alerts. amdsmi
is a ctypes binding, so the GIL is released during every query and the training thread is not slowed.
"""
from __future__ import annotations

import re
import threading
import time
from typing import Any, Dict, List, Optional

import torch


def _bdf(device: torch.device) -> Optional[str]:
    if device.type != "cuda":
        return None
    try:
        p = torch.cuda.get_device_properties(device)
        return f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}".lower()
    except Exception:  # noqa: BLE001
        return None


class _Agg:
    def __init__(self):
        self.n, self.sum, self.max = 0, 0.0, None

    def add(self, v) -> None:
        if v is None:
            return
        v = float(v)
        self.n += 1
        self.sum += v
        self.max = v if self.max is None else max(self.max, v)

    def summary(self) -> Optional[Dict[str, float]]:
        if not self.n:
            return None
        return {"mean": round(self.sum / self.n, 2), "max": round(self.max, 2)}


class TelemetrySampler:
    def __init__(self, device: torch.device, interval_s: float = 2.0, manager=None):
        from .gpu_manager import GPUManager

        self.device = device
        self.interval_s = interval_s
        self.mgr = manager or GPUManager()
        self.bdf = _bdf(device)
        self.aggs = {k: _Agg() for k in ("junction_temp_c", "hbm_temp_c", "edge_temp_c", "hbm_used_gib",
                                         "power_w", "gfx_util_pct", "hbm_activity_pct")}
        self.samples = 0
        self.source = "none"
        self.errors: List[str] = []
        self.links: Dict[str, int] = {}
        self.ecc_uncorrectable = 0
        self.worst = "healthy"
        # one entry per distinct alert (numbers masked: "Power 1359W near limit" and "Power 1379W ..." are one
        # alert), {message (latest wording), count, first_s, last_s} -- the reference's message formats are
        # kept (gpu_manager.py:93-98, 301-305), repeated samples are counted instead of listed
        self.alerts: Dict[str, Dict[str, Any]] = {}
        self.name = ""
        self._t0 = time.time()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def _mine(self, devs):
        if self.bdf:
            for d in devs:
                if d.pci_bus_id and d.pci_bus_id.lower().startswith(self.bdf):
                    return d
        idx = self.device.index if self.device.type == "cuda" and self.device.index is not None else 0
        return devs[idx] if idx < len(devs) else (devs[0] if devs else None)

    def sample(self) -> None:
        try:
            devs, self.source = self.mgr.query_devices()
        except Exception as e:  # noqa: BLE001
            if len(self.errors) < 5:
                self.errors.append(str(e)[:200])
            return
        d = self._mine(devs)
        if d is None:
            return
        self.samples += 1
        self.name = d.name
        self.aggs["junction_temp_c"].add(d.hotspot_temperature_celsius)
        self.aggs["hbm_temp_c"].add(d.hbm_temperature_celsius)
        self.aggs["edge_temp_c"].add(d.edge_temperature_celsius)
        self.aggs["hbm_used_gib"].add(d.memory_used_mib / 1024.0)
        self.aggs["power_w"].add(d.power_draw_watts)
        self.aggs["gfx_util_pct"].add(d.gpu_utilization_pct)
        self.aggs["hbm_activity_pct"].add(d.memory_activity_pct)
        self.links = {}
        for ln in d.xgmi_links:
            self.links[ln.status] = self.links.get(ln.status, 0) + 1
        self.ecc_uncorrectable = max(self.ecc_uncorrectable, d.ecc_uncorrectable)
        rank = {"healthy": 0, "warning": 1, "critical": 2, "unreachable": 3}
        h = getattr(d.health, "value", str(d.health))
        if rank.get(h, 0) > rank.get(self.worst, 0):
            self.worst = h
        now = round(time.time() - self._t0, 1)
        for a in d.alerts:
            key = re.sub(r"\d+(\.\d+)?", "#", a)
            e = self.alerts.get(key)
            if e is None:
                if len(self.alerts) < 20:
                    self.alerts[key] = {"message": a, "count": 1, "first_s": now, "last_s": now}
            else:
                e.update(message=a, count=e["count"] + 1, last_s=now)

    def _loop(self) -> None:
        while not self._stop.is_set():
            t0 = time.time()
            self.sample()
            self._stop.wait(max(0.0, self.interval_s - (time.time() - t0)))

    def start(self) -> "TelemetrySampler":
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="gpu-telemetry")
            self._thread.start()
        return self

    def stop(self) -> Dict[str, Any]:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        return self.summary()

    def summary(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"source": self.source, "samples": self.samples, "interval_s": self.interval_s,
                               "device": self.name, "pci_bus_id": self.bdf, "health": self.worst,
                               "xgmi_links": self.links, "ecc_uncorrectable": self.ecc_uncorrectable}
        for k, a in self.aggs.items():
            s = a.summary()
            if s is not None:
                out[k] = s
        if self.alerts:
            out["alerts"] = list(self.alerts.values())
        if self.errors and not self.samples:
            out["errors"] = self.errors
        return out
