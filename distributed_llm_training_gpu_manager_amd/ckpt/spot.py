"""Spot / preemptible-instance resiliency (reference ``ai_engine/spot_resiliency.py:5-49``).

The reference class polls nothing (the AWS/GCP URLs are comments), its fault hook
``_simulate_interruption`` always returns False and the "emergency checkpoint" only
prints. Same class name and async API here, but real:

* polls the cloud metadata services with short timeouts (stdlib ``urllib``, no
  ``requests`` dependency): AWS IMDSv2 ``spot/instance-action`` (with a session
  token), GCP ``instance/preempted`` (``Metadata-Flavor: Google``), Azure
  ``scheduledevents`` (Preempt events); every URL is injectable so tests drive it
  with a local fake HTTP server;
* ``_simulate_interruption`` stays as the fault-injection hook (settable, or
  ``DLGM_SIMULATE_PREEMPTION=1``);
* on a notice the manager calls ``on_preemption`` -- by default it signals the
  supervised job's process group with SIGUSR1; the training ranks then take an
  emergency checkpoint through the async checkpointer at the next step boundary and
  exit with ``EXIT_PREEMPTED`` well inside the ~2-minute notice window, and the
  replacement instance restores with ``--resume=auto``.
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import threading
import time
import urllib.request
from typing import Any, Callable, Dict, List, Optional

AWS_TOKEN_URL = "http://169.254.169.254/latest/api/token"
AWS_ACTION_URL = "http://169.254.169.254/latest/meta-data/spot/instance-action"
GCP_PREEMPTED_URL = "http://metadata.google.internal/computeMetadata/v1/instance/preempted"
AZURE_EVENTS_URL = "http://169.254.169.254/metadata/scheduledevents?api-version=2020-07-01"


def _http(url: str, headers: Dict[str, str], timeout: float, method: str = "GET") -> Optional[str]:
    req = urllib.request.Request(url, headers=headers, method=method)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            if r.status != 200:
                return None
            return r.read().decode()
    except Exception:  # noqa: BLE001 - 404 / no route / timeout all mean "no notice"
        return None


class SpotInstanceResiliencyManager:
    def __init__(self, check_interval_sec: float = 5, provider: str = "auto", urls: Optional[Dict[str, str]] = None,
                 on_preemption: Optional[Callable[[Dict[str, Any]], None]] = None, timeout_s: float = 0.5,
                 target_pgid: Optional[int] = None):
        self.check_interval_sec = check_interval_sec
        self.provider = provider
        self.urls = {"aws_token": AWS_TOKEN_URL, "aws_action": AWS_ACTION_URL, "gcp": GCP_PREEMPTED_URL,
                     "azure": AZURE_EVENTS_URL, **(urls or {})}
        self.on_preemption = on_preemption
        self.timeout_s = timeout_s
        self.target_pgid = target_pgid
        self.is_running = False
        self.simulate = False
        self.notices: List[Dict[str, Any]] = []
        self._thread: Optional[threading.Thread] = None

    # ---- providers
    def _check_aws(self) -> Optional[Dict[str, Any]]:
        token = _http(self.urls["aws_token"], {"X-aws-ec2-metadata-token-ttl-seconds": "60"}, self.timeout_s, "PUT")
        hdr = {"X-aws-ec2-metadata-token": token} if token else {}
        body = _http(self.urls["aws_action"], hdr, self.timeout_s)
        if body:
            try:
                d = json.loads(body)
            except ValueError:
                d = {"raw": body}
            return {"provider": "aws", **d}
        return None

    def _check_gcp(self) -> Optional[Dict[str, Any]]:
        body = _http(self.urls["gcp"], {"Metadata-Flavor": "Google"}, self.timeout_s)
        if body and body.strip().upper() == "TRUE":
            return {"provider": "gcp", "action": "terminate"}
        return None

    def _check_azure(self) -> Optional[Dict[str, Any]]:
        body = _http(self.urls["azure"], {"Metadata": "true"}, self.timeout_s)
        if body:
            try:
                evs = json.loads(body).get("Events", [])
            except ValueError:
                return None
            pre = [e for e in evs if e.get("EventType") == "Preempt"]
            if pre:
                return {"provider": "azure", "action": "terminate", "events": pre}
        return None

    def _simulate_interruption(self) -> bool:
        """Fault-injection hook (the reference's, now settable)."""
        return self.simulate or os.environ.get("DLGM_SIMULATE_PREEMPTION", "0") == "1"

    def check_once(self) -> Optional[Dict[str, Any]]:
        if self._simulate_interruption():
            return {"provider": "simulated", "action": "terminate"}
        checks = {"aws": self._check_aws, "gcp": self._check_gcp, "azure": self._check_azure}
        order = list(checks) if self.provider == "auto" else [self.provider]
        for p in order:
            n = checks[p]()
            if n:
                return n
        return None

    # ---- reference async API
    async def monitor_preemption_notices(self, deepspeed_launcher_ref=None) -> Optional[Dict[str, Any]]:
        self.is_running = True
        while self.is_running:
            await asyncio.sleep(self.check_interval_sec)
            notice = await asyncio.get_running_loop().run_in_executor(None, self.check_once)
            if notice:
                await self._execute_emergency_checkpoint(deepspeed_launcher_ref, notice)
                return notice
        return None

    async def _execute_emergency_checkpoint(self, launcher, notice: Optional[Dict[str, Any]] = None) -> None:
        self._handle(notice or {"provider": "unknown"}, launcher)

    def _handle(self, notice: Dict[str, Any], launcher=None) -> None:
        notice = {**notice, "detected_at": time.time()}
        self.notices.append(notice)
        if self.on_preemption is not None:
            self.on_preemption(notice)
        elif self.target_pgid is not None:
            try:
                os.killpg(self.target_pgid, signal.SIGUSR1)
            except ProcessLookupError:
                pass
        elif launcher is not None and hasattr(launcher, "registry"):
            for job in launcher.registry.list():
                if job.status == "running":
                    launcher.registry.signal(job.spec.job_id, signal.SIGUSR1)

    # ---- thread API for non-async callers
    def start(self) -> None:
        if self._thread is not None:
            return
        self.is_running = True

        def loop():
            while self.is_running:
                notice = self.check_once()
                if notice:
                    self._handle(notice)
                    self.is_running = False
                    return
                time.sleep(self.check_interval_sec)

        self._thread = threading.Thread(target=loop, daemon=True, name="spot-monitor")
        self._thread.start()

    def stop(self) -> None:
        self.is_running = False
