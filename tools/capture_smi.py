#!/usr/bin/env python3
"""Record amdsmi / amd-smi outputs on a real MI355X box as test fixtures (tests/fixtures/amdsmi/).

The fixtures let the GPU-manager parsers be tested on CPU (no hardware in CI),
mirroring how the reference's nvidia-smi parsers take injected XML/CSV strings.
"""
import json
import os
import subprocess
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fixtures"
os.makedirs(OUT, exist_ok=True)


def jsonable(x):
    if isinstance(x, dict):
        return {str(k): jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v) for v in x]
    if isinstance(x, (int, float, str, bool)) or x is None:
        return x
    if hasattr(x, "name"):
        return str(x.name)
    return str(x)


for sub in ("static", "metric", "topology", "process", "xgmi", "list", "version"):
    try:
        r = subprocess.run(["amd-smi", sub, "--json"], capture_output=True, text=True, timeout=60)
        with open(os.path.join(OUT, f"amd-smi_{sub}.json"), "w") as f:
            f.write(r.stdout if r.returncode == 0 else json.dumps({"rc": r.returncode, "stderr": r.stderr[-2000:]}))
    except Exception as e:  # noqa: BLE001
        print(sub, e)

import amdsmi  # noqa: E402

amdsmi.amdsmi_init()
dump = {"lib_version": jsonable(amdsmi.amdsmi_get_lib_version())}
handles = amdsmi.amdsmi_get_processor_handles()
dump["n"] = len(handles)
devs = []
T = amdsmi.AmdSmiTemperatureType
M = amdsmi.AmdSmiTemperatureMetric
for h in handles[:1]:
    d = {}
    calls = {
        "asic": lambda: amdsmi.amdsmi_get_gpu_asic_info(h),
        "board": lambda: amdsmi.amdsmi_get_gpu_board_info(h),
        "bdf": lambda: amdsmi.amdsmi_get_gpu_device_bdf(h),
        "uuid": lambda: amdsmi.amdsmi_get_gpu_device_uuid(h),
        "driver": lambda: amdsmi.amdsmi_get_gpu_driver_info(h),
        "activity": lambda: amdsmi.amdsmi_get_gpu_activity(h),
        "vram": lambda: amdsmi.amdsmi_get_gpu_vram_usage(h),
        "power": lambda: amdsmi.amdsmi_get_power_info(h),
        "power_cap": lambda: amdsmi.amdsmi_get_power_cap_info(h),
        "procs": lambda: amdsmi.amdsmi_get_gpu_process_list(h),
        "ecc_total": lambda: amdsmi.amdsmi_get_gpu_total_ecc_count(h),
        "xgmi_link_status": lambda: amdsmi.amdsmi_get_gpu_xgmi_link_status(h),
        "link_metrics": lambda: amdsmi.amdsmi_get_link_metrics(h),
        "metrics": lambda: amdsmi.amdsmi_get_gpu_metrics_info(h),
        "kfd": lambda: amdsmi.amdsmi_get_gpu_kfd_info(h),
        "enum": lambda: amdsmi.amdsmi_get_gpu_enumeration_info(h),
    }
    for name in ("EDGE", "HOTSPOT", "VRAM", "HBM_0", "HBM_1", "HBM_2", "HBM_3"):
        calls[f"temp_{name}"] = (lambda n=name: amdsmi.amdsmi_get_temp_metric(h, getattr(T, n), M.CURRENT))
    for k, fn in calls.items():
        try:
            d[k] = jsonable(fn())
        except Exception as e:  # noqa: BLE001
            d[k] = {"error": str(e)}
    devs.append(d)
dump["devices"] = devs
with open(os.path.join(OUT, "amdsmi_py_dump.json"), "w") as f:
    json.dump(dump, f, indent=1)
amdsmi.amdsmi_shut_down()
print("captured to", OUT)
