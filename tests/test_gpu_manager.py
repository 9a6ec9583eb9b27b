"""amdsmi GPU manager: parsing of real MI355X amd-smi output (recorded fixtures), reference health rules."""
import json
import os

import pytest

from distributed_llm_training_gpu_manager_amd.health.gpu_manager import GPUHealthStatus, GPUManager

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
AMD = os.path.join(FIX, "amdsmi")


def _read(name):
    return open(os.path.join(AMD, name)).read()


def test_parse_recorded_mi355x_amdsmi_json():
    m = GPUManager()
    devs = m.parse_amdsmi_json(_read("amd-smi_static.json"), _read("amd-smi_metric.json"),
                               _read("amd-smi_process.json"), _read("amd-smi_xgmi.json"))
    assert len(devs) == 1
    d = devs[0]
    assert d.name == "AMD Instinct MI355 OAM" and d.gfx_arch == "gfx950" and d.pci_bus_id == "0000:f1:00.0"
    assert d.memory_total_mib == 294896 and d.memory_used_mib == 283
    assert d.hotspot_temperature_celsius == 45 and d.hbm_temperature_celsius == 33
    assert d.temperature_celsius == 45 and d.edge_temperature_celsius is None  # no edge sensor on MI355X
    assert d.power_draw_watts == 242 and d.power_limit_watts == 1400
    assert d.health == GPUHealthStatus.HEALTHY and d.is_available
    assert d.processes and d.processes[0].pid == 1263896
    assert len(d.xgmi_links) == 7 and all(l.status == "up" for l in d.xgmi_links)
    assert d.ecc_uncorrectable == 0


def test_fleet_from_injected_json_and_selection():
    m = GPUManager()
    fleet = m.get_fleet_status(static_json=_read("amd-smi_static.json"), metric_json=_read("amd-smi_metric.json"))
    assert fleet.total_gpus == 1 and fleet.available_gpus == 1 and fleet.source == "amd-smi-cli"
    assert m.select_best_gpu(1000, fleet=fleet).index == 0
    assert m.select_best_gpu(10 ** 7, fleet=fleet) is None


GOLD = json.load(open(os.path.join(FIX, "reference_golden", "assess_health.json")))


@pytest.mark.parametrize("i", range(len(GOLD)))
def test_assess_health_matches_reference(i):
    c = GOLD[i]
    h, alerts = GPUManager()._assess_health(c["temp"], c["util"], c["mem"], c["power"], c["limit"])
    assert h.value == c["health"] and alerts == c["alerts"]


def test_mi355x_specific_health():
    m = GPUManager()
    from distributed_llm_training_gpu_manager_amd.health.gpu_manager import XGMILink
    h, a = m._assess_mi355x(GPUHealthStatus.HEALTHY, [], 97, 0, [])
    assert h == GPUHealthStatus.CRITICAL and "HBM temperature" in a[0]
    h, a = m._assess_mi355x(GPUHealthStatus.HEALTHY, [], 40, 2, [])
    assert h == GPUHealthStatus.CRITICAL and "uncorrectable ECC" in a[0]
    h, a = m._assess_mi355x(GPUHealthStatus.HEALTHY, [], 40, 0, [XGMILink(status="down")])
    assert h == GPUHealthStatus.WARNING and "xGMI" in a[0]


def test_no_gpu_gives_empty_fleet_not_exception():
    m = GPUManager(amd_smi_path="/nonexistent/amd-smi", backend="cli")
    fleet = m.get_fleet_status()
    assert fleet.total_gpus == 0 and fleet.alerts == ["Unable to query amd-smi. No GPUs detected."]


def test_mock_fleet_is_mi355x():
    f = GPUManager().get_mock_fleet()
    assert f.total_gpus == 2 and f.available_gpus == 1 and f.devices[0].memory_total_mib == 294896
    assert f.devices[1].health == GPUHealthStatus.WARNING


NV_XML = """<?xml version="1.0"?><nvidia_smi_log><driver_version>535.1</driver_version><cuda_version>12.2</cuda_version>
<gpu><product_name>NVIDIA H100</product_name><uuid>GPU-1</uuid><pci><pci_bus_id>0000:01:00.0</pci_bus_id></pci>
<fan_speed>N/A</fan_speed><fb_memory_usage><total>81559 MiB</total><used>78000 MiB</used><free>3559 MiB</free></fb_memory_usage>
<utilization><gpu_util>97 %</gpu_util></utilization><temperature><gpu_temp>91 C</gpu_temp></temperature>
<gpu_power_readings><power_draw>690 W</power_draw><power_limit>700 W</power_limit></gpu_power_readings>
<processes><process_info><pid>42</pid><process_name>python</process_name><used_memory>78000 MiB</used_memory></process_info></processes>
</gpu></nvidia_smi_log>"""


def test_nvidia_parsers_for_mixed_fleets():
    m = GPUManager()
    d = m.parse_xml(NV_XML)[0]
    assert d.health == GPUHealthStatus.CRITICAL and d.processes[0].pid == 42 and d.cuda_version == "12.2"
    csv = "0, NVIDIA H100, GPU-1, 45, 10, 5, 1000, 81559, 80559, [Not Supported], [N/A], [Not Supported]\n"
    d = m.parse_csv(csv)[0]  # A6: no crash on [Not Supported]
    assert d.temperature_celsius == 45 and d.power_draw_watts == 0.0


def test_market_name_falls_back_when_libdrm_name_is_generic():
    """On the MI355X boxes libdrm's amdgpu.ids is missing and asic.market_name reads "AMD Radeon Graphics":
    the device is named from the board FRU product name, then the PCI device id, then the gfx target."""
    from distributed_llm_training_gpu_manager_amd.health.gpu_manager import market_name
    asic = {"market_name": "AMD Radeon Graphics", "device_id": "0x75a3", "target_graphics_version": "gfx950"}
    assert market_name(asic, {"product_name": "AMD Instinct MI355 OAM"}) == "AMD Instinct MI355 OAM"
    assert market_name(asic, {}) == "AMD Instinct MI355X"
    assert market_name({"market_name": "", "target_graphics_version": "gfx950"}) == "AMD Instinct MI350-series (gfx950)"
    assert market_name({"market_name": "AMD Instinct MI355 OAM"}, {"product_name": "x"}) == "AMD Instinct MI355 OAM"


def test_telemetry_alerts_are_deduplicated():
    """Repeated samples of one alert (numbers differ: "Power 1359W ...", "Power 1379W ...") collapse into one
    {message, count, first_s, last_s} entry; distinct alerts stay separate (reference formats kept)."""
    import torch
    from distributed_llm_training_gpu_manager_amd.health.gpu_manager import GPUDevice
    from distributed_llm_training_gpu_manager_amd.health.telemetry import TelemetrySampler

    class FakeMgr:
        def __init__(self):
            self.i = 0

        def query_devices(self):
            self.i += 1
            d = GPUDevice(index=0, name="AMD Instinct MI355X", memory_total_mib=294912,
                          alerts=[f"WARNING: Power {1350 + self.i}W near limit 1400W",
                                  "WARNING: Utilization 100% at max capacity"])
            return [d], "amdsmi"

    s = TelemetrySampler(torch.device("cpu"), interval_s=0.0, manager=FakeMgr())
    for _ in range(25):
        s.sample()
    out = s.summary()
    assert out["device"] == "AMD Instinct MI355X"
    alerts = out["alerts"]
    assert len(alerts) == 2, alerts
    power = next(a for a in alerts if "Power" in a["message"])
    assert power["count"] == 25 and power["message"] == "WARNING: Power 1375W near limit 1400W"
    assert power["first_s"] <= power["last_s"]
