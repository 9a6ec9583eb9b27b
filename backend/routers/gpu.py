"""GPU fleet endpoints (reference ``backend/routers/gpu.py``), served by the amdsmi GPU manager."""
from fastapi import APIRouter, HTTPException

from distributed_llm_training_gpu_manager_amd.health.gpu_manager import GPUFleetStatus, GPUManager

router = APIRouter()
manager = GPUManager()


def _fleet() -> GPUFleetStatus:
    return manager.get_fleet_status()


@router.get("/fleet", response_model=GPUFleetStatus)
def get_fleet_status():
    """Real-time status of all GPUs (empty fleet + alert when no GPU is visible, like the reference)."""
    return _fleet()


@router.get("/fleet/mock", response_model=GPUFleetStatus)
def get_mock_fleet():
    """Mock MI355X fleet for testing and development."""
    return manager.get_mock_fleet()


@router.get("/select")
def select_best_gpu(required_memory_mib: int = 0):
    """Best available GPU (most free HBM); falls back to the mock fleet when no GPU is visible.

    One selection path for both cases (fix A4: the reference's mock fallback did not sort).
    """
    fleet = _fleet()
    if fleet.total_gpus == 0:
        fleet = manager.get_mock_fleet()
    gpu = manager.select_best_gpu(required_memory_mib, fleet=fleet)
    if gpu is None:
        raise HTTPException(status_code=503, detail=f"No GPU available with {required_memory_mib} MiB free memory")
    return {
        "selected_gpu": gpu.model_dump(),
        "recommendation": f"Use GPU {gpu.index} ({gpu.name}) with {gpu.memory_free_mib} MiB free",
    }


@router.get("/devices/{index}")
def get_device(index: int):
    for device in _fleet().devices:
        if device.index == index:
            return device.model_dump()
    raise HTTPException(status_code=404, detail=f"GPU {index} not found")


@router.get("/alerts")
def get_gpu_alerts():
    fleet = _fleet()
    return {
        "total_alerts": len(fleet.alerts),
        "alerts": fleet.alerts,
        "devices_with_alerts": [
            {"gpu_index": d.index, "gpu_name": d.name, "health": d.health, "alerts": d.alerts}
            for d in fleet.devices if d.alerts
        ],
    }
