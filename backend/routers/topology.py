"""xGMI topology (replaces the reference's unmounted, hard-coded NVLink stub ``backend/routers/nvlink.py``)."""
from typing import Any, Dict

from fastapi import APIRouter

from backend.routers.gpu import manager

router = APIRouter()


@router.get("/topology")
def get_topology() -> Dict[str, Any]:
    """GPU<->GPU link matrix from amdsmi (link type + hops) and down/degraded xGMI links as bottlenecks."""
    return manager.topology()
