"""REST control plane: ``uvicorn backend.main:app --host 0.0.0.0 --port 8000``.

Same app metadata, CORS policy, router prefixes and ``/`` + ``/health`` payloads as
the reference (``backend/main.py:1-39``). Fixes: absolute imports so the
documented start command works (A1), the topology router is mounted (A2, now
xGMI via amdsmi), responses are JSON-safe for NaN/Inf (A14), and the GPU
telemetry is served from a background-polled snapshot (A27).
"""
import os
from contextlib import asynccontextmanager

from fastapi import FastAPI
from fastapi.middleware.cors import CORSMiddleware

from backend.routers import gpu, monitoring, topology, training

@asynccontextmanager
async def _lifespan(_app):
    # amdsmi telemetry is polled on a background thread; handlers serve the latest snapshot
    interval = float(os.environ.get("DLGM_TELEMETRY_INTERVAL_S", "5"))
    if interval > 0:
        gpu.manager.start_polling(interval)
    yield


app = FastAPI(
    lifespan=_lifespan,
    title="MLOps Platform API",
    description="GPU fleet management, ZeRO distributed training on AMD Instinct MI355X, and training health monitoring",
    version="1.0.0",
)

app.add_middleware(
    CORSMiddleware,
    allow_origins=["*"],
    allow_credentials=True,
    allow_methods=["*"],
    allow_headers=["*"],
)

app.include_router(gpu.router, prefix="/api/v1/gpu", tags=["gpu-management"])
app.include_router(training.router, prefix="/api/v1/training", tags=["distributed-training"])
app.include_router(monitoring.router, prefix="/api/v1/monitoring", tags=["loss-monitoring"])
app.include_router(topology.router, prefix="/api/v1", tags=["topology"])
app.include_router(topology.router, tags=["topology"])  # reference path /topology


@app.get("/")
def root():
    return {
        "name": "MLOps Platform API",
        "version": "1.0.0",
        "features": [
            "GPU Fleet Management",
            "DeepSpeed ZeRO-3 Launcher",
            "Training Loss Monitor",
        ],
        "backend": "AMD Instinct MI355X (ROCm / RCCL / HIP)",
    }


@app.get("/health")
def health_check():
    return {"status": "healthy"}


@app.get("/metrics")
def prometheus_metrics():
    """Prometheus scrape endpoint: training gauges (fed by /api/v1/monitoring/ingest) + GPU fleet."""
    from fastapi import Response

    from distributed_llm_training_gpu_manager_amd.utils import metrics as prom

    prom.observe_fleet(gpu.manager._snapshot)
    return Response(prom.render(), media_type=prom.CONTENT_TYPE_LATEST)
