"""Cross-cutting utilities: HIP-event phase timers, rank-aware logging, Prometheus metrics, GEMM tuning."""
from .logging import get_logger
from .timers import PhaseTimers

__all__ = ["PhaseTimers", "get_logger"]
