"""Entry point run by the launcher on every rank: ``python -m distributed_llm_training_gpu_manager_amd.train``."""
import os
import sys

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_training_gpu_manager_amd.engine.trainer import main
else:
    from .engine.trainer import main

if __name__ == "__main__":
    sys.exit(main())
