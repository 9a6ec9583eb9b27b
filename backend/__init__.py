"""FastAPI control plane (reference-compatible REST API) for the MI355X training framework."""
