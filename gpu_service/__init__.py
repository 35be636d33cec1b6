"""Model-serving service (FastAPI) on the MI355X engine (reference gpu_service/)."""
