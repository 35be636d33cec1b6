"""Models served by gpu_service (reference gpu_service/models.py).

Comma-separated env lists; names are engine presets (``bge-base-en``, ``llama-3-8b`` ...) or local HF
checkpoint directories.  As in the reference, no dialog model is served unless configured."""
import os


def _list(name: str, default: str):
    return [m.strip() for m in os.environ.get(name, default).split(",") if m.strip()]


embedder_models = _list("GPU_SERVICE_EMBEDDERS", "bge-base-en")
provider_models = _list("GPU_SERVICE_PROVIDERS", "")
