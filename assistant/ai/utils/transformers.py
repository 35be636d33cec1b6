"""Device selection (reference ai/utils/transformers.py:9-23): the MI355X (ROCm HIP device, exposed by
PyTorch as 'cuda') when present, else CPU."""
import logging

logger = logging.getLogger(__name__)


def get_torch_device() -> str:
    import torch

    if torch.cuda.is_available():
        logger.info("ROCm GPU available: %s", torch.cuda.get_device_name(0))
        return "cuda"
    logger.warning("no GPU: using the CPU")
    return "cpu"
