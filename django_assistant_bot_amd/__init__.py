"""django_assistant_bot_amd -- MI355X-native (gfx950) engine behind the assistant framework.

Subpackages
  ops/       hand-written HIP kernels (csrc/kernels) + plain-torch references
  models/    BERT/bge encoders and Llama-3 decoders (configs, weights, forward passes)
  engine/    tokenizer, continuous-batching LLM engine, embedding engine, vector index, RAG pipeline
  parallel/  torch.distributed (RCCL) process groups, tensor parallel, sharded index, DP ingest
  utils/     timing, profiling ranges, memory helpers
"""
__version__ = "0.1.0"

# The HIP runtime must be the one PyTorch ships (libamdhip64.so.7 from torch/lib): importing torch
# before the native extension makes the extension bind to that already-loaded runtime instead of
# pulling /opt/rocm's copy into the process first (two HIP runtime versions in one process fail).
import torch as _torch  # noqa: E402,F401
