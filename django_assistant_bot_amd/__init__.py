"""django_assistant_bot_amd -- MI355X-native (gfx950) engine behind the assistant framework.

Subpackages
  ops/       hand-written HIP kernels (csrc/kernels) + plain-torch references
  models/    BERT/bge encoders and Llama-3 decoders (configs, weights, forward passes)
  engine/    tokenizer, continuous-batching LLM engine, embedding engine, vector index, RAG pipeline
  parallel/  torch.distributed (RCCL) process groups, tensor parallel, sharded index, DP ingest
  utils/     timing, profiling ranges, memory helpers
"""
__version__ = "0.1.0"
