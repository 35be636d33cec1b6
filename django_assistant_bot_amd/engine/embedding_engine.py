"""Batched sentence-embedding engine (the GPU side of ``POST /embeddings/``).

The reference ``TransformersEmbedder.embeddings`` (ai/embedders/transformers.py:15-29) tokenises and
runs the encoder one text at a time, with no truncation (texts > 512 tokens fail on BERT).  Here texts
are tokenised natively in parallel, truncated to the model's max positions, sorted by length and
packed into variable-length batches of at most ``max_batch_tokens`` tokens (no padding), encoded on
the native kernels, mean-pooled exactly like the reference (all tokens incl. [CLS]/[SEP]) and
returned in the caller's order.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models import BertEncoder, EncoderConfig, encoder_config, random_encoder_weights
from .tokenizer import Tokenizer


class EmbeddingEngine:
    def __init__(self, model: str | EncoderConfig = "bge-base-en", device=None, weights: dict | None = None,
                 checkpoint: str | None = None, seed: int = 0, max_batch_tokens: int = 262144,
                 normalize: bool | None = None):
        self.cfg = encoder_config(model) if isinstance(model, str) else model
        if checkpoint is None and weights is None:
            from ..models.configs import checkpoint_dir

            checkpoint = checkpoint_dir(model)  # a local HF directory given as the model name
        self.device = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
        if weights is None:
            if checkpoint:
                from ..models import load_encoder_checkpoint

                weights = load_encoder_checkpoint(checkpoint, self.cfg)
            else:
                # bf16 on the GPU (MFMA); fp32 on the CPU, where bf16 GEMMs have no fast path
                dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
                weights = random_encoder_weights(self.cfg, self.device, seed=seed, dtype=dtype)
        self.model = BertEncoder(self.cfg, weights, self.device)
        self.tokenizer = Tokenizer.for_encoder(self.cfg, checkpoint)
        self.max_batch_tokens = max_batch_tokens
        self.normalize = self.cfg.normalize if normalize is None else normalize
        self.stats = {"texts": 0, "tokens": 0, "batches": 0}

    @property
    def dim(self) -> int:
        return self.cfg.hidden

    def tokenize(self, texts: list[str]):
        return self.tokenizer.encode_batch(texts, add_special=True, max_len=self.cfg.max_position)

    @torch.inference_mode()
    def embed_tokens(self, flat: np.ndarray, offsets: np.ndarray, normalize: bool | None = None,
                     out_dtype=torch.float32) -> torch.Tensor:
        """Pre-tokenised (flat ids, offsets) -> [n, H] on the engine device, caller order."""
        norm = self.normalize if normalize is None else normalize
        n = len(offsets) - 1
        lens = np.diff(offsets)
        order = np.argsort(-lens, kind="stable")
        out = torch.empty((n, self.cfg.hidden), dtype=out_dtype, device=self.device)
        pin = self.device.type == "cuda"

        def t(a):
            x = torch.from_numpy(np.ascontiguousarray(a))
            return (x.pin_memory() if pin else x).to(self.device, non_blocking=True)

        # batch boundaries over the length-sorted order: greedy token budget (vectorised)
        sorted_lens = lens[order]
        csum = np.concatenate([[0], np.cumsum(sorted_lens)])
        i = 0
        while i < n:
            # last j with csum[j] - csum[i] <= budget (at least one text per batch)
            j = int(np.searchsorted(csum, csum[i] + self.max_batch_tokens, side="right")) - 1
            j = max(j, i + 1)
            idx = order[i:j]
            seg_lens = sorted_lens[i:j]
            cu = np.zeros(len(idx) + 1, dtype=np.int32)
            np.cumsum(seg_lens, out=cu[1:])
            total = int(cu[-1])
            # gather index of every token of the batch and its position, without per-text slices
            seg_start = np.repeat(cu[:-1], seg_lens)
            pos = (np.arange(total, dtype=np.int64) - seg_start).astype(np.int32)
            ids = flat[np.repeat(offsets[idx], seg_lens) + pos].astype(np.int32, copy=False)
            emb = self.model.encode(t(ids), t(pos), t(cu), int(seg_lens.max()), normalize=norm)
            out[t(idx.astype(np.int64))] = emb.to(out_dtype)  # pinned + async: no stream sync per batch
            self.stats["batches"] += 1
            self.stats["tokens"] += total
            i = j
        self.stats["texts"] += n
        return out

    def embed(self, texts: list[str], normalize: bool | None = None, out_dtype=torch.float32) -> torch.Tensor:
        if not texts:
            return torch.empty((0, self.cfg.hidden), dtype=out_dtype, device=self.device)
        flat, offs = self.tokenize(list(texts))
        return self.embed_tokens(np.asarray(flat), np.asarray(offs), normalize, out_dtype)

    def embeddings(self, texts: list[str]) -> list[list[float]]:
        """JSON-ready float lists, the ``/embeddings/`` response body of the reference."""
        return self.embed(texts).float().cpu().tolist()
