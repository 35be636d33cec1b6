"""Config 2 of BASELINE.json: bge-base-en encoder (bf16) batch-embedding of synthetic chunks, one
process per GPU (data parallel, ``torch.distributed.run --nproc-per-node N``), vectors inserted into the
rank's shard of the HBM index as they are produced (parallel.dp_embed).

    python benchmarks/embed_bench.py --chunks 1000000 [--words 48]
    python benchmarks/embed_bench.py --gpus 8 ...     (starts its 8 ranks itself; or one rank under torchrun)

Prints one JSON line (rank 0): chunks/s and tokens/s for the whole job, time measured between barriers.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1_000_000)
    ap.add_argument("--words", type=int, default=48, help="mean words per chunk (+-50 %)")
    ap.add_argument("--model", default="bge-base-en")
    ap.add_argument("--max-batch-tokens", type=int, default=262144,
                    help="tokens per packed encoder batch (64k / 128k / 256k: 100.7k / 102.4k / 103.9k chunks/s, round 4)")
    ap.add_argument("--warmup-chunks", type=int, default=20000)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", 1)),
                    help="ranks; from a plain process the script starts them itself (parallel/launch.py)")
    args = ap.parse_args()

    from django_assistant_bot_amd.parallel.launch import check_world, maybe_spawn

    maybe_spawn(args.gpus, __file__)

    from bench import _WORDS
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.dp_embed import embed_corpus
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    info = pdist.init()
    check_world(args.gpus, info.world_size)
    eng = EmbeddingEngine(args.model, info.device, seed=0, max_batch_tokens=args.max_batch_tokens)
    words = np.array(_WORDS)

    def text_of(i: int) -> str:
        rng = np.random.default_rng(i)
        n = int(rng.integers(args.words // 2, args.words * 3 // 2 + 1))
        return " ".join(words[rng.integers(0, len(words), n)])

    # warm-up (kernels, allocator) on a disjoint id range
    embed_corpus(eng, text_of, args.warmup_chunks, info.rank, info.world_size, first_id=10**9)
    # synthetic corpus materialised before timing (generating random text is not ingest work;
    # tokenisation is, and stays inside the timed region)
    from django_assistant_bot_amd.parallel.dp_embed import owned_ids
    corpus = {int(i): text_of(int(i)) for i in owned_ids(args.chunks, info.rank, info.world_size)}
    index = ShardedIndex(eng.dim, info.device, capacity=args.chunks // max(1, info.world_size) + 1024)
    pdist.barrier(info)
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    tok0 = eng.stats["tokens"]
    t0 = time.perf_counter()
    _, _, total = embed_corpus(eng, corpus.__getitem__, args.chunks, info.rank, info.world_size, index=index,
                               doc_of=lambda ids: ids // 10)
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier(info)
    el = pdist.max_over_ranks(time.perf_counter() - t0, info.device)
    toks = torch.tensor([eng.stats["tokens"] - tok0], dtype=torch.float64,
                        device=info.device if info.backend == "nccl" else "cpu")
    if info.world_size > 1:
        torch.distributed.all_reduce(toks)
    if info.rank == 0:
        print(json.dumps({"metric": "bge-base batch-embed chunks/s (DP, into the sharded HBM index)",
                          "value": round(total / el, 1), "unit": "chunks/s", "n_gpus": info.world_size,
                          "chunks": total, "seconds": round(el, 2), "tokens_per_s": round(float(toks.item()) / el),
                          "mean_tokens_per_chunk": round(float(toks.item()) / max(total, 1), 1),
                          "dtype": "bf16", "data": "synthetic", "scaling": "strong",
                          "config": {"model": args.model, "parallelism": f"dp{info.world_size}",
                                     "max_batch_tokens": args.max_batch_tokens}}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
