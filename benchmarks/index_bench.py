#!/usr/bin/env python
"""BASELINE config 3: in-HBM cosine top-k index sharded across the GPUs of a node, partial top-k
merged over RCCL (the pgvector replacement).

Rows are owned by ``id % world``.  Each rank holds ``rows / world`` bf16 vectors.  A search of a
query batch:

1. all-gathers the queries;
2. each rank runs the fused score GEMM + radix top-k on its shard;
3. routes each rank's packed (score, id, doc) partials back to it with all_to_all (12 B per hit) and merges.

``ShardedIndex.search`` is the same path ``bench.py`` and the RAG pipeline use.

    python benchmarks/index_bench.py --rows 10000000 --batch 1 64 512
    python benchmarks/index_bench.py --gpus 8 ...     (starts its 8 ranks itself; or one rank under torchrun)

Reported per query batch size: latency per search call (max over ranks), queries/s over the whole
job, and the effective scan rate (index bytes read per second, summed over ranks).
"""
from __future__ import annotations

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
    ap.add_argument("--rows", type=int, default=10_000_000, help="rows in the whole (sharded) index")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=250)
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 64, 512], help="queries per rank per call")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sample-stride", type=int, default=0,
                    help="A/B: the threshold search's row-sample stride (0 = VectorIndex default)")
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", 1)),
                    help="ranks; from a plain process the script starts them itself (parallel/launch.py)")
    args = ap.parse_args()

    from django_assistant_bot_amd.parallel.launch import check_world, maybe_spawn

    maybe_spawn(args.gpus, __file__)

    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    if args.sample_stride:
        from django_assistant_bot_amd.engine.vector_index import VectorIndex

        VectorIndex.sample_stride = args.sample_stride
    info = pdist.init()
    check_world(args.gpus, info.world_size)
    dev, W, R = info.device, info.world_size, info.rank
    index = ShardedIndex(args.dim, dev, capacity=args.rows // W + 1024)
    g = torch.Generator(device=dev).manual_seed(7 + R)
    mine = np.arange(R, args.rows, W, dtype=np.int64)
    for s in range(0, len(mine), 1 << 20):
        ids = mine[s:s + (1 << 20)]
        index.add(ids, torch.randn((len(ids), args.dim), device=dev, generator=g), doc_ids=ids // 10,
                  groups=np.zeros(len(ids), dtype=np.int32))
    results = []
    for B in args.batch:
        q = torch.randn((B, args.dim), device=dev, generator=g)
        for _ in range(args.warmup):
            index.search(q, args.k)
        pdist.barrier(info)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.iters):
            sims, ids, docs = index.search(q, args.k)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        pdist.barrier(info)
        el = pdist.max_over_ranks(time.perf_counter() - t0, dev)
        per_call = el / args.iters
        res = {"queries_per_rank": B, "ms_per_search": round(1000 * per_call, 3),
               "queries_per_s": round(W * B / per_call, 1),
               "scan_TBps": round(args.rows * args.dim * 2 / per_call / 1e12, 2)}
        results.append(res)
        assert ids.shape == (B, args.k)
    if R == 0:
        print(json.dumps({"metric": "sharded in-HBM cosine top-k (RCCL all_to_all merge)", "n_gpus": W,
                          "rows": args.rows, "dim": args.dim, "k": args.k, "dtype": "bf16", "data": "synthetic",
                          "results": results}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
