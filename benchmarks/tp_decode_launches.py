"""Kernel launches of one tensor-parallel decode step, with and without the fused all-reduce + RMSNorm
(``allreduce_rmsnorm_kernel`` replaces slab_reduce + the one-shot all-reduce +
rmsnorm at every TP all-reduce site).

W ranks share the box's GPU (gloo default group, IPC all-reduce).  Each rank prefills a small batch,
then runs ONE eager decode step (the body the decode graph captures) under ``torch.profiler`` for
each setting and counts the kernels by name; rank 0 prints one JSON line.

    python benchmarks/tp_decode_launches.py [--model tiny-llama-70b-d128] [--world 2]
"""
import argparse
import collections
import datetime
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _family(name: str) -> str:
    for key in ("allreduce_rmsnorm_kernel", "allreduce_kernel", "slab_reduce", "rmsnorm_slab", "rmsnorm_kernel",
                "stream_gemm", "paged_decode", "rope_kv", "sample", "embed_gather", "chunk_topk"):
        if key in name:
            return key
    return "other:" + name.split("(")[0].split("<")[0][-48:]


def _rank(rank, world, port, args, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.profiler import ProfilerActivity, profile

    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.parallel import dist as pdist

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(0)
    try:
        group, tp_rank, _ = pdist.tp_groups(world)
        eng = LLMEngine(args.model, device="cuda:0", seed=3, max_batch=args.batch, max_model_len=1024,
                        kv_cache_gb=1.0, max_prefill_tokens=4096, tp_group=group, tp_size=world, tp_rank=tp_rank,
                        use_graphs=False)
        g = torch.Generator().manual_seed(5)
        sp = SamplingParams(max_new_tokens=64, temperature=1.0, top_k=50, top_p=0.95, ignore_eos=True)
        for i in range(args.batch):
            eng.add_request(torch.randint(100, 1000, (100 + 7 * i,), generator=g).tolist(), sp)
        while eng.waiting or eng.prefilling or eng._pending_prefill is not None:
            eng.step()
        res = {}
        for fused in (True, False):
            eng.model.tp_fused_norm = fused
            eng.step()  # one untimed step in this setting
            torch.cuda.synchronize()
            dist.barrier()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                eng.step()
                torch.cuda.synchronize()
            counts = collections.Counter()
            for ev in prof.events():
                if ev.device_type == torch.autograd.DeviceType.CUDA:
                    counts[_family(ev.name)] += 1
            res["fused" if fused else "unfused"] = dict(counts)
            dist.barrier()
        eng.model.custom_ar.check_error()
        if rank == 0:
            cfg = eng.cfg
            out = {"op": "tp-decode-launches", "model": args.model, "tp": world, "layers": cfg.layers,
                   "allreduce_sites_per_step": 2 * cfg.layers, "batch": args.batch,
                   "kernels_per_step": {k: sum(v.values()) for k, v in res.items()}, **res}
            print(json.dumps(out), flush=True)
            with open(out_path, "w") as f:
                f.write(json.dumps(out) + "\n")
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tiny-llama-70b-d128")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/tp_decode_launches.json")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    mp.spawn(_rank, args=(args.world, _free_port(), args, args.out), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
