"""BASELINE config 5's generator at its real size on ONE MI355X: Llama-3-70B
(80 layers, hidden 8192, 64 / 8 heads, FFN 28672, vocab 128256) tensor-parallel over 8 ranks that
share the card -- gloo default group, the one-shot IPC all-reduce for the TP partial sums inside the
HIP-graph decode, the vocabulary-parallel LM head.  Each rank random-inits only its own shard
(~17.5 GB of layers + the replicated 2.1 GB embedding + 1/8 of the head), so the whole group fits in
the card's 288 GB.

Reports per rank: HBM held (allocated / reserved), weight bytes, LM-head bytes, init and
graph-capture times; for the group: whether every rank produced the same sampled tokens (top-k 50,
top-p 0.95, temperature 1: the reference's generate() settings, /root/reference/assistant/ai/
providers/transformers.py:57-66), decode steps and the mean step time (8 ranks time-share one GPU,
so the step time is a rehearsal number, not the 8-GPU one).

    python benchmarks/tp70b_rehearsal.py [--world 8] [--batch 8] [--prompt 512] [--new 16]
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tensor_bytes(model) -> tuple[int, int]:
    total = model.embed.numel() * 2 + model.lm_head.numel() * 2 + model.final_norm.numel() * 2
    for L in model.layers:
        for t in (L.attn_norm, L.qkv_w, L.o_w, L.mlp_norm, L.gate_up_w, L.down_w):
            total += t.numel() * t.element_size()
    return total, model.lm_head.numel() * model.lm_head.element_size()


def _rank(rank, world, port, args, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.parallel import dist as pdist

    import datetime

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(0)

    def say(msg):  # progress on stdout (a silent multi-minute phase looks hung)
        print(f"[rank {rank}] {time.strftime('%H:%M:%S')} {msg}", flush=True)

    try:
        group, tp_rank, _ = pdist.tp_groups(world)
        t0 = time.perf_counter()
        eng = LLMEngine(args.model, device="cuda:0", seed=3, max_batch=args.batch, max_model_len=args.ctx,
                        kv_cache_gb=args.kv_gb, max_prefill_tokens=args.batch * args.prompt, tp_group=group,
                        tp_size=world, tp_rank=tp_rank)
        torch.cuda.synchronize()
        init_s = time.perf_counter() - t0
        say(f"engine ready in {init_s:.1f} s, {torch.cuda.memory_allocated() / 2 ** 30:.1f} GB allocated")
        wbytes, head_bytes = _tensor_bytes(eng.model)
        dist.barrier()
        t1 = time.perf_counter()
        eng.capture_all()
        torch.cuda.synchronize()
        capture_s = time.perf_counter() - t1
        say(f"{len(eng._graphs)} decode graphs captured in {capture_s:.1f} s")
        dist.barrier()
        g = torch.Generator().manual_seed(11)
        prompts = [torch.randint(100, eng.cfg.vocab_size, (args.prompt + 17 * i,), generator=g).tolist()
                   for i in range(args.batch)]
        sp = SamplingParams(max_new_tokens=args.new, temperature=1.0, top_k=50, top_p=0.95, ignore_eos=True)
        s0 = dict(eng.stats)
        t2 = time.perf_counter()
        outs = eng.generate(prompts, sp)
        torch.cuda.synchronize()
        gen_s = time.perf_counter() - t2
        say(f"generated in {gen_s:.1f} s")
        eng.model.custom_ar.check_error()
        toks = [o.token_ids for o in outs]
        gathered = [None] * world
        dist.all_gather_object(gathered, toks)
        free, total = torch.cuda.mem_get_info()
        mine = {"rank": rank, "init_s": round(init_s, 2), "capture_s": round(capture_s, 2),
                "graphs": len(eng._graphs), "hbm_allocated_gb": round(torch.cuda.memory_allocated() / 2 ** 30, 2),
                "hbm_reserved_gb": round(torch.cuda.memory_reserved() / 2 ** 30, 2),
                "weight_gb": round(wbytes / 2 ** 30, 2), "lm_head_gb": round(head_bytes / 2 ** 30, 3),
                "kv_blocks": eng.kv.num_blocks}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        if rank == 0:
            dec = eng.stats["decode_steps"] - s0["decode_steps"]
            res = {"op": "tp70b-rehearsal", "model": args.model, "tp": world, "layers": eng.cfg.layers,
                   "hidden": eng.cfg.hidden, "intermediate": eng.cfg.intermediate, "vocab": eng.cfg.vocab_size,
                   "vocab_parallel": eng.vp, "batch": args.batch, "prompt_tokens": args.prompt,
                   "new_tokens": args.new, "ranks_agree": all(x == toks for x in gathered),
                   "tokens_per_seq": [len(t) for t in toks], "decode_steps": dec,
                   "graph_replays": eng.stats["graph_replays"] - s0["graph_replays"],
                   "generate_s": round(gen_s, 2), "card_free_gb_after_load": round(free / 2 ** 30, 1),
                   "card_total_gb": round(total / 2 ** 30, 1), "per_rank": ranks}
            print(json.dumps(res), flush=True)
            with open(out_path, "w") as f:
                f.write(json.dumps(res) + "\n")
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--kv-gb", type=float, default=2.0)
    ap.add_argument("--out", default="gpurun_out/tp70b_rehearsal.json")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    mp.spawn(_rank, args=(args.world, _free_port(), args, args.out), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
