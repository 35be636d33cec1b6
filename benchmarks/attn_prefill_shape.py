"""Prefill attention at the headline's prefill-step shape: ~30 prompts of 989-1189 tokens (1089 mean,
the bench's RAG prompts) packed into one 32k-token step, causal, q read from the strided qkv
projection with RoPE on load (the model's call, models/llama.py _layer prefill path).  Against
uniform 1024-token sequences, so the loss from ragged lengths (partial 128-row query blocks) is
visible.  One JSON line per case: us, exact causal TF/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.kernel_bench import timeit  # noqa: E402
from django_assistant_bot_amd import ops  # noqa: E402

Hq, Hkv, D, bs = 32, 8, 128, 64


def case(name, lens, prefix=0, pool_blocks=0):
    """lens: query tokens per sequence; prefix: cached tokens before them (the prompt's system block
    comes from the prefix cache, so the engine's queries start at position 64)."""
    B = len(lens)
    ctx_l = [n + prefix for n in lens]
    T = int(sum(lens))
    nbl = [-(-n // bs) for n in ctx_l]
    nb = max(sum(nbl), pool_blocks)
    kc = torch.randn(nb, Hkv, bs, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.zeros((B, max(nbl)), dtype=torch.int32)
    # pool_blocks: the blocks scattered at random over a pool that large (the engine's per-layer KV
    # pool after many batches), else packed in order
    ids = torch.randperm(nb, generator=torch.Generator().manual_seed(1)).to(torch.int32) if pool_blocks else \
        torch.arange(nb, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nbl):
        bt[i, :n] = ids[o:o + n]
        o += n
    bt = bt.cuda()
    cu = torch.zeros(B + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(lens), 0)
    cu = cu.cuda()
    ctx = torch.tensor(ctx_l, dtype=torch.int32, device="cuda")
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").to(torch.bfloat16)
    q = qkv[:, :Hq * D].view(T, Hq, D)
    pos = torch.cat([torch.arange(prefix, prefix + n, dtype=torch.int32) for n in lens]).cuda()
    cs = ops.reference.rope_cos_sin(ops.reference.llama3_inv_freq(D, 500000.0, None), 8192).cuda()
    mx = int(max(lens))
    flop = sum(4.0 * Hq * D * n * ((n + 1) / 2 + prefix) for n in lens)
    res = {"case": name, "seqs": B, "tokens": T}
    times = {a: [] for a in ARMS}
    base = None
    npairs = (-(-max(lens) // 128) + 1) // 2
    g_r5 = max(1, min(npairs, npairs * Hq * B // 1024))
    for _ in range(ROUNDS):  # interleaved rounds: no arm is always the first one timed
        for arm, env in ARMS.items():
            if env is None:
                env = {"DAB_FLASH_LPT": "0", "DAB_FLASH_G": str(g_r5)}
            for k in ("DAB_FLASH_G", "DAB_FLASH_PAIR", "DAB_FLASH_LPT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            run = lambda: ops.flash_attention_paged(q, kc, vc, bt, cu, ctx, mx, causal=True, rope=(pos, cs))  # noqa: E731
            out = run()
            if base is None:
                base = out
            else:
                assert torch.equal(out, base), arm
            times[arm].append(timeit(run))
    for k in ("DAB_FLASH_G", "DAB_FLASH_PAIR", "DAB_FLASH_LPT"):
        os.environ.pop(k, None)
    for arm, ts in times.items():
        t = sorted(ts)[len(ts) // 2]
        res[f"{arm}_us"] = round(t * 1e6, 1)
        res[f"{arm}_tflops"] = round(flop / t / 1e12, 1)
    print(json.dumps(res), flush=True)


# default = heaviest-first walk, G = 2 (1 below 1024 workgroups); "r5" = the round-5 choice (G = pairs
# x heads x seqs / 1024, alternating walk); "fifo" = the alternating walk with the default G; gN =
# heaviest-first with G forced to N
ARMS = {"default": {}, "r5": None, "fifo": {"DAB_FLASH_LPT": "0"}, "g1": {"DAB_FLASH_G": "1"}, "g2": {"DAB_FLASH_G": "2"},
        "g4": {"DAB_FLASH_G": "4"}, "nopair": {"DAB_FLASH_PAIR": "0"}}
ROUNDS = 3


def main():
    g = torch.Generator().manual_seed(0)
    if os.environ.get("ATTN_SINGLE"):  # single prompts (time to first token): pairs vs one block per workgroup
        for lens in ([512], [1024], [2048], [4096], [1024] * 2, [1024] * 4):
            case(f"single-{len(lens)}x{lens[0]}", lens)
        return
    case("uniform-32x1024", [1024] * 32)
    case("uniform-8x4096", [4096] * 8)
    case("uniform-4x300", [300] * 4)
    # the engine's headline prefill step: 1089 +- 100-token prompts minus the 64-token cached system
    # block, packed up to 32,768 query tokens; and the classify fast step (774-token prompts)
    real, tot = [], 0
    while tot < 32768:
        n = min(int(torch.randint(989, 1190, (1,), generator=g)) - 64, 32768 - tot)
        real.append(n)
        tot += n
    case("engine-step", real, prefix=64)
    case("engine-step-scattered", real, prefix=64, pool_blocks=12000)
    case("engine-step-33", [990] * 33, prefix=64)  # the traced step: 33 sequences (1056 units)
    case("engine-classify", [710] * 46, prefix=64)
    lens = torch.randint(989, 1190, (30,), generator=g).tolist()
    case("ragged-30x989..1189", lens)


if __name__ == "__main__":
    main()
