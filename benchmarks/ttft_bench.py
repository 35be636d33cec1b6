"""Time to first token of ONE prompt (the reference's request-at-a-time shape: one HF ``generate``
per request) on Llama-3-8B, random init: the prefill step plus the first token's sampling, for prompt
lengths 16..1024, with the round-6 small-step paths (prefill <= 128 tokens on the streaming decode
layer, gemm_mid from M = 1) against the round-5 dispatch (MFMA 128 x 128 tiles below M = 192).
Median of 7 generations with max_new_tokens = 1 (prefix cache off, so every run prefills)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams  # noqa: E402


def main():
    eng = LLMEngine("llama-3-8b", device="cuda", max_batch=8, kv_cache_gb=8, prefix_cache=False)
    sp = SamplingParams(max_new_tokens=1, ignore_eos=True)
    g = torch.Generator().manual_seed(0)
    arms = {"r6": (type(eng.model).PREFILL_STREAM_MAX_M, ops.kernels.GEMM_MID_MIN_M), "r5": (0, 192)}
    for T in (16, 64, 100, 128, 187, 300, 1024):
        ids = torch.randint(0, 128000, (T,), generator=g).tolist()
        res = {"prompt_tokens": T}
        for _ in range(2):  # interleaved
            for arm, (pf, mid) in arms.items():
                eng.model.PREFILL_STREAM_MAX_M, ops.kernels.GEMM_MID_MIN_M = pf, mid
                eng.generate([ids], sp)  # warm
                ts = []
                for _ in range(7):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    eng.generate([ids], sp)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                res.setdefault(f"{arm}_ms", []).append(round(sorted(ts)[3] * 1e3, 2))
        for arm in arms:
            res[f"{arm}_ms"] = min(res[f"{arm}_ms"])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
