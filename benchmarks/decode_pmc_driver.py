"""Eager (no HIP graphs) Llama-3-8B engine run at the bench's decode shape, for rocprofv3 PMC passes:
128 sequences of ~1.1k-token prompts, one packed prefill, then ``--steps`` decode steps.  Every
kernel of the prefill and of the decode layer runs at its production configuration (the engine's
own choices), so `scripts/prof_decode_pmc.sh` can read per-kernel HBM bytes and MFMA / LDS counters.

    python benchmarks/decode_pmc_driver.py [--steps 8]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--prompt", type=int, default=1100)
    a = ap.parse_args()
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    eng = LLMEngine("llama-3-8b", torch.device("cuda"), max_batch=a.batch, use_graphs=False, seed=0)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(1000, 100000, a.prompt + int(rng.integers(0, 200))).tolist() for _ in range(a.batch)]
    outs = eng.generate(prompts, SamplingParams(max_new_tokens=a.steps, ignore_eos=True))
    torch.cuda.synchronize()
    print("decoded", sum(len(o.token_ids) for o in outs), "tokens;", eng.stats, flush=True)


if __name__ == "__main__":
    main()
