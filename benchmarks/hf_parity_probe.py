"""Teacher-forced greedy parity of the GPU engine against an HF fp32 Llama (the model of
tests/test_hf_dirs.py::test_llm_engine_runs_a_saved_hf_llama_on_gpu), per GEMM dispatch arm.

For every generated token: the gap between HF's best logit and HF's logit of the engine's token,
relative to the row's max |logit| (0 when the engine took HF's argmax).  Arms: the production
dispatch (mid-M prefill GEMMs on gemm_mid) and gemm_mid switched off (GEMM_MID_MIN_M raised).

    python benchmarks/hf_parity_probe.py [--tie 1]
"""
import argparse
import json
import os
import random
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bpe_dir(root: str) -> str:
    """The byte-level BPE tokenizer of tests/conftest.py::bpe_dir."""
    import tokenizers
    from tokenizers import decoders, models, pre_tokenizers, trainers

    tok = tokenizers.Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    rng = random.Random(0)
    words = ["topic", "question", "billing", "access", "small", "talk", "null", "true", "false", "name", "score"]
    corpus = [" ".join(rng.choice(words) + rng.choice(["", "s", "ing", '":', '"}', "{", ","]) for _ in range(12))
              for _ in range(3000)] + ['{"topic": "Billing"}', '{"question": 3}', "Доступ к аккаунту"] * 50
    trainer = trainers.BpeTrainer(vocab_size=1000, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  show_progress=False)
    tok.train_from_iterator(corpus, trainer)
    tok.add_tokens([f"<pad{i}>" for i in range(1000 - tok.get_vocab_size())])
    tok.add_special_tokens(["<|bos|>", "<|eos|>"])
    d = os.path.join(root, "bpe")
    os.makedirs(d, exist_ok=True)
    tok.save(os.path.join(d, "tokenizer.json"))
    return d


def gaps(hf, prompts, outs):
    res = []
    for p, t in zip(prompts, outs):
        with torch.no_grad():
            lg = hf(torch.tensor([p + t[:-1]])).logits[0, len(p) - 1:].float()
        for j, tok in enumerate(t):
            best = int(lg[j].argmax())
            res.append(0.0 if tok == best else float(lg[j, best] - lg[j, tok]) / float(lg[j].abs().max()))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tie", type=int, default=1)
    args = ap.parse_args()
    from django_assistant_bot_amd import ops
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from tests.test_hf_dirs import LLAMA3_SCALING, _llama_dir

    tmp = tempfile.mkdtemp()
    hf, d = _llama_dir(tmp, bpe_dir(tmp), rope_scaling=LLAMA3_SCALING, hidden=512, heads=4, kv_heads=2,
                       tie=bool(args.tie))
    texts = ["the quick brown fox", "jumps over the lazy dog again and again", "a" * 300]
    base_min = ops.kernels.GEMM_MID_MIN_M
    for arm, min_m in (("gemm_mid", base_min), ("no_gemm_mid", 1 << 30)):
        ops.kernels.GEMM_MID_MIN_M = min_m
        eng = LLMEngine(d, device="cuda", max_batch=8, block_size=64, num_blocks=64)
        prompts = [eng.tokenizer.encode(t) for t in texts]
        sp = SamplingParams(max_new_tokens=16, do_sample=False, temperature=0.0, ignore_eos=True)
        outs = [o.token_ids for o in eng.generate(prompts, sp)]
        g = gaps(hf, prompts, outs)
        print(json.dumps({"arm": arm, "tie": args.tie, "prompt_tokens": [len(p) for p in prompts],
                          "exact": round(sum(x == 0 for x in g) / len(g), 4), "max_gap_rel": round(max(g), 5),
                          "gaps_over_1pct": sorted(round(x, 4) for x in g if x > 0.01)}), flush=True)
        del eng
        torch.cuda.empty_cache()
    ops.kernels.GEMM_MID_MIN_M = base_min


if __name__ == "__main__":
    main()
