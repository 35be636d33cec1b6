"""LLMEngine scheduling on CPU (reference ops, native block manager): mixed prefill+decode steps must
give the same greedy tokens as the prefill-then-decode schedule, and the mixed path must actually run."""
import pytest
import torch

from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
from django_assistant_bot_amd.models import decoder_config, random_decoder_weights


def _engine(mixed: int, weights):
    return LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(weights), max_batch=8, block_size=16,
                     num_blocks=64, max_prefill_tokens=256, mixed_prefill_tokens=mixed, use_graphs=False)


def _weights():
    cfg = decoder_config("tiny-llama")
    return {k: v.float() for k, v in random_decoder_weights(cfg, dtype=torch.float32, seed=3).items()}


def _run_staggered(eng, prompts_a, prompts_b, steps_before_b=3):
    greedy = SamplingParams(max_new_tokens=12, do_sample=False, temperature=0.0, ignore_eos=True)
    rids = [eng.add_request(p, greedy) for p in prompts_a]
    for _ in range(steps_before_b):
        eng.step()
    rids += [eng.add_request(p, greedy) for p in prompts_b]
    while eng.has_unfinished():
        eng.step()
    return [eng.pop_output(r).token_ids for r in rids]


def test_mixed_steps_match_separate_schedule():
    w = _weights()
    a = [list(range(5, 5 + n)) for n in (20, 37)]
    b = [list(range(300, 300 + n)) for n in (50, 9, 70)]  # 70 > budget: split over several mixed steps
    ref_eng, mix_eng = _engine(0, w), _engine(32, w)
    ref = _run_staggered(ref_eng, a, b)
    got = _run_staggered(mix_eng, a, b)
    assert mix_eng.stats["mixed_steps"] > 0 and ref_eng.stats["mixed_steps"] == 0
    assert got == ref
    assert all(len(t) == 12 for t in got)


def test_mixed_step_accounting():
    eng = _engine(16, _weights())
    greedy = SamplingParams(max_new_tokens=8, do_sample=False, temperature=0.0, ignore_eos=True)
    eng.add_request(list(range(10, 30)), greedy)
    eng.step()  # pure prefill (nothing running)
    assert eng.stats["prefill_steps"] == 1 and len(eng.running) == 1
    eng.add_request(list(range(40, 80)), greedy)  # 40 tokens at budget 16 -> 3 mixed steps
    for _ in range(3):
        eng.step()
    assert eng.stats["mixed_steps"] == 3
    assert len(eng.running) == 2 and not eng.prefilling
    # the first request decoded one token per mixed step, the second got its first token at the end
    first, second = eng.running
    assert len(first.out) == 4
    assert len(second.out) == 1


def test_deadline_and_abort_free_blocks():
    eng = _engine(0, _weights())
    free0 = eng.blocks.num_free_blocks()
    sp = SamplingParams(max_new_tokens=50, do_sample=False, temperature=0.0, ignore_eos=True)
    a = eng.add_request(list(range(10, 40)), sp)
    b = eng.add_request(list(range(50, 70)), SamplingParams(max_new_tokens=50, ignore_eos=True, timeout_s=0.0))
    c = eng.add_request(list(range(80, 100)), sp)
    eng.step()
    assert eng.finished[b].finish_reason == "timeout"
    for _ in range(3):
        eng.step()
    assert eng.abort(a)
    assert not eng.abort(12345)
    out_a = eng.pop_output(a)
    assert out_a.finish_reason == "abort" and 1 <= len(out_a.token_ids) < 50
    while eng.has_unfinished():
        eng.step()
    assert len(eng.pop_output(c).token_ids) == 50
    assert eng.blocks.num_free_blocks() == free0


def test_worker_survives_injected_faults_and_flags_sticky_ones():
    from django_assistant_bot_amd.engine import serving

    eng = _engine(0, _weights())
    worker = serving.LLMWorker(eng)
    try:
        sp = SamplingParams(max_new_tokens=5, do_sample=False, temperature=0.0, ignore_eos=True)
        fired = []

        def fault_once(e):
            if not fired:
                fired.append(1)
                raise RuntimeError("injected step failure")
        eng.fault_hook = fault_once
        fut = worker.submit(list(range(5, 25)), sp)
        try:
            fut.result(timeout=60)
            raise AssertionError("expected the injected failure")
        except RuntimeError as exc:
            assert "injected" in str(exc)
        assert worker.faults == 1 and worker.healthy
        # the engine keeps serving after the reset, with the block pool intact
        out = worker.submit(list(range(5, 25)), sp).result(timeout=60)
        assert len(out.token_ids) == 5
        assert eng.blocks.num_free_blocks() == eng.blocks.num_blocks()
        # a sticky device error marks the worker unhealthy (gpu_service /health -> 503)
        eng.fault_hook = lambda e: (_ for _ in ()).throw(
            RuntimeError("HIP error: an illegal memory access was encountered"))
        fut = worker.submit(list(range(5, 25)), sp)
        try:
            fut.result(timeout=60)
        except RuntimeError:
            pass
        assert not worker.healthy and "illegal memory access" in worker.last_error
        serving._llm["fault-test"] = worker
        try:
            h = serving.health()
            assert not h["healthy"] and "fault-test" in h["unhealthy_workers"]
        finally:
            serving._llm.pop("fault-test", None)
    finally:
        worker.stop()


def test_worker_marks_a_broken_tp_group_unhealthy():
    """A TP step that raises ``CustomAllReduceError`` (a peer missed a one-shot all-reduce: the
    step's outputs are poisoned) fails the in-flight requests and turns the worker unhealthy, so
    gpu_service /health answers 503 and the launcher restarts the group."""
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.parallel.custom_allreduce import CustomAllReduceError

    eng = _engine(0, _weights())
    worker = serving.LLMWorker(eng)
    try:
        sp = SamplingParams(max_new_tokens=5, do_sample=False, temperature=0.0, ignore_eos=True)

        def broken(e):
            raise CustomAllReduceError("custom all-reduce: a TP peer did not arrive")
        eng.fault_hook = broken
        fut = worker.submit(list(range(5, 25)), sp)
        with pytest.raises(CustomAllReduceError):
            fut.result(timeout=60)
        assert not worker.healthy and "TP peer" in worker.last_error
        assert not eng.has_unfinished() and not eng.finished
        serving._llm["tp-test"] = worker
        try:
            assert not serving.health()["healthy"]
        finally:
            serving._llm.pop("tp-test", None)
    finally:
        worker.stop()


def _pipe_engine(pipeline: bool, weights):
    return LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(weights), max_batch=8, block_size=16,
                     num_blocks=64, max_prefill_tokens=256, use_graphs=False, pipeline_decode=pipeline)


def test_pipelined_decode_matches_synchronous():
    """Step t+1 launched before step t's tokens are read (ids from the device tokens) must produce
    exactly the synchronous engine's tokens: greedy decode with stop tokens (a stopped sequence's
    extra in-flight token is discarded), sampled decode with per-request lengths (host-predicted
    finishes; the CPU reference sampler draws per batch, so the batches must match too), and a
    request arriving mid-decode (the pipeline drains for its prefill)."""
    w = _weights()
    prompts = [list(range(7, 7 + n)) for n in (12, 30, 5, 44)]
    greedy = dict(do_sample=False, temperature=0.0)
    outs = {}
    for pipe in (False, True):
        eng = _pipe_engine(pipe, w)
        rids = []
        for i, p in enumerate(prompts):
            sp = SamplingParams(max_new_tokens=6 + 3 * i, temperature=0.9, top_k=20, top_p=0.9, seed=11,
                                ignore_eos=True)
            rids.append(eng.add_request(p, sp))
        while eng.has_unfinished():
            eng.step()
        sampled = [eng.pop_output(r).token_ids for r in rids]
        # greedy with a request arriving mid-decode (the pipelined engine is one step further when it
        # arrives; greedy tokens do not depend on the batch composition)
        rids = [eng.add_request(p, SamplingParams(max_new_tokens=20, **greedy)) for p in prompts]
        for _ in range(4):
            eng.step()
        late = eng.add_request(list(range(900, 925)), SamplingParams(max_new_tokens=9, **greedy))
        while eng.has_unfinished():
            eng.step()
        sampled.append(eng.pop_output(late).token_ids)
        free_run = [eng.pop_output(r).token_ids for r in rids]
        stops = tuple({t[3] for t in free_run})
        rids = [eng.add_request(p, SamplingParams(max_new_tokens=20, stop_token_ids=stops, **greedy)) for p in prompts]
        while eng.has_unfinished():
            eng.step()
        stopped = [(eng.pop_output(r).token_ids, eng.finished.get(r)) for r in rids]
        outs[pipe] = (sampled, free_run, [t for t, _ in stopped])
        assert eng.blocks.num_free_blocks() == eng.blocks.num_blocks()
        assert all(len(t) <= 4 for t in outs[pipe][2])
    assert outs[True] == outs[False]


def test_prefix_blocks_are_shared_from_the_launch_of_their_chunk():
    """full blocks of a prompt chunk enter the prefix cache when the chunk is launched, not
    when the whole prompt (or the deferred read-back) completes.  A request that shares a long
    prompt's first chunk and arrives while that prompt is still being prefilled reuses those blocks;
    its tokens equal a cold run's."""
    w = _weights()
    greedy = SamplingParams(max_new_tokens=6, do_sample=False, temperature=0.0, ignore_eos=True)
    shared = list(range(7, 7 + 128))
    long_prompt = shared + list(range(400, 400 + 300))  # 428 tokens: two 256-token prefill chunks
    other = shared + [900, 901, 902]
    eng = LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(w), max_batch=8, block_size=16,
                    num_blocks=96, max_prefill_tokens=256, use_graphs=False)
    r1 = eng.add_request(long_prompt, greedy)
    eng.step()  # first chunk (256 tokens) launched; the prompt is not complete yet
    assert eng.stats["prefill_tokens"] == 256
    r2 = eng.add_request(other, greedy)
    before = eng.blocks.prefix_hits()
    while eng.has_unfinished():
        eng.step()
    assert eng.blocks.prefix_hits() - before >= 128  # the shared 8 blocks came from the cache
    cold = LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(w), max_batch=8, block_size=16,
                     num_blocks=96, max_prefill_tokens=256, use_graphs=False, prefix_cache=False)
    c2 = cold.add_request(other, greedy)
    while cold.has_unfinished():
        cold.step()
    assert eng.pop_output(r2).token_ids == cold.pop_output(c2).token_ids
    assert len(eng.pop_output(r1).token_ids) == 6


def _preempt_run(eng, prompts, abort_idx=None, steps_before_abort=6):
    greedy = SamplingParams(max_new_tokens=40, do_sample=False, temperature=0.0, ignore_eos=True)
    rids = [eng.add_request(p, greedy) for p in prompts]
    for _ in range(steps_before_abort):
        eng.step()
    if abort_idx is not None:
        assert eng.abort(rids[abort_idx])
    while eng.has_unfinished():
        eng.step()
    return [eng.pop_output(r) for r in rids]


def test_preemption_recompute_matches_an_unconstrained_pool():
    """A KV pool too small for the batch: the youngest sequences are preempted (blocks freed,
    re-queued, prompt + generated tokens recomputed) and still produce the tokens of a run that never
    ran dry; an abort in the middle frees its blocks; prompts sharing a 32-token prefix reuse blocks.
    Every block is free at the end."""
    w = _weights()
    shared = list(range(500, 532))
    prompts = [shared + list(range(10 * i, 10 * i + 8 + 5 * i)) for i in range(6)]

    def engine(blocks):
        return LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(w), max_batch=8, block_size=16,
                         num_blocks=blocks, max_prefill_tokens=512, use_graphs=False)

    ref = [o.token_ids for o in _preempt_run(engine(256), prompts)]
    small = engine(18)  # 6 sequences need up to 6 x 7 blocks
    outs = _preempt_run(small, prompts)
    assert small.stats["preemptions"] > 0
    assert [o.token_ids for o in outs] == ref
    assert small.blocks.num_free_blocks() == small.blocks.num_blocks()
    # with an abort: the aborted request ends early, the others are unchanged
    small = engine(18)
    outs = _preempt_run(small, prompts, abort_idx=2)
    assert outs[2].finish_reason == "abort" and len(outs[2].token_ids) < 40
    assert [o.token_ids for i, o in enumerate(outs) if i != 2] == [t for i, t in enumerate(ref) if i != 2]
    assert small.blocks.num_free_blocks() == small.blocks.num_blocks()


def test_prefix_blocks_are_shared_within_one_prefill_step():
    """Requests admitted in the same prefill step share the blocks of their common prefix (committed
    as each chunk is scheduled): only the first computes them, and every request's greedy tokens
    equal a cold run without the prefix cache."""
    w = _weights()
    greedy = SamplingParams(max_new_tokens=5, do_sample=False, temperature=0.0, ignore_eos=True)
    shared = list(range(11, 11 + 64))  # 4 full 16-token blocks
    prompts = [shared + [300 + 7 * i + j for j in range(5 + i)] for i in range(5)]
    outs = {}
    for cache in (True, False):
        eng = LLMEngine(decoder_config("tiny-llama"), device="cpu", weights=dict(w), max_batch=8, block_size=16,
                        num_blocks=96, max_prefill_tokens=1024, use_graphs=False, prefix_cache=cache)
        rids = [eng.add_request(p, greedy) for p in prompts]
        eng.step()  # every prompt is admitted and prefilled in this one step
        if cache:
            assert eng.stats["prefill_tokens"] == sum(len(p) for p in prompts) - 4 * 64
            assert eng.blocks.prefix_hits() >= 4 * 64
        while eng.has_unfinished():
            eng.step()
        outs[cache] = [eng.pop_output(r).token_ids for r in rids]
    assert outs[True] == outs[False]
