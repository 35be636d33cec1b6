"""gpu_service under concurrent load on the GPU (one process, the engine workers of
``engine/serving.py``): 32 simultaneous /dialog/ requests share continuous-batching decode steps,
16 simultaneous /embeddings/ requests share packed encoder batches, and a request whose client gives
up (asyncio timeout) frees its engine slot.  Reference: gpu_service/gunicorn_conf.py ran two
independent workers, each answering one request at a time."""
import asyncio

import pytest

pytestmark = pytest.mark.gpu
fastapi = pytest.importorskip("fastapi")
httpx = pytest.importorskip("httpx")

from gpu_service import main as svc  # noqa: E402


@pytest.fixture(scope="module")
def app():
    from django_assistant_bot_amd.engine import serving

    svc.embedders.clear()
    svc.providers.clear()
    svc.indexes.clear()
    with serving._lock:
        serving._llm.pop("tiny-llama", None)
        serving._emb.pop("tiny-bert", None)
    svc.load_models(["tiny-bert"], ["tiny-llama"])
    a = svc.FastAPI()
    for r in svc.app.routes:
        a.router.routes.append(r)
    return a


def _client(app):
    return httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://svc", timeout=120)


def test_concurrent_dialog_and_embeddings_share_batches(app):
    from django_assistant_bot_amd.engine import serving

    llm = serving._llm["tiny-llama"]
    emb = serving._emb["tiny-bert"]
    steps0 = llm.engine.stats["decode_steps"]
    toks0 = llm.engine.stats["decode_tokens"]

    async def main():
        async with _client(app) as c:
            dialogs = [c.post("/dialog/", json={"model": "tiny-llama", "max_tokens": 24, "messages": [
                {"role": "user", "content": f"question number {i}"}]}) for i in range(32)]
            embeds = [c.post("/embeddings/", json={"model": "tiny-bert", "texts": [f"text {i} {j}" for j in range(8)]})
                      for i in range(16)]
            return await asyncio.gather(*dialogs, *embeds)

    rs = asyncio.run(main())
    assert all(r.status_code == 200 for r in rs)
    assert all(len(r.json()["embeddings"]) == 8 for r in rs[32:])
    steps = llm.engine.stats["decode_steps"] - steps0
    toks = llm.engine.stats["decode_tokens"] - toks0
    # continuous batching: far fewer decode steps than generated tokens
    assert steps > 0 and toks / steps > 4, (steps, toks)
    assert llm.engine.stats["graph_replays"] > 0
    assert emb.requests >= 16


def test_client_timeout_frees_the_engine_slot(app):
    """The caller gives up (what a client disconnect or the HTTP timeout does to the handler's
    await): ``LLMWorker.generate`` turns the cancellation into an engine abort."""
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams

    llm = serving._llm["tiny-llama"]
    toks0 = llm.engine.stats["decode_tokens"]

    async def main():
        try:  # ignore_eos: the generation cannot end on its own inside the timeout
            await asyncio.wait_for(llm.generate(list(range(3, 40)), SamplingParams(max_new_tokens=1500,
                                                                                    ignore_eos=True)), timeout=0.05)
        except asyncio.TimeoutError:
            return True
        return False

    assert asyncio.run(main())
    import time

    deadline = time.time() + 30
    while time.time() < deadline and (llm.engine.running or llm.engine.waiting or llm.engine.prefilling):
        time.sleep(0.05)
    assert not llm.engine.running and not llm.engine.waiting
    assert llm.engine.blocks.num_free_blocks() == llm.engine.blocks.num_blocks()
    # the generation was cut short, not run to its 1500 tokens
    assert llm.engine.stats["decode_tokens"] - toks0 < 1400
