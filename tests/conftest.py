import os
import random
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "django: needs Django / DRF installed")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def bpe_dir(tmp_path_factory):
    """A byte-level BPE tokenizer.json for tiny-llama (1000 trained tokens, <|bos|> = 1000,
    <|eos|> = 1001): the kind of vocabulary real checkpoints ship (Llama-3 is byte-level BPE)."""
    tokenizers = pytest.importorskip("tokenizers")
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
    n = tok.get_vocab_size()
    tok.add_tokens([f"<pad{i}>" for i in range(1000 - n)])
    tok.add_special_tokens(["<|bos|>", "<|eos|>"])
    assert tok.token_to_id("<|bos|>") == 1000 and tok.token_to_id("<|eos|>") == 1001
    d = tmp_path_factory.mktemp("bpe")
    tok.save(str(d / "tokenizer.json"))
    return str(d)


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """GPU tests that run for minutes (multi-process TP groups time-sharing the box's one GPU) print a
    line every 30 s to the real stderr, past pytest's capture, so a long but live test is never taken
    for a hung one by the GPU harness's silence watchdog."""
    if "gpu" not in request.node.keywords:
        yield
        return
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(30):
            sys.__stderr__.write(f"[heartbeat] {request.node.nodeid} running {time.time() - t0:.0f} s\n")
            sys.__stderr__.flush()

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
