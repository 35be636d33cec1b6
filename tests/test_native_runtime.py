"""Native host runtime (C++): tokenizer, paged-KV block manager with prefix caching, RAG aggregation."""
import numpy as np
import pytest

from django_assistant_bot_amd.ops import native


@pytest.fixture(scope="module")
def n():
    return native()


def _tok(n, vocab=30522, first=1000, cls=101, sep=102):
    c = n.TokenizerConfig()
    c.vocab_size, c.first_id, c.last_id, c.cls_id, c.sep_id = vocab, first, vocab, cls, sep
    return n.HashTokenizer(c)


def test_tokenizer_framing_truncation(n):
    t = _tok(n)
    ids = t.encode("Hello, World! hello", True, 0)
    assert ids[0] == 101 and ids[-1] == 102
    assert ids[1] == ids[5]  # case-insensitive: "Hello" == "hello" ([CLS] hello , world ! hello [SEP])
    assert len(t.encode("a b c d e f g", True, 5)) == 5
    assert t.encode("a b c", True, 5)[-1] == 102
    assert all(1000 <= i < 30522 for i in t.encode("words only", False, 0))


def test_tokenizer_unicode_and_batch(n):
    t = _tok(n)
    ru = t.encode("Привет, мир! ПРИВЕТ", False, 0)
    assert ru[0] == ru[4] and len(ru) == 5  # привет , мир ! привет
    flat, offs = t.encode_batch(["one two", "", "три четыре пять"], True, 0, 4)
    assert list(offs) == [0, 4, 6, 11]
    assert t.decode([int(x) for x in flat[offs[2]:offs[3]]], True) == "три четыре пять"
    assert n.HashTokenizer.count_words("  a  b\nc ") == 3


def test_tokenizer_decoder_mode_and_pseudo_words(n):
    t = _tok(n, vocab=128256, first=0, cls=128000, sep=-1)
    ids = t.encode("hi there", True, 0)
    assert ids[0] == 128000 and len(ids) == 3
    s = t.decode([5, 77, 12345], True)
    assert isinstance(s, str) and len(s.split()) == 3


def test_kv_manager_alloc_extend_free(n):
    m = n.KVBlockManager(8, 4, False)
    assert m.add_sequence(1, list(range(10)), 1) == 0
    assert m.num_free_blocks() == 5 and m.capacity_tokens(1) == 12
    assert m.extend(1, 2)
    assert not m.extend(1, 100)
    m.append_tokens(1, [7, 8])
    assert m.num_tokens(1) == 12
    slots = np.zeros(3, dtype=np.int64)
    m.slot_mapping_into(1, 3, 3, slots.ctypes.data)
    bl = m.blocks(1)
    assert list(slots) == [bl[0] * 4 + 3, bl[1] * 4 + 0, bl[1] * 4 + 1]
    bt = np.full((2, 5), -7, dtype=np.int32)
    m.block_table_into([1, -1], 5, bt.ctypes.data)
    assert list(bt[0][:3]) == list(bl) and list(bt[1]) == [0] * 5
    m.free_sequence(1)
    assert m.num_free_blocks() == 8
    assert m.add_sequence(2, list(range(40)), 0) == -1  # does not fit, nothing allocated
    assert m.num_free_blocks() == 8


def test_kv_manager_prefix_cache(n):
    m = n.KVBlockManager(16, 4, True)
    prompt = list(range(100, 111))  # 11 tokens -> 2 full blocks registrable
    assert m.add_sequence(1, prompt, 1) == 0
    m.commit_prefix(1, len(prompt))
    assert m.add_sequence(2, prompt + [5], 1) == 8  # two cached blocks reused
    shared = m.blocks(2)[:2]
    assert list(shared) == list(m.blocks(1)[:2])
    m.free_sequence(1)
    m.free_sequence(2)
    # cached blocks survive in the LRU and are reused by a third request
    assert m.add_sequence(3, prompt, 1) == 8
    assert m.prefix_hits() == 16
    m.free_sequence(3)
    # pressure evicts the cache instead of failing
    assert m.add_sequence(4, list(range(60)), 0) == 0
    assert m.num_free_blocks() == 1


def test_aggregate_documents_reference_semantics(n):
    # hits sorted by distance; doc 7 has 3 hits, doc 9 has 2, doc 5 has 1
    dist = np.array([0.1, 0.2, 0.25, 0.3, 0.4, 0.5], dtype=np.float32)
    docs = np.array([7, 9, 7, 5, 9, 7], dtype=np.int64)
    out = n.aggregate_documents(dist, docs, 2, 10)
    # doc 7: 1 - (0.1+0.25)/2 = 0.825 ; doc 9: 1 - (0.2+0.4)/2 = 0.7 ; doc 5 dropped (<2 hits)
    assert [d for d, _ in out] == [7, 9]
    assert abs(out[0][1] - 0.825) < 1e-6 and abs(out[1][1] - 0.7) < 1e-6
    assert len(n.aggregate_documents(dist, docs, 2, 1)) == 1
    dist[1] = np.inf  # filtered rows never count
    assert [d for d, _ in n.aggregate_documents(dist, docs, 2, 10)] == [7]


def test_merge_topk(n):
    vals = np.array([[0.9, 0.5, 0.1], [0.8, 0.7, -np.inf]], dtype=np.float32)
    ids = np.array([[1, 2, 3], [4, 5, -1]], dtype=np.int64)
    v, i = n.merge_topk(vals, ids, 4)
    assert list(i) == [1, 4, 5, 2] and np.allclose(v, [0.9, 0.8, 0.7, 0.5])


def test_kv_manager_packs_blocks_low_and_caps_cached_prefixes(n):
    """Fresh blocks come lowest id first (a batch's live blocks stay packed at the low end of the
    pool) and at most max(64, pool / 4) unreferenced prefix blocks are kept cached."""
    m = n.KVBlockManager(1024, 4, True)
    for s in range(100):  # 100 sequences x 3 registrable blocks, all freed -> 300 cached > cap 256
        m.add_sequence(s, [s * 1000 + i for i in range(13)], 0)
        m.commit_prefix(s, 13)
    for s in range(100):
        m.free_sequence(s)
    assert m.num_free_blocks() == 1024
    # the 44 oldest cached blocks went back to the free heap; a new sequence packs into the lowest
    # free ids (not the LRU tail of the pool)
    m.add_sequence(500, list(range(7000, 7040)), 0)
    got = list(m.blocks(500))
    assert got == sorted(got) and got[0] < 400 and len(got) == 10
    # the most recently cached prefixes still hit
    assert m.add_sequence(501, [99 * 1000 + i for i in range(13)], 0) == 12


def test_every_native_entry_point_called_from_python_is_bound(n):
    """Each ``native().<name>`` the Python package calls exists in the built extension (a binding lost
    in an edit otherwise only shows up on the GPU box)."""
    import pathlib
    import re

    root = pathlib.Path(__file__).resolve().parents[1]
    names = set()
    for d in ("django_assistant_bot_amd", "gpu_service", "benchmarks", "tests"):
        for f in (root / d).rglob("*.py"):
            names |= set(re.findall(r"native\(\)\.([A-Za-z_]\w*)", f.read_text()))
    assert len(names) > 20
    missing = sorted(x for x in names if not hasattr(n, x))
    assert not missing, missing


def test_build_scratch_guard_parses_resource_usage():
    """The build refuses kernels with a scratch frame (runtime-indexed register arrays moved to
    memory); the parser reads hipcc's -Rpass-analysis=kernel-resource-usage remarks."""
    from django_assistant_bot_amd.build import scratch_kernels

    log = "\n".join([
        "a.hip:1:1: remark: Function Name: _ZN3dab1kILi1EEEvv [-Rpass-analysis=kernel-resource-usage]",
        "a.hip:1:1: remark:     VGPRs: 96 [-Rpass-analysis=kernel-resource-usage]",
        "a.hip:1:1: remark:     ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]",
        "a.hip:9:1: remark: Function Name: _ZN3dab1kILi2EEEvv [-Rpass-analysis=kernel-resource-usage]",
        "a.hip:9:1: remark:     ScratchSize [bytes/lane]: 528 [-Rpass-analysis=kernel-resource-usage]",
    ])
    assert scratch_kernels(log) == [("_ZN3dab1kILi2EEEvv", 528)]
