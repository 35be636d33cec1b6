"""The native host runtime (KV block manager, tokenizer, retrieval aggregation, roctx shim) built and
run under AddressSanitizer+UBSan and ThreadSanitizer (host code only)."""
import shutil

import pytest

from django_assistant_bot_amd import build

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_runtime_selftest_under_sanitizer(kind, tmp_path):
    rc, log = build.selftest(kind, tmp_path)
    if rc and "cannot find" in log and "libtsan" in log:
        pytest.skip("sanitizer runtime not installed")
    assert rc == 0, log[-4000:]
    assert "runtime selftest ok" in log
