"""Port of /root/reference/tests/test_utils.py:6-36 (the 23 ``has_cjk_characters`` cases).

The reference file does not parse: line 23 nests ASCII double quotes inside a double-quoted
literal (``"...与"Dixy"订单..."``).  Here that case is written with single outer quotes so the
inner ``"Dixy"`` is part of the string, which is what the case intends.
"""
import pytest

from assistant.utils.language import has_cjk_characters


@pytest.mark.parametrize("input_str,expected", [
    # positive cases
    ("漢字", True),  # Chinese
    ("こんにちは", True),  # hiragana
    ("カタカナ", True),  # katakana
    ("한글", True),  # hangul
    ("Hello 你好", True),  # Latin + Chinese
    ("ＨＥＬＬＯ", True),  # full-width forms (FF00-FFEF)
    ("一", True),  # first CJK Unified Ideograph
    ("鿿", True),  # last CJK Unified Ideograph
    ("㐀", True),  # first of CJK Extension A
    ("䶿", True),  # last of CJK Extension A
    # real bot outputs
    ("Привет!很高兴见到你。有什么可以帮助你的吗？", True),
    ("Я可以帮助您处理订单相关的问题，包括查询订单状态、取消订单或向骑手留言。请告诉我您的具体需求。", True),
    ("Хорошо,谢谢 за интерес! Как я могу вам помочь?", True),
    ("Спасибо за ваш вопрос! Я хорошо,谢谢. Как я могу вам помочь с вашим заказом?", True),
    ('您好！我目前的任务是帮助您处理与"Dixy"订单相关的问题，具体包括以下几种方式：', True),
    ("Вы можете问我 о статусе вашего заказа", True),
    # negative cases
    ("", False),
    ("Hello World", False),
    ("Привет", False),
    ("12345!@#", False),
    ("αβγδε", False),
    ("😀🎉", False),
    ("Привет! 👋 Я ваш новый виртуальный ассистент", False),
])
def test_has_cjk_characters(input_str, expected):
    assert has_cjk_characters(input_str) == expected
