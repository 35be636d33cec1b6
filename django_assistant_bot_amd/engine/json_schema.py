"""JSON-Schema-constrained decoding: schema -> byte NFA for the native ``SchemaAutomaton``.

SURVEY.md 7.1 #4 asks for schema-constrained decoding so the reference's JSON steps (classify,
choose-known-question: /root/reference/assistant/bot/services/context_service/steps/classify.py:41-45,
choose_known_question.py:45-50, which retry until the answer has the right keys and types) succeed
in one generation.  A schema is compiled to a regular language over bytes:

  * objects emit their properties in schema order (``required`` lists the ones emitted; without it
    all are), no additional keys;
  * ``string`` (optional ``maxLength``), ``integer`` / ``number`` (an integer ``minimum`` ..
    ``maximum`` range of <= 256 values becomes an enumeration), ``boolean``, ``null``, ``enum`` /
    ``const`` of any JSON values, ``array`` (``items``, ``minItems``, ``maxItems``), ``anyOf`` /
    ``oneOf`` and type lists (alternatives);
  * whitespace between tokens is allowed up to ``max_ws`` bytes (tokenizers emit " value" tokens).

The NFA (Thompson construction) goes to C++ as edge lists; determinisation, the token-trie walk
and the per-state mask cache are native (csrc/runtime/json_grammar.cpp).  Recursive schemas
(``$ref``) are not regular and are refused.
"""
from __future__ import annotations

import json
import threading

from ..ops._lib import native

class SchemaError(ValueError):
    """A JSON Schema the constrained decoder cannot compile (a client error: /dialog/ answers 400)."""


_WS = [(0x09, 0x0A), (0x0D, 0x0D), (0x20, 0x20)]
_DIGIT = [(0x30, 0x39)]
_HEX = [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66)]
_STR_ASCII = [(0x20, 0x21), (0x23, 0x5B), (0x5D, 0x7F)]  # printable ASCII but '"' and '\\'


class _Nfa:
    def __init__(self):
        self.n = 0
        self.edges: list[list[int]] = []
        self.eps: list[list[int]] = []

    def state(self) -> int:
        self.n += 1
        if self.n > 200_000:
            raise SchemaError("schema too large for the constrained decoder")
        return self.n - 1

    # every builder returns a fragment (start, end)
    def cls(self, ranges):
        s, e = self.state(), self.state()
        for lo, hi in ranges:
            self.edges.append([s, lo, hi, e])
        return s, e

    def lit(self, b: bytes):
        s = cur = self.state()
        for c in b:
            nxt = self.state()
            self.edges.append([cur, c, c, nxt])
            cur = nxt
        return s, cur

    def seq(self, *frags):
        frags = [f for f in frags if f is not None]
        if not frags:
            s = self.state()
            return s, s
        for (_, e), (s2, _) in zip(frags, frags[1:]):
            self.eps.append([e, s2])
        return frags[0][0], frags[-1][1]

    def alt(self, *frags):
        s, e = self.state(), self.state()
        for fs, fe in frags:
            self.eps.append([s, fs])
            self.eps.append([fe, e])
        return s, e

    def opt(self, frag):
        s, e = frag
        self.eps.append([s, e])
        return frag

    def star(self, frag):
        s, e = self.state(), self.state()
        fs, fe = frag
        self.eps += [[s, fs], [fe, fs], [s, e], [fe, e]]
        return s, e


class _Compiler:
    def __init__(self, max_ws: int):
        self.a = _Nfa()
        self.max_ws = max_ws

    def ws(self):
        a = self.a
        return a.seq(*[a.opt(a.cls(_WS)) for _ in range(self.max_ws)])

    def string(self, max_len=None):
        a = self.a

        def char():  # one code point: printable ASCII but '"' / '\\', a UTF-8 sequence, or an escape
            esc = a.seq(a.lit(b"\\"), a.alt(a.cls([(ord(c), ord(c)) for c in '"\\/bfnrt']),
                                            a.seq(a.lit(b"u"), *[a.cls(_HEX) for _ in range(4)])))
            cont = lambda: a.cls([(0x80, 0xBF)])  # noqa: E731
            return a.alt(a.cls(_STR_ASCII), a.seq(a.cls([(0xC2, 0xDF)]), cont()),
                         a.seq(a.cls([(0xE0, 0xEF)]), cont(), cont()),
                         a.seq(a.cls([(0xF0, 0xF4)]), cont(), cont(), cont()), esc)

        if max_len is None:
            body = a.star(char())
        else:
            body = a.seq(*[a.opt(char()) for _ in range(int(max_len))])
        return a.seq(a.lit(b'"'), body, a.lit(b'"'))

    def integer(self):
        a = self.a
        return a.seq(a.opt(a.lit(b"-")), a.alt(a.lit(b"0"), a.seq(a.cls([(0x31, 0x39)]),
                                                                  *[a.opt(a.cls(_DIGIT)) for _ in range(15)])))

    def number(self):
        a = self.a
        frac = a.opt(a.seq(a.lit(b"."), a.cls(_DIGIT), *[a.opt(a.cls(_DIGIT)) for _ in range(15)]))
        exp = a.opt(a.seq(a.cls([(0x45, 0x45), (0x65, 0x65)]), a.opt(a.cls([(0x2B, 0x2B), (0x2D, 0x2D)])),
                          a.cls(_DIGIT), a.opt(a.cls(_DIGIT)), a.opt(a.cls(_DIGIT))))
        return a.seq(self.integer(), frac, exp)

    def literals(self, values):
        a = self.a
        return a.alt(*[a.lit(json.dumps(v, ensure_ascii=False).encode()) for v in values])

    def value(self, sch):
        a = self.a
        if sch is True or sch == {}:
            raise SchemaError("unconstrained sub-schemas are not supported (give a type)")
        if "$ref" in sch:
            raise SchemaError("recursive schemas ($ref) are not supported")
        if "enum" in sch:
            return self.literals(sch["enum"])
        if "const" in sch:
            return self.literals([sch["const"]])
        for k in ("anyOf", "oneOf"):
            if k in sch:
                return a.alt(*[self.value(s) for s in sch[k]])
        t = sch.get("type")
        if isinstance(t, list):
            return a.alt(*[self.value({**sch, "type": x}) for x in t])
        if t == "string":
            return self.string(sch.get("maxLength"))
        if t in ("integer", "number"):
            lo, hi = sch.get("minimum"), sch.get("maximum")
            if t == "integer" and lo is not None and hi is not None and 0 <= hi - lo < 256:
                return self.literals(list(range(int(lo), int(hi) + 1)))
            return self.integer() if t == "integer" else self.number()
        if t == "boolean":
            return self.literals([True, False])
        if t == "null":
            return a.lit(b"null")
        if t == "array":
            items = sch.get("items")
            if not isinstance(items, dict):
                raise SchemaError("arrays need an 'items' schema")
            lo = int(sch.get("minItems", 0))
            hi = sch.get("maxItems")
            sep = lambda: a.seq(self.ws(), a.lit(b","), self.ws(), self.value(items))  # noqa: E731
            if hi is None:
                rest = a.star(sep())
                tail = a.seq(*[sep() for _ in range(max(lo - 1, 0))], rest)
            else:
                hi = int(hi)
                if hi < max(lo, 1):
                    return a.seq(a.lit(b"["), self.ws(), a.lit(b"]"))
                tail = a.seq(*[sep() for _ in range(max(lo - 1, 0))],
                             *[a.opt(sep()) for _ in range(hi - max(lo, 1))])
            body = a.seq(self.value(items), tail)
            if lo == 0:
                body = a.opt(body)
            return a.seq(a.lit(b"["), self.ws(), body, self.ws(), a.lit(b"]"))
        if t == "object" or "properties" in sch:
            props = sch.get("properties", {})
            req = sch.get("required")
            keys = [k for k in props if req is None or k in req]
            parts = [a.lit(b"{"), self.ws()]
            for i, k in enumerate(keys):
                if i:
                    parts += [self.ws(), a.lit(b","), self.ws()]
                parts += [a.lit(json.dumps(k, ensure_ascii=False).encode()), self.ws(), a.lit(b":"), self.ws(),
                          self.value(props[k])]
            parts += [self.ws(), a.lit(b"}")]
            return a.seq(*parts)
        raise SchemaError(f"unsupported schema: {sch!r}")


def compile_schema(schema, max_ws: int = 4):
    """-> (n_states, start, accept, edges, eps) of the schema's byte NFA (leading whitespace
    allowed, nothing after the closing bracket).  Every malformed or unsupported schema raises
    ``SchemaError``."""
    try:
        if isinstance(schema, (str, bytes)):
            schema = json.loads(schema)
        if not isinstance(schema, dict):
            raise SchemaError("a decoding schema must be a JSON object")
        t = schema.get("type")
        if t not in ("object", "array") and "properties" not in schema:
            raise SchemaError("the top level of a decoding schema must be an object or an array")
        c = _Compiler(max_ws)
        s, e = c.a.seq(c.ws(), c.value(schema))
    except SchemaError:
        raise
    except (ValueError, TypeError, AttributeError, KeyError) as exc:  # malformed JSON / schema values
        raise SchemaError(f"invalid JSON schema: {exc}") from exc
    return c.a.n, s, [e], c.a.edges, c.a.eps


def schema_key(schema) -> str:
    """Canonical text of a schema (key order kept: properties are emitted in schema order)."""
    return json.dumps(json.loads(schema) if isinstance(schema, (str, bytes)) else schema, ensure_ascii=False,
                      separators=(",", ":"))


_lock = threading.Lock()


def automaton_for(tokenizer, eos_ids, schema):
    """The (cached per tokenizer and schema) native automaton of ``schema``."""
    from .json_constraint import vocab_for

    key = schema_key(schema)
    vocab = vocab_for(tokenizer, eos_ids)
    with _lock:
        cache = getattr(tokenizer, "_schema_automata", None)
        if cache is None:
            cache = tokenizer._schema_automata = {}
        a = cache.get(key)
        if a is None:
            if len(cache) >= 16:
                cache.clear()
            n, s, acc, edges, eps = compile_schema(key)
            a = cache[key] = native().SchemaAutomaton(vocab, n, s, acc, edges, eps)
        return a


def matcher_for(tokenizer, eos_ids, schema):
    return native().SchemaMatcher(automaton_for(tokenizer, eos_ids, schema))
