"""The JSON container skipper (native/src/json.cpp): the AVX2 block classifier (escape runs,
string interiors by prefix XOR, bracket popcounts) agrees with the scalar walk on JSON text,
whatever the block boundaries, escapes, nesting and string contents."""
import json
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from nanogpu import _native as N

_leaf = st.one_of(st.none(), st.booleans(), st.integers(-10 ** 6, 10 ** 6),
                  st.text(alphabet=st.sampled_from('ab"\\\\{}[],: \n\t\x01é '), max_size=12))
_doc = st.recursive(_leaf, lambda ch: st.one_of(st.lists(ch, max_size=5), st.dictionaries(st.text(max_size=6), ch, max_size=5)),
                    max_leaves=40)


@settings(max_examples=400, deadline=None)
@given(doc=st.one_of(st.lists(_doc), st.dictionaries(st.text(max_size=8), _doc)), pad=st.integers(0, 70),
       tail=st.sampled_from(["", ",", "]}", ' ,"x":1}', "\n"]), ascii_only=st.booleans())
def test_avx2_skip_agrees_with_the_scalar_walk(doc, pad, tail, ascii_only):
    text = (json.dumps(doc, ensure_ascii=ascii_only, separators=(",", ":") if pad % 2 else None)).encode()
    # a leading padding string inside the container shifts every byte across the 64-byte blocks
    if isinstance(doc, list):
        text = b'["' + b"\\\\" * (pad // 2) + b"q" * (pad % 2) + b'",' + text[1:] if text != b"[]" else text
    src = text + tail.encode()
    want = N.json_skip(src, True)
    assert want == len(text)
    assert N.json_skip(src, False) == want


@settings(max_examples=300, deadline=None)
@given(st.binary(min_size=1, max_size=300))
def test_avx2_skip_never_accepts_what_the_scalar_walk_refuses_or_ends_elsewhere(raw):
    src = b"[" + raw
    a, s = N.json_skip(src, False), N.json_skip(src, True)
    # on bytes that are not JSON the AVX2 walk may refuse a stray backslash the scalar walk
    # steps over; where both accept, they end at the same byte
    if a != -1:
        assert a == s


def test_the_avx2_walk_is_the_one_in_use_where_the_host_has_avx2():
    flags = open("/proc/cpuinfo").read().split()
    assert N.json_skip_uses_avx2() == ("avx2" in flags and "pclmulqdq" in flags)


def test_long_documents_cross_many_blocks():
    rng = random.Random(5)
    for n in (1, 63, 64, 65, 127, 128, 129, 1000, 5000):
        names = [f"node-{i:05d}" + ("\\\"x" if rng.random() < 0.1 else "") for i in range(n)]
        src = ("[" + ",".join(f'"{x}"' for x in names) + "]").encode()
        assert N.json_skip(src, False) == N.json_skip(src, True) == len(src)
        deep = b"[" * 64 + b"]" * 64
        assert N.json_skip(deep, False) == N.json_skip(deep, True) == len(deep)
        assert N.json_skip(b"[" * 65 + b"]" * 65, False) == N.json_skip(b"[" * 65 + b"]" * 65, True) == -1
    assert N.json_skip(b'["a\x01"]', False) == N.json_skip(b'["a\x01"]', True) == -1
    assert N.json_skip(b'["unterminated]', False) == -1
