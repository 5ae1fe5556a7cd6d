"""newName equality classes follow Python ``==`` (the ``!=`` test of
/root/reference/semmerge/compose.py:66), including the container corner cases."""
from collections import OrderedDict

import pytest

from semantic_merge_amd.marshal import _EqClasses, eq_key


def _same(a, b):
    eq = _EqClasses()
    return eq(a) == eq(b)


@pytest.mark.parametrize("a,b", [
    (bytearray(b"ab"), bytearray(b"ab")),
    (bytearray(b"ab"), b"ab"),
    ({1, 2}, frozenset({2, 1})),
    (1, 1.0),
    (True, 1),
    ([1, {"x": 2}], [1, {"x": 2}]),
    ({"a": 1, "b": 2}, {"b": 2, "a": 1}),
])
def test_equal_values_share_a_class(a, b):
    assert a == b
    assert _same(a, b)


@pytest.mark.parametrize("a,b", [
    (bytearray(b"ab"), bytearray(b"ba")),
    ([1], (1,)),
    ({1}, {2}),
    ("1", 1),
])
def test_unequal_values_differ(a, b):
    assert a != b
    assert not _same(a, b)


def test_nan_is_never_equal():
    eq = _EqClasses()
    x = float("nan")
    assert eq(x) != eq(x)


def test_ordered_dict_is_rejected():
    with pytest.raises(TypeError):
        eq_key(OrderedDict(a=1))
