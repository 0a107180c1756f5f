"""Host-side callbacks of the topk_rmv behaviour mirror (no GPU):
is_operation/1, is_replicate_tagged/1, can_compact/2, compact_ops/2,
require_state_downstream/1 (src/antidote_ccrdt_topk_rmv.erl:166-226).  The
reference has no test for these; expectations follow the source
(parity unpinned)."""
import pytest

from antidote_ccrdt_amd import antidote_ccrdt_topk_rmv as trmv

A = "dc1"


def add(tag, i, s, ts):
    return (tag, (i, s, (A, ts)))


def test_is_operation_and_tags():
    assert trmv.is_operation(("add", (1, 2)))
    assert trmv.is_operation(("rmv", 1))
    assert not trmv.is_operation(("add", ("a", 2)))
    assert not trmv.is_operation(("rmv", "a"))
    assert not trmv.is_operation(("inc", 1))
    assert trmv.is_replicate_tagged(add("add_r", 1, 1, 1))
    assert trmv.is_replicate_tagged(("rmv_r", (1, {})))
    assert not trmv.is_replicate_tagged(add("add", 1, 1, 1))
    assert trmv.require_state_downstream(("add", (1, 2)))


def test_compact_add_add_retags_lower_score():  # Q20: never merged
    e1, e2 = add("add", 1, 5, 1), add("add", 1, 3, 2)
    assert trmv.can_compact(e1, e2)
    assert trmv.compact_ops(e1, e2) == (add("add", 1, 5, 1), add("add_r", 1, 3, 2))
    assert trmv.compact_ops(e2, e1) == (add("add_r", 1, 3, 2), add("add", 1, 5, 1))
    assert not trmv.can_compact(add("add", 1, 5, 1), add("add", 2, 5, 1))


def test_compact_add_r_add():
    e1, e2 = add("add_r", 1, 5, 1), add("add", 1, 5, 1)
    assert trmv.compact_ops(e1, e2) == (("noop",), e2)
    e3 = add("add", 1, 6, 1)
    assert trmv.compact_ops(e1, e3) == (e1, e3)


def test_compact_add_rmv():
    e1 = add("add", 1, 5, 4)
    assert trmv.can_compact(e1, ("rmv", (1, {A: 4})))
    assert not trmv.can_compact(e1, ("rmv", (1, {A: 3})))
    assert not trmv.can_compact(e1, ("rmv", (2, {A: 9})))
    assert not trmv.can_compact(e1, ("rmv", (1, {})))  # missing DC reads 0
    assert trmv.compact_ops(e1, ("rmv", (1, {A: 9}))) == (("noop",), ("rmv", (1, {A: 9})))
    e2 = add("add_r", 1, 5, 4)
    assert trmv.compact_ops(e2, ("rmv_r", (1, {A: 9}))) == (("noop",), ("rmv_r", (1, {A: 9})))
    with pytest.raises(trmv.FunctionClause):  # no {add, _}, {rmv_r, _} clause (:207-212)
        trmv.compact_ops(e1, ("rmv_r", (1, {A: 9})))


def test_compact_rmv_rmv_merges_clocks():
    e1, e2 = ("rmv_r", (1, {A: 3, "dc2": 7})), ("rmv_r", (1, {A: 5}))
    assert trmv.can_compact(e1, e2)
    assert trmv.compact_ops(e1, e2) == (("noop",), ("rmv_r", (1, {A: 5, "dc2": 7})))
    assert trmv.compact_ops(e1, ("rmv", (1, {})))[1][0] == "rmv"


def test_compact_ops_has_no_catch_all():  # Q21
    with pytest.raises(trmv.FunctionClause):
        trmv.compact_ops(("rmv", (1, {})), add("add", 1, 1, 1))
