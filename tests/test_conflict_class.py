"""The drop-in returns the reference's own Conflict objects when the reference package
(semmerge) is importable, and this package's restatement (same fields) otherwise.  The
reference package is stood in by a module registered under its name, so the check
needs neither /root/reference nor a GPU."""
import sys
import types

import numpy as np

from semantic_merge_amd import materialize
from semantic_merge_amd.conflict import Conflict
from semantic_merge_amd.ops import Op, Target


def _ren(i, name):
    return Op(id=f"{i:08d}-op", schemaVersion=1, type="renameSymbol",
              target=Target(symbolId="sym-1", addressId=f"addr-{i}"),
              params={"newName": name}, guards={}, effects={}, provenance={"ts": i})


def test_restatement_without_reference(monkeypatch):
    monkeypatch.setattr(materialize, "_REF_DR", None)
    monkeypatch.setitem(sys.modules, "semmerge", None)   # import fails
    ops = [_ren(1, "a"), _ren(2, "b")]
    (c,) = materialize.materialize_conflicts(ops, np.array([[0, 1]]))
    assert isinstance(c, Conflict) and c.category == "DivergentRename"
    assert c.id == "conf-00000001-00000002" and c.opA == ops[0].to_dict()


def test_reference_factory_when_importable(monkeypatch):
    class RefConflict:  # the reference's class, as the stand-in package provides it
        def __init__(self, a, b):
            self.pair = (a.id, b.id)

    pkg = types.ModuleType("semmerge")
    mod = types.ModuleType("semmerge.conflict")
    mod.conflict_divergent_rename = lambda a, b: RefConflict(a, b)
    pkg.conflict = mod
    monkeypatch.setitem(sys.modules, "semmerge", pkg)
    monkeypatch.setitem(sys.modules, "semmerge.conflict", mod)
    monkeypatch.setattr(materialize, "_REF_DR", None)
    ops = [_ren(1, "a"), _ren(2, "b")]
    (c,) = materialize.materialize_conflicts(ops, np.array([[0, 1]]))
    assert isinstance(c, RefConflict) and c.pair == (ops[0].id, ops[1].id)
    monkeypatch.setattr(materialize, "_REF_DR", None)
