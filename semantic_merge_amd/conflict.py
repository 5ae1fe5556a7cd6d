"""Conflict payloads emitted by compose.

Restates the record of ``semmerge/conflict.py:10-31`` and the only category the
reference composer emits, ``DivergentRename`` (``conflict.py:34-49``).  The
device side only reports the pair of source indices; the payload is built here
from the *uncloned* input ops, exactly as the reference does.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List


@dataclass
class Conflict:
    id: str
    category: str
    symbolId: str
    addressIds: Dict[str, Any]
    opA: Dict[str, Any]
    opB: Dict[str, Any]
    minimalSlice: Dict[str, Any]
    suggestions: List[Dict[str, Any]]

    def to_dict(self) -> Dict[str, Any]:
        return {
            "id": self.id,
            "category": self.category,
            "symbolId": self.symbolId,
            "addressIds": self.addressIds,
            "opA": self.opA,
            "opB": self.opB,
            "minimalSlice": self.minimalSlice,
            "suggestions": self.suggestions,
        }


def divergent_rename(op_a, op_b) -> Conflict:
    """Payload for two same-symbol renames with different names (conflict.py:34-49)."""
    name_a = op_a.params.get("newName")
    name_b = op_b.params.get("newName")
    return Conflict(
        id=f"conf-{op_a.id[:8]}-{op_b.id[:8]}",
        category="DivergentRename",
        symbolId=op_a.target.symbolId,
        addressIds={"A": op_a.target.addressId, "B": op_b.target.addressId, "base": None},
        opA=op_a.to_dict(),
        opB=op_b.to_dict(),
        minimalSlice={"path": "", "start": 0, "end": 0, "code": ""},
        suggestions=[
            {"id": "keepA", "label": f"Rename to {name_a}", "ops": [op_a.id]},
            {"id": "keepB", "label": f"Rename to {name_b}", "ops": [op_b.id]},
        ],
    )
