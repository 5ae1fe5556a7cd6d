"""Op schema used at the compose boundary.

The reference's schema lives in ``semmerge/ops.py:31-103`` (``Target``, ``Op``,
``Op.to_dict`` key order, ``Op.from_dict`` coercions).  It must stay unchanged
for the drop-in to be transparent, so this module restates exactly the fields,
the ``to_dict`` key order and the ``from_dict`` coercions, and nothing else.
When the real ``semmerge`` package is importable, callers simply pass its
``Op`` instances: :func:`semantic_merge_amd.compose.compose_oplogs` only reads
attributes and rebuilds outputs with ``type(op)`` / ``type(op.target)``.
"""
from __future__ import annotations

import uuid
from dataclasses import dataclass
from typing import Any, Dict, Mapping, Optional

# Precedence table of the composer (semmerge/compose.py:130-149); unknown
# types rank 99 (compose.py:18).
PRECEDENCE: Dict[str, int] = {
    "moveDecl": 10,
    "renameSymbol": 11,
    "modifyImport": 12,
    "reorderImports": 13,
    "changeSignature": 20,
    "updateCall": 21,
    "addDecl": 30,
    "deleteDecl": 31,
    "extractMethod": 40,
    "inlineMethod": 41,
    "editStmtBlock": 50,
    "reorderParams": 51,
    "addParam": 52,
    "removeParam": 53,
    "moveFile": 60,
    "renameFile": 61,
    "modifyNamespace": 70,
}
UNKNOWN_PRECEDENCE = 99

# Dense device rank of each precedence value (order preserving): 0..17.
PREC_LEVELS = sorted(set(PRECEDENCE.values()) | {UNKNOWN_PRECEDENCE})
RANK_OF_PREC = {p: i for i, p in enumerate(PREC_LEVELS)}
KIND_RANK: Dict[str, int] = {t: RANK_OF_PREC[p] for t, p in PRECEDENCE.items()}
KIND_MOVE = KIND_RANK["moveDecl"]
KIND_RENAME = KIND_RANK["renameSymbol"]
KIND_UNKNOWN = RANK_OF_PREC[UNKNOWN_PRECEDENCE]
N_KINDS = len(PREC_LEVELS)


@dataclass
class Target:
    """Declaration an op acts on (ops.py:31-39)."""

    symbolId: str
    addressId: Optional[str] = None

    def to_dict(self) -> Dict[str, Any]:
        return {"symbolId": self.symbolId, "addressId": self.addressId}


@dataclass
class Op:
    """Semantic change record (ops.py:42-103)."""

    id: str
    schemaVersion: int
    type: str
    target: Target
    params: Dict[str, Any]
    guards: Dict[str, Any]
    effects: Dict[str, Any]
    provenance: Dict[str, Any]

    @staticmethod
    def new(op_type: str, target: Target, params=None, guards=None, effects=None,
            provenance=None) -> "Op":
        return Op(str(uuid.uuid4()), 1, op_type, target, params or {}, guards or {},
                  effects or {}, provenance or {})

    def to_dict(self) -> Dict[str, Any]:
        # Key order is part of the bit-exact JSON contract (ops.py:77-87).
        return {
            "id": self.id,
            "schemaVersion": self.schemaVersion,
            "type": self.type,
            "target": self.target.to_dict(),
            "params": self.params,
            "guards": self.guards,
            "effects": self.effects,
            "provenance": self.provenance,
        }

    @staticmethod
    def from_dict(data: Mapping[str, Any]) -> "Op":
        # Same coercions as ops.py:89-100.
        return Op(
            id=str(data["id"]),
            schemaVersion=int(data.get("schemaVersion", 1)),
            type=data["type"],
            target=Target(**data["target"]),
            params=dict(data.get("params", {})),
            guards=dict(data.get("guards", {})),
            effects=dict(data.get("effects", {})),
            provenance=dict(data.get("provenance", {})),
        )
