"""Drop-in ``compose_oplogs`` (semmerge/compose.py:11) running on the MI355X.

Same signature, same result objects, same exceptions for malformed ops:

    compose_oplogs(delta_a: List[Op], delta_b: List[Op]) -> (List[Op], List[Conflict])

Inputs are never mutated; outputs are fresh ``Op`` objects built with
``type(op)`` / ``type(op.target)`` (so reference ``Op`` instances round-trip),
and conflicts are built from the uncloned inputs, as in the reference.  Marshal and
materialise run in the native host module (csrc/smx_host.cpp), the merge on the GPU.  To wire
it into the reference CLI, rebind the module attribute the CLI looks up
(``semmerge.__main__.compose_oplogs``).
"""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple

from ._lib import dropin_session
from .marshal import marshal_native
from .materialize import materialize_conflicts, materialize_ops_native


def compose_oplogs(delta_a: Sequence[Any], delta_b: Sequence[Any]) -> Tuple[List[Any], List[Any]]:
    """Compose two op logs into one deterministic sequence plus DivergentRename conflicts."""
    ops_a = list(delta_a)
    ops_b = list(delta_b)
    with dropin_session() as sess:
        # marshalled straight into the session's pinned staging columns; the results are
        # views of its staging area too, materialised while the session is held
        soa = marshal_native(ops_a, ops_b, sess.staging(len(ops_a) + len(ops_b)))
        order, addr, file, ctx, pairs = sess.compose(soa, copy=False)
        ops = ops_a + ops_b
        out = materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx)
        conflicts = materialize_conflicts(ops, pairs)
    return out, conflicts
