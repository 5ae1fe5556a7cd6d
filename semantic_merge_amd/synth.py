"""Synthetic lift-shaped op logs.

The reference's producer is the TypeScript worker's ``lift`` (workers/ts/src/lift.ts:11-66):
one op per diff with a ``crypto.randomUUID()`` id, ``new Date().toISOString()``
timestamp (non-decreasing, millisecond resolution), and per-type params.  This
module generates logs of that shape deterministically from a seed:

* :func:`lift_soa` builds the device SoA directly with numpy (used at 100M ops,
  where Python ``Op`` objects would need ~160 GB);
* :func:`lift_op_dicts` renders the *same* logs as ``Op.to_dict()``-shaped dicts
  (feasible up to a few million ops) so the reference itself can compose them.

``tests/test_synth.py`` checks that marshalling the dicts reproduces the SoA.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from .marshal import SoA, TS_ISO, ID_UUID
from .ops import KIND_RANK

TYPE_MIX: Tuple[Tuple[str, float], ...] = (
    ("renameSymbol", 0.35),
    ("moveDecl", 0.25),
    ("editStmtBlock", 0.25),
    ("addDecl", 0.05),
    ("deleteDecl", 0.05),
    ("modifyImport", 0.05),
)
ADVERSARIAL_MIX: Tuple[Tuple[str, float], ...] = (
    ("renameSymbol", 0.60),
    ("moveDecl", 0.15),
    ("editStmtBlock", 0.15),
    ("addDecl", 0.04),
    ("deleteDecl", 0.03),
    ("modifyImport", 0.03),
)
BASE_MS = 1763078400000  # 2025-11-14T00:00:00.000Z
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


@dataclass
class LiftSpec:
    n_total: int
    n_sym: int
    seed: int
    ops_per_ms: int = 64
    divergent: float = 0.01
    names: int = 50
    n_files: int = 1000
    mix: Tuple[Tuple[str, float], ...] = TYPE_MIX
    # fraction of the symbol range each branch renames; 1.0 = both branches use all symbols
    rename_overlap: Optional[float] = None
    # robustness variant: each branch log randomly permuted (timestamps no longer monotone)
    shuffle: bool = False


CONFIGS: Dict[str, LiftSpec] = {
    # 1M ops, 10k symbols, seed 7
    "c2": LiftSpec(1_000_000, 10_000, 7),
    # config 3: 100M ops over 1M symbols, seed 11
    "c3": LiftSpec(100_000_000, 1_000_000, 11),
    # config 5: 20M ops, >= 60% renames, 30% of symbols renamed on both sides,
    # >= 64 renames per symbol, 4096 ops per ms (dense ties), seed 17
    "c5": LiftSpec(20_000_000, 100_000, 17, ops_per_ms=4096, mix=ADVERSARIAL_MIX,
                   rename_overlap=0.30),
    # robustness variants of configs 2 and 3: each branch log randomly permuted, which
    # forces the generic (radix) plan; reported, not targeted
    "c2s": LiftSpec(1_000_000, 10_000, 7, shuffle=True),
    "c3s": LiftSpec(100_000_000, 1_000_000, 11, shuffle=True),
}


def splitmix64(x: np.ndarray) -> np.ndarray:
    z = (x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & M64
    with np.errstate(over="ignore"):
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return z ^ (z >> np.uint64(31))


def _civil(days: np.ndarray):
    """Proleptic Gregorian (y, m, d) from days since 1970-01-01 (H. Hinnant)."""
    z = days + 719468
    era = np.floor_divide(z, 146097)
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = np.where(mp < 10, mp + 3, mp - 9)
    return y + (m <= 2), m, d


def iso_keys_from_ms(ms: np.ndarray) -> np.ndarray:
    """Vectorised marshal.iso_key of ``toISOString()`` renderings of ``ms``."""
    ms = ms.astype(np.int64)
    days = np.floor_divide(ms, 86_400_000)
    rem = ms - days * 86_400_000
    y, mo, d = _civil(days)
    hh = rem // 3_600_000
    mi = (rem // 60_000) % 60
    ss = (rem // 1000) % 60
    fff = rem % 1000
    whole = ((((y * 100 + mo) * 100 + d) * 100 + hh) * 100 + mi) * 100 + ss
    return (whole * 2000 + 2 * fff).astype(np.uint64)


def iso_string(ms: int) -> str:
    t = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc) + _dt.timedelta(milliseconds=int(ms))
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond // 1000:03d}Z"


@dataclass
class LiftLogs:
    """Generator state shared by the SoA and the dict renderings."""

    spec: LiftSpec
    n_a: int
    n_b: int
    type_idx: np.ndarray   # index into spec.mix
    sym: np.ndarray        # i64 symbol index
    ts_ms: np.ndarray      # i64
    id_hi: np.ndarray      # u64
    id_lo: np.ndarray      # u64
    name: np.ndarray       # i32 newName index (branch-local)
    dst: np.ndarray        # i32 move destination file

    @property
    def n(self) -> int:
        return self.n_a + self.n_b


def lift_logs(spec: LiftSpec) -> LiftLogs:
    rng = np.random.default_rng(spec.seed)
    n_a = spec.n_total // 2
    n_b = spec.n_total - n_a
    probs = np.array([p for _, p in spec.mix], dtype=np.float64)
    probs /= probs.sum()
    ren = [t for t, _ in spec.mix].index("renameSymbol")
    parts = []
    for side, n_s in enumerate((n_a, n_b)):
        t = rng.choice(len(spec.mix), size=n_s, p=probs).astype(np.int8)
        sym = rng.integers(0, spec.n_sym, size=n_s, dtype=np.int64)
        if spec.rename_overlap is not None:
            # A renames symbols in [0, lo_hi), B in [1 - lo_hi, 1) of the range:
            # the overlap (rename_overlap of the symbols) is renamed on both sides.
            span = int(spec.n_sym * (1.0 + spec.rename_overlap) / 2.0)
            r = rng.integers(0, span, size=n_s, dtype=np.int64)
            r = r if side == 0 else r + (spec.n_sym - span)
            sym = np.where(t == ren, r, sym)
        bits = rng.integers(0, 0xFFFFFFFFFFFFFFFF, size=(n_s, 2), dtype=np.uint64,
                            endpoint=True)
        hi =(bits[:, 0] & ~np.uint64(0xF000)) | np.uint64(0x4000)          # version 4
        lo = (bits[:, 1] & ~np.uint64(0xC000000000000000)) | np.uint64(0x8000000000000000)
        name = rng.integers(0, spec.names, size=n_s, dtype=np.int32)
        dst = rng.integers(0, spec.n_files, size=n_s, dtype=np.int32)
        ts = BASE_MS + np.arange(n_s, dtype=np.int64) // spec.ops_per_ms
        parts.append((t, sym, ts, hi, lo, name, dst))
    (ta, sa, tsa, ha, la, na_, da), (tb, sb, tsb, hb, lb, nb_, db) = parts
    # Divergent renames: B op k re-targeted to A op k's symbol when both are renames.
    m = min(n_a, n_b)
    flip = rng.random(m) < spec.divergent
    sel = flip & (ta[:m] == ren) & (tb[:m] == ren)
    sb = sb.copy()
    sb[:m][sel] = sa[:m][sel]
    if spec.shuffle:
        pa = rng.permutation(n_a)
        pb = rng.permutation(n_b)
        ta, sa, tsa, ha, la, na_, da = (x[pa] for x in (ta, sa, tsa, ha, la, na_, da))
        tb, sb, tsb, hb, lb, nb_, db = (x[pb] for x in (tb, sb, tsb, hb, lb, nb_, db))
    cat = np.concatenate
    return LiftLogs(spec, n_a, n_b, cat([ta, tb]), cat([sa, sb]), cat([tsa, tsb]),
                    cat([ha, hb]), cat([la, lb]), cat([na_, nb_]), cat([da, db]))


def lift_slice_soa(spec: LiftSpec, rank: int, world: int) -> Tuple[SoA, int, int]:
    """Rank's index slices of a merge of world x spec.n_total lift-shaped ops, generated
    without the rest of it (sharded benchmark: each rank loads its own slice).  Branch
    op k of the global logs has timestamp BASE_MS + k // ops_per_ms; rank r holds ops
    [r * n, (r + 1) * n) of each branch (n = n_total / 2), drawn from rng(seed, r);
    divergent renames pair A op k with B op k, so they stay inside one slice.
    Returns (slice SoA: A slice then B slice, global n_a, global n_b)."""
    if spec.shuffle or spec.rename_overlap is not None:
        raise ValueError("lift_slice_soa: plain lift-shaped specs only")
    n_s = spec.n_total // 2
    start = rank * n_s
    rng = np.random.default_rng([spec.seed, rank])
    probs = np.array([p for _, p in spec.mix], dtype=np.float64)
    probs /= probs.sum()
    ren = [t for t, _ in spec.mix].index("renameSymbol")
    parts = []
    for side in range(2):
        t = rng.choice(len(spec.mix), size=n_s, p=probs).astype(np.int8)
        sym = rng.integers(0, spec.n_sym, size=n_s, dtype=np.int64)
        bits = rng.integers(0, 0xFFFFFFFFFFFFFFFF, size=(n_s, 2), dtype=np.uint64, endpoint=True)
        hi = (bits[:, 0] & ~np.uint64(0xF000)) | np.uint64(0x4000)
        lo = (bits[:, 1] & ~np.uint64(0xC000000000000000)) | np.uint64(0x8000000000000000)
        name = rng.integers(0, spec.names, size=n_s, dtype=np.int32)
        dst = rng.integers(0, spec.n_files, size=n_s, dtype=np.int32)
        ts = BASE_MS + (start + np.arange(n_s, dtype=np.int64)) // spec.ops_per_ms
        parts.append([t, sym, ts, hi, lo, name, dst])
    (ta, sa), (tb, sb) = parts[0][:2], parts[1][:2]
    flip = rng.random(n_s) < spec.divergent
    sel = flip & (ta == ren) & (tb == ren)
    sb[sel] = sa[sel]
    cat = np.concatenate
    logs = LiftLogs(spec, n_s, n_s, *[cat([parts[0][i], parts[1][i]]) for i in range(7)])
    soa = lift_soa(logs)
    # move addresses are one string per global op index (like lift_soa on the whole merge)
    is_mv = soa.kind == KIND_RANK["moveDecl"]
    gidx = np.concatenate([start + np.arange(n_s), world * n_s + start + np.arange(n_s)])
    soa.v0[is_mv] = (2 * spec.names + spec.n_files + gidx[is_mv]).astype(np.int32)
    return soa, world * n_s, world * n_s


def _kind_table(spec: LiftSpec) -> np.ndarray:
    return np.array([KIND_RANK[t] for t, _ in spec.mix], dtype=np.uint8)


def lift_soa(logs: LiftLogs) -> SoA:
    """Device SoA of the logs.  String ids (implicit table):
    [0, 2*names) rename names (A then B), then n_files move files, then one
    newAddress per op index."""
    spec = logs.spec
    kind = _kind_table(spec)[logs.type_idx]
    side = (np.arange(logs.n) >= logs.n_a).astype(np.int32)
    v0 = np.full(logs.n, -1, np.int32)
    v1 = np.full(logs.n, -1, np.int32)
    is_ren = kind == KIND_RANK["renameSymbol"]
    is_mv = kind == KIND_RANK["moveDecl"]
    name_id = side * spec.names + logs.name
    v0[is_ren] = name_id[is_ren]
    v1[is_ren] = name_id[is_ren]
    base_addr = 2 * spec.names + spec.n_files
    v0[is_mv] = (base_addr + np.arange(logs.n, dtype=np.int64))[is_mv].astype(np.int32)
    v1[is_mv] = (2 * spec.names + logs.dst)[is_mv]
    return SoA(logs.n_a, logs.n_b, kind, iso_keys_from_ms(logs.ts_ms), logs.id_hi.copy(),
               logs.id_lo.copy(), logs.sym.astype(np.uint32), v0, v1, spec.n_sym, [],
               TS_ISO, ID_UUID)


def _uuid(hi: int, lo: int) -> str:
    h = f"{hi:016x}{lo:016x}"
    return f"{h[0:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}"


def lift_op_dicts(logs: LiftLogs) -> Tuple[List[dict], List[dict]]:
    """Render the logs as Op.to_dict()-shaped dicts shaped like lift.ts output."""
    spec = logs.spec
    types = [t for t, _ in spec.mix]
    symhex = splitmix64(np.arange(spec.n_sym, dtype=np.uint64))
    ts_cache: Dict[int, str] = {}
    out: List[dict] = []
    tl = logs.type_idx.tolist()
    syl = logs.sym.tolist()
    tsl = logs.ts_ms.tolist()
    hil = logs.id_hi.tolist()
    lol = logs.id_lo.tolist()
    nml = logs.name.tolist()
    dsl = logs.dst.tolist()
    for k in range(logs.n):
        side = "A" if k < logs.n_a else "B"
        s = syl[k]
        typ = types[tl[k]]
        ts = ts_cache.get(tsl[k])
        if ts is None:
            ts = ts_cache[tsl[k]] = iso_string(tsl[k])
        sid = f"{int(symhex[s]):016x}"
        f0 = f"src/f{s % spec.n_files}.ts"
        addr0 = f"{f0}::s{s}::0"
        prov = {"rev": "base", "timestamp": ts}
        if typ == "renameSymbol":
            new = f"{side}_name{nml[k]}"
            params = {"oldName": f"s{s}", "newName": new, "file": f0}
            guards = {"exists": True, "addressMatch": addr0}
            effects = {"summary": f"rename s{s}→{new}"}
        elif typ == "moveDecl":
            f1 = f"src/m{dsl[k]}.ts"
            new_addr = f"{f1}::s{s}::{k}"
            params = {"oldAddress": addr0, "newAddress": new_addr, "oldFile": f0, "newFile": f1}
            guards = {"exists": True, "addressMatch": addr0}
            effects = {"summary": f"move {addr0}→{new_addr}"}
        else:
            params = {"file": f0}
            guards = {}
            effects = {"summary": typ}
        out.append({
            "id": _uuid(hil[k], lol[k]),
            "schemaVersion": 1,
            "type": typ,
            "target": {"symbolId": sid, "addressId": addr0},
            "params": params,
            "guards": guards,
            "effects": effects,
            "provenance": prov,
        })
    return out[: logs.n_a], out[logs.n_a:]


def rga_batch(n_ops: int, n_lists: int, seed: int, values_per_list: int = 150,
              anchors_per_list: int = 20, authors: int = 4):
    """SURVEY §8(d) config 4 shape: RGA events over many independent lists
    (insert 0.7, delete 0.2, move 0.1), values from 150 per list, anchors from 20
    per list, t uniform in [0, 2^40), 4 authors, uuid4 opids.  Returns the
    ``RgaBatch`` image directly (order-preserving ranks; strings not materialised)."""
    from .crdt import RgaBatch
    rng = np.random.default_rng(seed)
    lid = rng.integers(0, n_lists, size=n_ops, dtype=np.int64)
    op = rng.choice(3, size=n_ops, p=[0.7, 0.1, 0.2]).astype(np.uint8)  # insert, move, delete
    val = lid * values_per_list + rng.integers(0, values_per_list, size=n_ops)
    anchor = rng.integers(0, anchors_per_list, size=n_ops, dtype=np.int64)
    t = rng.integers(0, 1 << 40, size=n_ops, dtype=np.int64)
    author = rng.integers(0, authors, size=n_ops, dtype=np.int64)
    bits = rng.integers(0, 0xFFFFFFFFFFFFFFFF, size=(n_ops, 2), dtype=np.uint64, endpoint=True)
    hi = (bits[:, 0] & ~np.uint64(0xF000)) | np.uint64(0x4000)
    lo = (bits[:, 1] & ~np.uint64(0xC000000000000000)) | np.uint64(0x8000000000000000)
    # value ids interned densely in first-seen order, like marshal_streams
    _, first, inv = np.unique(val, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    return RgaBatch(n_lists, lid.astype(np.uint32), op, rank[inv].astype(np.uint32),
                    anchor.astype(np.uint32), t, author.astype(np.uint32), hi, lo, [])
