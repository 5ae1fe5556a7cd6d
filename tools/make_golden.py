"""Generate tests/golden/ by running the REFERENCE implementation in this container.

The reference (``/root/reference/semmerge``) is imported read-only with
``PYTHONDONTWRITEBYTECODE`` semantics and a json-backed stand-in for ``orjson``
(only ``OpLog.to_json/from_json`` use it, ops.py:112-118; compose, conflict and
crdt never do).  Nothing from the reference is copied: the committed fixtures are
inputs and the reference's outputs (JSON), plus sha256 digests for the large
synthetic configs.  The GPU box never reads /root/reference.

    python tools/make_golden.py [--big] [--only oplog|applier|big|e2e]

``--big`` also composes the 1M-op config 2 (~25 s of reference CPU time);
``--only big`` composes only that.  ``--only e2e`` records config 1 (the
reference's tests/e2e_rename_move_decl.sh scenario) end to end: base tree, both op
logs, and the tree the reference's compose_oplogs + apply_ops leave.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import random
import sys
import time
import types
import uuid

sys.dont_write_bytecode = True
REF = os.environ.get("SMX_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)


def _import_reference():
    stub = types.ModuleType("orjson")
    stub.dumps = lambda obj, *a, **k: json.dumps(obj).encode()
    stub.loads = lambda s, *a, **k: json.loads(s)
    sys.modules.setdefault("orjson", stub)
    sys.path.insert(0, REF)
    from semmerge import compose, crdt, ops  # noqa: E402
    return compose, crdt, ops


def dumps_line(obj) -> str:
    return json.dumps(obj, ensure_ascii=False, separators=(",", ":"))


def digest(dicts) -> str:
    h = hashlib.sha256()
    for d in dicts:
        h.update(dumps_line(d).encode("utf-8"))
        h.update(b"\n")
    return h.hexdigest()


# ---------------------------------------------------------------------------
# random edge-case compose cases
TYPES = ["moveDecl", "renameSymbol", "editStmtBlock", "addDecl", "deleteDecl",
         "modifyImport", "reorderImports", "changeSignature", "updateCall", "extractMethod",
         "inlineMethod", "reorderParams", "addParam", "removeParam", "moveFile",
         "renameFile", "modifyNamespace", "customOp"]
NAMES = ["x", "y", "z", "3", 3, 3.0, True, 1, None, ["l"], {"d": 1}, ""]
ADDRS = ["a1", "a2", "a3", "", 5, None, "MISSING"]
FILES = ["f1.ts", "f2.ts", "", None, "MISSING"]


def rand_ts(rng, mode):
    if mode == "iso":
        return rng.choice(["2025-11-14T00:00:00.000Z", "2025-11-14T00:00:00.001Z",
                           "2025-11-14T00:00:00.002Z", "2025-11-14T00:00:00Z",
                           "1970-01-01T00:00:00Z", "1970-01-01T00:00:00.999Z", "MISSING"])
    return rng.choice(["2025-11-14T00:00:00.000Z", "2025-11-14T00:00:00Z", "abc", "b",
                       "2025-11-14 00:00:00", 5, None, "", "MISSING", "ä", "\U0001f600"])


def rand_id(rng, mode, pool):
    if mode == "uuid":
        if pool and rng.random() < 0.1:
            return rng.choice(pool)
        return str(uuid.UUID(int=rng.getrandbits(128), version=4))
    if mode == "short":
        return rng.choice(["op1", "op2", "op3", "a", "b", "", "op10", "é", "z" * 15])
    return rng.choice(["op-" + "x" * 20, "op-" + "y" * 20, "short", "a", "op-" + "x" * 19])


def rand_op(rng, ts_mode, id_mode, syms, pool):
    typ = rng.choice(TYPES[:6] * 4 + TYPES)
    params = {}
    if typ == "renameSymbol":
        params["oldName"] = "old"
        nn = rng.choice(NAMES + ["MISSING"])
        if nn != "MISSING":
            params["newName"] = nn
        f = rng.choice(FILES)
        if f != "MISSING":
            params["file"] = f
        if rng.random() < 0.2:
            params["newFile"] = rng.choice(["nf.ts", ""])
    elif typ == "moveDecl":
        params["oldAddress"] = "a0"
        a = rng.choice(ADDRS)
        if a != "MISSING":
            params["newAddress"] = a
        f = rng.choice(FILES)
        if f != "MISSING":
            params["newFile"] = f
        f2 = rng.choice(FILES)
        if f2 != "MISSING":
            params["file"] = f2
    else:
        if rng.random() < 0.5:
            params["file"] = "f.ts"
    if rng.random() < 0.15:
        params["renameContext"] = "pre"
    prov = {"rev": "base"}
    ts = rand_ts(rng, ts_mode)
    if ts != "MISSING":
        prov["timestamp"] = ts
    oid = rand_id(rng, id_mode, pool)
    pool.append(oid)
    return {
        "id": oid,
        "schemaVersion": 1,
        "type": typ,
        "target": {"symbolId": rng.choice(syms), "addressId": rng.choice(["ad0", None, "ad1"])},
        "params": params,
        "guards": {"exists": True, "nested": {"k": [1, {"z": None}]}} if rng.random() < 0.3 else {},
        "effects": {"summary": "s", "list": [1, 2]} if rng.random() < 0.3 else {},
        "provenance": prov,
    }


def make_cases(compose, ops_mod, n_cases: int, seed: int):
    rng = random.Random(seed)
    cases = []
    for c in range(n_cases):
        ts_mode = "iso" if c % 3 else "any"
        id_mode = ["uuid", "uuid", "short", "long"][c % 4]
        nsym = rng.choice([1, 2, 3, 5])
        syms = [f"s{i}" for i in range(nsym)]
        pool = []
        na = rng.choice([0, 1, 2, 3, 5, 8, 13, 25])
        nb = rng.choice([0, 1, 2, 3, 5, 8, 13, 25])
        if c % 5 == 0:  # rename-heavy to provoke walk regions
            A = [rand_op(rng, ts_mode, id_mode, syms, pool) for _ in range(na)]
            B = [rand_op(rng, ts_mode, id_mode, syms, pool) for _ in range(nb)]
            for d in A + B:
                if rng.random() < 0.8:
                    d["type"] = "renameSymbol"
                    d["params"]["newName"] = rng.choice(["p", "q", "r", None])
        else:
            A = [rand_op(rng, ts_mode, id_mode, syms, pool) for _ in range(na)]
            B = [rand_op(rng, ts_mode, id_mode, syms, pool) for _ in range(nb)]
        cases.append(run_case(compose, ops_mod, A, B))
    return cases


def run_case(compose, ops_mod, A, B):
    oa = [ops_mod.Op.from_dict(d) for d in A]
    ob = [ops_mod.Op.from_dict(d) for d in B]
    before = json.dumps([o.to_dict() for o in oa + ob])
    out, conf = compose.compose_oplogs(oa, ob)
    assert json.dumps([o.to_dict() for o in oa + ob]) == before, "reference mutated inputs"
    return {"A": A, "B": B, "out": [o.to_dict() for o in out],
            "conflicts": [c.to_dict() for c in conf]}


def scenarios(compose, ops_mod):
    """The reference's own test scenarios with fixed ids (tests/test_compose.py:10-25,
    tests/e2e_rename_move_decl.sh:22-65)."""
    mv = {"id": "7d2c9a4e-1b3f-4c8a-9e6d-2f1a0b9c8d7e", "schemaVersion": 1, "type": "moveDecl",
          "target": {"symbolId": "symbol-123", "addressId": "old-address"},
          "params": {"newAddress": "new-address"}, "guards": {}, "effects": {}, "provenance": {}}
    rn = {"id": "11111111-2222-4333-8444-555555555555", "schemaVersion": 1,
          "type": "renameSymbol", "target": {"symbolId": "symbol-foo", "addressId": "addr-old"},
          "params": {"oldName": "foo", "newName": "bar", "file": "src/util.ts"},
          "guards": {}, "effects": {}, "provenance": {}}
    mv2 = {"id": "66666666-7777-4888-9999-aaaaaaaaaaaa", "schemaVersion": 1, "type": "moveDecl",
           "target": {"symbolId": "symbol-foo", "addressId": "addr-old"},
           "params": {"oldAddress": "addr-old", "newAddress": "addr-new",
                      "oldFile": "src/util.ts", "newFile": "lib/util.ts"},
           "guards": {}, "effects": {}, "provenance": {}}
    return {
        "test_compose_move_only": run_case(compose, ops_mod, [mv], []),
        "e2e_rename_move_decl": run_case(compose, ops_mod, [rn], [mv2]),
    }


# ---------------------------------------------------------------------------
# synthetic configs: digests of the reference output
def synth_digest(compose, ops_mod, name, spec):
    from semantic_merge_amd import synth
    logs = synth.lift_logs(spec)
    A, B = synth.lift_op_dicts(logs)
    oa = [ops_mod.Op.from_dict(d) for d in A]
    ob = [ops_mod.Op.from_dict(d) for d in B]
    t0 = time.perf_counter()
    out, conf = compose.compose_oplogs(oa, ob)
    dt = time.perf_counter() - t0
    rec = {
        "name": name,
        "spec": {k: v for k, v in spec.__dict__.items() if k != "mix"},
        "mix": [list(x) for x in spec.mix],
        "n_out": len(out),
        "n_conflicts": len(conf),
        "out_sha256": digest(o.to_dict() for o in out),
        "conflicts_sha256": digest(c.to_dict() for c in conf),
        # first/last records verbatim, for a readable failure
        "out_head": [o.to_dict() for o in out[:3]],
        "conflicts_head": [c.to_dict() for c in conf[:2]],
        "reference_seconds": round(dt, 3),
    }
    print(f"{name}: n={spec.n_total} out={len(out)} conflicts={len(conf)} ref {dt:.2f}s",
          flush=True)
    return rec


# ---------------------------------------------------------------------------
# RGA cases
def make_rga_cases(crdt, n_cases: int, seed: int):
    rng = random.Random(seed)
    cases = []
    for c in range(n_cases):
        nvals = rng.choice([1, 2, 3, 6])
        vals = [f"v{i}" for i in range(nvals)]
        anchors = rng.choice([["root"], ["a", "b"], ["", "a", "ab", "b"]])
        authors = rng.choice([["u1"], ["u1", "u2"], ["A", "a", "b"]])
        events = []
        for _ in range(rng.choice([0, 1, 3, 8, 20, 40])):
            kind = rng.choices(["insert", "move", "delete"], [0.6, 0.25, 0.15])[0]
            key = [rng.choice(anchors), rng.choice([0, 1, 2, 5, -1, 2 ** 40]),
                   rng.choice(authors), rng.choice(["o1", "o2", "o3", "p"])]
            if c % 4 == 0:
                key[3] = str(uuid.UUID(int=rng.getrandbits(128), version=4))
            if kind == "delete":
                events.append(["delete", rng.choice(vals)])
            else:
                events.append([kind, rng.choice(vals), key])
        rga = crdt.RGA()
        for ev in events:
            if ev[0] == "insert":
                rga.insert(crdt.Key(*ev[2]), ev[1])
            elif ev[0] == "move":
                rga.move(ev[1], crdt.Key(*ev[2]))
            else:
                rga.delete(ev[1])
        cases.append({"events": events, "out": rga.materialize()})
    return cases


def make_rga_list_cases(crdt):
    """The reference's RGA.list state (crdt.py:26-27: every element in list order, with
    its key and tombstone) after each stream of tests/golden/rga_cases.json."""
    cases = json.load(open(os.path.join(GOLD, "rga_cases.json")))
    out = []
    for case in cases:
        rga = crdt.RGA()
        for ev in case["events"]:
            if ev[0] == "insert":
                rga.insert(crdt.Key(*ev[2]), ev[1])
            elif ev[0] == "move":
                rga.move(ev[1], crdt.Key(*ev[2]))
            else:
                rga.delete(ev[1])
        out.append([[[e.key.anchor, e.key.t, e.key.author, e.key.opid], e.value, e.tombstone]
                    for e in rga.list])
    return out


def make_rga_mutation_cases(crdt, n_cases: int, seed: int):
    """Scripts that mix RGA events with reads and in-place changes of the reference's
    mutable state RGA.list (crdt.py:26-27): appends, pops, tombstone flips, whole-list
    assignments, and an element held across later events (delete() sets its tombstone in
    place, crdt.py:40-43).  Each script keeps the list in key order (what insert() and
    move() maintain).  Recorded: the list after every "read", materialize() after every
    "materialize", the held element's tombstone after every "held"."""
    rng = random.Random(seed)

    def key():
        return [rng.choice(["", "a", "b"]), rng.choice([0, 1, 2, 7, -3]), rng.choice(["u1", "u2"]),
                rng.choice(["o1", "o2", "o3"])]

    def snap(rga):
        return [[[e.key.anchor, e.key.t, e.key.author, e.key.opid], e.value, e.tombstone] for e in rga.list]

    def tup(k):
        return (k.anchor, k.t, k.author, k.opid)

    cases = []
    for _ in range(n_cases):
        vals = ["v%d" % i for i in range(rng.choice([1, 2, 4]))]
        rga = crdt.RGA()
        held = None
        steps, rec = [], []
        for _ in range(rng.choice([4, 10, 25])):
            r = rng.random()
            if r < 0.35:
                step = ["insert", rng.choice(vals), key()]
                rga.insert(crdt.Key(*step[2]), step[1])
            elif r < 0.5:
                step = ["move", rng.choice(vals), key()]
                rga.move(step[1], crdt.Key(*step[2]))
            elif r < 0.6:
                step = ["delete", rng.choice(vals)]
                rga.delete(step[1])
            elif r < 0.68:
                step = ["read"]
                rec.append(snap(rga))
            elif r < 0.74:
                step = ["materialize"]
                rec.append(rga.materialize())
            elif r < 0.8:  # append past the last key (the list stays in key order)
                last = tup(rga.list[-1].key) if rga.list else None
                k = key()
                if last is not None and tuple(k) < last:
                    k = [last[0], last[1] + 1, last[2], last[3]]
                step = ["append", k, rng.choice(vals), rng.random() < 0.3]
                rga.list.append(crdt.Elem(crdt.Key(*step[1]), step[2], step[3]))
            elif r < 0.85 and rga.list:
                step = ["pop", rng.randrange(len(rga.list))]
                rga.list.pop(step[1])
            elif r < 0.9 and rga.list:
                step = ["set_tomb", rng.randrange(len(rga.list)), rng.random() < 0.5]
                rga.list[step[1]].tombstone = step[2]
            elif r < 0.93:
                items = sorted([(tuple(key()), rng.choice(vals), rng.random() < 0.3)
                                for _ in range(rng.choice([0, 1, 3]))], key=lambda x: x[0])
                step = ["assign", [[list(k), v, tb] for k, v, tb in items]]
                rga.list = [crdt.Elem(crdt.Key(*k), v, tb) for k, v, tb in items]
            elif r < 0.97 and rga.list:
                step = ["hold", rng.randrange(len(rga.list))]
                held = rga.list[step[1]]
            else:
                step = ["held"]
                rec.append(None if held is None else held.tombstone)
            steps.append(step)
        steps.append(["read"])
        rec.append(snap(rga))
        cases.append({"steps": steps, "out": rec})
    return cases


# ---------------------------------------------------------------------------
# OpLog.from_json cases (ops.py:106-121): JSON texts of op dicts with the coercions
# Op.from_dict applies (ops.py:89-100), and the reference's decoded ops -- or the
# exception class it raises.
def make_oplog_cases(ops_mod, n_cases: int, seed: int):
    rng = random.Random(seed)
    cases = []
    for c in range(n_cases):
        pool = []
        syms = ["s0", "s1", "sé"]
        items = [rand_op(rng, "iso" if c % 2 else "any", ["uuid", "short", "long"][c % 3], syms, pool)
                 for _ in range(rng.choice([0, 1, 2, 5, 9]))]
        for d in items:
            r = rng.random()
            if r < 0.1:
                d["schemaVersion"] = rng.choice(["2", 3.0, True, "7"])
            elif r < 0.2:
                del d["schemaVersion"]
            elif r < 0.3:
                d["id"] = rng.choice([123, 4.5, True, None, "ü-id"])
            for k in ("params", "guards", "effects", "provenance"):
                if rng.random() < 0.08:
                    del d[k]
            if rng.random() < 0.1 and "params" in d:
                d["params"]["unicode"] = "naïve ☃ \U0001f600"
                d["params"]["float"] = rng.choice([0.1, -2.5e-8, 1e300, 12345678901234567])
        bad = None
        if c % 10 == 9 and items:  # malformed input: the reference's exception
            bad = rng.choice(["type", "target", "symbolId", "schemaVersion", "id"])
            d = items[0]
            if bad == "type":
                del d["type"]
            elif bad == "target":
                del d["target"]
            elif bad == "symbolId":
                d["target"] = {"addressId": "x"}
            elif bad == "schemaVersion":
                d["schemaVersion"] = "v1"
            else:
                del d["id"]
        text = json.dumps(items, ensure_ascii=rng.random() < 0.5,
                          separators=rng.choice([(",", ":"), (", ", ": ")]),
                          indent=rng.choice([None, None, 2]))
        try:
            log = ops_mod.OpLog.from_json(text)
            cases.append({"text": text, "ops": [o.to_dict() for o in log.ops]})
        except Exception as e:  # noqa: BLE001 - the class name is the fixture
            cases.append({"text": text, "error": type(e).__name__})
    return cases


# ---------------------------------------------------------------------------
# applier cases (applier.py:14-104): a base tree, an op sequence, and the reference's
# merged tree (or the exception it raised, with the tree as it left it).  Paths stay
# inside the tree (no "..": the reference would write outside its temp directory).
def _tree(root):
    files, dirs = {}, []
    for dp, dn, fn in os.walk(root):
        rel = os.path.relpath(dp, root)
        if rel != ".":
            dirs.append(rel)
        for f in fn:
            with open(os.path.join(dp, f), "rb") as fh:
                files[os.path.normpath(os.path.join(rel, f))] = fh.read().decode("latin-1")
    return files, sorted(dirs)


def make_e2e_tree(compose, applier_mod, ops_mod):
    """Config 1: tests/e2e_rename_move_decl.sh:14-74 with fixed ids -- base tree
    src/util.ts, A renames foo -> bar, B moves the declaration to lib/util.ts; the
    reference's composed log and the merged tree its apply_ops leaves."""
    import pathlib
    import shutil
    import tempfile
    sc = scenarios(compose, ops_mod)["e2e_rename_move_decl"]
    base_files = {"src/util.ts": "export function foo(x: number) {\n  return x + 1;\n}\n"}
    tmp = tempfile.mkdtemp(prefix="smx_e2e_")
    try:
        for pth, text in base_files.items():
            full = pathlib.Path(tmp) / pth
            full.parent.mkdir(parents=True, exist_ok=True)
            full.write_text(text, encoding="utf-8")
        oa = [ops_mod.Op.from_dict(d) for d in sc["A"]]
        ob = [ops_mod.Op.from_dict(d) for d in sc["B"]]
        out, conf = compose.compose_oplogs(oa, ob)
        merged = applier_mod.apply_ops(pathlib.Path(tmp), out)
        try:
            files, dirs = _tree(merged)
        finally:
            shutil.rmtree(merged, ignore_errors=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    assert "function bar" in files["lib/util.ts"]
    return {"base": base_files, "A": sc["A"], "B": sc["B"], "out": [o.to_dict() for o in out],
            "conflicts": [c.to_dict() for c in conf], "files": files, "dirs": dirs}


def make_applier_cases(applier_mod, ops_mod, n_cases: int, seed: int):
    import shutil
    import tempfile
    rng = random.Random(seed)
    names = ["foo", "bar", "a.b", "$x", "x1", "foo_bar", "élan", "if", "Foo", "o"]
    paths = ["src/a.ts", "src/b.ts", "lib/c.ts", "d.ts", "src/deep/e.ts", "/abs/src/a.ts"]
    cases = []
    for c in range(n_cases):
        base = {}
        for pth in ("src/a.ts", "src/b.ts", "lib/c.ts", "d.ts"):
            if rng.random() < 0.85:
                words = [rng.choice(names + ["import x from 'y';", "(", ")", ".", "=", "1"])
                         for _ in range(rng.randint(0, 40))]
                text = " ".join(words)
                if rng.random() < 0.2:
                    text = text.replace(" ", "\r\n", 3)
                base[pth] = text
        ops = []
        for k in range(rng.randint(0, 14)):
            t = rng.choice(["renameSymbol"] * 5 + ["modifyImport"] * 2 + ["moveDecl"] * 2 + ["moveFile", "addDecl"])
            params = {}
            if t == "renameSymbol":
                params = {"file": rng.choice(paths + [None, ""]), "oldName": rng.choice(names + [None]),
                          "newName": rng.choice(names + ["\\g<0>!", "n\\n", None, 7])}
                if rng.random() < 0.2:
                    params["newFile"] = rng.choice(paths)
            elif t == "modifyImport":
                params = {"file": rng.choice(paths), "oldImport": rng.choice(["'y'", "x", None]),
                          "newImport": rng.choice(["'z'", "w", None])}
            elif t == "moveDecl":
                params = {"oldFile": rng.choice(paths + [None]), "newFile": rng.choice(paths + ["src/new/f.ts"]),
                          "file": rng.choice(paths + [None])}
            elif t == "moveFile":
                params = {"oldPath": rng.choice(paths + ["src", "lib"]),
                          "newPath": rng.choice(paths + ["moved", "src/deep", "lib2/c.ts"])}
            ops.append({"id": f"op{c}-{k}", "type": t, "target": {"symbolId": "s", "addressId": None},
                        "params": params})
        tmp = tempfile.mkdtemp(prefix="smx_gold_")
        try:
            for pth, text in base.items():
                full = os.path.join(tmp, "base", pth)
                os.makedirs(os.path.dirname(full), exist_ok=True)
                with open(full, "w", encoding="utf-8", newline="") as fh:
                    fh.write(text)
            os.makedirs(os.path.join(tmp, "base"), exist_ok=True)
            op_objs = [ops_mod.Op.from_dict(d) for d in ops]
            before = set(os.listdir(tempfile.gettempdir()))
            err = None
            try:
                out = applier_mod.apply_ops(os.path.join(tmp, "base"), op_objs)
            except Exception as e:  # noqa: BLE001 - the class name is the fixture
                err = type(e).__name__
                new = [d for d in set(os.listdir(tempfile.gettempdir())) - before
                       if d.startswith("semmerge_merged_")]
                out = os.path.join(tempfile.gettempdir(), new[0])
            files, dirs = _tree(out)
            shutil.rmtree(out)
        finally:
            shutil.rmtree(tmp)
        rec = {"base": base, "ops": ops, "files": files, "dirs": dirs}
        if err:
            rec["error"] = err
        cases.append(rec)
    return cases


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--only", choices=["oplog", "applier", "big", "e2e", "rga_list", "rga_mut"],
                    help="regenerate one fixture only")
    args = ap.parse_args()
    compose, crdt, ops_mod = _import_reference()
    os.makedirs(GOLD, exist_ok=True)
    if args.only in (None, "oplog"):
        with open(os.path.join(GOLD, "oplog_cases.json"), "w") as fh:
            json.dump(make_oplog_cases(ops_mod, 300, seed=112), fh, separators=(",", ":"), ensure_ascii=False)
    if args.only in (None, "applier"):
        from semmerge import applier as applier_mod
        with open(os.path.join(GOLD, "applier_cases.json"), "w") as fh:
            json.dump(make_applier_cases(applier_mod, ops_mod, 400, seed=77), fh, separators=(",", ":"),
                      ensure_ascii=False)
    if args.only == "rga_list":
        with open(os.path.join(GOLD, "rga_list_cases.json"), "w") as fh:
            json.dump(make_rga_list_cases(crdt), fh, separators=(",", ":"))
    if args.only == "rga_mut":
        with open(os.path.join(GOLD, "rga_mutation_cases.json"), "w") as fh:
            json.dump(make_rga_mutation_cases(crdt, 300, seed=31), fh, separators=(",", ":"))
    if args.only == "e2e":
        from semmerge import applier as applier_mod
        with open(os.path.join(GOLD, "e2e_tree.json"), "w") as fh:
            json.dump(make_e2e_tree(compose, applier_mod, ops_mod), fh, indent=1, ensure_ascii=False)
    if args.only == "big":
        from semantic_merge_amd import synth
        _save_digests([synth_digest(compose, ops_mod, "c2_1M", synth.CONFIGS["c2"])])
    if args.only:
        return

    cases = make_cases(compose, ops_mod, 600, seed=20251114)
    with open(os.path.join(GOLD, "compose_cases.json"), "w") as fh:
        json.dump(cases, fh, separators=(",", ":"))
    with open(os.path.join(GOLD, "compose_scenarios.json"), "w") as fh:
        json.dump(scenarios(compose, ops_mod), fh, indent=1)
    print(f"compose cases: {len(cases)}, "
          f"with conflicts: {sum(1 for c in cases if c['conflicts'])}")

    with open(os.path.join(GOLD, "rga_cases.json"), "w") as fh:
        json.dump(make_rga_cases(crdt, 600, seed=13), fh, separators=(",", ":"))

    from semantic_merge_amd import synth
    specs = [
        ("lift_20k", synth.LiftSpec(20_000, 200, 3)),
        ("lift_200k", synth.LiftSpec(200_000, 2_000, 5)),
        ("lift_100k_shuffled", synth.LiftSpec(100_000, 1_000, 9, shuffle=True)),
        ("adversarial_100k", synth.LiftSpec(100_000, 500, 17, ops_per_ms=4096,
                                            mix=synth.ADVERSARIAL_MIX, rename_overlap=0.30)),
    ]
    if args.big:
        specs.append(("c2_1M", synth.CONFIGS["c2"]))
    _save_digests([synth_digest(compose, ops_mod, name, spec) for name, spec in specs])


def _save_digests(recs) -> None:
    path = os.path.join(GOLD, "compose_digests.json")
    old = {}
    if os.path.exists(path):
        old = {r["name"]: r for r in json.load(open(path))}
    for r in recs:
        old[r["name"]] = r
    with open(path, "w") as fh:
        json.dump(list(old.values()), fh, indent=1, ensure_ascii=False)


if __name__ == "__main__":
    main()
