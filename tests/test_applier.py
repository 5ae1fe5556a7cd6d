"""Applier fast path (semantic_merge_amd/applier.py) against the
reference's own apply_ops (semmerge/applier.py:14-104): 400 base trees and op sequences
whose merged trees -- or the exception and the tree it left -- tools/make_golden.py
recorded by running the reference.  Byte-exact trees, same directories, same exception
class."""
import os
import shutil
import tempfile

import pytest

from semantic_merge_amd import applier
from semantic_merge_amd.ops import Op

from _util import load


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


def test_applier_matches_reference_trees(tmp_path):
    cases = load("applier_cases.json")
    assert len(cases) == 400 and sum("error" in c for c in cases) > 10
    for i, case in enumerate(cases):
        base = tmp_path / f"base{i}"
        base.mkdir()
        for pth, text in case["base"].items():
            full = base / pth
            full.parent.mkdir(parents=True, exist_ok=True)
            with open(full, "w", encoding="utf-8", newline="") as fh:
                fh.write(text)
        ops = [Op.from_dict(d) for d in case["ops"]]
        prefix = f"smx_applier_t{i}_"
        err = None
        try:
            out = applier.apply_ops(base, ops, prefix=prefix)
        except Exception as e:  # noqa: BLE001
            err = type(e).__name__
            (d,) = [x for x in os.listdir(tempfile.gettempdir()) if x.startswith(prefix)]
            out = os.path.join(tempfile.gettempdir(), d)
        try:
            assert err == case.get("error"), f"case {i}: {err} vs {case.get('error')}"
            files, dirs = _tree(out)
            assert files == case["files"], f"case {i}"
            assert dirs == case["dirs"], f"case {i}"
        finally:
            shutil.rmtree(out)


def test_applier_batches_file_io(tmp_path, monkeypatch):
    """k renames of one file: one read and one write (the reference does k of each)."""
    import pathlib
    (tmp_path / "src").mkdir()
    (tmp_path / "src" / "a.ts").write_text("foo bar foo\n", encoding="utf-8")
    reads, writes = [], []
    orig_r, orig_w = pathlib.Path.read_text, pathlib.Path.write_text
    monkeypatch.setattr(pathlib.Path, "read_text", lambda self, *a, **k: reads.append(self) or orig_r(self, *a, **k))
    monkeypatch.setattr(pathlib.Path, "write_text",
                        lambda self, *a, **k: writes.append(self) or orig_w(self, *a, **k))
    names = ["foo", "x1", "x2", "x3", "x4", "x5"]
    ops = [Op.from_dict({"id": f"o{k}", "type": "renameSymbol", "target": {"symbolId": "s"},
                         "params": {"file": "src/a.ts", "oldName": names[k], "newName": names[k + 1]}})
           for k in range(5)]
    out = applier.apply_ops(tmp_path, ops)
    try:
        assert (out / "src" / "a.ts").read_text() == "x5 bar x5\n"
        assert len(reads) == 2 and len(writes) == 1  # (+ the check above)
    finally:
        shutil.rmtree(out)


def test_composed_renames_equal_sequential_substitution(tmp_path):
    """Chains, swaps and cycles of identifier renames in one file: the one-pass
    composition equals the reference's one re.sub per op (applier.py:77-78)."""
    import random
    import re
    rng = random.Random(3)
    vocab = ["a", "b", "c", "ab", "a1", "_x", "é", "b_c", "z9"]
    for trial in range(200):
        text = "".join(rng.choice(vocab + [" ", ".", "(", ")", "\n", "-"]) for _ in range(300))
        (tmp_path / "f.ts").write_text(text, encoding="utf-8")
        pairs = [(rng.choice(vocab), rng.choice(vocab)) for _ in range(rng.randint(1, 12))]
        want = text
        for old, new in pairs:
            want = re.sub(rf"\b{re.escape(old)}\b", new, want)
        ops = [Op.from_dict({"id": f"o{k}", "type": "renameSymbol", "target": {"symbolId": "s"},
                             "params": {"file": "f.ts", "oldName": o, "newName": n}})
               for k, (o, n) in enumerate(pairs)]
        out = applier.apply_ops(tmp_path, ops)
        try:
            assert (out / "f.ts").read_text(encoding="utf-8") == want, (trial, pairs)
        finally:
            shutil.rmtree(out)
