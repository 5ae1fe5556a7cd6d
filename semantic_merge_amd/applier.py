r"""Applier fast path: ``apply_ops`` of ``semmerge/applier.py:14-94``
with the text edits batched per file.

The reference applies the composed ops one at a time to a copy of the base tree: every
``renameSymbol`` and ``modifyImport`` reads its whole file, rewrites it and writes it
back (``applier.py:66-94``), so a file touched by k ops is read and written k times.
Here each text file is read once, edited in memory in op order, and written once --
before any move (a move sees, and carries, the edited contents), before an exception
propagates, and at the end.  Edits are keyed by the file itself (device, inode), so
every spelling of a path reaches the same text.  Moves run
exactly as the reference runs them (``shutil.move``, ``applier.py:37-63``), so their
directory and overwrite semantics are the filesystem's own.  Text I/O uses the same
``Path.read_text`` / ``write_text`` calls (UTF-8, universal newlines), regex
substitution the same pattern and replacement template, so the final tree is the
reference's byte for byte, and a failing op leaves the tree the reference would leave.

Consecutive renames of one file whose old and new names are both identifiers (``\w+``)
are composed into one substitution pass: such a rename replaces whole tokens by whole
tokens and never moves a token boundary, so the sequence maps every token on its own --
token t becomes the fold of ``x -> new_i if x == old_i else x`` over the renames -- and
one ``\b(?:old_1|old_2|...)\b`` pass with that map gives the sequential result.  Any
other rename or import edit of the file first applies the pending renames.

This path is filesystem work; it has no device part.
"""
from __future__ import annotations

import logging
import pathlib
import re
import shutil
import tempfile
from typing import Dict, Iterable

logger = logging.getLogger("semmerge")
_IDENT = re.compile(r"\w+")


def _utf8_ok(s: str) -> bool:
    try:
        s.encode("utf-8")
        return True
    except UnicodeEncodeError:
        return False


def _normalize_relpath(value: str) -> pathlib.Path:
    """applier.py:97-104."""
    path = pathlib.Path(value)
    if path.is_absolute():
        try:
            path = path.relative_to(path.anchor)
        except ValueError:
            path = pathlib.Path(path.name)
    return path


class _Texts:
    """Files read once and edited in memory, keyed by the file itself (device, inode:
    every path spelling, symlink or hard link of one file shares its entry); dirty ones
    written back on flush through the path that loaded them."""

    def __init__(self) -> None:
        self.text: Dict[tuple, str] = {}
        self.dirty: Dict[tuple, bool] = {}
        self.path: Dict[tuple, pathlib.Path] = {}
        self.pending: Dict[tuple, list] = {}  # identifier renames not yet applied
        self._pat: Dict[str, "re.Pattern[str]"] = {}

    @staticmethod
    def key(path: pathlib.Path):
        """The file's identity, or None when the path does not exist (path.exists())."""
        try:
            st = path.stat()
        except (OSError, ValueError):
            return None
        return (st.st_dev, st.st_ino)

    def get(self, key, path: pathlib.Path) -> str:
        t = self.text.get(key)
        if t is None:
            t = path.read_text(encoding="utf-8")
            self.text[key] = t
            self.dirty[key] = False
            self.path[key] = path
        elif key in self.pending:
            t = self.apply_pending(key)
        return t

    def defer_rename(self, key, old: str, new: str) -> None:
        self.pending.setdefault(key, []).append((old, new))
        self.dirty[key] = True

    def apply_pending(self, key) -> str:
        ren = self.pending.pop(key, None)
        t = self.text[key]
        if not ren:
            return t
        final = {}
        for old, _ in ren:  # each token's image under the whole sequence
            if old not in final:
                x = old
                for o, n in ren:
                    if x == o:
                        x = n
                final[old] = x
        alive = {o: n for o, n in final.items() if o != n}
        if alive:
            pat = re.compile(r"\b(?:" + "|".join(map(re.escape, sorted(alive, key=len, reverse=True))) + r")\b")
            t = pat.sub(lambda m: alive[m.group(0)], t)
        self.text[key] = t
        return t

    def put(self, key, t: str, old: str, repl: str) -> None:
        if t != old and not _utf8_ok(repl):
            # the reference's write of this op fails (a lone surrogate from the new
            # name): the same write, with everything before it already on disk
            path = self.path[key]
            self.flush()
            path.write_text(t, encoding="utf-8")
        self.text[key] = t
        self.dirty[key] = True

    def pattern(self, old: str) -> "re.Pattern[str]":
        p = self._pat.get(old)
        if p is None:
            p = self._pat[old] = re.compile(rf"\b{re.escape(old)}\b")
        return p

    def flush(self) -> None:
        """Write back (and forget) every file."""
        try:
            for key in list(self.text):
                t = self.apply_pending(key)
                if self.dirty[key]:
                    self.path[key].write_text(t, encoding="utf-8")
        finally:
            self.text.clear()
            self.dirty.clear()
            self.path.clear()
            self.pending.clear()


def apply_ops(base_tree: pathlib.Path, ops: Iterable, prefix: str = "semmerge_merged_") -> pathlib.Path:
    """Apply *ops* onto a copy of *base_tree* and return the merged tree path
    (applier.py:14-34)."""
    base_tree = pathlib.Path(base_tree)
    out = pathlib.Path(tempfile.mkdtemp(prefix=prefix))
    shutil.copytree(base_tree, out, dirs_exist_ok=True)
    texts = _Texts()
    try:
        for op in ops:
            if op.type == "moveDecl":
                _move_decl(out, op, texts)
            elif op.type == "renameSymbol":
                _rename_symbol(out, op, texts)
            elif op.type == "modifyImport":
                _modify_import(out, op, texts)
            elif op.type == "moveFile":
                _move_file(out, op, texts)
            else:
                logger.debug("No applier hook for op %s", op.type)
    finally:
        texts.flush()
    return out


def _move(src: pathlib.Path, dst: pathlib.Path, texts: _Texts) -> None:
    texts.flush()  # the move sees (and carries) the edited contents; inodes may change
    dst.parent.mkdir(parents=True, exist_ok=True)
    shutil.move(src, dst)


def _move_decl(root: pathlib.Path, op, texts: _Texts) -> None:
    """applier.py:37-50."""
    old_file = op.params.get("oldFile") or op.params.get("file")
    new_file = op.params.get("newFile") or op.params.get("file")
    if not old_file or not new_file:
        return
    src = root / _normalize_relpath(old_file)
    dst = root / _normalize_relpath(new_file)
    if src == dst:
        return
    if not src.exists():
        logger.debug("moveDecl source missing: %s", src)
        return
    _move(src, dst, texts)


def _move_file(root: pathlib.Path, op, texts: _Texts) -> None:
    """applier.py:53-63."""
    old_path = op.params.get("oldPath")
    new_path = op.params.get("newPath")
    if not old_path or not new_path:
        return
    src = root / _normalize_relpath(old_path)
    dst = root / _normalize_relpath(new_path)
    if not src.exists():
        logger.debug("moveFile source missing: %s", src)
        return
    _move(src, dst, texts)


def _rename_symbol(root: pathlib.Path, op, texts: _Texts) -> None:
    """applier.py:66-79: word-boundary regex substitution of the old name."""
    file_path = op.params.get("file") or op.params.get("newFile")
    old_name = op.params.get("oldName")
    new_name = op.params.get("newName")
    if not file_path or not old_name or not new_name:
        return
    path = root / _normalize_relpath(file_path)
    key = texts.key(path)
    if key is None:
        logger.debug("renameSymbol target missing: %s", path)
        return
    old, repl = str(old_name), str(new_name)
    if _IDENT.fullmatch(old) and _IDENT.fullmatch(repl):
        if key not in texts.text:
            texts.get(key, path)  # read (and decode) the file now, as the reference does
        texts.defer_rename(key, old, repl)
        return
    code = texts.get(key, path)
    texts.put(key, texts.pattern(old).sub(repl, code), code, repl)


def _modify_import(root: pathlib.Path, op, texts: _Texts) -> None:
    """applier.py:82-94."""
    file_path = op.params.get("file")
    old_import = op.params.get("oldImport")
    new_import = op.params.get("newImport")
    if not file_path or old_import is None or new_import is None:
        return
    path = root / _normalize_relpath(file_path)
    key = texts.key(path)
    if key is None:
        logger.debug("modifyImport target missing: %s", path)
        return
    code = texts.get(key, path)
    repl = str(new_import)
    texts.put(key, str(code).replace(str(old_import), repl), code, repl)
