"""The ctypes mirrors in semantic_merge_amd/_abi.py have the C layout of include/smx.h
(sizes and field offsets, from a host C program compiled against the header)."""
import ctypes
import os
import subprocess
import tempfile

import pytest

from semantic_merge_amd import _abi

HDR_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
STRUCTS = {"smx_ops": _abi.SmxOps, "smx_compose_out": _abi.SmxComposeOut, "smx_shard": _abi.SmxShard,
           "smx_rga_ops": _abi.SmxRgaOps, "smx_rga_out": _abi.SmxRgaOut}


def test_ctypes_structs_match_header():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "smx.h"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        r = subprocess.run(["gcc", "-I", HDR_DIR, "-o", exe, src], capture_output=True, text=True)
        if r.returncode != 0 and "not found" in r.stderr:
            pytest.skip("no C compiler")
        assert r.returncode == 0, r.stderr
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {}
    for line in filter(None, out):
        parts = line.split()
        got[tuple(parts[:-1])] = int(parts[-1])
    for cname, py in STRUCTS.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)
