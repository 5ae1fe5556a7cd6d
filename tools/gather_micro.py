"""Random-lookup cost by entry shape and table size (see gather_micro.hip).

    python tools/gather_micro.py [--lookups 64000000] [--iters 10]

One JSON line per (shape, entries): ms per launch, ns per lookup and the table bytes.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
"""
import argparse
import ctypes as C
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SHAPES = {0: "streams only", 1: "4 B aligned", 2: "8 B aligned", 3: "6 B packed, 8 B load at 4-aligned",
          4: "16 B aligned", 5: "6 B packed, two dword loads", 6: "6 B packed, 1 of 4 via scalar loads",
          7: "6 B packed, 2 of 4 via scalar loads", 8: "6 B packed, all via scalar loads"}
BYTES = {0: 0, 1: 4, 2: 8, 3: 6.1, 4: 16, 5: 6.1, 6: 6.1, 7: 6.1, 8: 6.1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lookups", type=int, default=64_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--log2-entries", default="15,18,20")
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(HERE, "_build", "libsmx_gather_micro.so"))
    lib.gather_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int64, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    nq = a.lookups // 4
    g = torch.Generator(device=dev).manual_seed(1)
    idx = torch.randint(0, 2**31 - 1, (nq * 4,), device=dev, dtype=torch.int32, generator=g)
    out = torch.empty(nq * 4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    res = {}
    for rnd in range(3):
        for le in [int(x) for x in a.log2_entries.split(",")]:
            ne = 1 << le
            tab = torch.randint(0, 2**31 - 1, (ne * 4 + 64,), device=dev, dtype=torch.int32, generator=g)
            for v in SHAPES:
                rc = lib.gather_run(v, idx.data_ptr(), tab.data_ptr(), ne - 1, nq, out.data_ptr(), st.cuda_stream)
                assert rc == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.iters):
                    lib.gather_run(v, idx.data_ptr(), tab.data_ptr(), ne - 1, nq, out.data_ptr(), st.cuda_stream)
                e1.record(st)
                e1.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                res.setdefault((v, le), []).append(ms)
    for (v, le), ms in sorted(res.items()):
        m = sorted(ms)[len(ms) // 2]
        print(json.dumps({"shape": SHAPES[v], "entries": 1 << le, "table_MB": round(BYTES[v] * (1 << le) / 2**20, 2),
                          "ms": round(m, 4), "ns_per_lookup": round(m * 1e6 / (nq * 4), 4)}))


if __name__ == "__main__":
    main()
