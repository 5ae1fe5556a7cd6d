"""CRDT benchmark: 10M RGA events over 50k lists on one GPU,
device-resident; prints one JSON line with events/s, the 45 B/event roofline
fraction and the CPU oracle (1 thread) on a bounded sample."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from semantic_merge_amd import _abi, _lib, synth
    n, nl = int(os.environ.get("RGA_N", 10_000_000)), int(os.environ.get("RGA_LISTS", 50_000))
    b = synth.rga_batch(n, nl, 13)
    dev = torch.device("cuda")

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)

    vals = torch.empty(n, dtype=torch.int32, device=dev)
    src = torch.empty(n, dtype=torch.int32, device=dev)
    offs = torch.empty(nl + 1, dtype=torch.int64, device=dev)
    counts = torch.zeros(1, dtype=torch.int64, device=dev)
    lib = _lib.lib()
    ws = C.c_size_t(0)
    _lib.check(lib.smx_rga_workspace_bytes(n, nl, C.byref(ws)))
    wst = torch.empty(ws.value, dtype=torch.uint8, device=dev)
    out = _abi.SmxRgaOut(vals.data_ptr(), src.data_ptr(), offs.data_ptr(), counts.data_ptr())
    s = torch.cuda.current_stream().cuda_stream
    steps = int(os.environ.get("RGA_STEPS", 5))

    def timed(batch, flags):
        """ms per call of smx_rga_replay_ex on the batch, device-resident."""
        ins = [up(batch.list_id, np.int32), up(batch.op, np.uint8), up(batch.value, np.int32),
               up(batch.anchor, np.int32), up(batch.t, np.int64), up(batch.author, np.int32),
               up(batch.opid_hi, np.int64), up(batch.opid_lo, np.int64)]
        ops = _abi.SmxRgaOps(n, nl, *[t.data_ptr() for t in ins])
        for _ in range(2):
            _lib.check(lib.smx_rga_replay_ex(C.byref(ops), C.byref(out), wst.data_ptr(), ws.value, flags, s))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            _lib.check(lib.smx_rga_replay_ex(C.byref(ops), C.byref(out), wst.data_ptr(), ws.value, flags, s))
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    # the drop-in's shape: each list's events together (crdt.replay / RGA hand over
    # stream after stream), through SMX_RGA_GROUPED
    from semantic_merge_amd.crdt import RgaBatch
    p = np.argsort(b.list_id, kind="stable")
    bg = RgaBatch(nl, b.list_id[p], b.op[p], b.value[p], b.anchor[p], b.t[p], b.author[p], b.opid_hi[p],
                  b.opid_lo[p], [])
    dtg = timed(bg, _abi.RGA_GROUPED)
    del bg, p
    dt = timed(b, 0)  # config 4 as generated: list ids interleaved
    grouped = {"ms_per_step": round(dtg * 1e3, 3), "value": round(n / dtg, 1),
               "roofline_frac": round(45 * n / dtg / 1e9 / 8000.0, 4),
               "note": "the same events grouped list by list (the drop-in's shape), SMX_RGA_GROUPED: no partition"}
    if os.environ.get("RGA_NO_CPU"):  # A/B timing runs: the GPU legs only
        print(json.dumps({"ms_per_step": round(dt * 1e3, 3), "value": round(n / dt, 1), "grouped": grouped}))
        return
    from oracle import oracle
    m = min(n, 1_000_000)
    sel = b.list_id < np.uint32(max(1, nl * m // n))
    t1 = time.perf_counter()
    oracle.rga(nl, b.list_id[sel], b.op[sel], b.value[sel], b.anchor[sel], b.t[sel], b.author[sel],
               b.opid_hi[sel], b.opid_lo[sel])
    ct = time.perf_counter() - t1
    gbs = 45 * n / dt / 1e9
    print(json.dumps({"metric": "RGA replay throughput (events/s), 10M events over 50k lists",
                      "value": round(n / dt, 1), "unit": "events/s", "ms_per_step": round(dt * 1e3, 3),
                      "survivors": int(counts.item()),
                      "roofline": {"bound": "hbm", "bytes_per_event": 45, "achieved": round(gbs, 1),
                                   "peak": 8000.0, "unit": "GB/s", "frac": round(gbs / 8000.0, 4)},
                      "grouped": grouped,
                      "cpu_baseline": {"value": round(int(sel.sum()) / ct, 1), "unit": "events/s",
                                       "cores": 1, "kind": "port",
                                       "sample": f"{int(sel.sum())} events of the first lists, oracle/crdt_ref.c"}}))


if __name__ == "__main__":
    main()
