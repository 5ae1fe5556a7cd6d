"""Diagnostic: slot-staged output payload checks of k_window_f<true> (SMX_DIAG build
with -DWF_OUT2=1): per window, counts of slots whose staged sym / slot kind / inverse
map / element index disagree with the inputs (dbg words 17-20)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from semantic_merge_amd import _lib, synth
    lib = _lib.lib()
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(5000, 50, 1)))
    buf = torch.zeros(24 * 4096, dtype=torch.int64, device="cuda")
    lib.smx_debug_phase_buffer(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(buf.numel() * 8))
    dc = _lib.DeviceCompose(soa)
    dc.run()
    torch.cuda.synchronize()
    lib.smx_debug_phase_buffer(None, ctypes.c_size_t(0))
    d = buf.view(-1, 24).cpu().numpy()
    for w in range(4):
        print(w, "stamps set" if d[w, 0] else "-", "order violations", d[w, 5], "sl/fin", d[w, 17:19].tolist())
    import numpy as np
    from oracle import oracle
    got, ref = dc.results(), oracle.compose(soa)
    for nm, g, r in zip(("order", "addr", "file", "ctx", "conf"), got, ref):
        if g.shape == r.shape and np.array_equal(g, r):
            print(nm, "OK")
            continue
        bad = np.flatnonzero(g.reshape(-1) != r.reshape(-1))
        print(nm, f"{bad.size} differ of {g.size}, first {bad[:4].tolist()} last {bad[-4:].tolist()}")
        if nm == "order":
            i = bad[0]
            print("  got", g[i - 2: i + 12].tolist())
            print("  ref", r[i - 2: i + 12].tolist())
            print("  sets equal:", sorted(g.tolist()) == sorted(r.tolist()))
            print("  kinds of ref[i..]:", soa.kind[r[i: i + 12]].tolist(), "got:", soa.kind[g[i: i + 12]].tolist())
            for x in g[i: i + 4].tolist():
                q = int(np.flatnonzero(r == x)[0])
                print(f"  op {x}: got at {int(np.flatnonzero(g == x)[0])}, ref at {q}, ts {int(soa.ts[x])}, "
                      f"hi32 {int(soa.oid_hi[x]) >> 32:#x}, kind {int(soa.kind[x])}")
            print("  ts got:", [int(soa.ts[x]) % 100000 for x in g[i - 2: i + 10]])
            print("  ts ref:", [int(soa.ts[x]) % 100000 for x in r[i - 2: i + 10]])


if __name__ == "__main__":
    main()
