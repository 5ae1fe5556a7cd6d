"""Per-phase latency of k_window_f (diagnostic build path k_window_f<true>): lane 0 of
each workgroup stamps s_memtime after every barrier; this prints the mean cycles of
each phase per window, and the window-kernel time with and without stamping."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
NST = 24
NAMES = {0: "start", 1: "load", 3: "check+merge", 4: "msplit", 6: "ccnt-scan",
         7: "scatter", 8: "gbits", 9: "keys", 10: "rank", 21: "tiechk+renrank",
         11: "tiefix", 12: "rc-scan", 13: "stage1+posl", 14: "flags+cand", 15: "write1",
         16: "stage2+write2"}
ORDER = [0, 1, 3, 4, 6, 7, 8, 9, 10, 21, 11, 12, 13, 14, 15, 16]


def main():
    import torch
    from semantic_merge_amd import _lib, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    spec = synth.LiftSpec(**{**synth.CONFIGS[cfg].__dict__, "n_total": n})
    soa = synth.lift_soa(synth.lift_logs(spec))
    dc = _lib.DeviceCompose(soa)
    lib = _lib.lib()
    W = n // 256 + 16
    buf = torch.zeros(W * NST, dtype=torch.int64, device="cuda")

    def timed(reps=5):
        lib.smx_reset_stage_times()
        lib.smx_set_profiling(1)
        for _ in range(reps):
            dc.run()
        torch.cuda.synchronize()
        lib.smx_set_profiling(0)
        ms, calls = _lib.stage_times()["window"]
        return ms / max(calls, 1)

    dc.run()
    print(f"window plain   {timed():.3f} ms  (median of 3: {sorted(timed() for _ in range(3))[1]:.3f})")
    try:
        lib.smx_debug_phase_buffer
    except AttributeError:
        return
    lib.smx_debug_phase_buffer(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(buf.numel() * 8))
    dc.run()
    print(f"window stamped {timed():.3f} ms")
    buf.zero_()
    dc.run()
    torch.cuda.synchronize()
    lib.smx_debug_phase_buffer(None, ctypes.c_size_t(0))
    a = buf.cpu().numpy().reshape(-1, NST)
    a = a[a[:, 16] != 0]
    print(f"{len(a)} windows stamped")
    tot = (a[:, 16] - a[:, 0]).mean()
    prev = 0
    for i in ORDER[1:]:
        d = (a[:, i] - a[:, prev]).mean()
        print(f"  {NAMES[i]:10s} {d:9.0f} cyc  {100 * d / tot:5.1f}%")
        prev = i
    print(f"  {'total':10s} {tot:9.0f} cyc per window (lane-0 view)")
    st = np.sort(a[:, 0])
    print(f"  window start span {(st[-1] - st[0]):.0f} cyc; concurrent ~ {tot * len(a) / (a[:, 16].max() - st[0]):.0f} windows")


if __name__ == "__main__":
    main()
