"""Microbenchmark of k_emit's access pattern (see emit_micro.hip).

    python tools/emit_micro.py [--n 100000000]

Prints one line per (variant, table size): ms per launch and the stream rate.
"""
import argparse
import ctypes as C
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "stream 2r/4w SoA, no gather", 1: "SoA + 16B gather", 2: "AoS int4 out + gather",
         3: "SoA + gather, outputs shifted by 1", 4: "4/lane int4 loads + AoS out + gather",
         5: "SoA + 8B packed gather (8 MB at 2^20)", 6: "SoA + 4B gather (4 MB at 2^20)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(HERE, "_build", "libsmx_emit_micro.so"))
    lib.micro_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int64] + \
        [C.c_void_p] * 5 + [C.c_void_p]
    n = a.n // 4 * 4
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    order = torch.randint(0, n, (n,), device=dev, dtype=torch.int32, generator=g)
    sym = torch.randint(0, 2**31 - 1, (n,), device=dev, dtype=torch.int32, generator=g)
    fin = torch.randint(0, 2**31 - 1, (1 << 20, 4), device=dev, dtype=torch.int32, generator=g)
    outs = [torch.empty(n + 1, device=dev, dtype=torch.int32) for _ in range(4)]
    oa = torch.empty((n + 1, 4), device=dev, dtype=torch.int32)
    st = torch.cuda.current_stream(dev).cuda_stream
    for bits in (20, 17):
        for v in range(7):
            args = [v, order.data_ptr(), sym.data_ptr(), fin.data_ptr(), (1 << bits) - 1, n] + \
                [o.data_ptr() for o in outs] + [oa.data_ptr(), st]
            for _ in range(3):
                assert lib.micro_run(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                lib.micro_run(*args)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            hbm = n * (8 + 16)
            print(f"table 2^{bits} v{v} {NAMES[v]:40s} {ms:7.3f} ms  {hbm / ms / 1e6:7.0f} GB/s (24 B/op stream)",
                  flush=True)


if __name__ == "__main__":
    main()
