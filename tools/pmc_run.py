"""Driver for rocprofv3 --pmc passes: calibration kernels on a known byte count,
then the bench workload.  Run as: rocprofv3 --pmc X -- python3 tools/pmc_run.py"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
CALIB_BYTES = 1 << 30


def main():
    import torch
    so = os.path.join(REPO, "tools", "_build", "libsmx_calib.so")
    lib = ctypes.CDLL(so)
    buf = torch.zeros(CALIB_BYTES, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = lib.smx_calib_run(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(CALIB_BYTES),
                           ctypes.c_void_p(sink.data_ptr()),
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    del buf
    sys.argv = ["bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-pmc", "--no-e2e", "--no-async"] + sys.argv[1:]
    import runpy
    runpy.run_path(os.path.join(REPO, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
