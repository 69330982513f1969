#!/usr/bin/env python3
"""Diagnostic: sample the host side of `bench.py --config c1`'s driver loop
(tools/libsampler.so, SIGPROF every 50 us on the calling thread) and write the
raw samples to gpurun_out/host_samples.txt for tools/sampler_report.py."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from parameter_server_amd import filter as F
    import torch
    S = C.CDLL(os.path.join(ROOT, "tools", "libsampler.so"))
    S.sampler_stop.argtypes = [C.c_char_p]
    ctx = F.Context(0)
    F.set_clock(12345)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    a = bench.parse(["--config", "c1"] + sys.argv[1:])
    run, payload, nloc, extra = bench.build_workload(a, F, ctx, 0, 1, "cuda:0", g, a.n)
    run(50)
    torch.cuda.synchronize()
    steps = 10000
    S.sampler_start(50)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e6
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    n = S.sampler_stop(os.path.join(ROOT, "gpurun_out", "host_samples.txt").encode())
    import shutil  # the library the addresses belong to, for the report
    shutil.copy(os.path.join(ROOT, "parameter_server_amd", "libpsf.so"), os.path.join(ROOT, "gpurun_out", "host_samples_libpsf.so"))
    print(f"step {dt:.1f} us, {n} samples")


if __name__ == "__main__":
    main()
