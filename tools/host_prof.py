#!/usr/bin/env python3
"""Host time per code section of the C1 driver (diagnostic build with
-DPSF_HOST_PROF, tools/variants/hprof/libpsf.so): runs `bench.py --config c1`'s
workload and prints microseconds per step for each instrumented section."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PSF_LIBRARY_VARIANT", os.path.join(ROOT, "tools", "variants", "hprof", "libpsf.so"))
sys.path.insert(0, ROOT)
NAMES = {0: "copy tmpl->msg", 1: "encode_batch", 2: "enc sig launch", 3: "enc FF", 4: "enc KC finish",
         5: "copy delivered", 6: "decode_batch", 7: "dec FF", 8: "dec KC", 9: "ff_encode_batch_launch",
         10: "ff_decode_batch_launch", 11: "crc32c_batch_launch", 12: "presign", 13: "presign_launch (next)",
         14: "iteration (all)"}


def main():
    import bench
    from parameter_server_amd import _lib
    from parameter_server_amd import filter as F
    import torch
    L = _lib.lib()
    fn = L.psf_debug_host_prof
    fn.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int]
    ns, n = (C.c_int64 * 16)(), (C.c_int64 * 16)()
    ctx = F.Context(0)
    F.set_clock(12345)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    a = bench.parse(["--config", "c1"] + sys.argv[1:])
    run, payload, nloc, extra = bench.build_workload(a, F, ctx, 0, 1, "cuda:0", g, a.n)
    run(20)
    torch.cuda.synchronize()
    fn(ns, n, 1)
    steps = 200 if a.config == "c1" else 40
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e6
    fn(ns, n, 1)
    print(f"step {dt:.1f} us")
    if a.config in ("c4", "c5"):
        NAMES.update({0: "router decode_batch", 1: "router prefetch (slice_begin)", 5: "router decode finish",
                      12: "router slice_end", 13: "router encode_batch", 15: "router encode finish"})
    for i in range(16):
        if n[i]:
            print(f"{NAMES.get(i, i):28s} {ns[i] / steps / 1e3:8.2f} us/step  calls/step {n[i] / steps:.1f}")


if __name__ == "__main__":
    main()
