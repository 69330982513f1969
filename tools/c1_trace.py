"""Per-workgroup timeline of one fused min/max + encode launch (C1's batched
small-message path, ff_fused_batch), from a -DPSF_WG_TRACE build of libpsf:

    tools/build_variants.sh trace -DPSF_WG_TRACE
    PSF_LIBRARY_VARIANT=tools/variants/trace/libpsf.so python tools/c1_trace.py

Runs bench.py's C1 workload, arms the stamp buffer, runs one step and prints,
for the step's last fused launch, when the workgroups started, how long their
min/max items, the hand-off wait, the fold and their tiles took (10 ns ticks of
s_memrealtime), and the start / finish counts over time.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
import parameter_server_amd.filter as F  # noqa: E402
from parameter_server_amd import _lib  # noqa: E402


def main():
    args = bench.parse(["--config", "c1"] + sys.argv[1:])
    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ctx = F.Context(0)
    F.set_clock(12345)
    # the stamp buffer is armed before the first launch (a trace build's
    # kernels skip their stamps while it is null)
    buf = torch.zeros(8 * 16384, dtype=torch.int64, device=dev)
    L = _lib.lib()
    L.psf_debug_wg_trace.argtypes = [ctypes.c_void_p]
    assert L.psf_debug_wg_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    torch.cuda.synchronize()
    run, _, n, _ = bench.build_workload(args, F, ctx, 0, 1, dev, g, None)
    run(20)
    torch.cuda.synchronize()
    buf.zero_()
    torch.cuda.synchronize()
    run(1)
    torch.cuda.synchronize()
    tr = buf.cpu().numpy().view(np.uint64).reshape(-1, 8)
    grid = int(np.nonzero(tr[:, 2])[0].max()) + 1
    tr = tr[:grid].astype(np.int64)
    s0, e1 = tr[:, 0].min(), tr[:, 2].max()
    enc = tr[:, 1] != 0
    print(f"grid {grid}: {int((~enc).sum())} decode, {int(enc.sum())} encode workgroups; span {(e1 - s0) * 0.01:.2f} us")

    def pct(name, v):
        v = np.sort(v * 0.01)
        q = lambda f: v[int(f * (len(v) - 1))]  # noqa: E731
        print(f"  {name:<10} p0 {q(0):6.2f} p10 {q(.1):6.2f} p50 {q(.5):6.2f} p90 {q(.9):6.2f} max {q(1):6.2f}")
    d = tr[~enc]
    if len(d):
        print("decode workgroups")
        pct("start", d[:, 0] - s0)
        pct("total", d[:, 2] - d[:, 0])
    e = tr[enc]
    print("encode workgroups")
    pct("start", e[:, 0] - s0)
    # (a stamp older than the workgroup's entry is a previous launch's)
    has = e[:, 4] > e[:, 0]
    if has.any():
        own = has & (e[:, 6] > e[:, 0]) & (e[:, 7] > e[:, 6])
        if own.any():
            pct("claim", e[own, 6] - e[own, 0])
            pct("own run", e[own, 7] - e[own, 6])
            pct("rest", e[own, 4] - e[own, 7])
        pct("items", e[has, 4] - e[has, 0])
        pct("wait", e[has, 5] - e[has, 4])
        pct("fold", e[has, 1] - e[has, 5])
    pct("to q", e[:, 1] - e[:, 0])
    pct("tiles", e[:, 2] - e[:, 1])
    pct("total", e[:, 2] - e[:, 0])
    for t in np.arange(0, (e1 - s0) * 0.01 + 1.0, 1.0):
        st = int(((tr[:, 0] - s0) * 0.01 <= t).sum())
        fi = int(((tr[:, 2] - s0) * 0.01 <= t).sum())
        print(f"  t {t:5.1f} us: started {st:5d} finished {fi:5d}")


if __name__ == "__main__":
    main()
