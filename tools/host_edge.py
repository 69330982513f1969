#!/usr/bin/env python3
"""Host-edge (PCIe-inclusive) rate of the filter path (BASELINE north_star:
"the rate including H2D and D2H copies is also measured").

The reference's messages start and end in host memory: the worker's value
arrays are SArrays in host RAM, the encoded arrays leave through ZeroMQ frames
(van.cc:122-191), the server receives frames in host RAM (van.cc:244-255) and its
decoded arrays land in host RAM.  One step here does exactly that with pinned
host buffers:

  H2D values -> encode (HBM) -> D2H encoded frame      (worker)
  H2D frame  -> decode (HBM) -> D2H decoded values     (server)

through libpsf's RemoteNode with host-resident message buffers (the library
stages them into HBM; see Context::to_device).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 27)
    ap.add_argument("--nb", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import LOC_HOST

    ctx = F.Context(0)
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    F.set_clock(12345)
    x = torch.randn(a.n, generator=torch.Generator().manual_seed(1)).pin_memory()
    frame = torch.empty(a.n * a.nb, dtype=torch.uint8).pin_memory()
    out = torch.empty(a.n, dtype=torch.float32).pin_memory()

    def step():
        m = F.Message(request=True, push=True)
        m.add_value(x)  # host buffer: staged H2D by the library
        m.add_filter(FIXING_FLOAT, num_bytes=a.nb)
        worker.encode(m)
        p, nb, loc = m.value_ptr(0)
        to_host(frame, p, nb)  # D2H: the frame ZeroMQ would send
        w2 = m.clone()  # the Task (with min/max side-info) as the receiver parses it
        lib_set_host_value(w2, frame, nb)  # ... and the received frame as its value
        server.decode(w2)
        p, nb2, loc = w2.value_ptr(0)
        to_host(out, p, nb2)  # D2H of the decoded values

    def to_host(t, p, nbytes):
        import ctypes as C

        from parameter_server_amd._lib import check, lib
        check(lib().psf_copy_to_host(ctx.h, C.c_void_p(t.data_ptr()), C.c_void_p(p), nbytes))

    def lib_set_host_value(msg, t, nbytes):
        import ctypes as C

        from parameter_server_amd._lib import check, lib
        msg._refs.append(t)
        check(lib().psf_msg_set_value(msg.h, 0, C.c_void_p(t.data_ptr()), nbytes, LOC_HOST))

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    # device-resident reference point: the same chain without the copies
    payload = 4 * a.n
    pcie_bytes = 4 * a.n + a.n * a.nb + a.n * a.nb + 4 * a.n
    print(json.dumps({
        "what": "host-edge FIXING_FLOAT round trip incl. H2D/D2H (pinned host buffers)",
        "n": a.n, "num_bytes": a.nb, "ms_per_step": round(dt * 1e3, 3),
        "GiBps_payload": round(payload / dt / 2**30, 2),
        "pcie_bytes_per_step": pcie_bytes,
        "pcie_GBps": round(pcie_bytes / dt / 1e9, 2),
    }))


if __name__ == "__main__":
    main()
