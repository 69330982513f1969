"""GPU: the caching allocator is bounded (one cap per device).

A long-running server sees many distinct message sizes; the buffers its
codecs release stay cached for reuse only up to the context's cap (HBM and
pinned host memory), the least recently released going first.  Cycling 1000
distinct message sizes through a FIXING_FLOAT encode + decode keeps the cache
under the cap, every round trip stays bit-exact, and the cap is reported
(psf_context_memory_stats).  Reference: key_caching.h:69-70 keeps one cache
entry per (channel, key range), fixing_float.h:37-44 allocates a new output
per array -- the allocation pattern being bounded here."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_cache_bounded_over_1000_sizes(port):
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    ctx = F.Context(0, stream=torch.cuda.Stream())
    st = ctx.memory_stats()
    assert st["hbm_cap"] == 8 << 30 and st["pinned_cap"] == 1 << 30
    cap = 64 << 20
    ctx.set_cache_limit(cap, 16 << 20)  # the device's cap: every context on device 0
    assert F.device_memory_stats(0)["hbm_cap"] == cap
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    big = torch.randn(10_000_000, device="cuda")
    torch.cuda.synchronize()  # (big is written on torch's stream; the context runs on its own)
    F.set_clock(7)
    try:
        peak_alloc = 0
        for i in range(1000):
            n = (1 << 18) + i * 9001 + (i % 7)  # 1000 distinct sizes, 0.25 M .. 9.3 M values
            m = F.Message(request=True, push=True)
            m.add_value(big[:n])
            m.add_filter(FIXING_FLOAT, num_bytes=1)
            worker.encode(m)
            w = m.clone()
            server.decode(w)
            if i % 97 == 0:  # spot-check the values against the restatement
                codes = worker.value(m, 0).cpu().numpy()
                x = big[:n].cpu().numpy()
                s, pc, mn, mx = port.ff_encode(x, 1, 7)
                assert s == 0 and np.array_equal(codes, pc), i
                s, pd = port.ff_decode(pc, 1, mn, mx, np.float32)
                assert server.value(w, 0).cpu().numpy().tobytes() == pd.tobytes(), i
            del m, w
            st = ctx.memory_stats()
            assert st["hbm_cached"] <= cap, (i, st)
            assert F.device_memory_stats(0)["hbm_cached"] <= cap, i
            peak_alloc = max(peak_alloc, st["hbm_allocated"])
        ctx.sync()
        st = ctx.memory_stats()
        assert st["hbm_cached"] <= cap and st["hbm_evictions"] > 0, st
        # everything the messages held is back: allocated == cached (nothing live)
        assert st["hbm_allocated"] == st["hbm_cached"], st
        # live buffers of one round trip (codes n + decoded 4n bytes, < 48 MiB)
        # plus the capped cache
        assert peak_alloc <= cap + (48 << 20), peak_alloc
        ctx.set_cache_limit(0, 0)
        st = ctx.memory_stats()
        assert st["hbm_cached"] == 0 and st["hbm_allocated"] == 0 and st["pinned_cached"] == 0, st
    finally:
        F.set_clock(None)
        F.set_device_cache_limit(0, *F.DEFAULT_CACHE_LIMIT)
