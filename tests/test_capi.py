"""CPU: the C-ABI library (libpsf.so) loads, exports exactly what
include/psf.h declares, and its host logic (Message/Task/FilterConfig model,
RemoteNode chain order, KEY_CACHING state machine on host-resident keys) matches
the reference's recorded behaviour.  No kernel is launched here."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def _header_symbols():
    hdr = open(os.path.join(ROOT, "include", "psf.h")).read()
    return set(re.findall(r"\b(psf_[a-z0-9_]+)\s*\(", hdr))


def test_library_exports_every_declared_symbol():
    from parameter_server_amd import _lib
    so = _lib.LIB_PATH
    assert os.path.exists(so), "libpsf.so not built"
    out = subprocess.check_output(["nm", "-D", "--defined-only", so]).decode()
    exported = {line.split()[-1] for line in out.splitlines()}
    declared = _header_symbols()
    assert len(declared) >= 30
    assert declared <= exported, sorted(declared - exported)
    # the ctypes binding covers the same surface
    assert set(_lib.SIGNATURES) == declared


def test_library_loads_and_is_hip():
    import parameter_server_amd as p
    L = p.lib()
    assert b"gfx950" in L.psf_version()
    out = subprocess.check_output(["ldd", p._lib.LIB_PATH]).decode()
    assert "libamdhip64" in out


def test_header_constants_match_binding():
    from parameter_server_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "psf.h")).read()
    consts = dict(re.findall(r"#define (PSF_[A-Z0-9_]+) \(?(-?\d+)\)?", hdr))
    assert int(consts["PSF_ERR_BIN"]) == _lib.PSF_ERR_BIN
    assert int(consts["PSF_ERR_NBYTES"]) == _lib.PSF_ERR_NBYTES
    assert int(consts["PSF_FIXING_FLOAT"]) == _lib.FIXING_FLOAT
    assert int(consts["PSF_DT_FLOAT"]) == _lib.DT_FLOAT


def test_message_model_host_only():
    from parameter_server_amd import filter as F
    m = F.Message(request=True, push=True, key_channel=5, key_range=(10, 20))
    i = m.add_filter(3, num_bytes=2, fixed_point=[(-1.0, 1.0), (None, 2.0)])
    assert i == 0
    assert m.fixed_points(0) == [(True, -1.0, True, 1.0), (False, -1.0, True, 2.0)]
    assert m.add_filter(1, clear_cache_if_done=True) == 1
    assert m.signature(1) == (False, 0)
    with pytest.raises(F.PsfError):
        m.add_filter(9)  # filter.cc:19-20 unknown type
    c = m.clone()
    assert c.fixed_points(0) == m.fixed_points(0)
    assert c.num_values() == 0


def test_key_caching_host_keys_matches_restatement(scenario_golden):
    """KEY_CACHING on host-resident keys (host-only context, no GPU)."""
    import scenarios
    got = scenarios.run(scenarios.PsfImpl(device=None), scenarios.kc_scenario())
    want = scenario_golden["key_caching"]
    assert [g["name"] for g in got] == [w["name"] for w in want]
    for g, w in zip(got, want):
        assert g == w, (g["name"], g, w)


def test_fixing_float_needs_device_context():
    import torch
    from parameter_server_amd import filter as F
    ctx = F.HostContext()
    node = F.RemoteNode(ctx)
    m = F.Message()
    m.add_value(torch.ones(8))
    m.add_filter(3, num_bytes=1)
    with pytest.raises(F.PsfError):
        node.encode(m)


def test_default_device_knob():
    """psf_default_device: the device the reference-side adapter's contexts
    use (PSF_DEVICE, else 0; psf_set_default_device overrides)."""
    import subprocess
    import sys
    code = ("import parameter_server_amd as p; L = p.lib(); print(L.psf_default_device()); "
            "print(L.psf_set_default_device(-1) < 0, L.psf_set_default_device(3), L.psf_default_device())")
    env = dict(os.environ, PSF_DEVICE="5")
    out = subprocess.check_output([sys.executable, "-c", code], cwd=ROOT, env=env).decode().split()
    assert out == ["5", "True", "0", "3"]
    for bad in ("junk", "1 ", "-1"):  # malformed: device 0, with a warning on stderr
        env["PSF_DEVICE"] = bad
        r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
        assert r.returncode == 0 and r.stdout.split()[0] == "0"
        assert "PSF_DEVICE" in r.stderr and "warning" in r.stderr


def test_context_outlives_its_users_whatever_the_destroy_order():
    """A binding may finalise handles in any order (a garbage collector
    clearing a cycle): destroying the context before its node and router
    leaves them usable until they go, and nothing is freed twice."""
    import ctypes as C

    import numpy as np
    import torch

    from parameter_server_amd import KEY_CACHING, lib, shard
    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import check
    L = lib()
    ctx = F.HostContext()
    node = F.RemoteNode(ctx)
    router = shard.PushRouter(ctx, shard.server_ranges(3), 0, 1)
    keys = np.arange(0, 3000, 3, dtype=np.uint64) << np.uint64(50)
    m = F.Message(request=True, push=True, key_channel=4, key_range=shard.KEY_ALL)
    m.set_key(torch.from_numpy(keys.view(np.int64).copy()))
    m.add_filter(KEY_CACHING)
    check(L.psf_context_destroy(ctx.h))  # the handle goes first
    ctx.h = C.c_void_p()
    router.step({4: m})  # still alive through the router's reference
    assert len(router.results()) == 3
    node.encode(m)
    check(L.psf_router_destroy(router.h))
    router.h = None
    check(L.psf_node_destroy(node.h))  # the last user: the context goes now
    node.h = None
