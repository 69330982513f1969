"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference and oracle/_ref):
    python tests/golden/make_golden.py

Every fixture is produced by oracle/_ref/libpsref.so -- the reference's
unmodified src/filter headers + filter.cc + util/crc32c.cc -- and, before it is
written, re-computed by the plain-C restatement oracle/psf_port.c; any
disagreement aborts.  The fixtures are data only (inputs + expected outputs):
  ff_cases.npz / ff_cases.json   FIXING_FLOAT codes, side-info, decoded values
  crc32c.npz                     CRC32C vectors
  noise.npz                      NOISE outputs (f32, f64)
  snappy.npz                     snappy 1.1.8 RawCompress outputs (COMPRESSING)
  snappy_dec.npz                 snappy 1.1.8 RawUncompress verdicts + outputs on
                                 valid and mutated streams
  scenarios.json                 message-sequence records (KEY_CACHING, chain,
                                 FIXING_FLOAT message rules) from tests/scenarios.py
  even_divide.json               Range<Key>::EvenDivide server ranges (range.h)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
import scenarios  # noqa: E402


def ff_case_list():
    rng = np.random.default_rng(20240601)
    cases = []

    def add(name, x, nb, seed, mn=None, mx=None):
        cases.append(dict(name=name, x=x, nb=nb, seed=seed, mn=mn, mx=mx))

    for dt in (np.float32, np.float64):
        tag = "f32" if dt == np.float32 else "f64"
        x = rng.standard_normal(1027).astype(dt)
        for nb in range(1, 8):
            add(f"{tag}_gauss_nb{nb}", x, nb, 12345)
        add(f"{tag}_preset_clamp_nb1", (rng.standard_normal(515) * 3).astype(dt), 1, 777, -1.0, 1.0)
        add(f"{tag}_preset_clamp_nb3", (rng.standard_normal(515) * 3).astype(dt), 3, 778, -1.0, 1.0)
        add(f"{tag}_min_only_nb2", (rng.standard_normal(257)).astype(dt), 2, 9, -0.25, None)
        add(f"{tag}_max_only_nb2", (rng.standard_normal(257)).astype(dt), 2, 10, None, 0.5)
        for n in (1, 2, 3, 5, 8):
            add(f"{tag}_tiny{n}_nb1", rng.standard_normal(n).astype(dt), 1, 4242)
        add(f"{tag}_const_small", np.full(33, 3.0, dt), 1, 5)
        add(f"{tag}_const_ge32", np.full(33, 40.0, dt), 1, 5)
        add(f"{tag}_uniform_wide_nb2", rng.uniform(-1e4, 1e4, 300).astype(dt), 2, 31337)
        add(f"{tag}_positive_nb1", rng.uniform(5, 6, 300).astype(dt), 1, 1)
        specials = np.array([0.5, np.nan, np.inf, -np.inf, 3.0, -3.0, 1e30, -0.0, 0.0, 0.1,
                             1.0, -1.0], dtype=dt)
        for nb in (1, 2, 3, 4, 5):
            add(f"{tag}_specials_preset_nb{nb}", specials, nb, 99, -1.0, 1.0)
        add(f"{tag}_inf_computed", np.array([1.0, np.inf, 2.0, -5.0], dt), 1, 5)
        add(f"{tag}_neg_inf_computed", np.array([1.0, -np.inf, 2.0], dt), 2, 5)
    for seed in (-1, 0, 2**31 - 1, -2**31, 7, 1697000000):
        add(f"f32_seed{seed}_nb1", rng.standard_normal(300).astype(np.float32), 1, seed)
    add("f64_beyond_f32_range", np.array([1e300, -1e300, 0.0, 1.0], np.float64), 1, 3)
    add("f64_tiny_range", (1.0 + rng.standard_normal(200) * 1e-9).astype(np.float64), 3, 3)
    add("f32_preset_equal_rejected", np.ones(4, np.float32), 1, 3, 2.0, 2.0)
    return cases


def gen_ff(R, P):
    arrays, meta = {}, []
    for i, c in enumerate(ff_case_list()):
        x = c["x"]
        fixed = None if (c["mn"] is None and c["mx"] is None) else (c["mn"], c["mx"])
        r = R.ff_roundtrip(x, c["nb"], c["seed"], fixed=fixed)
        st, codes, mn, mx = P.ff_encode(x, c["nb"], c["seed"], c["mn"], c["mx"])
        m = dict(name=c["name"], nb=c["nb"], seed=c["seed"], preset_min=c["mn"], preset_max=c["mx"],
                 dtype="f32" if x.dtype == np.float32 else "f64", n=int(x.size))
        arrays[f"x{i}"] = x
        if r["status"] != 0:
            assert st != 0, (c["name"], "port accepted what the reference rejected", r)
            m["status"] = "error"
            m["error"] = r.get("error", "")
        else:
            assert st == 0, (c["name"], st)
            assert np.array_equal(r["codes"], codes), c["name"]
            assert np.float32(r["min"]).tobytes() == np.float32(mn).tobytes(), c["name"]
            assert np.float32(r["max"]).tobytes() == np.float32(mx).tobytes(), c["name"]
            st2, dec = P.ff_decode(codes, c["nb"], mn, mx, x.dtype)
            assert st2 == 0 and dec.tobytes() == r["decoded"].tobytes(), c["name"]
            m["status"] = "ok"
            m["min_bits"] = int(np.float32(r["min"]).view(np.uint32))
            m["max_bits"] = int(np.float32(r["max"]).view(np.uint32))
            arrays[f"codes{i}"] = r["codes"]
            arrays[f"dec{i}"] = r["decoded"]
        meta.append(m)
    np.savez_compressed(os.path.join(HERE, "ff_cases.npz"), **arrays)
    with open(os.path.join(HERE, "ff_cases.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"ff_cases: {len(meta)} cases")


def gen_crc(R, P):
    rng = np.random.default_rng(7)
    lens = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 100, 255, 256, 1000,
            2047, 2048, 2049, 4096, 10000, 65537]
    blobs, crcs, offs = [], [], [0]
    for n in lens:
        b = rng.integers(0, 256, n, dtype=np.uint8)
        c = R.crc32c(b.tobytes())
        assert c == P.crc32c(b.tobytes())
        blobs.append(b)
        crcs.append(c)
        offs.append(offs[-1] + n)
    check = R.crc32c(b"123456789")
    assert check == 0xE3069283
    np.savez_compressed(os.path.join(HERE, "crc32c.npz"), data=np.concatenate(blobs),
                        offsets=np.array(offs, np.int64), crc=np.array(crcs, np.uint32))
    print(f"crc32c: {len(lens)} vectors")


def gen_noise(R, P):
    import ctypes as C
    L = R.lib
    arrays = {}
    for tag, dt, code in (("f32", np.float32, 9), ("f64", np.float64, 10)):
        for j, (n, mean, sd) in enumerate(((1001, 0.25, 2.0), (64, 0.0, 1.0), (7, -3.0, 0.01))):
            v = np.linspace(-1, 1, n).astype(dt)
            node = L.psref_node_new()
            m = R.msg_new()
            L.psref_msg_add_value(m, v.ctypes.data_as(C.c_void_p), v.nbytes, code)
            fi = L.psref_msg_add_filter(m, 4)
            L.psref_fc_set_noise(m, fi, mean, sd)
            assert L.psref_node_encode(node, m) == 0
            out = R.msg_values(m)[0].view(dt)
            assert out.tobytes() == P.add_noise(v, mean, sd).tobytes()
            arrays[f"{tag}_{j}_in"] = v
            arrays[f"{tag}_{j}_out"] = out
            arrays[f"{tag}_{j}_param"] = np.array([mean, sd], np.float32)
            L.psref_msg_free(m)
            L.psref_node_free(node)
    np.savez_compressed(os.path.join(HERE, "noise.npz"), **arrays)
    print("noise: ok")


def gen_snappy(R):
    rng = np.random.default_rng(5)
    inputs = {
        "random": rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(),
        "zeros": bytes(100000),
        "pattern": (b"parameter_server " * 5000),
        "ff_codes": oracle.Port().ff_encode(rng.standard_normal(70000).astype(np.float32), 1, 1)[1].tobytes(),
        "sorted_keys": scenarios.sorted_keys(20000, 3).tobytes(),
        "floats": rng.standard_normal(30000).astype(np.float32).tobytes(),
        "tiny": b"abc",
        "one": b"\x00",
        "long_run_after_literal": b"xy" + bytes(70000) + b"z" * 10,
    }
    for n in (15, 16, 4096, 65535, 65536, 65537, 131072 + 100):
        inputs[f"keys_{n}"] = scenarios.sorted_keys(n // 8 + 1, n).tobytes()[:n]
        if n in (15, 16, 4096, 65537):
            inputs[f"random_{n}"] = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    inputs["runs"] = np.repeat(rng.integers(0, 256, 3000, dtype=np.uint8), rng.integers(1, 200, 3000)).tobytes()
    P = oracle.Port()
    arrays = {}
    for k, v in inputs.items():
        out = R.snappy_compress(v)
        assert P.snappy_compress(v) == out, k
        arrays[f"{k}_in"] = np.frombuffer(v, np.uint8)
        arrays[f"{k}_out"] = np.frombuffer(out, np.uint8)
    np.savez_compressed(os.path.join(HERE, "snappy.npz"), **arrays)
    print(f"snappy: {len(inputs)} vectors (snappy 1.1.8)")
    gen_snappy_malformed(R, P)


def gen_snappy_malformed(R, P):
    """RawUncompress verdicts of the reference's snappy on mutated streams
    (the decoder's CHECK paths: shared_array_inl.h:236,240)."""
    rng = np.random.default_rng(11)
    streams, status, outs = [], [], []
    srcs = [lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
            lambda n: scenarios.sorted_keys(n // 8 + 1, n).tobytes()[:n],
            lambda n: np.repeat(rng.integers(0, 4, n // 9 + 1, dtype=np.uint8), 9).tobytes()[:n]]
    hand = [b"", b"\x80", b"\xff\xff\xff\xff\x1f", b"\xff\xff\xff\xff\x0f", b"\x05\x10abcde",
            b"\x05\x10abcd", b"\x04\x01\x00", b"\x04\x00a\x01\x00", b"\x04\x00a\x01\x01",
            b"\x05\x00a\x0d\x01", b"\x02\x00a", b"\x01\x04ab", b"\x03\xf0\x02\x00\x00abc",
            b"\x0a\x00a\x0a\x01\x00", b"\x08\x00a\x12\x01\x00\x00\x00"]
    for h in hand:
        streams.append(h)
    for t in range(400):
        b = srcs[t % 3](int(rng.integers(0, 2500)))
        r = bytearray(R.snappy_compress(b))
        for _ in range(int(rng.integers(0, 3))):
            if not r:
                break
            i, op = int(rng.integers(0, len(r))), int(rng.integers(0, 4))
            if op == 0:
                r[i] = int(rng.integers(0, 256))
            elif op == 1:
                del r[i]
            elif op == 2:
                r.insert(i, int(rng.integers(0, 256)))
            else:
                del r[i:]
        streams.append(bytes(r))
    for s in streams:
        st, out = R.snappy_uncompress(s, cap=1 << 20)
        assert (st, out) == P.snappy_uncompress(s, cap=1 << 20), s[:16]
        status.append(st)
        outs.append(out)
    off = np.cumsum([0] + [len(s) for s in streams])
    ooff = np.cumsum([0] + [len(o) for o in outs])
    np.savez_compressed(os.path.join(HERE, "snappy_dec.npz"),
                        data=np.frombuffer(b"".join(streams), np.uint8), offsets=off.astype(np.int64),
                        status=np.array(status, np.int32),
                        out=np.frombuffer(b"".join(outs), np.uint8), out_offsets=ooff.astype(np.int64))
    print(f"snappy_dec: {len(streams)} streams, {sum(1 for s in status if s == 0)} valid")


def gen_even_divide():
    """Range<Key>::EvenDivide from the reference's own range.h
    (oracle/_ref/libpsrange.so), checked against oracle/slicing.py."""
    import ctypes as C

    from oracle import slicing
    L = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libpsrange.so"))
    L.psref_even_divide.argtypes = [C.c_uint64] * 4 + [C.POINTER(C.c_uint64)] * 2
    rng = np.random.default_rng(9)
    spaces = [(0, (1 << 64) - 1), (0, 10**9), (5, 5 + 7), (123456789, 1 << 63), ((1 << 64) - 1000, (1 << 64) - 1)]
    for _ in range(20):
        a, b = sorted(int(v) for v in rng.integers(0, 2**63, 2, dtype=np.uint64))
        spaces.append((a, b * 2))
    rows = []
    for (b, e) in spaces:
        for n in (1, 2, 3, 4, 5, 7, 8, 16, 64):
            for i in range(n):
                ob, oe = C.c_uint64(), C.c_uint64()
                assert L.psref_even_divide(b, e, n, i, C.byref(ob), C.byref(oe)) == 0
                assert slicing.even_divide(b, e, n, i) == (ob.value, oe.value), (b, e, n, i)
                rows.append([str(b), str(e), n, i, str(ob.value), str(oe.value)])
    with open(os.path.join(HERE, "even_divide.json"), "w") as f:
        json.dump(rows, f)
    print(f"even_divide: {len(rows)} rows")


def gen_scenarios(R):
    impl = scenarios.RefImpl(R)
    out = {
        "key_caching": scenarios.run(impl, scenarios.kc_scenario()),
        "chain_ctr": scenarios.run(impl, scenarios.chain_scenario()),
        "ff_message": scenarios.run(impl, scenarios.ff_message_scenario()),
        "compressing": scenarios.run(impl, scenarios.compress_scenario()),
    }
    with open(os.path.join(HERE, "scenarios.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("scenarios:", {k: len(v) for k, v in out.items()})


def main():
    oracle.build(ref=True)
    R, P = oracle.Ref(), oracle.Port()
    gen_ff(R, P)
    gen_crc(R, P)
    gen_noise(R, P)
    gen_snappy(R)
    gen_scenarios(R)
    gen_even_divide()


if __name__ == "__main__":
    main()
