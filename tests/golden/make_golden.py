"""Generate (or --check) the golden fixtures in tests/golden/.

    python tests/golden/make_golden.py           # write the fixtures
    python tests/golden/make_golden.py --check   # regenerate in memory, compare

The reference's filter path cannot be built in this image (it needs glog,
gflags, Eigen and the protobuf runtime), so the fixtures come
from the restatements, cross-checked where the real thing exists here:
  ff_cases.npz / ff_cases.json   FIXING_FLOAT codes, side-info, decoded values
                                 (oracle/psf_port.c; parity unpinned)
  crc32c.npz                     CRC32C vectors from the reference's own
                                 src/util/crc32c.cc (oracle/_ref), = the port
  noise.npz                      NOISE outputs from libstdc++'s own
                                 std::default_random_engine +
                                 std::normal_distribution (oracle/noise_std.cc,
                                 the calls add_noise.h makes), = psf_port.c
  snappy.npz                     snappy 1.1.8 RawCompress outputs from the
                                 library itself (/opt/conda), = snappy_port.c
  snappy_dec.npz                 snappy 1.1.8 RawUncompress verdicts + outputs
                                 on valid and mutated streams, same source
  scenarios.json                 message-sequence records (KEY_CACHING, the
                                 ctr chain, FIXING_FLOAT message rules,
                                 COMPRESSING) of oracle/chain.py
  even_divide.json               Range<Key>::EvenDivide (oracle/slicing.py)
The committed files were first written in round 1 by a harness that compiled
the reference's filter headers against hand-written stand-ins for the types
they need; that harness pins nothing and is gone, and --check shows the
restatements regenerate every file unchanged.
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


def gen_ff(P):
    arrays, meta = {}, []
    for i, c in enumerate(ff_case_list()):
        x = c["x"]
        st, codes, mn, mx = P.ff_encode(x, c["nb"], c["seed"], c["mn"], c["mx"])
        m = dict(name=c["name"], nb=c["nb"], seed=c["seed"], preset_min=c["mn"], preset_max=c["mx"],
                 dtype="f32" if x.dtype == np.float32 else "f64", n=int(x.size))
        arrays[f"x{i}"] = x
        if st != 0:
            m["status"] = "error"
        else:
            st2, dec = P.ff_decode(codes, c["nb"], mn, mx, x.dtype)
            assert st2 == 0, c["name"]
            m["status"] = "ok"
            m["min_bits"] = int(np.float32(mn).view(np.uint32))
            m["max_bits"] = int(np.float32(mx).view(np.uint32))
            arrays[f"codes{i}"] = codes
            arrays[f"dec{i}"] = dec
        meta.append(m)
    return {"ff_cases.npz": arrays, "ff_cases.json": meta}


def gen_crc(P):
    R = oracle.RefCrc32c()  # the reference's crc32c.cc
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
    assert R.crc32c(b"123456789") == 0xE3069283
    return {"crc32c.npz": dict(data=np.concatenate(blobs), offsets=np.array(offs, np.int64),
                               crc=np.array(crcs, np.uint32))}


def gen_noise(P):
    import oracle
    S = oracle.NoiseStd()
    arrays = {}
    for tag, dt in (("f32", np.float32), ("f64", np.float64)):
        for j, (n, mean, sd) in enumerate(((1001, 0.25, 2.0), (64, 0.0, 1.0), (7, -3.0, 0.01))):
            v = np.linspace(-1, 1, n).astype(dt)
            arrays[f"{tag}_{j}_in"] = v
            out = S.add_noise(v, np.float32(mean), np.float32(sd))
            assert out.tobytes() == P.add_noise(v, np.float32(mean), np.float32(sd)).tobytes()
            arrays[f"{tag}_{j}_out"] = out
            arrays[f"{tag}_{j}_param"] = np.array([mean, sd], np.float32)
    return {"noise.npz": arrays}


def gen_snappy(P, S):
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
    arrays = {}
    for k, v in inputs.items():
        out = S.compress(v)
        assert P.snappy_compress(v) == out, k
        arrays[f"{k}_in"] = np.frombuffer(v, np.uint8)
        arrays[f"{k}_out"] = np.frombuffer(out, np.uint8)
    return {"snappy.npz": arrays}


def gen_snappy_malformed(P, S):
    """RawUncompress verdicts of snappy 1.1.8 on valid and mutated streams
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
        r = bytearray(S.compress(b))
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
        st, out = S.uncompress(s, cap=1 << 20)
        assert (st, out) == P.snappy_uncompress(s, cap=1 << 20), s[:16]
        status.append(st)
        outs.append(out)
    off = np.cumsum([0] + [len(s) for s in streams])
    ooff = np.cumsum([0] + [len(o) for o in outs])
    return {"snappy_dec.npz": dict(data=np.frombuffer(b"".join(streams), np.uint8), offsets=off.astype(np.int64),
                                   status=np.array(status, np.int32),
                                   out=np.frombuffer(b"".join(outs), np.uint8),
                                   out_offsets=ooff.astype(np.int64))}


def gen_even_divide():
    """Range<Key>::EvenDivide (range.h:100-107) restated in oracle/slicing.py."""
    from oracle import slicing
    rng = np.random.default_rng(9)
    spaces = [(0, (1 << 64) - 1), (0, 10**9), (5, 5 + 7), (123456789, 1 << 63), ((1 << 64) - 1000, (1 << 64) - 1)]
    for _ in range(20):
        a, b = sorted(int(v) for v in rng.integers(0, 2**63, 2, dtype=np.uint64))
        spaces.append((a, b * 2))
    rows = []
    for (b, e) in spaces:
        for n in (1, 2, 3, 4, 5, 7, 8, 16, 64):
            for i in range(n):
                ob, oe = slicing.even_divide(b, e, n, i)
                rows.append([str(b), str(e), n, i, str(ob), str(oe)])
    return {"even_divide.json": rows}


def gen_scenarios(P):
    from oracle.chain import PortImpl
    impl = PortImpl(P)
    return {"scenarios.json": {
        "key_caching": scenarios.run(impl, scenarios.kc_scenario()),
        "chain_ctr": scenarios.run(impl, scenarios.chain_scenario()),
        "ff_message": scenarios.run(impl, scenarios.ff_message_scenario()),
        "compressing": scenarios.run(impl, scenarios.compress_scenario()),
    }}


def generate(snappy=True):
    P = oracle.Port()
    out = {}
    out.update(gen_ff(P))
    out.update(gen_crc(P))
    out.update(gen_noise(P))
    if snappy:
        S = oracle.Snappy118()
        out.update(gen_snappy(P, S))
        out.update(gen_snappy_malformed(P, S))
    out.update(gen_scenarios(P))
    out.update(gen_even_divide())
    return out


def _same(name, data):
    path = os.path.join(HERE, name)
    if name.endswith(".json"):
        return json.load(open(path)) == json.loads(json.dumps(data))
    old = np.load(path, allow_pickle=False)
    return sorted(old.files) == sorted(data) and all(
        old[k].dtype == np.asarray(data[k]).dtype and old[k].tobytes() == np.asarray(data[k]).tobytes()
        for k in data)


def check(snappy=True):
    """names of the committed fixtures the generators do NOT reproduce"""
    return [name for name, data in generate(snappy).items() if not _same(name, data)]


def main():
    if "--check" in sys.argv:
        bad = check()
        print("all fixtures reproduced" if not bad else f"differ: {bad}")
        sys.exit(1 if bad else 0)
    oracle.build()
    for name, data in generate().items():
        path = os.path.join(HERE, name)
        if name.endswith(".json"):
            with open(path, "w") as f:
                json.dump(data, f, indent=None if name == "even_divide.json" else 1)
        else:
            np.savez_compressed(path, **data)
        print("wrote", name)


if __name__ == "__main__":
    main()
