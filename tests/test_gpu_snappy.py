"""GPU: the COMPRESSING codec (snappy 1.1.8 raw format) through the C ABI.

Compress must be byte-identical to snappy 1.1.8 (tests/golden/snappy.npz from
the reference's libsnappy; the C restatement oracle/snappy_port.c for larger
seeded inputs).  Uncompress must reproduce RawUncompress's verdict and output
on valid and mutated streams (tests/golden/snappy_dec.npz), including valid
streams that no 1.1.8 encoder writes (literals and copies across 64 KiB output
fragments: the one-lane path)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _dev(b: bytes, offset: int = 0) -> torch.Tensor:
    a = np.frombuffer(b"\0" * offset + b, dtype=np.uint8).copy()
    return torch.from_numpy(a).cuda()[offset:]


def _inputs(rng, n, kind):
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "keys":
        return np.sort(rng.integers(0, 10**9, n // 8 + 1, dtype=np.uint64)).tobytes()[:n]
    if kind == "codes":
        return np.clip(rng.standard_normal(n) * 30 + 128, 0, 255).astype(np.uint8).tobytes()
    if kind == "runs":
        return np.repeat(rng.integers(0, 256, n // 50 + 1, dtype=np.uint8),
                         50).tobytes()[:n]
    if kind == "zeros":
        return bytes(n)
    if kind == "alpha4":  # short matches everywhere, many same-hash probes in a skip step
        return rng.integers(0, 4, n, dtype=np.uint8).tobytes()
    if kind == "periodic":  # long copies (>= 64 bytes: several match-length rounds)
        p = rng.integers(0, 256, int(rng.integers(5, 300)), dtype=np.uint8)
        x = np.resize(p, n)
        x[rng.integers(0, max(n, 1), n // 500 + 1)] ^= 1  # sparse breaks
        return x.tobytes()
    if kind == "text":
        words = [b"param", b"server", b"filter", b"key", b"value", b"  ", b"\n"]
        return b"".join(words[i] for i in rng.integers(0, len(words), n // 4 + 1))[:n]
    raise ValueError(kind)


def test_compress_matches_snappy_1_1_8_fixtures(ctx):
    a = np.load(os.path.join(GOLDEN, "snappy.npz"), allow_pickle=False)
    names = sorted(k[:-3] for k in a.files if k.endswith("_in"))
    assert len(names) >= 20
    for k in names:
        x, want = a[f"{k}_in"].tobytes(), a[f"{k}_out"].tobytes()
        got = ctx.snappy_compress(_dev(x)).cpu().numpy().tobytes()
        assert got == want, k
        back = ctx.snappy_uncompress(_dev(want)).cpu().numpy().tobytes()
        assert back == x, k


@pytest.mark.parametrize("kind", ["random", "keys", "codes", "runs", "zeros", "text", "alpha4", "periodic"])
def test_compress_random_sizes_vs_port(ctx, port, kind):
    rng = np.random.default_rng(len(kind) * 7 + ord(kind[0]))
    for n in [1, 14, 15, 16, 17, 63, 64, 65, 255, 256, 257, 4095, 65535, 65536, 65537, 300001, 3 << 20]:
        x = _inputs(rng, n, kind)
        want = port.snappy_compress(x)
        got = ctx.snappy_compress(_dev(x)).cpu().numpy().tobytes()
        assert got == want, (kind, n)
        back = ctx.snappy_uncompress(_dev(want)).cpu().numpy().tobytes()
        assert back == x, (kind, n)


def test_compress_unaligned_input(ctx, port):
    rng = np.random.default_rng(5)
    x = _inputs(rng, 200003, "keys")
    for off in (1, 3, 4, 8, 13):
        got = ctx.snappy_compress(_dev(x, off)).cpu().numpy().tobytes()
        assert got == port.snappy_compress(x), off


def test_compress_many_fragments_mixed_vs_port(ctx, port):
    """64 MiB = 1024 fragments (several per persistent workgroup, more than can
    be resident at once) alternating incompressible and compressible blocks of
    odd lengths, so fragment offsets in the stream land on every residue mod 4,
    into output buffers at byte offsets 0..3: byte-identical to 1.1.8."""
    rng = np.random.default_rng(77)
    parts, n = [], 0
    kinds = ("random", "codes", "keys", "runs", "text")
    while n < (64 << 20):
        b = _inputs(rng, int(rng.integers(30000, 300000)), kinds[len(parts) % len(kinds)])
        parts.append(b)
        n += len(b)
    x = b"".join(parts)[:64 << 20]
    want = port.snappy_compress(x)
    xd = _dev(x)
    cap = len(x) + len(x) // 6 + 32
    for off in (0, 1, 2, 3):
        buf = torch.zeros(cap + 4, dtype=torch.uint8, device="cuda")
        got = ctx.snappy_compress(xd, out=buf[off:]).cpu().numpy().tobytes()
        assert got == want, off
    back = ctx.snappy_uncompress(_dev(want)).cpu().numpy().tobytes()
    assert back == x


def test_decoder_verdicts_match_snappy_1_1_8(ctx):
    from parameter_server_amd._lib import PSF_ERR_CHECK, PsfError
    a = np.load(os.path.join(GOLDEN, "snappy_dec.npz"), allow_pickle=False)
    d, off, st, out, ooff = a["data"], a["offsets"], a["status"], a["out"], a["out_offsets"]
    nbad = 0
    for i in range(len(st)):
        s = d[off[i]:off[i + 1]].tobytes()
        want = out[ooff[i]:ooff[i + 1]].tobytes()
        if st[i] == -2:
            continue  # declared length beyond the fixture's cap: not a verdict
        try:
            got = ctx.snappy_uncompress(_dev(s)).cpu().numpy().tobytes()
            ok = True
        except PsfError as e:
            assert e.code == PSF_ERR_CHECK
            ok = False
        assert ok == (st[i] == 0), (i, s[:12], st[i])
        if ok:
            assert got == want, i
        else:
            nbad += 1
    assert nbad > 100


def _varint(n):
    out = bytearray()
    while n >= 128:
        out.append((n & 127) | 128)
        n >>= 7
    out.append(n)
    return bytes(out)


def _lit(b):
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    k = (n.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + b


def _copy2(off, ln):
    return bytes([2 | ((ln - 1) << 2), off & 255, off >> 8])


def _copy4(off, ln):
    return bytes([3 | ((ln - 1) << 2)]) + off.to_bytes(4, "little")


def test_valid_streams_across_fragments(ctx, port):
    """Valid streams a 1.1.8 encoder never writes: a literal straddling the
    64 KiB output boundary, a copy reaching into the previous fragment, a
    copy-4 tag, an overlapping copy (offset 1)."""
    rng = np.random.default_rng(9)
    blob = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    streams = []
    body = _lit(blob) + _copy2(65000, 64) + _copy4(1, 64) + _copy2(3, 60)
    streams.append(body)
    body = _lit(blob[:65530]) + _copy2(60000, 64) + _lit(b"xyz") + _copy4(65000, 30)
    streams.append(body)
    body = _lit(b"a") + b"".join(_copy2(1, 64) for _ in range(3000))
    streams.append(body)
    for body in streams:
        total = _count(body)
        s = _varint(total) + body
        st, want = port.snappy_uncompress(s, cap=1 << 24)
        assert st == 0
        got = ctx.snappy_uncompress(_dev(s)).cpu().numpy().tobytes()
        assert got == want


def _count(body):
    p, o = 0, 0
    while p < len(body):
        c = body[p]
        if c & 3 == 0:
            ln = (c >> 2) + 1
            h = 1
            if ln > 60:
                k = ln - 60
                ln = int.from_bytes(body[p + 1:p + 1 + k], "little") + 1
                h += k
            p += h + ln
        else:
            ln = 4 + ((c >> 2) & 7) if c & 3 == 1 else (c >> 2) + 1
            p += {1: 2, 2: 3, 3: 5}[c & 3]
        o += ln
    return o


def test_large_roundtrip_properties(ctx):
    """64 MiB of sorted keys: decode(encode(x)) == x and the stream parses."""
    n = 8 << 20
    keys = torch.sort(torch.randint(0, 10**12, (n,), dtype=torch.int64, device="cuda"))[0]
    s = ctx.snappy_compress(keys)
    assert s.numel() < keys.numel() * 8
    back = ctx.snappy_uncompress(s)
    assert torch.equal(back.view(torch.int64), keys)


def test_header_errors(ctx):
    from parameter_server_amd._lib import PsfError
    for bad in (b"\x80", b"\xff\xff\xff\xff\x1f", b"\x03ab", b"\x02\x00\x00"):
        with pytest.raises(PsfError):
            ctx.snappy_uncompress(_dev(bad))


def test_decode_size_hint_vs_header(ctx, port):
    """COMPRESSING's decode sizes the launch from the FilterConfig's recorded
    uncompressed size; the stream's own header decides (UncompressFrom reads
    GetUncompressedLength), so a record that disagrees with the header still
    decodes by the header, and a malformed stream is still rejected."""
    from parameter_server_amd import COMPRESSING, PsfError, lib
    from parameter_server_amd import filter as F
    data = np.random.default_rng(3).integers(0, 256, 100_003, dtype=np.uint8)
    data[:40000] = 7  # partly compressible
    s = port.snappy_compress(data.tobytes())
    for hint in (data.size, data.size - 1, data.size + 5, 7, 1 << 31):
        m = F.Message(request=True, push=True)
        m.add_value(_dev(s))
        idx = m.add_filter(COMPRESSING)
        assert lib().psf_fc_add_uncompressed(m.h, idx, hint) == 0
        node = F.RemoteNode(ctx)
        node.decode(m)
        p, n, loc = m.value_ptr(0)
        ctx.sync()
        got = F.copy_out(p, n, loc, "cuda:0").cpu().numpy().tobytes()
        assert got == data.tobytes(), hint
    bad = b"\xff\xff\xff\xff\xff" + s[5:]
    m = F.Message(request=True, push=True)
    m.add_value(_dev(bad))
    idx = m.add_filter(COMPRESSING)
    lib().psf_fc_add_uncompressed(m.h, idx, data.size)
    with pytest.raises(PsfError):
        F.RemoteNode(ctx).decode(m)


@pytest.mark.parametrize("where", [0, 5, 37])
def test_decode_stored_stream_with_shifted_tail(ctx, port, where):
    """Incompressible fragments (each one stored literal) with one fragment
    that has a match: every later fragment sits a few bytes off the place the
    stored-stream fast path (K-spec) assumes, and the ones it guesses right
    must agree with the linked positions; the decode is exact."""
    rng = np.random.default_rng(where)
    n = 40 * 65536 + 12345
    x = rng.integers(0, 256, n, dtype=np.uint8)
    base = where * 65536 + 3000
    x[base + 100:base + 140] = x[base:base + 40]  # one 40-byte match
    s = port.snappy_compress(x.tobytes())
    for off in (0, 1, 3):
        got = ctx.snappy_uncompress(_dev(s, off)).cpu().numpy()
        assert got.tobytes() == x.tobytes(), off


def test_compress_on_private_stream_is_complete_on_return(port):
    """psf_snappy_compress is synchronous: on a context with its own stream,
    the stream bytes are all in place when the call returns, so a reader on
    another stream (here torch's default one, no sync) sees the whole of it."""
    from parameter_server_amd import filter as F
    side = torch.cuda.Stream()
    ctx = F.Context(0, stream=side)
    rng = np.random.default_rng(21)
    x = rng.integers(0, 256, 48 << 20, dtype=np.uint8)
    x[::7] = 3  # some matches in every fragment
    with torch.cuda.stream(side):
        xd = torch.from_numpy(x).to("cuda", non_blocking=False)
    side.synchronize()
    with torch.cuda.stream(side):
        s = ctx.snappy_compress(xd)
    got = s.to("cpu").numpy().tobytes()  # copied on the default stream
    assert got == port.snappy_compress(x.tobytes())


def test_compress_stream_past_inline_scan(ctx, port):
    """A stream of more than 4096 fragments (256 MiB + 1 fragment + a tail):
    the per-stream offset scan runs as its own launch (shorter streams sum
    their fragment lengths in the placement); byte-identical to 1.1.8 and
    round-trips, with compressible fragments scattered among stored ones."""
    rng = np.random.default_rng(4097)
    n = 4097 * 65536 + 12345
    x = rng.integers(0, 256, n, dtype=np.uint8)
    for k in (0, 5, 4095, 4096):
        x[k * 65536:k * 65536 + 30000] = 7  # a few compressible fragments, one past 4096
    xb = x.tobytes()
    want = port.snappy_compress(xb)
    got = ctx.snappy_compress(_dev(xb)).cpu().numpy().tobytes()
    assert got == want
    back = ctx.snappy_uncompress(_dev(want)).cpu().numpy().tobytes()
    assert back == xb


@pytest.mark.parametrize("kind", ["random", "keys", "codes", "runs", "alpha4", "periodic", "text"])
def test_mutated_multifragment_streams_vs_port(ctx, port, kind):
    """Multi-fragment streams (3-128 fragments) with one or two edits past the
    header (a byte overwritten, deleted or inserted, or the tail cut): the
    batched scan, linker, index and fragment decoder reach RawUncompress's
    verdict (snappy.cc's SnappyDecoder, through oracle/snappy_port.c) and, on
    a stream that still parses, its exact output.  The fixtures in
    snappy_dec.npz are single-fragment; these reach the per-lane tag checks of
    every kernel of the multi-fragment path."""
    from parameter_server_amd._lib import PSF_ERR_CHECK, PsfError
    rng = np.random.default_rng(1000 + len(kind) * 31 + ord(kind[1]))
    nbad = ngood = 0
    for t in range(30):
        n = int(rng.integers(150_000, 1_600_000)) if t % 10 != 9 else 8 << 20
        x = _inputs(rng, n, kind)
        s = bytearray(port.snappy_compress(x))
        hdr = 1
        while s[hdr - 1] & 0x80:
            hdr += 1
        for _ in range(1 + t % 2):
            i = int(rng.integers(hdr, len(s)))
            op = int(rng.integers(0, 4)) if t else 0
            if op == 0:
                s[i] = (s[i] + int(rng.integers(1, 256))) & 255
            elif op == 1:
                del s[i]
            elif op == 2:
                s.insert(i, int(rng.integers(0, 256)))
            else:
                del s[i:]
        s = bytes(s)
        st, want = port.snappy_uncompress(s, cap=1 << 24)
        assert st != -2
        try:
            got = ctx.snappy_uncompress(_dev(s)).cpu().numpy().tobytes()
            ok = True
        except PsfError as e:
            assert e.code == PSF_ERR_CHECK
            ok = False
        assert ok == (st == 0), (kind, t, st)
        if ok:
            assert got == want, (kind, t)
            ngood += 1
        else:
            nbad += 1
    assert nbad > 0


def test_tag_dense_with_long_literals_roundtrip(ctx, port):
    """Sorted-key runs (tags of a few bytes) between random runs of 100-400
    bytes (literals longer than 64 bytes, so some straddle an 8 KiB window
    start of the stream and the chain enters that window past its first 64
    bytes): the windows are then linked by K2's walk instead of the parallel
    prefix (K2p), and the bytes must come back either way -- and the stream
    is 1.1.8's."""
    rng = np.random.default_rng(21)
    parts = []
    base = 0
    while sum(len(p) for p in parts) < (6 << 20):
        k = np.sort(rng.integers(base, base + 10**7, 256)).astype(np.uint64)
        base += 10**7
        parts.append(k.tobytes())
        parts.append(rng.integers(0, 256, int(rng.integers(100, 400)), dtype=np.uint8).tobytes())
    data = b"".join(parts)
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    s = ctx.snappy_compress(x)
    want = port.snappy_compress(data)
    got_s = s.cpu().numpy().tobytes()
    ok = got_s == want
    assert ok, (len(got_s), len(want))
    back = ctx.snappy_uncompress(s).cpu().numpy().tobytes()
    ok = back == data
    assert ok


def _lz_fragments(rng, nfrag, dist):
    """Per 64 KiB fragment: a random head, then pieces copied from `dist(rng)`
    bytes back (5-60 bytes each) with 1-3 fresh bytes between them, so the
    stream is tag-dense and its copies reach back that far."""
    out = bytearray()
    for _ in range(nfrag):
        f = bytearray(rng.integers(0, 256, 256, dtype=np.uint8).tobytes())
        while len(f) < 65536:
            d = min(int(dist(rng)), len(f))
            n = int(rng.integers(5, 61))
            src = len(f) - d
            for i in range(n):  # (byte by byte: the copy may overlap itself)
                f.append(f[src + i])
            f += rng.integers(0, 256, int(rng.integers(1, 4)), dtype=np.uint8).tobytes()
        out += f[:65536]
    return bytes(out)


@pytest.mark.parametrize("kind", ["far", "ring_edge"])
def test_tag_dense_far_copies_roundtrip(ctx, port, kind):
    """Tag-dense fragments whose copies reach far back (up to 60 KiB, or right
    around 8 KiB): the fragment decoder keeps the last 8 KiB of its output in
    LDS and reads older copy sources from the bytes it already wrote out.
    Compress is 1.1.8's, uncompress gives the bytes back."""
    rng = np.random.default_rng(77 if kind == "far" else 78)
    if kind == "far":
        dist = lambda r: r.integers(1, 60000)  # noqa: E731
    else:
        dist = lambda r: 8192 + r.integers(-70, 70)  # noqa: E731
    data = _lz_fragments(rng, 24, dist)
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    s = ctx.snappy_compress(x)
    want = port.snappy_compress(data)
    assert s.cpu().numpy().tobytes() == want
    back = ctx.snappy_uncompress(s).cpu().numpy().tobytes()
    assert back == data
