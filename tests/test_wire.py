"""CPU: the Task frame of the wire (van.cc:122-191) against protobuf itself.

The reference serialises Task with protobuf-generated C++.  The message types
come from the reference's own .proto files (system/proto/task.proto and its
imports: filter.proto, range.proto, param.proto, ...), compiled here by the
image's protoc (torch/bin/protoc) into a descriptor set and loaded into
protobuf's Python runtime.  Where /root/reference is absent the tests fall
back to descriptors typed from the same field numbers and types, and
test_fallback_descriptors_match_reference_proto pins that fallback to the
compiled ones.  Checks:

* libpsf's frame == protobuf's serialisation of the same fields, byte for byte;
* protobuf frames (any field order, packed repeats, unknown fields) parse to
  the same fields in libpsf;
* truncated / corrupted frames are rejected exactly where protobuf's C++
  ParseFromArray (parse + required fields) rejects them.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

pb = pytest.importorskip("google.protobuf")

REF_SRC = "/root/reference/src"


def _protoc():
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "bin", "protoc")
    return p if os.access(p, os.X_OK) else None


def _reference_types():
    """PS.Task / PS.FilterConfig compiled from the reference's task.proto (and
    everything it imports), or None where the reference or protoc is absent."""
    protoc = _protoc()
    if protoc is None or not os.path.exists(os.path.join(REF_SRC, "system/proto/task.proto")):
        return None
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ps.desc")
        subprocess.run([protoc, f"-I{REF_SRC}", "--include_imports", f"--descriptor_set_out={out}",
                        "system/proto/task.proto"], check=True, capture_output=True)
        with open(out, "rb") as f:
            fds = descriptor_pb2.FileDescriptorSet.FromString(f.read())
    pool = descriptor_pool.DescriptorPool()
    for fd in fds.file:  # dependencies first (--include_imports order)
        pool.Add(fd)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("PS.Task")), get(pool.FindMessageTypeByName("PS.FilterConfig"))


def _types():
    return _reference_types() or _fallback_types()


def _fallback_types():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="psf_wire_test.proto", package="PS", syntax="proto2")

    def msg(name, fields, nested=(), enums=()):
        m = fd.message_type.add(name=name)
        for e in enums:
            m.enum_type.add().CopyFrom(e)
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        for fname, num, typ, label, extra in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            for k, v in extra.items():
                setattr(f, k, v)
        return m

    OPT, REQ, REP = F.LABEL_OPTIONAL, F.LABEL_REQUIRED, F.LABEL_REPEATED
    dt = fd.enum_type.add(name="DataType")
    for i, n in enumerate(["OTHER", "INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32",
                           "UINT64", "FLOAT", "DOUBLE", "CHAR"]):
        dt.value.add(name=n, number=i)
    msg("PbRange", [("begin", 1, F.TYPE_UINT64, REQ, {}), ("end", 2, F.TYPE_UINT64, REQ, {})])
    msg("ParamCall", [("push", 1, F.TYPE_BOOL, OPT, {"default_value": "true"})])
    ffc = descriptor_pb2.DescriptorProto(name="FixedFloatConfig")
    ffc.field.add(name="min_value", number=1, type=F.TYPE_FLOAT, label=OPT, default_value="-1")
    ffc.field.add(name="max_value", number=2, type=F.TYPE_FLOAT, label=OPT, default_value="1")
    ty = descriptor_pb2.EnumDescriptorProto(name="Type")
    for n, v in (("KEY_CACHING", 1), ("COMPRESSING", 2), ("FIXING_FLOAT", 3), ("NOISE", 4)):
        ty.value.add(name=n, number=v)
    msg("FilterConfig", [
        ("type", 1, F.TYPE_ENUM, REQ, {"type_name": ".PS.FilterConfig.Type"}),
        ("clear_cache_if_done", 20, F.TYPE_BOOL, OPT, {"default_value": "false"}),
        ("num_bytes", 5, F.TYPE_INT32, OPT, {"default_value": "3"}),
        ("fixed_point", 4, F.TYPE_MESSAGE, REP, {"type_name": ".PS.FilterConfig.FixedFloatConfig"}),
        ("mean", 6, F.TYPE_FLOAT, OPT, {}),
        ("std", 7, F.TYPE_FLOAT, OPT, {}),
        ("signature", 2, F.TYPE_UINT32, OPT, {}),
        ("uncompressed_size", 3, F.TYPE_UINT64, REP, {}),
    ], nested=[ffc], enums=[ty])
    msg("Task", [
        ("control", 1, F.TYPE_BOOL, OPT, {"default_value": "false"}),  # outside the filter path
        ("request", 2, F.TYPE_BOOL, OPT, {"default_value": "false"}),
        ("customer_id", 3, F.TYPE_INT32, OPT, {}),      # outside
        ("time", 5, F.TYPE_INT32, OPT, {}),             # outside
        ("wait_time", 6, F.TYPE_INT32, REP, {}),        # outside
        ("key_range", 7, F.TYPE_MESSAGE, OPT, {"type_name": ".PS.PbRange"}),
        ("key_channel", 8, F.TYPE_INT32, OPT, {}),
        ("has_key", 9, F.TYPE_BOOL, OPT, {"default_value": "false"}),
        ("filter", 12, F.TYPE_MESSAGE, REP, {"type_name": ".PS.FilterConfig"}),
        ("key_type", 13, F.TYPE_ENUM, OPT, {"type_name": ".PS.DataType"}),
        ("value_type", 14, F.TYPE_ENUM, REP, {"type_name": ".PS.DataType"}),
        ("msg", 17, F.TYPE_BYTES, OPT, {}),             # outside
        ("param", 20, F.TYPE_MESSAGE, OPT, {"type_name": ".PS.ParamCall"}),
    ])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("PS.Task")), get(pool.FindMessageTypeByName("PS.FilterConfig"))


@pytest.fixture(scope="module")
def Task():
    return _types()[0]


def _fields(desc, seen=None):
    """(message, field) -> (number, type, label, default) over desc and the
    message types it reaches"""
    from google.protobuf import descriptor_pb2
    seen = {} if seen is None else seen
    if desc.full_name in seen:
        return seen
    p = descriptor_pb2.DescriptorProto()
    desc.CopyToProto(p)
    seen[desc.full_name] = {f.name: (f.number, f.type, f.label, f.type_name.split(".")[-1], f.default_value)
                            for f in p.field}
    for f in desc.fields:
        if f.message_type is not None:
            _fields(f.message_type, seen)
    return seen


def test_fallback_descriptors_match_reference_proto():
    ref = _reference_types()
    if ref is None:
        pytest.skip("reference .proto files or protoc absent")
    want, got = _fields(ref[0].DESCRIPTOR), _fields(_fallback_types()[0].DESCRIPTOR)
    assert set(got) <= set(want)
    for msg, fields in got.items():
        for name, spec in fields.items():
            assert want[msg][name] == spec, (msg, name)


def _random_psf_message(rng):
    """A libpsf message with random filter-path fields + the equivalent protobuf
    field assignments (in the same has-state)."""
    from parameter_server_amd import filter as F
    request = bool(rng.integers(2))
    has_param = bool(rng.integers(2))
    push = bool(rng.integers(2))
    ch = int(rng.integers(-5, 1000))
    kr = None if rng.integers(3) == 0 else tuple(sorted(int(v) for v in rng.integers(0, 2**63, 2)))
    m = F.Message(request=request, push=push, has_param=has_param, key_channel=ch, key_range=kr)
    spec = {"request": request, "key_channel": ch, "kr": kr, "param": (push if has_param else None),
            "filters": [], "values": []}
    for _ in range(int(rng.integers(0, 4))):
        t = int(rng.integers(1, 5))
        opts = {}
        if rng.integers(2):
            opts["num_bytes"] = int(rng.integers(-3, 9))
        if rng.integers(2):
            opts["clear_cache_if_done"] = bool(rng.integers(2))
        if rng.integers(2):
            opts["noise"] = (float(np.float32(rng.standard_normal())), float(np.float32(rng.random())))
        fps = []
        for _ in range(int(rng.integers(0, 3))):
            fps.append((None if rng.integers(3) == 0 else float(np.float32(rng.standard_normal())),
                        None if rng.integers(3) == 0 else float(np.float32(rng.standard_normal()))))
        opts["fixed_point"] = fps
        m.add_filter(t, **opts)
        spec["filters"].append((t, opts))
    return m, spec


def _pb_from_spec(Task, spec):
    t = Task()
    t.request = spec["request"]
    if spec["kr"] is not None:
        t.key_range.begin, t.key_range.end = spec["kr"]
    t.key_channel = spec["key_channel"]
    for ftype, opts in spec["filters"]:
        f = t.filter.add()
        f.type = ftype
        for mn, mx in opts.get("fixed_point", []):
            fp = f.fixed_point.add()
            if mn is not None:
                fp.min_value = mn
            if mx is not None:
                fp.max_value = mx
        if "num_bytes" in opts:
            f.num_bytes = opts["num_bytes"]
        if "noise" in opts:
            f.mean, f.std = opts["noise"]
        if "clear_cache_if_done" in opts:
            f.clear_cache_if_done = opts["clear_cache_if_done"]
    if spec["param"] is not None:
        t.param.push = spec["param"]
    return t


def test_serialize_matches_protobuf(Task):
    rng = np.random.default_rng(0)
    for _ in range(300):
        m, spec = _random_psf_message(rng)
        ours = m.task_bytes()
        want = _pb_from_spec(Task, spec).SerializeToString()
        assert ours == want, spec
        assert Task.FromString(ours) == Task.FromString(want)


def _random_pb(Task, rng):
    t = Task()
    if rng.integers(2):
        t.request = bool(rng.integers(2))
    if rng.integers(2):
        t.control = bool(rng.integers(2))
    if rng.integers(2):
        t.time = int(rng.integers(-10, 10**6))
    for _ in range(int(rng.integers(0, 3))):
        t.wait_time.append(int(rng.integers(0, 100)))
    if rng.integers(2):
        t.key_range.begin, t.key_range.end = (int(v) for v in rng.integers(0, 2**63, 2))
    if rng.integers(2):
        t.key_channel = int(rng.integers(-2**31, 2**31))
    if rng.integers(2):
        t.has_key = bool(rng.integers(2))
    if rng.integers(2):
        t.key_type = int(rng.integers(0, 12))
    for _ in range(int(rng.integers(0, 4))):
        t.value_type.append(int(rng.integers(0, 12)))
    if rng.integers(2):
        t.msg = bytes(rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8))
    for _ in range(int(rng.integers(0, 3))):
        f = t.filter.add()
        f.type = int(rng.integers(1, 5))
        if rng.integers(2):
            f.signature = int(rng.integers(0, 2**32))
        for _ in range(int(rng.integers(0, 3))):
            f.uncompressed_size.append(int(rng.integers(0, 2**40)))
        for _ in range(int(rng.integers(0, 3))):
            fp = f.fixed_point.add()
            if rng.integers(2):
                fp.min_value = float(rng.standard_normal())
            if rng.integers(2):
                fp.max_value = float(rng.standard_normal())
        if rng.integers(2):
            f.num_bytes = int(rng.integers(-100, 100))
        if rng.integers(2):
            f.mean = float(rng.standard_normal())
        if rng.integers(2):
            f.std = float(rng.standard_normal())
        if rng.integers(2):
            f.clear_cache_if_done = bool(rng.integers(2))
    if rng.integers(2):
        t.param.SetInParent()
        if rng.integers(2):
            t.param.push = bool(rng.integers(2))
    fields = Task.DESCRIPTOR.fields_by_name
    if "more" in fields and rng.integers(4) == 0:  # reference-only fields: skipped by libpsf
        t.more = bool(rng.integers(2))
    if "task" in fields and rng.integers(4) == 0:
        sub = t.task.add()
        sub.request = True
        sub.key_channel = int(rng.integers(0, 100))
        if rng.integers(2):
            sub.key_range.begin, sub.key_range.end = 1, 2
    if "ctrl" in fields and rng.integers(4) == 0:  # required Control.cmd / Node.role nested
        t.ctrl.cmd = int(rng.choice([1, 2, 10, 14]))
        for _ in range(int(rng.integers(0, 3))):
            nd = t.ctrl.node.add()
            nd.role = int(rng.choice([0, 1, 3]))
            if rng.integers(2):
                nd.hostname = "h%d" % rng.integers(100)
    return t


_OUTSIDE = ("control", "time", "wait_time", "msg", "customer_id", "more", "task", "ctrl")


def _filter_path_view(Task, t):
    """t without the fields the filter path does not carry; request and
    key_channel always present (libpsf always sends them)."""
    u = Task()
    u.CopyFrom(t)
    for f in _OUTSIDE:
        if f in Task.DESCRIPTOR.fields_by_name:
            u.ClearField(f)
    u.DiscardUnknownFields()  # e.g. unknown enum values: protobuf keeps them aside
    u.request = t.request
    u.key_channel = t.key_channel
    if t.HasField("param"):
        u.param.push = t.param.push  # default true made explicit
    return u


def test_parse_protobuf_frames(Task):
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(1)
    for _ in range(400):
        t = _random_pb(Task, rng)
        b = t.SerializeToString()
        m = F.Message.from_task_bytes(b)
        back = Task.FromString(m.task_bytes())
        want = _filter_path_view(Task, t)
        want.has_key = False  # no key frame attached: Van::Send clears has_key
        want.ClearField("has_key")
        assert back == want, (t, back)


def test_parse_packed_and_reordered(Task):
    """Packed repeated scalars and out-of-order fields (valid protobuf input)."""
    from parameter_server_amd import filter as F

    def varint(v):
        o = bytearray()
        while v >= 0x80:
            o.append((v & 0x7f) | 0x80)
            v >>= 7
        o.append(v)
        return bytes(o)

    def ld(field, payload):
        return varint(field << 3 | 2) + varint(len(payload)) + payload

    fc = ld(3, varint(5) + varint(300)) + varint(1 << 3) + varint(2)  # packed sizes, then type
    b = varint(8 << 3) + varint(7) + ld(14, varint(9) + varint(10) + varint(99)) + ld(12, fc) + \
        varint(2 << 3) + varint(1)
    m = F.Message.from_task_bytes(b)
    want = Task.FromString(b)
    assert Task.FromString(m.task_bytes()) == _filter_path_view(Task, want)


def test_malformed_frames_rejected_like_protobuf(Task):
    from google.protobuf.message import DecodeError

    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import PsfError
    rng = np.random.default_rng(2)
    agree = rejected = 0
    for i in range(4000):
        b = bytearray(_random_pb(Task, rng).SerializeToString())
        op = i % 3
        if b and op == 0:
            del b[int(rng.integers(0, len(b))):]
        elif b and op == 1:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        else:
            b.insert(int(rng.integers(0, len(b) + 1)), int(rng.integers(0, 256)))
        try:  # C++ ParseFromArray == parse + IsInitialized (required fields)
            ok_pb = Task.FromString(bytes(b)).IsInitialized()
        except DecodeError:
            ok_pb = False
        try:
            F.Message.from_task_bytes(bytes(b))
            ok = True
        except PsfError:
            ok = False
        assert ok == ok_pb, bytes(b)
        agree += 1
        rejected += not ok
    assert rejected > 100


def test_frames_follow_van_send(Task):
    """[Task][key][values] with has_key set from the key (van.cc:131-137)."""
    import torch

    from parameter_server_amd import filter as F
    m = F.Message(request=True, push=True, key_range=(0, 100))
    keys = torch.arange(5, dtype=torch.int64)
    m.set_key(keys)
    m.add_value(torch.ones(5))
    fr = m.frames()
    assert len(fr) == 3
    t = Task.FromString(fr[0])
    assert t.has_key and t.key_type == 8 and list(t.value_type) == [9]
    assert fr[1] == keys.numpy().tobytes() and fr[2] == np.ones(5, np.float32).tobytes()
    m2 = F.Message(request=False, push=False)
    m2.add_value(torch.ones(2))
    fr = m2.frames()
    assert len(fr) == 2 and not Task.FromString(fr[0]).HasField("has_key")


def test_nested_fields_outside_filter_path_checked_like_protobuf(Task):
    """Fields libpsf skips are still parsed as protobuf parses them: a nested
    Control without its required cmd, a nested Task whose key_range lacks end,
    an unknown enum value in a required field, a packed repeat cut inside a
    varint -- all rejected, and their well-formed twins accepted."""
    from google.protobuf.message import DecodeError

    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import PsfError
    fields = Task.DESCRIPTOR.fields_by_name
    if "ctrl" not in fields:
        pytest.skip("reference .proto files absent: the fallback Task has no ctrl / task fields")
    cases = []
    t = Task()
    t.ctrl.SetInParent()
    cases.append(t.SerializePartialToString())
    t.ctrl.cmd = 2
    cases.append(t.SerializePartialToString())
    t = Task()
    t.task.add().key_range.begin = 5
    cases.append(t.SerializePartialToString())
    t.task[0].key_range.end = 9
    cases.append(t.SerializePartialToString())
    cases.append(bytes([0x92, 0x01, 2, 8, 7]))  # ctrl { cmd: 7 } -- not a Control.Command
    cases.append(bytes([0x92, 0x01, 2, 8, 4]))  # ctrl { cmd: READY_TO_EXIT }
    cases.append(bytes([6 << 3 | 2, 2, 1, 0x81]))  # packed wait_time cut inside a varint
    cases.append(bytes([6 << 3 | 2, 2, 1, 0x01]))
    verdicts = []
    for b in cases:
        try:
            ok_pb = Task.FromString(b).IsInitialized()
        except DecodeError:
            ok_pb = False
        try:
            F.Message.from_task_bytes(b)
            ok = True
        except PsfError:
            ok = False
        assert ok == ok_pb, b
        verdicts.append(ok)
    assert verdicts == [False, True] * 4
