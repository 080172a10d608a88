"""Result encoding.  CPU half: the shortest-decimal float formatter of
csrc/fmt_float.h, built for the host from the same source (tests/fmt_host.cpp), against
Python's shortest repr (doubles) and numpy's unique Dragon4 (float32), rendered the way Rust's
Display prints them (pgwire 0.28.0 ToSqlText).  GPU half: qeh_encode_pg_datarows vs the
Python restatement in oracle/pg_text.py."""
import ctypes as C
import math
import os
import random
import struct
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pg_text  # noqa: E402


@pytest.fixture(scope="module")
def fmt(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("fmt") / "fmt_host.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", os.path.join(ROOT, "tests", "fmt_host.cpp"),
                           "-I", os.path.join(ROOT, "query-engine_amd", "csrc"), "-o", so])
    lib = C.CDLL(so)
    lib.fmt_f64_c.argtypes = [C.c_double, C.c_char_p]
    lib.fmt_f32_c.argtypes = [C.c_float, C.c_char_p]
    lib.fmt_i64_c.argtypes = [C.c_longlong, C.c_char_p]
    buf = C.create_string_buffer(512)

    def call(fn, v):
        n = fn(v, buf)
        return buf.raw[:n].decode()
    return (lambda v: call(lib.fmt_f64_c, v)), (lambda v: call(lib.fmt_f32_c, v)), (lambda v: call(lib.fmt_i64_c, v))


EDGE = [0.0, -0.0, 1.0, -1.0, 0.1, 0.2, 0.3, 1 / 3, 2 / 3, 1e21, 1e22, 1e23, 1e-7, 123.456, 5e-324, 1e-323,
        2.2250738585072014e-308, 2.225073858507201e-308, 1.7976931348623157e308, 2.0 ** 53, 2.0 ** 53 + 2,
        9007199254740993.0, 100.0, 1e15, 1e16, 1e17, 0.5, 2.0 ** -1074 * 3, float("nan"), float("inf"),
        -float("inf"), 4.35, 0.000123, 123456789012345680.0]


def test_known_answers_rust_display(fmt):
    f64, f32, i64 = fmt
    assert f64(1.0) == "1" and f64(-0.0) == "-0" and f64(0.1) == "0.1"
    assert f64(1e21) == "1000000000000000000000" and f64(1e-7) == "0.0000001"
    assert f64(float("nan")) == "NaN" and f64(float("inf")) == "inf" and f64(-float("inf")) == "-inf"
    assert f32(0.1) == "0.1" and f32(16777216.0) == "16777216" and f32(3.4028234663852886e38).startswith("3402823")
    assert i64(-(2 ** 63)) == str(-(2 ** 63)) and i64(0) == "0" and i64(2 ** 63 - 1) == str(2 ** 63 - 1)


def test_i64_digit_boundaries_and_random(fmt):
    """Integer text: every power-of-ten boundary (the digit count comes from the bit length and one
    table compare; 8-digit pieces), both signs, and random values of every bit length."""
    _, _, i64 = fmt
    vals = [0, 1, -1, 2 ** 63 - 1, -(2 ** 63)]
    for k in range(19):
        for d in (-1, 0, 1):
            x = 10 ** k + d
            if x < 2 ** 63:
                vals += [x, -x]
    r = random.Random(7)
    vals += [r.getrandbits(b) * r.choice((1, -1)) for b in range(1, 64) for _ in range(40)]
    for x in vals:
        assert i64(x) == str(x), x


def test_f64_edges_and_random_bits(fmt):
    f64 = fmt[0]
    for v in EDGE:
        assert f64(v) == pg_text.rust_f64(v), v
    rnd = random.Random(7)
    for _ in range(100_000):
        v = struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0]
        assert f64(v) == pg_text.rust_f64(v), v
    for _ in range(50_000):
        v = rnd.random() * 10.0 ** rnd.randint(-20, 20)
        assert f64(v) == pg_text.rust_f64(v), v


def test_f64_power_of_two_boundaries_and_subnormals(fmt):
    f64 = fmt[0]
    for e in range(-1074, 1024):
        v = math.ldexp(1.0, e)
        for w in (v, math.nextafter(v, 0.0), math.nextafter(v, math.inf)):
            if math.isfinite(w):
                assert f64(w) == pg_text.rust_f64(w), w
    for t in list(range(1, 200)) + [2 ** 52 - 1, 2 ** 51]:
        v = struct.unpack("<d", struct.pack("<Q", t))[0]
        assert f64(v) == pg_text.rust_f64(v), t


def test_f32_random_and_boundaries(fmt):
    f32 = fmt[1]
    rnd = np.random.default_rng(3)
    bits = rnd.integers(0, 2 ** 32, 100_000, dtype=np.uint64).astype(np.uint32)
    vals = bits.view(np.float32)
    for v in vals:
        assert f32(float(v)) == pg_text.rust_f32(v), v
    for e in range(-149, 128):
        v = np.float32(math.ldexp(1.0, e))
        for w in (v, np.nextafter(v, np.float32(0)), np.nextafter(v, np.float32(np.inf))):
            if np.isfinite(w):
                assert f32(float(w)) == pg_text.rust_f32(w), w


def _host_values(vals, valid):
    return [None if (valid is not None and not valid[i]) else vals[i] for i in range(len(vals))]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 1000, 100_003])
def test_pg_datarows_device_vs_oracle(ctx, n):
    """qeh_encode_pg_datarows == oracle/pg_text.py byte for byte, every type, NULLs included."""
    r = np.random.default_rng(n)
    f64 = r.standard_normal(n) * 10.0 ** r.integers(-30, 30, n)
    if n > 10:
        f64[:10] = [0.0, -0.0, 1.0, 0.1, 1e21, 1e-7, np.nan, np.inf, -np.inf, 5e-324]
    f32 = (r.standard_normal(n) * 10.0 ** r.integers(-8, 8, n)).astype(np.float32)
    cols = [
        ("int64", r.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64), r.random(n) > 0.1),
        ("int32", r.integers(-(2 ** 31), 2 ** 31 - 1, n).astype(np.int32), None),
        ("float64", f64, r.random(n) > 0.05),
        ("float32", f32, None),
        ("bool", r.random(n) > 0.5, r.random(n) > 0.2),
        ("utf8", np.array(["", "a", "héllo", "x" * 40, "tab\\tq"] * (n // 5) + ["z"] * (n % 5), dtype=object),
         r.random(n) > 0.1),
    ]
    dev = [ctx.upload(v, m) for _, v, m in cols]
    got = ctx.encode_pg_datarows(dev).to_bytes()
    want = pg_text.encode_rows([(dt, _host_values(list(v), m)) for dt, v, m in cols])
    assert len(got) == len(want) == n
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, g, w)


@pytest.mark.gpu
def test_pg_datarows_sliced_input_and_no_columns(ctx):
    v = np.arange(-50, 50, dtype=np.int64)
    d = ctx.upload(v, offset=3)
    got = ctx.encode_pg_datarows([d]).to_bytes()
    assert got == pg_text.encode_rows([("int64", list(v))])
    assert ctx.encode_pg_datarows([]).to_bytes() == []


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 77, 100_000])
def test_arrow_ipc_stream_round_trips_through_pyarrow(ctx, n):
    """qeh_encode_arrow_ipc (SerializedBatch::from_batch, network.rs:56-72): the stream decodes
    with pyarrow's IPC reader to the same batch, names and types; sliced inputs included."""
    import pyarrow as pa
    r = np.random.default_rng(n + 1)
    vals = {
        "g.i64": (r.integers(-(2 ** 62), 2 ** 62, n).astype(np.int64), r.random(n) > 0.1, pa.int64()),
        "g.i32": (r.integers(-1000, 1000, n).astype(np.int32), None, pa.int32()),
        "g.f64": (r.standard_normal(n), r.random(n) > 0.3, pa.float64()),
        "g.f32": (r.random(n).astype(np.float32), None, pa.float32()),
        "g.b": (r.random(n) > 0.5, r.random(n) > 0.2, pa.bool_()),
        "g.s": (np.array([f"v{i % 13}" * (i % 4) for i in range(n)], dtype=object), r.random(n) > 0.1, pa.string()),
    }
    dev = [ctx.upload(v, m, offset=(3 if k != "g.s" else 0)) for k, (v, m, _) in vals.items()]
    data = ctx.encode_arrow_ipc(dev, list(vals))
    got = pa.ipc.open_stream(pa.py_buffer(data)).read_all()
    want = pa.table({k: pa.array(list(v), type=t, mask=None if m is None else ~m) for k, (v, m, t) in vals.items()})
    assert got.schema.names == want.schema.names
    assert [f.type for f in got.schema] == [f.type for f in want.schema]
    assert got.num_rows == n
    for a, b in zip(got.columns, want.columns):
        assert a.to_pylist() == b.to_pylist()


@pytest.mark.gpu
def test_arrow_ipc_reused_pinned_buffers(ctx):
    """The encoder's pinned host buffers are kept after qeh_host_free and handed out again: a stream
    still held is never overwritten by a later encode, and a reused buffer carries the new stream whole."""
    import gc
    import pyarrow as pa
    r = np.random.default_rng(5)
    batches = [r.integers(-(2 ** 62), 2 ** 62, m).astype(np.int64) for m in (200_000, 190_000, 200_000, 120_000)]
    held = []
    for i, v in enumerate(batches):
        data = ctx.encode_arrow_ipc([ctx.upload(v)], ["x"])
        held.append((i, data))
        if i == 1:  # free the first two streams: the next encodes may take their buffers
            held.clear()
            gc.collect()
        got = pa.ipc.open_stream(pa.py_buffer(data)).read_all().column(0).to_numpy()
        assert np.array_equal(got, v)
    for i, data in held:
        assert np.array_equal(pa.ipc.open_stream(pa.py_buffer(data)).read_all().column(0).to_numpy(), batches[i])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 5, 65_537])
def test_arrow_ipc_decode_pyarrow_streams_and_round_trip(ctx, n):
    """qeh_decode_arrow_ipc (SerializedBatch::to_batch, network.rs:75-90) reads a stream written by
    pyarrow (sliced arrays: non-zero Utf8 offset base, bit offsets) and our own encoder's output."""
    import pyarrow as pa
    r = np.random.default_rng(n + 9)
    m = n + 7
    t = pa.table({
        "a": pa.array(r.integers(-(2 ** 40), 2 ** 40, m), pa.int64(), mask=r.random(m) < 0.1),
        "b": pa.array(r.random(m), pa.float64()),
        "c": pa.array([f"s{i}" if i % 3 else None for i in range(m)], pa.string()),
        "d": pa.array(r.random(m) < 0.5, pa.bool_(), mask=r.random(m) < 0.2),
        "e": pa.array(r.integers(0, 2 ** 32, m, dtype=np.uint64).astype(np.uint32), pa.uint32()),
        "f": pa.array(r.random(m).astype(np.float32), pa.float32()),
        "g": pa.array(r.integers(-100, 100, m).astype(np.int32), pa.int32()),
    }).slice(7, n)
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    if n == 0:  # pyarrow writes no batch for an empty table: to_batch's "No batch found" error
        from qe_hip import QehError
        with pytest.raises(QehError, match="No batch found"):
            ctx.decode_arrow_ipc(sink.getvalue().to_pybytes())
        return
    names, cols, rows = ctx.decode_arrow_ipc(sink.getvalue().to_pybytes())
    assert names == t.schema.names and rows == n
    for c, want in zip(cols, t.columns):
        v, valid = c.to_numpy()
        got = [None if (valid is not None and not valid[i]) else v[i] for i in range(n)]
        got = [x.item() if hasattr(x, "item") else x for x in got]
        assert got == want.to_pylist()
    # encoder -> decoder round trip on the device
    names2, cols2, rows2 = ctx.decode_arrow_ipc(ctx.encode_arrow_ipc(cols, names))
    assert names2 == names and rows2 == n
    def rows(c):
        v, valid = c.to_numpy()
        return [None if (valid is not None and not valid[i]) else v[i] for i in range(len(v))]
    for a, b in zip(cols, cols2):
        assert rows(a) == rows(b)


@pytest.mark.gpu
def test_arrow_ipc_decode_rejects_malformed(ctx):
    import pyarrow as pa
    from qe_hip import QehError
    sink = pa.BufferOutputStream()
    t = pa.table({"a": pa.array([1, 2, 3], pa.int64())})
    with pa.ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    data = sink.getvalue().to_pybytes()
    for bad in (data[:10], data[:len(data) // 2], b"\xff\xff\xff\xff" + b"\x10\x00\x00\x00" + b"\x00" * 16):
        with pytest.raises(QehError):
            ctx.decode_arrow_ipc(bad)
    # a Utf8 column whose offsets decrease: rejected before anything reaches the device
    st = pa.BufferOutputStream()
    ts = pa.table({"s": pa.array(["ab", "cd", "ef"])})
    with pa.ipc.new_stream(st, ts.schema) as w:
        w.write_table(ts)
    raw = bytearray(st.getvalue().to_pybytes())
    import struct as _st
    pat = _st.pack("<4i", 0, 2, 4, 6)
    at = bytes(raw).index(pat)
    raw[at:at + 16] = _st.pack("<4i", 0, 4, 2, 6)
    with pytest.raises(QehError, match="offsets"):
        ctx.decode_arrow_ipc(bytes(raw))
    # a buffer whose offset + length overflows int64 (2^62 + 2^62): rejected, never dereferenced
    bufs = _st.pack("<4q", 0, 0, 0, 24)  # validity (0, 0), values (0, 24) of the Int64 column
    raw = bytearray(data)
    at = bytes(raw).index(bufs)
    raw[at:at + 32] = _st.pack("<4q", 0, 0, 2 ** 62, 2 ** 62)
    with pytest.raises(QehError, match="outside the body"):
        ctx.decode_arrow_ipc(bytes(raw))
    only_schema = data[:data.index(b"\xff\xff\xff\xff", 8)]
    with pytest.raises(QehError, match="No batch found"):
        ctx.decode_arrow_ipc(only_schema + b"\xff\xff\xff\xff\x00\x00\x00\x00")
