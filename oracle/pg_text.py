"""CPU restatement of the reference's pgwire text encoding of result rows.

TEST INFRASTRUCTURE ONLY (the checker for tests/test_encode.py); the product path is
qeh_encode_pg_datarows on the device.

Follows crates/query-pgwire/src/result.rs:56-176: record_batch_to_rows builds one DataRowEncoder
per row and encode_value writes each cell through pgwire 0.28.0 (Cargo.lock:1993-1995; not
vendored, so its published behaviour is restated here): NULL -> field length -1 (result.rs:88-91);
Boolean -> "t" / "f"; Int32 / Int64 (and UInt32 widened to i64, result.rs:123-126) -> decimal;
Float32 / Float64 -> Rust's Display (`to_string`): the shortest decimal that reads back to the
same value, written without an exponent; Utf8 -> its bytes.  The DataRow message is the
PostgreSQL protocol's: 'D', Int32 length (self-inclusive), Int16 field count, then per field an
Int32 length (-1 for NULL) and the bytes, all big-endian.

Parity: the float rendering is pinned by Python's shortest repr (David Gay's dtoa mode 0) for
doubles and numpy's unique Dragon4 for float32; pgwire's own output is not available here
(parity unpinned against pgwire itself).
"""
from __future__ import annotations

import math
import struct
from decimal import Decimal
from typing import List, Optional, Sequence, Tuple

import numpy as np


def _positional(sign: bool, digits: str, exp: int) -> str:
    """digits * 10^exp without exponent, trailing zeros of the digits removed."""
    ds = digits.rstrip("0") or "0"
    exp += len(digits) - len(ds)
    nd, pt = len(ds), exp + len(ds)
    if pt <= 0:
        s = "0." + "0" * (-pt) + ds
    elif pt >= nd:
        s = ds + "0" * (pt - nd)
    else:
        s = ds[:pt] + "." + ds[pt:]
    return ("-" if sign else "") + s


def rust_f64(v: float) -> str:
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "inf" if v > 0 else "-inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    sign, digits, exp = Decimal(repr(v)).as_tuple()
    return _positional(bool(sign), "".join(map(str, digits)), exp)


def rust_f32(v) -> str:
    v = np.float32(v)
    if np.isnan(v):
        return "NaN"
    if np.isinf(v):
        return "inf" if v > 0 else "-inf"
    if v == 0:
        return "-0" if np.signbit(v) else "0"
    s = np.format_float_scientific(v, unique=True, exp_digits=1)  # "d.ddde±x", shortest for float32
    mant, e = s.split("e")
    sign = mant.startswith("-")
    mant = mant.lstrip("-")
    ip, _, fp = mant.partition(".")
    return _positional(sign, ip + fp, int(e) - len(fp))


def cell_text(dtype: str, value) -> Optional[bytes]:
    if value is None:
        return None
    if dtype == "bool":
        return b"t" if value else b"f"
    if dtype in ("int32", "int64", "uint32"):
        return str(int(value)).encode()
    if dtype == "float32":
        return rust_f32(value).encode()
    if dtype == "float64":
        return rust_f64(value).encode()
    if dtype == "utf8":
        return value.encode() if isinstance(value, str) else bytes(value)
    raise TypeError(dtype)


def data_row(cells: Sequence[Optional[bytes]]) -> bytes:
    body = struct.pack(">h", len(cells))
    for c in cells:
        body += struct.pack(">i", -1) if c is None else struct.pack(">i", len(c)) + c
    return b"D" + struct.pack(">i", 4 + len(body)) + body


def encode_rows(columns: Sequence[Tuple[str, list]]) -> List[bytes]:
    """columns: (dtype name, python values with None for NULL) -> one DataRow per row."""
    n = len(columns[0][1]) if columns else 0
    return [data_row([cell_text(dt, vals[i]) for dt, vals in columns]) for i in range(n)]
