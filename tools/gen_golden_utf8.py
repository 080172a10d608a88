#!/usr/bin/env python3
"""Generate tests/golden/utf8_cmp.npz (run in the build container only).

Utf8 comparisons as the reference calls them (operators.rs:509-538 -> arrow-rs cmp kernels on
StringArray) pinned by Arrow C++ (pyarrow): pc.equal / not_equal / less / less_equal / greater /
greater_equal on string arrays, column vs column and column vs a scalar literal, nulls
propagated.  Strings are stored as offsets (int32) + bytes (uint8); written with
allow_pickle=False.
"""
import os

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "utf8_cmp.npz")
N = 2048
FUNCS = {"eq": pc.equal, "neq": pc.not_equal, "lt": pc.less, "lt_eq": pc.less_equal,
         "gt": pc.greater, "gt_eq": pc.greater_equal}
LITERALS = ["", "M", "Bob", "ab", "ab\x00", "été", "zzzz"]


def strings(r, n):
    alphabet = ["a", "b", "B", "z", "é", "\x00", "Bo", "ab"]
    out = []
    for _ in range(n):
        k = int(r.integers(0, 6))
        out.append("".join(alphabet[int(j)] for j in r.integers(0, len(alphabet), k)))
    return out


def put(d, name, arr: pa.Array):
    arr = arr.cast(pa.string())
    offs = np.frombuffer(arr.buffers()[1], np.int32)[arr.offset:arr.offset + len(arr) + 1]
    data = np.frombuffer(arr.buffers()[2], np.uint8) if arr.buffers()[2] is not None else np.zeros(0, np.uint8)
    d[name + "_offsets"] = (offs - offs[0]).astype(np.int32)
    d[name + "_bytes"] = data[offs[0]:offs[-1]].copy()
    d[name + "_valid"] = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), bool)


def main():
    r = np.random.default_rng(77)
    a = pa.array(strings(r, N), pa.string(), mask=r.random(N) < 0.1)
    b = pa.array(strings(r, N), pa.string(), mask=r.random(N) < 0.1)
    d = {}
    put(d, "a", a)
    put(d, "b", b)
    put(d, "lit", pa.array(LITERALS, pa.string()))  # offsets + bytes: keeps trailing NULs
    for op, f in FUNCS.items():
        res = f(a, b)
        d[f"col_{op}_values"] = np.asarray(res.fill_null(False).to_numpy(zero_copy_only=False), bool)
        d[f"col_{op}_valid"] = ~np.asarray(res.is_null().to_numpy(zero_copy_only=False), bool)
        for j, lit in enumerate(LITERALS):
            res = f(a, pa.scalar(lit, pa.string()))
            d[f"lit{j}_{op}_values"] = np.asarray(res.fill_null(False).to_numpy(zero_copy_only=False), bool)
            d[f"lit{j}_{op}_valid"] = ~np.asarray(res.is_null().to_numpy(zero_copy_only=False), bool)
    np.savez_compressed(OUT, **d)
    print("wrote", OUT, len(d), "arrays")


if __name__ == "__main__":
    main()
