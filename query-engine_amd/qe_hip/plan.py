"""Python mirror of the reference's `PhysicalPlan` enum and `QueryExecutor`.

    crates/query-executor/src/physical_plan.rs:13-72   PhysicalPlan
    crates/query-executor/src/executor.rs:12-21        QueryExecutor::{new, execute}
    crates/query-executor/src/physical_plan.rs:8-11    DataSource::{scan, schema}

`QueryExecutor(ctx).execute(plan)` flattens the plan into include/qeh_plan.h
nodes, exports every DataSource's batches through the Arrow C Data Interface,
runs `qeh_execute_plan` on the device and imports the result as
`list[pyarrow.RecordBatch]` — the same shape as the reference's
`Result<Vec<RecordBatch>>` (an empty list where the reference returns
`vec![]`).  Errors raise QehError carrying the reference's message.
"""
from __future__ import annotations

import ctypes as C
import itertools
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import pyarrow as pa

from . import abi
from .expr import AggregateExpr, PhysicalExpr

# ---- plan ABI structs (include/qeh_plan.h) ------------------------------------
PLAN_SCAN, PLAN_PROJECTION, PLAN_FILTER, PLAN_HASH_JOIN, PLAN_HASH_AGGREGATE, PLAN_SORT, PLAN_LIMIT, \
    PLAN_SUBQUERY_SCAN, PLAN_WINDOW, PLAN_INDEX_SCAN = range(10)


class JoinType:
    Inner, Left, Right, Full, Cross = range(5)


class WindowFunctionType:
    RowNumber, Rank, DenseRank, Ntile, Lag, Lead, FirstValue, LastValue = range(8)


class ArrowSchemaC(C.Structure):
    pass


ArrowSchemaC._fields_ = [("format", C.c_char_p), ("name", C.c_char_p), ("metadata", C.c_char_p),
                         ("flags", C.c_int64), ("n_children", C.c_int64),
                         ("children", C.POINTER(C.POINTER(ArrowSchemaC))), ("dictionary", C.POINTER(ArrowSchemaC)),
                         ("release", C.CFUNCTYPE(None, C.POINTER(ArrowSchemaC))), ("private_data", C.c_void_p)]


class ArrowArrayC(C.Structure):
    pass


ArrowArrayC._fields_ = [("length", C.c_int64), ("null_count", C.c_int64), ("offset", C.c_int64),
                        ("n_buffers", C.c_int64), ("n_children", C.c_int64), ("buffers", C.POINTER(C.c_void_p)),
                        ("children", C.POINTER(C.POINTER(ArrowArrayC))), ("dictionary", C.POINTER(ArrowArrayC)),
                        ("release", C.CFUNCTYPE(None, C.POINTER(ArrowArrayC))), ("private_data", C.c_void_p)]


class QehAggExprC(C.Structure):
    _fields_ = [("func", C.c_int32), ("_pad", C.c_int32), ("expr", abi.QehExpr)]


class QehWindowExprC(C.Structure):
    _fields_ = [("func", C.c_int32), ("n_args", C.c_int32), ("args", C.POINTER(abi.QehExpr)),
                ("n_partition", C.c_int32), ("n_order", C.c_int32), ("partition_by", C.POINTER(abi.QehExpr)),
                ("order_by", C.POINTER(abi.QehExpr))]


class QehPlanNodeC(C.Structure):
    _fields_ = [("kind", C.c_int32), ("input", C.c_int32), ("left", C.c_int32), ("right", C.c_int32),
                ("source", C.c_int32), ("join_type", C.c_int32), ("has_predicate", C.c_int32), ("n_exprs", C.c_int32),
                ("predicate", abi.QehExpr), ("exprs", C.POINTER(abi.QehExpr)), ("ascending", C.POINTER(C.c_int8)),
                ("aggs", C.POINTER(QehAggExprC)), ("window", C.POINTER(QehWindowExprC)), ("n_aggs", C.c_int32),
                ("n_window", C.c_int32), ("skip", C.c_int64), ("fetch", C.c_int64), ("n_fields", C.c_int32),
                ("_pad", C.c_int32), ("field_names", C.POINTER(C.c_char_p))]


class QehPlanC(C.Structure):
    _fields_ = [("nodes", C.POINTER(QehPlanNodeC)), ("n_nodes", C.c_int32), ("root", C.c_int32)]


class QehSourceC(C.Structure):
    _fields_ = [("schema", C.POINTER(ArrowSchemaC)), ("batches", C.POINTER(C.POINTER(ArrowArrayC))),
                ("n_batches", C.c_int64), ("cache_key", C.c_uint64)]


# ---- DataSource -------------------------------------------------------------------
class DataSource:
    """`DataSource` trait: scan() -> list of RecordBatch, schema()."""

    def scan(self) -> List[pa.RecordBatch]:
        raise NotImplementedError

    def schema(self) -> pa.Schema:
        raise NotImplementedError

    def cache_key(self) -> int:
        """Non-zero: scan() returns the same batches for as long as this key is in use, so the
        executor may keep their device copy between queries (qeh_source.cache_key). 0: import
        on every execute, as the reference re-scans on every execute (executor.rs:71-76)."""
        return 0


_next_cache_key = itertools.count(1)


class MemoryDataSource(DataSource):
    """crates/query-storage/src/memory.rs:305-308: scan() clones the batches.

    `device_cache=True` keeps the imported columns resident on the device between queries; the
    key changes whenever the batches do (`insert`), so a stale copy is never read."""

    def __init__(self, schema: pa.Schema, batches: Sequence[pa.RecordBatch], device_cache: bool = False):
        self._schema = schema
        self._batches = list(batches)
        self._device_cache = device_cache
        self._key = next(_next_cache_key) if device_cache else 0

    def insert(self, batch: pa.RecordBatch):
        """memory.rs insert_batch: append, and retire the cached device copy's key."""
        self._batches.append(batch)
        if self._device_cache:
            self._key = next(_next_cache_key)

    def cache_key(self) -> int:
        return self._key

    def scan(self):
        return list(self._batches)

    def schema(self):
        return self._schema


# ---- PhysicalPlan ------------------------------------------------------------------
class PhysicalPlan:
    pass


@dataclass
class Scan(PhysicalPlan):
    source: DataSource
    schema: Optional[List[str]] = None


@dataclass
class Projection(PhysicalPlan):
    input: PhysicalPlan
    exprs: List[PhysicalExpr]
    schema: List[str]  # field names of the planner schema (table-prefixed, planner.rs:80-81)


@dataclass
class Filter(PhysicalPlan):
    input: PhysicalPlan
    predicate: PhysicalExpr


@dataclass
class HashJoin(PhysicalPlan):
    left: PhysicalPlan
    right: PhysicalPlan
    join_type: int
    on: Optional[PhysicalExpr]


@dataclass
class HashAggregate(PhysicalPlan):
    input: PhysicalPlan
    group_exprs: List[PhysicalExpr]
    aggr_exprs: List[AggregateExpr]


@dataclass
class Sort(PhysicalPlan):
    input: PhysicalPlan
    exprs: List[PhysicalExpr]
    ascending: List[bool]


@dataclass
class Limit(PhysicalPlan):
    input: PhysicalPlan
    skip: int
    fetch: Optional[int]


@dataclass
class SubqueryScan(PhysicalPlan):
    subquery: PhysicalPlan
    schema: Optional[List[str]] = None


@dataclass
class WindowExpr:
    func: int
    args: List[PhysicalExpr] = field(default_factory=list)
    partition_by: List[PhysicalExpr] = field(default_factory=list)
    order_by: List[PhysicalExpr] = field(default_factory=list)


@dataclass
class Window(PhysicalPlan):
    input: PhysicalPlan
    window_exprs: List[WindowExpr]
    schema: List[str]


@dataclass
class IndexScan(PhysicalPlan):
    source: DataSource
    index_name: str = ""
    lookup_keys: list = field(default_factory=list)
    is_range_scan: bool = False
    schema: Optional[List[str]] = None


# ---- flattening -------------------------------------------------------------------
class _Flattener:
    def __init__(self):
        self.nodes: List[QehPlanNodeC] = []
        self.keep: list = []
        self.sources: List[DataSource] = []

    def expr(self, e: PhysicalExpr) -> abi.QehExpr:
        c, arr = e.to_c()
        self.keep.append(arr)
        return c

    def exprs(self, es: Sequence[PhysicalExpr]):
        if not es:
            return None
        arr = (abi.QehExpr * len(es))(*[self.expr(e) for e in es])
        self.keep.append(arr)
        return arr

    def names(self, ns: Optional[Sequence[str]]):
        if not ns:
            return None, 0
        arr = (C.c_char_p * len(ns))(*[n.encode() for n in ns])
        self.keep.append(arr)
        return arr, len(ns)

    def add(self, p: PhysicalPlan) -> int:
        n = QehPlanNodeC(input=-1, left=-1, right=-1, source=-1, fetch=-1)
        if isinstance(p, (Scan, IndexScan)):
            n.kind = PLAN_SCAN if isinstance(p, Scan) else PLAN_INDEX_SCAN
            n.source = len(self.sources)
            self.sources.append(p.source)
        elif isinstance(p, Projection):
            n.kind = PLAN_PROJECTION
            n.input = self.add(p.input)
            n.n_exprs = len(p.exprs)
            n.exprs = self.exprs(p.exprs)
            n.field_names, n.n_fields = self.names(p.schema)
        elif isinstance(p, Filter):
            n.kind = PLAN_FILTER
            n.input = self.add(p.input)
            n.has_predicate = 1
            n.predicate = self.expr(p.predicate)
        elif isinstance(p, HashJoin):
            n.kind = PLAN_HASH_JOIN
            n.left = self.add(p.left)
            n.right = self.add(p.right)
            n.join_type = p.join_type
            if p.on is not None:
                n.has_predicate = 1
                n.predicate = self.expr(p.on)
        elif isinstance(p, HashAggregate):
            n.kind = PLAN_HASH_AGGREGATE
            n.input = self.add(p.input)
            n.n_exprs = len(p.group_exprs)
            n.exprs = self.exprs(p.group_exprs)
            if p.aggr_exprs:
                arr = (QehAggExprC * len(p.aggr_exprs))(*[QehAggExprC(a.func, 0, self.expr(a.expr)) for a in p.aggr_exprs])
                self.keep.append(arr)
                n.aggs = arr
            n.n_aggs = len(p.aggr_exprs)
        elif isinstance(p, Sort):
            n.kind = PLAN_SORT
            n.input = self.add(p.input)
            n.n_exprs = len(p.exprs)
            n.exprs = self.exprs(p.exprs)
            if p.exprs:
                asc = (C.c_int8 * len(p.exprs))(*[1 if (p.ascending[i] if i < len(p.ascending) else True) else 0
                                                  for i in range(len(p.exprs))])
                self.keep.append(asc)
                n.ascending = asc
        elif isinstance(p, Limit):
            n.kind = PLAN_LIMIT
            n.input = self.add(p.input)
            n.skip = p.skip
            n.fetch = -1 if p.fetch is None else p.fetch
        elif isinstance(p, SubqueryScan):
            n.kind = PLAN_SUBQUERY_SCAN
            n.input = self.add(p.subquery)
        elif isinstance(p, Window):
            n.kind = PLAN_WINDOW
            n.input = self.add(p.input)
            ws = []
            for w in p.window_exprs:
                ws.append(QehWindowExprC(w.func, len(w.args), self.exprs(w.args), len(w.partition_by), len(w.order_by),
                                         self.exprs(w.partition_by), self.exprs(w.order_by)))
            if ws:
                arr = (QehWindowExprC * len(ws))(*ws)
                self.keep.append(arr)
                n.window = arr
            n.n_window = len(ws)
            n.field_names, n.n_fields = self.names(p.schema)
        else:
            raise TypeError(f"unknown plan node {p!r}")
        self.nodes.append(n)
        return len(self.nodes) - 1


class QueryExecutor:
    """`QueryExecutor::new()` / `execute(&PhysicalPlan)` on the device."""

    def __init__(self, ctx):
        self.ctx = ctx
        lib = abi.load()
        self.fn = lib.qeh_execute_plan
        self.fn.restype = C.c_int
        self.fn.argtypes = [C.c_void_p, C.POINTER(QehPlanC), C.POINTER(QehSourceC), C.c_int,
                            C.POINTER(ArrowSchemaC), C.POINTER(ArrowArrayC), C.POINTER(C.c_int64)]

    def execute(self, plan: PhysicalPlan) -> List[pa.RecordBatch]:
        fl = _Flattener()
        root = fl.add(plan)
        nodes = (QehPlanNodeC * len(fl.nodes))(*fl.nodes)
        cplan = QehPlanC(C.cast(nodes, C.POINTER(QehPlanNodeC)), len(fl.nodes), root)
        exported = []  # (schema struct, [array structs]) to release after the call
        srcs = []
        for ds in fl.sources:
            batches = ds.scan()
            sch = ArrowSchemaC()
            ds.schema()._export_to_c(C.addressof(sch))
            arrs = []
            for b in batches:
                a = ArrowArrayC()
                b._export_to_c(C.addressof(a))
                arrs.append(a)
            ptrs = (C.POINTER(ArrowArrayC) * max(len(arrs), 1))(*[C.pointer(a) for a in arrs])
            srcs.append(QehSourceC(C.pointer(sch), C.cast(ptrs, C.POINTER(C.POINTER(ArrowArrayC))), len(arrs),
                                   int(ds.cache_key())))
            exported.append((sch, arrs, ptrs))
        src_arr = (QehSourceC * max(len(srcs), 1))(*srcs)
        out_s, out_a, nb = ArrowSchemaC(), ArrowArrayC(), C.c_int64()
        try:
            abi.check(self.fn(self.ctx.h, C.byref(cplan), src_arr, len(srcs), C.byref(out_s), C.byref(out_a),
                              C.byref(nb)))
        finally:
            for sch, arrs, _ in exported:
                for a in arrs:
                    if a.release:
                        a.release(C.pointer(a))
                if sch.release:
                    sch.release(C.pointer(sch))
        if nb.value == 0:
            return []
        return [pa.RecordBatch._import_from_c(C.addressof(out_a), C.addressof(out_s))]

    # ---- device-resident Scan cache (qeh_source_cache_*) ----
    def cache_stats(self) -> dict:
        lib = abi.load()
        e, b, h, m = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        abi.check(lib.qeh_source_cache_stats(self.ctx.h, C.byref(e), C.byref(b), C.byref(h), C.byref(m)))
        return {"entries": e.value, "bytes": b.value, "hits": h.value, "misses": m.value}

    def cache_evict(self, source: Optional[DataSource] = None):
        """Drop `source`'s device copy (all copies when None)."""
        lib = abi.load()
        key = 0 if source is None else int(source.cache_key())
        if source is not None and key == 0:
            return
        abi.check(lib.qeh_source_cache_evict(self.ctx.h, C.c_uint64(key)))

    def cache_budget(self, nbytes: int):
        lib = abi.load()
        abi.check(lib.qeh_source_cache_budget(self.ctx.h, C.c_int64(nbytes)))
