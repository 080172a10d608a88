"""`Merge` — combining partition results on the device.

Mirrors crates/query-distributed/src/operators.rs:75-224: `Merge(schema, strategy)`, with
`MergeStrategy.Concat` (flatten, :139-141), `SortedMerge(sort_columns)` (concat_batches, then a
lexsort by the named columns with per-column ascending / nulls_first; names that do not resolve
are skipped, and with none left the concatenation is returned, :143-193) and
`UnionDistinct(key_columns)` (the reference concatenates without deduplicating, :196-204).

A batch here is a list of `DeviceColumn`s in schema order; `partitions` is a list (one entry per
partition) of lists of batches, exactly the reference's `Vec<Vec<RecordBatch>>`.  SortedMerge
runs as one `qeh_merge_sorted` call (device concat + LSD radix sort + gathers).  Ties keep the
concatenation order (the device sort is stable; arrow's lexsort_to_indices may order ties
either way, so any tie order matches the reference).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

from .device import Context, DeviceColumn


@dataclass
class SortColumn:
    name: str
    ascending: bool = True
    nulls_first: bool = True


@dataclass
class Concat:
    pass


@dataclass
class SortedMerge:
    sort_columns: List[SortColumn] = field(default_factory=list)


@dataclass
class UnionDistinct:
    key_columns: List[str] = field(default_factory=list)


class MergeStrategy:
    Concat = Concat
    SortedMerge = SortedMerge
    UnionDistinct = UnionDistinct


Batch = List[DeviceColumn]


class Merge:
    def __init__(self, ctx: Context, schema: Sequence[str], strategy):
        self.ctx = ctx
        self._schema = list(schema)
        self.strategy = strategy

    @classmethod
    def concat(cls, ctx: Context, schema: Sequence[str]) -> "Merge":
        return cls(ctx, schema, Concat())

    @classmethod
    def sorted(cls, ctx: Context, schema: Sequence[str], sort_columns: Sequence[SortColumn]) -> "Merge":
        return cls(ctx, schema, SortedMerge(list(sort_columns)))

    def schema(self) -> List[str]:
        return list(self._schema)

    def execute(self, partitions: Sequence[Sequence[Batch]]) -> List[Batch]:
        batches = [b for p in partitions for b in p]
        if isinstance(self.strategy, (Concat, UnionDistinct)):
            return batches
        if not isinstance(self.strategy, SortedMerge):
            raise TypeError(f"unknown merge strategy {self.strategy!r}")
        if not batches:
            return []
        keys = [(self._schema.index(sc.name), sc) for sc in self.strategy.sort_columns if sc.name in self._schema]
        cols, _ = self.ctx.merge_sorted(batches, [i for i, _ in keys], [sc.ascending for _, sc in keys],
                                        [sc.nulls_first for _, sc in keys])
        return [cols]
