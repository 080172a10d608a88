"""`Partitioner` / `Exchange` on the device.

Mirrors crates/query-distributed/src/partition.rs (PartitionStrategy :21-46, Partition :56-90,
Partitioner :93-357) and operators.rs:15-73 (Exchange).  A batch is a `DeviceBatch` (field names
+ device columns), since the reference resolves key columns by name in each batch's schema.

* Hash: per batch, `qeh_partition_hash_move` over the named key columns (names that do not
  resolve are skipped; none resolving is the reference's "No key columns found in batch" error):
  partition ids, then the columns moved to partition-major order in one tile-ranked pass, sliced
  per partition; empty partition batches are not added (partition.rs:190-193).
* Range: `qeh_partition_range` (first boundary the Int64 value is below; NULL / other types -> 0).
  A missing key column is the reference's "Key column '<name>' not found" error.
* RoundRobin: whole batches, batch i -> partition i % n (partition.rs:215-229).
* Single: every batch in partition 0.

The partition a hashed key lands in differs from the reference's SipHash choice; it is not
observable in query results, and rows with equal keys always share one.
Multi-GPU: `qe_hip.distributed.DistributedExecutor.exchange` sends partition p to rank p.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .device import Context, DeviceColumn


@dataclass
class DeviceBatch:
    names: List[str]
    columns: List[DeviceColumn]

    def num_rows(self) -> int:
        return len(self.columns[0]) if self.columns else 0


@dataclass
class Hash:
    key_columns: List[str]
    num_partitions: int


@dataclass
class Range:
    key_column: str
    boundaries: List[int]  # RangeBoundary::Int64 values; other boundary kinds never match


@dataclass
class RoundRobin:
    num_partitions: int = 4  # PartitionStrategy::default (partition.rs:48-52)


@dataclass
class Single:
    pass


class PartitionStrategy:
    Hash = Hash
    Range = Range
    RoundRobin = RoundRobin
    Single = Single


@dataclass
class Partition:
    index: int
    batches: List[DeviceBatch] = field(default_factory=list)
    worker: Optional[int] = None

    def add_batch(self, batch: DeviceBatch):
        self.batches.append(batch)

    def row_count(self) -> int:
        return sum(b.num_rows() for b in self.batches)

    def assign_to(self, worker_id: int):
        self.worker = worker_id


class PartitionError(RuntimeError):
    pass


def _fnv_fmix(data: bytes) -> int:
    h = 0xcbf29ce484222325
    for b in data:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    h ^= h >> 33
    h = (h * 0xff51afd7ed558ccd) & 0xFFFFFFFFFFFFFFFF
    h ^= h >> 33
    h = (h * 0xc4ceb9fe1a85ec53) & 0xFFFFFFFFFFFFFFFF
    return h ^ (h >> 33)


class Partitioner:
    def __init__(self, ctx: Context, strategy):
        self.ctx = ctx
        self.strategy = strategy

    @classmethod
    def hash(cls, ctx: Context, key_columns: Sequence[str], num_partitions: int) -> "Partitioner":
        return cls(ctx, Hash(list(key_columns), num_partitions))

    @classmethod
    def round_robin(cls, ctx: Context, num_partitions: int) -> "Partitioner":
        return cls(ctx, RoundRobin(num_partitions))

    def num_partitions(self) -> int:
        s = self.strategy
        if isinstance(s, Hash):
            return s.num_partitions
        if isinstance(s, Range):
            return len(s.boundaries) + 1
        if isinstance(s, RoundRobin):
            return s.num_partitions
        return 1

    # ---- device partition of one batch: (counts, partition-major permutation) ----
    def batch_permutation(self, batch: DeviceBatch):
        s = self.strategy
        if isinstance(s, Hash):
            idx = [batch.names.index(n) for n in s.key_columns if n in batch.names]
            if not idx:
                raise PartitionError("No key columns found in batch")
            keys = [batch.columns[i] for i in idx]
            counts = (C.c_int64 * s.num_partitions)()
            out = abi.QehColumn()
            abi.check(self.ctx.lib.qeh_partition_hash(self.ctx.h, self.ctx._cols(keys), len(keys), s.num_partitions,
                                                      counts, C.byref(out)))
            return np.array(counts[:], np.int64), self.ctx._wrap(out)
        if isinstance(s, Range):
            if s.key_column not in batch.names:
                raise PartitionError(f"Key column '{s.key_column}' not found")
            key = batch.columns[batch.names.index(s.key_column)]
            b = np.ascontiguousarray(np.asarray(s.boundaries, np.int64))
            counts = (C.c_int64 * (len(b) + 1))()
            out = abi.QehColumn()
            abi.check(self.ctx.lib.qeh_partition_range(self.ctx.h, C.byref(key.c),
                                                       b.ctypes.data_as(C.POINTER(C.c_int64)), len(b), counts,
                                                       C.byref(out)))
            return np.array(counts[:], np.int64), self.ctx._wrap(out)
        raise TypeError("batch_permutation: row-level strategies only (Hash, Range)")

    def batch_move(self, batch: DeviceBatch):
        """(counts, the batch's columns in partition-major order): Hash moves the columns in one
        device pass (qeh_partition_hash_move), Range through the permutation."""
        s = self.strategy
        if isinstance(s, Hash):
            idx = [batch.names.index(n) for n in s.key_columns if n in batch.names]
            if not idx:
                raise PartitionError("No key columns found in batch")
            return self.ctx.partition_hash_move([batch.columns[i] for i in idx], s.num_partitions, batch.columns)
        counts, perm = self.batch_permutation(batch)
        return counts, [self.ctx.take(c, perm) for c in batch.columns]

    def partition(self, batches: Sequence[DeviceBatch]) -> List[Partition]:
        s = self.strategy
        parts = [Partition(i) for i in range(self.num_partitions())]
        if isinstance(s, Single):
            for b in batches:
                parts[0].add_batch(b)
            return parts
        if isinstance(s, RoundRobin):
            for i, b in enumerate(batches):
                parts[i % s.num_partitions].add_batch(b)
            return parts
        for b in batches:
            counts, moved = self.batch_move(b)
            off = 0
            for p, cnt in enumerate(counts):
                if cnt:
                    parts[p].add_batch(DeviceBatch(list(b.names), [self.ctx.slice(c, off, int(cnt)) for c in moved]))
                off += int(cnt)
        return parts

    def route(self, key: bytes) -> int:
        """Partitioner::route (partition.rs:343-356): Hash and RoundRobin hash the key bytes."""
        s = self.strategy
        if isinstance(s, (Hash, RoundRobin)):
            return _fnv_fmix(bytes(key)) % s.num_partitions
        return 0


class Exchange:
    """operators.rs:15-73."""

    def __init__(self, ctx: Context, strategy, num_partitions: int):
        self.ctx = ctx
        self.strategy = strategy
        self._n = num_partitions

    @classmethod
    def hash(cls, ctx: Context, columns: Sequence[str], num_partitions: int) -> "Exchange":
        return cls(ctx, Hash(list(columns), num_partitions), num_partitions)

    @classmethod
    def round_robin(cls, ctx: Context, num_partitions: int) -> "Exchange":
        return cls(ctx, RoundRobin(num_partitions), num_partitions)

    @classmethod
    def gather(cls, ctx: Context) -> "Exchange":
        return cls(ctx, Single(), 1)

    def execute(self, batches: Sequence[DeviceBatch]) -> List[Partition]:
        return Partitioner(self.ctx, self.strategy).partition(batches)

    def route(self, key: bytes) -> int:
        return Partitioner(self.ctx, self.strategy).route(key)

    def num_partitions(self) -> int:
        return self._n
