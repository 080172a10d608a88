"""Multi-GPU execution: one process per GPU, torch.distributed over RCCL/xGMI.

Reference model (SURVEY.md §8 row e): the reference only simulates
distribution — hash partitioning (crates/query-distributed/src/partition.rs:151-212),
Exchange (operators.rs:15-73) and partial/final aggregate and shuffle-join stage
shapes (planner.rs:200-249) — and never executes workers.  Here the same
stages run for real:

  * shuffle(key, cols): device hash partition + move into partition-major
    order (qeh_partition_hash_move) -> ONE all_to_all per column over RCCL
    (counts first, so every rank knows its receive splits).
  * hash_join_inner: shuffle both sides by the join key, local device join.
  * group_by: local partial aggregate -> shuffle partial states by the first
    group key -> final aggregate on the owning rank (partial/final stages).
  * row_number: hash shuffle by the partition key, local ROW_NUMBER, reverse
    all-to-all, scatter back into input order.
  * sort: sample splitters, range partition, exchange, stable local sort.
  * join_filter_aggregate_broadcast (the BASELINE metric path): the dimension
    is replicated (broadcast join), every rank runs the fused kernel on its
    fact shard, then the partial states are shuffled by group key and merged.

The collectives carry device tensors under the "nccl" backend (RCCL on ROCm)
and host tensors under "gloo" (CPU rehearsal of the same code path).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import abi
from .device import NP_OF, Context, DeviceColumn, order_keys
from .expr import AggregateFunction as AF

TORCH_OF = {abi.DT_INT64: torch.int64, abi.DT_FLOAT64: torch.float64, abi.DT_INT32: torch.int32,
            abi.DT_FLOAT32: torch.float32, abi.DT_UINT32: torch.int32}


def exchange(send_counts: torch.Tensor, payloads: Sequence[torch.Tensor], group=None,
             byte_splits: Optional[dict] = None) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """All-to-all of partition-major payloads.  send_counts[r] rows of every
    payload go to rank r.  Returns (recv_counts, received payloads).
    byte_splits: {payload index: per-rank element counts} for payloads whose
    split is not the row split (the bytes of Utf8 columns); their receive
    sizes are exchanged first."""
    world = dist.get_world_size(group)
    send_counts = send_counts.to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    ins = [int(x) for x in send_counts.tolist()]
    outs = [int(x) for x in recv_counts.tolist()]
    assert len(ins) == world
    received = []
    for i, p in enumerate(payloads):
        pin, pout = ins, outs
        if byte_splits and i in byte_splits:
            sc = torch.tensor(byte_splits[i], dtype=torch.int64, device=send_counts.device)
            rc = torch.empty_like(sc)
            dist.all_to_all_single(rc, sc, group=group)
            pin, pout = [int(x) for x in byte_splits[i]], [int(x) for x in rc.tolist()]
        out = torch.empty((sum(pout),) + tuple(p.shape[1:]), dtype=p.dtype, device=p.device)
        dist.all_to_all_single(out, p.contiguous(), output_split_sizes=pout, input_split_sizes=pin, group=group)
        received.append(out)
    return recv_counts, received


# partial -> final aggregate decomposition (distributed/planner.rs:200-249 stage shape)
FINAL_OF = {AF.Count: AF.Sum, AF.Sum: AF.Sum, AF.Min: AF.Min, AF.Max: AF.Max}


class DistributedExecutor:
    def __init__(self, ctx: Context, group=None):
        self.ctx = ctx
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        self._keep: list = []  # tensors backing wrapped columns

    # ---- column <-> tensor ------------------------------------------------------
    def _bits_to_bytes(self, col: DeviceColumn, bits_ptr: int) -> torch.Tensor:
        """Bit-packed buffer (values of a Boolean column or any validity) -> one uint8 per row."""
        n = len(col)
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        c = abi.QehColumn()
        C.pointer(c)[0] = col.c
        c.validity = bits_ptr
        if n:
            abi.check(self.ctx.lib.qeh_validity_to_bytes(self.ctx.h, c, out.data_ptr()))
        return out

    def _to_tensors(self, col: DeviceColumn) -> List[torch.Tensor]:
        """Column -> payload tensors: values (Boolean: a byte per row; Utf8: int32 lengths, then
        the bytes), then validity bytes when the column has a bitmap."""
        n = len(col)
        if col.dtype in (abi.DT_UTF8, abi.DT_BOOL):
            if self.device == "cuda":
                if col.dtype == abi.DT_BOOL:
                    out = [self._bits_to_bytes(col, col.c.values)]
                else:
                    offs = torch.empty(n + 1, dtype=torch.int32, device="cuda")
                    self.ctx.copy_d2d(offs.data_ptr(), col.c.offsets + 4 * col.c.offset, 4 * (n + 1))
                    self.ctx.sync()
                    o0, o1 = (int(x) for x in offs[[0, n]].tolist())
                    data = torch.empty(max(o1 - o0, 0), dtype=torch.uint8, device="cuda")
                    if o1 > o0:
                        self.ctx.copy_d2d(data.data_ptr(), col.c.values + o0, o1 - o0)
                    out = [(offs[1:] - offs[:-1]).contiguous(), data]
                if col.c.validity:
                    out.append(self._bits_to_bytes(col, col.c.validity))
                return out
            v, m = col.to_numpy()
            if col.dtype == abi.DT_BOOL:
                out = [torch.from_numpy(np.asarray(v, np.uint8))]
            else:
                enc = [x.encode() for x in v]
                out = [torch.tensor([len(b) for b in enc], dtype=torch.int32),
                       torch.from_numpy(np.frombuffer(b"".join(enc), np.uint8).copy())]
            if col.c.validity:
                out.append(torch.from_numpy(m.astype(np.uint8)))
            return out
        tdt = TORCH_OF[col.dtype]
        if self.device == "cuda":
            vals = torch.empty(n, dtype=tdt, device="cuda")
            if n:
                item = vals.element_size()
                self.ctx.copy_d2d(vals.data_ptr(), col.c.values + col.c.offset * item, n * item)
            out = [vals]
            if col.c.validity:
                vb = torch.empty(n, dtype=torch.uint8, device="cuda")
                abi.check(self.ctx.lib.qeh_validity_to_bytes(self.ctx.h, col.c, vb.data_ptr()))
                out.append(vb)
            return out
        v, m = col.to_numpy()
        out = [torch.from_numpy(np.ascontiguousarray(v))]
        if col.c.validity:
            out.append(torch.from_numpy(m.astype(np.uint8)))
        return out

    def _from_tensors(self, dtype: int, vals, valid: Optional[torch.Tensor]) -> DeviceColumn:
        if dtype in (abi.DT_UTF8, abi.DT_BOOL):
            return self._from_tensors_var(dtype, vals, valid)
        n = vals.shape[0]
        if self.device == "cuda":
            bitmap = 0
            if valid is not None:
                bm = torch.zeros(((n + 63) // 64) * 8 + 8, dtype=torch.uint8, device="cuda")
                abi.check(self.ctx.lib.qeh_bytes_to_validity(self.ctx.h, valid.data_ptr(), n, bm.data_ptr()))
                self._keep.append(bm)
                bitmap = bm.data_ptr()
            self._keep.append(vals)
            return self.ctx.wrap_device(dtype, vals.data_ptr(), n, bitmap)
        v = vals.numpy().astype(NP_OF[dtype], copy=False)
        m = None if valid is None else valid.numpy().astype(bool)
        return self.ctx.upload(v, m)

    def _bytes_to_bits(self, b: torch.Tensor) -> torch.Tensor:
        n = b.shape[0]
        bm = torch.zeros(((n + 63) // 64) * 8 + 8, dtype=torch.uint8, device="cuda")
        if n:
            abi.check(self.ctx.lib.qeh_bytes_to_validity(self.ctx.h, b.data_ptr(), n, bm.data_ptr()))
        self._keep.append(bm)
        return bm

    def _from_tensors_var(self, dtype: int, vals, valid: Optional[torch.Tensor]) -> DeviceColumn:
        if self.device == "cuda":
            bitmap = self._bytes_to_bits(valid).data_ptr() if valid is not None else 0
            if dtype == abi.DT_BOOL:
                return self.ctx.wrap_device(dtype, self._bytes_to_bits(vals).data_ptr(), vals.shape[0], bitmap)
            lens, data = vals
            n = lens.shape[0]
            offs = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
            if n:
                offs[1:] = torch.cumsum(lens.to(torch.int64), 0).to(torch.int32)
            if data.shape[0] == 0:
                data = torch.zeros(8, dtype=torch.uint8, device="cuda")
            self._keep.extend([offs, data])
            return self.ctx.wrap_device(dtype, data.data_ptr(), n, bitmap, offsets=offs.data_ptr(),
                                        values_bytes=int(offs[-1].item()) if n else 0)
        m = None if valid is None else valid.numpy().astype(bool)
        if dtype == abi.DT_BOOL:
            return self.ctx.upload(vals.numpy().astype(bool), m)
        lens, data = vals
        raw = data.numpy().tobytes()
        cum = np.concatenate([[0], np.cumsum(lens.numpy().astype(np.int64))])
        strs = np.array([raw[cum[i]:cum[i + 1]].decode() for i in range(len(cum) - 1)], dtype=object)
        return self.ctx.upload(strs, m)

    def _sync(self):
        if self.device == "cuda":
            self.ctx.sync()

    # ---- shuffle -----------------------------------------------------------------
    def _exchange_columns(self, cols: Sequence[DeviceColumn], counts) -> Tuple[List[DeviceColumn], List[int]]:
        """All-to-all of partition-major columns: counts[r] leading rows go to rank r (Utf8
        bytes travel with their own per-rank byte counts)."""
        payloads, shape, byte_splits = [], [], {}
        bounds = np.concatenate([[0], np.cumsum(np.asarray(counts, np.int64))])
        for t in cols:
            ts = self._to_tensors(t)
            nvals = 2 if t.dtype == abi.DT_UTF8 else 1
            shape.append((t.dtype, len(ts) > nvals))
            if t.dtype == abi.DT_UTF8:  # bytes per destination from the row lengths
                lens = ts[0].to("cpu").numpy().astype(np.int64)
                cum = np.concatenate([[0], np.cumsum(lens)])
                byte_splits[len(payloads) + 1] = [int(cum[bounds[r + 1]] - cum[bounds[r]]) for r in range(self.world)]
            payloads.extend(ts)
        self._sync()
        recv_counts, recv = exchange(torch.tensor(np.asarray(counts), dtype=torch.int64, device=self.device), payloads,
                                     self.group, byte_splits)
        out, i = [], 0
        for dtype, nullable in shape:
            nvals = 2 if dtype == abi.DT_UTF8 else 1
            vals = recv[i:i + nvals]
            valid = recv[i + nvals] if nullable else None
            i += nvals + (1 if nullable else 0)
            out.append(self._from_tensors(dtype, vals[0] if nvals == 1 else vals, valid))
        return out, [int(x) for x in recv_counts.tolist()]

    def shuffle(self, key: DeviceColumn, cols: Sequence[DeviceColumn]) -> List[DeviceColumn]:
        """Route every row to rank hash(key) % world (partition.rs:151-212)."""
        counts, moved = self.ctx.partition_hash_move([key], self.world, cols)  # one device pass
        out, _ = self._exchange_columns(moved, counts)
        return out

    def exchange(self, strategy, batch) -> "object":
        """Exchange::execute across ranks (operators.rs:15-73, generalised to N GPUs): the
        device partitioner (qe_hip.partition) splits this rank's batch into world_size
        partitions — Hash / Range strategies must produce exactly world_size of them; Single
        gathers everything on rank 0 — and partition p is sent to rank p in one all-to-all.
        Returns the DeviceBatch this rank received (source-rank-major, stable)."""
        from .partition import DeviceBatch, Partitioner, Single
        if isinstance(strategy, Single):
            n = batch.num_rows()
            counts = np.zeros(self.world, np.int64)
            counts[0] = n
            cols = list(batch.columns)
        else:
            pt = Partitioner(self.ctx, strategy)
            if pt.num_partitions() != self.world:
                raise ValueError(f"exchange over {self.world} ranks needs {self.world} partitions, "
                                 f"strategy gives {pt.num_partitions()}")
            counts, cols = pt.batch_move(batch)
        recv, _ = self._exchange_columns(cols, counts)
        return DeviceBatch(list(batch.names), recv)

    # ---- operators -----------------------------------------------------------------
    def hash_join_inner(self, probe_key_idx: int, probe_cols: Sequence[DeviceColumn], build_key_idx: int,
                        build_cols: Sequence[DeviceColumn]):
        """Shuffle join: both sides hash-partitioned by the key, local device join."""
        p = self.shuffle(probe_cols[probe_key_idx], probe_cols)
        b = self.shuffle(build_cols[build_key_idx], build_cols)
        return self.ctx.hash_join_inner(p[probe_key_idx], p, b[build_key_idx], b)

    def _final(self, keys: Sequence[DeviceColumn], partials: Sequence[DeviceColumn], aggs: Sequence[Tuple[int, int]]):
        shuffled = self.shuffle(keys[0], list(keys) + list(partials))
        nk = len(keys)
        fk, fa, g = self.ctx.hash_aggregate(shuffled[:nk], shuffled[nk:],
                                            [(FINAL_OF[f], i) for i, (f, _) in enumerate(aggs)])
        return fk, fa, g

    def group_by(self, keys: Sequence[DeviceColumn], inputs: Sequence[DeviceColumn], aggs: Sequence[Tuple[int, int]]):
        """Partial aggregate locally, shuffle partial states by the first key,
        final aggregate on the owning rank.  Each rank returns the groups it owns."""
        for f, _ in aggs:
            if f not in FINAL_OF:
                raise NotImplementedError("distributed AVG needs SUM+COUNT partials; compose it from them")
        pk, pa_, g = self.ctx.hash_aggregate(keys, inputs, aggs)
        if g == 0 and not pk:
            pk = [self.ctx.empty(k.dtype, 0) for k in keys]
            pa_ = [self.ctx.empty(abi.DT_INT64, 0) for _ in aggs]
        return self._final(pk, pa_, aggs)

    def join_filter_aggregate_broadcast(self, probe_cols, probe_key_idx, predicate, build_key, build_group_keys,
                                        aggs):
        """Broadcast join: `build_*` replicated on every rank, `probe_cols` = this
        rank's shard.  Fused local pipeline, then partial/final merge."""
        for f, _ in aggs:
            if f not in FINAL_OF:
                raise NotImplementedError("distributed AVG needs SUM+COUNT partials; compose it from them")
        pk, pa_, g = self.ctx.join_filter_aggregate(probe_cols, probe_key_idx, predicate, build_key,
                                                    build_group_keys, aggs)
        return self._final(pk, pa_, aggs)

    def row_number(self, part_keys: Sequence[DeviceColumn], order_keys: Sequence[DeviceColumn],
                   ascending: Sequence[bool]) -> DeviceColumn:
        """ROW_NUMBER() OVER (PARTITION BY .. ORDER BY ..) over rank-sharded rows
        (global input order = rank-major).  Rows are hash-shuffled by the first
        partition key, so each PARTITION BY group lives on one rank and is numbered
        there (received order = source-rank-major, stable within a source, i.e. the
        global input order that breaks ties); the numbers go back by the reverse
        all-to-all and are scattered into this rank's input order."""
        counts, perm = self.ctx.hash_partition(part_keys[0], self.world)
        cols = list(part_keys) + list(order_keys)
        recv, recv_counts = self._exchange_columns([self.ctx.take(c, perm) for c in cols], counts)
        npk = len(part_keys)
        rn = self.ctx.row_number(recv[:npk], recv[npk:], list(ascending))
        back, _ = self._exchange_columns([rn], recv_counts)  # reverse: return what each source sent
        return self.ctx.scatter(back[0], perm)

    def window(self, func: int, part_keys: Sequence[DeviceColumn], order_keys: Sequence[DeviceColumn],
               ascending: Sequence[bool], arg: Optional[DeviceColumn] = None, param: int = 0,
               default=None) -> DeviceColumn:
        """Any ``WindowFunctionType`` OVER (PARTITION BY .. ORDER BY ..) over rank-sharded rows,
        placed like ``row_number``: hash shuffle by the first partition key (with the order keys
        and the argument), ``qeh_window`` on the owning rank, reverse all-to-all, then a gather
        through the inverse permutation (the results of LAG/LEAD/… carry NULLs)."""
        if not part_keys:
            raise ValueError("distributed window functions need a PARTITION BY key")
        counts, perm = self.ctx.hash_partition(part_keys[0], self.world)
        cols = list(part_keys) + list(order_keys) + ([arg] if arg is not None else [])
        recv, recv_counts = self._exchange_columns([self.ctx.take(c, perm) for c in cols], counts)
        npk, nok = len(part_keys), len(order_keys)
        res = self.ctx.window(func, recv[:npk], recv[npk:npk + nok], list(ascending),
                              arg=recv[npk + nok] if arg is not None else None, param=param, default=default)
        back, _ = self._exchange_columns([res], recv_counts)
        inv = self.ctx.scatter(self.ctx.upload(np.arange(len(part_keys[0]), dtype=np.uint32)), perm)
        return self.ctx.take(back[0], inv)

    def sort(self, cols: Sequence[DeviceColumn], key_idx: Sequence[int], ascending: Sequence[bool],
             samples_per_rank: int = 4096) -> List[DeviceColumn]:
        """ORDER BY over rank-sharded rows: range-partition on the first sort key
        with splitters from an all-gathered sample, then a stable local sort.  The
        global result is rank 0's rows, then rank 1's, ...  Equal first keys share a
        rank and arrive source-rank-major, so the result is stable."""
        k0 = cols[key_idx[0]]
        n = len(k0)
        sample = np.empty(0, np.int64)
        if n:
            idx = np.unique(np.linspace(0, n - 1, min(n, samples_per_rank)).astype(np.uint32))
            sv, sm = self.ctx.take(k0, self.ctx.upload(idx)).to_numpy()
            sample = order_keys(sv if sm is None else sv[sm])
        objs = [None] * self.world
        dist.all_gather_object(objs, sample, group=self.group)
        allk = np.sort(np.concatenate(objs)) if objs else np.empty(0, np.int64)
        if len(allk):
            splitters = allk[[(i + 1) * len(allk) // self.world for i in range(self.world - 1)]]
        else:
            splitters = np.zeros(self.world - 1, np.int64)
        counts, perm = self.ctx.range_partition(k0, splitters, bool(ascending[0]))
        recv, _ = self._exchange_columns([self.ctx.take(c, perm) for c in cols], counts)
        p = self.ctx.sort_indices([recv[i] for i in key_idx], list(ascending))
        return [self.ctx.take(c, p) for c in recv]

    def gather_to_root(self, cols: Sequence[DeviceColumn]) -> Optional[List[Tuple[np.ndarray, Optional[np.ndarray]]]]:
        """Collect every rank's result rows on rank 0 (host arrays)."""
        local = [c.to_numpy() for c in cols]
        objs = [None] * self.world
        dist.all_gather_object(objs, local, group=self.group)
        if self.rank != 0:
            return None
        out = []
        for j in range(len(cols)):
            vals = np.concatenate([o[j][0] for o in objs])
            masks = [o[j][1] if o[j][1] is not None else np.ones(len(o[j][0]), bool) for o in objs]
            out.append((vals, np.concatenate(masks)))
        return out
