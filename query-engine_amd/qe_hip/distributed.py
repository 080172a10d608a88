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
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import abi
from .device import NP_OF, Context, DeviceColumn, order_keys
from .expr import AggregateFunction as AF
from .plan import WindowFunctionType as W

TORCH_OF = {abi.DT_INT64: torch.int64, abi.DT_FLOAT64: torch.float64, abi.DT_INT32: torch.int32,
            abi.DT_FLOAT32: torch.float32, abi.DT_UINT32: torch.int32}


def exchange(send_counts: torch.Tensor, payloads: Sequence[torch.Tensor], group=None,
             byte_splits: Optional[dict] = None) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """All-to-all of partition-major payloads (host-level helper used by the CPU tests).
    send_counts[r] rows of every payload go to rank r.  Returns (recv_counts, received).
    byte_splits: {payload index: per-rank element counts} for payloads whose split is not the
    row split (the bytes of Utf8 columns).  All sizes travel in ONE all_gather of a metadata
    vector; the payloads then move with one all_to_all_single each."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    byte_splits = byte_splits or {}
    keys = sorted(byte_splits)
    meta = np.concatenate([np.asarray(send_counts.cpu().numpy() if isinstance(send_counts, torch.Tensor) else send_counts,
                                      np.int64)] + [np.asarray(byte_splits[i], np.int64) for i in keys])
    dev = payloads[0].device if payloads else torch.device("cpu")
    M = _allgather_meta(meta, world, dev, group)
    recv_counts = torch.tensor(M[:, rank], dtype=torch.int64)
    received = []
    for i, p in enumerate(payloads):
        if i in byte_splits:
            j = keys.index(i)
            S = M[:, world * (j + 1):world * (j + 2)]
        else:
            S = M[:, :world]
        pin = [int(x) for x in S[rank]]
        pout = [int(x) for x in S[:, rank]]
        received.append(_all_to_all(p, pin, pout, _peak_remote(S), group))
    return recv_counts, received


def _allgather_meta(meta: np.ndarray, world: int, device, group=None) -> np.ndarray:
    """all_gather of one int64 vector per rank -> [world, len] on the host (one host sync)."""
    return _allgather_meta_t(torch.from_numpy(np.ascontiguousarray(meta, np.int64)).to(device), world, group)


def _allgather_meta_t(t: torch.Tensor, world: int, group=None) -> np.ndarray:
    out = torch.empty(world * t.numel(), dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t.to(torch.int64).contiguous(), group=group)
    return out.cpu().numpy().reshape(world, -1)


# Largest message per peer in one RCCL round of an exchange.  RCCL 2.26 (the torch wheel's)
# loses the second half of a world-1 all_to_all self-send once it passes ~1 GB
# (tools/debug/a2a_big.py: 0.8 GB intact, 1.6 GB half wrong); large exchanges therefore never
# self-send through RCCL and move in rounds of at most this many bytes per peer.
A2A_CHUNK_BYTES = int(os.environ.get("QEH_A2A_CHUNK_BYTES", 256 << 20))


def _peak_remote(splits: np.ndarray) -> int:
    """Largest off-diagonal entry of a [world, world] split matrix (rows rank i sends to rank j):
    the most any rank sends to another.  Every rank holds the same matrix (it comes from one
    all_gather), so every rank derives the same round count from it."""
    m = np.array(splits, np.int64, copy=True).reshape(len(splits), -1)
    np.fill_diagonal(m, 0)
    return int(m.max()) if m.size else 0


def _a2a_rounds(pin: Sequence[int], pout: Sequence[int], me: int, row_bytes: int, chunk_bytes: int,
                peak: int) -> List[List[Tuple[int, int, int, int]]]:
    """The round plan of a chunked all-to-all (shared by every backend): rounds[t][r] =
    (a, b, c, d) — rows [a, b) of the partition for rank r are sent and rows [c, d) of what rank r
    sends here are received in round t (offsets inside the partitions).  At most chunk_bytes per
    peer per round; the local partition (r == me) never takes part.  The round count comes from
    `peak` (_peak_remote of the job-wide split matrix), not from this rank's own splits, so every
    rank issues the same number of collectives — a rank with nothing left to move joins the later
    rounds with empty slices (gloo's all-to-all is a collective every rank must enter)."""
    world = len(pin)
    cap = max(chunk_bytes // max(row_bytes, 1), 1)
    n_rounds = (peak + cap - 1) // cap
    rounds = []
    for t in range(n_rounds):
        plan = []
        for r in range(world):
            if r == me:
                plan.append((0, 0, 0, 0))
                continue
            plan.append((min(t * cap, pin[r]), min((t + 1) * cap, pin[r]),
                         min(t * cap, pout[r]), min((t + 1) * cap, pout[r])))
        rounds.append(plan)
    return rounds


def _all_to_all(p: torch.Tensor, pin: Sequence[int], pout: Sequence[int], peak: int, group=None,
                istarts: Optional[Sequence[int]] = None, pad: int = 0) -> torch.Tensor:
    """Variable all-to-all of one partition-major payload: pin[r] leading rows go to rank r,
    pout[r] rows arrive from rank r; peak = _peak_remote of the job-wide split matrix.  With
    `istarts`, rank r's rows are p[istarts[r] : istarts[r] + pin[r]] instead (per-destination blocks
    at fixed places, as qeh_shuffle_items_pack leaves them); `pad` rows of slack after the received
    rows (world > 1).  The local partition never goes through the collective
    (one copy, or the input itself at world size 1); the remote partitions move in the rounds of
    _a2a_rounds (at most A2A_CHUNK_BYTES per peer each).  Only the collective of a round depends on
    the backend: under "nccl" grouped send/recv of the views (dist.all_to_all over views,
    ncclGroupStart/End, no packing); under "gloo" the round's slices are packed into one buffer for
    all_to_all_single and unpacked into their places."""
    world = len(pin)
    me = dist.get_rank(group)
    if world == 1:
        if istarts is not None:
            p = p[int(istarts[0]):int(istarts[0]) + int(pin[0])]
        return p if p.is_contiguous() else p.contiguous()
    p = p.contiguous()
    shape = tuple(p.shape[1:])
    out = torch.empty((sum(pout) + pad,) + shape, dtype=p.dtype, device=p.device)
    ioff = np.concatenate([[0], np.cumsum(pin)]).astype(np.int64) if istarts is None else \
        np.asarray([int(x) for x in istarts], np.int64)
    ooff = np.concatenate([[0], np.cumsum(pout)]).astype(np.int64)
    if pin[me]:
        out[ooff[me]:ooff[me] + pout[me]].copy_(p[ioff[me]:ioff[me] + pin[me]])
    row_bytes = p.element_size() * int(np.prod(shape, dtype=np.int64))
    grouped = dist.get_backend(group) == "nccl"
    for plan in _a2a_rounds(pin, pout, me, row_bytes, A2A_CHUNK_BYTES, peak):
        ins = [p[ioff[r] + a:ioff[r] + b] for r, (a, b, _, _) in enumerate(plan)]
        outs = [out[ooff[r] + c:ooff[r] + d] for r, (_, _, c, d) in enumerate(plan)]
        if grouped:
            dist.all_to_all(outs, ins, group=group)
        else:
            recv = torch.empty((sum(o.shape[0] for o in outs),) + shape, dtype=p.dtype, device=p.device)
            dist.all_to_all_single(recv, torch.cat(ins) if ins else p[:0], output_split_sizes=[o.shape[0] for o in outs],
                                   input_split_sizes=[i.shape[0] for i in ins], group=group)
            q = 0
            for o in outs:
                o.copy_(recv[q:q + o.shape[0]])
                q += o.shape[0]
    return out


def _without_bitmap(ctx: Context, col: DeviceColumn) -> DeviceColumn:
    """A view of `col` without its validity bitmap (for columns known to hold no NULL)."""
    c = abi.QehColumn()
    C.pointer(c)[0] = col.c
    c.owned = 0
    c.validity = None
    c.null_count = 0
    d = DeviceColumn(ctx, c)
    d.parent = col
    return d


class _DeviceView:
    """__cuda_array_interface__ over a library-owned device buffer: torch.as_tensor wraps it
    without a copy and keeps this object (and the column it references) alive."""

    def __init__(self, ptr: int, n: int, typestr: str, owner):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2,
                                         "strides": None}


TYPESTR = {abi.DT_INT64: "<i8", abi.DT_FLOAT64: "<f8", abi.DT_INT32: "<i4", abi.DT_FLOAT32: "<f4",
           abi.DT_UINT32: "<u4"}


# partial -> final aggregate decomposition (distributed/planner.rs:200-249 stage shape)
FINAL_OF = {AF.Count: AF.Sum, AF.Sum: AF.Sum, AF.Min: AF.Min, AF.Max: AF.Max}


class DistributedExecutor:
    def __init__(self, ctx: Context, group=None, device: Optional[str] = None):
        """device: where payloads live during collectives — "cuda" under "nccl" (RCCL), "cpu" under
        "gloo" by default.  device="cuda" with gloo keeps the device-tensor code paths (zero-copy
        views, the overlapped dimension all-gather, the dense final aggregate) with gloo staging
        through the host: the multi-rank rehearsal of the RCCL path on one GPU."""
        self.ctx = ctx
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
        self.last_final = None  # how the last broadcast join merged its partial states

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
            item = torch.empty(0, dtype=tdt).element_size()
            if n:  # a zero-copy view of the column's values (the view keeps the column alive)
                vals = torch.as_tensor(_DeviceView(col.c.values + col.c.offset * item, n, TYPESTR[col.dtype], col),
                                       device="cuda")
            else:
                vals = torch.empty(0, dtype=tdt, device="cuda")
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
            keep = [vals]
            bitmap = 0
            if valid is not None:
                bm = torch.zeros(((n + 63) // 64) * 8 + 8, dtype=torch.uint8, device="cuda")
                if n:
                    abi.check(self.ctx.lib.qeh_bytes_to_validity(self.ctx.h, valid.data_ptr(), n, bm.data_ptr()))
                keep.append(bm)
                bitmap = bm.data_ptr()
            if n == 0:  # a non-null pointer for empty columns
                keep[0] = torch.empty(1, dtype=vals.dtype, device="cuda")
            d = self.ctx.wrap_device(dtype, keep[0].data_ptr(), n, bitmap)
            d.parent = keep  # the torch buffers live as long as the column
            return d
        v = vals.numpy().astype(NP_OF[dtype], copy=False)
        m = None if valid is None else valid.numpy().astype(bool)
        return self.ctx.upload(v, m)

    def _bytes_to_bits(self, b: torch.Tensor) -> torch.Tensor:
        n = b.shape[0]
        bm = torch.zeros(((n + 63) // 64) * 8 + 8, dtype=torch.uint8, device="cuda")
        if n:
            abi.check(self.ctx.lib.qeh_bytes_to_validity(self.ctx.h, b.data_ptr(), n, bm.data_ptr()))
        return bm

    def _from_tensors_var(self, dtype: int, vals, valid: Optional[torch.Tensor]) -> DeviceColumn:
        if self.device == "cuda":
            keep = []
            bitmap = 0
            if valid is not None:
                keep.append(self._bytes_to_bits(valid))
                bitmap = keep[-1].data_ptr()
            if dtype == abi.DT_BOOL:
                keep.append(self._bytes_to_bits(vals))
                d = self.ctx.wrap_device(dtype, keep[-1].data_ptr(), vals.shape[0], bitmap)
                d.parent = keep
                return d
            lens, data = vals
            n = lens.shape[0]
            offs = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
            if n:
                offs[1:] = torch.cumsum(lens.to(torch.int64), 0).to(torch.int32)
            if data.shape[0] == 0:
                data = torch.zeros(8, dtype=torch.uint8, device="cuda")
            keep.extend([offs, data])
            d = self.ctx.wrap_device(dtype, data.data_ptr(), n, bitmap, offsets=offs.data_ptr(),
                                     values_bytes=int(data.shape[0]) if n else 0)
            d.parent = keep
            return d
        m = None if valid is None else valid.numpy().astype(bool)
        if dtype == abi.DT_BOOL:
            return self.ctx.upload(vals.numpy().astype(bool), m)
        lens, data = vals
        raw = data.numpy().tobytes()
        cum = np.concatenate([[0], np.cumsum(lens.numpy().astype(np.int64))])
        strs = np.array([raw[cum[i]:cum[i + 1]].decode() for i in range(len(cum) - 1)], dtype=object)
        return self.ctx.upload(strs, m)

    def _sync(self):
        """Order the library's queue before torch / RCCL work: a host wait, unless the context
        runs on torch's current stream (set_stream), where stream order already does it."""
        if self.device == "cuda":
            if getattr(self.ctx, "stream_handle", None) == torch.cuda.current_stream().cuda_stream:
                return
            self.ctx.sync()

    def _sync_torch(self):
        """Order torch / RCCL work before the library's queue reads its results: a wait on
        torch's current stream, unless the context runs on it."""
        if self.device == "cuda" and getattr(self.ctx, "stream_handle", None) != torch.cuda.current_stream().cuda_stream:
            torch.cuda.current_stream().synchronize()

    # ---- shuffle -----------------------------------------------------------------
    def _exchange_columns(self, cols: Sequence[DeviceColumn], counts) -> Tuple[List[DeviceColumn], List[int]]:
        """All-to-all of partition-major columns: counts[r] leading rows go to rank r.
        One all_gather carries every rank's row counts, per-column has-validity flags and the
        per-destination byte counts of Utf8 columns; nullability is then agreed across ranks
        (a column is sent with validity bytes when ANY rank's shard has a bitmap, all-valid bytes
        from the shards without one) so every rank issues the same sequence of collectives.
        Then one all_to_all_single per payload, with no further host round trip."""
        w, me = self.world, self.rank
        counts = np.asarray(counts, np.int64)
        bounds = np.concatenate([[0], np.cumsum(counts)])
        tens = [self._to_tensors(t) for t in cols]
        flags = np.array([1 if t.c.validity else 0 for t in cols], np.int64)
        utf8 = [j for j, t in enumerate(cols) if t.dtype == abi.DT_UTF8]
        byte_counts = []
        for j in utf8:  # bytes per destination from the row lengths (device cumsum, gathered below)
            lens = tens[j][0].to(torch.int64)
            cum = torch.zeros(len(lens) + 1, dtype=torch.int64, device=lens.device)
            if len(lens):
                cum[1:] = torch.cumsum(lens, 0)
            b = torch.as_tensor(bounds, dtype=torch.int64, device=lens.device)
            byte_counts.append(cum[b[1:]] - cum[b[:-1]])
        self._sync()
        meta = [torch.as_tensor(counts, device=self.device), torch.as_tensor(flags, device=self.device)] + \
               [bc.to(self.device) for bc in byte_counts]
        meta_t = torch.cat(meta) if meta else torch.zeros(0, dtype=torch.int64, device=self.device)
        M = _allgather_meta_t(meta_t, w, self.group)
        sin, sout = [int(x) for x in M[me, :w]], [int(x) for x in M[:, me]]
        peak = _peak_remote(M[:, :w])
        nullable = M[:, w:w + len(cols)].max(axis=0) > 0 if len(cols) else np.zeros(0, bool)
        out = []
        for j, t in enumerate(cols):
            ts = tens[j]
            nvals = 2 if t.dtype == abi.DT_UTF8 else 1
            vals = []
            for q in range(nvals):
                if t.dtype == abi.DT_UTF8 and q == 1:
                    u = utf8.index(j)
                    off = w + len(cols) + w * u
                    S = M[:, off:off + w]
                    vals.append(_all_to_all(ts[1], [int(x) for x in S[me]], [int(x) for x in S[:, me]],
                                            _peak_remote(S), self.group))
                else:
                    vals.append(_all_to_all(ts[q], sin, sout, peak, self.group))
            valid = None
            if nullable[j]:
                vb = ts[nvals] if len(ts) > nvals else torch.ones(len(t), dtype=torch.uint8, device=self.device)
                valid = _all_to_all(vb, sin, sout, peak, self.group)
            out.append(self._from_tensors(t.dtype, vals[0] if nvals == 1 else vals, valid))
        self._sync_torch()
        return out, sout

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
        if self.world == 1:
            # one rank: the shuffle is the identity and every group's partial state is already its
            # only one (the local aggregate emits each group once), so the final merge is the identity
            return list(keys), list(partials), len(keys[0]) if keys else 0
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
        if g == 0:
            pk, pa_ = self._empty_partials(keys, inputs, aggs)
        return self._final(pk, pa_, aggs)

    def _empty_partials(self, keys, inputs, aggs):
        """Zero-row partial states with the types every other rank's partials have (SUM of a
        float -> Float64, of an integer -> Int64; COUNT -> Int64; MIN / MAX keep the input type),
        so all ranks exchange identically typed columns."""
        def out_dt(f, c):
            t = inputs[c].dtype
            if f == AF.Count:
                return abi.DT_INT64
            if f == AF.Sum:
                return abi.DT_FLOAT64 if t in (abi.DT_FLOAT64, abi.DT_FLOAT32) else abi.DT_INT64
            return t
        return ([self.ctx.empty(k.dtype, 0) for k in keys], [self.ctx.empty(out_dt(f, c), 0) for f, c in aggs])

    def allgather_columns(self, cols: Sequence[DeviceColumn]) -> List[DeviceColumn]:
        """Every rank's shard of `cols`, concatenated in rank order, on every rank: the
        broadcast side of a broadcast join.  Fixed-width columns move with one padded
        all_gather each (ring, bandwidth-optimal on xGMI); validity travels as bytes when any
        shard has a bitmap.  Utf8 / Boolean shards go through the all-to-all exchange."""
        n = len(cols[0]) if cols else 0
        flags = [1 if c.c.validity else 0 for c in cols]
        M = _allgather_meta_t(torch.tensor([n] + flags, dtype=torch.int64, device=self.device), self.world,
                              self.group)
        rows = [int(x) for x in M[:, 0]]
        if any(c.dtype in (abi.DT_UTF8, abi.DT_BOOL) for c in cols):
            rep = [self.ctx.concat([c] * self.world) if self.world > 1 else c for c in cols]
            out, _ = self._exchange_columns(rep, [n] * self.world)
            return out
        nullable = M[:, 1:].max(axis=0) > 0 if cols else []
        mx = max(rows) if rows else 0
        out = []
        tens = [self._to_tensors(c) for c in cols]
        self._sync()  # the views / validity bytes are produced on the library's queue
        for j, c in enumerate(cols):
            ts = tens[j]
            vals = self._gather_padded(ts[0], n, mx, rows)
            valid = None
            if nullable[j]:
                vb = ts[1] if len(ts) > 1 else torch.ones(n, dtype=torch.uint8, device=self.device)
                valid = self._gather_padded(vb, n, mx, rows)
            out.append(self._from_tensors(c.dtype, vals, valid))
        self._sync_torch()
        return out

    def _gather_padded(self, t: torch.Tensor, n: int, mx: int, rows: Sequence[int]) -> torch.Tensor:
        if self.world == 1:
            return t
        if n < mx:
            pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
            pad[:n] = t
            t = pad
        buf = torch.empty(self.world * mx, dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(buf, t.contiguous(), group=self.group)
        if all(r == mx for r in rows):
            return buf
        return torch.cat([buf[q * mx:q * mx + rows[q]] for q in range(self.world)])

    def join_filter_aggregate_broadcast(self, probe_cols, probe_key_idx, predicate, build_key, build_group_keys,
                                        aggs, build_sharded: bool = False):
        """Broadcast join (the BASELINE metric path): `probe_cols` = this rank's fact shard.
        With build_sharded, `build_*` are this rank's shard of the dimension.  Two forms:
          * table (default when the shape allows it, _broadcast_table): every rank inserts its
            dimension shard into a DIRECT u16 table over the job-wide key range and the ranks sum
            the tables (one RCCL all-reduce of range x 2 B) -- each rank builds 1/N of the table
            and receives a table, not the dimension;
          * all-gather: the dimension shards are all-gathered (over RCCL under "nccl") and every
            rank builds the whole table.
        Otherwise `build_*` are replicated already.  Then the fused local pipeline, and the partial
        per-group states are merged on the owning rank (partial/final aggregate,
        distributed/planner.rs:200-249): one dense all-reduce for a bounded integer group key,
        else a shuffle of the partial states."""
        for f, _ in aggs:
            if f not in FINAL_OF:
                raise NotImplementedError("distributed AVG needs SUM+COUNT partials; compose it from them")
        # which aggregate inputs may hold NULLs, agreed across ranks (each rank sees only its fact
        # shard's bitmaps; the final stage's choice of collectives must be the same on every rank)
        probe_flags = [1 if probe_cols[c].c.validity else 0 for _, c in aggs]
        probe_nullable = None
        self.last_build = "replicated"
        if build_sharded and not os.environ.get("QEH_NO_ITEMS_BCAST"):
            out = self._broadcast_items(probe_cols, probe_key_idx, predicate, build_key, build_group_keys, aggs)
            if out is not None:
                self.last_build = "items"
                return out
        if build_sharded:
            st = self._build_stats(build_key, build_group_keys, probe_flags,
                                   probe=(probe_cols, probe_key_idx, predicate, aggs))
            full = None
            if st is not None:
                probe_nullable = st["agreed"]
                if not os.environ.get("QEH_NO_TABLE_BCAST"):
                    out = self._broadcast_table(st, probe_cols, probe_key_idx, predicate, build_key, build_group_keys,
                                                aggs, probe_nullable)
                    if out is not None:
                        self.last_build = "table"
                        return out
                full = self._allgather_beside_phase_a(st, probe_cols, probe_key_idx, predicate, aggs)
            if full is None:
                full = self.allgather_columns([build_key] + list(build_group_keys))
            self.last_build = "allgather"
            build_key, build_group_keys = full[0], full[1:]
        if probe_nullable is None:
            probe_nullable = self._agree_max(probe_flags)
        pk, pa_, g = self.ctx.join_filter_aggregate(probe_cols, probe_key_idx, predicate, build_key,
                                                    build_group_keys, aggs)
        if g == 0:
            pk, pa_ = self._empty_partials(build_group_keys, probe_cols, aggs)
        gcol = build_group_keys[0] if len(build_group_keys) == 1 else None
        dense = None
        if gcol is not None and gcol.dtype in (abi.DT_INT64, abi.DT_INT32) and not gcol.c.validity and len(gcol):
            self._sync()
            gk = self._to_tensors(gcol)[0]
            lo, hi = (int(q) for q in torch.stack([gk.min().to(torch.int64), gk.max().to(torch.int64)]).tolist())
            dense = self._final_dense(lo, hi, probe_nullable, pk, pa_, aggs)
        self.last_final = "dense" if dense is not None else "shuffle"
        if dense is not None:
            return dense
        return self._final(pk, pa_, aggs)

    def _agree_max(self, flags: Sequence[int]) -> np.ndarray:
        """Element-wise max of a small int vector over the ranks (one all_reduce; none at world 1)."""
        f = np.asarray(flags, np.int64)
        if self.world == 1 or len(f) == 0:
            return f
        t = torch.as_tensor(f, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.cpu().numpy()

    def _build_stats(self, build_key, build_group_keys, probe_flags: Sequence[int], probe=None):
        """One small all_gather of every dimension shard's [rows, key min / max, group key min / max,
        has-bitmap] and the fact shard's aggregate-input bitmap flags: the job-wide ranges both
        device broadcast forms plan from.  None when the shape is outside them (decided from
        schema-level facts, identical on every rank).  Every later branch depends only on gathered
        values, so all ranks take the same one."""
        cols = [build_key] + list(build_group_keys)
        if (self.device != "cuda" or len(build_group_keys) != 1 or build_key.dtype != abi.DT_INT64
                or build_group_keys[0].dtype not in (abi.DT_INT64, abi.DT_INT32)):
            return None
        n = len(build_key)
        flags = [1 if any(c.c.validity for c in cols) else 0] + list(probe_flags)
        # [rows, key min / max, group key min / max, flags] written on the device by one library call
        # (min / max kernels, no host wait), gathered over the ranks, read back once
        row = torch.empty(5 + len(flags), dtype=torch.int64, device="cuda")
        self._sync_torch()
        self.ctx.broadcast_stats(build_key, build_group_keys[0], flags, row.data_ptr())
        self._sync()
        if self.world > 1:
            out = torch.empty(self.world * row.numel(), dtype=torch.int64, device="cuda")
            dist.all_gather_into_tensor(out, row, group=self.group)
            row = out
        # the rows' copy to the host is queued ahead of phase A: a copy queued behind it would wait for
        # phase A's workgroups to leave the CUs (the copy engine's blit kernel needs a CU), so the host
        # would sit idle for the whole of phase A before it could queue the build and phase B
        # (one pinned buffer per row size, reused every step: M below is copied out of it)
        pinned = getattr(self, "_stats_pinned", None)
        if pinned is None or pinned.numel() != row.numel():
            pinned = self._stats_pinned = torch.empty(row.numel(), dtype=torch.int64, pin_memory=True)
        row_host = pinned
        row_host.copy_(row, non_blocking=True)
        copied = torch.cuda.Event()
        copied.record()
        prelaunched = False
        # the table form's u16 table of the previous step, zeroed here -- ahead of phase A on the queue --
        # for this step to reuse when its key range is the same: zeroed behind phase A it waited for
        # phase A's CUs (0.67 ms for 20 MB), and the table insert, its count and phase B's set-up with it
        table_zeroed = False
        tc = getattr(self, "_table_cache", None)
        if tc is not None and probe is not None and not os.environ.get("QEH_NO_TABLE_CACHE"):
            tc.zero_()
            table_zeroed = True
        if probe is not None and not os.environ.get("QEH_HOST_PLAN"):
            # phase A planned on the device from the gathered rows: it starts while the host reads them
            self._sync_torch()
            self.ctx.join_filter_aggregate_prelaunch_stats(*probe, row.data_ptr(), self.world, 5 + len(flags))
            prelaunched = True
        copied.synchronize()
        M = row_host.numpy().reshape(self.world, -1).copy()
        rows = [int(x) for x in M[:, 0]]
        total = sum(rows)
        out = {"M": M, "rows": rows, "total": total, "n": n, "cols": cols, "bitmap": bool(M[:, 5].max() > 0),
               "agreed": M[:, 6:].max(axis=0), "gdtype": build_group_keys[0].dtype, "prelaunched": prelaunched,
               "stats_dev": row, "table_zeroed": table_zeroed}
        if total:
            live = M[M[:, 0] > 0]
            out["krange"] = [int(live[:, 1].min()), int(live[:, 2].max()), total]
            out["grange"] = [int(live[:, 3].min()), int(live[:, 4].max()), total]
        return out

    ITEMS_SLICES = 160       # slices an item buffer holds (the library's kSliceMaxF)
    ITEMS_STATE_WORDS = 3584  # group slots x value slots the fused pipeline's phase B keeps in LDS
    ITEMS_MIN_TABLE_BYTES = 6 << 20  # smaller key ranges take the single fused pass (the library's rule)

    def _broadcast_items(self, probe_cols, probe_key_idx, predicate, build_key, build_group_keys, aggs):
        """The items form of the broadcast join (include/qeh.h qeh_fused_items_*; the fused pipeline of
        N = 1 with its build side sharded): every rank groups ITS dimension shard by 2^16-key slice into
        4-B items, one all-gather moves the items (4 B per dimension row, one region per rank and
        slice), and phase B builds each slice's LDS entries from every rank's region -- no 2-B-per-key
        table, no table all-reduce and no table reads in phase B, and phase A is the fused pipeline's
        kernel.  Phase A is queued (planned on the device from the gathered stats rows) before the host
        reads the rows.  Whether the form runs is decided from gathered values only -- each rank's
        shape check travels in its stats row -- so every rank issues the same collectives; a plan the
        device declines, a region overflow or a key on two ranks come back in the status lane of the
        lanes' all-reduce, and every rank then returns None (the caller takes the table / all-gather
        form).  Returns the dense final ([keys], aggs, groups) or None."""
        if (self.device != "cuda" or len(build_group_keys) != 1 or build_key.dtype != abi.DT_INT64
                or build_group_keys[0].dtype not in (abi.DT_INT64, abi.DT_INT32)
                or any(f not in (AF.Count, AF.Sum) for f, _ in aggs)):
            return None
        gkc = build_group_keys[0]
        local_ok = 1 if self.ctx.fused_items_check(probe_cols, probe_key_idx, predicate, aggs) else 0
        bitmap = 1 if (build_key.c.validity or gkc.c.validity) else 0
        row_len = 7  # [rows, key min, max, group key min, max, has-bitmap, shape ok]
        row = torch.empty(row_len, dtype=torch.int64, device="cuda")
        self._sync_torch()
        self.ctx.broadcast_stats(build_key, gkc, [bitmap, local_ok], row.data_ptr())
        self._sync()
        if self.world > 1:
            out = torch.empty(self.world * row_len, dtype=torch.int64, device="cuda")
            dist.all_gather_into_tensor(out, row, group=self.group)
            row = out
        pinned = getattr(self, "_items_pinned", None)
        if pinned is None or pinned.numel() != row.numel():
            pinned = self._items_pinned = torch.empty(row.numel(), dtype=torch.int64, pin_memory=True)
        pinned.copy_(row, non_blocking=True)  # queued ahead of phase A (a copy behind it would wait for it)
        copied = torch.cuda.Event()
        copied.record()
        handle = None
        if local_ok:  # phase A planned on the device from the gathered rows, while the host reads them
            self._sync_torch()
            try:
                handle = self.ctx.fused_items_begin(probe_cols, probe_key_idx, predicate, aggs, row.data_ptr(),
                                                    self.world, row_len)
            except abi.QehError:
                handle = None  # (an OOM on this rank: it still joins every collective below, see `failed`)
        copied.synchronize()
        M = pinned.numpy().reshape(self.world, row_len).copy()
        live = M[M[:, 0] > 0]
        total = int(M[:, 0].sum())
        n_sum = sum(1 for f, _ in aggs if f == AF.Sum)
        ok = bool(M[:, 6].min() == 1 and M[:, 5].max() == 0 and total > 0)
        if ok:
            kmin, kmax = int(live[:, 1].min()), int(live[:, 2].max())
            gmin, gmax = int(live[:, 3].min()), int(live[:, 4].max())
            R, G = kmax - kmin + 1, gmax - gmin + 1
            F = (R + (1 << 16) - 1) >> 16
            ok = (1 <= F <= self.ITEMS_SLICES and G * (1 + n_sum) <= self.ITEMS_STATE_WORDS
                  and 2 * R >= self.ITEMS_MIN_TABLE_BYTES)
        if not ok:
            if handle is not None:
                self.ctx.fused_items_abort(handle)
            return None
        # this rank's build rows grouped by slice (spans of ~8 K rows, one run per slice each), all-gathered:
        # 4 B per dimension row (+ the runs' padding to 16 B); every rank uses the same shape
        nb, span = self.ctx.fused_items_shape(int(M[:, 0].max()), self.world)
        OW = 2 * (self.ITEMS_SLICES + 1)
        # A library error on this rank only (begin / build / finish: e.g. out of memory) must not leave the
        # other ranks waiting in a collective: this rank sends empty items and a set status lane, so every
        # rank's lanes come back flagged and every rank returns None together.
        failed = handle is None
        items = torch.zeros(nb * span, dtype=torch.int32, device="cuda")
        offs = torch.zeros(nb * OW, dtype=torch.int32, device="cuda")
        self._sync_torch()
        if not failed:
            try:
                self.ctx.fused_items_build(handle, build_key, gkc, nb, span, items.data_ptr(), offs.data_ptr())
            except abi.QehError:
                failed = True
                items.zero_(), offs.zero_()
        self._sync()
        if self.world > 1:
            gi = torch.empty(self.world * nb * span, dtype=torch.int32, device="cuda")
            go = torch.empty(self.world * nb * OW, dtype=torch.int32, device="cuda")
            dist.all_gather_into_tensor(gi, items, group=self.group)
            dist.all_gather_into_tensor(go, offs, group=self.group)
            items, offs = gi, go
        nl = (1 + len(aggs)) * G + 1  # + the status lane
        lanes = torch.empty(nl, dtype=torch.float64, device="cuda")
        self._sync_torch()
        if not failed:
            try:
                self.ctx.fused_items_finish(handle, items.data_ptr(), span, offs.data_ptr(), self.world * nb, G,
                                            lanes.data_ptr())
            except abi.QehError:
                failed = True
            handle = None  # (finish frees it, also when it fails)
        if failed:
            if handle is not None:
                self.ctx.fused_items_abort(handle)
            lanes.zero_()
            lanes[nl - 1] = 1.0
        self._sync()
        if self.world > 1:
            dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
        self._sync_torch()
        got, ov, g, bad = self.ctx.dense_states_take_status(
            lanes.data_ptr(), len(aggs), gmin, G, self.world, self.rank, gkc.dtype,
            [abi.DT_INT64 if f == AF.Count else abi.DT_FLOAT64 for f, _ in aggs])
        if bad != 0.0:  # declined, overflowed or a repeated key on some rank (the same lane on every rank)
            return None
        self.last_final = "dense"
        return [got], ov, g

    def _broadcast_table(self, st, probe_cols, probe_key_idx, predicate, build_key, build_group_keys, aggs,
                         probe_nullable):
        """The table form of the broadcast join: phase A is launched from the job-wide key range
        (qeh_join_filter_aggregate_prelaunch), this rank's dimension shard goes into a zeroed DIRECT
        u16 table over that range (entry = group slot + 1, qeh_direct_group_table_insert), one RCCL
        all-reduce sums the ranks' tables (unique keys: one writer per entry), and the fused probe
        runs against the sum (qeh_join_filter_aggregate_table).  A repeated key shows as fewer
        non-empty entries than build rows -- the same count on every rank, since every rank holds
        the same summed table -- and returns None (the caller all-gathers instead).  None too when
        the shape does not fit: NULLs, a key range above 4 x rows, more than 4096 groups."""
        total = st["total"]
        if st["bitmap"] or not total:
            return None
        kmin, kmax, _ = st["krange"]
        gmin, gmax, _ = st["grange"]
        R, G = kmax - kmin + 1, gmax - gmin + 1
        # QEH_TABLE_MAX_SPARSITY: key range per build row allowed (bench.py's one-rank rehearsal holds 1/N
        # of the rows over the whole range)
        sparsity = float(os.environ.get("QEH_TABLE_MAX_SPARSITY", "4"))
        if R > sparsity * total + 1024 or R >= (1 << 31) or G > 4096 or self.world * (G + 1) >= (1 << 16):
            # declined: drop the cached table so later steps stop zeroing it (and its memory is freed)
            self._table_cache = None
            return None
        if not st["prelaunched"]:
            self.ctx.join_filter_aggregate_prelaunch(probe_cols, probe_key_idx, predicate, aggs, st["krange"],
                                                     st["grange"])
        tc = getattr(self, "_table_cache", None)
        if st.get("table_zeroed") and tc is not None and tc.numel() == (R + 1) // 2:
            table = tc  # zeroed ahead of phase A in _build_stats
        else:
            table = torch.zeros((R + 1) // 2, dtype=torch.int32, device="cuda")  # R u16 entries (+1 pad)
            # cached for the next step (zeroed ahead of its phase A) up to TABLE_CACHE_MAX_BYTES
            cache = not os.environ.get("QEH_NO_TABLE_CACHE") and R * 2 <= self.TABLE_CACHE_MAX_BYTES
            self._table_cache = table if cache else None
        self._sync_torch()  # zeroed before the library writes
        lanes_ok = (G <= self.DENSE_MAX_KEYS and not os.environ.get("QEH_NO_TABLE_LANES")
                    and all((f == AF.Count or (f == AF.Sum and probe_cols[c].dtype == abi.DT_FLOAT64 and not probe_nullable[j]))
                            for j, (f, c) in enumerate(aggs)))
        no_wait = lanes_ok and not os.environ.get("QEH_SYNC_TABLE_CHECK")
        if st["n"]:
            # the ranges are the job's own min / max, so every row is in range; the no-wait form skips
            # the range check's host read (a row it skipped would show in the non-empty count below)
            self.ctx.direct_group_table_insert(build_key, build_group_keys[0], kmin, R, gmin, table.data_ptr(),
                                               check=not no_wait)
        self._sync()
        if self.world > 1:
            dist.all_reduce(table, op=dist.ReduceOp.SUM, group=self.group)  # u16 pairs: no carries (checked above)
        self._sync_torch()
        if no_wait:
            # no host wait until the final states: the duplicate check (non-empty entries of the summed
            # table, the same on every rank) and the operator's status words (error bits, a slice region
            # overflow on this rank) stay on the device; the status rides the lanes' all-reduce as one
            # extra lane, so every rank sees every rank's flags and all take the same branch below
            status = torch.empty(4, dtype=torch.int32, device="cuda")
            # (1 + aggregates) lanes per group slot + the status lane the library writes last, then one
            # word outside the all-reduced lanes for the table's non-empty count (int64 bits): the two
            # checks come back in one 16-B read, with no torch kernels between the step's end and it
            nl = (1 + len(aggs)) * G + 1
            lanes_buf = torch.empty(nl + 1, dtype=torch.float64, device="cuda")
            lanes = lanes_buf[:nl]
            self._sync_torch()
            # entries above G (a build key on two ranks sums to world x its entry) are cleared before
            # the probe reads the table: the kernels index group states with entry - 1 unchecked
            self.ctx.u16_table_check_dev(table.data_ptr(), R, G, lanes_buf[nl:].data_ptr())
            self.ctx.join_filter_aggregate_table_lanes_async(probe_cols, probe_key_idx, predicate, table.data_ptr(), kmin,
                                                             R, G, aggs, lanes.data_ptr(), status.data_ptr())
            self._sync()
            if self.world > 1:
                dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
            self._sync_torch()
            ok, ov, g = self.ctx.dense_states_take(lanes.data_ptr(), len(aggs), gmin, G, self.world, self.rank,
                                                   st["gdtype"],
                                                   [abi.DT_INT64 if f == AF.Count else abi.DT_FLOAT64 for f, _ in aggs])
            tail = lanes_buf[nl - 1:].cpu().numpy()  # [status lane, non-empty count]
            nz, bad = int(tail[1:].view(np.int64)[0]), float(tail[0]) != 0.0
            self.last_table_redo = False
            if nz != total:
                return None  # a build key repeats: the general path handles multi-match joins
            if bad:  # some rank's operator overflowed a slice region (or failed): redo it with the checks inline
                self.last_table_redo = True
                lanes = torch.empty((1 + len(aggs)) * G, dtype=torch.float64, device="cuda")
                self._sync_torch()
                self.ctx.join_filter_aggregate_table_lanes(probe_cols, probe_key_idx, predicate, table.data_ptr(),
                                                           kmin, R, G, aggs, lanes.data_ptr())
                self._sync()
                if self.world > 1:
                    dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
                self._sync_torch()
                ok, ov, g = self.ctx.dense_states_take(lanes.data_ptr(), len(aggs), gmin, G, self.world, self.rank,
                                                       st["gdtype"],
                                                       [abi.DT_INT64 if f == AF.Count else abi.DT_FLOAT64 for f, _ in aggs])
            self.last_final = "dense"
            return [ok], ov, g
        if self.ctx.u16_count_nonzero(table.data_ptr(), R) != total:
            return None  # a build key repeats: the general path handles multi-match joins
        if lanes_ok:
            # the fused operator writes the dense final stage's lanes itself (row counts, COUNT / float
            # SUM partials per group slot): no compaction, output columns or re-scatter of the partials
            lanes = torch.empty((1 + len(aggs)) * G, dtype=torch.float64, device="cuda")
            self._sync_torch()
            self.ctx.join_filter_aggregate_table_lanes(probe_cols, probe_key_idx, predicate, table.data_ptr(), kmin, R,
                                                       G, aggs, lanes.data_ptr())
            self._sync()
            if self.world > 1:
                dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
            self._sync_torch()
            ok, ov, g = self.ctx.dense_states_take(lanes.data_ptr(), len(aggs), gmin, G, self.world, self.rank,
                                                   st["gdtype"],
                                                   [abi.DT_INT64 if f == AF.Count else abi.DT_FLOAT64 for f, _ in aggs])
            self.last_final = "dense"
            return [ok], ov, g
        pk, pa_, g = self.ctx.join_filter_aggregate_table(probe_cols, probe_key_idx, predicate, table.data_ptr(), kmin,
                                                          R, gmin, G, st["gdtype"], aggs)
        if g == 0:
            pk, pa_ = self._empty_partials(build_group_keys, probe_cols, aggs)
        dense = self._final_dense(gmin, gmax, probe_nullable, pk, pa_, aggs)
        self.last_final = "dense" if dense is not None else "shuffle"
        return dense if dense is not None else self._final(pk, pa_, aggs)

    def _allgather_beside_phase_a(self, st, probe_cols, probe_key_idx, predicate, aggs):
        """The dimension all-gather overlapped with phase A of the fused operator: with the
        job-wide ranges of _build_stats, the padded column all-gathers are issued asynchronously,
        phase A is launched from the ranges (qeh_join_filter_aggregate_prelaunch) while they run,
        and only then does the queue wait for them.  None when the shape does not allow it (the
        caller all-gathers first)."""
        if self.world == 1 or st["bitmap"] or not st["total"]:
            return None
        rows, n = st["rows"], st["n"]
        ts = [self._to_tensors(c)[0] for c in st["cols"]]
        mx = max(rows)
        bufs, works = [], []
        for t in ts:
            if n < mx:
                pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
                pad[:n] = t
                t = pad
            buf = torch.empty(self.world * mx, dtype=t.dtype, device=t.device)
            works.append(dist.all_gather_into_tensor(buf, t.contiguous(), group=self.group, async_op=True))
            bufs.append(buf)
        if not st["prelaunched"]:
            self.ctx.join_filter_aggregate_prelaunch(probe_cols, probe_key_idx, predicate, aggs, st["krange"],
                                                     st["grange"])
        for w in works:
            w.wait()
        out = []
        dts = [abi.DT_INT64, st["gdtype"]]
        for dt, buf in zip(dts, bufs):
            if any(r != mx for r in rows):
                buf = torch.cat([buf[q * mx:q * mx + rows[q]] for q in range(self.world)])
            out.append(self._from_tensors(dt, buf, None))
        self._sync_torch()
        return out

    DENSE_MAX_KEYS = 1 << 20
    TABLE_CACHE_MAX_BYTES = 256 << 20  # the table form's u16 table kept for the next step up to this size

    def _final_dense(self, lo: int, hi: int, probe_nullable, pk, pa_, aggs):
        """Final aggregate of a broadcast join by all-reduce instead of a shuffle, when the single
        group key is a non-null integer of the (whole) dimension whose job-wide range [lo, hi] spans
        at most DENSE_MAX_KEYS values: every rank scatters its partial states into dense arrays
        indexed by key - lo, one all_reduce per reduction op (SUM for float SUMs, COUNTs and a
        presence flag; SUM / MIN / MAX over int64 for integer aggregates) merges them, and each
        rank keeps the groups with (key - lo) % world == rank.  Same result as _final (partial
        states merged per group, each group on one rank) with one or two collectives instead of a
        partition kernel, a metadata all_gather, an all-to-all per column and a hash aggregate.
        None when not applicable (the caller shuffles).  probe_nullable[j]: aggregate j's input has
        a bitmap on some rank (agreed across ranks); lo / hi are the same on every rank, so every
        rank decides the same way."""
        if len(pk) != 1:
            return None
        kinds = []
        for j, ((f, c), col) in enumerate(zip(aggs, pa_)):
            # partial states can be NULL only where an input value can (all-NULL group)
            if f not in FINAL_OF or (f != AF.Count and probe_nullable[j]):
                return None
            if f in (AF.Min, AF.Max) and col.dtype not in (abi.DT_INT64, abi.DT_INT32):
                return None  # float MIN / MAX keep the shuffle (total-order semantics)
            kinds.append(f)
        R = hi - lo + 1
        if R > self.DENSE_MAX_KEYS or R <= 0:
            return None
        if (pk[0].dtype in (abi.DT_INT64, abi.DT_INT32) and not pk[0].c.validity
                and all(f == AF.Count or (f == AF.Sum and c.dtype == abi.DT_FLOAT64) for f, c in zip(kinds, pa_))):
            # every lane is a COUNT or a float SUM: exact in f64, so one lane buffer, one library scatter,
            # one all-reduce and one library take (the torch path below issues ~15 small kernels)
            lanes = torch.zeros((1 + len(pa_)) * R, dtype=torch.float64, device="cuda")
            self._sync_torch()
            # (SUM partials carry a bitmap but no NULL: every input is non-null, checked above)
            self.ctx.dense_states_f64(pk[0], [_without_bitmap(self.ctx, c) for c in pa_], lo, R, lanes.data_ptr())
            self._sync()
            if self.world > 1:
                dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
            self._sync_torch()
            ok, ov, g = self.ctx.dense_states_take(lanes.data_ptr(), len(pa_), lo, R, self.world, self.rank, pk[0].dtype,
                                                   [c.dtype for c in pa_])
            return [ok], ov, g
        self._sync()
        gk = self._to_tensors(pk[0])[0]
        dev = gk.device
        idx = self._to_tensors(pk[0])[0].to(torch.int64) - lo
        vals = [self._to_tensors(c)[0] for c in pa_]
        # f64 lanes: presence, float SUMs, COUNTs (exact below 2^53); i64 lanes: integer SUM / MIN / MAX
        fl = [None] + [j for j, f in enumerate(kinds) if f == AF.Count or (f == AF.Sum and vals[j].is_floating_point())]
        il = {op: [j for j, f in enumerate(kinds) if f == op and j not in fl] for op in (AF.Sum, AF.Min, AF.Max)}
        fbuf = torch.zeros((len(fl), R), dtype=torch.float64, device=dev)
        fbuf[0].index_fill_(0, idx, 1.0)
        for q, j in enumerate(fl[1:], 1):
            fbuf[q].index_copy_(0, idx, vals[j].to(torch.float64))
        dist.all_reduce(fbuf, op=dist.ReduceOp.SUM, group=self.group)
        ibufs = {}
        for op, js in il.items():
            if not js:
                continue
            init = {AF.Sum: 0, AF.Min: np.iinfo(np.int64).max, AF.Max: np.iinfo(np.int64).min}[op]
            b = torch.full((len(js), R), init, dtype=torch.int64, device=dev)
            for q, j in enumerate(js):
                b[q].index_copy_(0, idx, vals[j].to(torch.int64))
            rop = {AF.Sum: dist.ReduceOp.SUM, AF.Min: dist.ReduceOp.MIN, AF.Max: dist.ReduceOp.MAX}[op]
            dist.all_reduce(b, op=rop, group=self.group)
            ibufs[op] = (js, b)
        keys = torch.arange(R, device=dev)
        own = (fbuf[0] > 0) & (keys % self.world == self.rank)
        sel = torch.nonzero(own).flatten()
        out_keys = [self._from_tensors(pk[0].dtype, (sel + lo).to(TORCH_OF[pk[0].dtype]).contiguous(), None)]
        out_aggs = [None] * len(kinds)
        for q, j in enumerate(fl[1:], 1):
            out_aggs[j] = fbuf[q][sel]
        for js, b in ibufs.values():
            for q, j in enumerate(js):
                out_aggs[j] = b[q][sel]
        cols = [self._from_tensors(c.dtype, v.to(TORCH_OF[c.dtype]).contiguous(), None) for c, v in zip(pa_, out_aggs)]
        self._sync_torch()
        return out_keys, cols, int(sel.shape[0])

    def join_filter_aggregate_shuffle(self, probe_cols, probe_key_idx, predicate, build_key, build_group_keys,
                                      aggs):
        """Hash-partitioned join + aggregate (BASELINE config 4; the reference's shuffle-join and
        partial/final aggregate stage shapes, distributed/planner.rs:200-249, with hash
        partitioning by key, partition.rs:151-212).  Both inputs are this rank's shards:
          1. the probe side is filtered locally, keeping only the join key and the aggregate
             inputs (the predicate reads probe columns only);
          2. both sides are hash-partitioned by the join key on the device and exchanged with
             one all-to-all per column, so every key's probe and build rows meet on one rank;
          3. the local fused join + aggregate runs on what arrived, and the partial per-group
             states are shuffled by group key and merged on the owning rank."""
        for f, _ in aggs:
            if f not in FINAL_OF:
                raise NotImplementedError("distributed AVG needs SUM+COUNT partials; compose it from them")
        if self.world == 1:
            # one partition: both hash exchanges and the final merge are the identity, so the plan
            # is the local fused operator on this rank's rows
            pk, pa_, g = self.ctx.join_filter_aggregate(probe_cols, probe_key_idx, predicate, build_key,
                                                        build_group_keys, aggs)
            if g == 0:
                pk, pa_ = self._empty_partials(build_group_keys, probe_cols, aggs)
            return self._final(pk, pa_, aggs)
        if self.device == "cuda" and len(build_group_keys) == 1 and not os.environ.get("QEH_NO_ITEMS_SHUFFLE"):
            out = self._shuffle_items(probe_cols, probe_key_idx, predicate, build_key, build_group_keys, aggs)
            if out is not None:
                self.last_shuffle = "items"
                return out
        self.last_shuffle = "two_pass"
        need = sorted({probe_key_idx} | {c for _, c in aggs})
        remap = {c: i for i, c in enumerate(need)}
        pcounts = None
        if predicate is not None and len(need) <= 4:
            # filter fused into the exchange's partition pass (one read of the probe columns)
            try:
                pcounts, pmoved = self.ctx.filter_partition_hash_move(probe_cols, predicate, probe_key_idx,
                                                                      self.world, need)
            except abi.QehError as e:
                if e.status != abi.QEH_E_UNSUPPORTED:
                    raise
        if pcounts is None:
            if predicate is not None:
                cols, _ = self.ctx.filter(probe_cols, predicate, out_idx=need)
            else:
                cols = [probe_cols[i] for i in need]
            pk_col = cols[remap[probe_key_idx]]
            pcounts, pmoved = self.ctx.partition_hash_move([pk_col], self.world, cols)
        bcols = [build_key] + list(build_group_keys)
        bcounts, bmoved = self.ctx.partition_hash_move([build_key], self.world, bcols)
        precv, _ = self._exchange_columns(pmoved, pcounts)
        brecv, _ = self._exchange_columns(bmoved, bcounts)
        local_aggs = [(f, remap[c]) for f, c in aggs]
        pk, pa_, g = self.ctx.join_filter_aggregate(precv, remap[probe_key_idx], None, brecv[0], brecv[1:],
                                                    local_aggs)
        if g == 0:
            pk, pa_ = self._empty_partials(build_group_keys, probe_cols, aggs)
        return self._final(pk, pa_, aggs)

    def _shuffle_items(self, probe_cols, probe_key_idx, predicate, build_key, build_group_keys, aggs):
        """The items form of the shuffle join (include/qeh.h qeh_shuffle_items_*): every rank runs the fused
        pipeline's phase A over its fact shard with the regions laid out per destination rank -- the
        partition function is ((k - kmin) >> 16) % world, a modulo hash of the join key's 2^16-key slice --
        packs each destination's regions into one block of 10-B items (16-bit key offset, value), and one
        all-to-all per payload moves the blocks; each rank's phase B aggregates what it received against
        its slices' dimension rows (all-gathered as 4-B items, as the broadcast items form does) into the
        dense final stage's lanes.  The receiving rank needs no pipeline of its own over (key, value)
        rows, and the wire carries 10 B per selected fact row instead of 16.  Decided from gathered
        values only; a declined plan or an overflow on any rank (gathered with the block totals), or a
        key on two ranks (the status lane), returns None on every rank (the two-pass form follows)."""
        if (len(build_group_keys) != 1 or build_key.dtype != abi.DT_INT64
                or build_group_keys[0].dtype not in (abi.DT_INT64, abi.DT_INT32)
                or any(f not in (AF.Count, AF.Sum) for f, _ in aggs)):
            return None
        gkc = build_group_keys[0]
        W, me = self.world, self.rank
        local_ok = 1 if self.ctx.fused_items_check(probe_cols, probe_key_idx, predicate, aggs) else 0
        bitmap = 1 if (build_key.c.validity or gkc.c.validity) else 0
        row_len = 7  # [rows, key min, max, group key min, max, has-bitmap, shape ok]
        row = torch.empty(row_len, dtype=torch.int64, device="cuda")
        self._sync_torch()
        self.ctx.broadcast_stats(build_key, gkc, [bitmap, local_ok], row.data_ptr())
        self._sync()
        out = torch.empty(W * row_len, dtype=torch.int64, device="cuda")
        dist.all_gather_into_tensor(out, row, group=self.group)
        row = out
        pinned = getattr(self, "_shuffle_pinned", None)
        if pinned is None or pinned.numel() != row.numel():
            pinned = self._shuffle_pinned = torch.empty(row.numel(), dtype=torch.int64, pin_memory=True)
        pinned.copy_(row, non_blocking=True)  # queued ahead of phase A
        copied = torch.cuda.Event()
        copied.record()
        handle = None
        if local_ok:
            self._sync_torch()
            try:
                handle = self.ctx.shuffle_items_begin(probe_cols, probe_key_idx, predicate, aggs, row.data_ptr(), W,
                                                      me, row_len)
            except abi.QehError:
                handle = None  # (this rank still joins the block-totals all-gather below, with ok = 0)
        copied.synchronize()
        M = pinned.numpy().reshape(W, row_len).copy()
        live = M[M[:, 0] > 0]
        n_sum = sum(1 for f, _ in aggs if f == AF.Sum)
        ok = bool(M[:, 6].min() == 1 and M[:, 5].max() == 0 and int(M[:, 0].sum()) > 0)
        if ok:
            kmin, kmax = int(live[:, 1].min()), int(live[:, 2].max())
            gmin, gmax = int(live[:, 3].min()), int(live[:, 4].max())
            R, G = kmax - kmin + 1, gmax - gmin + 1
            F = (R + (1 << 16) - 1) >> 16
            ok = (1 <= F <= self.ITEMS_SLICES and G * (1 + n_sum) <= self.ITEMS_STATE_WORDS
                  and 2 * R >= self.ITEMS_MIN_TABLE_BYTES)
        if not ok:
            if handle is not None:
                self.ctx.fused_items_abort(handle)
            return None
        # this rank's dimension rows grouped by slice, all-gathered (every rank builds only its own slices)
        nb, span = self.ctx.fused_items_shape(int(M[:, 0].max()), W)
        OW = 2 * (self.ITEMS_SLICES + 1)
        items = torch.empty(nb * span, dtype=torch.int32, device="cuda")
        offs = torch.empty(nb * OW, dtype=torch.int32, device="cuda")
        self._sync_torch()
        # phase A's regions packed per destination (waits for phase A); the flag and the block totals of
        # every rank in one all-gather -- a library error on this rank (e.g. out of memory) sends ok = 0, so
        # every rank takes the two-pass form together instead of waiting in a collective
        pk_ok, kp, vp, cp, blockcap, E, totals = False, 0, 0, 0, 0, 0, np.zeros(W, np.int64)
        if handle is not None:
            try:
                self.ctx.fused_items_build(handle, build_key, gkc, nb, span, items.data_ptr(), offs.data_ptr())
                pk_ok, kp, vp, cp, blockcap, E, totals = self.ctx.shuffle_items_pack(handle, W)
            except abi.QehError:
                pk_ok = False
        if not pk_ok:
            totals = np.zeros(W, np.int64)
        meta = torch.tensor(list(totals) + [1 if pk_ok else 0], dtype=torch.int64, device="cuda")
        Mt = _allgather_meta_t(meta, W, self.group)
        if int(Mt[:, W].min()) == 0:
            if handle is not None:
                self.ctx.fused_items_abort(handle)
            return None
        gi = torch.empty(W * nb * span, dtype=torch.int32, device="cuda")
        go = torch.empty(W * nb * OW, dtype=torch.int32, device="cuda")
        dist.all_gather_into_tensor(gi, items, group=self.group)
        dist.all_gather_into_tensor(go, offs, group=self.group)
        # (this rank's own block stays in phase A's regions: nothing to or from itself)
        pin, pout = [int(x) for x in Mt[me, :W]], [int(x) for x in Mt[:, me]]
        pin[me] = pout[me] = 0
        peak = _peak_remote(Mt[:, :W])
        starts = [q * blockcap for q in range(W)]
        nacol = vp != 0
        # (received keys / values with slack: phase B's pair loads may read one item past a count; the
        # 16-bit keys travel as 32-bit pairs -- every block and total is even -- which gloo also carries)
        keys_t = torch.as_tensor(_DeviceView(kp, W * blockcap // 2, "<i4", handle))
        rk = _all_to_all(keys_t, [c // 2 for c in pin], [c // 2 for c in pout], peak // 2, self.group,
                         [x // 2 for x in starts], pad=2)
        rv = None
        if nacol:
            vals_t = torch.as_tensor(_DeviceView(vp, W * blockcap, "<i8", handle))
            rv = _all_to_all(vals_t, pin, pout, peak, self.group, starts, pad=4)
        cnt_t = torch.as_tensor(_DeviceView(cp, W * E, "<i4", handle))
        rc = _all_to_all(cnt_t, [E] * W, [E] * W, E, self.group)
        src_off = np.concatenate([[0], np.cumsum(pout)[:-1]]).astype(np.int64)
        nl = (1 + len(aggs)) * G + 1
        lanes = torch.empty(nl, dtype=torch.float64, device="cuda")
        self._sync_torch()
        self.ctx.shuffle_items_finish(handle, rk.data_ptr(), rv.data_ptr() if rv is not None else 0, rc.data_ptr(),
                                      src_off, gi.data_ptr(), span, go.data_ptr(), W * nb, G, lanes.data_ptr())
        self._sync()
        dist.all_reduce(lanes, op=dist.ReduceOp.SUM, group=self.group)
        self._sync_torch()
        got, ov, g, bad = self.ctx.dense_states_take_status(
            lanes.data_ptr(), len(aggs), gmin, G, W, me, gkc.dtype,
            [abi.DT_INT64 if f == AF.Count else abi.DT_FLOAT64 for f, _ in aggs])
        if bad != 0.0:
            return None
        self.last_final = "dense"
        return [got], ov, g

    def _moved_shuffle_ok(self, part_keys, cols) -> bool:
        """The fused window shuffle applies: one non-null 16-B aligned Int64 PARTITION BY key, every
        moved column a non-null Int64 / Float64, at most 16 ranks (QEH_DIST_WINDOW_PERM=1: the
        permutation + take / scatter form)."""
        if len(part_keys) != 1 or self.world > 16 or os.environ.get("QEH_DIST_WINDOW_PERM"):
            return False
        k = part_keys[0].c
        if k.dtype != abi.DT_INT64 or (k.validity and k.null_count != 0) or ((k.values or 0) + k.offset * 8) % 16:
            return False
        return all(c.dtype in (abi.DT_INT64, abi.DT_FLOAT64) and not (c.c.validity and c.c.null_count != 0) for c in cols)

    def _moved_window(self, part_keys, cols, local_fn) -> DeviceColumn:
        """The window shuffle as two streaming passes instead of a permutation, a take per column and a
        scatter: qeh_partition_hash_move carries (key, order keys, argument) to their rank in one pass,
        the rank computes the function on what it received (source-rank-major = global input order,
        stable within a source), the reverse all-to-all returns each source's rows in the order it sent
        them, and qeh_partition_hash_unmove puts them back into input order (the same stable ranking,
        gathering instead of scattering)."""
        counts, moved = self.ctx.partition_hash_move([part_keys[0]], self.world, cols)
        recv, recv_counts = self._exchange_columns(moved, counts)
        res = local_fn(recv)
        back, _ = self._exchange_columns([res], recv_counts)
        return self.ctx.partition_hash_unmove(part_keys[0], self.world, [back[0]])[0]

    def row_number(self, part_keys: Sequence[DeviceColumn], order_keys: Sequence[DeviceColumn],
                   ascending: Sequence[bool]) -> DeviceColumn:
        """ROW_NUMBER() OVER (PARTITION BY .. ORDER BY ..) over rank-sharded rows
        (global input order = rank-major).  Rows are hash-shuffled by the first
        partition key, so each PARTITION BY group lives on one rank and is numbered
        there (received order = source-rank-major, stable within a source, i.e. the
        global input order that breaks ties); the numbers go back by the reverse
        all-to-all into this rank's input order (_moved_window, or a permutation and
        a scatter for shapes it does not take)."""
        cols = list(part_keys) + list(order_keys)
        if self._moved_shuffle_ok(part_keys, cols):
            npk = len(part_keys)
            return self._moved_window(part_keys, cols,
                                      lambda recv: self.ctx.row_number(recv[:npk], recv[npk:], list(ascending)))
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
        cols = list(part_keys) + list(order_keys) + ([arg] if arg is not None else [])
        npk, nok = len(part_keys), len(order_keys)
        if func in (W.RowNumber, W.Rank, W.DenseRank, W.Ntile) and self._moved_shuffle_ok(part_keys, cols):
            # non-null Int64 results: back through the moved route
            return self._moved_window(part_keys, cols, lambda recv: self.ctx.window(
                func, recv[:npk], recv[npk:npk + nok], list(ascending),
                arg=recv[npk + nok] if arg is not None else None, param=param, default=default))
        counts, perm = self.ctx.hash_partition(part_keys[0], self.world)
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
