"""Packed row exchange: the hash-partition shuffle of an index build (Spark's
``repartition(numBuckets, indexedCols)``, ``CreateActionBase.scala:129-130``; Hybrid Scan's
appended-row shuffle, ``RuleUtils.scala:519-578``) as ONE uneven all-to-all per batch of rows.

Row ``i`` goes to rank ``dest[i]``: its bucket's owner (``bucket[i] % world`` by default, else the
session's owner map, ``parallel/placement.py``).  Every
column of a batch — values, validity bytes, bucket ids — is packed by one kernel
(``csrc/kernels/exchange.hip``) into a byte buffer with one contiguous segment per destination,
so a batch costs one counts all-to-all (device tensors, no host round trip before it), one small
D2H of the counts and segment layout (``all_to_all_single`` takes its split sizes on the host),
and one payload all-to-all.  Over RCCL on an MI355X node each rank pair has its own xGMI link,
so a single all-to-all drives all 7 links of a GPU at once; one collective per column would pay
the per-call latency C times and leave the links idle in between.

Batches are independent: ``RowExchange.add`` can be called as soon as a batch of source files
has been decoded (the payload all-to-all runs on the communicator's stream while the next batch
decodes), and ``finish`` unpacks every (batch, source rank, column) run of the received buffers
into the final columns with one copy-table kernel.  Received rows are ordered by (batch,
source rank, source row order) — deterministic for a fixed file-to-rank assignment.

CPU tensors (gloo rehearsals, CPU tests) take a numpy implementation of the same layout, so the
multi-rank tests exercise the same split sizes and unpack table as the device path.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

ALIGN = 16


def _align(x):
    return (x + ALIGN - 1) // ALIGN * ALIGN


def segment_layout(counts: Sequence[int], elem_bytes: Sequence[int]) -> np.ndarray:
    """Host mirror of ``hs_xch_scan``: ``[W, C+1]`` byte offsets of (segment d, column c) from
    the buffer start; column ``C`` is the end of segment d."""
    W, Cn = len(counts), len(elem_bytes)
    lay = np.zeros((W, Cn + 1), dtype=np.int64)
    off = 0
    for d in range(W):
        for c in range(Cn):
            lay[d, c] = off
            off += _align(int(counts[d]) * int(elem_bytes[c]))
        lay[d, Cn] = off
    return lay


def segment_bytes(count: int, elem_bytes: Sequence[int]) -> int:
    return sum(_align(int(count) * int(e)) for e in elem_bytes)


class _Batch:
    __slots__ = ("recv", "counts", "work", "keep")

    def __init__(self, recv, counts, work, keep):
        self.recv, self.counts, self.work, self.keep = recv, counts, work, keep


class RowExchange:
    """Batched packed all-to-all of a fixed column list (same dtypes on every rank)."""

    def __init__(self, ctx, dtypes: Sequence, device=None):
        import torch
        self.ctx = ctx
        self.world = ctx.world if ctx is not None else 1
        self.dtypes = list(dtypes)
        self.elem_bytes = [torch.empty(0, dtype=d).element_size() for d in self.dtypes]
        self.device = device
        self.batches: List[_Batch] = []
        self.sent_bytes = 0      # bytes this rank sent to other ranks (excludes its own slice)
        # double-buffered counts: a batch's payload all-to-all is issued when the NEXT batch
        # arrives (or at finish), by which time its counts / layout D2H has long completed, so
        # add() never blocks the host on the device (decode of the next files keeps going)
        self._pending = None
        self.host_waits = 0      # add() calls that had to wait for a counts copy
        if len(self.dtypes) > 32:
            raise ValueError("RowExchange: at most 32 columns")
        if self.world > 64:
            raise ValueError("RowExchange: at most 64 ranks")

    # -- collectives ---------------------------------------------------------------------------
    def _a2a(self, out, inp, out_splits=None, in_splits=None, async_op=False):
        import torch.distributed as dist
        ctx = self.ctx
        if ctx is None:                     # single process: the "exchange" is a local copy
            out.copy_(inp)
            return None
        if ctx._staged(inp):
            ctx.all_to_all_single(out, inp, out_splits, in_splits)   # host-staged, synchronous
            return None
        w = dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                                   input_split_sizes=in_splits, async_op=async_op)
        return w if async_op else None

    # -- send side -------------------------------------------------------------------------------
    def add(self, columns: Sequence, bucket, dest=None) -> None:
        """Exchange one batch: row ``i`` of every column goes to rank ``dest[i]`` (default
        ``bucket[i] % world``).  The pack kernel routes by ``route % world``, so an owner-map
        destination (< world) passes through it unchanged."""
        if dest is not None:
            bucket = dest.to(bucket.dtype) if dest.dtype != bucket.dtype else dest
        if len(columns) != len(self.dtypes):
            raise ValueError("RowExchange.add: column count mismatch")
        for c, dt in zip(columns, self.dtypes):
            if c.dtype != dt or c.shape[0] != bucket.shape[0]:
                raise ValueError(f"RowExchange.add: column {c.dtype}/{tuple(c.shape)} vs "
                                 f"{dt}/{tuple(bucket.shape)}")
        if bucket.is_cuda:
            self._add_device(columns, bucket)
        else:
            self._add_host(columns, bucket)

    def _add_device(self, columns, bucket) -> None:
        import torch
        from ..ops import _lib as NL
        L = NL.lib()
        W, Cn = self.world, len(columns)
        dev = bucket.device
        n = int(bucket.numel())
        tile_rows = int(L.hs_xch_tile_rows())
        ntiles = (n + tile_rows - 1) // tile_rows
        bucket = bucket.contiguous()
        cols = [c.contiguous() for c in columns]
        tile = torch.empty(max(ntiles * W, 1), dtype=torch.int64, device=dev)
        meta = torch.empty(2 * W + W * (Cn + 1), dtype=torch.int64, device=dev)
        row_bytes = sum(self.elem_bytes)
        send = torch.empty(max(n * row_bytes + ALIGN * W * Cn, 1), dtype=torch.uint8, device=dev)
        p = NL.XchParams()
        for i, c in enumerate(cols):
            p.src[i] = c.data_ptr()
            p.elem_bytes[i] = self.elem_bytes[i]
        p.ncols, p.world = Cn, W
        NL.check(L.hs_xch_pack(C.byref(p), NL.ptr(bucket), n, NL.ptr(tile), NL.ptr(meta),
                               NL.ptr(send), NL.stream_ptr()), "hs_xch_pack")
        send_cnt = meta[:W]
        recv_cnt = meta[W:2 * W]
        self._a2a(recv_cnt, send_cnt.clone())
        host = torch.empty(meta.numel(), dtype=torch.int64, pin_memory=True)
        host.copy_(meta, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        prev, self._pending = self._pending, (ev, host, send, tile, meta, cols, bucket, dev)
        if prev is not None:
            self._issue_payload(prev)

    def _issue_payload(self, pend) -> None:
        """Payload all-to-all of a packed batch whose counts copy was queued earlier."""
        import torch
        ev, host, send, tile, meta, cols, bucket, dev = pend
        W, Cn = self.world, len(self.dtypes)
        if not ev.query():
            self.host_waits += 1
        ev.synchronize()
        h = host.numpy()
        sc, rc = h[:W].copy(), h[W:2 * W].copy()
        lay = h[2 * W:].reshape(W, Cn + 1)
        send_splits = [int(lay[d, Cn] - lay[d, 0]) for d in range(W)]
        recv_splits = [segment_bytes(int(rc[s]), self.elem_bytes) for s in range(W)]
        total_send = int(lay[W - 1, Cn]) if W else 0
        recv = torch.empty(max(sum(recv_splits), 1), dtype=torch.uint8, device=dev)
        work = self._a2a(recv[:sum(recv_splits)], send[:total_send], recv_splits, send_splits,
                         async_op=True)
        self.sent_bytes += sum(send_splits) - send_splits[self.ctx.rank if self.ctx else 0]
        self.batches.append(_Batch(recv, rc, work, (send, tile, meta, cols, bucket)))

    def _add_host(self, columns, bucket) -> None:
        import torch
        W = self.world
        b = bucket.numpy()
        dest = (b % W).astype(np.int64)
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=W).astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(counts)])
        lay = segment_layout(counts, self.elem_bytes)
        send = np.zeros(max(int(lay[-1, -1]) if W else 0, 1), dtype=np.uint8)
        arrs = [c.numpy() for c in columns]
        for d in range(W):
            idx = order[starts[d]:starts[d + 1]]
            for ci, (a, eb) in enumerate(zip(arrs, self.elem_bytes)):
                o = int(lay[d, ci])
                send[o:o + len(idx) * eb] = np.ascontiguousarray(a[idx]).view(np.uint8)
        recv_cnt = torch.empty(W, dtype=torch.int64)
        self._a2a(recv_cnt, torch.from_numpy(counts))
        rc = recv_cnt.numpy().copy()
        send_splits = [int(lay[d, -1] - lay[d, 0]) for d in range(W)]
        recv_splits = [segment_bytes(int(rc[s]), self.elem_bytes) for s in range(W)]
        recv = torch.empty(max(sum(recv_splits), 1), dtype=torch.uint8)
        self._a2a(recv[:sum(recv_splits)], torch.from_numpy(send[:int(lay[-1, -1])]),
                  recv_splits, send_splits)
        self.sent_bytes += sum(send_splits) - send_splits[self.ctx.rank if self.ctx else 0]
        self.batches.append(_Batch(recv, rc, None, None))

    # -- receive side ----------------------------------------------------------------------------
    def received_rows(self) -> int:
        if self._pending is not None:
            pend, self._pending = self._pending, None
            self._issue_payload(pend)
        return int(sum(int(b.counts.sum()) for b in self.batches))

    def finish(self) -> List:
        """Wait for every batch and unpack the received runs into one tensor per column."""
        import torch
        if self._pending is not None:
            pend, self._pending = self._pending, None
            self._issue_payload(pend)
        total = self.received_rows()
        dev = self.batches[0].recv.device if self.batches else (self.device or "cpu")
        outs = [torch.empty(total, dtype=dt, device=dev) for dt in self.dtypes]
        for b in self.batches:
            if b.work is not None:
                b.work.wait()   # stream-orders the unpack after the payload all-to-all
        runs = []               # (batch recv tensor, byte offset, column, row offset, count)
        row = 0
        for b in self.batches:
            seg = 0
            for s in range(self.world):
                cnt = int(b.counts[s])
                off = seg
                for ci, eb in enumerate(self.elem_bytes):
                    if cnt:
                        runs.append((b.recv, off, ci, row, cnt))
                    off += _align(cnt * eb)
                seg = off
                row += cnt
        if dev != "cpu" and getattr(dev, "type", dev) == "cuda":
            self._unpack_device(runs, outs)
        else:
            for recv, off, ci, r0, cnt in runs:
                eb = self.elem_bytes[ci]
                src = recv[off:off + cnt * eb].view(self.dtypes[ci])
                outs[ci][r0:r0 + cnt].copy_(src)
        self.batches = []
        return outs

    def _unpack_device(self, runs, outs) -> None:
        import torch
        from ..ops import _lib as NL
        if not runs:
            return
        tab = (NL.XchCopy * len(runs))()
        mx = 0
        for i, (recv, off, ci, r0, cnt) in enumerate(runs):
            eb = self.elem_bytes[ci]
            tab[i].src = recv.data_ptr() + off
            tab[i].dst = outs[ci].data_ptr() + r0 * eb
            tab[i].count = cnt
            tab[i].elem_bytes = eb
            mx = max(mx, cnt)
        raw = np.frombuffer(bytes(tab), dtype=np.uint8)
        dev = outs[0].device
        h = torch.from_numpy(raw.copy()).pin_memory()
        d = torch.empty(h.numel(), dtype=torch.uint8, device=dev)
        d.copy_(h, non_blocking=True)
        NL.check(NL.lib().hs_xch_unpack(NL.ptr(d), len(runs), mx, NL.stream_ptr()),
                 "hs_xch_unpack")
        for recv in {id(r[0]): r[0] for r in runs}.values():
            recv.record_stream(torch.cuda.current_stream(dev))
        d.record_stream(torch.cuda.current_stream(dev))


def exchange_rows(columns: Sequence, bucket, ctx) -> List:
    """One-batch convenience: ``RowExchange(...).add(columns, bucket); finish()``."""
    ex = RowExchange(ctx, [c.dtype for c in columns], bucket.device)
    ex.add(columns, bucket)
    return ex.finish()


def pack_reference(columns: Sequence[np.ndarray], bucket: np.ndarray, world: int):
    """numpy oracle of ``hs_xch_pack``: (send bytes, per-destination counts, layout)."""
    eb = [a.dtype.itemsize for a in columns]
    dest = bucket.astype(np.int64) % world
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=world).astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)])
    lay = segment_layout(counts, eb)
    send = np.zeros(int(lay[-1, -1]), dtype=np.uint8)
    for d in range(world):
        idx = order[starts[d]:starts[d + 1]]
        for ci, a in enumerate(columns):
            o = int(lay[d, ci])
            send[o:o + len(idx) * eb[ci]] = np.ascontiguousarray(a[idx]).view(np.uint8)
    return send, counts, lay
