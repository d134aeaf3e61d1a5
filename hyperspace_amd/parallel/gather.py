"""Row results of a sharded query to every rank, on the device, without pickling.

A row-producing query over bucket-sharded indexes (each rank holds the buckets its owner map gives it, ``parallel/placement.py``) ends
with every rank holding the result rows of its own buckets as device columns.  The reference's
driver collect (PlanAnalyzer.scala:217 and Spark's ``collect``) becomes here:

1. one all-gather of the per-rank row counts (int64 tensor);
2. agreement on which columns carry a validity mask (one small all-reduce) and, for string
   columns, one job-global sorted dictionary (``parallel/dictionary.union_sorted``: raw-buffer
   all-gather) with local codes remapped on the device;
3. every column's fixed-width values (and masks) packed per rank into ONE uint8 buffer, padded
   to the largest rank's row count, and ONE ``all_gather_into_tensor`` (RCCL over xGMI; gloo
   stages through host memory);
4. the gathered slices concatenated back into device columns in rank order.
"""
from __future__ import annotations

from typing import List

import numpy as np


def _all_gather_flat(ctx, buf):
    """``world`` copies of ``buf`` (same size on every rank) concatenated in rank order."""
    import torch
    import torch.distributed as dist
    if ctx.backend == "nccl":
        out = torch.empty(buf.numel() * ctx.world, dtype=buf.dtype, device=buf.device)
        dist.all_gather_into_tensor(out, buf)
        return out
    src = buf.cpu()
    outs = [torch.empty_like(src) for _ in range(ctx.world)]
    dist.all_gather(outs, src)
    return torch.cat(outs).to(buf.device)


def gather_device_columns(ctx, cols: List, n_local: int) -> List:
    """All ranks' rows of ``cols`` (DeviceColumns of equal length ``n_local``), concatenated in
    rank order, on every rank."""
    import torch
    from ..exec.device_table import DeviceColumn
    from ..ops import kernels as K
    from .dictionary import union_sorted
    if not cols:
        return cols
    dev = cols[0].data.device
    cdev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
    cnt = torch.tensor([n_local], dtype=torch.int64, device=cdev)
    counts = _all_gather_flat(ctx, cnt).cpu().numpy().astype(np.int64)
    nmax = int(counts.max()) if len(counts) else 0
    need_valid = ctx.agree_any([c.valid is not None for c in cols])
    # string columns: one job-global dictionary, local codes remapped on the device
    datas, dicts = [], []
    for c in cols:
        data = c.data[:n_local]
        gd = None
        if c.dictionary is not None:
            gd = union_sorted(c.dictionary, ctx)
            if n_local and not c.dictionary.equals(gd):
                from .dictionary import remap_table
                table = torch.from_numpy(remap_table(c.dictionary, gd)).to(dev)
                data = K.lookup_i32(table, data) if len(c.dictionary) else torch.zeros_like(data)
        datas.append(data.contiguous())
        dicts.append(gd)
    widths = [d.element_size() for d in datas]
    row_bytes = sum(widths) + sum(1 for v in need_valid if v)
    buf = torch.zeros(max(nmax, 1) * row_bytes, dtype=torch.uint8, device=dev)
    off = 0
    layout = []
    for c, d, w, nv in zip(cols, datas, widths, need_valid):
        seg = buf[off:off + nmax * w]
        if n_local:
            seg[:n_local * w].copy_(d.view(torch.uint8).reshape(-1))
        layout.append((off, w))
        off += nmax * w
        if nv:
            vseg = buf[off:off + nmax]
            if n_local:
                if c.valid is not None:
                    vseg[:n_local].copy_(c.valid[:n_local])
                else:
                    vseg[:n_local].fill_(1)
            layout.append((off, 1))
            off += nmax
        else:
            layout.append(None)
    allbuf = _all_gather_flat(ctx, buf.to(cdev) if ctx.backend == "nccl" else buf)
    allbuf = allbuf.to(dev)
    stride = max(nmax, 1) * row_bytes
    out = []
    for i, (c, d, gd) in enumerate(zip(cols, datas, dicts)):
        (doff, w), vl = layout[2 * i], layout[2 * i + 1]
        pieces, vpieces = [], []
        for r in range(ctx.world):
            n = int(counts[r])
            if not n:
                continue
            base = r * stride
            pieces.append(allbuf[base + doff: base + doff + n * w])
            if vl is not None:
                vpieces.append(allbuf[base + vl[0]: base + vl[0] + n])
        data = torch.cat(pieces).view(d.dtype) if pieces else d[:0]
        valid = torch.cat(vpieces) if vl is not None and vpieces else None
        if vl is not None and valid is None:
            valid = torch.zeros(0, dtype=torch.uint8, device=dev)
        out.append(DeviceColumn(data, valid, c.atype, gd if gd is not None else c.dictionary))
    return out


__all__ = ["gather_device_columns"]
