"""Job-global sorted string dictionaries for multi-rank builds and shuffles.

String columns live on the device as int32 codes into a *sorted* dictionary (code order ==
string order), so a multi-rank build or shuffle needs one dictionary shared by every rank.
Each rank contributes its local sorted unique values as two raw buffers (int64 offsets + UTF-8
bytes); they cross ranks with two tensor all-gathers (sizes, then payload padded to the largest
rank) — no pickled Python objects — and every rank merges the same inputs into the same sorted
union.  Codes then move to the union with one device gather through a local -> global table.
"""
from __future__ import annotations

from typing import List

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc


def _to_buffers(arr: pa.Array):
    a = arr.cast(pa.large_string())
    if a.null_count:
        a = a.drop_null()
    bufs = a.buffers()
    offs = np.frombuffer(bufs[1], dtype=np.int64)[a.offset:a.offset + len(a) + 1]
    chars = np.frombuffer(bufs[2], dtype=np.uint8)[offs[0]:offs[-1]] if bufs[2] is not None and \
        len(a) else np.zeros(0, np.uint8)
    return (offs - offs[0]).astype(np.int64), np.ascontiguousarray(chars)


def _from_buffers(offs: np.ndarray, chars: np.ndarray) -> pa.Array:
    n = len(offs) - 1
    if n <= 0:
        return pa.array([], pa.string())
    return pa.LargeStringArray.from_buffers(n, pa.py_buffer(offs.tobytes()),
                                            pa.py_buffer(chars.tobytes())).cast(pa.string())


def all_gather_bytes(ctx, payload: np.ndarray) -> List[np.ndarray]:
    """Every rank's uint8 ``payload`` (sizes may differ), in rank order."""
    import torch
    import torch.distributed as dist
    dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
    n = torch.tensor([payload.size], dtype=torch.int64, device=dev)
    sizes = torch.empty(ctx.world, dtype=torch.int64, device=dev)
    if ctx.backend == "nccl":
        dist.all_gather_into_tensor(sizes, n)
    else:
        parts = list(sizes.chunk(ctx.world))
        dist.all_gather(parts, n)
        sizes = torch.cat(parts)
    sizes = sizes.cpu().numpy()
    mx = max(int(sizes.max()), 1)
    buf = np.zeros(mx, np.uint8)
    buf[:payload.size] = payload
    src = torch.from_numpy(buf).to(dev)
    if ctx.backend == "nccl":
        out = torch.empty(mx * ctx.world, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, src)
        flat = out.cpu().numpy()
        return [flat[r * mx:r * mx + int(sizes[r])] for r in range(ctx.world)]
    outs = [torch.empty(mx, dtype=torch.uint8) for _ in range(ctx.world)]
    dist.all_gather(outs, src)
    return [o.numpy()[:int(s)] for o, s in zip(outs, sizes)]


def union_sorted(local: pa.Array, ctx) -> pa.Array:
    """The sorted union of every rank's string values (``local`` need not be unique/sorted)."""
    local = pc.unique(local.cast(pa.string()).drop_null()) if len(local) else \
        pa.array([], pa.string())
    if ctx is None or ctx.world <= 1:
        return local.sort()
    offs, chars = _to_buffers(local)
    head = np.array([len(offs), len(chars)], dtype=np.int64).view(np.uint8)
    payload = np.concatenate([head, offs.view(np.uint8), chars])
    arrays = []
    for p in all_gather_bytes(ctx, payload):
        no, nc = (int(x) for x in p[:16].view(np.int64))
        o = p[16:16 + 8 * no].view(np.int64)
        c = p[16 + 8 * no:16 + 8 * no + nc]
        arrays.append(_from_buffers(o, c))
    allv = pa.concat_arrays(arrays) if arrays else pa.array([], pa.string())
    return pc.unique(allv).sort() if len(allv) else allv


def remap_table(local_dict: pa.Array, global_dict: pa.Array) -> np.ndarray:
    """int32 positions of ``local_dict`` values in ``global_dict`` (both sorted, local a subset)."""
    if len(local_dict) == 0:
        return np.zeros(1, np.int32)
    idx = pc.index_in(local_dict.cast(pa.string()), value_set=global_dict)
    if idx.null_count:
        raise ValueError("remap_table: local dictionary value missing from the union")
    return np.asarray(idx.to_numpy(zero_copy_only=False), dtype=np.int32)
