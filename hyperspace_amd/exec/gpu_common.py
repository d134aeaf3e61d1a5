"""Names shared by the device executor's modules (``exec/gpu.py`` and its operator families
``gpu_agg`` / ``gpu_join`` / ``gpu_semi`` / ``gpu_hash``): imports, limits, the device relation
``DRel``, prepared lowerings and the query future."""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from ..index import constants as C
from ..ops import _lib as NL
from ..ops import kernels as K
from ..plan import expressions as E
from ..plan import physical as X
from ..utils import murmur3
from ..utils.conf import HyperspaceConf
from ..utils.tracing import TRACER, stage
from . import compile as CP
from . import jit, jit_runs, join_index
from .arrow_eval import key
from .device_cache import (DeviceTableCache, _files_key, load_bucketed_index, load_flat,
                           seeded_index)
from .device_table import DeviceColumn, DeviceTable
from .graphs import GraphCache, ScanAggGraph, range_bounds
from .graphs import GraphPending as _GraphPending, _cbuf

log = logging.getLogger("hyperspace_amd.exec.gpu")

# per-wavefront list size of a run top-K aggregate (hash_agg.TopKPlan.K): LIMIT must be below
H_TOPK_K = 32
Unsupported = CP.Unsupported
MAX_GROUPS_SCAN = 3000
MAX_GROUPS_JOIN = 2400
# LDS bytes a dense aggregate's group table may take (32 bytes per group x aggregate: sum, min,
# max, count) beside the rest of the kernel's LDS (160 KiB per CU on gfx950)
GROUP_LDS_SCAN = 144 << 10
GROUP_LDS_JOIN = 112 << 10


def _group_limit(limit: int, lds: int, naggs: int) -> int:
    """Most groups a dense aggregate of ``naggs`` aggregates (+ COUNT(*)) keeps in LDS."""
    return max(1, min(limit, lds // (32 * (naggs + 1))))
# a grouped aggregate with more groups than this returns candidates of ORDER BY ... LIMIT from
# the device top-k instead of copying every group to the host
TOPK_MIN_GROUPS = 4096


class _NeedHash(CP.Unsupported):
    """The dense (LDS) grouped aggregate does not apply; run the hash-mode aggregate
    (exec/hash_agg.py) instead of falling back to the host."""


class DRel:
    def __init__(self, table: DeviceTable, colmap: Dict[int, str], attrs: List[E.Attribute],
                 conds: Optional[list] = None, bucketed: bool = False,
                 sort_attrs: Optional[List[E.Attribute]] = None,
                 bucket_attrs: Optional[List[E.Attribute]] = None, num_buckets: int = 0,
                 parts: Optional[List["DRel"]] = None, split: bool = False):
        self.table = table
        self.colmap = colmap
        self.attrs = attrs
        self.conds = list(conds or [])
        self.bucketed = bucketed
        self.sort_attrs = list(sort_attrs or [])
        self.bucket_attrs = list(bucket_attrs or [])
        self.num_buckets = num_buckets
        # BucketUnion: co-partitioned parts (each sorted within its buckets); table is None
        self.parts = parts
        # distributed: this rank holds a file split of a non-index relation (rows not yet routed
        # to their bucket owners)
        self.split = split
        # computed projection columns of this query (exec/project.py), by colmap name
        self.extra: Dict[str, DeviceColumn] = {}

    def col(self, a: E.Attribute) -> DeviceColumn:
        if self.parts:
            raise Unsupported("column access on a bucket union")
        name = self.colmap.get(a.expr_id)
        if name is None:
            raise Unsupported(f"attribute {a.sql()} not available on device")
        c = self.extra.get(name)
        return c if c is not None else self.table.columns[name]

    def is_computed(self, a: E.Attribute) -> bool:
        return self.colmap.get(a.expr_id) in self.extra

    def copy(self, **kw) -> "DRel":
        d = DRel(self.table, dict(self.colmap), list(self.attrs), list(self.conds), self.bucketed,
                 self.sort_attrs, self.bucket_attrs, self.num_buckets, self.parts, self.split)
        d.extra = dict(self.extra)
        for k, v in kw.items():
            setattr(d, k, v)
        return d


_SCHEMAS: dict = {}


def arrow_table(arrays, names) -> pa.Table:
    """``pa.Table.from_arrays(arrays, names=names)`` through a cached schema: building the
    schema from names costs several times the table itself, on every query result."""
    key = (tuple(names), tuple(a.type for a in arrays))
    sch = _SCHEMAS.get(key)
    if sch is None:
        if len(_SCHEMAS) >= 512:
            _SCHEMAS.clear()
        sch = _SCHEMAS[key] = pa.schema([pa.field(n, a.type) for n, a in zip(names, arrays)])
    return pa.Table.from_arrays(arrays, schema=sch)


def _finalize_array(fn, s, c, mn, mx) -> pa.Array:
    """Vectorized ``CP.finalize_value`` over the groups of a hash-mode aggregate."""
    c = np.asarray(c, dtype=np.int64)
    if isinstance(fn, E.Count):
        return pa.array(c, type=pa.int64())
    null = c == 0
    if isinstance(fn, E.Avg):
        with np.errstate(divide="ignore", invalid="ignore"):
            return pa.array(np.where(null, 0.0, s / np.maximum(c, 1)), mask=null)
    v = s if isinstance(fn, E.Sum) else (mn if isinstance(fn, E.Min) else mx)
    v = np.where(null, 0.0, v)
    if CP.int_result(fn):
        return pa.array(np.rint(v).astype(np.int64), mask=null)
    t = fn.child.data_type
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_date32(t):
        return pa.array(np.rint(v).astype(np.int32), mask=null).view(pa.date32())
    if isinstance(fn, (E.Min, E.Max)) and CP._int_coded(t):
        return pa.array(np.rint(v).astype(np.int64), mask=null).cast(t)
    if isinstance(fn, (E.Min, E.Max)) and pa.types.is_decimal(t):
        return pa.array([CP.finalize_value(fn, 0.0, 1, x, x) if not nl else None
                         for x, nl in zip(v, null)], type=t)
    return pa.array(v.astype(np.float64), mask=null)


def _eval_vec(e, vals, gmap, n: int) -> pa.Array:
    """Output expression of an aggregate over whole result columns."""
    import pyarrow.compute as pc
    if isinstance(e, E.AggregateFunction):
        return vals[id(e)]
    if isinstance(e, E.Attribute):
        if e.expr_id in gmap:
            return gmap[e.expr_id]
        raise Unsupported(f"result column {e.sql()}")
    if isinstance(e, E.Literal):
        return pa.array([e.value] * n)
    if isinstance(e, E.Alias):
        return _eval_vec(e.child, vals, gmap, n)
    if isinstance(e, E.Cast):
        return _eval_vec(e.child, vals, gmap, n).cast(e.data_type)
    if isinstance(e, E.BinaryArithmetic):
        a = _eval_vec(e.left, vals, gmap, n)
        b = _eval_vec(e.right, vals, gmap, n)
        if isinstance(e, E.Add):
            return pc.add(a, b)
        if isinstance(e, E.Subtract):
            return pc.subtract(a, b)
        if isinstance(e, E.Multiply):
            return pc.multiply(a, b)
        a = pc.cast(a, pa.float64())
        b = pc.cast(b, pa.float64())
        return pc.if_else(pc.equal(b, 0.0), pa.scalar(None, pa.float64()), pc.divide(a, b))
    raise Unsupported(f"result expression {type(e).__name__}")


def _combine_aggs(a, b):
    """Merge two (sum, count, min, max) partial aggregate tuples in place of ``a``."""
    import torch
    a[0].add_(b[0])
    a[1].add_(b[1])
    torch.minimum(a[2], b[2], out=a[2])
    torch.maximum(a[3], b[3], out=a[3])
    return a


def _warm_torch_kernels(device) -> None:
    """Run the PyTorch elementwise / reduction / scan kernels the query paths use once, on
    tiny tensors: ROCm loads a kernel's code object on its first launch (tens of ms each),
    which would otherwise land in the first query that needs it (profiled: floor_divide,
    cumsum, compare + any of the join setup, ~250 ms of a cold Q3)."""
    import torch
    for dt in (torch.int64, torch.int32):
        x = torch.arange(64, dtype=dt, device=device)
        y = x.flip(0)
        (x // 3, x % 3, x + y, x - y, x * y, x == y, x != y, x < y, x <= y, x > y, x >= y,
         torch.cumsum(x, 0), torch.cumsum((x + 1) // 2, 0, out=torch.empty_like(x)),
         torch.aminmax(x), x.max(), x.min(), x.sum(), (x == y).any(), (x == y).all(),
         torch.nonzero(x > 3), x.index_select(0, y.long()), torch.where(x > 3, x, y),
         x.clamp(0, 9), torch.repeat_interleave(x[:4].long(), 2), x.long(), x.int(),
         x.to(torch.float64), torch.minimum(x, y), torch.maximum(x, y), x[1:] == x[:-1],
         (x[1:] != 0) & (x[:-1] != 0), torch.zeros_like(x), torch.full_like(x, 7))
    v = torch.ones(64, dtype=torch.uint8, device=device)
    (v.bool(), v & v, v == 0, v.any(), v.sum(), v.bool().any(), torch.nonzero(v))
    f = torch.linspace(0, 1, 64, dtype=torch.float64, device=device)
    (f + f, f * f, f / 3, f < 0.5, torch.aminmax(f), f.sum(), torch.minimum(f, f),
     torch.maximum(f, f), torch.isnan(f), f.to(torch.int64))
    torch.cuda.synchronize(device)


def _needs_eval(c: E.Expression) -> bool:
    """A predicate over computed values (arithmetic, or a cast that changes a column's values):
    the scan kernels' predicate compiler takes column / literal comparisons (it looks through
    value-preserving casts only), so such a conjunct is evaluated as a computed column."""
    for x in c.iter_tree():
        if isinstance(x, E.BinaryArithmetic):
            return True
        if isinstance(x, E.Cast) and not isinstance(x.child, E.Literal) and \
                not _lossless_cast(x.child.data_type, x.dtype):
            return True
    return False


def _lossless_cast(src: pa.DataType, dst: pa.DataType) -> bool:
    if src == dst:
        return True
    if pa.types.is_integer(src) and pa.types.is_integer(dst):
        return dst.bit_width >= src.bit_width and \
            pa.types.is_signed_integer(dst) >= pa.types.is_signed_integer(src)
    if pa.types.is_float64(dst):
        return pa.types.is_floating(src) or \
            (pa.types.is_integer(src) and src.bit_width <= 32) or pa.types.is_decimal(src)
    return False


def _prefix_sorted(r: DRel, exprs) -> bool:
    if r.parts:
        return all(_prefix_sorted(x, exprs) for x in r.parts)
    if len(exprs) > len(r.sort_attrs):
        return False
    for e, s in zip(exprs, r.sort_attrs):
        if not isinstance(e, E.Attribute):
            return False
        if r.colmap.get(e.expr_id) != r.colmap.get(s.expr_id):
            return False
    return True


def _eval_scalar(e, agg_val, attr_val):
    if isinstance(e, E.AggregateFunction):
        return agg_val(e)
    if isinstance(e, E.Attribute):
        return attr_val(e)
    if isinstance(e, E.Literal):
        return e.value
    if isinstance(e, E.Alias):
        return _eval_scalar(e.child, agg_val, attr_val)
    if isinstance(e, E.Cast):
        return _eval_scalar(e.child, agg_val, attr_val)
    if isinstance(e, E.BinaryArithmetic):
        a = _eval_scalar(e.left, agg_val, attr_val)
        b = _eval_scalar(e.right, agg_val, attr_val)
        if a is None or b is None:
            return None
        if isinstance(e, E.Add):
            return a + b
        if isinstance(e, E.Subtract):
            return a - b
        if isinstance(e, E.Multiply):
            return a * b
        return None if b == 0 else a / b
    raise Unsupported(f"result expression {type(e).__name__}")


_SEMI_LITS: dict = {}


def _semi_fail_key(node) -> tuple:
    """Memo key of a semi-join whose build keys repeated: the join node AND the literal values
    under it - a plan-cache hit re-submits the same nodes with other literals, whose filtered
    build side may well be unique."""
    hit = _SEMI_LITS.get(id(node))
    if hit is not None and hit[0] is node:
        lits = hit[1]
    else:
        # the literal OBJECTS under a node are fixed (a bound plan-cache hit rewrites their
        # values in place): walk the subtree once per node, read the values per query
        from ..plan.plan_cache import _iter_literals
        lits = []
        _iter_literals(node, lits, set())
        if len(_SEMI_LITS) >= 256:
            _SEMI_LITS.clear()
        _SEMI_LITS[id(node)] = (node, lits)
    try:
        vals = tuple(x.value for x in lits)
        hash(vals)
    except TypeError:
        vals = tuple(id(x) for x in lits)
    return (id(node), vals)


class _Stale(Exception):
    """A prepared lowering no longer matches the query (the normal path runs instead)."""


class _GraphPrep:
    __slots__ = ("key", "g", "k", "compacts", "values", "GA", "packed", "marked", "tpl")

    def __init__(self, key, g, k, compacts, values, GA):
        self.key, self.g, self.k, self.compacts, self.values, self.GA = \
            key, g, k, compacts, values, GA
        self.tpl = None     # packed block of the literal-independent slots (Args.patch)
        self.packed: Dict[tuple, tuple] = {}     # literal vector -> (range bounds, args block)
        self.marked = None    # the side stream every persistent buffer was marked in use by


def bucket_chunks(per_bucket, budget: int) -> List[tuple]:
    """Contiguous bucket ranges [lo, hi) whose estimated resident bytes (``per_bucket``, the
    decoded bytes of every index of a plan per bucket) stay within half of ``budget`` - the
    pass's tables plus what its kernels derive - one bucket at least per range."""
    cap = max(budget // 2, 1)
    chunks, lo, acc = [], 0, 0.0
    for b, wb in enumerate(per_bucket):
        if acc and acc + wb > cap:
            chunks.append((lo, b))
            lo, acc = b, 0.0
        acc += float(wb)
    chunks.append((lo, len(per_bucket)))
    return chunks


def _literals(exprs) -> list:
    """The Literal nodes under ``exprs`` (depth first)."""
    out = []
    stack = list(reversed(list(exprs)))
    while stack:
        e = stack.pop()
        if isinstance(e, E.Literal):
            out.append(e)
        else:
            stack.extend(reversed(getattr(e, "children", ()) or ()))
    return out


class _ScanPrep:
    """Literal-independent lowering of a fused scan aggregate (GpuBackend._dense_agg), plus
    the literal-dependent part per literal vector (``lowered``): the plan cache binds a query's
    literals into the same Literal nodes of the cached plan, so their values key the range
    bounds, bound predicates and aggregate terms - a repeated parameter set (a dashboard's
    queries) skips predicate compilation altogether."""
    __slots__ = ("final", "r", "col_info", "descs", "gs", "params", "graph", "placement",
                 "lits", "lowered", "tbound")

    def __init__(self, final, r, col_info, descs, gs, params, graph, placement):
        self.final, self.r, self.col_info, self.descs, self.gs = final, r, col_info, descs, gs
        self.params, self.graph, self.placement = params, graph, placement
        self.lits = _literals(list(r.conds) + list(final.aggregates))
        self.lowered: Dict[tuple, tuple] = {}
        # (implied condition ids, bound predicates) of a lowering whose literals CP.rebind can
        # re-read: a new literal vector skips the CNF conversion and column binding
        self.tbound = None

    def literal_key(self):
        try:
            k = tuple(x.value for x in self.lits)
            hash(k)
            return k
        except TypeError:
            return None

    def tables(self):
        return (self.r.table,)

    def run(self, be, fns, group):
        return be._scan_agg(self.r, fns, group, self)

    def fast(self, be, fns, group):
        """``run`` for a literal vector whose lowering and graph block are cached, with no
        re-validation beyond the graph's (``_AggProgram`` checked residency); None otherwise."""
        gp = self.graph
        if gp is None:
            return None
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        hit = gp.packed.get(lkey) if low is not None else None
        if hit is None or low[1].always_false or be.graphs.peek(gp.key) is not gp.g:
            return None
        g = gp.g
        side = gp.marked
        if side is None and (g.on_side or HyperspaceConf.side_stream_scans(be.session.conf)):
            return None     # the full path moves warm replays to the side stream first
        agreed, G, gbase, gdict, gtype = self.gs
        be._groups_agreed = agreed is True
        if side is None:
            handle = g.launch(hit[0], hit[1])
        else:
            import torch
            for x in hit[2]:
                _use_on(x, side)
            # on the side stream, ordered after this stream's queued work (one native call)
            handle = g.launch(hit[0], hit[1], stream=side, after=torch.cuda.current_stream())
        return (_GraphPending(g, handle), None, None, None, G, gbase, gdict, gtype)


class _JoinPrep:
    """Literal-independent lowering of a co-located merge-join aggregate: the two resident
    relations, column slots, group domain and the kernel launcher (jit.MergeJoinLauncher).
    A submission re-binds the predicates and aggregate terms and launches."""
    __slots__ = ("final", "node", "left", "right", "lk", "rk", "col_info", "descs", "launcher",
                 "gtail", "placement", "agreed", "lits", "lowered", "lconds", "tjoin")

    def __init__(self, final, node, left, right, lk, rk, col_info, descs, launcher, gtail,
                 placement, agreed, lconds=None):
        self.final, self.node, self.left, self.right = final, node, left, right
        self.lk, self.rk, self.col_info, self.descs = lk, rk, col_info, descs
        self.launcher, self.gtail, self.placement, self.agreed = launcher, gtail, placement, agreed
        # the left conjuncts the recorded launch bound (same order: predicate slots match)
        self.lconds = list(left.conds) if lconds is None else list(lconds)
        conds = list(left.conds) + list(right.conds) + \
            ([node.condition] if node.condition is not None else [])
        self.lits = _literals(conds + list(final.aggregates))
        self.lowered: Dict[tuple, tuple] = {}   # literal vector -> (params, keep, specs)
        self.tjoin = None     # (join params, (left, right) bound predicates) to CP.rebind

    literal_key = _ScanPrep.literal_key

    def tables(self):
        return (self.left.table, self.right.table)

    def run(self, be, fns, group):
        left = self.left
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        if low is None and be._range_spec(left, left.conds) is not None:
            raise _Stale()        # the new literals bound the left key: ranges change
        nd = len(self.descs)
        with stage("join.agg_kernel"):
            if low is None:
                jp = None
                col_info, descs = self.col_info, self.descs
                if self.tjoin is not None:
                    tjp, (tlb, trb) = self.tjoin
                    lb, rb = CP.rebind(tlb), CP.rebind(trb)
                    if lb is not None and rb is not None:
                        jp = NL.JoinParams.from_buffer_copy(tjp)
                        for i, pr in enumerate(lb.preds + rb.preds):
                            jp.preds[i] = pr
                        keep = (lb, rb)
                if jp is None:
                    jp, col_info, descs, keep = be._join_params(
                        left, self.right, self.lk, self.rk, self.node.condition,
                        lconds=self.lconds, slots=(self.col_info, self.descs))
                    if keep[0].rebindable and keep[1].rebindable:
                        self.tjoin = (NL.JoinParams.from_buffer_copy(jp), keep)
                specs = be._agg_specs(fns, col_info)
                if len(descs) != nd:
                    raise _Stale()
                if lkey is not None:
                    if len(self.lowered) >= 1024:
                        self.lowered.clear()
                    self.lowered[lkey] = (jp, keep, specs)
            else:
                jp, keep, specs = low
                col_info = self.col_info
            G, gbase = self.gtail[0], self.gtail[1]
            if keep[0].always_false or keep[1].always_false:
                out = be._empty_agg(len(specs), G)
            else:
                for i, a in enumerate(specs):
                    jp.aggs[i] = a
                jp.naggs = len(specs)
                if group is not None:
                    jp.group_col = col_info(group).slot if G > 1 else -1
                    jp.num_groups, jp.group_base = G, gbase
                if isinstance(self.launcher, jit_runs.TwoPhaseLauncher):
                    out = self.launcher.launch(
                        jp, lkey, graph=HyperspaceConf.join_graph_enabled(be.session.conf))
                    if isinstance(out, _GraphPending):
                        out = (out, None, None, None)
                else:
                    out = self.launcher.launch(jp)
        be._groups_agreed = self.agreed
        return (*out, *self.gtail)

    def fast(self, be, fns, group):
        """``run`` replaying the captured two-phase pipeline for a cached literal vector; None
        when that does not apply (the full ``run`` / planning path runs instead)."""
        launcher = self.launcher
        if not isinstance(launcher, jit_runs.TwoPhaseLauncher) or launcher.graph is None:
            return None
        lkey = self.literal_key()
        low = self.lowered.get(lkey) if lkey is not None else None
        if low is None or lkey not in launcher.gblocks:
            return None
        jp, keep, specs = low
        if keep[0].always_false or keep[1].always_false:
            return None
        out = launcher.launch(jp, lkey, graph=True)
        be._groups_agreed = self.agreed
        return (out, None, None, None, *self.gtail)


class _HashPrep:
    """Literal-independent setup of a hash-mode join aggregate (GpuBackend._hash_agg): the
    co-partitioned relations, functional-dependency grouping, group domains and top-K request,
    plus per literal vector the lowering ``_join_hash_pair`` made (join parameters, hash key
    plan, ranges) - the plan cache binds a query's literals into the same Literal nodes of the
    cached plan, so their values key it."""
    __slots__ = ("final", "order", "limit", "node", "tables", "setup", "placement", "epoch",
                 "lits", "lowered")

    def __init__(self, final, order, limit, node, tables, setup, placement, epoch):
        self.final, self.order, self.limit, self.node = final, order, limit, node
        self.tables, self.setup, self.placement, self.epoch = tables, setup, placement, epoch
        left, right = setup[0], setup[1]
        conds = list(left.conds if left is not None else []) + \
            list(right.conds if right is not None else []) + \
            ([node.condition] if getattr(node, "condition", None) is not None else [])
        self.lits = _literals(conds + list(final.aggregates))
        self.lowered: Dict[tuple, tuple] = {}

    def literal_key(self, extra=None):
        try:
            k = (tuple(x.value for x in self.lits), extra)
            hash(k)
            return k
        except TypeError:
            return None

    def keep_lowered(self, key, low) -> None:
        if len(self.lowered) >= 1024:
            self.lowered.clear()
        self.lowered[key] = low


class _AggProgram:
    """Prepared re-submission of a fused aggregate plan (GpuBackend._register_program): a
    plan-cache hit binds its literals into the cached plan's nodes and the program replays the
    prepared lowering of its literal vector - a captured hipGraph (scan: ``ScanAggGraph``;
    two-phase merge join: ``TwoPhaseGraph``) - and queues the cross-rank combine, skipping the
    executor's plan walk and every per-query lowering check.  A literal vector it has not seen
    is lowered by the prep itself (``prep.run``, still no plan walk).  Valid while the
    device-table cache has evicted nothing since it was made (``epoch``); any other miss
    (eviction, placement change, a prep gone stale, graph dropped) returns None and the full
    path runs (and re-registers)."""
    __slots__ = ("final", "fns", "group", "prep", "epoch", "n")

    def __init__(self, be, final, fns, group, prep, epoch):
        self.final, self.fns, self.group, self.prep, self.epoch = final, fns, group, prep, epoch
        self.n = 0

    def submit(self, be, plan, t0):
        if be.cache.epoch != self.epoch:
            return None
        self.n += 1
        if self.n % 64 == 0 and not all(be._holds(t) for t in self.prep.tables()):
            return None      # (also keeps the tables recent in the cache's LRU)
        res = self.prep.fast(be, self.fns, self.group)
        if res is None:
            # a literal vector this program has not lowered yet: its literal-dependent lowering
            # runs here (what the executor's _dense_agg would run for this prep) instead of
            # after a walk of the plan; anything the prep cannot take returns to that path
            if self.prep.placement != be._placement_tag():
                return None
            be._groups_agreed = False
            try:
                res = self.prep.run(be, self.fns, self.group)
            except _Stale:
                return None
            if res is None:
                return None
        finish = be._agg_finish(self.final, self.fns, self.group, res)
        return QueryFuture(be, plan, finish, "native", None, t0)


def _gather_tables(d, t: pa.Table) -> pa.Table:
    """Every rank's (small) result table, concatenated in rank order: Arrow IPC bytes through
    one row all-gather (``DistContext.all_gather_rows``), no pickling."""
    import pyarrow.ipc as ipc
    sink = pa.BufferOutputStream()
    with ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    b = sink.getvalue().to_pybytes()
    n = len(b)
    words = np.frombuffer(b + b"\0" * ((-n) % 8), dtype=np.int64)
    allr = d.all_gather_rows(np.concatenate([[n], words]).astype(np.int64).reshape(-1, 1))
    allr = allr.reshape(-1)
    out, i = [], 0
    while i < len(allr):
        nb = int(allr[i])
        nw = (nb + 7) // 8
        out.append(ipc.open_stream(pa.py_buffer(allr[i + 1:i + 1 + nw].tobytes()[:nb])).read_all())
        i += 1 + nw
    out = [x if x.schema.equals(t.schema) else x.cast(t.schema) for x in out]
    return pa.concat_tables(out)


def _fd_columns(attrs, cols, fd, gmap: dict) -> None:
    """``gmap[attr]`` from the device functional-dependency lookup (``TopKPlan.unpack``'s
    rows, 64-bit values and validity per right column)."""
    import torch
    rows, vals, valid = fd
    if (rows < 0).any():
        raise RuntimeError("functional-dependency lookup: a group key has no right row")
    for a, c, v, ok in zip(attrs, cols, vals, valid):
        nd = np.dtype(str(c.data.dtype).replace("torch.", ""))
        x = v.view(np.float64).astype(nd) if c.is_float else v.astype(nd)
        dc = DeviceColumn(torch.from_numpy(x), None if ok.all() else
                          torch.from_numpy(ok.astype(np.uint8)), c.atype, c.dictionary)
        arr = dc.to_arrow()
        if not arr.type.equals(a.data_type):
            try:
                arr = arr.cast(a.data_type)
            except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                pass
        gmap[a.expr_id] = arr


class _NoCondition:
    """A join node stand-in without a residual condition (``_copart_semi``'s derived join)."""
    condition = None


def _strip_exchange(p):
    """The child below a [Sort(local) <-] hash Exchange (a join side Spark would shuffle), or
    None when ``p`` does not start with one."""
    if isinstance(p, X.SortExec) and not p.global_sort:
        p = p.child
    if isinstance(p, X.ShuffleExchangeExec) and isinstance(p.partitioning, X.HashPartitioning):
        return p.child
    return None


_PLAN_BYTES: dict = {}


def _plan_bytes(p) -> int:
    """Bytes of the files under a physical plan's scans (the build side of a semi-join is the
    side with fewer); memoized per plan node (its file listings are fixed)."""
    hit = _PLAN_BYTES.get(id(p))
    if hit is not None and hit[0] is p:
        return hit[1]
    n = _plan_bytes_walk(p)
    if len(_PLAN_BYTES) >= 256:
        _PLAN_BYTES.clear()
    _PLAN_BYTES[id(p)] = (p, n)
    return n


def _plan_bytes_walk(p) -> int:
    n = 0
    for s in p.collect(lambda x: isinstance(x, X.FileSourceScanExec)):
        try:
            n += sum(int(f.length) for f in s.relation.location.all_files())
        except Exception:  # noqa: BLE001 - a relation without a file listing counts 0
            pass
    return n


def _use_on(x, stream) -> None:
    """``x.record_stream(stream)`` once per (tensor, stream): the caching allocator keeps the
    streams a block was used on until the block is freed, and then waits for the work queued
    on each of them by that time, so one record covers every later use on the stream."""
    if getattr(x, "_hs_used_on", None) is not stream:
        x.record_stream(stream)
        x._hs_used_on = stream


def _compact_buffers(enc) -> list:
    """Device tensors of a compact encoding whose pointers go into a kernel's argument block
    (codes, and a grouped 16-bit form's group bases and wide codes)."""
    out = [enc.codes]
    g = getattr(enc, "g16", None)
    for e in (enc, g if g else None):
        if e is None:
            continue
        for name in ("gbase", "wide", "codes"):
            x = getattr(e, name, None)
            if x is not None and hasattr(x, "record_stream") and all(x is not y for y in out):
                out.append(x)
    return out


class QueryFuture:
    """Handle of a submitted query (``GpuBackend.collect_async``)."""

    def __init__(self, backend, plan, finish, path: str, reason, t0: float):
        self.backend, self.plan = backend, plan
        self.plan_fn = None         # builds the plan when ``plan`` was a bound cached plan
        self._finish = finish
        self.path, self.reason = path, reason
        self._t0 = t0
        self._value = None
        self._done = False

    def result(self) -> pa.Table:
        if not self._done:
            try:
                self._value = self._finish()
            except Unsupported as e:   # e.g. a result expression the device path cannot finish
                plan = self.plan if self.plan is not None else self.plan_fn()
                f = self.backend._fallback(plan, e, self._t0)
                self._value, self.path, self.reason = f.result(), f.path, f.reason
                self.backend.last_path, self.backend.fallback_reason = self.path, self.reason
            self._done = True
            self._finish = None
            self.backend.metrics["last_query_s"] = time.perf_counter() - self._t0
        return self._value


__all__ = [n for n in list(globals()) if not n.startswith("__")]
