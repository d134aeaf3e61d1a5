"""Joins: co-partitioned inputs (packed multi-key and remapped string keys), probe-pruned ranges,
the fused merge-join aggregate over bucket-union parts, row-producing inner / outer / semi /
anti joins, and the device shuffle (repartition, row exchange)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL, kernels as K
from ..plan import expressions as E, physical as X
from ..utils.conf import HyperspaceConf
from ..utils.tracing import stage
from . import compile as CP, jit, join_index
from .arrow_eval import key
from ..parallel.placement import routes_by_key
from .device_table import DeviceColumn, DeviceTable
from .gpu_common import (_combine_aggs, _group_limit, _NeedHash, _prefix_sorted, DRel,
                         GROUP_LDS_JOIN, MAX_GROUPS_JOIN, Unsupported)


class JoinOps:
    """Join operators of ``GpuBackend`` (exec/gpu.py)."""

    # a filtered right side drives the join when it keeps fewer than 1 / PROBE_RATIO of the left
    # rows; only tried when the right table itself is this much smaller than the left
    PROBE_RATIO = 64
    PROBE_MAX = 1 << 20

    def _probe_ranges(self, left: DRel, right: DRel, lk, rk):
        """Key-probe ranges of ``left`` for a selective, filtered ``right`` (a dimension filtered
        down to a few keys against a large fact index sorted by the join key): the right rows
        passing their predicates are selected first, and each distinct (bucket, key) of them
        becomes one equality range search in the left's bucket, so the join scans only the
        matching key runs of the left instead of every left row.  None when the shape does not
        qualify (then the left's own ranges drive the join).  Left-side predicates are not
        applied by these ranges; the caller evaluates all of them per row."""
        import torch
        if left.parts or right.parts or not right.conds or not left.bucketed:
            return None
        nl, nr = left.table.num_rows or 0, right.table.num_rows or 0
        if nl < (1 << 20) or nr * 8 > nl:
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.offsets is not None:
            return None
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}.get(lc.hs_type)
        if width is None or rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        # a pair whose filtered side turned out not selective twice is not probed again (the
        # selection costs a scan of the right side and a host sync per query)
        pk_ = (id(left.table), id(right.table))
        misses = self.__dict__.setdefault("_probe_misses", {})
        if misses.get(pk_, 0) >= 2:
            return None
        with stage("join.probe_select"):
            rows = self._selected_rows(right)
            npass = int(rows.numel())
        if npass * self.PROBE_RATIO > nl or npass > self.PROBE_MAX:
            if len(misses) > 4096:
                misses.clear()
            misses[pk_] = misses.get(pk_, 0) + 1
            return None
        with stage("join.probe_ranges"):
            g = K.gather_columns([rc], rows)[0]
            vals = g.data.to(torch.int64).cpu().numpy()
            ok = np.ones(len(vals), dtype=bool)
            if g.valid is not None:
                ok &= g.valid.cpu().numpy().astype(bool)
            rows_h = rows.cpu().numpy()
            off = right.table.bucket_offsets_host
            bk = np.searchsorted(off, rows_h, side="right") - 1
            lo, hi = -(1 << (width - 1)), (1 << (width - 1)) - 1
            ok &= (vals >= lo) & (vals <= hi)
            vals, bk = vals[ok], bk[ok]
            if width == 64:
                u = (vals.view(np.uint64) ^ np.uint64(1 << 63))
            else:
                u = (vals + (1 << (width - 1))).astype(np.uint64)
            probes = np.unique(np.stack([bk.astype(np.uint64), u], axis=1), axis=0) \
                if len(u) else np.zeros((0, 2), np.uint64)
            self.last_join_probes = len(probes)
            pb = torch.from_numpy(probes[:, 0].astype(np.int32)).to(self.device)
            pk = torch.from_numpy(probes[:, 1].view(np.int64).copy()).to(self.device)
            if len(probes) == 0:
                z = torch.zeros(0, dtype=torch.int64, device=self.device)
                return z, z.clone(), torch.zeros(0, dtype=torch.int32, device=self.device)
            return K.probe_ranges(lc, left.table.bucket_offsets, pb, pk)

    def _domain_pruned_ranges(self, left: DRel, right: DRel, lk, rk):
        """Left ranges restricted to the right join key's [min, max] when that domain is
        narrower than the left's (a zone-map join filter on the sorted left key): e.g. the
        Hybrid Scan pair (index lineitem, appended orders) whose keys are disjoint costs a range
        search instead of a scan.  None when the left has its own key ranges, the shape is not
        integer / resident, or the domains do not prune."""
        if left.parts or right.parts or not left.bucketed or not left.sort_attrs:
            return None
        if self._range_spec(left, left.conds) is not None:
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.hs_transient or rc.hs_transient:
            return None
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}.get(lc.hs_type)
        if width is None or rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        llo, lspan = self._local_domain(lc)
        rlo, rspan = self._local_domain(rc)
        if lspan == 0:
            return None
        lhi, rhi = llo + lspan - 1, rlo + rspan - 1
        if rspan > 0 and rlo <= llo and rhi >= lhi:
            return None                     # the right covers the left's keys: nothing to prune
        import torch
        tmin, tmax = -(1 << (width - 1)), (1 << (width - 1)) - 1
        if rspan == 0 or rlo > min(lhi, tmax) or rhi < max(llo, tmin):
            z = torch.zeros(0, dtype=torch.int64, device=self.device)
            return z, z.clone(), torch.zeros(0, dtype=torch.int32, device=self.device)
        lo = K.sortable_image(max(rlo, tmin), lc.hs_type)
        hi = K.sortable_image(min(rhi, tmax), lc.hs_type)
        with stage("join.domain_prune"):
            return K.range_search(lc, left.table.bucket_offsets, None, lo, True, hi, True)

    # ------------------------------------------------------------------------------------------
    # Repartition (device shuffle for non-index inputs)
    # ------------------------------------------------------------------------------------------
    def _repartition(self, r: DRel, part: X.HashPartitioning) -> DRel:
        """Hash Exchange (K3) on the device: Spark-compatible Murmur3 bucket ids, then one
        (bucket, keys) sort so the result is bucketed and sorted like an index.  With several
        ranks, rows first move to their bucket's owner (the owner map, ``parallel/placement.py``) with
        RCCL all-to-all, so
        the output is co-partitioned with the index tables of the same bucket count."""
        d = self._dist()
        if not all(isinstance(e, E.Attribute) for e in part.expressions):
            raise Unsupported("hash partitioning on expressions")
        keys = list(part.expressions)
        if (r.bucketed and not r.parts and not r.split and r.num_buckets == part.num_partitions
                and [a.expr_id for a in r.bucket_attrs] == [k.expr_id for k in keys]
                and _prefix_sorted(r, keys)):
            # an index table loaded bucket-major is already hash-partitioned by these keys into
            # this many buckets (same Murmur3 + pmod) and sorted inside each bucket — the
            # exchange the planner asked for would reproduce exactly this layout
            return r
        if (d is None or d.world == 1) and not r.parts and not r.split and \
                getattr(r.table, "global_key", None) is not None:
            cached = self._repartition_cached(r, keys, part.num_partitions)
            if cached is not None:
                return cached
        cols = self._materialize(r, list(dict.fromkeys(r.attrs + keys)))
        kcols = [cols[k.expr_id] for k in keys]
        import torch
        B = part.num_partitions
        with stage("shuffle.hash"):
            bucket, counts = K.murmur3_bucket(kcols, B)
        if d is not None and d.world > 1:
            with stage("shuffle.all_to_all"):
                om = self._owner_map(B, d.world)
                k0 = kcols[0]
                if om.splits and not (routes_by_key(k0.atype) and k0.dictionary is None):
                    om = om.unsplit()       # only integer keys follow the key-range cuts
                # (a null key goes to its bucket's first piece, where the loader keeps an
                # index's nulls: they sort first)
                cols, bucket = self._exchange_rows(
                    d, cols, bucket, om.dest(bucket, k0.data if om.splits else None,
                                             k0.valid if om.splits else None))
            kcols = [cols[k.expr_id] for k in keys]
            counts = K.histogram(bucket, B)
        n = int(bucket.numel())
        with stage("shuffle.sort"):
            perm = K.sort_permutation(kcols, extra_leading=(bucket, 16))
        names = list(cols.keys())
        gathered = K.gather_columns([cols[i] for i in names], perm)
        for c in gathered:
            c.hs_transient = True       # built for this query only (not the cached repartition)
        off_host = np.concatenate([[0], np.cumsum(counts.cpu().numpy())]).astype(np.int64)
        table = DeviceTable({f"c{i}": c for i, c in zip(names, gathered)}, n,
                            torch.from_numpy(off_host).to(self.device), off_host)
        colmap = {i: f"c{i}" for i in names}
        return DRel(table, colmap, list(r.attrs), [], True, keys, keys, B)

    def _repartition_cached(self, r: DRel, keys, B: int) -> Optional[DRel]:
        """Single rank, resident source table (e.g. the appended files of a Hybrid Scan): the
        bucketed + sorted layout of the *unfiltered* rows depends only on the table, so it is
        built once and cached on the table; the query's filters stay pending on the result
        and run inside the consuming kernel.  Queries with new literals reuse the layout."""
        need = list(dict.fromkeys(list(r.attrs) + list(keys) +
                                  [a for c in r.conds for a in c.references()]))
        if any(a.expr_id not in r.colmap or r.is_computed(a) for a in need):
            return None
        names = sorted({r.colmap[a.expr_id] for a in need})
        knames = tuple(r.colmap[k.expr_id] for k in keys)
        t = r.table
        cache = t.__dict__.setdefault("_repart", {})
        ck = (tuple(names), knames, B)
        nt = cache.get(ck)
        if nt is None:
            import torch
            kcols = [t.columns[n] for n in knames]
            with stage("shuffle.hash"):
                bucket, counts = K.murmur3_bucket(kcols, B)
            with stage("shuffle.sort"):
                perm = K.sort_permutation(kcols, extra_leading=(bucket, 16))
            gathered = K.gather_columns([t.columns[n] for n in names], perm)
            off_host = np.concatenate([[0], np.cumsum(counts.cpu().numpy())]).astype(np.int64)
            nt = DeviceTable(dict(zip(names, gathered)), t.num_rows,
                             torch.from_numpy(off_host).to(self.device), off_host)
            nt.global_key = ("repartition", t.global_key, ck)
            nt._hs_sources = [t]      # current while the source table is resident
            nt._hs_cache_key = nt.global_key
            cache[ck] = nt
        colmap = {a.expr_id: r.colmap[a.expr_id] for a in need}
        return DRel(nt, colmap, list(r.attrs), list(r.conds), True, list(keys), list(keys), B)

    def _exchange_rows(self, d, cols: Dict[int, DeviceColumn], bucket, dest=None):
        """Route every row to its bucket's owner rank (``dest``, default ``bucket % world``:
        parallel/placement.py) with ONE packed all-to-all
        (``parallel/exchange.py``).  Ranks first agree on column layouts: a validity mask exists
        on every rank if it exists on any (one small all-reduce), and string dictionaries are
        unified (raw-buffer all-gather, ``parallel/dictionary.py``) with codes remapped on the
        device."""
        import torch
        from ..parallel.dictionary import remap_table, union_sorted
        from ..parallel.exchange import RowExchange
        ids = list(cols)
        need_valid = d.agree_any([cols[i].valid is not None for i in ids])
        datas, valids, dicts = [], [], []
        for j, i in enumerate(ids):
            c = cols[i]
            data = c.data
            gdict = None
            if c.dictionary is not None:
                gdict = union_sorted(c.dictionary, d)
                if len(c.dictionary) == 0:
                    data = torch.zeros_like(data)
                elif not c.dictionary.equals(gdict):
                    remap = torch.from_numpy(remap_table(c.dictionary, gdict)).to(self.device)
                    data = K.lookup_i32(remap, data)
            v = c.valid
            if need_valid[j] and v is None:
                v = torch.ones(data.shape[0], dtype=torch.uint8, device=self.device)
            datas.append(data)
            valids.append(v if need_valid[j] else None)
            dicts.append(gdict)
        send = datas + [v for v in valids if v is not None] + [bucket]
        moved = RowExchange(d, [t.dtype for t in send], self.device)
        moved.add(send, bucket, dest)
        got = moved.finish()
        out = {}
        vi = len(ids)
        for j, i in enumerate(ids):
            mv = None
            if valids[j] is not None:
                mv = got[vi]
                vi += 1
            out[i] = DeviceColumn(got[j], mv, cols[i].atype, dicts[j])
        return out, got[-1]

    # ------------------------------------------------------------------------------------------
    # Joins
    # ------------------------------------------------------------------------------------------
    JOIN_TYPES = ("inner", "left", "right", "full", "leftsemi", "leftanti")

    def _join_inputs(self, p: X.SortMergeJoinExec):
        if p.join_type not in self.JOIN_TYPES:
            raise Unsupported(f"{p.join_type} join on device")
        if not all(isinstance(k, E.Attribute) for k in list(p.left_keys) + list(p.right_keys)):
            raise Unsupported("expression join keys")
        left, right = self._rel(p.left), self._rel(p.right)
        if not (left.bucketed and right.bucketed) or left.num_buckets != right.num_buckets:
            raise Unsupported("join inputs not co-partitioned on device")
        if not _prefix_sorted(left, list(p.left_keys)):
            raise Unsupported("left not sorted by join key")
        if not _prefix_sorted(right, list(p.right_keys)):
            raise Unsupported("right not sorted by join key")
        if len(p.left_keys) > 1:
            return self._packed_join_keys(left, right, list(p.left_keys), list(p.right_keys))
        lk, rk = p.left_keys[0], p.right_keys[0]
        kinds = set()
        strings = []
        for side, k in ((left, lk), (right, rk)):
            for part in side.parts or [side]:
                c = part.col(k)
                strings.append(c.dictionary is not None)
                kinds.add(c.is_float)
        if any(strings):
            if not all(strings):
                raise Unsupported("mixed string / non-string join keys")
            left, right = self._string_join_keys(left, right, lk, rk)
        elif len(kinds) > 1:
            raise Unsupported("mixed int/float join keys")
        return left, right, lk, rk

    def _packed_join_keys(self, left: DRel, right: DRel, lks, rks):
        """Multi-column equi-join (e.g. ``(l_partkey, l_suppkey) = (ps_partkey, ps_suppkey)``):
        both sides are sorted by the key columns inside every bucket, so packing the integer
        keys into one 64-bit value — ``(k1 - lo1) << bits2 | (k2 - lo2)`` with the SAME bases
        and widths on both sides — preserves the lexicographic order and equality.  The packed
        column (null if any component is null) is cached on each table, and the single-key join
        machinery (merge join or join index) runs on it."""
        # string key components: codes into the sorted union of every part's dictionary (the
        # same remap as a single string key, _string_join_keys), so they compare across sides
        # and keep each bucket's order; then they pack like integers
        for lk, rk in zip(lks, rks):
            strs = [x.col(k).dictionary is not None
                    for side, k in ((left, lk), (right, rk)) for x in (side.parts or [side])]
            if any(strs):
                if not all(strs):
                    raise Unsupported("mixed string / non-string join keys")
                left, right = self._string_join_keys(left, right, lk, rk)
        lparts, rparts = left.parts or [left], right.parts or [right]
        lcols = [[x.col(k) for x in lparts] for k in lks]
        rcols = [[x.col(k) for x in rparts] for k in rks]
        if any(c.is_float for cs in lcols + rcols for c in cs):
            raise Unsupported("multi-key join on float keys")
        spans = []
        for lcs, rcs in zip(lcols, rcols):
            doms = [d for d in (self._local_domain(c) for c in lcs + rcs) if d[1] > 0]
            lo = min((d[0] for d in doms), default=0)
            hi = max((d[0] + d[1] - 1 for d in doms), default=0)
            # codes: 0 = null on the left, 1 = null on the right, 2 + (v - lo) = value
            spans.append((lo, max(1, int(hi - lo + 2).bit_length())))
        if sum(b for _, b in spans) > 62:
            raise Unsupported("multi-key join keys do not pack into 64 bits")
        spec = tuple(spans)
        la = E.Attribute("__hs_jkey", pa.int64(), True)
        ra = E.Attribute("__hs_jkey", pa.int64(), True)

        def pack(side, keys, code, attr):
            parts = [self._packed(x, keys, spec, code) for x in (side.parts or [side])]
            for x in parts:
                x.colmap[attr.expr_id] = "__hs_jkey"
                x.sort_attrs = [attr]
            if side.parts:
                return side.copy(parts=parts)
            return parts[0]
        return pack(left, lks, 0, la), pack(right, rks, 1, ra), la, ra

    def _packed(self, r: DRel, keys, spec, side: int) -> DRel:
        """``side`` 0/1 = the code of a null component on this side: nulls sort first within
        their prefix (the index order, NULLS FIRST) and never equal anything on the other side,
        so the packed column is sorted per bucket and needs no validity mask."""
        import torch
        t = r.table
        names = tuple(r.colmap[k.expr_id] for k in keys)
        cache = t.__dict__.setdefault("_packed_keys", {})
        nt = cache.get((names, spec, side))
        if nt is None:
            packed = torch.zeros(t.num_rows, dtype=torch.int64, device=self.device)
            for name, (lo, bits) in zip(names, spec):
                c = t.columns[name]
                code = c.data.long() - (lo - 2)
                if c.valid is not None:
                    code = torch.where(c.valid.bool(), code, torch.full_like(code, side))
                packed = (packed << bits) | code
            cols = dict(t.columns)
            cols["__hs_jkey"] = DeviceColumn(packed, None, pa.int64())
            nt = DeviceTable(cols, t.num_rows, t.bucket_offsets, t.bucket_offsets_host)
            for a in ("global_key", "_full_ranges"):
                if a in t.__dict__:
                    nt.__dict__[a] = t.__dict__[a]
            cache[(names, spec, side)] = nt
        return r.copy(table=nt, colmap=dict(r.colmap))

    def _string_join_keys(self, left: DRel, right: DRel, lk, rk):
        """Join on string keys.  Strings live in HBM as codes into per-table *sorted*
        dictionaries, so codes of different tables are not comparable — but codes into the
        sorted union of all their dictionaries are, and they keep each bucket's sort order
        (code order == string order).  Every part's key column (both sides; a Hybrid Scan side
        is a bucket union of the index and its shuffled appended rows) is remapped once (one
        int32 gather) into the union's code space; the remapped tables are cached on the
        originals, so the join index and span caches see stable tables across queries."""
        sides = [(left, lk), (right, rk)]
        dicts = []
        for side, k in sides:
            for part in side.parts or [side]:
                dicts.append(part.col(k).dictionary)
        if all(d is dicts[0] or d.equals(dicts[0]) for d in dicts[1:]):
            return left, right
        ukey = tuple(id(d) for d in dicts)
        hit = self._unions.get(ukey)
        if hit is None or any(a is not b for a, b in zip(hit[0], dicts)):
            import pyarrow.compute as pc
            union = pc.unique(pa.concat_arrays([d.cast(pa.string()) for d in dicts])).sort()
            hit = (tuple(dicts), union)
            self._unions[ukey] = hit
        union = hit[1]

        def remap(side, k):
            if side.parts:
                return side.copy(parts=[self._remapped(x, k, union) for x in side.parts])
            return self._remapped(side, k, union)
        return remap(left, lk), remap(right, rk)

    def _remapped(self, r: DRel, attr, union) -> DRel:
        import pyarrow.compute as pc
        import torch
        name = r.colmap[attr.expr_id]
        t = r.table
        cache = t.__dict__.setdefault("_remap", {})
        hit = cache.get((name, id(union)))
        if hit is None or hit[0] is not union:
            c = t.columns[name]
            pos = pc.index_in(c.dictionary.cast(pa.string()), value_set=union)
            remap = torch.from_numpy(pos.to_numpy(zero_copy_only=False).astype(np.int32)) \
                .to(self.device)
            data = remap[c.data.long()] if len(pos) else torch.zeros_like(c.data)
            cols = dict(t.columns)
            cols[name] = DeviceColumn(data, c.valid, c.atype, union)
            nt = DeviceTable(cols, t.num_rows, t.bucket_offsets, t.bucket_offsets_host)
            for a in ("global_key", "_full_ranges"):
                if a in t.__dict__:
                    nt.__dict__[a] = t.__dict__[a]
            hit = (union, nt)
            cache[(name, id(union))] = hit
        return r.copy(table=hit[1])

    def _join_params(self, left: DRel, right: DRel, lk, rk, residual, extra_attrs=(),
                     lconds=None, slots=None):
        col_info, descs = slots if slots is not None else \
            self._column_infos([(left, 0), (right, 8)])
        lslot = col_info(lk).slot
        rslot = col_info(rk).slot
        lb = CP.bind(CP.to_cnf(left.conds if lconds is None else lconds), col_info, self.device, 0)
        rconds = list(right.conds) + ([residual] if residual is not None else [])
        rb = CP.bind(CP.to_cnf(rconds), col_info, self.device, 1000)
        for a in extra_attrs:
            col_info(a)
        p = NL.JoinParams()
        preds = lb.preds + rb.preds
        if len(preds) > NL.MAX_PREDS:
            raise Unsupported("too many join predicates")
        for i, pr in enumerate(preds):
            p.preds[i] = pr
        p.nlp, p.npreds = len(lb.preds), len(preds)
        p.lkey, p.rkey = lslot, rslot
        p.key_is_float = 1 if left.col(lk).is_float else 0
        p.group_col = -1
        return p, col_info, descs, (lb, rb)

    def _join_rel(self, p: X.SortMergeJoinExec) -> DRel:
        """Row-producing co-located join: matched (left row, right row) pairs from the join
        kernels, then per join type — inner: the pairs; left/right/full outer: plus the
        unmatched rows of the preserved side(s) (rows passing that side's own filters, marked
        by a scatter of the matched ids and selected in order) padded with NULLs (gather index
        -1); left semi / anti: the left rows that do / do not appear in a pair.  Reference: the
        rule rewrites any join type (JoinIndexRule.scala:58), Spark's bucketed SortMergeJoin
        runs it."""
        left, right, lk, rk = self._join_inputs(p)
        if left.parts or right.parts:
            return self._join_rel_union(p, left, right, lk, rk)
        return self._join_rel_pair(p, left, right, lk, rk)

    def _join_rel_union(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk) -> DRel:
        """Inner join rows over BucketUnion inputs (Hybrid Scan: index buckets plus appended
        rows shuffled by the index bucket spec): an inner join distributes over union, so each
        (left part, right part) pair runs as its own co-located join and the row sets are
        concatenated; string columns whose parts carry different dictionaries are re-coded
        over the union of the dictionaries."""
        out_attrs = list(p.output)
        if p.join_type == "inner":
            pieces = [self._join_rel_pair(p, lp, rp, lk, rk)
                      for lp in (left.parts or [left]) for rp in (right.parts or [right])]
            return self._concat_rels([[x.col(a) for a in out_attrs] for x in pieces], out_attrs)
        return self._join_rel_parts_outer(p, left.parts or [left], right.parts or [right],
                                          lk, rk)

    def _join_rel_parts_outer(self, p: X.SortMergeJoinExec, lparts, rparts, lk, rk) -> DRel:
        """Outer / semi / anti join rows over BucketUnion parts (Hybrid Scan of either side): the
        matched pairs of every (left part, right part) pair, and a row of a preserved side is
        unmatched only if NO part of the other side matched it - its match marks are OR-ed over
        the other side's parts before the unmatched rows (passing the row's own side filters)
        are selected and padded with NULLs.  Same rows as the join of the unions
        (JoinIndexRule.scala:57-58 rewrites any join type; RuleUtils.scala:439-441 puts the
        BucketUnion under it)."""
        import torch
        jt = p.join_type
        out_attrs = list(p.output)
        lset = {a.expr_id for a in p.left.output}
        lattrs = [a for a in out_attrs if a.expr_id in lset]
        rattrs = [a for a in out_attrs if a.expr_id not in lset]
        inner = X.SortMergeJoinExec(p.left_keys, p.right_keys, "inner", p.condition, p.left,
                                    p.right)
        lmarks: List = [None] * len(lparts)
        rmarks: List = [None] * len(rparts)
        pieces = []
        for i, lp in enumerate(lparts):
            for j, rp in enumerate(rparts):
                ol, orr = self._pair_rows(inner, lp, rp, lk, rk)
                if jt in ("left", "full", "leftsemi", "leftanti"):
                    m = K.mark_rows(ol, int(lp.table.num_rows or 0))
                    lmarks[i] = m if lmarks[i] is None else torch.maximum(lmarks[i], m)
                if jt in ("right", "full"):
                    m = K.mark_rows(orr, int(rp.table.num_rows or 0))
                    rmarks[j] = m if rmarks[j] is None else torch.maximum(rmarks[j], m)
                if jt in ("left", "right", "full"):
                    lg = K.gather_columns([lp.col(a) for a in lattrs], ol)
                    rg = K.gather_columns([rp.col(a) for a in rattrs], orr)
                    pieces.append(lg + rg)
        ncols = len(rattrs)
        for i, lp in enumerate(lparts):
            if jt not in ("left", "full", "leftsemi", "leftanti"):
                break
            sel = self._selected_rows(lp)
            want = 1 if jt == "leftsemi" else 0
            rows = K.select_marked(sel, lmarks[i], want)
            lg = K.gather_columns([lp.col(a) for a in lattrs], rows)
            if jt in ("leftsemi", "leftanti"):
                pieces.append(lg)
                continue
            pad = torch.full_like(rows, -1)
            rg = K.gather_columns([rparts[0].col(a) for a in rattrs], pad, padded=True) \
                if ncols else []
            pieces.append(lg + rg)
        if jt in ("right", "full"):
            for j, rp in enumerate(rparts):
                sel = self._selected_rows(rp)
                rows = K.select_marked(sel, rmarks[j], 0)
                pad = torch.full_like(rows, -1)
                lg = K.gather_columns([lparts[0].col(a) for a in lattrs], pad, padded=True) \
                    if lattrs else []
                rg = K.gather_columns([rp.col(a) for a in rattrs], rows)
                pieces.append(lg + rg)
        attrs = lattrs + rattrs if jt not in ("leftsemi", "leftanti") else lattrs
        rel = self._concat_rels(pieces, attrs)
        if [a.expr_id for a in attrs] != [a.expr_id for a in out_attrs]:
            rel.attrs = out_attrs
        return rel

    def _pair_rows(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk):
        """(left row ids, right row ids) of the inner join pairs of one part pair (each side's
        own predicates applied, the join condition evaluated)."""
        import torch
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, p.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        for s_, c in descs.items():
            jp.cols[s_] = c.desc()
        if keep[0].always_false or keep[1].always_false:
            e = torch.empty(0, dtype=torch.int64, device=self.device)
            return e, e
        max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
        return K.join_pairs(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)

    def _concat_rels(self, pieces: List[List[DeviceColumn]], out_attrs) -> DRel:
        """One flat device relation over ``out_attrs`` from row sets ``pieces`` (per piece the
        columns in ``out_attrs`` order); string columns with different dictionaries are
        re-coded over their union."""
        import torch
        from ..parallel.dictionary import remap_table
        cols = {}
        for ai, a in enumerate(out_attrs):
            cs = [x[ai] for x in pieces]
            dicts = [c.dictionary for c in cs]
            gd = None
            if any(d is not None for d in dicts):
                gd = dicts[0]
                if not all(d is not None and d.equals(gd) for d in dicts):
                    import pyarrow.compute as pc
                    allv = pa.concat_arrays([d.cast(pa.string()) for d in dicts if d is not None])
                    gd = pc.unique(allv).sort()
            datas = []
            for c in cs:
                d = c.data
                if gd is not None and c.dictionary is not None and not c.dictionary.equals(gd) \
                        and d.numel():
                    tab = torch.from_numpy(remap_table(c.dictionary, gd)).to(self.device)
                    d = K.lookup_i32(tab, d)
                datas.append(d)
            valid = None
            if any(c.valid is not None for c in cs):
                valid = torch.cat([c.valid if c.valid is not None else
                                   torch.ones(c.data.numel(), dtype=torch.uint8,
                                              device=self.device) for c in cs])
            col = DeviceColumn(torch.cat(datas), valid, cs[0].atype, gd)
            col.hs_transient = True
            cols[key(a)] = col
        n = sum(int(x[0].data.numel()) for x in pieces) if out_attrs else 0
        off = np.array([0, n], dtype=np.int64)
        table = DeviceTable(cols, n, torch.from_numpy(off).to(self.device), off)
        return DRel(table, {a.expr_id: key(a) for a in out_attrs}, out_attrs)

    def _join_rel_pair(self, p: X.SortMergeJoinExec, left: DRel, right: DRel, lk, rk) -> DRel:
        jt = p.join_type
        out_attrs = list(p.output)
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk) if jt in ("inner", "leftsemi") else None
        if probed is None and jt in ("inner", "leftsemi", "right"):
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            with stage("join.ranges"):
                rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, p.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        if keep[0].always_false or keep[1].always_false:
            import torch
            ol = orr = torch.empty(0, dtype=torch.int64, device=self.device)
        else:
            max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
            ol, orr = K.join_pairs(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)
        lset = {a.expr_id for a in p.left.output}
        lattrs = [a for a in out_attrs if a.expr_id in lset]
        rattrs = [a for a in out_attrs if a.expr_id not in lset]
        padded = jt in ("left", "right", "full")
        if jt != "inner":
            import torch
            with stage("join.outer_rows"):
                if jt in ("left", "full", "leftsemi", "leftanti"):
                    lsel = self._selected_rows(left)
                    lmark = K.mark_rows(ol, int(left.table.num_rows or 0))
                if jt in ("leftsemi", "leftanti"):
                    ol = K.select_marked(lsel, lmark, 1 if jt == "leftsemi" else 0)
                    orr = ol[:0]
                    rattrs = []
                else:
                    extra_l, extra_r = [], []
                    if jt in ("left", "full"):
                        um = K.select_marked(lsel, lmark, 0)
                        extra_l.append(um)
                        extra_r.append(torch.full_like(um, -1))
                    if jt in ("right", "full"):
                        rsel = self._selected_rows(right)
                        rmark = K.mark_rows(orr, int(right.table.num_rows or 0))
                        um = K.select_marked(rsel, rmark, 0)
                        extra_l.append(torch.full_like(um, -1))
                        extra_r.append(um)
                    ol = torch.cat([ol] + extra_l)
                    orr = torch.cat([orr] + extra_r)
        lg = K.gather_columns([left.col(a) for a in lattrs], ol,
                              padded=padded and jt in ("right", "full"))
        rg = K.gather_columns([right.col(a) for a in rattrs], orr,
                              padded=padded and jt in ("left", "full"))
        cols = {}
        for a, c in list(zip(lattrs, lg)) + list(zip(rattrs, rg)):
            c.hs_transient = True
            cols[key(a)] = c
        n = int(ol.numel())
        import torch
        off = np.array([0, n], dtype=np.int64)
        table = DeviceTable(cols, n, torch.from_numpy(off).to(self.device), off)
        return DRel(table, {a.expr_id: key(a) for a in out_attrs}, out_attrs)

    def _join_agg(self, node: X.SortMergeJoinExec, fns, group):
        """Fused join + aggregate.  A side that is a BucketUnion (Hybrid Scan: index buckets plus
        appended rows shuffled by the index bucket spec) is a list of co-partitioned sorted parts;
        an inner join distributes over union, so every (left part, right part) pair runs as its
        own co-located join and the partial aggregates combine — the index side is never
        re-sorted together with the appended rows."""
        left, right, lk, rk = self._join_inputs(node)
        lparts, rparts = left.parts or [left], right.parts or [right]
        gs = (None, 1, 0, None, None)
        if group is not None:
            side = lparts if any(group.expr_id in x.colmap for x in lparts) else rparts
            gs = self._group_spec_parts(side, group, _group_limit(MAX_GROUPS_JOIN, GROUP_LDS_JOIN,
                                                                  len(fns)))
            if gs is None:
                return (*self._empty_agg(len(fns) + 1), 1, 0, None, None)
        agreed, G, gbase, gdict, gtype = gs
        self._groups_agreed = agreed is True
        out = None
        for lp in lparts:
            for rp in rparts:
                part = self._join_agg_pair(node, lp, rp, lk, rk, fns, group, G, gbase)
                out = part if out is None else _combine_aggs(out, part)
        if len(lparts) * len(rparts) > 1:
            self._join_rec = None       # a bucket union: no single replayable launch
        return (*out, G, gbase, gdict, gtype)

    def _group_spec_parts(self, parts, group, limit):
        specs = [self._group_spec(x, group, limit) for x in parts if group.expr_id in x.colmap]
        specs = [s for s in specs if s is not None]
        if not specs:
            return None
        if len(specs) == 1:
            return specs[0]
        if any(s[3] is not None for s in specs):
            raise _NeedHash("string group key over a bucket union")
        lo = min(s[2] for s in specs)
        hi = max(s[2] + s[1] for s in specs)
        if hi - lo > limit:
            raise _NeedHash("group domain too large for LDS aggregation")
        return (True if all(s[0] is True for s in specs) else None), hi - lo, lo, None, specs[0][4]

    def _run_match_ok(self, jp, left: DRel, right: DRel, rk, descs, rstart) -> bool:
        """Whether this join takes the run-keyed two-phase form over the left table's full
        ranges with unique right keys - the form whose launcher can keep its key match
        (``jit_runs.TwoPhaseLauncher._record``) when join indexes are enabled."""
        from . import jit_join, jit_runs
        if not HyperspaceConf.codegen_enabled(self.session.conf) or not jit_runs.RT2_MATCH:
            return False
        fr = getattr(left.table, "_full_ranges", None)
        if fr is None or rstart is not fr[0] or jit.key_has_dups(right.col(rk)):
            return False
        comp = self._compacts(descs)
        if not jit.merge_join_ok(jp, comp, right.table.num_rows, left.table.num_rows) or \
                not jit_runs.applies(jp):
            return False
        return jit_join._with_runs(jp, comp)[1] is not None

    def _join_agg_pair(self, node, left: DRel, right: DRel, lk, rk, fns, group, G, gbase):
        # drive the kernel from a much smaller side (the appended part of a hybrid scan).  Only
        # then: one work item per driving row is cheapest when each finds few matches, so a
        # many-to-one pair like lineitem⋈orders (4:1) keeps the many side driving — swapping it
        # made TPC-H Q3 2.5x slower on MI355X (profiles/bench_sf100_r1_v5.json)
        if right.table.num_rows * 64 < left.table.num_rows:
            left, right, lk, rk = right, left, rk, lk
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, node.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        specs = self._agg_specs(fns, col_info)
        if group is not None:
            col_info(group)
            jp.group_col = col_info(group).slot if G > 1 else -1
            jp.num_groups, jp.group_base = G, gbase
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        for i, a in enumerate(specs):
            jp.aggs[i] = a
        jp.naggs = len(specs)
        if keep[0].always_false or keep[1].always_false or left.table.num_rows == 0 or \
                right.table.num_rows == 0:
            return self._empty_agg(len(specs), G)
        max_tiles = K.join_max_tiles(left.table.num_rows, rlen.numel())
        conf = self.session.conf
        jindex = HyperspaceConf.join_index_enabled(conf)
        if jindex and self._run_match_ok(jp, left, right, rk, descs, rstart):
            # a unique-key run-keyed join keeps its key match in run form instead (the two-phase
            # launcher records it on its second launch): the faster join index
            jindex = False
        if HyperspaceConf.codegen_enabled(conf) and jindex and \
                not getattr(self, "_merge_join_only", False) and \
                getattr(left.table, "global_key", None) is not None and \
                getattr(right.table, "global_key", None) is not None and \
                join_index.eligible(left.table, right.table, left.col(lk), right.col(rk)):
            # both sides are resident index tables: join through the cached join index
            with stage("join.index"):
                fs, fl, fb = self._full_ranges(left.table)
                jidx = join_index.get_join_index(jp, left.table, right.table, left.col(lk),
                                                 right.col(rk), fs, fl, fb)
            with stage("join.index_agg_kernel"):
                return jit.join_index_agg(jp, rstart, rlen, jidx, self._compacts(descs),
                                          nrows=left.table.num_rows,
                                          rnrows=right.table.num_rows)
        with stage("join.agg_kernel"):
            if HyperspaceConf.codegen_enabled(self.session.conf):
                fr = getattr(left.table, "_full_ranges", None)
                comp = self._compacts(descs)
                if jit.merge_join_ok(jp, comp, right.table.num_rows, left.table.num_rows):
                    jit.LAST_MJ_LAUNCHER[0] = None
                    out = jit.merge_join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets,
                                             comp, nrows=left.table.num_rows,
                                             cache_spans=fr is not None and rstart is fr[0],
                                             rdup=jit.key_has_dups(right.col(rk)),
                                             record=HyperspaceConf.join_index_enabled(conf))
                    if fr is not None and rstart is fr[0] and probed is None:
                        # full ranges, no probing: the launch can be replayed for this pair
                        # (``implied`` then holds only isnotnull(key) conjuncts the full ranges
                        # satisfy; the replay binds the same left conjuncts as this launch)
                        self._join_rec = (left, right, lk, rk, col_info, descs,
                                          jit.LAST_MJ_LAUNCHER[0], specs,
                                          [c for c in left.conds if id(c) not in implied])
                    return out
                return jit.join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles,
                                    self._compacts(descs),
                                    cache_spans=fr is not None and rstart is fr[0])
            return K.join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, max_tiles)
