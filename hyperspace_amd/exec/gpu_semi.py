"""Semi-joins of a non-co-partitioned build side: key bitmaps (exchanged as keys or bitmaps
across ranks), the probe's run-form walk, projection semi-joins, and the co-partitioned
rewrite of a (customer x orders) build onto an orders-key index."""
from __future__ import annotations

from typing import Optional

import pyarrow as pa

from ..index import constants as C
from ..ops import _lib as NL, kernels as K
from ..plan import expressions as E, physical as X
from ..utils.conf import HyperspaceConf
from ..utils.tracing import stage
from . import compile as CP, jit, jit_runs
from .arrow_eval import key
from .device_table import DeviceColumn
from .gpu_common import (_group_limit, _NoCondition, _plan_bytes, _semi_fail_key, _strip_exchange,
                         DRel, GROUP_LDS_JOIN, GROUP_LDS_SCAN, MAX_GROUPS_JOIN, MAX_GROUPS_SCAN)


class SemiJoinOps:
    """Semi-join operators of ``GpuBackend`` (exec/gpu.py)."""

    # ------------------------------------------------------------------------------------------
    # Semi-join through a key-domain bitmap (csrc/kernels/key_bitmap.hip)
    # ------------------------------------------------------------------------------------------
    def _semi_join_agg(self, node: X.SortMergeJoinExec, fns, group):
        """An inner equi-join whose aggregate reads only one side (the probe) and whose other
        side (the build) needs an Exchange - it is not co-partitioned with the probe, e.g. the
        output of another join (TPC-H Q3: (customer x orders) x lineitem; JoinIndexRule cannot
        rewrite a join whose side is a join, JoinIndexRule.scala:100-105,149-150) - runs as a
        scan of the probe side filtered by a bitmap of the build keys, when those keys are
        unique (then the join matches each probe row at most once and multiplies nothing).
        That replaces the Exchange + Sort of both sides and the merge join.  None when the
        shape does not qualify (or the build keys repeat): the general join runs instead."""
        if node.condition is not None or len(node.left_keys) != 1:
            return None
        conf = self.session.conf
        if not HyperspaceConf.codegen_enabled(conf) or \
                str(conf.get("spark.hyperspace.mi.semiJoinBitmap.enabled", "true")).lower() != "true":
            return None
        failed = self.__dict__.setdefault("_semi_failed", {})
        fkey = _semi_fail_key(node)
        if failed.get(fkey) is node:
            return None
        need = set()
        for fn in fns:
            need.update(a.expr_id for a in fn.references())
        if group is not None:
            need.add(group.expr_id)
        lk, rk = node.left_keys[0], node.right_keys[0]
        if not (isinstance(lk, E.Attribute) and isinstance(rk, E.Attribute)):
            return None
        sides = []
        for probe, build, pk, bk in ((node.right, node.left, rk, lk), (node.left, node.right, lk, rk)):
            if not need <= {a.expr_id for a in probe.output}:
                continue
            binner = _strip_exchange(build)
            if binner is None:
                continue
            sides.append((_plan_bytes(build), probe, binner, pk, bk))
        if not sides:
            return None
        _, probe, binner, pk, bk = min(sides, key=lambda x: x[0])
        if not all(pa.types.is_integer(a.data_type) for a in (pk, bk)):
            return None
        pinner = _strip_exchange(probe) or probe
        out = self._copart_semi(pinner, pk, binner, bk, fns, group)
        if out is not None:
            return out
        with stage("semi.build"):
            brel = self._rel(binner)
            if brel.parts:
                return None
            keys = self._materialize(brel, [bk])[bk.expr_id]
            bm = self._semi_bitmap(keys)
        if bm is None:
            if len(failed) > 256:
                failed.clear()
            failed[fkey] = node
            return None
        words, lo, nbits = bm
        prel = self._rel(pinner)
        if prel.parts:
            return None
        cond = CP.KeyBitmap(pk, words, lo, nbits)
        self.last_semi_join = {"build_keys": int(keys.data.numel()), "bitmap_bits": nbits,
                               "probe": "scan"}
        with stage("semi.probe"):
            out = self._semi_runs(prel, pk, words, lo, nbits, fns, group)
            if out is not None:
                self.last_semi_join["probe"] = "runs"
                return out
            return self._scan_agg(prel.copy(conds=prel.conds + [cond]), fns, group)

    def _copart_semi(self, pinner, pk, binner, bk, fns, group):
        """The semi-join's build as a co-partitioned join: a build ``Project/Filter <- inner
        join(orders side, customer side)`` whose kept key ``bk`` comes from the orders side
        (TPC-H Q3: ``(customer x orders) x lineitem``), when another index over the same orders
        files is bucketed by ``bk`` like the probe index is by ``pk`` and covers the orders
        side's columns.  Then the probe joins that index bucket by bucket - the two-phase
        run-keyed merge join of ``_join_agg_pair`` - with the orders side's own filters plus
        ``o_custkey`` in a bitmap of the (unique) customer keys as right-side predicates: one
        small bitmap (the customer key domain, L2-resident) instead of the orders-key bitmap
        (75 MB at SF100, probed at random) and no all-gather of it across ranks.  An inner join
        with unique customer keys pairs every passing orders row with exactly one customer, so
        ``(C x O) x L = L x (O where o_custkey in C)``.  None when the shape or the indexes do
        not qualify."""
        conf = self.session.conf
        if str(conf.get("spark.hyperspace.mi.coPartitionedSemiJoin.enabled", "true")).lower() \
                != "true" or not HyperspaceConf.codegen_enabled(conf):
            return None
        above, node = [], binner
        while isinstance(node, (X.ProjectExec, X.FilterExec)):
            if isinstance(node, X.ProjectExec) and \
                    not all(isinstance(e, E.Attribute) for e in node.project_list):
                return None
            above.append(node)
            node = node.child
        if not (isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner" and
                node.condition is None and len(node.left_keys) == 1):
            return None
        pick = None
        for o, c, ok, ck in ((node.left, node.right, node.left_keys[0], node.right_keys[0]),
                             (node.right, node.left, node.right_keys[0], node.left_keys[0])):
            if any(a.expr_id == bk.expr_id for a in o.output):
                pick = (o, c, ok, ck)
        if pick is None:
            return None
        oside, cside, ojk, cjk = pick
        if not all(isinstance(k, E.Attribute) and pa.types.is_integer(k.data_type)
                   for k in (ojk, cjk)):
            return None
        oids = {a.expr_id for a in oside.output}
        upper = [f for f in above if isinstance(f, X.FilterExec)]
        if any(not {a.expr_id for a in f.condition.references()} <= oids for f in upper):
            return None
        chain, leaf = [], _strip_exchange(oside) or oside
        while isinstance(leaf, (X.ProjectExec, X.FilterExec)):
            chain.append(leaf)
            leaf = leaf.child
        if not isinstance(leaf, X.FileSourceScanExec) or not leaf.relation.is_index():
            return None
        ascan = self._copart_scan(leaf, bk, pinner)
        if ascan is None:
            return None
        prel = self._rel(pinner)
        if prel.parts or not prel.bucketed or prel.num_buckets != ascan.relation.index.num_buckets \
                or not prel.sort_attrs or prel.sort_attrs[0].expr_id != pk.expr_id or \
                pk.data_type != bk.data_type:
            return None
        gs = (None, 1, 0, None, None)
        if group is not None:
            if group.expr_id not in prel.colmap:
                return None
            gs = self._group_spec(prel, group, _group_limit(MAX_GROUPS_JOIN, GROUP_LDS_JOIN,
                                                            len(fns)))
            if gs is None:
                return (*self._empty_agg(len(fns) + 1), 1, 0, None, None)
        with stage("semi.build"):
            crel = self._rel(_strip_exchange(cside) or cside)
            if crel.parts:
                return None
            src = crel.col(cjk) if crel.bucketed and crel.sort_attrs and \
                crel.sort_attrs[0].expr_id == cjk.expr_id and not crel.is_computed(cjk) else None
            bm = self._filtered_bitmap(crel, cjk, src)
            nkeys = None
            if bm is None:
                keys = self._materialize(crel, [cjk])[cjk.expr_id]
                nkeys = int(keys.data.numel())
                bm = self._semi_bitmap(keys, src)
        if bm is None:
            return None
        words, lo, nbits = bm
        orel = self._scan_memo(ascan)
        for n in reversed(chain):
            orel = self._unary(n, orel)
        for f in reversed(upper):
            orel = self._unary(f, orel)
        orel = orel.copy(conds=orel.conds + [CP.KeyBitmap(ojk, words, lo, nbits)])
        self.last_semi_join = {"build_keys": nkeys, "bitmap_bits": nbits, "probe": "copart",
                               "index": ascan.relation.index.name,
                               "build": "materialized" if nkeys is not None else "fused"}
        agreed, G, gbase, gdict, gtype = gs
        self._groups_agreed = agreed is True
        self._join_rec = None
        # the two-phase run-keyed merge join tests the orders predicates once per lineitem key
        # run; a join index would gather o_custkey per lineitem row (at random)
        self._merge_join_only = True
        try:
            with stage("semi.probe"):
                out = self._join_agg_pair(_NoCondition, prel, orel, pk, bk, fns, group, G, gbase)
        finally:
            self._merge_join_only = False
        self._join_rec = None
        return (*out, G, gbase, gdict, gtype)

    def _copart_scan(self, scan: X.FileSourceScanExec, key, pinner):
        """A scan of an index over the same source files as ``scan``'s index, bucketed by
        ``key`` alone with the probe index's bucket count and holding every column ``scan``
        outputs (``_copart_semi``); the scan node is kept per (scan, index) so the device
        cache and scan memo see one node.  None when no index qualifies."""
        from ..hyperspace import get_context
        from ..actions import states
        from ..rules import rule_utils as RU
        from ..index import tags as T
        from ..plan import logical as L
        idx = scan.relation.index
        probe_scans = pinner.collect(lambda x: isinstance(x, X.FileSourceScanExec))
        if len(probe_scans) != 1 or not probe_scans[0].relation.is_index():
            return None
        nb = probe_scans[0].relation.index.num_buckets
        names = {a.name.lower() for a in scan.output}
        if C.DATA_FILE_NAME_ID.lower() in names:
            return None        # lineage ids are per index: a hybrid-scan delete filter stays
        found = None
        for e in get_context(self.session).index_collection_manager.get_indexes([states.ACTIVE]):
            if e.name == idx.name or e.num_buckets != nb or \
                    [c.lower() for c in e.indexed_columns] != [key.name.lower()] or \
                    not names <= {n.lower() for n in e.schema.names} or \
                    e.source_file_info_set != idx.source_file_info_set:
                continue
            found = e
            break
        if found is None:
            return None
        memo = self.__dict__.setdefault("_copart_scans", {})
        mk = (id(scan), found.name)
        hit = memo.get(mk)
        if hit is not None and hit[0] is scan and hit[1] is found:
            return hit[2]
        loc = found.with_cached_tag(None, T.INMEMORYFILEINDEX_INDEX_ONLY,
                                    lambda: RU._index_file_index(found))
        k, v = C.INDEX_RELATION_IDENTIFIER
        schema = pa.schema([f for f in found.schema if f.name != C.DATA_FILE_NAME_ID])
        rel = L.HadoopFsRelation(loc, None, schema, found.bucket_spec, "parquet", {k: v},
                                 index=found)
        ascan = X.FileSourceScanExec(rel, list(scan.output), [], [], True)
        if len(memo) > 64:
            memo.clear()
        memo[mk] = (scan, found, ascan)
        return ascan

    def _semi_runs(self, r: DRel, key, words, lo: int, nbits: int, fns, group):
        """The semi-join probe over the probe key's run form (``jit_runs.semi_runs_agg``): a
        resident index relation sorted by the key (an index's bucket-sorted indexed column, so
        its rows form runs of equal keys) tests the build bitmap once per run and scans its
        own predicates and aggregates bit-parallel.  None when the shape does not qualify (the
        plain scan with a per-row bitmap predicate runs instead)."""
        conf = self.session.conf
        if not (jit_runs.RS_BITS and HyperspaceConf.codegen_enabled(conf)) or \
                str(conf.get("spark.hyperspace.mi.semiRuns.enabled", "true")).lower() != "true":
            return None
        if r.table is None or r.parts or r.extra or r.split or not r.bucketed or \
                not r.sort_attrs or r.sort_attrs[0].expr_id != key.expr_id:
            return None
        col_info, descs = self._column_infos([(r, 0)])
        kslot = col_info(key).slot
        implied: set = set()
        spec = self._range_spec(r, r.conds, implied)
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        specs = self._agg_specs(fns, col_info)
        gs = self._group_spec(r, group, _group_limit(MAX_GROUPS_SCAN, GROUP_LDS_SCAN, len(fns)))
        if gs is None:
            return None
        agreed, G, gbase, gdict, gtype = gs
        gslot = col_info(group).slot if (group is not None and G > 1) else -1
        if any(sl >= jit_runs.SPLIT for sl in descs) or len(bound.preds) > NL.MAX_PREDS:
            return None
        comp = self._compacts(descs)
        if not comp or kslot not in comp or r.col(key).valid is not None:
            return None
        from .encoding import key_runs
        runs = key_runs(comp[kslot])
        if runs is None:
            return None
        comp = dict(comp)
        comp[kslot] = runs
        rstart, rlen, _ = self._ranges(r, r.conds) if spec is not None else \
            self._full_ranges(r.table)
        self._groups_agreed = agreed is True
        if bound.always_false:
            return (*self._empty_agg(len(specs), G), G, gbase, gdict, gtype)
        p = NL.JoinParams()
        for s_, c in descs.items():
            p.cols[s_] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.nlp = p.npreds = len(bound.preds)
        for i, a in enumerate(specs):
            p.aggs[i] = a
        p.naggs = len(specs)
        p.lkey, p.rkey, p.key_is_float = kslot, kslot, 0
        p.group_col, p.num_groups, p.group_base = gslot, G, gbase
        out = jit_runs.semi_runs_agg(p, rstart, rlen, comp, runs, r.table.num_rows, words, lo,
                                     nbits)
        return (*out, G, gbase, gdict, gtype)

    def _semi_project(self, p: X.ProjectExec) -> Optional[DRel]:
        """``Project <- Filter* <- inner join`` whose projection and filters read one side only:
        that side filtered by a bitmap of the other side's (unique) keys - a semi-join, no
        row pairs materialized (TPC-H Q3's customer x orders feeding the lineitem join).  None
        when the shape does not qualify or the other side's keys repeat."""
        filters, node = [], p.child
        while isinstance(node, X.FilterExec):
            filters.append(node)
            node = node.child
        if not (isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner" and
                node.condition is None and len(node.left_keys) == 1):
            return None
        conf = self.session.conf
        if not HyperspaceConf.codegen_enabled(conf) or \
                str(conf.get("spark.hyperspace.mi.semiJoinBitmap.enabled", "true")).lower() != "true" \
                or str(conf.get("spark.hyperspace.mi.semiProject.enabled", "true")).lower() != "true":
            return None
        failed = self.__dict__.setdefault("_semi_failed", {})
        fkey = _semi_fail_key(node)
        if failed.get(fkey) is node:
            return None
        need = set()
        for e in p.project_list:
            need.update(a.expr_id for a in e.references())
        for f in filters:
            need.update(a.expr_id for a in f.condition.references())
        lk, rk = node.left_keys[0], node.right_keys[0]
        if not (isinstance(lk, E.Attribute) and isinstance(rk, E.Attribute)) or \
                not all(pa.types.is_integer(a.data_type) for a in (lk, rk)):
            return None
        cands = []
        for probe, build, pk, bk in ((node.right, node.left, rk, lk),
                                     (node.left, node.right, lk, rk)):
            if need <= {a.expr_id for a in probe.output}:
                cands.append((_plan_bytes(build), probe, build, pk, bk))
        if not cands:
            return None
        _, probe, build, pk, bk = min(cands, key=lambda x: x[0])
        binner = _strip_exchange(build) or build
        pinner = _strip_exchange(probe) or probe
        with stage("semi.build"):
            brel = self._rel(binner)
            if brel.parts:
                return None
            keys = self._materialize(brel, [bk])[bk.expr_id]
            bm = self._semi_bitmap(keys)
        if bm is None:
            if len(failed) > 256:
                failed.clear()
            failed[fkey] = node
            return None
        words, lo, nbits = bm
        r = self._rel(pinner)
        if r.parts:
            return None
        r = r.copy(conds=r.conds + [CP.KeyBitmap(pk, words, lo, nbits)])
        for f in reversed(filters):
            r = self._unary(f, r)
        return self._unary(p, r)

    def _filtered_bitmap(self, r: DRel, key: E.Attribute, src: Optional[DeviceColumn]):
        """(words, lo, nbits) of the keys of ``r``'s rows passing its predicates, built by one
        filter-to-bitmap launch (``K.scan_bitmap``) - no selected-row materialization, so no
        host synchronization - when ``src`` is the resident, sorted index key column those rows
        come from, single rank, with a cached domain that fits the bitmap and no repeated key
        (then every selection of it is unique too).  None when that does not hold (the
        materializing path runs)."""
        d = self._dist()
        if (d is not None and d.world > 1) or src is None or src.valid is not None or \
                getattr(src, "hs_transient", False) or \
                src.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64) or r.table is None or \
                r.split or r.extra or jit.key_has_dups(src):
            return None
        lo, span = self._local_domain(src)
        if span == 0 or span > K.MAX_BITMAP_BITS:
            return None
        implied: set = set()
        rstart, rlen, _ = self._ranges(r, r.conds, implied)
        col_info, descs = self._column_infos([(r, 0)])
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        kslot = col_info(key).slot
        if len(bound.preds) > NL.MAX_PREDS:
            return None
        if bound.always_false:
            import torch
            return torch.zeros(max((span + 63) // 64, 1), dtype=torch.int64,
                               device=self.device), lo, span
        p = NL.ScanParams()
        for s_, c in descs.items():
            p.cols[s_] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.npreds = len(bound.preds)
        p.naggs, p.group_col = 0, -1
        words = K.scan_bitmap(p, rstart, rlen, K.ranges_to_tiles(rlen), kslot, lo, span)
        return words, lo, span

    def _semi_bitmap(self, keys: DeviceColumn, src: Optional[DeviceColumn] = None):
        """(words, lo, nbits) of the build keys over every rank's keys, or None when they are
        not unique, not integer, empty everywhere or span more than K.MAX_BITMAP_BITS.
        ``src``: the resident, sorted index key column the keys were selected from - its
        (cached) domain bounds them and, when it repeats no key, so is every selection of it:
        the bitmap is built with no host synchronization."""
        import torch
        d = self._dist()
        if (d is None or d.world == 1) and src is not None and src.valid is None and \
                not getattr(src, "hs_transient", False) and \
                src.hs_type in (NL.I8, NL.I16, NL.I32, NL.I64) and not jit.key_has_dups(src):
            lo, span = self._local_domain(src)
            if span == 0 or span > K.MAX_BITMAP_BITS:
                return None
            words, _ = K.key_bitmap(keys, lo, span, check=False)
            return words, lo, span
        dom = K.key_domain(keys)
        if d is None or d.world == 1:
            if dom is None:
                return None
            lo, hi, n = dom
            if hi - lo + 1 > K.MAX_BITMAP_BITS:
                return None
            words, dup = K.key_bitmap(keys, lo, hi - lo + 1)
            return None if dup else (words, lo, hi - lo + 1)
        # every rank: every rank's (lo, hi, count) in one small all-gather, then whichever
        # moves fewer bytes over xGMI: the keys themselves (32-bit offsets from the global low
        # key when the domain allows; every rank builds the whole bitmap and checks uniqueness
        # itself), or each rank's bitmap of its own keys, OR-ed, with a uniqueness check by
        # population count.  Every rank sees the same counts and the same "any rank's keys carry
        # a validity mask" flag (a rank materializes one only when its split has nulls), so all
        # take the same branch - the keys route ships raw values, so it needs no nulls anywhere.
        from ..parallel.gather import _all_gather_flat
        big = 1 << 62
        lo, hi, n = dom if dom is not None else (big, -big, 0)
        cdev = d.device if d.backend == "nccl" else torch.device("cpu")
        info = torch.tensor([lo, hi, n, int(keys.valid is not None)], dtype=torch.int64,
                            device=cdev)
        allinfo = _all_gather_flat(d, info).view(d.world, 4).cpu().numpy()
        any_valid = bool(allinfo[:, 3].any())
        allinfo = allinfo[:, :3]
        ns = allinfo[:, 2]
        gn = int(ns.sum())
        if gn == 0:
            return None
        live = allinfo[ns > 0]
        glo, ghi = int(live[:, 0].min()), int(live[:, 1].max())
        if ghi - glo + 1 > K.MAX_BITMAP_BITS:
            return None
        nbits = ghi - glo + 1
        wide = nbits > (1 << 31) - 1
        key_bytes = gn * (8 if wide else 4)
        bitmap_bytes = (d.world - 1) * ((nbits + 63) // 64) * 8
        self.last_semi_exchange = "keys" if key_bytes < bitmap_bytes and not any_valid else \
            "bitmap"
        if key_bytes < bitmap_bytes and not any_valid:
            nmax = int(ns.max())
            dt = torch.int64 if wide else torch.int32
            buf = torch.zeros(nmax, dtype=dt, device=self.device)
            if n:
                buf[:n] = (keys.data.long() - glo).to(dt)
            allk = d.all_gather_tensor(buf).view(d.world, nmax)
            cat = torch.cat([allk[r, :int(ns[r])] for r in range(d.world) if ns[r]])
            words, dup = K.key_bitmap(DeviceColumn(cat, None, pa.int64() if wide else pa.int32()),
                                      0, nbits)
            return None if dup else (words, glo, nbits)
        self.last_semi_exchange = "bitmap"
        if dom is not None:
            words, _ = K.key_bitmap(keys, glo, nbits)
        else:
            words = torch.zeros((nbits + 63) // 64, dtype=torch.int64, device=self.device)
        allw = d.all_gather_tensor(words).view(d.world, -1)
        words = allw[0].clone()
        for r in range(1, d.world):
            words.bitwise_or_(allw[r])
        if K.bitmap_popcount(words) != gn:
            return None
        return words, glo, nbits
