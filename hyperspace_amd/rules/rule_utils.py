"""Candidate selection, index plan rewrite and Hybrid Scan (reference
``index/rules/RuleUtils.scala:37-579``)."""
from __future__ import annotations

from typing import List, Optional

from ..index import constants as C
from ..index import signatures as S
from ..index import tags as T
from ..index.log_entry import FileInfo
from ..plan import expressions as E
from ..plan import logical as L
from ..plan.optimizer import optimize_in
from ..utils import path_utils as P
from ..utils.conf import HyperspaceConf
from ..utils.file_utils import FileStatus


def _ctx(session):
    from ..hyperspace import get_context
    return get_context(session)


def get_logical_relation(plan: L.LogicalPlan) -> Optional[L.LogicalRelation]:
    lrs = plan.collect(lambda p: isinstance(p, L.LogicalRelation))
    return lrs[0] if len(lrs) == 1 else None


def is_index_applied(rel: L.HadoopFsRelation) -> bool:
    k, v = C.INDEX_RELATION_IDENTIFIER
    return rel.options.get(k) == v


def get_candidate_indexes(session, indexes: list, plan: L.LogicalRelation) -> list:
    conf = session.conf
    hybrid = HyperspaceConf.hybrid_scan_enabled(conf)
    delete_enabled = HyperspaceConf.hybrid_scan_delete_enabled(conf)
    sig_cache = {}

    def signature_valid(entry) -> bool:
        def compute():
            sig = entry.signature
            if sig.provider not in sig_cache:
                sig_cache[sig.provider] = S.create(sig.provider).signature(plan, session)
            s = sig_cache[sig.provider]
            return s is not None and s == sig.value
        return entry.with_cached_tag(plan, T.SIGNATURE_MATCHED, compute)

    if not hybrid:
        return [i for i in indexes if i.created and signature_valid(i)]

    app_thr = HyperspaceConf.hybrid_scan_appended_ratio_threshold(conf)
    del_thr = HyperspaceConf.hybrid_scan_deleted_ratio_threshold(conf)
    files = _ctx(session).source_provider_manager.all_files(plan)
    inputs = [FileInfo(f.path, f.length, f.modification_time, C.UNKNOWN_FILE_ID) for f in files]
    total = sum(f.size for f in inputs)
    cur_cfg = [str(app_thr), str(del_thr)]
    for idx in indexes:
        tagged = idx.get_tag_value(plan, T.HYBRIDSCAN_RELATED_CONFIGS)
        if tagged is None or tagged != cur_cfg:
            idx.unset_tag_value(plan, T.IS_HYBRIDSCAN_CANDIDATE)
            idx.set_tag_value(plan, T.HYBRIDSCAN_RELATED_CONFIGS, cur_cfg)

    def is_candidate(entry) -> bool:
        def compute():
            src = entry.source_file_info_set
            common = [f for f in inputs if f in src]
            common_cnt = len(common)
            common_bytes = sum(f.size for f in common)
            appended_ratio = 1 - common_bytes / float(total) if total else 0.0
            src_bytes = entry.source_files_size_in_bytes
            deleted_ratio = 1 - common_bytes / float(src_bytes) if src_bytes else 0.0
            deleted_cnt = len(src) - common_cnt
            append_delete = delete_enabled and entry.has_lineage_column and common_cnt > 0 and \
                appended_ratio < app_thr and deleted_ratio < del_thr
            append_only = deleted_cnt == 0 and common_cnt > 0 and appended_ratio < app_thr
            ok = append_delete or append_only
            if ok:
                entry.set_tag_value(plan, T.COMMON_SOURCE_SIZE_IN_BYTES, common_bytes)
                entry.set_tag_value(plan, T.HYBRIDSCAN_REQUIRED,
                                    not (common_cnt == len(src) and common_cnt == len(inputs)))
            return ok
        return entry.with_cached_tag(plan, T.IS_HYBRIDSCAN_CANDIDATE, compute)

    return [i for i in indexes if i.created and is_candidate(i)]


def _statuses(paths_or_infos) -> List[FileStatus]:
    out = []
    for f in paths_or_infos:
        if isinstance(f, FileInfo):
            out.append(FileStatus(f.name, f.size, f.modified_time))
        elif isinstance(f, FileStatus):
            out.append(f)
    return out


def _index_file_index(index, extra: list = ()) -> L.FileIndex:
    infos = sorted(index.content.file_infos, key=lambda f: f.name)
    files = _statuses(infos) + list(extra)
    return L.FileIndex([f.path for f in files], files)


_SCHEMA_FOR: dict = {}


def _index_schema_for(index, base: L.LogicalRelation, with_lineage: bool):
    """Index columns that exist in the base relation (+ lineage); memoized on the (immutable)
    schema objects since rules evaluate it for every candidate of every query."""
    import pyarrow as pa
    ischema, bschema = index.schema, base.relation.schema
    k = (id(ischema), id(bschema), with_lineage)
    hit = _SCHEMA_FOR.get(k)
    if hit is not None and hit[0] is ischema and hit[1] is bschema:
        return hit[2]
    base_fields = {(f.name, str(f.type)) for f in bschema}
    fields = [f for f in ischema
              if (f.name, str(f.type)) in base_fields or
              (with_lineage and f.name == C.DATA_FILE_NAME_ID)]
    out = pa.schema(fields)
    if len(_SCHEMA_FOR) > 1024:
        _SCHEMA_FOR.clear()
    _SCHEMA_FOR[k] = (ischema, bschema, out)
    return out


def _index_relation(session, index, base: L.LogicalRelation, location, schema, use_bucket_spec):
    k, v = C.INDEX_RELATION_IDENTIFIER
    rel = L.HadoopFsRelation(location, None, schema,
                             index.bucket_spec if use_bucket_spec else None, "parquet", {k: v},
                             index=index)
    names = set(schema.names)
    out = [a for a in base.output if a.name in names]
    return rel, out


def transform_plan_to_use_index(session, index, plan: L.LogicalPlan, use_bucket_spec: bool):
    lr = get_logical_relation(plan)
    assert lr is not None
    hybrid_required = HyperspaceConf.hybrid_scan_enabled(session.conf) and \
        bool(index.get_tag_value(lr, T.HYBRIDSCAN_REQUIRED))
    if hybrid_required or index.has_source_update:
        out = transform_plan_to_use_hybrid_scan(session, index, plan, use_bucket_spec)
    else:
        out = transform_plan_to_use_index_only_scan(session, index, plan, use_bucket_spec)
    assert out is not plan
    return out


def transform_plan_to_use_index_only_scan(session, index, plan, use_bucket_spec):
    def fn(p):
        if isinstance(p, L.LogicalRelation) and not p.relation.is_index():
            loc = index.with_cached_tag(None, T.INMEMORYFILEINDEX_INDEX_ONLY,
                                        lambda: _index_file_index(index))
            rel, out = _index_relation(session, index, p, loc, _index_schema_for(index, p, False),
                                       use_bucket_spec)
            return p.copy(relation=rel, output=out)
        return None
    return plan.transform_down(fn)


def transform_plan_to_use_hybrid_scan(session, index, plan, use_bucket_spec):
    conf = session.conf
    unhandled: list = []

    def fn(p):
        if not isinstance(p, L.LogicalRelation) or p.relation.is_index():
            return None
        if not HyperspaceConf.hybrid_scan_enabled(conf) and index.has_source_update:
            deleted = sorted(index.deleted_files, key=lambda f: f.name)
            appended = sorted(index.appended_files, key=lambda f: f.name)
        else:
            mgr = _ctx(session).source_provider_manager
            tracker = index.file_id_tracker
            cur = [FileInfo.from_status(f, tracker.add_file(f), True) for f in mgr.all_files(p)]
            src = index.source_file_info_set
            if HyperspaceConf.hybrid_scan_delete_enabled(conf) and index.has_lineage_column:
                exist = [f for f in cur if f in src]
                appended = [f for f in cur if f not in src]
                deleted = sorted(src - set(exist), key=lambda f: f.name) if len(exist) < len(src) else []
            else:
                appended = [f for f in cur if f not in src]
                deleted = []
        partitioned = len(p.relation.location.partition_schema) > 0
        if use_bucket_spec or not index.has_parquet_as_source_format or deleted or partitioned:
            unhandled.extend(appended)
            loc = index.with_cached_tag(None, T.INMEMORYFILEINDEX_INDEX_ONLY,
                                        lambda: _index_file_index(index))
        else:
            loc = _index_file_index(index, _statuses(appended))
        schema = _index_schema_for(index, p, bool(deleted))
        rel, out = _index_relation(session, index, p, loc, schema, use_bucket_spec)
        if not deleted:
            return p.copy(relation=rel, output=out)
        import pyarrow as pa
        lineage = E.Attribute(C.DATA_FILE_NAME_ID, pa.int64(), False)
        new_rel = p.copy(relation=rel, output=out + [lineage])
        ids = [E.Literal(f.id, pa.int64()) for f in deleted]
        thr = int(conf.get(C.SQL_IN_SET_CONVERSION_THRESHOLD, "10"))
        filt = optimize_in(L.Filter(E.Not(E.In(lineage, ids)), new_rel), thr)
        return L.Project(out, filt)

    index_plan = plan.transform_up(fn)
    if not unhandled:
        return index_plan
    appended_plan = transform_plan_to_read_appended_files(session, index, plan, unhandled)
    if use_bucket_spec:
        bs = index.bucket_spec.copy(sort_column_names=())
        return L.BucketUnion([index_plan, transform_plan_to_shuffle_using_bucket_spec(bs, appended_plan)], bs)
    return L.Union([index_plan, appended_plan])


def transform_plan_to_read_appended_files(session, index, plan, appended: list):
    import pyarrow as pa
    k, v = C.INDEX_RELATION_IDENTIFIER

    def fn(p):
        if not isinstance(p, L.LogicalRelation) or p.relation.is_index():
            return None
        rel = p.relation
        mgr = _ctx(session).source_provider_manager
        bp = mgr.partition_base_path(rel.location)
        opts = dict(rel.options)
        opts[k] = v
        if bp is not None:
            opts["basePath"] = bp
        statuses = _statuses(appended)
        from ..io.reader import discover_partitions
        pspec = rel.location.partition_spec
        if len(pspec.columns):
            pspec = discover_partitions(statuses, [bp] if bp else [], bp)
            pspec.columns = rel.location.partition_spec.columns
        loc = L.FileIndex([f.path for f in statuses], statuses, pspec)
        idx_names = set(index.schema.names)
        part_names = set(rel.partition_schema.names)
        data_schema = pa.schema([f for f in rel.data_schema if f.name in idx_names])
        part_schema = rel.partition_schema
        new_rel = L.HadoopFsRelation(loc, part_schema, data_schema, None, rel.file_format, opts)
        out = [a for a in p.output if a.name in idx_names or a.name in part_names]
        return p.copy(relation=new_rel, output=out)

    out = plan.transform_down(fn)
    assert out is not plan
    return out


def transform_plan_to_shuffle_using_bucket_spec(bucket_spec: L.BucketSpec, plan: L.LogicalPlan):
    def indexed_attrs(p):
        m = {a.name: a for a in p.output}
        return [m.get(n) for n in bucket_spec.bucket_column_names]

    injected = [False]

    def fn(p):
        if injected[0]:
            return None
        is_project = isinstance(p, L.Project)
        candidate = (is_project and (isinstance(p.child, L.LogicalRelation) or (
            isinstance(p.child, L.Filter) and isinstance(p.child.child, L.LogicalRelation)))) or \
            (isinstance(p, L.Filter) and isinstance(p.child, L.LogicalRelation)) or \
            isinstance(p, L.LogicalRelation)
        if not candidate:
            return None
        attrs = indexed_attrs(p)
        if is_project and not all(a is not None for a in attrs):
            return None
        injected[0] = True
        return _Marker(L.RepartitionByExpression([a for a in attrs if a is not None], p,
                                                 bucket_spec.num_buckets))

    shuffled = plan.transform_down(fn)
    shuffled = _unmark(shuffled)
    assert injected[0]
    return shuffled


class _Marker(L.LogicalPlan):
    """Stops transform_down from descending into a freshly injected shuffle."""

    def __init__(self, inner):
        self.inner = inner
        self.children = ()

    @property
    def output(self):
        return self.inner.output

    def with_children(self, children):
        return self


def _unmark(plan):
    def fn(p):
        if isinstance(p, _Marker):
            return p.inner
        return None
    return plan.transform_up(fn)
