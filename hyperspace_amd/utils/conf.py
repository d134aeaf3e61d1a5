"""Typed configuration accessors (reference ``util/HyperspaceConf.scala:26-110``).

``RuntimeConf`` is the session conf (``spark.conf`` analog): a plain string map read at use time,
so changes take effect immediately.
"""
from __future__ import annotations

from ..index import constants as C


class RuntimeConf:
    def __init__(self, initial=None):
        self._m = {}
        self.version = 0   # bumped on every change (plan-cache key, plan/plan_cache.py)
        for k, v in (initial or {}).items():
            self.set(k, v)

    def set(self, key: str, value) -> None:
        if isinstance(value, bool):
            value = "true" if value else "false"
        value = str(value)
        if self._m.get(key) != value:
            self._m[key] = value
            self.version += 1

    def get(self, key: str, default=None):
        return self._m.get(key, default)

    def get_option(self, key: str):
        return self._m.get(key)

    def unset(self, key: str) -> None:
        if self._m.pop(key, None) is not None:
            self.version += 1

    def contains(self, key: str) -> bool:
        return key in self._m

    def get_all(self) -> dict:
        return dict(self._m)


_BOOLS: dict = {}


def _b(v: str) -> bool:
    r = _BOOLS.get(v)
    if r is None:
        r = str(v).strip().lower() == "true"
        if isinstance(v, str) and len(_BOOLS) < 1024:
            _BOOLS[v] = r
    return r


class HyperspaceConf:
    @staticmethod
    def hybrid_scan_enabled(conf) -> bool:
        return _b(conf.get(C.INDEX_HYBRID_SCAN_ENABLED, C.INDEX_HYBRID_SCAN_ENABLED_DEFAULT))

    @staticmethod
    def hybrid_scan_deleted_ratio_threshold(conf) -> float:
        return float(conf.get(C.INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD,
                              C.INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD_DEFAULT))

    @staticmethod
    def hybrid_scan_delete_enabled(conf) -> bool:
        return HyperspaceConf.hybrid_scan_deleted_ratio_threshold(conf) > 0.0

    @staticmethod
    def hybrid_scan_appended_ratio_threshold(conf) -> float:
        return float(conf.get(C.INDEX_HYBRID_SCAN_APPENDED_RATIO_THRESHOLD,
                              C.INDEX_HYBRID_SCAN_APPENDED_RATIO_THRESHOLD_DEFAULT))

    @staticmethod
    def optimize_file_size_threshold(conf) -> int:
        return int(conf.get(C.OPTIMIZE_FILE_SIZE_THRESHOLD, str(C.OPTIMIZE_FILE_SIZE_THRESHOLD_DEFAULT)))

    @staticmethod
    def num_buckets_for_index(conf) -> int:
        for k in (C.INDEX_NUM_BUCKETS, C.INDEX_NUM_BUCKETS_LEGACY):
            if conf.contains(k):
                return int(conf.get(k))
        return C.INDEX_NUM_BUCKETS_DEFAULT

    @staticmethod
    def index_lineage_enabled(conf) -> bool:
        return _b(conf.get(C.INDEX_LINEAGE_ENABLED, C.INDEX_LINEAGE_ENABLED_DEFAULT))

    @staticmethod
    def file_based_source_builders(conf) -> str:
        return conf.get(C.FILE_BASED_SOURCE_BUILDERS, C.FILE_BASED_SOURCE_BUILDERS_DEFAULT)

    @staticmethod
    def supported_file_formats_for_default_file_based_source(conf) -> str:
        return conf.get(C.DEFAULT_SOURCE_SUPPORTED_FORMATS, C.DEFAULT_SOURCE_SUPPORTED_FORMATS_DEFAULT)

    @staticmethod
    def case_sensitive(conf) -> bool:
        return _b(conf.get(C.SQL_CASE_SENSITIVE, "false"))

    @staticmethod
    def shuffle_partitions(conf) -> int:
        return int(conf.get(C.SQL_SHUFFLE_PARTITIONS, "200"))

    @staticmethod
    def auto_broadcast_join_threshold(conf) -> int:
        return int(conf.get(C.SQL_AUTO_BROADCAST_JOIN_THRESHOLD, str(10 * 1024 * 1024)))

    @staticmethod
    def exec_device(conf) -> str:
        return conf.get(C.EXEC_DEVICE, C.EXEC_DEVICE_DEFAULT).lower()

    @staticmethod
    def device_cache_bytes(conf) -> int:
        return int(conf.get(C.DEVICE_CACHE_BYTES, C.DEVICE_CACHE_BYTES_DEFAULT))

    @staticmethod
    def index_file_codec(conf) -> str:
        return conf.get(C.INDEX_FILE_CODEC, C.INDEX_FILE_CODEC_DEFAULT).lower()

    @staticmethod
    def index_row_group_rows(conf) -> int:
        return int(conf.get(C.INDEX_ROW_GROUP_ROWS, C.INDEX_ROW_GROUP_ROWS_DEFAULT))

    @staticmethod
    def codegen_enabled(conf) -> bool:
        return _b(conf.get(C.CODEGEN_ENABLED, C.CODEGEN_ENABLED_DEFAULT))

    @staticmethod
    def fd_group_enabled(conf) -> bool:
        """GROUP BY (join key, right columns) over a unique right key groups by the key and
        looks the right columns up for the result groups (exec/gpu.py ``_fd_grouping``)."""
        return _b(conf.get("spark.hyperspace.mi.fdGroup.enabled", "true"))

    @staticmethod
    def hipgraph_enabled(conf) -> bool:
        return _b(conf.get(C.HIPGRAPH_ENABLED, C.HIPGRAPH_ENABLED_DEFAULT))

    @staticmethod
    def join_graph_enabled(conf) -> bool:
        return HyperspaceConf.hipgraph_enabled(conf) and \
            _b(conf.get(C.JOIN_GRAPH_ENABLED, C.JOIN_GRAPH_ENABLED_DEFAULT))

    @staticmethod
    def run_topk_enabled(conf) -> bool:
        return _b(conf.get(C.RUN_TOPK_ENABLED, C.RUN_TOPK_ENABLED_DEFAULT))

    @staticmethod
    def prepared_submit_enabled(conf) -> bool:
        return _b(conf.get(C.PREPARED_SUBMIT_ENABLED, C.PREPARED_SUBMIT_ENABLED_DEFAULT))

    @staticmethod
    def gc_freeze_enabled(conf) -> bool:
        return _b(conf.get(C.GC_FREEZE_ENABLED, C.GC_FREEZE_ENABLED_DEFAULT))

    @staticmethod
    def side_stream_scans(conf) -> bool:
        return _b(conf.get(C.SIDE_STREAM_SCANS, C.SIDE_STREAM_SCANS_DEFAULT))

    @staticmethod
    def side_stream_priority(conf) -> int:
        """torch stream priority of the scan side stream (-1 high, 0 normal)."""
        v = str(conf.get(C.SIDE_STREAM_PRIORITY, C.SIDE_STREAM_PRIORITY_DEFAULT)).lower()
        if v not in ("high", "normal"):
            raise ValueError(f"{C.SIDE_STREAM_PRIORITY} must be high or normal, got {v}")
        return -1 if v == "high" else 0

    @staticmethod
    def index_placement(conf) -> str:
        v = str(conf.get(C.INDEX_PLACEMENT, C.INDEX_PLACEMENT_DEFAULT)).lower()
        if v not in ("sharded", "replicated"):
            raise ValueError(f"{C.INDEX_PLACEMENT} must be sharded or replicated, got {v}")
        return v

    @staticmethod
    def hbm_reserve_bytes(conf) -> int:
        return int(conf.get(C.HBM_RESERVE_BYTES, C.HBM_RESERVE_BYTES_DEFAULT))

    @staticmethod
    def build_hbm_budget_bytes(conf) -> int:
        return int(conf.get(C.BUILD_HBM_BUDGET_BYTES, C.BUILD_HBM_BUDGET_BYTES_DEFAULT))

    @staticmethod
    def plan_cache_enabled(conf) -> bool:
        return _b(conf.get(C.PLAN_CACHE_ENABLED, C.PLAN_CACHE_ENABLED_DEFAULT))

    @staticmethod
    def join_index_enabled(conf) -> bool:
        return _b(conf.get(C.JOIN_INDEX_ENABLED, C.JOIN_INDEX_ENABLED_DEFAULT))

    @staticmethod
    def hbm_compression_enabled(conf) -> bool:
        return _b(conf.get(C.HBM_COMPRESSION_ENABLED, C.HBM_COMPRESSION_ENABLED_DEFAULT))
