"""All configuration keys and on-disk constants (reference ``index/IndexConstants.scala:21-107``).

Key strings are identical to the reference so existing configurations keep working.  Keys under
``spark.hyperspace.mi.*`` are MI355X-specific additions (device executor, HBM budget, ...).
"""

INDEXES_DIR = "indexes"
INDEX_SYSTEM_PATH = "spark.hyperspace.system.path"
WAREHOUSE_DIR = "spark.sql.warehouse.dir"

INDEX_NUM_BUCKETS_LEGACY = "spark.hyperspace.index.num.buckets"
INDEX_NUM_BUCKETS = "spark.hyperspace.index.numBuckets"
# Compiled default of spark.sql.shuffle.partitions (Appendix B quirk 8): NOT the runtime value.
INDEX_NUM_BUCKETS_DEFAULT = 200

INDEX_HYBRID_SCAN_ENABLED = "spark.hyperspace.index.hybridscan.enabled"
INDEX_HYBRID_SCAN_ENABLED_DEFAULT = "false"
INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD = "spark.hyperspace.index.hybridscan.maxDeletedRatio"
INDEX_HYBRID_SCAN_DELETED_RATIO_THRESHOLD_DEFAULT = "0.2"
INDEX_HYBRID_SCAN_APPENDED_RATIO_THRESHOLD = "spark.hyperspace.index.hybridscan.maxAppendedRatio"
INDEX_HYBRID_SCAN_APPENDED_RATIO_THRESHOLD_DEFAULT = "0.3"

INDEX_RELATION_IDENTIFIER = ("indexRelation", "true")

INDEX_CACHE_EXPIRY_DURATION_SECONDS = "spark.hyperspace.index.cache.expiryDurationInSeconds"
INDEX_CACHE_EXPIRY_DURATION_SECONDS_DEFAULT = "300"

HYPERSPACE_LOG = "_hyperspace_log"
INDEX_VERSION_DIRECTORY_PREFIX = "v__"
LATEST_STABLE_LOG_NAME = "latestStable"

DISPLAY_MODE = "spark.hyperspace.explain.displayMode"
HIGHLIGHT_BEGIN_TAG = "spark.hyperspace.explain.displayMode.highlight.beginTag"
HIGHLIGHT_END_TAG = "spark.hyperspace.explain.displayMode.highlight.endTag"


class DisplayMode:
    CONSOLE = "console"
    PLAIN_TEXT = "plaintext"
    HTML = "html"


DATA_FILE_NAME_ID = "_data_file_id"
INDEX_LINEAGE_ENABLED = "spark.hyperspace.index.lineage.enabled"
INDEX_LINEAGE_ENABLED_DEFAULT = "false"

REFRESH_MODE_INCREMENTAL = "incremental"
REFRESH_MODE_FULL = "full"
REFRESH_MODE_QUICK = "quick"

OPTIMIZE_FILE_SIZE_THRESHOLD = "spark.hyperspace.index.optimize.fileSizeThreshold"
OPTIMIZE_FILE_SIZE_THRESHOLD_DEFAULT = 256 * 1024 * 1024
OPTIMIZE_MODE_QUICK = "quick"
OPTIMIZE_MODE_FULL = "full"
OPTIMIZE_MODES = (OPTIMIZE_MODE_QUICK, OPTIMIZE_MODE_FULL)

UNKNOWN_FILE_ID = -1

LINEAGE_PROPERTY = "lineage"
HAS_PARQUET_AS_SOURCE_FORMAT_PROPERTY = "hasParquetAsSourceFormat"

GLOBBING_PATTERN_KEY = "spark.hyperspace.source.globbingPattern"

EVENT_LOGGER_CLASS_KEY = "spark.hyperspace.eventLoggerClass"
FILE_BASED_SOURCE_BUILDERS = "spark.hyperspace.index.sources.fileBasedBuilders"
FILE_BASED_SOURCE_BUILDERS_DEFAULT = "hyperspace_amd.sources.default.DefaultFileBasedSourceBuilder"
DEFAULT_SOURCE_SUPPORTED_FORMATS = \
    "spark.hyperspace.index.sources.defaultFileBasedSource.supportedFileFormats"
DEFAULT_SOURCE_SUPPORTED_FORMATS_DEFAULT = "avro,csv,json,orc,parquet,text"

# Spark SQL keys the engine honours.
SQL_CASE_SENSITIVE = "spark.sql.caseSensitive"
SQL_SHUFFLE_PARTITIONS = "spark.sql.shuffle.partitions"
SQL_AUTO_BROADCAST_JOIN_THRESHOLD = "spark.sql.autoBroadcastJoinThreshold"
SQL_IN_SET_CONVERSION_THRESHOLD = "spark.sql.optimizer.inSetConversionThreshold"

# ---- MI355X-native additions -------------------------------------------------------------
# Execution device for physical plans: "auto" (GPU when available), "gpu", "cpu".
EXEC_DEVICE = "spark.hyperspace.mi.execution.device"
EXEC_DEVICE_DEFAULT = "auto"
# Per-GPU HBM budget for the resident index-column cache (bytes); 0 = disabled.
DEVICE_CACHE_BYTES = "spark.hyperspace.mi.deviceCacheBytes"
DEVICE_CACHE_BYTES_DEFAULT = str(160 * 1024 ** 3)
# Index data file codec written by the build: "snappy" (Spark's default Parquet codec, as the
# reference writes; pages compressed on the device, decoded by the device Snappy inflate) or
# "none" (uncompressed).
INDEX_FILE_CODEC = "spark.hyperspace.mi.index.codec"
INDEX_FILE_CODEC_DEFAULT = "snappy"
# Rows per Parquet row group in index files (row-group stats drive pruning).
INDEX_ROW_GROUP_ROWS = "spark.hyperspace.mi.index.rowGroupRows"
INDEX_ROW_GROUP_ROWS_DEFAULT = "1048576"
# Fault-injection hook for action crash tests: after_begin | mid_op | before_end.
# whole-stage code generation (hipRTC) for the fused scan/join aggregate kernels
CODEGEN_ENABLED = "spark.hyperspace.mi.codegen.enabled"
CODEGEN_ENABLED_DEFAULT = "true"
# lossless frame-of-reference / decimal-scale compaction of HBM columns read by generated kernels
HBM_COMPRESSION_ENABLED = "spark.hyperspace.mi.hbmCompression.enabled"
# on by default since the generated kernels load each thread's rows as aligned vectors
# (jit.SCAN_VEC / JI_VEC): narrow codes then cut HBM bytes instead of only adding decode work
# (SF100 Q6+Q3: 988 -> 1133 q/s, profiles/sweep_r1_compaction_vec.txt)
HBM_COMPRESSION_ENABLED_DEFAULT = "true"
# replay captured hipGraphs of the scan pipeline (exec/graphs.py)
HIPGRAPH_ENABLED = "spark.hyperspace.mi.hipGraph.enabled"
HIPGRAPH_ENABLED_DEFAULT = "true"
# warm captured scan pipelines replay on a side stream, overlapping the work queued on the
# query's stream (exec/gpu.py GpuBackend._scan_agg_graph)
SIDE_STREAM_SCANS = "spark.hyperspace.mi.sideStreamScans.enabled"
SIDE_STREAM_SCANS_DEFAULT = "true"
# the side stream's queue priority: "high" lets the scan pipeline's kernels dispatch ahead of the
# join kernels' queued waves - measured slower at SF100 (1875 vs 2489 q/s: the scan's waves then
# take the CUs the critical-path join needs, profiles/bench_side_priority_r6.jsonl)
SIDE_STREAM_PRIORITY = "spark.hyperspace.mi.sideStreamScans.priority"
SIDE_STREAM_PRIORITY_DEFAULT = "normal"
# replay the run-keyed two-phase merge join (tags, bits scan, fold, result copy) as one captured
# hipGraph per lowering (graphs.TwoPhaseGraph); needs hipGraph.enabled
JOIN_GRAPH_ENABLED = "spark.hyperspace.mi.joinGraph.enabled"
JOIN_GRAPH_ENABLED_DEFAULT = "true"
# plan-cache hits of a fused aggregate with a known literal vector replay the prepared
# lowering directly (exec/gpu.py _AggProgram), skipping the executor's plan walk
PREPARED_SUBMIT_ENABLED = "spark.hyperspace.mi.preparedSubmit.enabled"
PREPARED_SUBMIT_ENABLED_DEFAULT = "true"
# when a new prepared program is registered (warm-up of a query shape), move every object
# alive at that point out of the cyclic GC's scans (gc.freeze after a young-generation collect):
# a full collection over the engine's long-lived state (plans, lowerings, Arrow / torch objects)
# costs tens of ms of host time in the middle of a serving loop (utils/hostgc.py)
GC_FREEZE_ENABLED = "spark.hyperspace.mi.host.gcFreeze.enabled"
GC_FREEZE_ENABLED_DEFAULT = "true"
# ORDER BY <sum / count> LIMIT k over the key-run hash walk keeps whole keys in per-wavefront
# top-K lists instead of hash-table slots (hash_agg.TopKPlan)
RUN_TOPK_ENABLED = "spark.hyperspace.mi.runTopK.enabled"
RUN_TOPK_ENABLED_DEFAULT = "true"
# cached join index (left row -> first matching right row, int32 in HBM) for joins of two
# device-resident index tables with unique integer right keys: the fused join aggregate becomes a
# streaming scan of the left table plus a gather, no per-tile span search (exec/join_index.py).
# Off by default: the run-keyed two-phase merge join is faster on the TPC-H Q3 shape (0.74 vs
# 0.93-1.53 ms per query at SF100, bench.py's join_index side key) and replays as a prepared
# program; the join index stays available per session
JOIN_INDEX_ENABLED = "spark.hyperspace.mi.joinIndex.enabled"
JOIN_INDEX_ENABLED_DEFAULT = "false"
# Query-time placement of index buckets across the ranks of a torch.distributed job:
#  "sharded"    each bucket (or key-range piece of a heavy bucket) is resident on one rank only
#               (the owner map of parallel/placement.py); every query runs on all ranks and
#               partial results combine with one RCCL all-gather (strong scaling of one query);
#  "replicated" every rank holds all buckets in its HBM (an SF100 index set is ~36 GB of a
#               288 GB MI355X) and answers queries alone, with no collective (read replicas:
#               query throughput scales with ranks).  Index builds are sharded either way.
INDEX_PLACEMENT = "spark.hyperspace.mi.index.placement"
INDEX_PLACEMENT_DEFAULT = "sharded"
# parameterized plan cache: queries that differ only in literal values reuse one planning
# (plan/plan_cache.py)
PLAN_CACHE_ENABLED = "spark.hyperspace.mi.planCache.enabled"
PLAN_CACHE_ENABLED_DEFAULT = "true"
# HBM arena reserved at engine start (bytes; capped at 80% of free HBM): allocated once and
# kept in torch's caching allocator so builds and queries do not hipMalloc multi-GB columns
HBM_RESERVE_BYTES = "spark.hyperspace.mi.hbmReserveBytes"
HBM_RESERVE_BYTES_DEFAULT = str(64 * 1024 ** 3)
# HBM an index build may use (decoded source + sort workspace); a build whose estimate exceeds
# it runs in bucket-range passes (exec/device_build.py).  0 = 60% of the free HBM at build time.
BUILD_HBM_BUDGET_BYTES = "spark.hyperspace.mi.build.hbmBudgetBytes"
BUILD_HBM_BUDGET_BYTES_DEFAULT = "0"
FAULT_INJECTION = "spark.hyperspace.mi.faultInjection"
