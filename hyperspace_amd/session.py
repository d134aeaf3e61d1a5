"""Session: the SparkSession analog that owns conf, readers, the optimizer extension points and
the execution backend.

* ``extra_optimizations`` / ``extra_strategies`` mirror ``spark.experimental`` — this is where
  ``enableHyperspace`` injects ``JoinIndexRule``, ``FilterIndexRule`` and ``BucketUnionStrategy``
  (``package.scala:35-79``).
* ``backend()`` picks the executor from ``spark.hyperspace.mi.execution.device``: the MI355X HIP
  executor when a GPU is present (``auto``), else the pyarrow oracle.
* In a ``torch.distributed`` job (one process per GPU, RCCL over xGMI) the session carries the
  rank/world so index builds shuffle with all-to-all and queries run on owned buckets.
"""
from __future__ import annotations

import getpass
import os
import threading
import uuid
from typing import Optional

import pyarrow as pa

from .index import constants as C
from .plan import logical as L
from .plan.dataframe import DataFrame
from .io.reader import DataFrameReader
from .utils.conf import HyperspaceConf, RuntimeConf

_active = threading.local()


class Session:
    def __init__(self, conf: Optional[dict] = None, app_name: str = "hyperspace-amd",
                 warehouse_dir: Optional[str] = None):
        base = {C.WAREHOUSE_DIR: os.path.abspath(warehouse_dir or "spark-warehouse"),
                C.SQL_SHUFFLE_PARTITIONS: "200"}
        base.update(conf or {})
        self.conf = RuntimeConf(base)
        self.app_name = app_name
        self.app_id = f"local-{uuid.uuid4().hex[:12]}"
        try:
            self.user = getpass.getuser()
        except Exception:  # noqa: BLE001
            self.user = "unknown"
        self.extra_optimizations: list = []
        self.extra_strategies: list = []
        self._backends: dict = {}
        self.dist = None  # parallel.dist.DistContext when running under torch.distributed
        Session.set_active(self)
        if str(self.conf.get(C.EXEC_DEVICE, "")).lower() == "gpu":
            # engine start: HIP context, kernel libraries and the pinned staging pool come up
            # with the session, not inside its first index build or query
            self.backend()

    # -- active session --------------------------------------------------------------------------
    @staticmethod
    def set_active(s: "Session") -> None:
        _active.session = s

    @staticmethod
    def active() -> "Session":
        s = getattr(_active, "session", None)
        if s is None:
            s = Session()
        return s

    getActiveSession = active

    # -- data -----------------------------------------------------------------------------------
    @property
    def read(self) -> DataFrameReader:
        return DataFrameReader(self)

    def createDataFrame(self, data, schema=None) -> DataFrame:
        if isinstance(data, pa.Table):
            t = data
        elif isinstance(data, dict):
            t = pa.table(data)
        else:
            import pandas as pd
            if isinstance(data, pd.DataFrame):
                t = pa.Table.from_pandas(data, preserve_index=False)
            else:
                rows = list(data)
                names = schema if isinstance(schema, (list, tuple)) else \
                    [f"_{i + 1}" for i in range(len(rows[0]))]
                t = pa.table({n: [r[i] for r in rows] for i, n in enumerate(names)})
        if isinstance(schema, pa.Schema):
            t = t.cast(schema)
        return DataFrame(self, L.LocalRelation(t))

    create_dataframe = createDataFrame

    # -- catalog / SQL ----------------------------------------------------------------------------
    @property
    def catalog(self):
        """Temporary views and warehouse tables (hyperspace_amd/catalog.py)."""
        c = self.__dict__.get("_catalog")
        if c is None:
            from .catalog import Catalog
            c = self._catalog = Catalog(self)
        return c

    def sql(self, query: str) -> DataFrame:
        """A DataFrame for a SQL SELECT over temporary views and tables (plan/sql.py)."""
        from .plan.sql import sql
        return sql(self, query)

    def table(self, name: str) -> DataFrame:
        return self.catalog.lookup(name)

    @property
    def case_sensitive(self) -> bool:
        # read on every name resolution of every DataFrame built: memoized per conf version
        c = self.conf
        memo = self.__dict__.get("_cs_memo")
        if memo is None or memo[0] is not c or memo[1] != c.version:
            memo = self.__dict__["_cs_memo"] = (c, c.version, HyperspaceConf.case_sensitive(c))
        return memo[2]

    # -- execution ------------------------------------------------------------------------------
    def gpu_available(self) -> bool:
        try:
            import torch
            return torch.cuda.is_available()
        except Exception:  # noqa: BLE001
            return False

    def device_kind(self) -> str:
        mode = HyperspaceConf.exec_device(self.conf)
        if mode == "cpu":
            return "cpu"
        if mode == "gpu":
            return "gpu"
        return "gpu" if self.gpu_available() else "cpu"

    def backend(self):
        kind = self.device_kind()
        if kind not in self._backends:
            if kind == "gpu":
                from .exec.gpu import GpuBackend
                self._backends[kind] = GpuBackend(self)
            else:
                from .exec.cpu import CpuBackend
                self._backends[kind] = CpuBackend(self)
        return self._backends[kind]

    # -- hyperspace enable/disable (package.scala Implicits) ----------------------------------------
    def enableHyperspace(self) -> "Session":
        from .rules import enable
        enable(self)
        if HyperspaceConf.gc_freeze_enabled(self.conf) and self.device_kind() == "gpu":
            from .utils import hostgc
            hostgc.settle(full=True)      # a serving phase starts: freeze the settled heap
        return self

    def disableHyperspace(self) -> "Session":
        from .rules import disable
        disable(self)
        return self

    def isHyperspaceEnabled(self) -> bool:
        from .rules import is_enabled
        return is_enabled(self)

    @property
    def sparkUser(self):
        return self.user


def get_or_create(**kw) -> Session:
    s = getattr(_active, "session", None)
    return s if s is not None else Session(**kw)
