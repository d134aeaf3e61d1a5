"""Public API facade (reference ``Hyperspace.scala:26-204``, ``python/hyperspace/hyperspace.py:9-192``).

Method names, arguments and defaults match the reference's Python binding so user code ports by
changing the import::

    from hyperspace_amd import Hyperspace, IndexConfig, Session
    hs = Hyperspace(session)
    hs.createIndex(df, IndexConfig("idx", ["k"], ["v"]))
    Hyperspace.enable(session)
"""
from __future__ import annotations

import sys
import threading
import weakref

from .index import constants as C
from .index.config import IndexConfig
from .index.manager import CachingIndexCollectionManager
from .sources.manager import FileBasedSourceProviderManager

_ctx_local = threading.local()


class HyperspaceContext:
    def __init__(self, session):
        self.session_ref = weakref.ref(session)
        self.index_collection_manager = CachingIndexCollectionManager(session)
        self.source_provider_manager = FileBasedSourceProviderManager(session)

    @property
    def indexCollectionManager(self):
        return self.index_collection_manager

    @property
    def sourceProviderManager(self):
        return self.source_provider_manager


def get_context(session=None) -> HyperspaceContext:
    """Per-thread context, recreated when the session changes (``Hyperspace.scala:169-181``)."""
    if session is None:
        from .session import Session
        session = Session.active()
    ctx = getattr(_ctx_local, "ctx", None)
    if ctx is None or ctx.session_ref() is not session:
        ctx = HyperspaceContext(session)
        _ctx_local.ctx = ctx
    return ctx


class Hyperspace:
    def __init__(self, spark):
        self.spark = spark

    @property
    def _mgr(self):
        return get_context(self.spark).index_collection_manager

    def indexes(self):
        return self._mgr.indexes()

    def createIndex(self, dataFrame, indexConfig: IndexConfig) -> None:
        self._mgr.create(dataFrame, indexConfig)

    def deleteIndex(self, indexName: str) -> None:
        self._mgr.delete(indexName)

    def restoreIndex(self, indexName: str) -> None:
        self._mgr.restore(indexName)

    def vacuumIndex(self, indexName: str) -> None:
        self._mgr.vacuum(indexName)

    def refreshIndex(self, indexName: str, mode: str = C.REFRESH_MODE_FULL) -> None:
        self._mgr.refresh(indexName, mode)

    def optimizeIndex(self, indexName: str, mode: str = C.OPTIMIZE_MODE_QUICK) -> None:
        self._mgr.optimize(indexName, mode)

    def cancel(self, indexName: str) -> None:
        self._mgr.cancel(indexName)

    def explain(self, df, verbose: bool = False, redirectFunc=lambda x: sys.stdout.write(x)) -> None:
        from .plananalysis.analyzer import explain_string
        redirectFunc(explain_string(df, self.spark, self._mgr.indexes(), verbose))

    def index(self, indexName: str):
        return self._mgr.index(indexName)

    @staticmethod
    def enable(spark):
        spark.enableHyperspace()
        return spark

    @staticmethod
    def disable(spark):
        spark.disableHyperspace()
        return spark

    @staticmethod
    def isEnabled(spark) -> bool:
        return spark.isHyperspaceEnabled()
