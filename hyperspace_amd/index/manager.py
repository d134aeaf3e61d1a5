"""Index management layer (reference ``IndexManager.scala:24-107``,
``IndexCollectionManager.scala:28-185``, ``CachingIndexCollectionManager.scala:38-170``)."""
from __future__ import annotations

from typing import List, Optional, Sequence

from ..actions import states
from ..actions.create import CreateAction
from ..actions.lifecycle import CancelAction, DeleteAction, RestoreAction, VacuumAction
from ..actions.optimize import OptimizeAction
from ..actions.refresh import RefreshAction, RefreshIncrementalAction, RefreshQuickAction
from ..exceptions import HyperspaceException
from . import constants as C
from . import statistics as ST
from .cache import CREATION_TIME_BASED, IndexCacheFactoryImpl
from .factories import (FileSystemFactoryImpl, IndexDataManagerFactoryImpl,
                        IndexLogManagerFactoryImpl)
from .path_resolver import PathResolver


class IndexManager:
    def indexes(self):
        raise NotImplementedError

    def create(self, df, config) -> None:
        raise NotImplementedError

    def delete(self, name: str) -> None:
        raise NotImplementedError

    def restore(self, name: str) -> None:
        raise NotImplementedError

    def vacuum(self, name: str) -> None:
        raise NotImplementedError

    def refresh(self, name: str, mode: str) -> None:
        raise NotImplementedError

    def optimize(self, name: str, mode: str) -> None:
        raise NotImplementedError

    def cancel(self, name: str) -> None:
        raise NotImplementedError

    def get_indexes(self, states_: Sequence[str] = ()) -> list:
        raise NotImplementedError

    def index(self, name: str):
        raise NotImplementedError


class IndexCollectionManager(IndexManager):
    def __init__(self, session, log_manager_factory=None, data_manager_factory=None,
                 fs_factory=None):
        self.session = session
        self.log_manager_factory = log_manager_factory or IndexLogManagerFactoryImpl()
        self.data_manager_factory = data_manager_factory or IndexDataManagerFactoryImpl()
        self.fs_factory = fs_factory or FileSystemFactoryImpl()

    def _resolver(self):
        return PathResolver(self.session.conf)

    def _get_log_manager(self, name: str):
        path = self._resolver().get_index_path(name)
        if self.fs_factory.create(path).exists(path):
            return self.log_manager_factory.create(path)
        return None

    def _with_log_manager(self, name: str):
        lm = self._get_log_manager(name)
        if lm is None:
            raise HyperspaceException(f"Index with name {name} could not be found.")
        return lm

    def _data_manager(self, name: str):
        return self.data_manager_factory.create(self._resolver().get_index_path(name))

    def create(self, df, config) -> None:
        path = self._resolver().get_index_path(config.indexName)
        dm = self.data_manager_factory.create(path)
        lm = self._get_log_manager(config.indexName) or self.log_manager_factory.create(path)
        CreateAction(self.session, df, config, lm, dm).run()

    def delete(self, name: str) -> None:
        DeleteAction(self._with_log_manager(name), self.session).run()

    def restore(self, name: str) -> None:
        RestoreAction(self._with_log_manager(name), self.session).run()

    def vacuum(self, name: str) -> None:
        lm = self._with_log_manager(name)
        VacuumAction(lm, self._data_manager(name), self.session).run()

    def refresh(self, name: str, mode: str = C.REFRESH_MODE_FULL) -> None:
        lm = self._with_log_manager(name)
        dm = self._data_manager(name)
        m = mode.lower()
        if m == C.REFRESH_MODE_INCREMENTAL:
            RefreshIncrementalAction(self.session, lm, dm).run()
        elif m == C.REFRESH_MODE_FULL:
            RefreshAction(self.session, lm, dm).run()
        elif m == C.REFRESH_MODE_QUICK:
            RefreshQuickAction(self.session, lm, dm).run()
        else:
            raise HyperspaceException(f"Unsupported refresh mode '{mode}' found.")

    def optimize(self, name: str, mode: str = C.OPTIMIZE_MODE_QUICK) -> None:
        lm = self._with_log_manager(name)
        OptimizeAction(self.session, lm, self._data_manager(name), mode).run()

    def cancel(self, name: str) -> None:
        CancelAction(self._with_log_manager(name), self.session).run()

    def _log_managers(self):
        root = self._resolver().system_path
        fs = self.fs_factory.create(root)
        if not fs.exists(root):
            return []
        return [self.log_manager_factory.create(s.path) for s in fs.list_status(root) if s.is_dir]

    def get_indexes(self, states_: Sequence[str] = ()) -> list:
        out = []
        for lm in self._log_managers():
            e = lm.get_latest_log()
            if e is not None and (not states_ or e.state in states_):
                out.append(e)
        return out

    def indexes(self):
        from ..plan.dataframe import DataFrame
        from ..plan import logical as L
        rows = [ST.statistics(e) for e in self.get_indexes() if e.state != states.DOESNOTEXIST]
        return DataFrame(self.session, L.LocalRelation(ST.to_table(rows)))

    def index(self, name: str):
        from ..plan.dataframe import DataFrame
        from ..plan import logical as L
        lm = self._with_log_manager(name)
        e = lm.get_latest_stable_log()
        if e is None or e.state.upper() == states.DOESNOTEXIST:
            raise HyperspaceException(f"No latest stable log found for index {name}.")
        return DataFrame(self.session, L.LocalRelation(ST.to_table([ST.statistics(e, True)], True)))


class CachingIndexCollectionManager(IndexCollectionManager):
    def __init__(self, session, cache_factory=None, log_manager_factory=None,
                 data_manager_factory=None, fs_factory=None):
        super().__init__(session, log_manager_factory, data_manager_factory, fs_factory)
        self.cache = (cache_factory or IndexCacheFactoryImpl()).create(session, CREATION_TIME_BASED)

    def get_indexes(self, states_: Sequence[str] = ()) -> list:
        cached = self.cache.get()
        if cached is None:
            cached = super().get_indexes(())
            self.cache.set(cached)
        return [e for e in cached if not states_ or e.state in states_]

    def snapshot(self):
        """The cached index-metadata list the rules read (a new object after every refill:
        mutating API calls and TTL expiry), so its identity versions cached plans."""
        cached = self.cache.get()
        if cached is None:
            cached = super().get_indexes(())
            self.cache.set(cached)
        return cached

    def clear_cache(self) -> None:
        self.cache.clear()

    def _mutating(name):
        def wrapper(self, *a, **kw):
            self.clear_cache()
            try:
                return getattr(IndexCollectionManager, name)(self, *a, **kw)
            finally:
                self.clear_cache()
        wrapper.__name__ = name
        return wrapper

    create = _mutating("create")
    delete = _mutating("delete")
    restore = _mutating("restore")
    vacuum = _mutating("vacuum")
    refresh = _mutating("refresh")
    optimize = _mutating("optimize")
    cancel = _mutating("cancel")
