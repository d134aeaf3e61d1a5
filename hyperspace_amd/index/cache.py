"""Index-list cache (reference ``index/Cache.scala:23-41``, ``IndexCacheFactory.scala:24-40``,
``CachingIndexCollectionManager.scala:137-169``).

Creation-time based expiry (``spark.hyperspace.index.cache.expiryDurationInSeconds``).  Unlike the
reference (Appendix B quirk 5), the cached list is filtered by the requested states, and
``cancel`` clears the cache too.
"""
from __future__ import annotations

import time
from typing import Generic, Optional, TypeVar

from . import constants as C

T = TypeVar("T")


class Clock:
    def get_time(self) -> int:
        return int(time.time() * 1000)


class Cache(Generic[T]):
    def get(self) -> Optional[T]:
        raise NotImplementedError

    def set(self, entry: T) -> None:
        raise NotImplementedError

    def clear(self) -> None:
        raise NotImplementedError


class CreationTimeBasedIndexCache(Cache):
    def __init__(self, session, clock: Clock = None):
        self.session = session
        self.clock = clock or Clock()
        self._entries = []
        self._last = 0

    def get(self):
        if self._last > 0:
            exp = int(self.session.conf.get(C.INDEX_CACHE_EXPIRY_DURATION_SECONDS,
                                            C.INDEX_CACHE_EXPIRY_DURATION_SECONDS_DEFAULT))
            if self.clock.get_time() < self._last + exp * 1000:
                return self._entries
        return None

    def set(self, entry) -> None:
        self._entries = entry
        self._last = self.clock.get_time()

    def clear(self) -> None:
        self._last = 0


CREATION_TIME_BASED = "CREATION_TIME_BASED"


class IndexCacheFactory:
    def create(self, session, cache_type: str) -> Cache:
        raise NotImplementedError


class IndexCacheFactoryImpl(IndexCacheFactory):
    def create(self, session, cache_type: str = CREATION_TIME_BASED) -> Cache:
        if cache_type == CREATION_TIME_BASED:
            return CreationTimeBasedIndexCache(session)
        raise ValueError(f"Unknown cache type: {cache_type}")
