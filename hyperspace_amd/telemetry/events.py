"""Telemetry events and pluggable loggers (reference ``telemetry/HyperspaceEvent.scala:28-156``,
``telemetry/HyperspaceEventLogging.scala:30-68``).

The sink is chosen by ``spark.hyperspace.eventLoggerClass`` (a dotted Python class path) and
defaults to ``NoOpEventLogger``.  Unlike the reference's lazy JVM singleton, the logger is resolved
per session so tests can swap it; events also carry device metrics (rows, bytes, kernel ms).
"""
from __future__ import annotations

import importlib
import logging
from dataclasses import dataclass, field
from typing import Any, List, Optional

from ..exceptions import HyperspaceException
from ..index import constants as C

log = logging.getLogger(__name__)


@dataclass
class AppInfo:
    sparkUser: str
    appId: str
    appName: str


class HyperspaceEvent:
    pass


class HyperspaceIndexCRUDEvent(HyperspaceEvent):
    pass


@dataclass
class CreateActionEvent(HyperspaceIndexCRUDEvent):
    appInfo: AppInfo
    indexConfig: Any
    index: Optional[Any]
    originalPlan: str
    message: str


@dataclass
class _IndexEvent(HyperspaceIndexCRUDEvent):
    appInfo: AppInfo
    index: Any
    message: str


class DeleteActionEvent(_IndexEvent):
    pass


class RestoreActionEvent(_IndexEvent):
    pass


class VacuumActionEvent(_IndexEvent):
    pass


class RefreshActionEvent(_IndexEvent):
    pass


class CancelActionEvent(_IndexEvent):
    pass


class RefreshIncrementalActionEvent(_IndexEvent):
    pass


class RefreshQuickActionEvent(_IndexEvent):
    pass


class OptimizeActionEvent(_IndexEvent):
    pass


@dataclass
class HyperspaceIndexUsageEvent(HyperspaceEvent):
    appInfo: AppInfo
    indexes: List[Any]
    planBeforeRule: str
    planAfterRule: str
    message: str


@dataclass
class QueryExecutionEvent(HyperspaceEvent):
    """MI355X addition: per-query device metrics (rows scanned, bytes, time per stage)."""
    appInfo: AppInfo
    device: str
    metrics: dict = field(default_factory=dict)


class EventLogger:
    def log_event(self, event: HyperspaceEvent) -> None:
        raise NotImplementedError


class NoOpEventLogger(EventLogger):
    def log_event(self, event: HyperspaceEvent) -> None:
        pass


_logger_cache: dict = {}


def get_event_logger(conf) -> EventLogger:
    name = conf.get(C.EVENT_LOGGER_CLASS_KEY) if conf is not None else None
    if not name:
        return NoOpEventLogger()
    if name in _logger_cache:
        return _logger_cache[name]
    try:
        mod, _, cls = name.rpartition(".")
        inst = getattr(importlib.import_module(mod), cls)()
    except Exception as e:  # noqa: BLE001
        raise HyperspaceException(f"Unable to instantiate event logger from provided class {name}") from e
    if not isinstance(inst, EventLogger) and not hasattr(inst, "log_event"):
        raise HyperspaceException(f"Unable to instantiate event logger from provided class {name}")
    _logger_cache[name] = inst
    return inst


class HyperspaceEventLogging:
    """Mixin: ``self.session`` must be set."""

    def log_event(self, event: HyperspaceEvent) -> None:
        get_event_logger(getattr(self, "session", None) and self.session.conf).log_event(event)
