"""Action state machine (reference ``actions/Action.scala:34-107``).

``run`` = log "started" -> validate -> begin (write ``baseId+1`` with the transient state) -> op
-> end (drop ``latestStable``, write ``baseId+2`` with the final state, recreate
``latestStable``) -> log "succeeded".  A failed log write means another writer won the optimistic
race ("Could not acquire proper state").  ``NoChangesException`` turns the call into a logged no-op.

MI355X additions: fault-injection points (``spark.hyperspace.mi.faultInjection`` =
``after_begin|mid_op|before_end``) and SPMD awareness — under ``torch.distributed``
only the coordinator rank writes the log while every rank takes part in ``op`` (the build).
"""
from __future__ import annotations

import logging
import time

from ..exceptions import HyperspaceException, NoChangesException
from ..index import constants as C
from ..telemetry.events import AppInfo, get_event_logger

log = logging.getLogger(__name__)


class FaultInjected(HyperspaceException):
    pass


class Action:
    transient_state: str = ""
    final_state: str = ""

    def __init__(self, log_manager, session=None):
        self.log_manager = log_manager
        self.session = session
        latest = log_manager.get_latest_id()
        self.base_id = latest if latest is not None else -1

    # -- to override ----------------------------------------------------------------------------
    def log_entry(self):
        raise NotImplementedError

    def validate(self) -> None:
        pass

    def op(self) -> None:
        raise NotImplementedError

    def event(self, app_info: AppInfo, message: str):
        raise NotImplementedError

    # -- machinery ------------------------------------------------------------------------------
    def _dist(self):
        return getattr(self.session, "dist", None) if self.session is not None else None

    def _is_coordinator(self) -> bool:
        d = self._dist()
        return d is None or d.rank == 0

    def _barrier(self) -> None:
        d = self._dist()
        if d is not None:
            d.barrier()

    def _fault(self, point: str) -> None:
        """Raise at ``point`` if the fault-injection conf names it.  ``point@r`` limits the fault
        to rank ``r`` (SPMD failure tests: one rank fails, every rank must observe it)."""
        spec = self.session.conf.get(C.FAULT_INJECTION) if self.session is not None else None
        if not spec:
            return
        name, _, rank = str(spec).partition("@")
        if name != point:
            return
        d = self._dist()
        if rank and int(rank) != (d.rank if d is not None else 0):
            return
        raise FaultInjected(f"fault injected at {point}")

    def _op_with_faults(self) -> None:
        self.op()
        self._fault("mid_op")

    def _save_entry(self, id: int, entry) -> None:
        entry.timestamp = int(time.time() * 1000)
        if not self.log_manager.write_log(id, entry):
            raise HyperspaceException("Could not acquire proper state")

    def _agreed(self, fn, coordinator_only: bool = False) -> None:
        """Run ``fn`` (on every rank, or on the coordinator only) and make its outcome unanimous:
        under SPMD a failure on any rank is re-raised on every rank — the same exception kind,
        so a ``NoChangesException`` stays a no-op everywhere — instead of leaving the other ranks
        blocked in the next barrier.  Doubles as that barrier."""
        d = self._dist()
        if d is None:
            fn()
            return
        err = None
        try:
            if not coordinator_only or d.rank == 0:
                fn()
        except Exception as e:  # noqa: BLE001 — shared with the other ranks below
            err = e
        outcomes = d.all_gather_object(
            None if err is None else (isinstance(err, NoChangesException), str(err)))
        if err is not None:
            raise err
        failed = [o for o in outcomes if o is not None]
        if failed:
            no_change, msg = failed[0]
            raise NoChangesException(msg) if no_change else HyperspaceException(
                f"failed on another rank: {msg}")

    def _begin(self) -> None:
        def write():
            entry = self.log_entry()
            entry.state = self.transient_state
            entry.id = self.base_id + 1
            self._save_entry(self.base_id + 1, entry)
        self._agreed(write, coordinator_only=True)

    def end_log_entry(self):
        """Entry committed by ``end`` (the same as ``begin``'s unless an action overrides it)."""
        return self.log_entry()

    def _end(self) -> None:
        def commit():
            entry = self.end_log_entry()
            entry.state = self.final_state
            entry.id = self.base_id + 2
            if not self.log_manager.delete_latest_stable_log():
                raise HyperspaceException("Could not delete latest stable log")
            self._save_entry(self.base_id + 2, entry)
            if not self.log_manager.create_latest_stable_log(self.base_id + 2):
                log.warning("Unable to recreate latest stable log")
        self._agreed(commit, coordinator_only=True)

    def _app_info(self) -> AppInfo:
        s = self.session
        if s is None:
            return AppInfo("", "", "")
        return AppInfo(s.user, s.app_id, s.app_name)

    def _log_event(self, message: str) -> None:
        try:
            ev = self.event(self._app_info(), message)
        except Exception:  # noqa: BLE001 — event construction must never fail the action
            return
        get_event_logger(self.session.conf if self.session else None).log_event(ev)

    def run(self) -> None:
        try:
            self._log_event("Operation started.")
            self._barrier()   # every rank has pinned base_id / target paths
            # nobody writes the log before every rank validated
            self._agreed(self.validate)
            self._begin()
            self._fault("after_begin")
            # every rank's share of the build finished before the coordinator commits
            self._agreed(self._op_with_faults)
            self._fault("before_end")
            self._end()
            self._log_event("Operation succeeded.")
        except NoChangesException as e:
            self._log_event(f"No-op operation recorded: {e.msg}")
            log.warning(e.msg)
        except Exception as e:
            self._log_event(f"Operation failed: {e}")
            raise
