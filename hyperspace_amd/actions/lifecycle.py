"""Metadata-only lifecycle actions (reference ``DeleteAction.scala:24-48``,
``RestoreAction.scala:24-48``, ``VacuumAction.scala:24-57``, ``CancelAction.scala:35-76``)."""
from __future__ import annotations

from ..exceptions import HyperspaceException
from ..telemetry.events import (CancelActionEvent, DeleteActionEvent, RestoreActionEvent,
                                VacuumActionEvent)
from . import states
from .base import Action


class _ExistingEntryAction(Action):
    what = ""

    def __init__(self, log_manager, session=None):
        super().__init__(log_manager, session)
        self._entry = None

    def log_entry(self):
        if self._entry is None:
            e = self.log_manager.get_log(self.base_id)
            if e is None:
                raise HyperspaceException(f"LogEntry must exist for {self.what} operation")
            self._entry = e
        return self._entry


class DeleteAction(_ExistingEntryAction):
    what = "delete"
    transient_state = states.DELETING
    final_state = states.DELETED

    def validate(self):
        if self.log_entry().state.upper() != states.ACTIVE:
            raise HyperspaceException(f"Delete is only supported in {states.ACTIVE} state. "
                                      f"Current state is {self.log_entry().state}")

    def op(self):
        pass

    def event(self, app_info, message):
        return DeleteActionEvent(app_info, self.log_entry(), message)


class RestoreAction(_ExistingEntryAction):
    what = "restore"
    transient_state = states.RESTORING
    final_state = states.ACTIVE

    def validate(self):
        if self.log_entry().state.upper() != states.DELETED:
            raise HyperspaceException(f"Restore is only supported in {states.DELETED} state. "
                                      f"Current state is {self.log_entry().state}")

    def op(self):
        pass

    def event(self, app_info, message):
        return RestoreActionEvent(app_info, self.log_entry(), message)


class VacuumAction(_ExistingEntryAction):
    what = "vacuum"
    transient_state = states.VACUUMING
    final_state = states.DOESNOTEXIST

    def __init__(self, log_manager, data_manager, session=None):
        super().__init__(log_manager, session)
        self.data_manager = data_manager

    def validate(self):
        if self.log_entry().state.upper() != states.DELETED:
            raise HyperspaceException(f"Vacuum is only supported in {states.DELETED} state. "
                                      f"Current state is {self.log_entry().state}")

    def op(self):
        if not self._is_coordinator():
            return
        latest = self.data_manager.get_latest_version_id()
        if latest is not None:
            for i in range(latest, -1, -1):
                self.data_manager.delete(i)

    def event(self, app_info, message):
        return VacuumActionEvent(app_info, self.log_entry(), message)


class CancelAction(_ExistingEntryAction):
    """Roll a crashed action back to the last stable state.

    The reference documents "save the next log entry with the contents of the last active state
    log entry" but commits the *crashed* entry with the stable state (``CancelAction.scala:36-40``),
    so cancelling a crashed refresh leaves an ACTIVE entry pointing at a half-written ``v__=n``.
    Here the final entry carries the last stable entry's content, as documented."""
    what = "cancel"
    transient_state = states.CANCELLING

    _final = None

    def end_log_entry(self):
        stable = self.log_manager.get_latest_stable_log()
        if self.final_state == states.DOESNOTEXIST or stable is None:
            return self.log_entry()
        return stable

    @property
    def final_state(self):
        # Decided from the state *before* begin() overwrites it with CANCELLING.
        if self._final is None:
            if self.log_entry().state == states.VACUUMING:
                self._final = states.DOESNOTEXIST
            else:
                stable = self.log_manager.get_latest_stable_log()
                self._final = states.DOESNOTEXIST if stable is None else stable.state
        return self._final

    def validate(self):
        _ = self.final_state
        if self.log_entry().state in states.STABLE_STATES:
            raise HyperspaceException(
                f"Cancel() is not supported in {sorted(states.STABLE_STATES)} states. "
                f"Current state is {self.log_entry().state}")

    def op(self):
        pass

    def event(self, app_info, message):
        return CancelActionEvent(app_info, self.log_entry(), message)
