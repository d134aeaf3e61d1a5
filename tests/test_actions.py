"""Action state-machine tests against fake log/data managers — the mock-based tier of the
reference (``ActionTest.scala:55-63``, ``CancelActionTest.scala``, ``DeleteActionTest.scala``,
``RestoreActionTest.scala``, ``VacuumActionTest.scala``), using the same DI seams
(``index/factories.py``) instead of Mockito."""
from __future__ import annotations

import pytest

from hyperspace_amd.actions import states as S
from hyperspace_amd.actions.base import Action
from hyperspace_amd.actions.lifecycle import (CancelAction, DeleteAction, RestoreAction,
                                              VacuumAction)
from hyperspace_amd.exceptions import HyperspaceException, NoChangesException
from hyperspace_amd.index.data_manager import IndexDataManager
from hyperspace_amd.index.log_manager import IndexLogManager


class Entry:
    """``TestLogEntry.scala``: a log entry that only carries its state."""

    def __init__(self, state: str):
        self.state = state
        self.id = 0
        self.timestamp = 0
        self.enabled = True


class FakeLogManager(IndexLogManager):
    def __init__(self, latest_id=None, entry=None, stable=None, write_ok=True):
        self.latest_id = latest_id
        self.entry = entry
        self.stable = stable
        self.write_ok = write_ok
        self.calls = []

    def get_log(self, id):
        return self.entry

    def get_latest_id(self):
        return self.latest_id

    def get_latest_log(self):
        return self.entry

    def get_latest_stable_log(self):
        return self.stable

    def create_latest_stable_log(self, id):
        self.calls.append(("create_latest_stable", id))
        return True

    def delete_latest_stable_log(self):
        self.calls.append(("delete_latest_stable",))
        return True

    def write_log(self, id, entry):
        self.calls.append(("write", id, entry.state))
        return self.write_ok


class FakeDataManager(IndexDataManager):
    def __init__(self, latest=None):
        self.latest = latest
        self.deleted = []

    def get_latest_version_id(self):
        return self.latest

    def get_path(self, id):
        return f"/idx/v__={id}"

    def delete(self, id):
        self.deleted.append(id)


class DummyAction(Action):
    transient_state = S.CREATING
    final_state = S.ACTIVE

    def __init__(self, lm, validate_exc=None):
        super().__init__(lm)
        self.validate_exc = validate_exc
        self.ops = 0

    def log_entry(self):
        return Entry(S.ACTIVE)

    def validate(self):
        if self.validate_exc is not None:
            raise self.validate_exc

    def op(self):
        self.ops += 1

    def event(self, app_info, message):
        return None


# ---------------------------------------------------------------------------------- Action.run
def test_run_writes_transient_then_final_and_moves_latest_stable():
    lm = FakeLogManager(latest_id=None)
    a = DummyAction(lm)
    a.run()
    assert a.ops == 1
    assert lm.calls == [("write", 0, S.CREATING), ("delete_latest_stable",),
                        ("write", 1, S.ACTIVE), ("create_latest_stable", 1)]


def test_run_continues_from_latest_id():
    lm = FakeLogManager(latest_id=4)
    DummyAction(lm).run()
    assert [c for c in lm.calls if c[0] == "write"] == [("write", 5, S.CREATING),
                                                        ("write", 6, S.ACTIVE)]


def test_run_fails_when_another_writer_won():
    lm = FakeLogManager(latest_id=0, write_ok=False)
    a = DummyAction(lm)
    with pytest.raises(HyperspaceException, match="Could not acquire proper state"):
        a.run()
    assert a.ops == 0


def test_no_changes_exception_is_a_logged_no_op():
    lm = FakeLogManager(latest_id=1)
    a = DummyAction(lm, NoChangesException("nothing to do"))
    a.run()  # swallowed
    assert lm.calls == [] and a.ops == 0


def test_validation_failure_writes_nothing():
    lm = FakeLogManager(latest_id=1)
    with pytest.raises(HyperspaceException, match="bad"):
        DummyAction(lm, HyperspaceException("bad")).run()
    assert lm.calls == []


# ---------------------------------------------------------------------------------- Cancel
def test_cancel_from_active_state_final_is_active():
    lm = FakeLogManager(latest_id=None, entry=Entry(S.ACTIVE), stable=Entry(S.ACTIVE))
    assert CancelAction(lm).final_state == S.ACTIVE


def test_cancel_from_transient_goes_to_last_stable_state():
    lm = FakeLogManager(latest_id=None, entry=Entry(S.REFRESHING), stable=Entry(S.ACTIVE))
    assert CancelAction(lm).final_state == S.ACTIVE
    lm = FakeLogManager(latest_id=None, entry=Entry(S.RESTORING), stable=Entry(S.DELETED))
    assert CancelAction(lm).final_state == S.DELETED


def test_cancel_from_vacuuming_goes_to_does_not_exist():
    lm = FakeLogManager(latest_id=None, entry=Entry(S.VACUUMING), stable=Entry(S.ACTIVE))
    assert CancelAction(lm).final_state == S.DOESNOTEXIST


def test_cancel_without_stable_state_goes_to_does_not_exist():
    lm = FakeLogManager(latest_id=None, entry=Entry(S.REFRESHING), stable=None)
    assert CancelAction(lm).final_state == S.DOESNOTEXIST


@pytest.mark.parametrize("state", sorted(S.STABLE_STATES))
def test_cancel_rejected_in_stable_states(state):
    lm = FakeLogManager(latest_id=3, entry=Entry(state), stable=Entry(state))
    with pytest.raises(HyperspaceException, match="Cancel"):
        CancelAction(lm).run()


def test_cancel_commits_cancelling_then_stable_state():
    lm = FakeLogManager(latest_id=7, entry=Entry(S.OPTIMIZING), stable=Entry(S.ACTIVE))
    CancelAction(lm).run()
    assert [c for c in lm.calls if c[0] == "write"] == [("write", 8, S.CANCELLING),
                                                        ("write", 9, S.ACTIVE)]


# ---------------------------------------------------------------------------------- Delete / Restore
@pytest.mark.parametrize("cls,ok_state", [(DeleteAction, S.ACTIVE), (RestoreAction, S.DELETED)])
def test_lifecycle_validate_by_state(cls, ok_state):
    cls(FakeLogManager(latest_id=1, entry=Entry(ok_state))).validate()
    for st in (S.CREATING, S.DELETING, S.REFRESHING, S.VACUUMING, S.RESTORING, S.OPTIMIZING,
               S.DOESNOTEXIST, S.CANCELLING, S.ACTIVE, S.DELETED):
        if st == ok_state:
            continue
        with pytest.raises(HyperspaceException):
            cls(FakeLogManager(latest_id=1, entry=Entry(st))).validate()


def test_delete_and_restore_state_transitions():
    lm = FakeLogManager(latest_id=1, entry=Entry(S.ACTIVE))
    DeleteAction(lm).run()
    assert [c[2] for c in lm.calls if c[0] == "write"] == [S.DELETING, S.DELETED]
    lm = FakeLogManager(latest_id=3, entry=Entry(S.DELETED))
    RestoreAction(lm).run()
    assert [c[2] for c in lm.calls if c[0] == "write"] == [S.RESTORING, S.ACTIVE]


def test_missing_log_entry_is_an_error():
    with pytest.raises(HyperspaceException, match="LogEntry must exist"):
        DeleteAction(FakeLogManager(latest_id=0, entry=None)).validate()


# ---------------------------------------------------------------------------------- Vacuum
def test_vacuum_validate_only_from_deleted():
    VacuumAction(FakeLogManager(latest_id=1, entry=Entry(S.DELETED)), FakeDataManager()).validate()
    for st in (S.ACTIVE, S.CREATING, S.DOESNOTEXIST):
        with pytest.raises(HyperspaceException, match="Vacuum"):
            VacuumAction(FakeLogManager(latest_id=1, entry=Entry(st)), FakeDataManager()).validate()


def test_vacuum_op_deletes_every_data_version():
    dm = FakeDataManager(latest=2)
    lm = FakeLogManager(latest_id=5, entry=Entry(S.DELETED))
    VacuumAction(lm, dm).run()
    assert dm.deleted == [2, 1, 0]
    assert [c[2] for c in lm.calls if c[0] == "write"] == [S.VACUUMING, S.DOESNOTEXIST]


def test_vacuum_with_no_data_is_fine():
    dm = FakeDataManager(latest=None)
    VacuumAction(FakeLogManager(latest_id=5, entry=Entry(S.DELETED)), dm).run()
    assert dm.deleted == []
