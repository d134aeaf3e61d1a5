"""Operation log, data versions and path resolution on the local FS (reference
``IndexLogManagerImplTest.scala:91-197``, ``IndexDataManager``/``PathResolver`` semantics), plus
the concurrent-writer race the reference never tests."""
import multiprocessing as mp
import os
import threading

from hyperspace_amd.index.data_manager import IndexDataManagerImpl
from hyperspace_amd.index.log_manager import IndexLogManagerImpl
from hyperspace_amd.index.path_resolver import PathResolver
from hyperspace_amd.utils.conf import RuntimeConf

from test_log_entry import _expected


def _entry(state, id_=0):
    e = _expected()
    e.state = state
    e.id = id_
    return e


def test_latest_id_and_get_log(tmp_path):
    lm = IndexLogManagerImpl(str(tmp_path / "idx"))
    assert lm.get_latest_id() is None and lm.get_latest_log() is None
    assert lm.write_log(0, _entry("CREATING", 0))
    assert lm.write_log(1, _entry("ACTIVE", 1))
    assert lm.write_log(10, _entry("REFRESHING", 10))
    assert lm.get_latest_id() == 10
    assert lm.get_log(1).state == "ACTIVE"
    assert lm.get_latest_log().state == "REFRESHING"
    assert lm.get_log(5) is None
    # temp files never linger
    assert all(not n.startswith("temp") for n in os.listdir(tmp_path / "idx" / "_hyperspace_log"))


def test_write_log_fails_on_existing_id(tmp_path):
    lm = IndexLogManagerImpl(str(tmp_path / "idx"))
    assert lm.write_log(0, _entry("CREATING"))
    assert not lm.write_log(0, _entry("ACTIVE"))
    assert lm.get_log(0).state == "CREATING"


def test_latest_stable_log(tmp_path):
    lm = IndexLogManagerImpl(str(tmp_path / "idx"))
    lm.write_log(0, _entry("CREATING"))
    assert lm.get_latest_stable_log() is None
    assert not lm.create_latest_stable_log(0)      # not a stable state
    assert not lm.create_latest_stable_log(7)      # does not exist
    lm.write_log(1, _entry("ACTIVE", 1))
    lm.write_log(2, _entry("DELETING", 2))
    # no latestStable file: scan downward for a stable state
    assert lm.get_latest_stable_log().id == 1
    assert lm.create_latest_stable_log(1)
    assert os.path.exists(tmp_path / "idx" / "_hyperspace_log" / "latestStable")
    assert lm.get_latest_stable_log().state == "ACTIVE"
    assert lm.delete_latest_stable_log()
    assert lm.delete_latest_stable_log()  # idempotent
    assert not os.path.exists(tmp_path / "idx" / "_hyperspace_log" / "latestStable")


def test_concurrent_writers_threads_exactly_one_wins(tmp_path):
    lm = IndexLogManagerImpl(str(tmp_path / "idx"))
    results = []
    barrier = threading.Barrier(16)

    def go(i):
        barrier.wait()
        results.append(lm.write_log(3, _entry("ACTIVE", 3)))
    ts = [threading.Thread(target=go, args=(i,)) for i in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert sum(results) == 1


def _proc_write(path, q):
    lm = IndexLogManagerImpl(path)
    q.put(lm.write_log(0, _entry("CREATING")))


def test_concurrent_writers_processes_exactly_one_wins(tmp_path):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_proc_write, args=(str(tmp_path / "idx"), q)) for _ in range(6)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
    wins = [q.get(timeout=10) for _ in ps]
    assert sum(wins) == 1


def test_data_manager_versions(tmp_path):
    dm = IndexDataManagerImpl(str(tmp_path / "idx"))
    assert dm.get_latest_version_id() is None
    for v in (0, 3, 1):
        os.makedirs(tmp_path / "idx" / f"v__={v}")
    os.makedirs(tmp_path / "idx" / "_hyperspace_log")
    assert dm.get_latest_version_id() == 3
    assert dm.get_path(4).endswith("/idx/v__=4")
    dm.delete(3)
    assert dm.get_latest_version_id() == 1


def test_path_resolver_case_insensitive_and_defaults(tmp_path):
    conf = RuntimeConf({"spark.sql.warehouse.dir": str(tmp_path / "wh")})
    r = PathResolver(conf)
    assert r.system_path.endswith("/wh/indexes")
    conf.set("spark.hyperspace.system.path", str(tmp_path / "sys"))
    os.makedirs(tmp_path / "sys" / "MyIndex")
    assert PathResolver(conf).get_index_path("myindex").endswith("/sys/MyIndex")
    assert PathResolver(conf).get_index_path("other").endswith("/sys/other")
