"""Device table cache accounting (exec/device_cache.py): the HBM budget covers what queries
derive from a resident table (compacted copies, join indexes), re-measured on every hit."""
import pyarrow as pa
import torch

from hyperspace_amd.exec.device_cache import DeviceTableCache
from hyperspace_amd.exec.device_table import DeviceColumn, DeviceTable
from hyperspace_amd.exec.encoding import Compact


class _F:
    def __init__(self, path):
        self.path, self.length, self.modification_time = path, 1, 1


def _table(n=100):   # 100 int32 rows = 400 bytes
    return DeviceTable({"a": DeviceColumn(torch.zeros(n, dtype=torch.int32), None, pa.int32())}, n)


def test_budget_counts_derived_structures_and_evicts_lru():
    c = DeviceTableCache(1000)
    files = {k: [_F(k)] for k in "xyz"}
    tx = c.get(files["x"], ["a"], (), _table)
    c.get(files["y"], ["a"], (), _table)
    assert c.resident_bytes == 800 and c.hits == 0
    # a query attaches a compacted copy (+100 B) to x: re-measured on the next hit
    tx.columns["a"].compact = Compact(torch.zeros(100, dtype=torch.int8), 1, 0, None, 0)
    assert c.get(files["x"], ["a"], (), _table) is tx
    assert c.resident_bytes == 900
    # z does not fit next to x (500) and y (400): the least recently used (y) goes
    c.get(files["z"], ["a"], (), _table)
    assert c.resident_bytes == 900
    assert c.get(files["x"], ["a"], (), _table) is tx and c.hits == 2
    misses = c.misses
    c.get(files["y"], ["a"], (), _table)
    assert c.misses == misses + 1
