"""Heavy-bucket key-range split of the sharded placement (parallel/placement.py split_heavy):
a bucket heavier than total/W is cut at split keys of its leading indexed column into pieces on
distinct ranks, every row keeps exactly one owner, and shuffles route a cut bucket's rows by key.
The reference leaves skew to the user (docs/_docs/04-ug-faqs.md:107-132); the multi-rank
device run is tests/test_distributed.py::test_heavy_bucket_cut_into_key_ranges."""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest
import torch

from hyperspace_amd.io.writer import bucket_file_name
from hyperspace_amd.parallel import placement as PL
from hyperspace_amd.utils.file_utils import FileStatus


def test_equal_weights_reproduce_modulo():
    m = PL.split_heavy([10.0] * 12, 4, lambda b, k: [1, 2, 3])
    assert m.owners.tolist() == [b % 4 for b in range(12)] and not m.splits
    assert (m.owners == PL.lpt([10.0] * 12, 4)).all()


def test_heavy_bucket_pieces_on_distinct_ranks():
    w = [700.0] + [30.0] * 10                      # total 1000, W = 4: cap 250
    m = PL.split_heavy(w, 4, lambda b, k: [100 * i for i in range(1, k)])
    ranks, bounds = m.splits[0]
    assert len(ranks) == 3 and len(set(ranks.tolist())) == 3
    assert bounds.tolist() == [100, 200]
    assert m.owners[0] == ranks[0]
    # every rank's load is far below the unsplit LPT's 700
    assert m.loads(w).max() < 0.5 * PL.OwnerMap.balanced(w, 4).loads(w).max()
    seen = []
    for r in range(4):
        cuts = m.ranges(r)
        if r in ranks.tolist():
            assert 0 in m.owned(r) and 0 in cuts
            seen.append(cuts[0])
        else:
            assert 0 not in m.owned(r) and 0 not in cuts
    assert sorted(seen, key=lambda x: (x[0] is not None, x[0] or 0)) == \
        [(None, 100), (100, 200), (200, None)]
    # the other buckets stay whole, each with one owner
    for b in range(1, 11):
        assert sum(b in m.owned(r) for r in range(4)) == 1


def test_unsplittable_heavy_bucket_stays_whole():
    m = PL.split_heavy([700.0] + [30.0] * 10, 4, lambda b, k: None)
    assert not m.splits
    assert (m.owners == PL.lpt([700.0] + [30.0] * 10, 4)).all()


def test_dest_routes_cut_bucket_rows_by_key():
    m = PL.OwnerMap([0, 1, 2, 3], 4, {2: ([3, 1], [50])})
    bucket = torch.tensor([2, 2, 2, 0, 1, 3], dtype=torch.int32)
    keys = torch.tensor([10, 50, 99, 7, 8, 9], dtype=torch.int64)
    assert m.dest(bucket, keys).tolist() == [3, 1, 1, 0, 1, 3]
    with pytest.raises(ValueError):
        m.dest(bucket)
    assert m.key != PL.OwnerMap([3, 1, 2, 3], 4).key
    with pytest.raises(ValueError):
        PL.OwnerMap([0, 1], 2, {0: ([1, 1], [5])})           # pieces on one rank


def _bucket_files(tmp_path, b, keys, stats: bool, rg: int):
    name = bucket_file_name(0, "00000000-0000-0000-0000-000000000000", b, "snappy")
    path = tmp_path / name
    pq.write_table(pa.table({"k": np.sort(keys).astype(np.int64),
                             "v": np.arange(len(keys), dtype=np.int64)}),
                   path, row_group_size=rg, write_statistics=stats)
    return [FileStatus(str(path), path.stat().st_size, 0)]


@pytest.mark.parametrize("stats", [True, False])
def test_bucket_bounds_at_row_quantiles(tmp_path, stats):
    keys = np.repeat(np.arange(1000, dtype=np.int64), 4)           # 4000 rows, 1000 keys
    files = _bucket_files(tmp_path, 3, keys, stats, 100)
    bounds, frac = PL.bucket_bounds(files, 8, "k")(3, 4)
    assert len(bounds) == 3 and bounds == sorted(bounds)
    for got, q in zip(bounds, (250, 500, 750)):
        assert abs(got - q) <= 25
    assert len(frac) == 4 and abs(sum(frac) - 1) < 1e-9 and max(frac) < 0.3
    assert PL.bucket_bounds(files, 8, "k")(5, 4) is None            # no such bucket
    one = _bucket_files(tmp_path / ".." / tmp_path.name, 6, np.full(500, 9), stats, 100)
    assert PL.bucket_bounds(one, 8, "k")(6, 3) is None              # one key: cannot cut


def test_session_map_split_switch(tmp_path):
    from hyperspace_amd import Session
    keys = np.arange(3000, dtype=np.int64)
    files = _bucket_files(tmp_path, 0, keys, True, 200)
    w = [3000.0, 100.0, 100.0, 100.0]
    for enabled, expect_split in (("true", True), ("false", False)):
        s = Session(conf={PL.HEAVY_SPLIT: enabled})
        m = PL.session_map(s, 4, 2, w, PL.bucket_bounds(files, 4, "k"))
        assert bool(m.splits) == expect_split
        assert PL.session_map(s, 4, 2) is m                          # sticky


def test_hot_key_bucket_is_not_cut(tmp_path):
    """90% of the bucket's rows on one key: any cut leaves one piece with most rows, so the
    bucket stays whole (the plain balanced map gives it a rank of its own)."""
    keys = np.concatenate([np.full(9000, 500), np.arange(1000)]).astype(np.int64)
    files = _bucket_files(tmp_path, 0, keys, False, 1000)
    w = [10000.0, 300.0, 300.0, 300.0]
    m = PL.split_heavy(w, 2, PL.bucket_bounds(files, 4, "k"))
    assert not m.splits and (m.owners == PL.lpt(w, 2)).all()
