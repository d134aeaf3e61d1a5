"""BASELINE config #5 plumbing on the host executor at a tiny scale: TPC-DS-shaped tables
(``models/tpcds.py``), covering indexes on the three tables, the star join through the indexes,
an incremental refresh after appended fact files, and the independent pyarrow-dataset oracle."""
import argparse
import os
import sys

import numpy as np

from hyperspace_amd.models import tpcds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tpcds_domains(tmp_path):
    d = tpcds.date_dim()
    assert d.num_rows == tpcds.DATE_ROWS
    assert d.column("d_date_sk")[0].as_py() == 2_415_022
    assert str(d.column("d_date")[0].as_py()) == "1900-01-02"
    assert tpcds.item_rows(300) == 264_000 and tpcds.item_rows(100) == 204_000
    assert tpcds.store_sales_rows(300) == 864_121_200
    t = tpcds.store_sales_chunk(0.01, 4, 1)
    sk = t.column("ss_sold_date_sk").to_numpy()
    assert sk.min() >= tpcds.SALES_LO and sk.max() <= tpcds.SALES_HI
    assert t.column("ss_item_sk").to_numpy().max() <= tpcds.item_rows(0.01)
    ext = t.column("ss_ext_sales_price").to_numpy()
    np.testing.assert_allclose(ext, np.round(t.column("ss_quantity").to_numpy() *
                                             t.column("ss_sales_price").to_numpy(), 2))


def test_tpcds_3way_config_cpu(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import configs
    args = argparse.Namespace(device="cpu", buckets=4, steps=3, data_dir=str(tmp_path),
                              tpcds_sf=0.02, sf=1.0)
    out = configs.config_tpcds_3way(args)
    assert out["base_match"] and out["refreshed_match"], out
    assert set(out["base_indexes_in_plan"]) == {"ss_item", "item_idx", "date_idx"}, out
    assert "ss_item" in out["refreshed_indexes_in_plan"]
    assert out["refreshed_lines"] >= out["base_lines"]
