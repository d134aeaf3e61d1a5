"""Index path resolution (reference ``index/PathResolver.scala:30-76``).

System path = ``spark.hyperspace.system.path`` or ``${spark.sql.warehouse.dir}/indexes``; index
name lookup is case-insensitive over the existing directories.
"""
from __future__ import annotations

from ..utils import file_utils as FU
from ..utils import path_utils as P
from . import constants as C


class PathResolver:
    def __init__(self, conf):
        self.conf = conf

    @property
    def system_path(self) -> str:
        default = P.join(P.make_absolute(self.conf.get(C.WAREHOUSE_DIR, "spark-warehouse")),
                         C.INDEXES_DIR)
        value = self.conf.get(C.INDEX_SYSTEM_PATH, default)
        return value if P.is_qualified(value) else P.make_absolute(value)

    def get_index_path(self, name: str) -> str:
        root = self.system_path
        fs = FU.get_fs(root)
        if fs.exists(root):
            for s in fs.list_status(root):
                if s.name.lower() == name.lower():
                    return s.path
        return P.join(root, name)
