"""Session catalog: temporary views and persistent (managed / external) tables.

The reference's users reach indexed data through Spark's catalog as often as through paths:
``df.createOrReplaceTempView("t1")`` + ``spark.sql("SELECT ... FROM t1, t2 WHERE ...")``
(``E2EHyperspaceRulesTest.scala:261-282``, ``python/hyperspace/tests/test_indexutilization.py:
45-46``) and ``df.write.option("path", p).saveAsTable("t1")`` + ``spark.table("t1")``
(``E2EHyperspaceRulesTest.scala:316-341``).  The rules see through both: a view is its logical
plan, a table is a relation over its files, so index rewrites apply unchanged.

* Temporary views live in the session (a name -> logical plan map; case-insensitive unless
  ``spark.sql.caseSensitive``).
* Tables are persisted under the warehouse directory: ``<warehouse>/_catalog/<name>.json``
  records the table's location and format (a managed table's data goes to
  ``<warehouse>/<name>``; ``option("path", ...)`` makes it external), so a later session over
  the same warehouse sees it - the role of Spark's metastore.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import threading
from typing import Dict, List, Optional

from .exceptions import HyperspaceException
from .index import constants as C


_IDENT = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*$")


class Catalog:
    def __init__(self, session):
        self._session = session
        self._views: Dict[str, object] = {}
        self._lock = threading.Lock()

    # -- naming ------------------------------------------------------------------------------
    def _norm(self, name: str) -> str:
        return name if self._session.case_sensitive else name.lower()

    def _warehouse(self) -> str:
        return str(self._session.conf.get(C.WAREHOUSE_DIR))

    def _meta_path(self, name: str) -> str:
        return os.path.join(self._warehouse(), "_catalog", f"{name.lower()}.json")

    @staticmethod
    def _check_name(name: str) -> None:
        """Table names are identifiers: a managed table's data directory and its catalog record
        are built from the name, and drop / overwrite delete that directory."""
        if not isinstance(name, str) or not _IDENT.match(name):
            raise HyperspaceException(f"Invalid table name '{name}' (expected an identifier)")

    # -- temporary views ---------------------------------------------------------------------
    def create_temp_view(self, name: str, plan, replace: bool) -> None:
        with self._lock:
            k = self._norm(name)
            if not replace and k in self._views:
                raise HyperspaceException(f"Temporary view '{name}' already exists")
            self._views[k] = plan

    def dropTempView(self, name: str) -> bool:
        with self._lock:
            return self._views.pop(self._norm(name), None) is not None

    def temp_view(self, name: str):
        return self._views.get(self._norm(name))

    # -- tables ------------------------------------------------------------------------------
    def table_meta(self, name: str) -> Optional[dict]:
        if not isinstance(name, str) or not _IDENT.match(name):
            return None
        p = self._meta_path(name)
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)

    def save_table(self, name: str, writer, mode: str) -> None:
        """``DataFrameWriter.saveAsTable``: write the data and record the table."""
        self._check_name(name)
        meta = self.table_meta(name)
        if meta is not None:
            if mode in ("errorifexists", "error"):
                raise HyperspaceException(f"Table '{name}' already exists")
            if mode == "ignore":
                return
        path = writer._options.get("path")
        managed = path is None
        if managed:
            path = os.path.join(self._warehouse(), name.lower())
        if meta is not None and mode == "overwrite" and meta.get("managed") and \
                os.path.exists(meta["path"]):
            if writer.reads_from(meta["path"]):
                # e.g. spark.table('t').filter(..).write.mode('overwrite').saveAsTable('t'): the
                # data is computed inside save, after this delete (Spark refuses it as well)
                raise HyperspaceException(
                    f"Cannot overwrite table '{name}' that is also being read from")
            shutil.rmtree(meta["path"])
        writer.save(path)
        os.makedirs(os.path.dirname(self._meta_path(name)), exist_ok=True)
        rec = {"name": name, "path": os.path.abspath(path), "format": writer._format,
               "managed": managed, "options": {k: v for k, v in writer._options.items()
                                               if k != "path"}}
        tmp = self._meta_path(name) + ".tmp"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, self._meta_path(name))

    def dropTable(self, name: str) -> bool:
        self._check_name(name)
        meta = self.table_meta(name)
        if meta is None:
            return False
        if meta.get("managed") and os.path.exists(meta["path"]):
            shutil.rmtree(meta["path"])
        os.remove(self._meta_path(name))
        return True

    def tableExists(self, name: str) -> bool:
        return self.temp_view(name) is not None or self.table_meta(name) is not None

    def listTables(self) -> List[str]:
        out = sorted(self._views)
        d = os.path.join(self._warehouse(), "_catalog")
        if os.path.isdir(d):
            out += sorted(f[:-5] for f in os.listdir(d) if f.endswith(".json"))
        return out

    def lookup(self, name: str):
        """The DataFrame of a temp view or table ``name``."""
        from .plan.dataframe import DataFrame
        plan = self.temp_view(name)
        if plan is not None:
            return DataFrame(self._session, plan)
        meta = self.table_meta(name)
        if meta is None:
            raise HyperspaceException(f"Table or view not found: {name}")
        r = self._session.read.format(meta.get("format", "parquet"))
        for k, v in (meta.get("options") or {}).items():
            r = r.option(k, v)
        return r.load(meta["path"])
