"""Session catalog: temporary views + managed tables under the warehouse directory.

The reference's stream sink targets the managed table ``hospital_unbounded_table``
(ref.py:44, ref.py:115) and the batch section reads it back by name through SQL
(ref.py:123-128); both resolve here.
"""
from __future__ import annotations

import os
import shutil
from dataclasses import dataclass
from typing import Dict, List, Optional

from ..io import table as tbl


_GLOBAL_VIEWS: dict = {}  # global_temp database: shared by the sessions of this process


@dataclass
class Table:
    name: str
    database: Optional[str]
    description: Optional[str]
    tableType: str
    isTemporary: bool


class Catalog:
    def __init__(self, session):
        self._session = session
        self._views: Dict[str, object] = {}

    # ------------------------------------------------------------------ locations
    @property
    def warehouse(self) -> str:
        return self._session.conf.get("spark.sql.warehouse.dir", os.path.join(os.getcwd(), "spark-warehouse"))

    def _table_path(self, name: str) -> str:
        return os.path.join(self.warehouse, name.split(".")[-1])

    # ------------------------------------------------------------------ views
    def _register_view(self, name: str, df, replace: bool) -> None:
        if not replace and name in self._views:
            raise ValueError(f"temporary view {name!r} already exists")
        self._views[name] = df

    def dropTempView(self, name: str) -> bool:
        return self._views.pop(name, None) is not None

    # global temporary views live in the ``global_temp`` database, shared by the sessions of the process
    def _register_global_view(self, name: str, df, replace: bool) -> None:
        if not replace and name in _GLOBAL_VIEWS:
            raise ValueError(f"global temporary view {name!r} already exists")
        _GLOBAL_VIEWS[name] = df

    def dropGlobalTempView(self, name: str) -> bool:
        return _GLOBAL_VIEWS.pop(name, None) is not None

    # ------------------------------------------------------------------ tables
    def _save_table(self, name: str, df, mode: str) -> None:
        tbl.write_frame(df, self._table_path(name), "append" if mode == "append" else mode, operation="WRITE")

    def _resolve(self, name: str):
        if name in self._views:
            return self._views[name]
        if name.startswith("global_temp."):
            v = _GLOBAL_VIEWS.get(name.split(".", 1)[1])
            if v is None:
                raise LookupError(f"Table or view not found: {name}")
            return v
        path = self._table_path(name)
        if tbl.exists(path):
            return tbl.read_table(self._session, path)
        raise LookupError(f"Table or view not found: {name}")

    def tableExists(self, tableName: str, dbName: Optional[str] = None) -> bool:
        return tableName in self._views or tbl.exists(self._table_path(tableName))

    def listTables(self, dbName: Optional[str] = None) -> List[Table]:
        out = [Table(n, None, None, "TEMPORARY", True) for n in sorted(self._views)]
        wh = self.warehouse
        if os.path.isdir(wh):
            for d in sorted(os.listdir(wh)):
                if tbl.exists(os.path.join(wh, d)):
                    out.append(Table(d, "default", None, "MANAGED", False))
        return out

    def dropTable(self, name: str) -> None:
        path = self._table_path(name)
        comm = self._session._comm
        comm.barrier()
        if comm.is_root and os.path.isdir(path):
            shutil.rmtree(path)
        comm.barrier()

    def history(self, name: str):
        return tbl.history(self._table_path(name))

    def currentDatabase(self) -> str:
        return "default"

    def listDatabases(self):
        return ["default"]

    def cacheTable(self, name: str) -> None:  # data is resident already
        return None

    def clearCache(self) -> None:
        return None
