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

    def cacheTable(self, name: str, storageLevel=None) -> None:  # data is resident already
        self._resolve(name)

    def clearCache(self) -> None:
        return None

    def isCached(self, tableName: str) -> bool:
        """Frames are materialised in device memory, so a resolvable table is always "cached"."""
        try:
            self._resolve(tableName)
            return True
        except LookupError:
            return False

    def uncacheTable(self, tableName: str) -> None:
        return None

    def refreshTable(self, tableName: str) -> None:
        return None

    def refreshByPath(self, path: str) -> None:
        return None

    def recoverPartitions(self, tableName: str) -> None:
        return None

    # ------------------------------------------------------------------ metadata
    def currentCatalog(self) -> str:
        return "spark_catalog"

    def setCurrentCatalog(self, catalogName: str) -> None:
        if catalogName != "spark_catalog":
            raise ValueError(f"catalog {catalogName!r} not found")

    def listCatalogs(self, pattern: Optional[str] = None):
        return [CatalogMetadata("spark_catalog", None)]

    def setCurrentDatabase(self, dbName: str) -> None:
        if dbName != "default":
            raise ValueError(f"database {dbName!r} not found (only 'default' and 'global_temp' exist)")

    def databaseExists(self, dbName: str) -> bool:
        return dbName in ("default", "global_temp")

    def getDatabase(self, dbName: str):
        if not self.databaseExists(dbName):
            raise LookupError(f"database {dbName!r} not found")
        return Database(dbName, "spark_catalog", None, self.warehouse if dbName == "default" else None)

    def getTable(self, tableName: str) -> Table:
        name = tableName.split(".")[-1]
        if tableName in self._views:
            return Table(tableName, None, None, "TEMPORARY", True)
        if tableName.startswith("global_temp.") and name in _GLOBAL_VIEWS:
            return Table(name, "global_temp", None, "TEMPORARY", True)
        if tbl.exists(self._table_path(tableName)):
            return Table(name, "default", None, "MANAGED", False)
        raise LookupError(f"Table or view not found: {tableName}")

    def listColumns(self, tableName: str, dbName: Optional[str] = None):
        df = self._resolve(tableName if dbName in (None, "default") else f"{dbName}.{tableName}")
        return [CatalogColumn(f.name, f.metadata.get("comment") if f.metadata else None, f.dataType.simpleString(),
                              f.nullable, False, False) for f in df.schema.fields]

    def listFunctions(self, dbName: Optional[str] = None, pattern: Optional[str] = None):
        import fnmatch
        from . import functions as F
        names = sorted({n for n in dir(F) if not n.startswith("_") and callable(getattr(F, n)) and n[0].islower()}
                       | set(_registered_udfs()))
        if pattern:
            names = [n for n in names if fnmatch.fnmatch(n, pattern.replace("*", "*"))]
        return [Function(n, None, None, None, "TEMPORARY" if n in _registered_udfs() else "BUILTIN",
                         n in _registered_udfs()) for n in names]

    def functionExists(self, functionName: str, dbName: Optional[str] = None) -> bool:
        from . import functions as F
        return functionName in _registered_udfs() or callable(getattr(F, functionName.lower(), None))

    def getFunction(self, functionName: str):
        if not self.functionExists(functionName):
            raise LookupError(f"function {functionName!r} not found")
        tmp = functionName in _registered_udfs()
        return Function(functionName, None, None, None, "TEMPORARY" if tmp else "BUILTIN", tmp)

    def registerFunction(self, name: str, f, returnType=None):
        return self._session.udf.register(name, f, returnType)

    def createTable(self, tableName: str, path: Optional[str] = None, source: Optional[str] = None,
                    schema=None, description: Optional[str] = None, **options):
        """A managed table (empty, with ``schema``) or, with ``path``, an external table: the files
        at ``path`` are registered under the name."""
        if path is not None:
            df = self._session.read.format(source or "parquet").options(**options).load(path) if schema is None \
                else self._session.read.format(source or "parquet").schema(schema).options(**options).load(path)
            self._register_view(tableName, df, replace=False)
            return df
        if schema is None:
            raise ValueError("createTable needs a schema or a path")
        from .types import StructType, parse_ddl_schema
        st = schema if isinstance(schema, StructType) else parse_ddl_schema(schema)
        df = self._session._empty_frame(st)
        tbl.write_frame(df, self._table_path(tableName), "error", operation="CREATE TABLE")
        return self._resolve(tableName)

    createExternalTable = createTable


@dataclass
class Database:
    name: str
    catalog: Optional[str]
    description: Optional[str]
    locationUri: Optional[str]


@dataclass
class CatalogMetadata:
    name: str
    description: Optional[str]


@dataclass
class CatalogColumn:
    name: str
    description: Optional[str]
    dataType: str
    nullable: bool
    isPartition: bool
    isBucket: bool


@dataclass
class Function:
    name: str
    catalog: Optional[str]
    namespace: Optional[str]
    description: Optional[str]
    className: str
    isTemporary: bool


def _registered_udfs() -> Dict[str, object]:
    from .functions import REGISTERED_UDFS
    return REGISTERED_UDFS
