"""Metastore / catalog: databases, managed tables, temp views.

Persisted as JSON under the warehouse directory so ``saveAsTable`` tables
survive the session (ML 00c - Delta Review.py:67-70,178-179;
Labs/ML 09L:41-42).
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Dict


class Table:
    def __init__(self, name, database, tableType, isTemporary, location=None, fmt=None):
        self.name = name
        self.database = database
        self.tableType = tableType
        self.isTemporary = isTemporary
        self.location = location
        self.format = fmt

    def __repr__(self):
        return f"Table(name='{self.name}', database='{self.database}', tableType='{self.tableType}', " \
               f"isTemporary={self.isTemporary})"


class Database:
    def __init__(self, name, locationUri):
        self.name = name
        self.locationUri = locationUri
        self.description = ""

    def __repr__(self):
        return f"Database(name='{self.name}', locationUri='{self.locationUri}')"


class Catalog:
    def __init__(self, session):
        self._session = session
        self._temp: Dict[str, object] = {}
        self._functions = {}
        self._current = "default"

    # ---------------------------------------------------------- storage
    @property
    def _root(self):
        return os.path.abspath(self._session.conf.get("cdnaml.warehouse.dir"))

    def _meta_path(self):
        return os.path.join(self._root, "_catalog.json")

    def _load(self):
        p = self._meta_path()
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        return {"databases": {"default": {"location": os.path.join(self._root)}}, "tables": {}}

    def _save(self, meta):
        if self._session.comm.rank != 0:
            return
        os.makedirs(self._root, exist_ok=True)
        tmp = self._meta_path() + ".tmp"
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(tmp, self._meta_path())

    def _qualify(self, name: str):
        name = name.strip("`")
        if "." in name:
            db, t = name.split(".", 1)
        else:
            db, t = self._current, name
        return db.lower(), t.lower()

    # ---------------------------------------------------------- databases
    def createDatabase(self, name, ifNotExists=True, location=None):
        meta = self._load()
        name = name.lower()
        if name in meta["databases"]:
            if not ifNotExists:
                raise RuntimeError(f"Database '{name}' already exists")
            return
        loc = location or os.path.join(self._root, f"{name}.db")
        meta["databases"][name] = {"location": loc}
        self._save(meta)

    def dropDatabase(self, name, ifExists=True, cascade=False):
        meta = self._load()
        name = name.lower()
        if name not in meta["databases"]:
            if ifExists:
                return
            raise RuntimeError(f"Database '{name}' not found")
        tables = [k for k in meta["tables"] if k.startswith(name + ".")]
        if tables and not cascade:
            raise RuntimeError(f"Database {name} is not empty")
        for k in tables:
            t = meta["tables"].pop(k)
            if t.get("managed") and self._session.comm.rank == 0:
                shutil.rmtree(t["location"], ignore_errors=True)
        meta["databases"].pop(name)
        self._save(meta)
        if self._current == name:
            self._current = "default"

    def setCurrentDatabase(self, name):
        meta = self._load()
        if name.lower() not in meta["databases"]:
            raise RuntimeError(f"Database '{name}' not found")
        self._current = name.lower()

    def currentDatabase(self):
        return self._current

    def listDatabases(self):
        return [Database(k, v["location"]) for k, v in self._load()["databases"].items()]

    def databaseExists(self, name):
        return name.lower() in self._load()["databases"]

    # ---------------------------------------------------------- tables
    def _table_location(self, name):
        db, t = self._qualify(name)
        meta = self._load()
        if db not in meta["databases"]:
            raise RuntimeError(f"Database '{db}' not found")
        base = meta["databases"][db]["location"]
        return os.path.join(base, t)

    def _register_table(self, name, location, fmt, managed):
        meta = self._load()
        db, t = self._qualify(name)
        if db not in meta["databases"]:
            meta["databases"][db] = {"location": os.path.join(self._root, f"{db}.db")}
        meta["tables"][f"{db}.{t}"] = {"location": location, "format": fmt, "managed": managed}
        self._save(meta)

    def _table_info(self, name):
        db, t = self._qualify(name)
        return self._load()["tables"].get(f"{db}.{t}")

    def tableExists(self, name, dbName=None):
        if dbName:
            name = f"{dbName}.{name}"
        return name.lower() in self._temp or self._table_info(name) is not None

    def dropTable(self, name, ifExists=True):
        meta = self._load()
        db, t = self._qualify(name)
        info = meta["tables"].pop(f"{db}.{t}", None)
        if info is None:
            if not ifExists:
                raise RuntimeError(f"Table {name} not found")
            return
        if info.get("managed") and self._session.comm.rank == 0:
            shutil.rmtree(info["location"], ignore_errors=True)
        self._save(meta)

    def listTables(self, dbName=None):
        db = (dbName or self._current).lower()
        out = [Table(k.split(".", 1)[1], db, "MANAGED" if v.get("managed") else "EXTERNAL", False, v["location"],
                     v.get("format")) for k, v in self._load()["tables"].items() if k.startswith(db + ".")]
        out += [Table(k, None, "TEMPORARY", True) for k in self._temp]
        return out

    def _register_temp(self, name, df):
        self._temp[name.lower()] = df

    def dropTempView(self, name):
        return self._temp.pop(name.lower(), None) is not None

    def _lookup(self, name):
        key = name.strip("`").lower()
        if key in self._temp:
            return self._temp[key]
        info = self._table_info(name)
        if info is None:
            from .sql.column import AnalysisException
            raise AnalysisException(f"Table or view not found: {name}")
        r = self._session.read
        if info.get("format") == "delta":
            return r.format("delta").load(info["location"])
        return r.format(info.get("format") or "parquet").load(info["location"])

    def cacheTable(self, name):
        self._lookup(name).cache()

    def uncacheTable(self, name):
        self._lookup(name).unpersist()

    def clearCache(self):
        pass

    def refreshTable(self, name):
        pass
