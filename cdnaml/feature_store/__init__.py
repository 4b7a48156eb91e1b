"""Feature store (ML 10 - Feature Store.py:61-348).

``FeatureStoreClient`` over this framework's versioned (Delta-layout) tables:

* ``create_table`` / ``create_feature_table(name, keys, features_df, schema,
  description, partition_columns)``, ``write_table(name, df, mode)`` with
  ``overwrite`` (schema-merging: columns absent from the new frame read back
  as nulls, ML 10:332,343) and ``merge`` (upsert on the primary keys);
* ``read_table(name, as_of_delta_timestamp)`` (time travel), ``get_table`` /
  ``get_feature_table`` (``.path_data_sources``, ``.description``…);
* ``FeatureLookup`` + ``create_training_set(df, lookups, label,
  exclude_columns).load_df()`` — a key join executed by the engine's
  distributed hash join (all-to-all over RCCL when multi-GPU);
* ``log_model(model, artifact_path, flavor, training_set, …)`` packages the
  model with a ``feature_spec.json`` and ``score_batch(model_uri, df)`` looks
  the features up by key before predicting.

Metadata lives next to the catalog under ``<warehouse>/_feature_store``.
"""
from __future__ import annotations

import datetime
import functools
import json
import os
import time
from typing import Any, Dict, List, Optional, Union

from ..sql import types as T

__all__ = ["FeatureStoreClient", "FeatureLookup", "TrainingSet", "FeatureTable", "feature_table"]


def feature_table(fn):
    """Marks a feature-computation function (ML 10:93).  Calling it returns the
    DataFrame and tags it with the file sources of its inputs."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        df = fn(*args, **kwargs)
        srcs = []
        for a in list(args) + list(kwargs.values()):
            if hasattr(a, "_plan"):
                srcs.extend(_lineage_sources(a._plan))
        try:
            df._fs_sources = sorted(set(srcs))
        except AttributeError:
            pass
        return df
    wrapper._is_feature_table = True
    return wrapper


def _lineage_sources(plan) -> List[str]:
    out, stack, seen = [], [plan], set()
    while stack:
        p = stack.pop()
        if id(p) in seen:
            continue
        seen.add(id(p))
        out.extend(getattr(p, "source_paths", None) or [])
        if not getattr(p, "source_paths", None) and getattr(p, "files", None):
            out.extend(sorted({os.path.dirname(f) for f in p.files}))
        stack.extend(getattr(p, "children", []) or [])
    return out


class FeatureLookup:
    def __init__(self, table_name: str, lookup_key: Union[str, List[str]], feature_names=None,
                 rename_outputs: Optional[Dict[str, str]] = None, feature_name=None, output_name=None):
        self.table_name = table_name
        self.lookup_key = [lookup_key] if isinstance(lookup_key, str) else list(lookup_key)
        if feature_name is not None:
            feature_names = [feature_name]
            if output_name:
                rename_outputs = {feature_name: output_name}
        self.feature_names = [feature_names] if isinstance(feature_names, str) else feature_names
        self.rename_outputs = dict(rename_outputs or {})

    def to_dict(self):
        return {"table_name": self.table_name, "lookup_key": self.lookup_key, "feature_names": self.feature_names,
                "rename_outputs": self.rename_outputs}

    @classmethod
    def from_dict(cls, d):
        return cls(d["table_name"], d["lookup_key"], d.get("feature_names"), d.get("rename_outputs"))

    def __repr__(self):
        return f"FeatureLookup(table_name={self.table_name!r}, lookup_key={self.lookup_key!r})"


class FeatureTable:
    def __init__(self, meta: dict):
        self._m = meta
        self.name = meta["name"]
        self.table_id = meta["table_id"]
        self.description = meta.get("description", "")
        self.primary_keys = meta["keys"]
        self.partition_columns = meta.get("partition_columns", [])
        self.features = meta.get("features", [])
        self.path_data_sources = meta.get("path_data_sources", [])
        self.creation_timestamp = meta.get("creation_timestamp")
        self.timestamp_keys = meta.get("timestamp_keys", [])

    @property
    def keys(self):
        return self.primary_keys

    def __repr__(self):
        return f"<FeatureTable: name={self.name!r}, keys={self.primary_keys}, features={self.features}>"


class TrainingSet:
    def __init__(self, client: "FeatureStoreClient", df, lookups: List[FeatureLookup], label, exclude_columns):
        self._client = client
        self._df = df
        self.feature_lookups = lookups
        self.label = label
        self.exclude_columns = exclude_columns

    def _joined(self, df, drop_label=False):
        out = df
        for lk in self.feature_lookups:
            ft = self._client.read_table(lk.table_name)
            keys = lk.lookup_key
            tkeys = self._client.get_table(lk.table_name).primary_keys
            feats = lk.feature_names or [c for c in ft.columns if c not in tkeys]
            sel = ft.select(*([ft[k].alias(ik) for k, ik in zip(tkeys, keys)] +
                              [ft[f].alias(lk.rename_outputs.get(f, f)) for f in feats]))
            out = out.join(sel, on=keys, how="left")
        excl = [self.exclude_columns] if isinstance(self.exclude_columns, str) else list(self.exclude_columns or [])
        if drop_label and self.label:
            excl.append(self.label)
        keep = [c for c in out.columns if c not in excl]
        return out.select(*keep)

    def load_df(self):
        return self._joined(self._df)

    def feature_spec(self) -> dict:
        cols = [c for c in self.load_df().columns if c != self.label]
        return {"feature_lookups": [lk.to_dict() for lk in self.feature_lookups], "label": self.label,
                "exclude_columns": self.exclude_columns, "input_columns": cols,
                "source_columns": [c for c in self._df.columns if c != self.label]}


class FeatureStoreClient:
    def __init__(self, feature_store_uri=None, model_registry_uri=None, spark=None):
        from ..session import SparkSession
        self._spark = spark or SparkSession.builder.getOrCreate()

    # ------------------------------------------------------------ metadata
    def _root(self):
        r = os.path.join(os.path.abspath(self._spark.conf.get("cdnaml.warehouse.dir")), "_feature_store")
        os.makedirs(r, exist_ok=True)
        return r

    def _meta_path(self, name):
        return os.path.join(self._root(), self._qualify(name) + ".json")

    def _qualify(self, name):
        return name if "." in name else f"{self._spark.catalog.currentDatabase()}.{name}"

    def _load_meta(self, name) -> dict:
        p = self._meta_path(name)
        if not os.path.exists(p):
            raise ValueError(f"Feature table '{self._qualify(name)}' does not exist.")
        with open(p) as f:
            return json.load(f)

    def _save_meta(self, meta):
        if self._spark.comm.rank != 0:
            return
        p = self._meta_path(meta["name"])
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(tmp, p)

    # ------------------------------------------------------------ tables
    def create_table(self, name, primary_keys, df=None, schema: Optional[T.StructType] = None,
                     description: str = "", partition_columns=None, timestamp_keys=None, path=None, tags=None,
                     **kw) -> FeatureTable:
        qn = self._qualify(name)
        if os.path.exists(self._meta_path(qn)):
            raise ValueError(f"Feature table '{qn}' already exists. Use a different name or drop it first.")
        keys = [primary_keys] if isinstance(primary_keys, str) else list(primary_keys)
        if df is None and schema is None:
            raise ValueError("Either schema or df must be provided")
        sch = schema or df.schema
        for k in keys:
            if k not in sch.names:
                raise ValueError(f"primary key {k!r} is not a column of the feature table")
        db = qn.split(".")[0]
        self._spark.catalog.createDatabase(db, ifNotExists=True)
        meta = {"name": qn, "table_id": f"{abs(hash((qn, time.time()))) % 10 ** 12:012d}", "keys": keys,
                "description": description, "partition_columns": list(partition_columns or []),
                "timestamp_keys": list(timestamp_keys or []),
                "features": [c for c in sch.names if c not in keys],
                "path_data_sources": list(getattr(df, "_fs_sources", []) or []),
                "creation_timestamp": int(time.time() * 1000), "tags": dict(tags or {})}
        self._save_meta(meta)
        if df is not None:
            self.write_table(qn, df, mode="overwrite")
        else:
            empty = self._spark.createDataFrame([], sch)
            self._write(qn, empty, "overwrite", meta)
        return FeatureTable(self._load_meta(qn))

    def create_feature_table(self, name, keys, features_df=None, schema=None, description="",
                             partition_columns=None, **kw) -> FeatureTable:
        return self.create_table(name, keys, features_df, schema, description, partition_columns, **kw)

    def _write(self, qn, df, mode, meta):
        w = df.write.format("delta").mode(mode).option("mergeSchema", "true")
        if meta.get("partition_columns"):
            w = w.partitionBy(*meta["partition_columns"])
        w.saveAsTable(qn)

    def write_table(self, name, df, mode: str = "merge", checkpoint_location=None, trigger=None):
        qn = self._qualify(name)
        meta = self._load_meta(qn)
        keys = meta["keys"]
        missing = [k for k in keys if k not in df.columns]
        if missing:
            raise ValueError(f"DataFrame is missing primary key column(s) {missing}")
        if mode == "overwrite":
            self._write(qn, df, "overwrite", meta)
        elif mode == "merge":
            if self._spark.catalog.tableExists(qn):
                cur = self._spark.table(qn)
                # upsert: keep current rows whose key is not in df, then add df (schemas merged)
                kept = cur.join(df.select(*keys), on=keys, how="left_anti")
                self._write(qn, _union_by_name(kept, df), "overwrite", meta)
            else:
                self._write(qn, df, "overwrite", meta)
        else:
            raise ValueError(f"Unsupported mode {mode!r}: use 'overwrite' or 'merge'")
        cols = self._spark.table(qn).columns
        meta["features"] = [c for c in cols if c not in keys]
        srcs = getattr(df, "_fs_sources", None)
        if srcs:
            meta["path_data_sources"] = sorted(set(meta.get("path_data_sources", [])) | set(srcs))
        self._save_meta(meta)

    def read_table(self, name, as_of_delta_timestamp=None, **kw):
        qn = self._qualify(name)
        self._load_meta(qn)
        if as_of_delta_timestamp is None:
            return self._spark.table(qn)
        ts = as_of_delta_timestamp
        if isinstance(ts, (datetime.datetime, datetime.date)):
            ts = ts.isoformat(sep=" ") if isinstance(ts, datetime.datetime) else ts.isoformat()
        loc = self._spark.catalog._table_location(qn)
        return self._spark.read.format("delta").option("timestampAsOf", str(ts)).load(loc)

    def get_table(self, name) -> FeatureTable:
        return FeatureTable(self._load_meta(name))

    get_feature_table = get_table

    def drop_table(self, name):
        qn = self._qualify(name)
        self._load_meta(qn)
        self._spark.sql(f"DROP TABLE IF EXISTS {qn}")
        if self._spark.comm.rank == 0:
            os.remove(self._meta_path(qn))

    def set_feature_table_tag(self, table_name, key, value):
        meta = self._load_meta(table_name)
        meta.setdefault("tags", {})[key] = value
        self._save_meta(meta)

    # ------------------------------------------------------------ training / scoring
    def create_training_set(self, df, feature_lookups: List[FeatureLookup], label, exclude_columns=None
                            ) -> TrainingSet:
        for lk in feature_lookups:
            self._load_meta(lk.table_name)
            for k in lk.lookup_key:
                if k not in df.columns:
                    raise ValueError(f"lookup key {k!r} is not a column of the input DataFrame")
        return TrainingSet(self, df, list(feature_lookups), label, exclude_columns or [])

    def log_model(self, model, artifact_path: str, *, flavor, training_set: TrainingSet,
                  registered_model_name: Optional[str] = None, input_example=None, signature=None, **kw):
        from .. import tracking
        from ..tracking import fluent
        if fluent.active_run() is None:
            raise RuntimeError("fs.log_model requires an active run (with mlflow.start_run())")
        flavor.log_model(model, artifact_path, input_example=input_example, signature=signature)
        spec = training_set.feature_spec()
        spec["flavor"] = getattr(flavor, "FLAVOR_NAME", getattr(flavor, "__name__", "unknown"))
        tracking.log_dict(spec, f"{artifact_path}/feature_store/feature_spec.json")
        if registered_model_name:
            rid = fluent.active_run().info.run_id
            return tracking.register_model(f"runs:/{rid}/{artifact_path}", registered_model_name)
        return None

    def score_batch(self, model_uri: str, df, result_type: str = "double"):
        from ..tracking import artifacts, pyfunc
        path = artifacts.resolve(model_uri)
        sp = os.path.join(path, "feature_store", "feature_spec.json")
        if not os.path.exists(sp):
            raise ValueError(f"{model_uri} was not logged with FeatureStoreClient.log_model")
        with open(sp) as f:
            spec = json.load(f)
        ts = TrainingSet(self, df, [FeatureLookup.from_dict(d) for d in spec["feature_lookups"]], None, [])
        joined = ts._joined(df)
        cols = spec["input_columns"]
        udf = pyfunc.spark_udf(self._spark, model_uri, result_type=result_type)
        return joined.withColumn("prediction", udf(*cols))


def _union_by_name(a, b):
    """Union two frames by column name; columns missing on one side become nulls."""
    from ..sql import functions as F
    cols = list(a.columns) + [c for c in b.columns if c not in a.columns]
    sch_a, sch_b = a.schema, b.schema

    def typed(df, sch_other, c):
        if c in df.columns:
            return F.col(c)
        return F.lit(None).cast(sch_other[c].dataType).alias(c)
    aa = a.select(*[typed(a, sch_b, c) for c in cols])
    bb = b.select(*[typed(b, sch_a, c) for c in cols])
    return aa.union(bb)
