"""Course harness parity: compat imports, synthetic datasets, classroom helpers, dbutils
(Labs/ML 00L end to end)."""
import os
import sys

import numpy as np
import pytest

from cdnaml.utils import Classroom, dbutils, to_hash
from cdnaml.utils import datasets as D


def test_spark_hash_matches_course_expected_hashes(spark):
    # Labs/ML 00L:145-146 expected constants, produced by Spark's abs(hash(str(answer)))
    assert to_hash(spark, "8") == 1276280174
    assert to_hash(spark, "100000") == 972882115


def test_compat_aliases(spark):
    import cdnaml.compat as compat
    installed = compat.install()
    try:
        assert "pyspark.ml.regression" in installed
        from pyspark.ml.regression import RandomForestRegressor  # noqa: F401
        from pyspark.sql.functions import col, translate  # noqa: F401
        from pyspark.sql import SparkSession
        import mlflow
        import mlflow.sklearn  # noqa: F401
        from mlflow.tracking import MlflowClient  # noqa: F401
        from mlflow.models.signature import infer_signature  # noqa: F401
        from hyperopt import fmin, tpe, hp, SparkTrials  # noqa: F401
        from sparkdl.xgboost import XgboostRegressor  # noqa: F401
        from delta.tables import DeltaTable  # noqa: F401
        import databricks.koalas as ks  # noqa: F401
        from databricks import automl, feature_store  # noqa: F401
        from databricks.feature_store import FeatureLookup, feature_table  # noqa: F401
        assert SparkSession.builder.getOrCreate() is spark
        assert mlflow.pyspark.ml.autolog is not None
    finally:
        compat.uninstall()
    assert "pyspark" not in sys.modules or not sys.modules["pyspark"].__name__.startswith("cdnaml")


def test_dbutils_fs(tmp_path, monkeypatch):
    monkeypatch.setenv("CDNAML_DBFS_ROOT", str(tmp_path))
    dbutils.fs.mkdirs("dbfs:/user/a/dir")
    dbutils.fs.put("dbfs:/user/a/dir/x.txt", "hello", overwrite=True)
    assert dbutils.fs.head("/dbfs/user/a/dir/x.txt") == "hello"
    names = [f.name for f in dbutils.fs.ls("dbfs:/user/a")]
    assert names == ["dir/"]
    dbutils.fs.cp("dbfs:/user/a/dir", "dbfs:/user/b", recurse=True)
    assert dbutils.fs.ls("dbfs:/user/b")[0].size == 5
    with pytest.raises(IOError):
        dbutils.fs.rm("dbfs:/user/a", False)
    assert dbutils.fs.rm("dbfs:/user/a", True)
    dbutils.widgets.text("reinstall", "false")
    assert dbutils.widgets.get("reinstall") == "false"


def test_generators_have_course_schemas():
    raw = D.airbnb_raw(n=500)
    assert set(D.KEEP) <= set(raw.columns)
    assert raw.price.str.startswith("$").all()
    clean = D.airbnb_clean(raw)
    assert len([c for c in clean.columns if c.endswith("_na")]) == 10
    assert clean.neighbourhood_cleansed.nunique() > 32  # forces maxBins=40 (ML 06:110)
    assert clean.price.max() <= 10000 and (clean.price > 0).all()
    m = D.airbnb_mlflow_csv(clean)
    assert str(m.neighbourhood_cleansed.dtype) == "int64" and "zipcode" in m.columns
    # ML 12:131 is the schema after .drop(["zipcode"])
    assert list(m.drop(["zipcode"], axis=1).columns[:4]) == ["host_total_listings_count", "neighbourhood_cleansed",
                                                          "latitude", "longitude"]
    p = D.people_with_dups(n_unique=1000, n_dups=30)
    assert len(p) == 1030
    key = p.firstName.str.lower() + p.middleName.str.lower() + p.lastName.str.lower() + \
        p.ssn.str.replace("-", "") + p.birthDate
    assert key.nunique() == 1000
    r, mv = D.movielens(n_users=100, n_movies=80, n_ratings=3000)
    assert set(r.columns) == {"userId", "movieId", "rating"} and set(mv.columns) == {"ID", "title"}
    assert r.rating.between(1, 5).all()
    c = D.covid_time()
    assert list(c.columns) == ["date", "time", "test", "negative", "confirmed", "released", "deceased"]
    assert (np.diff(c.confirmed) >= 0).all()


def test_iot_generator(spark):
    df = D.iot(spark, 1000)
    assert df.columns == ["record_id", "device_id", "feature_1", "feature_2", "feature_3", "label"]
    assert df.select("device_id").distinct().count() == 10


def test_install_datasets_tree(spark, tmp_path):
    root = D.install_datasets(str(tmp_path / "datasets"), spark, scale=0.03)
    sf = os.path.join(root, "airbnb", "sf-listings")
    for rel in ("sf-listings-2019-03-06.csv", "sf-listings-2019-03-06-clean.parquet",
                "sf-listings-2019-03-06-clean.delta/_delta_log", "airbnb-cleaned-mlflow.csv",
                "models/sf-listings-2019-03-06/pipeline_model/metadata"):
        assert os.path.exists(os.path.join(sf, rel)), rel
    parts = [f for f in os.listdir(os.path.join(sf, "sf-listings-2019-03-06-clean-100p.parquet"))
             if f.endswith(".parquet")]
    assert len(parts) == 100
    raw = spark.read.csv(os.path.join(sf, "sf-listings-2019-03-06.csv"), header="true", inferSchema="true",
                         multiLine="true", escape='"')
    assert "description" in raw.columns and dict(raw.dtypes)["price"] == "string"
    from cdnaml.ml import PipelineModel
    pm = PipelineModel.load(os.path.join(sf, "models/sf-listings-2019-03-06/pipeline_model"))
    df = spark.read.format("delta").load(os.path.join(sf, "sf-listings-2019-03-06-clean.delta"))
    assert pm.transform(df).select("prediction").count() == df.count()
    assert os.path.exists(os.path.join(root, "movielens", "ratings.parquet"))
    assert os.path.exists(os.path.join(root, "COVID", "coronavirusdataset", "Time.csv"))


def test_dedup_lab_with_classroom(spark, tmp_path, monkeypatch):
    """Labs/ML 00L end to end on the synthetic people file, validated with the lab's own hashes
    (scaled: 1,000 unique people; the full-size check uses the same code path)."""
    from cdnaml.sql.functions import col, lower, translate
    monkeypatch.setenv("CDNAML_DBFS_ROOT", str(tmp_path))
    cr = Classroom(spark, lesson="ML 00L", install=False)
    ddir = os.path.join(str(tmp_path), "people")
    os.makedirs(ddir)
    D.people_with_dups(n_unique=100000, n_dups=3000).to_csv(os.path.join(ddir, "people-with-dups.txt"), sep=":",
                                                            index=False)
    df = spark.read.csv(os.path.join(ddir, "people-with-dups.txt"), header=True, sep=":", inferSchema=True)
    assert df.count() == 103000
    spark.conf.set("spark.sql.shuffle.partitions", 8)
    dedup = (df.select(col("*"), lower(col("firstName")).alias("lcFirstName"),
                       lower(col("lastName")).alias("lcLastName"), lower(col("middleName")).alias("lcMiddleName"),
                       translate(col("ssn"), "-", "").alias("ssnNums"))
             .dropDuplicates(["lcFirstName", "lcMiddleName", "lcLastName", "ssnNums", "gender", "birthDate",
                              "salary"])
             .drop("lcFirstName", "lcMiddleName", "lcLastName", "ssnNums"))
    dest = cr.working_dir + "/people.parquet"
    dedup.write.mode("overwrite").parquet(dest.replace("dbfs:/", str(tmp_path) + "/"))
    part_files = len([f for f in dbutils.fs.ls(dest) if f.path.endswith(".parquet")])
    final_count = spark.read.parquet(dest.replace("dbfs:/", str(tmp_path) + "/")).count()
    assert cr.validate_your_answer("01 Parquet File Exists", 1276280174, part_files)
    assert cr.validate_your_answer("02 Expected 100000 Records", 972882115, final_count)


def test_validate_schema_and_all_done(spark, tmp_path, monkeypatch):
    """H3 validateYourSchema (UTIL:175-194) and H7 allDone (UTIL:297-351)."""
    monkeypatch.setenv("CDNAML_DBFS_ROOT", str(tmp_path))
    cr = Classroom(spark, lesson="ML 01", install=False)
    df = spark.createDataFrame([(1.0, "a")], ["price", "city"])
    assert cr.validateYourSchema("01 schema", df, "price", "double")
    assert cr.validateYourSchema("02 schema", df, "city")
    assert not cr.validateYourSchema("03 schema", df, "city", "double")
    assert not cr.validateYourSchema("04 schema", df, "missing", "double")
    assert cr.test_results["03 schema contains city:double"] == {"passed": False, "answer": "city:string"}
    assert cr.test_results["04 schema"]["answer"] == "-not found-"
    spark.conf.set("com.databricks.training.suppress.hidden_fn", "true")
    html = cr.allDone({"username": ("v", cr.username, "your user name"),
                       "validateYourAnswer": ("f", "what, expectedHash, answer", "checks an answer"),
                       "hidden_fn": ("f", "x", "not shown"),
                       cr.database: ("d", cr.database, "your database")})
    assert "validateYourAnswer" in html and "username" in html and cr.database in html
    assert "hidden_fn" not in html and html.endswith("All done!")


def test_one_dbfs_namespace(tmp_path, monkeypatch):
    """dbfs:/x, /dbfs/x, file:/dbfs/x and file:///dbfs/x are one file for spark.read/write, Delta, dbutils and
    pandas (Includes/Reset.py:11; ML 05:69); a dbfs: URI never lands on the host root."""
    import pandas as pd

    import cdnaml
    from cdnaml.sql.readwriter import _strip_dbfs
    from cdnaml.utils.dbutils import dbutils, to_local
    from cdnaml.utils.notebook import mount_dbfs_fuse, unmount_dbfs_fuse

    root = str(tmp_path / "dbfs")
    monkeypatch.setenv("CDNAML_DBFS_ROOT", root)
    for p in ("dbfs:/user/a/x.csv", "dbfs:user/a/x.csv", "/dbfs/user/a/x.csv", "file:/dbfs/user/a/x.csv",
              "file:///dbfs/user/a/x.csv"):
        assert to_local(p) == os.path.join(root, "user/a/x.csv"), p
        assert _strip_dbfs(p) == to_local(p)
    assert to_local("file:///tmp/q") == "/tmp/q" and to_local("/tmp/q") == "/tmp/q"
    with pytest.raises(ValueError):
        to_local("dbfs:/../../etc/passwd")
    spark = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(tmp_path / "wh")).getOrCreate()
    df = spark.createDataFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0]}))
    df.write.mode("overwrite").parquet("dbfs:/user/a/t.parquet")
    assert os.path.isdir(os.path.join(root, "user/a/t.parquet"))
    assert spark.read.parquet("/dbfs/user/a/t.parquet").count() == 3
    assert any(f.name.endswith(".parquet") for f in dbutils.fs.ls("dbfs:/user/a/t.parquet"))
    df.write.format("delta").mode("overwrite").save("dbfs:/user/a/d")
    assert spark.read.format("delta").load("file:/dbfs/user/a/d").count() == 3
    assert mount_dbfs_fuse()
    try:
        pd.DataFrame({"b": [1, 2]}).to_csv("/dbfs/user/a/p.csv", index=False)
        assert pd.read_csv("dbfs:/user/a/p.csv".replace("dbfs:/", "/dbfs/")).b.sum() == 3
        assert spark.read.csv("dbfs:/user/a/p.csv", header=True).count() == 2
    finally:
        unmount_dbfs_fuse()
    assert not hasattr(pd.read_csv, "__wrapped__")
    spark.stop()


def test_structfield_spark_equality_and_hash():
    """Labs/ML 05L:257 takes set(a.schema.fields) ^ set(b.schema.fields); Spark compares nullable/metadata."""
    from cdnaml.sql import types as T

    a = T.StructType([T.StructField("x", T.DoubleType()), T.StructField("y", T.StringType())])
    b = T.StructType([T.StructField("x", T.DoubleType()), T.StructField("z", T.LongType())])
    assert {f.name for f in set(a.fields) ^ set(b.fields)} == {"y", "z"}
    assert T.StructField("x", T.DoubleType(), True) != T.StructField("x", T.DoubleType(), False)
    assert T.StructField("x", T.DoubleType(), metadata={"k": 1}) != T.StructField("x", T.DoubleType())
    assert hash(T.StructField("x", T.DoubleType())) == hash(T.StructField("x", T.DoubleType()))


def test_notebook_namespace_and_cells(tmp_path, monkeypatch):
    """The Databricks globals + Classroom-Setup names (H1/H12) and the cell splitter/runner."""
    import cdnaml
    from cdnaml.utils import notebook as N

    monkeypatch.setenv("CDNAML_DBFS_ROOT", str(tmp_path / "dbfs"))
    spark = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(tmp_path / "wh")).getOrCreate()
    ns = N.notebook_namespace(spark, lesson="unit", install=False, quiet_display=True)
    try:
        for k in ("spark", "sc", "sql", "table", "display", "displayHTML", "dbutils", "username", "userhome",
                  "datasets_dir", "working_dir", "validateYourAnswer", "toHash", "untilStreamIsReady", "FILL_IN"):
            assert k in ns, k
        assert ns["datasets_dir"].startswith("dbfs:/user/") and "@" not in ns["cleaned_username"]
        src = ("# Databricks notebook source\n# MAGIC %md # title\n\n# COMMAND ----------\n\n"
               "# MAGIC %run ./Includes/Classroom-Setup\n\n# COMMAND ----------\n\n"
               "df = spark.range(5)\ndf.createOrReplaceTempView('v')\n\n# COMMAND ----------\n\n"
               "# MAGIC %sql\n# MAGIC SELECT COUNT(*) AS c FROM v\n\n# COMMAND ----------\n\n"
               "# just a comment\n\n# COMMAND ----------\n\nassert sql('SELECT * FROM v').count() == 5\n"
               "x = 1 / 0\n")
        cells = N.split_cells(src)
        assert [c.kind for c in cells] == ["md", "run", "python", "sql", "python"]
        p = tmp_path / "nb.py"
        p.write_text(src)
        r = N.run_notebook(str(p), ns)
        assert [c.ok for c in r.cells] == [True, True, False]
        assert r.cells[-1].error.startswith("ZeroDivisionError") and r.cells[-1].line > 1
    finally:
        N.unmount_dbfs_fuse()
        spark.stop()
