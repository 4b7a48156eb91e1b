"""K16 relational operators in the device hash tables (csrc/kernels/hashagg.hip) against pandas: groupBy
aggregates over int / multi-column / string / float keys with nulls, dropDuplicates (first row of every key, in
input order), and inner / outer / semi / anti joins with unique and duplicated build keys.  Every test also
checks that the hash-table kernels ran (no silent fallback), and one forces partition overflow to check the
portable fallback gives the same answer."""
import numpy as np
import pandas as pd
import pytest
import torch

from cdnaml.ops import _lib, kernels as K, relops as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spark():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.lib()
    import cdnaml
    return cdnaml.SparkSession.builder.getOrCreate()


@pytest.fixture
def calls(monkeypatch):
    seen = {"groups": 0, "join": 0}
    hg, jt = K.hash_groups, K.join_table

    def hash_groups(*a, **k):
        seen["groups"] += 1
        return hg(*a, **k)

    def join_table(*a, **k):
        seen["join"] += 1
        return jt(*a, **k)
    monkeypatch.setattr(K, "hash_groups", hash_groups)
    monkeypatch.setattr(K, "join_table", join_table)
    return seen


@pytest.fixture(params=["local", "partitioned"])
def path(request, monkeypatch):
    """Both K16 aggregation paths: per-chunk LDS tables + merge (few keys), and the radix-partitioned tables."""
    monkeypatch.setattr(R, "LOCAL_FIRST", request.param == "local")
    return request.param


def _frame(n, seed, nkeys=5000):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=n)
    v[rng.random(n) < 0.05] = np.nan          # nulls in the value column (pandas NaN -> Spark null)
    return pd.DataFrame({"k": rng.integers(0, nkeys, n), "k2": rng.integers(-3, 4, n).astype(np.int32),
                         "s": rng.choice(["ann", "bob", "cé", None], n), "v": v,
                         "i": rng.integers(-1000, 1000, n), "id": np.arange(n)})


def test_groupby_int_key_all_table_aggregates(spark, calls, path):
    from cdnaml.sql import functions as F
    pdf = _frame(300_000, 1)
    df = spark.createDataFrame(pdf)
    got = (df.groupBy("k").agg(F.count("*").alias("n"), F.sum("v").alias("s"), F.avg("v").alias("m"),
                               F.min("v").alias("lo"), F.max("i").alias("hi"), F.count("v").alias("nv"),
                               F.sum("i").alias("si"), F.first("id").alias("f"), F.last("id").alias("l"))
           .toPandas())
    assert calls["groups"] == 1
    g = pdf.groupby("k")
    ref = pd.DataFrame({"n": g.size(), "s": g["v"].sum(), "m": g["v"].mean(), "lo": g["v"].min(),
                        "hi": g["i"].max(), "nv": g["v"].count(), "si": g["i"].sum(), "f": g["id"].first(),
                        "l": g["id"].last()}).reset_index()
    assert got["k"].tolist() == ref["k"].tolist()          # groups come out in key order
    for c in ("n", "hi", "nv", "si", "f", "l"):
        assert got[c].tolist() == ref[c].tolist(), c
    for c in ("s", "m", "lo"):
        np.testing.assert_allclose(got[c].to_numpy(float), ref[c].to_numpy(float), rtol=1e-12, atol=1e-12)


def test_groupby_generic_aggregates_use_table_group_ids(spark, calls, path):
    from cdnaml.sql import functions as F
    pdf = _frame(200_000, 2, nkeys=300)
    df = spark.createDataFrame(pdf)
    got = df.groupBy("k").agg(F.stddev("v").alias("sd"), F.countDistinct("k2").alias("nd"),
                              F.avg("i").alias("m")).toPandas()
    assert calls["groups"] == 1
    g = pdf.groupby("k")
    np.testing.assert_allclose(got["sd"].to_numpy(float), g["v"].std().to_numpy(), rtol=1e-9)
    assert got["nd"].tolist() == g["k2"].nunique().tolist()
    np.testing.assert_allclose(got["m"].to_numpy(float), g["i"].mean().to_numpy(), rtol=1e-12)


def test_groupby_multi_column_and_string_keys_with_nulls(spark, calls, path):
    from cdnaml.sql import functions as F
    pdf = _frame(250_000, 3)
    df = spark.createDataFrame(pdf)
    got = df.groupBy("s", "k2").agg(F.count("*").alias("n"), F.max("v").alias("mx")).toPandas()
    got1 = df.groupBy("s").count().toPandas()
    assert calls["groups"] == 2
    ref = pdf.groupby(["s", "k2"], dropna=False).agg(n=("v", "size"), mx=("v", "max")).reset_index()
    # Spark order: nulls first, then by value
    ref = ref.assign(_null=ref["s"].notna()).sort_values(["_null", "s", "k2"], kind="stable").drop(columns="_null")
    assert [None if x is None or x != x else x for x in got["s"]] == \
        [None if x is None or x != x else x for x in ref["s"]]
    assert got["k2"].tolist() == ref["k2"].tolist()
    assert got["n"].tolist() == ref["n"].tolist()
    np.testing.assert_allclose(got["mx"].to_numpy(float), ref["mx"].to_numpy(float), rtol=0)
    assert sorted(got1["count"].tolist()) == sorted(pdf.groupby("s", dropna=False).size().tolist())


def test_groupby_float_key_nan_negzero_null(spark, calls, path):
    """Float keys: -0.0 and 0.0 are one group, NaN is one group sorted last, null is one group sorted first."""
    from cdnaml.sql import functions as F
    rng = np.random.default_rng(4)
    n = 100_000
    x = rng.choice([0.5, -0.0, 0.0, 2.25, -7.0, 3.5], n)
    v = rng.normal(size=n)
    pdf = pd.DataFrame({"x": x, "v": v})
    df = (spark.createDataFrame(pdf)
          .withColumn("x", F.when(F.col("v") > 1.5, None).when(F.col("x") == 3.5, F.lit(float("nan")))
                      .otherwise(F.col("x"))))
    got = df.groupBy("x").agg(F.count("*").alias("n")).toPandas()
    assert calls["groups"] == 1
    null = v > 1.5
    expect = [int(null.sum())]
    for k in (-7.0, 0.0, 0.5, 2.25):
        expect.append(int(((x == k) & ~null).sum()))
    expect.append(int(((x == 3.5) & ~null).sum()))
    assert got["n"].tolist() == expect
    gx = got["x"].tolist()
    assert gx[0] is None or gx[0] != gx[0]
    assert gx[1:5] == [-7.0, 0.0, 0.5, 2.25] and gx[5] != gx[5]


def test_dropduplicates_first_rows_in_order(spark, calls, path):
    pdf = _frame(400_000, 5, nkeys=20_000)
    df = spark.createDataFrame(pdf)
    out = df.dropDuplicates(["k", "k2"])
    got = out.toPandas()
    assert calls["groups"] == 1
    assert out.rdd.getNumPartitions() == int(spark.conf.get("spark.sql.shuffle.partitions"))
    ref = pdf.drop_duplicates(["k", "k2"], keep="first")
    assert sorted(got["id"].tolist()) == ref["id"].tolist()
    # within every output partition rows keep the input order
    for part in out._plan.execute():
        assert bool((part.columns["id"].values.diff() > 0).all())
    s = df.dropDuplicates(["s"]).toPandas()
    assert sorted(s["id"].tolist()) == pdf.drop_duplicates(["s"], keep="first")["id"].tolist()


def _merge_ref(l, r, on, how):
    lk, rk = l.dropna(subset=[on]), r.dropna(subset=[on])
    m = lk.merge(rk, on=on, how="inner", suffixes=("", "_r"))
    return m


@pytest.mark.parametrize("dup", [False, True])
def test_join_matches_pandas(spark, calls, dup):
    rng = np.random.default_rng(6 + dup)
    n = 300_000
    left = pd.DataFrame({"k": rng.integers(0, 40_000, n).astype(float), "a": np.arange(n)})
    left.loc[rng.random(n) < 0.02, "k"] = np.nan                    # null keys never match
    kk = np.arange(0, 40_000, 3)
    if dup:
        kk = np.concatenate([kk, kk[::5]])
    right = pd.DataFrame({"k": kk.astype(float), "b": np.arange(len(kk))})
    L, R = spark.createDataFrame(left), spark.createDataFrame(right)
    ref = _merge_ref(left, right, "k", "inner").sort_values(["a", "b"]).reset_index(drop=True)
    got = L.join(R, on="k").toPandas()
    assert got["a"].tolist() == ref["a"].tolist() and got["b"].tolist() == ref["b"].tolist()
    assert calls["join"] >= 1
    matched = set(ref["a"])
    semi = L.join(R, on="k", how="left_semi").toPandas()
    anti = L.join(R, on="k", how="left_anti").toPandas()
    assert semi["a"].tolist() == sorted(matched)
    assert anti["a"].tolist() == [a for a in range(n) if a not in matched]
    lo = L.join(R, on="k", how="left").toPandas()
    assert len(lo) == len(ref) + (n - len(matched)) and lo["b"].isna().sum() == n - len(matched)
    fo = L.join(R, on="k", how="full").toPandas()
    rmatched = set(ref["b"])
    assert len(fo) == len(lo) + (len(right) - len(rmatched))


def test_join_two_int_keys_packed(spark, calls):
    rng = np.random.default_rng(8)
    n = 200_000
    left = pd.DataFrame({"u": rng.integers(0, 500, n), "m": rng.integers(0, 300, n).astype(np.int32),
                         "a": np.arange(n)})
    right = pd.DataFrame({"u": rng.integers(0, 500, 20_000), "m": rng.integers(0, 300, 20_000),
                          "b": np.arange(20_000)}).drop_duplicates(["u", "m"])
    got = spark.createDataFrame(left).join(spark.createDataFrame(right), on=["u", "m"]).toPandas()
    ref = left.merge(right, on=["u", "m"]).sort_values("a")
    assert calls["join"] == 1
    assert got["a"].tolist() == ref["a"].tolist() and got["b"].tolist() == ref["b"].tolist()


def test_partition_overflow_falls_back(spark, monkeypatch):
    """A table too small for its partition's keys reports overflow; the operator then takes the portable path
    and returns the same groups."""
    from cdnaml.sql import functions as F
    pdf = _frame(150_000, 9, nkeys=100_000)
    df = spark.createDataFrame(pdf)
    ref = df.groupBy("k").agg(F.sum("i").alias("s")).toPandas()
    monkeypatch.setattr(R, "_hp_shape", lambda n, na: (64, 56, 1))
    assert K.hash_groups(torch.arange(10_000, device="cuda")) is None
    got = df.groupBy("k").agg(F.sum("i").alias("s")).toPandas()
    assert got["k"].tolist() == ref["k"].tolist() and got["s"].tolist() == ref["s"].tolist()
    dd = df.dropDuplicates(["k"]).count()
    assert dd == pdf["k"].nunique()


def test_hash_groups_all_distinct_keys(spark):
    """1e6 distinct keys (every partition near its target fill) in one pass, exact counts and first rows."""
    g = torch.Generator(device="cuda").manual_seed(3)
    keys = torch.randperm(1_000_000, generator=g, device="cuda") * 7919 - (1 << 40)
    keys = torch.cat([keys, keys[:1000]])
    r = K.hash_groups(keys)
    assert r is not None and r["G"] == 1_000_000
    pos = r["pos"]
    k, c, f = r["key"][pos], r["cnt"][pos], r["first"][pos].long()
    assert torch.equal(keys[f], k)
    assert int(c.sum()) == keys.numel() and int((c == 2).sum()) == 1000


def test_gather_cols_and_bucket_compact(spark):
    """K19 multi-column gather == torch indexing for every element width (and Batch.take's null masks);
    bucket compaction == a stable numpy grouping of the kept rows by bucket."""
    g = torch.Generator(device="cuda").manual_seed(1)
    n, m = 300_000, 200_000
    cols = [torch.randint(0, 255, (n,), generator=g, device="cuda", dtype=torch.int64).to(dt)
            for dt in (torch.uint8, torch.int16, torch.int32, torch.int64, torch.float32, torch.float64)]
    cols += [torch.rand(n, generator=g, device="cuda") > 0.5] * 4
    idx = torch.randint(0, n, (m,), generator=g, device="cuda")
    got = K.gather_cols(cols + [torch.zeros((n, 3), device="cuda")], idx)
    assert got[-1] is None
    for c, o in zip(cols, got[:-1]):
        assert torch.equal(c[idx] if c.dtype != torch.bool else c[idx].view(torch.uint8), o.view(c.dtype).view(
            torch.uint8) if c.dtype == torch.bool else o)
    keep = torch.randint(0, 6, (n,), generator=g, device="cuda").to(torch.uint8)
    keep[keep == 5] = 0
    ix, counts = K.bucket_compact(keep, 4)
    k = keep.cpu().numpy()
    ref = np.concatenate([np.nonzero(k == b + 1)[0] for b in range(4)])
    assert np.array_equal(ix.cpu().numpy(), ref)
    assert counts.cpu().tolist() == [int((k == b + 1).sum()) for b in range(4)]
