"""pandas API on the engine (Koalas; ML 14 - Koalas.py:85-194)."""
import os

import numpy as np
import pandas as pd
import pytest

import cdnaml.pandas_api as ks


@pytest.fixture
def parquet_path(spark, tmp_path):
    rng = np.random.default_rng(0)
    n = 300
    pdf = pd.DataFrame({"property_type": rng.choice(["Apartment", "House", "Condo"], n, p=[.6, .3, .1]),
                        "bedrooms": rng.integers(0, 4, n).astype(float), "price": rng.uniform(50, 500, n)})
    p = os.path.join(str(tmp_path), "listings.parquet")
    spark.createDataFrame(pdf).write.parquet(p)
    return p, pdf


def test_koalas_notebook_flow(spark, parquet_path):
    path, pdf = parquet_path
    kdf = ks.read_parquet(path)
    head = kdf.head().to_pandas()
    assert list(head.index) == [0, 1, 2, 3, 4]
    ks.set_option("compute.default_index_type", "distributed-sequence")
    try:
        assert ks.get_option("compute.default_index_type") == "distributed-sequence"
        assert len(ks.read_parquet(path)) == 300
    finally:
        ks.reset_option("compute.default_index_type")
    with pytest.raises(ValueError):
        ks.set_option("compute.default_index_type", "bogus")
    df = spark.read.parquet(path)
    k1, k2 = ks.DataFrame(df), df.to_koalas()
    assert k1.shape == k2.shape == (300, 3)
    assert k2.to_spark().count() == 300
    vc = k2["property_type"].value_counts().to_pandas()
    ref = pdf.property_type.value_counts()
    assert vc.to_dict() == ref.to_dict() and list(vc.index) == list(ref.index)
    ks.options.plotting.backend = "matplotlib"
    assert ks.options.plotting.backend == "matplotlib"
    ax = k2[["bedrooms", "price"]].plot.hist(x="bedrooms", y="price", bins=20)
    assert ax is not None
    g = k2.filter(items=["bedrooms", "price"])
    assert list(g.columns) == ["bedrooms", "price"]
    kdf = k2
    distinct = ks.sql("select distinct(property_type) from {kdf}").to_pandas()
    assert set(distinct.property_type) == {"Apartment", "House", "Condo"}


def test_koalas_ops_match_pandas(spark, parquet_path):
    path, pdf = parquet_path
    k = ks.read_parquet(path)
    np.testing.assert_allclose(k.price.mean(), pdf.price.mean())
    np.testing.assert_allclose(k.describe().loc["mean", "price"], pdf.price.mean())
    gm = k.groupby("property_type").mean().to_pandas()
    np.testing.assert_allclose(gm.loc["House", "price"], pdf[pdf.property_type == "House"].price.mean())
    k["p2"] = k.price * 2 + 1
    np.testing.assert_allclose(k.p2.to_numpy(), pdf.price.to_numpy() * 2 + 1)
    assert k[k.price > 400].shape[0] == int((pdf.price > 400).sum())
    top = k.sort_values("price", ascending=False).head(3).to_pandas()
    np.testing.assert_allclose(top.price.values, np.sort(pdf.price.values)[::-1][:3])
    sl = k.iloc[10:13].to_pandas()
    np.testing.assert_allclose(sl.price.values, pdf.price.values[10:13])
    fp = ks.from_pandas(pd.DataFrame({"a": [1, 2, 3]}, index=[10, 20, 30]))
    assert list(fp.to_pandas().index) == [10, 20, 30]
    assert fp.a.str is not None and k.property_type.str.lower().to_pandas().iloc[0].islower()
