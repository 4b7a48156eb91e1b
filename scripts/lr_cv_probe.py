"""Probe: MLE 03 logistic CV folds on cpu vs cuda (per-fold metric, iterations, objective, coefficients)."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import session_device  # noqa: E402


def run(device, root):
    import cdnaml
    import cdnaml.compat as compat
    from cdnaml.utils import datasets as D
    out = {}
    with session_device(device):
        os.environ["CDNAML_DBFS_ROOT"] = os.path.join(root, f"dbfs_{device}")
        spark = cdnaml.SparkSession.builder.getOrCreate()
        compat.install()
        ds = D.install_datasets(os.path.join(root, "datasets"), spark, scale=0.3)
        from pyspark.sql.functions import col, when
        from pyspark.sql import functions as F
        from pyspark.ml.classification import LogisticRegression
        from pyspark.ml.feature import RFormula
        from pyspark.ml.evaluation import BinaryClassificationEvaluator
        data = spark.read.format("delta").load(os.path.join(ds, "airbnb", "sf-listings",
                                                            "sf-listings-2019-03-06-clean.delta"))
        data = data.withColumn("priceClass", when(col("price") >= 150, 1.0).otherwise(0.0))
        train, _ = data.randomSplit([0.8, 0.2], seed=42)
        rf = RFormula(formula="priceClass ~ . - price", handleInvalid="skip").fit(train)
        t = rf.transform(train)
        tagged = t._with_global_uniform(42, "__u").withColumn("__fold", F.floor(F.col("__u") * 3).cast("int"))
        ev = BinaryClassificationEvaluator(labelCol="priceClass")
        for f in range(3):
            tr = tagged.filter(F.col("__fold") != f).drop("__fold")
            va = tagged.filter(F.col("__fold") == f).drop("__fold")
            for reg, en in ((0.1, 0.0), (0.1, 0.5)):
                m = LogisticRegression(labelCol="priceClass", regParam=reg, elasticNetParam=en).fit(tr)
                h = m.summary.objectiveHistory
                out[(f, reg, en)] = dict(n=tr.count(), it=m.summary.totalIterations, loss=h[-1], h=h,
                                         coef=m.coefficients.toArray(), b=m.intercept,
                                         auc=ev.evaluate(m.transform(va)))
        compat.uninstall()
        spark.stop()
    return out


if __name__ == "__main__":
    root = tempfile.mkdtemp()
    a = run("cpu", root)
    b = run("cuda", root)
    for k in a:
        x, y = a[k], b[k]
        nh = min(len(x["h"]), len(y["h"]))
        hd = [abs(x["h"][i] - y["h"][i]) / abs(x["h"][i]) for i in range(nh)]
        first = next((i for i, v in enumerate(hd) if v > 1e-12), None)
        print(k, "n", x["n"], y["n"], "it", x["it"], y["it"], "loss rel", abs(x["loss"] - y["loss"]) / abs(x["loss"]),
              "coef maxrel", float(np.max(np.abs(x["coef"] - y["coef"]) / np.maximum(np.abs(x["coef"]), 1e-3))),
              "auc", x["auc"], y["auc"], "hist first >1e-12 at", first, "of", nh,
              "hd[0..4]", [f"{v:.1e}" for v in hd[:5]], flush=True)
