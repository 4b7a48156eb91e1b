"""AutoML (ML 09 - AutoML.py:35-90, Labs/ML 09L).

``automl.regress(train_df, target_col="price", primary_metric="rmse",
timeout_minutes=5, max_trials=10)`` / ``automl.classify(...)``:

1. data exploration — column statistics logged as an artifact of the
   experiment's exploration run;
2. a deterministic train / validation / test split (60/20/20, Philox keyed
   by row id, so it does not depend on the GPU count);
3. TPE search (this package's hyperopt) over model families of THIS engine —
   linear/logistic models, random forests and XGBoost-style GBDT — each trial
   a full distributed fit on the GPUs, logged as a tracking run with
   ``val_*`` / ``test_*`` metrics and the fitted pipeline (``model`` artifact,
   servable with ``pyfunc.spark_udf`` on the raw columns);
4. ``AutoMLSummary`` with ``best_trial.mlflow_run_id`` etc.
"""
from __future__ import annotations

import math
import time
from typing import List, Optional

import numpy as np

__all__ = ["regress", "classify", "AutoMLSummary", "TrialInfo"]


class TrialInfo:
    def __init__(self, run_id, metrics, params, model_description, duration, model_path):
        self.mlflow_run_id = run_id
        self.metrics = metrics
        self.params = params
        self.model_description = model_description
        self.duration = duration
        self.model_path = model_path
        self.notebook_path = None
        self.notebook_url = None

    def load_model(self):
        from ..tracking import spark as flavor
        return flavor.load_model(self.model_path)

    def __repr__(self):
        m = ", ".join(f"{k}={v:.4g}" for k, v in sorted(self.metrics.items()))
        return f"TrialInfo(run_id={self.mlflow_run_id}, model={self.model_description}, {m})"


class AutoMLSummary:
    def __init__(self, experiment, trials: List[TrialInfo], primary_metric: str, larger_better: bool,
                 exploration_run_id: Optional[str]):
        self.experiment = experiment
        self.trials = trials
        self.primary_metric = primary_metric
        self._larger = larger_better
        self.output_table_name = None
        self.exploration_run_id = exploration_run_id

    @property
    def best_trial(self) -> TrialInfo:
        if not self.trials:
            raise RuntimeError("AutoML produced no successful trial")
        return self.trials[0]

    def __repr__(self):
        return f"AutoMLSummary(experiment={self.experiment.name!r}, trials={len(self.trials)}, " \
               f"best={self.best_trial!r})"


_REG_METRICS = {"rmse": False, "mse": False, "mae": False, "r2": True}
_CLS_METRICS = {"f1": True, "accuracy": True, "roc_auc": True, "log_loss": False, "precision": True,
                "recall": True}


def _space(kind: str):
    from ..hyperopt import hp
    if kind == "regress":
        models = [
            {"type": "linear", "regParam": hp.loguniform("lin_reg", math.log(1e-4), math.log(1.0)),
             "elasticNetParam": hp.uniform("lin_en", 0.0, 1.0)},
            {"type": "rf", "maxDepth": hp.quniform("rf_depth", 3, 10, 1),
             "numTrees": hp.quniform("rf_trees", 10, 100, 10)},
            {"type": "xgb", "max_depth": hp.quniform("xgb_depth", 3, 8, 1),
             "learning_rate": hp.loguniform("xgb_lr", math.log(0.03), math.log(0.3)),
             "n_estimators": hp.quniform("xgb_n", 50, 300, 50)},
        ]
    else:
        models = [
            {"type": "logistic", "regParam": hp.loguniform("log_reg", math.log(1e-4), math.log(1.0)),
             "elasticNetParam": hp.uniform("log_en", 0.0, 1.0)},
            {"type": "rf", "maxDepth": hp.quniform("rfc_depth", 3, 10, 1),
             "numTrees": hp.quniform("rfc_trees", 10, 100, 10)},
            {"type": "xgb", "max_depth": hp.quniform("xgbc_depth", 3, 8, 1),
             "learning_rate": hp.loguniform("xgbc_lr", math.log(0.03), math.log(0.3)),
             "n_estimators": hp.quniform("xgbc_n", 50, 300, 50)},
        ]
    return hp.choice("model", models)


def _build(kind, cfg, target, cat_cols, num_cols, max_bins):
    from ..ml import Pipeline
    from ..ml.classification import LogisticRegression, RandomForestClassifier
    from ..ml.feature import Imputer, StringIndexer, VectorAssembler
    from ..ml.regression import LinearRegression, RandomForestRegressor
    from ..ml.xgboost import XgboostClassifier, XgboostRegressor
    stages = []
    idx = [f"{c}__idx" for c in cat_cols]
    if cat_cols:
        stages.append(StringIndexer(inputCols=cat_cols, outputCols=idx, handleInvalid="keep"))
    imp = [f"{c}__imp" for c in num_cols]
    if num_cols:
        stages.append(Imputer(strategy="median", inputCols=num_cols, outputCols=imp))
    stages.append(VectorAssembler(inputCols=idx + imp, outputCol="__features", handleInvalid="keep"))
    t = cfg["type"]
    common = dict(featuresCol="__features", labelCol=target)
    if t == "linear":
        m = LinearRegression(regParam=cfg["regParam"], elasticNetParam=cfg["elasticNetParam"], **common)
    elif t == "logistic":
        m = LogisticRegression(regParam=cfg["regParam"], elasticNetParam=cfg["elasticNetParam"], **common)
    elif t == "rf":
        cls = RandomForestRegressor if kind == "regress" else RandomForestClassifier
        m = cls(maxDepth=int(cfg["maxDepth"]), numTrees=int(cfg["numTrees"]), maxBins=max_bins, seed=42, **common)
    else:
        cls = XgboostRegressor if kind == "regress" else XgboostClassifier
        m = cls(max_depth=int(cfg["max_depth"]), learning_rate=float(cfg["learning_rate"]),
                n_estimators=int(cfg["n_estimators"]), random_state=42, **common)
    return Pipeline(stages=stages + [m]), t


def _metrics(kind, pred, target, prefix):
    from ..ml.evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator, \
        RegressionEvaluator
    out = {}
    if kind == "regress":
        for m in ("rmse", "mse", "mae", "r2"):
            out[f"{prefix}_{m}"] = RegressionEvaluator(labelCol=target, metricName=m).evaluate(pred)
    else:
        for m, name in (("accuracy", "accuracy"), ("f1", "f1"), ("weightedPrecision", "precision"),
                        ("weightedRecall", "recall"), ("logLoss", "log_loss")):
            try:
                out[f"{prefix}_{name}"] = MulticlassClassificationEvaluator(labelCol=target,
                                                                            metricName=m).evaluate(pred)
            except Exception:  # noqa: BLE001 - metric unsupported for this output
                pass
        try:
            out[f"{prefix}_roc_auc"] = BinaryClassificationEvaluator(labelCol=target).evaluate(pred)
        except Exception:  # noqa: BLE001 - multiclass
            pass
    return out


def _run(kind, dataset, target_col, primary_metric, timeout_minutes, max_trials, exclude_cols=None,
         experiment_dir=None, max_bins=64, **kw):
    from .. import tracking
    from ..hyperopt import Trials, fmin, tpe
    from ..sql import types as T
    from ..sql import functions as F
    table = {"regress": _REG_METRICS, "classify": _CLS_METRICS}[kind]
    if primary_metric not in table:
        raise ValueError(f"primary_metric must be one of {sorted(table)}")
    larger = table[primary_metric]
    if target_col not in dataset.columns:
        raise ValueError(f"target column {target_col!r} not in the dataset")
    excl = set(exclude_cols or []) | {target_col}
    cat_cols, num_cols = [], []
    for f in dataset.schema.fields:
        if f.name in excl:
            continue
        if isinstance(f.dataType, T.StringType) or isinstance(f.dataType, T.BooleanType):
            cat_cols.append(f.name)
        elif f.dataType.is_numeric:
            num_cols.append(f.name)
    df = dataset.withColumn(target_col, F.col(target_col).cast("double"))
    for c in num_cols:
        df = df.withColumn(c, F.col(c).cast("double"))  # Imputer needs doubles (ML 01:194-207)
    train, val, test = df.randomSplit([0.6, 0.2, 0.2], seed=42)
    for c in cat_cols:
        train = train.withColumn(c, F.col(c).cast("string"))
        val = val.withColumn(c, F.col(c).cast("string"))
        test = test.withColumn(c, F.col(c).cast("string"))
    stamp = time.strftime("%Y-%m-%d_%H:%M:%S")
    exp_name = f"{experiment_dir or '/automl'}/{target_col}-{stamp}"
    exp = tracking.set_experiment(exp_name)
    # data exploration summary
    with tracking.start_run(run_name="data-exploration") as er:
        stats = dataset.summary().toPandas()
        tracking.log_text(stats.to_markdown() if hasattr(stats, "to_markdown") else stats.to_string(),
                          "data_exploration.md")
        tracking.log_params({"target_col": target_col, "n_categorical": len(cat_cols), "n_numeric": len(num_cols)})
        explore_id = er.info.run_id
    deadline = time.time() + 60.0 * timeout_minutes
    infos: List[TrialInfo] = []
    sign = -1.0 if larger else 1.0
    sig_cols = [c for c in dataset.columns if c not in excl]

    def objective(cfg):
        if time.time() > deadline:
            return {"status": "fail", "loss": None, "failure": "timeout"}
        t0 = time.time()
        pipe, desc = _build(kind, cfg, target_col, cat_cols, num_cols, max_bins)
        with tracking.start_run(run_name=f"{desc}") as run:
            model = pipe.fit(train)
            mets = {}
            mets.update(_metrics(kind, model.transform(train), target_col, "training"))
            mets.update(_metrics(kind, model.transform(val), target_col, "val"))
            mets.update(_metrics(kind, model.transform(test), target_col, "test"))
            tracking.log_metrics(mets)
            params = {k: (v if not isinstance(v, float) else round(v, 6)) for k, v in cfg.items()}
            tracking.log_params(params)
            ex = dataset.select(*sig_cols).limit(5).toPandas()
            tracking.spark.log_model(model, "model", input_example=ex,
                                     signature=tracking.models.infer_signature(ex))
            rid = run.info.run_id
        infos.append(TrialInfo(rid, mets, params, desc, time.time() - t0, f"runs:/{rid}/model"))
        return {"status": "ok", "loss": sign * mets[f"val_{primary_metric}"]}

    fmin(objective, _space(kind), algo=tpe.suggest, max_evals=max_trials, trials=Trials(),
         rstate=np.random.default_rng(42), timeout=60.0 * timeout_minutes, catch_eval_exceptions=True)
    infos.sort(key=lambda t: sign * t.metrics[f"val_{primary_metric}"])
    return AutoMLSummary(exp, infos, primary_metric, larger, explore_id)


def regress(dataset, target_col: str, primary_metric: str = "r2", timeout_minutes: float = 120,
            max_trials: int = 20, exclude_cols=None, experiment_dir=None, **kw) -> AutoMLSummary:
    return _run("regress", dataset, target_col, primary_metric, timeout_minutes, max_trials, exclude_cols,
                experiment_dir, **kw)


def classify(dataset, target_col: str, primary_metric: str = "f1", timeout_minutes: float = 120,
             max_trials: int = 20, exclude_cols=None, experiment_dir=None, **kw) -> AutoMLSummary:
    return _run("classify", dataset, target_col, primary_metric, timeout_minutes, max_trials, exclude_cols,
                experiment_dir, **kw)
