from ..models.xgboost import XgboostClassifier, XgboostClassifierModel, XgboostRegressor, XgboostRegressorModel  # noqa: F401
