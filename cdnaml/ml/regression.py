from ..models.regression import (DecisionTreeRegressionModel, DecisionTreeRegressor, GBTRegressionModel,  # noqa: F401
                                 GBTRegressor, IsotonicRegression, IsotonicRegressionModel, LinearRegression,
                                 LinearRegressionModel, RandomForestRegressionModel, RandomForestRegressor)
