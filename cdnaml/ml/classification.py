from ..models.classification import (DecisionTreeClassificationModel, DecisionTreeClassifier,  # noqa: F401
                                     GBTClassificationModel, GBTClassifier, LinearSVC, LinearSVCModel,
                                     LogisticRegression, LogisticRegressionModel, NaiveBayes, NaiveBayesModel,
                                     RandomForestClassificationModel, RandomForestClassifier)
