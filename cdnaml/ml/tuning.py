from ..models.tuning import (CrossValidator, CrossValidatorModel, ParamGridBuilder,  # noqa: F401
                             TrainValidationSplit, TrainValidationSplitModel)
