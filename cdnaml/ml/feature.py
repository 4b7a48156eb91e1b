from ..models.feature import *  # noqa: F401,F403
from ..models.feature import (Bucketizer, Imputer, ImputerModel, IndexToString, MinMaxScaler,  # noqa: F401
                              MinMaxScalerModel, Normalizer, OneHotEncoder, OneHotEncoderModel, PCA, PCAModel,
                              QuantileDiscretizer, RFormula, RFormulaModel, SQLTransformer, StandardScaler,
                              StandardScalerModel, StringIndexer, StringIndexerModel, VectorAssembler)
