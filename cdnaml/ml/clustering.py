from ..models.clustering import BisectingKMeans, KMeans, KMeansModel, KMeansSummary  # noqa: F401
