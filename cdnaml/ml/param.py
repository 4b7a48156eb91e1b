from ..models.param import Param, Params, TypeConverters  # noqa: F401
