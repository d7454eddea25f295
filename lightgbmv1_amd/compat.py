"""Optional-dependency shims (reference python-package/lightgbm/compat.py).

Python 3 only.  pandas / scikit-learn / matplotlib / graphviz / datatable are optional;
the corresponding features raise a clear error when the package is missing.
"""
import json  # noqa: F401

import numpy as np  # noqa: F401

string_type = str
numeric_types = (int, float, bool)
integer_types = (int,)
range_ = range
zip_ = zip


def argc_(func):
    """Count the positional arguments of a function."""
    import inspect
    return len(inspect.signature(func).parameters)


def decode_string(bytestring):
    return bytestring.decode("utf-8")


try:
    from pandas import DataFrame as pd_DataFrame
    from pandas import Series as pd_Series
    PANDAS_INSTALLED = True
except ImportError:  # pragma: no cover
    PANDAS_INSTALLED = False

    class pd_Series(object):  # noqa: N801
        pass

    class pd_DataFrame(object):  # noqa: N801
        pass

try:
    import matplotlib  # noqa: F401
    MATPLOTLIB_INSTALLED = True
except ImportError:
    MATPLOTLIB_INSTALLED = False

try:
    import graphviz  # noqa: F401
    GRAPHVIZ_INSTALLED = True
except ImportError:
    GRAPHVIZ_INSTALLED = False

try:
    import datatable
    dt_DataTable = datatable.Frame
    DATATABLE_INSTALLED = True
except ImportError:
    DATATABLE_INSTALLED = False

    class dt_DataTable(object):  # noqa: N801
        pass

try:
    from sklearn.base import BaseEstimator, ClassifierMixin, RegressorMixin
    from sklearn.exceptions import NotFittedError
    from sklearn.model_selection import GroupKFold, StratifiedKFold
    from sklearn.preprocessing import LabelEncoder
    from sklearn.utils.class_weight import compute_sample_weight
    from sklearn.utils.multiclass import check_classification_targets
    from sklearn.utils.validation import _check_sample_weight, assert_all_finite, check_array, check_X_y
    SKLEARN_INSTALLED = True
    _LGBMModelBase = BaseEstimator
    _LGBMRegressorBase = RegressorMixin
    _LGBMClassifierBase = ClassifierMixin
    _LGBMLabelEncoder = LabelEncoder
    LGBMNotFittedError = NotFittedError
    _LGBMStratifiedKFold = StratifiedKFold
    _LGBMGroupKFold = GroupKFold
    import inspect as _inspect
    if "ensure_all_finite" in _inspect.signature(check_array).parameters:  # scikit-learn >= 1.6
        def _finite_kw(kw):
            if "force_all_finite" in kw:
                kw["ensure_all_finite"] = kw.pop("force_all_finite")
            return kw

        def _LGBMCheckXY(*args, **kw):  # noqa: N802
            return check_X_y(*args, **_finite_kw(kw))

        def _LGBMCheckArray(*args, **kw):  # noqa: N802
            return check_array(*args, **_finite_kw(kw))
    else:
        _LGBMCheckXY = check_X_y
        _LGBMCheckArray = check_array
    _LGBMCheckSampleWeight = _check_sample_weight
    _LGBMAssertAllFinite = assert_all_finite
    _LGBMCheckClassificationTargets = check_classification_targets
    _LGBMComputeSampleWeight = compute_sample_weight
except ImportError:  # pragma: no cover
    SKLEARN_INSTALLED = False
    _LGBMModelBase = object
    _LGBMClassifierBase = object
    _LGBMRegressorBase = object
    _LGBMLabelEncoder = None
    LGBMNotFittedError = ValueError
    _LGBMStratifiedKFold = None
    _LGBMGroupKFold = None
    _LGBMCheckXY = None
    _LGBMCheckArray = None
    _LGBMCheckSampleWeight = None
    _LGBMAssertAllFinite = None
    _LGBMCheckClassificationTargets = None
    _LGBMComputeSampleWeight = None
