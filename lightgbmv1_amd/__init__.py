"""lightgbmv1_amd -- MI355X-native gradient boosting with the LightGBM v3 API.

``import lightgbmv1_amd as lgb`` gives the same entry points as the reference package
(reference python-package/lightgbm/__init__.py): Dataset, Booster, train, cv, callbacks,
scikit-learn estimators and plotting helpers.  Set ``device_type='gpu'`` to train on the
MI355X learner (HIP kernels in src/device/).
"""
from .basic import Booster, Dataset, LightGBMError, device_count, device_synchronize, get_timers
from .callback import EarlyStopException, early_stopping, print_evaluation, record_evaluation, reset_parameter
from .engine import CVBooster, cv, train

try:
    from .sklearn import LGBMClassifier, LGBMModel, LGBMRanker, LGBMRegressor
except ImportError:  # pragma: no cover
    pass
try:
    from .plotting import create_tree_digraph, plot_importance, plot_metric, plot_split_value_histogram, plot_tree
except ImportError:  # pragma: no cover
    pass

__version__ = "3.0.0.99"

__all__ = ["Dataset", "Booster", "CVBooster", "LightGBMError",
           "train", "cv",
           "LGBMModel", "LGBMRegressor", "LGBMClassifier", "LGBMRanker",
           "print_evaluation", "record_evaluation", "reset_parameter", "early_stopping", "EarlyStopException",
           "plot_importance", "plot_split_value_histogram", "plot_metric", "plot_tree", "create_tree_digraph",
           "device_count", "device_synchronize", "get_timers"]
