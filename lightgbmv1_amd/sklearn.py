"""scikit-learn estimators over the MI355X booster.

API parity with the reference's python-package/lightgbm/sklearn.py (LightGBM 3.0):
``LGBMModel`` (sklearn-style parameter names mapped onto booster parameters, ``fit`` with
eval sets / early stopping / callbacks / init_model, ``predict`` with raw / leaf /
contribution outputs, fitted attributes ``booster_``, ``best_iteration_``, ``best_score_``,
``evals_result_``, ``feature_importances_``, ``n_features_``, ``objective_``),
``LGBMRegressor``, ``LGBMClassifier`` (label encoding, ``predict_proba``, class weights)
and ``LGBMRanker`` (query groups, ``eval_at``).  Custom objectives / metrics follow the
reference calling conventions: ``objective(y_true, y_pred[, weight[, group]]) -> grad, hess``
and ``metric(y_true, y_pred[, weight[, group]]) -> (name, value, is_higher_better)``.
Pass ``device_type='gpu'`` (or ``device='gpu'``) to train on the HIP learner.
"""
import inspect

import numpy as np

from .basic import Booster, Dataset, LightGBMError, _ConfigAliases
from .compat import (SKLEARN_INSTALLED, LGBMNotFittedError, _LGBMAssertAllFinite, _LGBMCheckArray,
                     _LGBMCheckClassificationTargets, _LGBMCheckSampleWeight, _LGBMCheckXY,
                     _LGBMClassifierBase, _LGBMComputeSampleWeight, _LGBMLabelEncoder, _LGBMModelBase,
                     _LGBMRegressorBase, pd_DataFrame)
from .engine import train

_MULTI_OBJECTIVES = {"multiclass", "softmax", "multiclassova", "multiclass_ova", "ova", "ovr"}


def _n_args(func):
    return len(inspect.signature(func).parameters)


def _reshape_class_major(arr, num_data):
    """Booster buffers of multi-model objectives are [class][row]; sklearn wants [row][class]."""
    k = arr.size // num_data
    if k > 1:
        return arr.reshape(k, num_data).T
    return arr


class _ObjectiveFunctionWrapper(object):
    """Adapt a sklearn-style objective ``f(y_true, y_pred[, weight[, group]])`` to ``fobj``."""

    def __init__(self, func):
        self.func = func

    def __call__(self, preds, dataset):
        labels = dataset.get_label()
        n = _n_args(self.func)
        num_data = labels.size
        pred_view = _reshape_class_major(np.asarray(preds), num_data)
        if n == 2:
            grad, hess = self.func(labels, pred_view)
        elif n == 3:
            grad, hess = self.func(labels, pred_view, dataset.get_weight())
        elif n == 4:
            grad, hess = self.func(labels, pred_view, dataset.get_weight(), dataset.get_group())
        else:
            raise TypeError("Self-defined objective function should have 2, 3 or 4 arguments, got %d" % n)
        grad = np.asarray(grad, dtype=np.float64)
        hess = np.asarray(hess, dtype=np.float64)
        weight = dataset.get_weight()
        if grad.ndim == 2:  # multiclass: back to the booster's class-major layout
            if weight is not None:
                grad = grad * weight[:, None]
                hess = hess * weight[:, None]
            return grad.T.ravel(), hess.T.ravel()
        if weight is not None and grad.size == weight.size:
            grad = grad * weight
            hess = hess * weight
        return grad, hess


class _EvalFunctionWrapper(object):
    """Adapt a sklearn-style metric ``f(y_true, y_pred[, weight[, group]])`` to ``feval``."""

    def __init__(self, func):
        self.func = func

    def __call__(self, preds, dataset):
        labels = dataset.get_label()
        n = _n_args(self.func)
        pred_view = _reshape_class_major(np.asarray(preds), labels.size)
        if n == 2:
            return self.func(labels, pred_view)
        if n == 3:
            return self.func(labels, pred_view, dataset.get_weight())
        if n == 4:
            return self.func(labels, pred_view, dataset.get_weight(), dataset.get_group())
        raise TypeError("Self-defined eval function should have 2, 3 or 4 arguments, got %d" % n)


class LGBMModel(_LGBMModelBase):
    """Implementation of the scikit-learn API for gradient boosting on MI355X."""

    def __init__(self, boosting_type="gbdt", num_leaves=31, max_depth=-1, learning_rate=0.1, n_estimators=100,
                 subsample_for_bin=200000, objective=None, class_weight=None, min_split_gain=0.,
                 min_child_weight=1e-3, min_child_samples=20, subsample=1., subsample_freq=0,
                 colsample_bytree=1., reg_alpha=0., reg_lambda=0., random_state=None, n_jobs=-1, silent=True,
                 importance_type="split", **kwargs):
        if not SKLEARN_INSTALLED:
            raise LightGBMError("scikit-learn is required for lightgbmv1_amd.sklearn")
        self.boosting_type = boosting_type
        self.objective = objective
        self.num_leaves = num_leaves
        self.max_depth = max_depth
        self.learning_rate = learning_rate
        self.n_estimators = n_estimators
        self.subsample_for_bin = subsample_for_bin
        self.min_split_gain = min_split_gain
        self.min_child_weight = min_child_weight
        self.min_child_samples = min_child_samples
        self.subsample = subsample
        self.subsample_freq = subsample_freq
        self.colsample_bytree = colsample_bytree
        self.reg_alpha = reg_alpha
        self.reg_lambda = reg_lambda
        self.random_state = random_state
        self.n_jobs = n_jobs
        self.silent = silent
        self.importance_type = importance_type
        self.class_weight = class_weight
        self._Booster = None
        self._evals_result = None
        self._best_score = None
        self._best_iteration = None
        self._other_params = {}
        self._objective = objective
        self._class_weight = None
        self._class_map = None
        self._n_features = None
        self._n_features_in = None
        self._classes = None
        self._n_classes = None
        self.set_params(**kwargs)

    def _more_tags(self):
        return {"allow_nan": True, "X_types": ["2darray", "sparse", "1dlabels"]}

    def get_params(self, deep=True):
        params = super().get_params(deep=deep)
        params.update(self._other_params)
        return params

    def set_params(self, **params):
        for key, value in params.items():
            setattr(self, key, value)
            if hasattr(self, "_" + key):
                setattr(self, "_" + key, value)
            self._other_params[key] = value
        return self

    # ------------------------------------------------------------------ parameters
    def _default_objective(self):
        return "regression"

    def _booster_params(self):
        params = self.get_params()
        params.pop("silent", None)
        params.pop("importance_type", None)
        params.pop("n_estimators", None)
        params.pop("class_weight", None)
        if isinstance(params.get("random_state"), np.random.RandomState):
            params["random_state"] = params["random_state"].randint(np.iinfo(np.int32).max)
        for alias in _ConfigAliases.get("objective"):
            params.pop(alias, None)
        if self._n_classes is not None and self._n_classes > 2:
            for alias in _ConfigAliases.get("num_class"):
                params.pop(alias, None)
            params["num_class"] = self._n_classes
        if callable(self._objective):
            self._fobj = _ObjectiveFunctionWrapper(self._objective)
            params["objective"] = "None"
        else:
            self._fobj = None
            params["objective"] = self._objective
        # sklearn names -> booster names (the booster also accepts these as aliases)
        rename = {"boosting_type": "boosting", "min_split_gain": "min_gain_to_split",
                  "min_child_weight": "min_sum_hessian_in_leaf", "min_child_samples": "min_data_in_leaf",
                  "subsample": "bagging_fraction", "subsample_freq": "bagging_freq",
                  "colsample_bytree": "feature_fraction", "reg_alpha": "lambda_l1", "reg_lambda": "lambda_l2",
                  "random_state": "seed", "n_jobs": "num_threads", "subsample_for_bin": "bin_construct_sample_cnt"}
        out = {}
        for k, v in params.items():
            if k == "random_state" and v is None:
                continue
            out[rename.get(k, k)] = v
        if "device" in out and "device_type" not in out:
            out["device_type"] = out.pop("device")
        out["verbose"] = -1 if self.silent else out.get("verbose", 1)
        return out

    # ------------------------------------------------------------------ fit
    def fit(self, X, y, sample_weight=None, init_score=None, group=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_class_weight=None, eval_init_score=None, eval_group=None,
            eval_metric=None, early_stopping_rounds=None, verbose=True, feature_name="auto",
            categorical_feature="auto", callbacks=None, init_model=None):
        """Build a gradient boosting model from the training set (X, y)."""
        self._objective = self.objective if self.objective is not None else self._default_objective()
        params = self._booster_params()
        evals_result = {}
        # metric: eval_metric (string / list / callable) adds to the params' metric
        feval = None
        if callable(eval_metric):
            feval = _EvalFunctionWrapper(eval_metric)
            eval_metric = None
        elif isinstance(eval_metric, (list, tuple)):
            fns = [m for m in eval_metric if callable(m)]
            if fns:
                feval = [_EvalFunctionWrapper(m) for m in fns]
            eval_metric = [m for m in eval_metric if not callable(m)]
        if self._fobj is not None and "metric" not in params and not any(
                a in params for a in _ConfigAliases.get("metric")):
            params["metric"] = "None"
        original_metric = None
        for alias in _ConfigAliases.get("metric"):
            if alias in params:
                original_metric = params.pop(alias)
        if eval_metric:
            em = [eval_metric] if isinstance(eval_metric, str) else list(eval_metric)
            if original_metric is None and isinstance(self._objective, str):
                # keep the objective's default metric (objective names are metric aliases)
                original_metric = self._objective
            om = [] if original_metric is None else (
                [original_metric] if isinstance(original_metric, str) else list(original_metric))
            params["metric"] = list(dict.fromkeys(em + om))
        elif original_metric is not None:
            params["metric"] = original_metric

        if not isinstance(X, pd_DataFrame) and not hasattr(X, "tocsr"):
            _X, _y = _LGBMCheckXY(X, y, accept_sparse=True, force_all_finite=False, ensure_min_samples=2)
            if sample_weight is not None:
                sample_weight = _LGBMCheckSampleWeight(sample_weight, _X)
        else:
            _X, _y = X, y
        if self._class_weight is None:
            self._class_weight = self.class_weight
        if self._class_weight is not None:
            cw = _LGBMComputeSampleWeight(self._class_weight, _y)
            sample_weight = cw if sample_weight is None else np.multiply(sample_weight, cw)
        self._n_features = _X.shape[1]
        self._n_features_in = self._n_features

        train_set = Dataset(_X, label=_y, weight=sample_weight, group=group, init_score=init_score,
                            params=params)
        valid_sets, valid_names = [], []
        if eval_set is not None:
            if isinstance(eval_set, tuple):
                eval_set = [eval_set]

            def _pick(coll, i):
                if coll is None:
                    return None
                if isinstance(coll, dict):
                    return coll.get(i)
                return coll[i] if i < len(coll) else None

            for i, (vx, vy) in enumerate(eval_set):
                if vx is X and vy is y:
                    vs = train_set
                else:
                    vw = _pick(eval_sample_weight, i)
                    vcw = _pick(eval_class_weight, i)
                    if vcw is not None:
                        if self._class_map is not None:
                            vcw = {self._class_map[k]: v for k, v in vcw.items()}
                        extra = _LGBMComputeSampleWeight(vcw, vy)
                        vw = extra if vw is None else np.multiply(vw, extra)
                    vs = Dataset(vx, label=vy, weight=vw, group=_pick(eval_group, i),
                                 init_score=_pick(eval_init_score, i), reference=train_set, params=params)
                valid_sets.append(vs)
                name = _pick(eval_names, i)
                valid_names.append(name if name is not None else "valid_%d" % i)

        if isinstance(init_model, LGBMModel):
            init_model = init_model.booster_
        self._Booster = train(params, train_set, self.n_estimators, valid_sets=valid_sets or None,
                              valid_names=valid_names or None, fobj=self._fobj, feval=feval,
                              init_model=init_model, feature_name=feature_name,
                              categorical_feature=categorical_feature, early_stopping_rounds=early_stopping_rounds,
                              evals_result=evals_result, verbose_eval=verbose, callbacks=callbacks)
        if evals_result:
            self._evals_result = evals_result
        if early_stopping_rounds is not None and early_stopping_rounds > 0:
            self._best_iteration = self._Booster.best_iteration
        self._best_score = self._Booster.best_score
        self.fitted_ = True
        # free the training data; the booster keeps the model only
        self._Booster.free_dataset()
        return self

    # ------------------------------------------------------------------ predict
    def predict(self, X, raw_score=False, start_iteration=0, num_iteration=None, pred_leaf=False,
                pred_contrib=False, **kwargs):
        """Return the predicted value for each sample."""
        if self._n_features is None:
            raise LGBMNotFittedError("Estimator not fitted, call `fit` before exploiting the model.")
        if not isinstance(X, pd_DataFrame) and not hasattr(X, "tocsr"):
            X = _LGBMCheckArray(X, accept_sparse=True, force_all_finite=False)
        n_features = X.shape[1]
        if self._n_features != n_features:
            raise ValueError("Number of features of the model must match the input. Model n_features_ is %s and "
                             "input n_features is %s " % (self._n_features, n_features))
        return self._Booster.predict(X, raw_score=raw_score, start_iteration=start_iteration,
                                     num_iteration=num_iteration, pred_leaf=pred_leaf,
                                     pred_contrib=pred_contrib, **kwargs)

    # ------------------------------------------------------------------ fitted attributes
    def _check_fitted(self):
        if self._n_features is None:
            raise LGBMNotFittedError("No n_features found. Need to call fit beforehand.")

    @property
    def n_features_(self):
        self._check_fitted()
        return self._n_features

    @property
    def n_features_in_(self):
        self._check_fitted()
        return self._n_features_in

    @property
    def best_score_(self):
        self._check_fitted()
        return self._best_score

    @property
    def best_iteration_(self):
        self._check_fitted()
        return self._best_iteration

    @property
    def objective_(self):
        self._check_fitted()
        return self._objective

    @property
    def booster_(self):
        if self._Booster is None:
            raise LGBMNotFittedError("No booster found. Need to call fit beforehand.")
        return self._Booster

    @property
    def evals_result_(self):
        self._check_fitted()
        return self._evals_result

    @property
    def feature_importances_(self):
        self._check_fitted()
        return self._Booster.feature_importance(importance_type=self.importance_type)

    @property
    def feature_name_(self):
        self._check_fitted()
        return self._Booster.feature_name()


class LGBMRegressor(_LGBMRegressorBase, LGBMModel):
    """Gradient boosting regressor."""

    def fit(self, X, y, sample_weight=None, init_score=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_init_score=None, eval_metric=None, early_stopping_rounds=None,
            verbose=True, feature_name="auto", categorical_feature="auto", callbacks=None, init_model=None):
        return super().fit(X, y, sample_weight=sample_weight, init_score=init_score, eval_set=eval_set,
                           eval_names=eval_names, eval_sample_weight=eval_sample_weight,
                           eval_init_score=eval_init_score, eval_metric=eval_metric,
                           early_stopping_rounds=early_stopping_rounds, verbose=verbose, feature_name=feature_name,
                           categorical_feature=categorical_feature, callbacks=callbacks, init_model=init_model)


class LGBMClassifier(_LGBMClassifierBase, LGBMModel):
    """Gradient boosting classifier."""

    def _default_objective(self):
        return "binary" if (self._n_classes or 2) <= 2 else "multiclass"

    def fit(self, X, y, sample_weight=None, init_score=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_class_weight=None, eval_init_score=None, eval_metric=None,
            early_stopping_rounds=None, verbose=True, feature_name="auto", categorical_feature="auto",
            callbacks=None, init_model=None):
        _LGBMAssertAllFinite(y)
        _LGBMCheckClassificationTargets(y)
        self._le = _LGBMLabelEncoder().fit(y)
        _y = self._le.transform(y)
        self._class_map = dict(zip(self._le.classes_, self._le.transform(self._le.classes_)))
        if isinstance(self.class_weight, dict):
            self._class_weight = {self._class_map[k]: v for k, v in self.class_weight.items()}
        self._classes = self._le.classes_
        self._n_classes = len(self._classes)
        if self._n_classes > 2:
            if eval_metric in ("logloss", "binary_logloss"):
                eval_metric = "multi_logloss"
            elif eval_metric in ("error", "binary_error"):
                eval_metric = "multi_error"
        else:
            if eval_metric in ("logloss", "multi_logloss"):
                eval_metric = "binary_logloss"
            elif eval_metric in ("error", "multi_error"):
                eval_metric = "binary_error"
        if eval_set is not None:
            if isinstance(eval_set, tuple):
                eval_set = [eval_set]
            # the training pair stays identical (LGBMModel.fit reuses the training Dataset)
            eval_set = [(X, _y) if (vx is X and vy is y) else (vx, self._le.transform(vy)) for vx, vy in eval_set]
        super().fit(X, _y, sample_weight=sample_weight, init_score=init_score, eval_set=eval_set,
                    eval_names=eval_names, eval_sample_weight=eval_sample_weight, eval_class_weight=eval_class_weight,
                    eval_init_score=eval_init_score, eval_metric=eval_metric,
                    early_stopping_rounds=early_stopping_rounds, verbose=verbose, feature_name=feature_name,
                    categorical_feature=categorical_feature, callbacks=callbacks, init_model=init_model)
        return self

    def predict(self, X, raw_score=False, start_iteration=0, num_iteration=None, pred_leaf=False,
                pred_contrib=False, **kwargs):
        result = self.predict_proba(X, raw_score, start_iteration, num_iteration, pred_leaf, pred_contrib, **kwargs)
        if callable(self._objective) or raw_score or pred_leaf or pred_contrib:
            return result
        return self._le.inverse_transform(np.argmax(result, axis=1))

    def predict_proba(self, X, raw_score=False, start_iteration=0, num_iteration=None, pred_leaf=False,
                      pred_contrib=False, **kwargs):
        """Return the predicted probability for each class for each sample."""
        result = super().predict(X, raw_score, start_iteration, num_iteration, pred_leaf, pred_contrib, **kwargs)
        if callable(self._objective) and not (raw_score or pred_leaf or pred_contrib):
            return result
        if self._n_classes > 2 or raw_score or pred_leaf or pred_contrib:
            return result
        return np.vstack((1. - result, result)).transpose()

    @property
    def classes_(self):
        if self._classes is None:
            raise LGBMNotFittedError("No classes found. Need to call fit beforehand.")
        return self._classes

    @property
    def n_classes_(self):
        if self._n_classes is None:
            raise LGBMNotFittedError("No classes found. Need to call fit beforehand.")
        return self._n_classes


class LGBMRanker(LGBMModel):
    """Gradient boosting ranker (lambdarank by default)."""

    def _default_objective(self):
        return "lambdarank"

    def fit(self, X, y, sample_weight=None, init_score=None, group=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_init_score=None, eval_group=None, eval_metric=None, eval_at=(1, 2, 3, 4, 5),
            early_stopping_rounds=None, verbose=True, feature_name="auto", categorical_feature="auto",
            callbacks=None, init_model=None):
        if group is None:
            raise ValueError("Should set group for ranking task")
        if eval_set is not None:
            if eval_group is None:
                raise ValueError("Eval_group cannot be None when eval_set is not None")
            if len(eval_group) != len(eval_set if isinstance(eval_set, list) else [eval_set]):
                raise ValueError("Length of eval_group should be equal to eval_set")
            if isinstance(eval_group, dict) and any(i not in eval_group or eval_group[i] is None
                                                    for i in range(len(eval_group))) or \
                    (isinstance(eval_group, list) and any(g is None for g in eval_group)):
                raise ValueError("Should set group for all eval datasets for ranking task; "
                                 "if you use dict, the index should start from 0")
        self._eval_at = eval_at
        self._other_params["eval_at"] = list(eval_at)
        self.eval_at = list(eval_at)
        super().fit(X, y, sample_weight=sample_weight, init_score=init_score, group=group, eval_set=eval_set,
                    eval_names=eval_names, eval_sample_weight=eval_sample_weight, eval_init_score=eval_init_score,
                    eval_group=eval_group, eval_metric=eval_metric, early_stopping_rounds=early_stopping_rounds,
                    verbose=verbose, feature_name=feature_name, categorical_feature=categorical_feature,
                    callbacks=callbacks, init_model=init_model)
        return self


__all__ = ["LGBMModel", "LGBMRegressor", "LGBMClassifier", "LGBMRanker"]
