"""High-level training API: ``train`` and ``cv`` (reference python-package/lightgbm/engine.py).

Behaviour (parameter aliases overriding arguments, callback ordering, early stopping,
init_model continuation, fold construction) follows the reference; the loops drive the
native booster through basic.Booster.
"""
import collections
import copy
import warnings
from operator import attrgetter

import numpy as np

from . import callback
from .basic import Booster, Dataset, LightGBMError, _ConfigAliases, _InnerPredictor
from .compat import SKLEARN_INSTALLED, _LGBMGroupKFold, _LGBMStratifiedKFold, integer_types, string_type

_RANKING_OBJECTIVES = {"lambdarank", "rank_xendcg", "xendcg", "xe_ndcg", "xe_ndcg_mart", "xendcg_mart"}


def _normalize_params(params, fobj, num_boost_round, early_stopping_rounds):
    """Apply objective / iteration / early-stopping aliases; parameters in ``params`` win."""
    params = copy.deepcopy(params)
    if fobj is not None:
        for key in _ConfigAliases.get("objective"):
            params.pop(key, None)
        params["objective"] = "none"
    for key in _ConfigAliases.get("num_iterations"):
        if key in params:
            num_boost_round = params.pop(key)
            warnings.warn("Found `{}` in params. Will use it instead of argument".format(key))
    params["num_iterations"] = num_boost_round
    for key in _ConfigAliases.get("early_stopping_round"):
        if key in params:
            early_stopping_rounds = params.pop(key)
            warnings.warn("Found `{}` in params. Will use it instead of argument".format(key))
    params["early_stopping_round"] = early_stopping_rounds
    if num_boost_round <= 0:
        raise ValueError("num_boost_round should be greater than zero.")
    return params, num_boost_round, early_stopping_rounds


def _init_predictor(init_model, params):
    if isinstance(init_model, string_type):
        return _InnerPredictor(model_file=init_model, pred_parameter=params)
    if isinstance(init_model, Booster):
        return init_model._to_predictor(dict(init_model.params, **params))
    return None


def _split_callbacks(callbacks):
    """Return (before_iteration, after_iteration) callbacks sorted by their ``order``."""
    before = sorted((cb for cb in callbacks if getattr(cb, "before_iteration", False)), key=attrgetter("order"))
    after = sorted((cb for cb in callbacks if not getattr(cb, "before_iteration", False)), key=attrgetter("order"))
    return before, after


def _user_callbacks(callbacks):
    if callbacks is None:
        return set()
    for pos, cb in enumerate(callbacks):
        if not hasattr(cb, "order"):
            cb.order = pos - len(callbacks)
    return set(callbacks)


def _env(model, params, it, begin, end, results):
    return callback.CallbackEnv(model=model, params=params, iteration=it, begin_iteration=begin,
                                end_iteration=end, evaluation_result_list=results)


def train(params, train_set, num_boost_round=100, valid_sets=None, valid_names=None, fobj=None, feval=None,
          init_model=None, feature_name="auto", categorical_feature="auto", early_stopping_rounds=None,
          evals_result=None, verbose_eval=True, learning_rates=None, keep_training_booster=False, callbacks=None):
    """Perform the training with given parameters; returns the trained Booster."""
    params, num_boost_round, early_stopping_rounds = _normalize_params(params, fobj, num_boost_round,
                                                                       early_stopping_rounds)
    first_metric_only = params.get("first_metric_only", False)
    predictor = _init_predictor(init_model, params)
    init_iteration = predictor.num_total_iteration if predictor is not None else 0
    if not isinstance(train_set, Dataset):
        raise TypeError("Training only accepts Dataset object")
    train_set._update_params(params)._set_predictor(predictor).set_feature_name(feature_name) \
        .set_categorical_feature(categorical_feature)

    train_in_valid = False
    train_data_name = "training"
    other_valid, other_names = [], []
    if valid_sets is not None:
        if isinstance(valid_sets, Dataset):
            valid_sets = [valid_sets]
        if isinstance(valid_names, string_type):
            valid_names = [valid_names]
        for pos, vset in enumerate(valid_sets):
            if vset is train_set:  # evaluated through the training scores
                train_in_valid = True
                if valid_names is not None:
                    train_data_name = valid_names[pos]
                continue
            if not isinstance(vset, Dataset):
                raise TypeError("Training only accepts Dataset object")
            other_valid.append(vset._update_params(params).set_reference(train_set))
            has_name = valid_names is not None and len(valid_names) > pos
            other_names.append(valid_names[pos] if has_name else "valid_" + str(pos))

    cbs = _user_callbacks(callbacks)
    if verbose_eval is True:
        cbs.add(callback.print_evaluation())
    elif isinstance(verbose_eval, integer_types):
        cbs.add(callback.print_evaluation(verbose_eval))
    if early_stopping_rounds is not None and early_stopping_rounds > 0:
        cbs.add(callback.early_stopping(early_stopping_rounds, first_metric_only, verbose=bool(verbose_eval)))
    if learning_rates is not None:
        cbs.add(callback.reset_parameter(learning_rate=learning_rates))
    if evals_result is not None:
        cbs.add(callback.record_evaluation(evals_result))
    cbs_before, cbs_after = _split_callbacks(cbs)

    try:
        booster = Booster(params=params, train_set=train_set)
        if train_in_valid:
            booster.set_train_data_name(train_data_name)
        for vset, vname in zip(other_valid, other_names):
            booster.add_valid(vset, vname)
    finally:
        train_set._reverse_update_params()
        for vset in other_valid:
            vset._reverse_update_params()
    booster.best_iteration = 0

    end_iteration = init_iteration + num_boost_round
    results = []
    for it in range(init_iteration, end_iteration):
        for cb in cbs_before:
            cb(_env(booster, params, it, init_iteration, end_iteration, None))
        booster.update(fobj=fobj)
        results = []
        if valid_sets is not None:
            if train_in_valid:
                results.extend(booster.eval_train(feval))
            results.extend(booster.eval_valid(feval))
        try:
            for cb in cbs_after:
                cb(_env(booster, params, it, init_iteration, end_iteration, results))
        except callback.EarlyStopException as stop:
            booster.best_iteration = stop.best_iteration + 1
            results = stop.best_score
            break
    booster.best_score = collections.defaultdict(collections.OrderedDict)
    for dataset_name, eval_name, score, _ in results:
        booster.best_score[dataset_name][eval_name] = score
    if not keep_training_booster:
        booster.model_from_string(booster.model_to_string(), False).free_dataset()
    return booster


class CVBooster(object):
    """Auxiliary container of the per-fold boosters of ``cv``; forwards method calls to every fold."""

    def __init__(self):
        self.boosters = []
        self.best_iteration = -1

    def _append(self, booster):
        self.boosters.append(booster)

    def __getattr__(self, name):
        def forward(*args, **kwargs):
            ret = []
            for booster in self.boosters:
                ret.append(getattr(booster, name)(*args, **kwargs))
            return ret
        return forward


def _fold_indices(full_data, folds, nfold, params, seed, stratified, shuffle):
    num_data = full_data.num_data()
    if folds is not None:
        if not hasattr(folds, "__iter__") and not hasattr(folds, "split"):
            raise AttributeError("folds should be a generator or iterator of (train_idx, test_idx) tuples "
                                 "or scikit-learn splitter object with split method")
        if hasattr(folds, "split"):
            group_info = full_data.get_group()
            if group_info is not None:
                groups = np.repeat(range(len(group_info)), repeats=np.asarray(group_info, dtype=np.int32))
            else:
                groups = np.zeros(num_data, dtype=np.int32)
            return folds.split(X=np.zeros(num_data), y=full_data.get_label(), groups=groups)
        return folds
    is_ranking = any(params.get(key, "") in _RANKING_OBJECTIVES for key in _ConfigAliases.get("objective"))
    if is_ranking:
        if not SKLEARN_INSTALLED:
            raise LightGBMError("Scikit-learn is required for ranking cv.")
        group_info = np.asarray(full_data.get_group(), dtype=np.int32)
        groups = np.repeat(range(len(group_info)), repeats=group_info)
        return _LGBMGroupKFold(n_splits=nfold).split(X=np.zeros(num_data), groups=groups)
    if stratified:
        if not SKLEARN_INSTALLED:
            raise LightGBMError("Scikit-learn is required for stratified cv.")
        skf = _LGBMStratifiedKFold(n_splits=nfold, shuffle=shuffle, random_state=seed if shuffle else None)
        return skf.split(X=np.zeros(num_data), y=full_data.get_label())
    order = np.random.RandomState(seed).permutation(num_data) if shuffle else np.arange(num_data)
    step = int(num_data / nfold)
    tests = [order[i:i + step] for i in range(0, num_data, step)]
    trains = [np.concatenate([tests[j] for j in range(nfold) if j != k]) for k in range(nfold)]
    return zip(trains, tests)


def _make_n_folds(full_data, folds, nfold, params, seed, fpreproc=None, stratified=True, shuffle=True,
                  eval_train_metric=False):
    """Build one Booster per fold (train subset + valid subset)."""
    full_data = full_data.construct()
    ret = CVBooster()
    for train_idx, test_idx in _fold_indices(full_data, folds, nfold, params, seed, stratified, shuffle):
        train_part = full_data.subset(sorted(train_idx))
        valid_part = full_data.subset(sorted(test_idx))
        fold_params = params
        if fpreproc is not None:
            train_part, valid_part, fold_params = fpreproc(train_part, valid_part, params.copy())
        booster = Booster(fold_params, train_part)
        if eval_train_metric:
            booster.add_valid(train_part, "train")
        booster.add_valid(valid_part, "valid")
        ret._append(booster)
    return ret


def _agg_cv_result(raw_results, eval_train_metric=False):
    """Mean and standard deviation of each metric over the folds."""
    values = collections.OrderedDict()
    higher_better = {}
    for fold_result in raw_results:
        for data_name, metric, value, hb in fold_result:
            key = "{} {}".format(data_name, metric) if eval_train_metric else metric
            higher_better[key] = hb
            values.setdefault(key, []).append(value)
    return [("cv_agg", k, np.mean(v), higher_better[k], np.std(v)) for k, v in values.items()]


def cv(params, train_set, num_boost_round=100, folds=None, nfold=5, stratified=True, shuffle=True, metrics=None,
       fobj=None, feval=None, init_model=None, feature_name="auto", categorical_feature="auto",
       early_stopping_rounds=None, fpreproc=None, verbose_eval=None, show_stdv=True, seed=0, callbacks=None,
       eval_train_metric=False, return_cvbooster=False):
    """Perform the cross-validation; returns {'metric-mean': [...], 'metric-stdv': [...]}."""
    if not isinstance(train_set, Dataset):
        raise TypeError("Training only accepts Dataset object")
    params, num_boost_round, early_stopping_rounds = _normalize_params(params, fobj, num_boost_round,
                                                                       early_stopping_rounds)
    first_metric_only = params.get("first_metric_only", False)
    predictor = _init_predictor(init_model, params)
    if metrics is not None:
        for key in _ConfigAliases.get("metric"):
            params.pop(key, None)
        params["metric"] = metrics
    train_set._update_params(params)._set_predictor(predictor).set_feature_name(feature_name) \
        .set_categorical_feature(categorical_feature)

    history = collections.defaultdict(list)
    cvfolds = _make_n_folds(train_set, folds=folds, nfold=nfold, params=params, seed=seed, fpreproc=fpreproc,
                            stratified=stratified, shuffle=shuffle, eval_train_metric=eval_train_metric)
    cbs = _user_callbacks(callbacks)
    if early_stopping_rounds is not None and early_stopping_rounds > 0:
        cbs.add(callback.early_stopping(early_stopping_rounds, first_metric_only, verbose=False))
    if verbose_eval is True:
        cbs.add(callback.print_evaluation(show_stdv=show_stdv))
    elif isinstance(verbose_eval, integer_types):
        cbs.add(callback.print_evaluation(verbose_eval, show_stdv=show_stdv))
    cbs_before, cbs_after = _split_callbacks(cbs)

    for it in range(num_boost_round):
        for cb in cbs_before:
            cb(_env(cvfolds, params, it, 0, num_boost_round, None))
        cvfolds.update(fobj=fobj)
        agg = _agg_cv_result(cvfolds.eval_valid(feval), eval_train_metric)
        for _, key, mean, _, std in agg:
            history[key + "-mean"].append(mean)
            history[key + "-stdv"].append(std)
        try:
            for cb in cbs_after:
                cb(_env(cvfolds, params, it, 0, num_boost_round, agg))
        except callback.EarlyStopException as stop:
            cvfolds.best_iteration = stop.best_iteration + 1
            for key in history:
                history[key] = history[key][:cvfolds.best_iteration]
            break
    if return_cvbooster:
        history["cvbooster"] = cvfolds
    return dict(history)
