"""Training callbacks (the callback contract of the LightGBM v3 Python API; reference
python-package/lightgbm/callback.py).

A callback is a callable taking a ``CallbackEnv`` with two attributes the training loops in
engine.py read: ``order`` (callbacks run sorted by it) and ``before_iteration`` (run before
the boosting round instead of after).  Here each callback is a small class; ``early_stopping``
raises ``EarlyStopException`` which the loops catch to truncate the model.
"""
import collections
import warnings

from .basic import _ConfigAliases


class EarlyStopException(Exception):
    """Raised by early_stopping; carries the best iteration (0-based) and its evaluation list."""

    def __init__(self, best_iteration, best_score):
        super().__init__()
        self.best_iteration = best_iteration
        self.best_score = best_score


CallbackEnv = collections.namedtuple(
    "LightGBMCallbackEnv",
    ["model", "params", "iteration", "begin_iteration", "end_iteration", "evaluation_result_list"])


def _format_eval_result(value, show_stdv=True):
    """'<data>'s <metric>: <value>[ + <stdv>]' of one (data, metric, value, higher_better[, stdv]) tuple."""
    if len(value) not in (4, 5):
        raise ValueError("Wrong metric value")
    text = "%s's %s: %g" % (value[0], value[1], value[2])
    if len(value) == 5 and show_stdv:
        text += " + %g" % value[4]
    return text


def _format_results(results, show_stdv=True):
    return "\t".join(_format_eval_result(r, show_stdv) for r in results)


class _Callback:
    order = 0
    before_iteration = False


class _PrintEvaluation(_Callback):
    order = 10

    def __init__(self, period, show_stdv):
        self.period = period
        self.show_stdv = show_stdv

    def __call__(self, env):
        rnd = env.iteration + 1
        if self.period > 0 and env.evaluation_result_list and rnd % self.period == 0:
            print("[%d]\t%s" % (rnd, _format_results(env.evaluation_result_list, self.show_stdv)))


def print_evaluation(period=1, show_stdv=True):
    """Print the evaluation results every ``period`` rounds."""
    return _PrintEvaluation(period, show_stdv)


class _RecordEvaluation(_Callback):
    order = 20

    def __init__(self, store):
        self.store = store

    def __call__(self, env):
        for data_name, metric, value in (r[:3] for r in env.evaluation_result_list):
            self.store.setdefault(data_name, collections.OrderedDict()).setdefault(metric, []).append(value)


def record_evaluation(eval_result):
    """Record the evaluation history into the dict ``eval_result``:
    ``{data_name: {metric: [value per round]}}`` (cleared first)."""
    if not isinstance(eval_result, dict):
        raise TypeError("eval_result should be a dictionary")
    eval_result.clear()
    return _RecordEvaluation(eval_result)


class _ResetParameter(_Callback):
    order = 10
    before_iteration = True

    def __init__(self, schedules):
        self.schedules = schedules

    def __call__(self, env):
        rnd = env.iteration - env.begin_iteration
        changed = {}
        for key, schedule in self.schedules.items():
            if isinstance(schedule, list):
                if len(schedule) != env.end_iteration - env.begin_iteration:
                    raise ValueError("Length of list {} has to equal to 'num_boost_round'.".format(repr(key)))
                value = schedule[rnd]
            else:
                value = schedule(rnd)
            if value != env.params.get(key, None):
                changed[key] = value
        if changed:
            env.model.reset_parameter(changed)
            env.params.update(changed)


def reset_parameter(**kwargs):
    """Reset parameters before every round: each value is a list (one entry per round) or a
    function of the round index (counted from the first round of this training call)."""
    return _ResetParameter(kwargs)


class _MetricTracker:
    """Best value so far of one (dataset, metric) entry of the evaluation list."""

    def __init__(self, higher_better):
        self.higher_better = higher_better
        self.best = None
        self.best_iter = 0
        self.best_results = None

    def offer(self, value, iteration, results):
        if self.best is None or (value > self.best if self.higher_better else value < self.best):
            self.best = value
            self.best_iter = iteration
            self.best_results = results


class _EarlyStopping(_Callback):
    order = 30

    def __init__(self, stopping_rounds, first_metric_only, verbose):
        self.stopping_rounds = stopping_rounds
        self.first_metric_only = first_metric_only
        self.verbose = verbose
        self.trackers = None
        self.enabled = True
        self.first_metric = ""

    def _start(self, env):
        self.trackers = []
        self.enabled = not any(env.params.get(a, "") == "dart" for a in _ConfigAliases.get("boosting"))
        if not self.enabled:
            warnings.warn("Early stopping is not available in dart mode")
            return
        if not env.evaluation_result_list:
            raise ValueError("For early stopping, at least one dataset and eval metric is required for evaluation")
        if self.verbose:
            print("Training until validation scores don't improve for {} rounds".format(self.stopping_rounds))
        # cv reports "<dataset> <metric>" names: the metric is the last word
        self.first_metric = env.evaluation_result_list[0][1].split(" ")[-1]
        self.trackers = [_MetricTracker(r[3]) for r in env.evaluation_result_list]

    def _stop(self, tracker, metric_words, headline):
        if self.verbose:
            print("%s\n[%d]\t%s" % (headline, tracker.best_iter + 1, _format_results(tracker.best_results)))
            if self.first_metric_only:
                print("Evaluated only: {}".format(metric_words[-1]))
        raise EarlyStopException(tracker.best_iter, tracker.best_results)

    def __call__(self, env):
        if self.trackers is None:
            self._start(env)
        if not self.enabled:
            return
        last_round = env.iteration == env.end_iteration - 1
        results = env.evaluation_result_list
        for tracker, (data_name, metric, value) in zip(self.trackers, (r[:3] for r in results)):
            tracker.offer(value, env.iteration, results)
            words = metric.split(" ")
            if self.first_metric_only and words[-1] != self.first_metric:
                continue
            # training-set entries (lgb.cv's "train ..." aggregates, the booster's own training
            # data) never trigger a stop; they only report at the last round
            on_train = (data_name == "cv_agg" and words[0] == "train") or data_name == env.model._train_data_name
            if not on_train and env.iteration - tracker.best_iter >= self.stopping_rounds:
                self._stop(tracker, words, "Early stopping, best iteration is:")
            if last_round:
                self._stop(tracker, words, "Did not meet early stopping. Best iteration is:")


def early_stopping(stopping_rounds, first_metric_only=False, verbose=True):
    """Stop training when no validation metric improved for ``stopping_rounds`` rounds (all
    metrics, or only the first with ``first_metric_only``); disabled for dart."""
    return _EarlyStopping(stopping_rounds, first_metric_only, verbose)
