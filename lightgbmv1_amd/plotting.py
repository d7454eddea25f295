"""Plotting helpers (reference python-package/lightgbm/plotting.py).

``plot_importance``, ``plot_split_value_histogram``, ``plot_metric`` and ``plot_tree`` draw
with matplotlib; ``create_tree_digraph`` builds a graphviz Digraph from the booster's JSON
dump.  Both libraries are optional: a function raises ImportError naming the missing
package when called without it.
"""
from copy import deepcopy

import numpy as np

from .basic import Booster
from .compat import GRAPHVIZ_INSTALLED, MATPLOTLIB_INSTALLED
from .sklearn import LGBMModel


def _require_matplotlib(what):
    if not MATPLOTLIB_INSTALLED:
        raise ImportError("You must install matplotlib to %s." % what)
    import matplotlib.pyplot as plt
    return plt


def _check_limits(lim, name):
    if not isinstance(lim, tuple) or len(lim) != 2:
        raise TypeError("%s must be a tuple of 2 elements." % name)


def _as_booster(obj):
    if isinstance(obj, LGBMModel):
        return obj.booster_
    if isinstance(obj, Booster):
        return obj
    raise TypeError("booster must be Booster or LGBMModel.")


def _new_axes(ax, figsize, dpi):
    plt = _require_matplotlib("plot")
    if ax is None:
        if figsize is not None:
            _check_limits(figsize, "figsize")
        _, ax = plt.subplots(1, 1, figsize=figsize, dpi=dpi)
    return ax


def _fmt(value, precision):
    if precision is None or isinstance(value, (int, np.integer)):
        return str(value)
    return "{0:.{1}f}".format(value, precision)


def plot_importance(booster, ax=None, height=0.2, xlim=None, ylim=None, title="Feature importance",
                    xlabel="Feature importance", ylabel="Features", importance_type="split", max_num_features=None,
                    ignore_zero=True, figsize=None, dpi=None, grid=True, precision=3, **kwargs):
    """Horizontal bar chart of feature importances ("split" counts or total "gain")."""
    _require_matplotlib("plot importance")
    booster = _as_booster(booster)
    importance = booster.feature_importance(importance_type=importance_type)
    names = booster.feature_name()
    if not len(importance):
        raise ValueError("Booster's feature_importance is empty.")
    pairs = sorted(zip(names, importance), key=lambda x: x[1])
    if ignore_zero:
        pairs = [p for p in pairs if p[1] > 0]
    if max_num_features is not None and max_num_features > 0:
        pairs = pairs[-max_num_features:]
    labels, values = zip(*pairs) if pairs else ((), ())
    ax = _new_axes(ax, figsize, dpi)
    ylocs = np.arange(len(values))
    ax.barh(ylocs, values, align="center", height=height, **kwargs)
    for x, y in zip(values, ylocs):
        ax.text(x + 1, y, _fmt(x, precision) if importance_type == "gain" else x, va="center")
    ax.set_yticks(ylocs)
    ax.set_yticklabels(labels)
    if xlim is not None:
        _check_limits(xlim, "xlim")
    else:
        xlim = (0, (max(values) if values else 1) * 1.1)
    ax.set_xlim(xlim)
    if ylim is not None:
        _check_limits(ylim, "ylim")
    else:
        ylim = (-1, len(values))
    ax.set_ylim(ylim)
    if title is not None:
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.grid(grid)
    return ax


def plot_split_value_histogram(booster, feature, bins=None, ax=None, width_coef=0.8, xlim=None, ylim=None,
                               title="Split value histogram for feature with @index/name@ @feature@",
                               xlabel="Feature split value", ylabel="Count", figsize=None, dpi=None, grid=True,
                               **kwargs):
    """Histogram of the thresholds a numerical feature was split at."""
    _require_matplotlib("plot split value histogram")
    booster = _as_booster(booster)
    hist, split_bins = booster.get_split_value_histogram(feature=feature, bins=bins, xgboost_style=False)
    if np.count_nonzero(hist) == 0:
        raise ValueError("Cannot plot split value histogram, because feature {} was not used in splitting"
                         .format(feature))
    width = width_coef * (split_bins[1] - split_bins[0])
    centred = (split_bins[:-1] + split_bins[1:]) / 2
    ax = _new_axes(ax, figsize, dpi)
    ax.bar(centred, hist, align="center", width=width, **kwargs)
    if xlim is not None:
        _check_limits(xlim, "xlim")
    else:
        r = split_bins[-1] - split_bins[0]
        xlim = (split_bins[0] - r * 0.2, split_bins[-1] + r * 0.2)
    ax.set_xlim(xlim)
    from matplotlib.ticker import MaxNLocator
    ax.yaxis.set_major_locator(MaxNLocator(integer=True))
    if ylim is not None:
        _check_limits(ylim, "ylim")
    else:
        ylim = (0, max(hist) * 1.1)
    ax.set_ylim(ylim)
    if title is not None:
        title = title.replace("@feature@", str(feature)).replace(
            "@index/name@", "name" if isinstance(feature, str) else "index")
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.grid(grid)
    return ax


def plot_metric(booster, metric=None, dataset_names=None, ax=None, xlim=None, ylim=None,
                title="Metric during training", xlabel="Iterations", ylabel="auto", figsize=None, dpi=None,
                grid=True):
    """Metric curves recorded during training (``evals_result`` dict or a fitted LGBMModel)."""
    _require_matplotlib("plot metric")
    if isinstance(booster, LGBMModel):
        eval_results = deepcopy(booster.evals_result_)
    elif isinstance(booster, dict):
        eval_results = deepcopy(booster)
    else:
        raise TypeError("booster must be dict or LGBMModel.")
    if not eval_results:
        raise ValueError("eval results cannot be empty.")
    ax = _new_axes(ax, figsize, dpi)
    names = list(eval_results.keys()) if dataset_names is None else list(dataset_names)
    if not names:
        raise ValueError("dataset_names cannot be empty.")
    first = eval_results[names[0]]
    if metric is None:
        if len(first) > 1:
            import warnings
            warnings.warn("More than one metric available, picking one to plot.")
        metric, results = next(iter(first.items()))
    else:
        if metric not in first:
            raise KeyError("No given metric in eval results.")
        results = first[metric]
    num_iteration = len(results)
    max_result, min_result = max(results), min(results)
    x = range(num_iteration)
    ax.plot(x, results, label=names[0])
    for name in names[1:]:
        results = eval_results[name][metric]
        max_result, min_result = max(max(results), max_result), min(min(results), min_result)
        ax.plot(x, results, label=name)
    ax.legend(loc="best")
    if xlim is not None:
        _check_limits(xlim, "xlim")
    else:
        xlim = (0, num_iteration)
    ax.set_xlim(xlim)
    if ylim is not None:
        _check_limits(ylim, "ylim")
    else:
        r = max_result - min_result
        ylim = (min_result - r * 0.2, max_result + r * 0.2)
    ax.set_ylim(ylim)
    if ylabel == "auto":
        ylabel = metric
    if title is not None:
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.grid(grid)
    return ax


def _tree_to_digraph(tree_info, show_info, feature_names, precision, orientation, constraints, **kwargs):
    if not GRAPHVIZ_INSTALLED:
        raise ImportError("You must install graphviz to plot tree.")
    from graphviz import Digraph

    def node_label(root, total_count):
        if "split_index" in root:
            name = "split%d" % root["split_index"]
            feat = root["split_feature"]
            fname = feature_names[feat] if feature_names is not None else "feature_%d" % feat
            op = "&#8804;" if root["decision_type"] == "<=" else "="
            label = "<B>%s</B> %s <B>%s</B>" % (fname, op, _fmt(root["threshold"], precision))
            for info in ("split_gain", "internal_value", "internal_weight", "internal_count"):
                if info in show_info:
                    label += "<br/>%s %s" % (info.split("_")[-1], _fmt(root[info], precision))
            if "data_percentage" in show_info:
                label += "<br/>%s%% of data" % _fmt(root["internal_count"] / total_count * 100, 2)
            return name, label, root
        name = "leaf%d" % root["leaf_index"]
        label = "leaf %d: <B>%s</B>" % (root["leaf_index"], _fmt(root["leaf_value"], precision))
        if "leaf_weight" in show_info:
            label += "<br/>weight: %s" % _fmt(root["leaf_weight"], precision)
        if "leaf_count" in show_info:
            label += "<br/>count: %s" % root["leaf_count"]
        if "data_percentage" in show_info:
            label += "<br/>%s%% of data" % _fmt(root["leaf_count"] / total_count * 100, 2)
        return name, label, root

    graph = Digraph(**kwargs)
    rankdir = "LR" if orientation == "horizontal" else "TB"
    graph.attr("graph", nodesep="0.05", ranksep="0.3", rankdir=rankdir)
    root = tree_info["tree_structure"]
    total = root.get("internal_count", root.get("leaf_count", 1)) or 1

    def add(node, parent=None, decision=None):
        name, label, n = node_label(node, total)
        fill = "white"
        if constraints and "split_feature" in n and constraints[n["split_feature"]] != 0:
            fill = "#ddffdd" if constraints[n["split_feature"]] == 1 else "#ffdddd"
        shape = "rectangle" if "split_index" in n else "ellipse"
        graph.node(name, label="<" + label + ">", shape=shape, style="filled", fillcolor=fill)
        if "split_index" in n:
            # the left edge is the "<=" / "in set" branch; missing values follow default_left
            add(n["left_child"], name, "yes" + (" (missing)" if n.get("default_left") else ""))
            add(n["right_child"], name, "no" + ("" if n.get("default_left") else " (missing)"))
        if parent is not None:
            graph.edge(parent, name, decision)

    add(root)
    return graph


def create_tree_digraph(booster, tree_index=0, show_info=None, precision=3, orientation="horizontal", **kwargs):
    """graphviz Digraph of one tree of the booster."""
    booster = _as_booster(booster)
    model = booster.dump_model()
    trees = model["tree_info"]
    feature_names = model.get("feature_names")
    monotone = model.get("monotone_constraints")
    if tree_index < len(trees):
        tree_info = trees[tree_index]
    else:
        raise IndexError("tree_index is out of range.")
    return _tree_to_digraph(tree_info, show_info or [], feature_names, precision, orientation, monotone, **kwargs)


def plot_tree(booster, ax=None, tree_index=0, figsize=None, dpi=None, show_info=None, precision=3,
              orientation="horizontal", **kwargs):
    """Render one tree (graphviz) into a matplotlib Axes."""
    _require_matplotlib("plot tree")
    import io

    import matplotlib.image as image
    ax = _new_axes(ax, figsize, dpi)
    graph = create_tree_digraph(booster=booster, tree_index=tree_index, show_info=show_info, precision=precision,
                                orientation=orientation, **kwargs)
    s = io.BytesIO()
    s.write(graph.pipe(format="png"))
    s.seek(0)
    ax.imshow(image.imread(s))
    ax.axis("off")
    return ax
