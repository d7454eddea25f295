"""Single source of truth for every training / IO / predict parameter.

The generator ``tools/gen_params.py`` turns this table into:
  * ``include/lgbm_amd/config_fields.inc``  (C++ struct members)
  * ``src/config/config_auto.cpp``          (alias table, typed parser with range checks,
                                             model-file "parameters:" serializer)
  * ``lightgbmv1_amd/utils/param_table.py`` (Python alias table)
  * ``docs/Parameters.md``                  (reference documentation)

Every parameter name and alias accepted by the reference is listed here
(reference: include/LightGBM/config.h:84-988, src/io/config_auto.cpp:10-170).
Parameters marked ``save=False`` are not written to the model's
``parameters:`` section (the reference omits the task/IO-only keys there,
src/io/config_auto.cpp:616-721).  New MI355X-specific parameters are additive
and documented with ``[new]``.
"""

# (name, ctype, default, aliases, checks, save, doc)
#   ctype: int | double | bool | string | vint | vint8 | vdouble | vstring | size_t
#   checks: list of (op, value) pairs, e.g. [(">=", 0)]
P = []


def p(name, ctype, default, aliases=(), checks=(), save=True, doc="", section="core"):
    P.append(dict(name=name, ctype=ctype, default=default, aliases=list(aliases),
                  checks=list(checks), save=save, doc=doc, section=section))


# ---------------------------------------------------------------- core
S = "core"
p("config", "string", "", ["config_file"], save=False, doc="path of config file", section=S)
p("task", "string", "train", ["task_type"], save=False,
  doc="train | predict | convert_model | refit", section=S)
p("objective", "string", "regression", ["objective_type", "app", "application"], save=False,
  doc="regression, regression_l1, huber, fair, poisson, quantile, mape, gamma, tweedie, "
      "binary, multiclass, multiclassova, cross_entropy, cross_entropy_lambda, lambdarank, rank_xendcg",
  section=S)
p("boosting", "string", "gbdt", ["boosting_type", "boost"], save=False, doc="gbdt | rf | dart | goss",
  section=S)
p("data", "string", "", ["train", "train_data", "train_data_file", "data_filename"], doc="training data path",
  section=S)
p("valid", "vstring", [], ["test", "valid_data", "valid_data_file", "test_data", "test_data_file",
                           "valid_filenames"], doc="validation data paths", section=S)
p("num_iterations", "int", 100, ["num_iteration", "n_iter", "num_tree", "num_trees", "num_round",
                                 "num_rounds", "num_boost_round", "n_estimators"], [(">=", 0)],
  doc="number of boosting iterations", section=S)
p("learning_rate", "double", 0.1, ["shrinkage_rate", "eta"], [(">", 0.0)], doc="shrinkage rate", section=S)
p("num_leaves", "int", 31, ["num_leaf", "max_leaves", "max_leaf"], [(">", 1), ("<=", 131072)],
  doc="max number of leaves in one tree", section=S)
p("tree_learner", "string", "serial", ["tree", "tree_type", "tree_learner_type"], save=False,
  doc="serial | feature | data | voting", section=S)
p("num_threads", "int", 0, ["num_thread", "nthread", "nthreads", "n_jobs"], doc="host threads", section=S)
p("device_type", "string", "cpu", ["device"], save=False,
  doc="cpu | gpu (gpu = the MI355X HIP learner)", section=S)
p("seed", "int", 0, ["random_seed", "random_state"], save=False,
  doc="master seed; derives the other seeds when set", section=S)

# ---------------------------------------------------------------- learning control
S = "learning"
p("force_col_wise", "bool", False, section=S)
p("force_row_wise", "bool", False, section=S)
p("histogram_pool_size", "double", -1.0, ["hist_pool_size"], section=S,
  doc="max cache size in MB for historical histograms (<0: no limit)")
p("max_depth", "int", -1, section=S, doc="limit the max depth of the tree (<=0: no limit)")
p("min_data_in_leaf", "int", 20, ["min_data_per_leaf", "min_data", "min_child_samples"], [(">=", 0)],
  section=S)
p("min_sum_hessian_in_leaf", "double", 1e-3, ["min_sum_hessian_per_leaf", "min_sum_hessian",
                                              "min_hessian", "min_child_weight"], [(">=", 0.0)], section=S)
p("bagging_fraction", "double", 1.0, ["sub_row", "subsample", "bagging"], [(">", 0.0), ("<=", 1.0)],
  section=S)
p("pos_bagging_fraction", "double", 1.0, ["pos_sub_row", "pos_subsample", "pos_bagging"],
  [(">", 0.0), ("<=", 1.0)], section=S)
p("neg_bagging_fraction", "double", 1.0, ["neg_sub_row", "neg_subsample", "neg_bagging"],
  [(">", 0.0), ("<=", 1.0)], section=S)
p("bagging_freq", "int", 0, ["subsample_freq"], section=S)
p("bagging_seed", "int", 3, ["bagging_fraction_seed"], section=S)
p("feature_fraction", "double", 1.0, ["sub_feature", "colsample_bytree"], [(">", 0.0), ("<=", 1.0)],
  section=S)
p("feature_fraction_bynode", "double", 1.0, ["sub_feature_bynode", "colsample_bynode"],
  [(">", 0.0), ("<=", 1.0)], section=S)
p("feature_fraction_seed", "int", 2, section=S)
p("extra_trees", "bool", False, section=S)
p("extra_seed", "int", 6, section=S)
p("early_stopping_round", "int", 0, ["early_stopping_rounds", "early_stopping", "n_iter_no_change"],
  section=S)
p("first_metric_only", "bool", False, section=S)
p("max_delta_step", "double", 0.0, ["max_tree_output", "max_leaf_output"], section=S)
p("lambda_l1", "double", 0.0, ["reg_alpha"], [(">=", 0.0)], section=S)
p("lambda_l2", "double", 0.0, ["reg_lambda", "lambda"], [(">=", 0.0)], section=S)
p("min_gain_to_split", "double", 0.0, ["min_split_gain"], [(">=", 0.0)], section=S)
p("drop_rate", "double", 0.1, ["rate_drop"], [(">=", 0.0), ("<=", 1.0)], section=S)
p("max_drop", "int", 50, section=S)
p("skip_drop", "double", 0.5, [], [(">=", 0.0), ("<=", 1.0)], section=S)
p("xgboost_dart_mode", "bool", False, section=S)
p("uniform_drop", "bool", False, section=S)
p("drop_seed", "int", 4, section=S)
p("top_rate", "double", 0.2, [], [(">=", 0.0), ("<=", 1.0)], section=S)
p("other_rate", "double", 0.1, [], [(">=", 0.0), ("<=", 1.0)], section=S)
p("min_data_per_group", "int", 100, [], [(">", 0)], section=S)
p("max_cat_threshold", "int", 32, [], [(">", 0)], section=S)
p("cat_l2", "double", 10.0, [], [(">=", 0.0)], section=S)
p("cat_smooth", "double", 10.0, [], [(">=", 0.0)], section=S)
p("max_cat_to_onehot", "int", 4, [], [(">", 0)], section=S)
p("top_k", "int", 20, ["topk"], [(">", 0)], section=S)
p("monotone_constraints", "vint8", [], ["mc", "monotone_constraint"], section=S)
p("monotone_constraints_method", "string", "basic", ["monotone_constraining_method", "mc_method"],
  section=S)
p("monotone_penalty", "double", 0.0, ["monotone_splits_penalty", "ms_penalty", "mc_penalty"],
  [(">=", 0.0)], section=S)
p("feature_contri", "vdouble", [], ["feature_contrib", "fc", "fp", "feature_penalty"], section=S)
p("forcedsplits_filename", "string", "", ["fs", "forced_splits_filename", "forced_splits_file",
                                          "forced_splits"], section=S)
p("refit_decay_rate", "double", 0.9, [], [(">=", 0.0), ("<=", 1.0)], section=S)
p("cegb_tradeoff", "double", 1.0, [], [(">=", 0.0)], section=S)
p("cegb_penalty_split", "double", 0.0, [], [(">=", 0.0)], section=S)
p("cegb_penalty_feature_lazy", "vdouble", [], section=S)
p("cegb_penalty_feature_coupled", "vdouble", [], section=S)
p("path_smooth", "double", 0.0, [], [(">=", 0.0)], section=S)
p("interaction_constraints", "string", "", section=S)
p("verbosity", "int", 1, ["verbose"], section=S)
p("input_model", "string", "", ["model_input", "model_in"], save=False, section=S)
p("output_model", "string", "LightGBM_model.txt", ["model_output", "model_out"], save=False, section=S)
p("saved_feature_importance_type", "int", 0, section=S)
p("snapshot_freq", "int", -1, ["save_period"], save=False, section=S)

# ---------------------------------------------------------------- dataset
S = "dataset"
p("max_bin", "int", 255, [], [(">", 1)], section=S)
p("max_bin_by_feature", "vint", [], section=S)
p("min_data_in_bin", "int", 3, [], [(">", 0)], section=S)
p("bin_construct_sample_cnt", "int", 200000, ["subsample_for_bin"], [(">", 0)], section=S)
p("data_random_seed", "int", 1, ["data_seed"], section=S)
p("is_enable_sparse", "bool", True, ["is_sparse", "enable_sparse", "sparse"], section=S)
p("enable_bundle", "bool", True, ["is_enable_bundle", "bundle"], section=S)
p("use_missing", "bool", True, section=S)
p("zero_as_missing", "bool", False, section=S)
p("feature_pre_filter", "bool", True, section=S)
p("pre_partition", "bool", False, ["is_pre_partition"], section=S)
p("two_round", "bool", False, ["two_round_loading", "use_two_round_loading"], section=S)
p("header", "bool", False, ["has_header"], section=S)
p("label_column", "string", "", ["label"], section=S)
p("weight_column", "string", "", ["weight"], section=S)
p("group_column", "string", "", ["group", "group_id", "query_column", "query", "query_id"], section=S)
p("ignore_column", "string", "", ["ignore_feature", "blacklist"], section=S)
p("categorical_feature", "string", "", ["cat_feature", "categorical_column", "cat_column"], section=S)
p("forcedbins_filename", "string", "", section=S)
p("save_binary", "bool", False, ["is_save_binary", "is_save_binary_file"], save=False, section=S)

# ---------------------------------------------------------------- predict
S = "predict"
p("start_iteration_predict", "int", 0, save=False, section=S)
p("num_iteration_predict", "int", -1, save=False, section=S)
p("predict_raw_score", "bool", False, ["is_predict_raw_score", "predict_rawscore", "raw_score"],
  save=False, section=S)
p("predict_leaf_index", "bool", False, ["is_predict_leaf_index", "leaf_index"], save=False, section=S)
p("predict_contrib", "bool", False, ["is_predict_contrib", "contrib"], save=False, section=S)
p("predict_disable_shape_check", "bool", False, save=False, section=S)
p("pred_early_stop", "bool", False, save=False, section=S)
p("pred_early_stop_freq", "int", 10, save=False, section=S)
p("pred_early_stop_margin", "double", 10.0, save=False, section=S)
p("output_result", "string", "LightGBM_predict_result.txt",
  ["predict_result", "prediction_result", "predict_name", "prediction_name", "pred_name", "name_pred"],
  save=False, section=S)

# ---------------------------------------------------------------- convert
S = "convert"
p("convert_model_language", "string", "", save=False, section=S)
p("convert_model", "string", "gbdt_prediction.cpp", ["convert_model_file"], save=False, section=S)

# ---------------------------------------------------------------- objective
S = "objective"
p("objective_seed", "int", 5, section=S)
p("num_class", "int", 1, ["num_classes"], [(">", 0)], section=S)
p("is_unbalance", "bool", False, ["unbalance", "unbalanced_sets"], section=S)
p("scale_pos_weight", "double", 1.0, [], [(">", 0.0)], section=S)
p("sigmoid", "double", 1.0, [], [(">", 0.0)], section=S)
p("boost_from_average", "bool", True, section=S)
p("reg_sqrt", "bool", False, section=S)
p("alpha", "double", 0.9, [], [(">", 0.0)], section=S)
p("fair_c", "double", 1.0, [], [(">", 0.0)], section=S)
p("poisson_max_delta_step", "double", 0.7, [], [(">", 0.0)], section=S)
p("tweedie_variance_power", "double", 1.5, [], [(">=", 1.0), ("<", 2.0)], section=S)
p("lambdarank_truncation_level", "int", 20, [], [(">", 0)], section=S)
p("lambdarank_norm", "bool", True, section=S)
p("label_gain", "vdouble", [], section=S)

# ---------------------------------------------------------------- metric
S = "metric"
p("metric", "vstring", [], ["metrics", "metric_types"], save=False, section=S)
p("metric_freq", "int", 1, ["output_freq"], [(">", 0)], save=False, section=S)
p("is_provide_training_metric", "bool", False, ["training_metric", "is_training_metric",
                                                "train_metric"], save=False, section=S)
p("eval_at", "vint", [], ["ndcg_eval_at", "ndcg_at", "map_eval_at", "map_at"], section=S)
p("multi_error_top_k", "int", 1, [], [(">", 0)], section=S)
p("auc_mu_weights", "vdouble", [], section=S)

# ---------------------------------------------------------------- network
S = "network"
p("num_machines", "int", 1, ["num_machine"], [(">", 0)], section=S)
p("local_listen_port", "int", 12400, ["local_port", "port"], [(">", 0)], section=S)
p("time_out", "int", 120, [], [(">", 0)], section=S)
p("machine_list_filename", "string", "", ["machine_list_file", "machine_list", "mlist"], section=S)
p("machines", "string", "", ["workers", "nodes"], section=S)

# ---------------------------------------------------------------- device (reference: GPU section)
S = "device"
p("gpu_platform_id", "int", -1, section=S, doc="accepted for compatibility; ignored (HIP has no platforms)")
p("gpu_device_id", "int", -1, section=S, doc="HIP device ordinal (-1: current / LOCAL_RANK)")
p("gpu_use_dp", "bool", False, section=S, doc="accumulate device histograms in fp64")
# [new] MI355X-specific knobs
p("hist_rows_per_block", "int", 0, save=False, section=S,
  doc="[new] rows per histogram workgroup (0: auto)")
p("gpu_hist_precision", "string", "auto", save=False, section=S,
  doc="[new] device histogram precision: fx32 (per-row 32-bit fixed point (g, h) packed in one "
      "int64 word), fx64 (two int64 words, 31-bit rows; what gpu_use_dp selects) or auto (fx64 "
      "for the listwise objectives lambdarank / rank_xendcg, whose per-query gradients span a "
      "wide dynamic range, else fx32)")
p("deterministic", "bool", False, save=False, section=S,
  doc="[new] fixed-order device reductions (bitwise reproducible histograms)")
p("gpu_rccl", "bool", True, save=False, section=S,
  doc="[new] use RCCL for device collectives when a communicator is registered")
