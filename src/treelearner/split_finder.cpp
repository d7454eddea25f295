// Sequential split search (reference semantics, see split_finder.h).
#include "split_finder.h"

#include <algorithm>
#include <cmath>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

SplitParams MakeSplitParams(const Config& cfg) {
  SplitParams p;
  p.lambda_l1 = cfg.lambda_l1;
  p.lambda_l2 = cfg.lambda_l2;
  p.max_delta_step = cfg.max_delta_step;
  p.path_smooth = cfg.path_smooth;
  p.min_gain_to_split = cfg.min_gain_to_split;
  p.min_sum_hessian_in_leaf = cfg.min_sum_hessian_in_leaf;
  p.min_data_in_leaf = cfg.min_data_in_leaf;
  p.cat_l2 = cfg.cat_l2;
  p.cat_smooth = cfg.cat_smooth;
  p.max_cat_threshold = cfg.max_cat_threshold;
  p.min_data_per_group = cfg.min_data_per_group;
  p.max_cat_to_onehot = cfg.max_cat_to_onehot;
  p.use_l1 = cfg.lambda_l1 > 0;
  p.use_max_output = cfg.max_delta_step > 0;
  p.use_smoothing = cfg.path_smooth > kEpsilon;
  p.use_mc = !cfg.monotone_constraints.empty();
  return p;
}

namespace {

inline double G(const hist_t* h, int i) { return h[2 * i]; }
inline double H(const hist_t* h, int i) { return h[2 * i + 1]; }

void ScanNumerical(const FeatureMeta& m, const SplitParams& p, const hist_t* h, double sum_g, double sum_h,
                   data_size_t num_data, ConstraintRange c, double min_gain_shift, SplitInfo* out, int rand_thr,
                   double parent_output, bool reverse, bool skip_default_bin, bool na_as_missing, bool use_rand,
                   bool* splittable) {
  const int offset = m.offset;
  double best_lg = NAN, best_lh = NAN, best_gain = kMinScore;
  data_size_t best_lc = 0;
  uint32_t best_thr = static_cast<uint32_t>(m.num_bin);
  const double cnt_factor = num_data / sum_h;
  if (reverse) {
    double rg = 0.0, rh = kEpsilon;
    data_size_t rc = 0;
    int t = m.num_bin - 1 - offset - (na_as_missing ? 1 : 0);
    const int t_end = 1 - offset;
    for (; t >= t_end; --t) {
      if (skip_default_bin && (t + offset) == static_cast<int>(m.default_bin)) continue;
      const double g = G(h, t), hh = H(h, t);
      rg += g;
      rh += hh;
      rc += static_cast<data_size_t>(common::RoundInt(hh * cnt_factor));
      if (rc < p.min_data_in_leaf || rh < p.min_sum_hessian_in_leaf) continue;
      const data_size_t lc = num_data - rc;
      if (lc < p.min_data_in_leaf) break;
      const double lh = sum_h - rh;
      if (lh < p.min_sum_hessian_in_leaf) break;
      const double lg = sum_g - rg;
      if (use_rand && t - 1 + offset != rand_thr) continue;
      const double gain = SplitGain(lg, lh, rg, rh, p.lambda_l2, p, c, m.monotone_type, lc, rc, parent_output);
      if (gain <= min_gain_shift) continue;
      *splittable = true;
      if (gain > best_gain) {
        best_lc = lc;
        best_lg = lg;
        best_lh = lh;
        best_thr = static_cast<uint32_t>(t - 1 + offset);
        best_gain = gain;
      }
    }
  } else {
    double lg = 0.0, lh = kEpsilon;
    data_size_t lc = 0;
    int t = 0;
    const int t_end = m.num_bin - 2 - offset;
    if (na_as_missing && offset == 1) {
      lg = sum_g;
      lh = sum_h - kEpsilon;
      lc = num_data;
      for (int i = 0; i < m.num_bin - offset; ++i) {
        lg -= G(h, i);
        lh -= H(h, i);
        lc -= static_cast<data_size_t>(common::RoundInt(H(h, i) * cnt_factor));
      }
      t = -1;
    }
    for (; t <= t_end; ++t) {
      if (skip_default_bin && (t + offset) == static_cast<int>(m.default_bin)) continue;
      if (t >= 0) {
        lg += G(h, t);
        lh += H(h, t);
        lc += static_cast<data_size_t>(common::RoundInt(H(h, t) * cnt_factor));
      }
      if (lc < p.min_data_in_leaf || lh < p.min_sum_hessian_in_leaf) continue;
      const data_size_t rc = num_data - lc;
      if (rc < p.min_data_in_leaf) break;
      const double rh = sum_h - lh;
      if (rh < p.min_sum_hessian_in_leaf) break;
      const double rg = sum_g - lg;
      if (use_rand && t + offset != rand_thr) continue;
      const double gain = SplitGain(lg, lh, rg, rh, p.lambda_l2, p, c, m.monotone_type, lc, rc, parent_output);
      if (gain <= min_gain_shift) continue;
      *splittable = true;
      if (gain > best_gain) {
        best_lc = lc;
        best_lg = lg;
        best_lh = lh;
        best_thr = static_cast<uint32_t>(t + offset);
        best_gain = gain;
      }
    }
  }
  if (*splittable && best_gain > out->gain + min_gain_shift) {
    out->threshold = best_thr;
    out->left_output = LeafOutputConstrained(best_lg, best_lh, p.lambda_l2, p, c, best_lc, parent_output);
    out->left_count = best_lc;
    out->left_sum_gradient = best_lg;
    out->left_sum_hessian = best_lh - kEpsilon;
    out->right_output =
        LeafOutputConstrained(sum_g - best_lg, sum_h - best_lh, p.lambda_l2, p, c, num_data - best_lc, parent_output);
    out->right_count = num_data - best_lc;
    out->right_sum_gradient = sum_g - best_lg;
    out->right_sum_hessian = sum_h - best_lh - kEpsilon;
    out->gain = best_gain - min_gain_shift;
    out->default_left = reverse;
  }
}

void FindNumerical(const FeatureMeta& m, const SplitParams& p, bool extra, const hist_t* h, double sum_g,
                   double sum_h, data_size_t num_data, ConstraintRange c, double parent_output, SplitInfo* out,
                   bool* splittable) {
  *splittable = false;
  out->monotone_type = m.monotone_type;
  const double gain_shift = LeafGain(sum_g, sum_h, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth,
                                     num_data, parent_output, p.use_l1, p.use_max_output, p.use_smoothing);
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  int rand_thr = 0;
  if (extra && m.num_bin - 2 > 0) rand_thr = m.rand.NextInt(0, m.num_bin - 2);
  auto scan = [&](bool rev, bool skip_def, bool na) {
    ScanNumerical(m, p, h, sum_g, sum_h, num_data, c, min_gain_shift, out, rand_thr, parent_output, rev, skip_def,
                  na, extra, splittable);
  };
  if (m.num_bin > 2 && m.missing_type != MissingType::None) {
    if (m.missing_type == MissingType::Zero) {
      scan(true, true, false);
      scan(false, true, false);
    } else {
      scan(true, false, true);
      scan(false, false, true);
    }
  } else {
    scan(true, false, false);
    if (m.missing_type == MissingType::NaN) out->default_left = false;
  }
}

void FindCategorical(const FeatureMeta& m, const SplitParams& p, bool extra, const hist_t* h, double sum_g,
                     double sum_h, data_size_t num_data, ConstraintRange c, double parent_output, SplitInfo* out,
                     bool* splittable) {
  *splittable = false;
  out->default_left = false;
  double best_gain = kMinScore, best_lg = 0, best_lh = 0;
  data_size_t best_lc = 0;
  double gain_shift;
  if (p.use_smoothing) {
    gain_shift = LeafGainGivenOutput(sum_g, sum_h, p.lambda_l1, p.lambda_l2, parent_output, p.use_l1);
  } else {
    gain_shift = LeafGain(sum_g, sum_h, p.lambda_l1, p.lambda_l2, p.max_delta_step, 0, num_data, 0, p.use_l1,
                          p.use_max_output, 0);
  }
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const int offset = m.offset;
  const int bin_start = 1 - offset;
  const int bin_end = m.num_bin - offset;
  double l2 = p.lambda_l2;
  const bool onehot = m.num_bin <= p.max_cat_to_onehot;
  int best_thr = -1, best_dir = 1, used_bin = -1;
  const double cnt_factor = num_data / sum_h;
  std::vector<int> sorted;
  int rand_thr = 0;
  if (onehot) {
    if (extra && bin_end - bin_start > 0) rand_thr = m.rand.NextInt(bin_start, bin_end);
    for (int t = bin_start; t < bin_end; ++t) {
      const double g = G(h, t), hh = H(h, t);
      data_size_t cnt = static_cast<data_size_t>(common::RoundInt(hh * cnt_factor));
      if (cnt < p.min_data_in_leaf || hh < p.min_sum_hessian_in_leaf) continue;
      data_size_t other = num_data - cnt;
      if (other < p.min_data_in_leaf) continue;
      double oh = sum_h - hh - kEpsilon;
      if (oh < p.min_sum_hessian_in_leaf) continue;
      double og = sum_g - g;
      if (extra && t != rand_thr) continue;
      double gain = SplitGain(og, oh, g, hh + kEpsilon, l2, p, c, 0, other, cnt, parent_output);
      if (gain <= min_gain_shift) continue;
      *splittable = true;
      if (gain > best_gain) {
        best_thr = t;
        best_lg = g;
        best_lh = hh + kEpsilon;
        best_lc = cnt;
        best_gain = gain;
      }
    }
  } else {
    for (int i = bin_start; i < bin_end; ++i) {
      if (common::RoundInt(H(h, i) * cnt_factor) >= p.cat_smooth) sorted.push_back(i);
    }
    used_bin = static_cast<int>(sorted.size());
    l2 += p.cat_l2;
    auto ctr = [&](int i) { return G(h, i) / (H(h, i) + p.cat_smooth); };
    std::stable_sort(sorted.begin(), sorted.end(), [&](int a, int b) { return ctr(a) < ctr(b); });
    const int dirs[2] = {1, -1};
    const int starts[2] = {0, used_bin - 1};
    const int max_num_cat = std::min(p.max_cat_threshold, (used_bin + 1) / 2);
    int max_threshold = std::max(std::min(max_num_cat, used_bin) - 1, 0);
    if (extra && max_threshold > 0) rand_thr = m.rand.NextInt(0, max_threshold);
    *splittable = false;
    for (int o = 0; o < 2; ++o) {
      const int dir = dirs[o];
      int pos = starts[o];
      data_size_t cnt_group = 0;
      double lg = 0.0, lh = kEpsilon;
      data_size_t lc = 0;
      for (int i = 0; i < used_bin && i < max_num_cat; ++i) {
        const int t = sorted[pos];
        pos += dir;
        const double g = G(h, t), hh = H(h, t);
        data_size_t cnt = static_cast<data_size_t>(common::RoundInt(hh * cnt_factor));
        lg += g;
        lh += hh;
        lc += cnt;
        cnt_group += cnt;
        if (lc < p.min_data_in_leaf || lh < p.min_sum_hessian_in_leaf) continue;
        data_size_t rc = num_data - lc;
        if (rc < p.min_data_in_leaf || rc < p.min_data_per_group) break;
        double rh = sum_h - lh;
        if (rh < p.min_sum_hessian_in_leaf) break;
        if (cnt_group < p.min_data_per_group) continue;
        cnt_group = 0;
        double rg = sum_g - lg;
        if (extra && i != rand_thr) continue;
        double gain = SplitGain(lg, lh, rg, rh, l2, p, c, 0, lc, rc, parent_output);
        if (gain <= min_gain_shift) continue;
        *splittable = true;
        if (gain > best_gain) {
          best_lc = lc;
          best_lg = lg;
          best_lh = lh;
          best_thr = i;
          best_gain = gain;
          best_dir = dir;
        }
      }
    }
  }
  if (*splittable) {
    out->left_output = LeafOutputConstrained(best_lg, best_lh, l2, p, c, best_lc, parent_output);
    out->left_count = best_lc;
    out->left_sum_gradient = best_lg;
    out->left_sum_hessian = best_lh - kEpsilon;
    out->right_output = LeafOutputConstrained(sum_g - best_lg, sum_h - best_lh, l2, p, c, num_data - best_lc,
                                              parent_output);
    out->right_count = num_data - best_lc;
    out->right_sum_gradient = sum_g - best_lg;
    out->right_sum_hessian = sum_h - best_lh - kEpsilon;
    out->gain = best_gain - min_gain_shift;
    out->cat_threshold.clear();
    if (onehot) {
      out->num_cat_threshold = 1;
      out->cat_threshold.push_back(static_cast<uint32_t>(best_thr + offset));
    } else {
      out->num_cat_threshold = best_thr + 1;
      for (int i = 0; i < out->num_cat_threshold; ++i) {
        int t = best_dir == 1 ? sorted[i] : sorted[used_bin - 1 - i];
        out->cat_threshold.push_back(static_cast<uint32_t>(t + offset));
      }
    }
    out->monotone_type = 0;
  }
}

}  // namespace

void FindBestThreshold(const FeatureMeta& meta, const SplitParams& p, bool extra_trees, const hist_t* hist,
                       double sum_gradient, double sum_hessian, data_size_t num_data, ConstraintRange c,
                       double parent_output, SplitInfo* out, bool* is_splittable) {
  out->default_left = true;
  out->gain = kMinScore;
  const double sh = sum_hessian + 2 * kEpsilon;
  if (meta.bin_type == BinType::Numerical) {
    FindNumerical(meta, p, extra_trees, hist, sum_gradient, sh, num_data, c, parent_output, out, is_splittable);
  } else {
    FindCategorical(meta, p, extra_trees, hist, sum_gradient, sh, num_data, c, parent_output, out, is_splittable);
  }
  out->gain *= meta.penalty;
}

void GatherInfoForThreshold(const FeatureMeta& m, const SplitParams& p, const hist_t* h, double sum_g,
                            double sum_h, uint32_t threshold, data_size_t num_data, double parent_output,
                            SplitInfo* out) {
  const int smooth = p.use_smoothing;
  if (m.bin_type == BinType::Numerical) {
    const double gain_shift = LeafGainGivenOutput(sum_g, sum_h, p.lambda_l1, p.lambda_l2, parent_output, 1);
    const double min_gain_shift = gain_shift + p.min_gain_to_split;
    const int offset = m.offset;
    double rg = 0.0, rh = kEpsilon;
    data_size_t rc = 0;
    const bool skip_default = m.missing_type == MissingType::Zero;
    const bool na = m.missing_type == MissingType::NaN;
    int t = m.num_bin - 1 - offset - (na ? 1 : 0);
    const int t_end = 1 - offset;
    const double cnt_factor = num_data / sum_h;
    for (; t >= t_end; --t) {
      if (static_cast<uint32_t>(t + offset) < threshold) break;
      if (skip_default && (t + offset) == static_cast<int>(m.default_bin)) continue;
      rg += G(h, t);
      rh += H(h, t);
      rc += static_cast<data_size_t>(common::RoundInt(H(h, t) * cnt_factor));
    }
    const double lg = sum_g - rg, lh = sum_h - rh;
    const data_size_t lc = num_data - rc;
    const double gain =
        LeafGain(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, parent_output, 1, 1, smooth) +
        LeafGain(rg, rh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc, parent_output, 1, 1, smooth);
    if (std::isnan(gain) || gain <= min_gain_shift) {
      out->gain = kMinScore;
      Log::Warning("'Forced Split' will be ignored since the gain getting worse.");
      return;
    }
    out->threshold = threshold;
    out->left_output = LeafOutputRaw(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc,
                                     parent_output, 1, 1, smooth);
    out->left_count = lc;
    out->left_sum_gradient = lg;
    out->left_sum_hessian = lh - kEpsilon;
    out->right_output = LeafOutputRaw(sum_g - lg, sum_h - lh, p.lambda_l1, p.lambda_l2, p.max_delta_step,
                                      p.path_smooth, rc, parent_output, 1, 1, smooth);
    out->right_count = num_data - lc;
    out->right_sum_gradient = sum_g - lg;
    out->right_sum_hessian = sum_h - lh - kEpsilon;
    out->gain = gain - min_gain_shift;
    out->default_left = true;
    return;
  }
  // categorical one-hot forced split
  out->default_left = false;
  const double gain_shift = LeafGainGivenOutput(sum_g, sum_h, p.lambda_l1, p.lambda_l2, parent_output, 1);
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  if (threshold >= static_cast<uint32_t>(m.num_bin) || threshold == 0) {
    out->gain = kMinScore;
    Log::Warning("Invalid categorical threshold split");
    return;
  }
  const double cnt_factor = num_data / sum_h;
  const double g = G(h, threshold - m.offset), hh = H(h, threshold - m.offset);
  const data_size_t lc = static_cast<data_size_t>(common::RoundInt(hh * cnt_factor));
  const data_size_t rc = num_data - lc;
  const double lh = hh + kEpsilon, rh = sum_h - lh, lg = g, rg = sum_g - g;
  const double gain =
      LeafGain(rg, rh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc, parent_output, 1, 1, smooth) +
      LeafGain(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, parent_output, 1, 1, smooth);
  if (std::isnan(gain) || gain <= min_gain_shift) {
    out->gain = kMinScore;
    Log::Warning("'Forced Split' will be ignored since the gain getting worse.");
    return;
  }
  out->left_output = LeafOutputRaw(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc,
                                   parent_output, 1, 1, smooth);
  out->left_count = lc;
  out->left_sum_gradient = lg;
  out->left_sum_hessian = lh - kEpsilon;
  out->right_output = LeafOutputRaw(rg, rh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc,
                                    parent_output, 1, 1, smooth);
  out->right_count = rc;
  out->right_sum_gradient = sum_g - lg;
  out->right_sum_hessian = rh - kEpsilon;
  out->gain = gain - min_gain_shift;
  out->num_cat_threshold = 1;
  out->cat_threshold.assign(1, threshold);
}

}  // namespace lgbm_amd
