// Test support of the device learner: read back the state the last device-grown tree left
// in HBM (leaf partitions, raw fixed-point histogram slots, the packed per-row (g, h), the
// fixed-point scales) and check every leaf's device best split against the CPU split finder
// (src/treelearner/split_finder.cpp, the sequential formulation of reference
// feature_histogram.hpp) run on the same dequantised histogram.  Used by
// tests/test_gpu_kernels.py through LGBM_AMD_BoosterDevice* in the C API; nothing here runs
// during training.
#include <hip/hip_runtime.h>

#include <cmath>
#include <sstream>

#include "gpu_tree_learner.h"
#include "lgbm_amd/log.h"

#define HIPCHECK(x)                                                                               \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

namespace lgbm_amd {

namespace {
// JSON number (non-finite values as null)
std::string Num(double v) {
  if (!std::isfinite(v)) return "null";
  std::ostringstream o;
  o.precision(17);
  o << v;
  return o.str();
}
// whether the split that created `leaf` histogrammed / scanned its children: not for the
// tree's last split, nor when both children are too small to split or at max_depth (the
// skip rule of StepChildren in src/device/device_common.h)
bool LeafScanned(const Tree* tree, int leaf, const Config& cfg) {
  if (tree->num_leaves() <= 1) return true;
  const int p = tree->leaf_parent(leaf);
  if (p == tree->num_leaves() - 2) return false;
  const int sib = tree->left_child(p) == ~leaf ? tree->right_child(p) : tree->left_child(p);
  const int md = cfg.min_data_in_leaf;
  if (tree->leaf_count(leaf) < 2 * md && tree->data_count(sib) < 2 * md) return false;
  return !(cfg.max_depth > 0 && tree->leaf_depth(leaf) >= cfg.max_depth);
}
}  // namespace

bool GPUTreeLearner::DebugLeafState(const Tree* tree, int leaf, std::vector<int32_t>* rows,
                                    std::vector<long long>* hist, std::vector<int8_t>* bin_valid, double* sums) {
  if (spec_live_) {
    Log::Fatal("device learner: the device holds the next tree (launched speculatively); set "
               "LGBM_AMD_SPECULATE=0 to inspect the last tree's device state");
  }
  if (!device_mode_ || d_leaves_ == nullptr || tree == nullptr || leaf < 0 || leaf >= tree->num_leaves()) {
    return false;
  }
  HIPCHECK(hipSetDevice(device_id_));
  HIPCHECK(hipStreamSynchronize(stream_));
  dev::Leaf lf;
  HIPCHECK(hipMemcpy(&lf, d_leaves_ + leaf, sizeof(lf), hipMemcpyDeviceToHost));
  rows->assign(static_cast<size_t>(lf.count), 0);
  const int32_t* buf = lf.buf == 0 ? d_idx_ : d_tmp_ + static_cast<int64_t>(lf.buf - 1) * num_data_;
  if (lf.count > 0) {
    HIPCHECK(hipMemcpy(rows->data(), buf + lf.begin, sizeof(int32_t) * lf.count, hipMemcpyDeviceToHost));
  }
  ReadHist(lf, leaf, hist);
  std::vector<int8_t> flags(num_features_);
  HIPCHECK(hipMemcpy(flags.data(), d_splittable_ + static_cast<size_t>(lf.frow) * num_features_, num_features_,
                     hipMemcpyDeviceToHost));
  bin_valid->assign(static_cast<size_t>(total_bins_), 0);
  const bool scanned = LeafScanned(tree, leaf, *config_);
  for (int f = 0; f < num_features_ && scanned; ++f) {
    if (flags[f] == 0) continue;
    const size_t off = data_->FeatureHistOffset(f);
    for (int t = 0; t < data_->FeatureHistSize(f); ++t) (*bin_valid)[off + t] = 1;
  }
  sums[0] = lf.sum_g;
  sums[1] = lf.sum_h;
  sums[2] = lf.global_count;
  return true;
}

bool GPUTreeLearner::DebugGradients(std::vector<float>* g, std::vector<float>* h, double* scales) {
  if (d_gh_ == nullptr) return false;
  HIPCHECK(hipSetDevice(device_id_));
  HIPCHECK(hipStreamSynchronize(stream_));
  std::vector<dev::GH> gh(static_cast<size_t>(num_data_));
  // (rows of the bin matrix may carry their (g, h): a strided copy)
  HIPCHECK(hipMemcpy2D(gh.data(), sizeof(dev::GH), d_gh_, sizeof(dev::GH) * static_cast<size_t>(args_.gh_stride),
                       sizeof(dev::GH), gh.size(), hipMemcpyDeviceToHost));
  g->resize(gh.size());
  h->resize(gh.size());
  for (size_t i = 0; i < gh.size(); ++i) {
    (*g)[i] = gh[i].g;
    (*h)[i] = gh[i].h;
  }
  HIPCHECK(hipMemcpy(scales, d_scales_, 2 * sizeof(double), hipMemcpyDeviceToHost));
  return true;
}

std::string GPUTreeLearner::DebugCheckSplits(const Tree* tree) {
  if (spec_live_) {
    Log::Fatal("device learner: the device holds the next tree (launched speculatively); set "
               "LGBM_AMD_SPECULATE=0 to inspect the last tree's device state");
  }
  std::ostringstream js;
  if (!device_mode_ || tree == nullptr) return "{\"device_mode\": false}";
  double scales[4];
  HIPCHECK(hipSetDevice(device_id_));
  HIPCHECK(hipStreamSynchronize(stream_));
  HIPCHECK(hipMemcpy(scales, d_scales_, 4 * sizeof(double), hipMemcpyDeviceToHost));
  const int L = tree->num_leaves();
  std::vector<dev::Leaf> leaves(L);
  std::vector<DeviceSplit> best(L);
  HIPCHECK(hipMemcpy(leaves.data(), d_leaves_, sizeof(dev::Leaf) * L, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(best.data(), d_best_, sizeof(DeviceSplit) * L, hipMemcpyDeviceToHost));
  const size_t nh = 2 * static_cast<size_t>(total_bins_);
  std::vector<long long> raw(nh);
  std::vector<hist_t> fh;
  int checked = 0, mismatched = 0, gain_mismatch = 0, direction_ties = 0;
  double max_rel = 0.0;
  std::ostringstream details;
  for (int l = 0; l < L; ++l) {
    const dev::Leaf& lf = leaves[l];
    if (!LeafScanned(tree, l, *config_)) continue;  // no split is evaluated
    ReadHist(lf, l, &raw);
    ConstraintRange c;
    c.min = lf.cmin;
    c.max = lf.cmax;
    double parent_output = lf.output;
    if (l == 0 && tree->num_leaves() == 1) {
      SplitParams rp = params_;
      rp.use_l1 = 1;
      rp.use_max_output = 1;
      rp.use_smoothing = 0;
      rp.use_mc = 1;
      parent_output = LeafOutputConstrained(lf.sum_g, lf.sum_h, params_.lambda_l2, rp, c, lf.global_count, 0);
    }
    // features the device did not evaluate for this leaf (its parent could not split on them)
    // have no histogram in the slot: the CPU finder skips them too
    std::vector<int8_t> flags(num_features_);
    HIPCHECK(hipMemcpy(flags.data(), d_splittable_ + static_cast<size_t>(lf.frow) * num_features_, num_features_,
                       hipMemcpyDeviceToHost));
    SplitInfo host_best;
    std::vector<double> gains(num_features_, -INFINITY);
    for (int f = 0; f < num_features_; ++f) {
      if (flags[f] == 0) continue;
      const size_t off = 2 * data_->FeatureHistOffset(f);
      const int n = data_->FeatureHistSize(f);
      fh.assign(2 * static_cast<size_t>(n), 0.0);
      for (int t = 0; t < n; ++t) {
        fh[2 * t] = static_cast<double>(raw[off + 2 * t]) * scales[2];
        fh[2 * t + 1] = static_cast<double>(raw[off + 2 * t + 1]) * scales[3];
      }
      data_->FixHistogram(f, lf.sum_g, lf.sum_h, fh.data());
      SplitInfo ns;
      bool splittable = false;
      FindBestThreshold(meta_[f], params_, false, fh.data(), lf.sum_g, lf.sum_h, lf.global_count, c, parent_output,
                        &ns, &splittable);
      ns.feature = data_->RealFeatureIndex(f);
      ns.inner_feature = f;
      if (ns.monotone_type != 0) ns.gain *= MonotoneSplitPenalty(lf.depth, config_->monotone_penalty);
      gains[f] = ns.gain;
      if (ns > host_best) host_best = ns;
    }
    const DeviceSplit& d = best[l];
    if (d.feature < 0 && !(host_best.gain > 0 && std::isfinite(host_best.gain))) {
      ++checked;  // neither side found a split
      continue;
    }
    ++checked;
    const double hg = host_best.gain, dg = d.gain;
    const double rel = std::fabs(hg - dg) / std::max(1.0, std::fabs(hg));
    max_rel = std::max(max_rel, std::isfinite(rel) ? rel : 1e30);
    // the device's feature must be a best one (ties within tolerance allowed), with its
    // threshold and direction matching the CPU finder's for that feature
    bool ok = d.feature >= 0 && rel <= 1e-6;
    if (ok && d.feature != host_best.inner_feature) {
      ok = std::fabs(gains[d.feature] - hg) / std::max(1.0, std::fabs(hg)) <= 1e-6;
    }
    if (ok && d.feature == host_best.inner_feature && !d.is_categorical) {
      ok = static_cast<uint32_t>(d.threshold) == host_best.threshold && d.left_count == host_best.left_count;
      // the same threshold found by both scan directions with equal gain and equal counts
      // (the missing / default bin is empty in this leaf): which direction wins is decided
      // by the last bits of two differently-ordered sums, on the host as in the reference
      if (ok && (d.default_left != 0) != host_best.default_left) ++direction_ties;
    }
    if (rel > 1e-6) ++gain_mismatch;
    if (!ok) {
      ++mismatched;
      if (mismatched <= 8) {
        details << (mismatched > 1 ? ", " : "") << "{\"leaf\": " << l << ", \"device_feature\": " << d.feature
                << ", \"device_threshold\": " << d.threshold << ", \"device_gain\": " << Num(dg)
                << ", \"device_left_count\": " << d.left_count << ", \"host_feature\": " << host_best.inner_feature
                << ", \"host_threshold\": " << host_best.threshold << ", \"host_gain\": " << Num(hg)
                << ", \"host_left_count\": " << host_best.left_count << "}";
      }
    }
  }
  js.precision(17);
  js << "{\"device_mode\": true, \"leaves\": " << L << ", \"checked\": " << checked << ", \"mismatched\": "
     << mismatched << ", \"gain_mismatch\": " << gain_mismatch << ", \"direction_ties\": " << direction_ties
     << ", \"max_rel_gain_diff\": " << Num(max_rel) << ", \"layout\": \""
     << (sparse_rows_ ? "sparse" : args_.nibbles ? "4" : (args_.bin_bytes == 1 ? "8" : (args_.bin_bytes == 2 ? "16" : "mixed")))
     << "\", \"hist_tiles\": " << args_.hist_tiles << ", \"details\": [" << details.str() << "]}";
  return js.str();
}

}  // namespace lgbm_amd
