// Best-split search on device histograms (reference src/treelearner/feature_histogram.hpp:
// FindBestThresholdSequentially, FuncForNumricalL3, FixHistogram; serial_tree_learner.cpp
// FindBestSplitsFromHistograms).
//
// k_find: grid (num_features, 2 leaves), one 256-thread workgroup per (feature, leaf).  It
// materialises the feature's histogram in the leaf's pool slot -- the histogrammed child
// takes the step's reduced histogram (or sums the few partials of a small leaf itself), the
// other child subtracts it from the parent slot in place, exact in int64 -- stages it
// dequantised in LDS, then evaluates every threshold of the forward and reverse scans in
// parallel from ONE workgroup prefix scan (the reverse scan's right sums are the range total
// minus the prefix), with the reference's missing-value handling, min_data / min_hessian
// filters, hessian-estimated counts, L1 / max_delta_step / path smoothing / monotone
// constraints.  Ties keep the threshold the sequential scan would keep.  Per-feature results
// go to feat_best.  The last workgroup of the step to finish (a device-scope counter) then
// records the step and picks the next split (pick.h), so the next k_split starts from one
// small Step record.
#include "split_scan.h"

namespace lgbm_amd {
namespace dev {


// KIND 0: every feature of a dataset without categorical features; 1: the numerical
// features of a dataset with some (the categorical ones only get their bookkeeping here);
// 2: the categorical features (grid over KArgs::cat_list).  The categorical scan has its
// own register / LDS footprint, so it runs in a kernel of its own (inlined: a called
// function costs ~700 B/lane of stack and ran ~10x slower).

// extra_trees: whether the host learner scans f at node mi (the feature is used by the tree,
// its parent could split on it, the node samples it and its constraints allow it) and so
// draws FeatureMeta::rand.NextInt(0, num_bin - 2) (split_finder.cpp FindNumerical)
__device__ __forceinline__ int XtDraws(const KArgs& a, const Feature& F, int f, int mi, IcMask icmask, bool gate) {
  if (!gate || F.num_bin - 2 <= 0) return 0;
  if (a.node_mask != nullptr && !a.node_mask[static_cast<size_t>(mi) * a.p.num_features + f]) return 0;
  if (a.feat_icmask != nullptr && !IcAny(icmask & a.feat_icmask[f])) return 0;
  return 1;
}

// ---- voting-parallel extra_trees (KArgs::xt_base_glob)
// the owner of elected slot i of side (0: the smaller leaf) -- the reference's CopyLocalHistogram:
// each rank in turn takes ceil(elected / world) histograms, alternating smaller-leaf and
// larger-leaf slots and starting each rank with a smaller-leaf one
__device__ int VoteOwner(const KArgs& a, bool root, int side, int i) {
  const int k = a.p.vote_k, W = a.p.world;
  int n0 = 0, n1 = 0;
  for (int j = 0; j < k; ++j) {
    n0 += a.vote_list[j] >= 0 ? 1 : 0;
    n1 += (!root && a.vote_list[k + j] >= 0) ? 1 : 0;
  }
  const int total = n0 + n1, avg = (total + W - 1) / W;
  int used = 0, si = 0, li = 0;
  for (int m = 0; m < W; ++m) {
    const int want = min(avg, total - used);
    int cnt = 0;
    while (cnt < want) {
      if (si < n0) {
        if (side == 0 && si == i) return m;
        ++si;
        ++cnt;
      }
      if (cnt >= want) break;
      if (li < n1) {
        if (side == 1 && li == i) return m;
        ++li;
        ++cnt;
      }
    }
    used += cnt;
  }
  return -1;
}
// whether the global scan of side evaluates f (ComputeBestSplitForFeature's is_feature_used:
// the tree's and the node's samples, the interaction constraints) -- and so draws
__device__ bool VoteXtUsed(const KArgs& a, int f, int side, int mi_base, IcMask icm) {
  if (!a.tree_mask[f]) return false;
  if (a.node_mask != nullptr && !a.node_mask[static_cast<size_t>(mi_base + side) * a.p.num_features + f]) return false;
  if (a.feat_icmask != nullptr && !IcAny(icm & a.feat_icmask[f])) return false;
  return true;
}
// the draws rank r's global scans make of f this step (smaller leaf first)
__device__ int VoteXtDraws(const KArgs& a, bool root, int r, int f, int mi_base, IcMask icm, int sides_upto) {
  const int k = a.p.vote_k;
  int d = 0;
  for (int side = 0; side < sides_upto; ++side) {
    for (int j = 0; j < k; ++j) {
      if (a.vote_list[side * k + j] != f) continue;
      if (VoteOwner(a, root, side, j) == r && VoteXtUsed(a, f, side, mi_base, icm)) ++d;
      break;
    }
  }
  return d;
}
// the step's row of global draw counts, every (rank, feature), strided over the scan's grid
__device__ void VoteXtCountRow(const KArgs& a, bool root, int s, int mi_base, bool skip, IcMask icm) {
  const int nf = a.p.num_features, W = a.p.world;
  const size_t n = static_cast<size_t>(W) * nf;
  const int32_t* prev = root ? nullptr : a.xt_cum_glob + static_cast<size_t>(s) * n;
  int32_t* row = a.xt_cum_glob + static_cast<size_t>(root ? 0 : s + 1) * n;
  const size_t wg = static_cast<size_t>(blockIdx.y) * gridDim.x + blockIdx.x;
  const size_t nwg = static_cast<size_t>(gridDim.x) * gridDim.y;
  for (size_t e = wg * blockDim.x + threadIdx.x; e < n; e += nwg * blockDim.x) {
    const int r = static_cast<int>(e / nf), f = static_cast<int>(e % nf);
    const int d = (!skip && a.feat[f].num_bin - 2 > 0) ? VoteXtDraws(a, root, r, f, mi_base, icm, root ? 1 : 2) : 0;
    row[e] = (prev != nullptr ? prev[e] : 0) + d;
  }
}
// the random threshold of elected slot i (side) of f: the owner's next draw, after its draw for
// the smaller leaf's slot of f this step
__device__ int VoteXtThreshold(const KArgs& a, const Feature& F, int f, int side, int i, bool root, int s, int mi_base,
                               IcMask icm) {
  const int nf = a.p.num_features, W = a.p.world;
  if (F.num_bin - 2 <= 0 || !VoteXtUsed(a, f, side, mi_base, icm)) return 0;
  const int r = VoteOwner(a, root, side, i);
  if (r < 0) return 0;
  const int before = side == 1 ? VoteXtDraws(a, root, r, f, mi_base, icm, 1) : 0;
  const int prev = root ? 0 : a.xt_cum_glob[(static_cast<size_t>(s) * W + r) * nf + f];
  const uint32_t x = LcgSkip(a.xt_base_glob[static_cast<size_t>(r) * nf + f], prev + before + 1);
  return static_cast<int>((x & 0x7fffffffu) % static_cast<uint32_t>(F.num_bin - 2));
}

// GatherInfoForThreshold (reference feature_histogram.hpp; host split_finder.cpp): the split of
// a forced node at bin `thr` from the leaf's histogram, one thread.  hv holds the raw bins;
// the most frequent bin is rebuilt from the leaf totals first (FixHistogram).  Invalid (gain
// no better than the leaf's own): gain -inf, the pick then drops the forced splits.
__device__ void ForcedGather(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p, int thr,
                             FeatureBest* out, int* cat_bin) {
  const int nb = F.num_bin - F.offset, offset = F.offset;
  const double sum_g = L.sg, sum_h = L.sh - 2 * kEpsilon;  // the leaf's raw sums
  hv.fix_t = -1;
  if (F.mfb > 0) {
    double og = 0.0, oh = 0.0;
    for (int t = 0; t < nb; ++t) {
      if (t == F.mfb) continue;
      og += hv.RawG(t);
      oh += hv.RawH(t);
    }
    hv.fix_t = F.mfb;
    hv.fix_g = sum_g - og;
    hv.fix_h = sum_h - oh;
  }
  const int smooth = p.use_smoothing;
  const double gain_shift = LeafGainGivenOutput(sum_g, sum_h, p.lambda_l1, p.lambda_l2, L.parent_out, 1);
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const double cnt_factor = L.n / sum_h;
  FeatureBest o = {};
  o.gain = -INFINITY;
  o.feature = -1;
  o.real_feature = -1;
  *cat_bin = -1;  // (the forced category: the set published by the caller)
  double lg, lh, rg, rh;
  int lc, rc;
  if (!F.is_cat) {
    rg = 0.0;
    rh = kEpsilon;
    rc = 0;
    const bool skip_default = F.missing_type == 1, na = F.missing_type == 2;
    for (int t = nb - 1 - (na ? 1 : 0); t >= 1 - offset; --t) {
      if (static_cast<uint32_t>(t + offset) < static_cast<uint32_t>(thr)) break;
      if (skip_default && t + offset == F.default_bin) continue;
      rg += hv.G(t);
      rh += hv.H(t);
      rc += RoundIntD(hv.H(t) * cnt_factor);
    }
    lg = sum_g - rg;
    lh = sum_h - rh;
    lc = L.n - rc;
    o.default_left = 1;
  } else {
    if (thr >= F.num_bin || thr == 0) {
      *out = o;
      return;
    }
    const double hh = hv.H(thr - offset);
    lc = RoundIntD(hh * cnt_factor);
    rc = L.n - lc;
    lh = hh + kEpsilon;
    rh = sum_h - lh;
    lg = hv.G(thr - offset);
    rg = sum_g - lg;
    o.default_left = 0;
    o.ncat = 1;
    *cat_bin = thr;
  }
  const double gain = LeafGain(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, L.parent_out, 1, 1,
                               smooth) +
                      LeafGain(rg, rh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc, L.parent_out, 1, 1,
                               smooth);
  if (!(gain > min_gain_shift)) {  // (NaN included)
    *out = o;
    return;
  }
  o.thr = F.is_cat ? 0 : thr;
  o.lo = LeafOutputRaw(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, L.parent_out, 1, 1,
                       smooth);
  o.ro = LeafOutputRaw(sum_g - lg, sum_h - lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc,
                       L.parent_out, 1, 1, smooth);
  o.lc = lc;
  o.rc = L.n - lc;
  o.lg = lg;
  o.lh = lh - kEpsilon;
  o.rg = sum_g - lg;
  o.rh = sum_h - lh - kEpsilon;
  o.gain = gain - min_gain_shift;
  o.mono = 0;
  o.feature = -2;  // (set by the caller)
  *out = o;
}

template <bool ROOT, int KIND, int NT>
struct FindShared {
  BlockScratch<NT> sc;
  ScanScratch<NT> ssc;
  Cand sc2[NT / kWave];
  typename std::conditional<KIND == 2, CatScratchT<kFindCatNarrow>,
                            typename std::conditional<KIND == 3, CatScratchT<kFindMaxCatBins>, int>::type>::type cat_sc;
  unsigned long long s_red[2 * NT];  // direct partial sums of narrow features
};

// the scan of one (feature, child) by one workgroup: every thread of the workgroup takes the
// same path (the kernel's pick tail needs all of them)
// side: the child (0: the smaller one); d0_in / drew: categorical extra_trees only -- the draws
// the smaller child's scan of this feature consumed, and this scan's (see k_find)
template <bool ROOT, int KIND, bool SIMPLE, int NT>
__device__ __forceinline__ void FindBody(const KArgs& a, double* s_bins, FindShared<ROOT, KIND, NT>& sh, const int side,
                                         const int d0_in, int* drew) {
  if (drew != nullptr) *drew = 0;
  constexpr bool CAT = KIND >= 2;  // (3: the wide categorical variant)
  constexpr int kFindThreads = NT;
  const long long t_entry = wall_clock64();
  // voting-parallel global scan: the features the vote elected for this side's leaf (an
  // empty slot still takes part in the step's workgroup count)
  const bool vote_global = a.p.vote_phase == 2;
  int f = CAT ? a.cat_list[blockIdx.x] : (a.feat_list != nullptr ? a.feat_list[blockIdx.x] : static_cast<int>(blockIdx.x));
  if (f < 0 && !vote_global) return;  // a padded owner slot (distributed learners: no pick in this kernel)
  if (vote_global) f = a.vote_list[blockIdx.y * a.p.vote_k + blockIdx.x];
  const bool vote_empty = vote_global && f < 0;
  if (vote_empty) f = 0;
  const int tid = threadIdx.x;
  const int units = a.hist_units;
  // ---- independent loads first (one round trip): the feature, its mask, the scales and the
  // Step record
  const Feature F = a.feat[f];
  const int8_t tree_used = a.tree_mask[f];
  const Step* st = a.st;
  // intermediate monotone constraints: sides 2.. re-scan the leaves the last split re-bounded
  // (SerialTreeLearner::RecomputeBestSplitForLeaf: the leaf's histogram, the sums and count of
  // its current best split, parent output 0, every feature of the tree it could split on; no
  // node sampling, flags untouched).  An unused slot only counts its arrival.
  const bool rescan = !ROOT && side >= 2;
  int rleaf = -1;
  if (rescan) {
    if (side - 2 >= a.mt_upd[0]) return;
    rleaf = a.mt_upd[side - 1];
  }
  const int mi_base = ROOT ? 0 : st->bynode_next;  // this step's per-node masks (advanced by the pick)
  int8_t used = tree_used;  // evaluated at this node (feature_fraction_bynode)
  // (voting: the local scan evaluates every feature, the global scan of the elected ones
  // applies the node's sample -- VotingParallelTreeLearner::FindBestSplits)
  if (a.node_mask != nullptr && !rescan && a.p.vote_phase != 1) {
    used = used && a.node_mask[static_cast<size_t>(mi_base + side) * a.p.num_features + f];
  }
  // (voting: every feature is scanned -- the vote may elect one this rank could not split, and
  // its local histogram must exist; see k_round_find)
  const int8_t parent_ok = (ROOT || a.p.vote_phase != 0) ? 1
                           : rescan ? a.splittable[static_cast<size_t>(a.leaves[rleaf].frow) * a.p.num_features + f]
                                    : a.parent_flags[f];
  const double ig = a.scales[2], ih = a.scales[3];
  int s = 0, pc = 0, skip = 0;
  ChildInfo c;
  SideInfo sd;
  ChildStats cl;
  if (rescan) {
    s = st->cs.s;
    const Leaf& lf = a.leaves[rleaf];
    const DeviceSplit& rbest = a.best[rleaf];  // (the sums and counts only: no copy of the category set)
    sd.lr = 0;
    sd.leaf = rleaf;
    sd.slot = lf.slot;
    sd.frow = lf.frow;
    sd.is_hist = 1;
    sd.global_count = rbest.left_count + rbest.right_count;
    cl.sum_g = rbest.left_sum_gradient + rbest.right_sum_gradient;
    cl.sum_h = rbest.left_sum_hessian + rbest.right_sum_hessian;
    cl.output = 0.0;
    cl.cmin = lf.cmin;
    cl.cmax = lf.cmax;
    cl.depth = lf.depth;
    cl.slot = lf.slot;
    cl.leaf = rleaf;
    cl.frow = lf.frow;
    cl.icmask = kIcAll;
  } else if (!ROOT) {
    s = st->cs.s;
    pc = st->cs.part_count;
    c = StepChildren(a, st);
    sd = StepSide(a, st, c, side);
    cl = st->lr[sd.lr];
    skip = c.skip;
  }
  // extra_trees: per feature and node, the smaller child draws before the larger one
  // (SerialTreeLearner::FindBestSplitsFromHistograms); draw k of the tree is the base state
  // stepped k times.  The smaller child's workgroup appends the step's count row.
  int xt_thr = kNoRandThr;
  uint32_t xt_r = 0u;
  if (a.xt_base != nullptr && CAT) {
    // categorical: whether a scan draws depends on its histogram (the sorted scan's
    // max_threshold), so k_find scans both children in one workgroup, the smaller one first,
    // and appends the step's count row itself
    const int prev = ROOT ? 0 : a.xt_cum[static_cast<size_t>(s) * a.p.num_features + f];
    xt_r = LcgSkip(a.xt_base[f], prev + (side == 1 ? d0_in : 0) + 1) & 0x7fffffffu;
  } else if (a.xt_base != nullptr && vote_global) {
    // voting: the owner's draw from the global generator set (KArgs::xt_base_glob)
    const IcMask icm = ROOT ? kIcAll : cl.icmask;
    xt_thr = 0;
    if (!vote_empty && !skip) xt_thr = VoteXtThreshold(a, F, f, side, blockIdx.x, ROOT, s, mi_base, icm);
    VoteXtCountRow(a, ROOT, s, mi_base, skip != 0, icm);
  } else if (a.xt_base != nullptr) {
    const int nf = a.p.num_features;
    const int prev = ROOT ? 0 : a.xt_cum[static_cast<size_t>(s) * nf + f];
    // (voting's local scans: the features whose parent's local scan could split, no node
    // sample and no interaction constraints -- VotingParallelTreeLearner::FindBestSplits)
    const bool vote_local = a.p.vote_phase == 1;
    const bool gate = tree_used && (vote_local ? (ROOT || a.parent_flags[f] != 0) : parent_ok) && !skip;
    const IcMask icm = ROOT ? kIcAll : cl.icmask;  // both children carry the same constraints
    const int d0 = vote_local ? (gate && F.num_bin - 2 > 0 ? 1 : 0) : XtDraws(a, F, f, mi_base, icm, gate);
    const int d1 = ROOT ? 0 : vote_local ? d0 : XtDraws(a, F, f, mi_base + 1, icm, gate);
    if (side == 0 && tid == 0) a.xt_cum[static_cast<size_t>(ROOT ? 0 : s + 1) * nf + f] = prev + d0 + d1;
    xt_thr = 0;  // num_bin <= 2: no draw, threshold 0 only
    if (side == 0 ? d0 : d1) {
      const uint32_t x = LcgSkip(a.xt_base[f], prev + (side == 1 ? d0 : 0) + 1);
      xt_thr = static_cast<int>(x & 0x7fffffffu) % (F.num_bin - 2);
    }
  }
  const int nbf = F.num_bin - F.offset;
  const int nb2 = 2 * nbf;
  int parity = 0, nblk_direct = -1;
  if (!ROOT) {
    parity = (s + 1) & 1;
    // zero this feature's bins of the buffer the next step reduces into (data-parallel:
    // the whole owner-major buffer is cleared before each reduction)
    if (!CAT && side == 0 && a.rs_pos == nullptr && !vote_global) {
      long long* nxt = StepScratch(a, parity + 1);
      for (int i = tid; i < nb2; i += kFindThreads) nxt[2 * F.hist_offset + i] = 0;
    }
    if (skip) return;
    KTraceAt(a, s, kTrFindEntry, t_entry);
    KTrace(a, s, kTrFindHdr);
    const int nblk = StepBlocks(a, pc);
    if (DirectPartials(a, nblk, s) && !vote_global && !rescan) nblk_direct = nblk;
  }
  const SplitParams& p = a.p.sp;
  LeafCtx L;
  int depth, slot;
  if (ROOT) {
    const double* rsum = a.p.vote_phase == 1 ? a.root_local : a.root;  // voting: local, then global
    const double sg = rsum[0], shh = rsum[1];
    const int n = static_cast<int>(rsum[2]);
    ConstraintRange cr;
    cr.min = -DBL_MAX;
    cr.max = DBL_MAX;
    SplitParams rp = p;
    rp.use_l1 = 1;
    rp.use_max_output = 1;
    rp.use_smoothing = 0;
    rp.use_mc = 1;
    const double out0 = LeafOutputConstrained(sg, shh, p.lambda_l2, rp, cr, n, 0);
    const bool first = vote_global ? blockIdx.x == 0 : f == 0;
    if (first && tid == 0 && !CAT) {  // (write-through: the root pick rewrites leaf 0)
      Leaf& lf = a.leaves[0];
      if (a.p.vote_phase == 1) {
        PublishF64(&lf.lsum_g, sg);
        PublishF64(&lf.lsum_h, shh);
      } else {
        PublishF64(&lf.sum_g, sg);
        PublishF64(&lf.sum_h, shh);
        PublishI32(&lf.global_count, n);
        PublishF64(&lf.output, out0);
        PublishI32(&a.st->root_count, n);
      }
    }
    L.sg = sg;
    L.sh = shh + 2 * kEpsilon;
    L.n = n;
    L.parent_out = out0;
    L.c = cr;
    depth = 0;
    slot = 0;
  } else {
    L.sg = cl.sum_g;
    L.sh = cl.sum_h + 2 * kEpsilon;
    L.n = sd.global_count;
    L.parent_out = cl.output;
    L.c.min = cl.cmin;
    L.c.max = cl.cmax;
    depth = cl.depth;
    slot = sd.slot;
    if (a.p.vote_phase == 1) {
      // voting local scan: this rank's rows of the child -- the histogrammed child's sums from
      // k_split, the other one's as the parent's minus those
      const double hg = static_cast<double>(static_cast<long long>(st->loc_acc[0])) * ig;
      const double hh = static_cast<double>(static_cast<long long>(st->loc_acc[1])) * ih;
      const double lsg = sd.is_hist ? hg : st->cs.plsum_g - hg;
      const double lsh = sd.is_hist ? hh : st->cs.plsum_h - hh;
      L.sg = lsg;
      L.sh = lsh + 2 * kEpsilon;
      L.n = sd.lr == 0 ? c.total_left : pc - c.total_left;
      if (blockIdx.x == 0 && tid == 0) {
        a.leaves[sd.leaf].lsum_g = lsg;
        a.leaves[sd.leaf].lsum_h = lsh;
      }
    }
  }
  if (vote_empty) return;
  // CEGB lazy penalties: this child's unpaid-row count of f -- the root's from k_cegb_root; the
  // histogrammed child's from k_cegb_step, the other one's as the split leaf's snapshot minus
  // it, 0 for the split feature (its rows were just paid) -- stored per leaf by the numerical
  // kernel (every feature has a workgroup there) for the children's own steps
  int unpaid = 0;
  if (a.cegb_lazy != nullptr) {
    const int nfc = a.p.num_features;
    if (ROOT) {
      unpaid = a.cegb_cnt[f];
    } else if (rescan) {
      unpaid = a.cegb_cnt[static_cast<size_t>(rleaf) * nfc + f];
    } else {
      const size_t po = static_cast<size_t>(s & 1) * nfc + f;
      const int hs = a.cegb_scratch[po];
      unpaid = f == st->cs.split.feature ? 0 : (sd.is_hist ? hs : a.cegb_snap[po] - hs);
      if (!CAT && tid == 0) a.cegb_cnt[static_cast<size_t>(sd.leaf) * nfc + f] = unpaid;
    }
  }
  if (KIND == 1 && F.is_cat) return;  // the categorical kernel scans it
  if (CAT && !F.is_cat) return;       // (voting global scan: an elected numerical feature)
  // interaction constraints: like a sampled-out feature, a disallowed one is not evaluated
  // here but keeps its histogram and its splittable flag
  // (voting's local scan evaluates it: its features are the tree's sample and the parent's flags)
  if (a.feat_icmask != nullptr && a.p.vote_phase != 1 && !IcAny((ROOT ? kIcAll : cl.icmask) & a.feat_icmask[f])) used = 0;
  int8_t* flags = a.splittable + static_cast<size_t>(ROOT ? a.leaves[0].frow : sd.frow) * a.p.num_features;
  FeatureBest* fb_out = &a.feat_best[FeatBestIndex(a, side, f)];
  if (tree_used && !parent_ok) {
    // the parent could not split on f: neither child evaluates it, the smaller child's row
    // says so and the larger child keeps the parent's row (SerialTreeLearner::FindBestSplits)
    if (side == 0 && tid == 0) flags[f] = 0;
    if (tid == 0) {
      FeatureBest none = {};
      none.gain = -INFINITY;
      none.feature = none.real_feature = -1;
      PublishRecord(fb_out, none);
    }
    return;
  }
  L.cnt_factor = L.n / L.sh;
  const double gain_shift = LeafGain(L.sg, L.sh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, L.n,
                                     L.parent_out, p.use_l1, p.use_max_output, p.use_smoothing);
  L.min_gain_shift = gain_shift + p.min_gain_to_split;

  FeatureBest o;
  o.gain = -INFINITY;
  o.feature = f;
  o.real_feature = F.real_index;
  o.thr = 0;
  o.default_left = 1;
  o.lc = o.rc = 0;
  o.mono = 0;
  o.ncat = 0;
  o.flag = -1;
  o.pad = 0;
  o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
  // a sampled-out feature (bynode) still materialises its histogram: descendants subtract it
  if (tree_used && (!F.is_cat || F.num_bin <= kFindMaxCatBins)) {
    const int nh = 2 * a.p.total_bins;
    // (voting global scan: the elected feature's histogram summed over the ranks, read in place)
    long long* dst = vote_global ? a.vote_hist + static_cast<size_t>(side * a.p.vote_k + blockIdx.x) * 2 *
                                                     a.p.max_feature_bins
                                 : a.hist + static_cast<size_t>(slot) * nh + 2 * F.hist_offset;
    const long long* src = (vote_global || rescan) ? dst
                           : a.owned_hist != nullptr ? a.owned_hist + 2 * a.owned_off[f]
                                                     : StepScratch(a, parity) + 2 * F.hist_offset;
    const size_t pstride = static_cast<size_t>(units) * a.p.total_bins;
    const unsigned long long* part = a.partials + static_cast<size_t>(units) * F.hist_offset;
    const bool stage = a.p.max_feature_bins <= kFindLdsBins;
    double* sg = s_bins;
    double* shv = s_bins + (stage ? a.p.max_feature_bins : 0);
    const bool subtract = !ROOT && !sd.is_hist && !vote_global;  // parent - the histogrammed child, in place
    // a feature with fewer bins than threads sums its direct partials with every thread:
    // kFindThreads / nbf threads per bin stride over the row blocks, then combine in LDS
    // (one thread per bin walking hundreds of partials would be a chain of round trips)
    const bool spread = nblk_direct > 1 && 2 * nbf <= kFindThreads;
    // the parent's bins (first bin of each thread): loaded up front, so their round trip
    // overlaps the partial-sum loads instead of following them
    long long pg0 = 0, ph0 = 0;
    if (subtract && tid < nbf) {
      pg0 = dst[2 * tid];
      ph0 = dst[2 * tid + 1];
    }
    if (spread) {
      for (int j = tid; j < 2 * nbf; j += kFindThreads) sh.s_red[j] = 0ull;
      __syncthreads();
      const int per = kFindThreads / nbf;
      const int i = tid % nbf, r = tid / nbf;
      if (r < per) {
        constexpr int kC = 8;
        long long g = 0, h = 0;
        for (int k0 = r; k0 < nblk_direct; k0 += per * kC) {
          unsigned long long v0[kC], v1[kC];
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            const int k = k0 + cc * per;
            const unsigned long long* q = part + k * pstride + static_cast<size_t>(units) * i;
            v0[cc] = k < nblk_direct ? q[0] : 0ull;
            v1[cc] = (k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            long long pgv, phv;
            UnpackPartial(v0[cc], v1[cc], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
        atomicAdd(&sh.s_red[2 * i], static_cast<unsigned long long>(g));
        atomicAdd(&sh.s_red[2 * i + 1], static_cast<unsigned long long>(h));
      }
      __syncthreads();
    }
    for (int i = tid; i < nbf; i += kFindThreads) {
      long long g = 0, h = 0;
      if (spread) {
        g = static_cast<long long>(sh.s_red[2 * i]);
        h = static_cast<long long>(sh.s_red[2 * i + 1]);
      } else if (nblk_direct >= 0) {
        // small leaf: sum the few per-block partials here (k_hist_reduce skipped them),
        // chunks of kDirectChunk independent loads in flight
        for (int k0 = 0; k0 < nblk_direct; k0 += kDirectChunk) {
          unsigned long long v0[kDirectChunk], v1[kDirectChunk];
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            const unsigned long long* q = part + (k0 + k) * pstride + static_cast<size_t>(units) * i;
            v0[k] = k0 + k < nblk_direct ? q[0] : 0ull;
            v1[k] = (k0 + k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            long long pgv, phv;
            UnpackPartial(v0[k], v1[k], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
      } else {
        g = src[2 * i];
        h = src[2 * i + 1];
      }
      if (subtract) {
        g = (i == tid ? pg0 : dst[2 * i]) - g;
        h = (i == tid ? ph0 : dst[2 * i + 1]) - h;
      }
      dst[2 * i] = g;
      dst[2 * i + 1] = h;
      if (stage) {
        sg[i] = static_cast<double>(g) * ig;
        shv[i] = static_cast<double>(h) * ih;
      }
    }
    __syncthreads();  // the workgroup's stores become visible to all its threads
    if (!ROOT) KTrace(a, s, kTrFindLoaded);
    // voting extra_trees: the reference's local scans skip the features the parent's local scan
    // could not split (at its random threshold) -- their histograms exist for the vote, they
    // propose nothing and draw nothing (VotingParallelTreeLearner::FindBestSplits)
    const bool vote_skip = a.p.vote_phase == 1 && a.xt_base != nullptr && !ROOT && !rescan && !a.parent_flags[f];
    if (!used || vote_skip) {
      if (tid == 0) {
        if (vote_skip) flags[f] = 0;
        FeatureBest none = {};
        none.gain = -INFINITY;
        none.feature = none.real_feature = -1;
        PublishRecord(fb_out, none);
      }
      return;
    }
    HistView hv;
    hv.lg = stage ? sg : nullptr;
    hv.lh = stage ? shv : nullptr;
    hv.h = dst;
    hv.inv_g = ig;
    hv.inv_h = ih;
    bool splittable;
    if constexpr (CAT) {
      splittable = FindCategoricalBlock(F, hv, L, p, &o, a.feat_cat + FeatBestIndex(a, side, f) * kMaxCatWords, &sh.sc,
                                        &sh.cat_sc, a.xt_base != nullptr, xt_r, drew);
    } else {
      splittable = FindNumericalBlock<SIMPLE, NT>(F, hv, L, p, depth, a.p.monotone_penalty, &o, &sh.sc, &sh.ssc, sh.sc2,
                                              xt_thr);
    }
    // (the local scan's flags stay; thread 0's: the categorical scan decides on thread 0 only)
    if (tid == 0 && !vote_global && !rescan) {
      flags[f] = splittable ? 1 : 0;
      o.flag = splittable ? 1 : 0;
    }
    // SerialTreeLearner::EvalFeature order: the CEGB cost (the raw candidate remembered for the
    // coupled-penalty refund), then the monotone depth penalty
    if (a.p.cegb && tid == 0) {
      const int leaf = ROOT ? 0 : sd.leaf;
      if (a.cegb_mem != nullptr) {  // (read by the pick's refunds: write-through)
        const size_t mi = static_cast<size_t>(leaf) * a.p.num_features + f;
        PublishRecord(&a.cegb_mem[mi], o);
        if (CAT) {
          PublishCatCopy(a.cegb_mem_cat + mi * kMaxCatWords, a.feat_cat + FeatBestIndex(a, side, f) * kMaxCatWords);
        }
      }
      double delta = a.p.cegb_split * L.n;
      if (a.cegb_coupled != nullptr && !a.cegb_used[f]) delta += a.cegb_coupled[f];
      if (a.cegb_lazy != nullptr) delta += a.cegb_lazy[f] * static_cast<double>(unpaid);
      o.gain -= delta;
    }
    if (!CAT && !SIMPLE && F.monotone != 0) o.gain *= MonotonePenalty(depth, a.p.monotone_penalty);
    // a forced node on this child and feature: its split at the forced threshold (published
    // for the pick, which applies it as split k)
    if (a.forced_n > 0 && tid == 0 && !vote_global && !rescan) {
      const int k = ROOT ? 0 : (s < a.forced_n ? a.forced_child[2 * s + sd.lr] : -1);
      if (k >= 0 && k < a.forced_n && a.forced_feat[k] == f) {
        FeatureBest fo = {};
        fo.flag = -1;
        int fbin;
        ForcedGather(F, hv, L, p, a.forced_thr[k], &fo, &fbin);
        if (fo.feature == -2) {
          fo.feature = f;
          fo.real_feature = F.real_index;
        }
        PublishCatSingle(a.forced_cat + static_cast<size_t>(k) * kMaxCatWords, fbin);
        PublishRecord(&a.forced_best[k], fo);
      }
    }
    if (!ROOT) KTrace(a, s, kTrFindScanned);
  } else {
    o.feature = -1;
  }
  if (tid == 0) PublishRecord(fb_out, o);
}

#ifndef LGBM_FIND_WAVE_OCC
// one-wave split scans: waves per SIMD the register budget allows.  2 (256 VGPRs): at 4 the
// non-root kernels spilled 72-76 bytes per lane, and trees grown with them changed with
// unrelated code edits (one-split-per-step categorical trees, voting ranks that disagreed)
// while the spill-free build stayed exact -- tests/test_gpu_distributed.py voting cases
#define LGBM_FIND_WAVE_OCC 2
#endif
constexpr unsigned kFindFlatMax = 128;  // split-scan grids up to this size count arrivals on one counter

// NT: threads per workgroup -- kFindThreads, or one wave (kWave) when every feature has at
// most kWave stored bins (many narrow features: four times the workgroups in flight, and no
// cross-wave steps in the scans)
template <bool ROOT, int KIND, bool SIMPLE, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == kWave ? LGBM_FIND_WAVE_OCC : 1))) void k_find(KArgs a) {
  extern __shared__ double s_bins[];  // [2][max_feature_bins] dequantised (g, h), if they fit
  __shared__ FindShared<ROOT, KIND, NT> sh;
  __shared__ PickLds pl;
  __shared__ int s_last;
  Step* st = a.st;
  if (!ROOT && st->done) return;
  if (KIND >= 2 && a.xt_base != nullptr) {
    // categorical extra_trees: the larger child's draw follows the smaller child's, whose count
    // depends on its histogram -- workgroup (f, 0) scans both children in order and appends the
    // feature's count row (over the numerical kernel's); workgroups (f, 1) only arrive
    if (blockIdx.y == 0) {
      int d0 = 0, d1 = 0;
      FindBody<ROOT, KIND, SIMPLE, NT>(a, s_bins, sh, 0, 0, &d0);
      if (!ROOT) {
        __syncthreads();
        FindBody<ROOT, KIND, SIMPLE, NT>(a, s_bins, sh, 1, d0, &d1);
      }
      if (threadIdx.x == 0) {
        const int nf = a.p.num_features, f = a.cat_list[blockIdx.x];
        const int s = ROOT ? 0 : st->cs.s;
        const int prev = ROOT ? 0 : a.xt_cum[static_cast<size_t>(s) * nf + f];
        a.xt_cum[static_cast<size_t>(ROOT ? 0 : s + 1) * nf + f] = prev + d0 + d1;
      }
    }
  } else {
    FindBody<ROOT, KIND, SIMPLE, NT>(a, s_bins, sh, blockIdx.y, 0, nullptr);
  }
  // single process: the last workgroup of the step records it and picks the next split
  // (with categorical features the numerical kernel runs first and does not count)
  if (!a.pick_in_find || (KIND == 1)) return;
  // hand-off to the picking workgroup: what it reads of this launch (per-feature results,
  // category sets, CEGB candidates, the root's leaf record) was stored write-through
  // (PublishRecord); every wave drains its stores, then one lane counts the arrival.  Other
  // results (histograms, flags) are read by later kernels only.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ArrivalRelease();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nwg = gridDim.x * gridDim.y;
    int last = 0;
    if (nwg <= kFindFlatMax) {
      last = atomicAdd(&st->find_count, 1u) == nwg - 1 ? 1 : 0;
    } else {
      // one counter serialises thousands of arrivals (~12 ns each at the memory-side atomic
      // unit, tools/microbench/wg_throughput.hip): kFindSub counters take a share each, the last
      // of a share reports to find_count (and resets its counter for the next step)
      const unsigned id = blockIdx.y * gridDim.x + blockIdx.x, g = id % kFindSub;
      const unsigned members = (nwg - g + kFindSub - 1) / kFindSub;
      uint32_t* sub = a.find_sub + g * kFindSubStride;
      if (atomicAdd(sub, 1u) == members - 1) {
        atomicExch(sub, 0u);
        last = atomicAdd(&st->find_count, 1u) == kFindSub - 1 ? 1 : 0;
      }
    }
    if (last) {  // one agent-scope acquire for the workgroup (then the barrier below)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int s = ROOT ? -1 : st->cs.s;
  if (!ROOT && a.ktrace != nullptr && threadIdx.x == 0 && s < a.p.num_leaves) {
    a.ktrace[s * kTraceSlots + kTrPickEntry] = wall_clock64();
  }
  PickAndRecord(a, st, ROOT, &pl, s, reinterpret_cast<unsigned char*>(s_bins));
  if (!ROOT && a.ktrace != nullptr && threadIdx.x == 0 && s < a.p.num_leaves) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[s * kTraceSlots + kTrPickExit] = wall_clock64();
    a.ktrace[s * kTraceSlots + kTrClk1] = __builtin_amdgcn_s_memtime();
  }
}

// the step's bookkeeping and the next pick alone (distributed learners)
__global__ __launch_bounds__(kFindThreads) void k_pick(KArgs a, int root) {
  __shared__ PickLds pl;
  Step* st = a.st;
  if (st->done) return;
  PickAndRecord(a, st, root != 0, &pl);
}

static size_t FindLds(const KArgs& a) {
  const size_t bins = a.p.max_feature_bins <= kFindLdsBins ? 2 * sizeof(double) * static_cast<size_t>(a.p.max_feature_bins) : 0;
  // intermediate monotone: the picking workgroup walks the tree in this LDS (MonoInterLds)
  return a.p.mono_inter ? std::max(bins, MonoInterLds(a.p.num_leaves)) : bins;
}
// plain gain formulas (no L1 / max_delta_step / path smoothing / monotone constraints)
static bool SimpleGains(const KArgs& a) {
  const SplitParams& p = a.p.sp;
  return !p.use_l1 && !p.use_max_output && !p.use_smoothing && !p.use_mc;
}
template <bool ROOT>
static void LaunchFind(const KArgs& a, hipStream_t s) {
  if (a.num_scan <= 0) return;  // a rank that owns no feature
  // (intermediate monotone: sides 2.. re-scan up to num_leaves re-bounded leaves)
  const int sides = ROOT ? 1 : (a.p.mono_inter ? 2 + a.p.num_leaves : 2);
  const dim3 g(a.num_scan, sides);
  const size_t lds = FindLds(a);
  const bool simple = SimpleGains(a);
  const bool narrow = a.p.max_feature_bins <= kWave;  // (categorical scans keep kFindThreads)
  const dim3 b(narrow ? kWave : kFindThreads), bc(kFindThreads);
  if (a.p.has_cat) {
    if (narrow) {
      if (simple) hipLaunchKernelGGL((k_find<ROOT, 1, true, kWave>), g, b, lds, s, a);
      else hipLaunchKernelGGL((k_find<ROOT, 1, false, kWave>), g, b, lds, s, a);
    } else {
      if (simple) hipLaunchKernelGGL((k_find<ROOT, 1, true, kFindThreads>), g, b, lds, s, a);
      else hipLaunchKernelGGL((k_find<ROOT, 1, false, kFindThreads>), g, b, lds, s, a);
    }
    const int ncat = a.p.vote_phase == 2 ? a.num_scan : a.p.has_cat;  // voting: every elected slot
    if (a.p.has_cat > 0 && a.p.wide_cat) hipLaunchKernelGGL((k_find<ROOT, 3, false, kFindThreads>), dim3(ncat, sides), bc, lds, s, a);
    else if (a.p.has_cat > 0) hipLaunchKernelGGL((k_find<ROOT, 2, false, kFindThreads>), dim3(ncat, sides), bc, lds, s, a);
  } else if (narrow) {
    if (simple) hipLaunchKernelGGL((k_find<ROOT, 0, true, kWave>), g, b, lds, s, a);
    else hipLaunchKernelGGL((k_find<ROOT, 0, false, kWave>), g, b, lds, s, a);
  } else {
    if (simple) hipLaunchKernelGGL((k_find<ROOT, 0, true, kFindThreads>), g, b, lds, s, a);
    else hipLaunchKernelGGL((k_find<ROOT, 0, false, kFindThreads>), g, b, lds, s, a);
  }
}
void FindRoot(const KArgs& a, hipStream_t s) { LaunchFind<true>(a, s); }
void FindStep(const KArgs& a, hipStream_t s) { LaunchFind<false>(a, s); }
void PickStep(const KArgs& a, hipStream_t s, bool root) {
  hipLaunchKernelGGL(k_pick, dim3(1), dim3(kFindThreads), 0, s, a, root ? 1 : 0);
}

}  // namespace dev
}  // namespace lgbm_amd
