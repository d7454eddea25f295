// POD records shared by the HIP kernels (src/device/*.hip) and the host orchestration
// of the MI355X tree learner (src/treelearner/gpu_tree_learner.cpp).  All of them live
// in HBM for the whole training run; the host only writes them at (re)initialisation and
// reads the per-tree split records back once per tree.
#pragma once

#include <cstdint>

#include "lgbm_amd/split_info.h"
#include "lgbm_amd/split_math.h"

namespace lgbm_amd {
namespace dev {

constexpr int kMaxLeaves = 1024;  // device-mode tree size limit (num_leaves)
constexpr int kFindSub = 32;      // split-scan arrival sub-counters (KArgs::find_sub)
constexpr int kFindSubStride = 32;  // uint32 words between sub-counters: one 128-byte line each

// interleaved (gradient, hessian) of one row: one 8-byte gather per row
struct alignas(8) GH {
  float g;
  float h;
};

// per inner feature, everything the split scan and the partition need
struct Feature {
  int32_t group;        // storage column (feature group)
  int32_t hist_offset;  // first histogram bin of this feature (Dataset::FeatureHistOffset)
  int32_t num_bin;      // BinMapper::num_bin
  int32_t offset;       // 1 when the most frequent bin is 0 (bin 0 is not stored)
  int32_t default_bin;
  int32_t mfb;          // most frequent bin
  int32_t missing_type;  // 0 none, 1 zero, 2 NaN
  int32_t is_cat;
  int32_t sub_lo, sub_hi;  // this feature's [lo, hi) range inside the group's bin space
  int32_t real_index;
  int32_t monotone;
  // where the group's bin sits: byte offset inside a row of the row-major matrix, its width
  // there -- 0 8-bit, 1 16-bit, 2 / 3 the low / high 4 bits of the byte (4-bit storage,
  // GroupBinOf) -- and the byte offset of its column in the column-major copy (one byte per
  // row for 8- and 4-bit groups)
  int32_t gbyte;
  int32_t gwide;
  int64_t col_off;
  double penalty;
};

// tree-growth parameters (uniform for the launch)
struct Params {
  SplitParams sp{};
  int32_t num_leaves{};
  int32_t max_depth{};
  int32_t num_features{};
  int32_t num_groups{};
  int32_t row_stride{};  // bytes (or uint16 elements) per row in the bin matrix
  int32_t total_bins{};  // histogram length in bins
  double monotone_penalty{};
  int32_t data_parallel{};  // leaf sizes/decisions from global (split-estimated) counts
  int32_t max_feature_bins{};  // max stored bins of one feature (split-scan LDS staging)
  int32_t has_cat{};           // number of categorical features (KArgs::cat_list; their own split-scan kernel)
  int32_t wide_cat{};          // some categorical feature has > kFindCatNarrow bins (the wide categorical kernel)
  int32_t direct_from_split{}; // splits >= this have no reduce kernel: the split scan sums the partials
  int32_t trace_repeat{};      // diagnostics (LGBM_AMD_KTRACE_REPEAT): run the traced pick twice
  // voting-parallel split scans (reference voting_parallel_tree_learner.cpp): 0 off, 1 the
  // local scan (rank-local sums / counts / parameters, every feature), 2 the global scan of the
  // elected features (KArgs::vote_list, histograms in KArgs::vote_hist)
  int32_t vote_phase{};
  int32_t vote_k{};  // top_k: features each rank proposes and the vote elects, per leaf
  int32_t world{};   // ranks
  // > 0: 1 + min_data_in_leaf of the children-skip rule (StepChildren) when sp holds other
  // parameters -- voting's local scans run with min_data_in_leaf / world, but the reference
  // skips a step's scans by the global parameter (SerialTreeLearner::BeforeFindBestSplit)
  int32_t skip_min_data{};
  // cost-effective gradient boosting (split and coupled feature penalties): a candidate's gain
  // loses cegb_split * rows_in_leaf + KArgs::cegb_coupled[f] while f is unused by the model
  int32_t cegb{};
  double cegb_split{};
  // intermediate monotone constraints (KArgs::mt_*): a split re-bounds leaves across the tree,
  // which the next split scan re-scans
  int32_t mono_inter{};
};

// per-leaf state
// interaction-constraint sets of a leaf / feature: bit k of the words is constraint k (up to
// kMaxIcConstraints; more run host-assisted).  constexpr helpers (host and device)
constexpr int kIcWords = 4;
constexpr int kMaxIcConstraints = 64 * kIcWords;
struct IcMask {
  uint64_t w[kIcWords];
  constexpr IcMask operator&(const IcMask& o) const {
    IcMask r{};
    for (int i = 0; i < kIcWords; ++i) r.w[i] = w[i] & o.w[i];
    return r;
  }
  constexpr void Set(int k) { w[k >> 6] |= uint64_t{1} << (k & 63); }
};
// any constraint in common (a leaf may split on a feature iff IcAny(leaf & feature))
constexpr bool IcAny(const IcMask& m) {
  uint64_t x = 0;
  for (int i = 0; i < kIcWords; ++i) x |= m.w[i];
  return x != 0;
}
static_assert(kIcWords == 4, "kIcAll lists kIcWords words");
constexpr IcMask kIcAll = {{~uint64_t{0}, ~uint64_t{0}, ~uint64_t{0}, ~uint64_t{0}}};

struct Leaf {
  int32_t begin;         // local index range in the partition array
  int32_t count;         // local rows
  int32_t global_count;  // rows over all ranks (== count without data-parallel)
  int32_t depth;
  int32_t slot;          // histogram slot
  int32_t buf;           // which index buffer (KArgs::idx / tmp) holds the leaf's rows
  int32_t frow;          // row of KArgs::splittable (kept across trees; round growth: the leaf's RNode)
  int32_t pad;
  IcMask icmask;        // interaction constraints consistent with the leaf's branch (bit k: constraint k)
  double sum_g, sum_h, output;
  double lsum_g, lsum_h;  // voting-parallel: this rank's (local) sums of the leaf's rows
  double cmin, cmax;  // monotone constraint range
};

// a child's statistics as known from its parent's split (plus, once the partition is done,
// its histogram slot)
struct ChildStats {
  double sum_g, sum_h, output, cmin, cmax;
  int32_t global_count, depth, slot, leaf;
  int32_t frow;        // splittable row the child's scan writes
  IcMask icmask;       // Leaf::icmask
};

// the split being applied, as chosen by the partition kernel's pick
struct CurSplit {
  int32_t s;            // split index
  int32_t leaf, new_leaf;
  int32_t part_begin, part_count;  // the leaf's rows before the split
  int32_t src_buf;      // index buffer holding them (the children go to the other one)
  int32_t child_depth;
  int32_t parent_slot;  // histogram slot of the leaf (the new leaf's slot is its own id)
  int32_t parent_frow, new_frow;  // splittable rows of the leaf and of the new leaf
  double plsum_g, plsum_h;  // voting-parallel: the leaf's local sums (Leaf::lsum_*)
  Feature feat;         // the split feature's record
  DeviceSplit split;
};

// per-tree control record.  Each field is written by one kernel of a step and only read by
// later kernels (or by the writing workgroup itself):
//   pick (last split-scan workgroup, or k_pick): cs, lr, hist_left, bookkeeping fields
//   split (k_split, atomics): cursors
//   split scan (atomics): find_count
struct Step {
  int32_t done;       // tree finished: every later kernel of the tree exits
  int32_t nsplit;     // splits applied (= index of the next split)
  int32_t fresh;      // leaves with new per-feature results in feat_best: 0, 1 (root), 2
  int32_t smaller, larger;
  int32_t hist_left;  // k_split histograms the left child of cs (the pick's estimated counts), else the right
  uint32_t find_count;  // split-scan workgroups of the step that finished (the last one picks)
  int32_t root_count;   // global rows of the tree's root
  int32_t bynode_base, bynode_next;  // per-node feature masks: this step's / next free mask index
  int32_t cur_left, cur_right;      // partition cursors: rows placed left / right so far
  int32_t forced_abort;             // forced splits: a forced split was invalid; normal picks from then on
  // voting-parallel: fixed-point (g, h) sums of the rows k_split histogrammed (the local sums
  // of that child), accumulated with atomics; cleared by the pick
  unsigned long long loc_acc[2];
  CurSplit cs;
  ChildStats lr[2];     // left / right child of cs
};

// best threshold of one feature for one leaf (output of one split-scan wave)
// one bin's inclusive prefix over a feature's bins of a node (extra_trees rounds, KArgs::
// node_pre): (g, h) sums and the rows estimated per bin, the default bin left out as the scan
// leaves it out
struct XtPre {
  double g, h;
  int32_t c;
  int32_t pad;
};

struct FeatureBest {
  double gain;
  double lg, lh, rg, rh, lo, ro;
  int32_t feature, real_feature, thr, default_left, lc, rc, mono;
  int16_t ncat;  // categorical: categories in the left set (KArgs::feat_cat, <= kFindMaxCatBins); 0: numerical
  // the scan's "feature had a valid split" flag it wrote into KArgs::splittable (-1: none
  // written) -- gathered with the record, so distributed rounds complete every rank's rows
  int8_t flag;
  int8_t pad;
};
static_assert(sizeof(FeatureBest) == 88, "FeatureBest: eleven 8-byte words");

// voting-parallel: one rank's proposal for a leaf (reference LightSplitInfo: the local best
// split's gain and its local row count)
struct VoteEntry {
  double gain;
  int32_t feature;  // inner feature index, -1: none
  int32_t count;    // local rows of the leaf (left + right count of the local split)
};

// record of one applied split, read back by the host to rebuild the Tree
struct SplitRecord {
  int32_t leaf;
  int32_t left_count, right_count;  // counts stored in the model (global)
  int32_t pad;
  DeviceSplit split;
};

// ---- round growth (speculative multi-leaf expansion, round_kernels.hip)
// Leaf-wise growth applies one split at a time, but expanding a leaf -- partitioning its rows
// by its best split, histogramming and scanning both children -- depends on that leaf's rows
// only.  A round expands up to KArgs::round_k leaves at once (the current leaves of highest
// gain); the planner then replays the sequential best-first order (reference
// serial_tree_learner.cpp:152-202): it accepts the argmax leaf while its expansion is
// computed and stops at the first one whose expansion is not, which the next round expands.
// Expansions never accepted only cost work: histograms are exact integer sums, so the rows a
// pending expansion reordered inside its leaf's range change nothing.
//
// Speculation also reaches below the leaves: the children of an expanded leaf that is not
// accepted yet are 'virtual' nodes with exact best splits, rows (in the expansion's output
// buffer) and histograms, so the planner may expand them too (up to KArgs::round_vmax levels
// below a leaf), and a replay then accepts whole chains of splits.  Nodes are indexed by their
// splittable row (Leaf::frow).  A node at depth d reads index buffer d mod M and writes its
// children to (d + 1) mod M, M = round_vmax + 2 buffers: no expansion at most round_vmax
// levels below a leaf rewrites the buffer holding that leaf's rows, so every leaf's rows stay
// valid whichever of the speculative expansions below it the tree never accepts.
constexpr int kMaxRoundExp = 16;  // nodes expanded per round, upper bound
constexpr int kMaxRoundVmax = 14;  // speculation depth below a leaf, upper bound (buffers: + 2)

// one node being expanded by the current round (written by the planner)
struct ExpPlan {
  int32_t node;                  // the node (its splittable row)
  int32_t part_begin, part_count, src_buf, dst_buf;
  int32_t hist_left;             // the left child's rows are histogrammed (fewer by the estimate), else the right's
  int32_t blk_off, nblk;         // the expansion's row blocks inside the round's partial histograms
  int32_t slot_parent, slot_new;  // histogram slots: the subtracted child keeps the parent's, the histogrammed one is new
  int32_t frow_parent;           // the leaf's splittable row (its children skip what it could not split)
  int32_t frow_child[2];         // the children's rows (fresh rows)
  Feature feat;                  // the split feature's record
  DeviceSplit split;
  ChildStats lr[2];              // left / right child as known from the split
};

// one node of a tree under round growth (index: its splittable row): the root and both
// children of every expansion; written by the planner only
struct RNode {
  int32_t begin, count, buf;  // rows (local; known once the round expanding its parent is partitioned)
  int32_t expanded;           // its best split was applied: children child, child + 1
  int32_t child;
  int32_t total_left;         // expanded: local rows that went left
  ChildStats st;              // statistics from the parent's split (the root: its leaf's)
};

// per-tree control record of round growth
struct Round {
  int32_t done;       // tree finished: every later kernel of the tree exits
  int32_t nsplit;     // splits accepted so far
  int32_t nexp;       // expansions of the current round
  int32_t round;      // index of the current round (reduce-buffer parity)
  int32_t rpb;        // rows per row block of the current round
  int32_t nblk;       // row blocks of the current round (all expansions)
  int32_t next_slot, next_frow;  // next free histogram slot / splittable row
  int32_t rounds;     // rounds planned (diagnostics)
  int32_t accepted_max;  // most splits accepted by one round (diagnostics)
  uint32_t child_done;   // children of the round whose best split is folded (plan in the split scan)
  int32_t k_cur;         // expansions per round for this tree (set by the host; 0: KArgs::round_k)
  int32_t bynode_next;   // per-node sampling on round growth: the next draw (row of KArgs::node_mask)
  int32_t cur[kMaxRoundExp][2];  // partition cursors of each expansion: rows placed left / right
  // voting-parallel: the fixed-point (g, h) sums of each expansion's histogrammed child over
  // this rank's rows (its local sums; the other child's are the parent's minus these)
  unsigned long long loc_acc[kMaxRoundExp][2];
  ExpPlan e[kMaxRoundExp];
};

}  // namespace dev
}  // namespace lgbm_amd
