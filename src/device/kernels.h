// Host-side launch interface of the MI355X tree-learner kernels (src/device/kernels.hip).
// Every launcher is stream-ordered and performs no host synchronisation, so a whole tree
// (root + num_leaves-1 split steps) can be enqueued back to back or captured into one
// hipGraph.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "device_types.h"

namespace lgbm_amd {
namespace dev {

// pointers and constants shared by the tree-growth kernels
struct KArgs {
  Params p{};
  const void* bins{};          // row-major bin matrix, [rows][row_stride] of uint8 / uint16
  const Feature* feat{};       // [num_features]
  const int32_t* group_off{};  // [num_groups] first histogram bin of each storage column
  const int8_t* tree_mask{};   // [num_features] feature used by this tree
  const int8_t* node_mask{};   // [2 * num_leaves - 1][num_features] per-node samples (feature_fraction_bynode), or null
  // per-node sampling under interaction constraints (bynode_rng non-null; k_bynode_step draws
  // the children's node_mask rows): the tree's node pool (inner features in the host sampler's
  // order), the sample size before filtering, the generator state, a [num_features] scratch
  const int32_t* bynode_pool{};
  int32_t bynode_pool_n{}, bynode_cnt{};
  uint32_t* bynode_rng{};
  int32_t* bynode_scratch{};
  const GH* gh{};              // interleaved (gradient, hessian) per row
  int32_t* idx{};              // partition index buffer 0 (root rows)
  int32_t* tmp{};              // partition index buffer 1 (leaves alternate: Leaf::buf), then 2.. at buf_stride
  int64_t buf_stride{};        // int32 between index buffers 1, 2, ... (round growth: RowBuf)
  Leaf* leaves{};              // [num_leaves]
  Step* st{};
  SplitRecord* rec{};          // [num_leaves - 1]
  // round growth, one process: pinned host memory (fine-grained) the last plan of a tree fills
  // with the tree's split records (from word kHostOutHeaderWords) and then its scalars
  // [done, splits, rounds, nodes] -- the host waits on that flag instead of the stream (null:
  // the host copies the Round record and the records)
  int32_t* host_out{};
  DeviceSplit* best{};         // [num_leaves]
  // histograms hold fixed-point sums: int64 (g * scale_g, h * scale_h) per bin, exact and
  // order-independent (LDS float atomics are slow on gfx950; integer ones are not)
  long long* hist{};           // [num_leaves][total_bins][2]
  long long* scratch{};        // [2][scratch_stride] the histogram being built (step parity)
  int64_t scratch_stride{};    // int64 per parity buffer: 2 * total_bins, or the padded owner-major layout
  // per-row-block partial histograms, [hist_max_blocks][total_bins][hist_units] u64: one packed
  // (g | h) word per bin (hist_units 1) or int64 g, int64 h (hist_units 2, gpu_use_dp)
  unsigned long long* partials{};
  const double* scales{};      // [scale_g, scale_h, 1/scale_g, 1/scale_h] of the current tree
  double* root{};              // [sum_g, sum_h, count]
  double* root_blk{};          // [2 * 2 * CUs] per-workgroup partials of RootSum (summed in a fixed order)
  int32_t num_rows{};          // local rows in the root (or the explicit range); upper bound if num_rows_dev
  const int32_t* num_rows_dev{};  // root rows held on the device (a bag drawn on the device), or null
  int32_t root_identity{};     // root rows are 0..num_rows-1 (indices written by the root pass)
  // row layout: every group 8-bit (bin_bytes 1, 4 per word), every group 16-bit (2, 2 per
  // word), or mixed (0): each word holds 8-bit groups or 16-bit groups only, in group order
  // (a 16-bit group starts a new word), word_g0 / word_wide describe the words.  nibbles: every
  // group has at most 16 bins and sits in 4 bits, eight to a word (bin_bytes is then 1: the
  // groups are byte-addressable as (byte >> 4 * high) & 15, Feature::gwide 2 / 3)
  int32_t bin_bytes{};
  int32_t nibbles{};
  int32_t words_per_row{};     // 32-bit words of bins per row
  // 32-bit words between consecutive rows of `bins` (>= words_per_row).  With gh_stride > 1 the
  // rows carry their (g, h) in their last two words (gh points at row 0's): a gathered row is
  // one 64-B (or 128-B) line instead of a bins row straddling lines plus a separate (g, h) line
  int32_t row_words{};
  int64_t gh_stride{};         // GH elements between consecutive rows' (g, h): 1 (compact array) or row_words / 2
  const int32_t* word_g0{};    // [words_per_row + 1] first group of each word (mixed layouts)
  const int8_t* word_wide{};   // [words_per_row] word holds 16-bit groups (mixed layouts)
  // row-sparse storage (reference MultiValSparseBin, multi_val_sparse_bin.hpp): the stored
  // histogram bins of row r -- group_off[g] + bin for every group whose bin is not 0,
  // ascending -- are sp_bin[sp_ptr[r] .. sp_ptr[r + 1]); null: the word matrix `bins`.  The
  // histogram column tiles are then plain bin ranges of tile_bins each
  const int64_t* sp_ptr{};
  const uint16_t* sp_bin{};
  int32_t sp_team{};           // threads per row of a row-sparse gather (4..64, by the mean stored bins)
  int32_t hist_tiles{};        // column tiles of the histogram kernel
  int32_t tile_words{};        // words per column tile
  int32_t tile_bins{};         // max histogram bins of one tile (LDS words)
  int32_t range_begin{};       // explicit-range histogram (host-assisted mode)
  int32_t hist_rows_cap{};     // max rows of one row block (packed fixed-point headroom; fixed, not a function of N)
  int32_t hist_max_blocks{};   // row blocks of a histogram (partials capacity)
  int32_t hist_units{};        // u64 words per histogram bin in LDS / partials: 1 packed, 2 wide (gpu_use_dp)
  int32_t split_grid{};        // workgroups of a k_split launch (row blocks are dealt round-robin)
  int32_t root_grid{};         // workgroups of a root / range histogram launch
  int32_t blk_min_rows{};      // k_split: parent rows per row block, lower bound
  int32_t pick_in_find{};      // the last split-scan workgroup of a step picks the next split (else k_pick)
  // distributed learners (reference data_parallel_tree_learner.cpp / feature_parallel_*):
  // features are owned by ranks in storage-group blocks; a rank scans its own.  Data-parallel
  // with feature_fraction < 1 re-assigns the tree's used groups to the least-loaded rank by
  // bins every tree (reference DataParallelTreeLearner::BeforeTrain); slots past the rank's
  // features hold -1 (the grids keep one size for the captured graphs)
  const int32_t* feat_list{};  // [num_scan] inner features this rank scans (null: all; -1: none)
  int32_t num_scan{};          // features this rank scans (capacity)
  const int32_t* fb_index{};   // feat_best slot of feature f for side 0 (null: f); side 1 adds fb_side
  int32_t fb_side{};
  // data-parallel: the reduce kernel writes bin b at rs_pos[b] (owner-major blocks, padded
  // to equal size for the reduce-scatter; -1: a group no rank scans this tree) and the split
  // scan reads owned feature f's globally summed bins from owned_hist at 2 * owned_off[f];
  // null: the local scratch
  const int32_t* rs_pos{};
  const long long* owned_hist{};
  const int32_t* owned_off{};
  int32_t owned_bin_lo{};
  // histogram column range (feature-parallel: the words of this rank's features)
  int32_t tile_w0{}, tile_w1{};
  const uint8_t* bins_col{};   // column-major copy of the bin matrix (group columns at Feature::col_off)
  int32_t num_data{};          // rows of the matrix (column stride of bins_col)
  int32_t host_mode{};         // partition: the host wrote Step::cs (host-assisted growth)
  FeatureBest* feat_best{};    // [2][num_features] per-feature best split of the two leaves
  uint32_t* feat_cat{};        // [2][num_features][kMaxCatWords] category sets of categorical bests
  long long* ktrace{};         // optional [num_leaves][kTraceSlots] in-kernel timestamps (LGBM_AMD_KTRACE)
  // per-leaf "feature had a valid split" flags (the host learner's splittable_ rows): a
  // child skips a feature its parent could not split.  Rows are reached through Leaf::frow
  // (swapped with the histogram hand-over) and persist across trees, as the host rows do;
  // parent_flags is the parent's row, snapshot by the partition kernel
  int8_t* splittable{};        // [num_leaves][num_features]
  int8_t* parent_flags{};      // [num_features]
  const int32_t* cat_list{};   // [Params::has_cat] the categorical features
  // interaction constraints (<= 32): bit k set iff constraint k holds the feature, or null.
  // A leaf may split on f iff IcAny(Leaf::icmask & feat_icmask[f]) (ColSampler::GetByNode)
  const IcMask* feat_icmask{};  // [num_features]
  // extra_trees: each feature's generator state at the tree's start (FeatureMeta::rand) and the
  // running count of its draws, one row per split step (row 0: the root scan, row s + 1: after
  // step s; rows of steps not run stay 0), or null
  const uint32_t* xt_base{};   // [num_features]
  int32_t* xt_cum{};           // [num_leaves][num_features]
  // voting-parallel extra_trees: the global scans draw from a second generator set, only on the
  // rank that owns the elected histogram (reference voting_parallel_tree_learner.cpp:61-90,
  // CopyLocalHistogram); every rank replays every owner's draws: the states of every rank's set
  // at the tree's start ([world][num_features]) and their running counts ([num_leaves][world]
  // [num_features], rows as xt_cum), or null.  The local scans draw from xt_base / xt_cum.
  const uint32_t* xt_base_glob{};
  int32_t* xt_cum_glob{};
  // voting-parallel (Params::vote_phase): this rank's root sums before the all-reduce, the
  // proposals of every rank ([world][2][vote_k], this rank's block at rank), the elected
  // features per leaf ([2][vote_k], -1 padded) and their histograms ([2][vote_k][max_feature_bins]
  // (g, h) int64, summed over the ranks before the global scan)
  // CEGB (Params::cegb): tradeoff * coupled penalty per inner feature (or null), the model-wide
  // "feature already split on" flags, and every (leaf, feature) raw candidate ([num_leaves]
  // [num_features], category sets alongside) for the refund when a feature is first used
  const double* cegb_coupled{};
  int8_t* cegb_used{};
  FeatureBest* cegb_mem{};
  uint32_t* cegb_mem_cat{};
  // CEGB lazy penalties (cegb_penalty_feature_lazy; reference cost_effective_gradient_boosting.hpp
  // CalculateOndemandCosts / UpdateLeafBestSplits): tradeoff * penalty per inner feature, or
  // null; a row-major bitset of the (row, feature) pairs already paid for (cegb_paid_words words
  // per row, kept over the model); every leaf's count of unpaid rows per feature; per step
  // parity, the histogrammed child's counts and the split leaf's snapshot (k_cegb_step)
  const double* cegb_lazy{};
  uint32_t* cegb_paid{};
  int32_t cegb_paid_words{};
  int32_t* cegb_cnt{};      // [num_leaves][num_features]
  int32_t* cegb_scratch{};  // [2][num_features]
  int32_t* cegb_snap{};     // [2][num_features]
  // intermediate monotone constraints (Params::mono_inter; reference monotone_constraints.hpp
  // IntermediateLeafConstraints, host src/treelearner/monotone_constraints.cpp): the tree's
  // topology as the picks grow it, each leaf's membership of a monotone subtree, and the leaves
  // the last split re-bounded (mt_upd[0] of them, then their ids), which the next split scan
  // re-scans as sides 2.. (feat_best rows 2..) and the next pick folds into KArgs::best
  int32_t* mt_leaf_parent{};  // [num_leaves] internal node above each leaf (-1: the root leaf)
  int32_t* mt_node{};         // [num_leaves - 1][3] parent, left, right (child >= 0 node, else ~leaf)
  int8_t* mt_in_sub{};        // [num_leaves]
  int32_t* mt_upd{};          // [1 + num_leaves]
  // forced splits (reference serial_tree_learner.cpp ForceSplits), in the static BFS order of
  // the forced-split JSON tree: node k is applied as split k (while every earlier one was valid)
  // to leaf forced_leaf[k] on inner feature forced_feat[k] at bin forced_thr[k]; the children
  // of split s carry nodes forced_child[2s] (left) / forced_child[2s + 1] (right) or -1.  The
  // split scan of such a child's feature fills forced_best / forced_cat[k] (the reference's
  // GatherInfoForThreshold), the pick applies it
  int32_t forced_n{};
  const int32_t* forced_feat{};
  const int32_t* forced_thr{};
  const int32_t* forced_leaf{};
  const int32_t* forced_child{};
  FeatureBest* forced_best{};
  uint32_t* forced_cat{};
  // feature-parallel: forced_best / forced_cat are this rank's block of forced_world blocks of
  // forced_n records, gathered after each scan; the pick takes the owner's (the only valid one)
  int32_t forced_world{};
  const FeatureBest* forced_all{};
  const uint32_t* forced_cat_all{};
  // arrival sub-counters of large split-scan grids, [kFindSub] at kFindSubStride words: each on
  // a cache line of its own (atomics to one line serialise like atomics to one word)
  uint32_t* find_sub{};
  const double* root_local{};
  VoteEntry* vote_buf{};
  int32_t vote_rank{};
  int32_t* vote_list{};
  long long* vote_hist{};
  // round growth (round_kernels.hip; null rd: one split per step): up to round_k nodes are
  // expanded per round.  Their children's per-feature results go to feat_best rows 2j + lr,
  // each child node's best split to cbest[node] (category sets in cbest_cat); child_cnt holds
  // each child's split-scan arrival counters ([2 * kMaxRoundExp][kFindSub], kFindSubStride
  // apart); the reduced histogram of expansion j sits at scratch + (parity * round_k + j) * 2 *
  // total_bins
  Round* rd{};
  RNode* rnode{};            // [round_nodes] the tree's nodes (index: splittable row)
  FeatureBest* cbest{};      // [round_nodes] each node's best split
  uint32_t* cbest_cat{};     // [round_nodes][kMaxCatWords]
  uint32_t* child_cnt{};
  int32_t round_k{};
  int32_t round_vmax{};   // speculation depth below a leaf (index buffers: round_vmax + 2)
  int32_t round_nodes{};  // node capacity (splittable rows of a tree)
  int32_t round_emax{};   // expansions of a tree, upper bound (histogram slots - 1, (round_nodes - 1) / 2)
  int32_t round_need_div{};  // > 0: at most max(1, splits still possible / round_need_div) picks per round (A/B: off)
  int32_t round_predict{};   // the next round's picks: 1 bottleneck order keys (PredictBottleneck), 0 the step-by-step walk
  int32_t round_grid{};  // workgroups of a round's split kernel (row blocks: the round's rows / round_grid)
  int32_t round_gr{};    // independent row gathers per thread in its histogram phase (2, 4, 8)
  int32_t round_fused{};  // 1: partition + histograms in one kernel (k_round_split), 0: two (k_round_part, k_round_hist)
  int32_t plan_in_find{};  // the round's last split-scan workgroup plans (else k_round_plan)
  // distributed round growth (data- / feature-parallel): per-feature results rank-major,
  // [world][2 * round_k][max_owned] (a rank's local feature index from fb_index), all-gathered
  // before k_round_childbest; data-parallel: the round's histograms reduced into round_send
  // ([world][round_k][rs_block][2] int64, owner-major), reduce-scattered into round_owned
  // ([round_k][rs_block][2]: this rank's owned bins of every expansion)
  int32_t round_dist{};
  // voting-parallel round growth: phase 1 scans every feature of both children of every
  // expansion on this rank's histograms and sums (Params::vote_phase 1); the round's proposals
  // ([world][2 * round_k][vote_k] in vote_buf), elected features ([2 * round_k][vote_k] in
  // vote_list) and their histograms ([2 * round_k][vote_k][2 * max_feature_bins] in vote_hist)
  // feed phase 2, the global scan of the elected features (grid (vote_k, 2 * round_k))
  int32_t round_vote{};
  double* rnode_lsum{};  // voting rounds: this rank's (g, h) sums of every node's rows, [round_nodes][2]
  int32_t max_owned{};
  int32_t rs_block{};
  long long* round_send{};
  long long* round_owned{};
  // per-node feature sampling on round growth (one process, no interaction constraints): the scans
  // evaluate every feature of a node (KArgs::node_mask is not applied) and keep the per-feature
  // results per node (node_fb [round_nodes][num_features]); the replay folds a node's results
  // with its sample once it knows the split that created the node (draw 1 + 2 s, smaller child
  // first) and keeps the reference's splittable flags per leaf id (leaf_rows [num_leaves]
  // [num_features], persisting across trees; the children scan with their parent's leaf row).
  // Speculation stays at the current leaves (the draws of deeper nodes are not known yet)
  int32_t round_bynode{};
  FeatureBest* node_fb{};
  int8_t* leaf_rows{};
  // extra_trees on round growth (one process, numerical features without a rebuilt most
  // frequent bin): each random threshold is the next draw of its feature's generator in the
  // sequential order, so a scan cannot know it.  The scans store every node's per-bin inclusive
  // prefix sums (node_pre [round_nodes][total_bins]; exact: the bins are integers on the
  // fixed-point grid) and the replay draws each child's thresholds in the host loop's order
  // (smaller child first, per feature) and evaluates them from the prefixes; the draws counted
  // so far are xt_cum row 1.  Flags per leaf id as with per-node sampling (leaf_rows)
  int32_t round_xt{};
  XtPre* node_pre{};
  // CEGB coupled penalties on round growth (one process, no lazy penalties or monotone
  // constraints): the scans publish raw candidates (node_fb); the replay refunds a feature's
  // first use to the other leaves, remembers each child's candidates (cegb_mem, per leaf id)
  // and subtracts the penalties of the used set it has reached; the plan expands only leaves
  // no refund can change (and the blocker, which is accepted before any other split)
  int32_t round_cegb{};
  // per-node sampling with categorical features: each categorical feature's category set per
  // node ([round_nodes][node_cat_slots][kMaxCatWords]; node_cat_slot: the feature's slot, -1
  // for a numerical one), copied to the node's best when the replay picks it
  uint32_t* node_fb_cat{};
  const int32_t* node_cat_slot{};
  int32_t node_cat_slots{};
};

// in-kernel timestamp slots (first workgroup, first thread; constant 100 MHz clock)
enum TraceSlot {
  kTrSplitEntry = 0, kTrSplitRows, kTrSplitSide, kTrSplitResv, kTrSplitGather, kTrSplitAccum, kTrSplitExit,
  kTrRedEntry, kTrRedExit,
  kTrFindEntry, kTrFindLoaded, kTrFindScanned, kTrFindExit, kTrPickEntry, kTrPickExit,
  kTrPick1, kTrPick2, kTrPick3, kTrPick4, kTrFindHdr, kTrPW1, kTrPW2, kTrPickRep,
  kTrClk0 = 28, kTrClk1 = 29,  // s_memtime (shader clock) at kTrPick1 / kTrPickExit
  kTraceSlots = 32
};

constexpr int kFindMaxCatBins = 4096;  // categorical features scanned on device (<= 32 * kMaxCatWords)
constexpr int kFindCatNarrow = 1024;   // ... by the regular categorical kernel; wider ones by its wide variant
constexpr int kHistThreads = 1024;     // histogram workgroup (16 waves)
constexpr int kSparsePerThread = 4;    // row-sparse gathers: entries per thread and row loaded up front
constexpr int kHistMinRows = 1024;     // rows per histogram row block, lower bound
constexpr int kHistRowsCap = 16384;    // rows per row block, upper bound (packed fixed point)
#ifndef LGBM_REDUCE_CHUNK
#define LGBM_REDUCE_CHUNK 32
#endif
constexpr int kReduceChunk = LGBM_REDUCE_CHUNK;  // partial histograms summed per reduce thread
#ifndef LGBM_DIRECT_CHUNK
#define LGBM_DIRECT_CHUNK 16
#endif
// a step histogram of at most this many row blocks is summed by the split scan itself, every
// block's partial of a bin loaded in one round of independent loads (no reduce kernel)
constexpr int kDirectChunk = LGBM_DIRECT_CHUNK;
constexpr int kPartThreads = 1024;
constexpr int kSplitRows = 4;          // k_split: rows per thread of a sub-tile
constexpr int kSplitSub = kPartThreads * kSplitRows;

// row blocks (partial histograms) of `count` rows on a grid of `grid` workgroups: a multiple
// of the grid once the rows exceed one block per workgroup (every workgroup then handles
// the same number of blocks), blocks of at least min_rows and at most rows_cap rows.
// Deterministic: shared by the histogram, reduce and split-scan kernels.
__host__ __device__ inline int HistBlocksFor(int count, int grid, int rows_cap, int min_rows) {
  if (count <= 0) return 0;
  const long long per_round = static_cast<long long>(grid) * rows_cap;
  const int rounds = static_cast<int>((count + per_round - 1) / per_round);
  const long long target = static_cast<long long>(rounds) * grid;
  int rpb = static_cast<int>((count + target - 1) / target);
  if (rpb < min_rows) rpb = min_rows;
  return (count + rpb - 1) / rpb;
}

int HistGridBlocks();  // workgroups of a root histogram (2 per CU)
void PrepareKernels();  // per-kernel attributes (large dynamic LDS); once per process, before any capture
void SetNumCUs(int n);

// interleave (g, h); per-workgroup max|g| / max h into max_parts[PackBlocks(n)][2]
void PackGH(const float* g, const float* h, GH* gh, int64_t gh_stride, int64_t n, float* max_parts, hipStream_t s);
int PackBlocks(int64_t n);
// fixed-point scales of this tree from absmax: packed (hist_units 1) scales leave headroom
// for rows_cap rows per row block; wide ones (2) quantise each row to 31 bits of max|g|
void ComputeScales(const uint32_t* absmax, int rows_cap, int hist_units, double* scales, hipStream_t s);
// the tree's device state reset; optionally zero `zero_bytes` at `zero` (8-byte words) and copy
// the tree's feature mask from fine-grained host memory into KArgs::tree_mask
void TreeBegin(const KArgs& a, hipStream_t s, void* zero = nullptr, size_t zero_bytes = 0,
               const int8_t* mask_host = nullptr, int nmask = 0);
void RootSum(const KArgs& a, hipStream_t s);
int RootSumBlocks();  // (KArgs::root_blk holds 2 doubles per block)
// histograms: per-row-block partials, then an exact int64 reduction into scratch buffer 0
void HistRoot(const KArgs& a, hipStream_t s);
void HistRange(const KArgs& a, hipStream_t s);  // rows idx[range_begin, +num_rows)
// one split step: (k_split) the split picked into Step::cs is applied to the parent's rows
// and one child's rows are histogrammed into row-block partials; (reduce=true) the partials
// are summed into the step's scratch buffer unless the split scan sums them itself
void SplitStep(const KArgs& a, hipStream_t s, bool reduce);
// host-assisted growth: apply the split the host wrote into Step::cs (no histogram)
void Partition(const KArgs& a, hipStream_t s);
// split scans of the root / the two children of the step (per-feature results); with
// KArgs::pick_in_find the last workgroup also records the step and picks the next split
void FindRoot(const KArgs& a, hipStream_t s);
// CEGB lazy penalties (KArgs::cegb_lazy): the root's unpaid counts (cegb_cnt row 0 and both
// scratch rows pre-zeroed by the caller); per step after the partition, the split feature paid
// on the split leaf's rows and the histogrammed child's unpaid counts
void CegbRoot(const KArgs& a, hipStream_t s);
// LDS of the picking workgroup's intermediate-monotone tree walk (pick.h MonoInterUpdate); the
// device path takes num_leaves <= kMonoInterMaxLeaves
constexpr int kMonoInterMaxLeaves = 512;
inline size_t MonoInterLds(int num_leaves) {
  return static_cast<size_t>(num_leaves + 1) * (20 * sizeof(int32_t) + 2 * sizeof(double));
}
void CegbStep(const KArgs& a, hipStream_t s);
// interaction constraints + feature_fraction_bynode: the step's two node masks (bynode_kernels.hip)
void ByNodeStep(const KArgs& a, hipStream_t s);
void FindStep(const KArgs& a, hipStream_t s);
// the step's bookkeeping and the next pick as a kernel of its own (distributed learners:
// it runs after the per-feature results were gathered from every rank)
void PickStep(const KArgs& a, hipStream_t s, bool root);
// round growth (KArgs::rd): the root's pick and first plan (after FindRoot without a pick),
// then per round the fused partition + histogram of every expansion, the reduction of their
// large histograms, the children's split scans (+ each child's best split), and the plan
// (replay of the best-first order, next expansions).  A finished tree's kernels exit at once.
void RoundRootPlan(const KArgs& a, hipStream_t s);
void RoundStep(const KArgs& a, hipStream_t s);  // single process: split + reduce + scans (+ plan)
// distributed rounds: the collectives go between the parts
void RoundSplitReduce(const KArgs& a, hipStream_t s);
void RoundFind(const KArgs& a, hipStream_t s);
void RoundChildBestAndPlan(const KArgs& a, hipStream_t s);
// voting-parallel rounds: the proposals of every child of the round from the phase-1 scan, and
// after their allgather the elections and the elected features' local histograms; then the
// phase-2 (global) scan of the elected features
void RoundVoteLocal(const KArgs& a, hipStream_t s);
void RoundVoteElect(const KArgs& a, hipStream_t s);
void RoundFindElected(const KArgs& a, hipStream_t s);
size_t RoundPlanLds(int num_leaves, int nodes);
// voting-parallel: this rank's top-k proposals per leaf from the local scan (into its block
// of vote_buf); after the allgather, the election and the elected features' local histograms
// (into vote_hist, for the all-reduce); the global scan is FindRoot / FindStep with
// Params::vote_phase = 2
void VoteLocal(const KArgs& a, hipStream_t s, bool root);
void VoteElect(const KArgs& a, hipStream_t s, bool root);

// score[k] += value[leaf(row)] for every partitioned row of the finished tree
void AddLeafScore(const KArgs& a, const double* leaf_values, int num_leaves, double* score, hipStream_t s);

// generic tree traversal over binned rows (out-of-bag rows, DART drops, refits)
struct DevTree {
  int32_t num_leaves{};
  const int32_t* split_feature_inner{};
  const uint32_t* threshold_in_bin{};
  const int8_t* decision_type{};
  const int32_t* left_child{};
  const int32_t* right_child{};
  const double* leaf_value{};
  const int32_t* cat_boundaries_inner{};
  const uint32_t* cat_threshold_inner{};
  unsigned long long* bm_work{};  // [num_leaves - 1][4] decision bitmaps over 8-bit group bins (workspace)
  int32_t* bm_meta{};             // [num_leaves - 1] packed (group, left, right) (workspace)
  int32_t bm_ready{};             // bm_work / bm_meta already hold this tree's bitmaps (TreeFromRecords)
};
void AddTreeScore(const KArgs& a, const DevTree& t, const int32_t* rows, int64_t num_rows, double* score,
                  hipStream_t s);
// The tree of the first nsplit split records (KArgs::rec) in the DevTree layout, leaf values
// times `shrinkage`, exactly as Tree::Split / SplitCategorical and Tree::Shrinkage build them on
// the host (categorical sets kMaxCatWords words each): the training scores can take the tree
// while the host builds its own.  `blob` holds TreeFromRecordsBytes(max_leaves) bytes; the
// returned DevTree points into it (bm_work / bm_meta left null).
size_t TreeFromRecordsBytes(int max_leaves);
constexpr int kHostOutHeaderWords = 16;  // KArgs::host_out: the scalars' words before the records
// With bm_work / bm_meta (and TreeBitmapsApply) the same launch builds the score walk's bitmaps
// (DevTree::bm_ready): one launch instead of two on the tree's critical path.
DevTree TreeFromRecords(const KArgs& a, int nsplit, int max_leaves, double shrinkage, char* blob, hipStream_t s,
                        unsigned long long* bm_work = nullptr, int32_t* bm_meta = nullptr);
// whether AddTreeScore walks every row with the bitmap kernel (8-bit word rows of <= 64 bytes,
// <= 255 internal nodes); otherwise a partition-ordered scatter of leaf values is cheaper
bool TreeBitmapsApply(const KArgs& a, int num_leaves);

void Iota(int32_t* p, int64_t n, hipStream_t s);

// element-wise reduction over the buffers of up to kMaxPeerBufs ranks sharing the device
// (the in-process device communicator): out[i] = op(src_0[off + i], ..., src_{n-1}[off + i])
constexpr int kMaxPeerBufs = 16;
struct PeerBufs {
  const void* p[kMaxPeerBufs]{};
};
enum PeerOp { kPeerSumF64 = 0, kPeerSumF32 = 1, kPeerSumI64 = 2, kPeerMaxU32 = 3 };
void ReducePeers(const PeerBufs& src, int n, size_t offset, void* out, size_t count, int op, hipStream_t s);

// One-shot peer collectives over symmetric windows (src/device/peer_kernels.hip, used by
// src/network/peer_comm.cpp).  Every rank owns one window, mapped into every peer (the same
// device for thread ranks, hipIpc handles over xGMI across processes):
//   [kPeerFlagBytes: u64 flags[2][kMaxPeerBufs] -- arrival / departure epochs written by each
//    peer] [stage: this rank's input of the collective in progress]
// A collective is ONE kernel: wait until the peers left the previous collective's stage, copy
// the input into the own stage, publish an arrival epoch to every peer, wait for every peer's
// arrival, read the peers' stages directly (reduce / gather), publish a departure epoch.  No
// host rendezvous: the kernels are captured into the learner's graphs.  Every wait is bounded
// (timeout -> status code, the host raises); a collective whose guard flag is set is skipped on
// every rank (the guard is replicated state, e.g. Round::done).
constexpr size_t kPeerFlagBytes = 4096;
enum PeerKind { kPeerAllreduce = 0, kPeerReduceScatter = 1, kPeerAllgather = 2, kPeerBroadcast = 3 };
// status words (host-mapped): [0] error code, [1] abort request from the host, [2] epoch of the error
enum PeerStatus { kPeerOk = 0, kPeerTimeout = 1, kPeerInjected = 2, kPeerAborted = 3 };
struct PeerArgs {
  char* win[kMaxPeerBufs]{};  // every rank's window (self included)
  int32_t n{}, rank{}, kind{}, op{}, root{};
  int32_t elem{};             // element bytes (reductions) or 4 / 1 (gathers, broadcast)
  long long fail_epoch{};     // fault injection: this rank stops at that collective (0: never)
  const char* send{};
  char* recv{};
  size_t count{};             // elements of this chunk (reduce-scatter: per block)
  size_t stride{};            // reduce-scatter: elements between send blocks; allgather: elements per rank
  size_t off{};               // chunk offset in elements
  unsigned long long* ctl{};  // local device words: [0] epoch, [1] copy arrivals, [2] read departures, [3] error
  unsigned int* status{};     // host-mapped PeerStatus words
  const int32_t* guard{};     // optional: nonzero -> skipped
  long long timeout_ticks{};  // 100 MHz wall-clock ticks
};
void PeerCollective(const PeerArgs& a, hipStream_t s);

// score scaling helpers
void AddConst(double* score, int64_t n, double v, hipStream_t s);
void MulConst(double* score, int64_t n, double v, hipStream_t s);

// point-wise objective gradients: kind = DeviceGradKind
struct GradArgs {
  int32_t kind{};
  int32_t num_class{};
  int64_t num_data{};
  double p0{}, p1{}, p2{};
  double lw0{}, lw1{};
  const float* label{};
  const float* weights{};      // may be null
  const float* label_weight{};  // MAPE per-row factor, may be null
  const double* score{};       // [num_class][num_data]
  float* grad{};
  float* hess{};
  int32_t write_split{};       // also write grad / hess (else only gh: UnpackGH materialises them on demand)
  GH* gh{};                    // optional fused packing (one model per iteration; rows gh_stride apart):
  int64_t gh_stride{};
  float* max_parts{};          //   interleaved (g, h), per-workgroup max|g| / max h and
  double* root_parts{};        //   (sum g, sum h), [GradientBlocks][2] each
};
void Gradients(const GradArgs& g, hipStream_t s);
// the bitmap score walk (TreeBitmapsApply, every row) that also writes the next iteration's
// (g, h) into ga.gh and the ga.max_parts / ga.root_parts partials of AddTreeScoreGradParts
// workgroups (point-wise objectives, one model per iteration)
void AddTreeScoreGrad(const KArgs& a, const DevTree& t, int64_t num_rows, double* score, const GradArgs& ga,
                      hipStream_t s);
int AddTreeScoreGradParts(int64_t num_rows);
bool AddTreeScoreGradKind(int kind);  // objectives AddTreeScoreGrad supports
// grad / hess from the interleaved (g, h) (rows gh_stride apart)
void UnpackGH(const GH* gh, int64_t gh_stride, int64_t n, float* grad, float* hess, hipStream_t s);
// listwise ranking gradients (LambdaRank-NDCG / XE-NDCG), one workgroup per query
constexpr int kRankKindLambdarank = 15;
constexpr int kRankKindXendcg = 16;
constexpr int kRankMaxDocs = 2048;       // documents of one query staged in LDS
constexpr int kRankSigmoidBins = 1024 * 1024;  // the reference's sigmoid table size
struct RankArgs {
  int32_t kind{};
  int32_t num_queries{};
  const int32_t* qb{};          // [num_queries + 1] query boundaries
  const float* label{};
  const float* weights{};       // per-row weights, may be null
  const double* score{};
  float* grad{};
  float* hess{};
  const double* inv_max_dcg{};  // [num_queries] 1 / max DCG@truncation (lambdarank)
  const double* label_gain{};   // label -> gain
  const double* discount{};     // position -> 1 / log2(2 + i)
  double sigmoid{};
  double sig_min{}, sig_max{}, sig_factor{};  // sigmoid table domain and bins per unit
  const double* sig_table{};    // [kRankSigmoidBins] the host objective's sigmoid table (lambdarank)
  int32_t norm{};               // lambdarank_norm
  uint32_t* rng{};              // [num_queries] LCG states (xendcg), advanced in place
  // queries of more than kRankMaxDocs documents (one 1024-thread workgroup each over a global
  // scratch of their rows instead of LDS): their indices and [num_data] scratch arrays
  const int32_t* big_q{};
  int32_t num_big{};
  double *big_d0{}, *big_d1{}, *big_dh{};
  float* big_f{};
  int32_t *big_i0{}, *big_i1{}, *big_i2{};
  // queries of at most kRankMaxDocs documents: the most documents of one (the LDS staging is
  // sized to it), and lambdarank's pair scratch -- query q's (high sorted position, low
  // document) float pairs at pair_off[q] -- so that each pair is evaluated once (null: twice)
  int32_t max_docs{};
  float2* pair_buf{};
  const int64_t* pair_off{};
};
void RankGradients(const RankArgs& ra, hipStream_t s);
size_t RankLdsBytes(int max_docs);  // k_lambdarank's dynamic LDS for queries of up to max_docs documents

// row sampling (bagging / GOSS) with the reference's per-1024-row generators: in-bag rows
// (ascending) then out-of-bag rows, and the in-bag count, written on the device
constexpr int kSampleBlockRows = 1024;
struct SampleArgs {
  int64_t num_data{};
  int64_t num_blocks{};      // SampleBlocks(num_data)
  int32_t goss{};            // 0 bagging, 1 GOSS
  int32_t balanced{};        // bagging with pos/neg fractions (label > 0 is positive)
  int32_t num_class{};       // GOSS: models per iteration (row weight = sum over them of |g * h|)
  double fraction{}, pos_fraction{}, neg_fraction{};
  double top_rate{}, other_rate{};
  const float* label{};      // balanced bagging
  float* grad{};             // GOSS: [num_class][num_data]; sampled small-gradient rows are rescaled
  float* hess{};
  uint32_t* rng{};           // [num_blocks] generator states, advanced in place
  uint8_t* codes{};          // [num_data] scratch
  int32_t* block_cnt{};      // [num_blocks] scratch
  int32_t* block_off{};      // [num_blocks] scratch
  int32_t* bag{};            // [num_data] out: in-bag rows
  int32_t* oob{};            // [num_data] out: out-of-bag rows
  int32_t* bag_count{};      // out: number of in-bag rows
};
int SampleBlocks(int64_t n);
void SampleRows(const SampleArgs& s, hipStream_t st);

// batch prediction of a flattened forest on raw feature values (row per thread)
constexpr int kMaxPredClasses = 16;
struct ForestArgs {
  int32_t num_trees{};
  int32_t num_class{};        // trees per iteration (<= kMaxPredClasses)
  int32_t num_cols{};
  int32_t is_double{};        // data: float64 (else float32)
  int32_t row_major{};
  int64_t num_rows{};
  const void* data{};
  const int32_t* node_off{};  // [num_trees + 1] first internal node of each tree
  const int32_t* leaf_off{};  // [num_trees] first leaf value of each tree
  const int32_t* feature{};   // [nodes] real feature index
  const double* threshold{};  // [nodes] (categorical: index into the tree's cat boundaries)
  const int8_t* dtype{};      // [nodes] decision type
  const int32_t* left{};      // [nodes] children, leaves as ~leaf
  const int32_t* right{};
  const double* leaf_value{};
  const int32_t* cat_bound_off{};  // [num_trees] offset of the tree's cat_boundaries
  const int32_t* cat_bound{};
  const int32_t* cat_bits_off{};   // [num_trees] offset of the tree's cat_threshold words
  const uint32_t* cat_bits{};
  double* out{};              // [num_rows][num_class] raw scores
};
void PredictForest(const ForestArgs& f, hipStream_t s);

// validation metrics on device scores (one model per iteration)
constexpr int kMetricL2 = 1, kMetricRMSE = 2, kMetricL1 = 3, kMetricBinLogloss = 4, kMetricBinError = 5,
              kMetricAUC = 6, kMetricQuantile = 7, kMetricHuber = 8, kMetricFair = 9, kMetricPoisson = 10,
              kMetricMape = 11, kMetricGamma = 12, kMetricGammaDeviance = 13, kMetricTweedie = 14, kMetricXent = 15,
              kMetricMultiLogloss = 20, kMetricMultiError = 21, kMetricAucMu = 22, kMetricNDCG = 30,
              kMetricMAP = 31;
struct MetricArgs {
  int32_t kind{};
  int32_t convert{};       // score -> prediction: 0 identity, 1 sigmoid(sigmoid * s), 2 sign(s) * s^2, 3 exp,
                         // 4 softmax over the classes, 5 sigmoid per class
  double sigmoid{};
  double param{};          // alpha (quantile, huber), fair_c, tweedie_variance_power
  int64_t n{};
  const double* score{};   // [num_class][n]
  const float* label{};
  const float* weights{};  // may be null
  int32_t num_class{}, top_k{};
  // query metrics: per query [nk] values, summed over queries in fixed order
  int32_t nq{}, nk{};
  const int32_t* qb{};       // [nq + 1]
  const float* qw{};         // [nq] or null
  const int32_t* eval_at{};  // [nk]
  const double* qconst{};    // NDCG: [nq][nk] 1 / max DCG (<= 0: no relevant document); MAP: [nq] relevant documents;
                           // AUC-mu: [num_class][num_class] auc_mu_weights
  const double* label_gain{};
  const double* discount{};  // [kRankMaxDocs]
  int32_t big{};           // a query has more than kRankMaxDocs documents (scratch then holds n rows)
  void* scratch{};         // MetricScratchBytes(n, nq * nk) (query metrics: n = 0 unless big)
  double* out{};           // [0] weighted loss sum (or AUC accumulator), [1] AUC positive weight; query: [nk];
                         // AUC-mu: per class pair (i < j) accumulator and class-j count
};
size_t MetricScratchBytes(int64_t n, int64_t query_values = 0);
void EvalMetric(const MetricArgs& m, hipStream_t s);

// percentile leaf-output renewal (L1 / quantile / MAPE): per leaf of the finished tree, the
// alpha-percentile of its rows' residuals label - score (weighted if weights != null)
struct RenewArgs {
  const Leaf* leaves{};
  const int32_t* idx{};
  const int32_t* tmp{};
  int64_t buf_stride{};  // KArgs::buf_stride
  const float* label{};
  const double* score{};
  const float* weights{};    // or null
  const int64_t* offsets{};  // [num_leaves + 1] first row of each leaf in the gathered order
  int32_t num_leaves{};
  double alpha{};
  double* keys{};  // (carved from scratch)
  double* vals{};
  double* out{};   // [num_leaves]
  void* scratch{};  // RenewScratchBytes
};
size_t RenewScratchBytes(int64_t n, int leaves);
void RenewLeafOutputs(RenewArgs r, int64_t n, hipStream_t s);

int GradientBlocks(int64_t n);
// absmax = (max |g|, max h, rows_cap, 0) (and root = (sum g, sum h, n) if root_parts) from
// per-workgroup partials
// (scales non-null: also the tree's fixed-point scales from the result, as ComputeScales -- one
// process, where no all-reduce of absmax comes between)
void ReduceParts(const float* max_parts, const double* root_parts, int nparts, int64_t n, int rows_cap,
                 uint32_t* absmax, double* root, hipStream_t s, int units = 0, double* scales = nullptr);

}  // namespace dev
}  // namespace lgbm_amd
