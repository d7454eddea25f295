// Every environment knob of the native library, and the tuned defaults behind them, in one
// table.  Training parameters live in Config (tools/param_spec.py); these variables are not
// parameters: none changes a model unless its row says so (docs/ENVIRONMENT.md has the same
// table with the A/B each default came from).  Values are read at each use, so tests may change
// them between trainings in one process.
#pragma once

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace lgbm_amd {
namespace tuning {

// ---- tuned defaults (profiles/ cites the A/B of each)
constexpr int kRoundWidth = 8;             // expansions per round (r04_round_width.md)
constexpr int kRoundWidthNarrow = 6;       // ... for trees whose last tree's speculation was not accepted
constexpr double kRoundAdaptRows = 4e6;    // rows per rank from which the width adapts per tree
constexpr int kRoundLeavesPerWidth = 10;    // wide trees: the width is num_leaves / 10, 8 to 16 (r06_round_width_255.md)
constexpr double kRoundAutoRows = 16e6;    // rows per rank from which round growth is timed against one split per step
constexpr int kRoundHistory = 3;           // rounds enqueued per tree: the most of the last N trees
constexpr int kRoundSegment = 4;           // rounds per segment graph
constexpr int kRoundFirstTree = 16;        // rounds enqueued for the first tree
constexpr int kScoreWalkWgPerCu = 32;      // score walk workgroups per CU (r02_v9)
constexpr int kRootWgPerCu = 2;            // root histogram workgroups per CU (r04_final_remeasure.md)
constexpr int kPeerStageMbThreads = 16;    // peer comm stage, thread ranks (MiB)
constexpr int kPeerStageMbProcesses = 64;  // peer comm stage, one process per GPU (MiB)
// lambdarank pair scratch (cnt^2 float pairs per LDS-staged query, each pair evaluated once):
// at most this share of the free device memory when the tables are uploaded, and at most
// kRankPairCapMb; above it the kernel evaluates each pair from both ends (same gradients)
constexpr double kRankPairFreeShare = 0.125;
constexpr int kRankPairCapMb = 6144;
// NDCG / MAP on the device rank each document against every other of its query (one workgroup
// per query): validation sets with a longer query are evaluated on the host
constexpr int kQueryMetricDeviceMaxDocs = 16384;

// ---- the variables: X(id, name, what it does)
#define LGBM_AMD_KNOBS(X)                                                                                        \
  /* observability (no effect on results) */                                                                   \
  X(IterLog, "LGBM_AMD_ITER_LOG", "path: one JSON line per iteration (phase times, rounds, graph use, bytes)")  \
  X(Ktrace, "LGBM_AMD_KTRACE", "1: in-kernel wall-clock phase stamps of each round / split")                    \
  X(KtraceRepeat, "LGBM_AMD_KTRACE_REPEAT", "1: the traced pick runs twice (warm timing)")                     \
  X(KernelProbe, "LGBM_AMD_KERNEL_PROBE", "1: time back-to-back launches of every step kernel after a tree")     \
  X(Timetag, "LGBM_AMD_TIMETAG", "1: host phase timers (common::PhaseTimer)")                                  \
  X(Roctx, "LGBM_AMD_ROCTX", "1: roctx ranges around the host phases")                                         \
  X(PoisonArgs, "LGBM_AMD_POISON_ARGS", "1: argument structs filled with 0xA5 before their call sites set them")  \
  /* reference paths: parity tests and A/Bs */                                                                 \
  X(HostAssist, "LGBM_AMD_HOST_ASSIST", "1: host-assisted growth over device histograms")                      \
  X(DistHostAssist, "LGBM_AMD_DIST_HOST_ASSIST", "1: host-assisted per-node sampling / CEGB when distributed")  \
  X(HostBagging, "LGBM_AMD_HOST_BAGGING", "1: bagging / GOSS drawn on the host")                               \
  X(HostMetrics, "LGBM_AMD_HOST_METRICS", "1: metrics evaluated on the host")                                  \
  X(HostRenew, "LGBM_AMD_HOST_RENEW", "1: percentile leaf renewal on the host")                                \
  X(HostPredict, "LGBM_AMD_HOST_PREDICT", "1: C API prediction on the host")                                   \
  X(HostSparse, "LGBM_AMD_HOST_SPARSE", "0/1: dense / sparse host storage of every group")                     \
  X(DeviceBinning, "LGBM_AMD_DEVICE_BINNING", "0/1: value-to-bin on the host / the GPU")                       \
  X(NoGraph, "LGBM_AMD_NO_GRAPH", "1: kernels launched eagerly instead of from hipGraphs")                     \
  X(GraphCollectives, "LGBM_AMD_GRAPH_COLLECTIVES", "0: distributed split steps launched eagerly")             \
  X(StaticOwners, "LGBM_AMD_STATIC_OWNERS", "1: data-parallel keeps static feature owners")                    \
  X(RoundFused, "LGBM_AMD_ROUND_FUSED", "0: separate partition and histogram kernels per round")               \
  X(PlanInFind, "LGBM_AMD_PLAN_IN_FIND", "0: the round's plan in a kernel of its own")                         \
  X(FuseGrad, "LGBM_AMD_FUSE_GRAD", "0: the score walk does not compute the next gradients")                   \
  X(EarlyScore, "LGBM_AMD_EARLY_SCORE", "0: the training scores take the tree after the host has built it")     \
  X(GraphCopyNodes, "LGBM_AMD_GRAPH_COPY_NODES", "1: the tree's scratch zeroing / mask upload as memset / memcpy nodes")  \
  X(ByNodeRounds, "LGBM_AMD_BYNODE_ROUNDS", "0: per-node feature sampling grows one split per step instead of rounds")  \
  X(XtRounds, "LGBM_AMD_XT_ROUNDS", "0: extra_trees grows one split per step instead of rounds")                \
  X(CegbRounds, "LGBM_AMD_CEGB_ROUNDS", "0: CEGB coupled penalties refunded on one split per step until every feature is used")  \
  X(HostOut, "LGBM_AMD_HOST_OUT", "0: the host copies a round tree's records instead of its last plan writing them")  \
  X(Speculate, "LGBM_AMD_SPECULATE", "1: the next tree is launched when this one ends, before GBDT asks for it")  \
  /* storage layout (same models) */                                                                           \
  X(NibbleBins, "LGBM_AMD_NIBBLE_BINS", "1: 4-bit rows for groups of <= 16 bins (auto above 32 GiB)")          \
  X(ColumnCopy, "LGBM_AMD_COLUMN_COPY", "0/1: column-major copy of the bins (auto below 8 GiB)")                \
  X(SparseRows, "LGBM_AMD_SPARSE_ROWS", "0/1: row-sparse device storage (auto by density)")                    \
  X(UniformBins, "LGBM_AMD_UNIFORM_BINS", "1: every group at the widest group's width")                        \
  X(GhInRows, "LGBM_AMD_GH_IN_ROWS", "0/1: (g, h) beside the bins in each row or apart")                       \
  X(RowAlignWords, "LGBM_AMD_ROW_ALIGN_WORDS", "n: row stride rounded up to n words")                          \
  X(HistTileWords, "LGBM_AMD_HIST_TILE_WORDS", "n: histogram column tile width (words)")                       \
  X(HistRowsCap, "LGBM_AMD_HIST_ROWS_CAP", "n: rows per partial histogram block")                              \
  X(TextBlockBytes, "LGBM_AMD_TEXT_BLOCK_BYTES", "n: text reader block size (tests)")                          \
  /* tuning (same models; defaults above) */                                                                   \
  X(RoundK, "LGBM_AMD_ROUND_K", "n: expansions per round, fixed (1: one split per step)")                      \
  X(RoundVmax, "LGBM_AMD_ROUND_VMAX", "n: speculation depth below a leaf (14)")                                \
  X(RoundAuto, "LGBM_AMD_ROUND_AUTO", "0/1: never / always time round growth against one split per step")      \
  X(RoundHist, "LGBM_AMD_ROUND_HIST", "n: rounds enqueued = the most of the last n trees")                     \
  X(RoundMargin, "LGBM_AMD_ROUND_MARGIN", "n: extra rounds enqueued per tree")                                 \
  X(RoundSeg, "LGBM_AMD_ROUND_SEG", "n: rounds per segment graph")                                             \
  X(RoundRoot, "LGBM_AMD_ROUND_ROOT", "n: rounds in the root graph (0: the enqueued count)")                   \
  X(RoundGrid, "LGBM_AMD_ROUND_GRID", "n: round split workgroups")                                             \
  X(RoundGr, "LGBM_AMD_ROUND_GR", "n: rows gathered per pass in the round split kernel")                      \
  X(RoundNeedDiv, "LGBM_AMD_ROUND_NEED_DIV", "n: picks per round capped by remaining splits / n")              \
  X(RoundPredict, "LGBM_AMD_ROUND_PREDICT", "0/1: next round's picks by the step walk / bottleneck keys")     \
  X(SplitGrid, "LGBM_AMD_SPLIT_GRID", "n: one-split-per-step split workgroups")                                \
  X(BlkMinRows, "LGBM_AMD_BLK_MIN_ROWS", "n: smallest row block")                                              \
  X(DirectFromSplit, "LGBM_AMD_DIRECT_FROM_SPLIT", "n: split steps whose partials the split scan sums itself")  \
  X(BmWgPerCu, "LGBM_AMD_BM_WG_PER_CU", "n: score walk workgroups per CU")                                     \
  X(RootWgPerCu, "LGBM_AMD_ROOT_WG_PER_CU", "n: root histogram workgroups per CU")                             \
  X(RankPairMb, "LGBM_AMD_RANK_PAIR_MB", "n: lambdarank pair scratch budget (MiB; 0: no scratch)")            \
  /* distributed */                                                                                            \
  X(PeerStageMb, "LGBM_AMD_PEER_STAGE_MB", "n: peer comm stage size (MiB)")                                    \
  X(Network, "LGBM_AMD_NETWORK", "host network transport (tcp / mpi)")                                         \
  X(MpiLib, "LGBM_AMD_MPI_LIB", "path of the MPI library to load")

enum class Knob : int {
#define LGBM_AMD_KNOB_ID(id, name, doc) id,
  LGBM_AMD_KNOBS(LGBM_AMD_KNOB_ID)
#undef LGBM_AMD_KNOB_ID
      kCount
};

inline const char* Name(Knob k) {
  static const char* const names[] = {
#define LGBM_AMD_KNOB_NAME(id, name, doc) name,
      LGBM_AMD_KNOBS(LGBM_AMD_KNOB_NAME)
#undef LGBM_AMD_KNOB_NAME
  };
  return names[static_cast<int>(k)];
}

// the variable's value (nullptr: unset)
inline const char* Get(Knob k) { return std::getenv(Name(k)); }
// set to a value starting with '1' / '0'
inline bool On(Knob k) {
  const char* e = Get(k);
  return e != nullptr && e[0] == '1';
}
inline bool Off(Knob k) {
  const char* e = Get(k);
  return e != nullptr && e[0] == '0';
}
// the integer value, or dflt when unset
inline int Int(Knob k, int dflt) {
  const char* e = Get(k);
  return e != nullptr ? std::atoi(e) : dflt;
}

// LGBM_AMD_POISON_ARGS=1 (tests): a device argument struct whose call site sets every field the
// kernel reads is filled with 0xA5 bytes first, so a forgotten field reads garbage on every run
// instead of whatever the stack held (round 5: an unset GradArgs::write_split passed on one box
// and zeroed the gradients on another)
template <typename T>
inline void PoisonArgs(T* a) {
  static_assert(std::is_trivially_copyable<T>::value, "plain argument struct");
  if (On(Knob::PoisonArgs)) std::memset(static_cast<void*>(a), 0xA5, sizeof(T));
}

}  // namespace tuning
}  // namespace lgbm_amd
