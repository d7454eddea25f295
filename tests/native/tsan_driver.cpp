// ThreadSanitizer driver (`make tsan`): the library's own threads and its
// locking under concurrent C API use, with OpenMP at one thread (libgomp is not
// instrumented, so its barriers would read as races).
//   1. two_round loading: the pipelined block reader thread hands blocks to the parser;
//   2. a trainer thread adds iterations (exclusive booster lock) while three threads predict
//      dense rows (shared lock) and one reads evaluation results;
//   3. two boosters with row-wise CPU histograms train at once on the same Dataset (its
//      row-major copy is built once under the Dataset's lock; each learner owns its scratch).
// usage: tsan_driver <train file> <num features>; exit status 0 = no failed call (TSan reports
// go to stderr and make the process exit non-zero through TSAN_OPTIONS=exitcode).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "lgbm_amd/c_api.h"

#define CHECK_CALL(x)                                                                 \
  do {                                                                                \
    if ((x) != 0) {                                                                   \
      std::fprintf(stderr, "call failed: %s: %s\n", #x, LGBM_GetLastError());         \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int nfeat = std::atoi(argv[2]);
  DatasetHandle ds = nullptr;
  CHECK_CALL(LGBM_DatasetCreateFromFile(argv[1], "two_round=true num_threads=1 max_bin=63 verbose=-1", nullptr, &ds));
  BoosterHandle bst = nullptr;
  CHECK_CALL(LGBM_BoosterCreate(ds, "objective=binary num_leaves=15 num_threads=1 metric=auc verbose=-1", &bst));
  int fin = 0;
  for (int i = 0; i < 3; ++i) CHECK_CALL(LGBM_BoosterUpdateOneIter(bst, &fin));
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  ts.emplace_back([&] {
    int f = 0;
    for (int i = 0; i < 12; ++i) CHECK_CALL(LGBM_BoosterUpdateOneIter(bst, &f));
    stop = true;
  });
  for (int t = 0; t < 3; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937 rng(t);
      std::normal_distribution<double> nd;
      std::vector<double> x(200 * static_cast<size_t>(nfeat));
      std::vector<double> out(200);
      do {
        for (auto& v : x) v = nd(rng);
        int64_t len = 0;
        CHECK_CALL(LGBM_BoosterPredictForMat(bst, x.data(), C_API_DTYPE_FLOAT64, 200, nfeat, 1, C_API_PREDICT_NORMAL,
                                             0, -1, "num_threads=1", &len, out.data()));
      } while (!stop);
    });
  }
  ts.emplace_back([&] {
    do {
      int it = 0, n = 0;
      CHECK_CALL(LGBM_BoosterGetCurrentIteration(bst, &it));
      CHECK_CALL(LGBM_BoosterGetEvalCounts(bst, &n));
      std::vector<double> r(n + 1);
      CHECK_CALL(LGBM_BoosterGetEval(bst, 0, &n, r.data()));
    } while (!stop);
  });
  for (auto& t : ts) t.join();
  int it = 0;
  CHECK_CALL(LGBM_BoosterGetCurrentIteration(bst, &it));
  CHECK_CALL(LGBM_BoosterFree(bst));
  // 3. two row-wise boosters on one Dataset, trained concurrently
  BoosterHandle rw[2] = {nullptr, nullptr};
  for (auto& b : rw) {
    CHECK_CALL(LGBM_BoosterCreate(ds, "objective=binary num_leaves=15 num_threads=1 force_row_wise=true verbose=-1", &b));
  }
  std::vector<std::thread> rt;
  for (auto& b : rw) {
    rt.emplace_back([&b] {
      int f = 0;
      for (int i = 0; i < 5; ++i) CHECK_CALL(LGBM_BoosterUpdateOneIter(b, &f));
    });
  }
  for (auto& t : rt) t.join();
  int it2[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    CHECK_CALL(LGBM_BoosterGetCurrentIteration(rw[k], &it2[k]));
    CHECK_CALL(LGBM_BoosterFree(rw[k]));
  }
  CHECK_CALL(LGBM_DatasetFree(ds));
  std::printf("tsan driver ok: %d iterations, row-wise boosters %d / %d\n", it, it2[0], it2[1]);
  return (it == 15 && it2[0] == 5 && it2[1] == 5) ? 0 : 3;
}
