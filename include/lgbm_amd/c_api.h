/* C API of lightgbmv1_amd.  Function names, argument lists, return codes and constants are
 * those of the reference C API (reference include/LightGBM/c_api.h:27-1290) so existing
 * bindings (Python ctypes, R, JNI) can target this library unchanged.  Extensions for the
 * MI355X runtime are prefixed LGBM_AMD_. */
#ifndef LGBM_AMD_C_API_H_
#define LGBM_AMD_C_API_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define LGBM_EXTERN_C extern "C"
#else
#define LGBM_EXTERN_C
#endif
#define LIGHTGBM_C_EXPORT LGBM_EXTERN_C __attribute__((visibility("default")))

typedef void* DatasetHandle;
typedef void* BoosterHandle;
typedef void* FastConfigHandle;

#define C_API_DTYPE_FLOAT32 (0)
#define C_API_DTYPE_FLOAT64 (1)
#define C_API_DTYPE_INT32 (2)
#define C_API_DTYPE_INT64 (3)

#define C_API_PREDICT_NORMAL (0)
#define C_API_PREDICT_RAW_SCORE (1)
#define C_API_PREDICT_LEAF_INDEX (2)
#define C_API_PREDICT_CONTRIB (3)

#define C_API_MATRIX_TYPE_CSR (0)
#define C_API_MATRIX_TYPE_CSC (1)

#define C_API_FEATURE_IMPORTANCE_SPLIT (0)
#define C_API_FEATURE_IMPORTANCE_GAIN (1)

LIGHTGBM_C_EXPORT const char* LGBM_GetLastError();
LIGHTGBM_C_EXPORT int LGBM_RegisterLogCallback(void (*callback)(const char*));

LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromFile(const char* filename, const char* parameters,
                                                 const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromSampledColumn(double** sample_data, int** sample_indices, int32_t ncol,
                                                          const int* num_per_col, int32_t num_sample_row,
                                                          int32_t num_total_row, const char* parameters,
                                                          DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateByReference(const DatasetHandle reference, int64_t num_total_row,
                                                    DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRows(DatasetHandle dataset, const void* data, int data_type, int32_t nrow,
                                           int32_t ncol, int32_t start_row);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRowsByCSR(DatasetHandle dataset, const void* indptr, int indptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t nindptr, int64_t nelem, int64_t num_col, int64_t start_row);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSR(const void* indptr, int indptr_type, const int32_t* indices,
                                                const void* data, int data_type, int64_t nindptr, int64_t nelem,
                                                int64_t num_col, const char* parameters, const DatasetHandle reference,
                                                DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSRFunc(void* get_row_funptr, int num_rows, int64_t num_col,
                                                    const char* parameters, const DatasetHandle reference,
                                                    DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSC(const void* col_ptr, int col_ptr_type, const int32_t* indices,
                                                const void* data, int data_type, int64_t ncol_ptr, int64_t nelem,
                                                int64_t num_row, const char* parameters, const DatasetHandle reference,
                                                DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromMat(const void* data, int data_type, int32_t nrow, int32_t ncol,
                                                int is_row_major, const char* parameters,
                                                const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromMats(int32_t nmat, const void** data, int data_type, int32_t* nrow,
                                                 int32_t ncol, int is_row_major, const char* parameters,
                                                 const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetSubset(const DatasetHandle handle, const int32_t* used_row_indices,
                                            int32_t num_used_row_indices, const char* parameters, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetFeatureNames(DatasetHandle handle, const char** feature_names,
                                                  int num_feature_names);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetFeatureNames(DatasetHandle handle, const int len, int* num_feature_names,
                                                  const size_t buffer_len, size_t* out_buffer_len,
                                                  char** feature_names);
LIGHTGBM_C_EXPORT int LGBM_DatasetFree(DatasetHandle handle);
LIGHTGBM_C_EXPORT int LGBM_DatasetSaveBinary(DatasetHandle handle, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_DatasetDumpText(DatasetHandle handle, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetField(DatasetHandle handle, const char* field_name, const void* field_data,
                                           int num_element, int type);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetField(DatasetHandle handle, const char* field_name, int* out_len,
                                           const void** out_ptr, int* out_type);
LIGHTGBM_C_EXPORT int LGBM_DatasetUpdateParamChecking(const char* old_parameters, const char* new_parameters);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetNumData(DatasetHandle handle, int* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetNumFeature(DatasetHandle handle, int* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetAddFeaturesFrom(DatasetHandle target, DatasetHandle source);

LIGHTGBM_C_EXPORT int LGBM_BoosterCreate(const DatasetHandle train_data, const char* parameters, BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterCreateFromModelfile(const char* filename, int* out_num_iterations,
                                                      BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterLoadModelFromString(const char* model_str, int* out_num_iterations,
                                                      BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterFree(BoosterHandle handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterShuffleModels(BoosterHandle handle, int start_iter, int end_iter);
LIGHTGBM_C_EXPORT int LGBM_BoosterMerge(BoosterHandle handle, BoosterHandle other_handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterAddValidData(BoosterHandle handle, const DatasetHandle valid_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterResetTrainingData(BoosterHandle handle, const DatasetHandle train_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterResetParameter(BoosterHandle handle, const char* parameters);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumClasses(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterUpdateOneIter(BoosterHandle handle, int* is_finished);
LIGHTGBM_C_EXPORT int LGBM_BoosterRefit(BoosterHandle handle, const int32_t* leaf_preds, int32_t nrow, int32_t ncol);
LIGHTGBM_C_EXPORT int LGBM_BoosterUpdateOneIterCustom(BoosterHandle handle, const float* grad, const float* hess,
                                                      int* is_finished);
LIGHTGBM_C_EXPORT int LGBM_BoosterRollbackOneIter(BoosterHandle handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetCurrentIteration(BoosterHandle handle, int* out_iteration);
LIGHTGBM_C_EXPORT int LGBM_BoosterNumModelPerIteration(BoosterHandle handle, int* out_tree_per_iteration);
LIGHTGBM_C_EXPORT int LGBM_BoosterNumberOfTotalModel(BoosterHandle handle, int* out_models);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEvalCounts(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEvalNames(BoosterHandle handle, const int len, int* out_len,
                                               const size_t buffer_len, size_t* out_buffer_len, char** out_strs);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetFeatureNames(BoosterHandle handle, const int len, int* out_len,
                                                  const size_t buffer_len, size_t* out_buffer_len, char** out_strs);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumFeature(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEval(BoosterHandle handle, int data_idx, int* out_len, double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumPredict(BoosterHandle handle, int data_idx, int64_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetPredict(BoosterHandle handle, int data_idx, int64_t* out_len,
                                             double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForFile(BoosterHandle handle, const char* data_filename,
                                                 int data_has_header, int predict_type, int start_iteration,
                                                 int num_iteration, const char* parameter,
                                                 const char* result_filename);
LIGHTGBM_C_EXPORT int LGBM_BoosterCalcNumPredict(BoosterHandle handle, int num_row, int predict_type,
                                                 int start_iteration, int num_iteration, int64_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_FastConfigFree(FastConfigHandle fastConfig);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSR(BoosterHandle handle, const void* indptr, int indptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t nindptr, int64_t nelem, int64_t num_col, int predict_type,
                                                int start_iteration, int num_iteration, const char* parameter,
                                                int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictSparseOutput(BoosterHandle handle, const void* indptr, int indptr_type,
                                                      const int32_t* indices, const void* data, int data_type,
                                                      int64_t nindptr, int64_t nelem, int64_t num_col_or_row,
                                                      int predict_type, int start_iteration, int num_iteration,
                                                      const char* parameter, int matrix_type, int64_t* out_len,
                                                      void** out_indptr, int32_t** out_indices, void** out_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterFreePredictSparse(void* indptr, int32_t* indices, void* data, int indptr_type,
                                                    int data_type);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRow(BoosterHandle handle, const void* indptr, int indptr_type,
                                                         const int32_t* indices, const void* data, int data_type,
                                                         int64_t nindptr, int64_t nelem, int64_t num_col,
                                                         int predict_type, int start_iteration, int num_iteration,
                                                         const char* parameter, int64_t* out_len,
                                                         double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                                                 const int start_iteration, const int num_iteration,
                                                                 const int data_type, const int64_t num_col,
                                                                 const char* parameter,
                                                                 FastConfigHandle* out_fastConfig);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRowFast(FastConfigHandle fastConfig_handle, const void* indptr,
                                                             const int indptr_type, const int32_t* indices,
                                                             const void* data, const int64_t nindptr,
                                                             const int64_t nelem, int64_t* out_len,
                                                             double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSC(BoosterHandle handle, const void* col_ptr, int col_ptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t ncol_ptr, int64_t nelem, int64_t num_row, int predict_type,
                                                int start_iteration, int num_iteration, const char* parameter,
                                                int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMat(BoosterHandle handle, const void* data, int data_type, int32_t nrow,
                                                int32_t ncol, int is_row_major, int predict_type,
                                                int start_iteration, int num_iteration, const char* parameter,
                                                int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRow(BoosterHandle handle, const void* data, int data_type,
                                                         int ncol, int is_row_major, int predict_type,
                                                         int start_iteration, int num_iteration,
                                                         const char* parameter, int64_t* out_len,
                                                         double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                                                 const int start_iteration, const int num_iteration,
                                                                 const int data_type, const int32_t ncol,
                                                                 const char* parameter,
                                                                 FastConfigHandle* out_fastConfig);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRowFast(FastConfigHandle fastConfig_handle, const void* data,
                                                             int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMats(BoosterHandle handle, const void** data, int data_type,
                                                 int32_t nrow, int32_t ncol, int predict_type, int start_iteration,
                                                 int num_iteration, const char* parameter, int64_t* out_len,
                                                 double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterSaveModel(BoosterHandle handle, int start_iteration, int num_iteration,
                                            int feature_importance_type, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_BoosterSaveModelToString(BoosterHandle handle, int start_iteration, int num_iteration,
                                                    int feature_importance_type, int64_t buffer_len,
                                                    int64_t* out_len, char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterDumpModel(BoosterHandle handle, int start_iteration, int num_iteration,
                                            int feature_importance_type, int64_t buffer_len, int64_t* out_len,
                                            char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double* out_val);
LIGHTGBM_C_EXPORT int LGBM_BoosterSetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double val);
LIGHTGBM_C_EXPORT int LGBM_BoosterFeatureImportance(BoosterHandle handle, int num_iteration, int importance_type,
                                                    double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetUpperBoundValue(BoosterHandle handle, double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLowerBoundValue(BoosterHandle handle, double* out_results);

LIGHTGBM_C_EXPORT int LGBM_NetworkInit(const char* machines, int local_listen_port, int listen_time_out,
                                       int num_machines);
LIGHTGBM_C_EXPORT int LGBM_NetworkFree();
LIGHTGBM_C_EXPORT int LGBM_NetworkInitWithFunctions(int num_machines, int rank, void* reduce_scatter_ext_fun,
                                                    void* allgather_ext_fun);

/* ---- MI355X extensions ---- */
/* size in bytes of the RCCL unique id blob exchanged by the launcher */
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclUniqueIdSize(int* out);
/* rank 0 creates the id; every rank then calls LGBM_AMD_RcclInit with the same blob */
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclGetUniqueId(char* out_id);
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclInit(int num_ranks, int rank, int device_id, const char* unique_id);
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclFree();
/* one process per GPU: capture-safe peer collectives over hipIpc-mapped windows (xGMI);
   needs the host Network (LGBM_NetworkInit*) for the handle exchange */
LIGHTGBM_C_EXPORT int LGBM_AMD_PeerCommInit(int device_id, double timeout_s);
/* releases the device comm (peer or RCCL) after every rank's kernels are done */
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommFree();
/* microseconds per device collective (kind 0 int64 reduce-scatter, 1 allgather, 2 int64
   all-reduce) over `iters` back-to-back calls, graph-captured or eager; every rank calls it */
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommBench(int kind, int64_t bytes, int iters, int graph, double* out_us);
/* runs every device collective on small buffers and checks the sums (1 = ok) */
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclSelfTest(int* out_ok);
// the same all-reduces captured into a hipGraph and replayed (the device learner's tree graph)
LIGHTGBM_C_EXPORT int LGBM_AMD_RcclGraphSelfTest(int* out_ok);
/* number of visible GPUs (0 without a device) */
/* in-process ranks for tests: a hub of thread transports (timeout_s > 0 bounds every
 * collective; fail_rank / fail_at_call inject a fault); each rank's thread then joins it
 * and trains as that rank (Network state is thread-local) */
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkCreateThreadHub(int num_ranks, double timeout_s, int fail_rank,
                                                      int fail_at_call, void** out);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkJoinThreadHub(void* hub, int rank);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkFreeThreadHub(void* hub);
// test support of the device learner (tests/test_gpu_kernels.py): group-bin matrix of a
// dataset (row-major num_data x num_groups; boundaries: first histogram bin of each group,
// num_groups + 1 entries); call with null buffers to get num_groups first
LIGHTGBM_C_EXPORT int LGBM_AMD_DatasetGetGroupBins(DatasetHandle handle, int32_t* bins, int64_t* boundaries,
                                                   int* num_groups);
// the state the last device-grown tree left in HBM: a leaf's rows (count first with rows ==
// null), its raw fixed-point histogram slot (2 * total_bins int64: g, h) and sums
// (sum_g, sum_h, count); the rows' packed (g, h) and the fixed-point scales
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterDeviceLeafState(BoosterHandle handle, int leaf, int32_t* rows, int* count,
                                                      int64_t* hist, int8_t* bin_valid, int64_t* hist_len,
                                                      double* sums);
/* the gradients the last iteration trained on (device or host learner); *n = entries */
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterLastGradients(BoosterHandle handle, float* grad, float* hess, int64_t* n);
// growth counters of the device learner summed over the trees trained so far: out[0] trees,
// [1] of them grown device-resident, [2] rounds, [3] expansions, [4] splits, [5] bytes moved by
// device collectives (no synchronisation: cheap inside a timed loop)
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterGrowthStats(BoosterHandle handle, double* out, int n);
// free / total bytes of the current HIP device (hipMemGetInfo)
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceMemInfo(int64_t* free_bytes, int64_t* total_bytes);
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterDeviceGradients(BoosterHandle handle, float* grad, float* hess,
                                                      double* scales);
// JSON report of the leaves' device best splits checked against the CPU split finder
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterDeviceCheckSplits(BoosterHandle handle, int64_t buffer_len, int64_t* out_len,
                                                        char* out_str);
// for external collective functions (LGBM_NetworkInitWithFunctions) that fail: makes the
// collective that called them raise on this thread instead of using an unfilled buffer
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkReportExternalError(const char* msg);
// raw host collectives of the calling thread's network (the mesh training uses): allgather of
// block_len[r] bytes from every rank r; reduce-scatter / all-reduce sums of doubles
// (block_count[r] items of the input go to rank r)
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkRank(int* out);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkNumMachines(int* out);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkAllgather(const void* input, const int64_t* block_len, void* output);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkReduceScatterSumF64(const double* input, const int64_t* block_count,
                                                          double* output);
LIGHTGBM_C_EXPORT int LGBM_AMD_NetworkAllreduceSumF64(const double* input, int64_t count, double* output);
// in-process device communicators (thread ranks sharing one GPU)
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommCreateThreadHub(int num_ranks, double timeout_s, int fail_rank, int fail_at_call,
                                                         void** out);
/* kind 0: host-rendezvous device comm (eager); 1: capture-safe one-shot peer comm */
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommCreateThreadHubEx(int num_ranks, double timeout_s, int fail_rank,
                                                           int fail_at_call, int kind, void** out);
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommJoinThreadHub(void* hub, int rank);
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCommFreeThreadHub(void* hub);
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceSynchronize();
LIGHTGBM_C_EXPORT int LGBM_AMD_DeviceCount(int* out);
/* phase timers (LGBM_AMD_TIMETAG) as "name=seconds;..." */
LIGHTGBM_C_EXPORT int LGBM_AMD_GetTimers(int64_t buffer_len, int64_t* out_len, char* out_str);
/* save the model as a standalone C++ translation unit (convert_model) */
LIGHTGBM_C_EXPORT int LGBM_AMD_BoosterSaveModelToIfElse(BoosterHandle handle, int num_iteration,
                                                        const char* filename);

#endif /* LGBM_AMD_C_API_H_ */
