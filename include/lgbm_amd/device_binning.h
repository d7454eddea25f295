// Value -> bin mapping of dense matrices on the device (src/device/bin_kernels.hip;
// reference include/LightGBM/bin.h:132 ValueToBin).
#pragma once

#include <cstdint>
#include <vector>

#include "lgbm_amd/config.h"

namespace lgbm_amd {

class Dataset;

// device binning for an nrow x ncol matrix: LGBM_AMD_DEVICE_BINNING=0 never, =1 whenever a HIP
// device is visible, otherwise for device_type=gpu and at least 4M values
bool UseDeviceBinning(const Config& cfg, int64_t nrow, int64_t ncol);

// Writes the group columns of every group whose members are all numerical columns of the
// matrix (float32 or float64, row- or column-major) into `ds`, bit-identical to pushing the
// rows on the host.  Returns per column whether it was handled (the caller pushes the rest).
std::vector<char> DeviceBinDenseMatrix(Dataset* ds, const void* data, bool is_f64, int32_t nrow, int32_t ncol,
                                       bool row_major, const Config& cfg);

}  // namespace lgbm_amd
