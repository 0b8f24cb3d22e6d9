// The br512p16 blind rotation (params_sqrd_lvl_64 PBS, sixteen points per lane), compiled apart from kernels.hip
// so that it gets its own code-generation flags (Makefile P16FLAGS).
#include <hip/hip_runtime.h>

#define TAE_P16_INSTANTIATE
#include "br512p16.hpp"

namespace tae {
namespace br512p16 {
template __global__ void br_kernel<3, 12>(TAE_P16_PARAMS);
}  // namespace br512p16
}  // namespace tae
