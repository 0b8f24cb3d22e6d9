// The br512lat blind rotation (params_sqrd_lvl_64, small batches), compiled apart from kernels.hip so that it
// gets its own code-generation flags (Makefile LATFLAGS).
#include <hip/hip_runtime.h>

#define TAE_LAT_INSTANTIATE
#include "br512lat.hpp"

namespace tae {
namespace br512lat {
template __global__ void br_kernel<3, 12>(TAE_LAT_PARAMS);
}  // namespace br512lat
}  // namespace tae
