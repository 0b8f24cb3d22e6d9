// The br512x4 blind-rotation instantiations (params_sqrd_lvl_64 PBS, shortint_1bit bootstrap, vertical
// packing), compiled apart from kernels.hip so that they get their own code-generation flags (Makefile X4FLAGS).
#include <hip/hip_runtime.h>

#define TAE_X4_INSTANTIATE
#include "br512x4.hpp"

namespace tae {
namespace br512x4 {
template __global__ void br_kernel<3, true, 12>(TAE_X4_PARAMS);
template __global__ void br_kernel<7, true, 6>(TAE_X4_PARAMS);
template __global__ void br_kernel<1, false, 13>(TAE_X4_PARAMS);
}  // namespace br512x4
}  // namespace tae
