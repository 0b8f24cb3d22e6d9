// The br1024 blind rotations (N = 1024: the 8-bit model, lvl_1 / 4 / 256) and their selectors, compiled apart
// from kernels.hip so that they get their own code-generation flags (Makefile B1KFLAGS).
#include <hip/hip_runtime.h>

#define TAE_B1K_INSTANTIATE
#include "br1024.hpp"
#include "br1024w.hpp"

namespace tae {
namespace br1024w {
template __global__ void br_kernel<6, 7>(TAE_B1KW_PARAMS);
}  // namespace br1024w
}  // namespace tae
