// Complex f64 value as stored in the Fourier-domain keys (16-byte aligned for dwordx4 access).
#pragma once

namespace tae {
struct alignas(16) cplx {
    double re, im;
};
}  // namespace tae
