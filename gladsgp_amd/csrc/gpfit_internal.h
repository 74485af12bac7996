// Internal (non-exported) entry points shared between the library's translation units.
#pragma once
#include <hip/hip_runtime.h>

// z_b[r] = sum_{k<=r, k<n} Linv_b[r,k] w_b[k] for r0 <= r < r1   (linalg.hip)
hipError_t gpfit_trmv_rows_launch(const double* Linv, int ld, long long sL, const double* w,
                                  int ldw, double* z, int ldz, int r0, int r1, int n, int batch,
                                  hipStream_t st);
hipError_t gpfit_trmv_launch(const double* Linv, int ld, long long sL, const double* w,
                             int ldw, double* z, int ldz, int rows, int n, int batch,
                             hipStream_t st);
