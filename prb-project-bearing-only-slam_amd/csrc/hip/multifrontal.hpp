// GPU supernodal multifrontal Cholesky (hip/multifrontal.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace bos {
struct Multifrontal;
namespace dev {

struct MfDevice;

// Upload the static tree / maps and allocate factor buffers. Returns 0 or < 0 with err.
int mf_create(const Multifrontal& F, MfDevice** out, std::string& err);
void mf_destroy(MfDevice* d);
// Numeric factorization of H (read from the block array A through the assembly map, fp64), fused
// with the forward substitution: x (permuted order) holds b on entry and L^{-1} b on exit.
hipError_t mf_factor(MfDevice* d, const double* A, double* x, hipStream_t s);
// Backward substitution: x <- L^{-T} x, completing x = H^{-1} b.
hipError_t mf_solve(MfDevice* d, double* x, hipStream_t s);
// device counter of non-positive pivots met by the last factorization
int32_t* mf_info_ptr(const MfDevice* d);
// work-queue tickets (kMfTickets ints), zero between iterations
int32_t* mf_tickets_ptr(const MfDevice* d);
constexpr int kMfTickets = 3;

}  // namespace dev
}  // namespace bos
