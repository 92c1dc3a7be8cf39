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
// device word of the last factorization: count of non-positive pivots, | kMfStall when a dataflow
// launch timed out waiting for a dependency (its results are then invalid)
int32_t* mf_info_ptr(const MfDevice* d);
constexpr int32_t kMfStall = 1 << 30;
// work-queue tickets (kMfTickets ints, then kMfTickets exit counters); every flow launch leaves its
// ticket zero (the last wave out resets it)
int32_t* mf_tickets_ptr(const MfDevice* d);
constexpr int kMfTickets = 3;
// Test hook (bos_debug_inject_stall): the next factor flow launch starts at ticket 1, so its first
// front is never processed and its parent's wait times out — the stall path, end to end.
hipError_t mf_debug_skip_next_front(MfDevice* d, hipStream_t s);

}  // namespace dev
}  // namespace bos
