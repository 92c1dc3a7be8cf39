// GPU supernodal multifrontal Cholesky (hip/multifrontal.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace bos {
struct Multifrontal;
namespace dev {

struct MfDevice;

// Upload the static tree / maps and allocate factor buffers. owner (per supernode, plan.hpp
// Shard::sn_owner) null: one GPU, every front in program 0. Otherwise program 0 = the fronts owned
// by `rank`, program 1 = the replicated top (owner -1); other ranks' fronts are never processed.
// Returns 0 or < 0 with err.
int mf_create(const Multifrontal& F, const int8_t* owner, int rank, MfDevice** out, std::string& err);
void mf_destroy(MfDevice* d);
// Numeric factorization of a program's fronts (H read from the block array A through the assembly
// map, fp64), fused with the forward substitution: x (permuted order) holds b on entry and L^{-1} b
// on exit for those fronts' dofs. Sharded: program 0 (own subtrees), then — once the other ranks'
// subtree roots' U / u are in place — program 1 (the top).
hipError_t mf_factor(MfDevice* d, int program, const double* A, double* x, hipStream_t s);
// fp32 J+H with factored pose-landmark blocks whose pose-landmark and landmark-diagonal entries only
// the folds read (bos::mf_fold_reads_fp32): the folds read them from the fp32 block array A32 (the
// factored region starting at pl_lo), so the fp64 copy need not hold them. Null: the folds read A.
void mf_set_fold_source(MfDevice* d, const float* A32, int64_t pl_lo);
// Backward substitution of a program's fronts (x <- L^{-T} x); sharded: program 1, then program 0.
hipError_t mf_solve(MfDevice* d, int program, double* x, hipStream_t s);
// the update matrices / u-vectors (offsets Multifrontal::U_off / u_off): exchange 1 reads and
// writes the subtree roots' there
double* mf_update_ptr(const MfDevice* d);
double* mf_uvec_ptr(const MfDevice* d);
// device word of the last factorization: count of non-positive pivots, | kMfStall when a dataflow
// launch timed out waiting for a dependency (its results are then invalid)
int32_t* mf_info_ptr(const MfDevice* d);
// device word the dataflow launches compare completion flags with: must be bumped (step_mark
// kernel, kernels.hpp) once per GN step before the step's first mf_factor; all flows of one step
// (factor and backward, both programs when sharded) share it
uint32_t* mf_epoch_ptr(const MfDevice* d);
// Diagnostics: the dataflow launches write 8 realtime stamps per front into stamps ([2][nsuper][8]:
// factor, backward); null (the default) turns them off.
void mf_debug_set_stamps(MfDevice* d, unsigned long long* stamps);
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
