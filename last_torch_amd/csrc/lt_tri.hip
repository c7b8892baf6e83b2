// lt_tri.hip -- the trigram checkpointing recursions (FullNGram n = 2,
// V <= 32, Log, W staged in LDS): alpha and beta of every utterance side by
// side in one launch (workgroups [0, B) forward, [B, 2B) backward), as
// fwdbwd_kernel, with the den role of den_fwd_tri / den_bwd_tri
// (lt_kernels.h): one lane per destination pair (forward) or source pair
// (backward), every term of a state in that lane's registers. The numerator
// and loader roles are fwd_body / bwd_body's own. lattices.py:379-496 and
// 686-799 (alignments.py:286-318, contexts.py:207-256).
#include "lt_kernels.h"

namespace {
// VT = 32: V a compile-time constant; VT = 1: any V <= 32
template <bool BF16, int VT>
__global__ __launch_bounds__(1024) void tri_fwdbwd_kernel(const KArgs af, const KArgs ab, int nb) {
  // diagnostic builds: LT_DBG 16 / 32 time one direction alone (results wrong)
  if ((int)blockIdx.x < nb) {
    if (!LT_ABL(af, 16)) fwd_body<M_LOG, BF16, true, 2, 9, VT>(af, blockIdx.x);
  } else if (!LT_ABL(af, 32)) {
    bwd_body<BF16, true, false, 2, 9, true, (int)sizeof(KArgs), VT>(ab, blockIdx.x - nb);
  }
}
}  // namespace

namespace lt_impl {
int launch_tri_fwdbwd(const Plan& pf, const Plan& pb, bool bf16, int nb, hipStream_t st) {
  if (nb == 0) return LT_OK;
  const bool v32 = pf.a.g.V == 32;
  const void* k = bf16 ? (v32 ? (const void*)tri_fwdbwd_kernel<true, 32>
                              : (const void*)tri_fwdbwd_kernel<true, 1>)
                       : (v32 ? (const void*)tri_fwdbwd_kernel<false, 32>
                              : (const void*)tri_fwdbwd_kernel<false, 1>);
  const int lds = pf.lds_bytes > pb.lds_bytes ? pf.lds_bytes : pb.lds_bytes;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  KArgs af = pf.a, ab = pb.a;
  void* args[] = {(void*)&af, (void*)&ab, (void*)&nb};
  e = hipLaunchKernel(k, dim3(2 * nb), dim3(pf.threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
}  // namespace lt_impl
