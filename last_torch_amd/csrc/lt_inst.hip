// lt_inst.hip -- instantiates the forward / backward lattice kernels for one
// terms-per-lane value P (compile with -DLT_P=<P>); see lt_kernels.h.
#include "lt_kernels.h"

#if !defined(LT_P) || !defined(LT_LG) || !defined(LT_LGN)
#error "compile with -DLT_LG=<log2 lanes per group or -1> -DLT_LGN=<name> -DLT_P=<terms>"
#endif

#define LT_CAT4_(a, b, c, d) a##b##c##d
#define LT_CAT4(a, b, c, d) LT_CAT4_(a, b, c, d)

namespace {
template <typename K>
int launch_one(K kernel, const lt_impl::Plan& pl, int grid, hipStream_t st) {
  if (grid == 0) return LT_OK;
  hipError_t e = hipFuncSetAttribute((const void*)kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, pl.lds_bytes);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(pl.threads), pl.lds_bytes, st, pl.a);
  e = hipGetLastError();
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
template <int MODE>
int fwd_m(const lt_impl::Plan& pl, bool bf16, int grid, hipStream_t st) {
  if (bf16) return pl.wst ? launch_one(fwd_kernel<MODE, true, true, LT_LG, LT_P>, pl, grid, st)
                          : launch_one(fwd_kernel<MODE, true, false, LT_LG, LT_P>, pl, grid, st);
  return pl.wst ? launch_one(fwd_kernel<MODE, false, true, LT_LG, LT_P>, pl, grid, st)
                : launch_one(fwd_kernel<MODE, false, false, LT_LG, LT_P>, pl, grid, st);
}
}  // namespace

namespace lt_impl {
int LT_CAT4(launch_fwd_, LT_LGN, _, LT_P)(int mode, const Plan& pl, bool bf16, int grid, hipStream_t st) {
  switch (mode) {
    case M_LOG: return fwd_m<M_LOG>(pl, bf16, grid, st);
    case M_MAX: return fwd_m<M_MAX>(pl, bf16, grid, st);
    default: return fwd_m<M_REAL>(pl, bf16, grid, st);
  }
}
// the checkpointing pair (fwdbwd_kernel): same geometry for both plans
int LT_CAT4(launch_fwdbwd_, LT_LGN, _, LT_P)(const Plan& pf, const Plan& pb, bool bf16, int nb,
                                           hipStream_t st) {
  if (nb == 0) return LT_OK;
  const void* k = bf16 ? (pf.wst ? (const void*)fwdbwd_kernel<true, true, LT_LG, LT_P>
                                 : (const void*)fwdbwd_kernel<true, false, LT_LG, LT_P>)
                       : (pf.wst ? (const void*)fwdbwd_kernel<false, true, LT_LG, LT_P>
                                 : (const void*)fwdbwd_kernel<false, false, LT_LG, LT_P>);
  const int lds = pf.lds_bytes > pb.lds_bytes ? pf.lds_bytes : pb.lds_bytes;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  KArgs af = pf.a, ab = pb.a;
  void* args[] = {(void*)&af, (void*)&ab, (void*)&nb};
  e = hipLaunchKernel(k, dim3(2 * nb), dim3(pf.threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
// the frame-serial fallback's forward and backward in one launch (same
// geometry for both plans, direct dW stores)
int LT_CAT4(launch_serial_, LT_LGN, _, LT_P)(const Plan& pf, const Plan& pb, bool bf16, int nb,
                                           hipStream_t st) {
  if (nb == 0) return LT_OK;
  const void* k = bf16 ? (pf.wst ? (const void*)serial_kernel<true, true, true, LT_LG, LT_P>
                                 : (const void*)serial_kernel<true, false, true, LT_LG, LT_P>)
                       : (pf.wst ? (const void*)serial_kernel<false, true, true, LT_LG, LT_P>
                                 : (const void*)serial_kernel<false, false, true, LT_LG, LT_P>);
  const int lds = pf.lds_bytes > pb.lds_bytes ? pf.lds_bytes : pb.lds_bytes;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  KArgs af = pf.a, ab = pb.a;
  void* args[] = {(void*)&af, (void*)&ab};
  e = hipLaunchKernel(k, dim3(nb), dim3(pf.threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
int LT_CAT4(launch_bwd_, LT_LGN, _, LT_P)(const Plan& pl, bool bf16, int grid, hipStream_t st) {
  if (pl.ck) {
    if (bf16) return pl.wst ? launch_one(bwd_kernel<true, true, false, LT_LG, LT_P, true>, pl, grid, st)
                            : launch_one(bwd_kernel<true, false, false, LT_LG, LT_P, true>, pl, grid, st);
    return pl.wst ? launch_one(bwd_kernel<false, true, false, LT_LG, LT_P, true>, pl, grid, st)
                  : launch_one(bwd_kernel<false, false, false, LT_LG, LT_P, true>, pl, grid, st);
  }
  if (bf16) {
    if (pl.wst) return pl.dst ? launch_one(bwd_kernel<true, true, true, LT_LG, LT_P>, pl, grid, st)
                              : launch_one(bwd_kernel<true, true, false, LT_LG, LT_P>, pl, grid, st);
    return pl.dst ? launch_one(bwd_kernel<true, false, true, LT_LG, LT_P>, pl, grid, st)
                  : launch_one(bwd_kernel<true, false, false, LT_LG, LT_P>, pl, grid, st);
  }
  if (pl.wst) return pl.dst ? launch_one(bwd_kernel<false, true, true, LT_LG, LT_P>, pl, grid, st)
                            : launch_one(bwd_kernel<false, true, false, LT_LG, LT_P>, pl, grid, st);
  return pl.dst ? launch_one(bwd_kernel<false, false, true, LT_LG, LT_P>, pl, grid, st)
                : launch_one(bwd_kernel<false, false, false, LT_LG, LT_P>, pl, grid, st);
}
}  // namespace lt_impl
