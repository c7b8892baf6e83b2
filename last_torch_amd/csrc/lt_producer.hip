// lt_producer.hip -- the joint weight function's arc weights on the matrix
// cores (first step: the producer, not yet inside the
// recursions). JointWeightFn (weight_fns.py:174-227) computes, for every
// frame row f = (b, t) and context state c,
//
//   W[f, c, y] = bias[y] + sum_h Wo[y, h] * tanh(Pc[c, h] + Pf[f, h])
//
// with Pc = context_projection(context embeddings) [C, H], Pf =
// blank_projection(frames) [rows, H] (both plain GEMMs, left to the caller)
// and Wo / bias the stacked (blank, vocab) output projections [R = V+1, H].
// PyTorch materialises the [rows, C, H] hidden tensor (4.3 GB fp32 at the
// bench shape with H = 512); here each hidden tile is formed in registers
// as the A operand of v_mfma_f32_32x32x16_bf16 and never leaves the CU.
//
// Tiling: the flattened (f, c) rows are cut into 32-row wave tiles; a wave
// computes its tile against one or two 32-column tiles of y (R <= 64), K = H
// in steps of 16. Wo lives in LDS as bf16 [R][H] (loaded once per
// persistent workgroup). Hidden values and Wo are rounded to bf16, products
// accumulate in fp32 (MI355X_MICROARCH.md: dense bf16 MFMA).
#include "lt_kernels.h"

namespace {

struct JArgs {
  const float* pc;    // [C, H]
  const float* pf;    // [rows, H]
  const float* wo;    // [R, H]
  const float* bias;  // [R]
  void* W;            // [rows, C, R]
  long long rows;
  int C, H, R;
};

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// tanh(x) = 1 - 2 / (1 + e^{2x}): saturates to +-1 (exp over/underflow)
LT_DEVINL float fast_tanh(float x) {
  const float e = __expf(2.f * x);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
}

template <bool OBF16>
__global__ __launch_bounds__(256) void joint_weights_kernel(const JArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned short wol[];  // [R][H] bf16
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, R = a.R, C = a.C;
  for (int i = tid; i < R * H; i += blockDim.x) wol[i] = f2bf(a.wo[i]);
  __syncthreads();
  const long long M = a.rows * C;
  const long long ntile = (M + 31) / 32;
  const int r = lane & 31, hk = 8 * (lane >> 5);
  const int y0 = r, y1 = 32 + r;
  const bool v0 = y0 < R, v1 = y1 < R;
  const float b0 = v0 ? a.bias[y0] : 0.f, b1 = v1 ? a.bias[y1] : 0.f;
  const bf16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long long tile = (long long)blockIdx.x * 4 + wave; tile < ntile;
       tile += (long long)gridDim.x * 4) {
    const long long m = tile * 32 + r;
    const bool mv = m < M;
    const long long f = mv ? m / C : 0;
    const int c = mv ? (int)(m - f * C) : 0;
    const float* pc = a.pc + (long long)c * H + hk;
    const float* pf = a.pf + f * H + hk;
    f32x16 acc0 = {}, acc1 = {};
    for (int k0 = 0; k0 < H; k0 += 16) {
      const float4 c0 = *(const float4*)(pc + k0), c1 = *(const float4*)(pc + k0 + 4);
      const float4 f0 = *(const float4*)(pf + k0), f1 = *(const float4*)(pf + k0 + 4);
      const float x[8] = {c0.x + f0.x, c0.y + f0.y, c0.z + f0.z, c0.w + f0.w,
                          c1.x + f1.x, c1.y + f1.y, c1.z + f1.z, c1.w + f1.w};
      bf16x8 af;
#pragma unroll
      for (int j = 0; j < 8; ++j) af[j] = (short)f2bf(mv ? fast_tanh(x[j]) : 0.f);
      const bf16x8 bf0 = v0 ? *(const bf16x8*)(wol + y0 * H + k0 + hk) : zero8;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf0, acc0, 0, 0, 0);
      if (R > 32) {
        const bf16x8 bf1 = v1 ? *(const bf16x8*)(wol + y1 * H + k0 + hk) : zero8;
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf1, acc1, 0, 0, 0);
      }
    }
    // C/D: column y = lane & 31 (+32), row (i & 3) + 8 (i >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const long long mr = tile * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      if (mr >= M) continue;
      if (v0) stw<OBF16>(a.W, mr * R + y0, acc0[i] + b0);
      if (R > 32 && v1) stw<OBF16>(a.W, mr * R + y1, acc1[i] + b1);
    }
  }
}

}  // namespace

extern "C" {

int lt_joint_weights(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                     const float* ctx_proj, const float* frame_proj, const float* out_weight,
                     const float* out_bias, void* W, int32_t weight_dtype, void* stream) {
  if (rows < 0 || num_states < 1 || hidden < 1 || out_dim < 1)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: bad sizes");
  if (hidden % 16 || out_dim > 64)
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights: needs hidden % 16 == 0, V+1 <= 64");
  const long long lds = 2LL * out_dim * hidden;
  if (lds > 128 * 1024)
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights: output projection exceeds LDS");
  if (rows == 0) return LT_OK;
  if (!ctx_proj || !frame_proj || !out_weight || !out_bias || !W)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: null pointer");
  if (((uintptr_t)ctx_proj | (uintptr_t)frame_proj) & 15)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: projections must be 16-byte aligned");
  JArgs a;
  a.pc = ctx_proj; a.pf = frame_proj; a.wo = out_weight; a.bias = out_bias; a.W = W;
  a.rows = rows; a.C = num_states; a.H = hidden; a.R = out_dim;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long tiles = (rows * num_states + 31) / 32;
  const long long want = (tiles + 3) / 4;
  const int grid = (int)std::min<long long>(want, 4LL * cus);  // persistent: Wo loaded once per WG
  const bool bf = weight_dtype == LT_DTYPE_BF16;
  const void* k = bf ? (const void*)joint_weights_kernel<true> : (const void*)joint_weights_kernel<false>;
  hipStream_t st = (hipStream_t)stream;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  void* args[] = {&a};
  const hipError_t e = hipLaunchKernel(k, dim3(grid), dim3(256), args, (size_t)lds, st);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

}  // extern "C"
