// lt_producer.hip -- the joint weight function's arc weights and their
// gradients on the matrix cores (first half: the
// producer as its own launches, not yet inside the recursions).
// JointWeightFn (weight_fns.py:174-227) computes, for every frame row
// f = (b, t) and context state c,
//
//   W[f, c, y] = bias[y] + sum_h Wo[y, h] * tanh(Pc[c, h] + Pf[f, h])
//
// with Pc = context_projection(context embeddings) [C, H], Pf =
// frame_projection(frames) [rows, H] (both plain GEMMs, left to the caller)
// and Wo / bias the stacked (blank, vocab) output projections [R = V+1, H].
// PyTorch materialises the [rows, C, H] hidden tensor (4.3 GB fp32 at the
// bench shape with H = 512); here each hidden tile is formed in registers
// as an operand of v_mfma_f32_32x32x16_bf16 and never leaves the CU.
//
// Kernels:
//   joint_exp_kernel         e^{2 Pc} (and e^{2 Pf} for the row-tile form), the
//                            |projection| > 40 flag
//   joint_weights_fb_kernel  forward, one workgroup per 32-frame block, waves
//                            walk the context states (the default)
//   joint_weights_kernel     forward, 32 flattened (f, c) rows per wave tile
//                            (blocks that exceed LDS)
//   joint_backward_kernel    d_wo, d_pf, d_pc (+ bias) per 32-frame block
//   joint_reduce_kernel      fixed-order sum of the per-workgroup partials
// Wo and the hidden values enter the forward products as bf16
// (LT_JOINT_BF16) or split-bf16 (LT_JOINT_SPLIT: hi + lo each, three
// products, fp32-faithful); the backward uses split-bf16 products; all sums
// are fp32.
#include "lt_joint.h"

namespace {

struct JArgs {
  const float* pc;    // [C, H]
  const float* pf;    // [rows, H]
  const float* ec;    // [C, H]    e^{2 pc} (workspace)
  const float* ef;    // [rows, H] e^{2 pf} (workspace)
  const int* big;     // != 0: some |projection| > kSplitMax, use the direct path
  const float* wo;    // [R, H]
  const float* bias;  // [R]
  void* W;            // [rows, C, R]
  long long rows;
  int C, H, R;
};

// e^{2x} of both projections, and the direct-path flag (rows * H and C * H
// values, float4 per thread).
__global__ __launch_bounds__(256) void joint_exp_kernel(const JArgs a, float* ec, float* ef,
                                                        int* big) {
  const long long nc = (long long)a.C * a.H / 4, nf = a.rows * a.H / 4;
  bool over = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nc + nf;
       i += (long long)gridDim.x * blockDim.x) {
    const bool isc = i < nc;
    const float4 x = isc ? ((const float4*)a.pc)[i] : ((const float4*)a.pf)[i - nc];
    const float m = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
    over |= !(m <= kSplitMax);  // NaN counts as over
    const f32x2 lo = exp2x(f32x2{x.x, x.y}), hi = exp2x(f32x2{x.z, x.w});
    const float4 e = {lo.x, lo.y, hi.x, hi.y};
    if (isc) ((float4*)ec)[i] = e;
    else ((float4*)ef)[i - nc] = e;
  }
  if (__any(over) && (threadIdx.x & 63) == 0) atomicOr(big, 1);
}

// One wave: a 32-row tile of the flattened (f, c) rows against one or two
// 32-column tiles of y (TWO: R > 32), K = H in steps of 16.
template <bool OBF16, bool TWO, bool SP>
__global__ __launch_bounds__(256) void joint_weights_kernel(const JArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned short wol[];  // [R][H + 8] bf16 (x2: SP)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, R = a.R, C = a.C, HP = H + 8;  // padded rows: no LDS bank conflicts
  const int WL = R * HP;  // SP: the lo block's offset
  stage_wo<SP>(a.wo, wol, R, H, HP, WL, tid, blockDim.x);
  __syncthreads();
  const bool split = *a.big == 0;
  const long long M = a.rows * C;
  const long long ntile = (M + 31) / 32;
  const int r = lane & 31, hk = 8 * (lane >> 5);
  const int y0 = r, y1 = 32 + r;
  const bool v0 = y0 < R, v1 = y1 < R;
  const float b0 = v0 ? a.bias[y0] : 0.f, b1 = v1 ? a.bias[y1] : 0.f;
  // columns past R read row R - 1 (valid) and are never stored
  const unsigned short* w0 = wol + (v0 ? y0 : R - 1) * HP + hk;
  const unsigned short* w1 = wol + (v1 ? y1 : R - 1) * HP + hk;
  const unsigned short* w0l = w0 + WL;
  const unsigned short* w1l = w1 + WL;
  for (long long tile = (long long)blockIdx.x * 4 + wave; tile < ntile;
       tile += (long long)gridDim.x * 4) {
    const long long m = tile * 32 + r;
    const long long mm = m < M ? m : M - 1;  // rows past M load row M - 1, never stored
    const long long f = mm / C;
    const int c = (int)(mm - f * C);
    f32x16 acc0 = {}, acc1 = {};
    if (split) {
      const float* pc = a.ec + (long long)c * H + hk;
      const float* pf = a.ef + f * H + hk;
#pragma unroll 2
      for (int k0 = 0; k0 < H; k0 += 16) {
        const float4 c0 = *(const float4*)(pc + k0), c1 = *(const float4*)(pc + k0 + 4);
        const float4 f0 = *(const float4*)(pf + k0), f1 = *(const float4*)(pf + k0 + 4);
        const f32x2 tp[4] = {tanh_from_exp(f32x2{c0.x, c0.y} * f32x2{f0.x, f0.y}),
                             tanh_from_exp(f32x2{c0.z, c0.w} * f32x2{f0.z, f0.w}),
                             tanh_from_exp(f32x2{c1.x, c1.y} * f32x2{f1.x, f1.y}),
                             tanh_from_exp(f32x2{c1.z, c1.w} * f32x2{f1.z, f1.w})};
        joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
      }
    } else {
      const float* pc = a.pc + (long long)c * H + hk;
      const float* pf = a.pf + f * H + hk;
#pragma unroll 2
      for (int k0 = 0; k0 < H; k0 += 16) {
        const float4 c0 = *(const float4*)(pc + k0), c1 = *(const float4*)(pc + k0 + 4);
        const float4 f0 = *(const float4*)(pf + k0), f1 = *(const float4*)(pf + k0 + 4);
        const f32x2 tp[4] = {tanh_from_exp(exp2x(f32x2{c0.x + f0.x, c0.y + f0.y})),
                             tanh_from_exp(exp2x(f32x2{c0.z + f0.z, c0.w + f0.w})),
                             tanh_from_exp(exp2x(f32x2{c1.x + f1.x, c1.y + f1.y})),
                             tanh_from_exp(exp2x(f32x2{c1.z + f1.z, c1.w + f1.w}))};
        joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
      }
    }
    // C/D: column y = lane & 31 (+32), row (i & 3) + 8 (i >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const long long mr = tile * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      if (mr >= M) continue;
      if (v0) stw<OBF16>(a.W, mr * R + y0, acc0[i] + b0);
      if (TWO && v1) stw<OBF16>(a.W, mr * R + y1, acc1[i] + b1);
    }
  }
}

template <bool OBF16, bool SP>
const void* pick(bool two) {
  return two ? (const void*)joint_weights_kernel<OBF16, true, SP>
             : (const void*)joint_weights_kernel<OBF16, false, SP>;
}

// Frame-block form (used when a block fits LDS): a workgroup stages 32
// frames' e^{2 pf} (or pf on the direct path) in LDS once and its waves walk
// the context states, so the per-tile operands come from LDS plus one
// broadcast row of e^{2 pc}; the row-tile form above re-reads both per tile.
template <bool OBF16, bool TWO, bool SP>
__global__ __launch_bounds__(1024) void joint_weights_fb_kernel(const JArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned short wfl[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int H = a.H, R = a.R, C = a.C, HP = H + 8, FS = H + 4;
  const int WL = (R * HP + 7) & ~7;                           // SP: the lo block's offset
  float* fb = (float*)(wfl + (SP ? 2 : 1) * WL);  // [32][H + 4] fp32
  float* crow = fb + 32 * FS + wave * H;             // [waves][H] fp32
  stage_wo<SP>(a.wo, wfl, R, H, HP, WL, tid, blockDim.x);
  const bool csplit = *a.big == 0;  // every |pc| <= kSplitMax (the pre-pass's flag)
  const int rows = (int)a.rows;  // < 2^31 / H (host check)
  const int nblk = (rows + 31) / 32;
  const int r = lane & 31, hk = 8 * (lane >> 5), half = lane >> 5;
  const int y0 = r, y1 = 32 + r;
  const bool v0 = y0 < R, v1 = y1 < R;
  const float b0 = v0 ? a.bias[y0] : 0.f, b1 = v1 ? a.bias[y1] : 0.f;
  const unsigned short* w0 = wfl + (v0 ? y0 : R - 1) * HP + hk;
  const unsigned short* w1 = wfl + (v1 ? y1 : R - 1) * HP + hk;
  const unsigned short* w0l = w0 + WL;
  const unsigned short* w1l = w1 + WL;
  const int h4 = H / 4;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    __syncthreads();  // Wo staged / previous block's reads done
    // stage pf, decide split vs direct for this block, then turn the block
    // into e^{2 pf} in place (each thread its own elements)
    bool over = false;
    for (int e = tid; e < 32 * h4; e += blockDim.x) {
      const int m = e / h4, k4 = e - m * h4;
      const int f = 32 * blk + m;
      const float4 v = f < rows ? ((const float4*)a.pf)[(size_t)f * h4 + k4]
                                : float4{0.f, 0.f, 0.f, 0.f};
      const float mx = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
      over |= !(mx <= kSplitMax);  // NaN counts as over
      *(float4*)(fb + m * FS + 4 * k4) = v;
    }
    const bool split = csplit && !__syncthreads_or(over);
    if (split) {
      for (int e = tid; e < 32 * h4; e += blockDim.x) {
        const int m = e / h4, k4 = e - m * h4;
        float4* q = (float4*)(fb + m * FS + 4 * k4);
        const float4 v = *q;
        const f32x2 lo = exp2x(f32x2{v.x, v.y}), hi = exp2x(f32x2{v.z, v.w});
        *q = float4{lo.x, lo.y, hi.x, hi.y};
      }
    }
    const float* csrc = split ? a.ec : a.pc;
    __syncthreads();
    const float* fr = fb + r * FS + hk;
    // this wave's context row (e^{2 pc[c]} or pc[c]) goes through a private
    // LDS slice, loaded one tile ahead
    float4 p0, p1, p2, p3;
    const float4 z4 = {0.f, 0.f, 0.f, 0.f};
    auto load_row = [&](int cc) {
      const float4* src = (const float4*)(csrc + (size_t)cc * H);
      p0 = lane < h4 ? src[lane] : z4;
      p1 = lane + 64 < h4 ? src[lane + 64] : z4;
      p2 = lane + 128 < h4 ? src[lane + 128] : z4;
      p3 = lane + 192 < h4 ? src[lane + 192] : z4;
    };
    if (wave < C) load_row(wave);
    for (int c = wave; c < C; c += nw) {
      float4* cw = (float4*)crow;
      if (lane < h4) cw[lane] = p0;
      if (lane + 64 < h4) cw[lane + 64] = p1;
      if (lane + 128 < h4) cw[lane + 128] = p2;
      if (lane + 192 < h4) cw[lane + 192] = p3;
      if (c + nw < C) load_row(c + nw);
      const float* cr = crow + hk;
      f32x16 acc0 = {}, acc1 = {};
      if (split) {
#pragma unroll 2
        for (int k0 = 0; k0 < H; k0 += 16) {
          const float4 c0 = *(const float4*)(cr + k0), c1 = *(const float4*)(cr + k0 + 4);
          const float4 f0 = *(const float4*)(fr + k0), f1 = *(const float4*)(fr + k0 + 4);
          const f32x2 tp[4] = {tanh_from_exp(f32x2{c0.x, c0.y} * f32x2{f0.x, f0.y}),
                               tanh_from_exp(f32x2{c0.z, c0.w} * f32x2{f0.z, f0.w}),
                               tanh_from_exp(f32x2{c1.x, c1.y} * f32x2{f1.x, f1.y}),
                               tanh_from_exp(f32x2{c1.z, c1.w} * f32x2{f1.z, f1.w})};
          joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
        }
      } else {
#pragma unroll 2
        for (int k0 = 0; k0 < H; k0 += 16) {
          const float4 c0 = *(const float4*)(cr + k0), c1 = *(const float4*)(cr + k0 + 4);
          const float4 f0 = *(const float4*)(fr + k0), f1 = *(const float4*)(fr + k0 + 4);
          const f32x2 tp[4] = {tanh_from_exp(exp2x(f32x2{c0.x + f0.x, c0.y + f0.y})),
                               tanh_from_exp(exp2x(f32x2{c0.z + f0.z, c0.w + f0.w})),
                               tanh_from_exp(exp2x(f32x2{c1.x + f1.x, c1.y + f1.y})),
                               tanh_from_exp(exp2x(f32x2{c1.z + f1.z, c1.w + f1.w}))};
          joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
        }
      }
      // C/D: column y = lane & 31 (+32), row = frame (i & 3) + 8 (i >> 2) + 4 half
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int f = 32 * blk + (i & 3) + 8 * (i >> 2) + 4 * half;
        if (f >= rows) continue;
        const long long mr = (long long)f * C + c;
        if (v0) stw<OBF16>(a.W, mr * R + y0, acc0[i] + b0);
        if (TWO && v1) stw<OBF16>(a.W, mr * R + y1, acc1[i] + b1);
      }
    }
  }
}

template <bool OBF16, bool SP>
const void* pick_fb(bool two) {
  return two ? (const void*)joint_weights_fb_kernel<OBF16, true, SP>
             : (const void*)joint_weights_fb_kernel<OBF16, false, SP>;
}

// Wo bf16 (hi, and lo for SP), the frame block, a context row per wave
long long fb_lds(int H, int R, int nw, bool sp) {
  return (sp ? 4LL : 2LL) * (((long long)R * (H + 8) + 7) & ~7LL) + 4LL * 32 * (H + 4) +
         4LL * nw * H;
}

// waves per frame-block workgroup: the fewest in [4, 16] that give the
// fewest context tiles per wave (C = 33: 11 waves x 3 tiles, not 8 x 5)
int fb_waves(int C) {
  int best = 4;
  for (int w = 5; w <= 16; ++w)
    if ((C + w - 1) / w < (C + best - 1) / best) best = w;
  return best;
}

size_t ws_bytes(long long rows, int C, int H) {
  return 256 + 4 * (size_t)H * ((size_t)C + (size_t)rows);
}

}  // namespace

extern "C" {

int lt_joint_weights_workspace_bytes(int64_t rows, int32_t num_states, int32_t hidden,
                                     size_t* bytes) {
  if (!bytes || rows < 0 || num_states < 1 || hidden < 1)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights_workspace_bytes: bad arguments");
  *bytes = ws_bytes(rows, num_states, hidden);
  return LT_OK;
}

int lt_joint_weights(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                     const float* ctx_proj, const float* frame_proj, const float* out_weight,
                     const float* out_bias, void* W, int32_t weight_dtype, void* workspace,
                     size_t workspace_bytes, void* stream) {
  return lt_joint_weights_ex(rows, num_states, hidden, out_dim, ctx_proj, frame_proj, out_weight,
                             out_bias, W, weight_dtype, LT_JOINT_BF16, workspace, workspace_bytes,
                             stream);
}

int lt_joint_weights_ex(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                        const float* ctx_proj, const float* frame_proj, const float* out_weight,
                        const float* out_bias, void* W, int32_t weight_dtype, int32_t precision,
                        void* workspace, size_t workspace_bytes, void* stream) {
  if (rows < 0 || num_states < 1 || hidden < 1 || out_dim < 1)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: bad sizes");
  if (precision != LT_JOINT_BF16 && precision != LT_JOINT_SPLIT)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: precision must be LT_JOINT_BF16 or LT_JOINT_SPLIT");
  const bool sp = precision == LT_JOINT_SPLIT;
  if (hidden % 16 || out_dim > 64)
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights: needs hidden % 16 == 0, V+1 <= 64");
  const long long lds = (sp ? 4LL : 2LL) * out_dim * (hidden + 8);
  if (lds > 128 * 1024)
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights: output projection exceeds LDS");
  if (rows == 0) return LT_OK;
  if (!ctx_proj || !frame_proj || !out_weight || !out_bias || !W || !workspace)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: null pointer");
  if (((uintptr_t)ctx_proj | (uintptr_t)frame_proj | (uintptr_t)workspace) & 15)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: projections and workspace must be 16-byte aligned");
  if (workspace_bytes < ws_bytes(rows, num_states, hidden))
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights: workspace too small");
  JArgs a;
  char* ws = (char*)workspace;
  int* big = (int*)ws;
  float* ec = (float*)(ws + 256);
  float* ef = ec + (size_t)num_states * hidden;
  a.pc = ctx_proj; a.pf = frame_proj; a.ec = ec; a.ef = ef; a.big = big;
  a.wo = out_weight; a.bias = out_bias; a.W = W;
  a.rows = rows; a.C = num_states; a.H = hidden; a.R = out_dim;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(big, 0, sizeof(int), st);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  const int fnw = fb_waves(num_states);
  const long long lfb = fb_lds(hidden, out_dim, fnw, sp);
  const bool use_fb = lfb <= 160 * 1024 && hidden <= 1024 && rows * (long long)hidden < (1LL << 31);
  {
    // the frame-block kernel forms e^{2 pf} itself: the pre-pass then covers pc only
    JArgs ax = a;
    if (use_fb) ax.rows = 0;
    const long long n4 = ((long long)num_states + ax.rows) * hidden / 4;
    const int grid = (int)std::max<long long>(1, std::min<long long>((n4 + 255) / 256, 8LL * cus));
    void* args[] = {&ax, &ec, &ef, &big};
    e = hipLaunchKernel((const void*)joint_exp_kernel, dim3(grid), dim3(256), args, 0, st);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  const bool bf = weight_dtype == LT_DTYPE_BF16, two = out_dim > 32;
  void* args[] = {&a};
  if (use_fb) {
    // frame-block form: one workgroup of fnw waves per CU
    const void* k = sp ? (bf ? pick_fb<true, true>(two) : pick_fb<false, true>(two))
                       : (bf ? pick_fb<true, false>(two) : pick_fb<false, false>(two));
    if (lfb > 64 * 1024) {
      e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfb);
      if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
    }
    const int grid = (int)std::min<long long>((rows + 31) / 32, cus);
    e = hipLaunchKernel(k, dim3(grid), dim3(64 * fnw), args, (size_t)lfb, st);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
    return LT_OK;
  }
  const long long tiles = (rows * num_states + 31) / 32;
  const long long want = (tiles + 3) / 4;
  const int grid = (int)std::min<long long>(want, 4LL * cus);  // persistent: Wo loaded once per WG
  const void* k = sp ? (bf ? pick<true, true>(two) : pick<false, true>(two))
                     : (bf ? pick<true, false>(two) : pick<false, false>(two));
  if (lds > 64 * 1024) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  e = hipLaunchKernel(k, dim3(grid), dim3(256), args, (size_t)lds, st);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Backward of the joint weight function (the adjoint of lt_joint_weights):
// with g = dL/dW [rows * C, R], hid = tanh(pc[c] + pf[f]) recomputed in fp32,
//   gw[m, h]   = sum_r g[m, r] wo[r, h]          (MFMA, K = R)
//   dh[m, h]   = gw[m, h] (1 - hid[m, h]^2)
//   d_wo[r, h] = sum_m g[m, r] hid[m, h]          (MFMA, K = the tile's 32 rows)
//   d_pf[f, h] = sum_c dh[(f, c), h]              (registers, over the C tiles)
//   d_pc[c, h] = sum_f dh[(f, c), h]              (column sum per tile, LDS)
// A tile is 32 frames x ONE context state c: a workgroup takes a block of 32
// frames and walks c = 0..C-1, so pf stays in registers for the block, pc is
// one value per lane and tile, and d_pf accumulates in registers (no atomics).
// Products are split-bf16 (x = hi + lo; hi*hi + hi*lo + lo*hi), about 16
// mantissa bits, sums fp32. Each wave owns 32 hidden columns for the whole
// launch, so its d_wo block stays in registers; the MFMA output layout of
// gw / hid (row (i & 3) + 8 (i >> 2) + 4 half) is used directly as the K
// operand of d_wo (the K order only has to agree between A and B).
namespace {

struct JBArgs {
  const float* pc;   // [C, H]
  const float* pf;   // [rows, H]
  const float* wo;   // [R, H]
  const float* g;    // [rows * C, R]
  float* dpf;        // [rows, H]
  float* part;       // [grid][C + R][H] per-workgroup d_pc, d_wo
  long long rows;
  int C, H, R;
};

typedef short bf16x4 __attribute__((ext_vector_type(4)));
// 8 bf16: p[0..3] and p[8..11] (8-byte aligned)
LT_DEVINL bf16x8 tpair(const unsigned short* p) {
  const bf16x4 a = *(const bf16x4*)p, b = *(const bf16x4*)(p + 8);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int KB, bool TWO, int NW>  // KB = ceil(R / 16) K blocks of gw; TWO: R > 32; NW waves
__global__ __launch_bounds__(64 * NW) void joint_backward_kernel(const JBArgs a) {
  extern __shared__ __attribute__((aligned(16))) float bl[];
  constexpr int GS = KB * 16 + 4;   // fp32 g tile row stride (floats)
  constexpr int GB = KB * 16 + 8;   // bf16 g tile row stride: [m][r]
  constexpr int RB = TWO ? 64 : 32;  // rows of the transposed bf16 tile: [r][m]
  constexpr int TS = 32 + 4;        // its row stride
  constexpr int GN = 32 * KB * 16;  // g tile elements staged per tile
  constexpr int nthr = 64 * NW, HW = 32 * NW;
  // 8 waves share each staged g value: split it once at staging (PRE);
  // smaller workgroups split in each wave instead (fewer staging stores)
  constexpr bool PRE = NW == 8;
  // per buffer (bytes): fp32 [32][GS] | (PRE) hi, lo [32][GB] | hi, lo [RB][TS]
  // -- small workgroups allocate the fp32 tile only, so more of them fit a
  // CU (round 4: at H = 32, one wave per workgroup, 3 -> 9 workgroups a CU)
  constexpr int BUFB = 4 * 32 * GS + (PRE ? 2 * 2 * 32 * GB + 2 * 2 * RB * TS : 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, R = a.R, C = a.C;
  // this workgroup's hidden columns: [h0, h0 + HW)
  const int h0 = blockIdx.y * HW;
  // double-buffered g tile: fp32 (bias sums), bf16 hi/lo splits [m][r] (gw's
  // A operand) and transposed [r][m] (d_wo's A operand), split once here
  // instead of in every wave
  float* dpc = (float*)((char*)bl + 2 * BUFB);  // [C][HW]
  for (int e = tid; e < C * HW; e += nthr) dpc[e] = 0.f;
  const int half = lane >> 5, col = lane & 31;
  const int hl = wave * 32 + col, h = h0 + hl;
  const int rows = (int)a.rows;  // rows * max(C, H) < 2^31 (host check)
  const int nblk = (rows + 31) / 32;
  bf16x8 woh[KB], wol[KB];  // B[k = r][n = h] of gw
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = 16 * kb + 8 * half + j;
      v[j] = r < R ? a.wo[(long long)r * H + h] : 0.f;
    }
    split8(v, woh[kb], wol[kb]);
  }
  f32x16 dwo0 = {}, dwo1 = {};
  float dbias = 0.f;  // thread tid < R of blockIdx.y == 0: sum of g[:, tid]
  constexpr int GPT = (GN + nthr - 1) / nthr;  // staged g values per thread
  float gnext[GPT];
  // tile (blk, c): rows (f = 32 blk + m, c), m < 32
  auto load_g = [&](int blk, int c) {
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
      const int e = tid + u * nthr;
      const int m = e / (KB * 16), r = e - m * (KB * 16);
      const int f = 32 * blk + m;
      gnext[u] = (e < GN && blk < nblk && f < rows && r < R)
                     ? a.g[((size_t)f * C + c) * R + r] : 0.f;
    }
  };
  int buf = 0;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    // this lane's 16 frames (MFMA output rows) and their projections
    float pfv[16], dpf[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = 32 * blk + (i & 3) + 8 * (i >> 2) + 4 * half;
      pfv[i] = f < rows ? a.pf[(size_t)f * H + h] : 0.f;
      dpf[i] = 0.f;
    }
    load_g(blk, 0);
    for (int c = 0; c < C; ++c, buf ^= 1) {
      char* bb = (char*)bl + buf * BUFB;
      float* gt = (float*)bb;
      unsigned short* gh = (unsigned short*)(bb + 4 * 32 * GS);
      unsigned short* gl = gh + 32 * GB;
      unsigned short* th = gl + 32 * GB;
      unsigned short* tl = th + RB * TS;
#pragma unroll
      for (int u = 0; u < GPT; ++u) {
        const int e = tid + u * nthr;
        if (e < GN) {
          const int m = e / (KB * 16), r = e - m * (KB * 16);
          const float v = gnext[u];
          const unsigned short hi = __builtin_bit_cast(unsigned short, (__bf16)v);
          const unsigned short lo =
              __builtin_bit_cast(unsigned short, (__bf16)(v - __uint_as_float((unsigned)hi << 16)));
          gt[m * GS + r] = v;
          if constexpr (PRE) {
            gh[m * GB + r] = hi;
            gl[m * GB + r] = lo;
            if (r < RB) {
              th[r * TS + m] = hi;
              tl[r * TS + m] = lo;
            }
          }
        }
      }
      __syncthreads();  // one barrier per tile: the other buffer is written next
      if (c + 1 < C) load_g(blk, c + 1);  // in flight during this tile
      if (blockIdx.y == 0 && tid < R)
        for (int m = 0; m < 32; ++m) dbias += gt[m * GS + tid];
      const float pcv = a.pc[c * H + h];
      // gw: A[m = col][k = r]
      f32x16 gw = {};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        bf16x8 ah, al;
        if constexpr (PRE) {
          ah = *(const bf16x8*)(gh + col * GB + 16 * kb + 8 * half);
          al = *(const bf16x8*)(gl + col * GB + 16 * kb + 8 * half);
        } else {
          const float4 x0 = *(const float4*)(gt + col * GS + 16 * kb + 8 * half);
          const float4 x1 = *(const float4*)(gt + col * GS + 16 * kb + 8 * half + 4);
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split8(v, ah, al);
        }
        gw = mfma3(ah, al, woh[kb], wol[kb], gw);
      }
      float csum = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        // K slot (half, j) <-> row m(i = 8q + j, half): this lane's own rows
        float hv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * q + j;
          const float e = __builtin_amdgcn_exp2f((pcv + pfv[i]) * (2.f * kLog2e));
          const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
          hv[j] = t;  // rows past `rows` have g = 0: no contribution to d_wo
          const float d = gw[i] * (1.f - t * t);
          dpf[i] += d;
          csum += d;
        }
        bf16x8 hh, hlo;
        split8(hv, hh, hlo);
        // A[r][k slot (half, j)] = g[m][r], m = 16q + 4 half + (j & 3) + 8 (j >> 2):
        // two runs of 4 in the transposed tile
        const int tm = 16 * q + 4 * half;
        if constexpr (PRE) {
          dwo0 = mfma3(tpair(th + col * TS + tm), tpair(tl + col * TS + tm), hh, hlo, dwo0);
          if (TWO)
            dwo1 = mfma3(tpair(th + (32 + col) * TS + tm), tpair(tl + (32 + col) * TS + tm), hh,
                         hlo, dwo1);
        } else {  // split in this wave (fewer staging stores for small workgroups)
          float gv[8];
          bf16x8 gh8, gl8;
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] = gt[(tm + (j & 3) + 8 * (j >> 2)) * GS + col];
          split8(gv, gh8, gl8);
          dwo0 = mfma3(gh8, gl8, hh, hlo, dwo0);
          if (TWO) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = gt[(tm + (j & 3) + 8 * (j >> 2)) * GS + 32 + col];
            split8(gv, gh8, gl8);
            dwo1 = mfma3(gh8, gl8, hh, hlo, dwo1);
          }
        }
      }
      csum += __shfl_xor(csum, 32);
      if (half == 0) dpc[c * HW + hl] += csum;  // this wave owns column hl
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = 32 * blk + (i & 3) + 8 * (i >> 2) + 4 * half;
      if (f < rows) a.dpf[(size_t)f * H + h] = dpf[i];
    }
  }
  // per-workgroup partials: d_pc rows [0, C), d_wo rows [C, C + R), d_bias after them
  float* part = a.part + (long long)blockIdx.x * ((long long)(C + R) * H + 64);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = (i & 3) + 8 * (i >> 2) + 4 * half;
    if (r < R) part[(long long)(C + r) * H + h] = dwo0[i];
    if (TWO && r + 32 < R) part[(long long)(C + r + 32) * H + h] = dwo1[i];
  }
  if (blockIdx.y == 0 && tid < R) part[(long long)(C + R) * H + tid] = dbias;
  __syncthreads();
  for (int e = tid; e < C * HW; e += nthr) {
    const int c = e / HW;
    part[(long long)c * H + h0 + (e - c * HW)] = dpc[e];
  }
}

// out[e] = sum_g part[g][e] (fixed order: deterministic); part rows are
// d_pc [C*H] | d_wo [R*H] | d_bias [R] with a per-workgroup stride. One wave
// per output element: lane l sums the partials l, l + 64, ... in order, then
// a fixed xor butterfly (the serial sum over thousands of partials was
// latency-bound: 0.4 ms at 2,048 workgroups)
__global__ __launch_bounds__(256) void joint_reduce_kernel(const float* part, int grid,
                                                           long long stride, long long npc,
                                                           long long nwo, int R, float* dpc,
                                                           float* dwo, float* dbias) {
  const long long n = npc + nwo + R;
  const int lane = threadIdx.x & 63;
  for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < n;
       e += ((long long)gridDim.x * blockDim.x) >> 6) {
    float s = 0.f;
    for (int b = lane; b < grid; b += 64) s += part[(long long)b * stride + e];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) {
      if (e < npc) dpc[e] = s;
      else if (e < npc + nwo) dwo[e - npc] = s;
      else dbias[e - npc - nwo] = s;
    }
  }
}

template <int KB, bool TWO>
const void* pick_nw(int nw) {
  return nw == 8 ? (const void*)joint_backward_kernel<KB, TWO, 8>
       : nw == 4 ? (const void*)joint_backward_kernel<KB, TWO, 4>
       : nw == 2 ? (const void*)joint_backward_kernel<KB, TWO, 2>
                 : (const void*)joint_backward_kernel<KB, TWO, 1>;
}

// waves per workgroup: the largest of 8, 4, 2, 1 dividing hidden / 32
int bwd_waves(int H) {
  const int n = H / 32;
  return n % 8 == 0 ? 8 : n % 4 == 0 ? 4 : n % 2 == 0 ? 2 : 1;
}

long long bwd_lds(int C, int H, int R) {  // keep in sync with BUFB
  const int KB = (R + 15) / 16, RB = R > 32 ? 64 : 32;
  const bool pre = bwd_waves(H) == 8;
  const long long bufb =
      4LL * 32 * (KB * 16 + 4) + (pre ? 4LL * 32 * (KB * 16 + 8) + 4LL * RB * 36 : 0);
  return 2 * bufb + 4LL * C * 32 * bwd_waves(H);
}

int bwd_grid(long long rows, int C, int H, int R) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long tiles = (rows + 31) / 32;  // blocks of 32 frames
  const int gy = std::max(1, H / (32 * bwd_waves(H)));
  // as many resident workgroups per CU as LDS and waves allow (at most 8
  // waves' worth of workgroups: 1-wave workgroups are latency-bound alone)
  const long long lds = std::max<long long>(1, bwd_lds(C, H, R));
  const long long per_cu = std::max<long long>(
      1, std::min<long long>(160 * 1024 / lds, std::max(1, 8 / bwd_waves(H))));
  const long long gx = std::max<long long>(1, cus * per_cu / gy);
  return (int)std::max<long long>(1, std::min<long long>(tiles, gx));
}

long long bwd_stride(int C, int H, int R) { return (long long)(C + R) * H + 64; }

}  // namespace

extern "C" {

int lt_joint_weights_backward_workspace_bytes(int64_t rows, int32_t num_states, int32_t hidden,
                                              int32_t out_dim, size_t* bytes) {
  if (!bytes || rows < 0 || num_states < 1 || hidden < 32 || out_dim < 1)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights_backward_workspace_bytes: bad arguments");
  *bytes = 4 * (size_t)bwd_grid(rows, num_states, hidden, out_dim) * bwd_stride(num_states, hidden, out_dim);
  return LT_OK;
}

int lt_joint_weights_backward(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                              const float* ctx_proj, const float* frame_proj,
                              const float* out_weight, const float* grad_W, float* d_ctx_proj,
                              float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                              void* workspace, size_t workspace_bytes, void* stream) {
  const int C = num_states, H = hidden, R = out_dim;
  if (rows < 0 || C < 1 || H < 1 || R < 1)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights_backward: bad sizes");
  if (H % 32 || R > 64)
    return lt_impl::set_error(LT_EUNSUPPORTED,
                              "lt_joint_weights_backward: needs hidden % 32 == 0, V+1 <= 64");
  const long long lds = bwd_lds(C, H, R);
  if (lds > 160 * 1024)
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights_backward: d_ctx_proj block exceeds LDS");
  if (rows * (long long)C >= (1LL << 31) || rows * (long long)H >= (1LL << 31))
    return lt_impl::set_error(LT_EUNSUPPORTED, "lt_joint_weights_backward: rows * C or rows * H >= 2^31");
  if (!ctx_proj || !out_weight || !d_ctx_proj || !d_out_weight || !d_out_bias ||
      (rows > 0 && (!frame_proj || !grad_W || !d_frame_proj || !workspace)))
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights_backward: null pointer");
  size_t need = 0;
  (void)lt_joint_weights_backward_workspace_bytes(rows, C, H, R, &need);
  if (rows > 0 && workspace_bytes < need)
    return lt_impl::set_error(LT_EINVAL, "lt_joint_weights_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (rows == 0) {
    e = hipMemsetAsync(d_ctx_proj, 0, 4 * (size_t)C * H, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_out_weight, 0, 4 * (size_t)R * H, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_out_bias, 0, 4 * (size_t)R, st);
    return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  JBArgs a;
  a.pc = ctx_proj; a.pf = frame_proj; a.wo = out_weight; a.g = grad_W;
  a.dpf = d_frame_proj; a.part = (float*)workspace;
  a.rows = rows; a.C = C; a.H = H; a.R = R;
  const int grid = bwd_grid(rows, C, H, R);
  const int nw = bwd_waves(H);
  const int KB = (R + 15) / 16;
  const void* k = KB == 1 ? pick_nw<1, false>(nw) : KB == 2 ? pick_nw<2, false>(nw)
                : KB == 3 ? pick_nw<3, true>(nw) : pick_nw<4, true>(nw);
  if (lds > 64 * 1024) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  void* args[] = {&a};
  e = hipLaunchKernel(k, dim3(grid, H / (32 * nw)), dim3(64 * nw), args, (size_t)lds, st);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  long long stride = bwd_stride(C, H, R), npc = (long long)C * H, nwo = (long long)R * H;
  int gridv = grid, Rv = R;
  const int rg = (int)std::min<long long>((npc + nwo + R + 3) / 4, 8192);  // a wave per element
  void* rargs[] = {&a.part, &gridv, &stride, &npc, &nwo, &Rv, &d_ctx_proj, &d_out_weight,
                   &d_out_bias};
  e = hipLaunchKernel((const void*)joint_reduce_kernel, dim3(rg), dim3(256), rargs, 0, st);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

}  // extern "C"
