// lt_joint.h -- device helpers of the joint weight function's matrix-core
// producer (JointWeightFn, weight_fns.py:174-227), shared by the producer
// launches (lt_producer.hip), the fused joint lattice loss (lt_joint.hip)
// and the pipelined recursions' producer helpers (lt_pipe.hip):
//   W[f, c, y] = bias[y] + sum_h Wo[y, h] * tanh(Pc[c, h] + Pf[f, h])
// on v_mfma_f32_32x32x16_bf16 with split-bf16 (or plain bf16) products and
// fp32 sums. Every consumer forms a W element through the same K steps
// (joint_tile), so the fused paths reproduce the producer's W bit for bit.
#pragma once
#include "lt_kernels.h"

namespace {

// Projections beyond this magnitude take the direct path: e^{2x} of both
// factors then stays within [e^-80, e^80], so their product is finite or
// saturates to inf / 0 (tanh = +-1) without inf * 0.
constexpr float kSplitMax = 40.f;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// two fp32 -> packed bf16 (v_cvt_pk_bf16_f32, round to nearest even)
LT_DEVINL unsigned pk_bf16(f32x2 v) {
  const bf16x2 h = {(__bf16)v.x, (__bf16)v.y};
  return __builtin_bit_cast(unsigned, h);
}

// tanh from p = e^{2x}: 1 - 2 / (1 + p) (p = inf -> 1, p = 0 -> -1)
LT_DEVINL f32x2 tanh_from_exp(f32x2 p) {
  const f32x2 one = {1.f, 1.f}, m2 = {-2.f, -2.f};
  const f32x2 d = p + one;
  const f32x2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return r * m2 + one;
}

LT_DEVINL f32x2 exp2x(f32x2 x) {  // e^{2x}
  const f32x2 k = {2.f * kLog2e, 2.f * kLog2e};
  const f32x2 y = x * k;
  return f32x2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
}

LT_DEVINL void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  u32x4 h, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2 x = {v[2 * p], v[2 * p + 1]};
    const unsigned hp = pk_bf16(x);
    const f32x2 xh = {__uint_as_float(hp << 16), __uint_as_float(hp & 0xffff0000u)};
    h[p] = hp;
    l[p] = pk_bf16(x - xh);
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

LT_DEVINL f32x16 mfma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

// One K step (16 hidden units) of a hidden tile against one or two Wo
// column tiles. tp: the lane's 8 tanh values (fp32). SP (split-bf16, the
// precision of lt_joint_weights_ex's LT_JOINT_SPLIT): tanh = hi + lo and
// Wo = hi + lo in bf16, hi*hi + hi*lo + lo*hi on the matrix cores (about 16
// mantissa bits, fp32 sums); else one bf16 product.
template <bool SP, bool TWO>
LT_DEVINL void joint_kstep(const f32x2 (&tp)[4], const unsigned short* w0, const unsigned short* w1,
                           const unsigned short* w0l, const unsigned short* w1l, f32x16& acc0,
                           f32x16& acc1) {
  if constexpr (SP) {
    const float v[8] = {tp[0].x, tp[0].y, tp[1].x, tp[1].y, tp[2].x, tp[2].y, tp[3].x, tp[3].y};
    bf16x8 ah, al;
    split8(v, ah, al);
    acc0 = mfma3(ah, al, *(const bf16x8*)w0, *(const bf16x8*)w0l, acc0);
    if (TWO) acc1 = mfma3(ah, al, *(const bf16x8*)w1, *(const bf16x8*)w1l, acc1);
  } else {
    const u32x4 t = {pk_bf16(tp[0]), pk_bf16(tp[1]), pk_bf16(tp[2]), pk_bf16(tp[3])};
    const bf16x8 af = __builtin_bit_cast(bf16x8, t);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, *(const bf16x8*)w0, acc0, 0, 0, 0);
    if (TWO) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, *(const bf16x8*)w1, acc1, 0, 0, 0);
  }
}

// Wo [R, H] fp32 -> LDS rows of HP bf16: hi, and for SP the residual lo
// (wo - hi) in a second block of R * HP (WL elements after the first)
template <bool SP>
LT_DEVINL void stage_wo(const float* wo, unsigned short* w, int R, int H, int HP, int WL, int tid,
                        int nthr) {
  for (int i = tid; i < R * H; i += nthr) {
    const int y = i / H, hh = i - y * H;
    const float v = wo[i];
    const unsigned short hi = f2bf(v);
    w[y * HP + hh] = hi;
    if (SP) w[WL + y * HP + hh] = f2bf(v - __uint_as_float((unsigned)hi << 16));
  }
}


// One 32 x 32 (TWO: 32 x 64) tile of Wo * tanh(Pc + Pf) (no bias): lane row
// r = lane & 31, K half hk = 8 (lane >> 5); pcr / pfr point at the row's
// e^{2 Pc} / e^{2 Pf} (split) or Pc / Pf (direct) plus hk; w0 / w1 (and the
// lo blocks for SP) at the Wo bf16 rows of the lane's columns plus hk. The
// K order is h = 0, 16, ... -- the producer kernels' -- so a W element comes
// out the same whichever tile it sits in.
template <bool SP, bool TWO>
LT_DEVINL void joint_tile(bool split, const float* pcr, const float* pfr, int H,
                          const unsigned short* w0, const unsigned short* w1,
                          const unsigned short* w0l, const unsigned short* w1l, f32x16& acc0,
                          f32x16& acc1) {
  if (split) {
#pragma unroll 2
    for (int k0 = 0; k0 < H; k0 += 16) {
      const float4 c0 = *(const float4*)(pcr + k0), c1 = *(const float4*)(pcr + k0 + 4);
      const float4 f0 = *(const float4*)(pfr + k0), f1 = *(const float4*)(pfr + k0 + 4);
      const f32x2 tp[4] = {tanh_from_exp(f32x2{c0.x, c0.y} * f32x2{f0.x, f0.y}),
                           tanh_from_exp(f32x2{c0.z, c0.w} * f32x2{f0.z, f0.w}),
                           tanh_from_exp(f32x2{c1.x, c1.y} * f32x2{f1.x, f1.y}),
                           tanh_from_exp(f32x2{c1.z, c1.w} * f32x2{f1.z, f1.w})};
      joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
    }
  } else {
#pragma unroll 2
    for (int k0 = 0; k0 < H; k0 += 16) {
      const float4 c0 = *(const float4*)(pcr + k0), c1 = *(const float4*)(pcr + k0 + 4);
      const float4 f0 = *(const float4*)(pfr + k0), f1 = *(const float4*)(pfr + k0 + 4);
      const f32x2 tp[4] = {tanh_from_exp(exp2x(f32x2{c0.x + f0.x, c0.y + f0.y})),
                           tanh_from_exp(exp2x(f32x2{c0.z + f0.z, c0.w + f0.w})),
                           tanh_from_exp(exp2x(f32x2{c1.x + f1.x, c1.y + f1.y})),
                           tanh_from_exp(exp2x(f32x2{c1.z + f1.z, c1.w + f1.w}))};
      joint_kstep<SP, TWO>(tp, w0 + k0, w1 + k0, w0l + k0, w1l + k0, acc0, acc1);
    }
  }
}

}  // namespace
