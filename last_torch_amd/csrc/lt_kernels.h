// lt_kernels.h -- device code shared by the kernel translation units.
// Included by lt_inst.hip (compiled once per terms-per-lane value P, so the
// template instantiations build in parallel) and by lt_lattice.hip (host
// side, C ABI, scatter / backtrace kernels).
#pragma once
// MI355X (gfx950 / CDNA4) kernels for the GNAT recognition
// lattice hot path of theadamsabra/last_torch, behind the C ABI declared in
// include/lt_lattice.h.
//
// What is computed (reference file:line in last_torch/):
//   * denominator forward  alpha_{t+1} = FrameDependent.forward(alpha_t, W_t)
//       lattices.py:379-496, alignments.py:286-297, contexts.py:207-230
//   * denominator backward beta_t + arc marginals (FrameDependent.backward)
//       lattices.py:686-799, alignments.py:300-318, contexts.py:232-256
//   * numerator (string) forward / backward
//       lattices.py:250-377, alignments.py:320-329
//   * MaxTropical Viterbi + backtrace (shortest_path)
//       lattices.py:185-247, semirings.py:354-401 (tie rules)
//
// Execution design:
//   One workgroup per utterance; the recursion over frames is serial, the
//   live front (all C context states, all U+1 string positions) is spread
//   over the workgroup:
//     waves [0, den_waves)            : denominator front, L lanes per
//                                       context state ("group"), each lane a
//                                       slice of the state's in/out arcs;
//                                       group reductions with DPP.
//     waves [den, den+aux)            : numerator front (one lane per string
//                                       position) + (backward) the coalesced
//                                       dW store of the previous frame.
//     waves [den+aux, +load)          : loaders: LDS-DMA (global_load_lds
//                                       dwordx4) of frame t+P into a ring of
//                                       S = P+1 slots while frame t computes.
//   One LDS barrier per frame. HBM is touched only by the streamed W rows,
//   the (small) alpha checkpoints and dW.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

// Timing-ablation switches: live only in diagnostic builds (make diag,
// -DLT_DIAG); in the product build every LT_ABL is the constant false and
// the compiler drops the branch.
#ifdef LT_DIAG
#define LT_ABL(args, bits) ((((args).dbg) & (bits)) != 0)
#else
#define LT_ABL(args, bits) false
#endif

#include <algorithm>
#include <string>
#include <cstdlib>

// Tuning and dispatch overrides from the environment (LT_CHUNK_LEN,
// LT_PIPE_SLOTS, ...): read only by diagnostic builds (make diag, LT_DIAG).
// The product library ignores the environment: its designs and launch
// shapes are fixed per problem, and a caller picks a design explicitly
// through lt_loss_grad_ex.
namespace lt_impl {
inline int tune_int(const char* name, int dflt) {
#ifdef LT_DIAG
  const char* s = getenv(name);
  return (s && *s) ? atoi(s) : dflt;
#else
  (void)name;
  return dflt;
#endif
}
inline const char* tune_str(const char* name) {
#ifdef LT_DIAG
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
}  // namespace lt_impl

#include "../../include/lt_lattice.h"

#define LT_DEVINL __device__ __forceinline__

namespace {

// ---------------------------------------------------------------------------
// FullNGram index maps (contexts.py:181-256)
// ---------------------------------------------------------------------------
struct NGram {
  int V;    // vocab size
  int n;    // context size (order)
  int C;    // number of states  sum_{i<=n} V^i
  int An;   // ascending states  sum_{i<n}  V^i
  int Apn;  // sum_{i<n-1} V^i   (first source row feeding full-order states)
  int Vn1;  // V^(n-1) (n >= 1), 0 for n == 0
  int K;    // lexical in-arcs per full-order destination (V+1, or V for n=0)
};

enum { M_LOG = 0, M_MAX = 1, M_REAL = 2 };

constexpr float kInf = __builtin_huge_valf();

// Destination q's lexical in-arcs, as arithmetic progressions:
//   source  p_k = a0 + k*astr,  W element  e_k = w0 + k*wstr,  k in [0, kq)
// (term order index o = 0 is the blank self loop, o = k+1 lexical arc k; the
//  reference reduces the V+1 sources in ascending p, contexts.py:226-229).
struct DestDesc {
  int kq, a0, astr, w0, wstr;
};

__host__ __device__ inline DestDesc dest_desc(const NGram& g, int q) {
  DestDesc d;
  const int R = g.V + 1;
  if (g.n == 0) {  // single state, V lexical self loops y = 1..V
    d.kq = g.V; d.a0 = 0; d.astr = 0; d.w0 = 1; d.wstr = 1;
  } else if (q == 0) {  // start state: no lexical in-arc (contexts.py:216-217)
    d.kq = 0; d.a0 = 0; d.astr = 0; d.w0 = 0; d.wstr = 0;
  } else if (q < g.An) {  // ascending: unique in-arc (contexts.py:222-225)
    const int p = (q - 1) / g.V, y = (q - 1) % g.V + 1;
    d.kq = 1; d.a0 = p; d.astr = 0; d.w0 = p * R + y; d.wstr = 0;
  } else {  // full order: V+1 sources, same label (contexts.py:226-229)
    const int jq = q - g.An;
    const int pb = g.Apn + jq / g.V, y = jq % g.V + 1;
    d.kq = g.K; d.a0 = pb; d.astr = g.Vn1; d.w0 = pb * R + y; d.wstr = g.Vn1 * R;
  }
  return d;
}

// next(p, y) = nb + y for y >= 1 (contexts.py:190-205); returns nb, and
// *zero = true for n == 0 (every lexical arc loops to state 0).
__host__ __device__ inline int next_base(const NGram& g, int p, bool* zero) {
  *zero = (g.n == 0);
  if (g.n <= 1) return 0;  // n = 1: next(p, y) = y for every p
  if (p < g.An) return p * g.V;
  return ((p - g.An) % g.Vn1) * g.V + g.An - 1;
}

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
constexpr float kLog2e = 1.4426950408889634f;
LT_DEVINL float lt_exp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }
// exp(x - c) with cl = c * log2(e) precomputed: one FMA + v_exp_f32.
LT_DEVINL float lt_exp_off(float x, float cl) { return __builtin_amdgcn_exp2f(__builtin_fmaf(x, kLog2e, -cl)); }
// Arguments are sums of exp() with the max term == 1 (>= 1) or exactly 0.
LT_DEVINL float lt_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
// log(x) for log-space recursions that take one log per frame for T frames:
// v_log_f32's error (about an ulp of log2 x, and biased) adds up over the
// frames (measured: ~1e-3 after 1,000 FrameLabelDependent(2) frames). Here
// x = 2^e m with m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(z), z = (m - 1) /
// (m + 1), |z| <= 0.1716, by five terms of its series (truncation < 1e-9);
// the result's only sizeable error is its final rounding (unbiased). Zero,
// negative, infinite and NaN arguments go through v_log_f32 (-inf, NaN, inf).
LT_DEVINL float lt_log_acc(float x) {
  if (!(x > 0.f) || x == __builtin_inff()) return lt_log(x);
  int e = __builtin_amdgcn_frexp_expf(x);
  float m = __builtin_amdgcn_frexp_mantf(x);  // [0.5, 1)
  if (m < 0.70710678f) {
    m *= 2.f;
    --e;
  }
  const float z = __builtin_amdgcn_rcpf(m + 1.f) * (m - 1.f);
  const float z2 = z * z;
  float p = 1.f / 9.f;
  p = __builtin_fmaf(p, z2, 1.f / 7.f);
  p = __builtin_fmaf(p, z2, 1.f / 5.f);
  p = __builtin_fmaf(p, z2, 1.f / 3.f);
  p = __builtin_fmaf(p, z2, 1.f);
  const float lm = 2.f * z * p;
  const float ef = (float)e;
  return __builtin_fmaf(ef, 0.693145751953125f, __builtin_fmaf(ef, 1.428606765330187e-06f, lm));
}

// Log-space values as an exact integer part plus a small fraction, (i, f):
// the value is i + f with i integer-valued (or -inf: the semiring zero) and
// f in [0, 1) after each step. The string (numerator) recursions need it:
// their positions span hundreds of nats within one frame (the positions
// ahead of the alignment's diagonal), so a value kept relative to one
// offset per frame is rounded at its own magnitude -- 2^-24 * 80 at 80 nats
// below the frame's max, every frame -- while (i, f) rounds only the
// fraction. lae_split: (ia, fa) (+) (ib, fb) = log(e^(ia+fa) + e^(ib+fb))
// (semirings.py:248-255), the result's integer part taken from the larger
// term (exact), its fraction f1 + log(1 + e^d) with d = (i2 - i1) + (f2 - f1)
// <= 0 (d's rounding reaches the result only through e^d).
LT_DEVINL void lae_split(float ia, float fa, float ib, float fb, float& io, float& fo) {
  constexpr float ninf = -__builtin_inff();
  ia = fa == ninf ? ninf : ia;  // a masked arc (w = -inf) is the zero term
  ib = fb == ninf ? ninf : ib;
  // the larger term by its whole value (the integer parts' difference is
  // exact; both zero: NaN, false -> b, masked below)
  const bool ab = (ia - ib) + (fa - fb) >= 0.f;
  const float i1 = ab ? ia : ib, f1 = ab ? fa : fb;
  const float i2 = ab ? ib : ia, f2 = ab ? fb : fa;
  const float d = (i2 - i1) + (f2 - f1);  // i2 = -inf: -inf (exp 0); both -inf: NaN (masked)
  const float r = f1 + lt_log_acc(1.f + __builtin_amdgcn_exp2f(d * kLog2e));
  const float fl = floorf(r);
  const bool zero = i1 == ninf;
  const bool fin = __builtin_isfinite(r);  // +inf / NaN weights propagate as the value
  io = zero ? i1 : (fin ? i1 + fl : r);
  fo = (zero || !fin) ? 0.f : r - fl;
}
// (i, f) of a plain log value x (finite or -inf)
LT_DEVINL void split_of(float x, float& i, float& f) {
  const bool fin = __builtin_isfinite(x);
  i = fin ? floorf(x) : x;
  f = fin ? x - floorf(x) : 0.f;
}

template <int CTRL>
LT_DEVINL float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
LT_DEVINL int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// Partner exchange for butterfly stage s of a power-of-two lane group.
// Stages 0-3 stay inside a DPP row (quad_perm / half_mirror / mirror);
// stages 4-5 go through ds_bpermute. Valid for max / sum / (max,idx) merges
// because after stage s every lane of a 2^s block holds the same value.
// Butterfly stages of a power-of-two lane group. Stages 0-3 stay inside a
// DPP row (quad_perm / row_half_mirror / row_mirror); stages 4-5 go through
// ds_bpermute. Valid for max / sum / (max,idx) merges because after stage s
// every lane of a 2^s block already holds the same value.
template <int S>
LT_DEVINL float xchg(float v) {
  if constexpr (S == 0) return dppf<0xB1>(v);
  else if constexpr (S == 1) return dppf<0x4E>(v);
  else if constexpr (S == 2) return dppf<0x141>(v);
  else if constexpr (S == 3) return dppf<0x140>(v);
  else return __shfl_xor(v, 1 << S);
}
template <int S>
LT_DEVINL int xchgi(int v) {
  if constexpr (S == 0) return dppi<0xB1>(v);
  else if constexpr (S == 1) return dppi<0x4E>(v);
  else if constexpr (S == 2) return dppi<0x141>(v);
  else if constexpr (S == 3) return dppi<0x140>(v);
  else return __shfl_xor(v, 1 << S);
}
#define LT_STAGES(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5)

// Fused butterfly stage for stages 0-3: one v_max/v_add with a DPP source
// operand (the compiler otherwise emits v_mov_dpp + canonicalize + max).
// s_nop 1 covers the VALU-write -> DPP-read hazard of the input.
#define LT_DPP_OP(NAME, OPC)                                                            \
  template <int S>                                                                      \
  LT_DEVINL float NAME(float v) {                                                       \
    float r;                                                                            \
    if constexpr (S == 0)                                                               \
      asm("s_nop 1\n\t" OPC " %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" \
          : "=v"(r) : "v"(v));                                                          \
    else if constexpr (S == 1)                                                          \
      asm("s_nop 1\n\t" OPC " %0, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" \
          : "=v"(r) : "v"(v));                                                          \
    else if constexpr (S == 2)                                                          \
      asm("s_nop 1\n\t" OPC " %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf"     \
          : "=v"(r) : "v"(v));                                                          \
    else                                                                                \
      asm("s_nop 1\n\t" OPC " %0, %1, %1 row_mirror row_mask:0xf bank_mask:0xf"          \
          : "=v"(r) : "v"(v));                                                          \
    return r;                                                                           \
  }
LT_DPP_OP(dpp_max, "v_max_f32_dpp")
LT_DPP_OP(dpp_add, "v_add_f32_dpp")
#undef LT_DPP_OP

// max / sum over lanes 8k+7 (k = 0..7) of the wave, returned wave-uniform;
// every other lane must hold the identity. row_shr:8 folds lane 7 into 15
// of each row, row_bcast:15 rows 0/2 into 1/3, row_bcast:31 rows 0-1 into
// 2-3; lane 63 ends with the total.
template <bool MAX>
LT_DEVINL float xlane_reduce(float v) {
  float r1, r2, r3;
  if constexpr (MAX) {
    asm("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf"
        : "=v"(r1) : "v"(v));
    asm("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf"
        : "=v"(r2) : "v"(r1));
    asm("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "=v"(r3) : "v"(r2));
  } else {
    asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf"
        : "=v"(r1) : "v"(v));
    asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf"
        : "=v"(r2) : "v"(r1));
    asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "=v"(r3) : "v"(r2));
  }
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r3), 63));
}

LT_DEVINL float grp_max(float v, int lg) {
#define LT_MAXST(S) if (lg > S) v = fmaxf(v, xchg<S>(v));
  LT_STAGES(LT_MAXST)
#undef LT_MAXST
  return v;
}
LT_DEVINL float grp_sum(float v, int lg) {
#define LT_SUMST(S) if (lg > S) v += xchg<S>(v);
  LT_STAGES(LT_SUMST)
#undef LT_SUMST
  return v;
}
// first-max (lowest index wins ties): semirings.py:363 (blank term has the
// lowest index) and :382 (torch.argmax returns the first maximum).
LT_DEVINL void grp_argmax(float& v, int& i, int lg) {
#define LT_ARGST(S)                                   \
  if (lg > S) {                                       \
    const float pv = xchg<S>(v);                      \
    const int pi = xchgi<S>(i);                       \
    if (pv > v || (pv == v && pi < i)) { v = pv; i = pi; } \
  }
  LT_STAGES(LT_ARGST)
#undef LT_ARGST
}

// Log-semiring plus exactly as _LogAddExp.forward (semirings.py:248-255):
// c = max(a,b), non-finite c replaced by 0.
LT_DEVINL float log_plus(float a, float b) {
  float c = fmaxf(a, b);
  if (!__builtin_isfinite(c)) c = 0.f;
  return c + lt_log(lt_exp(a - c) + lt_exp(b - c));
}

template <int MODE>
LT_DEVINL float s_zero() { return MODE == M_REAL ? 0.f : -kInf; }
template <int MODE>
LT_DEVINL float s_one() { return MODE == M_REAL ? 1.f : 0.f; }
template <int MODE>
LT_DEVINL float s_times(float a, float b) { return MODE == M_REAL ? a * b : a + b; }
template <int MODE>
LT_DEVINL float s_plus(float a, float b) {
  if (MODE == M_LOG) return log_plus(a, b);
  if (MODE == M_MAX) return (a >= b) ? a : b;  // Maximum: choose a iff a >= b
  return a + b;
}

template <bool BF16, typename I>
LT_DEVINL float ldw(const unsigned char* p, I e) {
  if constexpr (BF16) {
    return __uint_as_float(((unsigned)((const unsigned short*)p)[e]) << 16);
  } else {
    return ((const float*)p)[e];
  }
}
LT_DEVINL unsigned short f2bf(float f) {  // round to nearest even, NaN kept
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
template <bool BF16>
LT_DEVINL void stw(void* p, long long e, float v) {
  if constexpr (BF16) ((unsigned short*)p)[e] = f2bf(v);
  else ((float*)p)[e] = v;
}

#ifdef LT_STAMPS
// Diagnostic build only: block 0 records s_memtime at three points of every
// frame for every wave (lane 0): [wave][i][k], k = 0 loop top, 1 after the
// barrier, 2 end of the frame's work. Never in the shipped library.
#define LT_STAMP(a, is_stamper, role_, i_, k_)                                      \
  do {                                                                             \
    if (blockIdx.x == 0 && a.stamps && (threadIdx.x & 63) == 0)                    \
      a.stamps[((long long)(threadIdx.x >> 6) * a.T + (i_)) * 4 + (k_)] =           \
          (long long)__builtin_amdgcn_s_memtime();                                  \
  } while (0)
#else
#define LT_STAMP(a, is_stamper, role_, i_, k_) \
  do {                                          \
  } while (0)
#endif

// LDS barrier: drains this wave's LDS ops, then s_barrier. The asm has a
// memory clobber so the compiler cannot move LDS accesses across it, and it
// does NOT wait on vmcnt: loads in flight (LDS-DMA ring) and global stores
// (checkpoints) survive the barrier.
LT_DEVINL void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One LDS-DMA wave instruction: 64 lanes x 16 B from per-lane global
// addresses into the contiguous 1 KiB at LDS byte address `lds_addr`
// (wave-uniform, passed in M0). Issued from inline asm so the compiler's
// waitcnt pass does not drain it at unrelated LDS reads; the loader waits
// for it with a counted vmcnt (wait_vmcnt) before the consuming barrier.
LT_DEVINL void glds16(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// glds16 with the sc1 cache policy: the 16 bytes come from L2 (past this
// CU's L1), so data another CU published in the same launch is read fresh
// without an agent-scope acquire (buffer_inv sc1) first
LT_DEVINL void glds16_sc1(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

#define LT_VMCNT_CASE(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
LT_DEVINL void wait_vmcnt(int n) {
  switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
    LT_VMCNT_CASE(0) LT_VMCNT_CASE(1) LT_VMCNT_CASE(2) LT_VMCNT_CASE(3)
    LT_VMCNT_CASE(4) LT_VMCNT_CASE(5) LT_VMCNT_CASE(6) LT_VMCNT_CASE(7)
    LT_VMCNT_CASE(8) LT_VMCNT_CASE(9) LT_VMCNT_CASE(10) LT_VMCNT_CASE(11)
    LT_VMCNT_CASE(12) LT_VMCNT_CASE(13) LT_VMCNT_CASE(14) LT_VMCNT_CASE(15)
    LT_VMCNT_CASE(16) LT_VMCNT_CASE(17) LT_VMCNT_CASE(18) LT_VMCNT_CASE(19)
    LT_VMCNT_CASE(20) LT_VMCNT_CASE(21) LT_VMCNT_CASE(22) LT_VMCNT_CASE(23)
    LT_VMCNT_CASE(24) LT_VMCNT_CASE(25) LT_VMCNT_CASE(26) LT_VMCNT_CASE(27)
    LT_VMCNT_CASE(28) LT_VMCNT_CASE(29) LT_VMCNT_CASE(30) LT_VMCNT_CASE(31)
    LT_VMCNT_CASE(32) LT_VMCNT_CASE(33) LT_VMCNT_CASE(34) LT_VMCNT_CASE(35)
    LT_VMCNT_CASE(36) LT_VMCNT_CASE(37) LT_VMCNT_CASE(38) LT_VMCNT_CASE(39)
    LT_VMCNT_CASE(40) LT_VMCNT_CASE(41) LT_VMCNT_CASE(42) LT_VMCNT_CASE(43)
    LT_VMCNT_CASE(44) LT_VMCNT_CASE(45) LT_VMCNT_CASE(46) LT_VMCNT_CASE(47)
    LT_VMCNT_CASE(48) LT_VMCNT_CASE(49) LT_VMCNT_CASE(50) LT_VMCNT_CASE(51)
    LT_VMCNT_CASE(52) LT_VMCNT_CASE(53) LT_VMCNT_CASE(54) LT_VMCNT_CASE(55)
    LT_VMCNT_CASE(56) LT_VMCNT_CASE(57) LT_VMCNT_CASE(58) LT_VMCNT_CASE(59)
    LT_VMCNT_CASE(60) LT_VMCNT_CASE(61) LT_VMCNT_CASE(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}

// ---------------------------------------------------------------------------
// Kernel arguments (passed by value)
// ---------------------------------------------------------------------------
constexpr int kMaxStreams = 3;
enum { F_DEN = 1, F_NUM = 2, F_LOCAL = 4, F_LOSS = 8 };

struct KArgs {
  const unsigned char* W;
  const int* nfr;
  const int* labels;
  const int* nlab;
  const float* grad;
  const float* log_z_in;
  const float* num_in;
  float* dist;       // den result (log_z / path weight)
  float* alpha;      // [B,T,C] den alpha history
  float* num;        // [B]
  float* alpha_num;  // [B,T,U+1]
  float* loss;       // [B]
  unsigned char* bp; // [B,T,C] Viterbi backpointers
  int* qstar;        // [B] Viterbi final state
  void* dW;          // [B,T,C,V+1]
  float* nm_side;    // [B,T,U+1,2] numerator marginals (direct path)
  int* ctx_side;     // [B,U+1,2]    numerator arc rows (direct path)
  float* beta;       // [B,T,C]   den beta_{t+1} per frame t (checkpointing backward)
  float* beta_num;   // [B,T,U+1] num beta_{t+1} per frame t
  int* arcs;         // [B,4(U+1)] numerator arc table (forward writes, marginal pass reads)
  int B, T, U, flags;
  const int* only;   // nullable: only utterances with only[b] != 0 run (the chunked
                     // path's fallback, lt_chunk.hip); the others return at once
  long long* stamps; // diagnostic build (-DLT_STAMPS) only: per-step clocks
  int dbg;           // ablation bitmask (LT_DBG, timing experiments only): 1 skip den
                     // compute, 2 skip numerator, 4 loaders issue nothing, 8 no barrier
  NGram g;
  int FR;            // C*(V+1) elements per frame
  int den_groups;    // denominator groups (forward: destinations, backward: sources)
  int den_q0;        // state of group 0 (forward n >= 1: 1, the start state is extra0)
  int extra0;        // forward n >= 1: den lane 0 also does the start state (blank only)
  int den_fast;      // every den lane owns at most one group (slices precomputed)
  int den_xg;        // backward: last source state reduced by wave 0's spare lanes
  int Pr;            // terms per lane (block size of the lane slice, <= template P)
  // layout
  int L, lgL, den_waves, aux_waves, load_waves;
  int S, P, slot_bytes;
  // staged streams, fixed slots: 0 = W rows, 1 = alpha rows, 2 = alpha_num
  // rows; st_ninstr[s] == 0 means stream s is not staged. Only indexed with
  // compile-time constants (runtime-indexed kernel-argument arrays would be
  // copied to scratch).
  const unsigned char* st_base[kMaxStreams];
  long long st_row[kMaxStreams];   // bytes per frame row
  int st_ninstr[kMaxStreams];      // LDS-DMA wave instructions per frame
  int st_off[kMaxStreams];         // byte offset inside a slot
  int gw0, gw1;                    // instructions per frame of loader wave 0 / 1
  int off_ring, off_a, off_na, off_ctx, off_ylab, off_dbuf, off_nbuf, off_misc;
  int off_tb;        // trigram V = 32 backward: the padded beta rows [2][kTriBPad]
  // the trigram overlap (lt_tri.hip, tri_mix_kernel): nullable; [2B] frames
  // whose checkpoint rows are final, published every kTriPub frames (forward:
  // rows [0, p); backward: rows [nf - 1 - p, nf))
  unsigned* prog;
};

// The kernel arguments re-read from the kernarg segment through a pointer
// the compiler cannot see through: each role loop then loads only the
// fields it uses (scalar loads at the use), instead of the whole KArgs being
// hoisted to the kernel entry and kept live (SGPR spills) across all roles.
// KOFF: the byte offset of this role's KArgs among the kernel's arguments
// (fwdbwd_kernel's second KArgs sits at sizeof(KArgs)).
template <int KOFF = 0>
LT_DEVINL const KArgs& fresh_args() {
  typedef const __attribute__((address_space(4))) KArgs* KP;
  KP p = (KP)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
              KOFF);
  asm volatile("" : "+s"(p));
  return *(const KArgs*)p;
}

LT_DEVINL unsigned lds_base_addr(unsigned char* lds) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
}

// Issue loader wave `lw`'s LDS-DMA instructions for frame t into `slot`.
// The frame's instructions are numbered across the streams in slot order
// (stream 0 first); wave lw issues numbers lw, lw + load_waves, ...
// Streams are visited with compile-time indices so every parameter stays in
// SGPRs (a runtime-indexed kernel argument becomes a vector load whose
// vmcnt wait would drain the DMA ring).
template <int S>
LT_DEVINL void issue_stream(const KArgs& a, long long bt, unsigned sbase, int first, int lw,
                            int lane) {
  const int ni = a.st_ninstr[S];
  if (ni == 0) return;
  const long long row = a.st_row[S];
  const long long off = bt * row;
  const long long g1 = (off + row + 15) >> 4;
  const unsigned char* base = a.st_base[S];
  const unsigned dst = sbase + a.st_off[S];
  // first k with (first + k) % load_waves == lw
  int k = lw - first % a.load_waves;
  if (k < 0) k += a.load_waves;
  for (; k < ni; k += a.load_waves) {
    long long gg = (off >> 4) + (long long)k * 64 + lane;
    if (gg > g1 - 1) gg = g1 - 1;  // in-bounds duplicate, lands past the row
    glds16(base + gg * 16, dst + k * 1024);
  }
}
LT_DEVINL void issue_frame(const KArgs& a, int b, int t, int slot, int lw, int lane,
                           unsigned ldsb) {
  const unsigned sbase = ldsb + a.off_ring + slot * a.slot_bytes;
  const long long bt = (long long)b * a.T + t;
  issue_stream<0>(a, bt, sbase, 0, lw, lane);
  issue_stream<1>(a, bt, sbase, a.st_ninstr[0], lw, lane);
  issue_stream<2>(a, bt, sbase, a.st_ninstr[0] + a.st_ninstr[1], lw, lane);
}

// Address (in LDS) of stream S's row for frame t held in `slot`.
template <int S>
LT_DEVINL const unsigned char* slot_row(unsigned char* lds, const KArgs& a, int b, int t,
                                        int slot) {
  const long long off = ((long long)b * a.T + t) * a.st_row[S];
  return lds + a.off_ring + slot * a.slot_bytes + a.st_off[S] + (int)(off & 15);
}

// Walk the context DFA along the label string (contexts.py:109-146) and the
// numerator gather indices (lattices.py:314-338): ctx[u] = c_u*(V+1),
// ylab[u] = safe class of labels[u] (0 -> 1, lattices.py:314-315), u < U.
// Phase 1 (all aux lanes): labels -> ylab (raw). Phase 2 (one lane, after a
// barrier): the serial walk over LDS.
LT_DEVINL void load_labels(const KArgs& a, int b, int* ylab, int al, int aux_lanes) {
  for (int u = al; u < a.U; u += aux_lanes) ylab[u] = a.labels[(long long)b * a.U + u];
}
LT_DEVINL void walk_states(const KArgs& a, int* ctx, int* ylab) {
  const NGram& g = a.g;
  const int R = g.V + 1;
  int c = 0;
  for (int u = 0; u <= a.U; ++u) {
    ctx[u] = c * R;
    if (u < a.U) {
      int y = ylab[u];
      if (y < 0 || y > g.V) y = 0;
      ylab[u] = y < 1 ? 1 : y;
      if (y != 0) {
        bool z;
        const int nb = next_base(g, c, &z);
        c = z ? 0 : nb + y;
      }
    } else {
      ylab[u] = 1;
    }
  }
}

// Numerator arc table of utterance b for the marginal pass: entry k = 2u is
// position u's blank arc (frame element c_u*(V+1)), k = 2u+1 its lexical arc
// c_u*(V+1) + y_{u+1} (u < U; -1 for u = U). link[k] = head << 30 | (next+1):
// entries sharing an element form a chain in ascending k whose head (lowest
// k) sums it, so the subtraction order is fixed (deterministic dW).
LT_DEVINL void write_arc_table(const KArgs& a, int b, const int* ctx, const int* ylab, int tid,
                               int nthr) {
  const int NP = a.U + 1, NK = 2 * NP;
  int* off = a.arcs + (long long)b * 2 * NK;
  int* link = off + NK;
  auto arc = [&](int k) {
    const int u = k >> 1;
    return (k & 1) == 0 ? ctx[u] : (u < a.U ? ctx[u] + ylab[u] : -1);
  };
  for (int k = tid; k < NK; k += nthr) {
    const int o = arc(k);
    int head = o >= 0 ? 1 : 0, nxt = -1;
    if (o >= 0) {
      for (int k2 = 0; k2 < NK; ++k2) {
        if (arc(k2) != o) continue;
        if (k2 < k) head = 0;
        else if (k2 > k && nxt < 0) nxt = k2;
      }
    }
    off[k] = o;
    link[k] = (head << 30) | (nxt + 1);
  }
}

// Lane slice of a forward group (destination q): term order index
// o in [j*P, j*P+P) of {blank, lexical k = o-1}; aoff = alpha index,
// woff = W element of the frame. Returns the count of valid terms.
template <int P>
LT_DEVINL int fwd_slice(const NGram& g, int q, int j, int Pr, int* aoff, int* woff) {
  const DestDesc d = dest_desc(g, q);
  const int nterm = d.kq + 1, R = g.V + 1;
  int nv = 0;
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int o = j * Pr + m;
    int ai = 0, wi = 0;
    if (m < Pr && o < nterm) {
      if (o == 0) { ai = q; wi = q * R; }
      else { const int k = o - 1; ai = d.a0 + k * d.astr; wi = d.w0 + k * d.wstr; }
      nv = m + 1;
    }
    aoff[m] = ai;
    woff[m] = wi;
  }
  return nv;
}

// Lane slice of a backward group (source p): labels y in [j*P, j*P+P);
// woff = W element p*(V+1)+y, boff = beta index of next(p, y).
template <int P>
LT_DEVINL int bwd_slice(const NGram& g, int p, int j, int Pr, int* woff, int* boff) {
  bool zero;
  const int nb = next_base(g, p, &zero);
  const int R = g.V + 1;
  int nv = 0;
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int y = j * Pr + m;
    int wi = 0, bi = 0;
    if (m < Pr && y <= g.V) {
      wi = p * R + y;
      bi = (y == 0) ? p : (zero ? 0 : nb + y);
      nv = m + 1;
    }
    woff[m] = wi;
    boff[m] = bi;
  }
  return nv;
}

// Group reductions with a compile-time group size 2^LG (LG < 0: runtime lg).
template <int LG>
LT_DEVINL float gmax(float v, int lg) {
  if constexpr (LG < 0) {
    return grp_max(v, lg);
  } else {
    if constexpr (LG > 0) v = dpp_max<0>(v);
    if constexpr (LG > 1) v = dpp_max<1>(v);
    if constexpr (LG > 2) v = dpp_max<2>(v);
    if constexpr (LG > 3) v = dpp_max<3>(v);
    if constexpr (LG > 4) v = fmaxf(v, xchg<4>(v));
    if constexpr (LG > 5) v = fmaxf(v, xchg<5>(v));
    return v;
  }
}
template <int LG>
LT_DEVINL float gsum(float v, int lg) {
  if constexpr (LG < 0) {
    return grp_sum(v, lg);
  } else {
    if constexpr (LG > 0) v = dpp_add<0>(v);
    if constexpr (LG > 1) v = dpp_add<1>(v);
    if constexpr (LG > 2) v = dpp_add<2>(v);
    if constexpr (LG > 3) v = dpp_add<3>(v);
    if constexpr (LG > 4) v += xchg<4>(v);
    if constexpr (LG > 5) v += xchg<5>(v);
    return v;
  }
}
template <int S>
LT_DEVINL void argmax_stage(float& v, int& i) {
  const float pv = xchg<S>(v);
  const int pi = xchgi<S>(i);
  if (pv > v || (pv == v && pi < i)) { v = pv; i = pi; }
}
template <int LG>
LT_DEVINL void gargmax(float& v, int& i, int lg) {
  if constexpr (LG < 0) {
    grp_argmax(v, i, lg);
  } else {
    if constexpr (LG > 0) argmax_stage<0>(v, i);
    if constexpr (LG > 1) argmax_stage<1>(v, i);
    if constexpr (LG > 2) argmax_stage<2>(v, i);
    if constexpr (LG > 3) argmax_stage<3>(v, i);
    if constexpr (LG > 4) argmax_stage<4>(v, i);
    if constexpr (LG > 5) argmax_stage<5>(v, i);
  }
}

// Balanced reductions over a lane's register slice (short dependency chains).
template <int P>
LT_DEVINL float tree_max(const float* x) {
  float t[P];
#pragma unroll
  for (int m = 0; m < P; ++m) t[m] = x[m];
#pragma unroll
  for (int w = 1; w < P; w *= 2)
#pragma unroll
    for (int m = 0; m + w < P; m += 2 * w) t[m] = fmaxf(t[m], t[m + w]);
  return t[0];
}
template <int P>
LT_DEVINL float tree_sum(const float* x) {
  float t[P];
#pragma unroll
  for (int m = 0; m < P; ++m) t[m] = x[m];
#pragma unroll
  for (int w = 1; w < P; w *= 2)
#pragma unroll
    for (int m = 0; m + w < P; m += 2 * w) t[m] = t[m] + t[m + w];
  return t[0];
}

// Semiring reduction of a group's terms (x[m] for m >= nv already = zero).
// Log follows _LogSumExp.forward (semirings.py:279-286); Max returns the
// first maximum's term order index in *bi (semirings.py:363, :382).
template <int MODE, int LG, int P>
LT_DEVINL float group_reduce(const float* x, int lgL, int o0, int* bi) {
  if constexpr (MODE == M_LOG) {
    float mx = gmax<LG>(tree_max<P>(x), lgL);
    const float c = __builtin_isfinite(mx) ? mx : 0.f;
    const float cl = c * kLog2e;
    float e[P];
#pragma unroll
    for (int m = 0; m < P; ++m) e[m] = lt_exp_off(x[m], cl);
    const float s = gsum<LG>(tree_sum<P>(e), lgL);
    return c + lt_log(s);
  } else if constexpr (MODE == M_MAX) {
    float r = x[0];
    int i = o0;
#pragma unroll
    for (int m = 1; m < P; ++m)
      if (x[m] > r) { r = x[m]; i = o0 + m; }
    gargmax<LG>(r, i, lgL);
    *bi = i;
    return r;
  } else {
    return gsum<LG>(tree_sum<P>(x), lgL);
  }
}

// Per-role frame loops. Every role runs exactly nf iterations with one LDS
// barrier each (the only cross-wave synchronisation); each loop carries only
// its own loop state, and frame addresses advance incrementally.
LT_DEVINL void idle_loop(int nf) {
  for (int i = 0; i < nf; ++i) lds_barrier();
}

// Loader: frame f(i) = reverse ? nf-1-i : i goes to slot i % S; at step i
// frame f(i+P) is issued after the barrier and frame f(i+1) is waited for
// before the next one (counted vmcnt).
LT_DEVINL void loader_loop(const KArgs& a, int b, int nf, bool reverse, int lw, int lane,
                           unsigned ldsb, int ahead = 0) {
  const int gw = lw == 0 ? a.gw0 : a.gw1;
  int slot = 0;
  [[maybe_unused]] const bool st = lw == 0 && lane == 0;
  for (int i = 0; i < nf; ++i) {
    LT_STAMP(a, st, 2, i, 0);
    if (!LT_ABL(a, 4)) {
      // frame i + ahead must have landed by this barrier
      int later = (a.P - 1 < nf - 1 - i) ? a.P - 1 : nf - 1 - i;
      later -= ahead;
      wait_vmcnt(later < 0 ? 0 : later * gw);
    }
    lds_barrier();
    LT_STAMP(a, st, 2, i, 1);
    if (i + a.P < nf && !LT_ABL(a, 4)) {
      const int s2 = slot + a.P >= a.S ? slot + a.P - a.S : slot + a.P;
      const int f = reverse ? nf - 1 - (i + a.P) : i + a.P;
      issue_frame(a, b, f, s2, lw, lane, ldsb);
    }
    slot = (slot + 1 == a.S) ? 0 : slot + 1;
    LT_STAMP(a, st, 2, i, 2);
  }
}

// Cursor over the rows of one stream for successive frames: LDS address of
// the staged row (ring slot + 16-B misalignment) and the global row.
struct Cursor {
  int soff;        // slot * slot_bytes
  int mis;         // global byte offset & 15
  int dmis;        // row bytes & 15, signed step
  long long goff;  // global byte offset of the row
  long long step;  // +-row bytes
};
LT_DEVINL Cursor make_cursor(long long row, long long first_row_index, bool reverse) {
  Cursor c;
  c.soff = 0;
  c.goff = first_row_index * row;
  c.mis = (int)(c.goff & 15);
  c.dmis = (int)(row & 15);
  if (reverse) c.dmis = -c.dmis;
  c.step = reverse ? -row : row;
  return c;
}
LT_DEVINL void advance(Cursor& c, const KArgs& a) {
  c.soff += a.slot_bytes;
  if (c.soff == a.S * a.slot_bytes) c.soff = 0;
  c.mis = (c.mis + c.dmis) & 15;
  c.goff += c.step;
}

// Log numerator offsets: the recursion holds the string vector relative to
// an integer offset O near its max (exact), so its roundings stay 2^-24 of
// small numbers however long the utterance; history rows and num are O +
// value, rounded once. The offset every lane subtracts at step k is the
// floor of the max of the vector step k-1 read, taken by the first aux wave
// into an LDS ping-pong slot (misc + kNumSub) between two barriers.
constexpr int kNumSub = 8;
LT_DEVINL float num_sub_take(const KArgs& a, unsigned char* lds, const float* vec, int NP, int al,
                             int k) {
  float* sub = (float*)(lds + a.off_misc) + kNumSub;
  const float sp = sub[(k + 1) & 1];  // written at step k - 1
  if (al < 64) {                      // the first aux wave: this step's input max
    float m = -kInf;
    for (int u = al; u < NP; u += 64) m = fmaxf(m, vec[u]);
    m = gmax<6>(m, 6);
    if (al == 0) sub[k & 1] = floorf(__builtin_isfinite(m) ? m : 0.f);
  }
  return sp;
}
LT_DEVINL void num_sub_init(const KArgs& a, unsigned char* lds, int al) {
  if (al == 0) {
    float* sub = (float*)(lds + a.off_misc) + kNumSub;
    sub[0] = 0.f;
    sub[1] = 0.f;
  }
}

// The denominator's Log vector the same way: its offset slots at misc +
// kDenSub, the max taken by the first den wave over the C states.
constexpr int kDenSub = 12;
LT_DEVINL float den_sub_take(const KArgs& a, unsigned char* lds, const float* vec, int C, int tid,
                             int k) {
  float* sub = (float*)(lds + a.off_misc) + kDenSub;
  const float sp = sub[(k + 1) & 1];
  if (tid < 64) {
    float m = -kInf;
    for (int q = tid; q < C; q += 64) m = fmaxf(m, vec[q]);
    m = gmax<6>(m, 6);
    if (tid == 0) sub[k & 1] = floorf(__builtin_isfinite(m) ? m : 0.f);
  }
  return sp;
}
LT_DEVINL void den_sub_init(const KArgs& a, unsigned char* lds, int tid) {
  if (tid == 0) {
    float* sub = (float*)(lds + a.off_misc) + kDenSub;
    sub[0] = 0.f;
    sub[1] = 0.f;
  }
}

// ---------------------------------------------------------------------------
// Forward kernel: denominator and/or numerator, Log / MaxTropical / Real.
// ---------------------------------------------------------------------------
template <int MODE, bool BF16, bool WST, int LG, int P>
LT_DEVINL float den_fwd_loop(const KArgs& a, unsigned char* lds, float* abuf, int b, int nf,
                             int tid) {
  const NGram& g = a.g;
  const int C = g.C;
  const int lgL = LG >= 0 ? LG : a.lgL;
  const int L = 1 << lgL;
  const int j = tid & (L - 1);
  const int grp = tid >> lgL;
  const int ngrp = (a.den_waves * 64) >> lgL;
  const bool fast = a.den_fast;
  const bool has = grp < a.den_groups;
  int aoff[P], woff[P];
  int nv = 0;
  const int q = a.den_q0 + grp;
  if (fast && has) nv = fwd_slice<P>(g, q, j, a.Pr, aoff, woff);
  const unsigned char* ring = lds + a.off_ring + a.st_off[0];
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * (BF16 ? 2 : 4),
                          (long long)b * a.T, false);
  float* hist = a.alpha ? a.alpha + (long long)b * a.T * C : nullptr;
  unsigned char* bpp = a.bp ? a.bp + (long long)b * a.T * C : nullptr;
  // Log: alpha relative to an integer offset O near its max (den_sub_take),
  // history rows O + value; MaxTropical / Real: exact values, no offset
  float O = 0.f, sp = 0.f;
  // one destination group: terms -> semiring sum -> alpha_{t+1}[q]
  auto group = [&](int qq, const int* ao, const int* wo, int n2, const unsigned char* wrow,
                   const float* acur, float* anxt) {
    float x[P];
    float aself = 0.f;
#pragma unroll
    for (int m = 0; m < P; ++m) {
      const float av = acur[ao[m]];
      const float wv = ldw<BF16>(wrow, wo[m]);
      if (m == 0) aself = av;
      x[m] = m < n2 ? s_times<MODE>(av, wv) : s_zero<MODE>();
    }
    int bi = 0;
    const float r = group_reduce<MODE, LG, P>(x, lgL, j * a.Pr, &bi);
    if (j == 0) {
      anxt[qq] = MODE == M_LOG ? r - sp : r;
      if (hist) hist[qq] = MODE == M_LOG ? O + aself : aself;
      if (MODE == M_MAX && bpp) bpp[qq] = (unsigned char)bi;
    }
  };
  auto start_state = [&](const unsigned char* wrow, const float* acur, float* anxt) {
    if (a.extra0 && tid == 0) {  // blank self loop only
      const float av = acur[0];
      const float r = s_times<MODE>(av, ldw<BF16>(wrow, 0));
      anxt[0] = MODE == M_LOG ? r - sp : r;
      if (hist) hist[0] = MODE == M_LOG ? O + av : av;
      if (MODE == M_MAX && bpp) bpp[0] = 0;
    }
  };
  auto take = [&](int i, const float* acur) {
    if constexpr (MODE == M_LOG) sp = den_sub_take(a, lds, acur, C, tid, i);
  };
  if (fast) {
    for (int i = 0; i < nf; ++i) {
      LT_STAMP(a, tid == 0, 0, i, 0);
      lds_barrier();
      LT_STAMP(a, tid == 0, 0, i, 1);
      const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
      const float* acur = abuf + (i & 1) * C;
      float* anxt = abuf + ((i + 1) & 1) * C;
      take(i, acur);
      if (has) group(q, aoff, woff, nv, wrow, acur, anxt);
      start_state(wrow, acur, anxt);
      O += sp;
      advance(cw, a);
      if (hist) hist += C;
      if (bpp) bpp += C;
      LT_STAMP(a, tid == 0, 0, i, 2);
    }
  } else {
    const int R = g.V + 1;
    const bool fstep = g.n >= 1 && ngrp % g.V == 0;
    const int fda = fstep ? ngrp / g.V : 0;
    for (int i = 0; i < nf; ++i) {
      lds_barrier();
      const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
      const float* acur = abuf + (i & 1) * C;
      float* anxt = abuf + ((i + 1) & 1) * C;
      take(i, acur);
      // a lane's slice advances by a constant from one pass to the next once
      // its destination is a full-order state and ngrp is a multiple of V
      // (the source base moves by ngrp / V, the label stays): no per-pass
      // index math (trigram: 5.5 passes a frame)
      int ao[P], wo[P], n2 = 0, qprev = -1;
      for (int qq = a.den_q0 + grp; qq < C; qq += ngrp) {
        if (fstep && qprev >= g.An) {
#pragma unroll
          for (int m = 0; m < P; ++m) {
            const bool blank = m == 0 && j == 0;
            ao[m] += m < n2 ? (blank ? ngrp : fda) : 0;
            wo[m] += m < n2 ? (blank ? ngrp * R : fda * R) : 0;
          }
        } else {
          n2 = fwd_slice<P>(g, qq, j, a.Pr, ao, wo);
        }
        qprev = qq;
        group(qq, ao, wo, n2, wrow, acur, anxt);
      }
      start_state(wrow, acur, anxt);
      O += sp;
      advance(cw, a);
      if (hist) hist += C;
      if (bpp) bpp += C;
    }
  }
  return O;
}

// ---------------------------------------------------------------------------
// Trigram den recursions (FullNGram n = 2, V <= 32, Log; lt_tri.hip).
// The full-order destinations come in V blocks of V (contexts.py:226-229):
// block j holds the states (j+1, y), y = 1..V, whose V+1 sources are
// p_k = 1 + j + k V (the order-1 state j+1, then the order-2 states
// (x, j+1)), and their lexical arcs are the label runs W[p_k, 1..V]. A den
// lane owns the two destinations y and y+16 of one block and reduces all
// 2 x (V+2) of their terms in registers: no lane groups, no cross-lane sums,
// one pass per frame. alpha[p_k] is one address per block (four blocks a
// wave: four banks), the W reads are 16 consecutive labels per block.
// The backward lane owns two source rows p and p + 576. At V = 32
// (den_bwd_tri32) the beta rows are padded to blocks 33 floats apart and the
// labels walked in natural order from immediate offsets; at runtime V the
// lane walks its labels from a lane-dependent start. Either way 32
// consecutive sources read 32 different banks both in W (rows 66 B apart)
// and in beta (next(p, y) = nb(p) + y, one block of V per source).
// Log vectors stay relative to an integer offset: the max of the vector a
// step writes goes through an LDS slot (ds_max on an order-preserving int
// image, three slots in rotation) to the next step, which subtracts its
// floor (the same rounding scheme as den_sub_take, without a serial pass).
// ---------------------------------------------------------------------------
// 16-byte units of W / dW (marg_kernel, the trigram overlap's marginal role)
template <bool BF16>
LT_DEVINL void unpack_unit(const uint4 q, float* w) {
  if constexpr (BF16) {
    const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[2 * i] = __uint_as_float(u[i] << 16);
      w[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  } else {
    w[0] = __uint_as_float(q.x); w[1] = __uint_as_float(q.y);
    w[2] = __uint_as_float(q.z); w[3] = __uint_as_float(q.w);
  }
}
template <bool BF16>
LT_DEVINL void store_unit(unsigned char* p, const float* v) {
  uint4 q;
  if constexpr (BF16) {
    q.x = f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    q.y = f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    q.z = f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
    q.w = f2bf(v[6]) | ((unsigned)f2bf(v[7]) << 16);
  } else {
    q.x = __float_as_uint(v[0]); q.y = __float_as_uint(v[1]);
    q.z = __float_as_uint(v[2]); q.w = __float_as_uint(v[3]);
  }
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u qv = {q.x, q.y, q.z, q.w};
  __builtin_nontemporal_store(qv, (v4u*)p);  // dW is written once: one 16-byte store
}


// The trigram overlap's progress words (KArgs::prog, tri_mix_kernel): every
// kTriPub frames the waves that store checkpoint rows (den and numerator
// roles) drain their stores before the frame's barrier, and thread 0
// publishes the count after it (an sc1 store; the marginal workgroups on the
// same XCD poll it with sc1 loads and read the rows with sc1 loads)
#ifndef LT_TRI_PUB
#define LT_TRI_PUB 16  // (64: 3.28-3.29 ms at cfg5, 16: 3.25-3.26, 8: 3.36-3.39; profiles/r06_tri_pub_ab.txt)
#endif
constexpr int kTriPub = LT_TRI_PUB;
LT_DEVINL bool tri_pub_frame(const KArgs& a, int i) { return a.prog && i > 0 && i % kTriPub == 0; }
LT_DEVINL void tri_pub_drain(const KArgs& a, int i) {
  if (tri_pub_frame(a, i)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
LT_DEVINL void tri_pub_store(const KArgs& a, int b, int dir, unsigned v) {
  if (a.prog && threadIdx.x == 0)
    __hip_atomic_store(a.prog + 2 * b + dir, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kTriDenWaves = 9;
#ifndef LT_TRI_LOAD
#define LT_TRI_LOAD 4
#endif
constexpr int kTriLoadWaves = LT_TRI_LOAD;  // loader waves of the trigram launch
LT_DEVINL int tri_enc(float f) {  // order-preserving int image of a float
  const int i = __float_as_int(f);
  return i ^ ((i >> 31) & 0x7fffffff);
}
LT_DEVINL float tri_dec(int i) { return __int_as_float(i ^ ((i >> 31) & 0x7fffffff)); }

// the wave's max into the step's slot (lane 0, LDS atomic)
LT_DEVINL void tri_publish_max(int* slot, float v) {
  v = gmax<6>(v, 6);  // butterfly: every lane holds the wave's max
  if ((threadIdx.x & 63) == 0) atomicMax(slot, tri_enc(v));
}

// VT: V as a compile-time constant (32: every address an immediate offset
// from one lane base, no per-term address registers), 0 = runtime V
template <bool BF16, bool WST, int VT>
LT_DEVINL float den_fwd_tri(const KArgs& a, unsigned char* lds, float* abuf, int b, int nf,
                            int tid) {
  const NGram& g = a.g;
  const int V = VT > 0 ? VT : g.V, R = V + 1;
  const int C = VT > 0 ? 1 + VT + VT * VT : g.C;
  int* slot = (int*)(lds + a.off_misc) + 2;
  const int blk = tid >> 4, yl = tid & 15;
  const int y0 = yl + 1, y1 = yl + 17;
  const bool pairs = tid < 16 * V && y0 <= V;
  const bool v1 = y1 <= V;
  const int pb = 1 + blk;  // Apn = 1, An = V + 1 for n = 2
  const int qa = V + 1 + blk * V + y0 - 1, qb = qa + 16;
  const int lo = tid - 16 * V;  // low-order destination (start state, order-1 states)
  const bool low = lo >= 0 && lo <= V;
  if (tid == 0) {
    slot[0] = tri_enc(0.f);  // max of alpha_0
    slot[1] = tri_enc(-kInf);
    slot[2] = tri_enc(-kInf);
  }
  const unsigned char* ring = lds + a.off_ring + a.st_off[0];
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * (BF16 ? 2 : 4),
                          (long long)b * a.T, false);
  float* hist = a.alpha ? a.alpha + (long long)b * a.T * C : nullptr;
  float O = 0.f;
  for (int i = 0; i < nf; ++i) {
    tri_pub_drain(a, i);
    lds_barrier();
    if (tri_pub_frame(a, i)) tri_pub_store(a, b, 0, (unsigned)i);
    const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
    const float* acur = abuf + (i & 1) * C;
    float* anxt = abuf + ((i + 1) & 1) * C;
    const int s3 = i % 3;
    const float mprev = tri_dec(slot[s3]);
    const float sp = __builtin_isfinite(mprev) ? floorf(mprev) : 0.f;
    if (tid == 0) slot[s3 == 0 ? 2 : s3 - 1] = tri_enc(-kInf);  // slot of step i + 2
    float lmax = -kInf;
    if (pairs) {
      // the lane's two destinations one after the other (33 terms in
      // registers at a time: no spills at four waves per SIMD)
#pragma unroll 1
      for (int d = 0; d < 2; ++d) {
        const int q = d ? qb : qa, y = d ? y1 : y0;
        if (d && !v1) break;
        float x[33];
        const float aq = acur[q];
        if (hist) hist[q] = O + aq;
        const float tq = aq + ldw<BF16>(wrow, q * R);  // blank self loop
        float m = tq;
#pragma unroll
        for (int k = 0; k < 33; ++k) {
          if (k <= V) {
            const int p = pb + k * V;
            x[k] = acur[p] + ldw<BF16>(wrow, p * R + y);
          } else {
            x[k] = -kInf;
          }
          m = fmaxf(m, x[k]);
        }
        // one logsumexp over blank + lexical terms with the safe max
        // (semirings.py:248-255, 279-286)
        const float c = __builtin_isfinite(m) ? m : 0.f;
        const float l = c * kLog2e;
        float s = lt_exp_off(tq, l);
#pragma unroll
        for (int k = 0; k < 33; ++k) s += lt_exp_off(x[k], l);
        const float r = (c + lt_log(s)) - sp;
        anxt[q] = r;
        lmax = fmaxf(lmax, r);
      }
    } else if (low) {
      const int q = lo;
      const float aq = acur[q];
      if (hist) hist[q] = O + aq;
      const float tb = aq + ldw<BF16>(wrow, q * R);  // blank self loop
      float r;
      if (q == 0) {
        r = tb;  // the start state has no lexical in-arc (contexts.py:216-217)
      } else {
        const float tl = acur[0] + ldw<BF16>(wrow, q);  // from state 0, label q
        r = log_plus(tb, tl);
      }
      r -= sp;
      anxt[q] = r;
      lmax = r;
    }
    tri_publish_max(slot + (s3 == 2 ? 0 : s3 + 1), lmax);
    O += sp;
    advance(cw, a);
    if (hist) hist += C;
  }
  return O;
}

template <int MODE, bool BF16, bool WST>
LT_DEVINL float num_fwd_loop(const KArgs& a, unsigned char* lds, float* nbuf, const int* ctx,
                             const int* ylab, int b, int nf, int al, int aux_lanes) {
  const int NP = a.U + 1;
  int ob = 0, olm = 0;
  if (al < NP) {
    ob = ctx[al];
    if (al >= 1) olm = ctx[al - 1] + ylab[al - 1];
  }
  const unsigned char* ring = lds + a.off_ring + a.st_off[0];
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * (BF16 ? 2 : 4),
                          (long long)b * a.T, false);
  float* hist = a.alpha_num ? a.alpha_num + (long long)b * a.T * NP : nullptr;
  float O = 0.f;  // Log: the vector's integer offset (MaxTropical / Real: 0, exact values)
  for (int i = 0; i < nf; ++i) {
    LT_STAMP(a, al == 0, 1, i, 0);
    tri_pub_drain(a, i);
    lds_barrier();
    LT_STAMP(a, al == 0, 1, i, 1);
    const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
    const float* ncur = nbuf + (i & 1) * NP;
    float* nnxt = nbuf + ((i + 1) & 1) * NP;
    const float sp = MODE == M_LOG ? num_sub_take(a, lds, ncur, NP, al, i) : 0.f;
    for (int u = al; u < NP; u += aux_lanes) {
      int o0 = ob, o2 = olm;
      if (u != al) { o0 = ctx[u]; o2 = ctx[u - 1] + ylab[u - 1]; }
      const float cu = ncur[u];
      const float xb = s_times<MODE>(cu, ldw<BF16>(wrow, o0));
      float xl = s_zero<MODE>();
      if (u >= 1) xl = s_times<MODE>(ncur[u - 1], ldw<BF16>(wrow, o2));
      if (hist) hist[u] = MODE == M_LOG ? O + cu : cu;
      nnxt[u] = MODE == M_LOG ? s_plus<MODE>(xb, xl) - sp : s_plus<MODE>(xb, xl);
    }
    O += sp;
    advance(cw, a);
    if (hist) hist += NP;
    LT_STAMP(a, al == 0, 1, i, 2);
  }
  return O;
}

// DEN > 0: the den role runs den_fwd_tri (trigram, lt_tri.hip; DEN = 32: V = 32, 1: any V)
template <int MODE, bool BF16, bool WST, int LG, int P, int DEN = 0>
LT_DEVINL void fwd_body(const KArgs& a, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const NGram& g = a.g;
  const int C = g.C, NP = a.U + 1;
  const bool do_den = a.flags & F_DEN, do_num = a.flags & F_NUM;
  if (a.only && !a.only[b]) return;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);

  float* abuf = (float*)(lds + a.off_a);    // [2][C]
  float* nbuf = (float*)(lds + a.off_na);   // [2][NP]
  int* ctx = (int*)(lds + a.off_ctx);
  int* ylab = (int*)(lds + a.off_ylab);
  float* misc = (float*)(lds + a.off_misc);
  const unsigned ldsb = lds_base_addr(lds);

  const int den_lanes = a.den_waves * 64;
  const int aux_lanes = a.aux_waves * 64;
  const int role = wave < a.den_waves ? 0 : (wave < a.den_waves + a.aux_waves ? 1 : 2);
  const int lw = wave - a.den_waves - a.aux_waves;  // loader wave index
  const int al = tid - den_lanes;                   // aux lane index

  // ---- prologue
  if (role == 2) {
    const int pre = nf < a.P ? nf : a.P;
    for (int f = 0; f < pre; ++f) issue_frame(a, b, f, f, lw, lane, ldsb);
  } else if (role == 0) {
    if (do_den)
      for (int q = tid; q < C; q += den_lanes) abuf[q] = (q == 0) ? s_one<MODE>() : s_zero<MODE>();
    den_sub_init(a, lds, tid);
  } else if (do_num) {
    for (int u = al; u < NP; u += aux_lanes) nbuf[u] = (u == 0) ? s_one<MODE>() : s_zero<MODE>();
    load_labels(a, b, ylab, al, aux_lanes);
    num_sub_init(a, lds, al);
  }
  lds_barrier();
  if (role == 1 && do_num && al == 0) walk_states(a, ctx, ylab);
  lds_barrier();
  float noff = 0.f;  // the numerator vector's final offset (Log)
  float doff = 0.f;  // the denominator vector's final offset (Log)

  // ---- frame loop (alignment scan, lattices.py:856-892), one loop per role
  if (role == 2) {
    loader_loop(a, b, nf, false, lw, lane, ldsb);
  } else if (role == 0) {
    if (do_den && !LT_ABL(a, 1)) {
      if constexpr (DEN > 0) doff = den_fwd_tri<BF16, WST, DEN == 1 ? 0 : DEN>(a, lds, abuf, b, nf, tid);
      else doff = den_fwd_loop<MODE, BF16, WST, LG, P>(a, lds, abuf, b, nf, tid);
    } else {
      idle_loop(nf);
    }
  } else {
    if (do_num && !LT_ABL(a, 2))
      noff = num_fwd_loop<MODE, BF16, WST>(a, lds, nbuf, ctx, ylab, b, nf, al, aux_lanes);
    else idle_loop(nf);
  }
  // the trigram overlap: every row final (the storing roles drain first)
  if (a.prog && role != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  tri_pub_store(a, b, 0, (unsigned)nf);

  // ---- finalize: shortest distance = (+)_q alpha_T[q] (lattices.py:496)
  const int fin = nf & 1;
  if (role == 0 && do_den) {
    const float* af = abuf + fin * C;
    if (wave == 0) {
      float r;
      int bi = 0x7fffffff;
      if constexpr (MODE == M_LOG) {
        float mx = -kInf;
        for (int q = lane; q < C; q += 64) mx = fmaxf(mx, af[q]);
        mx = gmax<6>(mx, 6);
        const float c = __builtin_isfinite(mx) ? mx : 0.f;
        float s = 0.f;
        for (int q = lane; q < C; q += 64) s += lt_exp(af[q] - c);
        s = gsum<6>(s, 6);
        r = doff + (c + lt_log(s));
      } else if constexpr (MODE == M_MAX) {
        r = -kInf;
        for (int q = lane; q < C; q += 64)
          if (bi == 0x7fffffff || af[q] > r) { r = af[q]; bi = q; }
        gargmax<6>(r, bi, 6);
      } else {
        float s = 0.f;
        for (int q = lane; q < C; q += 64) s += af[q];
        r = gsum<6>(s, 6);
      }
      if (lane == 0) {
        misc[0] = r;
        if (a.dist) a.dist[b] = r;
        if (MODE == M_MAX && a.qstar) a.qstar[b] = bi;
      }
    }
    if (a.alpha) {  // padding frames carry alpha (lattices.py:460-461)
      const long long n = (long long)(a.T - nf) * C;
      float* dst = a.alpha + ((long long)b * a.T + nf) * C;
      for (long long e = tid; e < n; e += den_lanes)
        dst[e] = MODE == M_LOG ? doff + af[e % C] : af[e % C];
    }
  } else if (role == 1 && do_num) {
    const float* nfin = nbuf + fin * NP;
    if (al == 0) {
      const int nl = a.nlab[b];
      // lattices.py:375-377: (+) over positions equal to num_labels
      const float r = (nl >= 0 && nl <= a.U) ? (MODE == M_LOG ? noff + nfin[nl] : nfin[nl])
                                             : s_zero<MODE>();
      misc[1] = r;
      if (a.num) a.num[b] = r;
    }
    if (a.alpha_num) {
      const long long n = (long long)(a.T - nf) * NP;
      float* dst = a.alpha_num + ((long long)b * a.T + nf) * NP;
      for (long long e = al; e < n; e += aux_lanes)
        dst[e] = MODE == M_LOG ? noff + nfin[e % NP] : nfin[e % NP];
    }
  }
  if (a.flags & F_LOSS) {
    lds_barrier();
    if (tid == 0) {
      // lattices.py:178-183
      const float num = misc[1];
      a.loss[b] = (a.flags & F_LOCAL) ? -num : misc[0] - num;
    }
  }
  if (do_num && a.arcs) write_arc_table(a, b, ctx, ylab, tid, blockDim.x);
}

// ---------------------------------------------------------------------------
// Backward kernel (Log): beta recursion + arc marginals -> dW.
//   Den lanes store dW straight to HBM, once per element.
//   DST: the numerator marginals of the den lanes' frame are already in a
//        3-deep LDS buffer (numerator lanes run one frame ahead) and are
//        subtracted before the store.
//   !DST (large C*(V+1)): numerator marginals go to a side buffer and a
//        scatter kernel subtracts them afterwards.
// ---------------------------------------------------------------------------
template <bool BF16, bool WST, bool DST, int LG, int P, bool CK>
LT_DEVINL void den_bwd_loop(const KArgs& a, unsigned char* lds, float* bbuf, float* nbuf3,
                            int b, int nf, int tid, float gb, float log_z, bool do_den,
                            bool do_num) {
  const NGram& g = a.g;
  const int C = g.C, FR = a.FR;
  const int lgL = LG >= 0 ? LG : a.lgL;
  const int L = 1 << lgL;
  const int j = tid & (L - 1);
  const int grp = tid >> lgL;
  const int ngrp = (a.den_waves * 64) >> lgL;
  const bool fast = a.den_fast;
  const bool has = grp < a.den_groups;
  const bool sub_num = DST && do_num;
  // Spare-lane extra group (plan: den_xg): the last source state E = C-1 is
  // reduced by the idle last lane (j = L-1) of every group in wave 0, so the
  // den role needs no partly filled extra wave; its reduction runs over lanes
  // 8k+7 with row_shr / row_bcast DPP and a readlane.
  const int E = C - 1;
  const bool xw = fast && a.den_xg && tid < 64;  // wave-uniform
  const bool xl = xw && j == L - 1;
  int woff[P], boff[P];
  int nv = 0;
  if (xl) nv = bwd_slice<P>(g, E, grp, a.Pr, woff, boff);
  else if (fast && has) nv = bwd_slice<P>(g, grp, j, a.Pr, woff, boff);
  const unsigned char* ringw = lds + a.off_ring + a.st_off[0];
  const unsigned char* ringa = lds + a.off_ring + a.st_off[1];
  const long long es = BF16 ? 2 : 4;
  const long long t_last = (long long)b * a.T + (nf - 1);
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)FR * es, t_last, true);
  Cursor ca = make_cursor(a.st_row[1] > 0 ? a.st_row[1] : (long long)C * 4, t_last, true);
  long long gframe = t_last * FR;  // global element offset of the frame
  // CK: beta_t (computed at step i for frame t = nf-1-i) is frame t-1's
  // checkpoint row; the row of frame nf-1 (beta_nf = 0) is the prologue's.
  float* brow = (CK && a.beta) ? a.beta + (t_last - 1) * C : nullptr;
  // beta relative to an integer offset Ob near its max (den_sub_take): the
  // recursion's roundings stay small; rows are Ob + value, and a marginal's
  // exponent takes the large terms as (alpha - log_z) + Ob first
  float Ob = 0.f, dsub = 0.f;
  // one source group: beta_t[p] (alignments.py:315-316) and, unless CK, the
  // marginals of its out-arcs (alignments.py:311-314) -> dW
  auto group = [&](int p, const int* wo, const int* bo, int n2, const unsigned char* wrow,
                   const float* arow, const float* bcur, float* bnxt, const float* ncur,
                   void* dWf, float* crow, bool xwv) {
      // every LDS read first, unconditionally (slots past the slice read
      // in-bounds dummies), so they issue back to back
      float wv[P], bv[P], nm[P];
#pragma unroll
      for (int m = 0; m < P; ++m) {
        wv[m] = ldw<BF16>(wrow, wo[m]);
        bv[m] = bcur[bo[m]];
        nm[m] = (!CK && sub_num) ? ncur[wo[m]] : 0.f;
      }
      const bool xlv = xwv && j == L - 1;
      const int pl = xlv ? E : p;
      const float ap = (!CK && do_den) ? arow[pl] : 0.f;
      float v[P];
      if (CK || do_den) {
        float x[P];
#pragma unroll
        for (int m = 0; m < P; ++m) x[m] = m < n2 ? wv[m] + bv[m] : -kInf;
        const float lmax = tree_max<P>(x);
        float mx;
        if (xwv) {
          const float gm = gmax<LG>(xlv ? -kInf : lmax, lgL);
          const float em = xlane_reduce<true>(xlv ? lmax : -kInf);
          mx = xlv ? em : gm;
        } else {
          mx = gmax<LG>(lmax, lgL);
        }
        const float c = __builtin_isfinite(mx) ? mx : 0.f;
        const float cl = c * kLog2e;
#pragma unroll
        for (int m = 0; m < P; ++m) x[m] = lt_exp_off(x[m], cl);
        const float ls = tree_sum<P>(x);
        float s;
        if (xwv) {
          const float gs = gsum<LG>(xlv ? 0.f : ls, lgL);
          const float es2 = xlane_reduce<false>(xlv ? ls : 0.f);
          s = xlv ? es2 : gs;
        } else {
          s = gsum<LG>(ls, lgL);
        }
        if (j == 0 || (xwv && tid == L - 1)) {
          const float bval = (c + lt_log(s)) - dsub;
          bnxt[pl] = bval;
          if (CK && crow) crow[pl] = (Ob + dsub) + bval;
        }
        if constexpr (CK) return;
        // marginal exp(alpha + w + beta' - log_z) = e * exp(c + alpha - log_z)
        // (no finite out-term: no marginal, whatever alpha - log_z is)
        const float sp = (gb == 0.f || !__builtin_isfinite(mx))
                             ? 0.f : lt_exp(((ap - log_z) + Ob) + c) * gb;
#pragma unroll
        for (int m = 0; m < P; ++m) v[m] = x[m] * sp - nm[m];
      } else {
#pragma unroll
        for (int m = 0; m < P; ++m) v[m] = -nm[m];
      }
      // branch-free stores: slots past the lane's slice rewrite the last valid
      // element with its own value
      if (n2 > 0) {
        const int wl = wo[0];
        float vl = v[0];
        int wlast = wl;
#pragma unroll
        for (int m = 1; m < P; ++m)
          if (m < n2) { wlast = wo[m]; vl = v[m]; }
#pragma unroll
        for (int m = 0; m < P; ++m) {
          const bool ok = m < n2;
          stw<BF16>(dWf, (ok ? wo[m] : wlast), ok ? v[m] : vl);
        }
      }
  };
  int k3 = 0;  // numerator marginal buffer of this frame (i % 3)
  // per-frame pointers, then the role's work; fast and general paths are
  // separate loops so each keeps only its own state live
  auto step = [&](int i, auto&& work) {
    LT_STAMP(a, tid == 0, 0, i, 0);
    lds_barrier();
    LT_STAMP(a, tid == 0, 0, i, 1);
    const int cur = i & 1;
    const unsigned char* wrow = WST ? ringw + cw.soff + cw.mis : a.W + cw.goff;
    const float* arow = (const float*)(ringa + ca.soff + ca.mis);
    const float* bcur = bbuf + cur * C;
    float* bnxt = bbuf + (cur ^ 1) * C;
    const float* ncur = nbuf3 + k3 * FR;
    void* dWf = CK ? nullptr
                   : (BF16 ? (void*)((unsigned short*)a.dW + gframe)
                           : (void*)((float*)a.dW + gframe));
    float* crow = (brow && i < nf - 1) ? brow : nullptr;
    dsub = den_sub_take(a, lds, bcur, C, tid, i);
    work(wrow, arow, bcur, bnxt, ncur, dWf, crow);
    Ob += dsub;
    advance(cw, a);
    if (!CK) advance(ca, a);
    gframe -= FR;
    if (brow) brow -= C;
    k3 = (k3 == 2) ? 0 : k3 + 1;
    LT_STAMP(a, tid == 0, 0, i, 2);
  };
  if (fast && xw) {
    for (int i = 0; i < nf; ++i)
      step(i, [&](const unsigned char* wrow, const float* arow, const float* bcur, float* bnxt,
                  const float* ncur, void* dWf, float* crow) {
        group(grp, woff, boff, nv, wrow, arow, bcur, bnxt, ncur, dWf, crow, true);
      });
  } else if (fast) {
    for (int i = 0; i < nf; ++i)
      step(i, [&](const unsigned char* wrow, const float* arow, const float* bcur, float* bnxt,
                  const float* ncur, void* dWf, float* crow) {
        if (has) group(grp, woff, boff, nv, wrow, arow, bcur, bnxt, ncur, dWf, crow, false);
      });
  } else {
    // a lane's slice advances by a constant from one pass to the next once
    // its source is a full-order state and ngrp is a multiple of V^(n-1)
    // (next(p, y) - y is then unchanged): W moves by ngrp rows, the blank's
    // beta index by ngrp, the lexical ones not at all
    const int R = g.V + 1;
    const bool bstep = g.n == 1 || (g.n >= 2 && ngrp % g.Vn1 == 0);
    for (int i = 0; i < nf; ++i)
      step(i, [&](const unsigned char* wrow, const float* arow, const float* bcur, float* bnxt,
                  const float* ncur, void* dWf, float* crow) {
        int wo[P], bo[P], n2 = 0, pprev = -1;
        for (int p = grp; p < C; p += ngrp) {
          if (bstep && pprev >= g.An) {
#pragma unroll
            for (int m = 0; m < P; ++m) {
              const bool blank = m == 0 && j == 0;
              wo[m] += m < n2 ? ngrp * R : 0;
              bo[m] += (m < n2 && blank) ? ngrp : 0;
            }
          } else {
            n2 = bwd_slice<P>(g, p, j, a.Pr, wo, bo);
          }
          pprev = p;
          group(p, wo, bo, n2, wrow, arow, bcur, bnxt, ncur, dWf, crow, false);
        }
      });
  }
}

// Trigram checkpointing backward den recursion (see den_fwd_tri): beta_t[p]
// = (+)_y W[p, y] + beta_{t+1}[next(p, y)] (alignments.py:315-316,
// contexts.py:232-256) for the sources p = tid and tid + 576 of this lane;
// beta_t is frame t-1's checkpoint row (the CK convention of den_bwd_loop).
// V = 32: beta rows kept padded in LDS, each next-state block of 32 followed
// by one unused float (block b at 33 b, state (b, y) at 33 b + y - 1), so
// a lane reads its block and its W row in natural label order at immediate
// offsets from two lane bases: consecutive sources (consecutive b) then sit
// 33 floats apart, 32 different banks, with no per-term address arithmetic
// (the skewed order above cost two integer ops a term and was the long pole
// of the launch)
constexpr int kTriBPad = 1088;  // padded row: 33 + 33 * 32 - 1 floats
LT_DEVINL int tri_pad(int s) { return s < 33 ? s : s + ((s - 33) >> 5); }

// a W row of 33 weights from LDS. The row's 2-byte alignment varies with p
// (66 B rows): plain loads would be merged into unaligned 16-byte reads,
// measured 0.7 ms slower per cfg5 call than one read per weight
template <bool BF16>
LT_DEVINL void tri_row(const unsigned char* wrow, int e, float* w) {
  // volatile LDS (address space 3) loads: one ds_read per weight, unmerged
  typedef const volatile __attribute__((address_space(3))) unsigned short lds_u16;
  typedef const volatile __attribute__((address_space(3))) float lds_f32;
#pragma unroll
  for (int k = 0; k < 33; ++k) {
    if constexpr (BF16)
      w[k] = __uint_as_float((unsigned)((lds_u16*)wrow)[e + k] << 16);
    else
      w[k] = ((lds_f32*)wrow)[e + k];
  }
}

template <bool BF16, bool WST>
LT_DEVINL void den_bwd_tri32(const KArgs& a, unsigned char* lds, int b, int nf, int tid) {
  static_assert(WST, "the V = 32 role reads W from the LDS ring");
  constexpr int V = 32, R = 33, C = 1 + 32 + 32 * 32;
  int* slot = (int*)(lds + a.off_misc) + 2;
  float* pbuf = (float*)(lds + a.off_tb);  // [2][kTriBPad]
  const int nthr = kTriDenWaves * 64;
  const bool h0 = tid < C, h1 = tid + nthr < C;
  const int p0 = h0 ? tid : 0, p1 = h1 ? tid + nthr : 0;
  // next(p, y) = nb + y (nb = 32 b, or 0 for the start state): padded 33 b - 1 + y
  bool z;
  const int n0 = next_base(a.g, p0, &z), n1 = next_base(a.g, p1, &z);
  const int nb0 = n0 ? n0 + (n0 >> 5) - 1 : 0, nb1 = n1 ? n1 + (n1 >> 5) - 1 : 0;
  const int q0 = tri_pad(p0), q1 = tri_pad(p1);
  // beta_T = 0 (before the loop's first barrier)
  for (int e = tid; e < kTriBPad; e += nthr) pbuf[e] = 0.f;
  if (tid == 0) {
    slot[0] = tri_enc(0.f);  // max of beta_T = 0
    slot[1] = tri_enc(-kInf);
    slot[2] = tri_enc(-kInf);
  }
  const unsigned char* ring = lds + a.off_ring + a.st_off[0];
  const long long t_last = (long long)b * a.T + (nf - 1);
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * (BF16 ? 2 : 4),
                          t_last, true);
  float* brow = a.beta ? a.beta + (t_last - 1) * C : nullptr;
  float Ob = 0.f;
  for (int i = 0; i < nf; ++i) {
    tri_pub_drain(a, i);
    lds_barrier();
    if (tri_pub_frame(a, i)) tri_pub_store(a, b, 1, (unsigned)i);
    const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
    const float* bcur = pbuf + (i & 1) * kTriBPad;
    float* bnxt = pbuf + ((i + 1) & 1) * kTriBPad;
    const int s3 = i % 3;
    const float mprev = tri_dec(slot[s3]);
    const float sp = __builtin_isfinite(mprev) ? floorf(mprev) : 0.f;
    if (tid == 0) slot[s3 == 0 ? 2 : s3 - 1] = tri_enc(-kInf);
    float* crow = (brow && i < nf - 1) ? brow : nullptr;
    float lmax = -kInf;
#pragma unroll 1
    for (int d = 0; d < 2; ++d) {
      if (!(d ? h1 : h0)) break;
      const int p = d ? p1 : p0;
      const float* bn = bcur + (d ? nb1 : nb0);
      float w[R];
      tri_row<BF16>(wrow, p * R, w);
      float x[V];
      const float tp = w[0] + bcur[d ? q1 : q0];  // blank self loop
      float m = tp;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        x[k] = w[k + 1] + bn[k + 1];
        m = fmaxf(m, x[k]);
      }
      const float c = __builtin_isfinite(m) ? m : 0.f;
      const float l = c * kLog2e;
      float s = lt_exp_off(tp, l);
#pragma unroll
      for (int k = 0; k < V; ++k) s += lt_exp_off(x[k], l);
      const float r = (c + lt_log(s)) - sp;
      bnxt[d ? q1 : q0] = r;
      if (crow) crow[p] = (Ob + sp) + r;
      lmax = fmaxf(lmax, r);
    }
    tri_publish_max(slot + (s3 == 2 ? 0 : s3 + 1), lmax);
    Ob += sp;
    advance(cw, a);
    if (brow) brow -= C;
  }
}

template <bool BF16, bool WST, int VT>
LT_DEVINL void den_bwd_tri(const KArgs& a, unsigned char* lds, float* bbuf, int b, int nf,
                           int tid) {
  if constexpr (VT == 32) {
    den_bwd_tri32<BF16, WST>(a, lds, b, nf, tid);
    return;
  }
  const NGram& g = a.g;
  const int V = VT > 0 ? VT : g.V, R = V + 1;
  const int C = VT > 0 ? 1 + VT + VT * VT : g.C;
  int* slot = (int*)(lds + a.off_misc) + 2;
  const int nthr = kTriDenWaves * 64;
  const bool h0 = tid < C, h1 = tid + nthr < C;
  const int p0 = h0 ? tid : 0, p1 = h1 ? tid + nthr : 0;
  bool z;
  const int nb0 = next_base(g, p0, &z), nb1 = next_base(g, p1, &z);
  const int ys = (tid & 63) % V;  // the lane's first label - 1
  if (tid == 0) {
    slot[0] = tri_enc(0.f);  // max of beta_T = 0
    slot[1] = tri_enc(-kInf);
    slot[2] = tri_enc(-kInf);
  }
  const unsigned char* ring = lds + a.off_ring + a.st_off[0];
  const long long t_last = (long long)b * a.T + (nf - 1);
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * (BF16 ? 2 : 4),
                          t_last, true);
  float* brow = a.beta ? a.beta + (t_last - 1) * C : nullptr;
  float Ob = 0.f;
  for (int i = 0; i < nf; ++i) {
    lds_barrier();
    const unsigned char* wrow = WST ? ring + cw.soff + cw.mis : a.W + cw.goff;
    const float* bcur = bbuf + (i & 1) * C;
    float* bnxt = bbuf + ((i + 1) & 1) * C;
    const int s3 = i % 3;
    const float mprev = tri_dec(slot[s3]);
    const float sp = __builtin_isfinite(mprev) ? floorf(mprev) : 0.f;
    if (tid == 0) slot[s3 == 0 ? 2 : s3 - 1] = tri_enc(-kInf);
    float* crow = (brow && i < nf - 1) ? brow : nullptr;
    float lmax = -kInf;
#pragma unroll 1
    for (int d = 0; d < 2; ++d) {
      if (!(d ? h1 : h0)) break;
      const int p = d ? p1 : p0, nb = d ? nb1 : nb0;
      float x[32];
      const float tp = ldw<BF16>(wrow, p * R) + bcur[p];  // blank self loop
      float m = tp;
      int y = ys + 1;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        if (k < V) {
          x[k] = ldw<BF16>(wrow, p * R + y) + bcur[nb + y];
          y = y == V ? 1 : y + 1;
        } else {
          x[k] = -kInf;
        }
        m = fmaxf(m, x[k]);
      }
      const float c = __builtin_isfinite(m) ? m : 0.f;
      const float l = c * kLog2e;
      float s = lt_exp_off(tp, l);
#pragma unroll
      for (int k = 0; k < 32; ++k) s += lt_exp_off(x[k], l);
      const float r = (c + lt_log(s)) - sp;
      bnxt[p] = r;
      if (crow) crow[p] = (Ob + sp) + r;
      lmax = fmaxf(lmax, r);
    }
    tri_publish_max(slot + (s3 == 2 ? 0 : s3 + 1), lmax);
    Ob += sp;
    advance(cw, a);
    if (brow) brow -= C;
  }
}

// Numerator beta + marginals for one frame (the reverse of
// alignments.py:320-329): beta^n_t[u] from beta^n_{t+1}; marginals
// exp(alpha^n_t[u] + w + beta^n_{t+1} - num) * g accumulated (LDS atomics:
// several positions can share an arc) into `mdst` or written to the side
// buffer `side` (direct path).
template <bool BF16, bool DST>
LT_DEVINL void num_bwd_frame(const KArgs& a, const unsigned char* wrow, const float* anrow,
                             const float* ncur, float* nnxt, float* mdst, float* side,
                             const int* ctx, const int* ylab, int al, int num_lanes, int ob,
                             int ol, float gb, float numv, float Ob, float sp) {
  const int NP = a.U + 1;
  // beta^n in ncur is relative to the integer offset Ob (num_sub_take):
  // the marginal's exponent alpha^n + w + beta^n - num takes it with alpha^n
  // - num, the two large terms first
  for (int u = al; u < NP; u += num_lanes) {
    int o0 = ob, o1 = ol;
    if (u != al) { o0 = ctx[u]; o1 = u < a.U ? o0 + ylab[u] : 0; }
    const bool lex = u < a.U;
    // all reads first (o1 = 0 and the u+1 clamp are in-bounds dummies)
    const float wb = ldw<BF16>(wrow, o0);
    const float wl = ldw<BF16>(wrow, o1);
    const float bu = ncur[u];
    const float bu1 = ncur[lex ? u + 1 : u];
    const float an = (anrow[u] - numv) + Ob;
    const float xb = wb + bu;
    const float xl = lex ? wl + bu1 : -kInf;
    // log_plus (semirings.py:248-255) sharing its exponentials with the
    // marginals exp(an + x) = exp(x - c) * exp(an + c)
    float c = fmaxf(xb, xl);
    // no path through (t, u) on either arc: no marginal (alpha^n alone may
    // be far above num, and exp of it times a zero term is NaN)
    const bool live = __builtin_isfinite(c);
    if (!live) c = 0.f;
    const float eb = lt_exp(xb - c), el = lt_exp(xl - c);
    nnxt[u] = (c + lt_log(eb + el)) - sp;
    float mb = 0.f, ml = 0.f;
    if (gb != 0.f && live) {
      const float sc = lt_exp(an + c) * gb;
      mb = eb * sc;
      ml = el * sc;
    }
    if constexpr (DST) {
      if (mb != 0.f) atomicAdd(&mdst[o0], mb);
      if (ml != 0.f) atomicAdd(&mdst[o1], ml);
    } else {
      side[u * 2 + 0] = mb;
      side[u * 2 + 1] = ml;
    }
  }
}

// Numerator lanes of the backward. DST: they run one frame AHEAD of the
// denominator (frame nf-1 in the prologue, frame nf-2-i at step i) so that
// the den lanes can subtract the numerator marginals of their frame from
// the 3-deep LDS buffer and store dW once, straight to HBM.
template <bool BF16, bool WST, bool DST>
LT_DEVINL void num_bwd_loop(const KArgs& a, unsigned char* lds, float* nbb, float* nbuf3,
                            const int* ctx, const int* ylab, int b, int nf, int al, int num_lanes,
                            float gb, float numv) {
  const int NP = a.U + 1, FR = a.FR;
  int ob = 0, ol = 0;
  if (al < NP) {
    ob = ctx[al];
    ol = al < a.U ? ob + ylab[al] : 0;
  }
  const unsigned char* ringw = lds + a.off_ring + a.st_off[0];
  const unsigned char* ringn = lds + a.off_ring + a.st_off[2];
  const long long es = BF16 ? 2 : 4;
  const long long t_last = (long long)b * a.T + (nf - 1);
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)FR * es, t_last, true);
  Cursor cn = make_cursor(a.st_row[2], t_last, true);
  float* side = a.nm_side ? a.nm_side + t_last * NP * 2 : nullptr;
  const int lead = DST ? 1 : 0;  // frames ahead of the den lanes
  int nb = 0;                    // beta^n buffer parity
  int k3 = 0;                    // marginal buffer of the frame being computed
  float Ob = 0.f;  // beta^n's integer offset
  int k = 0;       // num_bwd_frame calls (the offset slots' parity)
  if (DST && nf > 0) {           // prologue frame nf-1 (after the caller's barrier)
    const unsigned char* wrow = WST ? ringw + cw.soff + cw.mis : a.W + cw.goff;
    const float* anrow = (const float*)(ringn + cn.soff + cn.mis);
    const float sp = num_sub_take(a, lds, nbb, NP, al, k++);
    num_bwd_frame<BF16, DST>(a, wrow, anrow, nbb, nbb + NP, nbuf3, nullptr, ctx, ylab, al,
                             num_lanes, ob, ol, gb, numv, Ob, sp);
    Ob += sp;
    advance(cw, a);
    advance(cn, a);
    nb = 1;
    k3 = 1;
  }
  [[maybe_unused]] const bool stamper = al == 0;
  for (int i = 0; i < nf; ++i) {
    LT_STAMP(a, stamper, 1, i, 0);
    lds_barrier();
    LT_STAMP(a, stamper, 1, i, 1);
    if (i + lead < nf) {
      float* mdst = nbuf3 + k3 * FR;
      if constexpr (DST) {  // re-zero the buffer the den lanes read last step
        float* stale = nbuf3 + ((k3 == 2) ? 0 : k3 + 1) * FR;
        for (int u = al; u < NP; u += num_lanes) {
          int o0 = ob, o1 = ol;
          if (u != al) { o0 = ctx[u]; o1 = u < a.U ? o0 + ylab[u] : 0; }
          stale[o0] = 0.f;
          stale[o1] = 0.f;
        }
      }
      const unsigned char* wrow = WST ? ringw + cw.soff + cw.mis : a.W + cw.goff;
      const float* anrow = (const float*)(ringn + cn.soff + cn.mis);
      const float sp = num_sub_take(a, lds, nbb + nb * NP, NP, al, k++);
      num_bwd_frame<BF16, DST>(a, wrow, anrow, nbb + nb * NP, nbb + (nb ^ 1) * NP, mdst, side,
                               ctx, ylab, al, num_lanes, ob, ol, gb, numv, Ob, sp);
      Ob += sp;
      advance(cw, a);
      advance(cn, a);
      if (side) side -= NP * 2;
      nb ^= 1;
      k3 = (k3 == 2) ? 0 : k3 + 1;
    }
    LT_STAMP(a, stamper, 1, i, 2);
  }
}

// Numerator lanes of the checkpointing backward: beta^n only, one frame per
// step in lockstep with the den lanes; beta^n_t is frame t-1's checkpoint row.
template <bool BF16, bool WST>
LT_DEVINL void num_beta_loop(const KArgs& a, unsigned char* lds, float* nbb, const int* ctx,
                             const int* ylab, int b, int nf, int al, int num_lanes) {
  const int NP = a.U + 1;
  int ob = 0, ol = 0;
  if (al < NP) {
    ob = ctx[al];
    ol = al < a.U ? ob + ylab[al] : 0;
  }
  const unsigned char* ringw = lds + a.off_ring + a.st_off[0];
  const long long es = BF16 ? 2 : 4;
  const long long t_last = (long long)b * a.T + (nf - 1);
  Cursor cw = make_cursor(a.st_row[0] > 0 ? a.st_row[0] : (long long)a.FR * es, t_last, true);
  float* row = a.beta_num ? a.beta_num + (t_last - 1) * NP : nullptr;
  int nb = 0;
  float Ob = 0.f;  // the vector's integer offset (num_sub_take); rows are Ob + value
  for (int i = 0; i < nf; ++i) {
    LT_STAMP(a, al == 0, 1, i, 0);
    tri_pub_drain(a, i);
    lds_barrier();
    LT_STAMP(a, al == 0, 1, i, 1);
    const unsigned char* wrow = WST ? ringw + cw.soff + cw.mis : a.W + cw.goff;
    const float* ncur = nbb + nb * NP;
    float* nnxt = nbb + (nb ^ 1) * NP;
    float* crow = (row && i < nf - 1) ? row : nullptr;
    const float sp = num_sub_take(a, lds, ncur, NP, al, i);
    Ob += sp;
    for (int u = al; u < NP; u += num_lanes) {
      int o0 = ob, o1 = ol;
      if (u != al) { o0 = ctx[u]; o1 = u < a.U ? o0 + ylab[u] : 0; }
      const bool lex = u < a.U;
      const float wb = ldw<BF16>(wrow, o0);
      const float wl = ldw<BF16>(wrow, o1);
      const float bu = ncur[u];
      const float bu1 = ncur[lex ? u + 1 : u];
      const float v = log_plus(wb + bu, lex ? wl + bu1 : -kInf) - sp;
      nnxt[u] = v;
      if (crow) crow[u] = Ob + v;
    }
    advance(cw, a);
    if (row) row -= NP;
    nb ^= 1;
    LT_STAMP(a, al == 0, 1, i, 2);
  }
}

// CK = true: the checkpointing backward. Only beta (den) and beta^n (num)
// are computed and written per frame (a.beta / a.beta_num); the arc
// marginals come later from marg_kernel, so this kernel can run
// concurrently with the forward (both depend only on W).
// DEN > 0: the den role runs den_bwd_tri (trigram checkpointing backward, as fwd_body)
template <bool BF16, bool WST, bool DST, int LG, int P, bool CK = false, int KOFF = 0, int DEN = 0>
LT_DEVINL void bwd_body(const KArgs& a, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const NGram& g = a.g;
  const int C = g.C, NP = a.U + 1, FR = a.FR;
  const bool do_den = a.flags & F_DEN, do_num = a.flags & F_NUM;
  if (a.only && !a.only[b]) return;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);

  float* bbuf = (float*)(lds + a.off_a);     // [2][C]  den beta
  float* nbb = (float*)(lds + a.off_na);     // [2][NP] num beta
  int* ctx = (int*)(lds + a.off_ctx);
  int* ylab = (int*)(lds + a.off_ylab);
  float* nbuf3 = (float*)(lds + a.off_nbuf); // [3][FR] num marginals (DST)
  const unsigned ldsb = lds_base_addr(lds);

  const int den_lanes = a.den_waves * 64;
  const int aux_lanes = a.aux_waves * 64;
  const int role = wave < a.den_waves ? 0 : (wave < a.den_waves + a.aux_waves ? 1 : 2);
  const int lw = wave - a.den_waves - a.aux_waves;
  const int al = tid - den_lanes;

  float gb = a.grad ? a.grad[b] : 1.f;
  const float log_z = do_den ? a.log_z_in[b] : 0.f;
  const float numv = do_num ? a.num_in[b] : 0.f;
  // unreachable label string (loss = +inf) or degenerate partition: dW = 0
  if ((do_num && !__builtin_isfinite(numv)) || (do_den && !__builtin_isfinite(log_z))) gb = 0.f;
  const int nl = do_num ? a.nlab[b] : 0;

  // ---- prologue
  if (role == 2) {
    const int pre = nf < a.P ? nf : a.P;
    for (int f = 0; f < pre; ++f) issue_frame(a, b, nf - 1 - f, f, lw, lane, ldsb);
  } else if (role == 0) {
    // beta_T = one for every state: all context states are final
    // (lattices.py:788-790)
    if (do_den) {
      float* crow = (CK && a.beta && nf > 0) ? a.beta + ((long long)b * a.T + nf - 1) * C
                                             : nullptr;
      for (int p = tid; p < C; p += den_lanes) {
        bbuf[p] = 0.f;
        if (crow) crow[p] = 0.f;
      }
    }
    den_sub_init(a, lds, tid);
  } else {
    if (do_num) {
      float* crow = (CK && a.beta_num && nf > 0)
                        ? a.beta_num + ((long long)b * a.T + nf - 1) * NP : nullptr;
      for (int u = al; u < NP; u += aux_lanes) {
        const float v = (u == nl) ? 0.f : -kInf;
        nbb[u] = v;
        if (crow) crow[u] = v;
      }
      load_labels(a, b, ylab, al, aux_lanes);
      num_sub_init(a, lds, al);
    }
    if (DST && do_num)
      for (int e = al; e < 3 * FR; e += aux_lanes) nbuf3[e] = 0.f;
  }
  lds_barrier();
  if (role == 1 && do_num && al == 0) walk_states(a, ctx, ylab);
  if (role == 2 && DST && do_num && nf > 0) {
    // the numerator lanes start one frame early: frame nf-1 must have landed
    const int pre = nf < a.P ? nf : a.P;
    wait_vmcnt((pre - 1) * (lw == 0 ? a.gw0 : a.gw1));
  }
  lds_barrier();
  if (!DST && do_num && role == 1 && a.ctx_side) {
    for (int u = al; u < NP; u += aux_lanes) {
      a.ctx_side[((long long)b * NP + u) * 2 + 0] = ctx[u];
      a.ctx_side[((long long)b * NP + u) * 2 + 1] = ylab[u];
    }
  }

  if (role == 2) {
    loader_loop(a, b, nf, true, lw, lane, ldsb, DST && do_num ? 1 : 0);
  } else if (role == 0) {
    if (!LT_ABL(a, 1) && (!CK || do_den)) {
      if constexpr (DEN > 0)
        den_bwd_tri<BF16, WST, DEN == 1 ? 0 : DEN>(fresh_args<KOFF>(), lds, bbuf, b, nf, tid);
      else
        den_bwd_loop<BF16, WST, DST, LG, P, CK>(fresh_args<KOFF>(), lds, bbuf, nbuf3, b, nf, tid,
                                                gb, log_z, do_den, do_num);
    } else {
      idle_loop(nf);
    }
  } else {
    if (do_num && !LT_ABL(a, 2)) {
      if constexpr (CK)
        num_beta_loop<BF16, WST>(fresh_args<KOFF>(), lds, nbb, ctx, ylab, b, nf, al, aux_lanes);
      else
        num_bwd_loop<BF16, WST, DST>(fresh_args<KOFF>(), lds, nbb, nbuf3, ctx, ylab, b, nf, al,
                                     aux_lanes, gb, numv);
    } else {
      idle_loop(nf);
    }
  }
  if constexpr (CK) {
    if (a.prog) {  // the trigram overlap: every row final (the storing roles drain first)
      if (role != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      tri_pub_store(a, b, 1, (unsigned)nf);
    }
    return;
  }
  lds_barrier();
  // padding frames get zero marginals (lattices.py:775-779)
  {
    const long long n = (long long)(a.T - nf) * FR;
    const long long base = ((long long)b * a.T + nf) * FR;
    const int nthr = blockDim.x;
    for (long long e = tid; e < n; e += nthr) stw<BF16>(a.dW, base + e, 0.f);
  }
}

template <int MODE, bool BF16, bool WST, int LG, int P>
__global__ __launch_bounds__(1024) void fwd_kernel(const KArgs a) {
  fwd_body<MODE, BF16, WST, LG, P>(a, blockIdx.x);
}
template <bool BF16, bool WST, bool DST, int LG, int P, bool CK = false>
__global__ __launch_bounds__(1024) void bwd_kernel(const KArgs a) {
  bwd_body<BF16, WST, DST, LG, P, CK>(a, blockIdx.x);
}
// The frame-serial loss + dW of one utterance in ONE launch (lt_loss_grad's
// fallback for the utterances only[b] marks): the Log forward (alpha,
// alpha^n, loss) and then, in the same workgroup, the backward with the
// marginals. The forward's global stores (checkpoints, log_z, num) are this
// workgroup's own, so a vmcnt drain and the barrier hand them over; every
// other workgroup returns at once (one launch a call instead of two).
template <bool BF16, bool WST, bool DST, int LG, int P>
__global__ __launch_bounds__(1024) void serial_kernel(const KArgs af, const KArgs ab) {
  fwd_body<M_LOG, BF16, WST, LG, P>(af, blockIdx.x);
  if (af.only && !af.only[blockIdx.x]) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bwd_body<BF16, WST, DST, LG, P, false, (int)sizeof(KArgs)>(ab, blockIdx.x);
}
// The checkpointing pair in one launch: workgroups [0, nb) run the Log
// forward (alpha, alpha^n, loss) and [nb, 2 nb) the checkpointing backward
// (beta, beta^n). Both depend only on W, so they run side by side, as
// two launches on two streams would, without the library owning a stream.
static_assert(sizeof(KArgs) % alignof(KArgs) == 0, "the second KArgs follows the first");
template <bool BF16, bool WST, int LG, int P>
__global__ __launch_bounds__(1024) void fwdbwd_kernel(const KArgs af, const KArgs ab, int nb) {
  if ((int)blockIdx.x < nb) fwd_body<M_LOG, BF16, WST, LG, P>(af, blockIdx.x);
  else bwd_body<BF16, WST, false, LG, P, true, (int)sizeof(KArgs)>(ab, blockIdx.x - nb);
}

}  // namespace

namespace lt_impl {
// The trigram overlap (lt_tri.hip, tri_mix_kernel): what its marginal
// workgroups read and write besides the recursions' KArgs
struct MixArgs {
  const unsigned char* W;
  const int* nfr;
  const int* labels;
  const float *alpha, *beta, *alpha_num, *beta_num;  // the recursions' checkpoint rows
  const float* grad;  // nullable (ones)
  void* dW;
  unsigned* prog;     // [2B] the recursions' progress (KArgs::prog)
  unsigned* xcc;      // [2B] XCD id + 1 of each recursion workgroup (0: not yet)
  unsigned* ctr;      // [8 * 32] per-XCD job counters, one 128-byte line each
  int* done;          // [B*T] frame done here (marg_kernel skips it)
  int B, T, U;
  int lds_bytes;      // the launch's dynamic LDS (the marginal waves' row regions)
  int dbg;            // diagnostic builds (LT_TRI_MIX_DBG): 1 the marginal role does nothing,
                      // 2 it waits for whole recursions, 4 it leaves every frame to marg_kernel,
                      // 8 done = XCD id + 1, 16 done = completion time and ts the recursions' times
  unsigned* ts;       // [4B] diagnostic (dbg 16): recursion start, end (s_memrealtime low bits)
  NGram g;
};

// log Z and the string's weight of one utterance from its checkpoint rows at
// a middle frame m: (+)_q alpha_m[q] beta_m[q] and (+)_u alpha^n_m[u] beta^n_m[u]
// (any frame gives both: every path crosses it). One wave, a fixed lane order
// and butterfly, so the trigram overlap's marginal role and marg_kernel get
// the same bits; sc1: rows another workgroup of the same launch published.
template <int NQ>  // values per lane: n <= 64 NQ
LT_DEVINL float mid_lse(const float* x, const float* y, int n, int lane, bool sc1) {
  float v[NQ];
  // every load in flight before the first use: sc1 (L1-bypassing) buffer
  // loads for rows another workgroup of the same launch wrote
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 4 * n, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 4 * n, 0x00020000);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = min(lane + 64 * i, n - 1);
    const float a = sc1 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, 4 * q, 0, 0x10)) : x[q];
    const float b = sc1 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, 4 * q, 0, 0x10)) : y[q];
    v[i] = lane + 64 * i < n ? a + b : -kInf;
  }
  float mx = -kInf;
#pragma unroll
  for (int i = 0; i < NQ; ++i) mx = fmaxf(mx, v[i]);
  mx = gmax<6>(mx, 6);
  const float c = __builtin_isfinite(mx) ? mx : 0.f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) s += lt_exp(v[i] - c);
  s = gsum<6>(s, 6);
  return c + lt_log(s);
}
LT_DEVINL float2 tri_mid_norm(const float* ar, const float* br, const float* anr,
                              const float* bnr, int C, int NP, int lane, bool sc1) {
  // C = 1057 (the V = 32 trigram), NP <= 128 (the overlap's shapes)
  const float lz = mid_lse<17>(ar, br, C, lane, sc1);
  const float nm = mid_lse<2>(anr, bnr, NP, lane, sc1);
  return make_float2(lz, nm);
}

struct Plan {
  KArgs a;
  int lg;    // template LG (log2 lanes per group), -1 = runtime
  int tmax;  // template P (register slice size)
  bool wst, dst;
  bool ck;   // checkpointing backward (beta rows only, no marginals)
  int threads;
  int lds_bytes;
};
// Defined in lt_inst.hip, one pair per P in LT_P_LIST.
// (LG, P) pairs with a compile-time group size (LG = log2 lanes per group)
// plus runtime-LG fallbacks (LG = -1, written M1 in names).
#define LT_VARIANTS(X) \
  X(3, 5) X(2, 9) X(1, 4) X(1, 3) X(2, 5) X(3, 3) X(2, 3) X(M1, 4) X(M1, 8) X(M1, 16)
#define LT_DECL(LG, P)                                                                   \
  int launch_fwd_##LG##_##P(int mode, const Plan& pl, bool bf16, int grid, hipStream_t st); \
  int launch_bwd_##LG##_##P(const Plan& pl, bool bf16, int grid, hipStream_t st);          \
  int launch_fwdbwd_##LG##_##P(const Plan& pf, const Plan& pb, bool bf16, int nb, hipStream_t st); \
  int launch_serial_##LG##_##P(const Plan& pf, const Plan& pb, bool bf16, int nb, hipStream_t st);
LT_VARIANTS(LT_DECL)
#undef LT_DECL
int set_error(int code, const char* msg);
// Whether `st` is being captured into a graph: launches whose hand-off words
// carry a host-chosen per-call tag then zero those words by a memset node,
// since every replay of the graph reuses the captured tag.
inline bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}
// lt_tri.hip: the trigram checkpointing pair (den_fwd_tri / den_bwd_tri roles)
int launch_tri_fwdbwd(const Plan& pf, const Plan& pb, bool bf16, int nb, hipStream_t st);
// lt_tri.hip: the same recursions with marginal workgroups on the idle CUs
// (tri_mix_kernel, V = 32); marg_kernel afterwards takes the frames not done
int launch_tri_mix(const Plan& pf, const Plan& pb, bool bf16, int nb, int marg_blocks,
                   const MixArgs& mx, hipStream_t st);
// lt_tri4.hip (diagnostic builds only): the V = 32 trigram recursions on
// quads of four workgroups
bool tri4_eligible(int V, int n, int B, int U, int cus);
int launch_tri4(const Plan& pl, bool bf16, float* alpha, float* beta, float* alpha_num,
                float* beta_num, float* log_z, float* num, float* loss, long long w_bytes,
                hipStream_t st);
// lt_lattice.hip: frame-serial loss (+ dW) for the utterances with only[b] != 0
size_t serial_side_bytes(const lt_problem* pb, int local_norm);
int serial_loss(const lt_problem* pb, int local_norm, const void* W, const int32_t* num_frames,
                const int32_t* labels, const int32_t* num_labels, const int* only, float* loss,
                float* log_z, float* num, float* alpha, float* alpha_num, const float* grad,
                void* dW, void* side, void* stream);
// lt_chunk.hip: chunked two-level scan (bigram Log)
bool chunk_eligible(const lt_problem* pb);
// lt_loss_grad's choice: the chunked scan while it is the faster design
bool chunk_preferred(const lt_problem* pb);
int chunk_loss_grad(const lt_problem* pb, int local_norm, const void* W, const int32_t* num_frames,
                    const int32_t* labels, const int32_t* num_labels, float* loss, float* log_z,
                    float* num, void* dW, void* state, size_t state_bytes, void* scratch,
                    size_t scratch_bytes, void* stream);
// lt_vit.hip: bigram MaxTropical forward (distance, best final state, backpointers)
bool vit_bigram_eligible(const lt_problem* pb);
// forward + backtrace (one launch when the backpointers fit its LDS);
// LT_EUNSUPPORTED after the forward: the caller runs the generic backtrace
int vit_bigram(const lt_problem* pb, const void* W, const int32_t* nfr, unsigned char* bp,
               int* qstar, float* dist, const float* grad, int64_t* labels, void* arcs,
               int32_t conv, void* stream);
int vit_backtrace_lds(const lt_problem* pb, int* seg);
int vit_backtrace(const lt_problem* pb, const unsigned char* bp, const int* qstar,
                  const int32_t* nfr, const float* grad, int64_t* labels, void* arcs,
                  int32_t conv, void* stream);
// The joint weight function's operands for the fused paths (lt_joint.hip):
// W[f, c, y] = bias[y] + sum_h wo[y, h] tanh(pc[c, h] + pf[f, h])
struct JointOps {
  int H;                  // hidden units (a multiple of 32)
  int prod;               // 1: split-bf16 products, 2: bf16 products
  const float *pc, *ec;   // [C, H] Pc and e^{2 Pc}
  const float *pf, *ef;   // [B*T, H] Pf and e^{2 Pf}
  const int *cbig, *fbig; // [1], [ceil(B*T / 32)]: some |projection| > 40 (direct tanh)
  const float *wo, *bias; // [R, H], [R]
};
// lt_pipe.hip: pipelined bigram Log recursions (alpha, and beta when dirs == 2)
bool pipe_eligible(const lt_problem* pb);
int launch_pipe(const lt_problem* pb, int local_norm, const void* W, const int32_t* nfr,
                const int32_t* labels, const int32_t* nlab, float* loss, float* log_z,
                float* num, float* alpha, float* alpha_num, float* beta, float* beta_num,
                int32_t* arcs, int dirs, int* err, void* stream, void* dW = nullptr,
                int mid = 0, void* mws = nullptr, const JointOps* jo = nullptr);
// mid mode (lt_loss_grad at large batches): workspace bytes; whether the
// grid fits co-resident (launch_pipe with W == nullptr answers the same)
size_t pipe_mid_workspace_bytes(const lt_problem* pb);
bool pipe_mid_fits(const lt_problem* pb);
}  // namespace lt_impl
namespace {
using lt_impl::MixArgs;
using lt_impl::tri_mid_norm;
}  // namespace
