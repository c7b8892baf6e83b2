// lt_pipe.hip -- barrier-free, producer/consumer pipelined recursions for the
// bigram lattice (FullNGram context_size = 1, 1 <= V <= 32) under the Log
// semiring: the alpha and beta passes of the checkpointing loss forward
// (lt_loss_forward with checkpoints), one workgroup per (utterance, direction).
//
// What is computed (reference file:line in last_torch/):
//   alpha_{t+1} = FrameDependent.forward(alpha_t, W_t)   alignments.py:286-297,
//                 FullNGram.forward_reduce                  contexts.py:207-230
//   beta_t      = FrameDependent.backward(beta_{t+1}, W_t) alignments.py:300-318,
//                 FullNGram.backward_broadcast              contexts.py:232-256
//   numerator alpha^n / beta^n over the label string       lattices.py:250-377,
//                                                           alignments.py:320-329
//   log_z, numerator, loss                                 lattices.py:131-183, 496
//
// Why a different kernel for this shape. With n = 1 every lexical arc with
// label y lands in state y (contexts.py:190-205), so each frame is a dense
// (V+1) x (V+1) log-semiring matrix-vector product. Written as per-destination
// logsumexps it costs one exp per arc on the serial frame chain. Here it is
// split into two factors,
//     lse_k(v_k + W_k) = (M + c) + log sum_k exp(v_k - M) * exp(W_k - c),
// with c the frame's max weight and M an upper bound of the state values:
//   * E = exp(W - c) depends only on W. Helper waves compute it for frames
//     ahead of the recursion (they also stage raw W for the numerator), so
//     no arc exp is on the chain;
//   * g_k = exp(v_k - M) is one exp per STATE, broadcast through LDS;
//   * the chain per frame is then: one exp, an LDS round trip, J fused
//     multiply-adds per lane, one DPP add and one log.
// Exactness: every product is <= 1 and the sum is kept only when it lies in
// [2^-60, 2^64]; dropped (underflowed) products are then < 2^-126, i.e.
// below fp32 rounding of the sum. Any state whose sum leaves that range
// (adversarial weight ranges, -inf / +inf arcs, dead lattices) makes the
// wave recompute the frame with the exact safe-max logsumexp of
// semirings.py:279-286 from the raw weights -- same results, slower.
// State values are kept relative to a per-utterance float-float base, so the
// chain accumulates no rounding; outputs are base + value rounded once.
//
// Execution: wave 0 = denominator (states 1..V on H lanes each, state 0
// alongside), wave 1 = numerator (PN string positions per lane, neighbours
// through DPP wave shifts), waves 2.. = helpers. Frames flow through a ring
// of K LDS slots guarded by per-slot tags (producer) and done counters
// (consumers); there is no workgroup barrier inside the frame loop. Every
// wait is bounded: a stalled pipeline raises an abort flag and the kernel
// drains instead of hanging.
#include "lt_joint.h"

#include <atomic>

namespace {

constexpr int kPipeMaxSlots = 32;
// 6 waves (den, num, 4 helpers); __launch_bounds__(384, 4) keeps them at
// <= 128 VGPRs so that two workgroups share a CU at large batches
constexpr int kPipeMaxHelpers = 4;

struct PArgs {
  const unsigned char* W;
  const int* nfr;
  const int* labels;
  const int* nlab;
  float* loss;
  float* log_z;
  float* num;
  float* alpha;      // [B,T,C]   alpha_t (pre-update) of frame t
  float* alpha_num;  // [B,T,NP]
  float* beta;       // [B,T,C]   beta_{t+1} of frame t
  float* beta_num;   // [B,T,NP]
  int* arcs;         // [B,4NP]
  int* err;          // nullable: set to 1 if a pipeline wait timed out
  int B, T, U, V, C, R, FR, flags;
  int H, lgH;        // lanes per state
  int J, JP, rowE;   // terms per lane part (<= template J), padded, floats per E row
  int K, NH, NLr;    // ring slots, helper waves, loads per lane actually needed
  int logn_x;        // unused (alignment)
  float logn;        // log(number of terms per state) for the running bound
  int off_ctl, off_g, off_u, off_ctx, off_ylab, off_ring, slot_bytes;
  int soff_e, soff_eb, soff_c;  // offsets inside a slot
  int dirs;          // 1: alpha only (blocks = B), 2: alpha + beta (blocks = 2B)
  unsigned w_bytes;  // bytes of W (< 2^32)
  long long* stamps; // diagnostic build (-DLT_STAMPS) only: [wave][T][4] s_memtime
  int stamp_block;
  int dbg;           // timing ablations (LT_PIPE_DBG): 1 no raw-W stores, 2 no E stores,
                     // 4 no den history, 8 no num history
  void* dW;          // [B,T,C,V+1], W's dtype (mid mode)
  // ---- in-workgroup marginals (lt_loss_grad at large batches, mid mode):
  // each recursion workgroup turns its second half of the frames into dW
  // from the W still in its ring (alpha: frames [nf/2, nf), beta: [0, nf/2))
  int mid;           // 0: off; 1: NM marginal waves per workgroup
  int NM;            // marginal waves (waves 2 + NH ...)
  int off_hring, off_nring, off_mw, mw_bytes;  // LDS: own den / num rows per slot, wave regions
  // the rows the other direction needs (steps i < s0 of each workgroup), as
  // 8-byte {value, tag} granules written by one sc1 store each: a consumer
  // polls its granules until the tags match (MI355X_MICROARCH.md, granule
  // hand-off R2: no progress counter, no publication lag)
  unsigned long long* gden[2];  // [B,T,C]  alpha rows (fwd), beta rows (bwd)
  unsigned long long* gnum[2];  // [B,T,NP] alpha^n rows, beta^n rows
  unsigned epoch;               // per call: tag = epoch * T + t
  unsigned long long* mflag;    // [2][B] band zeroed: (epoch, ~epoch), alpha side then beta side
  // ---- producer helpers (lt_loss_grad_joint): the helpers form each frame's
  // W from the joint weight function's projections (W never in HBM)
  int prod;            // 0: W from HBM; 1: split-bf16 products; 2: bf16 products
  int jH;              // hidden units H (a multiple of 32)
  const float* jpc;    // [C, H]  Pc (the direct path's operand)
  const float* jec;    // [C, H]  e^{2 Pc}
  const float* jpf;    // [B*T, H] Pf
  const float* jef;    // [B*T, H] e^{2 Pf}
  const int* jcbig;    // [1] some |Pc| > kSplitMax
  const int* jfbig;    // [ceil(B*T / 32)] some |Pf| of the 32-row block > kSplitMax
  const float* jwo;    // [R, H] Wo (blank row first)
  const float* jbias;  // [R]
  int off_wo, off_ec;  // LDS: Wo bf16 (hi, lo), e^{2 Pc} fp32 [C][H + 4]
  int off_jf;          // LDS: per producer helper two 1 KB slots of e^{2 Pf} rows
  int off_j32;         // LDS: per producer helper state 32's W rows of its next 32 frames
};
constexpr int kMidBand = 32;    // frames next to the middle zeroed before the granules flow
// floats per slot of the den (hring) and numerator (nring) row rings
constexpr int kHS = 64;

#ifdef LT_STAMPS
#define PSTAMP(a, w, i, k)                                                         \
  do {                                                                             \
    if ((int)blockIdx.x == (a).stamp_block && (a).stamps && (threadIdx.x & 63) == 0) \
      (a).stamps[((long long)(w) * (a).T + (i)) * 4 + (k)] =                        \
          (long long)__builtin_amdgcn_s_memtime();                                  \
  } while (0)
#else
#define PSTAMP(a, w, i, k) \
  do {                     \
  } while (0)
#endif

// control block (ints) at off_ctl
#ifndef LT_PIPE_MID
#define LT_PIPE_MID 2
#endif
constexpr int kPipeMidWaves = LT_PIPE_MID;  // marginal waves per workgroup in mid mode
constexpr int kProdHelpers = kPipeMaxHelpers + kPipeMidWaves;  // producer helpers at most
enum { CTL_TAG = 0, CTL_DEN = kPipeMaxSlots, CTL_NUM, CTL_ABORT, CTL_FIN0, CTL_FIN1, CTL_JBIG,
       CTL_MRG, CTL_N = CTL_MRG + kPipeMidWaves };

typedef __attribute__((address_space(3))) volatile int lds_vint;
typedef __attribute__((address_space(3))) float lds_float;
typedef float lt_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) lt_f4 lds_float4;
typedef __attribute__((address_space(3))) int lds_int;

LT_DEVINL __attribute__((address_space(3))) unsigned char* as3(unsigned char* p) {
  return (__attribute__((address_space(3))) unsigned char*)p;
}

// Bounded wait until *p >= v (LDS word written by another wave). Returns
// false (and raises the abort flag) on timeout or abort. NAP is the s_sleep
// argument between polls (64 clocks each): the recursion waves poll with 1;
// the helper and marginal waves, which run ahead of or behind the chain with
// slack, may nap longer (LT_PIPE_NAP) so their polls take fewer issue slots
// from the chain on the same SIMD.
#ifndef LT_PIPE_ROT
#define LT_PIPE_ROT 0
#endif
#ifndef LT_PIPE_NAP
#define LT_PIPE_NAP 1
#endif
template <int NAP = 1>
LT_DEVINL bool wait_ge(lds_vint* p, int v, lds_vint* abort_flag, int* err) {
  int n = 0;
  while (*p < v) {
    if (*abort_flag) return false;
    __builtin_amdgcn_s_sleep(NAP);
    if (++n > (1 << 21) / NAP) {
      *abort_flag = 1;
      if (err) atomicOr(err, 1);
      return false;
    }
  }
  asm volatile("" ::: "memory");
  return true;
}

LT_DEVINL void lds_release_store(lds_vint* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *p = v;
}

// ---- cross-workgroup stores --------------------------------------------------
// History rows go out with sc1 (write-through) stores; the mid mode's rows for
// the other direction are 8-byte {value, tag} granules (one sc1 store each).
typedef __attribute__((address_space(1))) float g_float;
typedef __attribute__((address_space(1))) int g_int;
LT_DEVINL void st_sc1(float* p, float v) {
  __hip_atomic_store((g_float*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
typedef __attribute__((address_space(1))) unsigned long long g_u64;
LT_DEVINL void st_gran(unsigned long long* p, float v, unsigned tag) {
  const unsigned long long g = (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
  __hip_atomic_store((g_u64*)p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- cross-lane helpers (full exec) -------------------------------------
template <int CTRL>
LT_DEVINL float dpp_mov(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v),
                                                    CTRL, 0xF, 0xF, false));
}
// full-wave max / sum, result uniform
LT_DEVINL float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v, -kInf));
  v = fmaxf(v, dpp_mov<0x4E>(v, -kInf));
  v = fmaxf(v, dpp_mov<0x141>(v, -kInf));
  v = fmaxf(v, dpp_mov<0x140>(v, -kInf));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-kInf),
                                                          __float_as_int(v), 0x142, 0xA, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-kInf),
                                                          __float_as_int(v), 0x143, 0xC, 0xF, false)));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
LT_DEVINL float wave_sum(float v) {
  v += dpp_mov<0xB1>(v, 0.f);
  v += dpp_mov<0x4E>(v, 0.f);
  v += dpp_mov<0x141>(v, 0.f);
  v += dpp_mov<0x140>(v, 0.f);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// sum / max over aligned groups of 2^lg lanes (all lanes of a group end equal)
LT_DEVINL float group_sum_lg(float v, int lg) {
  if (lg > 0) v += dpp_mov<0xB1>(v, 0.f);
  if (lg > 1) v += dpp_mov<0x4E>(v, 0.f);
  if (lg > 2) v += dpp_mov<0x141>(v, 0.f);
  if (lg > 3) v += dpp_mov<0x140>(v, 0.f);
  if (lg > 4) v += __shfl_xor(v, 16);
  if (lg > 5) v += __shfl_xor(v, 32);
  return v;
}
LT_DEVINL float group_max_lg(float v, int lg) {
  if (lg > 0) v = fmaxf(v, dpp_mov<0xB1>(v, -kInf));
  if (lg > 1) v = fmaxf(v, dpp_mov<0x4E>(v, -kInf));
  if (lg > 2) v = fmaxf(v, dpp_mov<0x141>(v, -kInf));
  if (lg > 3) v = fmaxf(v, dpp_mov<0x140>(v, -kInf));
  if (lg > 4) v = fmaxf(v, __shfl_xor(v, 16));
  if (lg > 5) v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}
// value of lane l-1 (lane 0 gets `fill`) / lane l+1 (lane 63 gets `fill`)
LT_DEVINL float from_prev_lane(float v, float fill) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(fill), __float_as_int(v),
                                                    0x138, 0xF, 0xF, false));
}
LT_DEVINL float from_next_lane(float v, float fill) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(fill), __float_as_int(v),
                                                    0x130, 0xF, 0xF, false));
}

LT_DEVINL float safe(float x) { return __builtin_isfinite(x) ? x : 0.f; }

// float-float accumulation of the per-utterance base (two-sum)
LT_DEVINL void ff_add(float& hi, float& lo, float x) {
  const float s = hi + x;
  const float bb = s - hi;
  const float e = (hi - (s - bb)) + (x - bb);
  hi = s;
  lo += e;
}

// ---- denominator wave ----------------------------------------------------
// In-place DPP reductions: one VALU op per stage (s_nop 1 covers the
// VALU-write -> DPP-read hazard); rows outside row_mask keep their value.
LT_DEVINL float wave_max_dpp(float v) {
  asm volatile(
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
LT_DEVINL float wave_sum_dpp(float v) {
  asm volatile(
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// sum over lane pairs (2l, 2l+1)
LT_DEVINL float pair_sum_dpp(float v) {
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
               : "+v"(v));
  return v;
}

typedef float lt_f2 __attribute__((ext_vector_type(2)));

// fwd (REV = false): lane (d, h), d = 1 + (lane >> lgH) in [1, C): destination
//   d, lexical terms from every source k in part h (k = h*J + j < C), plus the
//   blank self loop on h == 0. State 0 (blank only, contexts.py:216-217) is
//   kept exactly in log space on every lane.
// bwd (REV = true): lane (p, h), p in [1, C): source p, lexical terms y = k+1
//   (k = h*J + j < V) plus the blank on h == 0; state 0's V+1 terms are spread
//   one per lane and wave-summed (no other state depends on it in-frame).
//
// Representation: the vector is base + log(g) with g the LINEAR values
// published in gbuf (scaled forward algorithm). A frame is then
//   S_d = sum_k g_k E[k,d]  (+ blank),  E = exp(W - c_t)  (helpers)
//   g'_d = S_d * 2^-e,  base' = base + c_t + e ln 2,
// with e the exponent of the previous frame's max S (lagged, off the chain):
// no transcendental and no reduction on the chain. While every S lies in
// [2^-60, 2^64] each dropped (underflowed) product is below fp32 rounding of
// its sum and every published g >= 2^-124 is exact in log space; otherwise
// the frame is recomputed with the exact safe-max logsumexp
// (semirings.py:279-286) from log(g) (or the exact log values kept after a
// previous fallback) and the raw weights, and the vector is republished
// with its exact max as the new base.
template <int J, bool REV>
LT_DEVINL void den_pipe(const PArgs& a, unsigned char* lds, int b, int nf, int lane) {
  // reset the compiler's view of outstanding loads (other roles' paths):
  // otherwise it waits for vmcnt(0) -- this wave's history stores -- in-loop
  __builtin_amdgcn_s_waitcnt(0x0F70);
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  lds_float* gbuf = (lds_float*)(as3(lds) + a.off_g);
  lds_float* ubuf = (lds_float*)(as3(lds) + a.off_u);
  // lanes per state: compile-time for the J classes with a single H
  constexpr int LGH = J == 17 ? 1 : (J == 5 ? 2 : (J == 2 ? 3 : -1));
  const int C = a.C, V = a.V, R = a.R, JP = a.JP, rowE = a.rowE;
  const int lgH = LGH >= 0 ? LGH : a.lgH;
  const int H = 1 << lgH;
  const int d = 1 + (lane >> lgH);
  const int h = lane & (H - 1);
  const bool act = d < C;
  const int nlex = REV ? V : C;
  auto pos = [&](int k) { return (k / J) * JP + (k % J); };
  // each lane publishes one state: its own, or state 0 (fwd) / nothing
  // (bwd: dummy slot rowE) for lane 1 and lanes without a state
  const bool pub0 = lane == 1 || !act;
  const int pub_pos = pub0 ? (REV ? rowE : 0) : pos(REV ? d - 1 : d);
  const int hist_idx = pub0 ? 0 : d;
  const int nvalid = max(0, min(J, nlex - h * J));  // valid terms of this part
  const int rowi = act ? (REV ? d : d - 1) : 0;
  const int eoff = rowi * rowE + h * JP;              // this lane's E part (floats)
  const int ebi = act ? d : 0;
  const int z_pos = (REV && lane < V) ? pos(lane) : 0;  // bwd state-0 spread
  const lds_float* Gp = gbuf + h * JP;
  // state (relative to base_hi + base_lo)
  float g = (REV && act) ? 1.f : 0.f;  // own state, linear
  float g0 = 1.f;                      // state 0, linear (bwd) / exp(u0) (fwd)
  float u0 = 0.f;                      // fwd state 0, exact log (bwd: in mode 1)
  float uo = (REV && act) ? 0.f : -kInf;  // own state, exact log (mode 1 only)
  int mode = 1;                        // 1: ubuf holds exact logs (after init / fallback)
  int esc = 0;                         // normaliser exponent (lagged)
  float base_hi = 0.f, base_lo = 0.f;
  gbuf[pub_pos] = pub0 ? g0 : g;
  ubuf[pub_pos] = pub0 ? u0 : uo;
  float* hrow = (REV ? a.beta : a.alpha);
  const long long hstep = REV ? -(long long)C : (long long)C;
  lds_float* hring = (lds_float*)(as3(lds) + a.off_hring);  // mid mode
  const int mid_s0 = REV ? nf - nf / 2 : nf / 2;
  if (hrow) hrow += ((long long)b * a.T + (REV ? nf - 1 : 0)) * C + hist_idx;

  // the current step's operands (software-pipelined: step i+1's are loaded
  // while step i's off-chain work runs)
  float gv[J], ev[J];
  float ebl = 0.f, gz = 0.f, ez = 0.f, eb0 = 0.f, ct = 0.f, w00 = 0.f;
  auto load_step = [&](int slot) {
    unsigned char* sb = lds + a.off_ring + slot * a.slot_bytes;
    const lds_float* E = (const lds_float*)(as3(sb) + a.soff_e);
    const lds_float* Eb = (const lds_float*)(as3(sb) + a.soff_eb);
#pragma unroll
    for (int q = 0; q < J / 4; ++q) {
      const lt_f4 g4 = *(const lds_float4*)(Gp + 4 * q);
      const lt_f4 e4 = *(const lds_float4*)(E + eoff + 4 * q);
      gv[4 * q] = g4.x; gv[4 * q + 1] = g4.y; gv[4 * q + 2] = g4.z; gv[4 * q + 3] = g4.w;
      ev[4 * q] = e4.x; ev[4 * q + 1] = e4.y; ev[4 * q + 2] = e4.z; ev[4 * q + 3] = e4.w;
    }
#pragma unroll
    for (int j = 4 * (J / 4); j < J; ++j) {
      gv[j] = Gp[j];
      ev[j] = E[eoff + j];
    }
    ebl = Eb[ebi];
    if constexpr (REV) {
      gz = gbuf[z_pos];
      ez = E[z_pos];
      eb0 = Eb[0];
    }
    ct = *(const lds_float*)(as3(sb) + a.soff_c);
    w00 = *(const lds_float*)as3(sb);
  };
  int slot = 0;
  bool live = nf > 0;
  if (live) {
    live = wait_ge(ctl + CTL_TAG, 1, ctl + CTL_ABORT, a.err);
    asm volatile("" ::: "memory");
    if (live) load_step(0);
  }
  int tag_pref = nf > 1 ? ctl[CTL_TAG + (a.K > 1 ? 1 : 0)] : 0;
  int i = 0;
  for (; live && i < nf; ++i) {
    PSTAMP(a, 0, i, 0);
    const int nslot = (slot + 1 == a.K) ? 0 : slot + 1;
    // ---- the chain: S_d = sum_k g_k E[k,d] over part h (+ blank on h == 0)
    lt_f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < J / 4; ++q) {
      const lt_f2 g01 = {gv[4 * q], gv[4 * q + 1]}, g23 = {gv[4 * q + 2], gv[4 * q + 3]};
      const lt_f2 e01 = {ev[4 * q], ev[4 * q + 1]}, e23 = {ev[4 * q + 2], ev[4 * q + 3]};
      acc0 = __builtin_elementwise_fma(g01, e01, acc0);
      acc1 = __builtin_elementwise_fma(g23, e23, acc1);
    }
    float st = __builtin_fmaf(g, h == 0 ? ebl : 0.f, 0.f);
#pragma unroll
    for (int j = 4 * (J / 4); j < J; ++j) st = __builtin_fmaf(gv[j], ev[j], st);
    float S = ((acc0.x + acc0.y) + (acc1.x + acc1.y)) + st;
    if (LT_ABL(a, 64)) S = gv[0] + ev[0];  // timing ablation
    S = act ? S : 0.f;
    if constexpr (LGH == 1) S = pair_sum_dpp(S);
    else S = group_sum_lg(S, lgH);
    float S0 = 0.f;
    if constexpr (REV) {
      const float tz = __builtin_fmaf(g0, lane == 0 ? eb0 : 0.f, lane < V ? gz * ez : 0.f);
      S0 = wave_sum_dpp(tz);
    }
    // range check: positive finite floats order like their bit patterns
    const unsigned lo_b = 0x21800000u, span = 0x5f800000u - 0x21800000u;
    const bool bad_l = act && ((unsigned)__float_as_uint(S) - lo_b > span);
    bool bad = __builtin_amdgcn_ballot_w64(bad_l) != 0;
    if constexpr (REV) bad = bad || ((unsigned)__float_as_uint(S0) - lo_b > span);
    PSTAMP(a, 0, i, 1);
    // history value of row t: the pre-update vector (lattices.py:462)
    const float hlo = pub0 ? ((REV && !mode) ? lt_log(g0) : u0) : (mode ? uo : lt_log(g));
    const float hval = base_hi + (base_lo + hlo);
    if (a.mid) {
      hring[slot * kHS + hist_idx] = hval;  // the slot's marginal waves read it
      // the other direction turns this frame into marginals: its granule
      if (i < mid_s0) {
        const int t = REV ? nf - 1 - i : i;
        st_gran(a.gden[REV] + ((long long)b * a.T + t) * C + hist_idx, hval,
                a.epoch * (unsigned)a.T + (unsigned)t);
      }
    }
    float shift, gn, g0n;
    if (!bad) {
      // fast path: publish g' = S 2^-e (exact scaling), base += c + e ln2
      gn = __builtin_amdgcn_ldexpf(S, -esc);
      const float esh = (float)esc * 0.6931471805599453f;
      if constexpr (REV) {
        g0n = __builtin_amdgcn_ldexpf(S0, -esc);
      } else {
        u0 = ((u0 + w00) - ct) - esh;  // exact blank self loop of state 0
        g0n = lt_exp(u0);
      }
      gbuf[pub_pos] = pub0 ? g0n : gn;
      shift = ct + esh;
    } else {
      // exact frame from log values (relative to base) and the raw weights
      const lds_float* Wr = (const lds_float*)as3(lds + a.off_ring + slot * a.slot_bytes);
      float x[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int k = h * J + j;
        float xv = -kInf;
        if (act && j < nvalid) {
          float uk = mode ? ubuf[h * JP + j] : lt_log(gv[j]);
          if (!REV && k == 0) uk = u0;
          xv = REV ? uk + Wr[d * R + k + 1] : uk + Wr[k * R + d];
        }
        x[j] = xv;
      }
      const float uown = mode ? uo : lt_log(g);
      const float xb = (act && h == 0) ? uown + Wr[d * R] : -kInf;
      float m1 = xb;
#pragma unroll
      for (int j = 0; j < J; ++j) m1 = fmaxf(m1, x[j]);
      m1 = group_max_lg(m1, lgH);
      const float c1 = safe(m1);
      float s1 = (act && h == 0) ? lt_exp(xb - c1) : 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) s1 += lt_exp(x[j] - c1);
      s1 = group_sum_lg(s1, lgH);
      const float un = act ? c1 + lt_log(s1) : -kInf;  // relative to base
      float u0n;
      if constexpr (REV) {
        const float u0c = mode ? u0 : lt_log(g0);
        float xz = -kInf;
        if (lane == 0) xz = u0c + Wr[0];
        else if (lane <= V) {
          const int zp = pos(lane - 1);
          xz = (mode ? ubuf[zp] : lt_log(gbuf[zp])) + Wr[lane];
        }
        const float cz = safe(wave_max(xz));
        const float sz = wave_sum(lane <= V ? lt_exp(xz - cz) : 0.f);
        u0n = cz + lt_log(sz);
      } else {
        u0n = u0 + w00;
      }
      // republish relative to the exact max of the new vector
      const float mnew = safe(wave_max(fmaxf(un, u0n)));
      const float unr = un - mnew, u0r = u0n - mnew;
      gn = act ? lt_exp(unr) : 0.f;
      g0n = lt_exp(u0r);
      gbuf[pub_pos] = pub0 ? g0n : gn;
      ubuf[pub_pos] = pub0 ? u0r : unr;
      uo = unr;
      u0 = u0r;
      shift = mnew;
    }
    // ---- next step's operands (after the publish: LDS is in order per wave)
    if (i + 1 < nf) {
      if (tag_pref < i + 2 && !wait_ge(ctl + CTL_TAG + nslot, i + 2, ctl + CTL_ABORT, a.err))
        live = false;
      asm volatile("" ::: "memory");
      if (live) {
        load_step(nslot);
        tag_pref = ctl[CTL_TAG + ((nslot + 1 == a.K) ? 0 : nslot + 1)];
      }
    }
    // ---- off-chain work of step i
    if (hrow && !LT_ABL(a, 4)) {
      st_sc1(hrow, hval);
      hrow += hstep;
    }
    if (!bad) {
      // next normaliser: exponent of this frame's max S
      float mx = act ? S : 0.f;
      if constexpr (REV) mx = fmaxf(mx, S0);
      if (LT_ABL(a, 32))  // timing ablation: cheap normaliser
        esc = __builtin_amdgcn_frexp_expf(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(S))));
      else
        esc = __builtin_amdgcn_frexp_expf(wave_max_dpp(mx));
      mode = 0;
    } else {
      esc = 0;
      mode = 1;
    }
    g = act ? gn : 0.f;
    g0 = g0n;
    if (!LT_ABL(a, 32)) ff_add(base_hi, base_lo, shift);
    // slot of step i consumed (its reads were used above)
    asm volatile("" ::: "memory");
    if (lane == 0) *(ctl + CTL_DEN) = i + 1;
    PSTAMP(a, 0, i, 2);
    slot = nslot;
  }
  // final vector: padding rows (fwd, lattices.py:460-461) and log_z
  if (!REV) {
    const float lown = mode ? uo : lt_log(g);
    if (a.alpha) {
      const long long r0 = (long long)b * a.T;
      for (int t = nf; t < a.T; ++t)
        a.alpha[(r0 + t) * C + hist_idx] = base_hi + (base_lo + (pub0 ? u0 : lown));
    }
    // (+)_q alpha_T[q] (lattices.py:496): safe-max logsumexp
    const bool own = act && h == 0;
    const float mx = wave_max(fmaxf(own ? lown : -kInf, lane == 0 ? u0 : -kInf));
    const float c = safe(mx);
    float e = 0.f;
    if (own) e += lt_exp(lown - c);
    if (lane == 0) e += lt_exp(u0 - c);
    const float s = wave_sum(e);
    // log_z = base + c + log(s) (the base only shifts finite values)
    const float rel = c + lt_log(s);
    const float lz = __builtin_isfinite(rel) ? base_hi + (base_lo + rel) : rel;
    if (lane == 0) {
      ((lds_float*)(as3(lds) + a.off_ctl))[CTL_FIN0] = lz;
      if (a.log_z) a.log_z[b] = lz;
    }
  }
}

// ---- numerator wave --------------------------------------------------------
// Positions u = PN*lane + s. fwd: a'[u] = a[u] W[c_u,0] (+) a[u-1] W[c_{u-1},y_u]
// (alignments.py:320-329, lattices.py:314-338); bwd is its transpose.
template <int PN, bool REV>
LT_DEVINL void num_pipe(const PArgs& a, unsigned char* lds, int b, int nf, int lane) {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // see den_pipe
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  const lds_int* ctx = (const lds_int*)(as3(lds) + a.off_ctx);
  const lds_int* ylab = (const lds_int*)(as3(lds) + a.off_ylab);
  const int NP = a.U + 1, U = a.U;
  int ob[PN], ol[PN];
  float v[PN], o[PN];
  const int nl = a.nlab[b];
#pragma unroll
  for (int s = 0; s < PN; ++s) {
    const int u = PN * lane + s;
    ob[s] = 0;
    ol[s] = 0;
    if (u < NP) {
      ob[s] = ctx[u];
      if (!REV) ol[s] = u >= 1 ? ctx[u - 1] + ylab[u - 1] : 0;
      else ol[s] = u < U ? ctx[u] + ylab[u] : 0;
    }
    v[s] = 0.f;
    if (!REV) o[s] = (u == 0) ? 0.f : -kInf;
    else o[s] = (u == nl) ? 0.f : -kInf;
  }
  // every position is an exact integer part o plus a fraction v in [0, 1)
  // (lae_split, lt_kernels.h): the positions span hundreds of nats within a
  // frame, and a value kept relative to one offset per frame was rounded at
  // its own magnitude every frame (round 3: up to 26 units of 2^-24 |num|
  // after 1,000 frames, tools/ck_precision.py). History rows and num are
  // o + v, rounded once.
  float* hist = REV ? a.beta_num : a.alpha_num;
  lds_float* nring = (lds_float*)(as3(lds) + a.off_nring);  // mid mode
  int tag_next = nf > 0 ? ctl[CTL_TAG] : 0;
  const long long row0 = (long long)b * a.T;
  int slot = 0;
  for (int i = 0; i < nf; ++i, slot = (slot + 1 == a.K) ? 0 : slot + 1) {
    const int t = REV ? nf - 1 - i : i;
    PSTAMP(a, 1, i, 0);
    if (tag_next < i + 1 && !wait_ge(ctl + CTL_TAG + slot, i + 1, ctl + CTL_ABORT, a.err)) break;
    asm volatile("" ::: "memory");
    PSTAMP(a, 1, i, 1);
    const lds_float* Wr = (const lds_float*)as3(lds + a.off_ring + slot * a.slot_bytes);
    tag_next = ctl[CTL_TAG + ((slot + 1 == a.K) ? 0 : slot + 1)];
    float wb[PN], wl[PN];
#pragma unroll
    for (int s = 0; s < PN; ++s) {
      wb[s] = Wr[ob[s]];
      wl[s] = Wr[ol[s]];
    }
    if (a.mid) {
      const bool gr = i < (REV ? nf - nf / 2 : nf / 2);
      unsigned long long* gp = a.gnum[REV] + (row0 + t) * NP;
      const unsigned tag = a.epoch * (unsigned)a.T + (unsigned)t;
#pragma unroll
      for (int s = 0; s < PN; ++s)
        if (PN * lane + s < NP) {
          nring[slot * NP + PN * lane + s] = o[s] + v[s];
          if (gr) st_gran(gp + PN * lane + s, o[s] + v[s], tag);
        }
    }
    if (hist && !LT_ABL(a, 8)) {
      float* hr = hist + (row0 + t) * NP;
#pragma unroll
      for (int s = 0; s < PN; ++s)
        if (PN * lane + s < NP) st_sc1(hr + PN * lane + s, o[s] + v[s]);
    }
    if (LT_ABL(a, 16)) {  // timing ablation: no numerator arithmetic
#pragma unroll
      for (int s = 0; s < PN; ++s) v[s] = v[s] + wb[s] + wl[s];
    } else
    if constexpr (!REV) {
      const float pv = from_prev_lane(v[PN - 1], 0.f), po = from_prev_lane(o[PN - 1], -kInf);
      float no[PN], nv[PN];
#pragma unroll
      for (int s = 0; s < PN; ++s) {
        const int u = PN * lane + s;
        const float lo = s == 0 ? po : o[s - 1], lv = s == 0 ? pv : v[s - 1];
        lae_split(o[s], v[s] + wb[s], u >= 1 ? lo : -kInf, lv + wl[s], no[s], nv[s]);
        if (u >= NP) no[s] = -kInf;
      }
#pragma unroll
      for (int s = 0; s < PN; ++s) {
        o[s] = no[s];
        v[s] = nv[s];
      }
    } else {
      const float nxv = from_next_lane(v[0], 0.f), nxo = from_next_lane(o[0], -kInf);
      float no[PN], nv[PN];
#pragma unroll
      for (int s = 0; s < PN; ++s) {
        const int u = PN * lane + s;
        const float ro = s == PN - 1 ? nxo : o[s + 1], rv = s == PN - 1 ? nxv : v[s + 1];
        lae_split(o[s], wb[s] + v[s], u < U ? ro : -kInf, wl[s] + rv, no[s], nv[s]);
        if (u >= NP) no[s] = -kInf;
      }
#pragma unroll
      for (int s = 0; s < PN; ++s) {
        o[s] = no[s];
        v[s] = nv[s];
      }
    }
    asm volatile("" ::: "memory");  // LDS is in order per wave: no wait
    if (lane == 0) *(ctl + CTL_NUM) = i + 1;
    PSTAMP(a, 1, i, 2);
  }
  if (!REV) {
    if (a.alpha_num) {
      for (int t = nf; t < a.T; ++t) {
        float* hr = a.alpha_num + (row0 + t) * NP;
#pragma unroll
        for (int s = 0; s < PN; ++s)
          if (PN * lane + s < NP) hr[PN * lane + s] = o[s] + v[s];
      }
    }
    // lattices.py:375-377
#pragma unroll
    for (int s = 0; s < PN; ++s) {
      const int u = PN * lane + s;
      if (u < NP && u == nl) {
        ((lds_float*)(as3(lds) + a.off_ctl))[CTL_FIN1] = o[s] + v[s];
        if (a.num) a.num[b] = o[s] + v[s];
      }
    }
    if (lane == 0 && !(nl >= 0 && nl <= U)) {
      ((lds_float*)(as3(lds) + a.off_ctl))[CTL_FIN1] = -kInf;
      if (a.num) a.num[b] = -kInf;
    }
  }
}

// ---- helper waves ----------------------------------------------------------
// Helper hw handles steps hw, hw + NH, ...: loads frame t's weights (element
// e = lane + 64k, coalesced), the frame max c, E = exp(W - c) scattered into
// the consumer layout, raw W (fp32) for the numerator, then the slot tag.
// Loads are unconditional (NL per lane, a compile-time count) and every
// step issues exactly NL of them, so the compiler's in-order vmcnt waits
// leave the D-1 younger frames in flight; elements past the frame go to
// padding / a trash word, so the per-element work is branch-free.
template <bool BF16, int NL, bool REV>
LT_DEVINL void helper_pipe(const PArgs& a, unsigned char* lds, int b, int nf, int hw, int lane) {
  constexpr int D = 60 / NL < 8 ? 60 / NL : 8;  // frames in flight per helper (vmcnt <= 63)
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  const int FR = a.FR, R = a.R, NH = a.NH;
  const int es = BF16 ? 2 : 4;
  // scattered E offsets (bytes inside a slot) of this lane's elements
  int pe[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int e = lane + 64 * k;
    int o = a.soff_c + 8;  // trash word
    if (e < FR) {
      const int p = e / R, y = e - (e / R) * R;
      if (y == 0) {
        o = a.soff_eb + 4 * p;
      } else {
        const int row = REV ? p : y - 1;
        const int kk = REV ? y - 1 : p;
        o = a.soff_e + 4 * (row * a.rowE + (kk / a.J) * a.JP + (kk % a.J));
      }
    }
    pe[k] = o;
  }
  // W through a buffer descriptor: the frame's byte offset in soffset, the
  // lane's element in voffset; reads past the tensor return 0 (range check),
  // reads past the frame are ignored below
  const unsigned nbytes = (unsigned)__builtin_amdgcn_readfirstlane((int)a.w_bytes);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.W, (short)0, (int)nbytes, 0x00020000);
  const long long ub = (long long)b * a.T;
  if (nf <= 0) return;
  auto issue = [&](float* w, int i) {
    int ii = i < nf ? i : nf - 1;
    const int t = REV ? nf - 1 - ii : ii;
    // frame offset in the voffset (the range check covers voffset + imm)
    const unsigned foff =
        (unsigned)__builtin_amdgcn_readfirstlane((int)((ub + t) * (long long)FR * es));
    const unsigned vb = foff + (unsigned)(lane * es);
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int vo = (int)(vb + (unsigned)(64 * k * es));
      if constexpr (BF16)
        w[k] = __uint_as_float(((unsigned)__builtin_amdgcn_raw_buffer_load_b16(rsrc, vo, 0, 0))
                               << 16);
      else
        w[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, vo, 0, 0));
    }
    asm volatile("" ::: "memory");
  };
  int seen_den = 0, seen_num = 0;
  // mid mode: the first step whose frame this workgroup turns into marginals
  const int s0 = REV ? nf - nf / 2 : nf / 2;
  int slot = hw;  // slot of step i (advanced by NH per processed step; NH <= K)
  auto process = [&](const float* w, int i) -> bool {
    // the slot's previous frame (step i-K) must be consumed
    const int need = i - a.K + 1;
    PSTAMP(a, 2 + hw, i, 0);
    if (need > 0) {
      if (seen_den < need) {
        if (!wait_ge<LT_PIPE_NAP>(ctl + CTL_DEN, need, ctl + CTL_ABORT, a.err)) return false;
        seen_den = ctl[CTL_DEN];
      }
      if (seen_num < need) {
        if (!wait_ge<LT_PIPE_NAP>(ctl + CTL_NUM, need, ctl + CTL_ABORT, a.err)) return false;
        seen_num = ctl[CTL_NUM];
      }
      // mid mode: the marginal wave of the slot's previous step (need - 1)
      if (a.mid && need - 1 >= s0 &&
          !wait_ge<LT_PIPE_NAP>(ctl + CTL_MRG + (need - 1 - s0) % a.NM, need, ctl + CTL_ABORT, a.err))
        return false;
    }
    PSTAMP(a, 2 + hw, i, 1);
    float mx = -kInf;
#pragma unroll
    for (int k = 0; k < NL; ++k) mx = fmaxf(mx, lane + 64 * k < FR ? w[k] : -kInf);
    const float c = safe(wave_max(mx));
    const float cl = c * kLog2e;
    unsigned char* sb = lds + a.off_ring + slot * a.slot_bytes;
    lds_float* Wr = (lds_float*)as3(sb);
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      if (!LT_ABL(a, 1)) Wr[lane + 64 * k] = w[k];
      if (!LT_ABL(a, 2)) *(lds_float*)(as3(sb) + pe[k]) = lt_exp_off(w[k], cl);
    }
    if (lane == 0) {
      *(lds_float*)(as3(sb) + a.soff_c) = c;
      lds_release_store(ctl + CTL_TAG + slot, i + 1);
    }
    PSTAMP(a, 2 + hw, i, 2);
    return true;
  };
  float wv[D][NL];
#pragma unroll
  for (int r = 0; r < D; ++r) issue(wv[r], hw + r * NH);
  bool ok = true;
  for (int i0 = hw; i0 < nf; i0 += NH * D) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      const int i = i0 + r * NH;
      if (ok && i < nf) {
        ok = process(wv[r], i);
        slot += NH;
        if (slot >= a.K) slot -= a.K;
      }
      issue(wv[r], i + NH * D);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- producer helpers (lt_loss_grad_joint) ----------------------------------
// Helper hw forms frame t's arc weights itself instead of loading them: the
// joint weight function W[p, y] = bias[y] + sum_h Wo[y, h] tanh(Pc[p, h] +
// Pf[f, h]) (weight_fns.py:174-227) as two 32-state row tiles (states 0..31,
// then 32) x two 32-label column tiles on the matrix cores -- joint_tile,
// the producer's own K steps, so every element is bit-identical to
// lt_joint_weights_ex's W -- then the frame max, raw W and E = exp(W - c)
// into the slot as helper_pipe leaves them. The split (e^{2 Pc} e^{2 Pf}) or
// direct tanh is chosen per 32-row block of Pf as lt_joint_weights does. W
// never exists in HBM; the helpers work in the shadow of the frame chain.
template <bool REV, bool SP, int J>
LT_DEVINL void helper_prod(const PArgs& a, unsigned char* lds, int b, int nf, int hw, int lane) {
  constexpr int JP = J >= 4 ? (J + 3) / 4 * 4 : J;  // launch_pipe's padded part length
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  const int R = a.R, C = a.C, H = a.jH, HP = H + 8;
  const int WL = (R * HP + 7) & ~7;
  const unsigned short* wo = (const unsigned short*)(lds + a.off_wo);
  const float* ecl = (const float*)(lds + a.off_ec);
  const bool csplit = *a.jcbig == 0;
  const int r = lane & 31, hk = 8 * (lane >> 5), half = lane >> 5;
  const int y0 = r, y1 = 32 + r;
  const bool v0 = y0 < R, v1 = y1 < R;
  const float b0 = v0 ? a.jbias[y0] : 0.f, b1 = v1 ? a.jbias[y1] : 0.f;
  const unsigned short* w0 = wo + (v0 ? y0 : R - 1) * HP + hk;
  const unsigned short* w1 = wo + (v1 ? y1 : R - 1) * HP + hk;
  const unsigned short* w0l = w0 + WL;
  const unsigned short* w1l = w1 + WL;
  // the two row tiles' e^{2 Pc} rows (states r and 32 + r; rows past C
  // repeat the last state and are never stored)
  const float* ec0 = ecl + min(r, C - 1) * (H + 4) + hk;
  const float* ec1 = ecl + min(32 + r, C - 1) * (H + 4) + hk;
  // E's byte offset in a slot for element (p, y) (helper_pipe's layout):
  // y is fixed per lane and p an unrolled constant plus 4 half, so with J a
  // compile-time constant no element pays a division
  auto eoff = [&](int p, int y) {
    if (y == 0) return a.soff_eb + 4 * p;
    const int row = REV ? p : y - 1, kk = REV ? y - 1 : p;
    return a.soff_e + 4 * (row * a.rowE + (kk / J) * JP + (kk % J));
  };
  // e^{2 Pf} rows come through a two-slot LDS ring of this helper, one
  // LDS-DMA instruction a frame issued a step ahead, so no frame waits on
  // its own global load
  unsigned char* ring = lds + a.off_jf + hw * 2048;
  const unsigned ring_a = lds_base_addr(ring);
  auto row_of = [&](int i) {
    const int t = REV ? nf - 1 - i : i;
    return (long long)b * a.T + t;
  };
  auto issue = [&](int i, int sl) {
    const long long f = row_of(min(i, nf - 1));
    glds16(a.jef + f * H + 4 * min(lane, H / 4 - 1), ring_a + 1024u * sl);
  };
  int seen_den = 0, seen_num = 0;
  int slot = hw, rs = 0;
  // the prologue's per-utterance flag: no 32-row block of this utterance's
  // Pf rows exceeds kSplitMax (the common case: no per-frame flag read, whose
  // scalar load would share lgkmcnt with every LDS wait of the frame)
  const bool utt_split = *(const lds_vint*)(as3(lds) + a.off_ctl + 4 * CTL_JBIG) == 0;
  // state 32 (C = 33) fills one row of a 32-row tile: with every frame on the
  // split path its W rows are formed 32 frames at a time (tile rows = this
  // helper's next 32 frames; an element's value does not depend on the other
  // rows of its tile) and kept in LDS
  const bool batch32 = C > 32 && csplit && utt_split;
  lds_float* s32 = (lds_float*)(as3(lds) + a.off_j32 + hw * ((32 * R * 4 + 15) & ~15));
  const float* ec32 = ecl + 32 * (H + 4) + hk;
  int bn = 0;  // frames this helper has processed
  if (hw < nf) issue(hw, 0);
  for (int i = hw; i < nf; i += a.NH, rs ^= 1, ++bn) {
    PSTAMP(a, 2 + hw, i, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this frame's row is in the ring
    issue(i + a.NH, rs ^ 1);                             // the next one in flight
    const long long f = row_of(i);
    const bool split = csplit && (utt_split || a.jfbig[f >> 5] == 0);
    const float* efr = (const float*)(ring + 1024 * rs) + hk;
    const int need = i - a.K + 1;  // the slot's previous frame (step i - K) must be consumed
    if (need > 0) {
      if (seen_den < need) {
        if (!wait_ge<LT_PIPE_NAP>(ctl + CTL_DEN, need, ctl + CTL_ABORT, a.err)) break;
        seen_den = ctl[CTL_DEN];
      }
      if (seen_num < need) {
        if (!wait_ge<LT_PIPE_NAP>(ctl + CTL_NUM, need, ctl + CTL_ABORT, a.err)) break;
        seen_num = ctl[CTL_NUM];
      }
    }
    PSTAMP(a, 2 + hw, i, 1);
    unsigned char* sb = lds + a.off_ring + slot * a.slot_bytes;
    lds_float* Wr = (lds_float*)as3(sb);
    // W = acc + bias (the producer's own rounding) into the slot's raw W and
    // kept in registers for E = exp(W - c) once the frame max is known. Row
    // tile 0 holds states 0..31; of row tile 1 only state 32 (k = 0 of the
    // lower half) exists, since C <= 33 here (V <= 32, one context label).
    f32x16 x0 = {}, x1 = {};
    if (split) {
      joint_tile<SP, true>(true, ec0, efr, H, w0, w1, w0l, w1l, x0, x1);
    } else {  // a projection beyond kSplitMax: the direct tanh from Pc + Pf (rare)
      joint_tile<SP, true>(false, a.jpc + min(r, C - 1) * H + hk, a.jpf + f * H + hk, H, w0, w1,
                           w0l, w1l, x0, x1);
    }
    float mx = -kInf;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int p = (k & 3) + 8 * (k >> 2) + 4 * half;
      x0[k] += b0;
      x1[k] += b1;
      Wr[p * R + y0] = x0[k];
      if (v1) Wr[p * R + y1] = x1[k];
      mx = fmaxf(mx, v1 ? fmaxf(x0[k], x1[k]) : x0[k]);
    }
    float z0 = 0.f, z1 = 0.f;
    const bool last = C > 32 && half == 0;  // this lane holds state 32's W
    if (batch32) {
      if ((bn & 31) == 0) {  // rows: frames i + NH q, q = 0..31 (clamped)
        const int fi = min(i + a.NH * r, nf - 1);
        const float* efq = a.jef + row_of(fi) * H + hk;
        f32x16 t0 = {}, t1 = {};
        joint_tile<SP, true>(true, ec32, efq, H, w0, w1, w0l, w1l, t0, t1);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int q = (k & 3) + 8 * (k >> 2) + 4 * half;
          s32[q * R + y0] = t0[k] + b0;
          if (v1) s32[q * R + y1] = t1[k] + b1;
        }
      }
      if (last) {
        const int q = bn & 31;
        z0 = s32[q * R + y0];
        Wr[32 * R + y0] = z0;
        if (v1) {
          z1 = s32[q * R + y1];
          Wr[32 * R + y1] = z1;
        }
        mx = fmaxf(mx, v1 ? fmaxf(z0, z1) : z0);
      }
    } else if (C > 32) {
      f32x16 t0 = {}, t1 = {};
      if (split) {
        joint_tile<SP, true>(true, ec1, efr, H, w0, w1, w0l, w1l, t0, t1);
      } else {
        joint_tile<SP, true>(false, a.jpc + min(32 + r, C - 1) * H + hk, a.jpf + f * H + hk, H,
                             w0, w1, w0l, w1l, t0, t1);
      }
      z0 = t0[0] + b0;
      z1 = t1[0] + b1;
      if (last) {
        Wr[32 * R + y0] = z0;
        if (v1) Wr[32 * R + y1] = z1;
        mx = fmaxf(mx, v1 ? fmaxf(z0, z1) : z0);
      }
    }
    const float c = safe(wave_max(mx));
    const float cl = c * kLog2e;
    PSTAMP(a, 2 + hw, i, 2);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int p = (k & 3) + 8 * (k >> 2) + 4 * half;
      *(lds_float*)(as3(sb) + eoff(p, y0)) = lt_exp_off(x0[k], cl);
      if (v1) *(lds_float*)(as3(sb) + eoff(p, y1)) = lt_exp_off(x1[k], cl);
    }
    if (last) {
      *(lds_float*)(as3(sb) + eoff(32, y0)) = lt_exp_off(z0, cl);
      if (v1) *(lds_float*)(as3(sb) + eoff(32, y1)) = lt_exp_off(z1, cl);
    }
    if (lane == 0) {
      *(lds_float*)(as3(sb) + a.soff_c) = c;
      lds_release_store(ctl + CTL_TAG + slot, i + 1);
    }
    PSTAMP(a, 2 + hw, i, 3);
    slot += a.NH;
    if (slot >= a.K) slot -= a.K;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS outlives the wave
}

// ---- in-workgroup marginals (mid mode) --------------------------------------
// Marginal wave m of a recursion workgroup turns the frames of its steps
// i = s0 + m, s0 + m + NM, ... (the workgroup's far half: alpha frames
// [nf/2, nf), beta frames [0, nf/2)) into dW while the frame is still in the
// ring: the workgroup's own den / numerator rows of the step from LDS (hring,
// nring: the pre-update vectors the den and numerator waves leave there with
// the step), the other direction's rows of the frame from its granules (that
// direction passed the frame in its own first half).
//
// dW[b,t,p,y] = den - num marginals of frame t (alignments.py:311-317 for the
// denominator; the string arcs of lattices.py:314-338 for the numerator,
// summed per lattice arc in LDS, one wave's adds in program and lane order:
// deterministic). Each frame is normalised by its own total,
//   log_z = logsumexp_{p,y} alpha_t[p] + W_t[p,y] + beta_{t+1}[next(p,y)]
// (the forward-backward identity holds at every live frame), and likewise the
// numerator, so no frame waits for the end of the other pass. A frame whose
// total is zero (log_z = -inf, or an unreachable string) gets dW = 0, as
// lt_loss_backward does for those utterances.
template <bool BF16, int NL, int PN, bool EXACT, bool REV>
LT_DEVINL void mid_marg(const PArgs& a, unsigned char* lds, int b, int nf, int m, int lane) {
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  const lds_int* ctx = (const lds_int*)(as3(lds) + a.off_ctx);
  const lds_int* ylab = (const lds_int*)(as3(lds) + a.off_ylab);
  const lds_float* hring = (const lds_float*)(as3(lds) + a.off_hring);
  const lds_float* nring = (const lds_float*)(as3(lds) + a.off_nring);
  const int C = a.C, R = a.R, FR = a.FR, NP = a.U + 1, NK = 2 * NP, U = a.U, T = a.T;
  const bool do_den = a.flags & F_DEN;
  constexpr int es = BF16 ? 2 : 4;
  constexpr int NKL = 2 * PN;
  lds_float* A = (lds_float*)(as3(lds) + a.off_mw + m * a.mw_bytes);  // [64]
  lds_float* Bt = A + 64;         // [64]
  lds_float* AN = Bt + 64;        // [64 PN]
  lds_float* BN = AN + 64 * PN;   // [64 PN]
  lds_float* Sub = BN + 64 * PN;  // [64 NL]
  lds_float* AL = Sub + 64 * NL;  // [64] exp(alpha - max alpha)
  lds_float* BL = AL + 64;        // [64] exp(beta - max beta)
  // elements e = lane + 64k: source p, destination q (n = 1: the blank stays
  // in p, label y goes to state y; contexts.py:190-205); past the frame A[63]
  // packed per element: the byte offset of its E = exp(W - c) in the slot
  // (helper_pipe's consumer layout) in bits 0-15, p in 16-23, q in 24-31; the
  // den marginal of a frame is then a product of three linear factors, no
  // exp per element
  int pk[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int e = lane + 64 * k;
    int o = a.soff_c + 8, p = 63, q = 63;
    if (e < FR) {
      p = e / R;
      const int y = e - p * R;
      q = y == 0 ? p : y;
      if (y == 0) {
        o = a.soff_eb + 4 * p;
      } else {
        const int row = REV ? p : y - 1;
        const int kk = REV ? y - 1 : p;
        o = a.soff_e + 4 * (row * a.rowE + (kk / a.J) * a.JP + (kk % a.J));
      }
    }
    pk[k] = o | (p << 16) | (q << 24);
  }
  auto pof = [&](int k) { return (pk[k] >> 16) & 0xff; };
  auto qof = [&](int k) { return (int)((unsigned)pk[k] >> 24); };
  auto partial = [&](int k) { return EXACT ? k == NL - 1 : 64 * (k + 1) > FR; };
  // numerator arc slots kk = lane + 64 s: the arc's element (-1: none) and
  // its positions u and u or u+1 (lattices.py:314-338)
  int on[NKL], uab[NKL];
#pragma unroll
  for (int s2 = 0; s2 < NKL; ++s2) {
    const int kk = lane + 64 * s2;
    const int u = min(kk >> 1, NP - 1);
    uab[s2] = u | (min((kk & 1) ? u + 1 : u, NP - 1) << 16);
    int o = -1;
    if (kk < NK) {
      const int uu = kk >> 1;
      o = (kk & 1) == 0 ? ctx[uu] : (uu < U ? ctx[uu] + ylab[uu] : -1);
    }
    on[s2] = o;
  }
  const unsigned nbytes = (unsigned)__builtin_amdgcn_readfirstlane((int)a.w_bytes);
  const __amdgpu_buffer_rsrc_t dr =
      __builtin_amdgcn_make_buffer_rsrc(a.dW, (short)0, (int)nbytes, 0x00020000);
  constexpr unsigned kOff = 0xFFFFFFF0u;
  const int s0 = REV ? nf - nf / 2 : nf / 2;
  const long long ub = (long long)b * T;
  const unsigned long long* god = a.gden[REV ? 0 : 1];  // the other direction's rows
  const unsigned long long* gon = a.gnum[REV ? 0 : 1];
  auto store_frame = [&](int t, const float* x) {
    const unsigned vb = (unsigned)__builtin_amdgcn_readfirstlane((int)((ub + t) * (long long)FR * es)) +
                        (unsigned)(lane * es);
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      int vo = (int)(vb + (unsigned)(64 * k * es));
      if (partial(k) && lane + 64 * k >= FR) vo = (int)kOff;
      if constexpr (BF16)
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(x[k]), dr, vo, 0, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x[k]), dr, vo, 0, 0);
    }
  };
  // the other direction's granules of a step, prefetched one assigned step
  // ahead so their latency hides under the current frame's work
  unsigned long long gd = 0, gn[PN];
#pragma unroll
  for (int s2 = 0; s2 < PN; ++s2) gn[s2] = 0;
  auto fetch = [&](int i) {
    const int t = REV ? nf - 1 - i : i;
    if (do_den && lane < C)
      gd = __hip_atomic_load((const g_u64*)(god + (ub + t) * C + lane), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int s2 = 0; s2 < PN; ++s2) {
      const int u = lane + 64 * s2;
      if (u < NP)
        gn[s2] = __hip_atomic_load((const g_u64*)(gon + (ub + t) * NP + u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  auto tags_ok = [&](unsigned tag) {
    bool got = !(do_den && lane < C) || (unsigned)(gd >> 32) == tag;
#pragma unroll
    for (int s2 = 0; s2 < PN; ++s2)
      got = got && (lane + 64 * s2 >= NP || (unsigned)(gn[s2] >> 32) == tag);
    return got;
  };
  if (s0 + m < nf) fetch(s0 + m);
  for (int i = s0 + m; i < nf; i += a.NM) {
    const int t = REV ? nf - 1 - i : i;
    const int slot = i % a.K;
    // the own recursions are past step i: their rows of the step are in the rings
    if (do_den && !wait_ge<LT_PIPE_NAP>(ctl + CTL_DEN, i + 1, ctl + CTL_ABORT, a.err)) break;
    if (!wait_ge<LT_PIPE_NAP>(ctl + CTL_NUM, i + 1, ctl + CTL_ABORT, a.err)) break;
    // the other direction's rows of frame t: the prefetched granules, else
    // poll until every lane's tag matches (bounded; an abort drains)
    const unsigned tag = a.epoch * (unsigned)T + (unsigned)t;
    if (__builtin_amdgcn_ballot_w64(!tags_ok(tag)) != 0) {
      int n = 0;
      bool ok = true;
      for (;;) {
        __builtin_amdgcn_s_sleep(2);
        fetch(i);
        if (__builtin_amdgcn_ballot_w64(!tags_ok(tag)) == 0) break;
        if (*(ctl + CTL_ABORT)) { ok = false; break; }
        if (++n > (1 << 22)) {
          *(ctl + CTL_ABORT) = 1;
          if (a.err) atomicOr(a.err, 2);
          ok = false;
          break;
        }
      }
      if (!ok) break;
    }
    const float od = do_den ? __uint_as_float((unsigned)gd) : -kInf;
    float onv[PN];
#pragma unroll
    for (int s2 = 0; s2 < PN; ++s2)
      onv[s2] = lane + 64 * s2 < NP ? __uint_as_float((unsigned)gn[s2]) : -kInf;
    if (i + a.NM < nf) fetch(i + a.NM);
    // frame t's rows into this wave's region (A[lanes >= C] = -inf serves the
    // elements past the frame)
    const lds_float* hr = hring + slot * kHS;
    const lds_float* nr = nring + slot * NP;
    const float own = (do_den && lane < C) ? hr[lane] : -kInf;
    if constexpr (!REV) {  // own alpha_t, alpha^n_t; the beta side's beta_{t+1}, beta^n_{t+1}
      A[lane] = (do_den && lane < C) ? own : -kInf;
      Bt[lane] = (do_den && lane < C) ? od : 0.f;
#pragma unroll
      for (int s2 = 0; s2 < PN; ++s2) {
        const int u = lane + 64 * s2;
        AN[u] = u < NP ? nr[u] : -kInf;
        BN[u] = onv[s2];
      }
    } else {  // own beta_{t+1}, beta^n_{t+1}; the alpha side's alpha_t, alpha^n_t
      A[lane] = (do_den && lane < C) ? od : -kInf;
      Bt[lane] = (do_den && lane < C) ? own : 0.f;
#pragma unroll
      for (int s2 = 0; s2 < PN; ++s2) {
        const int u = lane + 64 * s2;
        AN[u] = onv[s2];
        BN[u] = u < NP ? nr[u] : -kInf;
      }
    }
    // linear factors of the two den rows, each over its own max
    const float va = (do_den && lane < C) ? (REV ? od : own) : -kInf;
    const float vb = (do_den && lane < C) ? (REV ? own : od) : -kInf;
    const float ma = safe(wave_max(va)), mb = safe(wave_max(vb));
    AL[lane] = lane < C ? lt_exp(va - ma) : 0.f;
    BL[lane] = lane < C ? lt_exp(vb - mb) : 0.f;
#pragma unroll
    for (int k = 0; k < NL; ++k) Sub[lane + 64 * k] = 0.f;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* sb = lds + a.off_ring + slot * a.slot_bytes;
    // the frame's raw weights (fp32) staged in the slot by the helpers
    const lds_float* Wr = (const lds_float*)as3((unsigned char*)sb);
    float x[NL];
    // den marginals exp(alpha + w + beta) / frame total as the products
    // exp(alpha - ma) exp(w - c) exp(beta - mb) over their sum: every product
    // is <= 1 and a dropped (underflowed) one is below 2^-126; with the sum at
    // or above 2^-64 that is below fp32 rounding of any marginal that matters.
    // Below it (or on a non-finite sum) the frame runs the exact log-space
    // sum with the safe max (semirings.py:279-286).
    float sd = 0.f;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const float ev = *(const lds_float*)as3((unsigned char*)sb + (pk[k] & 0xffff));
      const float pr = AL[pof(k)] * ev * BL[qof(k)];
      x[k] = (partial(k) && lane + 64 * k >= FR) ? 0.f : pr;
      sd += x[k];
    }
    sd = wave_sum(sd);
    if (do_den && !(sd >= 0x1p-64f && sd < kInf)) {
      float m1 = -kInf;
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        float w = Wr[lane + 64 * k];
        if (partial(k) && lane + 64 * k >= FR) w = -kInf;  // the next frame's weight
        x[k] = A[pof(k)] + w + Bt[qof(k)];
        m1 = fmaxf(m1, x[k]);
      }
      const float md = safe(wave_max(m1));
      sd = 0.f;
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        x[k] = lt_exp(x[k] - md);
        sd += x[k];
      }
      sd = wave_sum(sd);
    }
    const float rd = (do_den && sd > 0.f && sd < kInf) ? __builtin_amdgcn_rcpf(sd) : 0.f;
    float xn[NKL];
    float mn = -kInf;
#pragma unroll
    for (int s2 = 0; s2 < NKL; ++s2) {
      const float w = on[s2] >= 0 ? Wr[on[s2]] : -kInf;
      xn[s2] = AN[uab[s2] & 0xffff] + w + BN[uab[s2] >> 16];
      mn = fmaxf(mn, xn[s2]);
    }
    const float mns = safe(wave_max(mn));
    float sn = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < NKL; ++s2) {
      xn[s2] = lt_exp(xn[s2] - mns);
      sn += xn[s2];
    }
    sn = wave_sum(sn);
    const float rn = (sn > 0.f && sn < kInf) ? __builtin_amdgcn_rcpf(sn) : 0.f;
    // a frame with a zero total (log_z = -inf, or an unreachable string) gets
    // dW = 0, as lt_loss_backward does
    const bool zero = (do_den && rd == 0.f) || rn == 0.f;
    if (!zero) {
#pragma unroll
      for (int s2 = 0; s2 < NKL; ++s2)
        if (on[s2] >= 0)
          __hip_atomic_fetch_add(Sub + on[s2], xn[s2] * rn, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < NL; ++k) x[k] = x[k] * rd - Sub[lane + 64 * k];
    } else {
#pragma unroll
      for (int k = 0; k < NL; ++k) x[k] = 0.f;
    }
    // the slot's LDS reads are issued (LDS is in order per wave): step done
    asm volatile("" ::: "memory");
    if (lane == 0) *(ctl + CTL_MRG + m) = i + 1;
    store_frame(t, x);
  }
  // padding frames (lattices.py:775-779): zero marginals, from the alpha side
  if (!REV && m == 0) {
    float z[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) z[k] = 0.f;
    for (int t = nf; t < T; ++t) store_frame(t, z);
  }
}

template <int J, bool BF16, int PN, int D, int PROD = 0>
__global__ __launch_bounds__(64 * (2 + kPipeMaxHelpers + kPipeMidWaves), PROD ? 2 : 4) void pipe_kernel(const PArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int blk = (int)blockIdx.x;
  const bool rev = a.dirs == 2 && blk >= a.B;
  const int b = rev ? blk - a.B : blk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nthr = blockDim.x;
  const bool do_den = a.flags & F_DEN;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int NP = a.U + 1;

  // ---- prologue: control block, zeroed ring (E padding stays 0), labels
  lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
  for (int k = tid; k < CTL_N; k += nthr) ctl[k] = 0;
  {
    const int n16 = (a.K * a.slot_bytes) / 16;
    lds_float4* ring = (lds_float4*)(as3(lds) + a.off_ring);
    for (int k = tid; k < n16; k += nthr) ring[k] = lt_f4{0.f, 0.f, 0.f, 0.f};
    lds_float* gb = (lds_float*)(as3(lds) + a.off_g);
    lds_float* ubf = (lds_float*)(as3(lds) + a.off_u);
    for (int k = tid; k < a.rowE + 4; k += nthr) {
      gb[k] = 0.f;
      ubf[k] = -kInf;
    }
  }
  int* ctx = (int*)(lds + a.off_ctx);
  int* ylab = (int*)(lds + a.off_ylab);
  for (int u = tid; u < a.U; u += nthr) ylab[u] = a.labels[(long long)b * a.U + u];
  if constexpr (PROD != 0) {
    // the producer helpers' operands: Wo as bf16 (hi, and lo for split
    // products) with padded rows, e^{2 Pc} in fp32 rows of H + 4 (the helpers'
    // 16-byte row reads then fall in distinct banks)
    const int H = a.jH, HP = H + 8, WL = (a.R * HP + 7) & ~7;
    stage_wo<PROD == 1>(a.jwo, (unsigned short*)(lds + a.off_wo), a.R, H, HP, WL, tid, nthr);
    float* ec = (float*)(lds + a.off_ec);
    for (int k = tid; k < a.C * H; k += nthr) ec[k + 4 * (k / H)] = a.jec[k];
  }
  __syncthreads();
  if constexpr (PROD != 0) {
    // any 32-row block of this utterance's Pf rows over kSplitMax (ctl was
    // zeroed above, before the barrier)
    const long long r0 = (long long)b * a.T;
    for (long long k = (r0 >> 5) + tid; k <= ((r0 + a.T - 1) >> 5); k += nthr)
      if (a.jfbig[k]) ctl[CTL_JBIG] = 1;
  }
  if (tid == 0) {
    // walk_states (contexts.py:109-146) with the lattices.py:314-338 label rules
    const int R = a.R;
    int c = 0;
    for (int u = 0; u <= a.U; ++u) {
      ctx[u] = c * R;
      if (u < a.U) {
        int y = ylab[u];
        if (y < 0 || y > a.V) y = 0;
        ylab[u] = y < 1 ? 1 : y;
        if (y != 0) c = y;  // n = 1: next(p, y) = y
      } else {
        ylab[u] = 1;
      }
    }
  }
  if (!do_den && tid == 0) ctl[CTL_DEN] = 0x3fffffff;
  __syncthreads();
  if (a.mid) {
    // zero the granules this workgroup writes last -- the band of frames next
    // to the middle, which the other direction polls first -- then raise the
    // flag (epoch, ~epoch) behind every wave's stores: a poll of a granule not
    // yet written then sees a zero tag, never a stale or arbitrary one (the
    // frames further out are written before the band; mid_marg reaches them
    // only after a band frame of the same direction)
    const int h = nf / 2;
    const int f0 = rev ? h : max(0, h - kMidBand), f1 = rev ? min(nf, h + kMidBand) : h;
    const int NPr = a.U + 1;
    // sc1 (write-through) stores: visible to a reader on any XCD
    if (do_den)
      for (int k = tid; k < (f1 - f0) * a.C; k += nthr)
        __hip_atomic_store((g_u64*)(a.gden[rev] + ((long long)b * a.T + f0) * a.C + k), 0ULL,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = tid; k < (f1 - f0) * NPr; k += nthr)
      __hip_atomic_store((g_u64*)(a.gnum[rev] + ((long long)b * a.T + f0) * NPr + k), 0ULL,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store((g_u64*)(a.mflag + (rev ? 1 : 0) * a.B + b),
                         (unsigned long long)a.epoch | ((unsigned long long)~a.epoch << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // the roles may rotate over the waves by block (LT_PIPE_ROT), so the den
  // chains of workgroups sharing a CU need not sit on one SIMD: measured
  // 0.5-1.5 % slower at B = 256 for three rotations (r05_pipe_rot_ab.txt), off
  const int nwv = nthr >> 6;
  const int rot = LT_PIPE_ROT == 1 ? (blk >> 3) % nwv
                : LT_PIPE_ROT == 2 ? blk % nwv
                : LT_PIPE_ROT == 3 ? ((blk >> 8) & 1) * (nwv >> 1) : 0;
  const int role = LT_PIPE_ROT ? (wave + rot) % nwv : wave;
  if (role == 0) {
    __builtin_amdgcn_s_setprio(3);
    if (do_den) {
      if (rev) den_pipe<J, true>(a, lds, b, nf, lane);
      else den_pipe<J, false>(a, lds, b, nf, lane);
    }
  } else if (role == 1) {
    __builtin_amdgcn_s_setprio(2);
    if (rev) num_pipe<PN, true>(a, lds, b, nf, lane);
    else num_pipe<PN, false>(a, lds, b, nf, lane);
  } else if (role - 2 < a.NH) {
    constexpr int NL = J == 17 ? 18 : (J == 5 ? 5 : (J == 2 ? 2 : 1));
    if constexpr (PROD != 0) {
      if (rev) helper_prod<true, PROD == 1, J>(a, lds, b, nf, role - 2, lane);
      else helper_prod<false, PROD == 1, J>(a, lds, b, nf, role - 2, lane);
    } else {
      if (rev) helper_pipe<BF16, NL, true>(a, lds, b, nf, role - 2, lane);
      else helper_pipe<BF16, NL, false>(a, lds, b, nf, role - 2, lane);
    }
  } else if (a.mid && role - 2 - a.NH < a.NM) {
    if constexpr (PN <= 2) {  // mid mode: U < 128 (pipe_mid_fits)
      constexpr int NL = J == 17 ? 18 : (J == 5 ? 5 : (J == 2 ? 2 : 1));
      const int m = role - 2 - a.NH;
      // the other direction's band granules are zeroed (its flag carries this call's epoch)
      const unsigned long long want =
          (unsigned long long)a.epoch | ((unsigned long long)~a.epoch << 32);
      const unsigned long long* fl = a.mflag + (rev ? 0 : 1) * a.B + b;
      int n = 0;
      lds_vint* ctl = (lds_vint*)(as3(lds) + a.off_ctl);
      bool ok = true;
      while (__hip_atomic_load((const g_u64*)fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        if (*(ctl + CTL_ABORT)) { ok = false; break; }
        __builtin_amdgcn_s_sleep(4);
        if (++n > (1 << 22)) {
          *(ctl + CTL_ABORT) = 1;
          if (a.err) atomicOr(a.err, 2);
          ok = false;
          break;
        }
      }
      if (ok) {
        const bool exact = (a.FR + 63) / 64 == NL;
        if (rev) {
          if (exact) mid_marg<BF16, NL, PN, true, true>(a, lds, b, nf, m, lane);
          else mid_marg<BF16, NL, PN, false, true>(a, lds, b, nf, m, lane);
        } else {
          if (exact) mid_marg<BF16, NL, PN, true, false>(a, lds, b, nf, m, lane);
          else mid_marg<BF16, NL, PN, false, false>(a, lds, b, nf, m, lane);
        }
      }
    }
  }
  __syncthreads();
  if (!rev) {
    if (tid == 0 && a.loss) {
      const lds_float* fin = (const lds_float*)(as3(lds) + a.off_ctl);
      const float num = fin[CTL_FIN1];
      a.loss[b] = (a.flags & F_LOCAL) ? -num : fin[CTL_FIN0] - num;
    }
    if (a.arcs) {
      KArgs ka;
      ka.arcs = a.arcs;
      ka.U = a.U;
      write_arc_table(ka, b, ctx, ylab, tid, nthr);
    }
  }
  (void)NP;
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
int pipe_env(const char* name, int dflt) { return lt_impl::tune_int(name, dflt); }

template <int J, bool BF16, int PN>
int launch_pipe_t(const PArgs& a, int grid, int threads, int lds, hipStream_t st) {
  constexpr int D = 4;
  if (a.prod) {  // producer helpers: fp32 weights, V in (16, 32]
    if constexpr (J == 17 && !BF16) {
      const void* kp = a.prod == 1 ? (const void*)pipe_kernel<J, false, PN, D, 1>
                                   : (const void*)pipe_kernel<J, false, PN, D, 2>;
      hipError_t e = hipFuncSetAttribute(kp, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
      if (a.prod == 1)
        hipLaunchKernelGGL((pipe_kernel<J, false, PN, D, 1>), dim3(grid), dim3(threads), lds, st, a);
      else
        hipLaunchKernelGGL((pipe_kernel<J, false, PN, D, 2>), dim3(grid), dim3(threads), lds, st, a);
      e = hipGetLastError();
      return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
    } else {
      return lt_impl::set_error(LT_EUNSUPPORTED, "pipe producer helpers: fp32, 16 < V <= 32");
    }
  }
  const void* k = (const void*)pipe_kernel<J, BF16, PN, D>;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  if (pipe_env("LT_VERBOSE", 0)) {
    int occ = -1;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, threads, lds);
    fprintf(stderr, "[lt pipe] occupancy %d blocks/CU (threads %d, lds %d)\n", occ, threads, lds);
  }
  if (a.mid) {
    // every recursion workgroup must be resident at once: the marginal waves
    // of one direction wait on the other direction's first half
    int occ = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, threads, lds) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        (long long)occ * cus < grid)
      return lt_impl::set_error(LT_EUNSUPPORTED, "pipe mid: the grid is not co-resident");
    if (a.W == nullptr) return LT_OK;  // a fit query only
  }
  hipLaunchKernelGGL((pipe_kernel<J, BF16, PN, D>), dim3(grid), dim3(threads), lds, st, a);
  e = hipGetLastError();
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

template <int J, bool BF16>
int launch_pipe_pn(int PN, const PArgs& a, int grid, int threads, int lds, hipStream_t st) {
  if (PN == 1) return launch_pipe_t<J, BF16, 1>(a, grid, threads, lds, st);
  if (PN == 2) return launch_pipe_t<J, BF16, 2>(a, grid, threads, lds, st);
  return launch_pipe_t<J, BF16, 4>(a, grid, threads, lds, st);
}

template <bool BF16>
int launch_pipe_j(int J, int PN, const PArgs& a, int grid, int threads, int lds, hipStream_t st) {
  switch (J) {
    case 17: return launch_pipe_pn<17, BF16>(PN, a, grid, threads, lds, st);
    case 5: return launch_pipe_pn<5, BF16>(PN, a, grid, threads, lds, st);
    case 2: return launch_pipe_pn<2, BF16>(PN, a, grid, threads, lds, st);
    default: return launch_pipe_pn<1, BF16>(PN, a, grid, threads, lds, st);
  }
}

}  // namespace

namespace lt_impl {

bool pipe_eligible(const lt_problem* pb) {
  if (pipe_env("LT_NO_PIPE", 0)) return false;
  if (pb->context_size != 1 || pb->vocab_size < 1 || pb->vocab_size > 32) return false;
  if (pb->max_labels + 1 > 256) return false;
  const long long C = pb->vocab_size + 1;
  const long long es = pb->weight_dtype == LT_DTYPE_BF16 ? 2 : 4;
  const long long bytes = (long long)pb->batch * pb->max_frames * C * C * es;
  const long long rows = (long long)pb->batch * pb->max_frames * (pb->max_labels + 1) * 4;
  return bytes < 0xFFFFFFF0LL && rows < 0xFFFFFFF0LL;
}

// mid mode workspace: the granule rows (alpha, beta [B,T,C]; alpha^n, beta^n
// [B,T,U+1]; 8 bytes each), the band flags [2][B] and the error word
size_t pipe_mid_workspace_bytes(const lt_problem* pb) {
  const long long BT = (long long)pb->batch * pb->max_frames;
  const long long C = pb->vocab_size + 1, NP = pb->max_labels + 1;
  return (size_t)(8 * (2 * BT * C + 2 * BT * NP + 2LL * pb->batch) + 16);
}

static std::atomic<unsigned> g_mid_epoch{0};

bool pipe_mid_fits(const lt_problem* pb) {
  // (U < 128: the marginal waves' registers stay below the spill point)
  if (!pipe_eligible(pb) || pb->batch == 0 || pb->max_frames == 0 || pb->max_labels + 1 > 128)
    return false;
  lt_problem q = *pb;
  // the occupancy query of the launch itself (no W: nothing is launched)
  return launch_pipe(&q, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                     nullptr, nullptr, nullptr, nullptr, nullptr, 2, nullptr, nullptr, nullptr, 1,
                     nullptr) == LT_OK;
}

int launch_pipe(const lt_problem* pb, int local_norm, const void* W, const int32_t* nfr,
                const int32_t* labels, const int32_t* nlab, float* loss, float* log_z,
                float* num, float* alpha, float* alpha_num, float* beta, float* beta_num,
                int32_t* arcs, int dirs, int* err, void* stream, void* dW, int mid,
                void* mws, const JointOps* jo) {
  if (!pipe_eligible(pb)) return set_error(LT_EUNSUPPORTED, "pipe: shape not eligible");
  if (mid && (dirs != 2 || (!dW && W) || (!mws && W)))
    return set_error(LT_EINVAL, "pipe mid: both directions, dW and the workspace");
  PArgs a;
  memset(&a, 0, sizeof(a));
  const int V = pb->vocab_size, C = V + 1, R = V + 1, FR = C * R, U = pb->max_labels;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const int es = bf16 ? 2 : 4;
  a.W = (const unsigned char*)W;
  a.nfr = nfr; a.labels = labels; a.nlab = nlab;
  a.loss = loss; a.log_z = log_z; a.num = num;
  a.alpha = alpha; a.alpha_num = alpha_num; a.beta = beta; a.beta_num = beta_num;
  a.arcs = arcs; a.err = err;
  a.B = pb->batch; a.T = pb->max_frames; a.U = U; a.V = V; a.C = C; a.R = R; a.FR = FR;
  a.flags = F_NUM | F_LOSS | (local_norm ? F_LOCAL : F_DEN);
  int p2 = 1;
  while (p2 < V) p2 *= 2;
  a.H = 64 / p2;
  a.lgH = 0;
  while ((1 << a.lgH) < a.H) ++a.lgH;
  a.J = V > 16 ? 17 : (V > 8 ? 5 : (V > 4 ? 2 : 1));
  a.JP = a.J >= 4 ? (a.J + 3) / 4 * 4 : a.J;
  a.rowE = a.H * a.JP;
  if (a.H * a.J < C) return set_error(LT_EUNSUPPORTED, "pipe: lane plan");
  a.NLr = (FR + 63) / 64;
  a.NH = std::max(1, std::min(kPipeMaxHelpers, pipe_env("LT_PIPE_HELPERS", 4)));
  a.logn = logf((float)(V + 2));
  a.dirs = dirs;
#ifdef LT_DIAG
  a.dbg = pipe_env("LT_PIPE_DBG", 0);  // timing ablations: diagnostic builds only
#endif
#ifdef LT_STAMPS
  {
    const char* sp = lt_impl::tune_str("LT_STAMPS_PTR");
    a.stamps = sp ? (long long*)strtoull(sp, nullptr, 0) : nullptr;
    a.stamp_block = pipe_env("LT_STAMP_BLOCK", 0);
  }
#endif
  a.w_bytes = (unsigned)((long long)pb->batch * pb->max_frames * FR * es);
  const int PN = U + 1 <= 64 ? 1 : (U + 1 <= 128 ? 2 : 4);
  const int NP = U + 1;
  if (mid && PN > 2) return set_error(LT_EUNSUPPORTED, "pipe mid: labels < 128");
  auto al16 = [](long long x) { return (int)((x + 15) & ~15LL); };
  int off = 0;
  a.off_ctl = off; off += al16(CTL_N * 4);
  a.off_g = off; off += al16((a.rowE + 4) * 4);
  a.off_u = off; off += al16((a.rowE + 4) * 4);
  a.off_ctx = off; off += al16(NP * 4);
  a.off_ylab = off; off += al16(NP * 4);
  if (jo) {  // producer helpers: Wo bf16 (hi, lo) and e^{2 Pc} in LDS
    if (mid || bf16 || jo->H % 32 || jo->H < 32)
      return set_error(LT_EUNSUPPORTED, "pipe producer helpers: fp32, no mid mode, H % 32 == 0");
    a.prod = jo->prod;
    a.jH = jo->H;
    a.jpc = jo->pc; a.jec = jo->ec; a.jpf = jo->pf; a.jef = jo->ef;
    a.jcbig = jo->cbig; a.jfbig = jo->fbig; a.jwo = jo->wo; a.jbias = jo->bias;
    const int WL = (R * (jo->H + 8) + 7) & ~7;
    a.off_wo = off; off += al16((jo->prod == 1 ? 4LL : 2LL) * WL);
    a.off_ec = off; off += al16(4LL * C * (jo->H + 4));
    // producer helpers take the mid-mode waves' places too: their registers
    // (two waves per SIMD) leave one workgroup per CU at any grid, and their
    // MFMA work bounds the step otherwise
    a.NH = std::max(a.NH, kProdHelpers);
    a.off_jf = off; off += kProdHelpers * 2048;
    a.off_j32 = off; off += kProdHelpers * al16(32LL * R * 4);
    if (jo->H > 256) return set_error(LT_EUNSUPPORTED, "pipe producer helpers: H <= 256");
  }
  int so = 0;
  const int NLc = a.J == 17 ? 18 : (a.J == 5 ? 5 : (a.J == 2 ? 2 : 1));
  if (NLc * 64 < FR) return set_error(LT_EUNSUPPORTED, "pipe: helper load plan");
  so += al16(NLc * 64 * 4);  // raw W, padded to the helpers' load footprint
  a.soff_e = so; so += al16((long long)C * a.rowE * 4);
  a.soff_eb = so; so += al16(C * 4);
  a.soff_c = so; so += 16;
  a.slot_bytes = so;
  // LDS budget: two workgroups per CU when the grid exceeds the CU count
  const int grid = dirs * pb->batch;
  int cap = grid > 256 && !jo ? 80 * 1024 : 160 * 1024;
  cap = pipe_env("LT_PIPE_LDS", cap);
  // mid mode: the marginal waves' regions, and per ring slot the den and
  // numerator rows of its step
  int per_slot = so;
  if (mid) {
    a.mid = 1;
    a.NM = kPipeMidWaves;
    a.mw_bytes = 4 * (256 + 128 * PN + 64 * NLc);
    a.off_mw = off;
    off += al16((long long)a.NM * a.mw_bytes);
    per_slot = so + 4 * (kHS + ((NP + 3) & ~3));
  }
  a.off_ring = off;
  int K = (cap - off) / per_slot;
  K = std::min(K, std::min(kPipeMaxSlots, pipe_env("LT_PIPE_SLOTS", 16)));
  if (K < 2) return set_error(LT_EUNSUPPORTED, "pipe: ring does not fit in LDS");
  a.K = K;
  a.NH = std::min(a.NH, K);
  int lds = off + K * so;
  if (mid) {
    a.off_hring = lds;
    a.off_nring = a.off_hring + K * kHS * 4;
    lds = a.off_nring + K * ((NP + 3) & ~3) * 4;
  }
  const int threads = 64 * (2 + a.NH + (mid ? a.NM : 0));
  if (grid == 0) return LT_OK;
  hipStream_t st = (hipStream_t)stream;
  if (mid) {
    // rows only for the other direction (granules), no checkpoints, no arcs
    a.alpha = a.beta = a.alpha_num = a.beta_num = nullptr;
    a.arcs = nullptr;
    a.dW = dW;
    const long long BT = (long long)pb->batch * pb->max_frames;
    unsigned long long* g = (unsigned long long*)mws;
    a.gden[0] = g; g += W ? BT * C : 0;
    a.gden[1] = g; g += W ? BT * C : 0;
    a.gnum[0] = g; g += W ? BT * NP : 0;
    a.gnum[1] = g; g += W ? BT * NP : 0;
    a.mflag = g; g += W ? 2LL * pb->batch : 0;
    a.err = W ? (int*)g : nullptr;
    // tags epoch * T + t stay nonzero and unique until the epoch wraps
    unsigned ep = ++g_mid_epoch;
    const unsigned lim = 0xFFFFFFFEu / (unsigned)(pb->max_frames + 1);
    if (ep == 0 || ep >= lim) {
      g_mid_epoch = 1;
      ep = 1;
    }
    a.epoch = ep;
    if (W) {
      // a captured graph replays this epoch: zero the granules and band
      // flags per replay (a memset node), so no replay reads the last one's
      const size_t zb = lt_impl::stream_capturing(st)
                            ? (size_t)((char*)a.err - (char*)mws) + sizeof(int)
                            : sizeof(int);
      const hipError_t e =
          hipMemsetAsync(zb == sizeof(int) ? (void*)a.err : mws, 0, zb, st);
      if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
    }
  }
  if (pipe_env("LT_VERBOSE", 0))
    fprintf(stderr, "[lt pipe] V=%d H=%d J=%d JP=%d PN=%d NH=%d K=%d slot=%d lds=%d grid=%d\n",
            V, a.H, a.J, a.JP, PN, a.NH, K, so, lds, grid);
  return bf16 ? launch_pipe_j<true>(a.J, PN, a, grid, threads, lds, st)
              : launch_pipe_j<false>(a.J, PN, a, grid, threads, lds, st);
}

}  // namespace lt_impl
