// lt_lattice.hip -- MI355X (gfx950 / CDNA4) kernels for the GNAT recognition
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

#include <algorithm>
#include <string>

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
  if (g.n == 0) return 0;
  if (p < g.An) return p * g.V;
  return ((p - g.An) % g.Vn1) * g.V + g.An - 1;
}

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
LT_DEVINL float lt_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// Arguments are sums of exp() with the max term == 1 (>= 1) or exactly 0.
LT_DEVINL float lt_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }

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
  int B, T, U, flags;
  NGram g;
  int FR;            // C*(V+1) elements per frame
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
};

LT_DEVINL unsigned lds_base_addr(unsigned char* lds) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
}

// Issue the LDS-DMA instructions of loader wave `lw` for frame t into `slot`.
// Instruction gi of the frame (streams in slot order) belongs to loader wave
// gi % load_waves.
template <int S>
LT_DEVINL void issue_stream(const KArgs& a, int b, int t, int slot, int lw, int lane,
                            unsigned ldsb, int& gi) {
  const int ni = a.st_ninstr[S];
  if (ni == 0) return;
  const long long row = a.st_row[S];
  const long long off = ((long long)b * a.T + t) * row;
  const long long g0 = off >> 4;
  const long long g1 = (off + row + 15) >> 4;
  const unsigned dst0 = ldsb + a.off_ring + slot * a.slot_bytes + a.st_off[S];
  const unsigned char* base = a.st_base[S];
  for (int k = 0; k < ni; ++k, ++gi) {
    if (gi % a.load_waves != lw) continue;
    long long gg = g0 + (long long)k * 64 + lane;
    if (gg > g1 - 1) gg = g1 - 1;  // in-bounds duplicate, lands past the row
    glds16(base + gg * 16, dst0 + k * 1024);
  }
}
LT_DEVINL void issue_frame(const KArgs& a, int b, int t, int slot, int lw, int lane,
                           unsigned ldsb) {
  int gi = 0;
  issue_stream<0>(a, b, t, slot, lw, lane, ldsb, gi);
  issue_stream<1>(a, b, t, slot, lw, lane, ldsb, gi);
  issue_stream<2>(a, b, t, slot, lw, lane, ldsb, gi);
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
LT_DEVINL void walk_states(const KArgs& a, int b, int* ctx, int* ylab) {
  const NGram& g = a.g;
  const int R = g.V + 1;
  int c = 0;
  for (int u = 0; u <= a.U; ++u) {
    ctx[u] = c * R;
    if (u < a.U) {
      int y = a.labels[(long long)b * a.U + u];
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

// ---------------------------------------------------------------------------
// Forward kernel: denominator and/or numerator, Log / MaxTropical / Real.
// ---------------------------------------------------------------------------
template <int MODE, bool BF16, bool WST, int TMAX>
__global__ __launch_bounds__(1024) void fwd_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const NGram& g = a.g;
  const int C = g.C, R = g.V + 1, NP = a.U + 1;
  const bool do_den = a.flags & F_DEN, do_num = a.flags & F_NUM;
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

  // ---- prologue
  if (role == 2) {
    const int pre = nf < a.P ? nf : a.P;
    for (int f = 0; f < pre; ++f) issue_frame(a, b, f, f % a.S, lw, lane, ldsb);
  } else if (role == 0) {
    if (do_den)
      for (int q = tid; q < C; q += den_lanes) abuf[q] = (q == 0) ? s_one<MODE>() : s_zero<MODE>();
  } else {
    const int al = tid - den_lanes;
    if (do_num) {
      for (int u = al; u < NP; u += aux_lanes) nbuf[u] = (u == 0) ? s_one<MODE>() : s_zero<MODE>();
      if (al == 0) walk_states(a, b, ctx, ylab);
    }
  }
  lds_barrier();

  const int L = a.L, lgL = a.lgL;
  const int j = tid & (L - 1);
  const int grp0 = tid >> lgL;
  const int ngrp = den_lanes >> lgL;

  // ---- frame loop (alignment scan, lattices.py:856-892)
  for (int i = 0; i < nf; ++i) {
    const int t = i;
    const int slot = i % a.S;
    if (role == 2) {
      const int later = (a.P - 1 < nf - 1 - i) ? a.P - 1 : nf - 1 - i;
      wait_vmcnt(later * (lw == 0 ? a.gw0 : a.gw1));
    }
    lds_barrier();
    if (role == 2) {
      if (i + a.P < nf) issue_frame(a, b, i + a.P, (i + a.P) % a.S, lw, lane, ldsb);
      continue;
    }
    const unsigned char* wrow;
    if constexpr (WST) wrow = slot_row<0>(lds, a, b, t, slot);
    else wrow = a.W + ((long long)b * a.T + t) * (long long)a.FR * (BF16 ? 2 : 4);

    if (role == 0) {
      if (!do_den) continue;
      const float* acur = abuf + (i & 1) * C;
      float* anxt = abuf + ((i + 1) & 1) * C;
      for (int q = grp0; q < C; q += ngrp) {
        const DestDesc d = dest_desc(g, q);
        const int nterm = d.kq + 1;
        float xv[TMAX];
#pragma unroll
        for (int m = 0; m < TMAX; ++m) {
          const int o = j + m * L;
          float x = s_zero<MODE>();
          if (o < nterm) {
            float av, wv;
            if (o == 0) {
              av = acur[q];
              wv = ldw<BF16>(wrow, (long long)q * R);
            } else {
              const int k = o - 1;
              av = acur[d.a0 + k * d.astr];
              wv = ldw<BF16>(wrow, d.w0 + k * d.wstr);
            }
            x = s_times<MODE>(av, wv);
          }
          xv[m] = x;
        }
        float r;
        int bi = j;
        if constexpr (MODE == M_LOG) {
          float mx = xv[0];
#pragma unroll
          for (int m = 1; m < TMAX; ++m) mx = fmaxf(mx, xv[m]);
          mx = grp_max(mx, lgL);
          const float c = __builtin_isfinite(mx) ? mx : 0.f;
          float s = 0.f;
#pragma unroll
          for (int m = 0; m < TMAX; ++m) s += lt_exp(xv[m] - c);
          s = grp_sum(s, lgL);
          r = c + lt_log(s);
        } else if constexpr (MODE == M_MAX) {
          r = xv[0];
#pragma unroll
          for (int m = 1; m < TMAX; ++m)
            if (xv[m] > r) { r = xv[m]; bi = j + m * L; }
          grp_argmax(r, bi, lgL);
        } else {
          float s = 0.f;
#pragma unroll
          for (int m = 0; m < TMAX; ++m) s += xv[m];
          r = grp_sum(s, lgL);
        }
        if (j == 0) {
          const long long hb = ((long long)b * a.T + t) * C + q;
          if (a.alpha) a.alpha[hb] = acur[q];
          if (MODE == M_MAX && a.bp) a.bp[hb] = (unsigned char)bi;
          anxt[q] = r;
        }
      }
    } else {  // role 1: numerator positions (alignments.py:320-329)
      if (!do_num) continue;
      const float* ncur = nbuf + (i & 1) * NP;
      float* nnxt = nbuf + ((i + 1) & 1) * NP;
      for (int u = tid - den_lanes; u < NP; u += aux_lanes) {
        const float xb = s_times<MODE>(ncur[u], ldw<BF16>(wrow, ctx[u]));
        float xl = s_zero<MODE>();
        if (u >= 1) xl = s_times<MODE>(ncur[u - 1], ldw<BF16>(wrow, ctx[u - 1] + ylab[u - 1]));
        if (a.alpha_num) a.alpha_num[((long long)b * a.T + t) * NP + u] = ncur[u];
        nnxt[u] = s_plus<MODE>(xb, xl);
      }
    }
  }
  lds_barrier();

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
        mx = grp_max(mx, 6);
        const float c = __builtin_isfinite(mx) ? mx : 0.f;
        float s = 0.f;
        for (int q = lane; q < C; q += 64) s += lt_exp(af[q] - c);
        s = grp_sum(s, 6);
        r = c + lt_log(s);
      } else if constexpr (MODE == M_MAX) {
        r = -kInf;
        for (int q = lane; q < C; q += 64)
          if (bi == 0x7fffffff || af[q] > r) { r = af[q]; bi = q; }
        grp_argmax(r, bi, 6);
      } else {
        float s = 0.f;
        for (int q = lane; q < C; q += 64) s += af[q];
        r = grp_sum(s, 6);
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
      for (long long e = tid; e < n; e += den_lanes) dst[e] = af[e % C];
    }
  } else if (role == 1 && do_num) {
    const float* nfin = nbuf + fin * NP;
    const int al = tid - den_lanes;
    if (al == 0) {
      const int nl = a.nlab[b];
      // lattices.py:375-377: (+) over positions equal to num_labels
      const float r = (nl >= 0 && nl <= a.U) ? nfin[nl] : s_zero<MODE>();
      misc[1] = r;
      if (a.num) a.num[b] = r;
    }
    if (a.alpha_num) {
      const long long n = (long long)(a.T - nf) * NP;
      float* dst = a.alpha_num + ((long long)b * a.T + nf) * NP;
      for (long long e = al; e < n; e += aux_lanes) dst[e] = nfin[e % NP];
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
}

// ---------------------------------------------------------------------------
// Backward kernel (Log): beta recursion + arc marginals -> dW.
//   DST: dW frame staged in LDS (den marginals written by den lanes, numerator
//        marginals LDS-atomically accumulated by aux lanes, stored coalesced
//        one frame later by the aux lanes).
//   !DST: den lanes store straight to HBM; numerator marginals go to a side
//        buffer and a scatter kernel subtracts them (large C*(V+1)).
// ---------------------------------------------------------------------------
template <bool BF16, bool WST, bool DST, int TMAX>
__global__ __launch_bounds__(1024) void bwd_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const NGram& g = a.g;
  const int C = g.C, R = g.V + 1, NP = a.U + 1, FR = a.FR;
  const bool do_den = a.flags & F_DEN, do_num = a.flags & F_NUM;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);

  float* bbuf = (float*)(lds + a.off_a);     // [2][C]  den beta
  float* nbb = (float*)(lds + a.off_na);     // [2][NP] num beta
  int* ctx = (int*)(lds + a.off_ctx);
  int* ylab = (int*)(lds + a.off_ylab);
  float* dbuf = (float*)(lds + a.off_dbuf);  // [2][FR] den marginals
  float* mbuf = (float*)(lds + a.off_nbuf);  // [2][FR] num marginals
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
    for (int f = 0; f < pre; ++f) issue_frame(a, b, nf - 1 - f, f % a.S, lw, lane, ldsb);
  } else if (role == 0) {
    // beta_T = one for every state: all context states are final
    // (lattices.py:788-790)
    if (do_den) for (int p = tid; p < C; p += den_lanes) bbuf[p] = 0.f;
  } else {
    if (do_num) {
      for (int u = al; u < NP; u += aux_lanes) nbb[u] = (u == nl) ? 0.f : -kInf;
      if (al == 0) walk_states(a, b, ctx, ylab);
    }
    if (DST && do_num)
      for (int e = al; e < 2 * FR; e += aux_lanes) mbuf[e] = 0.f;
  }
  lds_barrier();
  if (!DST && do_num && role == 1 && a.ctx_side) {
    for (int u = al; u < NP; u += aux_lanes) {
      a.ctx_side[((long long)b * NP + u) * 2 + 0] = ctx[u];
      a.ctx_side[((long long)b * NP + u) * 2 + 1] = ylab[u];
    }
  }

  const int L = a.L, lgL = a.lgL;
  const int j = tid & (L - 1);
  const int grp0 = tid >> lgL;
  const int ngrp = den_lanes >> lgL;
  const int es = BF16 ? 2 : 4;

  for (int i = 0; i < nf; ++i) {
    const int t = nf - 1 - i;
    const int slot = i % a.S;
    const int cur = i & 1;
    if (role == 2) {
      const int later = (a.P - 1 < nf - 1 - i) ? a.P - 1 : nf - 1 - i;
      wait_vmcnt(later * (lw == 0 ? a.gw0 : a.gw1));
    }
    lds_barrier();
    if (role == 2) {
      if (i + a.P < nf) issue_frame(a, b, nf - 1 - (i + a.P), (i + a.P) % a.S, lw, lane, ldsb);
      continue;
    }
    const unsigned char* wrow;
    if constexpr (WST) wrow = slot_row<0>(lds, a, b, t, slot);
    else wrow = a.W + ((long long)b * a.T + t) * (long long)FR * es;

    if (role == 0) {
      if (!do_den) continue;
      const float* arow = (const float*)slot_row<1>(lds, a, b, t, slot);
      const float* bcur = bbuf + cur * C;
      float* bnxt = bbuf + (cur ^ 1) * C;
      for (int p = grp0; p < C; p += ngrp) {
        bool zero;
        const int nb = next_base(g, p, &zero);
        float xv[TMAX];
#pragma unroll
        for (int m = 0; m < TMAX; ++m) {
          const int y = j + m * L;
          float x = -kInf;
          if (y <= g.V) {
            const int dst = (y == 0) ? p : (zero ? 0 : nb + y);
            x = ldw<BF16>(wrow, (long long)p * R + y) + bcur[dst];
          }
          xv[m] = x;
        }
        float mx = xv[0];
#pragma unroll
        for (int m = 1; m < TMAX; ++m) mx = fmaxf(mx, xv[m]);
        mx = grp_max(mx, lgL);
        const float c = __builtin_isfinite(mx) ? mx : 0.f;
        float s = 0.f;
#pragma unroll
        for (int m = 0; m < TMAX; ++m) {
          xv[m] = lt_exp(xv[m] - c);
          s += xv[m];
        }
        s = grp_sum(s, lgL);
        if (j == 0) bnxt[p] = c + lt_log(s);
        // marginals exp(alpha + w + beta' - log_z) = e_y * exp(c + alpha - log_z)
        const float sp = (gb == 0.f) ? 0.f : lt_exp(c + arow[p] - log_z) * gb;
#pragma unroll
        for (int m = 0; m < TMAX; ++m) {
          const int y = j + m * L;
          if (y <= g.V) {
            const float v = xv[m] * sp;
            const long long e = (long long)p * R + y;
            if constexpr (DST) dbuf[cur * FR + e] = v;
            else stw<BF16>(a.dW, ((long long)b * a.T + t) * FR + e, v);
          }
        }
      }
    } else {  // role 1
      if constexpr (DST) {
        if (i >= 1) {  // store frame t+1 (computed last step)
          const int pv = cur ^ 1;
          const long long base = ((long long)b * a.T + (t + 1)) * FR;
          for (int e = al; e < FR; e += aux_lanes) {
            float v = do_den ? dbuf[pv * FR + e] : 0.f;
            if (do_num) { v -= mbuf[pv * FR + e]; mbuf[pv * FR + e] = 0.f; }
            stw<BF16>(a.dW, base + e, v);
          }
        }
      }
      if (!do_num) continue;
      const float* ncur = nbb + cur * NP;
      float* nnxt = nbb + (cur ^ 1) * NP;
      const float* anrow = (const float*)slot_row<2>(lds, a, b, t, slot);
      for (int u = al; u < NP; u += aux_lanes) {
        const float xb = ldw<BF16>(wrow, ctx[u]) + ncur[u];
        float xl = -kInf;
        if (u < a.U) xl = ldw<BF16>(wrow, ctx[u] + ylab[u]) + ncur[u + 1];
        nnxt[u] = log_plus(xb, xl);
        float mb = 0.f, ml = 0.f;
        if (gb != 0.f) {
          const float an = anrow[u] - numv;
          mb = lt_exp(an + xb) * gb;
          ml = lt_exp(an + xl) * gb;
        }
        if constexpr (DST) {
          if (mb != 0.f) atomicAdd(&mbuf[cur * FR + ctx[u]], mb);
          if (ml != 0.f) atomicAdd(&mbuf[cur * FR + ctx[u] + ylab[u]], ml);
        } else {
          float* ns = a.nm_side + (((long long)b * a.T + t) * NP + u) * 2;
          ns[0] = mb;
          ns[1] = ml;
        }
      }
    }
  }
  lds_barrier();
  if constexpr (DST) {
    if (role == 1 && nf >= 1) {  // last processed frame: t = 0
      const int pv = (nf - 1) & 1;
      const long long base = ((long long)b * a.T) * FR;
      for (int e = al; e < FR; e += aux_lanes) {
        float v = do_den ? dbuf[pv * FR + e] : 0.f;
        if (do_num) v -= mbuf[pv * FR + e];
        stw<BF16>(a.dW, base + e, v);
      }
    }
  }
  // padding frames get zero marginals (lattices.py:775-779); with no
  // denominator in the direct path nothing else wrote dW.
  {
    const int t0 = (!DST && !do_den) ? 0 : nf;
    const long long n = (long long)(a.T - t0) * FR;
    const long long base = ((long long)b * a.T + t0) * FR;
    const int nthr = blockDim.x;
    for (long long e = tid; e < n; e += nthr) stw<BF16>(a.dW, base + e, 0.f);
  }
}

// Direct path: subtract numerator marginals (one thread per (b,t), fixed u
// order, so the result is deterministic).
template <bool BF16>
__global__ void num_scatter_kernel(const KArgs a) {
  const long long bt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (bt >= (long long)a.B * a.T) return;
  const int b = (int)(bt / a.T), t = (int)(bt % a.T);
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  if (t >= nf) return;
  const int NP = a.U + 1;
  const long long base = bt * a.FR;
  const float* ns = a.nm_side + bt * NP * 2;
  const int* cs = a.ctx_side + (long long)b * NP * 2;
  for (int u = 0; u < NP; ++u) {
    const int e0 = cs[2 * u], e1 = e0 + cs[2 * u + 1];
    const float mb = ns[2 * u], ml = ns[2 * u + 1];
    if (mb != 0.f) stw<BF16>(a.dW, base + e0, ldw<BF16>((const unsigned char*)a.dW, base + e0) - mb);
    if (u < a.U && ml != 0.f)
      stw<BF16>(a.dW, base + e1, ldw<BF16>((const unsigned char*)a.dW, base + e1) - ml);
  }
}

// ---------------------------------------------------------------------------
// Viterbi backtrace: follows the backpointers written by fwd_kernel<M_MAX>.
// Equivalent to the vjp of _forward(MaxTropical) w.r.t. a zero lexical mask
// (lattices.py:219-244): the chosen arc at each frame, blank when the blank
// term won (including ties).
// ---------------------------------------------------------------------------
struct BtArgs {
  const unsigned char* bp;
  const int* qstar;
  const int* nfr;
  const float* grad;
  long long* labels;  // [B,T]
  void* arcs;         // [B,T,C,V+1] or null
  int B, T, conv, arcs_bf16;
  NGram g;
  int chunk;          // frames per LDS chunk
};

template <bool BF16>
__global__ __launch_bounds__(256) void backtrace_kernel(const BtArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int b = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
  const NGram& g = a.g;
  const int C = g.C, R = g.V + 1;
  const long long FR = (long long)C * R;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  long long* lab = a.labels + (long long)b * a.T;
  for (int t = nf + tid; t < a.T; t += nthr) lab[t] = 0;  // padding frames
  if (a.arcs) {
    const long long n = (long long)a.T * FR;
    for (long long e = tid; e < n; e += nthr) stw<BF16>(a.arcs, (long long)b * a.T * FR + e, 0.f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float gb = a.grad ? a.grad[b] : 1.f;
  int q = a.qstar[b];
  int* qs = (int*)lds;  // walker state broadcast
  unsigned char* rows = lds + 16;
  for (int t1 = nf; t1 > 0; t1 -= a.chunk) {
    const int t0 = t1 - a.chunk < 0 ? 0 : t1 - a.chunk;
    const unsigned char* src = a.bp + ((long long)b * a.T + t0) * C;
    const int nbytes = (t1 - t0) * C;
    for (int e = tid; e < nbytes; e += nthr) rows[e] = src[e];
    __syncthreads();
    if (tid == 0) {
      for (int t = t1 - 1; t >= t0; --t) {
        const int idx = rows[(t - t0) * C + q];
        long long lb = 0;
        int p = q, y = 0;
        if (idx != 0) {
          const DestDesc d = dest_desc(g, q);
          const int k = idx - 1;
          p = d.a0 + k * d.astr;
          y = d.w0 + k * d.wstr - p * R;
          lb = a.conv == LT_LABELS_REFERENCE ? (long long)(y - 1) : (long long)y;
        }
        lab[t] = lb;
        if (a.arcs) stw<BF16>(a.arcs, ((long long)b * a.T + t) * FR + (long long)p * R + y, gb);
        q = p;
      }
      qs[0] = q;
    }
    __syncthreads();
    q = qs[0];
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
thread_local std::string g_err = "ok";

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int make_ngram(int V, int n, NGram* g) {
  if (V <= 0) return fail(LT_EINVAL, "vocab_size must be > 0");
  if (n < 0) return fail(LT_EINVAL, "context_size must be >= 0");
  long long C = 0, pw = 1, An = 0, Apn = 0, Vn1 = 0;
  for (int i = 0; i <= n; ++i) {
    if (i < n) An += pw;
    if (i < n - 1) Apn += pw;
    if (i == n - 1) Vn1 = pw;
    C += pw;
    pw *= V;
    if (C > (1LL << 22)) return fail(LT_EUNSUPPORTED, "too many context states");
  }
  if (C * (V + 1) > (1LL << 30)) return fail(LT_EUNSUPPORTED, "frame too large");
  g->V = V; g->n = n; g->C = (int)C; g->An = (int)An; g->Apn = (int)Apn;
  g->Vn1 = (int)Vn1; g->K = (n == 0) ? V : V + 1;
  return LT_OK;
}

int check_problem(const lt_problem* pb, NGram* g) {
  if (!pb) return fail(LT_EINVAL, "null problem");
  if (pb->batch < 0 || pb->max_frames < 0 || pb->max_labels < 0)
    return fail(LT_EINVAL, "negative dimension");
  if (pb->weight_dtype != LT_DTYPE_F32 && pb->weight_dtype != LT_DTYPE_BF16)
    return fail(LT_EINVAL, "weight_dtype must be LT_DTYPE_F32 or LT_DTYPE_BF16");
  return make_ngram(pb->vocab_size, pb->context_size, g);
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return LT_OK;
  return fail(LT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int kLdsMax = 160 * 1024;
constexpr int kMaxWaves = 16;

int env_int(const char* name, int dflt) {
  const char* s = getenv(name);
  return (s && *s) ? atoi(s) : dflt;
}

int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

struct Plan {
  KArgs a;
  int tmax;
  bool wst, dst;
  int threads;
  int lds_bytes;
};

// Choose lanes-per-group, wave roles, LDS carve and ring depth.
//   kind 0: forward, kind 1: backward
int plan(const lt_problem* pb, const NGram& g, int kind, int flags, Plan* pl) {
  KArgs& a = pl->a;
  memset(&a, 0, sizeof(a));
  a.B = pb->batch; a.T = pb->max_frames; a.U = pb->max_labels; a.g = g;
  a.flags = flags;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const int es = bf16 ? 2 : 4;
  const int C = g.C, R = g.V + 1, NP = a.U + 1;
  a.FR = C * R;
  const long long FRB = (long long)a.FR * es;
  const bool do_den = flags & F_DEN, do_num = flags & F_NUM;

  // terms per group: forward K+1 (blank + lexical in-arcs), backward V+1
  const int nterm = kind == 0 ? g.K + 1 : g.V + 1;
  int L = 1;
  while (L < 64 && (nterm + L - 1) / L > 16) L *= 2;
  // prefer >= ~4 terms per lane while the groups fit in the den waves
  while (L < 16 && nterm / (2 * L) >= 4 && (long long)C * 2 * L <= 64LL * 10) L *= 2;
  const int envL = env_int("LT_DEN_LANES", 0);
  if (envL > 0 && (envL & (envL - 1)) == 0 && (nterm + envL - 1) / envL <= 16) L = envL;
  a.L = L;
  a.lgL = 0;
  while ((1 << a.lgL) < L) ++a.lgL;
  const int per = (nterm + L - 1) / L;
  pl->tmax = per <= 4 ? 4 : (per <= 8 ? 8 : 16);

  a.aux_waves = do_num ? std::min(ceil_div(NP, 64), 4) : (kind == 1 ? 1 : 0);
  a.load_waves = 2;
  int den = do_den ? ceil_div((long long)C * L, 64) : 0;
  den = std::min(den, kMaxWaves - a.aux_waves - a.load_waves);
  if (do_den && den < 1) den = 1;
  a.den_waves = den;
  if (!do_den && a.aux_waves == 0) a.aux_waves = 1;

  // LDS carve (bytes, 16-aligned pieces)
  auto al16 = [](long long x) { return (int)((x + 15) & ~15LL); };
  int off = 0;
  a.off_misc = off; off += 64;
  a.off_a = off; off += al16(2LL * C * 4);
  a.off_na = off; off += al16(2LL * NP * 4);
  a.off_ctx = off; off += al16((long long)NP * 4);
  a.off_ylab = off; off += al16((long long)NP * 4);
  int fixed = off;

  // staged marginals (backward)
  pl->dst = false;
  if (kind == 1) {
    const long long need = (do_den ? 2LL * a.FR * 4 : 0) + (do_num ? 2LL * a.FR * 4 : 0);
    const int ring_min = 4 * 1024 * 4;  // leave room for a few ring slots
    if (fixed + need + ring_min <= kLdsMax && env_int("LT_FORCE_DIRECT", 0) == 0) {
      pl->dst = true;
      a.off_dbuf = fixed;
      fixed += do_den ? al16(2LL * a.FR * 4) : 0;
      a.off_nbuf = fixed;
      fixed += do_num ? al16(2LL * a.FR * 4) : 0;
    }
  }

  // streams staged through the ring (fixed slots 0 = W, 1 = alpha, 2 = alpha_num)
  auto set_stream = [&](int s, long long row) {
    a.st_row[s] = row;
    const long long ngmax = (row + 15) / 16 + 1;
    a.st_ninstr[s] = row > 0 ? ceil_div(ngmax, 64) : 0;
  };
  int instr = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    const bool with_w = attempt == 0 && env_int("LT_NO_WSTAGE", 0) == 0;
    set_stream(0, with_w ? FRB : 0);
    set_stream(1, (kind == 1 && do_den) ? (long long)C * 4 : 0);
    set_stream(2, (kind == 1 && do_num) ? (long long)NP * 4 : 0);
    int slot = 0;
    instr = 0;
    for (int s = 0; s < kMaxStreams; ++s) {
      a.st_off[s] = slot;
      slot += a.st_ninstr[s] * 1024;
      instr += a.st_ninstr[s];
    }
    a.slot_bytes = slot;
    if (instr == 0) { a.S = 1; a.P = 0; break; }
    const int gmax = ceil_div(instr, a.load_waves);
    int S = (kLdsMax - al16(fixed)) / slot;
    S = std::min(S, env_int("LT_RING_SLOTS", 24));
    // outstanding DMA instructions per loader wave must stay <= 63
    while (S >= 3 && (S - 2) * gmax > 63) --S;
    if (S >= 2) {
      a.S = S; a.P = S - 1;
      break;
    }
    if (!with_w) return fail(LT_EUNSUPPORTED, "lattice row does not fit in LDS");
  }
  pl->wst = a.st_ninstr[0] > 0;
  if (instr == 0) a.load_waves = 0;
  a.gw0 = a.gw1 = 0;
  for (int k = 0; k < instr; ++k) (k % a.load_waves == 0 ? a.gw0 : a.gw1)++;
  a.off_ring = al16(fixed);
  pl->lds_bytes = a.off_ring + a.S * a.slot_bytes;
  if (pl->lds_bytes > kLdsMax) return fail(LT_EUNSUPPORTED, "LDS plan exceeds 160 KiB");
  pl->threads = 64 * (a.den_waves + a.aux_waves + a.load_waves);
  if (pl->threads > 1024) return fail(LT_EUNSUPPORTED, "too many waves");
  return LT_OK;
}

template <typename K>
int launch(K kernel, const Plan& pl, int grid, hipStream_t st) {
  if (grid == 0) return LT_OK;
  hipError_t e = hipFuncSetAttribute((const void*)kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, pl.lds_bytes);
  if (e != hipSuccess) return hip_check(e, "hipFuncSetAttribute");
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(pl.threads), pl.lds_bytes, st, pl.a);
  return hip_check(hipGetLastError(), "kernel launch");
}

template <int MODE, bool BF16, bool WST>
int launch_fwd_t(const Plan& pl, int grid, hipStream_t st) {
  switch (pl.tmax) {
    case 4: return launch(fwd_kernel<MODE, BF16, WST, 4>, pl, grid, st);
    case 8: return launch(fwd_kernel<MODE, BF16, WST, 8>, pl, grid, st);
    default: return launch(fwd_kernel<MODE, BF16, WST, 16>, pl, grid, st);
  }
}
template <int MODE>
int launch_fwd_m(const Plan& pl, bool bf16, int grid, hipStream_t st) {
  if (bf16) return pl.wst ? launch_fwd_t<MODE, true, true>(pl, grid, st)
                          : launch_fwd_t<MODE, true, false>(pl, grid, st);
  return pl.wst ? launch_fwd_t<MODE, false, true>(pl, grid, st)
                : launch_fwd_t<MODE, false, false>(pl, grid, st);
}
int launch_fwd(int mode, const Plan& pl, bool bf16, int grid, hipStream_t st) {
  switch (mode) {
    case M_LOG: return launch_fwd_m<M_LOG>(pl, bf16, grid, st);
    case M_MAX: return launch_fwd_m<M_MAX>(pl, bf16, grid, st);
    case M_REAL: return launch_fwd_m<M_REAL>(pl, bf16, grid, st);
  }
  return fail(LT_EINVAL, "bad semiring");
}

template <bool BF16, bool WST, bool DST>
int launch_bwd_t(const Plan& pl, int grid, hipStream_t st) {
  switch (pl.tmax) {
    case 4: return launch(bwd_kernel<BF16, WST, DST, 4>, pl, grid, st);
    case 8: return launch(bwd_kernel<BF16, WST, DST, 8>, pl, grid, st);
    default: return launch(bwd_kernel<BF16, WST, DST, 16>, pl, grid, st);
  }
}
int launch_bwd(const Plan& pl, bool bf16, int grid, hipStream_t st) {
  if (bf16) {
    if (pl.wst) return pl.dst ? launch_bwd_t<true, true, true>(pl, grid, st)
                              : launch_bwd_t<true, true, false>(pl, grid, st);
    return pl.dst ? launch_bwd_t<true, false, true>(pl, grid, st)
                  : launch_bwd_t<true, false, false>(pl, grid, st);
  }
  if (pl.wst) return pl.dst ? launch_bwd_t<false, true, true>(pl, grid, st)
                            : launch_bwd_t<false, true, false>(pl, grid, st);
  return pl.dst ? launch_bwd_t<false, false, true>(pl, grid, st)
                : launch_bwd_t<false, false, false>(pl, grid, st);
}

void bind_streams(KArgs& a, const void* W, const float* alpha, const float* alpha_num) {
  a.st_base[0] = (const unsigned char*)W;
  a.st_base[1] = (const unsigned char*)alpha;
  a.st_base[2] = (const unsigned char*)alpha_num;
  a.W = (const unsigned char*)W;
}

bool misaligned(const void* p) { return ((uintptr_t)p & 15) != 0; }

size_t side_bytes(const lt_problem* pb) {
  const long long NP = pb->max_labels + 1;
  const long long nm = (long long)pb->batch * pb->max_frames * NP * 2 * 4;
  const long long cs = (long long)pb->batch * NP * 2 * 4;
  return (size_t)(((nm + 255) & ~255LL) + cs);
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* lt_last_error(void) { return g_err.c_str(); }
const char* lt_version(void) { return "last_torch_amd-lattice 0.1.0 (gfx950)"; }

int lt_num_context_states(int32_t V, int32_t n, int64_t* out) {
  NGram g;
  const int rc = make_ngram(V, n, &g);
  if (rc != LT_OK) return rc;
  if (out) *out = g.C;
  return LT_OK;
}

int lt_den_forward(const lt_problem* pb, int32_t semiring, const void* W,
                   const int32_t* num_frames, float* dist, float* alpha, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (semiring < 0 || semiring > 2) return fail(LT_EINVAL, "bad semiring");
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !dist) return fail(LT_EINVAL, "null pointer");
  if (misaligned(W)) return fail(LT_EINVAL, "W must be 16-byte aligned");
  lt_problem p2 = *pb;
  p2.max_labels = 0;
  Plan pl;
  if ((rc = plan(&p2, g, 0, F_DEN, &pl))) return rc;
  bind_streams(pl.a, W, nullptr, nullptr);
  pl.a.nfr = num_frames;
  pl.a.dist = dist;
  pl.a.alpha = alpha;
  return launch_fwd(semiring, pl, pb->weight_dtype == LT_DTYPE_BF16, pb->batch,
                    (hipStream_t)stream);
}

int lt_num_forward(const lt_problem* pb, int32_t semiring, const void* W,
                   const int32_t* num_frames, const int32_t* labels,
                   const int32_t* num_labels, float* num, float* alpha_num, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (semiring < 0 || semiring > 2) return fail(LT_EINVAL, "bad semiring");
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !num_labels || !num || (pb->max_labels > 0 && !labels))
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W)) return fail(LT_EINVAL, "W must be 16-byte aligned");
  Plan pl;
  if ((rc = plan(pb, g, 0, F_NUM, &pl))) return rc;
  bind_streams(pl.a, W, nullptr, nullptr);
  pl.a.nfr = num_frames;
  pl.a.labels = labels;
  pl.a.nlab = num_labels;
  pl.a.num = num;
  pl.a.alpha_num = alpha_num;
  return launch_fwd(semiring, pl, pb->weight_dtype == LT_DTYPE_BF16, pb->batch,
                    (hipStream_t)stream);
}

int lt_loss_forward(const lt_problem* pb, int32_t local_norm, const void* W,
                    const int32_t* num_frames, const int32_t* labels,
                    const int32_t* num_labels, float* loss, float* log_z, float* num,
                    float* alpha, float* alpha_num, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !num_labels || !loss || (pb->max_labels > 0 && !labels))
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W)) return fail(LT_EINVAL, "W must be 16-byte aligned");
  const int flags = F_NUM | F_LOSS | (local_norm ? F_LOCAL : F_DEN);
  Plan pl;
  if ((rc = plan(pb, g, 0, flags, &pl))) return rc;
  bind_streams(pl.a, W, nullptr, nullptr);
  pl.a.nfr = num_frames;
  pl.a.labels = labels;
  pl.a.nlab = num_labels;
  pl.a.loss = loss;
  pl.a.dist = log_z;
  pl.a.num = num;
  pl.a.alpha = alpha;
  pl.a.alpha_num = alpha_num;
  return launch_fwd(M_LOG, pl, pb->weight_dtype == LT_DTYPE_BF16, pb->batch,
                    (hipStream_t)stream);
}

int lt_den_backward(const lt_problem* pb, const void* W, const int32_t* num_frames,
                    const float* log_z, const float* alpha, const float* grad, void* dW,
                    void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !log_z || !alpha || !dW) return fail(LT_EINVAL, "null pointer");
  if (misaligned(W) || misaligned(alpha)) return fail(LT_EINVAL, "W/alpha must be 16-byte aligned");
  lt_problem p2 = *pb;
  p2.max_labels = 0;
  Plan pl;
  if ((rc = plan(&p2, g, 1, F_DEN, &pl))) return rc;
  bind_streams(pl.a, W, alpha, nullptr);
  pl.a.nfr = num_frames;
  pl.a.log_z_in = log_z;
  pl.a.grad = grad;
  pl.a.dW = dW;
  return launch_bwd(pl, pb->weight_dtype == LT_DTYPE_BF16, pb->batch, (hipStream_t)stream);
}

int lt_loss_backward_workspace_bytes(const lt_problem* pb, int32_t local_norm, size_t* bytes) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  Plan pl;
  const int flags = F_NUM | (local_norm ? F_LOCAL : F_DEN);
  if ((rc = plan(pb, g, 1, flags, &pl))) return rc;
  if (bytes) *bytes = pl.dst ? 0 : side_bytes(pb);
  return LT_OK;
}

int lt_loss_backward(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels,
                     const int32_t* num_labels, const float* log_z, const float* num,
                     const float* alpha, const float* alpha_num, const float* grad, void* dW,
                     void* workspace, size_t workspace_bytes, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !num_labels || !num || !alpha_num || !dW ||
      (pb->max_labels > 0 && !labels) || (!local_norm && (!log_z || !alpha)))
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W) || (alpha && misaligned(alpha)) || misaligned(alpha_num))
    return fail(LT_EINVAL, "W/alpha/alpha_num must be 16-byte aligned");
  const int flags = F_NUM | (local_norm ? F_LOCAL : F_DEN);
  Plan pl;
  if ((rc = plan(pb, g, 1, flags, &pl))) return rc;
  bind_streams(pl.a, W, local_norm ? nullptr : alpha, alpha_num);
  KArgs& a = pl.a;
  a.nfr = num_frames;
  a.labels = labels;
  a.nlab = num_labels;
  a.log_z_in = log_z;
  a.num_in = num;
  a.grad = grad;
  a.dW = dW;
  if (!pl.dst) {
    const size_t need = side_bytes(pb);
    if (!workspace || workspace_bytes < need) return fail(LT_EINVAL, "workspace too small");
    const long long NP = pb->max_labels + 1;
    const long long nm = (long long)pb->batch * pb->max_frames * NP * 2 * 4;
    a.nm_side = (float*)workspace;
    a.ctx_side = (int*)((char*)workspace + ((nm + 255) & ~255LL));
  }
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = launch_bwd(pl, bf16, pb->batch, st))) return rc;
  if (!pl.dst) {
    const long long n = (long long)pb->batch * pb->max_frames;
    const int blocks = (int)((n + 255) / 256);
    if (blocks > 0) {
      if (bf16) hipLaunchKernelGGL(num_scatter_kernel<true>, dim3(blocks), dim3(256), 0, st, a);
      else hipLaunchKernelGGL(num_scatter_kernel<false>, dim3(blocks), dim3(256), 0, st, a);
      if ((rc = hip_check(hipGetLastError(), "scatter launch"))) return rc;
    }
  }
  return LT_OK;
}

int lt_viterbi_workspace_bytes(const lt_problem* pb, size_t* bytes) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  const long long bpb = (long long)pb->batch * pb->max_frames * g.C;
  if (bytes) *bytes = (size_t)(((bpb + 255) & ~255LL) + 4LL * pb->batch + 256);
  return LT_OK;
}

int lt_viterbi(const lt_problem* pb, const void* W, const int32_t* num_frames,
               int32_t label_convention, int64_t* labels, float* path_weight,
               const float* grad, void* arcs, void* workspace, size_t workspace_bytes,
               void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (!W || !num_frames || !labels || !path_weight || !workspace)
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W)) return fail(LT_EINVAL, "W must be 16-byte aligned");
  if (g.K + 1 > 255) return fail(LT_EUNSUPPORTED, "vocab too large for 8-bit backpointers");
  size_t need = 0;
  lt_viterbi_workspace_bytes(pb, &need);
  if (workspace_bytes < need) return fail(LT_EINVAL, "workspace too small");
  const long long bpb = (long long)pb->batch * pb->max_frames * g.C;
  unsigned char* bp = (unsigned char*)workspace;
  int* qstar = (int*)((char*)workspace + ((bpb + 255) & ~255LL));
  lt_problem p2 = *pb;
  p2.max_labels = 0;
  Plan pl;
  if ((rc = plan(&p2, g, 0, F_DEN, &pl))) return rc;
  bind_streams(pl.a, W, nullptr, nullptr);
  pl.a.nfr = num_frames;
  pl.a.dist = path_weight;
  pl.a.bp = bp;
  pl.a.qstar = qstar;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = launch_fwd(M_MAX, pl, bf16, pb->batch, st))) return rc;
  BtArgs bt;
  bt.bp = bp; bt.qstar = qstar; bt.nfr = num_frames; bt.grad = grad;
  bt.labels = (long long*)labels; bt.arcs = arcs;
  bt.B = pb->batch; bt.T = pb->max_frames;
  bt.conv = label_convention; bt.arcs_bf16 = bf16; bt.g = g;
  const int budget = 60 * 1024;
  bt.chunk = std::max(1, budget / g.C);
  const int shm = 16 + bt.chunk * g.C;
  if (bf16) hipLaunchKernelGGL(backtrace_kernel<true>, dim3(pb->batch), dim3(256), shm, st, bt);
  else hipLaunchKernelGGL(backtrace_kernel<false>, dim3(pb->batch), dim3(256), shm, st, bt);
  return hip_check(hipGetLastError(), "backtrace launch");
}

}  // extern "C"
