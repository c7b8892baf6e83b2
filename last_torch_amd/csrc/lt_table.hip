// lt_table.hip -- recognition-lattice kernels for ANY context dependency given
// as a next-state table and for both alignment lattices (reference
// file:line in last_torch/):
//   context   NextStateTable                       contexts.py:266-320
//             (or FullNGram.next_state_table()     contexts.py:258-263)
//   alignment FrameDependent          (K = 0)      alignments.py:250-329
//             FrameLabelDependent(K)  (K >= 1)     alignments.py:331-432
// driven as RecognitionLattice._forward / _string_forward / forward /
// shortest_path do (lattices.py:131-496), with alignment-state-invariant
// weights (lattices.py:444-447): every expansion of a frame uses the same W.
//
// forward_reduce is the (+) over each state's in-arcs (its intended
// semantics; the reference's NextStateTable.forward_reduce is defect D8).
// The in-arcs come as a CSR over the next state, ascending (source, label)
// -- the order FullNGram.forward_reduce reduces in, which fixes the
// MaxTropical tie rule (first argmax, semirings.py:382).
//
// One workgroup per utterance; the state vectors live in LDS and each frame
// is a few barrier-separated sweeps over the states (one per expansion). The
// FullNGram x FrameDependent shapes of the benchmark use the tuned kernels
// of lt_lattice.hip / lt_pipe.hip; this file is the general path.
#include <type_traits>
#include <vector>

#include "lt_kernels.h"

namespace {

struct TArgs {
  const unsigned char* W;
  const int* nfr;
  const int* table;   // [C, V] next state of (p, y)
  const int* in_off;  // [C+1]
  const int* in_arc;  // [C*V] arc id p*V + (y-1), grouped by next state
  const int* labels;  // [B, U]
  const int* nlab;    // [B]
  float* dist;        // den: distance [B]; num: numerator [B]
  float* alpha;       // history [B,T,S] (state before frame t), nullable
  float* loss;        // num forward with dist_in: loss [B]
  const float* den_in;  // log_z [B] (num forward: loss = log_z - num)
  const float* num_in;  // numerator [B] (backward)
  const float* hist;    // backward: alpha history [B,T,S]
  float* dW;            // fp32 gradient (bf16 W: a workspace copy, converted at the end)
  int* bp;              // Viterbi: [B,T,KK,C] winning in-arc position (-1: blank)
  unsigned char* win;   // Viterbi, K >= 1: [B,T,C] winning expansion count
  int* qstar;           // Viterbi: [B] best final state
  long long* vlabels;   // Viterbi: [B, T*A]
  int B, T, U, C, V, R, K, conv, local;
  int acc;  // tab_bwd_den_kernel: FrameLabelDependent dW sums in LDS
  const float* gin;  // den backward: per-utterance gradient factor [B] (nullable)
  // numerator backward run beside the denominator's (lt_table_loss_grad):
  // the chain heads' marginal sums go to nsub [B,T,2S] and their elements to
  // ntab [B,2S] (-1: none), subtracted from dW afterwards (tab_apply_kernel)
  float* nsub;
  int* ntab;
  // dense-bigram FrameLabelDependent (lt_table_loss_grad): the lexical alphas
  // L^i alpha_t, i = 1..K, [B,T,K,C], written by the forward and read by the
  // backward instead of recomputed (nullable)
  float* lx;
};

// Copies the graph arrays to LDS at g (ints: in_off [C+1], in_arc [C*V],
// table [C*V]) when GST, and returns the arrays to use (compile-time choice,
// so the compiler knows which memory every access goes to).
template <bool GST>
LT_DEVINL void t_graph(const TArgs& a, int* g, const int** in_off, const int** in_arc,
                       const int** table) {
  if constexpr (!GST) {
    *in_off = a.in_off;
    *in_arc = a.in_arc;
    *table = a.table;
    return;
  }
  const int C = a.C, CV = a.C * a.V;
  for (int i = threadIdx.x; i <= C; i += blockDim.x) g[i] = a.in_off[i];
  for (int i = threadIdx.x; i < CV; i += blockDim.x) {
    const int id = a.in_arc[i];
    const int p = id / a.V;
    g[C + 1 + i] = p | ((id - p * a.V) << 16);  // DenGraphP packing
    g[C + 1 + CV + i] = a.table[i];
  }
  *in_off = g;
  *in_arc = g + C + 1;
  *table = g + C + 1 + CV;
}

LT_DEVINL float t_safe(float x) { return __builtin_isfinite(x) ? x : 0.f; }
// _LogAddExp (semirings.py:248-255)
LT_DEVINL float t_lae(float a, float b) {
  const float m = fmaxf(a, b);
  const float c = t_safe(m);
  return c + lt_log_acc(lt_exp(a - c) + lt_exp(b - c));
}
// running logsumexp (m, s): the result is m + log(s) with the safe max
struct Lse {
  float m = -kInf, s = 0.f;
  LT_DEVINL void add(float x) {
    if (x == -kInf) return;
    if (x > m) {
      s = s * lt_exp(m - x) + 1.f;
      m = x;
    } else {
      s += lt_exp(x - m);
    }
  }
  LT_DEVINL float get() const { return s > 0.f ? m + lt_log_acc(s) : -kInf; }
};

template <int SR>
LT_DEVINL float t_zero() { return SR == M_REAL ? 0.f : -kInf; }
template <int SR>
LT_DEVINL float t_one() { return SR == M_REAL ? 1.f : 0.f; }
template <int SR>
LT_DEVINL float t_times(float a, float b) { return SR == M_REAL ? a * b : a + b; }

constexpr int kTabMaxThreads = 512;
#ifndef LT_TAB_BWD_WAVES
#define LT_TAB_BWD_WAVES 4  // waves of the dense FrameLabelDependent backward (2 or 4)
#endif
#ifndef LT_TAB_DENSE
#define LT_TAB_DENSE 1  // the dense-bigram FrameLabelDependent kernels (diagnostic builds: 0 = generic)
#endif

// Log vectors are kept relative to an integer offset near their maximum
// (exact in fp32), so a recursion over T frames rounds small numbers, not
// values of magnitude |log_z| (the tuned kernels' scheme): the
// offset after a frame is floor(max) of its new vector.
// That offset without a pass of its own: the threads that write the new
// vector's values fold them into an LDS slot (ds_max on an order-preserving
// int image) and, after the barrier that publishes the vector, every thread
// reads the slot. Three slots rotate: frame t writes slot t % 3, reads it
// after its barrier, and resets slot (t + 1) % 3 for the next frame (the
// last frame that read it was t - 2).
LT_DEVINL int t_ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
LT_DEVINL float t_unord(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }
struct MaxSlots {
  int* s;  // [3] in LDS
  LT_DEVINL void init() const {
    if (threadIdx.x < 3) s[threadIdx.x] = t_ord(-kInf);
  }
  LT_DEVINL void put(int t, float v) const { atomicMax(s + t % 3, t_ord(v)); }
  LT_DEVINL void reset_next(int t) const {
    if (threadIdx.x == 0) s[(t + 1) % 3] = t_ord(-kInf);
  }
  // after the barrier: the integer offset floor(max) (0 when not finite)
  LT_DEVINL float shift(int t) const {
    const float m = t_unord(s[t % 3]);
    return __builtin_isfinite(m) ? floorf(m) : 0.f;
  }
};

// Graph accessors: the context lattice (states p, in-arcs from the CSR) and
// the string acceptor (positions u, one in-arc from u-1; lattices.py:314-338).
struct DenGraph {
  const int* in_off;
  const int* in_arc;
  int V, R;
  LT_DEVINL int blank(int q) const { return q * R; }
  LT_DEVINL int nin(int q) const { return in_off[q + 1] - in_off[q]; }
  LT_DEVINL int pos0(int q) const { return in_off[q]; }
  LT_DEVINL void arc(int pos, int q, int* src, int* widx) const {
    (void)q;
    const int id = in_arc[pos];
    const int p = id / V;
    *src = p;
    *widx = p * R + (id - p * V) + 1;
  }
};
// The LDS copy of the CSR holds src | (label - 1) << 16 (no division).
struct DenGraphP {
  const int* in_off;
  const int* in_arc;
  int V, R;
  LT_DEVINL int blank(int q) const { return q * R; }
  LT_DEVINL int nin(int q) const { return in_off[q + 1] - in_off[q]; }
  LT_DEVINL int pos0(int q) const { return in_off[q]; }
  LT_DEVINL void arc(int pos, int q, int* src, int* widx) const {
    (void)q;
    const int v = in_arc[pos];
    const int p = v & 0xffff;
    *src = p;
    *widx = p * R + (v >> 16) + 1;
  }
};
struct NumGraph {
  const int* ctx;  // [S] ctx state * R
  const int* yn;   // [S] label class of the arc leaving u
  LT_DEVINL int blank(int u) const { return ctx[u]; }
  LT_DEVINL int nin(int u) const { return u >= 1 ? 1 : 0; }
  LT_DEVINL int pos0(int u) const { return u - 1; }
  LT_DEVINL void arc(int pos, int u, int* src, int* widx) const {
    (void)pos;
    *src = u - 1;
    *widx = ctx[u - 1] + yn[u - 1];
  }
};

// The string acceptor over a compact per-frame copy of its weights:
// wc[2u] = blank of u, wc[2u+1] = the arc leaving u (lattices.py:314-338)
struct NumGraphC {
  LT_DEVINL int blank(int u) const { return 2 * u; }
  LT_DEVINL int nin(int u) const { return u >= 1 ? 1 : 0; }
  LT_DEVINL int pos0(int u) const { return u - 1; }
  LT_DEVINL void arc(int pos, int u, int* src, int* widx) const {
    (void)pos;
    *src = u - 1;
    *widx = 2 * u - 1;
  }
};

// Register staging of a strided per-frame gather (element e -> ld(e)): the
// next frame's values are loaded while this frame computes, so a frame costs
// no memory round trip of its own (N rounds per thread; the rest is loaded
// directly when stored)
template <int N>
struct RegStage {
  float r[N];
  template <typename F>
  LT_DEVINL void fetch(int n, const F& ld) {
#pragma unroll
    for (int u = 0; u < N; ++u) {
      const int e = u * blockDim.x + threadIdx.x;
      r[u] = e < n ? ld(e) : 0.f;
    }
  }
  template <typename F>
  LT_DEVINL void store(float* dst, int n, const F& ld) const {
#pragma unroll
    for (int u = 0; u < N; ++u) {
      const int e = u * blockDim.x + threadIdx.x;
      if (e < n) dst[e] = r[u];
    }
    for (int e = N * blockDim.x + threadIdx.x; e < n; e += blockDim.x) dst[e] = ld(e);
  }
};

// (+) over the in-arcs of q of x[src] (x) w; MaxTropical keeps the first max
// xo: an offset taken off every x (the pending integer shift of a vector
// kept unshifted; 0 leaves x exact)
template <int SR, typename G, typename WR>
LT_DEVINL float t_reduce(const G& g, int q, const float* x, const WR& wr, int* argpos,
                         float xo = 0.f) {
  const int n = g.nin(q), p0 = g.pos0(q);
  if constexpr (SR == M_LOG) {
    Lse l;
    for (int k = 0; k < n; ++k) {
      int src, wi;
      g.arc(p0 + k, q, &src, &wi);
      l.add((x[src] - xo) + wr(wi));
    }
    return l.get();
  } else if constexpr (SR == M_MAX) {
    float r = -kInf;
    int ra = -1;
    for (int k = 0; k < n; ++k) {
      int src, wi;
      g.arc(p0 + k, q, &src, &wi);
      const float v = (x[src] - xo) + wr(wi);
      if (ra < 0 || v > r) {
        r = v;
        ra = p0 + k;
      }
    }
    if (argpos) *argpos = ra;
    return r;
  } else {
    float r = 0.f;
    for (int k = 0; k < n; ++k) {
      int src, wi;
      g.arc(p0 + k, q, &src, &wi);
      r += x[src] * wr(wi);
    }
    return r;
  }
}

// Merge a running logsumexp over G aligned lanes (xor shuffles; every lane of
// the wave takes part) -- the lanes then hold the group's total.
template <int G>
LT_DEVINL void lse_merge(Lse& l) {
  for (int o = 1; o < G; o <<= 1) {
    const float m2 = __shfl_xor(l.m, o, 64), s2 = __shfl_xor(l.s, o, 64);
    const float M = fmaxf(l.m, m2);
    if (M == -kInf) {
      l.s = 0.f;
    } else {
      l.s = l.s * lt_exp(l.m - M) + s2 * lt_exp(m2 - M);
      l.m = M;
    }
  }
}

// t_reduce with G lanes per state: lane j takes in-arcs j, j+G, ... and the
// partials merge over the group (MaxTropical: the first max by CSR position,
// as the serial reduce). `valid` false: the lane joins the shuffles only.
template <int SR, int G, typename Gr, typename WR>
LT_DEVINL float t_reduce_g(const Gr& g, int q, bool valid, const float* x, const WR& wr,
                           int* argpos, float xo = 0.f) {
  if constexpr (G == 1) {
    return valid ? t_reduce<SR>(g, q, x, wr, argpos, xo) : t_zero<SR>();
  } else {
    // the lane's terms are gathered NU at a time (independent LDS reads in
    // flight together), then folded in CSR order
    constexpr int NU = 8;
    const int j = threadIdx.x & (G - 1);
    const int n = valid ? g.nin(q) : 0, p0 = valid ? g.pos0(q) : 0;
    float acc = SR == M_REAL ? 0.f : -kInf;  // MAX: best; LOG: running max
    float ls = 0.f;                          // LOG: running sum at `acc`
    int ra = -1;
    for (int k0 = j; k0 < n; k0 += G * NU) {
      float v[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const int k = k0 + G * i;
        v[i] = SR == M_REAL ? 0.f : -kInf;
        if (k < n) {
          int src, wi;
          g.arc(p0 + k, q, &src, &wi);
          v[i] = SR == M_REAL ? x[src] * wr(wi) : (x[src] - xo) + wr(wi);
        }
      }
      if constexpr (SR == M_LOG) {
        float cm = v[0];
#pragma unroll
        for (int i = 1; i < NU; ++i) cm = fmaxf(cm, v[i]);
        if (cm == kInf) {  // +inf dominates (the reference's safe max)
          acc = kInf;
          ls = 1.f;
        } else if (cm != -kInf && acc != kInf) {
          float cs = 0.f;
#pragma unroll
          for (int i = 0; i < NU; ++i) cs += lt_exp(v[i] - cm);
          const float M = fmaxf(acc, cm);
          ls = ls * lt_exp(acc - M) + cs * lt_exp(cm - M);
          acc = M;
        }
      } else if constexpr (SR == M_MAX) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          const int k = k0 + G * i;
          if (k < n && (ra < 0 || v[i] > acc)) {
            acc = v[i];
            ra = p0 + k;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NU; ++i) acc += v[i];
      }
    }
    if constexpr (SR == M_LOG) {
      Lse l;
      l.m = acc;
      l.s = ls;
      lse_merge<G>(l);
      return l.get();
    } else if constexpr (SR == M_MAX) {
      float r = acc;
      for (int o = 1; o < G; o <<= 1) {
        const float r2 = __shfl_xor(r, o, 64);
        const int a2 = __shfl_xor(ra, o, 64);
        if (a2 >= 0 && (ra < 0 || r2 > r || (r2 == r && a2 < ra))) {
          r = r2;
          ra = a2;
        }
      }
      if (argpos) *argpos = ra;
      return r;
    } else {
      float r = acc;
      for (int o = 1; o < G; o <<= 1) r += __shfl_xor(r, o, 64);
      return r;
    }
  }
}

// context_states / next-label classes of the string (contexts.py:109-146,
// lattices.py:314-315 and 336-338); one thread
LT_DEVINL void t_walk(const TArgs& a, int b, int* ctx, int* yn) {
  int c = 0;
  for (int u = 0; u <= a.U; ++u) {
    ctx[u] = c * a.R;
    int y = u < a.U ? a.labels[(long long)b * a.U + u] : 1;
    if (u < a.U && (y < 0 || y > a.V)) y = 0;
    yn[u] = y < 1 ? 1 : y;
    if (u < a.U && y != 0) c = a.table[c * a.V + y - 1];
  }
}

// Frame staging: the first kPf*blockDim weights of frame t+1 are loaded into
// registers while frame t is processed (one memory round trip per frame,
// hidden), the rest of a large frame in batches of kPf loads per thread.
constexpr int kPf = 8;
template <bool BF16>
struct FrameStage {
  float r[kPf];
  LT_DEVINL void fetch(const unsigned char* wf, long long FR) {
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
      const long long e = (long long)u * blockDim.x + threadIdx.x;
      r[u] = (wf && e < FR) ? ldw<BF16>(wf, e) : 0.f;
    }
  }
  LT_DEVINL void store(float* wl, const unsigned char* wf, long long FR) {
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
      const long long e = (long long)u * blockDim.x + threadIdx.x;
      if (e < FR) wl[e] = r[u];
    }
    for (long long e0 = (long long)kPf * blockDim.x; e0 < FR; e0 += (long long)kPf * blockDim.x) {
      float t[kPf];
#pragma unroll
      for (int u = 0; u < kPf; ++u) {
        const long long e = e0 + (long long)u * blockDim.x + threadIdx.x;
        t[u] = e < FR ? ldw<BF16>(wf, e) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kPf; ++u) {
        const long long e = e0 + (long long)u * blockDim.x + threadIdx.x;
        if (e < FR) wl[e] = t[u];
      }
    }
  }
};

// ---- string forward in Log (lattices.py:250-377, alignments.py:320-329 and
// :420-432 for FrameLabelDependent): every position as an exact integer part
// plus a fraction (lae_split, lt_kernels.h) -- the positions span hundreds
// of nats within a frame, so one offset per frame would round each value at
// its own magnitude every frame (measured: up to 16 units of 2^-24 |num|
// after 1,000 FrameLabelDependent(2) frames). History rows and num are i + f.
template <bool BF16>
LT_DEVINL void tab_str_fwd_log(const TArgs& a, const int b, float* sm) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int U = a.U, S = U + 1, K = a.K;
  float* ia = sm;  // alpha: integer parts, fractions
  float* fa = ia + S;
  float* il = fa + S;  // the lexical chain L^i alpha
  float* fl = il + S;
  float* ic = fl + S;  // the frame's sum (FrameLabelDependent) / the new alpha
  float* fc = ic + S;
  int* ctx = (int*)(fc + S);
  int* yn = ctx + S;
  float* wl = (float*)(yn + S);  // [2S]: blank of u, then the arc leaving u
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  for (int u = tid; u < S; u += nthr) {
    ia[u] = u == 0 ? 0.f : -kInf;
    fa[u] = 0.f;
  }
  if (tid == 0) t_walk(a, b, ctx, yn);
  __syncthreads();
  const long long fbytes = (long long)a.C * a.R * (BF16 ? 2 : 4);
  const unsigned char* wb = a.W + (long long)b * a.T * fbytes;
  auto ldc = [&](const unsigned char* w) {
    return [=](int e) { return ldw<BF16>(w, ctx[e >> 1] + ((e & 1) ? yn[e >> 1] : 0)); };
  };
  RegStage<2> cs;
  cs.fetch(nf > 0 ? 2 * S : 0, ldc(wb));
  if (K == 0) {
    // FrameDependent: ONE barrier a frame -- (ia, fa) and (ic, fc) swap
    // roles each frame, and the next frame's two weights per position go to
    // the other compact buffer (il / fl, unused without expansions) while
    // this frame reads its own
    float* wl1 = il;  // [2S]
    if (nf > 0) {
      cs.store(wl, 2 * S, ldc(wb));
      cs.fetch(nf > 1 ? 2 * S : 0, ldc(wb + fbytes));
    }
    __syncthreads();
    float *pi = ia, *pf = fa, *qi = ic, *qf = fc;
    for (int t = 0; t < a.T; ++t) {
      if (a.alpha)
        for (int u = tid; u < S; u += nthr) a.alpha[((long long)b * a.T + t) * S + u] = pi[u] + pf[u];
      if (t >= nf) continue;  // padding frames carry alpha (lattices.py:460-461)
      const float* w = (t & 1) ? wl1 : wl;
      for (int u = tid; u < S; u += nthr)
        lae_split(pi[u], pf[u] + w[2 * u], u >= 1 ? pi[u - 1] : -kInf,
                  u >= 1 ? pf[u - 1] + w[2 * u - 1] : 0.f, qi[u], qf[u]);
      if (t + 1 < nf) {
        const unsigned char* wn = wb + (t + 1) * fbytes;
        cs.store((t & 1) ? wl : wl1, 2 * S, ldc(wn));
        cs.fetch(t + 2 < nf ? 2 * S : 0, ldc(wn + fbytes));
      }
      __syncthreads();
      float* ti = pi; pi = qi; qi = ti;
      float* tf = pf; pf = qf; qf = tf;
    }
    if (tid == 0) {
      const int nl = a.nlab[b];
      const float r = (nl >= 0 && nl <= a.U) ? pi[nl] + pf[nl] : -kInf;
      a.dist[b] = r;  // lattices.py:375-377
      if (a.loss) a.loss[b] = a.local ? -r : a.den_in[b] - r;  // lattices.py:131-183
    }
    return;
  }
  for (int t = 0; t < a.T; ++t) {
    if (a.alpha)
      for (int u = tid; u < S; u += nthr) a.alpha[((long long)b * a.T + t) * S + u] = ia[u] + fa[u];
    if (t >= nf) continue;  // padding frames carry alpha (lattices.py:460-461)
    const unsigned char* wf = wb + t * fbytes;
    cs.store(wl, 2 * S, ldc(wf));
    cs.fetch(t + 1 < nf ? 2 * S : 0, ldc(wf + fbytes));
    __syncthreads();
    if (K == 0) {
      for (int u = tid; u < S; u += nthr)
        lae_split(ia[u], fa[u] + wl[2 * u], u >= 1 ? ia[u - 1] : -kInf,
                  u >= 1 ? fa[u - 1] + wl[2 * u - 1] : 0.f, ic[u], fc[u]);
    } else {
      // terminated[0] = alpha (x) blank; the chain starts at alpha
      for (int u = tid; u < S; u += nthr) {
        ic[u] = ia[u];
        fc[u] = fa[u] + wl[2 * u];
        il[u] = ia[u];
        fl[u] = fa[u];
      }
      __syncthreads();
      for (int i = 1; i <= K; ++i) {
        // last = shift_down(last (x) lexical): position u takes u - 1's
        // value times the arc leaving u - 1 (ia / fa hold it for one sweep)
        for (int u = tid; u < S; u += nthr) {
          ia[u] = u >= 1 ? il[u - 1] : -kInf;
          fa[u] = u >= 1 ? fl[u - 1] + wl[2 * u - 1] : 0.f;
        }
        __syncthreads();
        for (int u = tid; u < S; u += nthr) {
          il[u] = ia[u];
          fl[u] = fa[u];
          // (lt_table_loss_grad: L^i alpha kept for the string backward)
          if (a.lx) a.lx[(((long long)b * a.T + t) * K + (i - 1)) * S + u] = ia[u] + fa[u];
          lae_split(ic[u], fc[u], ia[u], fa[u] + wl[2 * u], ic[u], fc[u]);
        }
        __syncthreads();
      }
    }
    __syncthreads();
    for (int u = tid; u < S; u += nthr) {
      ia[u] = ic[u];
      fa[u] = fc[u];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int nl = a.nlab[b];
    const float r = (nl >= 0 && nl <= a.U) ? ia[nl] + fa[nl] : -kInf;
    a.dist[b] = r;  // lattices.py:375-377
    if (a.loss) a.loss[b] = a.local ? -r : a.den_in[b] - r;  // lattices.py:131-183
  }
}

// ---- forward, FrameDependent (K = 0) context lattice: ONE barrier a frame --
// The vector of frame t is kept unshifted in one of two LDS buffers, its
// pending integer shift applied where it is read ((v - sp) + w, the same two
// roundings as a shifted copy would take); the frame's weights are staged in
// the other of two LDS frame buffers by the previous frame (registers loaded
// a frame ahead). So a frame is: reduce (reads v_t, writes v_{t+1} and its
// max slot, stores frame t + 1's weights), barrier.
template <bool BF16, int SR, bool VIT, bool STAGE>
LT_DEVINL void tab_fwd_k0_body(const TArgs& a, const int b, float* sm) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int S = a.C, R = a.R;
  int* gsm = (int*)sm;
  const int* g_off;
  const int* g_arc;
  const int* g_tab;
  t_graph<STAGE>(a, gsm, &g_off, &g_arc, &g_tab);
  (void)g_tab;
  float* base = sm + (STAGE ? (a.C + 1 + 2 * a.C * a.V + 3) / 4 * 4 : 0);
  float* cur = base;       // [S] frame t's vector (unshifted)
  float* nxt = base + S;   // [S]
  const long long FR = (long long)a.C * R;
  float* w0 = base + 6 * S;  // STAGE: [2][FR] (the host's fwd_lds(S) + 4 FR more)
  float* w1 = w0 + FR;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  for (int q = tid; q < S; q += nthr) cur[q] = q == 0 ? t_one<SR>() : t_zero<SR>();
  __shared__ int slot_mem[3];
  const MaxSlots slots{slot_mem};
  slots.init();
  using DG = typename std::conditional<STAGE, DenGraphP, DenGraph>::type;
  DG dg{g_off, g_arc, a.V, R};
  constexpr int G = 8;
  constexpr bool kOff = SR == M_LOG;
  const long long fbytes = FR * (BF16 ? 2 : 4);
  const unsigned char* wb = a.W + (long long)b * a.T * fbytes;
  FrameStage<BF16> fs;
  if (STAGE && nf > 0) {
    fs.fetch(wb, FR);
    fs.store(w0, wb, FR);
    fs.fetch(nf > 1 ? wb + fbytes : nullptr, FR);
  }
  __syncthreads();
  float O = 0.f, sp = 0.f;  // the offset of cur - sp (sp included)
  for (int t = 0; t < a.T; ++t) {
    if (kOff && t >= 1 && t - 1 < nf) {  // frame t - 1's shift, once
      sp = slots.shift(t - 1);
      O += sp;
    }
    if (a.alpha)
      for (int q = tid; q < S; q += nthr)
        a.alpha[((long long)b * a.T + t) * S + q] = O + (cur[q] - sp);
    if (t >= nf) continue;  // padding frames carry alpha (lattices.py:460-461)
    const unsigned char* wf = wb + t * fbytes;
    const float* wl = (t & 1) ? w1 : w0;
    auto wr = [&](int i) { return STAGE ? wl[i] : ldw<BF16>(wf, i); };
    int* bpt = VIT ? a.bp + ((long long)b * a.T + t) * a.C : nullptr;
    for (int q0 = 0; q0 < S; q0 += nthr / G) {  // FrameDependent.forward, alignments.py:286-297
      const int q = q0 + tid / G;
      const bool valid = q < S;
      int ap = -1;
      const float r = t_reduce_g<SR, G>(dg, q, valid, cur, wr, &ap, sp);
      if (!valid || (tid & (G - 1))) continue;
      const float bt = t_times<SR>(cur[q] - sp, wr(dg.blank(q)));
      float o;
      if constexpr (SR == M_LOG) {
        o = t_lae(bt, r);
      } else if constexpr (SR == M_MAX) {
        const bool keep = ap < 0 || bt >= r;  // Maximum keeps a iff a >= b
        o = keep ? bt : r;
        if (VIT) bpt[q] = keep ? -1 : ap;
      } else {
        o = bt + r;
      }
      nxt[q] = o;
      if (kOff) slots.put(t, o);
    }
    if (STAGE && t + 1 < nf) {  // frame t + 1 into the other buffer, t + 2 in flight
      fs.store((t & 1) ? w0 : w1, wf + fbytes, FR);
      fs.fetch(t + 2 < nf ? wf + 2 * fbytes : nullptr, FR);
    }
    if (kOff) slots.reset_next(t);
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  if (kOff && nf >= 1 && nf == a.T) {  // the last frame's shift (no padding frame applied it)
    sp = slots.shift(nf - 1);
    O += sp;
  }
  if (tid == 0) {
    // (+)_q alpha_T[q] (lattices.py:496); MaxTropical: first max state
    float r = t_zero<SR>();
    int qs = 0;
    if constexpr (SR == M_LOG) {
      Lse l;
      for (int q = 0; q < S; ++q) l.add(cur[q] - sp);
      r = O + l.get();
    } else if constexpr (SR == M_MAX) {
      r = cur[0];
      for (int q = 1; q < S; ++q)
        if (cur[q] > r) {
          r = cur[q];
          qs = q;
        }
    } else {
      for (int q = 0; q < S; ++q) r += cur[q];
    }
    a.dist[b] = r;
    if (VIT) a.qstar[b] = qs;
  }
}

// ---- dense bigram context, FrameLabelDependent(K >= 1): one wave -----------
// FullNGram bigram (contexts.py:207-256 with n = 1): C = V + 1 states, every
// state p goes to state y on label y, so each lexical expansion of
// FrameLabelDependent.forward (alignments.py:363-377) is v'[y] = (+)_p v[p] w[p][y]
// over all C sources and nothing enters state 0. The generic kernel spends a
// frame on seven barrier-separated sweeps (CSR gathers, shuffle merges); here
// ONE wave keeps a frame in registers: lane (j, h) owns destination y = j + 1
// and sources [17h, 17h + 17), the two halves' partial logsumexps swap by
// permlane32, the vector goes between expansions through a 36-float LDS row.
// The other waves of the workgroup leave at once (no barrier after the
// dispatch). Decided by every thread from the next-state table.
LT_DEVINL bool tab_dense_bigram(const TArgs& a) {
  __shared__ int s_dense;
  if (threadIdx.x == 0) s_dense = (a.C == a.V + 1 && a.V <= 32 && a.V >= 1) ? 1 : 0;
  __syncthreads();
  if (s_dense)
    for (int e = threadIdx.x; e < a.C * a.V; e += blockDim.x)
      if (a.table[e] != e % a.V + 1) s_dense = 0;  // (benign race: every writer stores 0)
  __syncthreads();
  const bool d = s_dense != 0;
  __syncthreads();  // (s_dense is read by every thread before any can reuse it)
  return d;
}

LT_DEVINL int tdslot(int p) { return p < 17 ? p : p + 3; }  // sources of half 1 at 20..

template <bool BF16>
LT_DEVINL void tab_fwd_dense(const TArgs& a, const int b, float* sm) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, h = lane >> 5;
  const int V = a.V, C = a.C, R = a.R, K = a.K;
  const int y = j + 1;
  const bool live = y <= V;
  const int ns = h ? C - 17 : (C < 17 ? C : 17);  // sources of this half
  float* vb = sm;  // [40] the vector between expansions (slots tdslot(p)), -inf elsewhere
  for (int e = lane; e < 40; e += 64) vb[e] = -kInf;
  (void)ns;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const long long FR = (long long)C * R;
  const unsigned char* wb0 = a.W + (long long)b * a.T * FR * (BF16 ? 2 : 4);
  // the lane's weights of a frame: its sources' arcs into y, y's blank, w[0][0]
  float wc[17], wbl = 0.f, w00 = 0.f, nwc[17], nwbl = 0.f, nw00 = 0.f;
  auto fetch = [&](int t, float* c, float& bl, float& z) {
    const unsigned char* wf = wb0 + (long long)t * FR * (BF16 ? 2 : 4);
#pragma unroll
    for (int m = 0; m < 17; ++m)
      c[m] = (m < ns && live) ? ldw<BF16>(wf, (long long)(17 * h + m) * R + y) : 0.f;
    bl = live ? ldw<BF16>(wf, (long long)y * R) : 0.f;
    z = ldw<BF16>(wf, 0);
  };
  if (nf > 0) fetch(0, nwc, nwbl, nw00);
  float ay = -kInf, a0 = 0.f;  // alpha relative to the offset O (start state: one = 0)
  float O = 0.f;
  for (int t = 0; t < a.T; ++t) {
    // (the history row after this frame's weights are in and the next
    // frame's loads issued: the wait for those at the next frame's top then
    // covers this store too, a frame later, instead of stalling on it now)
    auto hist_row = [&]() {
      if (a.alpha) {
        float* row = a.alpha + ((long long)b * a.T + t) * C;
        if (h == 0 && live) row[y] = O + ay;
        if (lane == 32) row[0] = O + a0;
      }
    };
    if (t >= nf) {  // padding frames carry alpha (lattices.py:460-461)
      hist_row();
      continue;
    }
#pragma unroll
    for (int m = 0; m < 17; ++m) wc[m] = nwc[m];
    wbl = nwbl;
    w00 = nw00;
    if (t + 1 < nf) fetch(t + 1, nwc, nwbl, nw00);  // next frame under this one
    hist_row();
    // terminated[0] = alpha (x) blank; the chain starts at alpha
    float acc = live ? ay + wbl : -kInf;
    const float acc0 = a0 + w00;
    float v = ay;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (h == 0 && live) vb[tdslot(y)] = v;
    if (lane == 32) vb[0] = a0;
    for (int i = 1; i <= K; ++i) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float x[17];
#pragma unroll
      for (int m = 0; m < 17; ++m) {
        // every read unconditional (a read under a branch waits its own
        // latency): slots past the sources hold -inf for good
        x[m] = vb[20 * h + m] + wc[m];
      }
      const float mx = tree_max<17>(x);  // (balanced: short dependency chains)
      const float ch = t_safe(mx);
      float ex[17];
#pragma unroll
      for (int m = 0; m < 17; ++m) ex[m] = lt_exp(x[m] - ch);
      const float ss = tree_sum<17>(ex);
      // the other half's (max, sum) by permlane32 swap; the same expression on
      // both halves (commuted operands), so both hold the same value
      const auto pm = __builtin_amdgcn_permlane32_swap(__float_as_int(mx), __float_as_int(mx), false, false);
      const auto ps = __builtin_amdgcn_permlane32_swap(__float_as_int(ss), __float_as_int(ss), false, false);
      const float omx = __int_as_float(h ? pm[0] : pm[1]);
      const float oss = __int_as_float(h ? ps[0] : ps[1]);
      const float oc = t_safe(omx);
      const float c = t_safe(fmaxf(mx, omx));
      const float S = h ? oss * lt_exp(oc - c) + ss * lt_exp(ch - c) : ss * lt_exp(ch - c) + oss * lt_exp(oc - c);
      v = live ? (S > 0.f ? c + lt_log_acc(S) : -kInf) : -kInf;
      acc = live ? t_lae(acc, v + wbl) : -kInf;
      if (a.lx) {
        float* r = a.lx + (((long long)b * a.T + t) * K + (i - 1)) * C;
        if (h == 0 && live) r[y] = O + v;
        if (lane == 32) r[0] = -kInf;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (h == 0 && live) vb[tdslot(y)] = v;
      if (lane == 32) vb[0] = -kInf;  // nothing enters the start state
    }
    // the new vector over a new integer offset (floor of its max)
    float m = fmaxf(acc, acc0);
    m = gmax<6>(m, 6);
    const float sp = __builtin_isfinite(m) ? floorf(m) : 0.f;
    ay = acc - sp;
    a0 = acc0 - sp;
    O += sp;
  }
  // (+)_q alpha_T[q] (lattices.py:496)
  float m = fmaxf(h == 0 && live ? ay : -kInf, a0);
  m = gmax<6>(m, 6);
  const float c = t_safe(m);
  float e = h == 0 && live ? lt_exp(ay - c) : 0.f;
  if (lane == 32) e += lt_exp(a0 - c);
  e = gsum<6>(e, 6);
  if (lane == 0) a.dist[b] = e > 0.f ? O + c + lt_log_acc(e) : -kInf;
}

// The dense forward on TWO waves (V = 32): wave w takes destinations
// y = 16w + 1 .. 16w + 16, four lanes a destination, each over a quarter of
// the sources (9); the quarters merge by two xor shuffles, the vector goes
// between expansions through a double-buffered LDS row, one barrier each.
template <bool BF16>
LT_DEVINL void tab_fwd_dense2(const TArgs& a, const int b, float* sm) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int jj = lane & 15, qd = lane >> 4;
  const int C = a.C, R = a.R, K = a.K;
  const int y = 16 * w + jj + 1;  // the lane's destination (V = 32: always live)
  float* vbuf = sm;               // [2][48] the vector (slot p), -inf past C
  float* xch = vbuf + 96;         // [2 waves][4] partial maxima / sums
  for (int e = tid; e < 96; e += 128) vbuf[e] = -kInf;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const long long FR = (long long)C * R;
  const unsigned char* wb0 = a.W + (long long)b * a.T * FR * (BF16 ? 2 : 4);
  float wc[9], wbl = 0.f, w00 = 0.f, nwc[9], nwbl = 0.f, nw00 = 0.f;
  auto fetch = [&](int t, float* c, float& bl, float& z) {
    const unsigned char* wf = wb0 + (long long)t * FR * (BF16 ? 2 : 4);
#pragma unroll
    for (int m = 0; m < 9; ++m) {
      const int p = 9 * qd + m;
      c[m] = p < C ? ldw<BF16>(wf, (long long)p * R + y) : 0.f;
    }
    bl = ldw<BF16>(wf, (long long)y * R);
    z = ldw<BF16>(wf, 0);
  };
  auto sync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  // merge (m, s) running logsumexps over the four quarter lanes of a destination
  auto merge4 = [&](float m, float s) {
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
      const float c = t_safe(fmaxf(m, m2));
      s = s * lt_exp(t_safe(m) - c) + s2 * lt_exp(t_safe(m2) - c);
      m = fmaxf(m, m2);
    }
    return s > 0.f ? t_safe(m) + lt_log_acc(s) : -kInf;
  };
  if (nf > 0) fetch(0, nwc, nwbl, nw00);
  float ay = -kInf, a0 = 0.f, O = 0.f;  // alpha relative to O (start state: one = 0)
  for (int t = 0; t < a.T; ++t) {
    auto hist_row = [&]() {
      if (a.alpha) {
        float* row = a.alpha + ((long long)b * a.T + t) * C;
        if (qd == 0) row[y] = O + ay;
        if (tid == 0) row[0] = O + a0;
      }
    };
    if (t >= nf) {  // padding frames carry alpha (lattices.py:460-461)
      hist_row();
      continue;
    }
#pragma unroll
    for (int m = 0; m < 9; ++m) wc[m] = nwc[m];
    wbl = nwbl;
    w00 = nw00;
    if (t + 1 < nf) fetch(t + 1, nwc, nwbl, nw00);
    hist_row();
    float acc = ay + wbl;
    const float acc0 = a0 + w00;
    if (qd == 0) vbuf[y] = ay;
    if (tid == 0) vbuf[0] = a0;
    sync();
    for (int i = 1; i <= K; ++i) {
      const float* src = vbuf + ((i - 1) & 1) * 48;
      float x[9];
#pragma unroll
      for (int m = 0; m < 9; ++m) x[m] = src[9 * qd + m] + wc[m];  // (-inf past C)
      const float mx = tree_max<9>(x);
      const float ch = t_safe(mx);
#pragma unroll
      for (int m = 0; m < 9; ++m) x[m] = lt_exp(x[m] - ch);
      const float v = merge4(mx, tree_sum<9>(x));
      acc = t_lae(acc, v + wbl);
      if (a.lx) {
        float* r = a.lx + (((long long)b * a.T + t) * K + (i - 1)) * C;
        if (qd == 0) r[y] = O + v;
        if (tid == 0) r[0] = -kInf;
      }
      if (i < K) {
        float* dst = vbuf + (i & 1) * 48;
        if (qd == 0) dst[y] = v;
        if (tid == 0) dst[0] = -kInf;  // nothing enters the start state
        sync();
      }
    }
    // the new vector over a new integer offset: the max over both waves
    float m = fmaxf(acc, acc0);
    m = gmax<6>(m, 6);
    if (lane == 0) xch[(t & 1) * 2 + w] = m;
    sync();
    const float mall = fmaxf(xch[(t & 1) * 2], xch[(t & 1) * 2 + 1]);
    const float sp = __builtin_isfinite(mall) ? floorf(mall) : 0.f;
    ay = acc - sp;
    a0 = acc0 - sp;
    O += sp;
  }
  // (+)_q alpha_T[q] (lattices.py:496): partial (max, sum) by wave, then thread 0
  float m = gmax<6>(ay, 6);
  m = fmaxf(m, a0);
  const float c = t_safe(m);
  float e = qd == 0 ? lt_exp(ay - c) : 0.f;
  e = gsum<6>(e, 6);
  if (w == 0) e += lt_exp(a0 - c);
  if (lane == 0) {
    xch[4 + 2 * w] = m;
    xch[5 + 2 * w] = e;
  }
  sync();
  if (tid == 0) {
    const float m0 = xch[4], e0 = xch[5], m1 = xch[6], e1 = xch[7];
    const float cc = t_safe(fmaxf(m0, m1));
    const float S = e0 * lt_exp(t_safe(m0) - cc) + e1 * lt_exp(t_safe(m1) - cc);
    a.dist[b] = S > 0.f ? O + cc + lt_log_acc(S) : -kInf;
  }
}

// ---- forward: den (NUM = false) or string (NUM = true) shortest distance ----
// STAGE: the frame's weights are copied to LDS once (coalesced) and the
// in-arc gathers read LDS; otherwise they read W from global memory.
template <bool BF16, int SR, bool NUM, bool VIT, bool STAGE>
LT_DEVINL void tab_fwd_body(const TArgs& a, const int b, float* sm) {
  if constexpr (NUM && SR == M_LOG) {
    tab_str_fwd_log<BF16>(a, b, sm);
    return;
  }
  if constexpr (!NUM) {
    if (a.K == 0) {
      tab_fwd_k0_body<BF16, SR, VIT, STAGE>(a, b, sm);
      return;
    }
  }
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int S = NUM ? a.U + 1 : a.C, K = a.K, R = a.R;
  int* gsm = (int*)sm;  // graph copy (STAGE): C+1 + 2*C*V ints
  const int* g_off;
  const int* g_arc;
  const int* g_tab;
  t_graph<STAGE>(a, gsm, &g_off, &g_arc, &g_tab);
  float* va = sm + (STAGE ? (a.C + 1 + 2 * a.C * a.V + 3) / 4 * 4 : 0);
  float* vl = va + S;
  float* vn = vl + S;
  float* acc = vn + S;
  int* ctx = (int*)(acc + S);
  int* yn = ctx + S;
  float* wl = (float*)(yn + S);  // STAGE: [C*(V+1)]; NUM: the compact weights [2S]
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  for (int q = tid; q < S; q += nthr) va[q] = q == 0 ? t_one<SR>() : t_zero<SR>();
  if (NUM && tid == 0) t_walk(a, b, ctx, yn);
  __shared__ int slot_mem[3];
  const MaxSlots slots{slot_mem};
  slots.init();
  __syncthreads();
  using DG = typename std::conditional<STAGE, DenGraphP, DenGraph>::type;
  DG dg{g_off, g_arc, a.V, R};
  NumGraphC ng;
  const long long FR = (long long)a.C * R;
  const int KK = K > 0 ? K : 1;
  constexpr int G = NUM ? 1 : 8;  // lanes per state in the in-arc reductions
  (void)g_tab;
  const long long fbytes = FR * (BF16 ? 2 : 4);
  const unsigned char* wb = a.W + (long long)b * a.T * fbytes;
  FrameStage<BF16> fs;
  if (STAGE) fs.fetch(nf > 0 ? wb : nullptr, FR);
  // the string's two weights per position, gathered one frame ahead
  auto ldc = [&](const unsigned char* w) {
    return [=](int e) { return ldw<BF16>(w, ctx[e >> 1] + ((e & 1) ? yn[e >> 1] : 0)); };
  };
  RegStage<2> cs;
  if (NUM) cs.fetch(nf > 0 ? 2 * S : 0, ldc(wb));
  constexpr bool kOff = SR == M_LOG;  // Log: va relative to the integer offset O
  float O = 0.f;
  // the vector after frame t (its writers put every value into the slot,
  // then a barrier): Log renormalised to a new integer offset
  auto settle = [&](int t, const float* src) {
    if constexpr (kOff) {
      const float sp = slots.shift(t);
      for (int q = tid; q < S; q += nthr) va[q] = src[q] - sp;
      O += sp;
    } else {
      for (int q = tid; q < S; q += nthr) va[q] = src[q];
    }
  };
  for (int t = 0; t < a.T; ++t) {
    if (a.alpha)
      for (int q = tid; q < S; q += nthr) a.alpha[((long long)b * a.T + t) * S + q] = O + va[q];
    if (t >= nf) continue;  // padding frames carry alpha (lattices.py:460-461)
    const unsigned char* wf = wb + t * fbytes;
    if (STAGE) {
      fs.store(wl, wf, FR);
      fs.fetch(t + 1 < nf ? wf + fbytes : nullptr, FR);  // next frame in flight
      __syncthreads();
    }
    if (NUM) {
      cs.store(wl, 2 * S, ldc(wf));
      cs.fetch(t + 1 < nf ? 2 * S : 0, ldc(wf + fbytes));
      __syncthreads();
    }
    auto wr = [&](int i) { return (STAGE || NUM) ? wl[i] : ldw<BF16>(wf, i); };
    int* bpt = VIT ? a.bp + (((long long)b * a.T + t) * KK) * a.C : nullptr;
    if (K == 0) {  // FrameDependent.forward, alignments.py:286-297
      for (int q0 = 0; q0 < S; q0 += nthr / G) {
        const int q = q0 + tid / G;
        const bool valid = q < S;
        int ap = -1;
        const float r = NUM ? t_reduce_g<SR, G>(ng, q, valid, va, wr, &ap)
                            : t_reduce_g<SR, G>(dg, q, valid, va, wr, &ap);
        if (!valid || (tid & (G - 1))) continue;
        const int bi = NUM ? ng.blank(q) : dg.blank(q);
        const float bt = t_times<SR>(va[q], wr(bi));
        float o;
        if constexpr (SR == M_LOG) {
          o = t_lae(bt, r);
        } else if constexpr (SR == M_MAX) {
          const bool keep = ap < 0 || bt >= r;  // Maximum keeps a iff a >= b
          o = keep ? bt : r;
          if (VIT) bpt[q] = keep ? -1 : ap;
        } else {
          o = bt + r;
        }
        vn[q] = o;
        if (kOff) slots.put(t, o);
      }
      if (kOff) slots.reset_next(t);
      __syncthreads();
      settle(t, vn);
      __syncthreads();
      continue;
    }
    // FrameLabelDependent.forward (alignments.py:363-377): terms (L^i a) (x)
    // blank, i = 0..K, summed (MaxTropical: the first max term wins)
    for (int q = tid; q < S; q += nthr) {
      const int bi = NUM ? ng.blank(q) : dg.blank(q);
      acc[q] = t_times<SR>(va[q], wr(bi));
      vl[q] = va[q];
      if (VIT) a.win[((long long)b * a.T + t) * a.C + q] = 0;
    }
    __syncthreads();
    for (int i = 1; i <= K; ++i) {
      for (int q0 = 0; q0 < S; q0 += nthr / G) {
        const int q = q0 + tid / G;
        const bool valid = q < S;
        int ap = -1;
        const float r = NUM ? t_reduce_g<SR, G>(ng, q, valid, vl, wr, &ap)
                            : t_reduce_g<SR, G>(dg, q, valid, vl, wr, &ap);
        if (!valid || (tid & (G - 1))) continue;
        vn[q] = r;
        if (VIT) bpt[(long long)(i - 1) * a.C + q] = ap;
      }
      __syncthreads();
      for (int q = tid; q < S; q += nthr) {
        const int bi = NUM ? ng.blank(q) : dg.blank(q);
        const float term = t_times<SR>(vn[q], wr(bi));
        if constexpr (SR == M_LOG) {
          acc[q] = t_lae(acc[q], term);
          if (i == K) slots.put(t, acc[q]);
        } else if constexpr (SR == M_MAX) {
          if (term > acc[q]) {
            acc[q] = term;
            if (VIT) a.win[((long long)b * a.T + t) * a.C + q] = (unsigned char)i;
          }
        } else {
          acc[q] += term;
        }
        vl[q] = vn[q];
      }
      if (kOff && i == K) slots.reset_next(t);
      __syncthreads();
    }
    settle(t, acc);
    __syncthreads();
  }
  if (tid == 0) {
    if (NUM) {
      const int nl = a.nlab[b];
      const float r = (nl >= 0 && nl <= a.U) ? O + va[nl] : t_zero<SR>();
      a.dist[b] = r;  // lattices.py:375-377
      if (a.loss) a.loss[b] = a.local ? -r : a.den_in[b] - r;  // lattices.py:131-183
    } else {
      // (+)_q alpha_T[q] (lattices.py:496); MaxTropical: first max state
      float r = t_zero<SR>();
      int qs = 0;
      if constexpr (SR == M_LOG) {
        Lse l;
        for (int q = 0; q < S; ++q) l.add(va[q]);
        r = O + l.get();
      } else if constexpr (SR == M_MAX) {
        r = va[0];
        for (int q = 1; q < S; ++q)
          if (va[q] > r) {
            r = va[q];
            qs = q;
          }
      } else {
        for (int q = 0; q < S; ++q) r += va[q];
      }
      a.dist[b] = r;
      if (VIT) a.qstar[b] = qs;
    }
  }
}

template <bool BF16, int SR, bool NUM, bool VIT, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_fwd_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  tab_fwd_body<BF16, SR, NUM, VIT, STAGE>(a, (int)blockIdx.x, sm);
}

// Log denominator (blocks [0, B)) and string (blocks [B, 2B)) forwards side
// by side; the loss is formed afterwards (tab_loss_kernel)
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_fwd2_kernel(const TArgs ad, const TArgs an) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int blk = (int)blockIdx.x;
  if (blk < ad.B) tab_fwd_body<BF16, M_LOG, false, false, STAGE>(ad, blk, sm);
  else tab_fwd_body<BF16, M_LOG, true, false, false>(an, blk - ad.B, sm);
}

__global__ void tab_loss_kernel(float* loss, const float* log_z, const float* num, int B,
                                int local) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) loss[b] = local ? -num[b] : log_z[b] - num[b];  // lattices.py:131-183
}

// ---- Viterbi backtrace (lattices.py:185-247, per utterance: no D6) ----------
// One workgroup per utterance: chunks of backpointer rows (and the in-arc
// table) are staged in LDS by the workgroup, one thread walks them (a frame
// costs LDS latencies, not dependent global loads). `chunk` frames per stage;
// `arcs_lds`: the in-arc table fits beside them.
__global__ __launch_bounds__(256) void tab_backtrace_lds_kernel(const TArgs a, int chunk,
                                                                 int arcs_lds) {
  extern __shared__ __attribute__((aligned(16))) int lsm[];
  const int b = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int C = a.C, V = a.V, K = a.K, KK = K > 0 ? K : 1, A = K > 0 ? K + 1 : 1;
  long long* lab = a.vlabels + (long long)b * a.T * A;
  for (long long i = tid; i < (long long)a.T * A; i += nthr) lab[i] = 0;
  int* arcs = lsm;                              // [C*V] (arcs_lds)
  int* bpl = lsm + (arcs_lds ? C * V : 0);      // [chunk][KK][C]
  unsigned char* wl = (unsigned char*)(bpl + (long long)chunk * KK * C);  // [chunk][C]
  if (arcs_lds)
    for (int i = tid; i < C * V; i += nthr) arcs[i] = a.in_arc[i];
  const int* arc_tab = arcs_lds ? arcs : a.in_arc;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // zeros land before the walk's labels
  __syncthreads();
  int q = a.qstar[b];
  for (int t1 = nf; t1 > 0; t1 -= chunk) {
    const int t0 = t1 - chunk < 0 ? 0 : t1 - chunk;
    const int* src = a.bp + ((long long)b * a.T + t0) * KK * C;
    for (int e = tid; e < (t1 - t0) * KK * C; e += nthr) bpl[e] = src[e];
    if (K > 0) {
      const unsigned char* ws = a.win + ((long long)b * a.T + t0) * C;
      for (int e = tid; e < (t1 - t0) * C; e += nthr) wl[e] = ws[e];
    }
    __syncthreads();
    if (tid == 0) {
      for (int t = t1 - 1; t >= t0; --t) {
        const int i = K > 0 ? wl[(t - t0) * C + q] : 1;
        for (int j = i; j >= 1; --j) {
          const int pos = bpl[((t - t0) * KK + j - 1) * C + q];
          if (pos < 0) break;  // FrameDependent: blank won
          const int id = arc_tab[pos];
          const int p = id / V, y = id - p * V + 1;
          lab[(long long)t * A + j - 1] = a.conv ? y - 1 : y;
          q = p;
        }
      }
    }
    __syncthreads();
  }
}

__global__ void tab_backtrace_kernel(const TArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int K = a.K, KK = K > 0 ? K : 1, A = K > 0 ? K + 1 : 1;
  long long* lab = a.vlabels + (long long)b * a.T * A;
  for (long long i = 0; i < (long long)a.T * A; ++i) lab[i] = 0;
  int q = a.qstar[b];
  for (int t = nf - 1; t >= 0; --t) {
    const int* bpt = a.bp + (((long long)b * a.T + t) * KK) * a.C;
    const int i = K > 0 ? a.win[((long long)b * a.T + t) * a.C + q] : 1;
    for (int j = i; j >= 1; --j) {
      const int pos = bpt[(long long)(j - 1) * a.C + q];
      if (pos < 0) break;  // FrameDependent: blank won
      const int id = a.in_arc[pos];
      const int p = id / a.V, y = id - p * a.V + 1;
      lab[(long long)t * A + j - 1] = a.conv ? y - 1 : y;
      q = p;
    }
  }
}

// ---- backward: denominator arc gradients -> dW (written for every frame) ---
// FrameDependent.backward (alignments.py:300-318) / FrameLabelDependent.backward
// (:379-419) in reverse frame order; the K+1 blank and K lexical marginals of
// a frame add up on the shared weights. Utterances whose loss is not finite,
// and padding frames, get dW = 0. do_den = 0 (local normalisation): zeros.
// SR = M_LOG: d log_z / dW, the arc marginals exp(alpha + w + beta - log_z);
// SR = M_REAL: d dist / dW = alpha * beta' (the Real semiring's (+, x),
// semirings.py:143-173, differentiated as plain arithmetic). a.gin (nullable):
// a per-utterance factor on every element (the incoming gradient).
template <int SR>
LT_DEVINL float t_plus(float a, float b) {
  if constexpr (SR == M_LOG) return t_lae(a, b);
  else return a + b;
}
// (+) over the G lanes of a group of per-lane partial sums
template <int SR, int G>
struct OutSum {
  Lse l;
  float r = 0.f;
  LT_DEVINL void add(float x) {
    if constexpr (SR == M_LOG) l.add(x);
    else r += x;
  }
  LT_DEVINL float merge() {
    if constexpr (SR == M_LOG) {
      lse_merge<G>(l);
      return l.get();
    } else {
      for (int o = 1; o < G; o <<= 1) r += __shfl_xor(r, o, 64);
      return r;
    }
  }
};

// ---- backward, FrameDependent (K = 0) context lattice: ONE barrier a frame --
// As tab_fwd_k0_body: beta kept unshifted in two buffers (its pending integer
// shift applied where it is read), the frame's weights and alpha row staged
// by the previous frame in the other of two LDS buffers. A frame: marginals
// and the new beta (and its max slot), the next frame's staging, barrier.
template <bool BF16, bool STAGE, int SR>
LT_DEVINL void tab_bwd_den_k0_body(const TArgs& a, const int b, float* sm) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int C = a.C, V = a.V, R = a.R;
  int* gsm = (int*)sm;
  const int* g_off;
  const int* g_arc;
  const int* g_tab;
  t_graph<STAGE>(a, gsm, &g_off, &g_arc, &g_tab);
  float* base = sm + (STAGE ? (C + 1 + 2 * C * V + 3) / 4 * 4 : 0);
  float* cur = base;          // [C] beta_{t+1} (unshifted)
  float* nxt = base + C;      // [C]
  float* la0 = base + 2 * C;  // [2][C] alpha rows
  const long long FR = (long long)C * R;
  float* w0 = base + 4 * C;   // STAGE: [2][FR]
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float lz = (a.local || SR == M_REAL) ? 0.f : a.den_in[b];
  const float nm = a.num_in[b];
  const float gb = a.gin ? a.gin[b] : 1.f;
  const bool live = !a.local && __builtin_isfinite(nm) && __builtin_isfinite(lz) && gb != 0.f;
  constexpr bool kOff = SR == M_LOG;
  float Ob = 0.f, sp = 0.f;
  auto mg = [&](float al_or_lo, float x) {
    if constexpr (SR == M_LOG) return lt_exp(al_or_lo + x) * gb;
    else return al_or_lo * x * gb;
  };
  auto af = [&](float alv) {
    if constexpr (SR == M_LOG) return (alv - lz) + Ob;
    else return alv;
  };
  for (int q = tid; q < C; q += nthr) cur[q] = t_one<SR>();  // every state final
  __shared__ int slot_mem[3];
  const MaxSlots slots{slot_mem};
  slots.init();
  using DG = typename std::conditional<STAGE, DenGraphP, DenGraph>::type;
  DG dg{g_off, g_arc, V, R};
  (void)dg;
  constexpr int G = 8;  // lanes per state
  const int esz = BF16 ? 2 : 4;
  auto ldh = [&](int t) {  // alpha row of frame t, gathered one frame ahead
    return [=](int e) { return a.hist[((long long)b * a.T + t) * C + e]; };
  };
  FrameStage<BF16> fs;
  RegStage<1> hs;
  if (live && nf > 0) {
    const unsigned char* wl = a.W + ((long long)b * a.T + nf - 1) * FR * esz;
    if (STAGE) {
      fs.fetch(wl, FR);
      fs.store(w0 + ((nf - 1) & 1) * FR, wl, FR);
      fs.fetch(nf > 1 ? wl - FR * esz : nullptr, FR);
    }
    hs.fetch(C, ldh(nf - 1));
    hs.store(la0 + ((nf - 1) & 1) * C, C, ldh(nf - 1));
    hs.fetch(nf > 1 ? C : 0, ldh(nf - 2));
  }
  __syncthreads();
  const int jg = tid & (G - 1);
  for (int t = a.T - 1; t >= 0; --t) {
    const int it = a.T - 1 - t;  // the order the frames run in (the slots rotate with it)
    const long long fo = ((long long)b * a.T + t) * FR;
    if (t >= nf || !live) {
      for (long long e = tid; e < FR; e += nthr) stw<false>(a.dW, fo + e, 0.f);
      continue;
    }
    if (kOff && t + 1 < nf) {  // frame t + 1's shift, once
      sp = slots.shift(it - 1);
      Ob += sp;
    }
    const unsigned char* wf = a.W + fo * esz;
    const float* wl = w0 + (t & 1) * FR;
    const float* la = la0 + (t & 1) * C;
    auto wr = [&](int i) { return STAGE ? wl[i] : ldw<BF16>(wf, i); };
    // G lanes per source state p: lane jg takes the labels y = jg+1, jg+1+G, ...
    for (int p0 = 0; p0 < C; p0 += nthr / G) {
      const int p = p0 + tid / G;
      const bool valid = p < C;
      const float bb = valid ? t_times<SR>(wr(p * R), cur[p] - sp) : 0.f;
      OutSum<SR, G> s;
      if (valid) {
        const float a0 = af(la[p]);
#pragma unroll 4
        for (int y = 1 + jg; y <= V; y += G) {
          const float bq = cur[g_tab[p * V + y - 1]] - sp;
          const float lb = t_times<SR>(wr(p * R + y), bq);
          stw<false>(a.dW, fo + p * R + y, mg(a0, SR == M_LOG ? lb : bq));
          s.add(lb);
        }
      }
      const float sv = s.merge();
      if (!valid || jg) continue;
      stw<false>(a.dW, fo + p * R, mg(af(la[p]), SR == M_LOG ? bb : cur[p] - sp));
      nxt[p] = t_plus<SR>(bb, sv);
      if (kOff) slots.put(it, nxt[p]);
    }
    if (t >= 1) {  // frame t - 1's weights and alpha row into the other buffers
      if (STAGE) {
        fs.store(w0 + ((t - 1) & 1) * FR, wf - FR * esz, FR);
        fs.fetch(t >= 2 ? wf - 2 * FR * esz : nullptr, FR);
      }
      hs.store(la0 + ((t - 1) & 1) * C, C, ldh(t - 1));
      hs.fetch(t >= 2 ? C : 0, ldh(t - 2));
    }
    if (kOff) slots.reset_next(it);
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
}

// The dense-bigram FrameLabelDependent(K) backward in ONE wave (Log; see
// tab_fwd_dense): lane p owns state p's row of the frame -- its blank and its
// V lexical weights in registers, its dW row accumulated in registers -- and,
// for the lexical alphas L^i alpha_t recomputed from the history row, state p
// as a destination (its column of the frame from an LDS copy). The same
// recursion as tab_bwd_den_body: blank marginals over the K+1 alphas, then
// the lexical levels j = K-1..0 with cur_j = bb (+) L(cur_{j+1}).
constexpr int kTabDenseKMax = 4;
template <bool BF16>
LT_DEVINL void tab_bwd_den_dense(const TArgs& a, const int b, float* sm) {
  const int p = threadIdx.x & 63;  // the lane's state (rows p < C)
  const int C = a.C, V = a.V, R = a.R, K = a.K;
  const bool row = p < C;
  float* wf = sm;                    // [C * R] the frame (columns read by destination lanes)
  float* vb = wf + ((C * R + 3) & ~3);  // [64] a vector broadcast
  float* dwb = vb + 64;              // [C * R] the previous frame's dW, stored a frame late
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float lz = a.local ? 0.f : a.den_in[b];
  const float nm = a.num_in[b];
  const float gb = a.gin ? a.gin[b] : 1.f;
  const bool live = !a.local && __builtin_isfinite(nm) && __builtin_isfinite(lz) && gb != 0.f;
  const long long FR = (long long)C * R;
  const unsigned char* wb0 = a.W + (long long)b * a.T * FR * (BF16 ? 2 : 4);
  float wr[33], nwr[33];  // the lane's row: blank w[p][0], lexical w[p][1..V]
  float hr = 0.f, nhr = 0.f;  // the history alpha_t[p]
  float nla[kTabDenseKMax + 1], fla[kTabDenseKMax + 1];  // lexical alphas from a.lx
  auto fetch = [&](int t, float* w, float& hv) {
    const unsigned char* f = wb0 + (long long)t * FR * (BF16 ? 2 : 4);
#pragma unroll
    for (int k = 0; k < 33; ++k) w[k] = (row && k < R) ? ldw<BF16>(f, (long long)p * R + k) : 0.f;
    hv = row ? a.hist[((long long)b * a.T + t) * C + p] : -kInf;
#pragma unroll
    for (int i = 1; i <= kTabDenseKMax; ++i)
      fla[i] = (a.lx && row && i <= K) ? a.lx[(((long long)b * a.T + t) * K + (i - 1)) * C + p] : -kInf;
  };
  if (live && nf > 0) fetch(nf - 1, nwr, nhr);
  float beta = 0.f;  // beta_{t+1}[p] relative to Ob (every state final: one)
  float Ob = 0.f;
  // frame tp's dW (in dwb) to memory: issued after the next frame's loads,
  // so the wait for those (a frame later) covers these stores as well
  long long pend = -1;
  auto flush = [&]() {
    if (pend < 0) return;
    const int h0 = (int)((4 - (((unsigned long long)(a.dW + pend) >> 2) & 3)) & 3);
    const int n4 = (int)((FR - h0) >> 2);
    if (p < h0) a.dW[pend + p] = dwb[p];
    for (int i = p; i < n4; i += 64) {
      const int e = h0 + 4 * i;
      *(float4*)(a.dW + pend + e) = make_float4(dwb[e], dwb[e + 1], dwb[e + 2], dwb[e + 3]);
    }
    for (int e = h0 + 4 * n4 + p; e < FR; e += 64) a.dW[pend + e] = dwb[e];
    pend = -1;
  };
  for (int t = a.T - 1; t >= 0; --t) {
    const long long fo = ((long long)b * a.T + t) * FR;
    if (t >= nf || !live) {
      for (long long e = p; e < FR; e += 64) a.dW[fo + e] = 0.f;
      continue;
    }
#pragma unroll
    for (int k = 0; k < 33; ++k) wr[k] = nwr[k];
    hr = nhr;
#pragma unroll
    for (int i = 1; i <= kTabDenseKMax; ++i) nla[i] = fla[i];
    if (t >= 1) fetch(t - 1, nwr, nhr);  // the previous frame under this one
    flush();  // frame t + 1's dW (its LDS reads in order before this frame's writes)
    // the frame into LDS (row by row), then the lane's column as a destination
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (row && !a.lx)
#pragma unroll
      for (int k = 0; k < 33; ++k)
        if (k < R) wf[p * R + k] = wr[k];
    if (p < 64) vb[p] = row ? hr : -kInf;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool dest = p >= 1 && p <= V;  // lexical destinations (nothing enters state 0)
    // lexical alphas: la[0] = alpha_t, la[i][p] = (+)_q la[i-1][q] w[q][p]
    // (lt_table_loss_grad: the forward's, from a.lx; else recomputed here)
    float la[kTabDenseKMax + 1];
    la[0] = hr;
#pragma unroll
    for (int i = 1; i <= kTabDenseKMax; ++i) la[i] = i <= K ? nla[i] : -kInf;
    float col[33];
    if (!a.lx) {
      const int pc = p < R ? p : R - 1;  // (reads clamped in bounds, unconditional)
#pragma unroll
      for (int k = 0; k < 33; ++k) col[k] = wf[(k < C ? k : C - 1) * R + pc];
    }
#pragma unroll
    for (int i = 1; i <= kTabDenseKMax; ++i) {
      if (i > K || a.lx) break;
      float x[33];
#pragma unroll
      for (int k = 0; k < 33; ++k) {
        // unconditional (a select would sink the read under a branch that
        // waits its own latency): vb is -inf past C, non-destinations masked below
        x[k] = vb[k] + col[k];
      }
      const float c = t_safe(tree_max<33>(x));
#pragma unroll
      for (int k = 0; k < 33; ++k) x[k] = lt_exp(x[k] - c);
      const float ss = tree_sum<33>(x);
      la[i] = dest && ss > 0.f ? c + lt_log_acc(ss) : -kInf;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      vb[p] = row ? la[i] : -kInf;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // blank marginals over the K + 1 alphas: exp((alpha - log_z) + Ob + w[p][0] + beta)
    const float bb = wr[0] + beta;
    float mb = 0.f;
#pragma unroll
    for (int i = 0; i <= kTabDenseKMax; ++i)
      if (i <= K) mb += lt_exp(((la[i] - lz) + Ob) + bb) * gb;
    float dacc[32];
#pragma unroll
    for (int y = 0; y < 32; ++y) dacc[y] = 0.f;
    float cur = bb;  // level K: blank[K] + beta
    for (int jj = K - 1; jj >= 0; --jj) {
      // cur over the states by LDS, then the lane's row: lb = w[p][y] + cur[y]
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      vb[p] = row ? cur : -kInf;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float lj = -kInf;
#pragma unroll
      for (int i = 0; i < kTabDenseKMax; ++i)
        if (i == jj) lj = la[i];
      const float af = (lj - lz) + Ob;
      float lb[32];
#pragma unroll
      for (int y = 0; y < 32; ++y) {
        // unconditional reads: vb is -inf past C and wr 0 past R (rows past C
        // have alpha -inf, so their sums are zero and never stored)
        lb[y] = wr[y + 1] + vb[y + 1];
      }
      const float c = t_safe(tree_max<32>(lb));
      // one exponential per arc, shared by the sum and the marginal:
      // exp(af + lb) = exp(lb - c) exp(af + c), and af + c is the log of the
      // row's largest arc marginal (a probability: no overflow)
      const float sc = lt_exp(af + c) * gb;
#pragma unroll
      for (int y = 0; y < 32; ++y) {
        lb[y] = lt_exp(lb[y] - c);
        dacc[y] += lb[y] * sc;
      }
      const float ss = tree_sum<32>(lb);
      const float sv = ss > 0.f ? c + lt_log_acc(ss) : -kInf;
      cur = row ? t_lae(bb, sv) : -kInf;
      (void)V;
    }
    // the frame's dW rows into dwb (row p at p R), stored contiguously by
    // every lane at the next frame's top (flush) or after the loop
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (row) {
      dwb[p * R] = mb;
#pragma unroll
      for (int y = 0; y < 32; ++y)
        if (y < V) dwb[p * R + y + 1] = dacc[y];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    pend = fo;
    // beta_t over a new integer offset (floor of its max)
    float m = row ? cur : -kInf;
    m = gmax<6>(m, 6);
    const float sp = __builtin_isfinite(m) ? floorf(m) : 0.f;
    beta = cur - sp;
    Ob += sp;
  }
  flush();
}

// The same backward on TWO waves when the forward left its lexical alphas
// (a.lx, lt_table_loss_grad): wave w takes labels y in [16w + 1, 16w + 16] of
// every row (lane p = state p), so a lane forms half the arcs of a level;
// the two halves' (max, sum) of each row's logsumexp meet through LDS at one
// barrier a level, combined in a fixed order (both waves get the same bits).
template <bool BF16, int NW>
LT_DEVINL void tab_bwd_den_dense2(const TArgs& a, const int b, float* sm) {
  constexpr int L = 32 / NW;  // labels a lane
  const int w = threadIdx.x >> 6, p = threadIdx.x & 63;
  const int C = a.C, R = a.R, K = a.K;
  const bool row = p < C;
  const int y0 = L * w;            // the wave's labels y0 + 1 .. y0 + L
  float* vb = sm;                  // [64] cur over the states (-inf past C)
  float* part = vb + 64;           // [2 levels][NW waves][max, sum][64]
  float* dwb = part + 2 * NW * 128;  // [C R] the frame's dW, stored a frame late
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float lz = a.local ? 0.f : a.den_in[b];
  const float nm = a.num_in[b];
  const float gb = a.gin ? a.gin[b] : 1.f;
  const bool live = !a.local && __builtin_isfinite(nm) && __builtin_isfinite(lz) && gb != 0.f;
  const long long FR = (long long)C * R;
  const unsigned char* wb0 = a.W + (long long)b * a.T * FR * (BF16 ? 2 : 4);
  float wr[L + 1], nwr[L + 1];  // w[p][0], then w[p][y0 + 1 .. y0 + L]
  float la[kTabDenseKMax + 1], nla[kTabDenseKMax + 1];
  auto fetch = [&](int t, float* wv, float* lv) {
    const unsigned char* f = wb0 + (long long)t * FR * (BF16 ? 2 : 4);
    wv[0] = row ? ldw<BF16>(f, (long long)p * R) : 0.f;
#pragma unroll
    for (int k = 1; k <= L; ++k)
      wv[k] = (row && y0 + k < R) ? ldw<BF16>(f, (long long)p * R + y0 + k) : 0.f;
    lv[0] = row ? a.hist[((long long)b * a.T + t) * C + p] : -kInf;
#pragma unroll
    for (int i = 1; i <= kTabDenseKMax; ++i)
      lv[i] = (row && i <= K) ? a.lx[(((long long)b * a.T + t) * K + (i - 1)) * C + p] : -kInf;
  };
  auto sync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  if (live && nf > 0) fetch(nf - 1, nwr, nla);
  float beta = 0.f, Ob = 0.f;  // beta_{t+1}[p] relative to Ob (every state final: one)
  long long pend = -1;
  auto flush = [&]() {  // frame pend's dW from dwb, every lane of the NW waves
    if (pend < 0) return;
    const int t2 = threadIdx.x;
    const int h0 = (int)((4 - (((unsigned long long)(a.dW + pend) >> 2) & 3)) & 3);
    const int n4 = (int)((FR - h0) >> 2);
    if (t2 < h0) a.dW[pend + t2] = dwb[t2];
    for (int i = t2; i < n4; i += 64 * NW) {
      const int e = h0 + 4 * i;
      *(float4*)(a.dW + pend + e) = make_float4(dwb[e], dwb[e + 1], dwb[e + 2], dwb[e + 3]);
    }
    for (int e = h0 + 4 * n4 + t2; e < FR; e += 64 * NW) a.dW[pend + e] = dwb[e];
    pend = -1;
  };
  for (int t = a.T - 1; t >= 0; --t) {
    const long long fo = ((long long)b * a.T + t) * FR;
    if (t >= nf || !live) {
      for (long long e = threadIdx.x; e < FR; e += 64 * NW) a.dW[fo + e] = 0.f;
      continue;
    }
#pragma unroll
    for (int k = 0; k <= L; ++k) wr[k] = nwr[k];
#pragma unroll
    for (int i = 0; i <= kTabDenseKMax; ++i) la[i] = nla[i];
    if (t >= 1) fetch(t - 1, nwr, nla);  // the previous frame under this one
    flush();  // frame t + 1's dW (its dwb writes came before that frame's last barrier)
    const float bb = wr[0] + beta;
    float mb = 0.f;  // the blank marginal over the K + 1 alphas (wave 0 stores it)
#pragma unroll
    for (int i = 0; i <= kTabDenseKMax; ++i)
      if (i <= K) mb += lt_exp(((la[i] - lz) + Ob) + bb) * gb;
    float dacc[L];
#pragma unroll
    for (int k = 0; k < L; ++k) dacc[k] = 0.f;
    float cur = row ? bb : -kInf;  // level K: blank[K] + beta
    for (int jj = K - 1; jj >= 0; --jj) {
      if (w == 0) vb[p] = cur;  // (both waves hold the same cur)
      sync();
      float lj = -kInf;
#pragma unroll
      for (int i = 0; i < kTabDenseKMax; ++i)
        if (i == jj) lj = la[i];
      const float af = (lj - lz) + Ob;
      float lb[L];
#pragma unroll
      for (int k = 0; k < L; ++k) lb[k] = wr[k + 1] + vb[y0 + k + 1];  // (unconditional)
      const float mx = tree_max<L>(lb);
      const float c = t_safe(mx);
      // one exponential per arc for the sum and the marginal (af + c: the log
      // of the half row's largest arc marginal, a probability)
      const float sc = lt_exp(af + c) * gb;
#pragma unroll
      for (int k = 0; k < L; ++k) {
        lb[k] = lt_exp(lb[k] - c);
        dacc[k] += lb[k] * sc;
      }
      const float ss = tree_sum<L>(lb);
      float* pl = part + (jj & 1) * NW * 128;
      pl[w * 128 + p] = mx;
      pl[w * 128 + 64 + p] = ss;
      sync();
      // the row's logsumexp from the waves' parts, in wave order on every wave
      float mm = -kInf;
#pragma unroll
      for (int v = 0; v < NW; ++v) mm = fmaxf(mm, pl[v * 128 + p]);
      const float cc = t_safe(mm);
      float S = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) S += pl[v * 128 + 64 + p] * lt_exp(t_safe(pl[v * 128 + p]) - cc);
      const float sv = S > 0.f ? cc + lt_log_acc(S) : -kInf;
      cur = row ? t_lae(bb, sv) : -kInf;
    }
    // the frame's dW into dwb (each wave its labels, wave 0 the blank)
    if (row) {
      if (w == 0) dwb[p * R] = mb;
#pragma unroll
      for (int k = 0; k < L; ++k)
        if (y0 + k + 1 < R) dwb[p * R + y0 + k + 1] = dacc[k];
    }
    sync();
    pend = fo;
    // beta_t over a new integer offset (floor of its max); the same on both waves
    float m = row ? cur : -kInf;
    m = gmax<6>(m, 6);
    const float sp = __builtin_isfinite(m) ? floorf(m) : 0.f;
    beta = cur - sp;
    Ob += sp;
  }
  flush();
}

template <bool BF16, bool STAGE, int SR>
LT_DEVINL void tab_bwd_den_body(const TArgs& a, const int b, float* sm) {
  if (a.K == 0) {
    tab_bwd_den_k0_body<BF16, STAGE, SR>(a, b, sm);
    return;
  }

  const int tid = threadIdx.x, nthr = blockDim.x;
  const int C = a.C, V = a.V, R = a.R, K = a.K;
  int* gsm = (int*)sm;
  const int* g_off;
  const int* g_arc;
  const int* g_tab;
  t_graph<STAGE>(a, gsm, &g_off, &g_arc, &g_tab);
  float* beta = sm + (STAGE ? (C + 1 + 2 * C * V + 3) / 4 * 4 : 0);
  float* nbA = beta + C;
  float* nbB = nbA + C;
  float* la = nbB + C;  // [K+1][C]
  float* wl = la + (long long)(K + 1) * C;  // STAGE: [C*(V+1)]
  float* dacc = wl + (long long)C * R;      // a.acc: the frame's lexical dW sums [C*(V+1)]
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float lz = (a.local || SR == M_REAL) ? 0.f : a.den_in[b];
  const float nm = a.num_in[b];
  const float gb = a.gin ? a.gin[b] : 1.f;
  const bool live = !a.local && __builtin_isfinite(nm) && __builtin_isfinite(lz) && gb != 0.f;
  const long long FR = (long long)C * R;
  // Log: beta relative to the integer offset Ob (MaxSlots); an arc's
  // marginal exp(alpha + w + beta' - log_z) takes the large terms first,
  // ((alpha - log_z) + Ob) + (w + beta'_rel)
  float Ob = 0.f;
  // the gradient of one arc: Log from (alpha - log_z + Ob) and w + beta'_rel;
  // Real alpha * beta' (the weight not included)
  auto mg = [&](float al_or_lo, float x) {
    if constexpr (SR == M_LOG) return lt_exp(al_or_lo + x) * gb;
    else return al_or_lo * x * gb;
  };
  // the alpha-side factor of mg: Log (alpha - log_z) + Ob, Real alpha
  auto af = [&](float alv) {
    if constexpr (SR == M_LOG) return (alv - lz) + Ob;
    else return alv;
  };
  for (int q = tid; q < C; q += nthr) beta[q] = t_one<SR>();  // every state final
  __shared__ int slot_mem[3];
  const MaxSlots slots{slot_mem};
  slots.init();
  __syncthreads();
  using DG = typename std::conditional<STAGE, DenGraphP, DenGraph>::type;
  DG dg{g_off, g_arc, V, R};
  constexpr int G = 8;  // lanes per state
  FrameStage<BF16> fs;
  if (STAGE && live && nf > 0)
    fs.fetch(a.W + ((long long)b * a.T + nf - 1) * FR * (BF16 ? 2 : 4), FR);
  auto ldh = [&](int t) {  // alpha row of frame t, gathered one frame ahead
    return [=](int e) { return a.hist[((long long)b * a.T + t) * C + e]; };
  };
  RegStage<1> hs;
  if (live && nf > 0) hs.fetch(C, ldh(nf - 1));
  for (int t = a.T - 1; t >= 0; --t) {
    const int it = a.T - 1 - t;  // the frames' order here (the offset slots rotate with it)
    const long long fo = ((long long)b * a.T + t) * FR;
    if (t >= nf || !live) {
      for (long long e = tid; e < FR; e += nthr) stw<false>(a.dW, fo + e, 0.f);
      continue;
    }
    const unsigned char* wf = a.W + fo * (BF16 ? 2 : 4);
    if (STAGE) {
      fs.store(wl, wf, FR);
      fs.fetch(t >= 1 ? wf - FR * (BF16 ? 2 : 4) : nullptr, FR);  // frame t-1 in flight
    }
    auto wr = [&](int i) { return STAGE ? wl[i] : ldw<BF16>(wf, i); };
    hs.store(la, C, ldh(t));
    hs.fetch(t >= 1 ? C : 0, ldh(t - 1));
    __syncthreads();
    for (int i = 1; i <= K; ++i) {  // lexical_alphas
      for (int q0 = 0; q0 < C; q0 += nthr / G) {
        const int q = q0 + tid / G;
        const bool valid = q < C;
        const float r = t_reduce_g<SR, G>(dg, q, valid, la + (long long)(i - 1) * C, wr, nullptr);
        if (valid && !(tid & (G - 1))) la[(long long)i * C + q] = r;
      }
      __syncthreads();
    }
    // G lanes per source state p: lane jg takes the labels y = jg+1, jg+1+G, ...
    const int jg = tid & (G - 1);
    for (int p0 = 0; p0 < C; p0 += nthr / G) {
      const int p = p0 + tid / G;
      const bool valid = p < C;
      const float bb = valid ? t_times<SR>(wr(p * R), beta[p]) : 0.f;
      OutSum<SR, G> s;
      if (K == 0 && valid) {
        const float a0 = af(la[p]);
#pragma unroll 4
        for (int y = 1 + jg; y <= V; y += G) {
          const float bq = beta[g_tab[p * V + y - 1]];
          const float lb = t_times<SR>(wr(p * R + y), bq);
          stw<false>(a.dW, fo + p * R + y, mg(a0, SR == M_LOG ? lb : bq));
          s.add(lb);
        }
      }
      const float sv = s.merge();
      if (!valid || jg) continue;
      if (K == 0) {
        stw<false>(a.dW, fo + p * R, mg(af(la[p]), SR == M_LOG ? bb : beta[p]));
        nbA[p] = t_plus<SR>(bb, sv);
        if (SR == M_LOG) slots.put(it, nbA[p]);
      } else {
        float mb = 0.f;
        for (int i = 0; i <= K; ++i)
          mb += mg(af(la[(long long)i * C + p]), SR == M_LOG ? bb : beta[p]);
        stw<false>(a.dW, fo + p * R, mb);
        nbA[p] = bb;  // blank[K] + beta
      }
    }
    if (SR == M_LOG && K == 0) slots.reset_next(it);
    __syncthreads();
    float* cur = nbA;
    float* nxt = nbB;
    for (int j = K - 1; j >= 0; --j) {
      for (int p0 = 0; p0 < C; p0 += nthr / G) {
        const int p = p0 + tid / G;
        const bool valid = p < C;
        OutSum<SR, G> s;
        if (valid) {
          const float lj = af(la[(long long)j * C + p]);
#pragma unroll 4
          for (int y = 1 + jg; y <= V; y += G) {
            const float cq = cur[g_tab[p * V + y - 1]];
            const float lb = t_times<SR>(wr(p * R + y), cq);
            const float m = mg(lj, SR == M_LOG ? lb : cq);
            const long long e = fo + p * R + y;
            // the same lane owns (p, y) for every j: accumulate in place
            // (in LDS when it fits; dW is written once, at j = 0)
            if (STAGE && a.acc) {
              const float v = (j == K - 1 ? 0.f : dacc[p * R + y]) + m;
              if (j == 0) stw<false>(a.dW, e, v);
              else dacc[p * R + y] = v;
            } else {
              stw<false>(a.dW, e, j == K - 1 ? m : ldw<false>((const unsigned char*)a.dW, e) + m);
            }
            s.add(lb);
          }
        }
        const float sv = s.merge();
        if (valid && !jg) {
          nxt[p] = t_plus<SR>(t_times<SR>(wr(p * R), beta[p]), sv);
          if (SR == M_LOG && j == 0) slots.put(it, nxt[p]);
        }
      }
      if (SR == M_LOG && j == 0) slots.reset_next(it);
      __syncthreads();
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    if constexpr (SR == M_LOG) {
      const float sp = slots.shift(it);
      for (int p = tid; p < C; p += nthr) beta[p] = cur[p] - sp;
      Ob += sp;
    } else {
      for (int p = tid; p < C; p += nthr) beta[p] = cur[p];
    }
    __syncthreads();
  }
}

template <bool BF16, bool STAGE, int SR>
__global__ __launch_bounds__(kTabMaxThreads) void tab_bwd_den_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  tab_bwd_den_body<BF16, STAGE, SR>(a, (int)blockIdx.x, sm);
}

// MaxTropical: the gradient of the shortest distance is the best path's
// indicator (semirings.py:354-401: the first maximum wins), times the
// incoming gradient. One thread per utterance walks the Viterbi backpointers
// (tab_fwd_kernel's VIT mode) as tab_backtrace_kernel does and adds g to
// every arc the path takes -- the blank of the frame's end state and its
// lexical arcs (alignment-state-invariant weights: an element taken twice in
// one frame gets 2g). dW (fp32) is zeroed beforehand.
__global__ void tab_onehot_kernel(const TArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  // An utterance of distance -inf (every path masked) still gets the first
  // maximum's path, as the reference's argmax backward gives it
  // (semirings.py:354-401: ties go to the blank / the first source), so
  // this walks the all-tie backpointers like any other.
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int K = a.K, KK = K > 0 ? K : 1;
  const long long FR = (long long)a.C * a.R;
  const float gb = a.gin ? a.gin[b] : 1.f;
  int q = a.qstar[b];
  for (int t = nf - 1; t >= 0; --t) {
    float* dw = a.dW + ((long long)b * a.T + t) * FR;
    const int* bpt = a.bp + (((long long)b * a.T + t) * KK) * a.C;
    if (K > 0) dw[(long long)q * a.R] += gb;  // the end state's blank
    const int i = K > 0 ? a.win[((long long)b * a.T + t) * a.C + q] : 1;
    for (int j = i; j >= 1; --j) {
      const int pos = bpt[(long long)(j - 1) * a.C + q];
      if (pos < 0) {  // FrameDependent: the blank self loop won
        dw[(long long)q * a.R] += gb;
        break;
      }
      const int id = a.in_arc[pos];
      const int p = id / a.V, y = id - p * a.V + 1;
      dw[(long long)p * a.R + y] += gb;
      q = p;
    }
  }
}

// ---- backward (Log): numerator marginals subtracted from dW ----------------
// The same recursion on the string acceptor; string arcs that share a lattice
// arc are summed by their chain head in ascending order (one writer per
// element and frame: deterministic).
// ---- string backward, FrameDependent (K = 0): ONE barrier a frame ----------
// Frame t's pass (marginals of its string arcs into mb / ml of parity t, the
// new beta into the other (i, f) buffer) runs beside frame t + 1's chain-head
// sums (mb / ml of the other parity) and the staging of frame t - 1's alpha
// row and weights; dh is read and rewritten by the same thread (its heads'
// index set), so it needs no second buffer.
template <bool BF16>
LT_DEVINL void tab_bwd_num_k0_body(const TArgs& a, const int b, float* sm) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int U = a.U, S = U + 1, NK = 2 * S;
  float* b0i = sm;  // [2] x (i [S], f [S]): beta_{t+1} and the new beta
  float* mb0 = b0i + 4 * S;  // [2] x (mb [S], ml [S])
  float* la0 = mb0 + 4 * S;  // [2][S] alpha history rows
  int* ctx = (int*)(la0 + 2 * S);
  int* yn = ctx + S;
  int* link = yn + S;               // [NK]
  float* wc0 = (float*)(link + NK);  // [2][2S]
  float* dh = wc0 + 4 * S;           // [NK]
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float nm = a.num_in[b];
  const float lz = a.local ? 0.f : a.den_in[b];
  const bool live = __builtin_isfinite(nm) && (a.local || __builtin_isfinite(lz));
  if (!live) {  // the denominator kernel wrote zeros
    if (a.ntab)
      for (int k = tid; k < NK; k += nthr) a.ntab[(long long)b * NK + k] = -1;
    return;
  }
  const int nl = a.nlab[b];
  if (tid == 0) t_walk(a, b, ctx, yn);
  for (int u = tid; u < S; u += nthr) {
    b0i[u] = u == nl ? 0.f : -kInf;
    b0i[S + u] = 0.f;
  }
  __syncthreads();
  auto elem = [&](int k) {  // W element of string entry k = 2u + kind, or -1
    const int u = k >> 1;
    return (k & 1) == 0 ? ctx[u] : (u < U ? ctx[u] + yn[u] : -1);
  };
  for (int k = tid; k < NK; k += nthr) {
    const int o = elem(k);
    int head = o >= 0 ? 1 : 0, nxt = -1;
    if (o >= 0)
      for (int k2 = 0; k2 < NK; ++k2) {
        if (elem(k2) != o) continue;
        if (k2 < k) head = 0;
        else if (k2 > k && nxt < 0) nxt = k2;
      }
    link[k] = (head << 30) | (nxt + 1);
    if (a.ntab) a.ntab[(long long)b * NK + k] = head ? o : -1;
  }
  __syncthreads();
  const long long FR = (long long)a.C * a.R;
  auto ldh = [&](int t) {
    return [=](int e) { return a.hist[((long long)b * a.T + t) * S + e]; };
  };
  auto ldc = [&](int t) {
    const unsigned char* w = a.W + ((long long)b * a.T + t) * FR * (BF16 ? 2 : 4);
    return [=](int e) { return ldw<BF16>(w, ctx[e >> 1] + ((e & 1) ? yn[e >> 1] : 0)); };
  };
  auto ldd = [&](int t) {
    const long long fo = ((long long)b * a.T + t) * FR;
    return [=](int k) {
      return (!a.nsub && (link[k] >> 30)) ? ldw<false>((const unsigned char*)a.dW, fo + elem(k))
                                          : 0.f;
    };
  };
  auto marg = [&](float alv, float i, float f) { return lt_exp(((alv - nm) + i) + f); };
  // the chain heads of frame t (its mb / ml parity, dh): nsub or dW
  auto heads = [&](int t) {
    const float* mb = mb0 + (t & 1) * 2 * S;
    const float* ml = mb + S;
    const long long fo = ((long long)b * a.T + t) * FR;
    for (int k = tid; k < NK; k += nthr) {
      const int lk = link[k];
      if (!(lk >> 30)) continue;
      float s = 0.f;
      for (int kk = k; kk >= 0; kk = (link[kk] & 0x3fffffff) - 1)
        s += (kk & 1) ? ml[kk >> 1] : mb[kk >> 1];
      if (a.nsub) a.nsub[((long long)b * a.T + t) * NK + k] = s;
      else stw<false>(a.dW, fo + elem(k), dh[k] - s);
    }
  };
  RegStage<1> hs;
  RegStage<2> cs, ds;
  if (nf > 0) {
    hs.fetch(S, ldh(nf - 1));
    cs.fetch(2 * S, ldc(nf - 1));
    hs.store(la0 + ((nf - 1) & 1) * S, S, ldh(nf - 1));
    cs.store(wc0 + ((nf - 1) & 1) * 2 * S, 2 * S, ldc(nf - 1));
    hs.fetch(nf > 1 ? S : 0, ldh(nf - 2));
    cs.fetch(nf > 1 ? 2 * S : 0, ldc(nf - 2));
    ds.fetch(NK, ldd(nf - 1));
  }
  __syncthreads();
  float *bi = b0i, *bf = b0i + S, *ci = b0i + 2 * S, *cf = b0i + 3 * S;
  for (int t = nf - 1; t >= 0; --t) {
    const float* la = la0 + (t & 1) * S;
    const float* wc = wc0 + (t & 1) * 2 * S;
    float* mb = mb0 + (t & 1) * 2 * S;
    float* ml = mb + S;
    for (int u = tid; u < S; u += nthr) {
      const float bbf = wc[2 * u] + bf[u];  // blank + beta: (bi[u], bbf)
      const bool lex = u < U;
      const float li = lex ? bi[u + 1] : -kInf, lf = lex ? wc[2 * u + 1] + bf[u + 1] : 0.f;
      mb[u] = marg(la[u], bi[u], bbf);
      ml[u] = lex ? marg(la[u], li, lf) : 0.f;
      lae_split(bi[u], bbf, li, lf, ci[u], cf[u]);
    }
    if (t + 1 < nf) heads(t + 1);  // (its dh in place: read before this thread's restage)
    ds.store(dh, NK, ldd(t));
    ds.fetch(t >= 1 ? NK : 0, ldd(t - 1));
    if (t >= 1) {
      hs.store(la0 + ((t - 1) & 1) * S, S, ldh(t - 1));
      cs.store(wc0 + ((t - 1) & 1) * 2 * S, 2 * S, ldc(t - 1));
      hs.fetch(t >= 2 ? S : 0, ldh(t - 2));
      cs.fetch(t >= 2 ? 2 * S : 0, ldc(t - 2));
    }
    __syncthreads();
    float* ti = bi; bi = ci; ci = ti;
    float* tf = bf; bf = cf; cf = tf;
  }
  if (nf > 0) {
    heads(0);
    __syncthreads();
  }
}

template <bool BF16>
LT_DEVINL void tab_bwd_num_body(const TArgs& a, const int b, float* sm) {
  if (a.K == 0) {
    tab_bwd_num_k0_body<BF16>(a, b, sm);
    return;
  }
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int U = a.U, S = U + 1, K = a.K, NK = 2 * S;
  // beta and the backward chain in the (i, f) representation of
  // tab_str_fwd_log: integer parts and fractions
  float* bi = sm;
  float* bf = bi + S;
  float* ai = bf + S;  // nbA
  float* af = ai + S;
  float* ci = af + S;  // nbB
  float* cf = ci + S;
  float* mb = cf + S;
  float* ml = mb + S;
  float* la = ml + S;  // [K+1][S]: alpha history row and its lexical chain (absolute)
  int* ctx = (int*)(la + (long long)(K + 1) * S);
  int* yn = ctx + S;
  int* link = yn + S;  // [NK]: head << 30 | (next entry + 1)
  float* wc = (float*)(link + NK);  // [2S] the frame's string weights (NumGraphC)
  float* dh = wc + 2 * S;           // [NK] dW at the chain heads' elements
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const float nm = a.num_in[b];
  const float lz = a.local ? 0.f : a.den_in[b];
  const bool live = __builtin_isfinite(nm) && (a.local || __builtin_isfinite(lz));
  if (!live) {  // the denominator kernel wrote zeros
    if (a.ntab)
      for (int k = tid; k < NK; k += nthr) a.ntab[(long long)b * NK + k] = -1;
    return;
  }
  const int nl = a.nlab[b];
  if (tid == 0) t_walk(a, b, ctx, yn);
  for (int u = tid; u < S; u += nthr) {
    bi[u] = u == nl ? 0.f : -kInf;
    bf[u] = 0.f;
  }
  __syncthreads();
  auto elem = [&](int k) {  // W element of string entry k = 2u + kind, or -1
    const int u = k >> 1;
    return (k & 1) == 0 ? ctx[u] : (u < U ? ctx[u] + yn[u] : -1);
  };
  for (int k = tid; k < NK; k += nthr) {
    const int o = elem(k);
    int head = o >= 0 ? 1 : 0, nxt = -1;
    if (o >= 0)
      for (int k2 = 0; k2 < NK; ++k2) {
        if (elem(k2) != o) continue;
        if (k2 < k) head = 0;
        else if (k2 > k && nxt < 0) nxt = k2;
      }
    link[k] = (head << 30) | (nxt + 1);
    if (a.ntab) a.ntab[(long long)b * NK + k] = head ? o : -1;
  }
  __syncthreads();
  NumGraphC ng;
  const long long FR = (long long)a.C * a.R;
  // every global read of a frame (alpha_num row, the string's weights, dW at
  // the heads) is gathered one frame ahead into registers
  auto ldh = [&](int t) {
    return [=](int e) { return a.hist[((long long)b * a.T + t) * S + e]; };
  };
  auto ldc = [&](int t) {
    const unsigned char* w = a.W + ((long long)b * a.T + t) * FR * (BF16 ? 2 : 4);
    return [=](int e) { return ldw<BF16>(w, ctx[e >> 1] + ((e & 1) ? yn[e >> 1] : 0)); };
  };
  auto ldd = [&](int t) {
    const long long fo = ((long long)b * a.T + t) * FR;
    return [=](int k) {
      return (!a.nsub && (link[k] >> 30)) ? ldw<false>((const unsigned char*)a.dW, fo + elem(k))
                                          : 0.f;
    };
  };
  // the forward's lexical alphas L^i alpha_t (lt_table_loss_grad), [K][S] a frame
  auto ldx = [&](int t) {
    return [=](int e) { return a.lx[((long long)b * a.T + t) * K * S + e]; };
  };
  RegStage<1> hs;
  RegStage<2> cs, ds;
  RegStage<2> xs;
  if (nf > 0) {
    hs.fetch(S, ldh(nf - 1));
    cs.fetch(2 * S, ldc(nf - 1));
    ds.fetch(NK, ldd(nf - 1));
    if (a.lx) xs.fetch(K * S, ldx(nf - 1));
  }
  // a string arc's marginal exp(alpha + w + beta' - num), beta' = (i, f):
  // the large terms first, ((alpha - num) + i) + (f + w)
  auto marg = [&](float alv, float i, float f) { return lt_exp(((alv - nm) + i) + f); };
  for (int t = nf - 1; t >= 0; --t) {
    const long long fo = ((long long)b * a.T + t) * FR;
    hs.store(la, S, ldh(t));
    cs.store(wc, 2 * S, ldc(t));
    ds.store(dh, NK, ldd(t));
    if (a.lx) xs.store(la + S, K * S, ldx(t));
    hs.fetch(t >= 1 ? S : 0, ldh(t - 1));
    cs.fetch(t >= 1 ? 2 * S : 0, ldc(t - 1));
    ds.fetch(t >= 1 ? NK : 0, ldd(t - 1));
    if (a.lx) xs.fetch(t >= 1 ? K * S : 0, ldx(t - 1));
    auto wr = [&](int i) { return wc[i]; };
    __syncthreads();
    for (int i = 1; i <= K && !a.lx; ++i) {  // (recomputed without the forward's)
      for (int u = tid; u < S; u += nthr)
        la[(long long)i * S + u] = t_reduce<M_LOG>(ng, u, la + (long long)(i - 1) * S, wr, nullptr);
      __syncthreads();
    }
    for (int u = tid; u < S; u += nthr) {
      const float bbf = wc[2 * u] + bf[u];  // blank + beta: (bi[u], bbf)
      if (K == 0) {
        const bool lex = u < U;
        const float li = lex ? bi[u + 1] : -kInf, lf = lex ? wc[2 * u + 1] + bf[u + 1] : 0.f;
        mb[u] = marg(la[u], bi[u], bbf);
        ml[u] = lex ? marg(la[u], li, lf) : 0.f;
        lae_split(bi[u], bbf, li, lf, ai[u], af[u]);
      } else {
        float sacc = 0.f;
        for (int i = 0; i <= K; ++i) sacc += marg(la[(long long)i * S + u], bi[u], bbf);
        mb[u] = sacc;
        ml[u] = 0.f;
        ai[u] = bi[u];  // next_beta = blank[K] + beta
        af[u] = bbf;
      }
    }
    __syncthreads();
    float *pi = ai, *pf = af, *qi = ci, *qf = cf;
    for (int j = K - 1; j >= 0; --j) {
      for (int u = tid; u < S; u += nthr) {
        const bool lex = u < U;
        const float li = lex ? pi[u + 1] : -kInf, lf = lex ? wc[2 * u + 1] + pf[u + 1] : 0.f;
        if (lex) ml[u] += marg(la[(long long)j * S + u], li, lf);
        lae_split(bi[u], wc[2 * u] + bf[u], li, lf, qi[u], qf[u]);
      }
      __syncthreads();
      float* t1 = pi;
      pi = qi;
      qi = t1;
      t1 = pf;
      pf = qf;
      qf = t1;
    }
    for (int k = tid; k < NK; k += nthr) {
      const int lk = link[k];
      if (!(lk >> 30)) continue;
      float s = 0.f;
      for (int kk = k; kk >= 0; kk = (link[kk] & 0x3fffffff) - 1)
        s += (kk & 1) ? ml[kk >> 1] : mb[kk >> 1];
      if (a.nsub) a.nsub[((long long)b * a.T + t) * NK + k] = s;
      else stw<false>(a.dW, fo + elem(k), dh[k] - s);
    }
    // beta_t: the last level's buffers become beta (their roles swap, no copy)
    if (pi == ai) {
      ai = bi; bi = pi;
      af = bf; bf = pf;
    } else {
      ci = bi; bi = pi;
      cf = bf; bf = pf;
    }
    __syncthreads();
  }
}

template <bool BF16>
__global__ __launch_bounds__(kTabMaxThreads) void tab_bwd_num_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  tab_bwd_num_body<BF16>(a, (int)blockIdx.x, sm);
}

// denominator (blocks [0, B)) and numerator (blocks [B, 2B)) backwards side
// by side; the numerator's sums land in nsub
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_bwd2_kernel(const TArgs ad, const TArgs an) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int blk = (int)blockIdx.x;
  if (blk < ad.B) tab_bwd_den_body<BF16, STAGE, M_LOG>(ad, blk, sm);
  else tab_bwd_num_body<BF16>(an, blk - ad.B, sm);
}

// The Log denominator of FrameLabelDependent(K >= 1) lattices: the dense-
// bigram kernels (tab_fwd_dense*, tab_bwd_den_dense*) when the next-state
// table is FullNGram's bigram, else the generic bodies. Kernels of their own,
// chosen by the host for K >= 1, so the K = 0 kernels keep their code.
template <bool BF16, bool STAGE>
LT_DEVINL void tab_fwd_den_fld(const TArgs& a, const int b, float* sm) {
  if (LT_TAB_DENSE && tab_dense_bigram(a)) {  // (a uniform decision: every thread took it)
    if (a.V == 32 && blockDim.x >= 128) {
      if (threadIdx.x < 128) tab_fwd_dense2<BF16>(a, b, sm);
    } else if (threadIdx.x < 64) {
      tab_fwd_dense<BF16>(a, b, sm);
    }
    return;
  }
  tab_fwd_body<BF16, M_LOG, false, false, STAGE>(a, b, sm);
}
template <bool BF16, bool STAGE>
LT_DEVINL void tab_bwd_den_fld(const TArgs& a, const int b, float* sm) {
  // (STAGE and acc: the launch's LDS holds two frames)
  if (LT_TAB_DENSE && STAGE && a.acc && a.K <= kTabDenseKMax && tab_dense_bigram(a)) {
    if (a.lx && a.V == 32 && blockDim.x >= 64 * LT_TAB_BWD_WAVES) {
      if (threadIdx.x < 64 * LT_TAB_BWD_WAVES) tab_bwd_den_dense2<BF16, LT_TAB_BWD_WAVES>(a, b, sm);
    } else if (threadIdx.x < 64) {
      tab_bwd_den_dense<BF16>(a, b, sm);
    }
    return;
  }
  tab_bwd_den_body<BF16, STAGE, M_LOG>(a, b, sm);
}
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_fwd_fld_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  tab_fwd_den_fld<BF16, STAGE>(a, (int)blockIdx.x, sm);
}
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_fwd2_fld_kernel(const TArgs ad, const TArgs an) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int blk = (int)blockIdx.x;
  if (blk < ad.B) tab_fwd_den_fld<BF16, STAGE>(ad, blk, sm);
  else tab_fwd_body<BF16, M_LOG, true, false, false>(an, blk - ad.B, sm);
}
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_bwd_den_fld_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  tab_bwd_den_fld<BF16, STAGE>(a, (int)blockIdx.x, sm);
}
template <bool BF16, bool STAGE>
__global__ __launch_bounds__(kTabMaxThreads) void tab_bwd2_fld_kernel(const TArgs ad, const TArgs an) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int blk = (int)blockIdx.x;
  if (blk < ad.B) tab_bwd_den_fld<BF16, STAGE>(ad, blk, sm);
  else tab_bwd_num_body<BF16>(an, blk - ad.B, sm);
}

// dW -= the numerator's chain-head sums (one writer per element and frame)
__global__ __launch_bounds__(256) void tab_apply_kernel(const TArgs a) {
  const int NK = 2 * (a.U + 1);
  const long long FR = (long long)a.C * a.R;
  const long long n = (long long)a.B * a.T * NK;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % NK);
    const long long bt = i / NK;
    const int b = (int)(bt / a.T), t = (int)(bt - (long long)b * a.T);
    const int el = a.ntab[(long long)b * NK + k];
    int nf = a.nfr[b];
    nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
    if (el < 0 || t >= nf) continue;
    a.dW[bt * FR + el] -= a.nsub[i];
  }
}

// fp32 gradient -> bf16 dW (one rounding of den - num, as the tuned kernels)
__global__ __launch_bounds__(256) void tab_to_bf16_kernel(const float* src, unsigned short* dst,
                                                          long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dst[i] = f2bf(src[i]);
}

// ---- gradients of the string distance, MaxTropical and Real ----------------
// RecognitionLattice._string_forward (lattices.py:250-377) differentiated as
// the reference's autograd does it, for FrameDependent (alignments.py:320-329)
// and FrameLabelDependent(K) (:420-432) string forwards over any next-state
// table (walk_states, contexts.py:109-146):
//   forward   term_i[u] = L_i[u] (x) bl[u], L_0 = alpha, L_i[u] = L_{i-1}[u-1]
//             (x) lx[u-1] (shift_down's zero below i); alpha'[u] = (+)_i term_i
//             (FrameDependent: alpha[u] bl[u] (+) alpha[u-1] lx[u-1])
//   MaxTropical: Maximum keeps the blank term on ties (semirings.py:363) and
//             Max the first expansion count i (:382); the gradient is grad_b
//             on the arcs of the winning path, walked back from the final
//             position -- num_labels while alpha_T there is above -inf, else
//             position 0 of where(is_final, ...), which passes a gradient
//             only when num_labels == 0 (lattices.py:375-377)
//   Real:     reverse accumulation of the same recursion (semirings.py:143-173)
// Positions whose arcs hit one lattice element (epsilon labels, a context
// revisited) are summed by their chain head in ascending position order, one
// writer per element and frame (deterministic). One workgroup per utterance.
// Workspace: MaxTropical the winning term per (t, u) (bytes), Real the alpha
// history (fp32). dW is zeroed by the caller's memset.
constexpr int kStrChunk = 32768;  // bytes of decisions staged per chunk (MaxTropical walk)
template <bool BF16, int SR>
__global__ __launch_bounds__(kTabMaxThreads) void tab_str_grad_kernel(const TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
  const int U = a.U, S = U + 1, K = a.K, T = a.T;
  const float zero = t_zero<SR>();
  int* ctx = (int*)sm;    // [S] context state of position u, times R
  int* yn = ctx + S;      // [S] label class of the arc leaving u
  int* nxb = yn + S;      // [S] next position with the same blank element (-1)
  int* nxl = nxb + S;     // [S] next position with the same lexical element (-1)
  int* hd = nxl + S;      // [S] bit 0 / 1: head of its blank / lexical chain
  float* xa = (float*)(hd + S);  // [S] alpha_t (forward) / alpha_t of the frame (backward)
  float* xb = xa + S;     // [S] alpha_{t+1} / beta_{t+1}
  float* xc = xb + S;     // [S] beta_t
  float* wb = xc + S;     // [S] the frame's blank weights
  float* wl = wb + S;     // [S] the frame's lexical weights (u < U)
  float* gb = wl + S;     // [S] blank gradients of the frame
  float* gl = gb + S;     // [S] lexical gradients
  float* L = gl + S;      // [K+1][S] Real FrameLabelDependent: L_i
  float* d0 = L + (K + 1) * S;  // [S] dL_{i+1}
  float* d1 = d0 + S;           // [S] dL_i
  int* marks = (int*)(d1 + S) + 4;  // [K+1][2] MaxTropical: a frame's marked elements, counts
  unsigned char* wc = (unsigned char*)(marks + ((2 * (K + 1) + 3) & ~3));  // decision chunk
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > T ? T : nf);
  const long long FR = (long long)a.C * a.R;
  const unsigned char* wbase = a.W + (long long)b * T * FR * (BF16 ? 2 : 4);
  unsigned char* dwbase = (unsigned char*)a.dW + (long long)b * T * FR * (BF16 ? 2 : 4);
  if (tid == 0) t_walk(a, b, ctx, yn);
  __syncthreads();
  for (int u = tid; u < S; u += nthr) {
    const int kb = ctx[u], kl = u < U ? ctx[u] + yn[u] : -1;
    int nB = -1, nL = -1, h = u < U ? 3 : 1;
    for (int v = u + 1; v < S && (nB < 0 || (kl >= 0 && nL < 0)); ++v) {
      if (nB < 0 && ctx[v] == kb) nB = v;
      if (kl >= 0 && nL < 0 && v < U && ctx[v] + yn[v] == kl) nL = v;
    }
    for (int v = 0; v < u; ++v) {
      if (ctx[v] == kb) h &= ~1;
      if (kl >= 0 && ctx[v] + yn[v] == kl) h &= ~2;
    }
    nxb[u] = nB;
    nxl[u] = nL;
    hd[u] = h;
    xa[u] = u == 0 ? t_one<SR>() : zero;
  }
  __syncthreads();
  // ---- forward: alpha_t (Real: to the history) / the winning term (Max)
  for (int t = 0; t < nf; ++t) {
    const unsigned char* wf = wbase + t * FR * (BF16 ? 2 : 4);
    for (int u = tid; u < S; u += nthr) {
      wb[u] = ldw<BF16>(wf, ctx[u]);
      wl[u] = u < U ? ldw<BF16>(wf, ctx[u] + yn[u]) : zero;
      if (SR == M_REAL) a.alpha[((long long)b * T + t) * S + u] = xa[u];
    }
    __syncthreads();
    for (int u = tid; u < S; u += nthr) {
      float r;
      int wi = 0;
      if (K == 0) {
        if constexpr (SR == M_MAX) {
          const float x = xa[u] + wb[u];
          const float y = u >= 1 ? xa[u - 1] + wl[u - 1] : zero;
          wi = (u >= 1 && !(x >= y)) ? 1 : 0;  // a NaN blank term at u = 0 ends the path there
          r = x >= y ? x : y;
        } else {
          r = xa[u] * wb[u] + (u >= 1 ? xa[u - 1] * wl[u - 1] : 0.f);
        }
      } else {
        r = t_times<SR>(xa[u], wb[u]);
        for (int i = 1; i <= K; ++i) {
          float l = zero;
          if (u >= i) {
            l = t_times<SR>(xa[u - i], wl[u - i]);
            for (int j = u - i + 1; j < u; ++j) l = t_times<SR>(l, wl[j]);
          }
          const float term = t_times<SR>(l, wb[u]);
          if constexpr (SR == M_MAX) {
            if (term > r) {
              r = term;
              wi = i;
            }
          } else {
            r += term;
          }
        }
      }
      xb[u] = r;
      if (SR == M_MAX) a.win[((long long)b * T + t) * S + u] = (unsigned char)wi;
    }
    __syncthreads();
    for (int u = tid; u < S; u += nthr) xa[u] = xb[u];
    __syncthreads();
  }
  const int nlb = a.nlab[b];
  const int fin = (nlb >= 0 && nlb <= U) ? nlb : -1;
  const float gv = a.gin ? a.gin[b] : 1.f;
  if (tid == 0 && a.dist) a.dist[b] = fin >= 0 ? xa[fin] : zero;
  if constexpr (SR == M_MAX) {
    // ---- backward: one thread walks the decisions, staged in chunks
    int q = fin < 0 ? -1 : (xa[fin] > -kInf ? fin : (fin == 0 ? 0 : -1));
    const int F = max(1, kStrChunk / S);
    for (int t1 = nf; t1 > 0; t1 -= F) {
      const int t0 = max(0, t1 - F);
      const unsigned char* src = a.win + ((long long)b * T + t0) * S;
      for (int i = tid; i < (t1 - t0) * S; i += nthr) wc[i] = src[i];
      __syncthreads();
      if (tid == 0 && q >= 0) {
        for (int t = t1 - 1; t >= t0; --t) {
          const int wi = wc[(t - t0) * S + q];
          int nm = 0;
          auto mark = [&](int e) {
            for (int m = 0; m < nm; ++m)
              if (marks[2 * m] == e) {
                ++marks[2 * m + 1];
                return;
              }
            marks[2 * nm] = e;
            marks[2 * nm + 1] = 1;
            ++nm;
          };
          if (K == 0) {
            mark(wi ? ctx[q - 1] + yn[q - 1] : ctx[q]);
            q -= wi;
          } else {
            mark(ctx[q]);
            for (int j = q - wi; j < q; ++j) mark(ctx[j] + yn[j]);
            q -= wi;
          }
          unsigned char* dwf = dwbase + (long long)t * FR * (BF16 ? 2 : 4);
          for (int m = 0; m < nm; ++m) stw<BF16>(dwf, marks[2 * m], (float)marks[2 * m + 1] * gv);
        }
      }
      __syncthreads();
    }
  } else {
    // ---- backward: beta and the arc gradients frame by frame
    for (int u = tid; u < S; u += nthr) xb[u] = u == fin ? gv : 0.f;
    __syncthreads();
    for (int t = nf - 1; t >= 0; --t) {
      const unsigned char* wf = wbase + t * FR * (BF16 ? 2 : 4);
      for (int u = tid; u < S; u += nthr) {
        wb[u] = ldw<BF16>(wf, ctx[u]);
        wl[u] = u < U ? ldw<BF16>(wf, ctx[u] + yn[u]) : 0.f;
        xa[u] = a.alpha[((long long)b * T + t) * S + u];
      }
      __syncthreads();
      if (K == 0) {
        for (int u = tid; u < S; u += nthr) {
          gb[u] = xa[u] * xb[u];
          gl[u] = u < U ? xa[u] * xb[u + 1] : 0.f;
          xc[u] = wb[u] * xb[u] + (u < U ? wl[u] * xb[u + 1] : 0.f);
        }
      } else {
        for (int u = tid; u < S; u += nthr) {
          float s = xa[u];
          L[u] = xa[u];
          for (int i = 1; i <= K; ++i) {
            float l = 0.f;
            if (u >= i) {
              l = xa[u - i] * wl[u - i];
              for (int j = u - i + 1; j < u; ++j) l *= wl[j];
            }
            L[i * S + u] = l;
            s += l;
          }
          gb[u] = xb[u] * s;
          gl[u] = 0.f;
          d0[u] = xb[u] * wb[u];  // dL_K
        }
        __syncthreads();
        for (int i = K - 1; i >= 0; --i) {
          for (int u = tid; u < S; u += nthr) {
            const float up = u < U ? d0[u + 1] : 0.f;
            d1[u] = xb[u] * wb[u] + (u < U ? wl[u] * up : 0.f);
            if (u < U) gl[u] += L[i * S + u] * up;
          }
          __syncthreads();
          for (int u = tid; u < S; u += nthr) d0[u] = d1[u];
          __syncthreads();
        }
        for (int u = tid; u < S; u += nthr) xc[u] = d0[u];
      }
      __syncthreads();
      unsigned char* dwf = dwbase + (long long)t * FR * (BF16 ? 2 : 4);
      for (int u = tid; u < S; u += nthr) {
        if (hd[u] & 1) {
          float s = 0.f;
          for (int v = u; v >= 0; v = nxb[v]) s += gb[v];
          stw<BF16>(dwf, ctx[u], s);
        }
        if (hd[u] & 2) {
          float s = 0.f;
          for (int v = u; v >= 0; v = nxl[v]) s += gl[v];
          stw<BF16>(dwf, ctx[u] + yn[u], s);
        }
        xb[u] = xc[u];
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int t_fail(int code, const char* msg) { return lt_impl::set_error(code, msg); }
int t_hip(hipError_t e, const char* what) {
  return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, what);
}
constexpr int kTabLds = 160 * 1024;

int t_check(const lt_graph* g, const lt_table_problem* pb) {
  if (!g || !pb) return t_fail(LT_EINVAL, "null graph / problem");
  if (g->num_states < 1 || g->vocab_size < 1 || g->expansions < 0 || g->expansions > 255)
    return t_fail(LT_EINVAL, "bad graph (states >= 1, vocab >= 1, 0 <= expansions <= 255)");
  if (!g->next_state || !g->in_offsets || !g->in_arcs) return t_fail(LT_EINVAL, "null graph arrays");
  if (pb->batch < 0 || pb->max_frames < 0 || pb->max_labels < 0)
    return t_fail(LT_EINVAL, "negative shape");
  if (pb->weight_dtype != LT_DTYPE_F32 && pb->weight_dtype != LT_DTYPE_BF16)
    return t_fail(LT_EINVAL, "bad dtype");
  return LT_OK;
}

TArgs t_args(const lt_graph* g, const lt_table_problem* pb, const void* W, const int32_t* nf) {
  TArgs a;
  memset(&a, 0, sizeof(a));
  a.W = (const unsigned char*)W;
  a.nfr = nf;
  a.table = g->next_state;
  a.in_off = g->in_offsets;
  a.in_arc = g->in_arcs;
  a.B = pb->batch;
  a.T = pb->max_frames;
  a.U = pb->max_labels;
  a.C = g->num_states;
  a.V = g->vocab_size;
  a.R = g->vocab_size + 1;
  a.K = g->expansions;
  return a;
}

// threads per utterance workgroup: the denominator reductions take 8 lanes
// per state, so 512 threads cover up to 64 states in one pass
int tab_threads(const TArgs& a) {
  const char* e = lt_impl::tune_str("LT_TAB_THREADS");
  const int t = (e && *e) ? atoi(e) : (a.C > 32 ? 512 : 256);
  return t >= 512 ? 512 : 256;
}

template <typename KF>
int t_launch(KF k, int grid, int lds_bytes, hipStream_t st, const TArgs& a) {
  if (lds_bytes > kTabLds) return t_fail(LT_EUNSUPPORTED, "table lattice state exceeds LDS");
  if (lds_bytes > 64 * 1024)
    if (int rc = t_hip(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           lds_bytes), "table LDS"))
      return rc;
  if (grid == 0) return LT_OK;
  hipLaunchKernelGGL(k, dim3(grid), dim3(tab_threads(a)), lds_bytes, st, a);
  return t_hip(hipGetLastError(), "table kernel launch");
}

template <typename KF>
int t_launch2(KF k, int grid, int lds_bytes, hipStream_t st, const TArgs& a1, const TArgs& a2) {
  if (lds_bytes > kTabLds) return t_fail(LT_EUNSUPPORTED, "table lattice state exceeds LDS");
  if (lds_bytes > 64 * 1024)
    if (int rc = t_hip(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           lds_bytes), "table LDS"))
      return rc;
  if (grid == 0) return LT_OK;
  hipLaunchKernelGGL(k, dim3(grid), dim3(tab_threads(a1)), lds_bytes, st, a1, a2);
  return t_hip(hipGetLastError(), "table kernel launch");
}

int fwd_lds(int S) { return 4 * (4 * S) + 8 * S; }
// stage a frame in LDS when it fits beside the state vectors
constexpr int kStageBudget = 144 * 1024;

template <bool BF16, bool STG>
int launch_t_fwd_s(int sr, bool num, bool vit, const TArgs& a, int lds, hipStream_t st) {
  if (vit) return t_launch(tab_fwd_kernel<BF16, M_MAX, false, true, STG>, a.B, lds, st, a);
  if (num) {
    if (sr == M_LOG) return t_launch(tab_fwd_kernel<BF16, M_LOG, true, false, false>, a.B, lds, st, a);
    if (sr == M_MAX) return t_launch(tab_fwd_kernel<BF16, M_MAX, true, false, false>, a.B, lds, st, a);
    return t_launch(tab_fwd_kernel<BF16, M_REAL, true, false, false>, a.B, lds, st, a);
  }
  if (sr == M_LOG)
    return a.K > 0 ? t_launch(tab_fwd_fld_kernel<BF16, STG>, a.B, lds, st, a)
                   : t_launch(tab_fwd_kernel<BF16, M_LOG, false, false, STG>, a.B, lds, st, a);
  if (sr == M_MAX) return t_launch(tab_fwd_kernel<BF16, M_MAX, false, false, STG>, a.B, lds, st, a);
  return t_launch(tab_fwd_kernel<BF16, M_REAL, false, false, STG>, a.B, lds, st, a);
}

int graph_lds(const TArgs& a) { return 4 * ((a.C + 1 + 2 * a.C * a.V + 3) / 4 * 4); }

template <bool BF16>
int launch_t_fwd(int sr, bool num, bool vit, const TArgs& a0, hipStream_t st) {
  TArgs a = a0;
  const int S = num ? a.U + 1 : a.C;
  const long long FR = (long long)a.C * a.R;
  // + the string's compact weights and the Log string's (i, f) arrays
  const int lds = fwd_lds(S) + (num ? 16 * S : 0);
  // STAGE: graph and frame in LDS (when both fit; the string forward reads
  // two weights per position and stages nothing)
  // (K = 0: tab_fwd_k0_body stages two frames)
  const long long staged = (long long)lds + graph_lds(a) + (a.K == 0 ? 8 : 4) * FR;
  if (!num && staged <= kStageBudget)
    return launch_t_fwd_s<BF16, true>(sr, num, vit, a, (int)staged, st);
  return launch_t_fwd_s<BF16, false>(sr, num, vit, a, lds, st);
}

int t_fwd(int sr, bool num, bool vit, const TArgs& a, bool bf16, hipStream_t st) {
  return bf16 ? launch_t_fwd<true>(sr, num, vit, a, st) : launch_t_fwd<false>(sr, num, vit, a, st);
}

struct GradLayout {
  size_t hd, hn, nsub, ntab, dwf, lx, lxn, total;
};
GradLayout grad_layout(const lt_graph* g, const lt_table_problem* pb) {
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  GradLayout l;
  const long long BT = (long long)pb->batch * pb->max_frames, NK = 2LL * (pb->max_labels + 1);
  l.hd = 0;
  l.hn = up(4 * BT * g->num_states);
  l.nsub = l.hn + up(4 * BT * (pb->max_labels + 1));
  l.ntab = l.nsub + up(4 * BT * NK);
  l.dwf = l.ntab + up(4LL * pb->batch * NK);
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  l.lx = l.dwf + (bf16 ? up(4 * BT * g->num_states * (g->vocab_size + 1)) : 0);
  l.lxn = l.lx + (g->expansions > 0 ? up(4 * BT * g->expansions * g->num_states) : 0);
  l.total = l.lxn + (g->expansions > 0 ? up(4 * BT * g->expansions * (pb->max_labels + 1)) : 0);
  return l;
}

}  // namespace

extern "C" {

int lt_graph_in_arcs(int32_t num_states, int32_t vocab_size, const int32_t* next_state,
                     int32_t* in_offsets, int32_t* in_arcs) {
  if (num_states < 1 || vocab_size < 1 || !next_state || !in_offsets || !in_arcs)
    return t_fail(LT_EINVAL, "lt_graph_in_arcs: bad arguments");
  const int C = num_states, V = vocab_size;
  for (int q = 0; q <= C; ++q) in_offsets[q] = 0;
  for (long long i = 0; i < (long long)C * V; ++i) {
    const int q = next_state[i];
    if (q < 0 || q >= C) return t_fail(LT_EINVAL, "next_state entry out of range");
    ++in_offsets[q + 1];
  }
  for (int q = 0; q < C; ++q) in_offsets[q + 1] += in_offsets[q];
  std::vector<int> fill(in_offsets, in_offsets + C);
  for (int p = 0; p < C; ++p)  // ascending (p, y) within each next state
    for (int y = 0; y < V; ++y) {
      const int q = next_state[(long long)p * V + y];
      in_arcs[fill[q]++] = p * V + y;
    }
  return LT_OK;
}

int lt_table_forward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                     const void* W, const int32_t* num_frames, float* dist, float* alpha,
                     void* stream) {
  if (int rc = t_check(g, pb)) return rc;
  if (semiring < 0 || semiring > 2) return t_fail(LT_EINVAL, "bad semiring");
  if (pb->batch == 0) return LT_OK;
  if ((!W && pb->max_frames > 0) || !num_frames || !dist) return t_fail(LT_EINVAL, "null pointer");
  TArgs a = t_args(g, pb, W, num_frames);
  a.dist = dist;
  a.alpha = alpha;
  return t_fwd(semiring, false, false, a, pb->weight_dtype == LT_DTYPE_BF16, (hipStream_t)stream);
}

int lt_table_num_forward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                         const void* W, const int32_t* num_frames, const int32_t* labels,
                         const int32_t* num_labels, float* num, void* stream) {
  if (int rc = t_check(g, pb)) return rc;
  if (semiring < 0 || semiring > 2) return t_fail(LT_EINVAL, "bad semiring");
  if (pb->batch == 0) return LT_OK;
  if ((!W && pb->max_frames > 0) || !num_frames || !num_labels || !num ||
      (pb->max_labels > 0 && !labels))
    return t_fail(LT_EINVAL, "null pointer");
  TArgs a = t_args(g, pb, W, num_frames);
  a.labels = labels;
  a.nlab = num_labels;
  a.dist = num;
  return t_fwd(semiring, true, false, a, pb->weight_dtype == LT_DTYPE_BF16, (hipStream_t)stream);
}

int lt_table_loss_grad_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                       size_t* bytes) {
  if (int rc = t_check(g, pb)) return rc;
  if (bytes) *bytes = grad_layout(g, pb).total;
  return LT_OK;
}

int lt_table_loss_grad(const lt_graph* g, const lt_table_problem* pb, int32_t local_norm,
                       const void* W, const int32_t* num_frames, const int32_t* labels,
                       const int32_t* num_labels, float* loss, float* log_z, float* num,
                       void* dW, void* workspace, size_t workspace_bytes, void* stream) {
  if (int rc = t_check(g, pb)) return rc;
  if (pb->batch == 0) return LT_OK;
  if ((!W && pb->max_frames > 0) || !num_frames || !num_labels || !loss || !log_z || !num ||
      (pb->max_labels > 0 && !labels))
    return t_fail(LT_EINVAL, "null pointer");
  const GradLayout l = grad_layout(g, pb);
  if (dW && (!workspace || workspace_bytes < l.total)) return t_fail(LT_EINVAL, "workspace too small");
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  float* hd = dW ? (float*)((char*)workspace + l.hd) : nullptr;
  float* hn = dW ? (float*)((char*)workspace + l.hn) : nullptr;
  TArgs a = t_args(g, pb, W, num_frames);
  a.labels = labels;
  a.nlab = num_labels;
  a.local = local_norm ? 1 : 0;
  const int C = a.C, S = a.U + 1, K = a.K;
  const long long FR = (long long)C * a.R;
  int rc;
  // ---- forwards: denominator (log_z, alpha history) and string side by side
  TArgs ad = a, an = a;
  ad.dist = log_z;
  ad.alpha = hd;
  ad.lx = (dW && K > 0) ? (float*)((char*)workspace + l.lx) : nullptr;
  an.dist = num;
  an.alpha = hn;
  an.lx = (dW && K > 0) ? (float*)((char*)workspace + l.lxn) : nullptr;
  if (!local_norm) {
    const int ln = fwd_lds(S) + 16 * S;
    const int ld = fwd_lds(C);
    const long long staged = (long long)ld + graph_lds(a) + (a.K == 0 ? 8 : 4) * FR;
    if (staged <= kStageBudget) {
      const int l2 = std::max((int)staged, ln);
      rc = K > 0 ? (bf16 ? t_launch2(tab_fwd2_fld_kernel<true, true>, 2 * a.B, l2, st, ad, an)
                         : t_launch2(tab_fwd2_fld_kernel<false, true>, 2 * a.B, l2, st, ad, an))
                 : (bf16 ? t_launch2(tab_fwd2_kernel<true, true>, 2 * a.B, l2, st, ad, an)
                         : t_launch2(tab_fwd2_kernel<false, true>, 2 * a.B, l2, st, ad, an));
    } else {
      const int l2 = std::max(ld, ln);
      rc = K > 0 ? (bf16 ? t_launch2(tab_fwd2_fld_kernel<true, false>, 2 * a.B, l2, st, ad, an)
                         : t_launch2(tab_fwd2_fld_kernel<false, false>, 2 * a.B, l2, st, ad, an))
                 : (bf16 ? t_launch2(tab_fwd2_kernel<true, false>, 2 * a.B, l2, st, ad, an)
                         : t_launch2(tab_fwd2_kernel<false, false>, 2 * a.B, l2, st, ad, an));
    }
    if (rc) return rc;
  } else {
    if ((rc = t_hip(hipMemsetAsync(log_z, 0, sizeof(float) * pb->batch, st), "memset"))) return rc;
    if ((rc = t_fwd(M_LOG, true, false, an, bf16, st))) return rc;
  }
  hipLaunchKernelGGL(tab_loss_kernel, dim3((pb->batch + 255) / 256), dim3(256), 0, st, loss,
                     (const float*)log_z, (const float*)num, pb->batch, a.local);
  if ((rc = t_hip(hipGetLastError(), "loss launch"))) return rc;
  if (!dW) return LT_OK;
  // ---- backwards side by side; then dW -= the numerator's head sums
  float* dwf = bf16 ? (float*)((char*)workspace + l.dwf) : (float*)dW;
  a.dist = nullptr;
  a.alpha = nullptr;
  a.loss = nullptr;
  a.num_in = num;
  a.den_in = log_z;
  a.dW = dwf;
  a.nsub = (float*)((char*)workspace + l.nsub);
  a.ntab = (int*)((char*)workspace + l.ntab);
  ad = a;
  an = a;
  ad.hist = hd;
  an.lx = (dW && K > 0) ? (float*)((char*)workspace + l.lxn) : nullptr;
  ad.lx = (dW && K > 0) ? (float*)((char*)workspace + l.lx) : nullptr;
  ad.nsub = nullptr;
  ad.ntab = nullptr;
  an.hist = hn;
  const int lds_d = 4 * (3 * C + (K + 1) * C);
  // (K = 0: the one-barrier string backward double-buffers its rows, 80 S)
  const int lds_n = 4 * (8 * S + (K + 1) * S) + 4 * (2 * S + 2 * S) + 4 * (2 * S + 2 * S) +
                    (K == 0 ? 12 * S : 0);
  // K = 0: the one-barrier den backward stages two frames
  if (lds_d + graph_lds(a) + (K == 0 ? 8 : 4) * FR <= kStageBudget) {
    // + the lexical dW sums of FrameLabelDependent(K > 0) when they fit too
    ad.acc = K > 0 && lds_d + graph_lds(a) + 8 * FR <= kStageBudget;
    const int l2 =
        std::max((int)(lds_d + graph_lds(a) + ((ad.acc || K == 0) ? 8 : 4) * FR), lds_n);
    rc = K > 0 ? (bf16 ? t_launch2(tab_bwd2_fld_kernel<true, true>, 2 * a.B, l2, st, ad, an)
                       : t_launch2(tab_bwd2_fld_kernel<false, true>, 2 * a.B, l2, st, ad, an))
               : (bf16 ? t_launch2(tab_bwd2_kernel<true, true>, 2 * a.B, l2, st, ad, an)
                       : t_launch2(tab_bwd2_kernel<false, true>, 2 * a.B, l2, st, ad, an));
  } else {
    const int l2 = std::max(lds_d, lds_n);
    rc = bf16 ? t_launch2(tab_bwd2_kernel<true, false>, 2 * a.B, l2, st, ad, an)
              : t_launch2(tab_bwd2_kernel<false, false>, 2 * a.B, l2, st, ad, an);
  }
  if (rc) return rc;
  {
    const long long n = (long long)a.B * a.T * 2 * S;
    const int blocks = (int)std::min<long long>(4096, (n + 255) / 256);
    if (blocks > 0) hipLaunchKernelGGL(tab_apply_kernel, dim3(blocks), dim3(256), 0, st, a);
    if ((rc = t_hip(hipGetLastError(), "numerator apply launch"))) return rc;
  }
  if (!bf16) return LT_OK;
  const long long n = (long long)a.B * a.T * C * a.R;
  const int blocks = (int)std::min<long long>(4096, (n + 255) / 256);
  if (blocks > 0)
    hipLaunchKernelGGL(tab_to_bf16_kernel, dim3(blocks), dim3(256), 0, st, dwf,
                       (unsigned short*)dW, n);
  return t_hip(hipGetLastError(), "bf16 conversion launch");
}

// lt_table_den_backward's workspace: an fp32 gradient for bf16 W, and for
// MaxTropical the Viterbi backpointers, winning expansion counts, best final
// states and distances
struct DenBwdLayout {
  size_t dwf, bp, win, qstar, dist, total;
};
static DenBwdLayout den_bwd_layout(const lt_graph* g, const lt_table_problem* pb, int semiring) {
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  const long long BT = (long long)pb->batch * pb->max_frames;
  const int KK = g->expansions > 0 ? g->expansions : 1;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  DenBwdLayout l;
  l.dwf = 0;
  // the fp32 gradient only for bf16 W (fp32 W accumulates straight into dW)
  l.bp = bf16 ? up(4 * BT * g->num_states * (g->vocab_size + 1)) : 0;
  l.win = l.bp;
  l.qstar = l.bp;
  l.dist = l.bp;
  l.total = l.bp;
  if (semiring == M_MAX) {
    l.win = l.bp + up(4 * BT * KK * g->num_states);
    l.qstar = l.win + up(BT * g->num_states);
    l.dist = l.qstar + up(4LL * pb->batch);
    l.total = l.dist + up(4LL * pb->batch);
  }
  return l;
}

int lt_table_den_backward_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                          int32_t semiring, size_t* bytes) {
  if (int rc = t_check(g, pb)) return rc;
  if (semiring < 0 || semiring > 2) return t_fail(LT_EINVAL, "bad semiring");
  if (bytes) *bytes = den_bwd_layout(g, pb, semiring).total;
  return LT_OK;
}

int lt_table_den_backward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                          const void* W, const int32_t* num_frames, const float* dist,
                          const float* alpha, const float* grad, void* dW, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (int rc = t_check(g, pb)) return rc;
  if (semiring < 0 || semiring > 2) return t_fail(LT_EINVAL, "bad semiring");
  if (pb->batch == 0) return LT_OK;
  const bool maxt = semiring == M_MAX;
  if ((!W && pb->max_frames > 0) || !num_frames || (!dW && pb->max_frames > 0) ||
      (!maxt && (!dist || (!alpha && pb->max_frames > 0))))
    return t_fail(LT_EINVAL, "null pointer");
  const DenBwdLayout l = den_bwd_layout(g, pb, semiring);
  if (l.total && (!workspace || workspace_bytes < l.total))
    return t_fail(LT_EINVAL, "workspace too small");
  if (pb->max_frames == 0) return LT_OK;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  float* dwf = bf16 ? (float*)((char*)workspace + l.dwf) : (float*)dW;
  TArgs a = t_args(g, pb, W, num_frames);
  a.gin = grad;
  a.dW = dwf;
  const int C = a.C, K = a.K;
  const long long FR = (long long)C * a.R;
  const long long n = (long long)a.B * a.T * FR;
  int rc;
  if (maxt) {
    // the best path (tab_fwd_kernel VIT), then its arcs
    a.bp = (int*)((char*)workspace + l.bp);
    a.win = (unsigned char*)workspace + l.win;
    a.qstar = (int*)((char*)workspace + l.qstar);
    a.dist = (float*)((char*)workspace + l.dist);
    if ((rc = t_fwd(M_MAX, false, true, a, bf16, st))) return rc;
    if ((rc = t_hip(hipMemsetAsync(dwf, 0, sizeof(float) * n, st), "memset"))) return rc;
    const int threads = 64;
    hipLaunchKernelGGL(tab_onehot_kernel, dim3((a.B + threads - 1) / threads), dim3(threads), 0,
                       st, a);
    if ((rc = t_hip(hipGetLastError(), "one-hot launch"))) return rc;
  } else {
    a.hist = alpha;
    a.den_in = dist;
    a.num_in = dist;  // the den-only backward: live while the distance is finite
    const int lds_d = 4 * (3 * C + (K + 1) * C);
    if (lds_d + graph_lds(a) + (K == 0 ? 8 : 4) * FR <= kStageBudget) {
      a.acc = K > 0 && lds_d + graph_lds(a) + 8 * FR <= kStageBudget;
      const int lds = (int)(lds_d + graph_lds(a) + ((a.acc || K == 0) ? 8 : 4) * FR);
      if (semiring == M_LOG)
        rc = a.K > 0 ? (bf16 ? t_launch(tab_bwd_den_fld_kernel<true, true>, a.B, lds, st, a)
                             : t_launch(tab_bwd_den_fld_kernel<false, true>, a.B, lds, st, a))
                     : (bf16 ? t_launch(tab_bwd_den_kernel<true, true, M_LOG>, a.B, lds, st, a)
                             : t_launch(tab_bwd_den_kernel<false, true, M_LOG>, a.B, lds, st, a));
      else
        rc = bf16 ? t_launch(tab_bwd_den_kernel<true, true, M_REAL>, a.B, lds, st, a)
                  : t_launch(tab_bwd_den_kernel<false, true, M_REAL>, a.B, lds, st, a);
    } else {
      if (semiring == M_LOG)
        rc = bf16 ? t_launch(tab_bwd_den_kernel<true, false, M_LOG>, a.B, lds_d, st, a)
                  : t_launch(tab_bwd_den_kernel<false, false, M_LOG>, a.B, lds_d, st, a);
      else
        rc = bf16 ? t_launch(tab_bwd_den_kernel<true, false, M_REAL>, a.B, lds_d, st, a)
                  : t_launch(tab_bwd_den_kernel<false, false, M_REAL>, a.B, lds_d, st, a);
    }
    if (rc) return rc;
  }
  if (!bf16) return LT_OK;
  const int blocks = (int)std::min<long long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(tab_to_bf16_kernel, dim3(blocks), dim3(256), 0, st, dwf, (unsigned short*)dW, n);
  return t_hip(hipGetLastError(), "bf16 conversion launch");
}

static size_t str_grad_bytes(const lt_table_problem* pb, int semiring) {
  const long long BTS = (long long)pb->batch * pb->max_frames * (pb->max_labels + 1);
  return (size_t)((semiring == M_MAX ? BTS : 4 * BTS) + 255) & ~(size_t)255;
}

// LDS bytes of tab_str_grad_kernel: the string positions' rows and, for
// MaxTropical, the decision chunk
static long long str_grad_lds(const lt_graph* g, const lt_table_problem* pb, int32_t semiring) {
  const long long S = pb->max_labels + 1, K = g->expansions;
  return 4LL * (5 * S + (9 + K + 1 + 2) * S + 4 + ((K + 1 + 3) & ~3) * 2) +
         (semiring == M_MAX ? std::max<long long>(kStrChunk, S) : 0);
}

int lt_table_num_backward_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                          int32_t semiring, size_t* bytes) {
  if (int rc = t_check(g, pb)) return rc;
  if (semiring != M_MAX && semiring != M_REAL)
    return t_fail(LT_EUNSUPPORTED, "lt_table_num_backward: MaxTropical or Real (Log: "
                                   "lt_table_loss_grad with local_norm)");
  // the string-gradient kernel's LDS (tab_str_grad_kernel): refused here, so a
  // caller asking before its forward learns it up front
  if (str_grad_lds(g, pb, semiring) > kTabLds)
    return t_fail(LT_EUNSUPPORTED, "string gradient: labels exceed LDS");
  if (bytes) *bytes = str_grad_bytes(pb, semiring);
  return LT_OK;
}

int lt_table_num_backward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                          const void* W, const int32_t* num_frames, const int32_t* labels,
                          const int32_t* num_labels, const float* grad, float* num, void* dW,
                          void* workspace, size_t workspace_bytes, void* stream) {
  size_t need = 0;
  if (int rc = lt_table_num_backward_workspace_bytes(g, pb, semiring, &need)) return rc;
  if (pb->batch == 0) return LT_OK;
  if ((!W && pb->max_frames > 0) || !num_frames || !num_labels || (!dW && pb->max_frames > 0) ||
      (pb->max_labels > 0 && !labels))
    return t_fail(LT_EINVAL, "null pointer");
  if (need && (!workspace || workspace_bytes < need)) return t_fail(LT_EINVAL, "workspace too small");
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  TArgs a = t_args(g, pb, W, num_frames);
  a.labels = labels;
  a.nlab = num_labels;
  a.gin = grad;
  a.dist = num;
  a.dW = (float*)dW;
  if (semiring == M_MAX) a.win = (unsigned char*)workspace;
  else a.alpha = (float*)workspace;
  const long long n = (long long)a.B * a.T * a.C * a.R;
  if (n > 0)
    if (int rc = t_hip(hipMemsetAsync(dW, 0, (size_t)n * (bf16 ? 2 : 4), st), "memset")) return rc;
  const long long lds = str_grad_lds(g, pb, semiring);  // checked by the workspace query
  if (semiring == M_MAX)
    return bf16 ? t_launch(tab_str_grad_kernel<true, M_MAX>, a.B, (int)lds, st, a)
                : t_launch(tab_str_grad_kernel<false, M_MAX>, a.B, (int)lds, st, a);
  return bf16 ? t_launch(tab_str_grad_kernel<true, M_REAL>, a.B, (int)lds, st, a)
              : t_launch(tab_str_grad_kernel<false, M_REAL>, a.B, (int)lds, st, a);
}

int lt_table_viterbi_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                     size_t* bytes) {
  if (int rc = t_check(g, pb)) return rc;
  const long long BT = (long long)pb->batch * pb->max_frames;
  const int KK = g->expansions > 0 ? g->expansions : 1;
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  if (bytes) *bytes = up(4 * BT * KK * g->num_states) + up(BT * g->num_states) + up(4LL * pb->batch);
  return LT_OK;
}

int lt_table_viterbi(const lt_graph* g, const lt_table_problem* pb, const void* W,
                     const int32_t* num_frames, int32_t label_convention, int64_t* labels,
                     float* path_weight, void* workspace, size_t workspace_bytes, void* stream) {
  if (int rc = t_check(g, pb)) return rc;
  if (pb->batch == 0) return LT_OK;
  if ((!W && pb->max_frames > 0) || !num_frames || !path_weight || (!labels && pb->max_frames > 0))
    return t_fail(LT_EINVAL, "null pointer");
  size_t need = 0;
  lt_table_viterbi_workspace_bytes(g, pb, &need);
  if (!workspace || workspace_bytes < need) return t_fail(LT_EINVAL, "workspace too small");
  const long long BT = (long long)pb->batch * pb->max_frames;
  const int KK = g->expansions > 0 ? g->expansions : 1;
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  TArgs a = t_args(g, pb, W, num_frames);
  a.bp = (int*)workspace;
  a.win = (unsigned char*)workspace + up(4 * BT * KK * g->num_states);
  a.qstar = (int*)((char*)a.win + up(BT * g->num_states));
  a.dist = path_weight;
  a.conv = label_convention;
  a.vlabels = (long long*)labels;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = t_fwd(M_MAX, false, true, a, pb->weight_dtype == LT_DTYPE_BF16, st)) return rc;
  // staged walk when a frame's backpointers fit in LDS, else one thread per
  // utterance straight from global memory
  const long long per_frame = 4LL * KK * a.C + (a.K > 0 ? a.C : 0);
  const long long arcs_bytes = 4LL * a.C * a.V;
  const long long budget = 60 * 1024;
  const int arcs_lds = arcs_bytes <= budget / 2 ? 1 : 0;
  const long long room = budget - (arcs_lds ? arcs_bytes : 0);
  const int chunk = (int)std::min<long long>(std::max(1, a.T), room / per_frame);
  if (chunk >= 1 && !lt_impl::tune_str("LT_TAB_BT_SERIAL")) {
    const int lds = (int)((arcs_lds ? arcs_bytes : 0) + chunk * per_frame + 16);
    hipLaunchKernelGGL(tab_backtrace_lds_kernel, dim3(a.B), dim3(256), lds, st, a, chunk, arcs_lds);
  } else {
    const int threads = 64;
    hipLaunchKernelGGL(tab_backtrace_kernel, dim3((a.B + threads - 1) / threads), dim3(threads), 0,
                       st, a);
  }
  return t_hip(hipGetLastError(), "backtrace launch");
}

}  // extern "C"
