// lt_cpu.cpp -- the host twin of the lattice library (include/lt_lattice_cpu.h).
//
// The same lattice as the HIP kernels -- alignments.FrameDependent x
// contexts.FullNGram under Log / MaxTropical / Real (lattices.py:131-496,
// 686-799, 185-247) -- for host memory, built with g++ alone. Utterances are
// independent, so they are dealt to a pool of host threads; inside one
// utterance the frame loop is serial and each frame is vectorised over the
// V labels of a destination block:
//
//   * Full-order destinations come in blocks of V (contexts.py:226-229): the
//     V states (a.., y) for y = 1..V share their V+1 source states
//     p_k = pb + k V^(n-1), and their arcs are the contiguous label runs
//     W[p_k, 1..V]. A block is one pass over K rows of W with a length-V
//     vector of running maxima (Log: a second pass sums the exponentials).
//   * The backward recursion of source p reads W[p, 0..V] and beta over the
//     V consecutive states next(p, 1..V) = nb(p) + 1..V (contexts.py:190-205,
//     232-256): both contiguous.
//   * Log vectors are kept relative to an integer offset near their maximum
//     (exact in fp32); marginals take the large terms (offsets, log_z) in
//     double first and exponentiate a small float.
#include "../../include/lt_lattice_cpu.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err = "ok";
std::atomic<int> g_threads{0};

int fail(int code, const char* msg) {
  g_err = msg;
  return code;
}

constexpr float kNegInf = -INFINITY;

// FullNGram topology (contexts.py:149-256)
struct Topo {
  int V, n, C, R;
  int An;   // states of order < n: sum_{i<n} V^i
  int Apn;  // sum_{i<n-1} V^i: the first source state feeding full-order states
  int Vn1;  // V^(n-1) (source stride inside a destination block)
  int K;    // lexical in-arcs of a full-order destination
};

int make_topo(const lt_problem* pb, Topo* t) {
  if (!pb) return fail(LT_EINVAL, "null problem");
  if (pb->batch < 0 || pb->max_frames < 0 || pb->max_labels < 0)
    return fail(LT_EINVAL, "negative dimension");
  if (pb->weight_dtype != LT_DTYPE_F32 && pb->weight_dtype != LT_DTYPE_BF16)
    return fail(LT_EINVAL, "weight_dtype must be LT_DTYPE_F32 or LT_DTYPE_BF16");
  const int V = pb->vocab_size, n = pb->context_size;
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
  t->V = V; t->n = n; t->C = (int)C; t->R = V + 1;
  t->An = (int)An; t->Apn = (int)Apn; t->Vn1 = (int)Vn1;
  t->K = n == 0 ? V : V + 1;
  return LT_OK;
}

// next(p, y) - y for y >= 1 (contexts.py:190-205); n = 0 loops to state 0
inline int next_base(const Topo& g, int p) {
  if (g.n == 0) return -1;
  if (g.n == 1) return 0;
  if (p < g.An) return p * g.V;
  return ((p - g.An) % g.Vn1) * g.V + g.An - 1;
}

// Arc weights of frame `row` as fp32 (weight_fns.py:69-75 layout): fp32 W
// is read in place, bf16 W widened once per frame into a per-thread buffer,
// so the frame loops below are plain float loops the compiler vectorises.
const float* frame_at(const void* W, bool bf16, long long row, long long FR) {
  if (!bf16) return (const float*)W + row * FR;
  thread_local std::vector<float> buf;
  if ((long long)buf.size() < FR) buf.resize(FR);
  const uint16_t* h = (const uint16_t*)W + row * FR;
  for (long long e = 0; e < FR; ++e) {
    const uint32_t u = (uint32_t)h[e] << 16;
    std::memcpy(&buf[e], &u, 4);
  }
  return buf.data();
}

// exp(x) in fp32 without a libm call, so loops over it vectorise:
// x = n ln2 + r (Cody-Waite, |r| <= ln2 / 2), e^r by its degree-6 Taylor
// polynomial (relative error < 2e-7 on that range), 2^n into the exponent.
// exp(-inf) = 0 and anything below -103.3 flushes to 0; +inf and anything
// above 88.7 give +inf; NaN propagates.
inline float exp_f(float x) {
  const float t = std::min(std::max(x, -104.f), 89.f);
  // round to nearest by the 1.5 * 2^23 shift; n in [-151, 129]
  const float nf = (t * 1.44269504088896341f + 12582912.f) - 12582912.f;
  const float r = std::fma(nf, -0.693145751953125f, std::fma(nf, -1.428606765330187e-06f, t));
  float p = 1.f / 720.f;
  p = std::fma(p, r, 1.f / 120.f);
  p = std::fma(p, r, 1.f / 24.f);
  p = std::fma(p, r, 1.f / 6.f);
  p = std::fma(p, r, 0.5f);
  p = std::fma(p, r, 1.f);
  p = std::fma(p, r, 1.f);
  // 2^n in two halves so n down to -150 stays representable through denormals
  const int n = (int)nf;
  const int n1 = n >> 1, n2 = n - n1;
  float s1, s2;
  const int32_t b1 = (n1 + 127) << 23, b2 = (n2 + 127) << 23;
  std::memcpy(&s1, &b1, 4);
  std::memcpy(&s2, &b2, 4);
  float v = p * s1 * s2;
  v = x < -103.3f ? 0.f : v;
  v = x > 88.72f ? INFINITY : v;
  return x != x ? x : v;
}

inline uint16_t to_bf16(float f) {  // round to nearest even, NaN kept
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
void store_row(void* dW, bool bf16, long long off, const float* v, int n) {
  if (bf16) {
    uint16_t* d = (uint16_t*)dW + off;
    for (int i = 0; i < n; ++i) d[i] = to_bf16(v[i]);
  } else {
    std::memcpy((float*)dW + off, v, sizeof(float) * n);
  }
}
void zero_rows(void* dW, bool bf16, long long off, long long n) {
  if (n <= 0) return;
  std::memset((char*)dW + off * (bf16 ? 2 : 4), 0, (size_t)n * (bf16 ? 2 : 4));
}

// semirings.py:248-255 / 279-286: c = max, a non-finite c is replaced by 0
inline float safe(float c) { return std::isfinite(c) ? c : 0.f; }

// The default pool size: the CPUs this process may run on (its affinity
// mask, which cgroup cpusets also narrow), not the machine's count.
int default_threads() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    const int n = CPU_COUNT(&set);
    if (n > 0) return n;
  }
  return (int)std::max(1u, std::thread::hardware_concurrency());
}

// Runs fn(b, worker) for every utterance b on the thread pool. An exception
// inside a worker (a per-utterance buffer that cannot be allocated) or a
// thread that cannot be started ends the call with an LT_* code instead of
// std::terminate: the other workers stop taking utterances, and the caller
// returns the code.
template <typename F>
int for_utterances(int B, F&& fn) {
  int nt = g_threads.load();
  if (nt <= 0) nt = default_threads();
  nt = std::max(1, std::min(nt, B));
  std::atomic<int> next{0};
  std::atomic<int> err{LT_OK};
  auto work = [&](int w) {
    try {
      for (int b = next++; b < B && err.load(std::memory_order_relaxed) == LT_OK; b = next++)
        fn(b, w);
    } catch (const std::bad_alloc&) {
      int ok = LT_OK;
      err.compare_exchange_strong(ok, LT_ENOMEM);
    } catch (...) {
      int ok = LT_OK;
      err.compare_exchange_strong(ok, LT_EINVAL);
    }
  };
  std::vector<std::thread> pool;
  try {
    pool.reserve(nt);
    for (int w = 1; w < nt; ++w) pool.emplace_back(work, w);
  } catch (...) {
    // fewer workers than asked: the ones started and this thread finish the batch
  }
  work(0);
  for (auto& th : pool) th.join();
  const int rc = err.load();
  if (rc == LT_ENOMEM) return fail(rc, "host memory exhausted in a worker");
  if (rc != LT_OK) return fail(rc, "exception in a worker");
  return LT_OK;
}

// ---------------------------------------------------------------------------
// One frame of the denominator forward (alignments.py:286-297 with
// contexts.py:207-230): a -> na. SR: LT_SEMIRING_LOG / MAX / REAL.
// MAX records backpointers (0 = blank, k + 1 = lexical in-arc k) in bp.
// ---------------------------------------------------------------------------
struct FwdScratch {
  std::vector<float> m, s;
  std::vector<int> bi;
  explicit FwdScratch(int V) : m(V), s(V), bi(V) {}
};

template <int SR>
void den_step(const Topo& g, const float* w, const float* a, float* na, int16_t* bp,
              FwdScratch& sc) {
  const int V = g.V, R = g.R;
  float* m = sc.m.data();
  float* s = sc.s.data();
  int* bi = sc.bi.data();
  auto blank = [&](int q) {
    const float wb = w[(long long)q * R];
    return SR == LT_SEMIRING_REAL ? a[q] * wb : a[q] + wb;
  };
  // combine a destination's blank term with its reduced lexical term
  auto finish = [&](int q, float bt, float lex, int k) {
    if (SR == LT_SEMIRING_MAX) {
      // Maximum chooses the blank term iff it is >= (semirings.py:363)
      if (bt >= lex) { na[q] = bt; if (bp) bp[q] = 0; }
      else { na[q] = lex; if (bp) bp[q] = (int16_t)(k + 1); }
    } else if (SR == LT_SEMIRING_REAL) {
      na[q] = bt + lex;
    } else {  // logaddexp (semirings.py:248-255)
      const float c = safe(std::max(bt, lex));
      na[q] = c + std::log(exp_f(bt - c) + exp_f(lex - c));
    }
  };
  if (g.n == 0) {  // one state, V lexical self loops (labels 1..V)
    const float a0 = a[0];
    float r = SR == LT_SEMIRING_REAL ? 0.f : kNegInf;
    int best = 0;
    if (SR == LT_SEMIRING_MAX) {
      r = a0 + w[1];
      for (int k = 1; k < V; ++k) {
        const float x = a0 + w[1 + k];
        if (x > r) { r = x; best = k; }  // first maximum (semirings.py:382)
      }
    } else if (SR == LT_SEMIRING_REAL) {
      for (int k = 0; k < V; ++k) r += a0 * w[1 + k];
    } else {
      float mx = kNegInf;
      for (int k = 0; k < V; ++k) mx = std::max(mx, a0 + w[1 + k]);
      const float c = safe(mx);
      float acc = 0.f;
      for (int k = 0; k < V; ++k) acc += exp_f(a0 + w[1 + k] - c);
      r = c + std::log(acc);
    }
    finish(0, blank(0), r, best);
    return;
  }
  // the start state: blank self loop only (contexts.py:216-217)
  na[0] = blank(0);
  if (SR == LT_SEMIRING_MAX && bp) bp[0] = 0;
  // ascending states: one lexical in-arc each (contexts.py:222-225)
  for (int q = 1; q < g.An; ++q) {
    const int p = (q - 1) / V, y = (q - 1) % V + 1;
    const float wl = w[(long long)p * R + y];
    finish(q, blank(q), SR == LT_SEMIRING_REAL ? a[p] * wl : a[p] + wl, 0);
  }
  // full-order destinations, one block of V per source run
  const int blocks = (g.C - g.An) / V;
  for (int blk = 0; blk < blocks; ++blk) {
    const int q0 = g.An + blk * V, pb = g.Apn + blk;
    if (SR == LT_SEMIRING_REAL) {
      for (int y = 0; y < V; ++y) m[y] = 0.f;
      for (int k = 0; k < g.K; ++k) {
        const int p = pb + k * g.Vn1;
        const float ap = a[p];
        const long long e0 = (long long)p * R + 1;
        for (int y = 0; y < V; ++y) m[y] += ap * w[e0 + y];
      }
      for (int y = 0; y < V; ++y) finish(q0 + y, blank(q0 + y), m[y], 0);
      continue;
    }
    {  // running maximum over the sources, in ascending k (first maximum wins)
      const int p = pb;
      const float ap = a[p];
      const long long e0 = (long long)p * R + 1;
      for (int y = 0; y < V; ++y) { m[y] = ap + w[e0 + y]; bi[y] = 0; }
    }
    for (int k = 1; k < g.K; ++k) {
      const int p = pb + k * g.Vn1;
      const float ap = a[p];
      const long long e0 = (long long)p * R + 1;
      if (SR == LT_SEMIRING_MAX) {
        for (int y = 0; y < V; ++y) {
          const float x = ap + w[e0 + y];
          if (x > m[y]) { m[y] = x; bi[y] = k; }
        }
      } else {
#pragma omp simd
        for (int y = 0; y < V; ++y) m[y] = std::max(m[y], ap + w[e0 + y]);
      }
    }
    if (SR == LT_SEMIRING_MAX) {
      for (int y = 0; y < V; ++y) finish(q0 + y, blank(q0 + y), m[y], bi[y]);
      continue;
    }
    // Log: logsumexp over the sources (semirings.py:279-286), then the blank
    for (int y = 0; y < V; ++y) { m[y] = safe(m[y]); s[y] = 0.f; }
    for (int k = 0; k < g.K; ++k) {
      const int p = pb + k * g.Vn1;
      const float ap = a[p];
      const long long e0 = (long long)p * R + 1;
#pragma omp simd
      for (int y = 0; y < V; ++y) s[y] += exp_f(ap + w[e0 + y] - m[y]);
    }
    for (int y = 0; y < V; ++y) finish(q0 + y, blank(q0 + y), m[y] + std::log(s[y]), 0);
  }
}

// Log vectors: subtract the integer part of the max (exact); returns it
float renorm(float* v, int n) {
  float mx = kNegInf;
  for (int i = 0; i < n; ++i) mx = std::max(mx, v[i]);
  if (!std::isfinite(mx)) return 0.f;
  const float sub = std::floor(mx);
  for (int i = 0; i < n; ++i) v[i] -= sub;
  return sub;
}

// (+) over a vector (the final sum, lattices.py:496 / 375-377)
double lse_abs(const float* v, int n, double off) {
  float mx = kNegInf;
  for (int i = 0; i < n; ++i) mx = std::max(mx, v[i]);
  const float c = safe(mx);
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += std::exp((double)v[i] - c);
  return off + c + std::log(s);
}

// ---------------------------------------------------------------------------
// Numerator (lattices.py:250-377): context state and next label per string
// position (walk_states, contexts.py:109-146; labels outside [0, V] are
// epsilon, label 0 reads as class 1: lattices.py:314-315, 337-338).
// ---------------------------------------------------------------------------
struct StringArcs {
  std::vector<int> ctx, ynext;
};
int next_state(const Topo& g, int p, int y) {
  if (g.n == 0) return 0;
  return next_base(g, p) + y;
}
void string_arcs(const Topo& g, int U, const int32_t* lab, StringArcs* s) {
  s->ctx.assign(U + 1, 0);
  s->ynext.assign(U + 1, 1);
  int c = 0;
  for (int u = 0; u <= U; ++u) {
    s->ctx[u] = c;
    int y = u < U ? lab[u] : 1;
    if (u < U && (y < 0 || y > g.V)) y = 0;
    s->ynext[u] = y < 1 ? 1 : y;
    if (u < U && y != 0) c = next_state(g, c, y);
  }
}

template <int SR>
void num_step(const Topo& g, const float* w, const StringArcs& sa, const float* a, float* na,
              int NP) {
  const int R = g.R;
  for (int u = 0; u < NP; ++u) {
    const float wb = w[(long long)sa.ctx[u] * R];
    const float bt = SR == LT_SEMIRING_REAL ? a[u] * wb : a[u] + wb;
    float lx = SR == LT_SEMIRING_REAL ? 0.f : kNegInf;  // shift_down (alignments.py:233-248)
    if (u >= 1) {
      const float wl = w[(long long)sa.ctx[u - 1] * R + sa.ynext[u - 1]];
      lx = SR == LT_SEMIRING_REAL ? a[u - 1] * wl : a[u - 1] + wl;
    }
    if (SR == LT_SEMIRING_REAL) na[u] = bt + lx;
    else if (SR == LT_SEMIRING_MAX) na[u] = bt >= lx ? bt : lx;
    else {
      const float c = safe(std::max(bt, lx));
      na[u] = c + std::log(exp_f(bt - c) + exp_f(lx - c));
    }
  }
}

// ---------------------------------------------------------------------------
// Per-utterance drivers
// ---------------------------------------------------------------------------
struct Problem {
  Topo g;
  int B, T, U;
  bool bf16;
  long long FR;
};

int load_problem(const lt_problem* pb, Problem* P) {
  int rc = make_topo(pb, &P->g);
  if (rc) return rc;
  P->B = pb->batch; P->T = pb->max_frames; P->U = pb->max_labels;
  P->bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  P->FR = (long long)P->g.C * P->g.R;
  return LT_OK;
}

inline int clamp_frames(const int32_t* nf, int b, int T) {
  const int v = nf[b];
  return v < 0 ? 0 : (v > T ? T : v);
}

// Denominator forward of utterance b. Log: `hist` rows relative to the
// per-frame offsets `off` (hist[t] + off[t] = alpha_t); returns log_z.
// Other semirings: exact values, offsets 0. alpha_abs (nullable) receives
// absolute rows, padding frames carrying alpha_nf.
template <int SR>
double den_forward_utt(const Problem& P, const void* W, int b, int nf, float* hist, float* off,
                       float* alpha_abs, int16_t* bp, std::vector<float>& a,
                       std::vector<float>& na, FwdScratch& sc) {
  const Topo& g = P.g;
  const int C = g.C;
  for (int q = 0; q < C; ++q)
    a[q] = q == 0 ? (SR == LT_SEMIRING_REAL ? 1.f : 0.f) : (SR == LT_SEMIRING_REAL ? 0.f : kNegInf);
  float O = 0.f;
  for (int t = 0; t < nf; ++t) {
    if (hist) std::memcpy(hist + (long long)t * C, a.data(), sizeof(float) * C);
    if (off) off[t] = O;
    if (alpha_abs)
      for (int q = 0; q < C; ++q) alpha_abs[(long long)t * C + q] = O + a[q];
    const float* w = frame_at(W, P.bf16, (long long)b * P.T + t, P.FR);
    den_step<SR>(g, w, a.data(), na.data(), bp ? bp + (long long)t * C : nullptr, sc);
    a.swap(na);
    if (SR == LT_SEMIRING_LOG) O += renorm(a.data(), C);
  }
  if (alpha_abs)
    for (int t = nf; t < P.T; ++t)
      for (int q = 0; q < C; ++q) alpha_abs[(long long)t * C + q] = O + a[q];
  if (SR == LT_SEMIRING_LOG) return lse_abs(a.data(), C, O);
  if (SR == LT_SEMIRING_REAL) {
    double s = 0.0;
    for (int q = 0; q < C; ++q) s += a[q];
    return s;
  }
  float r = a[0];
  for (int q = 1; q < C; ++q) r = std::max(r, a[q]);
  return r;
}

template <int SR>
double num_forward_utt(const Problem& P, const void* W, int b, int nf, const StringArcs& sa,
                       int nl, float* hist, float* off, float* alpha_abs, std::vector<float>& a,
                       std::vector<float>& na) {
  const int NP = P.U + 1;
  for (int u = 0; u < NP; ++u)
    a[u] = u == 0 ? (SR == LT_SEMIRING_REAL ? 1.f : 0.f) : (SR == LT_SEMIRING_REAL ? 0.f : kNegInf);
  float O = 0.f;
  for (int t = 0; t < nf; ++t) {
    if (hist) std::memcpy(hist + (long long)t * NP, a.data(), sizeof(float) * NP);
    if (off) off[t] = O;
    if (alpha_abs)
      for (int u = 0; u < NP; ++u) alpha_abs[(long long)t * NP + u] = O + a[u];
    const float* w = frame_at(W, P.bf16, (long long)b * P.T + t, P.FR);
    num_step<SR>(P.g, w, sa, a.data(), na.data(), NP);
    a.swap(na);
    if (SR == LT_SEMIRING_LOG) O += renorm(a.data(), NP);
  }
  if (alpha_abs)
    for (int t = nf; t < P.T; ++t)
      for (int u = 0; u < NP; ++u) alpha_abs[(long long)t * NP + u] = O + a[u];
  if (nl < 0 || nl > P.U) return SR == LT_SEMIRING_REAL ? 0.0 : -INFINITY;
  return (double)O + a[nl];
}

// Denominator backward of one utterance (alignments.py:300-318 in reverse
// frame order): beta_t from beta_{t+1}, and for every frame the marginals
//   exp(alpha_t[p] + W[p, y] + beta_{t+1}[next(p, y)] - log_z) * gb
// written to `dfr` (one frame, FR floats) and handed to emit(t, dfr).
// alpha_t = ah[t] + aoff[t] (aoff nullable = 0).
template <typename Emit>
void den_backward_utt(const Problem& P, const void* W, int b, int nf, const float* ah,
                      const float* aoff, double log_z, float gb, std::vector<float>& bcur,
                      std::vector<float>& bnxt, std::vector<float>& dfr, Emit&& emit) {
  const Topo& g = P.g;
  const int C = g.C, R = g.R, V = g.V;
  std::fill(bcur.begin(), bcur.end(), 0.f);  // every state is final (lattices.py:788-790)
  float Ob = 0.f;
  std::vector<float> x(R), bz(V);
  for (int t = nf - 1; t >= 0; --t) {
    const float* w = frame_at(W, P.bf16, (long long)b * P.T + t, P.FR);
    const double kt = (aoff ? (double)aoff[t] : 0.0) + Ob - log_z;
    const float* at = ah + (long long)t * C;
    for (int p = 0; p < C; ++p) {
      const long long e0 = (long long)p * R;
      const int nb = next_base(g, p);
      // beta over next(p, 1..V): contiguous (n = 0: every label loops to 0)
      if (nb < 0) std::fill(bz.begin(), bz.end(), bcur[0]);
      const float* bl = nb < 0 ? bz.data() : bcur.data() + nb + 1;
      float* xp = x.data();
      const float* wp = w + e0;
      xp[0] = wp[0] + bcur[p];
#pragma omp simd
      for (int y = 1; y <= V; ++y) xp[y] = wp[y] + bl[y - 1];
      float mx = kNegInf;
#pragma omp simd reduction(max : mx)
      for (int y = 0; y <= V; ++y) mx = std::max(mx, xp[y]);
      const bool live = std::isfinite(mx);
      const float c = live ? mx : 0.f;
      float s = 0.f;
#pragma omp simd reduction(+ : s)
      for (int y = 0; y <= V; ++y) { xp[y] = exp_f(xp[y] - c); s += xp[y]; }
      bnxt[p] = c + std::log(s);
      // no finite out-term: no marginal, whatever alpha is
      const float sp = (gb == 0.f || !live) ? 0.f : (float)std::exp((double)at[p] + c + kt) * gb;
      float* dp = dfr.data() + e0;
#pragma omp simd
      for (int y = 0; y <= V; ++y) dp[y] = xp[y] * sp;
    }
    emit(t, dfr.data());
    bcur.swap(bnxt);
    Ob += renorm(bcur.data(), C);
  }
}

int check_ptrs(const void* W, long long T) { return (!W && T > 0) ? 1 : 0; }

}  // namespace

extern "C" {

int lt_cpu_set_num_threads(int32_t n) {
  g_threads.store(n > 0 ? n : 0);
  return LT_OK;
}

int lt_cpu_num_threads(void) {
  const int nt = g_threads.load();
  return nt > 0 ? nt : default_threads();
}

const char* lt_cpu_last_error(void) { return g_err.c_str(); }

int lt_cpu_den_forward(const lt_problem* pb, int32_t semiring, const void* W,
                       const int32_t* num_frames, float* dist, float* alpha) {
  Problem P;
  int rc = load_problem(pb, &P);
  if (rc) return rc;
  if (semiring < LT_SEMIRING_LOG || semiring > LT_SEMIRING_REAL)
    return fail(LT_EINVAL, "semiring must be LT_SEMIRING_LOG, _MAX or _REAL");
  if (P.B == 0) return LT_OK;
  if (check_ptrs(W, P.T) || !num_frames || !dist) return fail(LT_EINVAL, "null pointer");
  const int C = P.g.C;
  rc = for_utterances(P.B, [&](int b, int) {
    std::vector<float> a(C), na(C);
    FwdScratch sc(P.g.V);
    const int nf = clamp_frames(num_frames, b, P.T);
    float* ab = alpha ? alpha + (long long)b * P.T * C : nullptr;
    double r;
    if (semiring == LT_SEMIRING_LOG)
      r = den_forward_utt<LT_SEMIRING_LOG>(P, W, b, nf, nullptr, nullptr, ab, nullptr, a, na, sc);
    else if (semiring == LT_SEMIRING_MAX)
      r = den_forward_utt<LT_SEMIRING_MAX>(P, W, b, nf, nullptr, nullptr, ab, nullptr, a, na, sc);
    else
      r = den_forward_utt<LT_SEMIRING_REAL>(P, W, b, nf, nullptr, nullptr, ab, nullptr, a, na, sc);
    dist[b] = (float)r;
  });
  return rc;
}

int lt_cpu_num_forward(const lt_problem* pb, int32_t semiring, const void* W,
                       const int32_t* num_frames, const int32_t* labels,
                       const int32_t* num_labels, float* num, float* alpha_num) {
  Problem P;
  int rc = load_problem(pb, &P);
  if (rc) return rc;
  if (semiring < LT_SEMIRING_LOG || semiring > LT_SEMIRING_REAL)
    return fail(LT_EINVAL, "semiring must be LT_SEMIRING_LOG, _MAX or _REAL");
  if (P.B == 0) return LT_OK;
  if (check_ptrs(W, P.T) || !num_frames || !num_labels || !num || (!labels && P.U > 0))
    return fail(LT_EINVAL, "null pointer");
  const int NP = P.U + 1;
  rc = for_utterances(P.B, [&](int b, int) {
    std::vector<float> a(NP), na(NP);
    StringArcs sa;
    string_arcs(P.g, P.U, labels ? labels + (long long)b * P.U : nullptr, &sa);
    const int nf = clamp_frames(num_frames, b, P.T);
    float* ab = alpha_num ? alpha_num + (long long)b * P.T * NP : nullptr;
    double r;
    if (semiring == LT_SEMIRING_LOG)
      r = num_forward_utt<LT_SEMIRING_LOG>(P, W, b, nf, sa, num_labels[b], nullptr, nullptr, ab, a, na);
    else if (semiring == LT_SEMIRING_MAX)
      r = num_forward_utt<LT_SEMIRING_MAX>(P, W, b, nf, sa, num_labels[b], nullptr, nullptr, ab, a, na);
    else
      r = num_forward_utt<LT_SEMIRING_REAL>(P, W, b, nf, sa, num_labels[b], nullptr, nullptr, ab, a, na);
    num[b] = (float)r;
  });
  return rc;
}

int lt_cpu_den_backward(const lt_problem* pb, const void* W, const int32_t* num_frames,
                        const float* log_z, const float* alpha, const float* grad, void* dW) {
  Problem P;
  int rc = load_problem(pb, &P);
  if (rc) return rc;
  if (P.B == 0) return LT_OK;
  if (check_ptrs(W, P.T) || !num_frames || !log_z || (!alpha && P.T > 0) || (!dW && P.T > 0))
    return fail(LT_EINVAL, "null pointer");
  const int C = P.g.C;
  rc = for_utterances(P.B, [&](int b, int) {
    std::vector<float> bc(C), bn(C), dfr(P.FR);
    const int nf = clamp_frames(num_frames, b, P.T);
    float gb = grad ? grad[b] : 1.f;
    if (!std::isfinite(log_z[b])) gb = 0.f;
    const long long base = (long long)b * P.T * P.FR;
    den_backward_utt(P, W, b, nf, alpha + (long long)b * P.T * C, nullptr, log_z[b], gb, bc, bn,
                     dfr, [&](int t, const float* d) {
                       store_row(dW, P.bf16, base + (long long)t * P.FR, d, (int)P.FR);
                     });
    zero_rows(dW, P.bf16, base + (long long)nf * P.FR, (long long)(P.T - nf) * P.FR);
  });
  return rc;
}

int lt_cpu_loss_grad(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels,
                     const int32_t* num_labels, const float* grad, float* loss,
                     float* log_z, float* num, void* dW) {
  Problem P;
  int rc = load_problem(pb, &P);
  if (rc) return rc;
  if (P.B == 0) return LT_OK;
  if (check_ptrs(W, P.T) || !num_frames || !num_labels || !loss || (!labels && P.U > 0))
    return fail(LT_EINVAL, "null pointer");
  const Topo& g = P.g;
  const int C = g.C, R = g.R, NP = P.U + 1;
  const bool den = !local_norm;
  rc = for_utterances(P.B, [&](int b, int) {
    const int nf = clamp_frames(num_frames, b, P.T);
    const int nl = num_labels[b];
    StringArcs sa;
    string_arcs(g, P.U, labels ? labels + (long long)b * P.U : nullptr, &sa);
    const bool want = dW != nullptr;
    // forward: den (global normalisation) and numerator, histories kept for
    // the backward
    std::vector<float> a(std::max(C, NP)), na(std::max(C, NP));
    std::vector<float> ah(want && den ? (size_t)nf * C : 0), aoff(want && den ? nf : 0);
    std::vector<float> nh(want ? (size_t)nf * NP : 0), noff(want ? nf : 0);
    FwdScratch sc(g.V);
    double lz = 0.0;
    if (den)
      lz = den_forward_utt<LT_SEMIRING_LOG>(P, W, b, nf, want ? ah.data() : nullptr,
                                            want ? aoff.data() : nullptr, nullptr, nullptr, a,
                                            na, sc);
    const double nv = num_forward_utt<LT_SEMIRING_LOG>(P, W, b, nf, sa, nl,
                                                       want ? nh.data() : nullptr,
                                                       want ? noff.data() : nullptr, nullptr, a,
                                                       na);
    loss[b] = (float)(den ? lz - nv : -nv);  // lattices.py:178-183
    if (log_z) log_z[b] = den ? (float)lz : 0.f;
    if (num) num[b] = (float)nv;
    if (!want) return;
    float gb = grad ? grad[b] : 1.f;
    // unreachable label string (loss = +inf) or degenerate partition: dW = 0
    if (!std::isfinite(nv) || (den && !std::isfinite(lz))) gb = 0.f;
    const long long base = (long long)b * P.T * P.FR;
    zero_rows(dW, P.bf16, base + (long long)nf * P.FR, (long long)(P.T - nf) * P.FR);
    // numerator backward: beta^n and its marginals, one frame at a time in
    // step with the den backward, subtracted from the den marginals of the
    // same frame (ascending u: deterministic when positions share an arc)
    std::vector<float> nb(NP), nbn(NP), dfr(P.FR, 0.f), bc(C), bn(C);
    for (int u = 0; u < NP; ++u) nb[u] = u == nl ? 0.f : kNegInf;
    float Obn = 0.f;
    auto num_frame = [&](int t, float* d) {
      const float* w = frame_at(W, P.bf16, (long long)b * P.T + t, P.FR);
      const double kt = (double)noff[t] + Obn - nv;
      const float* at = nh.data() + (long long)t * NP;
      for (int u = 0; u < NP; ++u) {
        const long long eb = (long long)sa.ctx[u] * R;
        const bool lex = u < P.U;
        const long long el = lex ? eb + sa.ynext[u] : eb;
        const float xb = w[eb] + nb[u];
        const float xl = lex ? w[el] + nb[u + 1] : kNegInf;
        const float mx = std::max(xb, xl);
        const bool live = std::isfinite(mx);
        const float c = live ? mx : 0.f;
        const float ebv = exp_f(xb - c), elv = exp_f(xl - c);
        nbn[u] = c + std::log(ebv + elv);
        if (gb != 0.f && live) {
          const float sp = (float)std::exp((double)at[u] + c + kt) * gb;
          d[eb] -= ebv * sp;
          if (lex) d[el] -= elv * sp;
        }
      }
      nb.swap(nbn);
      Obn += renorm(nb.data(), NP);
    };
    if (den) {
      den_backward_utt(P, W, b, nf, ah.data(), aoff.data(), lz, gb, bc, bn, dfr,
                       [&](int t, float* d) {
                         num_frame(t, d);
                         store_row(dW, P.bf16, base + (long long)t * P.FR, d, (int)P.FR);
                       });
    } else {
      for (int t = nf - 1; t >= 0; --t) {
        std::fill(dfr.begin(), dfr.end(), 0.f);
        num_frame(t, dfr.data());
        store_row(dW, P.bf16, base + (long long)t * P.FR, dfr.data(), (int)P.FR);
      }
    }
  });
  return rc;
}

int lt_cpu_viterbi(const lt_problem* pb, const void* W, const int32_t* num_frames,
                   int32_t label_convention, int64_t* labels, float* path_weight,
                   const float* grad, void* arcs) {
  Problem P;
  int rc = load_problem(pb, &P);
  if (rc) return rc;
  if (label_convention != LT_LABELS_TRUE && label_convention != LT_LABELS_REFERENCE)
    return fail(LT_EINVAL, "label_convention must be LT_LABELS_TRUE or LT_LABELS_REFERENCE");
  if (P.B == 0) return LT_OK;
  if (check_ptrs(W, P.T) || !num_frames || !path_weight || (!labels && P.T > 0))
    return fail(LT_EINVAL, "null pointer");
  const Topo& g = P.g;
  const int C = g.C, R = g.R, V = g.V;
  rc = for_utterances(P.B, [&](int b, int) {
    const int nf = clamp_frames(num_frames, b, P.T);
    std::vector<float> a(C), na(C);
    std::vector<int16_t> bp((size_t)std::max(nf, 1) * C);
    FwdScratch sc(V);
    den_forward_utt<LT_SEMIRING_MAX>(P, W, b, nf, nullptr, nullptr, nullptr, bp.data(), a, na,
                                     sc);
    int q = 0;  // best final state: first maximum (semirings.py:382)
    for (int k = 1; k < C; ++k)
      if (a[k] > a[q]) q = k;
    path_weight[b] = a[q];
    const float gv = grad ? grad[b] : 1.f;
    int64_t* lab = labels + (long long)b * P.T;
    std::vector<float> one(arcs ? P.FR : 0);
    const long long base = (long long)b * P.T * P.FR;
    if (arcs) zero_rows(arcs, P.bf16, base + (long long)nf * P.FR, (long long)(P.T - nf) * P.FR);
    for (int t = P.T - 1; t >= nf; --t) lab[t] = 0;
    for (int t = nf - 1; t >= 0; --t) {
      const int k = bp[(long long)t * C + q];
      long long e;
      if (k == 0) {  // blank self loop
        lab[t] = 0;
        e = (long long)q * R;
      } else {
        // lexical in-arc k-1 of q: its source and label (contexts.py:207-230)
        int p, y;
        if (g.n == 0) { p = 0; y = k; }
        else if (q < g.An) { p = (q - 1) / V; y = (q - 1) % V + 1; }
        else { p = g.Apn + (q - g.An) / V + (k - 1) * g.Vn1; y = (q - g.An) % V + 1; }
        lab[t] = label_convention == LT_LABELS_REFERENCE ? y - 1 : y;
        e = (long long)p * R + y;
        q = p;
      }
      if (arcs) {
        std::fill(one.begin(), one.end(), 0.f);
        one[e] = gv;
        store_row(arcs, P.bf16, base + (long long)t * P.FR, one.data(), (int)P.FR);
      }
    }
  });
  return rc;
}

}  // extern "C"
