/*
 * lattice_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the
 * reference algorithm (theadamsabra/last_torch) for the lattice hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline. The
 * product path (last_torch_amd) never calls it.
 *
 * Pinned against the reference itself: the fixtures tests/golden/lattice_*.npz
 * (and contexts.npz, semirings.npz) are made by tests/golden/make_golden.py
 * importing /root/reference/last_torch, and tests/test_oracle_golden.py checks
 * every function here against them.
 *
 * Restated, not re-derived: the per-frame steps follow the reference's own
 * tensor formulation, cited per function:
 *   FullNGram.next_state          contexts.py:190-205
 *   FullNGram.forward_reduce      contexts.py:207-230 (reshape [-1, V^n], sum dim -2)
 *   FullNGram.backward_broadcast  contexts.py:232-256
 *   FrameDependent.forward        alignments.py:286-297
 *   FrameDependent.backward       alignments.py:300-318
 *   FrameDependent.string_forward alignments.py:320-329, shift_down :233-248
 *   RecognitionLattice._forward   lattices.py:379-496 (padding :460-461)
 *   RecognitionLattice._string_forward lattices.py:250-377
 *   RecognitionLattice.forward    lattices.py:131-183
 *   RecognitionLattice.shortest_path lattices.py:185-247
 *   Log semiring                  semirings.py:184-305 (safe max: non-finite -> 0)
 *   MaxTropical tie rules         semirings.py:354-401
 *
 * Precision: Log and Real are evaluated in double; MaxTropical in float so
 * that values and tie decisions are bit-identical to the fp32 reference.
 * The gradient (never produced by the reference, defects D1-D4) is the
 * per-frame FrameDependent.backward composed in the correct reverse order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_LOG 0
#define ORC_MAX 1
#define ORC_REAL 2

typedef struct {
  int V, n, C, An, Apn, Vn;
} ngram_t;

static void ngram_init(int V, int n, ngram_t* g) {
  long long pw = 1, C = 0, An = 0, Apn = 0;
  for (int i = 0; i <= n; ++i) {
    if (i < n) An += pw;
    if (i < n - 1) Apn += pw;
    C += pw;
    if (i < n) pw *= V;
  }
  g->V = V; g->n = n; g->C = (int)C; g->An = (int)An; g->Apn = (int)Apn;
  g->Vn = (int)pw; /* V^n */
}

/* contexts.py:190-205 */
int orc_next_state(int V, int n, int state, int label) {
  ngram_t g;
  ngram_init(V, n, &g);
  if (label == 0) return state;
  if (state < g.An) return state * V + label;
  if (n == 0) return 0;
  int vn1 = 1;
  for (int i = 0; i < n - 1; ++i) vn1 *= V;
  return ((state - g.An) % vn1) * V + g.An + label - 1;
}

int orc_num_states(int V, int n) {
  ngram_t g;
  ngram_init(V, n, &g);
  return g.C;
}

/* ---------------- semiring scalar ops ---------------- */
static const double kNegInf = -INFINITY;

static double d_logaddexp(double a, double b) { /* semirings.py:248-255 */
  double c = a > b ? a : b;
  if (!isfinite(c)) c = 0.0;
  return c + log(exp(a - c) + exp(b - c));
}

static double d_logsumexp(const double* x, int n) { /* semirings.py:279-286 */
  if (n == 0) return kNegInf; /* Log.sum of empty -> zeros (semirings.py:213-220) */
  double c = x[0];
  for (int i = 1; i < n; ++i) if (x[i] > c) c = x[i];
  if (!isfinite(c)) c = 0.0;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += exp(x[i] - c);
  return c + log(s);
}

/* forward_reduce (contexts.py:207-230) on one [C, V] block of double
 * weights, semiring LOG or REAL. out[C]. */
static void forward_reduce_d(const ngram_t* g, const double* w, int semiring, double* out,
                             double* tmp) {
  const int V = g->V, C = g->C;
  int q = 0;
  if (g->n > 0) out[q++] = (semiring == ORC_REAL) ? 0.0 : kNegInf; /* zeros part */
  /* weights[..., :A'_n, :] flattened: one arc each (ascending states) */
  for (int e = 0; e < g->Apn * V; ++e) out[q++] = w[e];
  /* weights[..., A'_n:, :].reshape(-1, V^n), sum over dim -2 */
  const int rows = (C - g->Apn) * V / g->Vn;
  for (int jq = 0; jq < g->Vn; ++jq) {
    for (int k = 0; k < rows; ++k) tmp[k] = w[g->Apn * V + k * g->Vn + jq];
    if (semiring == ORC_REAL) {
      double s = 0.0;
      for (int k = 0; k < rows; ++k) s += tmp[k];
      out[q++] = s;
    } else {
      out[q++] = d_logsumexp(tmp, rows);
    }
  }
}

/* MaxTropical forward_reduce in float with Max's first-argmax. arg[q] is
 * the winning source row index k inside the reduced axis (or -1 if the
 * destination has no lexical arc); src/lab give the arc. */
static void forward_reduce_max(const ngram_t* g, const float* w, float* out, int* src, int* lab) {
  const int V = g->V, C = g->C;
  int q = 0;
  if (g->n > 0) { out[q] = -INFINITY; src[q] = -1; lab[q] = 0; q++; }
  for (int e = 0; e < g->Apn * V; ++e) {
    out[q] = w[e]; src[q] = e / V; lab[q] = e % V + 1; q++;
  }
  const int rows = (C - g->Apn) * V / g->Vn;
  for (int jq = 0; jq < g->Vn; ++jq) {
    int best = 0;
    float bv = w[g->Apn * V + jq];
    for (int k = 1; k < rows; ++k) {
      const float v = w[g->Apn * V + k * g->Vn + jq];
      if (v > bv) { bv = v; best = k; } /* torch.argmax: first maximum */
    }
    const int e = g->Apn * V + best * g->Vn + jq;
    out[q] = bv; src[q] = e / V; lab[q] = e % V + 1; q++;
  }
}

/* backward_broadcast (contexts.py:232-256): out[p*V + (y-1)] = beta[next(p,y)] */
static void backward_broadcast_d(const ngram_t* g, const double* beta, double* out) {
  const int V = g->V, C = g->C;
  if (g->n == 0) {
    for (int y = 0; y < V; ++y) out[y] = beta[0];
    return;
  }
  int r = 0;
  /* part_a: weights[..., 1:A_n] reshaped [-1, V] */
  for (int q = 1; q < g->An; ++q) out[r++] = beta[q];
  /* part_b: broadcast weights[..., A_n:] to [(1+V), V^n] then [-1, V] */
  for (int rep = 0; rep < 1 + V; ++rep)
    for (int jq = 0; jq < g->Vn; ++jq) out[r++] = beta[g->An + jq];
  (void)C;
}

/* ---------------- denominator ---------------- */

/* _forward (lattices.py:379-496) for one utterance.
 * W: [T, C, V+1] float; alpha_out: [T, C] (float) or NULL. */
static double den_forward_one(const ngram_t* g, int T, const float* W, int nf, int semiring,
                              double* alpha_hist /* [T+1, C] or NULL */, float* alpha_out) {
  const int C = g->C, V = g->V, R = V + 1;
  double* a = (double*)malloc(sizeof(double) * C);
  double* na = (double*)malloc(sizeof(double) * C);
  double* lw = (double*)malloc(sizeof(double) * C * V);
  double* red = (double*)malloc(sizeof(double) * C);
  double* tmp = (double*)malloc(sizeof(double) * (C + V + 2));
  for (int q = 0; q < C; ++q) a[q] = (q == 0) ? (semiring == ORC_REAL ? 1.0 : 0.0)
                                             : (semiring == ORC_REAL ? 0.0 : kNegInf);
  for (int t = 0; t < T; ++t) {
    if (alpha_out) for (int q = 0; q < C; ++q) alpha_out[(long long)t * C + q] = (float)a[q];
    if (alpha_hist) memcpy(alpha_hist + (long long)t * C, a, sizeof(double) * C);
    if (t >= nf) continue; /* padding carries alpha */
    const float* w = W + (long long)t * C * R;
    for (int p = 0; p < C; ++p)
      for (int y = 0; y < V; ++y) {
        const double wv = w[p * R + 1 + y];
        lw[p * V + y] = semiring == ORC_REAL ? a[p] * wv : a[p] + wv;
      }
    forward_reduce_d(g, lw, semiring, red, tmp);
    for (int q = 0; q < C; ++q) {
      const double bt = semiring == ORC_REAL ? a[q] * w[q * R] : a[q] + w[q * R];
      na[q] = semiring == ORC_REAL ? bt + red[q] : d_logaddexp(bt, red[q]);
    }
    memcpy(a, na, sizeof(double) * C);
  }
  if (alpha_hist) memcpy(alpha_hist + (long long)T * C, a, sizeof(double) * C);
  double r;
  if (semiring == ORC_REAL) {
    r = 0.0;
    for (int q = 0; q < C; ++q) r += a[q];
  } else {
    r = d_logsumexp(a, C);
  }
  free(a); free(na); free(lw); free(red); free(tmp);
  return r;
}

/* MaxTropical _forward + shortest_path for one utterance (float, exact).
 * labels_out[T] (int64) per convention (0 true labels, 1 reference y-1);
 * arcs_out [T, C, V+1] float or NULL (one-hot path indicator). */
static float viterbi_one(const ngram_t* g, int T, const float* W, int nf, int conv,
                         float* alpha_out, long long* labels_out, float* arcs_out) {
  const int C = g->C, V = g->V, R = V + 1;
  float* a = (float*)malloc(sizeof(float) * C);
  float* na = (float*)malloc(sizeof(float) * C);
  float* lw = (float*)malloc(sizeof(float) * C * V);
  float* red = (float*)malloc(sizeof(float) * C);
  int* src = (int*)malloc(sizeof(int) * C);
  int* lab = (int*)malloc(sizeof(int) * C);
  /* backpointers: -1 = blank, else source state, and label */
  int* bps = (int*)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1) * C);
  int* bpl = (int*)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1) * C);
  for (int q = 0; q < C; ++q) a[q] = q == 0 ? 0.0f : -INFINITY;
  for (int t = 0; t < T; ++t) {
    if (alpha_out) memcpy(alpha_out + (long long)t * C, a, sizeof(float) * C);
    if (t >= nf) continue;
    const float* w = W + (long long)t * C * R;
    for (int p = 0; p < C; ++p)
      for (int y = 0; y < V; ++y) lw[p * V + y] = a[p] + w[p * R + 1 + y];
    forward_reduce_max(g, lw, red, src, lab);
    for (int q = 0; q < C; ++q) {
      const float bt = a[q] + w[q * R];
      if (bt >= red[q]) { /* Maximum: choose a iff a >= b (semirings.py:363) */
        na[q] = bt; bps[t * C + q] = -1; bpl[t * C + q] = 0;
      } else {
        na[q] = red[q]; bps[t * C + q] = src[q]; bpl[t * C + q] = lab[q];
      }
    }
    memcpy(a, na, sizeof(float) * C);
  }
  int q = 0;
  float best = a[0];
  for (int k = 1; k < C; ++k) if (a[k] > best) { best = a[k]; q = k; } /* first argmax */
  if (arcs_out) memset(arcs_out, 0, sizeof(float) * (size_t)T * C * R);
  for (int t = T - 1; t >= 0; --t) {
    if (t >= nf) { labels_out[t] = 0; continue; }
    const int s = bps[t * C + q], y = bpl[t * C + q];
    if (s < 0) {
      labels_out[t] = 0;
      if (arcs_out) arcs_out[((long long)t * C + q) * R] = 1.0f;
    } else {
      labels_out[t] = conv == 1 ? (long long)(y - 1) : (long long)y;
      if (arcs_out) arcs_out[((long long)t * C + s) * R + y] = 1.0f;
      q = s;
    }
  }
  free(a); free(na); free(lw); free(red); free(src); free(lab); free(bps); free(bpl);
  return best;
}

/* ---------------- numerator ---------------- */

/* walk_states + gather indices (contexts.py:109-146, lattices.py:314-338). */
static void string_arcs(const ngram_t* g, int U, const int* labels, int* ctx, int* ynext) {
  int c = 0;
  for (int u = 0; u <= U; ++u) {
    ctx[u] = c;
    int y = (u < U) ? labels[u] : 1; /* context_next_labels pads with 1 */
    if (u < U && (y < 0 || y > g->V)) y = 0;
    ynext[u] = (y - 1 < 0) ? 1 : y; /* make_safe_classes */
    if (u < U && y != 0) c = orc_next_state(g->V, g->n, c, y);
  }
}

/* _string_forward for one utterance. alpha_out [T, U+1] float or NULL;
 * alpha_hist [T+1, U+1] double or NULL. */
static double num_forward_one(const ngram_t* g, int T, int U, const float* W, int nf,
                              const int* labels, int nl, int semiring, float* alpha_out,
                              double* alpha_hist) {
  const int NP = U + 1, R = g->V + 1, C = g->C;
  int* ctx = (int*)malloc(sizeof(int) * NP);
  int* yn = (int*)malloc(sizeof(int) * NP);
  string_arcs(g, U, labels, ctx, yn);
  double* a = (double*)malloc(sizeof(double) * NP);
  double* na = (double*)malloc(sizeof(double) * NP);
  const double zero = semiring == ORC_REAL ? 0.0 : kNegInf;
  const double one = semiring == ORC_REAL ? 1.0 : 0.0;
  for (int u = 0; u < NP; ++u) a[u] = u == 0 ? one : zero;
  for (int t = 0; t < T; ++t) {
    if (alpha_out) for (int u = 0; u < NP; ++u) alpha_out[(long long)t * NP + u] = (float)a[u];
    if (alpha_hist) memcpy(alpha_hist + (long long)t * NP, a, sizeof(double) * NP);
    if (t >= nf) continue;
    const float* w = W + (long long)t * C * R;
    for (int u = 0; u < NP; ++u) {
      const double wb = w[ctx[u] * R];
      double bt = semiring == ORC_REAL ? a[u] * wb : a[u] + wb;
      double lx = zero; /* shift_down: position 0 gets semiring zero */
      if (u >= 1) {
        const double wl = w[ctx[u - 1] * R + yn[u - 1]];
        lx = semiring == ORC_REAL ? a[u - 1] * wl : a[u - 1] + wl;
      }
      /* MaxTropical runs in float like the reference (exact, same operand order). */
      if (semiring == ORC_MAX) { bt = (float)bt; lx = (float)lx; }
      if (semiring == ORC_REAL) na[u] = bt + lx;
      else if (semiring == ORC_MAX) na[u] = (bt >= lx) ? bt : lx;
      else na[u] = d_logaddexp(bt, lx);
    }
    memcpy(a, na, sizeof(double) * NP);
  }
  if (alpha_hist) memcpy(alpha_hist + (long long)T * NP, a, sizeof(double) * NP);
  const double r = (nl >= 0 && nl <= U) ? a[nl] : zero;
  free(ctx); free(yn); free(a); free(na);
  return r;
}

/* ---------------- public entry points ---------------- */

/* dist[B], alpha [B,T,C] (nullable). MaxTropical runs in float. */
void orc_den_forward(int B, int T, int V, int n, const float* W, const int* nf, int semiring,
                     float* dist, float* alpha) {
  ngram_t g;
  ngram_init(V, n, &g);
  const long long FR = (long long)g.C * (V + 1);
  for (int b = 0; b < B; ++b) {
    int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    float* ab = alpha ? alpha + (long long)b * T * g.C : NULL;
    if (semiring == ORC_MAX) {
      long long* lab = (long long*)malloc(sizeof(long long) * (T > 0 ? T : 1));
      dist[b] = viterbi_one(&g, T, Wb, nfb, 0, ab, lab, NULL);
      free(lab);
    } else {
      dist[b] = (float)den_forward_one(&g, T, Wb, nfb, semiring, NULL, ab);
    }
  }
}

void orc_num_forward(int B, int T, int U, int V, int n, const float* W, const int* nf,
                     const int* labels, const int* nl, int semiring, float* num,
                     float* alpha_num) {
  ngram_t g;
  ngram_init(V, n, &g);
  const long long FR = (long long)g.C * (V + 1);
  for (int b = 0; b < B; ++b) {
    int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    float* an = alpha_num ? alpha_num + (long long)b * T * (U + 1) : NULL;
    num[b] = (float)num_forward_one(&g, T, U, W + (long long)b * T * FR, nfb,
                                    labels + (long long)b * U, nl[b], semiring, an, NULL);
  }
}

void orc_viterbi(int B, int T, int V, int n, const float* W, const int* nf, int conv,
                 long long* labels, float* weight, float* arcs) {
  ngram_t g;
  ngram_init(V, n, &g);
  const long long FR = (long long)g.C * (V + 1);
  for (int b = 0; b < B; ++b) {
    int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    weight[b] = viterbi_one(&g, T, W + (long long)b * T * FR, nfb, conv, NULL,
                            labels + (long long)b * T, arcs ? arcs + (long long)b * T * FR : NULL);
  }
}

/* Denominator marginals: the correct-order composition of
 * FrameDependent.backward (alignments.py:300-318) with padding per
 * lattices.py:775-779 and beta_T = Log.ones (lattices.py:788-790).
 * dW [B,T,C,V+1] += scale[b] * marginal. log_z out [B]. */
static void den_marginals_one(const ngram_t* g, int T, const float* W, int nf, double scale,
                              double* dW, double* log_z_out) {
  const int C = g->C, V = g->V, R = V + 1;
  double* ah = (double*)malloc(sizeof(double) * (size_t)(T + 1) * C);
  const double log_z = den_forward_one(g, T, W, nf, ORC_LOG, ah, NULL);
  if (log_z_out) *log_z_out = log_z;
  double* beta = (double*)malloc(sizeof(double) * C);
  double* nb = (double*)malloc(sizeof(double) * C);
  double* bb = (double*)malloc(sizeof(double) * C * V);
  double* tmp = (double*)malloc(sizeof(double) * (V + 2));
  for (int q = 0; q < C; ++q) beta[q] = 0.0;
  for (int t = nf - 1; t >= 0; --t) {
    const float* w = W + (long long)t * C * R;
    const double* al = ah + (long long)t * C;
    backward_broadcast_d(g, beta, bb);
    for (int p = 0; p < C; ++p) {
      const double blank_beta = w[p * R] + beta[p];
      const double ls = al[p] - log_z;
      if (scale != 0.0) dW[(long long)t * C * R + p * R] += scale * exp(blank_beta + ls);
      for (int y = 0; y < V; ++y) {
        const double lb = w[p * R + 1 + y] + bb[p * V + y];
        tmp[y] = lb;
        if (scale != 0.0) dW[(long long)t * C * R + p * R + 1 + y] += scale * exp(lb + ls);
      }
      nb[p] = d_logaddexp(blank_beta, d_logsumexp(tmp, V));
    }
    memcpy(beta, nb, sizeof(double) * C);
  }
  free(ah); free(beta); free(nb); free(bb); free(tmp);
}

/* Numerator marginals: beta over the string acceptor (the reverse of
 * alignments.py:320-329), gathered back onto W (lattices.py:314-324). */
static void num_marginals_one(const ngram_t* g, int T, int U, const float* W, int nf,
                              const int* labels, int nl, double scale, double* dW,
                              double* num_out) {
  const int NP = U + 1, R = g->V + 1, C = g->C;
  double* ah = (double*)malloc(sizeof(double) * (size_t)(T + 1) * NP);
  const double num = num_forward_one(g, T, U, W, nf, labels, nl, ORC_LOG, NULL, ah);
  if (num_out) *num_out = num;
  int* ctx = (int*)malloc(sizeof(int) * NP);
  int* yn = (int*)malloc(sizeof(int) * NP);
  string_arcs(g, U, labels, ctx, yn);
  double* beta = (double*)malloc(sizeof(double) * NP);
  double* nbt = (double*)malloc(sizeof(double) * NP);
  for (int u = 0; u < NP; ++u) beta[u] = (u == nl) ? 0.0 : kNegInf;
  const int ok = isfinite(num) && scale != 0.0;
  for (int t = nf - 1; t >= 0; --t) {
    const float* w = W + (long long)t * C * R;
    const double* al = ah + (long long)t * NP;
    for (int u = 0; u < NP; ++u) {
      const double xb = w[ctx[u] * R] + beta[u];
      const double xl = (u < U) ? w[ctx[u] * R + yn[u]] + beta[u + 1] : kNegInf;
      nbt[u] = d_logaddexp(xb, xl);
      if (ok) {
        dW[(long long)t * C * R + ctx[u] * R] += scale * exp(al[u] + xb - num);
        if (u < U) dW[(long long)t * C * R + ctx[u] * R + yn[u]] += scale * exp(al[u] + xl - num);
      }
    }
    memcpy(beta, nbt, sizeof(double) * NP);
  }
  free(ah); free(ctx); free(yn); free(beta); free(nbt);
}

/* d log_z / dW, scaled by grad[b] (nullable = 1). */
void orc_den_grad(int B, int T, int V, int n, const float* W, const int* nf, const float* grad,
                  float* log_z, float* dW) {
  ngram_t g;
  ngram_init(V, n, &g);
  const long long FR = (long long)g.C * (V + 1);
  double* acc = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1) * FR);
  for (int b = 0; b < B; ++b) {
    int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    memset(acc, 0, sizeof(double) * (size_t)T * FR);
    double lz;
    den_marginals_one(&g, T, W + (long long)b * T * FR, nfb, grad ? grad[b] : 1.0, acc, &lz);
    log_z[b] = (float)lz;
    for (long long e = 0; e < (long long)T * FR; ++e) dW[(long long)b * T * FR + e] = (float)acc[e];
  }
  free(acc);
}

/* RecognitionLattice.forward loss and its gradient (local_norm: -num only).
 * Utterances with an unreachable label string (num = -inf) get dW = 0. */
void orc_loss_grad(int B, int T, int U, int V, int n, const float* W, const int* nf,
                   const int* labels, const int* nl, int local_norm, const float* grad,
                   float* loss, float* log_z, float* num, float* dW) {
  ngram_t g;
  ngram_init(V, n, &g);
  const long long FR = (long long)g.C * (V + 1);
  double* acc = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1) * FR);
  for (int b = 0; b < B; ++b) {
    int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    const double gb = grad ? grad[b] : 1.0;
    const double nv = num_forward_one(&g, T, U, Wb, nfb, labels + (long long)b * U, nl[b],
                                      ORC_LOG, NULL, NULL);
    double lz = 0.0;
    if (!local_norm) lz = den_forward_one(&g, T, Wb, nfb, ORC_LOG, NULL, NULL);
    const int live = isfinite(nv) && (local_norm || isfinite(lz));
    memset(acc, 0, sizeof(double) * (size_t)T * FR);
    if (dW && live) {
      if (!local_norm) den_marginals_one(&g, T, Wb, nfb, gb, acc, NULL);
      num_marginals_one(&g, T, U, Wb, nfb, labels + (long long)b * U, nl[b], -gb, acc, NULL);
    }
    if (dW)
      for (long long e = 0; e < (long long)T * FR; ++e) dW[(long long)b * T * FR + e] = (float)acc[e];
    if (log_z) log_z[b] = (float)lz;
    if (num) num[b] = (float)nv;
    loss[b] = (float)(local_norm ? -nv : lz - nv);
  }
  free(acc);
}
