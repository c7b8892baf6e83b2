/*
 * table_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the
 * reference's recognition lattice for an ARBITRARY context dependency given
 * as a next-state table and for both alignment lattices:
 *   K = 0  FrameDependent                     alignments.py:250-329
 *   K >= 1 FrameLabelDependent(max_expansions=K) alignments.py:331-432
 * Only tests/ may load it, as the checker of the generic (table) kernels.
 *
 * Restated from (reference file:line):
 *   NextStateTable.next_state            contexts.py:291-298 (epsilon stays)
 *   forward_reduce: (+) over the in-arcs of each state (the intended
 *     semantics; NextStateTable.forward_reduce at contexts.py:300-313 sums
 *     with scatter 'sum' then takes max -- defect D8 -- so the table path is
 *     pinned through FullNGram.next_state_table(), contexts.py:258-263,
 *     whose results must equal FullNGram's, and through FrameLabelDependent
 *     fixtures made by the reference itself with FullNGram)
 *   backward_broadcast                   contexts.py:315-320
 *   FrameDependent.forward / backward / string_forward alignments.py:286-329
 *   FrameLabelDependent.forward          alignments.py:363-377 (terms stacked
 *     then summed: Log logsumexp, MaxTropical first argmax)
 *   FrameLabelDependent.backward         alignments.py:379-419
 *   FrameLabelDependent.string_forward   alignments.py:421-432
 *   RecognitionLattice._forward / _string_forward / forward / shortest_path
 *     lattices.py:131-496 (padding frames carry alpha, :460-461; string
 *     weights :314-338 with label 0 -> 1 and the pad label 1)
 *   Log semiring safe max (non-finite -> 0)  semirings.py:248-286
 *   MaxTropical ties: Maximum keeps a iff a >= b (semirings.py:363), Max
 *     picks the first argmax (semirings.py:382)
 *
 * With alignment-state-invariant weights (lattices.py:444-447) every
 * expansion uses the same W: lexical marginals of all expansions add up on
 * one arc weight, and so do the K+1 blank marginals.
 *
 * Precision: Log and Real in double; MaxTropical in float with the
 * reference's operand order (bit-exact). Gradients: the per-frame backward
 * composed in reverse frame order (the reference's _backward walks forward,
 * D4), numerator through the same recursion on the string acceptor.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TAB_LOG 0
#define TAB_MAX 1
#define TAB_REAL 2

static const double kNegInf = -INFINITY;

/* A lattice frame graph: S states, blank weight index per state, lexical
 * arcs (src, dst, widx) grouped by dst in ascending (src, label) order. */
typedef struct {
  int S, A;
  int* blank;           /* [S] W index of the state's blank arc */
  int* src, *dst, *wix; /* [A] */
  int* in_off;          /* [S+1] arcs into each state (CSR over dst) */
  int* out_off, *out_arc; /* [S+1], [A] arcs out of each state */
} graph_t;

static void graph_finish(graph_t* g) {
  g->in_off = (int*)calloc((size_t)(unsigned)g->S + 1, sizeof(int));
  g->out_off = (int*)calloc((size_t)(unsigned)g->S + 1, sizeof(int));
  g->out_arc = (int*)malloc(sizeof(int) * (g->A > 0 ? g->A : 1));
  for (int a = 0; a < g->A; ++a) { g->in_off[g->dst[a] + 1]++; g->out_off[g->src[a] + 1]++; }
  for (int s = 0; s < g->S; ++s) { g->in_off[s + 1] += g->in_off[s]; g->out_off[s + 1] += g->out_off[s]; }
  int* fill = (int*)calloc((size_t)(unsigned)g->S + 1, sizeof(int));
  for (int a = 0; a < g->A; ++a) g->out_arc[g->out_off[g->src[a]] + fill[g->src[a]]++] = a;
  free(fill);
}

static void graph_free(graph_t* g) {
  free(g->blank); free(g->src); free(g->dst); free(g->wix);
  free(g->in_off); free(g->out_off); free(g->out_arc);
}

/* context graph: states p, arcs p --y--> table[p][y-1], W index p*R + y;
 * arcs sorted by (dst, src, y) -- the reduce order of forward_reduce */
static void context_graph(int C, int V, const int* table, graph_t* g) {
  const int R = V + 1;
  g->S = C;
  g->A = C * V;
  g->blank = (int*)malloc(sizeof(int) * C);
  g->src = (int*)malloc(sizeof(int) * g->A);
  g->dst = (int*)malloc(sizeof(int) * g->A);
  g->wix = (int*)malloc(sizeof(int) * g->A);
  for (int p = 0; p < C; ++p) g->blank[p] = p * R;
  int a = 0;
  for (int q = 0; q < C; ++q)
    for (int p = 0; p < C; ++p)
      for (int y = 1; y <= V; ++y)
        if (table[p * V + y - 1] == q) { g->src[a] = p; g->dst[a] = q; g->wix[a] = p * R + y; ++a; }
  g->A = a;
  graph_finish(g);
}

/* lattices.py:314-338 / contexts.py:109-146: context state of each string
 * position and the weight of its lexical arc (label 0 -> 1, pad 1) */
static void string_graph(int C, int V, const int* table, int U, const int* labels, graph_t* g) {
  const int R = V + 1, NP = U + 1;
  (void)C;
  g->S = NP;
  g->A = U;
  g->blank = (int*)malloc(sizeof(int) * NP);
  g->src = (int*)malloc(sizeof(int) * (U > 0 ? U : 1));
  g->dst = (int*)malloc(sizeof(int) * (U > 0 ? U : 1));
  g->wix = (int*)malloc(sizeof(int) * (U > 0 ? U : 1));
  int c = 0;
  for (int u = 0; u < NP; ++u) {
    g->blank[u] = c * R;
    if (u < U) {
      int y = labels[u];
      if (y < 0 || y > V) y = 0;
      g->src[u] = u; g->dst[u] = u + 1; g->wix[u] = c * R + (y < 1 ? 1 : y);
      if (y != 0) c = table[c * V + y - 1];
    }
  }
  graph_finish(g);
}

static double lse(const double* x, int n) { /* semirings.py:279-286 */
  double m = kNegInf;
  for (int i = 0; i < n; ++i) m = x[i] > m ? x[i] : m;
  if (!isfinite(m)) m = 0.0;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += exp(x[i] - m);
  return m + log(s);
}
static double lae(double a, double b) { double x[2] = {a, b}; return lse(x, 2); }

/* One frame in double (Log / Real): in -> out over graph g, weights w. */
static void frame_d(const graph_t* g, int K, int sr, const float* w, const double* in, double* out,
                    double* last, double* nxt, double* terms, double* tmp) {
  const int S = g->S;
  const int real = sr == TAB_REAL;
  if (K == 0) { /* FrameDependent: (a (x) blank) (+) reduce(a (x) lex) */
    for (int q = 0; q < S; ++q) {
      const double bt = real ? in[q] * w[g->blank[q]] : in[q] + w[g->blank[q]];
      int n = 0;
      double r = real ? 0.0 : kNegInf;
      for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a) {
        const double x = real ? in[g->src[a]] * w[g->wix[a]] : in[g->src[a]] + w[g->wix[a]];
        if (real) r += x; else tmp[n++] = x;
      }
      if (!real) r = lse(tmp, n);
      out[q] = real ? bt + r : lae(bt, r);
    }
    return;
  }
  /* FrameLabelDependent(K): terms_i = (L^i a) (x) blank, summed over i */
  memcpy(last, in, sizeof(double) * S);
  for (int q = 0; q < S; ++q)
    terms[q] = real ? in[q] * w[g->blank[q]] : in[q] + w[g->blank[q]];
  for (int i = 1; i <= K; ++i) {
    for (int q = 0; q < S; ++q) {
      int n = 0;
      double r = real ? 0.0 : kNegInf;
      for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a) {
        const double x = real ? last[g->src[a]] * w[g->wix[a]] : last[g->src[a]] + w[g->wix[a]];
        if (real) r += x; else tmp[n++] = x;
      }
      nxt[q] = real ? r : lse(tmp, n);
    }
    memcpy(last, nxt, sizeof(double) * S);
    for (int q = 0; q < S; ++q)
      terms[(long long)i * S + q] = real ? last[q] * w[g->blank[q]] : last[q] + w[g->blank[q]];
  }
  for (int q = 0; q < S; ++q) {
    if (real) {
      double r = 0.0;
      for (int i = 0; i <= K; ++i) r += terms[(long long)i * S + q];
      out[q] = r;
    } else {
      for (int i = 0; i <= K; ++i) tmp[i] = terms[(long long)i * S + q];
      out[q] = lse(tmp, K + 1);
    }
  }
}

/* One MaxTropical frame in float with the reference's tie rules; records
 * the winning term (win[q], FLD) / blank-or-arc (FD: arg[q] = -1 blank) and
 * per expansion the winning in-arc (argk[i-1][q]). */
static void frame_max(const graph_t* g, int K, const float* w, const float* in, float* out,
                      float* last, float* nxt, float* terms, int* win, int* argk) {
  const int S = g->S;
  if (K == 0) {
    for (int q = 0; q < S; ++q) {
      const float bt = in[q] + w[g->blank[q]];
      float r = -INFINITY;
      int ra = -1;
      for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a) {
        const float x = in[g->src[a]] + w[g->wix[a]];
        if (ra < 0 || x > r) { r = x; ra = a; } /* first argmax */
      }
      const int blank_wins = !(ra >= 0) || bt >= r; /* Maximum: a >= b keeps a */
      out[q] = blank_wins ? bt : r;
      if (argk) argk[q] = blank_wins ? -1 : ra;
    }
    return;
  }
  memcpy(last, in, sizeof(float) * S);
  for (int q = 0; q < S; ++q) terms[q] = in[q] + w[g->blank[q]];
  for (int i = 1; i <= K; ++i) {
    for (int q = 0; q < S; ++q) {
      float r = -INFINITY;
      int ra = -1;
      for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a) {
        const float x = last[g->src[a]] + w[g->wix[a]];
        if (ra < 0 || x > r) { r = x; ra = a; }
      }
      nxt[q] = r;
      if (argk) argk[(long long)(i - 1) * S + q] = ra;
    }
    memcpy(last, nxt, sizeof(float) * S);
    for (int q = 0; q < S; ++q) terms[(long long)i * S + q] = last[q] + w[g->blank[q]];
  }
  for (int q = 0; q < S; ++q) {
    float m = terms[q];
    int mi = 0;
    for (int i = 1; i <= K; ++i)
      if (terms[(long long)i * S + q] > m) { m = terms[(long long)i * S + q]; mi = i; }
    out[q] = m;
    if (win) win[q] = mi;
  }
}

/* forward over T frames; alpha_hist [T+1][S] double (Log/Real) */
static double forward_d(const graph_t* g, int K, int sr, int T, long long FR, const float* W,
                        int nf, int start, double* hist, float* alpha_out, int final_state) {
  const int S = g->S;
  double* a = (double*)malloc(sizeof(double) * S);
  double* na = (double*)malloc(sizeof(double) * S);
  double* last = (double*)malloc(sizeof(double) * S);
  double* nxt = (double*)malloc(sizeof(double) * S);
  double* terms = (double*)malloc(sizeof(double) * (size_t)(K + 1) * S);
  int maxin = K + 1;
  for (int q = 0; q < S; ++q)
    if (g->in_off[q + 1] - g->in_off[q] > maxin) maxin = g->in_off[q + 1] - g->in_off[q];
  double* tmp = (double*)malloc(sizeof(double) * (maxin + 2));
  const int real = sr == TAB_REAL;
  for (int q = 0; q < S; ++q) a[q] = q == start ? (real ? 1.0 : 0.0) : (real ? 0.0 : kNegInf);
  for (int t = 0; t < T; ++t) {
    if (hist) memcpy(hist + (long long)t * S, a, sizeof(double) * S);
    if (alpha_out) for (int q = 0; q < S; ++q) alpha_out[(long long)t * S + q] = (float)a[q];
    if (t >= nf) continue;
    frame_d(g, K, sr, W + (long long)t * FR, a, na, last, nxt, terms, tmp);
    memcpy(a, na, sizeof(double) * S);
  }
  if (hist) memcpy(hist + (long long)T * S, a, sizeof(double) * S);
  double r;
  if (final_state >= 0) {
    r = final_state < S ? a[final_state] : (real ? 0.0 : kNegInf);
  } else if (real) {
    r = 0.0;
    for (int q = 0; q < S; ++q) r += a[q];
  } else {
    r = lse(a, S);
  }
  free(a); free(na); free(last); free(nxt); free(terms); free(tmp);
  return r;
}

/* ------------------------------------------------------------------------ */

/* dist[B] (+ alpha [B,T,C] nullable): RecognitionLattice._forward */
void tab_den_forward(int B, int T, int C, int V, int K, const int* table, const float* W,
                     const int* nf, int sr, float* dist, float* alpha) {
  graph_t g;
  context_graph(C, V, table, &g);
  const long long FR = (long long)C * (V + 1);
  float* a = (float*)malloc(sizeof(float) * C);
  float* na = (float*)malloc(sizeof(float) * C);
  float* last = (float*)malloc(sizeof(float) * C);
  float* nxt = (float*)malloc(sizeof(float) * C);
  float* terms = (float*)malloc(sizeof(float) * (size_t)(K + 1) * C);
  for (int b = 0; b < B; ++b) {
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    float* ab = alpha ? alpha + (long long)b * T * C : NULL;
    if (sr == TAB_MAX) {
      for (int q = 0; q < C; ++q) a[q] = q == 0 ? 0.f : -INFINITY;
      for (int t = 0; t < T; ++t) {
        if (ab) memcpy(ab + (long long)t * C, a, sizeof(float) * C);
        if (t >= nfb) continue;
        frame_max(&g, K, Wb + (long long)t * FR, a, na, last, nxt, terms, NULL, NULL);
        memcpy(a, na, sizeof(float) * C);
      }
      float m = a[0];
      for (int q = 1; q < C; ++q) m = a[q] > m ? a[q] : m;
      dist[b] = m;
    } else {
      dist[b] = (float)forward_d(&g, K, sr, T, FR, Wb, nfb, 0, NULL, ab, -1);
    }
  }
  free(a); free(na); free(last); free(nxt); free(terms);
  graph_free(&g);
}

/* num[B]: RecognitionLattice._string_forward */
void tab_num_forward(int B, int T, int U, int C, int V, int K, const int* table, const float* W,
                     const int* nf, const int* labels, const int* nl, int sr, float* num) {
  const long long FR = (long long)C * (V + 1);
  const int NP = U + 1;
  float* a = (float*)malloc(sizeof(float) * NP);
  float* na = (float*)malloc(sizeof(float) * NP);
  float* last = (float*)malloc(sizeof(float) * NP);
  float* nxt = (float*)malloc(sizeof(float) * NP);
  float* terms = (float*)malloc(sizeof(float) * (size_t)(K + 1) * NP);
  for (int b = 0; b < B; ++b) {
    graph_t g;
    string_graph(C, V, table, U, labels + (long long)b * U, &g);
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    const int fin = (nl[b] >= 0 && nl[b] <= U) ? nl[b] : NP;
    if (sr == TAB_MAX) {
      for (int u = 0; u < NP; ++u) a[u] = u == 0 ? 0.f : -INFINITY;
      for (int t = 0; t < nfb; ++t) {
        frame_max(&g, K, Wb + (long long)t * FR, a, na, last, nxt, terms, NULL, NULL);
        memcpy(a, na, sizeof(float) * NP);
      }
      num[b] = fin < NP ? a[fin] : -INFINITY;
    } else {
      num[b] = (float)forward_d(&g, K, sr, T, FR, Wb, nfb, 0, NULL, NULL, fin);
    }
    graph_free(&g);
  }
  free(a); free(na); free(last); free(nxt); free(terms);
}

/* Log-semiring backward of one utterance over graph g: marginals added to
 * acc (scaled by scale), alpha history ah [T+1][S] from forward_d, final
 * beta = 0 on `fin` (or all states when fin < 0). */
static void backward_d(const graph_t* g, int K, long long FR, const float* W, int nf,
                       const double* ah, double lz, int fin, double scale, double* acc) {
  const int S = g->S;
  double* beta = (double*)malloc(sizeof(double) * S);
  double* nb = (double*)malloc(sizeof(double) * S);
  double* la = (double*)malloc(sizeof(double) * (size_t)(K + 1) * S);
  double* lb = (double*)malloc(sizeof(double) * (g->A > 0 ? g->A : 1));
  int maxin = 2;
  for (int q = 0; q < S; ++q) {
    if (g->in_off[q + 1] - g->in_off[q] > maxin) maxin = g->in_off[q + 1] - g->in_off[q];
    if (g->out_off[q + 1] - g->out_off[q] > maxin) maxin = g->out_off[q + 1] - g->out_off[q];
  }
  double* tmp = (double*)malloc(sizeof(double) * (maxin + 2));
  for (int q = 0; q < S; ++q) beta[q] = (fin < 0 || q == fin) ? 0.0 : kNegInf;
  for (int t = nf - 1; t >= 0; --t) {
    const float* w = W + (long long)t * FR;
    const double* al = ah + (long long)t * S;
    double* dw = acc + (long long)t * FR;
    if (K == 0) { /* FrameDependent.backward, alignments.py:300-318 */
      for (int p = 0; p < S; ++p) {
        const double bb = w[g->blank[p]] + beta[p];
        dw[g->blank[p]] += scale * exp(al[p] + bb - lz);
        int n = 0;
        for (int o = g->out_off[p]; o < g->out_off[p + 1]; ++o) {
          const int a = g->out_arc[o];
          const double x = w[g->wix[a]] + beta[g->dst[a]];
          tmp[n++] = x;
          dw[g->wix[a]] += scale * exp(al[p] + x - lz);
        }
        nb[p] = lae(bb, lse(tmp, n));
      }
    } else { /* FrameLabelDependent.backward, alignments.py:379-419 */
      memcpy(la, al, sizeof(double) * S);
      for (int i = 1; i <= K; ++i)
        for (int q = 0; q < S; ++q) {
          int n = 0;
          for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a)
            tmp[n++] = la[(long long)(i - 1) * S + g->src[a]] + w[g->wix[a]];
          la[(long long)i * S + q] = lse(tmp, n);
        }
      for (int i = 0; i <= K; ++i)
        for (int p = 0; p < S; ++p)
          dw[g->blank[p]] += scale * exp(la[(long long)i * S + p] + w[g->blank[p]] + beta[p] - lz);
      for (int p = 0; p < S; ++p) nb[p] = w[g->blank[p]] + beta[p];
      for (int j = K - 1; j >= 0; --j) {
        for (int a = 0; a < g->A; ++a) lb[a] = w[g->wix[a]] + nb[g->dst[a]];
        for (int a = 0; a < g->A; ++a)
          dw[g->wix[a]] += scale * exp(lb[a] + la[(long long)j * S + g->src[a]] - lz);
        for (int p = 0; p < S; ++p) {
          int n = 0;
          for (int o = g->out_off[p]; o < g->out_off[p + 1]; ++o) tmp[n++] = lb[g->out_arc[o]];
          nb[p] = lae(w[g->blank[p]] + beta[p], lse(tmp, n));
        }
      }
    }
    memcpy(beta, nb, sizeof(double) * S);
  }
  free(beta); free(nb); free(la); free(lb); free(tmp);
}

/* RecognitionLattice.forward loss and d(sum_b grad[b] loss_b)/dW; local_norm:
 * loss = -num. Unreachable strings (num = -inf) get dW = 0. */
void tab_loss_grad(int B, int T, int U, int C, int V, int K, const int* table, const float* W,
                   const int* nf, const int* labels, const int* nl, int local_norm,
                   const float* grad, float* loss, float* log_z, float* num, float* dW) {
  graph_t gd;
  context_graph(C, V, table, &gd);
  const long long FR = (long long)C * (V + 1);
  const int NP = U + 1;
  double* hd = (double*)malloc(sizeof(double) * (size_t)(T + 1) * C);
  double* hn = (double*)malloc(sizeof(double) * (size_t)(T + 1) * NP);
  double* acc = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1) * FR);
  for (int b = 0; b < B; ++b) {
    graph_t gs;
    string_graph(C, V, table, U, labels + (long long)b * U, &gs);
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    const int fin = (nl[b] >= 0 && nl[b] <= U) ? nl[b] : NP;
    const double nv = forward_d(&gs, K, TAB_LOG, T, FR, Wb, nfb, 0, hn, NULL, fin);
    double lz = 0.0;
    if (!local_norm) lz = forward_d(&gd, K, TAB_LOG, T, FR, Wb, nfb, 0, hd, NULL, -1);
    const double gb = grad ? grad[b] : 1.0;
    memset(acc, 0, sizeof(double) * (size_t)T * FR);
    if (dW && isfinite(nv) && (local_norm || isfinite(lz))) {
      if (!local_norm) backward_d(&gd, K, FR, Wb, nfb, hd, lz, -1, gb, acc);
      backward_d(&gs, K, FR, Wb, nfb, hn, nv, fin, -gb, acc);
    }
    if (dW)
      for (long long e = 0; e < (long long)T * FR; ++e) dW[(long long)b * T * FR + e] = (float)acc[e];
    if (log_z) log_z[b] = (float)lz;
    if (num) num[b] = (float)nv;
    loss[b] = (float)(local_norm ? -nv : lz - nv);
    graph_free(&gs);
  }
  free(hd); free(hn); free(acc);
  graph_free(&gd);
}

/* d log_z / dW alone (the denominator's arc marginals; the gradient of
 * _forward's Log distance, lattices.py:379-496, and the marginals _backward
 * streams, lattices.py:686-799): backward_d over the context graph, as in
 * tab_loss_grad without the string. Utterances whose log_z is not finite
 * get zeros. */
void tab_den_grad(int B, int T, int C, int V, int K, const int* table, const float* W,
                  const int* nf, float* log_z, float* dW) {
  graph_t gd;
  context_graph(C, V, table, &gd);
  const long long FR = (long long)C * (V + 1);
  double* hd = (double*)malloc(sizeof(double) * (size_t)(T + 1) * C);
  double* acc = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1) * FR);
  for (int b = 0; b < B; ++b) {
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    const double lz = forward_d(&gd, K, TAB_LOG, T, FR, Wb, nfb, 0, hd, NULL, -1);
    memset(acc, 0, sizeof(double) * (size_t)T * FR);
    if (isfinite(lz)) backward_d(&gd, K, FR, Wb, nfb, hd, lz, -1, 1.0, acc);
    for (long long e = 0; e < (long long)T * FR; ++e) dW[(long long)b * T * FR + e] = (float)acc[e];
    if (log_z) log_z[b] = (float)lz;
  }
  free(hd); free(acc);
  graph_free(&gd);
}

/* RecognitionLattice.shortest_path per utterance (no D6 aliasing):
 * labels [B, T*A] (A = 1 for FrameDependent, K+1 for FrameLabelDependent):
 * slot i of frame t holds the label of the (i+1)-th lexical arc taken in
 * frame t (conv 1: y-1 as the reference's argmax, D5; conv 0: y), else 0;
 * weight [B] = the MaxTropical distance. */
void tab_viterbi(int B, int T, int C, int V, int K, const int* table, const float* W,
                 const int* nf, int conv, long long* labels, float* weight) {
  graph_t g;
  context_graph(C, V, table, &g);
  const long long FR = (long long)C * (V + 1);
  const int A = K == 0 ? 1 : K + 1, R = V + 1;
  const int KK = K == 0 ? 1 : K;
  float* a = (float*)malloc(sizeof(float) * C);
  float* na = (float*)malloc(sizeof(float) * C);
  float* last = (float*)malloc(sizeof(float) * C);
  float* nxt = (float*)malloc(sizeof(float) * C);
  float* terms = (float*)malloc(sizeof(float) * (size_t)(K + 1) * C);
  int* win = (int*)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1) * C);
  int* argk = (int*)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1) * KK * C);
  for (int b = 0; b < B; ++b) {
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    long long* lb = labels + (long long)b * T * A;
    for (long long i = 0; i < (long long)T * A; ++i) lb[i] = 0;
    for (int q = 0; q < C; ++q) a[q] = q == 0 ? 0.f : -INFINITY;
    for (int t = 0; t < nfb; ++t) {
      frame_max(&g, K, Wb + (long long)t * FR, a, na, last, nxt, terms, win + (long long)t * C,
                argk + (long long)t * KK * C);
      memcpy(a, na, sizeof(float) * C);
    }
    int q = 0;
    float m = a[0];
    for (int s = 1; s < C; ++s) if (a[s] > m) { m = a[s]; q = s; }
    weight[b] = m;
    for (int t = nfb - 1; t >= 0; --t) {
      const int* ak = argk + (long long)t * KK * C;
      if (K == 0) {
        const int arc = ak[q];
        if (arc >= 0) {
          const int y = g.wix[arc] % R;
          lb[(long long)t * A] = conv ? y - 1 : y;
          q = g.src[arc];
        }
      } else {
        const int i = win[(long long)t * C + q];
        for (int j = i; j >= 1; --j) {
          const int arc = ak[(long long)(j - 1) * C + q];
          const int y = g.wix[arc] % R;
          lb[(long long)t * A + j - 1] = conv ? y - 1 : y;
          q = g.src[arc];
        }
      }
    }
  }
  free(a); free(na); free(last); free(nxt); free(terms); free(win); free(argk);
  graph_free(&g);
}

/* MaxTropical gradient of one utterance over graph g: the reference
 * differentiates its MaxTropical distance through Maximum (a >= b keeps a,
 * semirings.py:354-371) and Max (first argmax, :373-401), so the gradient is
 * `scale` on every arc of the first-maximum path (an arc used twice in a
 * frame gets it twice). fin < 0: the distance is the Max over all states
 * (lattices.py:482-496); fin >= 0: the Max over where(is_final, alpha, -inf)
 * (lattices.py:375-377), whose argmax is fin while alpha_T[fin] > -inf and
 * position 0 otherwise -- the gradient then reaches alpha only if fin == 0.
 * Padding frames carry alpha (lattices.py:357-358, 460-461): no arcs. */
static void grad_max(const graph_t* g, int K, long long FR, const float* W, int nf, int fin,
                     double scale, double* acc, float* dist) {
  const int S = g->S, KK = K == 0 ? 1 : K;
  float* a = (float*)malloc(sizeof(float) * S);
  float* na = (float*)malloc(sizeof(float) * S);
  float* last = (float*)malloc(sizeof(float) * S);
  float* nxt = (float*)malloc(sizeof(float) * S);
  float* terms = (float*)malloc(sizeof(float) * (size_t)(K + 1) * S);
  int* win = (int*)malloc(sizeof(int) * (size_t)(nf > 0 ? nf : 1) * S);
  int* argk = (int*)malloc(sizeof(int) * (size_t)(nf > 0 ? nf : 1) * KK * S);
  for (int q = 0; q < S; ++q) a[q] = q == 0 ? 0.f : -INFINITY;
  for (int t = 0; t < nf; ++t) {
    frame_max(g, K, W + (long long)t * FR, a, na, last, nxt, terms, win + (long long)t * S,
              argk + (long long)t * KK * S);
    memcpy(a, na, sizeof(float) * S);
  }
  int q = -1;
  if (fin < 0) {
    q = 0;
    for (int s = 1; s < S; ++s) if (a[s] > a[q]) q = s;
    *dist = a[q];
  } else {
    *dist = fin < S ? a[fin] : -INFINITY;
    if (fin < S) q = a[fin] > -INFINITY ? fin : (fin == 0 ? 0 : -1);
  }
  for (int t = nf - 1; t >= 0 && q >= 0; --t) {
    double* dw = acc + (long long)t * FR;
    const int* ak = argk + (long long)t * KK * S;
    if (K == 0) {
      const int arc = ak[q];
      if (arc < 0) {
        dw[g->blank[q]] += scale;
      } else {
        dw[g->wix[arc]] += scale;
        q = g->src[arc];
      }
    } else {
      dw[g->blank[q]] += scale;  /* the terminating blank of the winning term */
      for (int j = win[(long long)t * S + q]; j >= 1; --j) {
        const int arc = ak[(long long)(j - 1) * S + q];
        dw[g->wix[arc]] += scale;
        q = g->src[arc];
      }
    }
  }
  free(a); free(na); free(last); free(nxt); free(terms); free(win); free(argk);
}

/* Real-semiring gradient of one utterance over graph g (the reference's
 * Real autograd is plain arithmetic, semirings.py:143-173): d dist / dW by
 * reverse accumulation in double through each frame's recursion --
 *   FrameDependent  a'[q] = a[q] w_b[q] + sum_{p->q} a[p] w          (alignments.py:320-329, 286-297)
 *   FrameLabelDependent  L_0 = a, L_i[q] = sum_{p->q} L_{i-1}[p] w,
 *                   a'[q] = w_b[q] sum_i L_i[q]                      (alignments.py:362-377, 420-432)
 * fin < 0: dist = sum_q a_T[q]; fin >= 0: a_T[fin] (0 when fin >= S). */
static void grad_real(const graph_t* g, int K, int T, long long FR, const float* W, int nf, int fin,
                      double scale, double* acc, float* dist) {
  const int S = g->S;
  double* ah = (double*)malloc(sizeof(double) * (size_t)(T + 1) * S);
  *dist = (float)forward_d(g, K, TAB_REAL, T, FR, W, nf, 0, ah, NULL, fin);
  double* beta = (double*)malloc(sizeof(double) * S);
  double* nb = (double*)malloc(sizeof(double) * S);
  double* la = (double*)malloc(sizeof(double) * (size_t)(K + 1) * S);
  double* dl = (double*)malloc(sizeof(double) * S);
  double* dn = (double*)malloc(sizeof(double) * S);
  for (int q = 0; q < S; ++q) beta[q] = (fin < 0 || q == fin) ? scale : 0.0;
  for (int t = nf - 1; t >= 0; --t) {
    const float* w = W + (long long)t * FR;
    const double* al = ah + (long long)t * S;
    double* dw = acc + (long long)t * FR;
    if (K == 0) {
      for (int p = 0; p < S; ++p) {
        dw[g->blank[p]] += al[p] * beta[p];
        double r = w[g->blank[p]] * beta[p];
        for (int o = g->out_off[p]; o < g->out_off[p + 1]; ++o) {
          const int a = g->out_arc[o];
          dw[g->wix[a]] += al[p] * beta[g->dst[a]];
          r += w[g->wix[a]] * beta[g->dst[a]];
        }
        nb[p] = r;
      }
    } else {
      memcpy(la, al, sizeof(double) * S);
      for (int i = 1; i <= K; ++i)
        for (int q = 0; q < S; ++q) {
          double r = 0.0;
          for (int a = g->in_off[q]; a < g->in_off[q + 1]; ++a)
            r += la[(long long)(i - 1) * S + g->src[a]] * w[g->wix[a]];
          la[(long long)i * S + q] = r;
        }
      for (int q = 0; q < S; ++q) {
        double s = 0.0;
        for (int i = 0; i <= K; ++i) s += la[(long long)i * S + q];
        dw[g->blank[q]] += beta[q] * s;
        dl[q] = beta[q] * w[g->blank[q]];  /* dL_K */
      }
      for (int i = K - 1; i >= 0; --i) {
        for (int p = 0; p < S; ++p) {
          double r = beta[p] * w[g->blank[p]];
          for (int o = g->out_off[p]; o < g->out_off[p + 1]; ++o) {
            const int a = g->out_arc[o];
            dw[g->wix[a]] += la[(long long)i * S + p] * dl[g->dst[a]];
            r += w[g->wix[a]] * dl[g->dst[a]];
          }
          dn[p] = r;
        }
        memcpy(dl, dn, sizeof(double) * S);
      }
      memcpy(nb, dl, sizeof(double) * S);
    }
    memcpy(beta, nb, sizeof(double) * S);
  }
  free(ah); free(beta); free(nb); free(la); free(dl); free(dn);
}

/* The gradient of the distance under semiring sr, per utterance scaled by
 * grad[b] (nullable: 1): string = 0 the denominator (_forward over the
 * context graph, lattices.py:379-496), string = 1 the numerator
 * (_string_forward over the string acceptor, lattices.py:250-377). dist [B]
 * gets the distance. Log: the marginals (backward_d), zero for a non-finite
 * distance; MaxTropical: grad_max; Real: grad_real. */
void tab_dist_grad(int B, int T, int U, int C, int V, int K, const int* table, const float* W,
                   const int* nf, const int* labels, const int* nl, int sr, int string,
                   const float* grad, float* dist, float* dW) {
  graph_t gd;
  context_graph(C, V, table, &gd);
  const long long FR = (long long)C * (V + 1);
  const int NP = U + 1;
  const int SM = C > NP ? C : NP;
  double* hist = (double*)malloc(sizeof(double) * (size_t)(T + 1) * SM);
  double* acc = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1) * FR);
  for (int b = 0; b < B; ++b) {
    graph_t gs;
    if (string) string_graph(C, V, table, U, labels + (long long)b * U, &gs);
    const graph_t* g = string ? &gs : &gd;
    const int nfb = nf[b] < 0 ? 0 : (nf[b] > T ? T : nf[b]);
    const float* Wb = W + (long long)b * T * FR;
    const int fin = string ? ((nl[b] >= 0 && nl[b] <= U) ? nl[b] : NP) : -1;
    const double gb = grad ? grad[b] : 1.0;
    memset(acc, 0, sizeof(double) * (size_t)T * FR);
    if (sr == TAB_MAX) {
      grad_max(g, K, FR, Wb, nfb, fin, gb, acc, dist + b);
    } else if (sr == TAB_REAL) {
      grad_real(g, K, T, FR, Wb, nfb, fin, gb, acc, dist + b);
    } else {
      const double d = forward_d(g, K, TAB_LOG, T, FR, Wb, nfb, 0, hist, NULL, fin);
      dist[b] = (float)d;
      if (isfinite(d)) backward_d(g, K, FR, Wb, nfb, hist, d, fin, gb, acc);
    }
    for (long long e = 0; e < (long long)T * FR; ++e) dW[(long long)b * T * FR + e] = (float)acc[e];
    if (string) graph_free(&gs);
  }
  free(hist); free(acc);
  graph_free(&gd);
}
