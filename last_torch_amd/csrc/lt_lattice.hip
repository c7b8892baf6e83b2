// lt_lattice.hip -- host side of the MI355X lattice library: C ABI
// (include/lt_lattice.h), launch planning, and the small scatter / Viterbi
// backtrace kernels. The frame-recursion kernels live in lt_kernels.h and
// are instantiated per terms-per-lane value by lt_inst.hip.
#include "lt_kernels.h"

namespace {
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

// Frame-indexed buffers ([B, T, ...]) may be null when T == 0 (an empty
// tensor has no storage); the kernels never touch them then.
#define LT_NEED(p) (!(p) && pb->max_frames > 0)

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

using lt_impl::Plan;

// Choose lanes-per-group, wave roles, LDS carve and ring depth.
//   kind 0: forward, kind 1: backward
int plan(const lt_problem* pb, const NGram& g, int kind, int flags, Plan* pl) {
  KArgs& a = pl->a;
  memset(&a, 0, sizeof(a));
  a.B = pb->batch; a.T = pb->max_frames; a.U = pb->max_labels; a.g = g;
  a.flags = flags;
  a.dbg = env_int("LT_DBG", 0);
#ifdef LT_STAMPS
  {
    const char* sp = getenv("LT_STAMPS_PTR");
    a.stamps = sp ? (long long*)strtoull(sp, nullptr, 0) : nullptr;
  }
#endif
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const int es = bf16 ? 2 : 4;
  const int C = g.C, NP = a.U + 1;
  a.FR = C * (g.V + 1);
  const long long FRB = (long long)a.FR * es;
  const bool do_den = flags & F_DEN, do_num = flags & F_NUM;

  a.aux_waves = do_num ? std::min(ceil_div(NP, 64), 4) : 0;
  if (kind == 1 && do_num) a.aux_waves = std::max(a.aux_waves, env_int("LT_BWD_AUX", 0));
  a.load_waves = 2;
  if (!do_den && a.aux_waves == 0) a.aux_waves = 1;
  const int max_den = kMaxWaves - a.aux_waves - a.load_waves;

  // Denominator groups. Forward: one group per destination with lexical
  // in-arcs; for n >= 1 the start state (blank self loop only) is done on
  // the side by den lane 0 (extra0). Backward: one group per source state.
  int nterm;
  if (kind == 0) {
    nterm = g.K + 1;
    if (g.n >= 1) { a.den_groups = C - 1; a.den_q0 = 1; a.extra0 = 1; }
    else { a.den_groups = 1; a.den_q0 = 0; a.extra0 = 0; }
  } else {
    nterm = g.V + 1;
    a.den_groups = C; a.den_q0 = 0; a.extra0 = 0;
  }
  int L = 1;
  while (L < 64 && ceil_div(nterm, L) > 16) L *= 2;
  const int den_cap = std::min(max_den, env_int("LT_MAX_DEN_WAVES", kind == 1 ? 5 : 4));
  while (L < 16 && ceil_div(nterm, 2 * L) >= 3 &&
         (long long)a.den_groups * 2 * L <= 64LL * den_cap)
    L *= 2;
  const int envL = env_int("LT_DEN_LANES", 0);
  if (envL > 0 && (envL & (envL - 1)) == 0 && envL <= 64 && ceil_div(nterm, envL) <= 16) L = envL;
  a.L = L;
  a.lgL = 0;
  while ((1 << a.lgL) < L) ++a.lgL;
  a.Pr = ceil_div(nterm, L);
  // compiled (LG, P) variants: exact pairs, else runtime-LG with P >= Pr
  static const int kFixed[][2] = {{3, 5}, {2, 9}, {1, 4}, {1, 3}, {2, 5}, {3, 3}, {2, 3}};
  pl->lg = -1;
  pl->tmax = a.Pr <= 4 ? 4 : (a.Pr <= 8 ? 8 : 16);
  for (const auto& v : kFixed)
    if (v[0] == a.lgL && v[1] == a.Pr) { pl->lg = v[0]; pl->tmax = v[1]; }

  // backward: the den lanes also store dW, so they exist without a denominator
  const bool den_role = do_den || kind == 1;
  int den = den_role ? ceil_div((long long)a.den_groups * L, 64) : 0;
  den = std::min(den, max_den);
  if (den_role && den < 1) den = 1;
  a.den_waves = den;
  a.den_fast = (den * 64 / L) >= a.den_groups;

  // LDS carve (bytes, 16-aligned pieces)
  auto al16 = [](long long x) { return (int)((x + 15) & ~15LL); };
  int off = 0;
  a.off_misc = off; off += 64;
  a.off_a = off; off += al16(2LL * C * 4);
  a.off_na = off; off += al16(2LL * NP * 4);
  a.off_ctx = off; off += al16((long long)NP * 4);
  a.off_ylab = off; off += al16((long long)NP * 4);
  int fixed = off;

  // staged numerator marginals (backward): 3 frames of FR floats
  pl->dst = false;
  if (kind == 1) {
    const long long need = do_num ? 3LL * a.FR * 4 : 0;
    const int ring_min = 4 * 1024 * 4;  // leave room for a few ring slots
    if (fixed + need + ring_min <= kLdsMax && env_int("LT_FORCE_DIRECT", 0) == 0) {
      pl->dst = true;
      a.off_nbuf = fixed;
      a.off_dbuf = fixed;
      fixed += al16(need);
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
  if (env_int("LT_VERBOSE", 0))
    fprintf(stderr,
            "[lt] kind=%d C=%d V=%d L=%d Pr=%d P=%d lg=%d den=%d aux=%d load=%d groups=%d fast=%d "
            "S=%d slot=%d lds=%d dst=%d wst=%d\n",
            kind, C, g.V, a.L, a.Pr, pl->tmax, pl->lg, a.den_waves, a.aux_waves, a.load_waves,
            a.den_groups, a.den_fast, a.S, a.slot_bytes, pl->lds_bytes, (int)pl->dst,
            (int)pl->wst);
  return LT_OK;
}

constexpr int M1 = -1;
int launch_fwd(int mode, const Plan& pl, bool bf16, int grid, hipStream_t st) {
#define LT_CASE(LG, P) \
  if (pl.lg == LG && pl.tmax == P) return lt_impl::launch_fwd_##LG##_##P(mode, pl, bf16, grid, st);
  LT_VARIANTS(LT_CASE)
#undef LT_CASE
  return fail(LT_EINVAL, "no kernel variant for this slice size");
}

int launch_bwd(const Plan& pl, bool bf16, int grid, hipStream_t st) {
#define LT_CASE(LG, P) \
  if (pl.lg == LG && pl.tmax == P) return lt_impl::launch_bwd_##LG##_##P(pl, bf16, grid, st);
  LT_VARIANTS(LT_CASE)
#undef LT_CASE
  return fail(LT_EINVAL, "no kernel variant for this slice size");
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

namespace lt_impl {
int set_error(int code, const char* msg) { return fail(code, msg); }
}  // namespace lt_impl

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
  if (LT_NEED(W) || !num_frames || !dist) return fail(LT_EINVAL, "null pointer");
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
  if (LT_NEED(W) || !num_frames || !num_labels || !num || (pb->max_labels > 0 && !labels))
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
  if (LT_NEED(W) || !num_frames || !num_labels || !loss || (pb->max_labels > 0 && !labels))
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
  if (LT_NEED(W) || !num_frames || !log_z || LT_NEED(alpha) || LT_NEED(dW))
    return fail(LT_EINVAL, "null pointer");
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
  if (LT_NEED(W) || !num_frames || !num_labels || !num || LT_NEED(alpha_num) || LT_NEED(dW) ||
      (pb->max_labels > 0 && !labels) || (!local_norm && (!log_z || LT_NEED(alpha))))
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
  if (LT_NEED(W) || !num_frames || LT_NEED(labels) || !path_weight || !workspace)
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
