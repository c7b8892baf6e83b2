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
  if (a.only && !a.only[b]) return;
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
// Arc marginals from checkpoints (the checkpointing loss backward).
//   dW[b,t,p,y] = g_b * ( exp(alpha_t[p] + W[p,y] + beta_{t+1}[next(p,y)] - log_z)
//                         - sum of the numerator marginals on that arc )
// (alignments.py:311-317 for the denominator; the numerator arcs are the
// string arcs of lattices.py:314-338, Appendix A.4). Every (b,t) is
// independent, so this is one streaming pass over W -> dW with the grid
// spanning B x T: tiles of F whole frames (small frames) or one slice of a
// frame (large frames). Numerator entries that share an arc are summed by
// the chain head in ascending order (deterministic).
// ---------------------------------------------------------------------------
// The marginal pass's experimental numerator mode 2 and XCD grouping exist
// in diagnostic builds only: compiled into the product kernel they cost the
// trigram slices 2.8 % even when off (cfg5 4.00 against 3.89 ms,
// profiles/r05_marg_opts_ab.txt)
#ifdef LT_DIAG
#define LT_MARG_OPTS 1
#else
#define LT_MARG_OPTS 0
#endif

struct MgArgs {
  const unsigned char* W;
  const int* nfr;
  const float* alpha;      // [B,T,C]
  const float* beta;       // [B,T,C]   beta_{t+1} at frame t
  const float* alpha_num;  // [B,T,NP]
  const float* beta_num;   // [B,T,NP]  beta^n_{t+1} at frame t
  const int* arcs;         // [B,2*NK]  (offsets, links), NK = 2*NP
  const float* log_z;
  const float* num;
  const float* grad;
  void* dW;
  int B, T, U, FR, do_den, do_num;
  NGram g;
  int F;         // frames per tile (whole-frame tiles), 1 for slice tiles
  int tpf;       // slices per frame (1 = whole-frame tiles)
  int TS;        // elements per slice (tpf > 1)
  int tiles;     // tiles per utterance
  unsigned mR, mF, mNK;  // magic multipliers for / (V+1), / FR, / NK
  int off_a, off_b, off_an, off_bn, off_arc, off_sub, off_nb, lds_bytes;
  // how a tile subtracts the numerator marginals (do_num): 0 the chain heads
  // rewrite their elements after the tile's stores; 1 (whole-frame tiles) a
  // dense per-element buffer; 2 a bit per element marks the heads, whose sums
  // sit in a compact array by rank (the den pass subtracts before its store)
  int nmode;
  int off_hm, off_hp, off_hv;
  int xcd;       // frame slices: the tpf slices of a frame on one XCD (blocks 8 apart)
  // the trigram overlap (lt_tri.hip): frames its marginal workgroups did are
  // skipped; every frame normalised by the middle-frame norm (tri_mid_norm)
  const int* done;  // [B*T] nullable
  int mid_norm;
};

// n / d from the magic m = ceil(2^32 / d), corrected to exact.
LT_DEVINL unsigned fdiv(unsigned n, unsigned d, unsigned m) {
  unsigned q = __umulhi(n, m);
  if (q * d > n) --q;
  else if ((q + 1) * d <= n) ++q;
  return q;
}
inline unsigned magic_of(unsigned d) { return (unsigned)((0x100000000ULL + d - 1) / d); }

constexpr int kMgUnits = 5;  // 16-byte units of W per thread and tile

// One tile: F whole frames (small frames) or one slice of a frame.
//   phase 0: the tile's W as 16-B units into registers; alpha/beta (+num)
//            rows and the arc table into LDS (whole-frame tiles also zero a
//            per-element numerator buffer)
//   phase 1: den marginals in registers -> dW, 16-B stores from the tile's
//            first 16-byte boundary (head and tail element by element).
//            Whole-frame tiles (tpf == 1) subtract the numerator first: each
//            chain head (one per lattice element the string uses) sums its
//            arcs' marginals into the buffer (its W element from L2, the
//            tile was just streamed).
//   phase 2: frame slices (tpf > 1: trigram-size frames, where a buffer the
//            size of the slice would cap the workgroups per CU): once the
//            tile's own stores have completed, the chain heads rewrite their
//            elements as den - num.
// SLICED: frames cut in tpf > 1 slices, one per workgroup (compiled apart, so the whole-frame
// tiles keep their own register budget)
template <bool BF16, bool SLICED>
LT_DEVINL void marg_tile(const MgArgs& a, const int job, unsigned char* lds) {
  constexpr int VE = BF16 ? 8 : 4;  // elements per 16-byte unit
  constexpr int ES = BF16 ? 2 : 4;
  const int tile = job % a.tiles;
  const int b = job / a.tiles;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const NGram& g = a.g;
  const int C = g.C, R = g.V + 1, NP = a.U + 1, NK = 2 * NP, FR = a.FR;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  // whole-frame tiles: F frames; frame slices: slice tile % tpf of frame
  // tile / tpf (one workgroup per slice: a workgroup taking a frame's slices
  // in turn over one load of its rows measured 1.66 ms against 1.40 ms at
  // cfg5, fewer workgroups in flight)
  const int t0 = !SLICED ? tile * a.F : tile / a.tpf;
  const int s0 = !SLICED ? 0 : tile % a.tpf;
  const int Fh = !SLICED ? min(a.F, a.T - t0) : 1;
  float gb = a.grad ? a.grad[b] : 1.f;
  float lz = a.do_den ? a.log_z[b] : 0.f;
  float nm = a.do_num ? a.num[b] : 0.f;
  if constexpr (SLICED) {
    // the trigram overlap: a frame its marginal workgroups did is skipped;
    // the others take the same middle-frame norm they did
    if (a.done && a.done[(long long)b * a.T + t0]) return;
    if (a.mid_norm) {
      __shared__ float s_mid[2];
      int nf0 = a.nfr[b];
      nf0 = nf0 < 0 ? 0 : (nf0 > a.T ? a.T : nf0);
      if (nf0 >= 2) {
        if (threadIdx.x < 64) {
          const int mid = nf0 / 2, C0 = a.g.C, NP0 = a.U + 1;
          const long long r0 = (long long)b * a.T;
          const float2 zn = tri_mid_norm(a.alpha + (r0 + mid) * C0, a.beta + (r0 + mid - 1) * C0,
                                         a.alpha_num + (r0 + mid) * NP0,
                                         a.beta_num + (r0 + mid - 1) * NP0, C0, NP0,
                                         threadIdx.x, false);
          if (threadIdx.x == 0) {
            s_mid[0] = zn.x;
            s_mid[1] = zn.y;
          }
        }
        __syncthreads();
        lz = s_mid[0];
        nm = s_mid[1];
      }
    }
  }
  if ((a.do_num && !__builtin_isfinite(nm)) || (a.do_den && !__builtin_isfinite(lz))) gb = 0.f;
  const int Fl = max(0, min(Fh, nf - t0));  // live frames of the tile
  // slice sl: elements [e_lo, e_hi) of each of the tile's frames, contiguous
  // in HBM; 16-byte units from its first aligned element h0 (a trigram frame
  // is 2 mod 16 bytes long, so most slices start misaligned); the h0 head
  // elements and the tail go element by element
  struct Slice {
    int e_lo, Ew, E, h0, nunits, ntail;
    long long base;
  };
  auto slice = [&](int sl) {
    Slice x;
    x.e_lo = !SLICED ? 0 : sl * a.TS;
    const int e_hi = !SLICED ? FR : min(FR, x.e_lo + a.TS);
    x.Ew = e_hi - x.e_lo;
    x.E = Fh * x.Ew;
    x.base = ((long long)b * a.T + t0) * FR + x.e_lo;
    x.h0 = min(x.E, (int)(((16 - ((x.base * ES) & 15)) & 15) / ES));
    x.nunits = (x.E - x.h0) / VE;
    x.ntail = x.h0 + (x.E - x.h0 - x.nunits * VE);
    return x;
  };
  if (Fl == 0 || gb == 0.f) {  // padding (lattices.py:775-779) / unreachable
    const float z[VE] = {};
    {
      const Slice x = slice(s0);
      unsigned char* dWu = (unsigned char*)a.dW + (x.base + x.h0) * ES;
      for (int u = tid; u < x.nunits; u += nthr) store_unit<BF16>(dWu + (long long)u * 16, z);
      for (int i = tid; i < x.ntail; i += nthr)
        stw<BF16>(a.dW, x.base + (i < x.h0 ? i : i + x.nunits * VE), 0.f);
    }
    return;
  }
  float* A = (float*)(lds + a.off_a);     // [F][C]
  float* Bt = (float*)(lds + a.off_b);    // [F][C]
  float* AN = (float*)(lds + a.off_an);   // [F][NP]
  float* BN = (float*)(lds + a.off_bn);   // [F][NP]
  int* aoff = (int*)(lds + a.off_arc);    // [NK] offsets, then [NK] links
  int* alink = aoff + NK;
  int* nbt = (int*)(lds + a.off_nb);      // [C] next_base (n >= 2)
  float* Sub = (float*)(lds + a.off_sub); // nmode 1: [E] numerator marginals per element
  const bool dense = !SLICED && a.do_num && a.nmode == 1;
  const bool sparse = LT_MARG_OPTS && a.do_num && a.nmode == 2;
  unsigned* hm = (unsigned*)(lds + a.off_hm);  // nmode 2: a bit per tile element (chain heads)
  int* hp = (int*)(lds + a.off_hp);            // nmode 2: exclusive popcount prefix of hm
  float* hv = (float*)(lds + a.off_hv);        // nmode 2: the heads' numerator marginals by rank

  // ---- phase 0: the first slice's W as 16-B units into registers; alpha /
  // beta (+num) rows and the arc table into LDS, once for every slice
  // (whole-frame tiles also zero a per-element numerator buffer)
  uint4 wq[kMgUnits];
  auto load_units = [&](const Slice& x) {
    const unsigned char* Wu = a.W + (x.base + x.h0) * ES;
#pragma unroll
    for (int r = 0; r < kMgUnits; ++r) {
      const int u = tid + r * 256;
      if (u < x.nunits) wq[r] = *(const uint4*)(Wu + (long long)u * 16);
    }
  };
  const Slice x = slice(s0);
  load_units(x);
  const long long row0 = (long long)b * a.T + t0;
  // every row load in flight at once (a strided load -> LDS loop would wait
  // one memory latency per trip)
  constexpr int NR = 2;  // rounds per thread covered in registers; the rest loop
  const int nA = a.do_den ? Fl * C : 0, nN = a.do_num ? Fl * NP : 0, nK = a.do_num ? 2 * NK : 0;
  const int* arcsrc = a.arcs + (long long)b * 2 * NK;
  float ra[NR], rb[NR], rn[NR], rm[NR];
  int rk[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int e = tid + i * 256;
    if (e < nA) { ra[i] = a.alpha[row0 * C + e]; rb[i] = a.beta[row0 * C + e]; }
    if (e < nN) { rn[i] = a.alpha_num[row0 * NP + e]; rm[i] = a.beta_num[row0 * NP + e]; }
    if (e < nK) rk[i] = arcsrc[e];
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int e = tid + i * 256;
    if (e < nA) { A[e] = ra[i]; Bt[e] = rb[i]; }
    if (e < nN) { AN[e] = rn[i]; BN[e] = rm[i]; }
    if (e < nK) aoff[e] = rk[i];
  }
  for (int e = tid + NR * 256; e < nA; e += nthr) {
    A[e] = a.alpha[row0 * C + e];
    Bt[e] = a.beta[row0 * C + e];
  }
  for (int e = tid + NR * 256; e < nN; e += nthr) {
    AN[e] = a.alpha_num[row0 * NP + e];
    BN[e] = a.beta_num[row0 * NP + e];
  }
  for (int e = tid + NR * 256; e < nK; e += nthr) aoff[e] = arcsrc[e];
  if (a.do_den && g.n >= 2)
    for (int p = tid; p < C; p += nthr) {
      bool z;
      nbt[p] = next_base(g, p, &z);
    }
  if (dense) {
    float4* S4 = (float4*)Sub;  // the region is padded to 16 bytes
    for (int e = tid; e < (x.E + 3) / 4; e += nthr) S4[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int nhw = (x.E + 31) >> 5;  // words of the head bits
  if (sparse)
    for (int w = tid; w < nhw; w += nthr) hm[w] = 0u;
  __syncthreads();

  const bool den = a.do_den;
  const bool zero_next = g.n == 0, nb_table = g.n >= 2;
  // numerator chains (deterministic: chain order = ascending k): chain i's
  // head of frame f, arc k (its element within the slice, or -1 when the
  // lattice element lies outside it)
  auto head = [&](const Slice& x, int i, int& f, int& k) {
    f = (int)fdiv((unsigned)i, (unsigned)NK, a.mNK);
    k = i - f * NK;
    const int o = aoff[k];
    if (!(alink[k] >> 30) || o < x.e_lo || o >= x.e_lo + x.Ew) return -1;
    return f * x.Ew + o - x.e_lo;
  };
  auto chain = [&](int f, int k, float wv) {
    float sacc = 0.f;
    for (int kk = k; kk >= 0; kk = (alink[kk] & 0x3fffffff) - 1) {
      const int u = kk >> 1;
      const float bn = BN[f * NP + ((kk & 1) ? u + 1 : u)];
      sacc += lt_exp(AN[f * NP + u] + wv + bn - nm);
    }
    return gb * sacc;
  };
  // den marginal of frame f's element el (within the frame) with weight w
  auto den_el = [&](int f, int el, float w) {
    const int p = (int)fdiv((unsigned)el, (unsigned)R, a.mR);
    const int y = el - p * R;
    const int q = y == 0 ? p : (zero_next ? 0 : (nb_table ? nbt[p] : 0) + y);
    return gb * lt_exp(A[f * C + p] + w + Bt[f * C + q] - lz);
  };
  constexpr int NH = 4;
  const int nI = a.do_num ? Fl * NK : 0;
  {
    const unsigned char* Wb = a.W + x.base * ES;
    unsigned char* dWu = (unsigned char*)a.dW + (x.base + x.h0) * ES;  // unit u at dWu + 16 u
    auto tail_el = [&](int i) { return i < x.h0 ? i : i + x.nunits * VE; };
    // the chain heads' W elements come from L2 (the slice was just
    // streamed), gathered for NH rounds at once
    int hel[NH], hf[NH], hk[NH];
    float hw[NH];
#pragma unroll
    for (int r = 0; r < NH; ++r) {
      const int i = tid + r * 256;
      hel[r] = i < nI ? head(x, i, hf[r], hk[r]) : -1;
      if (hel[r] >= 0) hw[r] = ldw<BF16>(Wb, hel[r]);
    }
    // rank of a head element among the tile's heads (nmode 2)
    auto hrank = [&](int el) {
      return hp[el >> 5] + __builtin_popcount(hm[el >> 5] & ((1u << (el & 31)) - 1u));
    };
    if (sparse) {
      // the heads' bits, the prefix of their counts (wave 0), then each
      // head's numerator sum at its rank; three barriers, no buffer per element
#pragma unroll
      for (int r = 0; r < NH; ++r)
        if (hel[r] >= 0) atomicOr(&hm[hel[r] >> 5], 1u << (hel[r] & 31));
      for (int i = tid + NH * 256; i < nI; i += nthr) {
        int f, k;
        const int el = head(x, i, f, k);
        if (el >= 0) atomicOr(&hm[el >> 5], 1u << (el & 31));
      }
      __syncthreads();
      if (tid < 64) {
        int carry = 0;
        for (int c0 = 0; c0 < nhw; c0 += 64) {
          const int w = c0 + tid;
          const int pc = w < nhw ? __builtin_popcount(hm[w]) : 0;
          int inc = pc;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(inc, d);
            if (tid >= d) inc += o;
          }
          if (w < nhw) hp[w] = carry + inc - pc;
          carry += __shfl(inc, 63);
        }
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < NH; ++r)
        if (hel[r] >= 0) hv[hrank(hel[r])] = chain(hf[r], hk[r], hw[r]);
      for (int i = tid + NH * 256; i < nI; i += nthr) {
        int f, k;
        const int el = head(x, i, f, k);
        if (el >= 0) hv[hrank(el)] = chain(f, k, ldw<BF16>(Wb, el));
      }
      __syncthreads();
    }
    if (dense) {  // whole frames: the chains' sums into Sub before the den pass
#pragma unroll
      for (int r = 0; r < NH; ++r)
        if (hel[r] >= 0) Sub[hel[r]] = chain(hf[r], hk[r], hw[r]);
      for (int i = tid + NH * 256; i < nI; i += nthr) {
        int f, k;
        const int el = head(x, i, f, k);
        if (el >= 0) Sub[el] = chain(f, k, ldw<BF16>(Wb, el));
      }
    }
    // den marginals of the register units
    float v[kMgUnits][VE];
#pragma unroll
    for (int r = 0; r < kMgUnits; ++r) {
      const int u = tid + r * 256;
#pragma unroll
      for (int c = 0; c < VE; ++c) v[r][c] = 0.f;
      if (u < x.nunits && den) {
        float w[VE];
        unpack_unit<BF16>(wq[r], w);
        const int e0 = x.h0 + u * VE;
        int f = !SLICED ? (int)fdiv((unsigned)e0, (unsigned)FR, a.mF) : 0;
        const int el0 = x.e_lo + e0 - f * x.Ew;
        int p = (int)fdiv((unsigned)el0, (unsigned)R, a.mR);
        int y = el0 - p * R;
        if (R >= VE) {
          // a unit spans at most two source rows (p0 and the next, possibly
          // in the next frame of the tile): their alpha and next-state bases
          // are read once, every element is branch-free
          const int p1r = p + 1;
          const bool fw = p1r == C;
          const int p1 = fw ? 0 : p1r, f1 = fw ? f + 1 : f;
          const float a0v = A[f * C + p], a1v = f1 < Fl ? A[f1 * C + p1] : 0.f;
          const int nb0 = nb_table ? nbt[p] : 0;
          const int nb1 = nb_table ? nbt[p1] : 0;
#pragma unroll
          for (int c = 0; c < VE; ++c) {
            const int yc = y + c;
            const bool w2 = yc >= R;
            const int yy = w2 ? yc - R : yc;
            const int pp = w2 ? p1 : p, ff = w2 ? f1 : f;
            const int q = yy == 0 ? pp : (zero_next ? 0 : (w2 ? nb1 : nb0) + yy);
            const float av = w2 ? a1v : a0v;
            const float xv = gb * lt_exp(av + w[c] + Bt[ff * C + q] - lz);
            v[r][c] = ff < Fl ? xv : 0.f;
          }
        } else {
#pragma unroll
          for (int c = 0; c < VE; ++c) {
            if (f < Fl) {
              const int q = y == 0 ? p : (zero_next ? 0 : (nb_table ? nbt[p] : 0) + y);
              v[r][c] = gb * lt_exp(A[f * C + p] + w[c] + Bt[f * C + q] - lz);
            }
            if (++y == R) {
              y = 0;
              if (++p == C) { p = 0; ++f; }
            }
          }
        }
      }
    }
    if (dense) __syncthreads();
#pragma unroll
    for (int r = 0; r < kMgUnits; ++r) {
      const int u = tid + r * 256;
      if (u < x.nunits) {
        if (dense) {
#pragma unroll
          for (int c = 0; c < VE; ++c) v[r][c] -= Sub[x.h0 + u * VE + c];
        } else if (sparse) {
          const int e0 = x.h0 + u * VE, w0 = e0 >> 5, sh = e0 & 31;
          unsigned bits = hm[w0] >> sh;
          if (sh + VE > 32) bits |= hm[w0 + 1] << (32 - sh);
          bits &= (1u << VE) - 1u;
          if (bits) {
#pragma unroll
            for (int c = 0; c < VE; ++c)
              if ((bits >> c) & 1u) v[r][c] -= hv[hrank(e0 + c)];
          }
        }
        store_unit<BF16>(dWu + (long long)u * 16, v[r]);
      }
    }
    // the head before the first 16-byte boundary and the tail: element by element
    for (int i = tid; i < x.ntail; i += nthr) {
      const int e = tail_el(i);
      const int f = !SLICED ? (int)fdiv((unsigned)e, (unsigned)FR, a.mF) : 0;
      float xv = 0.f;
      if (f < Fl) {
        if (den) xv = den_el(f, x.e_lo + e - f * x.Ew, ldw<BF16>(Wb, e));
        if (dense) xv -= Sub[e];
        else if (sparse && ((hm[e >> 5] >> (e & 31)) & 1u)) xv -= hv[hrank(e)];
      }
      stw<BF16>(a.dW, x.base + e, xv);
    }
    if (!a.do_num || dense || sparse) return;

    // ---- phase 2 (frame slices): the chain heads rewrite their elements as
    // den - num once the slice's own stores have completed in every wave
    // (same workgroup, same address, in order)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    auto rewrite = [&](int el, int f, int k, float wv) {
      const float d = den ? den_el(f, el - f * x.Ew + x.e_lo, wv) : 0.f;
      stw<BF16>(a.dW, x.base + el, d - chain(f, k, wv));
    };
#pragma unroll
    for (int r = 0; r < NH; ++r)
      if (hel[r] >= 0) rewrite(hel[r], hf[r], hk[r], hw[r]);
    for (int i = tid + NH * 256; i < nI; i += nthr) {
      int f, k;
      const int el = head(x, i, f, k);
      if (el >= 0) rewrite(el, f, k, ldw<BF16>(Wb, el));
    }
  }
}

constexpr int kMgScan = 16;  // frames per cleanup workgroup after the trigram overlap

template <bool BF16, bool SLICED>
__global__ __launch_bounds__(256) void marg_kernel(const MgArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int job = (int)blockIdx.x;
  if (SLICED && a.done) {
    // after the trigram overlap: each workgroup scans kMgScan frames' done
    // flags in one load and takes the slices of the frames left (usually
    // none: one short workgroup per kMgScan frames instead of one per slice)
    __shared__ int s_list[kMgScan], s_n;
    const long long nfr = (long long)a.B * a.T;
    const long long f0 = (long long)blockIdx.x * kMgScan;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    if (threadIdx.x < kMgScan && f0 + threadIdx.x < nfr && !a.done[f0 + threadIdx.x])
      s_list[atomicAdd(&s_n, 1)] = (int)threadIdx.x;
    __syncthreads();
    const int cnt = s_n;
    for (int i = 0; i < cnt * a.tpf; ++i) {
      const long long f = f0 + s_list[i / a.tpf];
      const int b = (int)(f / a.T), t = (int)(f - (long long)b * a.T);
      marg_tile<BF16, SLICED>(a, b * a.tiles + t * a.tpf + i % a.tpf, lds);
      __syncthreads();  // the tile's LDS before the next tile's
    }
    return;
  }
  if (SLICED && LT_MARG_OPTS && a.xcd) {
    // blocks 8 g tpf + 8 s + x take slice s of frame 8 g + x: a frame's
    // slices 8 block ids apart, so under round-robin dispatch they share one
    // XCD's L2 for the frame's alpha / beta rows, which each of them reads
    // (placement changes only speed)
    const int gs = 8 * a.tpf, g = job / gs, r = job - g * gs;
    job = (8 * g + (r & 7)) * a.tpf + (r >> 3);
    if (job >= a.B * a.tiles) return;
  }
  marg_tile<BF16, SLICED>(a, job, lds);
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

int env_int(const char* name, int dflt) { return lt_impl::tune_int(name, dflt); }

int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

using lt_impl::Plan;

// Choose lanes-per-group, wave roles, LDS carve and ring depth.
//   kind 0: forward, kind 1: backward (beta + marginals), kind 2: checkpointing
//   backward (beta rows only). lds_cap bounds the workgroup's LDS (the
//   forward and the checkpointing backward share CUs when they run together).
int plan(const lt_problem* pb, const NGram& g, int kind, int flags, Plan* pl,
         int lds_cap = 160 * 1024) {
  KArgs& a = pl->a;
  memset(&a, 0, sizeof(a));
  pl->ck = kind == 2;
  a.B = pb->batch; a.T = pb->max_frames; a.U = pb->max_labels; a.g = g;
  a.flags = flags;
#ifdef LT_DIAG
  a.dbg = env_int("LT_DBG", 0);  // timing ablations: diagnostic builds only
#endif
#ifdef LT_STAMPS
  {
    const char* sp = lt_impl::tune_str("LT_STAMPS_PTR");
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
  const int den_cap = std::min(max_den, env_int("LT_MAX_DEN_WAVES", kind != 0 ? 5 : 4));
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
  const int cap = std::min(lds_cap, kLdsMax);
  int den = den_role ? ceil_div((long long)a.den_groups * L, 64) : 0;
  den = std::min(den, max_den);
  if (den_role && den < 1) den = 1;
  // backward: when exactly one group would spill into an extra, nearly empty
  // wave, wave 0's idle last lanes (j = L-1 of its 64/L groups) reduce it
  a.den_xg = 0;
  if (kind != 0 && den >= 2 && (long long)a.den_groups * L == 64LL * (den - 1) + L &&
      L >= 2 && L <= 8 && (L - 1) * a.Pr >= nterm && (64 / L) * a.Pr >= nterm &&
      env_int("LT_NO_XG", 0) == 0) {
    a.den_xg = 1;
    --den;
  }
  a.den_waves = den;
  a.den_fast = (den * 64 / L) >= a.den_groups - a.den_xg;

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
    if (fixed + need + ring_min <= cap && env_int("LT_FORCE_DIRECT", 0) == 0) {
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
    int S = (cap - al16(fixed)) / slot;
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
  if (pl->lds_bytes > cap) return fail(LT_EUNSUPPORTED, "LDS plan exceeds the LDS budget");
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

// Tiles of the marginal pass: at most kMgUnits 16-byte units per thread.
// Whole-frame tiles take a multiple of the frames that keep every tile
// 16-byte aligned when the frame size allows it.
int plan_marg(const lt_problem* pb, const NGram& g, bool do_den, bool do_num, MgArgs* m,
              long long* grid) {
  memset(m, 0, sizeof(*m));
  const int C = g.C, R = g.V + 1, NP = pb->max_labels + 1, NK = 2 * NP;
  const long long FR = (long long)C * R;
  const int es = pb->weight_dtype == LT_DTYPE_BF16 ? 2 : 4;
  const int units = std::max(1, std::min(kMgUnits, env_int("LT_MARG_UNITS", kMgUnits)));
  const long long emax_cap = 256LL * units * (16 / es);
  m->B = pb->batch; m->T = pb->max_frames; m->U = pb->max_labels; m->FR = (int)FR; m->g = g;
  m->do_den = do_den; m->do_num = do_num;
  if (FR <= emax_cap) {
    m->tpf = 1;
    long long period = 1;  // frames per 16-byte-aligned run
    while ((period * FR * es) % 16) ++period;
    int F = (int)(emax_cap / FR);
    if (F >= period) F -= F % period;
    F = std::max(1, std::min(F, std::max(1, pb->max_frames)));
    m->F = F;
    m->TS = (int)FR;
    m->tiles = std::max(1, ceil_div(pb->max_frames, F));
  } else {
    m->tpf = (int)((FR + emax_cap - 1) / emax_cap);
    long long ts = (FR + m->tpf - 1) / m->tpf;
    ts = (ts + 15) & ~15LL;  // slice starts stay 16-byte aligned within a frame
    m->TS = (int)std::min<long long>(ts, emax_cap);
    m->tpf = (int)((FR + m->TS - 1) / m->TS);
    m->F = 1;
    m->tiles = std::max(1, pb->max_frames * m->tpf);
  }
  m->mR = magic_of((unsigned)R);
  m->mF = magic_of((unsigned)FR);
  m->mNK = magic_of((unsigned)NK);
  auto al16 = [](long long x) { return (int)((x + 15) & ~15LL); };
  int off = 0;
  m->off_a = off; off += do_den ? al16(4LL * m->F * C) : 0;
  m->off_b = off; off += do_den ? al16(4LL * m->F * C) : 0;
  m->off_nb = off; off += (do_den && g.n >= 2) ? al16(4LL * C) : 0;
  m->off_an = off; off += do_num ? al16(4LL * m->F * NP) : 0;
  m->off_bn = off; off += do_num ? al16(4LL * m->F * NP) : 0;
  m->off_arc = off; off += do_num ? al16(8LL * NK) : 0;
  // whole-frame tiles may keep a dense numerator buffer (one float per
  // element); without it (and for frame slices, tpf > 1) the chain heads
  // rewrite their elements after the tile's stores, and the tile's LDS is a
  // quarter (more workgroups per CU)
  m->nmode = do_num ? env_int("LT_MARG_NMODE", 1) : 0;
  if (m->nmode == 1 && m->tpf != 1) m->nmode = 0;  // no dense buffer for frame slices
  m->off_sub = off; off += m->nmode == 1 ? al16(4LL * m->F * FR) : 0;
  {
    const long long E = m->tpf == 1 ? (long long)m->F * FR : m->TS;
    const int nhw = (int)((E + 31) / 32);
    m->off_hm = off; off += m->nmode == 2 ? al16(4LL * nhw) : 0;
    m->off_hp = off; off += m->nmode == 2 ? al16(4LL * nhw) : 0;
    m->off_hv = off; off += m->nmode == 2 ? al16(4LL * m->F * NK) : 0;
  }
  m->lds_bytes = std::max(off, 16);
  if (off > kLdsMax) return fail(LT_EUNSUPPORTED, "marginal tile exceeds LDS");
  *grid = (long long)pb->batch * m->tiles;
  m->xcd = m->tpf > 1 ? env_int("LT_MARG_XCD", 0) : 0;  // measured: no change at cfg5
  if (m->xcd) {  // whole groups of eight frames (the padding blocks return)
    const long long frames = (long long)pb->batch * pb->max_frames;
    *grid = (frames + 7) / 8 * 8 * m->tpf;
  }
  if (*grid > 0x7fffffffLL) return fail(LT_EUNSUPPORTED, "marginal grid too large");
  return LT_OK;
}

// dW[b] *= grad[b] for lt_scale_grad (the incoming gradient of a fused
// lt_loss_grad); workgroups of utterances with grad[b] == 1 return at once.
template <bool BF16>
__global__ __launch_bounds__(256) void scale_kernel(void* dW, const float* grad, long long per,
                                                    int chunks) {
  const int b = blockIdx.x / chunks, c = blockIdx.x - (blockIdx.x / chunks) * chunks;
  const float g = grad[b];
  if (g == 1.f) return;
  const long long lo = per * c / chunks, hi = per * (c + 1) / chunks;
  const long long base = (long long)b * per;
  for (long long e = lo + threadIdx.x; e < hi; e += blockDim.x) {
    if constexpr (BF16) {
      unsigned short* p = (unsigned short*)dW + base + e;
      *p = f2bf(__uint_as_float((unsigned)*p << 16) * g);
    } else {
      float* p = (float*)dW + base + e;
      *p *= g;
    }
  }
}

// After a fused lt_loss_grad launch: a hand-off wait that timed out (error
// word non-zero, lt_pipe.hip) means some workgroup read rows that were never
// published, so every loss of the batch is replaced by NaN -- the failure is
// visible in the product path instead of a silently wrong dW.
__global__ __launch_bounds__(256) void handoff_check_kernel(const int* err, float* loss, int B) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  for (int b = threadIdx.x; b < B; b += blockDim.x) loss[b] = __builtin_nanf("");
}

int cu_count() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;
}

// lt_loss_grad workspace: checkpoints, arc table and the recursion
// backward's side buffer, each 256-byte aligned
struct GradWs {
  size_t alpha, beta, an, bn, arcs, side, mix, total;
};
GradWs grad_ws(const lt_problem* pb, int local_norm) {
  GradWs w;
  const long long B = pb->batch, T = pb->max_frames, NP = pb->max_labels + 1;
  NGram g;
  make_ngram(pb->vocab_size, pb->context_size, &g);
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  size_t o = 0;
  w.alpha = o; o += local_norm ? 0 : up(4 * B * T * g.C);
  w.beta = o; o += local_norm ? 0 : up(4 * B * T * g.C);
  w.an = o; o += up(4 * B * T * NP);
  w.bn = o; o += up(4 * B * T * NP);
  w.arcs = o; o += up(4 * B * 4 * NP);
  w.side = o; o += up((long long)side_bytes(pb));
  // the trigram overlap: progress words, XCD ids, per-XCD job counters, done flags
  // (and the diagnostic time stamps)
  w.mix = o; o += g.n == 2 ? up(4 * (8 * B + 8 * 32 + B * T)) : 0;
  w.total = o;
  return w;
}

// The trigram overlap's hand-over from lt_loss_grad to the lt_loss_forward
// / lt_loss_backward calls it makes (set only for their duration, this thread)
struct MixReq {
  MixArgs m;      // prog / xcc / ctr / done set; the rest filled at the launch
  int blocks;     // marginal workgroups
  bool launched;  // lt_loss_forward took the overlap route
};
thread_local MixReq* t_mix = nullptr;
thread_local const int* t_mix_done = nullptr;

}  // namespace

namespace lt_impl {
int set_error(int code, const char* msg) { return fail(code, msg); }

size_t serial_side_bytes(const lt_problem* pb, int local_norm) {
  size_t n = 0;
  if (lt_loss_backward_workspace_bytes(pb, local_norm, &n) != LT_OK) return 0;
  return n;
}

// The frame-serial recursion kernels (fwd_kernel, bwd_kernel) restricted to
// the utterances with only[b] != 0: loss / log_z / num and, when dW is given,
// alpha / alpha_num checkpoints plus the backward -> dW (scaled by grad).
// The chunked path (lt_chunk.hip) sends utterances outside its range here.
int serial_loss(const lt_problem* pb, int local_norm, const void* W, const int32_t* num_frames,
                const int32_t* labels, const int32_t* num_labels, const int* only, float* loss,
                float* log_z, float* num, float* alpha, float* alpha_num, const float* grad,
                void* dW, void* side, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  Plan pf;
  if ((rc = plan(pb, g, 0, F_NUM | F_LOSS | (local_norm ? F_LOCAL : F_DEN), &pf))) return rc;
  bind_streams(pf.a, W, nullptr, nullptr);
  pf.a.nfr = num_frames; pf.a.labels = labels; pf.a.nlab = num_labels;
  pf.a.loss = loss; pf.a.dist = local_norm ? nullptr : log_z; pf.a.num = num;
  pf.a.alpha = dW ? alpha : nullptr; pf.a.alpha_num = dW ? alpha_num : nullptr;
  pf.a.only = only;
  if (local_norm && log_z) {
    if ((rc = hip_check(hipMemsetAsync(log_z, 0, sizeof(float) * pb->batch, st), "memset")))
      return rc;
  }
  if (!dW) return launch_fwd(M_LOG, pf, bf16, pb->batch, st);
  Plan pl;
  if ((rc = plan(pb, g, 1, F_NUM | (local_norm ? F_LOCAL : F_DEN), &pl))) return rc;
  bind_streams(pl.a, W, local_norm ? nullptr : alpha, alpha_num);
  KArgs& a = pl.a;
  a.nfr = num_frames; a.labels = labels; a.nlab = num_labels;
  a.log_z_in = log_z; a.num_in = num; a.grad = grad; a.dW = dW;
  a.only = only;
  // forward and backward in one launch when the two plans share a geometry
  // (the usual case): lt_loss_grad's fallback then costs one (empty) launch
  if (pl.dst && pf.lg == pl.lg && pf.tmax == pl.tmax && pf.wst == pl.wst &&
      pf.threads == pl.threads) {
#define LT_CASE(LG, P) \
  if (pf.lg == LG && pf.tmax == P) return lt_impl::launch_serial_##LG##_##P(pf, pl, bf16, pb->batch, st);
    LT_VARIANTS(LT_CASE)
#undef LT_CASE
  }
  if ((rc = launch_fwd(M_LOG, pf, bf16, pb->batch, st))) return rc;
  if (!pl.dst) {
    const long long NP = pb->max_labels + 1;
    const long long nm = (long long)pb->batch * pb->max_frames * NP * 2 * 4;
    a.nm_side = (float*)side;
    a.ctx_side = (int*)((char*)side + ((nm + 255) & ~255LL));
  }
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
                    float* alpha, float* alpha_num, float* beta, float* beta_num,
                    int32_t* arcs, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (LT_NEED(W) || !num_frames || !num_labels || !loss || (pb->max_labels > 0 && !labels))
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W)) return fail(LT_EINVAL, "W must be 16-byte aligned");
  const bool ck = beta_num && arcs;
  if (ck && !local_norm && LT_NEED(beta)) return fail(LT_EINVAL, "beta is null");
  if (ck && (LT_NEED(alpha_num) || (!local_norm && LT_NEED(alpha))))
    return fail(LT_EINVAL, "checkpoints need alpha / alpha_num");
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const int flags = F_NUM | F_LOSS | (local_norm ? F_LOCAL : F_DEN);
  hipStream_t st = (hipStream_t)stream;
  // bigram with checkpoints: the pipelined two-factor alpha and beta
  // recursions in one launch (lt_pipe.hip). Without checkpoints the
  // frame-barrier kernel below is the faster one (measured: 0.45 vs 0.52 ms
  // at B=64), so the pipe only serves the checkpointing path.
  if (ck && lt_impl::pipe_eligible(pb))
    return lt_impl::launch_pipe(pb, local_norm, W, num_frames, labels, num_labels, loss, log_z,
                                num, alpha, alpha_num, beta, beta_num, arcs, 2, nullptr, stream);
  // With checkpoints, the beta pass (independent of alpha) and the alpha
  // pass, both on the caller's stream (the library forks no stream:
  // everything stays ordered on `stream` and capturable).
  Plan pf, pbk;
  if (ck) {
    const int bflags = F_NUM | (local_norm ? F_LOCAL : F_DEN);
    if ((rc = plan(pb, g, 2, bflags, &pbk, kLdsMax))) return rc;
    bind_streams(pbk.a, W, nullptr, nullptr);
    pbk.a.nfr = num_frames;
    pbk.a.labels = labels;
    pbk.a.nlab = num_labels;
    pbk.a.beta = local_norm ? nullptr : beta;
    pbk.a.beta_num = beta_num;
  }
  if ((rc = plan(pb, g, 0, flags, &pf, kLdsMax))) return rc;
  bind_streams(pf.a, W, nullptr, nullptr);
  pf.a.nfr = num_frames;
  pf.a.labels = labels;
  pf.a.nlab = num_labels;
  pf.a.loss = loss;
  pf.a.dist = log_z;
  pf.a.num = num;
  pf.a.alpha = alpha;
  pf.a.alpha_num = alpha_num;
  pf.a.arcs = ck ? arcs : nullptr;
#ifdef LT_DIAG
  if (lt_impl::tune_str("LT_PLAN_DEBUG")) {
    fprintf(stderr, "fwd plan lg=%d P=%d wst=%d threads=%d lds=%d\n", pf.lg, pf.tmax, pf.wst,
            pf.threads, pf.lds_bytes);
    if (ck)
      fprintf(stderr, "bwd plan lg=%d P=%d wst=%d threads=%d lds=%d\n", pbk.lg, pbk.tmax,
              pbk.wst, pbk.threads, pbk.lds_bytes);
  }
#endif
  // trigram with W staged in LDS: the den roles of lt_tri.hip (one lane per
  // state pair, every term in registers) in the same side-by-side launch.
  // Diagnostic builds only (LT_DIAG, LT_TRI4=1): the V = 32 recursions on
  // quads of four workgroups (lt_tri4.hip, measured slower); the
  // product library does not link lt_tri4.o
#ifdef LT_DIAG
  if (ck && !local_norm && g.n == 2 && g.V == 32 && alpha && beta) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        lt_impl::tri4_eligible(g.V, g.n, pb->batch, pb->max_labels, cus)) {
      const long long wb = (long long)pb->batch * pb->max_frames * g.C * (g.V + 1) * (bf16 ? 2 : 4);
      return lt_impl::launch_tri4(pf, bf16, alpha, beta, alpha_num, beta_num, log_z, num, loss,
                                  wb, st);
    }
  }
#endif
  if (ck && !local_norm && g.n == 2 && g.V >= 2 && g.V <= 32 && pf.wst && pbk.wst &&
      pf.a.aux_waves == pbk.a.aux_waves && pf.a.slot_bytes == pbk.a.slot_bytes &&
      (g.V != 32 || pbk.lds_bytes + 8 * kTriBPad <= kLdsMax) && env_int("LT_NO_TRI", 0) == 0) {
    if (g.V == 32) {  // den_bwd_tri32's padded beta rows, past the ring
      pbk.a.off_tb = pbk.lds_bytes;
      pbk.lds_bytes += 8 * kTriBPad;
    }
    for (Plan* pl : {&pf, &pbk}) {
      // four loader waves: a frame is 69 LDS-DMA wave instructions (bf16),
      // whose issue cost alone is a microsecond on two waves
      KArgs& ka = pl->a;
      ka.den_waves = kTriDenWaves;
      const int instr = ka.st_ninstr[0] + ka.st_ninstr[1] + ka.st_ninstr[2];
      ka.load_waves = std::min(kTriLoadWaves, std::max(1, instr));
      // loader_loop: wave 0 issues gw0 instructions a frame, the others gw1
      // (instr % load_waves <= 1 keeps that exact)
      while (ka.load_waves > 2 && instr % ka.load_waves > 1) --ka.load_waves;
      ka.gw0 = (instr + ka.load_waves - 1) / ka.load_waves;
      ka.gw1 = instr / ka.load_waves;
      pl->threads = 64 * (kTriDenWaves + ka.aux_waves + ka.load_waves);
    }
    if (t_mix && g.V == 32 && pb->batch % 8 == 0) {
      // lt_loss_grad's trigram route: marginal workgroups on the idle CUs in
      // the same launch (lt_tri.hip, tri_mix_kernel)
      pf.a.prog = pbk.a.prog = t_mix->m.prog;
      MixArgs mx = t_mix->m;
      mx.W = (const unsigned char*)W; mx.nfr = num_frames; mx.labels = labels;
      mx.alpha = alpha; mx.beta = beta; mx.alpha_num = alpha_num; mx.beta_num = beta_num;
      mx.B = pb->batch; mx.T = pb->max_frames; mx.U = pb->max_labels; mx.g = g;
      if ((rc = lt_impl::launch_tri_mix(pf, pbk, bf16, pb->batch, t_mix->blocks, mx, st))) return rc;
      t_mix->launched = true;
      return LT_OK;
    }
    return lt_impl::launch_tri_fwdbwd(pf, pbk, bf16, pb->batch, st);
  }
  // same geometry (the usual case): beta and alpha side by side in one
  // launch; else beta, then alpha
  if (ck && pf.lg == pbk.lg && pf.tmax == pbk.tmax && pf.wst == pbk.wst &&
      pf.threads == pbk.threads && env_int("LT_PAIR", 1)) {
#define LT_CASE(LG, P) \
  if (pf.lg == LG && pf.tmax == P) return lt_impl::launch_fwdbwd_##LG##_##P(pf, pbk, bf16, pb->batch, st);
    LT_VARIANTS(LT_CASE)
#undef LT_CASE
  }
  if (ck && (rc = launch_bwd(pbk, bf16, pb->batch, st))) return rc;
  return launch_fwd(M_LOG, pf, bf16, pb->batch, st);
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
                     const float* alpha, const float* alpha_num, const float* beta,
                     const float* beta_num, const int32_t* arcs, const float* grad, void* dW,
                     void* workspace, size_t workspace_bytes, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  if (beta_num && arcs) {  // checkpoints from lt_loss_forward: one streaming pass
    if (LT_NEED(W) || !num_frames || !num || LT_NEED(alpha_num) || LT_NEED(beta_num) ||
        LT_NEED(dW) || (!local_norm && (!log_z || LT_NEED(alpha) || LT_NEED(beta))))
      return fail(LT_EINVAL, "null pointer");
    if (misaligned(W) || misaligned(dW)) return fail(LT_EINVAL, "W/dW must be 16-byte aligned");
    MgArgs m;
    long long grid = 0;
    if ((rc = plan_marg(pb, g, !local_norm, true, &m, &grid))) return rc;
    m.W = (const unsigned char*)W; m.nfr = num_frames;
    m.alpha = alpha; m.beta = beta; m.alpha_num = alpha_num; m.beta_num = beta_num;
    m.arcs = arcs; m.log_z = log_z; m.num = num; m.grad = grad; m.dW = dW;
    m.done = t_mix_done;  // the trigram overlap's frames (lt_loss_grad only)
    m.mid_norm = t_mix_done != nullptr;
    if (grid == 0) return LT_OK;
    if (m.done && m.tpf > 1) grid = ceil_div((long long)pb->batch * pb->max_frames, kMgScan);
    hipStream_t st = (hipStream_t)stream;
    const bool bf = pb->weight_dtype == LT_DTYPE_BF16, sliced = m.tpf > 1;
    const void* k = bf ? (sliced ? (const void*)marg_kernel<true, true>
                                 : (const void*)marg_kernel<true, false>)
                       : (sliced ? (const void*)marg_kernel<false, true>
                                 : (const void*)marg_kernel<false, false>);
    if (m.lds_bytes > 64 * 1024 &&
        (rc = hip_check(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            m.lds_bytes), "marginal LDS")))
      return rc;
    void* args[] = {&m};
    if ((rc = hip_check(hipLaunchKernel(k, dim3((unsigned)grid), dim3(256), args, m.lds_bytes, st),
                        "marginal launch")))
      return rc;
    return hip_check(hipGetLastError(), "marginal launch");
  }
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
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  hipStream_t st = (hipStream_t)stream;
  if (lt_impl::vit_bigram_eligible(pb)) {
    // bigram: the chain, loader and backpointer waves of lt_vit.hip, the
    // backtrace in the same launch when it fits
    rc = lt_impl::vit_bigram(pb, W, num_frames, bp, qstar, path_weight, grad, labels, arcs,
                             label_convention, stream);
    if (rc != LT_EUNSUPPORTED) return rc;
  } else {
    lt_problem p2 = *pb;
    p2.max_labels = 0;
    Plan pl;
    if ((rc = plan(&p2, g, 0, F_DEN, &pl))) return rc;
    bind_streams(pl.a, W, nullptr, nullptr);
    pl.a.nfr = num_frames;
    pl.a.dist = path_weight;
    pl.a.bp = bp;
    pl.a.qstar = qstar;
    if ((rc = launch_fwd(M_MAX, pl, bf16, pb->batch, st))) return rc;
  }
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

// The design lt_loss_grad runs for this problem (LT_DESIGN_*): the chunked
// scan while it is faster, else the fused pipe launch, the checkpointing pair
// or the recursion pair (the environment overrides apply, as in the call).
static int loss_grad_design(const lt_problem* pb) {
  if (lt_impl::chunk_preferred(pb) && pb->max_frames > 0) return LT_DESIGN_CHUNK;
  // the one-launch fused pipe (mid mode) measured level with the checkpointing
  // pair at B = 192 / 256 (profiles/r03_mid_modes.txt), so it is not the
  // default; lt_loss_grad_ex runs it on request
  if (lt_impl::pipe_eligible(pb) && env_int("LT_MID", 0) && lt_impl::pipe_mid_fits(pb))
    return LT_DESIGN_FUSED_PIPE;
  const int cus = cu_count();
  const bool ck_def = 2 * pb->batch <= cus || (lt_impl::pipe_eligible(pb) && 2 * pb->batch <= 3 * cus);
  const bool ck = env_int("LT_CHECKPOINTS", ck_def ? 1 : 0) != 0;
  return ck ? LT_DESIGN_CHECKPOINTS : LT_DESIGN_RECURSION;
}

int lt_loss_grad_design(const lt_problem* pb, int32_t* design) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  if (!design) return fail(LT_EINVAL, "null pointer");
  *design = loss_grad_design(pb);
  return LT_OK;
}

// An explicit design for *pb: LT_DESIGN_AUTO resolves to lt_loss_grad's own
// choice; a design the shape cannot take is EUNSUPPORTED.
static int resolve_design(const lt_problem* pb, int32_t design, int* out) {
  if (design == LT_DESIGN_AUTO) {
    *out = loss_grad_design(pb);
    return LT_OK;
  }
  if (design == LT_DESIGN_CHUNK && !(lt_impl::chunk_eligible(pb) && pb->max_frames > 0))
    return fail(LT_EUNSUPPORTED, "design chunk: FullNGram n = 1, vocab_size <= 32, labels < 128");
  if (design == LT_DESIGN_FUSED_PIPE && !(lt_impl::pipe_eligible(pb) && pb->max_labels + 1 <= 128))
    return fail(LT_EUNSUPPORTED, "design fused pipe: bigram shapes, labels < 128");
  if (design < LT_DESIGN_CHUNK || design > LT_DESIGN_RECURSION)
    return fail(LT_EINVAL, "unknown design");
  *out = design;
  return LT_OK;
}

int lt_loss_grad_workspace_bytes_ex(const lt_problem* pb, int32_t local_norm, int32_t design,
                                    size_t* bytes) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  int d = 0;
  if ((rc = resolve_design(pb, design, &d))) return rc;
  if (d == LT_DESIGN_CHUNK) {
    size_t st = 0, sc = 0;
    if ((rc = lt_chunk_workspace_bytes(pb, local_norm, &st, &sc))) return rc;
    if (bytes) *bytes = ((st + 255) & ~(size_t)255) + sc;
    return LT_OK;
  }
  if (d == LT_DESIGN_FUSED_PIPE) {
    if (bytes) *bytes = lt_impl::pipe_mid_workspace_bytes(pb);
    return LT_OK;
  }
  if (bytes) *bytes = grad_ws(pb, local_norm).total;
  return LT_OK;
}

int lt_loss_grad_workspace_bytes(const lt_problem* pb, int32_t local_norm, size_t* bytes) {
  return lt_loss_grad_workspace_bytes_ex(pb, local_norm, LT_DESIGN_AUTO, bytes);
}

int lt_loss_grad_ex(const lt_problem* pb, int32_t local_norm, int32_t design_in, const void* W,
                    const int32_t* num_frames, const int32_t* labels, const int32_t* num_labels,
                    float* loss, float* log_z, float* num, void* dW, void* workspace,
                    size_t workspace_bytes, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  int design = 0;
  if ((rc = resolve_design(pb, design_in, &design))) return rc;
  if (pb->batch == 0) return LT_OK;
  if (LT_NEED(W) || !num_frames || !num_labels || !loss || !log_z || !num || LT_NEED(dW) ||
      (pb->max_labels > 0 && !labels))
    return fail(LT_EINVAL, "null pointer");
  if (misaligned(W) || misaligned(dW)) return fail(LT_EINVAL, "W/dW must be 16-byte aligned");
  if (design == LT_DESIGN_CHUNK) {
    // bigram: the chunked two-level scan (lt_chunk.hip), two launches (plus
    // the frame-serial pair, whose workgroups exit at once unless an
    // utterance leaves the fast path)
    size_t st = 0, sc = 0;
    if ((rc = lt_chunk_workspace_bytes(pb, local_norm, &st, &sc))) return rc;
    const size_t st_al = (st + 255) & ~(size_t)255;
    if (!workspace || workspace_bytes < st_al + sc) return fail(LT_EINVAL, "workspace too small");
    char* state = (char*)workspace;
    char* scratch = state + st_al;
    return lt_impl::chunk_loss_grad(pb, local_norm, W, num_frames, labels, num_labels, loss,
                                    log_z, num, dW, state, st, scratch, sc, stream);
  }
  if (design == LT_DESIGN_FUSED_PIPE && pb->max_frames > 0) {
    // bigram, large batches: one launch of the pipelined alpha || beta
    // recursions whose marginal waves turn the far half of each utterance's
    // frames into dW while the frames are in the ring (lt_pipe.hip, mid mode)
    const size_t need = lt_impl::pipe_mid_workspace_bytes(pb);
    if (!workspace || workspace_bytes < need) return fail(LT_EINVAL, "workspace too small");
    if ((rc = lt_impl::launch_pipe(pb, local_norm, W, num_frames, labels, num_labels, loss, log_z,
                                   num, nullptr, nullptr, nullptr, nullptr, nullptr, 2, nullptr,
                                   stream, dW, 1, workspace)))
      return rc;
    const long long BT = (long long)pb->batch * pb->max_frames;
    const int* err = (const int*)((char*)workspace +
                                  8 * (2 * BT * g.C + 2 * BT * (pb->max_labels + 1) +
                                       2LL * pb->batch));
    hipLaunchKernelGGL(handoff_check_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, err,
                       loss, pb->batch);
    return hip_check(hipGetLastError(), "hand-off check launch");
  }
  const GradWs w = grad_ws(pb, local_norm);
  if (!workspace || workspace_bytes < w.total) return fail(LT_EINVAL, "workspace too small");
  char* ws = (char*)workspace;
  float* alpha = local_norm ? nullptr : (float*)(ws + w.alpha);
  float* beta = local_norm ? nullptr : (float*)(ws + w.beta);
  float* an = (float*)(ws + w.an);
  float* bn = (float*)(ws + w.bn);
  int32_t* arcs = (int32_t*)(ws + w.arcs);
  const long long ptrs = (long long)pb->batch * pb->max_frames;
  if (ptrs == 0) {  // T = 0: loss from the empty lattice, dW is empty
    return lt_loss_forward(pb, local_norm, W, num_frames, labels, num_labels, loss, log_z, num,
                           alpha, an, nullptr, nullptr, nullptr, stream);
  }
  // checkpointing (alpha || beta, then the marginal pass) while 2B recursion
  // workgroups find CUs; with the pipelined bigram recursions up to 1.5 CUs
  // utterances (measured crossover ~1.75: tools/b256_check.py)
  if (design == LT_DESIGN_CHECKPOINTS || design == LT_DESIGN_FUSED_PIPE) {
    // trigram V = 32: the recursions with marginal workgroups on the CUs they
    // leave idle (lt_tri.hip), marg_kernel afterwards on the frames not done
    const int cus = cu_count();
    MixReq req;
    const bool mix = g.n == 2 && g.V == 32 && !local_norm && pb->batch % 8 == 0 &&
                     2 * pb->batch + 8 <= cus && pb->max_frames >= 2 && pb->max_frames < 65536 &&
                     lt_impl::tune_int("LT_TRI_MIX", 1) != 0;
    if (mix) {
      memset(&req, 0, sizeof(req));
      const long long B = pb->batch;
      unsigned* mw = (unsigned*)(ws + w.mix);
      req.m.prog = mw;
      req.m.xcc = mw + 2 * B;
      req.m.ctr = mw + 4 * B;
      req.m.done = (int*)(mw + 4 * B + 8 * 32);
      req.m.dW = dW;
      req.m.dbg = lt_impl::tune_int("LT_TRI_MIX_DBG", 0);
      req.m.ts = (unsigned*)(req.m.done + B * pb->max_frames);
      // marginal workgroups for the idle CUs (LT_TRI_MIX_EXTRA more, queued
      // for the recursions' CUs: measured 3.35 against 3.27 ms at cfg5 with 2B)
      req.blocks = cus - 2 * pb->batch + lt_impl::tune_int("LT_TRI_MIX_EXTRA", 0);
      if ((rc = hip_check(hipMemsetAsync(mw, 0, 4 * (size_t)(8 * B + 8 * 32 + B * pb->max_frames),
                                         (hipStream_t)stream),
                          "overlap memset")))
        return rc;
      t_mix = &req;
    }
    rc = lt_loss_forward(pb, local_norm, W, num_frames, labels, num_labels, loss, log_z, num,
                         alpha, an, beta, bn, arcs, stream);
    t_mix = nullptr;
    if (rc) return rc;
    t_mix_done = mix && req.launched ? req.m.done : nullptr;
    rc = lt_loss_backward(pb, local_norm, W, num_frames, labels, num_labels, log_z, num, alpha,
                          an, beta, bn, arcs, nullptr, dW, nullptr, 0, stream);
    t_mix_done = nullptr;
    return rc;
  }
  if ((rc = lt_loss_forward(pb, local_norm, W, num_frames, labels, num_labels, loss, log_z, num,
                            alpha, an, nullptr, nullptr, nullptr, stream)))
    return rc;
  return lt_loss_backward(pb, local_norm, W, num_frames, labels, num_labels, log_z, num, alpha,
                          an, nullptr, nullptr, nullptr, nullptr, dW, ws + w.side,
                          workspace_bytes - w.side, stream);
}

int lt_loss_grad(const lt_problem* pb, int32_t local_norm, const void* W,
                 const int32_t* num_frames, const int32_t* labels, const int32_t* num_labels,
                 float* loss, float* log_z, float* num, void* dW, void* workspace,
                 size_t workspace_bytes, void* stream) {
  return lt_loss_grad_ex(pb, local_norm, LT_DESIGN_AUTO, W, num_frames, labels, num_labels, loss,
                         log_z, num, dW, workspace, workspace_bytes, stream);
}

int lt_scale_grad(const lt_problem* pb, const float* grad, void* dW, void* stream) {
  NGram g;
  int rc = check_problem(pb, &g);
  if (rc) return rc;
  const long long per = (long long)pb->max_frames * g.C * (g.V + 1);
  if (pb->batch == 0 || per == 0) return LT_OK;
  if (!grad || LT_NEED(dW)) return fail(LT_EINVAL, "null pointer");
  const int chunks = (int)std::max<long long>(1, std::min<long long>(64, per / 4096));
  const long long grid = (long long)pb->batch * chunks;
  if (grid > 0x7fffffffLL) return fail(LT_EUNSUPPORTED, "grid too large");
  hipStream_t st = (hipStream_t)stream;
  if (pb->weight_dtype == LT_DTYPE_BF16)
    hipLaunchKernelGGL(scale_kernel<true>, dim3((unsigned)grid), dim3(256), 0, st, dW, grad, per,
                       chunks);
  else
    hipLaunchKernelGGL(scale_kernel<false>, dim3((unsigned)grid), dim3(256), 0, st, dW, grad,
                       per, chunks);
  return hip_check(hipGetLastError(), "scale launch");
}

}  // extern "C"
