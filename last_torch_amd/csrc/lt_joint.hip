// lt_joint.hip -- the joint weight function fused into the lattice loss
// (SURVEY.md 8(f) rank 1). lt_loss_joint_forward / _backward (and
// lt_loss_grad_joint, both in one call) run RecognitionLattice.forward
// (lattices.py:131-183) for FullNGram n = 1 x FrameDependent under Log with
// the arc weights of JointWeightFn (weight_fns.py:174-227, consumed per frame
// at lattices.py:446),
//   W[f, c, y] = bias[y] + sum_h Wo[y, h] tanh(Pc[c, h] + Pf[f, h]),
// and give the loss and the parameter gradients d_Pc, d_Pf, d_Wo, d_bias
// without W or dW = d loss / dW ever in HBM:
//   1 jf_prep_kernel   e^{2 Pc}, e^{2 Pf} and the direct-tanh flags per 32-row
//                      block of Pf (as lt_joint_weights decides them)
//   2 pipe_kernel      the alpha || beta recursions with checkpoints
//                      (lt_pipe.hip); its helper waves form each frame's W on
//                      the matrix cores (helper_prod) instead of loading it
//   3 jf_marg_kernel   per (utterance, block of 32 frames), for each context
//                      state c: the W tile [32 frames x R] on the matrix cores,
//                      its den - num marginals g (alignments.py:300-318 and
//                      the string arcs of lattices.py:314-338, as marg_kernel
//                      forms them) times the incoming gradient, then the
//                      producer's backward from g in LDS: gw = g Wo, dh =
//                      gw (1 - hid^2), d_Pf rows, d_Pc / d_Wo / d_bias partials
//   4 joint_reduce     the partials summed in a fixed order (deterministic)
// Every W element is formed through joint_tile's K steps, so it equals
// lt_joint_weights_ex's output bit for bit, and the loss equals the
// checkpointing design's on that materialised W.
#include "lt_joint.h"

namespace {

struct JFArgs {
  const float *pc, *ec, *pf, *ef, *wo, *bias;
  const int *cbig, *fbig;
  const int* nfr;
  const float *alpha, *beta, *alpha_num, *beta_num;  // pipe_kernel's checkpoints
  const int* arcs;                                   // [B][2 NK] string arc table
  const float *log_z, *num, *grad;
  const int* err;  // the forward's pipeline-timeout word (nonzero: every output NaN)
  float* dpf;   // [B*T, H]
  float* part;  // [B * nblk][(C + R) H + 64] per-block d_Pc, d_Wo, d_bias
  int B, T, U, C, R, H, NP, nblk;
  long long* stamps;  // diagnostic build (-DLT_STAMPS) only: [block][8] s_memtime
};

#ifdef LT_STAMPS
#define JSTAMP(a, k, v)                                                  \
  do {                                                                   \
    if ((a).stamps && (threadIdx.x & 63) == 0 && threadIdx.x < 64)       \
      (a).stamps[(long long)blockIdx.x * 8 + (k)] = (v);                 \
  } while (0)
#define JCLK() ((long long)__builtin_amdgcn_s_memtime())
#define JWAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define JSTAMP(a, k, v) \
  do {                  \
  } while (0)
#define JCLK() 0LL
#define JWAIT() \
  do {          \
  } while (0)
#endif

__host__ __device__ inline long long jf_stride(int C, int R, int H) { return (long long)(C + R) * H + 64; }

// e^{2 Pc}, e^{2 Pf}; cbig / fbig[row / 32] raised for |projection| > kSplitMax
// (NaN counts): the producer's split / direct decision (joint_exp_kernel and
// joint_weights_fb_kernel's per-block test)
__global__ __launch_bounds__(256) void jf_prep_kernel(const float* pc, const float* pf, float* ec,
                                                      float* ef, int* cbig, int* fbig, long long nc4,
                                                      long long nf4, int H) {
  const int h4 = H / 4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nc4 + nf4;
       i += (long long)gridDim.x * blockDim.x) {
    const bool isc = i < nc4;
    const float4 x = isc ? ((const float4*)pc)[i] : ((const float4*)pf)[i - nc4];
    const float m = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
    const f32x2 lo = exp2x(f32x2{x.x, x.y}), hi = exp2x(f32x2{x.z, x.w});
    const float4 e = {lo.x, lo.y, hi.x, hi.y};
    if (isc) ((float4*)ec)[i] = e;
    else ((float4*)ef)[i - nc4] = e;
    if (!(m <= kSplitMax)) {
      if (isc) atomicOr(cbig, 1);
      else atomicOr(fbig + (i - nc4) / h4 / 32, 1);
    }
  }
}

constexpr int kJfKB = 3;                 // K blocks of gw (R = V + 1 <= 48)
constexpr int kJfGS = kJfKB * 16 + 4;    // g tile row stride (floats)

template <int NW>
constexpr int jf_threads() { return 64 * NW; }

struct JfLds {
  int wo, A, Bt, AN, BN, aoff, hd, gt, wt, dpc, ec, ef, total;
};
JfLds jf_lds(int C, int R, int H, int NP, bool sp) {
  auto al16 = [](long long x) { return (int)((x + 15) & ~15LL); };
  JfLds l;
  const int WL = (R * (H + 8) + 7) & ~7;
  int o = 0;
  l.wo = o; o += al16((sp ? 4LL : 2LL) * WL);
  l.A = o; o += al16(4LL * 32 * C);
  l.Bt = o; o += al16(4LL * 32 * C);
  l.AN = o; o += al16(4LL * 32 * NP);
  l.BN = o; o += al16(4LL * 32 * NP);
  l.aoff = o; o += al16(4LL * 4 * NP);
  l.hd = o; o += al16(4LL * C * R);
  l.gt = o; o += al16(4LL * 2 * 32 * kJfGS);
  l.wt = o; o += al16(4LL * 32 * R);  // the raw W tile of the forward in progress
  l.dpc = o; o += al16(4LL * C * H);
  l.ec = o; o += al16(4LL * C * H);   // e^{2 Pc} (or Pc on the direct path)
  l.ef = o; o += al16(4LL * 32 * H);  // the block's e^{2 Pf} rows (or Pf)
  l.total = o;
  return l;
}

// n 4-byte words global -> LDS with 8 loads in flight per thread (a plain
// strided copy loop waits one memory latency per trip)
template <typename Tw>
LT_DEVINL void stage_words(Tw* dst, const Tw* src, int n, int tid, int nthr) {
  constexpr int U = 8;
  for (int e0 = tid; e0 < n; e0 += U * nthr) {
    Tw v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * nthr;
      if (e < n) v[u] = src[e];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * nthr;
      if (e < n) dst[e] = v[u];
    }
  }
}

// One workgroup per (utterance b, block of 32 frames); NW = H / 32 waves,
// wave w owning hidden columns [32 w, 32 w + 32) in the backward. For c =
// 0..C-1 (two g tiles in LDS, one barrier a tile): wave c % NW forms the W
// tile of state c and its marginals, then every wave runs the backward of
// that tile -- the split-bf16 products and K orders of joint_backward_kernel.
template <int NW, bool SP>
__global__ __launch_bounds__(64 * (NW < 2 ? 2 : NW), 2) void jf_marg_kernel(const JFArgs a,
                                                                          const JfLds l) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  // NW backward waves own the hidden columns; at least two waves, so one
  // forms the next tile's W and marginals while another runs a backward
  constexpr int NT = NW < 2 ? 2 : NW;
  constexpr int KB = kJfKB, GS = kJfGS, nthr = 64 * NT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5, col = lane & 31;
  const int H = a.H, R = a.R, C = a.C, NP = a.NP, NK = 2 * NP, HP = H + 8;
  const int WL = (R * HP + 7) & ~7;
  const int b = blockIdx.x / a.nblk, t0 = 32 * (blockIdx.x - b * a.nblk);
  unsigned short* wol = (unsigned short*)(lds + l.wo);
  float* A = (float*)(lds + l.A);
  float* Bt = (float*)(lds + l.Bt);
  float* AN = (float*)(lds + l.AN);
  float* BN = (float*)(lds + l.BN);
  int* aoff = (int*)(lds + l.aoff);
  int* alink = aoff + NK;
  int* hd = (int*)(lds + l.hd);
  float* gt = (float*)(lds + l.gt);
  float* dpc = (float*)(lds + l.dpc);
  float* wtl = (float*)(lds + l.wt);
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int Fh = min(32, a.T - t0);             // frames of the block in the utterance
  const int Fl = max(0, min(Fh, nf - t0));      // live frames
  const long long row0 = (long long)b * a.T + t0;
  float gb = a.grad ? a.grad[b] : 1.f;
  const float lz = a.log_z[b], nm = a.num[b];
  // an unreachable string (num = -inf) or a dead lattice: no gradient
  // (lt_loss_backward's rule)
  if (!__builtin_isfinite(nm) || !__builtin_isfinite(lz)) gb = 0.f;
  const int hl = min(wave, NW - 1) * 32 + col;  // this lane's hidden column (backward waves)
  float* part = a.part + (long long)blockIdx.x * jf_stride(C, R, H);
  // a forward whose pipeline wait timed out left its checkpoints unfinished:
  // NaN out, never a silent result
  const bool bad = *a.err != 0;
  if (Fl == 0 || gb == 0.f || bad) {  // padding frames / no gradient: zeros out
    const float z = bad ? __builtin_nanf("") : 0.f;
    for (int e = tid; e < 32 * H; e += nthr) {
      const int m = e / H;
      if (m < Fh) a.dpf[(row0 + m) * H + (e - m * H)] = z;
    }
    for (long long e = tid; e < jf_stride(C, R, H); e += nthr) part[e] = z;
    return;
  }
  JSTAMP(a, 0, JCLK());
  // ---- staging: Wo bf16, the checkpoint rows, the string arc table
  stage_wo<SP>(a.wo, wol, R, H, HP, WL, tid, nthr);
  stage_words(A, a.alpha + row0 * C, Fl * C, tid, nthr);
  stage_words(Bt, a.beta + row0 * C, Fl * C, tid, nthr);
  stage_words(AN, a.alpha_num + row0 * NP, Fl * NP, tid, nthr);
  stage_words(BN, a.beta_num + row0 * NP, Fl * NP, tid, nthr);
  stage_words(aoff, a.arcs + (long long)b * 2 * NK, 2 * NK, tid, nthr);
  for (int e = tid; e < C * R; e += nthr) hd[e] = -1;
  for (int e = tid; e < 2 * 32 * GS; e += nthr) gt[e] = 0.f;  // columns past R stay 0
  for (int e = tid; e < C * H; e += nthr) dpc[e] = 0.f;
  // the forward tiles' operands in LDS: e^{2 Pc} (Pc on the direct path)
  // and this block's rows of e^{2 Pf} (Pf for a block over kSplitMax)
  const bool csplit = *a.cbig == 0;
  float* ecl = (float*)(lds + l.ec);
  float* efl = (float*)(lds + l.ef);
  {
    stage_words(ecl, csplit ? a.ec : a.pc, C * H, tid, nthr);
    // rows of one 32-row block of the flattened rows share a source: at most
    // two blocks meet in this one
    const long long fa = row0, fb = row0 + Fh - 1;
    const bool sa = csplit && a.fbig[fa >> 5] == 0, sb = csplit && a.fbig[fb >> 5] == 0;
    if (sa == sb) {
      stage_words(efl, (sa ? a.ef : a.pf) + row0 * H, Fh * H, tid, nthr);
    } else {
      for (int e = tid; e < Fh * H; e += nthr) {
        const long long f = row0 + e / H;
        efl[e] = ((f >> 5) == (fa >> 5) ? (sa ? a.ef : a.pf) : (sb ? a.ef : a.pf))[row0 * H + e];
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < NK; k += nthr)
    if ((alink[k] >> 30) && aoff[k] >= 0) hd[aoff[k]] = k;  // one head per element
  __syncthreads();

  // ---- the forward tiles' lane state: row m = col (frame t0 + m), columns y0 / y1
  const int y0 = col, y1 = 32 + col;
  const bool v1 = y1 < R;
  const float b0 = a.bias[y0], b1 = v1 ? a.bias[y1] : 0.f;
  const unsigned short* w0 = wol + y0 * HP + 8 * half;
  const unsigned short* w1 = wol + (v1 ? y1 : R - 1) * HP + 8 * half;
  const long long fr = row0 + min(col, Fh - 1);
  const bool split = csplit && a.fbig[fr >> 5] == 0;
  const float* pfr = efl + col * H + 8 * half;
  // a block mixing split rows with a direct one (|Pf| > kSplitMax in another
  // 32-row block of the flattened rows) reads Pc from global on the direct rows
  const bool dir_mix = !split && csplit;
  // ---- the backward's lane state (joint_backward_kernel's): Wo as the B
  // operand of gw, this lane's 16 frames' Pf, the d_Pf / d_Wo accumulators
  bf16x8 woh[KB], wolo[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = 16 * kb + 8 * half + j;
      v[j] = r < R ? a.wo[(long long)r * H + hl] : 0.f;
    }
    split8(v, woh[kb], wolo[kb]);
  }
  float pfv[16], dpf[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = (i & 3) + 8 * (i >> 2) + 4 * half;
    pfv[i] = m < Fh ? a.pf[(row0 + m) * H + hl] : 0.f;
    dpf[i] = 0.f;
  }
  f32x16 dwo0 = {}, dwo1 = {};
  float dbias = 0.f;  // thread tid < R: sum of g[:, tid]
  JSTAMP(a, 1, JCLK());
  [[maybe_unused]] long long tf = 0, tc = 0, tb = 0, tw = 0;  // wave 0: W tile, marginals, barrier, backward

  for (int c = 0, buf = 0; c < C; ++c, buf ^= 1) {
    float* g = gt + buf * 32 * GS;
    const long long q0 = JCLK();
    if (wave == c % NT) {
      // W tile of state c: rows = the block's frames, columns = labels
      f32x16 acc0 = {}, acc1 = {};
      const float* pcr = (dir_mix ? a.pc : ecl) + (long long)c * H + 8 * half;
      joint_tile<SP, true>(split, pcr, pfr, H, w0, w1, w0 + WL, w1 + WL, acc0, acc1);
      JWAIT();
      const long long qm = JCLK();
      tf += qm - q0;
      tc -= qm;
      // den - num marginals (marg_tile's arithmetic, no contraction):
      // den = gb e^{alpha + w + beta' - log_z} for every element, straight
      // from the accumulators; then on the few elements with string arcs
      // num = gb sum e^{alpha^n + w + beta^n' - num} over their chain
      // (ascending arc order) and den - num in place
      float* wt = wtl;  // the forward wave's raw W tile (one forward at a time)
      const int q0 = y0 == 0 ? c : y0;        // next(c, y) of the bigram (contexts.py:190-205)
#pragma unroll
      for (int i0 = 0; i0 < 16; i0 += 4) {
        float av[4], bv0[4], bv1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = ((i0 + j) & 3) + 8 * ((i0 + j) >> 2) + 4 * half;
          av[j] = A[m * C + c];
          bv0[j] = Bt[m * C + q0];
          bv1[j] = v1 ? Bt[m * C + y1] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = i0 + j, m = (i & 3) + 8 * (i >> 2) + 4 * half;
          const float x0 = acc0[i] + b0, x1 = acc1[i] + b1;
          wt[m * R + y0] = x0;
          g[m * GS + y0] = m < Fl ? gb * lt_exp(av[j] + x0 + bv0[j] - lz) : 0.f;
          if (v1) {
            wt[m * R + y1] = x1;
            g[m * GS + y1] = m < Fl ? gb * lt_exp(av[j] + x1 + bv1[j] - lz) : 0.f;
          }
        }
      }
      // the labels of row c with string arcs, two at a time (one per half)
      unsigned long long has = __ballot(lane < R && hd[c * R + lane] >= 0);
      while (has) {
        const int ya = __builtin_ctzll(has);
        has &= has - 1;
        const int yb = has ? __builtin_ctzll(has) : -1;
        if (yb >= 0) has &= has - 1;
        const int y = half ? yb : ya;
        if (y >= 0) {
          const int m = col;
          const float w = wt[m * R + y];
          float sacc = 0.f;
          for (int kk = hd[c * R + y]; kk >= 0; kk = (alink[kk] & 0x3fffffff) - 1) {
            const int u = kk >> 1, ub = (kk & 1) ? u + 1 : u;
            sacc += lt_exp(AN[m * NP + u] + w + BN[m * NP + ub] - nm);
          }
          if (m < Fl) g[m * GS + y] = __fsub_rn(g[m * GS + y], __fmul_rn(gb, sacc));
        }
      }
      JWAIT();
      tc += JCLK();
    }
    const long long q1 = JCLK();
    __syncthreads();  // one barrier a tile: the other buffer is written next
    const long long q2 = JCLK();
    tw += q2 - q1;
    if (wave >= NW) continue;  // a forward-only wave
    // ---- backward of tile c (the NW backward waves, each its hidden columns)
    if (tid < R) {  // eight partial sums: the loads in flight together
      float p8[8] = {};
#pragma unroll
      for (int m = 0; m < 32; ++m) p8[m & 7] += g[m * GS + tid];
      dbias += ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
    }
    const float pcv = a.pc[(long long)c * H + hl];
    f32x16 gw = {};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const float4 x0 = *(const float4*)(g + col * GS + 16 * kb + 8 * half);
      const float4 x1 = *(const float4*)(g + col * GS + 16 * kb + 8 * half + 4);
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 ah, al;
      split8(v, ah, al);
      gw = mfma3(ah, al, woh[kb], wolo[kb], gw);
    }
    float csum = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * q + j;
        const float e = __builtin_amdgcn_exp2f((pcv + pfv[i]) * (2.f * kLog2e));
        const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
        hv[j] = t;
        const float d = gw[i] * (1.f - t * t);
        dpf[i] += d;
        csum += d;
      }
      bf16x8 hh, hlo;
      split8(hv, hh, hlo);
      const int tm = 16 * q + 4 * half;
      float gv[8];
      bf16x8 gh8, gl8;
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = g[(tm + (j & 3) + 8 * (j >> 2)) * GS + col];
      split8(gv, gh8, gl8);
      dwo0 = mfma3(gh8, gl8, hh, hlo, dwo0);
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = g[(tm + (j & 3) + 8 * (j >> 2)) * GS + 32 + col];
      split8(gv, gh8, gl8);
      dwo1 = mfma3(gh8, gl8, hh, hlo, dwo1);
    }
    csum += __shfl_xor(csum, 32);
    if (half == 0) dpc[c * H + hl] += csum;  // this wave owns column hl
    tb += JCLK() - q2;
  }
  JSTAMP(a, 2, JCLK());
  JSTAMP(a, 4, tf);
  JSTAMP(a, 5, tc);
  JSTAMP(a, 6, tw);
  JSTAMP(a, 7, tb);
  // ---- outputs: d_Pf rows (the block owns its frames), the partials
  if (wave < NW) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = (i & 3) + 8 * (i >> 2) + 4 * half;
      if (m < Fh) a.dpf[(row0 + m) * H + hl] = dpf[i];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = (i & 3) + 8 * (i >> 2) + 4 * half;
      if (r < R) part[(long long)(C + r) * H + hl] = dwo0[i];
      if (r + 32 < R) part[(long long)(C + r + 32) * H + hl] = dwo1[i];
    }
  }
  if (tid < R) part[(long long)(C + R) * H + tid] = dbias;
  __syncthreads();
  for (int e = tid; e < C * H; e += nthr) part[e] = dpc[e];
  JSTAMP(a, 3, JCLK());
}

// out[e] = sum over the blocks' partials in a fixed order (joint_reduce_kernel's
// scheme): d_Pc [C H] | d_Wo [R H] | d_bias [R]
__global__ __launch_bounds__(256) void jf_reduce_kernel(const float* part, int nparts,
                                                        long long stride, long long npc,
                                                        long long nwo, int R, float* dpc,
                                                        float* dwo, float* dbias) {
  const long long n = npc + nwo + R;
  const int lane = threadIdx.x & 63;
  for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < n;
       e += ((long long)gridDim.x * blockDim.x) >> 6) {
    float s = 0.f;
    for (int p = lane; p < nparts; p += 64) s += part[(long long)p * stride + e];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) {
      if (e < npc) dpc[e] = s;
      else if (e < npc + nwo) dwo[e - npc] = s;
      else dbias[e - npc - nwo] = s;
    }
  }
}

// ---- host side ---------------------------------------------------------------
// The forward's state (lt_loss_joint_forward -> _backward): the flags, e^{2 Pc},
// e^{2 Pf}, the pipe's checkpoints and arc table, log_z and num.
struct JfState {
  size_t cbig, fbig, ec, ef, alpha, beta, an, bn, arcs, lz, num, err, total;
};
JfState jf_state(const lt_problem* pb, int H) {
  auto up = [](long long x) { return (size_t)((x + 255) & ~255LL); };
  const long long B = pb->batch, BT = B * pb->max_frames, C = pb->vocab_size + 1,
                  NP = pb->max_labels + 1;
  JfState s;
  size_t o = 0;
  s.cbig = o; o += up(4);
  s.fbig = o; o += up(4 * ((BT + 31) / 32 + 1));
  s.ec = o; o += up(4 * C * H);
  s.ef = o; o += up(4 * BT * H);
  s.alpha = o; o += up(4 * BT * C);
  s.beta = o; o += up(4 * BT * C);
  s.an = o; o += up(4 * BT * NP);
  s.bn = o; o += up(4 * BT * NP);
  s.arcs = o; o += up(4 * B * 4 * NP);
  s.lz = o; o += up(4 * B);
  s.num = o; o += up(4 * B);
  s.err = o; o += up(4);
  s.total = o;
  return s;
}
size_t jf_scratch(const lt_problem* pb, int H) {
  const long long C = pb->vocab_size + 1, R = C;
  const long long nblk = (pb->max_frames + 31) / 32;
  return (size_t)(4 * pb->batch * nblk * jf_stride((int)C, (int)R, H) + 256);
}

int jf_check(const lt_problem* pb, const lt_joint_params* jp) {
  if (!pb || !jp) return lt_impl::set_error(LT_EINVAL, "joint loss: null problem / params");
  if (pb->batch < 0 || pb->max_frames < 0 || pb->max_labels < 0)
    return lt_impl::set_error(LT_EINVAL, "joint loss: negative shape");
  if (pb->context_size != 1 || pb->vocab_size <= 16 || pb->vocab_size > 32 ||
      pb->weight_dtype != LT_DTYPE_F32)
    return lt_impl::set_error(LT_EUNSUPPORTED,
                              "joint loss: FullNGram n = 1, 16 < vocab_size <= 32, fp32");
  if (jp->hidden < 32 || jp->hidden > 256 || jp->hidden % 32)
    return lt_impl::set_error(LT_EUNSUPPORTED, "joint loss: hidden in {32, 64, ..., 256}");
  if (jp->precision != LT_JOINT_SPLIT && jp->precision != LT_JOINT_BF16)
    return lt_impl::set_error(LT_EINVAL, "joint loss: precision LT_JOINT_SPLIT or LT_JOINT_BF16");
  if (!lt_impl::pipe_eligible(pb) || pb->max_labels + 1 > 128)
    return lt_impl::set_error(LT_EUNSUPPORTED, "joint loss: max_labels < 128");
  const JfLds l = jf_lds(pb->vocab_size + 1, pb->vocab_size + 1, jp->hidden, pb->max_labels + 1,
                         jp->precision == LT_JOINT_SPLIT);
  if (l.total > 160 * 1024) return lt_impl::set_error(LT_EUNSUPPORTED, "joint loss: LDS");
  return LT_OK;
}

__global__ __launch_bounds__(64) void jf_err_kernel(const int* err, float* loss, float* lz,
                                                     float* num, int B) {
  if (*err == 0) return;
  const float nan = __builtin_nanf("");
  for (int b = threadIdx.x; b < B; b += 64) {
    loss[b] = nan;
    lz[b] = nan;
    num[b] = nan;
  }
}

template <int NW>
int jf_launch_marg(const JFArgs& a, const JfLds& l, bool sp, hipStream_t st) {
  const void* k = sp ? (const void*)jf_marg_kernel<NW, true> : (const void*)jf_marg_kernel<NW, false>;
  if (l.total > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, l.total);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  const int grid = a.B * a.nblk;
  const int threads = 64 * (NW < 2 ? 2 : NW);
  if (sp)
    hipLaunchKernelGGL((jf_marg_kernel<NW, true>), dim3(grid), dim3(threads), l.total, st, a, l);
  else
    hipLaunchKernelGGL((jf_marg_kernel<NW, false>), dim3(grid), dim3(threads), l.total, st, a, l);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
}

}  // namespace

extern "C" {

int lt_loss_joint_workspace_bytes(const lt_problem* pb, const lt_joint_params* jp,
                                  size_t* state_bytes, size_t* scratch_bytes) {
  if (int rc = jf_check(pb, jp)) return rc;
  if (state_bytes) *state_bytes = jf_state(pb, jp->hidden).total;
  if (scratch_bytes) *scratch_bytes = jf_scratch(pb, jp->hidden);
  return LT_OK;
}

int lt_loss_joint_forward(const lt_problem* pb, const lt_joint_params* jp,
                          const int32_t* num_frames, const int32_t* labels,
                          const int32_t* num_labels, float* loss, float* log_z, float* num,
                          void* state, size_t state_bytes, void* stream) {
  if (int rc = jf_check(pb, jp)) return rc;
  const int H = jp->hidden, C = pb->vocab_size + 1;
  const JfState s = jf_state(pb, H);
  if (pb->batch == 0) return LT_OK;
  if (!num_frames || !num_labels || !loss || (pb->max_labels > 0 && !labels) || !state ||
      !jp->ctx_proj || !jp->out_weight || !jp->out_bias ||
      (pb->max_frames > 0 && !jp->frame_proj))
    return lt_impl::set_error(LT_EINVAL, "joint loss: null pointer");
  if (((uintptr_t)jp->ctx_proj | (uintptr_t)jp->frame_proj | (uintptr_t)state) & 15)
    return lt_impl::set_error(LT_EINVAL, "joint loss: projections / state must be 16-byte aligned");
  if (state_bytes < s.total) return lt_impl::set_error(LT_EINVAL, "joint loss: state too small");
  hipStream_t st = (hipStream_t)stream;
  char* sb = (char*)state;
  const long long BT = (long long)pb->batch * pb->max_frames;
  hipError_t e = hipMemsetAsync(sb + s.cbig, 0, s.ec - s.cbig, st);  // the flags
  if (e == hipSuccess) e = hipMemsetAsync(sb + s.err, 0, sizeof(int), st);  // the timeout word
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  {
    long long nc4 = (long long)C * H / 4, nf4 = BT * H / 4;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = (int)std::max<long long>(1, std::min<long long>((nc4 + nf4 + 255) / 256, 8LL * cus));
    hipLaunchKernelGGL(jf_prep_kernel, dim3(grid), dim3(256), 0, st, jp->ctx_proj, jp->frame_proj,
                       (float*)(sb + s.ec), (float*)(sb + s.ef), (int*)(sb + s.cbig),
                       (int*)(sb + s.fbig), nc4, nf4, H);
    if ((e = hipGetLastError()) != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  lt_impl::JointOps jo;
  jo.H = H;
  jo.prod = jp->precision == LT_JOINT_SPLIT ? 1 : 2;
  jo.pc = jp->ctx_proj; jo.ec = (const float*)(sb + s.ec);
  jo.pf = jp->frame_proj; jo.ef = (const float*)(sb + s.ef);
  jo.cbig = (const int*)(sb + s.cbig); jo.fbig = (const int*)(sb + s.fbig);
  jo.wo = jp->out_weight; jo.bias = jp->out_bias;
  float* lz = (float*)(sb + s.lz);
  float* nm = (float*)(sb + s.num);
  int rc = lt_impl::launch_pipe(pb, 0, nullptr, num_frames, labels, num_labels, loss, lz, nm,
                                (float*)(sb + s.alpha), (float*)(sb + s.an),
                                (float*)(sb + s.beta), (float*)(sb + s.bn), (int32_t*)(sb + s.arcs),
                                2, (int*)(sb + s.err), stream, nullptr, 0, nullptr, &jo);
  if (rc) return rc;
  // a pipeline wait that timed out (the pipe raised its abort and drained):
  // loss, log_z and num NaN, and the backward NaN too (jf_marg_kernel)
  hipLaunchKernelGGL(jf_err_kernel, dim3(1), dim3(64), 0, st, (const int*)(sb + s.err), loss, lz,
                     nm, (int)pb->batch);
  if ((e = hipGetLastError()) != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  if (log_z && (e = hipMemcpyAsync(log_z, lz, 4 * pb->batch, hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  if (num && (e = hipMemcpyAsync(num, nm, 4 * pb->batch, hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

int lt_loss_joint_backward(const lt_problem* pb, const lt_joint_params* jp,
                           const int32_t* num_frames, const float* grad, float* d_ctx_proj,
                           float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                           void* state, size_t state_bytes, void* scratch, size_t scratch_bytes,
                           void* stream) {
  if (int rc = jf_check(pb, jp)) return rc;
  const int H = jp->hidden, C = pb->vocab_size + 1, R = C;
  const JfState s = jf_state(pb, H);
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (pb->batch == 0 || pb->max_frames == 0) {
    e = hipMemsetAsync(d_ctx_proj, 0, 4 * (size_t)C * H, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_out_weight, 0, 4 * (size_t)R * H, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_out_bias, 0, 4 * (size_t)R, st);
    return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  if (!num_frames || !d_ctx_proj || !d_frame_proj || !d_out_weight || !d_out_bias || !state ||
      !scratch || !jp->ctx_proj || !jp->frame_proj || !jp->out_weight || !jp->out_bias)
    return lt_impl::set_error(LT_EINVAL, "joint loss backward: null pointer");
  if (state_bytes < s.total || scratch_bytes < jf_scratch(pb, H))
    return lt_impl::set_error(LT_EINVAL, "joint loss backward: workspace too small");
  const char* sb = (const char*)state;
  JFArgs a;
  a.pc = jp->ctx_proj; a.ec = (const float*)(sb + s.ec);
  a.pf = jp->frame_proj; a.ef = (const float*)(sb + s.ef);
  a.wo = jp->out_weight; a.bias = jp->out_bias;
  a.cbig = (const int*)(sb + s.cbig); a.fbig = (const int*)(sb + s.fbig);
  a.nfr = num_frames;
  a.alpha = (const float*)(sb + s.alpha); a.beta = (const float*)(sb + s.beta);
  a.alpha_num = (const float*)(sb + s.an); a.beta_num = (const float*)(sb + s.bn);
  a.arcs = (const int*)(sb + s.arcs);
  a.log_z = (const float*)(sb + s.lz); a.num = (const float*)(sb + s.num);
  a.grad = grad;
  a.err = (const int*)(sb + s.err);
  a.dpf = d_frame_proj;
  a.part = (float*)scratch;
  a.stamps = nullptr;
#ifdef LT_STAMPS
  {
    const char* sp = lt_impl::tune_str("LT_JSTAMPS_PTR");
    a.stamps = sp ? (long long*)strtoull(sp, nullptr, 0) : nullptr;
  }
#endif
  a.B = pb->batch; a.T = pb->max_frames; a.U = pb->max_labels; a.C = C; a.R = R; a.H = H;
  a.NP = pb->max_labels + 1;
  a.nblk = (pb->max_frames + 31) / 32;
  const bool sp = jp->precision == LT_JOINT_SPLIT;
  const JfLds l = jf_lds(C, R, H, a.NP, sp);
  int rc;
  switch (H / 32) {
    case 1: rc = jf_launch_marg<1>(a, l, sp, st); break;
    case 2: rc = jf_launch_marg<2>(a, l, sp, st); break;
    case 3: rc = jf_launch_marg<3>(a, l, sp, st); break;
    case 4: rc = jf_launch_marg<4>(a, l, sp, st); break;
    case 5: rc = jf_launch_marg<5>(a, l, sp, st); break;
    case 6: rc = jf_launch_marg<6>(a, l, sp, st); break;
    case 7: rc = jf_launch_marg<7>(a, l, sp, st); break;
    default: rc = jf_launch_marg<8>(a, l, sp, st); break;
  }
  if (rc) return rc;
  long long stride = jf_stride(C, R, H), npc = (long long)C * H, nwo = (long long)R * H;
  int nparts = a.B * a.nblk;
  const int rg = (int)std::min<long long>((npc + nwo + R + 3) / 4, 8192);  // a wave per element
  hipLaunchKernelGGL(jf_reduce_kernel, dim3(rg), dim3(256), 0, st, (const float*)scratch, nparts,
                     stride, npc, nwo, R, d_ctx_proj, d_out_weight, d_out_bias);
  e = hipGetLastError();
  return e == hipSuccess ? LT_OK : lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
}

int lt_loss_grad_joint(const lt_problem* pb, const lt_joint_params* jp, const int32_t* num_frames,
                       const int32_t* labels, const int32_t* num_labels, const float* grad,
                       float* loss, float* log_z, float* num, float* d_ctx_proj,
                       float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                       void* workspace, size_t workspace_bytes, void* stream) {
  size_t stb = 0, scb = 0;
  if (int rc = lt_loss_joint_workspace_bytes(pb, jp, &stb, &scb)) return rc;
  if (workspace_bytes < stb + scb)
    return lt_impl::set_error(LT_EINVAL, "lt_loss_grad_joint: workspace too small");
  if (int rc = lt_loss_joint_forward(pb, jp, num_frames, labels, num_labels, loss, log_z, num,
                                     workspace, stb, stream))
    return rc;
  return lt_loss_joint_backward(pb, jp, num_frames, grad, d_ctx_proj, d_frame_proj, d_out_weight,
                                d_out_bias, workspace, stb, (char*)workspace + stb, scb, stream);
}

}  // extern "C"
