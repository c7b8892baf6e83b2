// lt_tri.hip -- the trigram checkpointing recursions (FullNGram n = 2,
// V <= 32, Log, W staged in LDS): alpha and beta of every utterance side by
// side in one launch (workgroups [0, B) forward, [B, 2B) backward), as
// fwdbwd_kernel, with the den role of den_fwd_tri / den_bwd_tri
// (lt_kernels.h): one lane per destination pair (forward) or source pair
// (backward), every term of a state in that lane's registers. The numerator
// and loader roles are fwd_body / bwd_body's own. lattices.py:379-496 and
// 686-799 (alignments.py:286-318, contexts.py:207-256).
//
// The overlap (tri_mix_kernel, lt_loss_grad's trigram V = 32 route, round 6):
// the 2B recursion workgroups hold 2B CUs for the whole call while the rest of
// the chip idles, and the marginal pass (marg_kernel) used to run only after
// them. Here the launch also carries one marginal workgroup per idle CU. A
// frame's marginals need alpha_t and beta_{t+1} only, so frames become ready
// from the middle of the utterance outwards once both recursions have passed
// it (alignments.py:300-318: each frame's marginals are the reference's
// FrameDependent.backward of that frame). The recursions publish their
// checkpoint rows every kTriPub frames (KArgs::prog); a marginal workgroup
// takes the frames of the utterances whose two recursion workgroups share its
// XCD (their plain row stores sit in that XCD's L2, which its sc1 loads read),
// in the order they become ready, and marks each frame done. marg_kernel then
// runs as before on the frames not done (the others return at once), so a
// placement that shares no XCD or a wait that times out only moves work back
// to it. Every frame is normalised by log Z and the string's weight taken
// from the rows at the middle frame m = nf / 2 (alpha_m . beta_m,
// tri_mid_norm: the same fixed-order wave reduction in both kernels), so the
// result does not depend on which kernel took a frame.
#include "lt_kernels.h"

namespace {
// VT = 32: V a compile-time constant; VT = 1: any V <= 32
template <bool BF16, int VT>
__global__ __launch_bounds__(1024) void tri_fwdbwd_kernel(const KArgs af, const KArgs ab, int nb) {
  // diagnostic builds: LT_DBG 16 / 32 time one direction alone (results wrong)
  if ((int)blockIdx.x < nb) {
    if (!LT_ABL(af, 16)) fwd_body<M_LOG, BF16, true, 2, 9, VT>(af, blockIdx.x);
  } else if (!LT_ABL(af, 32)) {
    bwd_body<BF16, true, false, 2, 9, true, (int)sizeof(KArgs), VT>(ab, blockIdx.x - nb);
  }
}

LT_DEVINL unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
// diagnostic time stamps: the low 30 bits of the 100 MHz real-time counter
LT_DEVINL unsigned mix_rt() { return (unsigned)__builtin_amdgcn_s_memrealtime() & 0x3fffffffu; }
LT_DEVINL float uniform_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
LT_DEVINL unsigned ld_u32_sc1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
LT_DEVINL float ld_f32_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// n <= 64 NQ floats of a row into LDS: NQ sc1 buffer loads per lane issued
// together (a relaxed atomic load per element waits one latency each)
template <int NQ>
LT_DEVINL void row_sc1(const float* src, int n, float* dst, int lane) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 4 * n, 0x00020000);
  float v[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i)
    v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * (lane + 64 * i), 0, 0x10));
#pragma unroll
  for (int i = 0; i < NQ; ++i)
    if (lane + 64 * i < n) dst[lane + 64 * i] = v[i];
}
constexpr unsigned kMixSpins = 1u << 22;  // ~1 s of polling, then the frames go back to marg_kernel
constexpr int kMixUnits = 5;              // 16-byte units of W in flight per thread
constexpr int kMixUtt = 8;                // utterances a marginal workgroup keeps arc tables for

}  // namespace

namespace {

// One frame's marginals by ONE wave (every wave of a marginal workgroup takes
// frames on its own: no workgroup barrier, so one wave's memory latency
// hides behind the others): the frame's rows into the wave's LDS region, den
// elements with marg_tile's expressions stored by 16-byte units, then the
// string's chain heads rewrite their elements as den - num once the wave's
// own stores of the frame have completed (marg_tile's phase 2).
template <bool BF16>
LT_DEVINL void mix_frame(const MixArgs& m, int b, int t, float lz, float nm, float* A, float* Bt,
                         float* AN, float* BN, const int* aoff, const int* alink, const int* nbt,
                         int lane) {
  constexpr int VE = BF16 ? 8 : 4, ES = BF16 ? 2 : 4;
  constexpr int R = 33, C = 1 + 32 + 32 * 32, FR = C * R;
  const int NP = m.U + 1, NK = 2 * NP;
  {
    // the four rows by sc1 buffer loads (L1 bypassed: another workgroup of
    // this launch wrote them), every load in flight before the first LDS write.
    // Lanes read each other's row entries, so the hand-offs through the
    // wave's LDS region are wavefront-scope fences (a wave barrier alone
    // orders no memory for the compiler): the previous frame's reads before
    // these writes, these writes before this frame's reads
    const long long rc = ((long long)b * m.T + t) * C, rn = ((long long)b * m.T + t) * NP;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    row_sc1<17>(m.alpha + rc, C, A, lane);
    row_sc1<17>(m.beta + rc, C, Bt, lane);
    row_sc1<2>(m.alpha_num + rn, NP, AN, lane);
    row_sc1<2>(m.beta_num + rn, NP, BN, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this wave's row writes, before any lane reads them
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (m.dbg & 64) return;  // diagnostic: the rows only
  const float gb = m.grad ? m.grad[b] : 1.f;
  const long long base = ((long long)b * m.T + t) * FR;
  const int h0 = (int)(((16 - ((base * ES) & 15)) & 15) / ES);
  const int nunits = (FR - h0) / VE;
  const int ntail = h0 + (FR - h0 - nunits * VE);
  const unsigned char* Wu = m.W + (base + h0) * ES;
  unsigned char* dWu = (unsigned char*)m.dW + (base + h0) * ES;
  auto den_el = [&](int el, float w) {
    const int p = el / R, y = el - p * R;
    const int q = y == 0 ? p : nbt[p] + y;
    return gb * lt_exp(A[p] + w + Bt[q] - lz);
  };
  for (int u0 = lane; u0 < nunits; u0 += kMixUnits * 64) {
    uint4 wq[kMixUnits];
#pragma unroll
    for (int r = 0; r < kMixUnits; ++r) {
      const int u = min(u0 + r * 64, nunits - 1);  // every load issued (clamped): one wait
      if (m.dbg & 256) wq[r] = make_uint4(u, u, u, u);  // diagnostic: no W loads
      else if (m.dbg & 1024) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u q = __builtin_nontemporal_load((const v4u*)(Wu + (long long)u * 16));
        wq[r] = make_uint4(q.x, q.y, q.z, q.w);
      }
      else wq[r] = *(const uint4*)(Wu + (long long)u * 16);
    }
#pragma unroll
    for (int r = 0; r < kMixUnits; ++r) {
      const int u = u0 + r * 64;
      if (u >= nunits) break;
      float w[VE], v[VE];
      unpack_unit<BF16>(wq[r], w);
      const int e0 = h0 + u * VE;
      const int p = e0 / R;
      const int y = e0 - p * R;
      // a unit spans at most two source rows (R >= VE)
      const int p1 = min(p + 1, C - 1);
      const float a0v = A[p], a1v = A[p1];
      const int nb0 = nbt[p], nb1 = nbt[p1];
#pragma unroll
      for (int c = 0; c < VE; ++c) {
        const int yc = y + c;
        const bool w2 = yc >= R;
        const int yy = w2 ? yc - R : yc;
        const int pp = w2 ? p1 : p;
        const int q = yy == 0 ? pp : (w2 ? nb1 : nb0) + yy;
        const float av = w2 ? a1v : a0v;
        v[c] = gb * lt_exp(av + w[c] + Bt[q] - lz);
      }
      if (m.dbg & 128) {  // diagnostic: no dW stores (one conditional store keeps the math)
        if (v[0] == 12345.f) store_unit<BF16>(dWu + (long long)u * 16, v);
      } else if (BF16 && (m.dbg & 512)) {  // diagnostic: plain (temporal) stores
        unsigned q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          q[i] = f2bf(v[(2 * i) % VE]) | ((unsigned)f2bf(v[(2 * i + 1) % VE]) << 16);
        *(uint4*)(dWu + (long long)u * 16) = make_uint4(q[0], q[1], q[2], q[3]);
      } else {
        store_unit<BF16>(dWu + (long long)u * 16, v);
      }
    }
  }
  for (int i = lane; i < ntail; i += 64) {
    const int e = i < h0 ? i : i + nunits * VE;
    stw<BF16>(m.dW, base + e, den_el(e, ldw<BF16>(m.W + base * ES, e)));
  }
  // the chain heads rewrite their elements once the wave's stores of the
  // frame have completed (same wave, same address)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int k = lane; k < NK; k += 64) {
    const int o = aoff[k];
    if (o < 0 || !(alink[k] >> 30)) continue;
    const float wv = ldw<BF16>(m.W + base * ES, o);
    float sacc = 0.f;
    for (int kk = k; kk >= 0; kk = (alink[kk] & 0x3fffffff) - 1) {
      const int u = kk >> 1;
      const float bn = BN[(kk & 1) ? u + 1 : u];
      sacc += lt_exp(AN[u] + wv + bn - nm);
    }
    stw<BF16>(m.dW, base + o, den_el(o, wv) - gb * sacc);
  }
}

__host__ __device__ inline int al16i(int x) { return (x + 15) & ~15; }
// the marginal role's shared LDS (the utterances' tables) and one wave's rows
__host__ __device__ inline int mix_shared_bytes(int C, int NP, int B) {
  return al16i(4 * (C + kMixUtt * 4 * NP + 2 * (NP + 1) + B + 4 + 16 * 2 * kMixUtt));
}
__host__ __device__ inline int mix_row_bytes(int C, int NP) { return al16i(4 * (2 * C + 2 * NP)); }

// The marginal role of tri_mix_kernel (blocks [2B, grid)): the workgroup
// builds the tables of the utterances on its XCD, then every wave takes
// frames through the XCD's job counter on its own.
template <bool BF16>
LT_DEVINL void mix_marg(const MixArgs& m_in, unsigned char* lds, int lds_bytes) {
#ifdef LT_MIX_NODBG
  // diagnostic: the switches folded away. This build gives wrong chain-head
  // elements on every frame after a wave's first ("Open item")
  MixArgs m = m_in;
  m.dbg = 0;
#else
  const MixArgs& m = m_in;
#endif
  const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int B = m.B, C = m.g.C, NP = m.U + 1, NK = 2 * NP;
  int* nbt = (int*)lds;                  // [C] next_base of each state
  int* tabs = nbt + C;                   // [kMixUtt][2 NK] arc tables (offsets, links) by list slot
  int* ctx = tabs + kMixUtt * 2 * NK;    // [NP + 1]
  int* ylab = ctx + NP + 1;              // [NP + 1]
  int* list = ylab + NP + 1;             // [B] the utterances this XCD's marginal workgroups take
  int* sh = list + B;                    // [0] list length
  float* shf = (float*)(sh + 4);         // [16][2 kMixUtt] per wave: log Z, num by slot (NaN: not yet)
  const int shared = mix_shared_bytes(C, NP, B), rowb = mix_row_bytes(C, NP);
  int nwork = min(nthr >> 6, (lds_bytes - shared) / rowb);
  if (m.dbg & 2048) nwork = min(nwork, 8);  // diagnostic: fewer marginal waves
  if (m.dbg & 4096) nwork = min(nwork, 4);
  if (m.dbg & 1) return;
  const unsigned own = xcc_id() + 1;
  for (int p = tid; p < C; p += nthr) {
    bool z;
    nbt[p] = next_base(m.g, p, &z);
  }
  for (int i = tid; i < 16 * 2 * kMixUtt; i += nthr) shf[i] = __builtin_nanf("");
  if (tid == 0) {
    // the recursion workgroups' XCD ids (each writes its own at its start)
    int n = 0, abort = 0;
    for (int b = 0; b < B && !abort; ++b) {
      unsigned xf = 0, xb = 0;
      for (unsigned spins = 0; (xf == 0 || xb == 0) && spins < kMixSpins; ++spins) {
        xf = ld_u32_sc1(m.xcc + b);
        xb = ld_u32_sc1(m.xcc + B + b);
        if (xf == 0 || xb == 0) __builtin_amdgcn_s_sleep(8);
      }
      if (xf == 0 || xb == 0) abort = 1;
      int nf = m.nfr[b];
      nf = nf < 0 ? 0 : (nf > m.T ? m.T : nf);
      if (xf == own && xb == own && nf >= 2 && n < kMixUtt) list[n++] = b;
    }
    sh[0] = abort ? 0 : n;  // (past kMixUtt on one XCD: marg_kernel takes the rest)
  }
  __syncthreads();
  const int n = sh[0];
  if (n == 0 || nwork < 1) return;
  // every listed utterance's string arc table (marg_kernel's,
  // write_arc_table: contexts.py:109-146 walk, lattices.py:314-338 arcs)
  for (int k2 = 0; k2 < n; ++k2) {
    const int b = list[k2];
    for (int u = tid; u < m.U; u += nthr) ylab[u] = m.labels[(long long)b * m.U + u];
    __syncthreads();
    if (tid == 0) {
      const int Rr = m.g.V + 1;
      int c = 0;
      for (int u = 0; u <= m.U; ++u) {
        ctx[u] = c * Rr;
        if (u < m.U) {
          int y = ylab[u];
          if (y < 0 || y > m.g.V) y = 0;
          ylab[u] = y < 1 ? 1 : y;
          if (y != 0) {
            bool z;
            const int nb = next_base(m.g, c, &z);
            c = z ? 0 : nb + y;
          }
        } else {
          ylab[u] = 1;
        }
      }
    }
    __syncthreads();
    auto arc = [&](int k) {
      const int u = k >> 1;
      return (k & 1) == 0 ? ctx[u] : (u < m.U ? ctx[u] + ylab[u] : -1);
    };
    int* aoff = tabs + k2 * 2 * NK;
    int* alink = aoff + NK;
    for (int k = tid; k < NK; k += nthr) {
      const int o = arc(k);
      int head = o >= 0 ? 1 : 0, nxt = -1;
      if (o >= 0)
        for (int kk = 0; kk < NK; ++kk) {
          if (arc(kk) != o) continue;
          if (kk < k) head = 0;
          else if (kk > k && nxt < 0) nxt = kk;
        }
      aoff[k] = o;
      alink[k] = (head << 30) | (nxt + 1);
    }
    __syncthreads();
  }
  if (wave >= nwork) return;
  float* A = (float*)(lds + shared + wave * rowb);
  float* Bt = A + C;
  float* AN = Bt + C;
  float* BN = AN + NP;
  const int smax = (m.T + 1) / 2;
  unsigned* ctr = m.ctr + 32 * ((own - 1) & 7);  // this XCD's job counter (its own 128-byte line)
  for (;;) {
    int job = -1;
    if (lane == 0) {
      // the next job of this XCD: step s outwards from the middle, utterance
      // list[slot], the frame after (side 0) or before (side 1) the middle
      int j = 0, b = 0, t = -1, nf = 0, mid = 0, slot = 0;
      for (;;) {
        j = (int)atomicAdd(ctr, 1u);
        const int s = j / (2 * n), r = j - s * 2 * n;
        if (s >= smax) { t = -1; break; }
        slot = r >> 1;
        b = list[slot];
        nf = m.nfr[b];
        nf = nf < 0 ? 0 : (nf > m.T ? m.T : nf);
        mid = nf / 2;
        t = (r & 1) ? mid - 1 - s : mid + s;
        if (t >= 0 && t < nf) break;
      }
      if (t >= 0) {
        // frame t needs alpha row t and beta row t (beta_{t+1}); the middle
        // norm alpha row mid and beta row mid - 1
        unsigned need_f = (unsigned)max(t + 1, mid + 1);
        unsigned need_b = (unsigned)max(nf - 1 - t, nf - mid);
        if (m.dbg & 2) need_f = need_b = (unsigned)nf;  // diagnostic: wait for the whole recursions
        unsigned spins = 0;
        while ((ld_u32_sc1(m.prog + 2 * b) < need_f || ld_u32_sc1(m.prog + 2 * b + 1) < need_b) &&
               ++spins < kMixSpins) {
          if (m.dbg & 32) __builtin_amdgcn_s_sleep(127);
          else __builtin_amdgcn_s_sleep(8);
        }
        // a recursion that never came: marg_kernel takes the frame
        job = spins >= kMixSpins ? -1 : (slot << 26 | b << 16 | t);
      }
    }
    job = __builtin_amdgcn_readfirstlane(job);
    if (job < 0) return;
    const int slot = job >> 26, b = (job >> 16) & 1023, t = job & 0xffff;
    // the slot's norm as this wave computed it before (each wave keeps its
    // own copy: no LDS word is written by one wave while another reads it),
    // taken wave-uniform
    float* wn = shf + wave * 2 * kMixUtt + 2 * slot;
    float lz = uniform_f(wn[0]), nm = uniform_f(wn[1]);
    if (__builtin_isnan(lz) || __builtin_isnan(nm)) {
      // this utterance's middle norm (its rows are final: the job's wait
      // covered them), once per wave and utterance
      int nf = m.nfr[b];
      nf = nf < 0 ? 0 : (nf > m.T ? m.T : nf);
      const int mid = nf / 2;
      const long long r0 = (long long)b * m.T;
      const float2 zn = tri_mid_norm(m.alpha + (r0 + mid) * C, m.beta + (r0 + mid - 1) * C,
                                     m.alpha_num + (r0 + mid) * NP,
                                     m.beta_num + (r0 + mid - 1) * NP, C, NP, lane, true);
      lz = uniform_f(zn.x);
      nm = uniform_f(zn.y);
      if (lane == 0) {
        wn[0] = lz;
        wn[1] = nm;
      }
    }
    // a frame whose norm is not finite (an unreachable string, a dead
    // lattice) stays with marg_kernel, which zeroes it
    if (__builtin_isfinite(lz) && __builtin_isfinite(nm)) {
      const int* aoff = tabs + slot * 2 * NK;
      mix_frame<BF16>(m, b, t, lz, nm, A, Bt, AN, BN, aoff, aoff + NK, nbt, lane);
      // (diagnostic dbg 4: the frame is left to marg_kernel all the same)
      if (lane == 0 && !(m.dbg & 4))
        m.done[(long long)b * m.T + t] =
            (m.dbg & 8) ? (int)own
                        : (m.dbg & 16) ? (int)(mix_rt() | 0x40000000u) : 1;
    }
  }
}

// The recursions and the marginal workgroups in one launch: blocks [0, nb)
// forward, [nb, 2 nb) checkpointing backward (each publishing its XCD id and
// its progress), [2 nb, grid) marginals.
template <bool BF16>
__global__ __launch_bounds__(1024) void tri_mix_kernel(const KArgs af, const KArgs ab, int nb,
                                                       const MixArgs mx) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int x = blockIdx.x;
  if (x < 2 * nb) {
    const bool stamp = (mx.dbg & 16) && mx.ts && threadIdx.x == 0;
    if (stamp) mx.ts[x] = mix_rt();
    if (threadIdx.x == 0)
      __hip_atomic_store(mx.xcc + x, xcc_id() + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x < nb) fwd_body<M_LOG, BF16, true, 2, 9, 32>(af, x);
    else bwd_body<BF16, true, false, 2, 9, true, (int)sizeof(KArgs), 32>(ab, x - nb);
    if (stamp) mx.ts[2 * nb + x] = mix_rt();
    return;
  }
  mix_marg<BF16>(mx, lds, mx.lds_bytes);
}
}  // namespace

namespace lt_impl {
int launch_tri_fwdbwd(const Plan& pf, const Plan& pb, bool bf16, int nb, hipStream_t st) {
  if (nb == 0) return LT_OK;
  const bool v32 = pf.a.g.V == 32;
  const void* k = bf16 ? (v32 ? (const void*)tri_fwdbwd_kernel<true, 32>
                              : (const void*)tri_fwdbwd_kernel<true, 1>)
                       : (v32 ? (const void*)tri_fwdbwd_kernel<false, 32>
                              : (const void*)tri_fwdbwd_kernel<false, 1>);
  const int lds = pf.lds_bytes > pb.lds_bytes ? pf.lds_bytes : pb.lds_bytes;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  KArgs af = pf.a, ab = pb.a;
  void* args[] = {(void*)&af, (void*)&ab, (void*)&nb};
  e = hipLaunchKernel(k, dim3(2 * nb), dim3(pf.threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

// LDS bytes the marginal role wants (mix_marg: its tables and a row region
// for every wave of a 1024-thread workgroup, capped at the CU's 160 KB)
int tri_mix_lds(const NGram& g, int U, int B) {
  const int NP = U + 1;
  return std::min(160 * 1024, mix_shared_bytes(g.C, NP, B) + 16 * mix_row_bytes(g.C, NP));
}

int launch_tri_mix(const Plan& pf, const Plan& pb, bool bf16, int nb, int marg_blocks,
                   const MixArgs& mx, hipStream_t st) {
  if (nb == 0) return LT_OK;
  if (!mx.W || !mx.nfr || !mx.alpha || !mx.beta || !mx.alpha_num || !mx.beta_num || !mx.dW ||
      !mx.prog || !mx.xcc || !mx.ctr || !mx.done || (mx.U > 0 && !mx.labels) ||
      pf.a.prog != mx.prog || pb.a.prog != mx.prog || mx.g.V != 32 || mx.g.n != 2 || mx.B != nb)
    return set_error(LT_EINVAL, "trigram overlap: incomplete arguments");
  const void* k = bf16 ? (const void*)tri_mix_kernel<true> : (const void*)tri_mix_kernel<false>;
  int lds = pf.lds_bytes > pb.lds_bytes ? pf.lds_bytes : pb.lds_bytes;
  lds = std::max(lds, tri_mix_lds(mx.g, mx.U, mx.B));
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  KArgs af = pf.a, ab = pb.a;
  MixArgs m = mx;
  m.lds_bytes = lds;
  void* args[] = {(void*)&af, (void*)&ab, (void*)&nb, (void*)&m};
  e = hipLaunchKernel(k, dim3(2 * nb + marg_blocks), dim3(pf.threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
}  // namespace lt_impl
