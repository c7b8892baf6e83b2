// lt_vit.hip -- MaxTropical shortest-distance forward with backpointers for
// the bigram lattice (FullNGram n = 1, V <= 32, FrameDependent): the
// forward half of lt_viterbi (lattices.py:185-247 -> shortest_path through
// _forward in MaxTropical, lattices.py:379-496), frame-serial per utterance,
// bit-exact with the generic frame kernel (same terms, same order, same
// first-maximum rule: semirings.py MaxTropical, term order of
// contexts.py:226-229 with the blank self loop first).
//
// One workgroup of two waves per utterance, the whole chain in registers and
// LDS (vit_split_kernel):
//   lane (j, h): destination q = j + 1 (a core state), half h of its in-arcs:
//   h = 0 the blank self loop (term 0) and sources p = 0..16 (terms 1..17),
//   h = 1 sources p = 17..32 (terms 18..33); the halves meet through one
//   permlane32 swap (the earlier half wins ties). The start state 0 has only
//   its blank self loop. alpha sits in LDS (one write, five b128 reads per
//   frame); the frames stream into an LDS ring three frames ahead by
//   LDS-DMA (5 contiguous 1 KiB wave instructions a frame, counted vmcnt
//   waits) and each lane reads its 19 weights from LDS beside alpha. The
//   alpha chain takes the maximum by a max3 tree on wave 0; wave 1 forms the
//   backpointers (the first term equal to the maximum) behind it.
// Backpointers: one byte per (frame, state), the term index, as the generic
// kernel writes them (backtrace_kernel reads both).
#include "lt_kernels.h"

namespace {

struct VitArgs {
  const unsigned char* W;  // [B,T,C,R] fp32 / bf16
  const int* nfr;
  unsigned char* bp;       // [B,T,C]
  int* qstar;              // [B] best final state
  float* dist;             // [B] the shortest distance (MaxTropical)
  int B, T, V, C, R;
  int dbg;                 // diagnostic builds (LT_DIAG) only
  long long* stamps;       // diagnostic builds: [kVitStampSteps][4] s_memtime of block 0's chain
};

constexpr int kHalf = 17;  // sources per half (p < 17 in h = 0)

// alpha's LDS slots: half 0's sources at [0, 17), half 1's at [20, 36)
// (16-byte aligned for the b128 reads)
LT_DEVINL int aslot(int p) { return p < kHalf ? p : p + 3; }

LT_DEVINL float max_raw(float x, float y) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
LT_DEVINL float max3_raw(float x, float y, float z) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}

// 4 (2) consecutive 1 KiB LDS-DMA wave-instructions from one lane address:
// the instruction's immediate offset steps the global and the LDS address
// alike (M0 = the LDS base, set once)
LT_DEVINL void glds16x4(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024\n\t"
      "global_load_lds_dwordx4 %1, off offset:2048\n\t"
      "global_load_lds_dwordx4 %1, off offset:3072\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}
LT_DEVINL void glds16x2(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// one weight of an LDS-staged frame (bf16 widened)
template <bool BF16>
LT_DEVINL float vlds(const unsigned char* fr, int off) {
  if constexpr (BF16) return __uint_as_float((unsigned)*(const unsigned short*)(fr + off) << 16);
  else return *(const float*)(fr + off);
}

// Backtrace of the bigram backpointers in segments (one workgroup per
// utterance, the utterance's backpointers staged in LDS): every segment of S
// frames walks back from each of its C possible end states at once (the
// segment's start state per end state), one thread composes the segments
// from the best final state, then every segment emits its own frames'
// labels. Serial depth S + T/S + S instead of T. The walk itself is the
// generic backtrace's (lattices.py:229-247 through the one-hot arcs):
// backpointer 0 = the blank self loop (label 0, state kept), k + 1 = the
// arc from source k with label q.
struct VbtArgs {
  const unsigned char* bp;
  const int* qstar;
  const int* nfr;
  const float* grad;
  long long* labels;  // [B,T]
  void* arcs;         // [B,T,C,R] or null
  int B, T, C, R, conv, S;
};

template <bool BF16>
LT_DEVINL void st_arc(void* arcs, long long e, float v) {
  if constexpr (BF16) ((unsigned short*)arcs)[e] = (unsigned short)(__float_as_uint(v) >> 16);
  else ((float*)arcs)[e] = v;
}

// utterance b's backtrace by one workgroup of `nth` threads (any multiple of
// 64: every loop strides by the block it runs in -- vit_backtrace_kernel's 256
// or vit_split_kernel's 64 (2 + kBpWaves)), its backpointers staged in `lds`
// (vit_backtrace_lds bytes)
template <bool BF16>
LT_DEVINL void backtrace_body(const VbtArgs& a, int b, int tid, int nth, unsigned char* lds) {
  const int C = a.C, R = a.R, S = a.S;
  const long long FR = (long long)C * R;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  long long* lab = a.labels + (long long)b * a.T;
  for (int t = nf + tid; t < a.T; t += nth) lab[t] = 0;  // padding frames
  if (a.arcs) {
    const long long n = (long long)a.T * FR;
    for (long long e = tid; e < n; e += nth) st_arc<BF16>(a.arcs, (long long)b * a.T * FR + e, 0.f);
  }
  const int nseg = (nf + S - 1) / S;
  unsigned char* rows = lds;                          // [nf][C]
  unsigned char* start = lds + ((nf * C + 15) & ~15);  // [nseg][C]
  int* endq = (int*)(start + ((nseg * C + 15) & ~15));  // [nseg]
  const unsigned char* src = a.bp + (long long)b * a.T * C;
  const int nb = nf * C;
  if ((((uintptr_t)src) & 15) == 0) {
    // 16-byte loads, four in flight per thread before their LDS stores
    const int n16 = nb >> 4;
    for (int e = tid; e < n16; e += 4 * nth) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (e + nth * k < n16) v[k] = ((const uint4*)src)[e + nth * k];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (e + nth * k < n16) ((uint4*)rows)[e + nth * k] = v[k];
    }
    for (int e = (n16 << 4) + tid; e < nb; e += nth) rows[e] = src[e];
  } else {
    for (int e = tid * 4; e < nb; e += 4 * nth) {
      if (e + 4 <= nb && ((((uintptr_t)(src + e)) & 3) == 0)) {
        *(unsigned*)(rows + e) = *(const unsigned*)(src + e);
      } else {
        for (int k = e; k < nb && k < e + 4; ++k) rows[k] = src[k];
      }
    }
  }
  __syncthreads();
  // each (segment, end state): the state before the segment's first frame
  for (int x = tid; x < nseg * C; x += nth) {
    const int sg = x / C;
    int q = x - sg * C;
    const int t1 = min(nf, (sg + 1) * S);
    for (int t = t1 - 1; t >= sg * S; --t) {
      const int i = rows[t * C + q];
      q = i ? i - 1 : q;
    }
    start[x] = (unsigned char)q;
  }
  __syncthreads();
  if (tid == 0) {
    int q = nf > 0 ? a.qstar[b] : 0;
    for (int sg = nseg - 1; sg >= 0; --sg) {
      endq[sg] = q;
      q = start[sg * C + q];
    }
  }
  __syncthreads();
  if (a.arcs) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // zero fill before the scatter
  __syncthreads();
  const float gb = a.grad ? a.grad[b] : 1.f;
  for (int sg = tid; sg < nseg; sg += nth) {
    int q = endq[sg];
    const int t1 = min(nf, (sg + 1) * S);
    for (int t = t1 - 1; t >= sg * S; --t) {
      const int i = rows[t * C + q];
      const int p = i ? i - 1 : q, y = i ? q : 0;
      lab[t] = i ? (a.conv == LT_LABELS_REFERENCE ? (long long)(y - 1) : (long long)y) : 0LL;
      if (a.arcs) st_arc<BF16>(a.arcs, ((long long)b * a.T + t) * FR + (long long)p * R + y, gb);
      q = p;
    }
  }
}

// The alpha chain, a loader and the backpointers on separate waves of one
// workgroup (round 3: chain and backpointers apart, 0.882 -> 0.742 ms at
// cfg4 with two backpointer waves dealing the frames round robin).
//   wave 0, the chain: per frame one LDS round trip for alpha (5 b128 reads,
//     one store), 17 adds and a max3 tree, one permlane32 swap. Its weights
//     come from the transposed frame (below): 5 b128 reads issued during the
//     previous step, behind alpha's store. It issues no DMA and reads no raw
//     frame.
//   wave 1, the loader: streams the frames into an LDS-DMA ring kRing - 2
//     frames ahead (counted vmcnt waits) and writes each frame transposed
//     for the lanes -- lane l's 17 source weights, its blank self loop and
//     w[0][0] as five 16-byte groups at g * 1 KiB + 16 l (conflict-free b128
//     reads, fp32 whatever W's dtype) -- into a kTw-slot ring, published
//     through its progress word; a slot is reused once the chain and the
//     backpointer wave that own its frame are past it.
//   waves 2.., the backpointers: re-form frame t's terms from the same
//     alpha_t and weights (the same additions, so the same floats), take the
//     first term equal to alpha_{t+1}[q] and store the backpointer byte.
// The chain publishes its progress every kPub frames; the backpointer waves'
// slack on the alpha rows (kSAl) is checked against their progress as last
// read, re-read only when it runs short. Waits are bounded: a timed-out wait
// makes the utterance's distance NaN (no silent result).
#ifndef LT_VIT_BPW
#define LT_VIT_BPW 2
#endif
#ifndef LT_VIT_PUB
#define LT_VIT_PUB 2
#endif
#ifndef LT_VIT_PUBWAIT
#define LT_VIT_PUBWAIT 1  // the chain's progress store waits for its row store
#endif
#ifndef LT_VIT_NAP
#define LT_VIT_NAP 4  // s_sleep count of the followers' progress polls
#endif
// the rings' depths: the slack the loader and the chain have on the
// backpointer waves, which lag the chain by jitter more than by throughput
// (cfg4: kTw 16 -> 22 and kSAl 16 -> 32 with kRing 10 -> 8, 0.602 -> 0.565 ms;
// a third backpointer wave or a deeper DMA ring did not help); the
// diagnostic build's stamp buffer takes 4 KB of the LDS
#ifndef LT_VIT_TW
#ifdef LT_DIAG
#define LT_VIT_TW 20
#else
#define LT_VIT_TW 22
#endif
#endif
#ifndef LT_VIT_SAL
#define LT_VIT_SAL 32
#endif
#ifndef LT_VIT_BT_FUSE
#define LT_VIT_BT_FUSE 1  // the backtrace in the forward's launch when it fits
#endif
#ifndef LT_VIT_RING
#define LT_VIT_RING 8
#endif
constexpr int kRing = LT_VIT_RING;  // raw frames: kRing - 2 in flight, taken in pairs
constexpr int kTw = LT_VIT_TW;     // transposed frames
constexpr int kSAl = LT_VIT_SAL;   // alpha rows
constexpr int kPub = LT_VIT_PUB;   // the chain publishes its progress every kPub frames
constexpr int kBpWaves = LT_VIT_BPW;  // backpointer waves (frames dealt round robin)
static_assert(kBpWaves >= 1 && kBpWaves <= 8, "backpointer waves");
static_assert(kTw > 2 * kPub + 2 && kSAl > 2 * kPub + 3, "rings must leave the followers slack");
[[maybe_unused]] constexpr int kVitStampSteps = 128;  // diagnostic stamps (LT_DIAG)
constexpr int kWaitSpins = 1 << 24;                   // progress waits time out (the result is NaN)
constexpr int kPL = 1 + kBpWaves;                     // s_prog index of the loader

template <bool BF16, bool FULL>
__global__ __launch_bounds__(64 * (2 + kBpWaves)) void vit_split_kernel(const VitArgs a, const VbtArgs bt) {
  // alpha rows: [0, 17) and [20, 36) the two halves' sources (b128 reads),
  // [40, 72) spare slots for the chain's branch-free store
  __shared__ __attribute__((aligned(16))) float s_al[kSAl][72];
  __shared__ __attribute__((aligned(16))) unsigned char s_ring[kRing][5 * 1024];
  __shared__ __attribute__((aligned(16))) float4 s_tw[kTw][5][64];
  // [0] chain: alpha rows published; [1 + k] backpointer wave k: 1 + its last
  // frame done; [kPL] loader: transposed frames published
  __shared__ int s_prog[2 + kBpWaves];
  __shared__ int s_err;  // a progress wait timed out
#ifdef LT_DIAG
  __shared__ long long s_st[kVitStampSteps][4];
  const bool stamp = a.stamps != nullptr && blockIdx.x == 0;
#define VSTAMP(t, k) \
  do { if (stamp && (t) < kVitStampSteps && lane == 0) s_st[t][k] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define VSTAMP(t, k) do {} while (0)
#endif
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  const int V = FULL ? 32 : a.V, R = FULL ? 33 : a.R, C = V + 1;
  constexpr int es = BF16 ? 2 : 4;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int q = j + 1;
  const bool live = j < V;
  const int p0 = kHalf * h;
  const long long fbytes = (long long)C * R * es;
#ifdef LT_DIAG
  // timing ablations (wrong results): 1 the backpointer waves only publish,
  // 2 the loader skips the transposition, 4 the loader skips the DMA
  const int abl = a.dbg;
#else
  constexpr int abl = 0;
#endif
  const long long goff0 = (long long)b * a.T * fbytes;
  auto fclamp = [&](int t) { return min(t, max(nf - 1, 0)); };
  // alpha_0: the start state (MaxTropical one = 0), every other state zero;
  // every row's slots of absent sources (past V, and p = 33 of the upper
  // half) stay zero (-inf) for good, so a term is always alpha + w (the
  // loader writes 0 for an absent source's weight): no mask in the chain
  for (int e = tid; e < kSAl * 40; e += blockDim.x) (&s_al[0][0])[(e / 40) * 72 + e % 40] =
      e == 0 ? 0.f : -kInf;
  if (tid < 2 + kBpWaves) s_prog[tid] = 0;
  if (tid == 0) s_err = 0;
  __syncthreads();
  // frame t's weights of the lane from the transposed ring: its sources'
  // arcs, the blank self loop, w[0][0] (the start state's self loop)
  auto weights = [&](int t, float* w, float& self, float& w00) {
    const float4* tw = &s_tw[t % kTw][0][lane];
    float v[20];
#pragma unroll
    for (int g = 0; g < 5; ++g) {
      const float4 x = tw[64 * g];
      v[4 * g] = x.x; v[4 * g + 1] = x.y; v[4 * g + 2] = x.z; v[4 * g + 3] = x.w;
    }
#pragma unroll
    for (int m = 0; m < kHalf; ++m) w[m] = v[m];
    self = v[17];
    w00 = v[18];
  };
  // alpha_t of the lane's sources (al[0..16]) and of its destination (aq)
  auto alpha_rd = [&](int t, float* al, float& aq) {
    const float* acur = s_al[t % kSAl];
    aq = acur[aslot(min(q, V))];  // first: its address register is then free
#pragma unroll
    for (int g = 0; g < 5; ++g) {
      const float4 v = *(const float4*)(acur + 20 * h + 4 * g);
      al[4 * g + 0] = v.x; al[4 * g + 1] = v.y; al[4 * g + 2] = v.z; al[4 * g + 3] = v.w;
    }
  };
  // frame t's terms x (the lane's sources; absent ones -inf + 0) and xs (the
  // blank self loop), in packed adds
  auto terms_of = [&](const float* al, float aq, const float* w, float self, float* x, float& xs) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int m = 0; m < kHalf - 1; m += 2) {
      const f2 s2 = f2{al[m], al[m + 1]} + f2{w[m], w[m + 1]};
      x[m] = s2.x;
      x[m + 1] = s2.y;
    }
    const f2 s2 = f2{al[kHalf - 1], aq} + f2{w[kHalf - 1], self};
    x[kHalf - 1] = s2.x;
    xs = s2.y;
  };
  auto terms_w = [&](int t, const float* w, float self, float* x, float& xs) {
    float al[20], aq;
    alpha_rd(t, al, aq);
    terms_of(al, aq, w, self, x, xs);
  };
  auto wait_prog = [&](int k, int want) {
    int n = 0;
    for (; n < kWaitSpins; ++n) {
      const int v = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&s_prog[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (v >= want) break;
      // the followers (loader, backpointer waves) poll less often: each poll
      // is an LDS instruction beside the chain's round trips
      if (wave == 0) __builtin_amdgcn_s_sleep(1);
      else __builtin_amdgcn_s_sleep(LT_VIT_NAP);
    }
    if (n == kWaitSpins && lane == 0) s_err = 1;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  auto publish = [&](int k, int v) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this wave's LDS accesses done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&s_prog[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // backpointer wave k (1-based) owns frames k - 1, k - 1 + kBpWaves, ...:
  // the progress it must reach to have done every frame of its below `want`
  auto bp_need = [&](int k, int want) {
    const int lim = min(want, nf) - 1 - (k - 1);
    return lim < 0 ? 0 : (k - 1) + (lim / kBpWaves) * kBpWaves + 1;
  };
  if (wave == 0) {
    // ---- the chain
    float a0 = 0.f;
    int bseen = 0;  // min over the backpointer waves of their progress as last read
    int lseen = 0;  // the loader's progress as last read
    float w[kHalf], self = 0.f, w00 = 0.f, al[20], aq = 0.f;
    if (nf > 0) {
      wait_prog(kPL, 1);
      lseen = __builtin_amdgcn_readfirstlane(s_prog[kPL]);
      alpha_rd(0, al, aq);
      weights(0, w, self, w00);
    }
    for (int t = 0; t < nf; ++t) {
      VSTAMP(t, 0);
      float x[kHalf], xs;
      terms_of(al, aq, w, self, x, xs);
#ifdef LT_DIAG
      if (stamp) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        VSTAMP(t, 1);
      }
#endif
      // the max of the lane's 18 terms (the blank self loop on the lower
      // half only; absent sources are -inf), branch-free: 8 max3 + 1 max
      const float xb = h ? -kInf : xs;
      const float m0 = max3_raw(xb, x[0], x[1]);
      const float m1 = max3_raw(x[2], x[3], x[4]);
      const float m2 = max3_raw(x[5], x[6], x[7]);
      const float m3 = max3_raw(x[8], x[9], x[10]);
      const float m4 = max3_raw(x[11], x[12], x[13]);
      const float m5 = max3_raw(x[14], x[15], x[16]);
      const float mx = max_raw(max3_raw(m0, m1, m2), max3_raw(m3, m4, m5));
      auto pv = __builtin_amdgcn_permlane32_swap(__float_as_int(mx), __float_as_int(mx), false, false);
      const float r = max_raw(mx, __int_as_float(h ? pv[0] : pv[1]));
      // one store for every lane, no exec branch: the destination's value
      // (lower half), alpha[0] (lane 32), else a spare slot of the row
      float* anxt = s_al[(t + 1) % kSAl];
      a0 += w00;
      const int wslot = h == 0 ? (live ? aslot(q) : 40 + j) : (lane == 32 ? 0 : 40 + j);
      anxt[wslot] = lane == 32 ? a0 : r;
      if ((t + 1) % kPub == 0 || t + 1 == nf) {
        if (LT_VIT_PUBWAIT) {
          publish(0, t + 1);
        } else {
          // the row store above and this progress store are LDS writes of
          // one wave, which the LDS performs in issue order: a follower that
          // reads the progress and then the row sees the row without this
          // wave waiting for its store (the asm keeps the compiler's order)
          asm volatile("" ::: "memory");
          if (lane == 0)
            __hip_atomic_store(&s_prog[0], t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      VSTAMP(t, 2);
      // step t + 1's operands: alpha_{t+1} read right behind its store (LDS
      // keeps a wave's order), its latency under the rest of the step, then
      // frame t + 1's weights
      if (t + 1 < nf) {
        alpha_rd(t + 1, al, aq);
        if (lseen < t + 2) {
          wait_prog(kPL, t + 2);
          lseen = __builtin_amdgcn_readfirstlane(s_prog[kPL]);
        }
        weights(t + 1, w, self, w00);
      }
      // step t + 1 overwrites the alpha row alpha_{t + 2 - kSAl}: every
      // backpointer wave must be past frame t + 2 - kSAl
      const int want = t + 3 - kSAl;
      if (bseen < want) {
        int m = 0x7fffffff;
        for (int k = 1; k <= kBpWaves; ++k) {
          const int need = bp_need(k, want);
          if (need > 0) wait_prog(k, need);
          m = min(m, __builtin_amdgcn_readfirstlane(s_prog[k]));
        }
        bseen = m;
      }
      VSTAMP(t, 3);
    }
#ifdef LT_DIAG
    if (stamp) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (int i = lane; i < kVitStampSteps * 4; i += 64) a.stamps[i] = (&s_st[0][0])[i];
    }
#endif
    // the distance: (+)_q alpha_T[q] in MaxTropical, the first maximum
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float* af = s_al[nf % kSAl];
    float r = lane < C ? af[aslot(lane)] : -kInf;
    int ri = lane < C ? lane : 0x7fffffff;
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) {
      const float pv = __shfl_xor(r, sft);
      const int pi = __shfl_xor(ri, sft);
      if (pv > r || (pv == r && pi < ri)) { r = pv; ri = pi; }
    }
    if (lane == 0) {
      a.dist[b] = r;
      a.qstar[b] = ri;
    }
  } else if (wave == 1) {
    // ---- the loader: raw frames by LDS-DMA, transposed for the lanes
    const int ni = (int)(((fbytes + 30) / 16 + 63) / 64);
    // wave-instructions that never leave the frame: 4 (fp32 V = 32), 2 (bf16)
    const int kf = (int)min((long long)min(ni, 4), fbytes / 16 / 64);
    auto issue = [&](int t) {  // frame t (clamped) -> slot t % kRing
      if (abl & 4) return;
      const long long off = goff0 + (long long)fclamp(t) * fbytes;
      const long long a0 = off & ~15LL;
      const int n16 = (int)((off + fbytes - a0 + 15) >> 4);
      const unsigned dst = lds_base_addr(&s_ring[t % kRing][0]);
      // the first kf wave-instructions never leave the frame (or W): one lane
      // address, the instruction's 1 KiB step as its immediate offset; the
      // rest clamp each lane to the frame's last 16 bytes (inline asm, as
      // glds16: the compiler sees no LDS write to order its LDS reads behind)
      const unsigned char* gb = a.W + a0 + 16 * lane;
      if (kf == 4) glds16x4(gb, dst);
      else if (kf == 2) glds16x2(gb, dst);
      for (int i = (kf == 4 || kf == 2) ? kf : 0; i < ni; ++i) {
        int g = lane + 64 * i;
        g = g < n16 ? g : n16 - 1;
        glds16(a.W + a0 + 16LL * g, dst + 1024u * i);
      }
    };
    const int vb = (p0 * R + min(q, V)) * es;
    const int vself = min(q, V) * R * es;
    // frames in pairs: one LDS round trip and one progress store per two
    // frames (the loader paced the chain with one frame per trip)
    if (nf > 0)
      for (int d = 0; d < kRing - 2; ++d) issue(d);
    int cseen = 0, bseen = 0;
    for (int f = 0; f < nf; f += 2) {
      if (!(abl & 4)) wait_vmcnt((kRing - 4) * ni);  // frames f, f + 1 landed
      // the transposed slots held frames f - kTw and f + 1 - kTw: the chain
      // (it reads frame f' during step f' - 1; its progress f' + 1 covers
      // those reads) and the backpointer waves owning them must be past them
      const int fo = f + 1 - kTw;
      if (fo >= 0) {
        if (cseen < fo + 1) {
          wait_prog(0, min(fo + 1 + kPub, nf));
          cseen = __builtin_amdgcn_readfirstlane(s_prog[0]);
        }
        if (bseen < fo + 1) {
          int m = 0x7fffffff;
          for (int k = 1; k <= kBpWaves; ++k) {
            const int need = bp_need(k, fo + 1);
            if (need > 0) wait_prog(k, need);
            m = min(m, __builtin_amdgcn_readfirstlane(s_prog[k]));
          }
          bseen = m;
        }
      }
      if (!(abl & 2)) {
        float v[2][20];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const unsigned char* fr =
              &s_ring[(f + e) % kRing][0] + ((goff0 + (long long)fclamp(f + e) * fbytes) & 15);
#pragma unroll
          for (int m = 0; m < kHalf; ++m) {
            // an absent source (past V; p = 33 of the upper half): 0 (its
            // alpha slot is -inf for good)
            const bool ok = FULL ? (m < kHalf - 1 || h == 0) : p0 + m <= V;
            v[e][m] = ok ? vlds<BF16>(fr, vb + m * (FULL ? 33 : R) * es) : 0.f;
          }
          v[e][17] = vlds<BF16>(fr, vself);
          v[e][18] = vlds<BF16>(fr, 0);
          v[e][19] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float4* tw = &s_tw[(f + e) % kTw][0][lane];
#pragma unroll
          for (int g = 0; g < 5; ++g)
            tw[64 * g] = make_float4(v[e][4 * g], v[e][4 * g + 1], v[e][4 * g + 2], v[e][4 * g + 3]);
        }
      }
      // the raw slots of frames f - 2, f - 1 are free once this wave's reads
      // of them are done (the DMA writes LDS outside the wave's LDS order)
      __builtin_amdgcn_s_waitcnt(0xc07f);
      issue(f + kRing - 2);
      issue(f + kRing - 1);
      publish(kPL, f + 2);
    }
    wait_vmcnt(0);
  } else {
    // ---- the backpointers (wave 2 + k takes frames k, k + kBpWaves, ...):
    // the first term equal to alpha_{t+1}[q]
    // (group_reduce's first-maximum rule), the lower half first
    const int k1 = wave - 1;  // 1-based index of this backpointer wave
    const __amdgpu_buffer_rsrc_t bpr =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.bp + (long long)b * a.T * C), (short)0,
                                          a.T * C, 0x00020000);
    const int ib = h ? 18 : 1;  // term index of x[0]
    int seen = 0;  // the chain's progress as last read
    for (int t = k1 - 1; t < nf; t += kBpWaves) {
      if (seen < t + 1) {
        wait_prog(0, t + 1);
        seen = __builtin_amdgcn_readfirstlane(s_prog[0]);
      }
      if (abl & 1) {
        publish(k1, t + 1);
        continue;
      }
      float w[kHalf], self, w00, x[kHalf], xs;
      weights(t, w, self, w00);
      terms_w(t, w, self, x, xs);
      const float rq = s_al[(t + 1) % kSAl][aslot(min(q, V))];
      int ri = 99;
#pragma unroll
      for (int m = 16; m >= 0; --m) ri = x[m] == rq ? ib + m : ri;
      if (h == 0) ri = xs == rq ? 0 : ri;
      auto pi = __builtin_amdgcn_permlane32_swap(ri, ri, false, false);
      const int rlo = h ? pi[0] : ri, rhi = h ? ri : pi[1];
      const int bpv = lane == 32 ? 0 : (rlo < 99 ? rlo : rhi);
      if (((h == 0 && live) || lane == 32) && !(abl & 1))
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bpv, bpr, lane == 32 ? 0 : q, t * C, 0);
      publish(k1, t + 1);
      (void)w00;
    }
  }
  // every wave's global stores (the backpointers, qstar) done before the barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && s_err) a.dist[b] = __builtin_nanf("");  // a timed-out wait: no silent result
  // the backtrace in the same workgroup (bt.labels set when the utterance's
  // backpointers fit the transposed ring's LDS, vit_backtrace_lds): they are
  // this workgroup's own stores, read back after the barrier; no second
  // launch (cfg4: 0.636 -> 0.633 ms)
  if (bt.labels) backtrace_body<BF16>(bt, b, tid, (int)blockDim.x, (unsigned char*)&s_tw[0][0][0]);
}

template <bool BF16>
__global__ __launch_bounds__(256) void vit_backtrace_kernel(const VbtArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  backtrace_body<BF16>(a, blockIdx.x, threadIdx.x, (int)blockDim.x, lds);
}

}  // namespace

namespace lt_impl {
bool vit_bigram_eligible(const lt_problem* pb) {
  return pb->context_size == 1 && pb->vocab_size >= 1 && pb->vocab_size <= 32 &&
         lt_impl::tune_str("LT_VIT_GENERIC") == nullptr;
}

// MaxTropical forward (distance, best final state, backpointers) of every
// utterance; lt_viterbi's backtrace reads the backpointers.
namespace {
int vit_bigram_forward(const lt_problem* pb, const void* W, const int32_t* nfr, unsigned char* bp,
                       int* qstar, float* dist, void* stream, const VbtArgs* bt) {
  VitArgs a;
  a.W = (const unsigned char*)W;
  a.nfr = nfr;
  a.bp = bp;
  a.qstar = qstar;
  a.dist = dist;
  a.B = pb->batch;
  a.T = pb->max_frames;
  a.V = pb->vocab_size;
  a.C = a.V + 1;
  a.R = a.V + 1;
  a.dbg = 0;
  a.stamps = nullptr;
#ifdef LT_DIAG
  if (const char* d = lt_impl::tune_str("LT_VIT_DBG")) a.dbg = atoi(d);
  if (const char* sp = lt_impl::tune_str("LT_VIT_STAMPS")) a.stamps = (long long*)strtoull(sp, nullptr, 0);
#endif
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const bool full = a.V == 32;
  const void* k = full ? (bf16 ? (const void*)vit_split_kernel<true, true>
                               : (const void*)vit_split_kernel<false, true>)
                       : (bf16 ? (const void*)vit_split_kernel<true, false>
                               : (const void*)vit_split_kernel<false, false>);
  VbtArgs none{};
  void* args[] = {(void*)&a, (void*)(bt ? bt : &none)};
  hipError_t e =
      hipLaunchKernel(k, dim3(a.B), dim3(64 * (2 + kBpWaves)), args, 0, (hipStream_t)stream);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
}  // namespace

// LDS bytes of vit_backtrace for T frames (0: too long, use the generic one)
int vit_backtrace_lds(const lt_problem* pb, int* seg) {
  const int T = pb->max_frames, C = pb->vocab_size + 1;
  const int S = std::max(16, (T + 255) / 256);
  const int nseg = (T + S - 1) / S;
  const long long bytes = ((T * (long long)C + 15) & ~15LL) + ((nseg * C + 15) & ~15) + 4LL * nseg;
  *seg = S;
  return bytes <= 144 * 1024 ? (int)bytes : 0;
}

namespace {
VbtArgs bt_args(const lt_problem* pb, const unsigned char* bp, const int* qstar, const int32_t* nfr,
                const float* grad, int64_t* labels, void* arcs, int32_t conv) {
  VbtArgs a;
  a.bp = bp; a.qstar = qstar; a.nfr = nfr; a.grad = grad;
  a.labels = (long long*)labels; a.arcs = arcs;
  a.B = pb->batch; a.T = pb->max_frames; a.C = pb->vocab_size + 1; a.R = a.C; a.conv = conv;
  a.S = 0;
  return a;
}
}  // namespace

// the bigram forward and its backtrace in ONE launch while the utterance's
// backpointers fit the forward's transposed-ring LDS, else the two launches
int vit_bigram(const lt_problem* pb, const void* W, const int32_t* nfr, unsigned char* bp,
               int* qstar, float* dist, const float* grad, int64_t* labels, void* arcs,
               int32_t conv, void* stream) {
  VbtArgs bt = bt_args(pb, bp, qstar, nfr, grad, labels, arcs, conv);
  const int lds = vit_backtrace_lds(pb, &bt.S);
  if (LT_VIT_BT_FUSE && lds > 0 && lds <= (int)(kTw * 5 * 64 * sizeof(float4)))
    return vit_bigram_forward(pb, W, nfr, bp, qstar, dist, stream, &bt);
  int rc = vit_bigram_forward(pb, W, nfr, bp, qstar, dist, stream, nullptr);
  if (rc) return rc;
  if (lds > 0) return vit_backtrace(pb, bp, qstar, nfr, grad, labels, arcs, conv, stream);
  return LT_EUNSUPPORTED;  // the caller runs the generic backtrace
}

int vit_backtrace(const lt_problem* pb, const unsigned char* bp, const int* qstar,
                  const int32_t* nfr, const float* grad, int64_t* labels, void* arcs,
                  int32_t conv, void* stream) {
  VbtArgs a = bt_args(pb, bp, qstar, nfr, grad, labels, arcs, conv);
  const int lds = vit_backtrace_lds(pb, &a.S);
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const void* k = bf16 ? (const void*)vit_backtrace_kernel<true> : (const void*)vit_backtrace_kernel<false>;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  void* args[] = {(void*)&a};
  if (e == hipSuccess) e = hipLaunchKernel(k, dim3(a.B), dim3(256), args, lds, (hipStream_t)stream);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
}  // namespace lt_impl
