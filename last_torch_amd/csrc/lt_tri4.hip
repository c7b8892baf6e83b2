// lt_tri4.hip -- the trigram checkpointing recursions split four ways
// (FullNGram n = 2, V = 32, Log; lattices.py:379-496 and 686-799,
// alignments.py:286-318, contexts.py:207-256). One utterance direction (the
// alpha recursion, or the checkpointing beta recursion) runs on a quad of
// four workgroups instead of one, so the 2B recursions of a batch use 8B CUs:
//
//   member k of a quad owns the states whose "block" lies in J_k = [8k, 8k+8):
//     forward   destinations (j+1, y), the order-1 states j+1, (k = 0) state 0
//     backward  sources (x, z), z - 1 in J_k, the order-1 sources z, (k = 0) 0
//   and stages per frame only the W rows its terms read: the 32 runs of eight
//   rows (x, 8k+1 .. 8k+8), x = 1..32, the order-1 rows 8k+1 .. 8k+8 and
//   row 0 (33 runs x 8 rows + 1 of the frame's 1,057), by LDS-DMA.
//
// The recursions are all-to-all across the quad: alpha_{t+1}[(j+1, y)] reads
// alpha_t[(x, j+1)] for every x, and beta_t[(x, z)] reads beta_{t+1}[(z, y)]
// for every y. Each frame every lane publishes its new value as one 64-bit
// word (frame tag << 32 | float bits) into a two-frame exchange buffer, and
// the readers poll exactly the words they need until the tag is theirs: the
// word is its own flag, so a hand-off is one store and one load. A writer
// reuses a buffer two frames later only after reading the frame in between
// from every member, which every member published after reading the old one.
//
// All four members hold their vectors relative to one integer offset: the
// floor of the max of the vector one step older (each member publishes its
// states' max as a tagged word; the step after next reads all four), so
// every value, history row and exchange word means the same thing in every
// member and no rebasing is needed.
//
// Placement: blocks 32 g + 8 k + x for quad 8 g + x, so the members of a quad
// sit 8 block ids apart (one XCD where dispatch is round robin over the 8
// XCDs; the protocol is coherent at memory either way). Every quad member
// must be resident at once: the host launches this design only while 8B <= the
// CU count (one workgroup per CU by LDS), and every wait is bounded -- a
// timeout turns the utterance's outputs into NaN and raises the error word.
//
// The numerators (alpha^n with the arc table and num, beta^n) run on an
// eighth wave of member 0, a frame a step in lockstep with the quad,
// gathering their 2(U+1) weights a frame straight from HBM sixteen frames
// ahead; the loss takes log_z from the forward quad through a per-utterance
// counter (whichever side finishes second writes it). The marginal pass
// (marg_kernel) is unchanged.
//
// Measured (cfg5, B = 32, bf16): parity-green, but 3.3-3.5 us
// a frame against the one-workgroup kernel's 2.7 (lt_tri.hip), so only the
// diagnostic build runs it (LT_TRI4=1). The per-frame hand-off is the floor:
// stamps (tools/tri4_stamps.py) show 2,400-2,900 cycles a frame from a
// member's last store to its inputs all present, against the guide's 0.8-2.9
// us for a data-tagged one-to-one hand-off between CUs that stream loads
// (MI355X_MICROARCH.md, handoff-1to1), and ~2,800 cycles of compute whatever
// the terms per lane (34 or 17) or the weight-read form.
//
// Scratch: one static device buffer (the exchange words, zeroed by the host
// before every launch), so concurrent trigram losses on two streams of one
// device must not overlap.
#include "lt_kernels.h"

namespace {

constexpr int kT4MaxB = 32;          // utterances per launch (8B quad workgroups <= CUs)
constexpr int kT4Pub = 264;          // words a member publishes a frame (256 + 8 order-1)
constexpr int kT4SW = 8;             // state waves: two lanes a state (the terms in halves)
constexpr int kT4Aux = 8, kT4Ld = 9, kT4Num = 11;  // the aux wave, loaders 9-10, numerator
constexpr int kT4Wr = 12;            // the checkpoint-row writer
constexpr int kT4Waves = 13;
constexpr unsigned kT4Spin = 1u << 21;
constexpr int kT4ND = 8;             // numerator gather depth (frames in flight)

struct T4Scratch {
  unsigned long long x[2 * kT4MaxB][2][4][kT4Pub];  // tagged values [quad][frame & 1][member]
  unsigned long long mx[2 * kT4MaxB][2][4];          // tagged member maxes
  unsigned long long fin[kT4MaxB][36][2];            // forward: tagged final (max, sum) per wave
  float lz[kT4MaxB], num[kT4MaxB];
  unsigned long long xcc[2 * kT4MaxB][4];           // tagged XCD id of each member
  int cnt[kT4MaxB];
  int err;
  float dummy[128];
};
__device__ T4Scratch g_t4;

struct T4Args {
  const unsigned char* W;
  long long w_bytes;
  const int* nfr;
  const int* labels;
  const int* nlab;
  float* alpha;      // [B,T,C]  alpha_t per frame (checkpoint rows)
  float* beta;       // [B,T,C]  beta_{t+1} per frame
  float* alpha_num;  // [B,T,NP]
  float* beta_num;   // [B,T,NP]
  float* log_z;      // [B]
  float* num;        // [B]
  float* loss;       // [B]
  int B, T, U, G;    // G: groups of eight quads
  long long* stamps; // diagnostic build (-DLT_STAMPS): quad 0 [member][wave][T][4] s_memtime
};

#ifdef LT_STAMPS
#define T4STAMP(a, q, k, w, i, s)                                                            \
  do {                                                                                     \
    if ((a).stamps && (q) == 0 && (threadIdx.x & 63) == 0)                                 \
      (a).stamps[(((long long)(k) * kT4Waves + (w)) * (a).T + (i)) * 4 + (s)] =              \
          (long long)__builtin_amdgcn_s_memtime();                                         \
  } while (0)
#else
#define T4STAMP(a, q, k, w, i, s) \
  do {                            \
  } while (0)
#endif

// W geometry (V = 32): R = 33 labels a row, C = 1,057 states
constexpr int kV = 32, kR = 33, kC = 1 + 32 + 32 * 32;
template <bool BF16>
struct T4Geo {
  static constexpr int es = BF16 ? 2 : 4;
  static constexpr int RB = kR * es;                 // bytes a row
  static constexpr int RC = BF16 ? 35 : 67;          // 16-byte chunks a run (8 rows + misalignment;
                                                     // 35, not 34: run starts 140 dwords apart)
  static constexpr int RUNB = 16 * RC;
  static constexpr int NRC = 33 * RC;                // chunks of the 33 runs
  static constexpr int R0C = BF16 ? 6 : 10;          // chunks of row 0 (+ misalignment)
  static constexpr int NI = (NRC + R0C + 63) / 64;   // LDS-DMA instructions (16 B a lane)
  static constexpr int BLK = 1024 * NI;              // forward: blank weights (dword a lane)
  static constexpr int P = BF16 ? 3 : 3;             // ring slots
  template <bool REV>
  static constexpr int slot() { return BLK + (REV ? 0 : 1024); }
  template <bool REV>
  static constexpr int ninstr() { return NI + (REV ? 0 : 4); }
};

LT_DEVINL unsigned long long t4_word(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | __float_as_uint(v);
}
LT_DEVINL unsigned long long t4_poll(const unsigned long long* p) {
  unsigned long long v;
  asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
LT_DEVINL void t4_put(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A word for the quad: with every member on one XCD a plain store, which
// keeps the line in that XCD's L2 where the readers' L1-bypassing polls find
// it; else the write-through (sc1) store, which drops it from the L2.
// (inline asm: no compiler-inserted wait for the wave's older stores)
LT_DEVINL void t4_pub(unsigned long long* p, unsigned long long v, bool same_xcd) {
  if (same_xcd) asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}
LT_DEVINL unsigned t4_xcc() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
// Poll until every active lane's word carries `tag` (lanes with want = false
// take no part); returns the value, or NaN after the bound (and raises err).
LT_DEVINL float t4_take(const unsigned long long* p, unsigned tag, bool want, int* abort_lds) {
  float v = 0.f;
  bool done = !want;
  unsigned spins = 0;
  while (true) {
    if (!done) {
      const unsigned long long w = t4_poll(p);
      if ((unsigned)(w >> 32) == tag) {
        v = __uint_as_float((unsigned)w);
        done = true;
      }
    }
    if (__builtin_amdgcn_ballot_w64(!done) == 0) break;
    if (++spins > kT4Spin) {
      if (!done) v = __builtin_nanf("");
      if ((threadIdx.x & 63) == 0) {
        *(volatile int*)abort_lds = 1;
        __hip_atomic_store(&g_t4.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return v;
}

// global_load_lds_dword: 64 lanes x 4 B into the contiguous 256 B at M0
LT_DEVINL void glds4(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

template <bool BF16>
LT_DEVINL float t4_w(const unsigned char* p) {  // one weight from LDS, unmerged
  typedef const volatile __attribute__((address_space(3))) unsigned short lds_u16;
  typedef const volatile __attribute__((address_space(3))) float lds_f32;
  if constexpr (BF16)
    return __uint_as_float((unsigned)*(lds_u16*)p << 16);
  else
    return *(lds_f32*)p;
}

// plain (pipelined) LDS weight reads, for terms whose addresses are not
// contiguous (the compiler cannot merge them into unaligned wide reads)
template <bool BF16>
LT_DEVINL float t4_wn(const unsigned char* p) {
  typedef const __attribute__((address_space(3))) unsigned short lds_u16;
  typedef const __attribute__((address_space(3))) float lds_f32;
  if constexpr (BF16)
    return __uint_as_float((unsigned)*(lds_u16*)p << 16);
  else
    return *(lds_f32*)p;
}

// LDS of a member: the ring, then the staged sources [2][8][32], the
// order-1 sources of state 0 (backward) [2][32], the order-1 alpha (forward)
// [2][8], the max slots [3], the abort flag
template <bool BF16, bool REV>
struct T4Lds {
  typedef T4Geo<BF16> Gm;
  static constexpr int ring = 0;
  static constexpr int stage = Gm::P * Gm::template slot<REV>();
  static constexpr int stage1 = stage + 2 * 256 * 4;
  static constexpr int own1 = stage1 + 2 * 32 * 4;
  static constexpr int maxs = own1 + 2 * 8 * 4;
  static constexpr int abrt = maxs + 4 * 4;
  static constexpr int hv = abrt + 16;     // abrt: two flags, by step parity
  static constexpr int spb = hv + 2 * 272 * 4;  // the states' values [2][265] for the writer
  static constexpr int nring = spb + 16;        // the offsets sp [2]             // numerator weights [kT4ND][4][64] dwords
  static constexpr int total = nring + kT4ND * 1024;
};

// The loader waves: frame f of step i into slot i % P, chunks dealt to the two
// waves instruction by instruction (wave lw issues lw, lw + 2, ...)
template <bool BF16, bool REV>
LT_DEVINL void t4_issue(const T4Args& a, int b, int k, int nf, int i, int lw, int lane,
                        unsigned ldsb) {
  typedef T4Geo<BF16> Gm;
  if (i >= nf) return;
  const int f = REV ? nf - 1 - i : i;
  const long long fb = ((long long)b * a.T + f) * (long long)(kC * Gm::RB);
  const unsigned sb = ldsb + (i % Gm::P) * Gm::template slot<REV>();
  const long long last = a.w_bytes - 16;
#pragma unroll 1
  for (int w = lw; w < Gm::template ninstr<REV>(); w += 2) {
    if (w < Gm::NI) {
      const int g = 64 * w + lane;
      long long src;
      if (g < Gm::NRC) {
        const int r = g / Gm::RC, c = g - r * Gm::RC;
        const long long rs = (long long)(r == 0 ? 1 + 8 * k : 33 + 32 * (r - 1) + 8 * k) * Gm::RB;
        src = ((fb + rs) & ~15LL) + 16 * c;
      } else {
        src = (fb & ~15LL) + 16 * min(g - Gm::NRC, Gm::R0C - 1);
      }
      glds16(a.W + min(src, last), sb + 1024 * w);
    } else {  // forward blank weights W[(j+1, y), 0], one dword a lane
      const int e = 64 * (w - Gm::NI) + lane, jl = e >> 5, y = (e & 31) + 1;
      const long long row = 33 + 32 * (8 * k + jl) + (y - 1);
      glds4(a.W + ((fb + row * Gm::RB) & ~3LL), sb + Gm::BLK + 256 * (w - Gm::NI));
    }
  }
}

// lse over a blank term and 33 lexical terms (den_fwd_tri's order): the safe
// max, then the sum of exps, minus the offset sp
LT_DEVINL float t4_lse(float tb, const float (&x)[33], float sp) {
  float m = tb;
#pragma unroll
  for (int k = 0; k < 33; ++k) m = fmaxf(m, x[k]);
  const float c = __builtin_isfinite(m) ? m : 0.f;
  const float l = c * kLog2e;
  float s = lt_exp_off(tb, l);
#pragma unroll
  for (int k = 0; k < 33; ++k) s += lt_exp_off(x[k], l);
  return (c + lt_log(s)) - sp;
}

// The numerator wave of member 0 (u = lane, lane + 64), in lockstep with the
// quad (one frame a step, the same barriers): alpha^n with the arc table and
// num (REV = false), or beta^n (REV = true), as num_fwd_loop / num_beta_loop,
// its 2(U+1) weights a frame gathered from HBM kT4ND frames ahead.
// The numerator wave of member 0 (u = lane, lane + 64), in lockstep with the
// quad (one frame a step, the same barriers): alpha^n with the arc table and
// num (REV = false), or beta^n (REV = true), as num_fwd_loop / num_beta_loop.
// Its 2(U+1) weights a frame come by LDS-DMA, one dword a lane per weight,
// kT4ND frames ahead: a step issues exactly two stores and four DMA
// instructions, so the wait for frame i is an exact vmcnt.
template <bool BF16, bool REV>
struct T4Numer {
  int ob[2], ol[2];
  bool live[2], lex[2];
  float n[2];
  float O;
  int nf, NP, nl;
  unsigned ring;  // LDS byte address of the numerator ring
  // one store instruction per position and step whatever the lane mask (the
  // exact vmcnt): lanes past the string write a dummy word
  LT_DEVINL float* row(float* hist, const T4Args& a, int b, int t, int lane, int h) const {
    return live[h] ? hist + ((long long)b * a.T + t) * NP + lane + 64 * h : &g_t4.dummy[lane + 64 * h];
  }

  LT_DEVINL void issue(const T4Args& a, int b, int lane, int i) {
    const int ii = i < nf ? i : nf - 1;
    const int f = REV ? nf - 1 - ii : ii;
    const long long fb = ((long long)b * a.T + f) * (long long)(kC * kR * (BF16 ? 2 : 4));
    const unsigned dst = ring + (i % kT4ND) * 1024;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      glds4(a.W + ((fb + (long long)ob[h] * (BF16 ? 2 : 4)) & ~3LL), dst + 512 * h);
      glds4(a.W + ((fb + (long long)ol[h] * (BF16 ? 2 : 4)) & ~3LL), dst + 512 * h + 256);
    }
  }
  LT_DEVINL float take(const unsigned char* lds, const T4Args& a, int b, int i, int w, int lane,
                       int e) const {
    const unsigned dw = *(const volatile __attribute__((address_space(3))) unsigned*)(
        lds + (ring - lds_base_addr((unsigned char*)lds)) + (i % kT4ND) * 1024 + 256 * w + 4 * lane);
    if constexpr (BF16) {
      const int ii = i < nf ? i : nf - 1;
      const int f = REV ? nf - 1 - ii : ii;
      const long long fb = ((long long)b * a.T + f) * (long long)(kC * kR * 2);
      const int hs = (int)((fb + 2LL * e) & 2);
      return __uint_as_float((hs ? dw >> 16 : dw & 0xffffu) << 16);
    } else {
      return __uint_as_float(dw);
    }
  }
  LT_DEVINL void init(const T4Args& a, const KArgs& ka, int b, int lane, int nfr, int* ctx,
                      int* ylab, unsigned ring_addr) {
    nf = nfr;
    ring = ring_addr;
    const int U = a.U;
    NP = U + 1;
    for (int u = lane; u < U; u += 64) ylab[u] = a.labels[(long long)b * U + u];
    if (lane == 0) walk_states(ka, ctx, ylab);  // one wave: its LDS ops stay in order
    if (!REV && ka.arcs) write_arc_table(ka, b, ctx, ylab, lane, 64);
    nl = a.nlab[b];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = lane + 64 * h;
      live[h] = u < NP;
      const int uu = live[h] ? u : 0;
      ob[h] = ctx[uu];
      if (!REV) {
        lex[h] = live[h] && u >= 1;
        ol[h] = lex[h] ? ctx[uu - 1] + ylab[uu - 1] : 0;
      } else {
        lex[h] = live[h] && u < U;
        ol[h] = lex[h] ? ob[h] + ylab[uu] : 0;
      }
      n[h] = !REV ? (u == 0 ? 0.f : -kInf) : (u == nl ? 0.f : -kInf);
      if (!live[h]) n[h] = -kInf;
    }
    float* hist = REV ? a.beta_num : a.alpha_num;
    if (REV && nf > 0)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (live[h]) hist[((long long)b * a.T + nf - 1) * NP + lane + 64 * h] = n[h];
    if (nf > 0)
      for (int d = 0; d < kT4ND; ++d) issue(a, b, lane, d);
    O = 0.f;
  }
  LT_DEVINL void step(const unsigned char* lds, const T4Args& a, int b, int lane, int i) {
    // frame i's DMA: issued after it, frames i+1 .. kT4ND-1 of the prologue
    // (four each), the two stores of the step that issued it and the steps
    // since (four DMA, then two stores, each)
    wait_vmcnt(min(4 * (kT4ND - 1) + 2 * i, 6 * (kT4ND - 1) + 2));
    const int f = REV ? nf - 1 - i : i;
    float* hist = REV ? a.beta_num : a.alpha_num;
    float wb[2], wl[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      wb[h] = take(lds, a, b, i, 2 * h, lane, ob[h]);
      wl[h] = take(lds, a, b, i, 2 * h + 1, lane, ol[h]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read: it can refill
    issue(a, b, lane, i + kT4ND);
    float m = fmaxf(n[0], n[1]);
    m = gmax<6>(m, 6);
    const float sp = __builtin_isfinite(m) ? floorf(m) : 0.f;
    float nn[2];
    if (!REV) {
#pragma unroll
      for (int h = 0; h < 2; ++h) *row(hist, a, b, f, lane, h) = O + n[h];
      // n[u - 1]: lane - 1's value (lane 0 of the second half: lane 63's first)
      const float up0 = __shfl_up(n[0], 1);
      const float up1 = __shfl_up(n[1], 1);
      const float l63 = __shfl(n[0], 63);
      const float prev[2] = {up0, lane == 0 ? l63 : up1};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float xb = n[h] + wb[h];
        const float xl = lex[h] ? prev[h] + wl[h] : -kInf;
        nn[h] = log_plus(xb, xl) - sp;
      }
    } else {
      // n[u + 1]: lane + 1's value (lane 63 of the first half: lane 0's second)
      const float dn0 = __shfl_down(n[0], 1);
      const float dn1 = __shfl_down(n[1], 1);
      const float l0 = __shfl(n[1], 0);
      const float next[2] = {lane == 63 ? l0 : dn0, dn1};
#pragma unroll
      for (int h = 0; h < 2; ++h)
        nn[h] = log_plus(wb[h] + n[h], lex[h] ? wl[h] + next[h] : -kInf) - sp;
    }
    O += sp;
#pragma unroll
    for (int h = 0; h < 2; ++h) n[h] = live[h] ? nn[h] : -kInf;
    if (REV && i < nf - 1)
#pragma unroll
      for (int h = 0; h < 2; ++h) *row(hist, a, b, f - 1, lane, h) = O + n[h];
  }
  LT_DEVINL void finish(const T4Args& a, int b, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the wave
    if (REV) return;
    float* hist = a.alpha_num;
    // padding frames carry alpha^n (lattices.py:460-461); num = O + n[nl]
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (live[h])
        for (int t = nf; t < a.T; ++t) hist[((long long)b * a.T + t) * NP + lane + 64 * h] = O + n[h];
    const bool ok = nl >= 0 && nl <= a.U;
    const int src = ok ? nl : 0;
    const float nv0 = __shfl(n[0], src & 63), nv1 = __shfl(n[1], src & 63);
    const float nmv = ok ? O + (src < 64 ? nv0 : nv1) : -kInf;
    if (lane == 0) {
      if (a.num) a.num[b] = nmv;
      __hip_atomic_store(&g_t4.num[b], nmv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&g_t4.cnt[b], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 1) {
        const float lz = __hip_atomic_load(&g_t4.lz[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.loss) a.loss[b] = lz - nmv;
      }
    }
  }
};

// One checkpoint row of a member's states (the writer wave): forward, alpha
// rows [B][T][C] at row t; backward, beta rows, value vals[li] + O, the
// member's 256 order-2 states, 8 order-1 states and (member 0) state 0
template <bool REV>
LT_DEVINL void t4_rows(const T4Args& a, int b, int k, int t, const float* vals, float O, int lane) {
  float* base = REV ? a.beta : a.alpha;
  if (!base || t < 0) return;
  float* row = base + ((long long)b * a.T + t) * kC;
  for (int li = lane; li < 265; li += 64) {
    int p;
    if (li < 256) {
      const int hi = li >> 5, lo = li & 31;
      p = REV ? 33 + 32 * lo + 8 * k + hi : 33 + 32 * (8 * k + hi) + lo;
    } else if (li < 264) {
      p = 1 + 8 * k + (li - 256);
    } else {
      if (k != 0) break;
      p = 0;
    }
    row[p] = O + vals[li];
  }
}

template <bool BF16, bool REV>
LT_DEVINL void t4_member(const T4Args& a, const KArgs& ka, int q, int b, int k) {
  typedef T4Geo<BF16> Gm;
  typedef T4Lds<BF16, REV> L;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ int s_ctx[128], s_ylab[128];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned ldsb = lds_base_addr(lds);
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  float* stage = (float*)(lds + L::stage);
  float* stage1 = (float*)(lds + L::stage1);
  float* own1 = (float*)(lds + L::own1);
  int* maxs = (int*)(lds + L::maxs);
  int* abrt = (int*)(lds + L::abrt);
  float* hv = (float*)(lds + L::hv);
  float* spb = (float*)(lds + L::spb);
  unsigned long long(*X)[4][kT4Pub] = g_t4.x[q];
  unsigned long long(*MX)[4] = g_t4.mx[q];
  if (tid < 3) maxs[tid] = tri_enc(-kInf);
  if (tid == 3) abrt[0] = abrt[1] = 0;
  if (tid == 0) t4_put(&g_t4.xcc[q][k], t4_word(1u, __uint_as_float(t4_xcc())));
  // ---- prologue: loaders put frames 0 .. P-2 in flight
  const bool loader = wave == kT4Ld || wave == kT4Ld + 1;
  if (loader) {
    for (int i = 0; i < Gm::P - 1; ++i) t4_issue<BF16, REV>(a, b, k, nf, i, wave - kT4Ld, lane, ldsb);
  }
  T4Numer<BF16, REV> nu;
  const bool numer = wave == kT4Num && k == 0;
  if (numer) nu.init(a, ka, b, lane, nf, s_ctx, s_ylab, ldsb + L::nring);
  __syncthreads();
  // the lane's state: state waves two lanes a state (h: which half of its
  // terms), the aux wave's lanes 0..7 the order-1 states, lane 8 state 0
  const int e = tid >> 1, h = tid & 1;  // state waves: state 0..255
  const int hi = e >> 5, lo = e & 31;   // forward (jl, y - 1); backward (zl, x - 1)
  const bool sw = wave < kT4SW, aux = wave == kT4Aux;
  int p = -1;                           // the lane's state
  if (sw) p = REV ? 33 + 32 * lo + 8 * k + hi : 33 + 32 * (8 * k + hi) + lo;
  else if (aux && lane < 8) p = 1 + 8 * k + lane;
  else if (aux && lane == 8) p = 0;
  const bool lead = !sw || h == 0;      // the lane that writes the state's words and rows
  // the state's slot in the writer's buffer
  const int li = sw ? e : (lane < 8 ? 256 + lane : 264);
  // alpha_0: state 0 = 0, else -inf; beta at the last frame: 0 everywhere
  float v = REV ? 0.f : (p == 0 ? 0.f : -kInf);
  const bool writes_hist = lead && (p > 0 || (p == 0 && k == 0));
  if (p >= 0 && lead) hv[li] = v;
  if (aux && lane < 8 && !REV) own1[lane] = -kInf;  // alpha_0 of the order-1 states
  if (REV && writes_hist && nf > 0 && a.beta) a.beta[((long long)b * a.T + nf - 1) * kC + p] = 0.f;
  float O = 0.f;  // the common offset
  if (wave == 0) {  // are the four members on one XCD? (placement: speed only)
    const float xv = t4_take(&g_t4.xcc[q][lane & 3], 1u, lane < 4, abrt);
    const unsigned xi = __float_as_uint(xv);
    const unsigned x0 = __shfl(xi, 0);
    const bool same = __builtin_amdgcn_ballot_w64(lane < 4 && xi != x0) == 0;
    if (lane == 0) maxs[3] = same ? 1 : 0;
  }
  __syncthreads();
  const bool same_xcd = maxs[3] != 0;

  for (int i = 0; i < nf; ++i) {
    const int f = REV ? nf - 1 - i : i;
    T4STAMP(a, q, k, wave, i, 0);
    // a wait that times out raises this step's abort flag (by parity: a wave
    // already polling for step i + 1 cannot change what the others read here)
    int* ab = abrt + (i & 1);
    float m4 = -kInf;  // the max of the vector one step older: this step's offset
    // ---- this step's inputs (the words of step i), before the barrier
    if (sw || aux) {
      if (i >= 1) {
        const float mv = t4_take(&MX[(i - 1) & 1][lane & 3], (unsigned)i, lane < 4, ab);
        m4 = lane < 4 ? mv : -kInf;
      }
      m4 = fmaxf(m4, __shfl_xor(m4, 1));
      m4 = fmaxf(m4, __shfl_xor(m4, 2));
      m4 = __shfl(m4, 0);
      if (sw) {
        // forward: stage[jl][x - 1] = alpha_i[(x, j+1)]; backward:
        // stage[zl][y - 1] = beta_{t+1}[(z, y)] (the lead lanes, one word each)
        int m, idx, row, col;
        if (!REV) {
          const int jl = e & 7, xi = e >> 3;
          m = xi >> 3;
          idx = (xi & 7) * 32 + 8 * k + jl;
          row = jl;
          col = xi;
        } else {
          const int zl = e >> 5, yi = e & 31;
          m = yi >> 3;
          idx = (8 * k + zl) * 8 + (yi & 7);
          row = zl;
          col = yi;
        }
        float sv = REV ? 0.f : -kInf;  // step 0: alpha_0 (order 2) = -inf, beta = 0
        if (i >= 1) sv = t4_take(&X[i & 1][m][idx], (unsigned)i, lead, ab);
        if (lead) stage[(i & 1) * 256 + row * 32 + col] = sv;
      } else if (REV && k == 0) {
        // state 0's order-1 sources beta_{t+1}[y], y = lane + 1
        float sv = 0.f;
        if (i >= 1)
          sv = t4_take(&X[i & 1][(lane & 31) >> 3][256 + (lane & 7)], (unsigned)i, lane < 32, ab);
        if (lane < 32) stage1[(i & 1) * 32 + lane] = sv;
      }
    } else if (loader) {
      // loaders: frame i landed (frames i+1 .. i+P-2 may stay in flight)
      const int mine = (Gm::template ninstr<REV>() - (wave - kT4Ld) + 1) / 2;
      wait_vmcnt((Gm::P - 2) * mine);
    } else if (numer) {
      nu.step(lds, a, b, lane, i);
    }
    T4STAMP(a, q, k, wave, i, 1);
    lds_barrier();
    T4STAMP(a, q, k, wave, i, 2);
    if (*(volatile int*)ab) break;
    if (!sw && !aux) {
      // loaders: frame i - 1's slot is free, the frame P - 1 ahead goes in
      if (loader) t4_issue<BF16, REV>(a, b, k, nf, i + Gm::P - 1, wave - kT4Ld, lane, ldsb);
      // the writer: the checkpoint rows of the vector of step i (forward:
      // frame i's alpha; backward: the beta after frame nf - 1 - i, row
      // nf - 1 - i), from the values the state lanes left, and its offset
      if (wave == kT4Wr) {
        if (i >= 1) O += spb[(i - 1) & 1];
        if (!REV || i >= 1) t4_rows<REV>(a, b, k, REV ? nf - 1 - i : i, hv + (i & 1) * 272, O, lane);
      }
      continue;
    }
    // this member's max of the vector of step i (gathered during step i - 1)
    if (aux && lane == 0) {
      const float mm = tri_dec(maxs[i % 3]);
      maxs[i % 3] = tri_enc(-kInf);
      t4_pub(&MX[i & 1][k], t4_word((unsigned)(i + 1), mm), same_xcd);
    }
    const float sp = i == 0 ? 0.f : (__builtin_isfinite(m4) ? floorf(m4) : 0.f);
    if (wave == 0 && lane == 0) spb[i & 1] = sp;
    const long long fb = ((long long)b * a.T + f) * (long long)(kC * Gm::RB);
    const unsigned char* slot = lds + (i % Gm::P) * Gm::template slot<REV>();
    const int mis = (int)((fb + (long long)(1 + 8 * k) * Gm::RB) & 15);  // every run's
    const unsigned char* row0 = slot + 16 * Gm::NRC + (int)(fb & 15);
    const float* st = stage + (i & 1) * 256;
    const float a0 = __shfl(v, 8);  // aux wave: alpha_i[0] (lane 8), forward
    float r = -kInf;
    if (sw) {
      // half h of the state's terms, then the pair's logsumexp: each half's
      // safe max and sum, combined across the two lanes
      float t[17];
      if (!REV) {
        const int jl = hi, y = lo + 1;
        const unsigned char* vb = slot + mis + (jl * kR + y) * Gm::es + 16 * h * Gm::RUNB;
        const float* sx = st + jl * 32 + 16 * h;
        if (h == 0) {
          float wb;
          const unsigned dw = *(const volatile __attribute__((address_space(3))) unsigned*)(
              slot + Gm::BLK + 4 * e);
          if constexpr (BF16) {
            const long long row = 33 + 32 * (8 * k + jl) + (y - 1);
            const int hs = (int)((fb + row * Gm::RB) & 2);
            wb = __uint_as_float((hs ? dw >> 16 : dw & 0xffffu) << 16);
          } else {
            wb = __uint_as_float(dw);
          }
          t[16] = v + wb;                                   // the blank self loop
          t[0] = own1[(i & 1) * 8 + jl] + t4_w<BF16>(vb);  // from the order-1 state j+1
        } else {
          t[16] = -kInf;
          t[0] = sx[-1] + t4_wn<BF16>(vb);                  // x = 16
        }
        // terms x = 16 h + 1 .. 16 h + 15 (h = 1: 17 .. 31, and x = 32 below)
#pragma unroll
        for (int xx = 1; xx < 16; ++xx) t[xx] = sx[xx - 1] + t4_wn<BF16>(vb + xx * Gm::RUNB);
        if (h == 1) t[16] = sx[15] + t4_wn<BF16>(vb + 16 * Gm::RUNB);  // x = 32
      } else {
        const int zl = hi, xx = lo + 1;
        const unsigned char* vb = slot + mis + xx * Gm::RUNB + zl * kR * Gm::es + 16 * h * Gm::es;
        const float* sy = st + zl * 32 + 16 * h;
        // h = 0: the blank and labels 1..16; h = 1: labels 17..32 (row
        // positions 0..16 from vb)
        float w[17];
        if constexpr (BF16) {
          // nine aligned dwords and a funnel shift per pair: the row's
          // 2-byte alignment varies by lane
          typedef const __attribute__((address_space(3))) unsigned lds_u32;
          const uintptr_t va = (uintptr_t)vb;
          const unsigned char* b4 = (const unsigned char*)(va & ~(uintptr_t)3);
          const unsigned sh = (unsigned)(va & 2) * 8;
          unsigned d[9];
#pragma unroll
          for (int m = 0; m < 9; ++m) d[m] = *(lds_u32*)(b4 + 4 * m);
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const unsigned pr = __builtin_amdgcn_alignbit(d[m + 1], d[m], sh);
            w[2 * m] = __uint_as_float(pr << 16);
            w[2 * m + 1] = __uint_as_float(pr & 0xffff0000u);
          }
          w[16] = __uint_as_float((sh ? d[8] >> 16 : d[8] & 0xffffu) << 16);
        } else {
#pragma unroll
          for (int y = 0; y <= 16; ++y) w[y] = t4_wn<BF16>(vb + y * Gm::es);
        }
        t[0] = h == 0 ? v + w[0] : -kInf;
#pragma unroll
        for (int y = 1; y <= 16; ++y) t[y] = w[y] + sy[y - 1];
      }
      float m = t[0];
#pragma unroll
      for (int u = 1; u < 17; ++u) m = fmaxf(m, t[u]);
      const float c = __builtin_isfinite(m) ? m : 0.f;
      const float l = c * kLog2e;
      float ss = 0.f;
#pragma unroll
      for (int u = 0; u < 17; ++u) ss += lt_exp_off(t[u], l);
      const float co = __shfl_xor(c, 1), so = __shfl_xor(ss, 1);
      const float cc = fmaxf(ss > 0.f ? c : -kInf, so > 0.f ? co : -kInf);
      const float cf = __builtin_isfinite(cc) ? cc : 0.f;
      const float tot = ss * lt_exp(c - cf) + so * lt_exp(co - cf);
      // the pair adds in lane order, so both lanes hold the same value
      const float tot2 = h == 0 ? tot : so * lt_exp(co - cf) + ss * lt_exp(c - cf);
      r = (cf + lt_log(tot2)) - sp;
      if (lead) {
        t4_pub(&X[(i + 1) & 1][k][REV ? lo * 8 + hi : hi * 32 + lo], t4_word((unsigned)(i + 1), r),
               same_xcd);
        hv[((i + 1) & 1) * 272 + li] = r;  // its checkpoint row: the writer wave
      }
      v = r;
    } else if (p >= 0) {  // the aux wave's states
      if (!REV) {
        if (lane < 8) {  // order-1 state 1 + 8k + lane
          const float tb = v + t4_w<BF16>(slot + mis + lane * kR * Gm::es);
          const float tl = a0 + t4_w<BF16>(row0 + p * Gm::es);
          r = log_plus(tb, tl) - sp;
          own1[((i + 1) & 1) * 8 + lane] = r;
        } else {  // state 0: the blank self loop only (contexts.py:216-217)
          r = (v + t4_w<BF16>(row0)) - sp;
        }
      } else {
        float x[33];
        float tb;
        if (lane < 8) {  // order-1 source z = 1 + 8k + lane: row z of run 0
          const unsigned char* vb = slot + mis + lane * kR * Gm::es;
          tb = v + t4_w<BF16>(vb);
#pragma unroll
          for (int y = 1; y <= 32; ++y) x[y - 1] = t4_w<BF16>(vb + y * Gm::es) + st[lane * 32 + y - 1];
        } else {  // source 0: row 0, next(0, y) = the order-1 state y
          const float* s1 = stage1 + (i & 1) * 32;
          tb = v + t4_w<BF16>(row0);
#pragma unroll
          for (int y = 1; y <= 32; ++y) x[y - 1] = t4_w<BF16>(row0 + y * Gm::es) + s1[y - 1];
        }
        x[32] = -kInf;
        r = t4_lse(tb, x, sp);
        if (lane < 8) t4_pub(&X[(i + 1) & 1][k][256 + lane], t4_word((unsigned)(i + 1), r), same_xcd);
      }
      hv[((i + 1) & 1) * 272 + li] = r;
      v = r;
    }
    // this member's max of the new vector (state 0: every forward member holds
    // the same alpha[0]; backward, member 0 alone)
    float lm = (p > 0 || (p == 0 && (k == 0 || !REV))) ? r : -kInf;
    lm = gmax<6>(lm, 6);
    if (lane == 0) atomicMax(&maxs[(i + 1) % 3], tri_enc(lm));
    O += sp;
    T4STAMP(a, q, k, wave, i, 3);
  }
  lds_barrier();  // the last step's values and offset, for the writer
  if (wave == kT4Wr) {
    // forward: the padding frames carry alpha_nf (lattices.py:460-461)
    if (!REV && nf > 0 && !(abrt[0] | abrt[1])) {
      O += spb[(nf - 1) & 1];
      for (int t = nf; t < a.T; ++t) t4_rows<REV>(a, b, k, t, hv + (nf & 1) * 272, O, lane);
    } else if (!REV && nf == 0) {
      for (int t = 0; t < a.T; ++t) t4_rows<REV>(a, b, k, t, hv, 0.f, lane);
    }
    return;
  }
  if (loader) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the wave
    return;
  }
  const bool aborted = (*(volatile int*)abrt | *(volatile int*)(abrt + 1)) != 0;
  if (wave == kT4Num) {
    if (numer) {
      if (aborted) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else nu.finish(a, b, lane);
    }
    return;
  }
  if (REV) return;
  if (aborted) {
    if (k == 0 && wave == 0 && lane == 0) {
      if (a.log_z) a.log_z[b] = __builtin_nanf("");
      if (a.loss) a.loss[b] = __builtin_nanf("");
    }
    return;
  }
  // ---- forward end: padding frames carry alpha_nf (lattices.py:460-461);
  // log_z = O + log sum_q exp(alpha_nf[q]) over the quad's states: every wave
  // of every member publishes its (max, sum), member 0 wave 0 combines them
  const bool cnt = lead && (p > 0 || (p == 0 && k == 0));
  const float mx = gmax<6>(cnt ? v : -kInf, 6);
  const float c = __builtin_isfinite(mx) ? mx : 0.f;
  const float s = gsum<6>(cnt ? lt_exp(v - c) : 0.f, 6);
  if (lane == 0) {
    t4_put(&g_t4.fin[b][9 * k + wave][0], t4_word(1u, c));
    t4_put(&g_t4.fin[b][9 * k + wave][1], t4_word(1u, s));
  }
  if (k != 0 || wave != 0) return;
  const bool want = lane < 36;
  const float pc = t4_take(&g_t4.fin[b][want ? lane : 0][0], 1u, want, abrt);
  const float ps = t4_take(&g_t4.fin[b][want ? lane : 0][1], 1u, want, abrt);
  float M = (want && ps > 0.f) ? pc : -kInf;
  M = gmax<6>(M, 6);
  const float cm = __builtin_isfinite(M) ? M : 0.f;
  float S = (want && ps > 0.f) ? ps * lt_exp(pc - cm) : 0.f;
  S = gsum<6>(S, 6);
  if (lane == 0) {
    const float lz = (*(volatile int*)abrt | *(volatile int*)(abrt + 1)) ? __builtin_nanf("")
                                                                         : O + (cm + lt_log(S));
    if (a.log_z) a.log_z[b] = lz;
    __hip_atomic_store(&g_t4.lz[b], lz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(&g_t4.cnt[b], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 1) {
      const float nm = __hip_atomic_load(&g_t4.num[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.loss) a.loss[b] = lz - nm;
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(64 * kT4Waves) void tri4_kernel(const T4Args a, const KArgs ka) {
  const int bid = (int)blockIdx.x;
  const int nq = 2 * a.B;
  if (bid < 32 * a.G) {
    const int g = bid >> 5, r = bid & 31, k = r >> 3, q = 8 * g + (r & 7);
    if (q >= nq) return;
    if (q < a.B) t4_member<BF16, false>(a, ka, q, q, k);
    else t4_member<BF16, true>(a, ka, q, q - a.B, k);
  }
}

}  // namespace

namespace lt_impl {
// The quad design applies to V = 32 trigram Log checkpointing with B <= 32,
// U < 128, while the 8B member workgroups fit the CUs at once.
bool tri4_eligible(int V, int n, int B, int U, int cus) {
  // measured slower than the one-workgroup recursions (header): only the
  // diagnostic build runs it, on request (LT_TRI4=1)
  if (!tune_int("LT_TRI4", 0)) return false;
  return V == 32 && n == 2 && B >= 1 && B <= kT4MaxB && U < 128 && 8 * B <= cus;
}

int launch_tri4(const Plan& pl, bool bf16, float* alpha, float* beta, float* alpha_num,
                float* beta_num, float* log_z, float* num, float* loss, long long w_bytes,
                hipStream_t st) {
  const KArgs& ka = pl.a;
  T4Args a;
  a.W = ka.W;
  a.w_bytes = w_bytes;
  a.nfr = ka.nfr;
  a.labels = ka.labels;
  a.nlab = ka.nlab;
  a.alpha = alpha;
  a.beta = beta;
  a.alpha_num = alpha_num;
  a.beta_num = beta_num;
  a.log_z = log_z;
  a.num = num;
  a.loss = loss;
  a.B = ka.B;
  a.T = ka.T;
  a.U = ka.U;
  a.G = (2 * a.B + 7) / 8;
  a.stamps = nullptr;
#ifdef LT_STAMPS
  {
    const char* sp = tune_str("LT_T4_STAMPS");
    a.stamps = sp ? (long long*)strtoull(sp, nullptr, 0) : nullptr;
  }
#endif
  void* scratch = nullptr;
  hipError_t e = hipGetSymbolAddress(&scratch, HIP_SYMBOL(g_t4));
  if (e == hipSuccess) e = hipMemsetAsync(scratch, 0, sizeof(T4Scratch), st);
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  const void* k = bf16 ? (const void*)tri4_kernel<true> : (const void*)tri4_kernel<false>;
  const int lds = bf16 ? std::max(T4Lds<true, false>::total, T4Lds<true, true>::total)
                       : std::max(T4Lds<false, false>::total, T4Lds<false, true>::total);
  e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  KArgs kk = ka;
  void* args[] = {(void*)&a, (void*)&kk};
  const unsigned grid = 32u * a.G;
  e = hipLaunchKernel(k, dim3(grid), dim3(64 * kT4Waves), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}
}  // namespace lt_impl
