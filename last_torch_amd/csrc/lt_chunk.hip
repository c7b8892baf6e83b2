// lt_chunk.hip -- chunked-time two-level scan for the bigram Log lattice
// (FullNGram n = 1, V <= 32, FrameDependent): loss and d(loss)/dW with
// every utterance split into K chunks of L frames, so the serial chain per
// utterance is L + K steps instead of T.
//
// Reference (last_torch/): the denominator recursion lattices.py:379-496
// with FrameDependent.forward (alignments.py:286-297) and FullNGram
// forward_reduce (contexts.py:207-230); the backward / marginals of
// alignments.py:300-318 composed in reverse frame order (lattices.py:686-799,
// defect D4 fixed); the numerator lattices.py:250-377 with
// FrameDependent.string_forward (alignments.py:320-329); the loss
// lattices.py:131-183. Log semiring semirings.py:184-305 (safe max).
//
// Bigram structure (contexts.py:190-205): next(p, y) = y for y >= 1, the
// blank arc (y = 0) loops. States 1..V form a dense V x V "core"; state 0
// (the start) has only its blank self loop as in-arc. So one frame is the
// block matrix  M_t = [[w00, w0.], [0, Mc_t]]  in the log semiring, with
// Mc_t[p][q] = W[p][q] (+) (p == q ? W[p][0] : zero).
//
// Two launches (one call of lt_loss_grad):
//   A  one wave per chunk: the chunk's transfer matrix
//      P_k = M_{t0} ... M_{t1-1} in scaled linear space. The 32 x 32 core
//      product runs on the matrix cores (v_mfma_f32_32x32x2_f32: exact f32
//      FMA chains) as X <- E_t^T X with X = P^T, one column scale per start
//      state; the state-0 row and the state-0 self loop on the side. Also
//      the numerator's group bands (the string lattice's frame steps
//      composed over kGrp frames) and the frame offsets.
//   B  one workgroup per utterance: the den alpha / beta vectors at every
//      chunk boundary (K steps of a 33 x 33 log-semiring vector-matrix
//      product each), the numerator alpha / beta over the groups with the
//      values at the chunk boundaries kept; log_z, num, loss.
//      A and B share ck_ab_kernel: the walks follow A's chunks through
//      per-chunk ready flags (write-through stores, agent-scope acquire), so
//      they run beside the transfers instead of after them (B > CUs or
//      LT_CHUNK_FUSE=0: ck_combine_kernel after the launch).
//   C  ck_marg_kernel      one workgroup per chunk: the chunk's W staged in
//      LDS once; local den / num alpha and beta recursions from the
//      boundary values (four waves side by side), then the arc marginals of
//      every frame, normalised by the frame's own total (= Z up to
//      rounding), den minus num, times the incoming gradient -> dW.
// HBM traffic: W is read twice (A and C) and dW written once, plus G and the
// chunk records (~10 % of W) -- the SURVEY 8(d) accounting.
//
// Exactness of the scaled linear spaces: with every weight of a frame finite
// and max - min <= kRange (checked per frame in A; utterances that fail go
// to the frame-serial kernels), every core state reaches every core state in
// one frame with a weight within e^kRange of any other, so a value that
// underflows relative to its vector's max (< 2^-126) carries a marginal below
// e^(kRange - 87): nothing the tolerance can see. The start state, whose
// alpha/beta can drift arbitrarily far from the core's, is kept in log space
// throughout.
#include "lt_kernels.h"

#include <unistd.h>

#include <atomic>
#include <chrono>

namespace {

typedef float v16f __attribute__((ext_vector_type(16)));

// the strict range (lt_chunk_forward's fast path): every weight of a frame
// within e^61 of its max, as E = exp(W - c) >= kEmin
constexpr float kEmin = 0x1p-88f;
constexpr int kRec = 1248;      // floats per chunk record (whole 128-byte lines)
constexpr int kRowT = 36;       // row stride of the transposed core in a record
constexpr int kChunkLds = 40 * 1024;  // phase C LDS per workgroup (four per CU)
constexpr int kMargWaves = 4;   // phase C: waves per workgroup (recursions on 0-3)
constexpr int kGrp = 7;         // frames per numerator group (band offsets 0..kGrp)
constexpr float kCert = 64.f;   // phase C's per-frame certificate: log2(max alpha max beta e^c / Z)
#ifndef LT_AB_WAVES
#define LT_AB_WAVES 3
#endif
constexpr int kAbWaves = LT_AB_WAVES;  // ck_ab_kernel: waves per SIMD its registers allow
#ifndef LT_CK_APF
#define LT_CK_APF 1
#endif
constexpr int kApf = LT_CK_APF;  // phase A: frames in registers ahead (1 or 2)
static_assert(kApf == 1 || kApf == 2, "phase A prefetch depth");
constexpr unsigned kSpinMax = 1u << 20;
#ifndef LT_CK_SPLIT
#define LT_CK_SPLIT 0
#endif
#ifndef LT_CK_WPRIO
#define LT_CK_WPRIO 3
#endif
#ifndef LT_CK_PRIO
#define LT_CK_PRIO 3
#endif
#ifndef LT_CK_ROT
#define LT_CK_ROT 1
#endif
#ifndef LT_CK_PF
#define LT_CK_PF 0
#endif
// LT_CK_NOACQ: what one launch's workgroups hand each other (the records
// and bands phase A publishes for the phase-1 walks; the boundary rows the
// phase-2 walks publish for phase C) is read with sc1 loads, which bypass the
// reading CU's L1, instead of plain loads behind an agent-scope acquire
// (buffer_inv sc1: an L1 invalidation per poll, ~1.7 us and more with four
// workgroups on the CU, MI355X_MICROARCH.md)
#ifndef LT_CK_NOACQ
#define LT_CK_NOACQ 1
#endif
constexpr bool kNoAcq = LT_CK_NOACQ != 0;
#ifndef LT_CK_ALDS
#define LT_CK_ALDS 1
#endif
constexpr bool kALds = LT_CK_ALDS != 0;  // phase A: frames through an LDS ring (two slots a wave)
constexpr int kASlot = 5 * 1024;         // bytes per slot (a fp32 bigram frame: 5 DMA instructions)
constexpr int kALdsBytes = 4 * 2 * kASlot;  // dynamic LDS of phase A's workgroups
#ifndef LT_CK_BANDMIX
#define LT_CK_BANDMIX 0
#endif
constexpr bool kBandMix = LT_CK_BANDMIX != 0;  // phase A: band steps between the MFMAs
#ifndef LT_CK_EPIPE
#define LT_CK_EPIPE 0
#endif
constexpr bool kEpipe = LT_CK_EPIPE != 0;  // phase C den chains: the next frame's E a step ahead
#ifndef LT_WALK_SLOTS
#define LT_WALK_SLOTS 3
#endif
constexpr int kWalkSlots = LT_WALK_SLOTS;        // phase B: den walk record ring depth (LDS)
constexpr int kRecNi = (4 * kRec + 1023) / 1024;  // LDS-DMA wave instructions per record
constexpr int kWalkSlot = kRecNi * 1024;         // bytes per ring slot
constexpr int kWalkLds = 2 * kWalkSlots * kWalkSlot;  // dynamic LDS of the walk launches  // phase B's bound on polls without progress (~1 s)
// record layout (floats): [0, 1152) X^T rows: rec[i * 36 + j] = X[i][j] =
// P_scaled[j][i] (start core state j -> end core state i); [1152, 1184)
// per-start-state (column) power-of-two scales ej (int); [1184, 1216) the
// state-0 row rt[i]; 1216 rho (int, log2 scale of rt); 1217 pi (log of
// P00 relative to csum); 1218 csum (sum of the frames' offsets c_t);
// 1219 flag (range violation); 1220 live frames.
constexpr int kRecEj = 1152, kRecRt = 1184, kRecRho = 1216, kRecPi = 1217, kRecCs = 1218,
              kRecFlag = 1219, kRecN = 1220;

struct CkArgs {
  const unsigned char* W;  // [B,T,C,R] fp32 / bf16
  const int* nfr;
  const int* labels;       // [B,U]
  const int* nlab;
  const float* grad;       // [B] nullable (ones)
  float* rec;              // [B*K][kRec]
  float* nb;               // [B,K,NGc,NPG,kGrp+1] numerator group bands (log2)
  int* uflag;              // [B] 1: utterance goes to the frame-serial kernels
  float* abd;              // [B,K+1,CP] den alpha at chunk starts (log)
  float* bbd;              // [B,K+1,CP] den beta at chunk starts
  float* nabd;             // [B,K+1,NPG] num alpha at chunk starts
  float* nbbd;             // [B,K+1,NPG] num beta at chunk starts
  float* cf;               // [B,T] frame offsets c_t = ceil(max W_t) (phase A's)
  // hand-off words, tagged per call (no zeroing pass): a word carries this
  // call's tag or is not yet written in this call (an older call's tag, or
  // whatever the scratch held: a 62-bit / 40-bit random tag matches it with
  // probability 2^-62 / 2^-40)
  unsigned long long* ready;  // [B,K] ep_tag | state (1 ok, 2 / 3 out of range) of chunk k
  unsigned long long* prog;   // [B,4] pg_tag | phase 2's boundaries done per walk (< 2^24)
  unsigned long long ep_tag, pg_tag;
  float* mid;              // [B,2] phase 1's den alpha and num alpha offsets at the middle
  float* loss;
  float* log_z;            // state copies (read by C)
  float* num;
  float* lz_out;           // the caller's, nullable
  float* num_out;
  void* dW;
  int B, T, U, V, C, R, FR, NP, NPG, PPL, CP;
  int L, K;                // frames per chunk, chunks per utterance
  int NGc;                 // numerator groups per chunk, ceil(L / kGrp)
  int nc, wpos;            // ck_ab_kernel: nc walking workgroups (B fused, 0 not) from block wpos
  int nbs;                 // floats per chunk of numerator bands (whole 128-byte lines)
  int half;                // 1: the walks stop at the middle (phase 1), phase C's launch finishes them
  int cont;                // phase C's launch: blocks [0, B) finish the walks (phase 2)
  int local;               // LocallyNormalizedWeightFn: no denominator
  int strict;              // 1 (lt_chunk_forward): a chunk outside the strict range (flag 3)
                           // leaves the fast path in B; 0: phase C's certificate decides
  int dbg;                 // diagnostic builds (LT_DIAG) only: role ablations
  int pf;                  // phase C: prefetch distance in blocks (0: none), LT_CK_PF
  long long* stamps;       // diagnostic builds only: per-workgroup s_memtime marks
  long long FB;            // bytes per frame
  // phase A per-wave LDS carve
  int a_slots, a_ni, a_slot_bytes, a_wave_bytes, a_off_rt, a_off_tab;
  // phase B LDS carve
  int b_ni, b_slots, b_off_ra, b_off_rb, b_off_ga, b_off_gb, b_gslots, b_gslot, b_off_buf;
  // phase C LDS carve
  int c_ni, c_off_ad, c_off_bd, c_off_an, c_off_bn, c_off_nw, c_off_fs, c_off_tab, c_off_cf,
      c_off_buf, c_off_fl, c_off_e, c_bytes;
};

// lanes l and l ^ 32 combined (v_permlane32_swap: both halves get both)
LT_DEVINL float half_sum(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
// lane l ^ 32's value
LT_DEVINL float half_other(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return (threadIdx.x & 32) ? __int_as_float(p[0]) : __int_as_float(p[1]);
}
// lane l gets v of lane l-1 (lane 0: fill)
LT_DEVINL float from_prev(float v, float fill) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(fill), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
// lane 0 gets lane 63 (rotate right by one)
LT_DEVINL float rot_prev(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x13C, 0xF, 0xF, false));
}
LT_DEVINL float rot_next(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x134, 0xF, 0xF, false));
}

LT_DEVINL float safe_max(float m) { return __builtin_isfinite(m) ? m : 0.f; }
#ifdef LT_DIAG
#define CK_STAMP(k)                                                                  \
  do {                                                                               \
    if (a.stamps && !LT_ABL(a, 64 | 256) && threadIdx.x == 0)                         \
      a.stamps[(long long)blockIdx.x * 8 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
// phase B: per utterance b (the walking workgroup's), two marks per wave
#define CK_WSTAMP(k)                                                                 \
  do {                                                                               \
    if (a.stamps && LT_ABL(a, 64) && (threadIdx.x & 63) == 0)                         \
      a.stamps[(long long)b * 8 + (k)] = (long long)__builtin_amdgcn_s_memtime();     \
  } while (0)
// phase A (LT_CK_DBG bit 256): per chunk wave, after phase C's per-workgroup marks
#define CK_ASTAMP(k)                                                                 \
  do {                                                                               \
    if (a.stamps && LT_ABL(a, 256) && (threadIdx.x & 63) == 0)                        \
      a.stamps[(long long)a.B * a.K * 8 + (long long)id * 4 + (k)] =                  \
          (long long)__builtin_amdgcn_s_memtime();                                   \
  } while (0)
#else
#define CK_ASTAMP(k) \
  do {               \
  } while (0)
#define CK_WSTAMP(k) \
  do {               \
  } while (0)
#define CK_STAMP(k) \
  do {              \
  } while (0)
#endif
// max of three with no NaN quieting of the operands (a NaN in W is caught
// by the exponential test of phase A, not by the max)
LT_DEVINL float max3_raw(float x, float y, float z) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
// lane 0's float (readfirstlane is an int builtin: never pass it a float)
LT_DEVINL float first_lane(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// k index of k-step s in lane half h (the rows register s of the 32x32
// accumulator holds in that half): the MFMA's K order is free, so the
// accumulator feeds the next product's B operand with no data movement
LT_DEVINL int kstep(int s, int h) { return (s & 3) + 8 * (s >> 2) + 4 * h; }

template <bool BF16>
LT_DEVINL float ldsw(const unsigned char* fr, int e) {
  if constexpr (BF16) return __uint_as_float(((unsigned)((const unsigned short*)fr)[e]) << 16);
  else return ((const float*)fr)[e];
}

// LDS-DMA of `bytes` bytes at global byte offset `off` of `base` into LDS at
// `lds_addr` (1 KiB per wave instruction, `ni` instructions; the copy starts
// at the 16-byte granule holding `off`: the data sits at lds + (off & 15)).
// Lanes past the end re-load the last granule into the slack.
LT_DEVINL void dma_issue(const unsigned char* base, long long off, long long bytes,
                         unsigned lds_addr, int ni, int lane, int wave0 = 0, int nwaves = 1,
                         bool sc1 = false) {
  const long long a0 = off & ~15LL;
  const int n16 = (int)((off + bytes - a0 + 15) >> 4);
  for (int i = wave0; i < ni; i += nwaves) {
    int g = lane + 64 * i;
    g = g < n16 ? g : n16 - 1;
    if (sc1) glds16_sc1(base + a0 + 16LL * g, lds_addr + 1024u * i);
    else glds16(base + a0 + 16LL * g, lds_addr + 1024u * i);
  }
}

// One LDS-DMA dword per 128-byte line of [off, off + bytes) of `base`, every
// lane's dword landing in the same 256-byte LDS scratch (discarded): the
// lines come into the XCD's L2 (and the memory-side cache) for a block that
// will stage them later. 8 KiB of lines per wave instruction.
LT_DEVINL void pf_lines(const unsigned char* base, long long off, long long bytes,
                        unsigned lds_addr, int lane) {
  const long long a0 = off & ~127LL;
  const int nl = (int)((off + bytes - a0 + 127) >> 7);
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  for (int i = 0; 64 * i < nl; ++i) {
    const int g = min(lane + 64 * i, nl - 1);
    const void* src = base + a0 + 128LL * g;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds_addr)
        : "memory");
  }
}

// dma_issue's copy, wave instructions [i0, i1) only (one wave)
LT_DEVINL void dma_range(const unsigned char* base, long long off, long long bytes,
                         unsigned lds_addr, int i0, int i1, int lane) {
  const long long a0 = off & ~15LL;
  const int n16 = (int)((off + bytes - a0 + 15) >> 4);
  for (int i = i0; i < i1; ++i) {
    int g = lane + 64 * i;
    g = g < n16 ? g : n16 - 1;
    glds16(base + a0 + 16LL * g, lds_addr + 1024u * i);
  }
}

// wave-uniform max / sum over all 64 lanes with DPP only (no LDS round trip):
// butterflies inside each row of 16, then row_bcast:15 / row_bcast:31 fold
// rows 0-1 into 2-3, and lane 63 holds the total
template <bool MAX>
LT_DEVINL float wred(float v) {
  auto op = [](float x, float y) { return MAX ? fmaxf(x, y) : x + y; };
  v = op(v, xchg<0>(v));
  v = op(v, xchg<1>(v));
  v = op(v, xchg<2>(v));
  v = op(v, xchg<3>(v));
  const float r15 = __int_as_float(__builtin_amdgcn_update_dpp(
      MAX ? __float_as_int(v) : 0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v = op(v, r15);
  const float r31 = __int_as_float(__builtin_amdgcn_update_dpp(
      MAX ? __float_as_int(v) : 0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  v = op(v, r31);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
LT_DEVINL float wmax_u(float v) { return wred<true>(v); }
LT_DEVINL float wsum_u(float v) { return wred<false>(v); }

template <bool BF16>
LT_DEVINL float ldg(const unsigned char* base, long long e) {
  if constexpr (BF16) return __uint_as_float(((unsigned)((const unsigned short*)base)[e]) << 16);
  else return ((const float*)base)[e];
}

// Numerator gather offsets of string position u (contexts.py:109-146
// walk_states, lattices.py:314-338, bigram next(p, y) = y): boff = element of
// a frame holding the blank weight of position u (state ctx_u = last valid
// label before u, 0 if none), loff = element holding the weight of the arc
// into u (from ctx_{u-1} with label y_u; epsilon / out-of-range labels read
// label 1, make_safe_classes), -1 for u = 0 or u past the string. `lab` is
// the utterance's labels staged in LDS.
LT_DEVINL void string_offsets(const CkArgs& a, const int* lab, int u, int* boff, int* loff) {
  auto valid = [&](int y) { return y >= 1 && y <= a.V; };
  int ctx = 0, pc = 0;
  int j = min(u, a.U) - 1;
  for (; j >= 0; --j)
    if (valid(lab[j])) { ctx = lab[j]; break; }
  // ctx_{u-1}: the same scan one position earlier
  if (u >= 1) {
    if (j == u - 1) {  // label u-1 itself was the last valid one
      for (int i = u - 2; i >= 0; --i)
        if (valid(lab[i])) { pc = lab[i]; break; }
    } else {
      pc = ctx;
    }
  }
  *boff = u < a.NP ? ctx * a.R : -1;
  if (u == 0 || u >= a.NP) {
    *loff = -1;
  } else {
    const int y = lab[u - 1];
    *loff = pc * a.R + (valid(y) ? y : 1);
  }
}

// log-space plus in base-2 units: m + log2(1 + 2^(n - m)); both operands
// -inf gives -inf (the clamp turns the NaN of -inf - -inf into -200)
LT_DEVINL float lse2_b2(float x, float y) {
  const float m = fmaxf(x, y), n = fminf(x, y);
  return m + __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(fmaxf(n - m, -200.f)));
}

// ---------------------------------------------------------------------------
// A: chunk transfer matrices (one wave per chunk). Frame data is loaded
// straight into registers two frames ahead (the compiler's own waits).
// ---------------------------------------------------------------------------
template <bool BF16, int PPL>
struct FrameRegs {
  float w[16];      // W[k+1][i+1] for the lane's 16 k-steps
  float wr0;        // W[0][i+1]
  float wbl;        // W[lane][0]   (the blank column, lanes <= V)
  float wdg;        // W[i+1][0]
  float w00;        // W[0][0]
  float gb[PPL], gl[PPL];  // numerator arc weights of the lane's positions
};

// Per-lane byte offsets of load_frame's loads inside a frame, fixed over the
// chunk: the frame is one buffer resource (scalar base, bounded), so a load
// costs no address arithmetic. The lane's k-step rows sit at compile-time
// immediates past vb (FULL) or at scalar offsets (srow).
template <int PPL>
struct FrameOffs {
  int vb, vr0, vbl, vdg, vgb[PPL], vgl[PPL];
  int srow[16];
};
LT_DEVINL constexpr int krow(int s) { return (s & 3) + 8 * (s >> 2); }
template <bool BF16, int PPL>
LT_DEVINL void frame_offsets(const CkArgs& a, int lane, const int* boff, const int* loff,
                             FrameOffs<PPL>& o) {
  const int R = a.R, i = lane & 31, h = lane >> 5, es = BF16 ? 2 : 4;
  o.vb = ((4 * h + 1) * R + i + 1) * es;  // row kstep(s, h) + 1, column i + 1
  o.vr0 = (i + 1) * es;
  o.vbl = lane * R * es;
  o.vdg = (i + 1) * R * es;
#pragma unroll
  for (int r = 0; r < PPL; ++r) {
    o.vgb[r] = max(boff[r], 0) * es;
    o.vgl[r] = max(loff[r], 0) * es;
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) o.srow[s] = krow(s) * R * es;
}
template <bool BF16>
LT_DEVINL float ldb(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (BF16)
    return __uint_as_float((unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0) << 16);
  else
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// Every lane issues every load (rows and columns past V read neighbouring
// bytes of the chunk or, past its end, the resource's zeros; mask_frame
// replaces them): no load sits under a branch, so the compiler's vmcnt
// bookkeeping across the prefetch stays exact.
template <bool BF16, int PPL, bool FULL>
LT_DEVINL void load_frame(const unsigned char* Wf, int bytes, const FrameOffs<PPL>& o,
                          FrameRegs<BF16, PPL>& f) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)Wf, (short)0, bytes, 0x00020000);
  constexpr int es = BF16 ? 2 : 4;
#pragma unroll
  for (int s = 0; s < 16; ++s)
    f.w[s] = FULL ? ldb<BF16>(r, o.vb + krow(s) * 33 * es, 0) : ldb<BF16>(r, o.vb, o.srow[s]);
  f.wr0 = ldb<BF16>(r, o.vr0, 0);
  f.wbl = ldb<BF16>(r, o.vbl, 0);
  f.wdg = ldb<BF16>(r, o.vdg, 0);
  f.w00 = ldb<BF16>(r, 0, 0);
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    f.gb[q] = ldb<BF16>(r, o.vgb[q], 0);
    f.gl[q] = ldb<BF16>(r, o.vgl[q], 0);
  }
}
// load_frame's values from a frame staged in LDS (LT_CK_ALDS: `fr` = the
// frame's first byte in the wave's ring slot)
template <bool BF16, int PPL, bool FULL>
LT_DEVINL void lds_frame(const unsigned char* fr, const FrameOffs<PPL>& o,
                         FrameRegs<BF16, PPL>& f) {
  constexpr int es = BF16 ? 2 : 4;
  auto rd = [&](int off) -> float {
    if constexpr (BF16) return __uint_as_float((unsigned)*(const unsigned short*)(fr + off) << 16);
    else return *(const float*)(fr + off);
  };
#pragma unroll
  for (int s = 0; s < 16; ++s) f.w[s] = FULL ? rd(o.vb + krow(s) * 33 * es) : rd(o.vb + o.srow[s]);
  f.wr0 = rd(o.vr0);
  f.wbl = rd(o.vbl);
  f.wdg = rd(o.vdg);
  f.w00 = rd(0);
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    f.gb[q] = rd(o.vgb[q]);
    f.gl[q] = rd(o.vgl[q]);
  }
}
// the values load_frame read for nothing (FULL: V = 32, every core value live)
template <bool BF16, int PPL, bool FULL>
LT_DEVINL void mask_frame(int V, int lane, const int* boff, const int* loff,
                          FrameRegs<BF16, PPL>& f) {
  const int i = lane & 31, h = lane >> 5;
  if constexpr (!FULL) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (!(kstep(s, h) < V && i < V)) f.w[s] = -kInf;
    if (i >= V) { f.wr0 = -kInf; f.wdg = -kInf; }
  }
  if (lane > V) f.wbl = -kInf;
#pragma unroll
  for (int r = 0; r < PPL; ++r) {
    if (boff[r] < 0) f.gb[r] = -kInf;
    if (loff[r] < 0) f.gl[r] = -kInf;
  }
}

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Write-through (sc1) stores for what phase B reads in the same launch: the
// bytes leave the XCD's L2 with the store, so the publishing wave needs only
// its own s_waitcnt vmcnt(0) before the flag -- no L2 write-back fence
// (MI355X_MICROARCH.md: a per-wave release fence costs the whole L2's dirty
// lines). A buffer resource per chunk region (bounds-checked).
LT_DEVINL __amdgpu_buffer_rsrc_t wt_rsrc(void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000);
}
LT_DEVINL void st_wt(__amdgpu_buffer_rsrc_t r, int idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, 4 * idx, 0, 0x10);
}
LT_DEVINL void st_wt(__amdgpu_buffer_rsrc_t r, int idx, int v) {
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)v, r, 4 * idx, 0, 0x10);
}
LT_DEVINL void st_wt4(__amdgpu_buffer_rsrc_t r, int idx, float x, float y, float z, float w) {
  const v4u v = {__float_as_uint(x), __float_as_uint(y), __float_as_uint(z), __float_as_uint(w)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, 4 * idx, 0, 0x10);
}

// Chunk k of utterance b: the transfer record, the numerator bands and the
// frame offsets, then the hand-off to phase B: record and bands stored
// write-through (sc1), the wave's s_waitcnt vmcnt(0), then one relaxed
// agent-scope flag store (1: inside the strict range; 3: a masked (-inf) or
// far-below-max weight, which only the relaxed path takes, under phase C's
// per-frame certificate; 2: a NaN / +inf weight or an all -inf frame, always
// the frame-serial kernels); phase B polls it and acquires (ChunkReady).
template <bool BF16, int PPL, bool FULL>
LT_DEVINL void transfer_role(const CkArgs& a, int b, int k, int wave) {
  __shared__ __attribute__((aligned(16))) float s_rt[4][32];
  __shared__ __attribute__((aligned(16))) float s_dg[4][32];
  __shared__ int s_lab[4][128];
  __shared__ __attribute__((aligned(16))) float2 s_g[4][128 + kGrp + 1];
  const int lane = threadIdx.x & 63;
  const int id = b * a.K + k;
  CK_ASTAMP(0);
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int t0 = k * a.L;
  const int t1 = min(t0 + a.L, nf);
  if (t0 >= t1) return;  // no live frame: phase B never reads this record
  const int V = a.V, NPG = a.NPG;
  const int i = lane & 31, h = lane >> 5;
  const int nt = t1 - t0;
  float* rt = s_rt[wave];
  float* sdg = s_dg[wave];  // the frame's core blank self loops E[p][0], p = 1..32
  int* lab = s_lab[wave];
  float2* sg = s_g[wave];  // the frame's numerator arc weights (log2) by position
  for (int j = lane; j < a.U; j += 64) lab[j] = a.labels[(long long)b * a.U + j];
  if (lane < 32) rt[lane] = 0.f;
  if (lane <= kGrp) sg[64 * PPL + lane] = make_float2(-kInf, -kInf);  // past the string
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  int boff[PPL], loff[PPL];
#pragma unroll
  for (int r = 0; r < PPL; ++r) {
    const int u = lane + 64 * r;
    boff[r] = -1;
    loff[r] = -1;
    if (u < NPG) string_offsets(a, lab, u, &boff[r], &loff[r]);
  }
  const long long es = BF16 ? 2 : 4;
  const unsigned char* W0 = a.W + ((long long)b * a.T + t0) * a.FR * es;
  CK_ASTAMP(1);

  v16f X;  // X = P^T, column j (lane & 31) = start state j+1; identity
#pragma unroll
  for (int r = 0; r < 16; ++r) X[r] = (kstep(r, h) == i && i < V) ? 1.f : 0.f;
  int ej = 0;         // column power-of-two scale (lane's column)
  int rho = -100000;  // rt scale (log2)
  float pi = 0.f;     // log2 P00 - csum
  float csum = 0.f;   // sum of the frames' offsets c_t (integers, log2 units)
  int bad = 0;        // 2: a NaN / +inf weight or an all -inf frame; 3: outside the strict range
  // numerator group bands: nbd[r][d] = log2 weight of the paths from
  // position s = lane + 64 r at the group's first frame to s + d after its
  // last (the string lattice's frame steps, lattices.py:340-377, composed)
  float nbd[PPL][kGrp + 1];
  const __amdgpu_buffer_rsrc_t nbr = wt_rsrc(a.nb + (long long)id * a.nbs, 4 * a.nbs);

  // the next frame in registers; the loads are unconditional (clamped to
  // the chunk's last frame) so the compiler's vmcnt tracking stays exact
  FrameRegs<BF16, PPL> fr;
  FrameOffs<PPL> fo;
  frame_offsets<BF16, PPL>(a, lane, boff, loff, fo);
  // LT_CK_ALDS: this wave's two ring slots in the launch's dynamic LDS
  extern __shared__ __attribute__((aligned(16))) unsigned char ck_dyn[];
  unsigned char* aring = ck_dyn + wave * 2 * kASlot;
  float cfl_lane = 0.f;  // LT_CK_ALDS: lane f holds frame f's offset
  auto goff = [&](int f) { return ((long long)b * a.T + t0 + f) * a.FB; };
  auto aissue = [&](int f) {
    dma_issue(a.W, goff(f), a.FB, lds_base_addr(aring) + (unsigned)((f & 1) * kASlot), a.a_ni, lane);
  };
  auto aframe = [&](int f) -> const unsigned char* {
    return aring + (f & 1) * kASlot + (int)(goff(f) & 15);
  };
  (void)aissue; (void)aframe;
  auto frame_ptr = [&](int f) { return W0 + (long long)min(f, nt - 1) * a.FR * es; };
  auto frame_bytes = [&](int f) { return (nt - min(f, nt - 1)) * a.FR * (int)es; };
  auto step = [&](FrameRegs<BF16, PPL>& F, int f, bool reload) {
    mask_frame<BF16, PPL, FULL>(V, lane, boff, loff, F);
    // numerator: band step over the group (positions past the string read -inf)
    // (diagnostic builds: LT_CK_DBG bit 1024 skips it -- timing only)
    const bool bands = !LT_ABL(a, 1024);
    const int jg = f / kGrp, flg = f - jg * kGrp;  // wave-uniform
    if (kBandMix && bands) {
      // LT_CK_BANDMIX: this frame's weights published now (F is reloaded
      // below); the band steps themselves run between the core product's
      // MFMAs, which they do not depend on
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        sg[lane + 64 * r] = make_float2(F.gb[r] * kLog2e, F.gl[r] * kLog2e);
      if (flg == 0) {
#pragma unroll
        for (int r = 0; r < PPL; ++r)
#pragma unroll
          for (int d = 0; d <= kGrp; ++d) nbd[r][d] = d ? -kInf : 0.f;
      }
    }
    if (!kBandMix && bands) {
      const int j = jg, fl = flg;
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        sg[lane + 64 * r] = make_float2(F.gb[r] * kLog2e, F.gl[r] * kLog2e);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if (fl == 0) {
#pragma unroll
        for (int r = 0; r < PPL; ++r)
#pragma unroll
          for (int d = 0; d <= kGrp; ++d) nbd[r][d] = d ? -kInf : 0.f;
      }
#pragma unroll
      for (int r = 0; r < PPL; ++r) {
        float2 gv[kGrp + 1];
#pragma unroll
        for (int d = 0; d <= kGrp; ++d) gv[d] = sg[lane + 64 * r + d];
#pragma unroll
        for (int d = kGrp; d >= 1; --d)
          if (d <= fl + 1) nbd[r][d] = lse2_b2(nbd[r][d] + gv[d].x, nbd[r][d - 1] + gv[d].y);
        nbd[r][0] += gv[0].x;
      }
      if (fl == kGrp - 1 || f == nt - 1) {  // source-major: 32 bytes per position
        static_assert(kGrp + 1 == 8, "two float4 per position");
        const int g0 = j * (kGrp + 1) * NPG;
#pragma unroll
        for (int r = 0; r < PPL; ++r)
          if (lane + 64 * r < NPG) {
            const int u = lane + 64 * r;
            st_wt4(nbr, g0 + 8 * u, nbd[r][0], nbd[r][1], nbd[r][2], nbd[r][3]);
            st_wt4(nbr, g0 + 8 * u + 4, nbd[r][4], nbd[r][5], nbd[r][6], nbd[r][7]);
          }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (kALds) {
      // frame f + 2 into the slot frame f came through (its reads into F have
      // returned: F was just used)
      if (f + 2 < nt && !LT_ABL(a, 8192)) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        aissue(f + 2);
      }
    }
    // the frame's offset c = ceil(max W log2 e), an integer in log2 units
    // (masked values are -inf), so every sum of offsets is exact
    float mx = max3_raw(F.wr0, F.wbl, F.w[15]);
#pragma unroll
    for (int s = 0; s < 15; s += 3) mx = max3_raw(mx, max3_raw(F.w[s], F.w[s + 1], F.w[s + 2]), mx);
    mx = wmax_u(mx);
    const bool cfin = __builtin_isfinite(mx);
    const float cl = cfin ? ceilf(mx * kLog2e) : 0.f;
    if constexpr (kALds) cfl_lane = lane == f ? cl : cfl_lane;  // stored after the frames
    else if (lane == 0) a.cf[(long long)b * a.T + t0 + f] = cl;
    // E_t^T as the A operand: lane (i, h), k-step s -> E[k][i]. The core
    // diagonal's blank self loop (alignments.py:294-297) is added beside
    // the product (Dg X after the MFMAs, rt Dg in the state-0 row), which
    // keeps the lane's diagonal k-step out of the registers.
    // Flags ride on the exponentials: a NaN weight gives a NaN E (fails
    // e >= 0); a weight below e^-61 of the frame's max, or -inf, gives
    // E < kEmin (outside the strict range, kept as an exact zero or a
    // small value: the relaxed path's per-frame certificate covers it).
    // (diagnostic builds: bit 4096 skips the exponentials and flags -- timing only)
    const bool noexp = LT_ABL(a, 4096);
    const float dgv = (FULL || i < V) ? (noexp ? F.wdg : lt_exp_off(F.wdg, cl)) : 0.f;
    if (lane < 32) sdg[lane] = dgv;
    float A[16];
    float e0;
    if (noexp) {
#pragma unroll
      for (int s = 0; s < 16; ++s) A[s] = F.w[s];
      e0 = F.wr0;
    } else {
    const float ebl = lt_exp_off(F.wbl, cl);
    bool lnan = (lane <= V) && !(ebl >= 0.f);
    bool lwide = (lane <= V) && !(ebl >= kEmin);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool live = FULL || (kstep(s, h) < V && i < V);
      const float e = lt_exp_off(F.w[s], cl);
      lnan = lnan || (live && !(e >= 0.f));
      lwide = lwide || (live && !(e >= kEmin));
      A[s] = live ? e : 0.f;
    }
    const float e0r = lt_exp_off(F.wr0, cl);
    e0 = (FULL || i < V) ? e0r : 0.f;
    lnan = lnan || ((FULL || i < V) && !(e0r >= 0.f));
    lwide = lwide || ((FULL || i < V) && !(e0r >= kEmin));
    if (!cfin || __builtin_amdgcn_ballot_w64(lnan)) bad = 2;
    else if (bad == 0 && __builtin_amdgcn_ballot_w64(lwide)) bad = 3;
    }
    const float w00 = F.w00;
    // (diagnostic builds: bit 8192 keeps the chunk's first frame -- timing only)
    if constexpr (kALds) {
      // frame f + 1 from its ring slot: its DMA was issued at the start of
      // step f - 1; only frame f + 2's (issued at the start of this step)
      // may still be in flight
      if (reload && !LT_ABL(a, 8192)) {
        wait_vmcnt(f + 2 < nt ? a.a_ni : 0);
        lds_frame<BF16, PPL, FULL>(aframe(f + 1), fo, F);
      }
    } else if (reload && !LT_ABL(a, 8192)) {
      load_frame<BF16, PPL, FULL>(frame_ptr(f + kApf), frame_bytes(f + kApf), fo, F);
    }

    // state-0 row: r' = p00 * e0 + r Ec (VALU, beside the MFMAs), scaled by
    // a power of two so that its largest entry sits in [1/2, 1)
    {
      float part = h ? 0.f : dgv * rt[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 r4 = *(const float4*)(rt + 8 * g + 4 * h);
        part = __builtin_fmaf(A[4 * g + 0], r4.x, part);
        part = __builtin_fmaf(A[4 * g + 1], r4.y, part);
        part = __builtin_fmaf(A[4 * g + 2], r4.z, part);
        part = __builtin_fmaf(A[4 * g + 3], r4.w, part);
      }
      const float y = half_sum(part);
      const float lam = pi;  // log2 P00 - csum
      const int B0 = __builtin_isfinite(lam) ? max(rho, (int)floorf(lam)) : rho;
      float nr = ldexpf(y, max(rho - B0, -200)) + e0 * __builtin_amdgcn_exp2f(lam - (float)B0);
      nr = (FULL || i < V) ? nr : 0.f;
      int e;
      frexpf(wmax_u(lane < 32 ? nr : 0.f), &e);  // 0 (nothing reached): e = 0
      nr = ldexpf(nr, -e);
      rho = B0 + e;
      if (lane < 32) rt[lane] = nr;
    }
    pi += __builtin_fmaf(w00, kLog2e, -cl);
    csum += cl;

    // core: X <- E^T X on the matrix cores (exact f32 FMA chains)
    // (diagnostic builds: bit 2048 skips the product and the column scales -- timing only)
    if (LT_ABL(a, 2048)) return;
    v16f D = {};
    if constexpr (kBandMix) {
      // the numerator band steps (log space: two transcendentals each, every
      // d of the group computed and kept only while d <= fl + 1) between the
      // MFMAs of the core product: the wave issues them while its own
      // dependent MFMA chain runs
      float2 gv[PPL][kGrp + 1];
      if (bands) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < PPL; ++r)
#pragma unroll
          for (int d = 0; d <= kGrp; ++d) gv[r][d] = sg[lane + 64 * r + d];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        D = __builtin_amdgcn_mfma_f32_32x32x2f32(A[s], X[s], D, 0, 0, 0);
        const int r = s / kGrp, d = kGrp - s % kGrp;
        if (bands && r < PPL) {
          const float nv = lse2_b2(nbd[r][d] + gv[r][d].x, nbd[r][d - 1] + gv[r][d].y);
          nbd[r][d] = d <= flg + 1 ? nv : nbd[r][d];
        }
      }
      if (bands) {
#pragma unroll
        for (int r = 0; r < PPL; ++r) nbd[r][0] += gv[r][0].x;
        if (flg == kGrp - 1 || f == nt - 1) {  // source-major: 32 bytes per position
          const int g0 = jg * (kGrp + 1) * NPG;
#pragma unroll
          for (int r = 0; r < PPL; ++r)
            if (lane + 64 * r < NPG) {
              const int u = lane + 64 * r;
              st_wt4(nbr, g0 + 8 * u, nbd[r][0], nbd[r][1], nbd[r][2], nbd[r][3]);
              st_wt4(nbr, g0 + 8 * u + 4, nbd[r][4], nbd[r][5], nbd[r][6], nbd[r][7]);
            }
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) D = __builtin_amdgcn_mfma_f32_32x32x2f32(A[s], X[s], D, 0, 0, 0);
    }
    // + Dg X: row kstep(r, h) of X times that state's blank self loop
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 d4 = *(const float4*)(sdg + 8 * g + 4 * h);
      D[4 * g + 0] = __builtin_fmaf(d4.x, X[4 * g + 0], D[4 * g + 0]);
      D[4 * g + 1] = __builtin_fmaf(d4.y, X[4 * g + 1], D[4 * g + 1]);
      D[4 * g + 2] = __builtin_fmaf(d4.z, X[4 * g + 2], D[4 * g + 2]);
      D[4 * g + 3] = __builtin_fmaf(d4.w, X[4 * g + 3], D[4 * g + 3]);
    }
    // one power-of-two scale per column (start state j): its largest entry
    // in [1/2, 1) (a column with nothing reached keeps its scale)
    float cm = fmaxf(max3_raw(D[0], D[1], D[2]), max3_raw(D[3], D[4], D[5]));
#pragma unroll
    for (int r = 6; r < 16; r += 2) cm = max3_raw(cm, D[r], D[r + 1]);
    cm = fmaxf(cm, half_other(cm));
    int e;
    frexpf(cm, &e);
    e = cm > 0.f ? e : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) X[r] = ldexpf(D[r], -e);
    ej += e;
  };
  if constexpr (kALds) {
    // LT_CK_ALDS: the chunk's frames through a two-slot LDS ring per wave
    // (LDS-DMA, 16 bytes a lane, a_ni wave instructions a frame) and into F
    // one step ahead: frame f + 2's DMA is issued at the start of step f, so
    // every frame has more than a step to land (the register prefetch gave
    // it two thirds of one), with no registers held for it
    aissue(0);
    if (nt > 1) aissue(1);
    wait_vmcnt(nt > 1 ? a.a_ni : 0);
    lds_frame<BF16, PPL, FULL>(aframe(0), fo, fr);
    for (int f = 0; f < nt; ++f) step(fr, f, f + 1 < nt);
    if (lane < nt) a.cf[(long long)b * a.T + t0 + lane] = cfl_lane;
  } else if constexpr (kApf == 1) {
    // one frame in registers ahead
    load_frame<BF16, PPL, FULL>(frame_ptr(0), frame_bytes(0), fo, fr);
    for (int f = 0; f < nt; ++f) step(fr, f, f + 1 < nt);
  } else {
    // two frames in registers ahead, the buffers alternating (the reloads
    // are unconditional, clamped to the chunk's last frame, so the
    // compiler's vmcnt count across the two buffers stays exact)
    FrameRegs<BF16, PPL> fr2;
    load_frame<BF16, PPL, FULL>(frame_ptr(0), frame_bytes(0), fo, fr);
    load_frame<BF16, PPL, FULL>(frame_ptr(1), frame_bytes(1), fo, fr2);
    for (int f = 0; f < nt; f += 2) {
      step(fr, f, true);
      if (f + 1 < nt) step(fr2, f + 1, true);
    }
  }
  CK_ASTAMP(2);

  const __amdgpu_buffer_rsrc_t rr = wt_rsrc(a.rec + (long long)id * kRec, 4 * kRec);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    st_wt(rr, kstep(r, h) * kRowT + i, X[r]);
  }
  if (lane < 32) {
    st_wt(rr, kRecEj + lane, ej);
    st_wt(rr, kRecRt + lane, rt[lane]);
  }
  bad = __builtin_amdgcn_readfirstlane(bad);
  if (lane == 0) {
    st_wt(rr, kRecRho, rho);
    st_wt(rr, kRecPi, pi);
    st_wt(rr, kRecCs, csum);
    st_wt(rr, kRecFlag, bad);
    st_wt(rr, kRecN, nt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  CK_ASTAMP(3);
  // diagnostic builds: LT_CK_DBG bit 512 withholds utterance 0's chunk 1, so
  // its walks take the hand-off timeout route (tests/test_gpu_diag.py)
  const bool withhold = LT_ABL(a, 512) && b == 0 && k == 1;
  if (lane == 0 && !withhold)
    __hip_atomic_store((gu64*)(a.ready + id), a.ep_tag | (bad ? (unsigned)bad : 1u),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Phase B's side of the hand-off, one wave: chunks [0, hi] (forward walks)
// or [lo, Kl) (backward walks) are known published. ensure() polls 64 flags
// per pass with relaxed agent-scope loads (s_sleep between passes), and one
// agent-scope acquire follows every pass that extends the range, so the
// wave's own plain loads of the newly published records see them (no other
// wave reads through this acquire). A flag of 2 marks a chunk outside the
// fast path's range (bad). A bounded spin: on timeout (a placement that never
// schedules the producer) ok = 0, the range is taken as covered, and the
// utterance goes to the frame-serial kernels.
// A flag poll and the agent-scope acquire as inline asm, each ending in
// its own vmcnt(0): the compiler sees no memory instruction of its own in a
// walk's step loop, so it has no reason to drain the walk's in-flight
// LDS-DMA record loads at every step (it did for the builtin forms).
LT_DEVINL unsigned long long poll_flag(const unsigned long long* p) {
  unsigned long long v;
  asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// a chunk's state in this call (0: not yet published)
LT_DEVINL unsigned flag_state(unsigned long long v, unsigned long long tag) {
  return (v & ~3ull) == tag ? (unsigned)(v & 3) : 0u;
}
// boundaries a phase-2 walk has done in this call
LT_DEVINL int prog_count(unsigned long long v, unsigned long long tag) {
  return (v & ~0xFFFFFFull) == tag ? (int)(v & 0xFFFFFF) : 0;
}
// L1-bypassing loads of another workgroup's data published in this launch
// (LT_CK_NOACQ): 16 bytes, one float
// (a buffer load: the compiler counts it in vmcnt, unlike an asm load)
LT_DEVINL float4 ld_sc1x4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0x10);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
LT_DEVINL float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
LT_DEVINL void acquire_agent() {
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
}
struct ChunkReady {
  const unsigned long long* f;
  unsigned long long tag;
  int lo, hi, Kl, ok, bad, strict;
  LT_DEVINL ChunkReady(const unsigned long long* flags, unsigned long long tg, int kl, int st)
      : f(flags), tag(tg), lo(kl), hi(-1), Kl(kl), ok(1), bad(0), strict(st) {}
  LT_DEVINL void take(unsigned v, int lane, int* c) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(v != 0);
    *c = m == ~0ull ? 64 : __builtin_ctzll(~m);
    const unsigned long long live = *c == 64 ? ~0ull : ((1ull << *c) - 1);
    if (__builtin_amdgcn_ballot_w64(v == 2u || (strict && v == 3u)) & live) bad = 1;
  }
  LT_DEVINL void timeout() {
    ok = 0;
    hi = Kl - 1;
    lo = 0;
  }
  LT_DEVINL void ensure_fwd(int k, int lane) {
    k = min(k, Kl - 1);
    for (unsigned spins = 0; k > hi; ++spins) {
      const int x = hi + 1 + lane;
      const unsigned v = flag_state(poll_flag(f + min(x, Kl - 1)), tag) & (x < Kl ? ~0u : 0u);
      int c;
      take(v, lane, &c);
      if (c) {
        hi += c;
        if (!kNoAcq) acquire_agent();
      } else if (spins > kSpinMax) {
        timeout();
      } else {
        __builtin_amdgcn_s_sleep(4);
      }
    }
  }
  LT_DEVINL void ensure_bwd(int k, int lane) {
    k = max(k, 0);
    for (unsigned spins = 0; k < lo; ++spins) {
      const int x = lo - 1 - lane;
      const unsigned v = flag_state(poll_flag(f + max(x, 0)), tag) & (x >= 0 ? ~0u : 0u);
      int c;
      take(v, lane, &c);
      if (c) {
        lo -= c;
        if (!kNoAcq) acquire_agent();
      } else if (spins > kSpinMax) {
        timeout();
      } else {
        __builtin_amdgcn_s_sleep(4);
      }
    }
  }
};

// ---------------------------------------------------------------------------
// B: chunk boundaries (one workgroup per utterance, 4 waves). Records and
// numerator rows are prefetched into registers (the compiler's own waits).
// ---------------------------------------------------------------------------
struct RecAlpha {  // what lane i (< 32) needs of one record for the alpha step
  float4 x[8];     // X[i][0..31]
  float rt, sc;    // rt[i]; the source-row scale of lane p (rho or ej[p-1], log2)
  float pi, cs;    // log2 P00 - csum; csum (log2, an integer)
};
LT_DEVINL void load_rec_alpha(const float* rc, int lane, int V, RecAlpha& r) {
  // unconditional loads (lanes >= 32 re-read row lane & 31): exact vmcnt
#pragma unroll
  for (int g = 0; g < 8; ++g) r.x[g] = *(const float4*)(rc + (lane & 31) * kRowT + 4 * g);
  r.rt = rc[kRecRt + (lane & 31)];
  const int si = lane == 0 ? kRecRho : kRecEj + min(lane, 32) - 1;
  const int sc = ((const int*)rc)[si];
  r.sc = lane <= V ? (float)sc : 0.f;
  r.pi = rc[kRecPi];
  r.cs = rc[kRecCs];
}
struct RecBeta {   // lane (j, h): the rows of half h of column j
  float x[16];
  float rt, ej;    // rt[lane & 31], ej[j] (log2)
  float rho, pi, cs;
};
LT_DEVINL void load_rec_beta(const float* rc, int lane, RecBeta& r) {
  const int j = lane & 31, h = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) r.x[4 * g + q] = rc[(8 * g + 4 * h + q) * kRowT + j];
  r.rt = rc[kRecRt + j];
  r.ej = (float)((const int*)rc)[kRecEj + j];
  r.rho = (float)((const int*)rc)[kRecRho];
  r.pi = rc[kRecPi];
  r.cs = rc[kRecCs];
}

// The walks in two halves (lt_loss_grad): phase 1 runs beside phase A as far
// as the middle chunk boundary Kh = Kl / 2 -- alpha over chunks [0, Kh),
// beta over [Kh, Kl), the chunks phase A publishes first (outside-in) -- and
// phase 2 finishes them in phase C's launch, from the boundary rows and
// offsets phase 1 left, while C's workgroups take the chunks middle-out as
// their boundaries land. So the launch of A no longer waits for the second
// half of every walk (a walk is K steps of ~0.6 us, as long as A itself), and
// that half overlaps C. Phase 0: the whole walk in one go (lt_chunk_forward).
// Phase 2 publishes its boundary rows write-through (relaxed agent-scope
// stores) and, every kProgStep boundaries and at its end, after its own
// s_waitcnt vmcnt(0), the count of boundaries done to a progress word
// (CkArgs::prog) that phase C's workgroups poll before their boundary loads.
constexpr int kProgStep = 4;
enum { kWalkFull = 0, kWalkFirst = 1, kWalkRest = 2 };
LT_DEVINL void bd_store(float* p, float v, bool wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
LT_DEVINL void prog_publish(const CkArgs& a, int b, int w, int n, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    __hip_atomic_store((gu64*)(a.prog + 4LL * b + w), a.pg_tag | (unsigned)n, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// The walks' LDS, carved from the launch's dynamic LDS (no static LDS, so
// phase C's launch can hold them at its own four workgroups per CU): the den
// record rings, the numerator alpha's scatter table and beta's padded copy,
// the den step operand rows, three scalars.
constexpr int kWalkNvA = (128 + kGrp + 1) * (kGrp + 2);
constexpr int kWalkNvB = 128 + kGrp + 1;
constexpr int kWalkLdsBytes = kWalkLds + 4 * (kWalkNvA + kWalkNvB) + 4 * 128 + 16;
struct WalkLds {
  unsigned char* ring;
  float *nva, *nvb, *bc, *lz, *num;
  int* bad;
};
LT_DEVINL WalkLds walk_lds(unsigned char* base) {
  WalkLds w;
  w.ring = base;
  w.nva = (float*)(base + kWalkLds);
  w.nvb = w.nva + kWalkNvA;
  w.bc = w.nvb + kWalkNvB;
  w.lz = w.bc + 128;
  w.num = w.lz + 1;
  w.bad = (int*)(w.num + 1);
  return w;
}

// Phase B's numerator over the groups of kGrp frames (phase A's bands),
// base-2 log space. FWD, alpha (lattices.py:340-377 composed per group):
// al'[u] = (+)_d al[u - d] + N[u - d][d], scattered by destination through
// an LDS table; !FWD, beta (the reverse of alignments.py:320-329):
// be'[s] = (+)_d N[s][d] + be[s + d] from an LDS copy padded with -inf.
// Boundary values at every chunk start -> nabd / nbbd (log2, each vector
// relative to the walk's integer offset at that boundary: phase C normalises
// every frame by its own total, so only differences within a vector matter).
// D groups of bands in registers ahead.
template <int PPL, bool FWD, int D>
LT_DEVINL void num_walk(const CkArgs& a, int b, int lane, int nf, int Kl, int nl, float* lds,
                        float* s_num, ChunkReady& rd, int ph) {
  const int NPG = a.NPG;
  constexpr int NB = kGrp + 1;
  constexpr int TS = NB + 1;  // alpha's scatter table row stride (odd: no bank conflicts)
  const int NGc = a.NGc;
  const int ntl = nf - (Kl - 1) * a.L;  // live frames of the last chunk
  const int Q = Kl > 0 ? (Kl - 1) * NGc + (ntl + kGrp - 1) / kGrp : 0;
  const int Kh = Kl / 2, qh = Kh * NGc;  // the middle chunk boundary's group
  // this phase's groups [q0, q1): alpha walks them up, beta down
  const int q0 = ph == kWalkRest ? (FWD ? qh : 0) : (FWD ? 0 : (ph == kWalkFirst ? qh : 0));
  const int q1 = ph == kWalkRest ? (FWD ? Q : qh) : (FWD ? (ph == kWalkFirst ? qh : Q) : Q);
  const bool wt = ph == kWalkRest;
  const float* nb0 = a.nb + (long long)b * a.K * a.nbs;
  // alpha: tab[u][d] = al[u - d] + N[u - d][d] (rows u < d stay -inf);
  // beta: sv[s] = be[s] with sv[64 PPL, +NB) = -inf
  float* tab = lds;
  float* sv = lds;
  if constexpr (FWD) {
    for (int e = lane; e < (64 * PPL + NB) * TS; e += 64) tab[e] = -kInf;
  } else if (lane < NB) {
    sv[64 * PPL + lane] = -kInf;
  }
  float v[PPL];
  float off = 0.f;  // the vector's integer offset (log2): the walk holds v - off
  float* dst = (FWD ? a.nabd : a.nbbd) + (long long)b * (a.K + 1) * NPG;
  if (ph == kWalkRest) {  // phase 1's vector at the middle boundary, and alpha's offset
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int u = lane + 64 * r;
      const float x = dst[(long long)Kh * NPG + min(u, NPG - 1)];
      v[r] = u < NPG ? x : -kInf;
    }
    if (FWD) off = a.mid[2LL * b + 1];
  } else {
#pragma unroll
    for (int r = 0; r < PPL; ++r) v[r] = (lane + 64 * r == (FWD ? 0 : nl)) ? 0.f : -kInf;
    if (!FWD) {
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        if (lane + 64 * r < NPG) dst[(long long)Kl * NPG + lane + 64 * r] = v[r];
    }
  }
  int pub = 0;  // phase 2: boundaries published (progress word)
  auto publish = [&](int done, bool last) {
    if (wt && (last || done - pub >= kProgStep)) {
      prog_publish(a, b, FWD ? 2 : 3, done, lane);
      pub = done;
    }
  };
  // band rows N[s][0 .. kGrp] of group q for the lane's source positions
  float4 gq[D][PPL][2];
  auto bload = [&](int q, float4 (*g)[2]) {
    const int qc = min(max(q, 0), max(Q - 1, 0));
    if constexpr (FWD) rd.ensure_fwd(qc / NGc, lane);
    else rd.ensure_bwd(qc / NGc, lane);
    const int kc = qc / NGc;
    const float4* row = (const float4*)(nb0 + (long long)kc * a.nbs + (qc - kc * NGc) * NB * NPG);
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int uc = min(lane + 64 * r, NPG - 1);
      if constexpr (kNoAcq) {
        const __amdgpu_buffer_rsrc_t rr =
            __builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, 32 * NPG, 0x00020000);
        g[r][0] = ld_sc1x4(rr, 32 * uc);
        g[r][1] = ld_sc1x4(rr, 32 * uc + 16);
      } else {
        g[r][0] = row[2 * uc];
        g[r][1] = row[2 * uc + 1];
      }
    }
  };
  auto step = [&](float4 (*g)[2], int q, int qn) {
    if (FWD && q % NGc == 0) {  // a chunk starts here
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        if (lane + 64 * r < NPG) bd_store(dst + (long long)(q / NGc) * NPG + lane + 64 * r, v[r], wt);
      publish(q / NGc - Kh, false);
    }
    float n[PPL][NB];
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      n[r][0] = g[r][0].x; n[r][1] = g[r][0].y; n[r][2] = g[r][0].z; n[r][3] = g[r][0].w;
      n[r][4] = g[r][1].x; n[r][5] = g[r][1].y; n[r][6] = g[r][1].z; n[r][7] = g[r][1].w;
    }
    if constexpr (FWD) {
#pragma unroll
      for (int r = 0; r < PPL; ++r)
#pragma unroll
        for (int d = 0; d < NB; ++d) tab[(lane + 64 * r + d) * TS + d] = v[r] + n[r][d];
    } else {
#pragma unroll
      for (int r = 0; r < PPL; ++r) sv[lane + 64 * r] = v[r];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    float x[PPL][NB];
#pragma unroll
    for (int r = 0; r < PPL; ++r)
#pragma unroll
      for (int d = 0; d < NB; ++d)
        x[r][d] = FWD ? tab[(lane + 64 * r) * TS + d] : n[r][d] + sv[lane + 64 * r + d];
    bload(qn, g);
    float vm = -kInf;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      float m = x[r][0];
#pragma unroll
      for (int d = 1; d < NB; ++d) m = fmaxf(m, x[r][d]);
      const float ms = m == -kInf ? 0.f : m;
      float sum = 0.f;
#pragma unroll
      for (int d = 0; d < NB; ++d) sum += __builtin_amdgcn_exp2f(x[r][d] - ms);
      v[r] = lane + 64 * r < NPG ? ms + __builtin_amdgcn_logf(sum) : -kInf;
      vm = fmaxf(vm, v[r]);
    }
    // the vector relative to an integer offset near its max: the values a
    // marginal is made of stay small, so their rounding stays 2^-24 of
    // small numbers however long the utterance (the offset is exact)
    {
      const float mv = wmax_u(vm);
      const float fl = __builtin_isfinite(mv) ? floorf(mv) : 0.f;
#pragma unroll
      for (int r = 0; r < PPL; ++r) v[r] -= fl;
      off += fl;
    }
    if (!FWD && q % NGc == 0) {  // beta at the chunk's first frame
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        if (lane + 64 * r < NPG) bd_store(dst + (long long)(q / NGc) * NPG + lane + 64 * r, v[r], wt);
      publish(Kh - q / NGc, false);
    }
    __builtin_amdgcn_wave_barrier();
  };
  const int cnt = q1 - q0;
  auto qof = [&](int n) { return FWD ? q0 + n : q1 - 1 - n; };
#pragma unroll
  for (int d = 0; d < D; ++d) bload(qof(d), gq[d]);
  const int nmain = cnt - cnt % D;
  for (int n0 = 0; n0 < nmain; n0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) step(gq[d], qof(n0 + d), qof(n0 + d + D));
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (nmain + d < cnt) step(gq[d], qof(nmain + d), qof(nmain + d));
  if (ph == kWalkFirst) {
    if (FWD) {  // alpha at the middle boundary (phase 2's start) and its offset
#pragma unroll
      for (int r = 0; r < PPL; ++r)
        if (lane + 64 * r < NPG) dst[(long long)Kh * NPG + lane + 64 * r] = v[r];
      if (lane == 0) a.mid[2LL * b + 1] = off;
    }
    return;
  }
  publish(FWD ? (Kl - 1) - Kh : Kh, true);
  if constexpr (FWD) {
    float nv = -kInf;
#pragma unroll
    for (int r = 0; r < PPL; ++r)
      if (lane + 64 * r == nl) nv = v[r];
    nv = wmax_u(nv);
    if (lane == 0)
      *s_num = (nl >= 0 && nl <= a.U) ? (float)(((double)off + (double)nv) * 0.6931471805599453)
                                       : -kInf;
  }
}

// Utterance b's walks, one per wave, each following phase A's progress
// through the ready flags (ChunkReady) when A runs in the same launch; `ph`
// as above; `dyn` the launch's dynamic LDS (walk_lds).
template <int PPL, int D>
LT_DEVINL void combine_role(const CkArgs& a, int b, int wave, unsigned char* dyn, int ph) {
  const WalkLds wl = walk_lds(dyn);
  const int lane = threadIdx.x & 63;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int Kl = (nf + a.L - 1) / a.L;  // live chunks
  const int Kh = Kl / 2;                // the middle boundary (phases 1 and 2)
  const int V = a.V, C = a.C, CP = a.CP;
  const int nl = a.nlab[b];
  if (ph == kWalkRest && a.uflag[b]) return;  // phase 1 sent it to the frame-serial kernels
  if (threadIdx.x == 0) *wl.bad = 0;
  __syncthreads();
  CK_WSTAMP(2 * wave);
  ChunkReady rd(a.ready + (long long)b * a.K, a.ep_tag, Kl, a.strict);
  if (ph == kWalkRest) {  // every chunk published (phase A's launch is over)
    rd.lo = 0;
    rd.hi = Kl - 1;
  }
  const bool wt = ph == kWalkRest;

  // den walks: the records stream through a ring of kWalkSlots LDS slots
  // per wave by LDS-DMA (1 KiB contiguous per instruction), issued
  // kWalkSlots steps ahead; each step reads its record from LDS. (Records
  // gathered straight into registers -- a row per lane for alpha, a column
  // for beta -- stalled each step about as long as the rest of the step.)
  const unsigned ring_a = lds_base_addr(wl.ring) + (unsigned)(wave * kWalkSlots * kWalkSlot);
  const unsigned char* ring = wl.ring + wave * kWalkSlots * kWalkSlot;
  auto issue_rec = [&](int k, int n) {  // step n's record k (clamped to [0, Kl)) -> slot n mod kWalkSlots
    const int kc = min(max(k, 0), Kl - 1);
    dma_issue((const unsigned char*)a.rec, ((long long)b * a.K + kc) * (kRec * 4), kRec * 4,
              ring_a + (unsigned)((n % kWalkSlots) * kWalkSlot), kRecNi, lane, 0, 1, kNoAcq);
  };
  // step n's record has landed: the ring's issues and each step's one
  // boundary-row store, in issue order (vmcnt counts both, in order; the
  // flag polls and progress words drain it themselves)
  auto wait_rec = [&](int n) {
    wait_vmcnt(n < kWalkSlots ? kRecNi * (kWalkSlots - 1) + n : (kRecNi + 1) * kWalkSlots - kRecNi);
  };
  auto slot = [&](int n) { return (const float*)(ring + (n % kWalkSlots) * kWalkSlot); };

  if (wave == 0 && !a.local && !LT_ABL(a, 1)) {
    // ---- den alpha across chunks (lattices.py:379-496 in chunk steps), log2
    // units: lane p holds alpha[p] - O with O an integer offset near the
    // vector's max. The records' scales (ej, rho) and offsets (csum) are
    // integers, so O is exact and every stored value stays small: its
    // rounding is 2^-24 of a small number however long the utterance.
    float* bc = wl.bc;  // bc[j] = a_{j+1} (core source j), bc[32] = a_0
    float* dst = a.abd + (long long)b * (a.K + 1) * CP;
    const int k0 = ph == kWalkRest ? Kh : 0, k1 = ph == kWalkFirst ? Kh : Kl;
    float al, O;
    if (ph == kWalkRest) {  // phase 1's vector at the middle boundary and its offset
      const float x = dst[(long long)Kh * CP + min(lane, C - 1)];
      al = lane < C ? x : -kInf;
      O = a.mid[2LL * b];
    } else {
      al = lane == 0 ? 0.f : -kInf;  // lane p: alpha[p] - O
      O = 0.f;
      if (lane < C) dst[lane] = al;
    }
    int pub = 0;
    if (k1 > k0) {
      rd.ensure_fwd(k0 + kWalkSlots - 1, lane);
      for (int n = 0; n < kWalkSlots; ++n) issue_rec(k0 + n, n);
    }
    for (int k = k0; k < k1; ++k) {
      const int n = k - k0;
      wait_rec(n);
      RecAlpha R;
      load_rec_alpha(slot(n), lane, V, R);
      const float x = lane < C ? al + R.sc : -kInf;
      const float M = safe_max(wmax_u(x));
      const float av = lane < C ? __builtin_amdgcn_exp2f(x - M) : 0.f;
      if (lane >= 1 && lane <= 32) bc[lane - 1] = av;
      if (lane == 0) bc[32] = av;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int g = 0; g < 8; g += 2) {
        const float4 a0 = *(const float4*)(bc + 4 * g);
        const float4 a1 = *(const float4*)(bc + 4 * g + 4);
        s0 = __builtin_fmaf(R.x[g].x, a0.x, s0);
        s1 = __builtin_fmaf(R.x[g + 1].x, a1.x, s1);
        s0 = __builtin_fmaf(R.x[g].y, a0.y, s0);
        s1 = __builtin_fmaf(R.x[g + 1].y, a1.y, s1);
        s0 = __builtin_fmaf(R.x[g].z, a0.z, s0);
        s1 = __builtin_fmaf(R.x[g + 1].z, a1.z, s1);
        s0 = __builtin_fmaf(R.x[g].w, a0.w, s0);
        s1 = __builtin_fmaf(R.x[g + 1].w, a1.w, s1);
      }
      s0 = __builtin_fmaf(R.rt, bc[32], s0);
      const float cs = R.cs, pi = R.pi;
      // the slot's last read has returned: its next record goes in
      __builtin_amdgcn_s_waitcnt(0xc07f);
      rd.ensure_fwd(k + kWalkSlots, lane);
      issue_rec(k + kWalkSlots, n + kWalkSlots);
      const float fl = floorf(M);
      const float nq = (M - fl) + __builtin_amdgcn_logf(s0 + s1);  // lane i < 32: alpha'[i+1] - O'
      const float n0 = first_lane(al) + pi - fl;
      O += cs + fl;
      const float sh = from_prev(nq, -kInf);
      al = lane == 0 ? n0 : (lane < C ? sh : -kInf);
      if (lane < C) bd_store(dst + (long long)(k + 1) * CP + lane, al, wt);
      if (wt && k + 1 - Kh - pub >= kProgStep && k + 1 < k1) {
        prog_publish(a, b, 0, k + 1 - Kh, lane);
        pub = k + 1 - Kh;
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (ph == kWalkFirst) {
      if (lane == 0) a.mid[2LL * b] = O;
    } else {
      if (wt) prog_publish(a, b, 0, k1 - Kh, lane);
      // log_z = (+)_q alpha_T[q] (lattices.py:496), back to natural log once
      const float x = lane < C ? al : -kInf;
      const float M = safe_max(wmax_u(x));
      const float s = wsum_u(lane < C ? __builtin_amdgcn_exp2f(x - M) : 0.f);
      if (lane == 0)
        *wl.lz = (float)(((double)O + (double)(M + __builtin_amdgcn_logf(s))) * 0.6931471805599453);
    }
  } else if (wave == 1 && !a.local && !LT_ABL(a, 1)) {
    // ---- den beta across chunks: beta_T = one for every state
    // (lattices.py:788-790); log2, relative to an integer offset as alpha
    // (the offset itself is not needed: nothing reads beta's absolute value)
    float* bc = wl.bc + 64;
    const int h = lane >> 5;
    float* dst = a.bbd + (long long)b * (a.K + 1) * CP;
    const int k0 = ph == kWalkFirst ? Kh : 0, k1 = ph == kWalkRest ? Kh : Kl;  // chunks, walked down
    float be;  // lane p: beta[p] - O
    if (ph == kWalkRest) {
      const float x = dst[(long long)Kh * CP + min(lane, C - 1)];
      be = lane < C ? x : -kInf;
    } else {
      be = lane < C ? 0.f : -kInf;
      if (lane < C) dst[(long long)Kl * CP + lane] = be;
    }
    int pub = 0;
    if (k1 > k0) {
      rd.ensure_bwd(k1 - kWalkSlots, lane);
      for (int n = 0; n < kWalkSlots; ++n) issue_rec(k1 - 1 - n, n);
    }
    for (int n = 0; n < k1 - k0; ++n) {
      const int k = k1 - 1 - n;
      wait_rec(n);
      RecBeta R;
      load_rec_beta(slot(n), lane, R);
      const float xc = (lane >= 1 && lane < C) ? be : -kInf;  // core beta
      const float Mc = safe_max(wmax_u(xc));
      if (lane >= 1 && lane <= 32) bc[lane - 1] = lane < C ? __builtin_amdgcn_exp2f(xc - Mc) : 0.f;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      // lane (j, h): sum over end states i of half h of X[i][j] b_i
      float p0 = 0.f, p1 = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b4 = *(const float4*)(bc + 8 * g + 4 * h);
        p0 = __builtin_fmaf(R.x[4 * g + 0], b4.x, p0);
        p1 = __builtin_fmaf(R.x[4 * g + 1], b4.y, p1);
        p0 = __builtin_fmaf(R.x[4 * g + 2], b4.z, p0);
        p1 = __builtin_fmaf(R.x[4 * g + 3], b4.w, p1);
      }
      const float rp = lane < 32 ? R.rt * bc[lane & 31] : 0.f;
      const float ej = R.ej, rho = R.rho, pi = R.pi;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      rd.ensure_bwd(k - kWalkSlots, lane);
      issue_rec(k - kWalkSlots, n + kWalkSlots);
      const float fl = floorf(Mc);
      const float tot = half_sum(p0 + p1);
      const float nj = (Mc - fl) + ej + __builtin_amdgcn_logf(tot);  // lane j: beta'[j+1] - O'
      // state 0: the rt row and its own self loop
      const float rsum = wsum_u(rp);
      const float rterm = (Mc - fl) + rho + __builtin_amdgcn_logf(rsum);
      const float nb0 = lse2_b2(first_lane(be) + pi - fl, rterm);
      const float sh = from_prev(nj, -kInf);
      be = lane == 0 ? nb0 : (lane < C ? sh : -kInf);
      if (lane < C) bd_store(dst + (long long)k * CP + lane, be, wt);
      if (wt && Kh - k - pub >= kProgStep && k > k0) {
        prog_publish(a, b, 1, Kh - k, lane);
        pub = Kh - k;
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (wt) prog_publish(a, b, 1, Kh - k0, lane);
  } else if (wave == 2 && !LT_ABL(a, 2) && !LT_ABL(a, 128)) {
    num_walk<PPL, true, D>(a, b, lane, nf, Kl, nl, wl.nva, wl.num, rd, ph);
  } else if (wave == 3 && !LT_ABL(a, 2)) {
    num_walk<PPL, false, D>(a, b, lane, nf, Kl, nl, wl.nvb, nullptr, rd, ph);
  }
  // any chunk out of the fast path's range (a weight not finite, or a frame
  // spanning more than kRange; every walk has seen every chunk's flag) or a
  // hand-off timeout: the frame-serial kernels take the utterance
  if (lane == 0 && (rd.bad || !rd.ok)) *wl.bad = 1;
  CK_WSTAMP(2 * wave + 1);
  __syncthreads();
  if (ph == kWalkFirst) {  // phase 2 (phase C's launch) finishes the walks
    if (threadIdx.x == 0) a.uflag[b] = *wl.bad ? 1 : 0;
    return;
  }
  if (*wl.bad) {
    if (threadIdx.x == 0) a.uflag[b] = 1;
    return;
  }
  if (threadIdx.x == 0) {
    const float lz = a.local ? 0.f : *wl.lz;
    const float nm = *wl.num;
    // phase 2: phase C's workgroups took the chunks before log_z and num
    // existed; a denominator with no finite path, a NaN or an unreachable
    // string (the reference's semantics, dW = 0) goes to the frame-serial
    // kernels after the launch, which rewrite the utterance
    if (ph == kWalkRest && ((!a.local && !__builtin_isfinite(lz)) || !__builtin_isfinite(nm)))
      a.uflag[b] = 1;
    else if (ph == kWalkFull)
      a.uflag[b] = 0;
    a.log_z[b] = lz;
    a.num[b] = nm;
    if (a.lz_out) a.lz_out[b] = lz;
    if (a.num_out) a.num_out[b] = nm;
    a.loss[b] = a.local ? -nm : lz - nm;  // lattices.py:178-183
  }
}

// numerator band groups in registers ahead: the walk launches' (2 PPL loads
// each: vmcnt <= 63; PPL = 2 keeps the walk inside the fused launch's
// register budget) and phase C's (its four workgroups per CU)
template <int PPL>
constexpr int kWalkD = PPL == 1 ? 8 : (kAbWaves > 3 ? 4 : 5);
template <int PPL>
constexpr int kWalkDc = PPL == 1 ? 4 : 3;

// A and B in one launch: the nc = B workgroups at block indices [wpos, wpos
// + nc) walk one utterance each (nc = 0: ck_combine_kernel walks after the
// launch); every other wave computes one chunk, ordered outside-in -- level
// m holds chunks m and Kl-1-m of every utterance -- so the forward walks
// (chunk 0 up) and the backward walks (Kl-1 down) both find their next
// chunks among the first published. The walks start part-way through the
// chunks (wpos, host-chosen), so that they hold their wave slots only for
// the stretch they can follow A's front. Dispatch order is not assumed for
// correctness: a walk that never sees its chunk times out to the
// frame-serial kernels.
template <bool BF16, int PPL, bool FULL>
__global__ __launch_bounds__(256, kAbWaves) void ck_ab_kernel(const CkArgs a) {
  const int nc = a.nc;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int x = blockIdx.x;
  if (x >= a.wpos && x < a.wpos + nc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char ck_dyn[];
    if (LT_CK_WPRIO) __builtin_amdgcn_s_setprio(LT_CK_WPRIO);  // the walks' chains first
    combine_role<PPL, kWalkD<PPL>>(a, x - a.wpos, wave, ck_dyn, a.half ? kWalkFirst : kWalkFull);
    return;
  }
  if (x >= a.wpos) x -= nc;
  const long long j = (long long)x * 4 + wave;
  const int m = (int)(j / (2 * a.B));
  const int r = (int)(j - (long long)m * 2 * a.B);
  const int b = r < a.B ? r : r - a.B;
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int Kl = (nf + a.L - 1) / a.L;
  const int k = r < a.B ? m : Kl - 1 - m;
  if (r < a.B ? m > Kl - 1 - m : Kl - 1 - m <= m) return;  // past the middle (or no chunk)
  transfer_role<BF16, PPL, FULL>(a, b, k, wave);
}

template <int PPL>
__global__ __launch_bounds__(256) void ck_combine_kernel(const CkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ck_dyn[];
  combine_role<PPL, kWalkD<PPL>>(a, blockIdx.x, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                                 ck_dyn, a.half ? kWalkFirst : kWalkFull);
}

// Phase C's gather tables: per position, in LDS (labels staged by the whole
// workgroup first).
LT_DEVINL void gather_tables(const CkArgs& a, int b, int* lab, int* boff, int* loff, int tid,
                             int nthr) {
  for (int j = tid; j < a.U; j += nthr) lab[j] = a.labels[(long long)b * a.U + j];
  __syncthreads();
  for (int u = tid; u < a.NPG; u += nthr) {
    int bo, lo;
    string_offsets(a, lab, u, &bo, &lo);
    boff[u] = bo < 0 ? 0 : bo;
    loff[u] = lo;
  }
}

// ---------------------------------------------------------------------------
// C: local recursions + marginals -> dW (one workgroup per chunk)
// ---------------------------------------------------------------------------
template <bool BF16>
LT_DEVINL void store_dw(void* dW, long long e, float v) {
  if constexpr (BF16) ((unsigned short*)dW)[e] = f2bf(v);
  else ((float*)dW)[e] = v;
}

// per-frame scalars of phase C (log2): alpha's and beta's scales, the start
// state's alpha and beta, W[0][0]
constexpr int kFs = 8, kFsMa = 0, kFsA0 = 1, kFsMb = 2, kFsB0 = 3, kFsW00 = 4;
// phase C's per-frame progress bits: den alpha / beta have passed the frame
// (rows written, E_f read), numerator alpha / beta rows written
constexpr int kFlA = 1, kFlB = 2, kFlNA = 4, kFlNB = 8, kFlAll = 15;

template <bool BF16, int PPL, bool FULL>
__global__ __launch_bounds__(64 * kMargWaves, kMargWaves / 2) void ck_marg_kernel(const CkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.cont && (int)blockIdx.x < a.B) {  // phase 2 of utterance blockIdx.x's walks
    CK_STAMP(0);
    if (LT_CK_WPRIO) __builtin_amdgcn_s_setprio(LT_CK_WPRIO);
    combine_role<PPL, kWalkDc<PPL>>(a, blockIdx.x, wave, lds, kWalkRest);
    CK_STAMP(4);
    return;
  }
  // level j of utterance b: chunks middle-out (Kh, Kh - 1, Kh + 1, Kh - 2,
  // ...: the order phase 2's boundaries land in), then the padding chunks
  const int c = a.cont ? (int)blockIdx.x - a.B : (int)blockIdx.x;
  const int j = c / a.B, b = c - j * a.B;
  if (a.uflag[b]) return;  // the frame-serial kernels own this utterance
  int nf = a.nfr[b];
  nf = nf < 0 ? 0 : (nf > a.T ? a.T : nf);
  const int Kl = (nf + a.L - 1) / a.L, Kh = Kl / 2;
  const int k = j < 2 * Kh ? ((j & 1) ? Kh - 1 - (j >> 1) : Kh + (j >> 1)) : j;
  const int t0 = k * a.L;
  const int tend = min(t0 + a.L, a.T);
  const int t1 = max(t0, min(t0 + a.L, nf));
  // FULL: V = 32, every stride a compile-time constant
  const int V = FULL ? 32 : a.V, C = V + 1, R = V + 1, FR = C * R, CP = FULL ? 36 : a.CP;
  const int NPG = a.NPG, NP = a.NP;
  const int FRP = (FR + 3) & ~3;
  float g = a.grad ? a.grad[b] : 1.f;
  if (!a.cont) {  // (phase 2 checks log_z and num itself, once they exist)
    const float lz = a.log_z[b], nm = a.num[b];
    // a NaN, or a denominator with no finite path (the relaxed path admits
    // masked arcs): the frame-serial kernels own the utterance (the
    // reference's semantics for such lattices)
    if ((!a.local && !__builtin_isfinite(lz)) || __builtin_isnan(nm)) {
      if (tid == 0) a.uflag[b] = 1;
      return;
    }
    if (!__builtin_isfinite(nm)) g = 0.f;  // unreachable string: loss +inf, dW = 0
  }
  const long long e0 = ((long long)b * a.T + t0) * FR;
  if (t1 <= t0 || g == 0.f) {  // padding chunk / unreachable string: dW = 0
    const long long n = (long long)(tend - t0) * FR;
    for (long long e = tid; e < n; e += blockDim.x) store_dw<BF16>(a.dW, e0 + e, 0.f);
    return;
  }
  const int nt = t1 - t0;
  CK_STAMP(0);
  // the recursion roles rotate over the waves by workgroup (LT_CK_ROT), so
  // the two den chains of the workgroups sharing a CU need not sit on the
  // same two SIMDs
  const int role = LT_CK_ROT == 1 ? (wave + (int)(blockIdx.x >> 3)) & 3
                 : LT_CK_ROT == 2 ? (wave + (int)blockIdx.x) & 3 : wave;
  // split staging (LT_CK_SPLIT): each den chain stages the half of W it
  // reads first (alpha frames [0, hs), beta [hs, nt)) and starts on it while
  // the other waves gather the tables; the chains take the numerator's arc
  // weights out of their own frames before forming E there, and the
  // numerator waves follow the chains' frame bits. One barrier (tables,
  // offsets, flags), not two, and no wave waits for the whole chunk's DMA.
  const bool split = LT_CK_SPLIT && !a.local && !LT_ABL(a, 4 | 8);
  const int hs = (nt + 1) / 2;
  // stage the chunk's live frames
  const long long off = e0 * (BF16 ? 2 : 4);
  if (!split) {
    dma_issue(a.W, off, (long long)nt * a.FB, lds_base_addr(lds), a.c_ni, lane, wave, kMargWaves);
  } else if (role < 2) {
    const int n1 = (int)(((off & 15) + (long long)hs * a.FB + 1023) >> 10);
    dma_range(a.W, off, (long long)nt * a.FB, lds_base_addr(lds), role == 0 ? 0 : max(n1 - 1, 0),
              role == 0 ? n1 : a.c_ni, lane);
  }
  unsigned char* wch = lds + (off & 15);
  float* xa = (float*)(lds + a.c_off_ad);  // [L][CP] alpha_f, linear, max 1 (scale fs Ma)
  float* xb = (float*)(lds + a.c_off_bd);  // [L][CP] beta_{f+1} of the core, linear, max 1
  float* an = (float*)(lds + a.c_off_an);  // [L][NPG] numerator alpha_f (log2)
  float* bn = (float*)(lds + a.c_off_bn);  // [L][NPG] numerator beta_{f+1} (log2)
  float2* nw = (float2*)(lds + a.c_off_nw);  // [L][NPG] (blank of u, arc into u), log2
  float* fs = (float*)(lds + a.c_off_fs);    // [L][kFs]
  int* boff = (int*)(lds + a.c_off_tab);
  int* loff = boff + NPG;
  int* labs = loff + NPG;
  float* buf = (float*)(lds + a.c_off_buf) + 64 * wave;
  float* cfl = (float*)(lds + a.c_off_cf);
  int* fl = (int*)(lds + a.c_off_fl);
  int* ford = fl + a.L;
  int* njob = ford + a.L;
  int* cert_fail = njob + 1;  // a frame outside the certificate (any wave)
  // per-frame progress bits for the marginal pass (kFl*), the frames in
  // the order their inputs complete (middle first), a job counter
  auto init_flags = [&](int t) {
    if (t < nt) {
      fl[t] = 0;
      const int mid = (nt - 1) / 2;  // job j -> frames mid, mid+1, mid-1, mid+2, ...
      const int k = (t + 1) / 2;
      ford[t] = (t & 1) ? mid + k : mid - k;
    }
    if (t == 0) {
      *njob = 0;
      *cert_fail = 0;
    }
  };
  // the split staging's tables, offsets and flags: the numerator waves
  // (t2 = their thread in [0, 128)), the labels read by each of the two
  if (split && role >= 2) {
    const int t2 = (role - 2) * 64 + lane;
    if (t2 < nt) cfl[t2] = a.cf[(long long)b * a.T + t0 + t2];
    for (int j = lane; j < a.U; j += 64) labs[j] = a.labels[(long long)b * a.U + j];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    for (int u = t2; u < NPG; u += 128) {
      int bo, lo;
      string_offsets(a, labs, u, &bo, &lo);
      boff[u] = bo < 0 ? 0 : bo;
      loff[u] = lo;
    }
    init_flags(t2);
  }
  if (!split && tid < nt) cfl[tid] = a.cf[(long long)b * a.T + t0 + tid];
  // phase 2's boundaries this chunk needs (alpha at k, beta at k + 1): one
  // lane polls the walks' progress words, then the agent-scope acquire
  // before any wave's loads of them (after the barriers below); split: a
  // numerator wave's lane, whose loads do not queue behind the W DMA
  if (a.cont && (split ? (role == 2 && lane == 0) : tid == 0)) {
    const int need_a = k - Kh, need_b = Kh - (k + 1);
    const unsigned long long* pg = a.prog + 4LL * b;
    int ok = 1;
    for (unsigned spins = 0;; ++spins) {
      bool done = true;
      if (need_a > 0)
        done = (a.local || prog_count(poll_flag(pg + 0), a.pg_tag) >= need_a) &&
               prog_count(poll_flag(pg + 2), a.pg_tag) >= need_a;
      if (done && need_b > 0)
        done = (a.local || prog_count(poll_flag(pg + 1), a.pg_tag) >= need_b) &&
               prog_count(poll_flag(pg + 3), a.pg_tag) >= need_b;
      if (done) break;
      if (spins > kSpinMax) {  // phase 2 never ran (a placement that starves it)
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!kNoAcq) acquire_agent();
    CK_STAMP(6);
    fl[2 * a.L + 2] = ok;
  }
  if (!split) {
    gather_tables(a, b, labs, boff, loff, tid, blockDim.x);
    wait_vmcnt(0);
    __syncthreads();
  } else {  // LDS only: the den chains' W DMA stays in flight
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if (a.cont && !fl[2 * a.L + 2]) {
    if (tid == 0) a.uflag[b] = 1;
    return;
  }
  CK_STAMP(1);
  // E_f = exp(W_f - c_f) (c_f = phase A's integer offset, log2 units, so
  // E <= 1) is formed by the den recursions as they first read the frame,
  // from the staged W, and stored to E_f's home (in place over the f32
  // image, a float region of its own for bf16): alpha owns frames [0, hs),
  // beta [hs, nt), the ones each reaches first, and each reads the other's
  // frames as E once that frame's bit is set. No pass and barrier of its
  // own, one exponential per element. The marginals read E_f and leave the
  // frame's dW in its place.
  auto wrow = [&](int f) -> const unsigned char* { return wch + f * a.FB; };
  auto eptr = [&](int f) -> float* {
    return BF16 ? (float*)(lds + a.c_off_e) + f * FRP : (float*)(wch + f * a.FB);
  };
  auto ew = [](float w, float cl) -> float {
    return __builtin_amdgcn_exp2f(__builtin_fmaf(w, kLog2e, -cl));
  };
  // the numerator's arc weights leave W first (exact, log2); every read of
  // this pass issues before the barrier, every E store after it
  if (!split) {
    float2 g2[4];
    const int nnw = nt * NPG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int x = min(tid + 64 * kMargWaves * i, nnw - 1);
      const int f = x / NPG, u = x - f * NPG;
      const unsigned char* fr = wch + f * a.FB;
      const int lo = loff[u];
      const float wb = ldsw<BF16>(fr, boff[u]), wl = ldsw<BF16>(fr, max(lo, 0));
      g2[i] = make_float2(u < NP ? wb * kLog2e : -kInf, (u >= 1 && u < NP) ? wl * kLog2e : -kInf);
    }
    for (int x = tid + 4 * 64 * kMargWaves; x < nnw; x += 64 * kMargWaves) {  // long strings
      const int f = x / NPG, u = x - f * NPG;
      const unsigned char* fr = wch + f * a.FB;
      const int lo = loff[u];
      const float wb = ldsw<BF16>(fr, boff[u]), wl = ldsw<BF16>(fr, max(lo, 0));
      nw[x] = make_float2(u < NP ? wb * kLog2e : -kInf, (u >= 1 && u < NP) ? wl * kLog2e : -kInf);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (tid + 64 * kMargWaves * i < nnw) nw[tid + 64 * kMargWaves * i] = g2[i];
  }
  if (!split) {
    if (tid < nt) fs[tid * kFs + kFsW00] = ldsw<BF16>(wch + tid * a.FB, 0) * kLog2e;
    init_flags(tid);
    __syncthreads();  // nw, fs, fl and the job order for every wave
  }
  // split: frame f's numerator arc weights and W00, taken by the den chain
  // that owns f out of its W before E overwrites it (one wave, LDS in order)
  auto own_arcs = [&](int f, const unsigned char* fr) -> float {
    for (int u = lane; u < NPG; u += 64) {
      const int lo = loff[u];
      const float wb = ldsw<BF16>(fr, boff[u]), wl = ldsw<BF16>(fr, max(lo, 0));
      nw[f * NPG + u] =
          make_float2(u < NP ? wb * kLog2e : -kInf, (u >= 1 && u < NP) ? wl * kLog2e : -kInf);
    }
    const float w = ldsw<BF16>(fr, 0) * kLog2e;
    if (lane == 0) fs[f * kFs + kFsW00] = w;
    return w;
  };
  CK_STAMP(5);
  // every LDS load below is unconditional (clamped index, unused values
  // masked afterwards): a load under a branch would pay its full latency

  // a recursion wave has passed frame f (its rows written, E_f read): one
  // LDS atomic after its own LDS writes (in order within the wave)
  auto mark = [&](int f, int bit) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_or(fl + f, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto mark_all = [&](int bit) {
    for (int f = 0; f < nt; ++f) mark(f, bit);
  };
  auto wait_bits = [&](int f, int want) {
    for (;;) {
      const int bits = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(fl + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      if ((bits & want) == want) break;
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };

  // LT_CK_PRIO: the den chains issue ahead of the other waves on their SIMD
  if (LT_CK_PRIO && role < 2) __builtin_amdgcn_s_setprio(LT_CK_PRIO);
  if (role == 0 && !a.local && !LT_ABL(a, 4)) {
    // ---- den alpha in scaled linear space. Lane p in [1, V]: alpha_f[p] =
    // al 2^S (log2 units relative to the walk's offset); each frame the
    // vector is taken over its own max, xa = alpha_f / 2^Ma with Ma = S + the
    // exponent of the largest core value (or the start state's a0, a log2
    // scalar beside the chain: its only in-arc is its blank loop), and the
    // step runs on xa: alpha_{f+1}[q] = 2^(Ma + c) sum_p xa[p] E[p][q]. So
    // every product and sum is relative to the vector's max, whatever the
    // frame's range (masked -inf weights are exact zeros): a value lost to
    // underflow is below 2^-126 of that max, which the marginal pass's
    // per-frame certificate bounds. Lane (q, h): destination q+1, sources p
    // in [16h, 16h+16) (+ p = 32 in h = 1), the blank self loop in h = 0;
    // halves combined by permlane.
    const int q = lane & 31, h = lane >> 5;
    const int qe = min(q, V - 1) + 1;
    const bool core = lane >= 1 && lane <= V;
    const float* xp = a.abd + ((long long)b * (a.K + 1) + k) * CP + min(lane, C - 1);
    const float xr = kNoAcq ? ld_sc1(xp) : *xp;
    const float x0 = lane < C ? xr : -kInf;
    float a0 = first_lane(x0);
    float S = wmax_u(core ? x0 : -kInf);  // -inf: no core state reached yet
    float al = (core && S != -kInf) ? __builtin_amdgcn_exp2f(x0 - S) : 0.f;
    if (split) wait_vmcnt(0);  // this wave's half of W
    // frame f's E terms of the lane (its sources' arcs into qe, source 32,
    // qe's blank self loop) and W00: alpha's own frames [0, hs) from W, their
    // E stored to its home; beta's once beta has passed them
    auto get_e = [&](int f, float* e, float& e32, float& eb, float& w00) {
      const unsigned char* fr = wrow(f);
      float* ef = eptr(f);
      const float cl = cfl[f];
      w00 = fs[f * kFs + kFsW00];
      if (f < hs) {
        if (split) w00 = own_arcs(f, fr);
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ldsw<BF16>(fr, min(16 * h + m, C - 1) * R + qe);
        e32 = ldsw<BF16>(fr, min(32, C - 1) * R + qe);
        eb = ldsw<BF16>(fr, qe * R);
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ew(e[m], cl);
        e32 = ew(e32, cl);
        eb = ew(eb, cl);
#pragma unroll
        for (int m = 0; m < 16; ++m) ef[min(16 * h + m, C - 1) * R + qe] = e[m];
        ef[min(32, C - 1) * R + qe] = e32;
        ef[qe * R] = eb;
        if (lane == 0) ef[0] = 0.f;  // (0, 0) is taken in log2 (xb[0] = 0)
      } else {
        wait_bits(f, kFlB);
        if (split) w00 = fs[f * kFs + kFsW00];
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ef[min(16 * h + m, C - 1) * R + qe];
        e32 = ef[min(32, C - 1) * R + qe];
        eb = ef[qe * R];
      }
    };
    // LT_CK_EPIPE: alpha's own frames' E a step ahead (only those: fetching
    // one of beta's frames early would wait on beta while beta waits on this
    // chain's previous frame)
    float e[16], e32 = 0.f, eb = 0.f, w00 = 0.f;
    if (kEpipe && nt > 0) get_e(0, e, e32, eb, w00);  // hs >= 1: frame 0 is alpha's
    for (int f = 0; f < nt; ++f) {
      const float cl = cfl[f];
      if (!kEpipe || f >= hs) get_e(f, e, e32, eb, w00);
      const float mc = wmax_u(core ? al : 0.f);
      int ex;
      (void)frexpf(mc, &ex);
      const float Ma = safe_max(mc > 0.f ? fmaxf(a0, S + (float)ex) : a0);
      // xa = alpha_f over 2^Ma (the marginals' row) and the step's operand
      // row buf (36 floats, 0 past V)
      const float xv = lane == 0 ? __builtin_amdgcn_exp2f(a0 - Ma) : al * __builtin_amdgcn_exp2f(S - Ma);
      if (lane < 36) buf[lane] = xv;
      if (lane < C) xa[f * CP + lane] = xv;
      if (lane == 0) {
        fs[f * kFs + kFsMa] = Ma;
        fs[f * kFs + kFsA0] = a0;
      }
      // LT_CK_EPIPE: the next frame's E under this step's LDS round trip
      // (a wave issues in order: fetched at the top of the next step, its
      // loads and exponentials sat on the chain)
      float en[16], en32 = 0.f, enb = 0.f, wn00 = 0.f;
      if (kEpipe && f + 1 < hs) get_e(f + 1, en, en32, enb, wn00);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 b4 = *(const float4*)(buf + 16 * h + 4 * g4);
        s0 = __builtin_fmaf(b4.x, e[4 * g4 + 0], s0);
        s1 = __builtin_fmaf(b4.y, e[4 * g4 + 1], s1);
        s0 = __builtin_fmaf(b4.z, e[4 * g4 + 2], s0);
        s1 = __builtin_fmaf(b4.w, e[4 * g4 + 3], s1);
      }
      // h = 1: source 32 (buf[32] = 0 unless C > 32); h = 0: the blank loop of qe
      s0 = __builtin_fmaf(h ? buf[32] : buf[qe], h ? e32 : eb, s0);
      const float sq = half_sum(s0 + s1);  // lane q: alpha'[q+1] / 2^(Ma + c)
      S = Ma + cl;
      a0 += w00;
      const float sh = from_prev(sq, 0.f);
      al = core ? sh : 0.f;
      __builtin_amdgcn_wave_barrier();
      mark(f, kFlA);
      if (kEpipe && f + 1 < hs) {
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = en[m];
        e32 = en32;
        eb = enb;
        w00 = wn00;
      }
    }
  } else if (role == 1 && !a.local && !LT_ABL(a, 4)) {
    // ---- den beta, the same scaled linear space; frame f gets beta_{f+1}.
    // Each frame the core vector over its own max: xb = beta_{f+1} / 2^Mb;
    // the step runs on xb. Lane (j, h): core source j+1 over labels y in
    // [16h+1, 16h+16], the blank in h = 0; every lane also one term of the
    // start state's sum (log2 scalar b0: no core state depends on it).
    const int j = lane & 31, h = lane >> 5;
    const int pe = min(j, V - 1) + 1;
    const bool core = lane >= 1 && lane <= V;
    const float* xp = a.bbd + ((long long)b * (a.K + 1) + k + 1) * CP + min(lane, C - 1);
    const float xr = kNoAcq ? ld_sc1(xp) : *xp;
    const float x0 = lane < C ? xr : -kInf;
    float b0 = first_lane(x0);
    float S = safe_max(wmax_u(core ? x0 : -kInf));
    float be = core ? __builtin_amdgcn_exp2f(x0 - S) : 0.f;
    if (split) wait_vmcnt(0);  // this wave's half of W
    // frame f's E terms of the lane (source pe's arcs, its blank, E[0][j+1])
    // and W00: beta's own frames [hs, nt) from W, alpha's once alpha passed them
    auto get_e = [&](int f, float* e, float& eb, float& e0y, float& w00) {
      const unsigned char* fr = wrow(f);
      float* ef = eptr(f);
      const float cl = cfl[f];
      w00 = fs[f * kFs + kFsW00];
      if (f >= hs) {
        if (split) w00 = own_arcs(f, fr);
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ldsw<BF16>(fr, pe * R + min(16 * h + m + 1, V));
        eb = ldsw<BF16>(fr, pe * R);
        e0y = ldsw<BF16>(fr, min(j, V - 1) + 1);
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ew(e[m], cl);
        eb = ew(eb, cl);
        e0y = ew(e0y, cl);
#pragma unroll
        for (int m = 0; m < 16; ++m) ef[pe * R + min(16 * h + m + 1, V)] = e[m];
        ef[pe * R] = eb;
        ef[min(j, V - 1) + 1] = e0y;
        if (lane == 0) ef[0] = 0.f;
      } else {
        wait_bits(f, kFlA);
        if (split) w00 = fs[f * kFs + kFsW00];
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = ef[pe * R + min(16 * h + m + 1, V)];
        eb = ef[pe * R];
        e0y = ef[min(j, V - 1) + 1];
      }
    };
    // LT_CK_EPIPE: beta's own frames' E a step ahead (as alpha's)
    float e[16], eb = 0.f, e0y = 0.f, w00 = 0.f;  // e0y = E[0][j+1]
    if (kEpipe && nt - 1 >= hs) get_e(nt - 1, e, eb, e0y, w00);
    for (int f = nt - 1; f >= 0; --f) {
      const float cl = cfl[f];
      if (!kEpipe || f < hs) get_e(f, e, eb, e0y, w00);
      const float mc = wmax_u(be);
      int ex;
      (void)frexpf(mc, &ex);
      const float Mb = mc > 0.f ? S + (float)ex : S;
      const float xv = be * __builtin_amdgcn_exp2f(S - Mb);  // <= 1
      // buf[y-1] = xb[y] for core y; 0 past V
      if (lane >= 1 && lane <= 32) buf[lane - 1] = xv;
      if (lane < C) xb[f * CP + lane] = xv;
      if (lane == 0) {
        fs[f * kFs + kFsMb] = Mb;
        fs[f * kFs + kFsB0] = b0;
      }
      float en[16], enb = 0.f, en0y = 0.f, wn00 = 0.f;
      if (kEpipe && f - 1 >= hs) get_e(f - 1, en, enb, en0y, wn00);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 b4 = *(const float4*)(buf + 16 * h + 4 * g4);
        s0 = __builtin_fmaf(b4.x, e[4 * g4 + 0], s0);
        s1 = __builtin_fmaf(b4.y, e[4 * g4 + 1], s1);
        s0 = __builtin_fmaf(b4.z, e[4 * g4 + 2], s0);
        s1 = __builtin_fmaf(b4.w, e[4 * g4 + 3], s1);
      }
      const float bj = buf[j];
      s0 = __builtin_fmaf(h ? 0.f : bj, eb, s0);
      const float sj = half_sum(s0 + s1);  // lane j: beta_f[j+1] / 2^(Mb + c)
      // start state: (+)_y E[0][y] beta[y], then its own blank loop
      const float r0 = wsum_u(lane < 32 ? bj * e0y : 0.f);
      b0 = lse2_b2(b0 + w00, Mb + cl + __builtin_amdgcn_logf(r0));
      S = Mb + cl;
      const float sh = from_prev(sj, 0.f);
      be = core ? sh : 0.f;
      __builtin_amdgcn_wave_barrier();
      mark(f, kFlB);
      if (kEpipe && f - 1 >= hs) {
#pragma unroll
        for (int m = 0; m < 16; ++m) e[m] = en[m];
        eb = enb;
        e0y = en0y;
        w00 = wn00;
      }
    }
  } else if (role == 2 && !LT_ABL(a, 8)) {
    // ---- num alpha (log2): al'[u] = al[u] + blank(u) (+) al[u-1] + arc(u)
    float al[PPL];
    const float* src = a.nabd + ((long long)b * (a.K + 1) + k) * NPG;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int u = lane + 64 * r, uc = min(u, NPG - 1);
      const float v = kNoAcq ? ld_sc1(src + uc) : src[uc];  // log2, relative to the walk's offset
      al[r] = u < NPG ? v : -kInf;
    }
    for (int f = 0; f < nt; ++f) {
      if (split) wait_bits(f, f < hs ? kFlA : kFlB);  // nw[f] from its den chain
      float prev = -kInf, nv[PPL];
#pragma unroll
      for (int r = 0; r < PPL; ++r) {
        const int u = lane + 64 * r;
        if (u < NPG) an[f * NPG + u] = al[r];
        const float x = rot_prev(al[r]);
        const float pv = lane == 0 ? prev : x;
        prev = x;
        const float2 w = nw[f * NPG + min(u, NPG - 1)];
        nv[r] = lse2_b2(al[r] + w.x, pv + w.y);
      }
#pragma unroll
      for (int r = 0; r < PPL; ++r) al[r] = nv[r];
      __builtin_amdgcn_wave_barrier();
      mark(f, kFlNA);
    }
  } else if (role == 3 && !LT_ABL(a, 8)) {
    // ---- num beta (log2); frame f gets beta_{f+1}
    float be[PPL];
    const float* src = a.nbbd + ((long long)b * (a.K + 1) + k + 1) * NPG;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int u = lane + 64 * r, uc = min(u, NPG - 1);
      const float v = kNoAcq ? ld_sc1(src + uc) : src[uc];
      be[r] = u < NPG ? v : -kInf;
    }
    if (a.pf) {  // the chunk of the block about a.pf dispatches later, into L2
      const int c2 = c + a.pf;
      if (c2 < a.B * a.K) {
        const int j2 = c2 / a.B, b2 = c2 - j2 * a.B;
        int nf2 = a.nfr[b2];
        nf2 = nf2 < 0 ? 0 : (nf2 > a.T ? a.T : nf2);
        const int Kl2 = (nf2 + a.L - 1) / a.L, Kh2 = Kl2 / 2;
        const int k2 = j2 < 2 * Kh2 ? ((j2 & 1) ? Kh2 - 1 - (j2 >> 1) : Kh2 + (j2 >> 1)) : j2;
        const int t02 = k2 * a.L, t12 = max(t02, min(t02 + a.L, nf2));
        if (t12 > t02)
          pf_lines(a.W, ((long long)b2 * a.T + t02) * FR * (BF16 ? 2 : 4),
                   (long long)(t12 - t02) * a.FB, lds_base_addr((unsigned char*)buf), lane);
      }
    }
    for (int f = nt - 1; f >= 0; --f) {
      if (split) wait_bits(f, f < hs ? kFlA : kFlB);
      float nx[PPL], nv[PPL];
#pragma unroll
      for (int r = 0; r < PPL; ++r) nx[r] = rot_next(be[r]);
#pragma unroll
      for (int r = 0; r < PPL; ++r) {
        const int u = lane + 64 * r;
        if (u < NPG) bn[f * NPG + u] = be[r];
        const float nb = lane == 63 ? (r + 1 < PPL ? nx[r + 1 < PPL ? r + 1 : r] : -kInf) : nx[r];
        const float wb = nw[f * NPG + min(u, NPG - 1)].x;
        const float wl = nw[f * NPG + min(u + 1, NPG - 1)].y;
        nv[r] = lse2_b2(wb + be[r], (u + 1 < NP ? wl : -kInf) + nb);
      }
#pragma unroll
      for (int r = 0; r < PPL; ++r) be[r] = nv[r];
      __builtin_amdgcn_wave_barrier();
      mark(f, kFlNB);
    }
  } else {  // a recursion this chunk does not run (local / ablations): nothing to wait for
    mark_all(role == 0 ? kFlA : role == 1 ? kFlB : role == 2 ? kFlNA : kFlNB);
  }
  if (LT_CK_PRIO && role < 2) __builtin_amdgcn_s_setprio(0);
  CK_STAMP(2);

  // ---- marginals, one wave per frame: den - num, each normalised by its
  // frame total (alignments.py:311-317; numerator: reverse of :320-329).
  // Den in rows: lane (y, h) = column y = lane & 31 of rows p = 2 m + h,
  // then column 32 (lane p); arc (p, y) goes into q = y ? y : p. Den (p, y)
  // = E[p][y] xa[p] xb[q] 2^(Ma + Mb + c - Z) except (0, 0), the only arc
  // into the start state, taken in log2 (its beta may sit far above the
  // core's; xb[0] = 0 keeps it out of the sum). Every other den term is
  // <= 1 and the largest >= e^-61.
  constexpr int NROW = 17;  // row pairs: p = 2 m + h <= 33
  const int y = lane & 31, h = lane >> 5;
  const bool ycol = y < R;  // FULL: every lane
  int bo[PPL], lo[PPL];
#pragma unroll
  for (int r = 0; r < PPL; ++r) {
    const int uc = min(lane + 64 * r, NP - 1);
    bo[r] = boff[uc];
    lo[r] = max(loff[uc], 0);
  }
  // frames as jobs in the order their inputs complete (middle first): a
  // wave done with its recursion takes the next job and waits for that
  // frame's four bits, so the marginals overlap the longer recursions
  for (;;) {
    int jb = 0;
    if (lane == 0) jb = __hip_atomic_fetch_add(njob, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    jb = __builtin_amdgcn_readfirstlane(jb);
    if (jb >= nt || LT_ABL(a, 16)) break;
    const int f = ford[jb];
    for (;;) {
      const int bits = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(fl + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      if ((bits & kFlAll) == kFlAll) break;
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    float* fb = eptr(f);  // E_f, then the frame's dW in place
    // numerator terms (log2)
    float sb[PPL], sl[PPL];
    float mxn = -kInf;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int u = lane + 64 * r, uc = min(u, NP - 1);
      const float bu = bn[f * NPG + uc];
      const float2 w = nw[f * NPG + uc];
      const float tb = an[f * NPG + uc] + w.x + bu;
      const float tl = an[f * NPG + max(uc - 1, 0)] + w.y + bu;
      sb[r] = u < NP ? tb : -kInf;
      sl[r] = (u >= 1 && u < NP) ? tl : -kInf;
      mxn = fmaxf(mxn, fmaxf(sb[r], sl[r]));
    }
    mxn = safe_max(wmax_u(mxn));
    float zn = 0.f;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      sb[r] = __builtin_amdgcn_exp2f(sb[r] - mxn);
      sl[r] = __builtin_amdgcn_exp2f(sl[r] - mxn);
      zn += sb[r] + sl[r];
    }
    zn = wsum_u(zn);
    const float gn = zn > 0.f ? g / zn : 0.f;
    if (!a.local) {
      const float* xaf = xa + f * CP;
      const float* xbf = xb + f * CP;
      const int yc = min(y, R - 1);
      const float xby = xbf[yc];  // column y's beta (y >= 1)
      // rows: E, xa[p] and xb[p] (the blank column's beta) for p = 2 m + h
      float t[NROW], ra[NROW], rb[NROW];
#pragma unroll
      for (int m = 0; m < NROW; ++m) t[m] = fb[min(2 * m + h, C - 1) * R + yc];
#pragma unroll
      for (int m = 0; m < NROW; ++m) ra[m] = xaf[min(2 * m + h, C - 1)];
#pragma unroll
      for (int m = 0; m < NROW; ++m) rb[m] = xbf[min(2 * m + h, C - 1)];
      // column 32 (C = 33 only): lane p < 33
      const int pc = min(lane, C - 1);
      float tc = fb[pc * R + (R - 1)] * xaf[pc] * xbf[R - 1];
      const bool colc = R == 33 && lane < 33;
      tc = colc ? tc : 0.f;
      float sum = tc;
#pragma unroll
      for (int m = 0; m < NROW; ++m) {
        const bool live = ycol && 2 * m + h < C && (R < 33 || y < 32);
        const float v = t[m] * ra[m] * (y ? xby : rb[m]);
        t[m] = live ? v : 0.f;
        sum += t[m];
      }
      sum = wsum_u(sum);
      const float* fsf = fs + f * kFs;
      const float base = fsf[kFsMa] + fsf[kFsMb] + cfl[f];
      const float v00 = fsf[kFsA0] + fsf[kFsW00] + fsf[kFsB0];
      const float zl = lse2_b2(base + __builtin_amdgcn_logf(sum), v00);
      // the per-frame certificate of the scaled linear spaces (phases A, B
      // and C): every value lost to underflow anywhere -- an E below 2^-126,
      // a product or sum below 2^-126 of its vector's (or column's) max --
      // carries at most 2^(base - 126 + 15) of this frame's total 2^zl (base
      // = log2 of alpha_f's max x beta_{f+1}'s max x e^c, 2^15 the count of
      // such terms). base - zl <= kCert keeps that below 2^-47 of the
      // marginals' scale; a frame outside it (or a NaN / inf anywhere) sends
      // the utterance to the frame-serial kernels.
      if (!(base - zl <= kCert) && lane == 0) *cert_fail = 1;
      const float mult = g * __builtin_amdgcn_exp2f(base - zl);
      const float m00 = g * __builtin_amdgcn_exp2f(v00 - zl);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int m = 0; m < NROW; ++m) {
        const int p = 2 * m + h;
        if (ycol && p < C && (R < 33 || y < 32))
          fb[p * R + y] = (m == 0 && lane == 0) ? m00 : t[m] * mult;
      }
      if (colc) fb[pc * R + (R - 1)] = tc * mult;
    } else {
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      for (int e = lane; e < FR; e += 64) fb[e] = 0.f;
    }
    // string arcs sharing a lattice arc meet here (LDS adds, lane order)
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      const int u = lane + 64 * r;
      if (u < NP) {
        atomicAdd(fb + bo[r], -sb[r] * gn);
        if (u >= 1) atomicAdd(fb + lo[r], -sl[r] * gn);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if constexpr (BF16) {  // the frame's dW, rounded once, over its own W bytes
      unsigned short* fo = (unsigned short*)(wch + f * a.FB);
      for (int e = lane; e < FR; e += 64) fo[e] = f2bf(fb[e]);
    }
  }
  // the chunk's dW sits in LDS in place of its W: one streaming pass of
  // 16-byte stores (scalar stores only at the unaligned head and tail)
  __syncthreads();
  if (*cert_fail) {  // the frame-serial kernels redo this utterance after the launch
    if (tid == 0) a.uflag[b] = 1;
    return;
  }
  CK_STAMP(3);
  {
    const long long es = BF16 ? 2 : 4;
    const long long bytes = (long long)nt * a.FB;
    unsigned char* gdst = (unsigned char*)a.dW + off;  // same byte offset as W
    const long long head = min((long long)((16 - (off & 15)) & 15), bytes);
    const long long body = (bytes - head) & ~15LL;
    const unsigned char* src = wch;  // LDS image, (off & 15)-shifted like W
    for (long long x = tid; x < head / es; x += blockDim.x) {
      if constexpr (BF16) ((unsigned short*)gdst)[x] = ((const unsigned short*)src)[x];
      else ((float*)gdst)[x] = ((const float*)src)[x];
    }
    const uint4* s16 = (const uint4*)(src + head);
    uint4* d16 = (uint4*)(gdst + head);
    for (long long x = tid; x < body / 16; x += blockDim.x) d16[x] = s16[x];
    for (long long x = head + body + tid * es; x < bytes; x += blockDim.x * es) {
      if constexpr (BF16) *(unsigned short*)(gdst + x) = *(const unsigned short*)(src + x);
      else *(float*)(gdst + x) = *(const float*)(src + x);
    }
  }
  CK_STAMP(4);
  // padding frames of this chunk
  {
    const long long n = (long long)(tend - t1) * FR;
    const long long base = e0 + (long long)nt * FR;
    for (long long e = tid; e < n; e += blockDim.x) store_dw<BF16>(a.dW, base + e, 0.f);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
namespace {

int ck_env(const char* name, int dflt) { return lt_impl::tune_int(name, dflt); }
long long up256(long long x) { return (x + 255) & ~255LL; }
int al16(long long x) { return (int)((x + 15) & ~15LL); }

struct CkLayout {
  // state (kept from lt_chunk_forward to lt_chunk_backward)
  size_t uflag, lz, num, abd, bbd, nabd, nbbd, cf, mid, state;
  // scratch: forward = records + numerator bands; backward = the fallback's checkpoints
  size_t ready, rec, nb, f_alpha, f_an, f_loss, f_lz, f_num, f_side, scratch;
};

int ck_plan(const lt_problem* pb, int local_norm, CkArgs* a, CkLayout* w) {
  memset(a, 0, sizeof(*a));
  const int V = pb->vocab_size;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  const int es = bf16 ? 2 : 4;
  a->B = pb->batch; a->T = pb->max_frames; a->U = pb->max_labels;
  a->V = V; a->C = V + 1; a->R = V + 1; a->FR = a->C * a->R;
  a->NP = a->U + 1; a->NPG = (a->NP + 1) & ~1; a->PPL = (a->NPG + 63) / 64;
  a->CP = (a->C + 3) & ~3;
  a->local = local_norm ? 1 : 0;
#ifdef LT_DIAG
  a->dbg = ck_env("LT_CK_DBG", 0);
  a->pf = ck_env("LT_CK_PF", LT_CK_PF);
  if (const char* sp = lt_impl::tune_str("LT_CK_STAMPS")) a->stamps = (long long*)strtoull(sp, nullptr, 0);
#endif
  a->FB = (long long)a->FR * es;
  // A: per wave a ring of frame slots, the state-0 row and the gather tables
  const long long n16f = (a->FB + 30) / 16;
  a->a_ni = (int)((n16f + 63) / 64);
  a->a_slots = 3;
  a->a_slot_bytes = a->a_ni * 1024;
  a->a_off_rt = a->a_slots * a->a_slot_bytes;
  a->a_off_tab = a->a_off_rt + 128;
  a->a_wave_bytes = al16(a->a_off_tab + 8LL * a->NPG);
  // B: record rings (den alpha, den beta), G rings (num alpha, num beta)
  a->b_ni = (kRec * 4 + 15 + 1023) / 1024;
  a->b_slots = 4;
  a->b_off_ra = 0;
  a->b_off_rb = a->b_slots * a->b_ni * 1024;
  a->b_gslot = 1024;
  a->b_gslots = 16;
  a->b_off_ga = a->b_off_rb + a->b_slots * a->b_ni * 1024;
  a->b_off_gb = a->b_off_ga + a->b_gslots * a->b_gslot;
  a->b_off_buf = a->b_off_gb + a->b_gslots * a->b_gslot;
  // C: the chunk's frames, per-frame alpha/beta vectors, tables; L frames
  // per chunk chosen so that two workgroups share a CU
  auto c_bytes = [&](int L, CkArgs* t) {
    const long long n16 = ((long long)L * a->FB + 30) / 16;
    t->c_ni = (int)((n16 + 63) / 64);
    int off = t->c_ni * 1024;
    t->c_off_ad = off; off += al16(4LL * L * a->CP);
    t->c_off_bd = off; off += al16(4LL * L * a->CP);
    t->c_off_an = off; off += al16(4LL * L * a->NPG);
    t->c_off_bn = off; off += al16(4LL * L * a->NPG);
    t->c_off_nw = off; off += al16(8LL * L * a->NPG);
    t->c_off_fs = off; off += al16(4LL * L * kFs);
    t->c_off_tab = off; off += al16(8LL * a->NPG + 4LL * a->U);
    t->c_off_cf = off; off += al16(4LL * L);
    t->c_off_buf = off; off += 4 * 64 * 4;
    t->c_off_fl = off; off += al16(4LL * (2 * L + 3));
    t->c_off_e = off; off += bf16 ? al16(4LL * L * ((a->FR + 3) & ~3)) : 0;
    return off;
  };
  int L = std::max(1, std::min(32, ck_env("LT_CHUNK_LEN", 32)));
  // LDS per workgroup: kChunkLds lets four share a CU (the per-frame chains
  // of phase C are latency-bound: more workgroups in flight beat longer chunks)
  const int budget = ck_env("LT_CHUNK_LDS", kChunkLds);
  while (L > 4 && c_bytes(L, a) > budget) --L;
  if (c_bytes(L, a) > 160 * 1024) return lt_impl::set_error(LT_EUNSUPPORTED, "chunk: LDS");
  a->c_bytes = c_bytes(L, a);
  a->L = L;
  a->K = std::max(1, (a->T + L - 1) / L);
  if (a->K >= (1 << 24)) return lt_impl::set_error(LT_EUNSUPPORTED, "chunk: too many frames");
  a->NGc = (L + kGrp - 1) / kGrp;
  // workspace
  const long long B = a->B, K = a->K, T = a->T;
  size_t o = 0;
  w->uflag = o; o += up256(4 * B);
  w->lz = o; o += up256(4 * B);
  w->num = o; o += up256(4 * B);
  w->abd = o; o += up256(4 * B * (K + 1) * a->CP);
  w->bbd = o; o += up256(4 * B * (K + 1) * a->CP);
  w->nabd = o; o += up256(4 * B * (K + 1) * a->NPG);
  w->nbbd = o; o += up256(4 * B * (K + 1) * a->NPG);
  w->cf = o; o += up256(4 * B * T);
  w->mid = o; o += up256(8 * B);
  w->state = o;
  size_t s = 0;
  w->ready = s; s += up256(8LL * B * K + 32LL * B);  // ready flags, then the progress words
  w->rec = s; s += up256(4LL * B * K * kRec);
  a->nbs = (a->NGc * (kGrp + 1) * a->NPG + 31) & ~31;
  w->nb = s; s += up256(4LL * B * K * a->nbs);
  const size_t fwd = s;
  s = 0;
  w->f_alpha = s; s += up256(4LL * B * T * a->C);
  w->f_an = s; s += up256(4LL * B * T * a->NP);
  w->f_loss = s; s += up256(4 * B);
  w->f_lz = s; s += up256(4 * B);
  w->f_num = s; s += up256(4 * B);
  w->f_side = s; s += up256((long long)lt_impl::serial_side_bytes(pb, local_norm));
  w->scratch = std::max(fwd, s);
  return LT_OK;
}

void ck_bind(CkArgs* a, const CkLayout& w, void* state, void* scratch) {
  char* st = (char*)state;
  char* sc = (char*)scratch;
  a->uflag = (int*)(st + w.uflag);
  a->log_z = (float*)(st + w.lz);
  a->num = (float*)(st + w.num);
  a->abd = (float*)(st + w.abd);
  a->bbd = (float*)(st + w.bbd);
  a->nabd = (float*)(st + w.nabd);
  a->nbbd = (float*)(st + w.nbbd);
  a->cf = (float*)(st + w.cf);
  a->mid = (float*)(st + w.mid);
  a->rec = sc ? (float*)(sc + w.rec) : nullptr;
  a->nb = sc ? (float*)(sc + w.nb) : nullptr;
  a->ready = sc ? (unsigned long long*)(sc + w.ready) : nullptr;
  a->prog = sc ? (unsigned long long*)(sc + w.ready) + (long long)a->B * a->K : nullptr;
}

int ck_launch(const void* k, int grid, int lds, hipStream_t st, const CkArgs& a,
              int threads = 256) {
  if (grid <= 0) return LT_OK;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  void* args[] = {(void*)&a};
  e = hipLaunchKernel(k, dim3(grid), dim3(threads), args, lds, st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  return LT_OK;
}

int ck_check(const lt_problem* pb) {
  if (!pb) return lt_impl::set_error(LT_EINVAL, "null problem");
  if (pb->batch < 0 || pb->max_frames < 0 || pb->max_labels < 0)
    return lt_impl::set_error(LT_EINVAL, "negative dimension");
  if (pb->weight_dtype != LT_DTYPE_F32 && pb->weight_dtype != LT_DTYPE_BF16)
    return lt_impl::set_error(LT_EINVAL, "weight_dtype must be LT_DTYPE_F32 or LT_DTYPE_BF16");
  if (!lt_impl::chunk_eligible(pb))
    return lt_impl::set_error(LT_EUNSUPPORTED,
                              "chunked path: FullNGram n = 1, vocab_size <= 32, labels < 128");
  return LT_OK;
}

const void* ck_kernel_ab(int ppl, bool bf16, bool full) {
  if (full)
    return ppl == 1 ? (bf16 ? (const void*)ck_ab_kernel<true, 1, true>
                            : (const void*)ck_ab_kernel<false, 1, true>)
                    : (bf16 ? (const void*)ck_ab_kernel<true, 2, true>
                            : (const void*)ck_ab_kernel<false, 2, true>);
  return ppl == 1 ? (bf16 ? (const void*)ck_ab_kernel<true, 1, false>
                          : (const void*)ck_ab_kernel<false, 1, false>)
                  : (bf16 ? (const void*)ck_ab_kernel<true, 2, false>
                          : (const void*)ck_ab_kernel<false, 2, false>);
}
const void* ck_kernel_b(int ppl) {
  return ppl == 1 ? (const void*)ck_combine_kernel<1> : (const void*)ck_combine_kernel<2>;
}
int ck_cus() {
  static int cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) !=
                       hipSuccess)
    cus[dev] = 0;
  return cus[dev];
}
// This call's hand-off tags (CkArgs::ready / prog): splitmix64 over a
// per-process counter seeded from the clock and the pid, so consecutive calls
// never share a tag and a stale word from an earlier call (or scratch
// garbage) reads as "not yet published"; no memset before the launch.
unsigned long long ck_seed() {
  unsigned long long z = (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
  z ^= (unsigned long long)getpid() << 32;
  z ^= (unsigned long long)(uintptr_t)&ck_cus;
  return z;
}
void ck_tags(CkArgs& a) {
  static std::atomic<unsigned long long> ctr{ck_seed()};
  unsigned long long z = ctr.fetch_add(0x9E3779B97F4A7C15ull) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  a.ep_tag = ((z >> 2) | (1ull << 61)) << 2;                 // bits 2..63, never 0
  a.pg_tag = ((z & 0xFFFFFFFFFFull) | (1ull << 39)) << 24;  // bits 24..63, never 0
}
// Phases A and B: ONE launch with the walks among its workgroups, or A and B as two launches
// when the walks (one workgroup per utterance, at most one of the two
// workgroup slots per CU the launch's registers allow) could hold half the
// chip's slots while they wait (B > CUs), or LT_CHUNK_FUSE=0. The walks'
// block position, the fraction 1 - 48 / B of A's workgroups: a walk follows
// A's front and then needs about K x 0.55 us on its own, so small batches
// start it early and larger ones keep its slots for A longer
// (tools/walk_sweep.py: B = 64 best at 0-25 %, B = 128 at 50-65 %;
// LT_CHUNK_WALK_AT overrides, in percent).
int ck_launch_ab(CkArgs& a, bool bf16, hipStream_t st) {
  ck_tags(a);
  // Under stream capture the tag above is baked into the graph, so every
  // replay would carry the same one and see the previous replay's words as
  // published: zero them by a memset node instead (any nonzero tag is then
  // fresh). Eager calls keep the per-call tag and no memset.
  if (lt_impl::stream_capturing(st)) {
    const hipError_t e =
        hipMemsetAsync(a.ready, 0, 8ull * a.B * a.K + 32ull * a.B, st);
    if (e != hipSuccess) return lt_impl::set_error(LT_EHIP, hipGetErrorString(e));
  }
  const bool fuse = a.B <= ck_cus() && ck_env("LT_CHUNK_FUSE", 1) != 0;
  a.nc = fuse ? a.B : 0;
  const long long items = 2LL * a.B * ((a.K + 1) / 2);
  const long long nwa = (items + 3) / 4;
  const int at = ck_env("LT_CHUNK_WALK_AT", std::max(0, 100 - 4800 / std::max(a.B, 1)));
  a.wpos = (int)(nwa * std::min(std::max(at, 0), 100) / 100);
  int rc = ck_launch(ck_kernel_ab(a.PPL, bf16, a.V == 32), (int)(a.nc + nwa),
                     std::max(fuse ? kWalkLdsBytes : 0, kALds ? kALdsBytes : 0), st, a);
  if (rc || fuse) return rc;
  return ck_launch(ck_kernel_b(a.PPL), a.B, kWalkLdsBytes, st, a);
}
const void* ck_kernel_c(int ppl, bool bf16, bool full) {
  if (full)
    return ppl == 1 ? (bf16 ? (const void*)ck_marg_kernel<true, 1, true>
                            : (const void*)ck_marg_kernel<false, 1, true>)
                    : (bf16 ? (const void*)ck_marg_kernel<true, 2, true>
                            : (const void*)ck_marg_kernel<false, 2, true>);
  return ppl == 1 ? (bf16 ? (const void*)ck_marg_kernel<true, 1, false>
                          : (const void*)ck_marg_kernel<false, 1, false>)
                  : (bf16 ? (const void*)ck_marg_kernel<true, 2, false>
                          : (const void*)ck_marg_kernel<false, 2, false>);
}
int ck_lds_c(const CkArgs& a, bool bf16) {
  (void)bf16;
  int lds = a.c_bytes;
#ifdef LT_DIAG
  lds += ck_env("LT_CK_LDS_PAD", 0);  // occupancy experiments
#endif
  return lds;
}

}  // namespace

namespace lt_impl {
bool chunk_eligible(const lt_problem* pb) {
  if (ck_env("LT_CHUNK", 1) == 0) return false;
  if (pb->context_size != 1 || pb->vocab_size < 1 || pb->vocab_size > 32) return false;
  if (pb->max_labels + 1 > 128) return false;  // <= 2 string positions per lane
  const long long C = pb->vocab_size + 1;
  if ((long long)pb->batch * pb->max_frames * C * C >= (1LL << 31)) return false;
  return true;
}
// The chunked scan's phases A and C are throughput work that grows with B,
// while the frame-serial checkpointing design (pipe_kernel + marg_kernel)
// hides its chains behind idle CUs until 2B recursions fill them: measured
// crossover B ~ 178 on 256 CUs (round 4, profiles/r04_design_crossover.txt:
// chunk 0.641 / 0.801 / 0.966 / 1.130 / 1.294 ms against 0.746 / 0.863 /
// 0.924 / 0.994 / 1.121 ms at B = 128 / 160 / 192 / 224 / 256), so the chunked
// scan while 16 B <= 11 CUs (B <= 176). LT_CHUNK=1 forces the chunked scan,
// LT_CHUNK=0 forbids it.
bool chunk_preferred(const lt_problem* pb) {
  if (!chunk_eligible(pb)) return false;
  if (ck_env("LT_CHUNK", -1) == 1) return true;
  const long long cus = ck_cus();
  return cus <= 0 || 16LL * pb->batch <= 11LL * cus;
}
}  // namespace lt_impl

namespace lt_impl {
// lt_loss_grad's chunked route: A, B and C, then ONE frame-serial call for
// the utterances outside the fast path's range (it writes their loss, log_z,
// num and dW; its workgroups return at once for every other utterance).
// `state` / `scratch` as lt_chunk_workspace_bytes; the scratch's records
// and bands are dead once B has run, so the fallback reuses the region.
int chunk_loss_grad(const lt_problem* pb, int local_norm, const void* W, const int32_t* num_frames,
                    const int32_t* labels, const int32_t* num_labels, float* loss, float* log_z,
                    float* num, void* dW, void* state, size_t state_bytes, void* scratch,
                    size_t scratch_bytes, void* stream) {
  int rc = ck_check(pb);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  CkArgs a;
  CkLayout w;
  if ((rc = ck_plan(pb, local_norm, &a, &w))) return rc;
  if (state_bytes < w.state || scratch_bytes < w.scratch)
    return set_error(LT_EINVAL, "workspace too small");
  ck_bind(&a, w, state, scratch);
  a.W = (const unsigned char*)W;
  a.nfr = num_frames; a.labels = labels; a.nlab = num_labels;
  a.loss = loss;
  a.lz_out = log_z;
  a.num_out = num;
  a.dW = dW;
  hipStream_t st = (hipStream_t)stream;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  // the walks' second halves run in phase C's launch (blocks [0, B))
  a.half = 1;
  if ((rc = ck_launch_ab(a, bf16, st))) return rc;
  a.cont = 1;
  if ((rc = ck_launch(ck_kernel_c(a.PPL, bf16, a.V == 32), a.B + a.B * a.K,
                      std::max(ck_lds_c(a, bf16), kWalkLdsBytes), st, a, 64 * kMargWaves)))
    return rc;
  char* sc = (char*)scratch;
  return serial_loss(pb, local_norm, W, num_frames, labels, num_labels, a.uflag, loss, log_z, num,
                     (float*)(sc + w.f_alpha), (float*)(sc + w.f_an), nullptr, dW, sc + w.f_side,
                     stream);
}
}  // namespace lt_impl

extern "C" {

int lt_chunk_workspace_bytes(const lt_problem* pb, int32_t local_norm, size_t* state_bytes,
                             size_t* scratch_bytes) {
  int rc = ck_check(pb);
  if (rc) return rc;
  CkArgs a;
  CkLayout w;
  if ((rc = ck_plan(pb, local_norm, &a, &w))) return rc;
  if (state_bytes) *state_bytes = w.state;
  if (scratch_bytes) *scratch_bytes = w.scratch;
  return LT_OK;
}

int lt_chunk_forward(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels, const int32_t* num_labels,
                     float* loss, float* log_z, float* num, void* state, size_t state_bytes,
                     void* scratch, size_t scratch_bytes, void* stream) {
  int rc = ck_check(pb);
  if (rc) return rc;
  if (pb->batch == 0) return LT_OK;
  CkArgs a;
  CkLayout w;
  if ((rc = ck_plan(pb, local_norm, &a, &w))) return rc;
  if ((pb->max_frames > 0 && !W) || !num_frames || !num_labels || !loss ||
      (pb->max_labels > 0 && !labels) || !state || !scratch)
    return lt_impl::set_error(LT_EINVAL, "null pointer");
  if (((uintptr_t)W & 15) || ((uintptr_t)state & 15) || ((uintptr_t)scratch & 15))
    return lt_impl::set_error(LT_EINVAL, "W / workspaces must be 16-byte aligned");
  if (state_bytes < w.state || scratch_bytes < w.scratch)
    return lt_impl::set_error(LT_EINVAL, "workspace too small");
  ck_bind(&a, w, state, scratch);
  a.W = (const unsigned char*)W;
  a.nfr = num_frames; a.labels = labels; a.nlab = num_labels;
  a.loss = loss;
  a.lz_out = log_z;
  a.num_out = num;
  // the loss alone has no phase C to certify it: chunks outside the strict
  // range (every weight finite, within e^61 of its frame's max) leave here
  a.strict = 1;
  hipStream_t st = (hipStream_t)stream;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  if ((rc = ck_launch_ab(a, bf16, st))) return rc;
  // utterances outside the fast path's range: the frame-serial kernels
  // (their workgroups return at once for every other utterance)
  return lt_impl::serial_loss(pb, local_norm, W, num_frames, labels, num_labels, a.uflag, loss,
                              log_z ? log_z : a.log_z, num ? num : a.num, nullptr, nullptr,
                              nullptr, nullptr, nullptr, stream);
}

int lt_chunk_backward(const lt_problem* pb, int32_t local_norm, const void* W,
                      const int32_t* num_frames, const int32_t* labels, const int32_t* num_labels,
                      const float* grad, void* dW, void* state, size_t state_bytes, void* scratch,
                      size_t scratch_bytes, void* stream) {
  int rc = ck_check(pb);
  if (rc) return rc;
  if (pb->batch == 0 || pb->max_frames == 0) return LT_OK;
  CkArgs a;
  CkLayout w;
  if ((rc = ck_plan(pb, local_norm, &a, &w))) return rc;
  if (!W || !num_frames || !num_labels || !dW || (pb->max_labels > 0 && !labels) || !state ||
      !scratch)
    return lt_impl::set_error(LT_EINVAL, "null pointer");
  if (((uintptr_t)W & 15) || ((uintptr_t)state & 15) || ((uintptr_t)scratch & 15))
    return lt_impl::set_error(LT_EINVAL, "W / workspaces must be 16-byte aligned");
  if (state_bytes < w.state || scratch_bytes < w.scratch)
    return lt_impl::set_error(LT_EINVAL, "workspace too small");
  ck_bind(&a, w, state, nullptr);
  a.W = (const unsigned char*)W;
  a.nfr = num_frames; a.labels = labels; a.nlab = num_labels;
  a.grad = grad;
  a.dW = dW;
  hipStream_t st = (hipStream_t)stream;
  const bool bf16 = pb->weight_dtype == LT_DTYPE_BF16;
  if ((rc = ck_launch(ck_kernel_c(a.PPL, bf16, a.V == 32), a.B * a.K, ck_lds_c(a, bf16), st, a,
                      64 * kMargWaves)))
    return rc;
  char* sc = (char*)scratch;
  return lt_impl::serial_loss(pb, local_norm, W, num_frames, labels, num_labels, a.uflag,
                              (float*)(sc + w.f_loss), (float*)(sc + w.f_lz),
                              (float*)(sc + w.f_num), (float*)(sc + w.f_alpha),
                              (float*)(sc + w.f_an), grad, dW, sc + w.f_side, stream);
}

}  // extern "C"
