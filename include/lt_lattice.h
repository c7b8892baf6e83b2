/*
 * lt_lattice.h -- C ABI of the MI355X (gfx950) recognition-lattice kernels.
 *
 * This is the drop-in boundary for the hot path of theadamsabra/last_torch:
 * the semiring shortest distance / forward-backward over a GNAT recognition
 * lattice built from alignments.FrameDependent x contexts.FullNGram, under
 * semirings.Log / MaxTropical (and Real for the forward KATs).
 *
 * The reference has no FFI (it is pure PyTorch); every entry point below
 * replaces one method of last_torch/lattices.py.RecognitionLattice and is the
 * function that method's drop-in binds to (ctypes stub: INTEGRATION.md).
 *
 * Conventions
 *   - All pointers are DEVICE pointers (caller-owned, e.g. from the PyTorch
 *     caching allocator or hipMalloc). The library keeps no allocations.
 *   - Arc weights W are one contiguous row-major tensor [B, T, C, V+1]:
 *     W[b,t,p,0] = blank weight from context state p (weight_fns.py:69-71),
 *     W[b,t,p,y] = lexical weight of label y in 1..V (weight_fns.py:72-75).
 *     W must be 16-byte aligned; the 16-byte granule that holds its last byte
 *     must be readable (always true for hipMalloc / torch allocations).
 *     dtype: LT_DTYPE_F32 or LT_DTYPE_BF16; arithmetic is always fp32.
 *   - C = sum_{i=0..n} V^i context states (contexts.py:181-182).
 *   - Lengths (num_frames, num_labels) and labels are int32. Lengths are
 *     clamped to [0, T] / labels outside [0, V] are treated as epsilon (0).
 *   - Every call is asynchronous and ordered on `stream` (a hipStream_t;
 *     NULL = legacy default stream). Calls are reentrant.
 *   - Return value: LT_OK (0) or a negative LT_E* code; lt_last_error()
 *     gives a thread-local message. No C++ exception crosses the ABI.
 */
#ifndef LT_LATTICE_H_
#define LT_LATTICE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LT_OK 0
#define LT_EINVAL (-1)       /* bad argument / shape */
#define LT_EUNSUPPORTED (-2) /* configuration outside what the kernels do */
#define LT_EHIP (-3)         /* HIP runtime error (launch, attribute) */
#define LT_ENOMEM (-4)       /* host memory exhausted (the host twin's workers) */

#define LT_DTYPE_F32 0
#define LT_DTYPE_BF16 1

/* semirings.py: Log (184-305), MaxTropical (308-401), Real (143-173). */
#define LT_SEMIRING_LOG 0
#define LT_SEMIRING_MAX 1
#define LT_SEMIRING_REAL 2

/* shortest_path label convention.
 * LT_LABELS_REFERENCE reproduces lattices.py:242-244 exactly: a lexical
 * frame emits argmax over the 0-based vocab axis, i.e. label y as y-1.
 * LT_LABELS_TRUE emits y (1..V) as documented at lattices.py:204-206. */
#define LT_LABELS_TRUE 0
#define LT_LABELS_REFERENCE 1

typedef struct lt_problem {
  int32_t batch;        /* B: number of utterances (flattened batch dims)  */
  int32_t max_frames;   /* T: padded number of frames                      */
  int32_t vocab_size;   /* V: lexical vocabulary size (FullNGram.vocab_size) */
  int32_t context_size; /* n: FullNGram.context_size                       */
  int32_t max_labels;   /* U: padded number of labels (0 if unused)        */
  int32_t weight_dtype; /* LT_DTYPE_F32 or LT_DTYPE_BF16                    */
} lt_problem;

/* FullNGram.num_states() (contexts.py:181-182). */
int lt_num_context_states(int32_t vocab_size, int32_t context_size,
                          int64_t* num_states);

/* RecognitionLattice._forward (lattices.py:379-496): shortest distance of the
 * denominator lattice under `semiring`.
 *   dist  [B]        out: (+)_q alpha_T[q]
 *   alpha [B,T,C]    out (nullable): alpha_t before frame t, padding frames
 *                    carry (lattices.py:460-462, 886-890). fp32. */
int lt_den_forward(const lt_problem* pb, int32_t semiring, const void* W,
                   const int32_t* num_frames, float* dist, float* alpha,
                   void* stream);

/* ForwardBackward.backward / _backward (lattices.py:514-642, 686-799) done
 * right (reference defects D3/D4): backward weights + arc marginals.
 *   dW[b,t,p,y] = grad[b] * exp(alpha_t[p] + W[b,t,p,y] + beta_{t+1}[next(p,y)]
 *                 - log_z[b])   (alignments.py:300-318), 0 on padding frames.
 *   log_z, alpha: outputs of lt_den_forward(LOG). grad nullable (= ones).
 *   dW has W's dtype and shape. */
int lt_den_backward(const lt_problem* pb, const void* W,
                    const int32_t* num_frames, const float* log_z,
                    const float* alpha, const float* grad, void* dW,
                    void* stream);

/* RecognitionLattice._string_forward (lattices.py:250-377): numerator
 * (intersection with the label string) shortest distance.
 *   labels [B,U] int32, num_labels [B] int32
 *   num [B] out; alpha_num [B,T,U+1] out (nullable). */
int lt_num_forward(const lt_problem* pb, int32_t semiring, const void* W,
                   const int32_t* num_frames, const int32_t* labels,
                   const int32_t* num_labels, float* num, float* alpha_num,
                   void* stream);

/* RecognitionLattice.forward (lattices.py:131-183), fused denominator +
 * numerator in one launch (Log semiring).
 *   local_norm != 0: LocallyNormalizedWeightFn (lattices.py:178-179),
 *                    loss = -num and the denominator is skipped.
 *   loss [B] out; log_z [B], num [B] out; alpha [B,T,C], alpha_num
 *   [B,T,U+1] out (needed by lt_loss_backward; nullable otherwise).
 *   Checkpointing mode (beta_num and arcs non-NULL, and beta unless
 *   local_norm): the backward recursion -- which depends only on W -- runs
 *   here too (for the bigram in the same launch as the forward; otherwise
 *   launched before it on `stream`: the library forks no stream), writing
 *     beta     [B,T,C]    beta_{t+1} of frame t (alignments.py:315-316)
 *     beta_num [B,T,U+1]  numerator beta_{t+1} of frame t
 *     arcs     [B,4(U+1)] int32 numerator arc table
 *   so that lt_loss_backward is a single fully parallel streaming pass. */
int lt_loss_forward(const lt_problem* pb, int32_t local_norm, const void* W,
                    const int32_t* num_frames, const int32_t* labels,
                    const int32_t* num_labels, float* loss, float* log_z,
                    float* num, float* alpha, float* alpha_num, float* beta,
                    float* beta_num, int32_t* arcs, void* stream);

/* d loss / d W for lt_loss_forward (what loss.backward() in the reference
 * should produce; it raises there, D1/D3):
 *   dW = grad[b] * (den_marginals - num_marginals)   (global normalisation)
 *   dW = -grad[b] * num_marginals                    (local_norm != 0)
 * Utterances whose numerator is -inf (loss = +inf) get dW = 0.
 * With the checkpoints of lt_loss_forward (beta_num, arcs and, unless
 * local_norm, beta non-NULL) this is one streaming pass over (b, t) tiles;
 * otherwise the backward recursion runs here. workspace:
 * lt_loss_backward_workspace_bytes() bytes of device memory (0 for most
 * shapes and in checkpointing mode; then it may be NULL). */
int lt_loss_backward_workspace_bytes(const lt_problem* pb, int32_t local_norm,
                                     size_t* bytes);
int lt_loss_backward(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels,
                     const int32_t* num_labels, const float* log_z,
                     const float* num, const float* alpha,
                     const float* alpha_num, const float* beta,
                     const float* beta_num, const int32_t* arcs,
                     const float* grad, void* dW, void* workspace,
                     size_t workspace_bytes, void* stream);

/* Loss and its gradient in one call: loss, log_z, num as lt_loss_forward and
 *   dW = d(sum_b loss_b)/dW   (grad = ones; lt_scale_grad applies another)
 * -- what RecognitionLattice.forward followed by loss.sum().backward() means
 * to produce (lattices.py:131-183 with the backward of alignments.py:300-318;
 * D1/D3 in the reference). Utterances with num = -inf get dW = 0.
 * For the bigram (FullNGram n = 1, V <= 32, U <= 127) while 16 B <= 11 CUs
 * this is the chunked two-level scan below (two launches, plus one
 * frame-serial launch whose workgroups exit at once unless an utterance is
 * out of its range or a hand-off wait timed out; no memset: the hand-off
 * words carry a per-call tag, so the workspace's contents do not matter;
 * under stream capture, where every replay would reuse the captured tag, a
 * memset node zeroes them instead). Other
 * bigram shapes with 2B below the CU count run ONE fused launch (alpha and
 * beta recursions plus workgroups that turn every frame into marginals as
 * soon as both recursions have passed it; should a hand-off wait time out,
 * the affected loss is NaN, never a silent wrong value). Otherwise
 * lt_loss_forward + lt_loss_backward run in turn.
 *   workspace: lt_loss_grad_workspace_bytes() bytes of device memory. */
int lt_loss_grad_workspace_bytes(const lt_problem* pb, int32_t local_norm,
                                 size_t* bytes);
int lt_loss_grad(const lt_problem* pb, int32_t local_norm, const void* W,
                 const int32_t* num_frames, const int32_t* labels,
                 const int32_t* num_labels, float* loss, float* log_z,
                 float* num, void* dW, void* workspace, size_t workspace_bytes,
                 void* stream);
/* dW[b,...] *= grad[b] in place (grad [B] fp32), the chain rule for an
 * incoming gradient after lt_loss_grad; utterances with grad[b] == 1 cost
 * nothing. */
int lt_scale_grad(const lt_problem* pb, const float* grad, void* dW,
                  void* stream);

/* The bigram loss as a chunked two-level scan (lt_chunk.hip): FullNGram
 * n = 1, 1 <= vocab_size <= 32, max_labels <= 127, Log semiring. Each
 * utterance is cut into chunks of L frames (L from a 40 KB LDS budget per
 * workgroup: 6 for V = 32, U = 100, fp32); the serial chains are L frames
 * and T/L chunk steps (T/7 numerator group steps) instead of T.
 *   lt_chunk_forward  = RecognitionLattice.forward (lattices.py:131-183):
 *     loss [B] (log_z, num [B] nullable outputs); keeps the alpha / beta
 *     values at every chunk boundary in `state`.
 *   lt_chunk_backward = its gradient (alignments.py:300-318 composed in
 *     reverse, D1-D4 in the reference): dW = grad[b] * (den - num marginals)
 *     (grad nullable = ones), from `state` and W alone.
 * `state` must live from the forward to the backward; `scratch` only during
 * each call. Utterances with a frame whose weights are not all finite or
 * span more than 61 (max - min) run through the frame-serial kernels inside
 * the same calls (same results, slower). Sizes from
 * lt_chunk_workspace_bytes(); both buffers 16-byte aligned.
 * Phase A (chunk transfers) and phase B (the boundary walks) share one
 * launch while B <= CUs: per-chunk ready flags tagged per call (62-bit;
 * whatever `scratch` held reads as "not published"), write-through stores,
 * agent-scope acquire on the walks' side; a walk that never sees its chunk
 * times out and sends its utterance to the frame-serial kernels.
 * lt_loss_grad runs the same launches for every shape they take. */
int lt_chunk_workspace_bytes(const lt_problem* pb, int32_t local_norm, size_t* state_bytes,
                             size_t* scratch_bytes);
int lt_chunk_forward(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels,
                     const int32_t* num_labels, float* loss, float* log_z, float* num,
                     void* state, size_t state_bytes, void* scratch, size_t scratch_bytes,
                     void* stream);
int lt_chunk_backward(const lt_problem* pb, int32_t local_norm, const void* W,
                      const int32_t* num_frames, const int32_t* labels,
                      const int32_t* num_labels, const float* grad, void* dW, void* state,
                      size_t state_bytes, void* scratch, size_t scratch_bytes, void* stream);

/* RecognitionLattice.shortest_path (lattices.py:185-247) without the
 * cross-batch mask aliasing (D6): MaxTropical Viterbi with the reference's
 * tie rules (blank wins ties, semirings.py:363; first argmax among lexical
 * arcs and among final states, semirings.py:382).
 *   labels [B,T] int64 out (0 = blank; lexical per label_convention; 0 on
 *          padding frames), path_weight [B] out.
 *   arcs   [B,T,C,V+1] (nullable, W's dtype): if given, receives grad[b] on
 *          every arc of the best path and 0 elsewhere -- the vjp of
 *          _forward(MaxTropical) (grad nullable = ones).
 *   workspace: lt_viterbi_workspace_bytes() bytes of device memory.
 * The bigram (V <= 32) decodes and backtracks in one launch while an
 * utterance's backpointers fit the forward's LDS (T <= 2,300 at V = 32),
 * else the backtrace is a second launch. */
int lt_viterbi_workspace_bytes(const lt_problem* pb, size_t* bytes);
int lt_viterbi(const lt_problem* pb, const void* W, const int32_t* num_frames,
               int32_t label_convention, int64_t* labels, float* path_weight,
               const float* grad, void* arcs, void* workspace,
               size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * General lattices: any context dependency given as a next-state table and
 * either alignment lattice (lt_table.hip).
 *   context   contexts.NextStateTable (contexts.py:266-320), or any
 *             ContextDependency through its next_state_table() (FullNGram:
 *             contexts.py:258-263); forward_reduce is the (+) over in-arcs
 *             (the reference's NextStateTable.forward_reduce is defect D8)
 *   alignment expansions = 0: alignments.FrameDependent (alignments.py:250-329)
 *             expansions = K >= 1: alignments.FrameLabelDependent(K)
 *             (alignments.py:331-432), alignment-state-invariant weights
 *             (lattices.py:444-447)
 * W has the same [B, T, C, V+1] layout as above with C = num_states.
 * ------------------------------------------------------------------------ */
typedef struct lt_graph {
  int32_t num_states;        /* C */
  int32_t vocab_size;        /* V */
  int32_t expansions;        /* K: 0 FrameDependent, K >= 1 FrameLabelDependent */
  const int32_t* next_state; /* device [C, V]: next_state[p, y-1] (y = 1..V) */
  const int32_t* in_offsets; /* device [C+1]  } the arcs into each state, from */
  const int32_t* in_arcs;    /* device [C*V]  } lt_graph_in_arcs()            */
} lt_graph;

typedef struct lt_table_problem {
  int32_t batch, max_frames, max_labels, weight_dtype;
} lt_table_problem;

/* HOST helper: the in-arc CSR of a next-state table (host arrays): arcs
 * (id = p*V + y-1) grouped by next state, ascending (p, y) inside a group --
 * the reduce order, which fixes MaxTropical's first-argmax tie rule. */
int lt_graph_in_arcs(int32_t num_states, int32_t vocab_size, const int32_t* next_state,
                     int32_t* in_offsets, int32_t* in_arcs);

/* RecognitionLattice._forward (lattices.py:379-496): dist [B], alpha
 * [B,T,C] (state before frame t; nullable). Log / MaxTropical / Real. */
int lt_table_forward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                     const void* W, const int32_t* num_frames, float* dist, float* alpha,
                     void* stream);

/* RecognitionLattice._string_forward (lattices.py:250-377): num [B]. */
int lt_table_num_forward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                         const void* W, const int32_t* num_frames, const int32_t* labels,
                         const int32_t* num_labels, float* num, void* stream);

/* RecognitionLattice.forward (lattices.py:131-183) and, when dW is non-NULL,
 * d(sum_b loss_b)/dW (Log; local_norm: loss = -num). Unreachable strings:
 * loss = +inf, dW = 0. workspace: lt_table_loss_grad_workspace_bytes(). */
int lt_table_loss_grad_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                       size_t* bytes);
int lt_table_loss_grad(const lt_graph* g, const lt_table_problem* pb, int32_t local_norm,
                       const void* W, const int32_t* num_frames, const int32_t* labels,
                       const int32_t* num_labels, float* loss, float* log_z, float* num,
                       void* dW, void* workspace, size_t workspace_bytes, void* stream);

/* The gradient of lt_table_forward's distance (RecognitionLattice._forward
 * under autograd, lattices.py:379-496 with semirings.py:184-401; the
 * marginals of _backward / _forward_backward, lattices.py:498-799 with
 * FrameDependent.backward alignments.py:300-318 and
 * FrameLabelDependent.backward :379-419):
 *   LT_SEMIRING_LOG   dW = grad_b * d log_z / dW (the arc marginals); dist =
 *                     log_z and alpha = the [B,T,C] history of lt_table_forward
 *   LT_SEMIRING_REAL  dW = grad_b * d dist / dW = grad_b * alpha * beta'
 *                     (dist, alpha from lt_table_forward in Real)
 *   LT_SEMIRING_MAX   dW = grad_b on every arc of the best path (the first
 *                     maximum, as lt_table_viterbi), 0 elsewhere; dist and
 *                     alpha are not read (may be NULL)
 * grad [B] nullable (1). Padding frames get dW = 0; in Log / Real so do
 * utterances of non-finite distance, while MaxTropical marks the first
 * maximum's path whatever its weight (an all -inf utterance: the tie rules'
 * path, as the reference's argmax backward). workspace: lt_table_den_backward_workspace_bytes() (0 bytes for
 * fp32 W in Log / Real). */
int lt_table_den_backward_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                          int32_t semiring, size_t* bytes);
int lt_table_den_backward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                          const void* W, const int32_t* num_frames, const float* dist,
                          const float* alpha, const float* grad, void* dW, void* workspace,
                          size_t workspace_bytes, void* stream);

/* The gradient of lt_table_num_forward's string distance
 * (RecognitionLattice._string_forward under autograd, lattices.py:250-377,
 * through FrameDependent.string_forward alignments.py:320-329 or
 * FrameLabelDependent.string_forward :420-432):
 *   LT_SEMIRING_MAX   dW = grad_b on every arc of the best string-aligned
 *                     path (ties: the blank term / the fewest expansions,
 *                     semirings.py:354-401; an arc taken twice in a frame
 *                     gets 2 grad_b), walked back from num_labels -- or from
 *                     position 0 when alpha_T[num_labels] is -inf, which
 *                     carries a gradient only if num_labels == 0, as the
 *                     reference's Max over where(is_final, ...) does
 *   LT_SEMIRING_REAL  dW = grad_b * d num / dW (semirings.py:143-173)
 * Log: LT_EUNSUPPORTED (its gradient is lt_table_loss_grad with local_norm,
 * negated). grad [B] nullable (1); num [B] nullable out (the distance);
 * dW W's dtype and shape, zero off the string's arcs and on padding frames.
 * Arcs of several string positions on one lattice element sum in ascending
 * position order (deterministic). Any next-state table: FullNGram through
 * its next_state_table() (contexts.py:258-263). workspace:
 * lt_table_num_backward_workspace_bytes(). */
int lt_table_num_backward_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                          int32_t semiring, size_t* bytes);
int lt_table_num_backward(const lt_graph* g, const lt_table_problem* pb, int32_t semiring,
                          const void* W, const int32_t* num_frames, const int32_t* labels,
                          const int32_t* num_labels, const float* grad, float* num, void* dW,
                          void* workspace, size_t workspace_bytes, void* stream);

/* RecognitionLattice.shortest_path (lattices.py:185-247), per utterance (no
 * D6 aliasing): labels [B, T*A] int64 with A = 1 (FrameDependent) or K+1
 * (FrameLabelDependent): slot i of frame t = label of the (i+1)-th lexical
 * arc of that frame (label_convention as lt_viterbi), else 0; the last slot
 * of a FrameLabelDependent frame is always 0. path_weight [B] = the
 * MaxTropical distance. workspace: lt_table_viterbi_workspace_bytes(). */
int lt_table_viterbi_workspace_bytes(const lt_graph* g, const lt_table_problem* pb,
                                     size_t* bytes);
int lt_table_viterbi(const lt_graph* g, const lt_table_problem* pb, const void* W,
                     const int32_t* num_frames, int32_t label_convention, int64_t* labels,
                     float* path_weight, void* workspace, size_t workspace_bytes,
                     void* stream);

/* The design lt_loss_grad runs for *pb (a function of the shape and the
 * device's CU count only; the library reads no environment): LT_DESIGN_CHUNK the chunked
 * two-level scan (bigram, 5 * batch <= 3 * CUs), LT_DESIGN_FUSED_PIPE one
 * pipelined launch with the marginals beside the recursions,
 * LT_DESIGN_CHECKPOINTS alpha || beta with checkpoints then one streaming
 * marginal pass (the north-star B = 256), LT_DESIGN_RECURSION forward then a
 * backward recursion that writes dW. For bindings that call the two-call
 * entry points themselves and want lt_loss_grad's choice. */
#define LT_DESIGN_CHUNK 0
#define LT_DESIGN_FUSED_PIPE 1
#define LT_DESIGN_CHECKPOINTS 2
#define LT_DESIGN_RECURSION 3
#define LT_DESIGN_AUTO (-1)
int lt_loss_grad_design(const lt_problem* pb, int32_t* design);
/* lt_loss_grad with the design given explicitly (LT_DESIGN_AUTO: the call's
 * own choice, as lt_loss_grad): for callers that time or test one design at
 * a shape where lt_loss_grad would pick another. LT_EUNSUPPORTED when the
 * shape cannot take it (LT_DESIGN_CHUNK and LT_DESIGN_FUSED_PIPE are bigram
 * designs; LT_DESIGN_FUSED_PIPE, the one-launch pipe with the marginals in
 * the recursion workgroups, also needs U < 128 and its 2B workgroups
 * co-resident). Replaces the environment overrides of round 2. */
int lt_loss_grad_workspace_bytes_ex(const lt_problem* pb, int32_t local_norm, int32_t design,
                                    size_t* bytes);
int lt_loss_grad_ex(const lt_problem* pb, int32_t local_norm, int32_t design, const void* W,
                    const int32_t* num_frames, const int32_t* labels,
                    const int32_t* num_labels, float* loss, float* log_z, float* num,
                    void* dW, void* workspace, size_t workspace_bytes, void* stream);

/* Joint weight function on the matrix cores (replaces
 * the hidden-tensor path of JointWeightFn.forward, weight_fns.py:174-227):
 *   W[f, c, y] = out_bias[y] + sum_h out_weight[y, h] * tanh(ctx_proj[c, h] + frame_proj[f, h])
 * for f < rows (= B*T), c < num_states, y < out_dim (= V+1; <= 64), h < hidden
 * (a multiple of 16). ctx_proj [num_states, hidden], frame_proj [rows, hidden],
 * out_weight [out_dim, hidden], out_bias [out_dim]: fp32, 16-byte aligned. W
 * [rows, num_states, out_dim] in weight_dtype. The tanh values and out_weight
 * enter the products as bf16, sums are fp32. tanh(a + b) is formed from
 * e^{2a} e^{2b} (e^{2a} precomputed into the workspace, e^{2b} per block of
 * 32 frames) unless some |ctx_proj| or a block's |frame_proj| exceeds 40, in
 * which case that block evaluates e^{2(a+b)} directly.
 * workspace: lt_joint_weights_workspace_bytes() bytes, 16-byte aligned. */
int lt_joint_weights_workspace_bytes(int64_t rows, int32_t num_states, int32_t hidden,
                                     size_t* bytes);
int lt_joint_weights(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                     const float* ctx_proj, const float* frame_proj, const float* out_weight,
                     const float* out_bias, void* W, int32_t weight_dtype, void* workspace,
                     size_t workspace_bytes, void* stream);
/* lt_joint_weights with the product precision chosen: LT_JOINT_BF16 (as
 * lt_joint_weights) or LT_JOINT_SPLIT, the fp32-faithful mode for the
 * reference's fp32 JointWeightFn: the tanh values and out_weight each split
 * into bf16 hi + lo, hi*hi + hi*lo + lo*hi summed in fp32 (about 16 mantissa
 * bits per product, as lt_joint_weights_backward); out_weight then takes
 * twice the LDS (4 * out_dim * (hidden + 8) bytes <= 128 KB). */
#define LT_JOINT_BF16 0
#define LT_JOINT_SPLIT 1
int lt_joint_weights_ex(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                        const float* ctx_proj, const float* frame_proj, const float* out_weight,
                        const float* out_bias, void* W, int32_t weight_dtype, int32_t precision,
                        void* workspace, size_t workspace_bytes, void* stream);

/* Adjoint of lt_joint_weights (JointWeightFn's parameter gradients; the
 * reference gets them from autograd through weight_fns.py:174-227): with
 * grad_W = dL/dW [rows, num_states, out_dim] fp32 and hid = tanh(ctx_proj[c] +
 * frame_proj[f]) recomputed in fp32,
 *   d_out_weight[y, h] = sum_{f,c} grad_W[f, c, y] hid[f, c, h]
 *   d_out_bias[y]      = sum_{f,c} grad_W[f, c, y]
 *   dh[f, c, h]        = (sum_y grad_W[f, c, y] out_weight[y, h]) (1 - hid^2)
 *   d_ctx_proj[c, h]   = sum_f dh,   d_frame_proj[f, h] = sum_c dh
 * Products are split-bf16 (about 16 mantissa bits), sums fp32. Needs
 * hidden % 32 == 0, out_dim <= 64, rows * max(num_states, hidden) < 2^31 and
 * the d_ctx_proj block of one workgroup (4 * num_states * 32 * waves bytes,
 * waves = the largest of 8/4/2/1 dividing hidden / 32) plus 14 KB in LDS
 * (<= 160 KB). All outputs are overwritten, every sum in a fixed order
 * (deterministic). workspace: lt_joint_weights_backward_workspace_bytes(). */
int lt_joint_weights_backward_workspace_bytes(int64_t rows, int32_t num_states, int32_t hidden,
                                              int32_t out_dim, size_t* bytes);
int lt_joint_weights_backward(int64_t rows, int32_t num_states, int32_t hidden, int32_t out_dim,
                              const float* ctx_proj, const float* frame_proj,
                              const float* out_weight, const float* grad_W, float* d_ctx_proj,
                              float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                              void* workspace, size_t workspace_bytes, void* stream);

/* The joint weight function fused into the lattice loss (SURVEY.md 8(f)
 * rank 1; replaces lt_joint_weights -> lt_loss_grad -> lt_joint_weights_backward
 * for RecognitionLattice(JointWeightFn).forward + .backward, weight_fns.py:
 * 174-227 consumed at lattices.py:446): the loss of FullNGram n = 1 (16 <
 * vocab_size <= 32) x FrameDependent under Log, fp32, with
 *   W[b,t,c,y] = out_bias[y] + sum_h out_weight[y,h] tanh(ctx_proj[c,h] + frame_proj[b*T+t,h])
 * formed on the matrix cores where the recursions and the marginal pass use
 * it -- bit-identical to lt_joint_weights_ex's W in the same precision -- and
 * the parameter gradients formed from the marginals in LDS: neither W nor
 * d loss / dW is ever written to memory.
 *   lt_loss_joint_forward   loss [B] (log_z, num [B] nullable), keeping the
 *                           recursions' checkpoints in `state`
 *   lt_loss_joint_backward  d_ctx_proj [C,H], d_frame_proj [B*T,H],
 *                           d_out_weight [V+1,H], d_out_bias [V+1] of
 *                           sum_b grad[b] loss_b (grad nullable = ones;
 *                           unreachable strings contribute 0), from `state`
 *   lt_loss_grad_joint      both, one workspace (state then scratch)
 * hidden: a multiple of 32 up to 256 whose marginal-pass LDS image fits the
 * CU's 160 KB (lt_loss_joint_workspace_bytes returns LT_EUNSUPPORTED
 * otherwise): at max_labels = 100, H <= 192 with split products, H <= 224
 * with bf16 ones. max_labels < 128. A pipeline wait that timed out makes
 * loss / log_z / num and every gradient NaN (never a silent result). The
 * d_ctx_proj / d_out_weight / d_out_bias sums run in a fixed order
 * (deterministic). */
typedef struct lt_joint_params {
  int32_t hidden;           /* H */
  int32_t precision;        /* LT_JOINT_SPLIT or LT_JOINT_BF16 (forward products) */
  const float* ctx_proj;    /* [C, H]    */
  const float* frame_proj;  /* [B*T, H]  */
  const float* out_weight;  /* [V+1, H]: row 0 blank, row y label y */
  const float* out_bias;    /* [V+1]     */
} lt_joint_params;
int lt_loss_joint_workspace_bytes(const lt_problem* pb, const lt_joint_params* jp,
                                  size_t* state_bytes, size_t* scratch_bytes);
int lt_loss_joint_forward(const lt_problem* pb, const lt_joint_params* jp,
                          const int32_t* num_frames, const int32_t* labels,
                          const int32_t* num_labels, float* loss, float* log_z, float* num,
                          void* state, size_t state_bytes, void* stream);
int lt_loss_joint_backward(const lt_problem* pb, const lt_joint_params* jp,
                           const int32_t* num_frames, const float* grad, float* d_ctx_proj,
                           float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                           void* state, size_t state_bytes, void* scratch, size_t scratch_bytes,
                           void* stream);
int lt_loss_grad_joint(const lt_problem* pb, const lt_joint_params* jp, const int32_t* num_frames,
                       const int32_t* labels, const int32_t* num_labels, const float* grad,
                       float* loss, float* log_z, float* num, float* d_ctx_proj,
                       float* d_frame_proj, float* d_out_weight, float* d_out_bias,
                       void* workspace, size_t workspace_bytes, void* stream);

/* Thread-local description of the last error; never NULL. */
const char* lt_last_error(void);
/* Library version string. */
const char* lt_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LT_LATTICE_H_ */
