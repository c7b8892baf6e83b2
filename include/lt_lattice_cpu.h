/*
 * lt_lattice_cpu.h -- C ABI of the host (CPU) twin of the lattice library.
 *
 * Same computations and conventions as lt_lattice.h (same lt_problem, same
 * W layout [B, T, C, V+1] in fp32 or bf16, same label conventions, same
 * error codes), but every pointer is a HOST pointer and every call returns
 * when its results are written. It is built without HIP
 * (last_torch_amd/liblt_lattice_cpu.so), so a GPU-less host binds it the way
 * a ROCm host binds liblt_lattice.so ("the C++ CPU twin
 * exports the same set as lt_cpu_*"). Utterances run in parallel on a pool
 * of host threads; one utterance is one thread's serial frame loop.
 *
 * Arithmetic: fp32, as the reference (last_torch runs its recursions in the
 * weight dtype, lattices.py:482). Log vectors are held relative to an
 * integer offset near their maximum (exact), so their roundings stay those
 * of small numbers however long the utterance; MaxTropical runs the
 * reference's own float operations and tie rules (bit-exact).
 *
 * Reference entry points each function replaces (last_torch/):
 *   lt_cpu_den_forward   RecognitionLattice._forward        lattices.py:379-496
 *   lt_cpu_num_forward   RecognitionLattice._string_forward lattices.py:250-377
 *   lt_cpu_loss_grad     RecognitionLattice.forward + loss.sum().backward()
 *                        lattices.py:131-183, alignments.py:300-318
 *   lt_cpu_den_backward  _backward's marginals              lattices.py:686-799
 *   lt_cpu_viterbi       RecognitionLattice.shortest_path   lattices.py:185-247
 */
#ifndef LT_LATTICE_CPU_H_
#define LT_LATTICE_CPU_H_

#include "lt_lattice.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host threads used by the calls below (default: the host's hardware
 * concurrency). n <= 0 restores the default. */
int lt_cpu_set_num_threads(int32_t n);
int lt_cpu_num_threads(void);

/* lt_den_forward on the host: dist [B], alpha [B,T,C] (nullable; padding
 * frames carry alpha). semiring LT_SEMIRING_LOG / MAX / REAL. */
int lt_cpu_den_forward(const lt_problem* pb, int32_t semiring, const void* W,
                       const int32_t* num_frames, float* dist, float* alpha);

/* lt_num_forward on the host: num [B], alpha_num [B,T,U+1] (nullable). */
int lt_cpu_num_forward(const lt_problem* pb, int32_t semiring, const void* W,
                       const int32_t* num_frames, const int32_t* labels,
                       const int32_t* num_labels, float* num, float* alpha_num);

/* lt_den_backward on the host: dW = grad[b] * den marginals from log_z and
 * the alpha history of lt_cpu_den_forward(LOG). grad nullable (= ones). */
int lt_cpu_den_backward(const lt_problem* pb, const void* W, const int32_t* num_frames,
                        const float* log_z, const float* alpha, const float* grad, void* dW);

/* lt_loss_grad on the host: loss, log_z, num [B] (log_z / num nullable) and,
 * when dW is non-NULL, dW = grad[b] * d loss_b / dW (grad nullable = ones;
 * utterances with an unreachable string or a non-finite log_z get dW = 0;
 * padding frames 0). local_norm != 0: loss = -num (lattices.py:178-179). */
int lt_cpu_loss_grad(const lt_problem* pb, int32_t local_norm, const void* W,
                     const int32_t* num_frames, const int32_t* labels,
                     const int32_t* num_labels, const float* grad, float* loss,
                     float* log_z, float* num, void* dW);

/* lt_viterbi on the host: labels [B,T] int64, path_weight [B], arcs
 * [B,T,C,V+1] (nullable, W's dtype: grad[b] on the best path's arcs). */
int lt_cpu_viterbi(const lt_problem* pb, const void* W, const int32_t* num_frames,
                   int32_t label_convention, int64_t* labels, float* path_weight,
                   const float* grad, void* arcs);

const char* lt_cpu_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LT_LATTICE_CPU_H_ */
