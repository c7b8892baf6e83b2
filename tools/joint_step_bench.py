"""Times one training step of RecognitionLattice driven by JointWeightFn
(SharedEmbCacher + JointWeightFn, weight_fns.py:174-242): the frame and
context projections, the arc weights, the lattice loss + dW, and the
backward into every weight-function parameter. The step runs at the bench
lattice shape (B=64, T=1000, U=100, bigram V=32, C=33) with hidden size H and
feature size F. It is run twice: with the matrix-core producer
(lt_joint_weights / lt_joint_weights_backward), and with the PyTorch hidden
tensor (fused=False). The lattice kernels are the same in both. Prints one
JSON line per H."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import last_torch_amd as lt  # noqa: E402


def main():
  B, T, U, V, F = 64, 1000, 100, 32, 256
  dev = torch.device('cuda')
  for H in [int(h) for h in os.environ.get('HS', '512').split(',')]:
    torch.manual_seed(0)
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=1)
    cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=128,
                                           device=dev)
    wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=H, device=dev)
    lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                                weight_fn_cacher_factory=lambda _: cacher,
                                weight_fn_factory=lambda _: wfn)
    frames = torch.randn([B, T, F], device=dev)
    nf = torch.full([B], T, device=dev)
    labels = torch.randint(1, V + 1, [B, U], device=dev)
    nl = torch.full([B], U, device=dev)

    def step():
      loss = lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl)
      loss.sum().backward()
      return loss

    out = {'B': B, 'T': T, 'U': U, 'V': V, 'C': V + 1, 'F': F, 'H': H}
    for name, fused, prec in (('producer', True, 'fp32'), ('producer_bf16', True, 'bf16'),
                              ('pytorch_hidden', False, 'fp32')):
      wfn.fused = fused
      wfn.precision = prec
      for _ in range(3):  # lazy layers, allocator, clocks
        step()
      torch.cuda.synchronize()
      e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
      reps = 10
      e0.record()
      for _ in range(reps):
        loss = step()
      e1.record()
      torch.cuda.synchronize()
      out[f'{name}_step_ms'] = e0.elapsed_time(e1) / reps
      out[f'{name}_loss_mean'] = float(loss.mean())
    out['speedup'] = out['pytorch_hidden_step_ms'] / out['producer_step_ms']
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
