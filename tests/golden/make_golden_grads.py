"""Generates tests/golden/grads_*.npz: the reference's own autograd gradients
of its shortest distances under MaxTropical and Real, for the inputs of every
lattice_*.npz (FrameDependent) and fld_*.npz (FrameLabelDependent(K))
fixture.

Run in the development container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_grads.py /root/reference

The inputs are read back from the committed fixtures (W, num_frames, labels,
num_labels, V, n, K), so those fixtures are not regenerated. For each
semiring s in (MaxTropical, Real), with the arc-weight table as the leaf of
the reference's TableWeightFn (weight_fns.py:307-342):

  den_grad_<s>  d sum_b _forward(..., s)[0][b] / dW        lattices.py:379-496
  num_grad_<s>  d sum_b _string_forward(..., s)[b] / dW    lattices.py:250-377

by loss.backward() through the reference's code -- its Real semiring is
plain arithmetic (semirings.py:143-173) and its MaxTropical plus / sum
backward through Maximum (a >= b keeps a) and Max (first argmax,
semirings.py:354-401), so these gradients are sound there (only Log's are
broken). num_grad_<s> is recorded only for FrameDependent and
for FrameLabelDependent string forwards (one batch dim, D13 holds here).
"""
import glob
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def main(ref_path):
  os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
  sys.dont_write_bytecode = True
  sys.path.insert(0, ref_path)
  import last_torch as lt
  torch.set_default_dtype(torch.float32)

  def lattice_for(table, V, n, K):
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    align = (lt.alignments.FrameDependent() if K == 0
             else lt.alignments.FrameLabelDependent(max_expansions=K))
    return lt.RecognitionLattice(
        context=ctx, alignment=align,
        weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
        weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))

  def frames_for(B, T):
    return torch.broadcast_to(torch.arange(T)[None, :, None], [B, T, 1]).float()

  def grads(d, K):
    W = d['W']
    V, n = int(d['vocab_size']), int(d['context_size'])
    B, T = W.shape[:2]
    nf = torch.as_tensor(d['num_frames']).float()
    out = {}
    for sname in ('MaxTropical', 'Real'):
      s = getattr(lt.semirings, sname)
      table = torch.tensor(W, requires_grad=True)
      dist, _ = lattice_for(table, V, n, K)._forward(cache=None, frames=frames_for(B, T),
                                                     num_frames=nf, semiring=s)
      dist.sum().backward()
      out[f'den_{sname}'] = dist.detach().numpy().astype(np.float32)
      out[f'den_grad_{sname}'] = table.grad.numpy().astype(np.float32)
      table = torch.tensor(W, requires_grad=True)
      num = lattice_for(table, V, n, K)._string_forward(
          cache=None, frames=frames_for(B, T), num_frames=nf,
          labels=torch.as_tensor(d['labels']).float(),
          num_labels=torch.as_tensor(d['num_labels']).float(), semiring=s)
      num.sum().backward()
      g = table.grad
      out[f'num_{sname}'] = num.detach().numpy().astype(np.float32)
      out[f'num_grad_{sname}'] = (torch.zeros_like(table) if g is None else g).numpy().astype(
          np.float32)
    return out

  for path in sorted(glob.glob(os.path.join(OUT, 'lattice_*.npz')) +
                     glob.glob(os.path.join(OUT, 'fld_*.npz'))):
    name = os.path.basename(path)[:-4]
    with np.load(path) as z:
      d = {k: z[k] for k in z.files}
    K = int(d['K']) if 'K' in d else 0
    g = grads(d, K)
    # the distances must be the fixture's own (same reference, same inputs)
    for sname in ('MaxTropical', 'Real'):
      np.testing.assert_array_equal(g[f'den_{sname}'], d[f'den_{sname}'])
      np.testing.assert_array_equal(g[f'num_{sname}'], d[f'num_{sname}'])
    keep = {k: v for k, v in g.items() if 'grad' in k}
    np.savez_compressed(os.path.join(OUT, f'grads_{name}.npz'), **keep)
    print('wrote grads', name, {k: float(np.abs(v).sum()) for k, v in keep.items()})


if __name__ == '__main__':
  main(sys.argv[1] if len(sys.argv) > 1 else '/root/reference')
